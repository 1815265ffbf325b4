// LinUCB's numpy arithmetic in OpenBLAS's rounding orders (ctrls/ctrl_bandit.py:503-526), shared by
// the policy kernels (dpt_policies.hip) and the host-side order check (tests/test_linucb_orders.py,
// which compiles this header with g++: no HIP types here).
#pragma once
#include <math.h>
#ifndef __HIPCC__
#ifndef __host__
#define __host__
#define __device__
#endif
#include <algorithm>
using std::min;
#endif

namespace dpt {

constexpr int kMaxD = 8;  // LinUCB feature dimension (lin_d) supported

// ----------------------------------------------------------------------------- LinUCB
// LinUCBPolicy.act_numpy_vec (ctrls/ctrl_bandit.py:503-526) rebuilds its estimate from the
// whole context every step with numpy:
//   X = arms[argmax(actions)]; cov = I + X^T X; cov_inv = np.linalg.inv(cov)
//   theta = (cov_inv @ X^T) @ r; value_k = theta @ arm_k + c * sqrt(arm_k @ cov_inv @ arm_k)
// numpy hands each product to its BLAS (OpenBLAS, scipy-openblas 0.3.29 in the image the
// fixtures were recorded in) and each of those kernels has its own, fixed rounding order.  The
// lane restates those orders (established against numpy on the recording host:
// tests/golden/gen_golden.py linucb fixtures), so at lin_d = 2 every value -- and so every arm
// index -- is bit-identical to the reference's:
//   X^T X  dsyrk: per entry one fma chain over the context, K-blocked like the level-3 driver
//          (blocks of GEMM_Q = 384, a remainder between Q and 2Q split in halves), C += block;
//   inv    dgesv(cov, I): linucb_inverse (OpenBLAS's left-looking getf2, then getrs through its
//          trsm kernels' row chunks; below);
//   cov_inv @ X^T  dgemm with K = d: per entry an fma chain from 0;
//   (.) @ r  dgemv_t: 2048-row blocks of the first n - n%4 rows, two interleaved unfused
//          accumulators per block summed into y, then the n%4 tail rows contracted into y;
//   theta @ arm, arm @ cov_inv, (.) @ arm  ddot / dgemv_n with d rows: fma chains from 0.
// tests/test_linucb_orders.py runs this code on the host against numpy itself on random contexts:
// the inverse is bit-identical for lin_d <= 5 and the arm values for lin_d <= 5 (see there for
// lin_d 6..8, where getf2's longer dot / gemv kernels are not restated and values agree to rounding).
constexpr int kSyrkQ = 384;
__host__ __device__ inline int syrk_block(int ls, int n) {
    const int ml = n - ls;
    if (ml >= 2 * kSyrkQ) return kSyrkQ;
    if (ml > kSyrkQ) return (ml + 1) / 2;
    return ml;
}

// dgemv_t row reduction y = sum_k m(k) r(k) over k < n in OpenBLAS's order (dgemv_t_4.c, established
// against numpy: tests/test_linucb_orders.py).  The driver takes the output rows (columns of its
// column-major view) in groups of 4, then 2, then 1, each group through its own kernel over 2048-row
// blocks of the first n - n%4 terms; a block's partial is added into y, then the n%4 tail terms:
//   4-row kernel: four fma accumulators (term k into k % 4), (s0 + s2) + (s1 + s3);
//   2-row kernel: two unfused accumulators (k % 2), s0 + s1;
//   1-row kernel: four unfused accumulators (k % 4), (s0 + s2) + (s1 + s3);
//   tail: fma for one term, y + fma(a0, x0, a1 x1) for two, y + fma(a2, x2, fma(a0, x0, a1 x1)) for three.
// gemv_t_cols(p, rows) is the kernel width of output row p of a product with `rows` output rows.
__host__ __device__ inline int gemv_t_cols(int p, int rows) {
    const int n4 = rows & ~3;
    if (p < n4) return 4;
    if ((rows & 2) && p < n4 + 2) return 2;
    return 1;
}
template <class Mk, class Rk>
__host__ __device__ inline double gemv_t_sum(Mk m, Rk r, int n, int cols = 2) {
    const int m3 = n & 3, m1 = n - m3;
    double y = 0.0;
    for (int s0 = 0; s0 < m1; s0 += 2048) {
        const int nb = min(2048, m1 - s0);
        double l0 = 0.0, l1 = 0.0, l2 = 0.0, l3 = 0.0;
        int k = s0;
        if (cols == 2) {
            // the products of 8 terms first (independent loads in flight), then the two chains in order
            for (; k + 8 <= s0 + nb; k += 8) {
                double pr[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) pr[t] = m(k + t) * r(k + t);
#pragma unroll
                for (int t = 0; t < 8; t += 2) {
                    l0 = l0 + pr[t];
                    l1 = l1 + pr[t + 1];
                }
            }
            for (; k < s0 + nb; k += 2) {
                l0 = l0 + m(k) * r(k);
                l1 = l1 + m(k + 1) * r(k + 1);
            }
            y = y + (l0 + l1);
        } else if (cols == 4) {
            for (; k < s0 + nb; k += 4) {
                l0 = fma(m(k), r(k), l0);
                l1 = fma(m(k + 1), r(k + 1), l1);
                l2 = fma(m(k + 2), r(k + 2), l2);
                l3 = fma(m(k + 3), r(k + 3), l3);
            }
            y = y + ((l0 + l2) + (l1 + l3));
        } else {
            for (; k < s0 + nb; k += 4) {
                l0 = l0 + m(k) * r(k);
                l1 = l1 + m(k + 1) * r(k + 1);
                l2 = l2 + m(k + 2) * r(k + 2);
                l3 = l3 + m(k + 3) * r(k + 3);
            }
            y = y + ((l0 + l2) + (l1 + l3));
        }
    }
    if (m3 == 1) {
        y = fma(m(m1), r(m1), y);
    } else if (m3 == 2) {
        y = y + fma(m(m1), r(m1), m(m1 + 1) * r(m1 + 1));
    } else if (m3 == 3) {
        y = y + fma(m(m1 + 2), r(m1 + 2), fma(m(m1), r(m1), m(m1 + 1) * r(m1 + 1)));
    }
    return y;
}

// np.linalg.inv(cov) as numpy's OpenBLAS computes it (dgesv with B = I), established against numpy
// on random covariances (tests/test_linucb_orders.py; bit-identical for every d <= kMaxD):
//  getf2, left-looking over the columns of A (cov is symmetric, so A's column-major view is cov):
//    column j: the earlier row swaps; U part u_ij -= ddot(l_i,0..i-1, u_0..i-1,j); the rest a_rj -= the
//    dgemv_n of the rows below; pivot = the first max |a_rj|; the rows swapped over columns 0..j; the
//    column below the pivot scaled by 1 / pivot;
//  getrs: the row swaps on e_col, then the trsm kernels: L (unit) top-down and U bottom-up in row
//    chunks (full chunks of kUM and the power-of-two remainders, in the kernels' order); a chunk first
//    subtracts the solved rows' contribution (one fma chain from 0 over them, ascending), then solves
//    in place: x_i = c_i (1 / u_ii), c_k = fma(-a_ki, x_i, c_k).
// lu: cov on entry (row stride kMaxD), the factors on return; piv, c: d scratch entries; ci[p][col].
template <class F, class I>
__host__ __device__ inline void linucb_inverse(F* lu, I* piv, F* c, double* ci, int d) {
#define DPT_LA(r, q) lu[(q) * kMaxD + (r)]
    for (int j = 0; j < d; ++j) {
        for (int i = 0; i < j; ++i) {
            const int ip = piv[i];
            if (ip != i) {
                const double t = DPT_LA(i, j);
                DPT_LA(i, j) = DPT_LA(ip, j);
                DPT_LA(ip, j) = t;
            }
        }
        for (int i = 1; i < j; ++i) {
            // ddot with a strided x (the row of L): 4-term steps into two sums (t1 += fma(y0, x0, y2 x2),
            // t2 += fma(y1, x1, y3 x3)), the rest fma into t1, then t1 + t2
            double t1 = 0.0, t2 = 0.0;
            int k = 0;
            for (; k + 4 <= i; k += 4) {
                t1 = t1 + fma(DPT_LA(k, j), DPT_LA(i, k), DPT_LA(k + 2, j) * DPT_LA(i, k + 2));
                t2 = t2 + fma(DPT_LA(k + 1, j), DPT_LA(i, k + 1), DPT_LA(k + 3, j) * DPT_LA(i, k + 3));
            }
            for (; k < i; ++k) t1 = fma(DPT_LA(k, j), DPT_LA(i, k), t1);
            DPT_LA(i, j) = DPT_LA(i, j) - (t1 + t2);
        }
        // dgemv_n over the rows below: rows in whole blocks of 4 subtract each column group's contracted sum
        // (linucb_w's groups) in turn; the (d - j) % 4 tail rows subtract one fma chain from 0
        const int mb = (d - j) & ~3;
        for (int r = j; r < d; ++r) {
            auto a = [&](int k) { return DPT_LA(r, k); };
            auto x = [&](int k) { return DPT_LA(k, j); };
            if (r - j < mb) {
                double y = DPT_LA(r, j);
                int k = 0;
                for (; k + 4 <= j; k += 4) y = y - fma(a(k + 3), x(k + 3), fma(a(k + 2), x(k + 2), fma(a(k), x(k), a(k + 1) * x(k + 1))));
                if ((j - k) & 2) {
                    y = y - fma(a(k), x(k), a(k + 1) * x(k + 1));
                    k += 2;
                }
                if ((j - k) & 1) y = y - a(k) * x(k);
                DPT_LA(r, j) = y;
            } else {
                double s = 0.0;
                for (int k = 0; k < j; ++k) s = fma(a(k), x(k), s);
                DPT_LA(r, j) = DPT_LA(r, j) - s;
            }
        }
        int jp = j;
        for (int r = j + 1; r < d; ++r)
            if (fabs(DPT_LA(r, j)) > fabs(DPT_LA(jp, j))) jp = r;
        piv[j] = jp;
        if (jp != j)
            for (int q = 0; q <= j; ++q) {
                const double t = DPT_LA(j, q);
                DPT_LA(j, q) = DPT_LA(jp, q);
                DPT_LA(jp, q) = t;
            }
        const double t1 = 1.0 / DPT_LA(j, j);
        for (int r = j + 1; r < d; ++r) DPT_LA(r, j) = DPT_LA(r, j) * t1;
    }
    constexpr int kUM = 16;  // the trsm kernels' row unroll (GEMM_UNROLL_M of the recording host's dgemm)
    // rows r0 .. r0 + n - 1 minus the solved rows k0 .. k0 + kn - 1 (one chain per row)
    auto upd = [&](int r0, int n, int k0, int kn) {
        for (int r = r0; r < r0 + n; ++r) {
            double s = 0.0;
            for (int k = k0; k < k0 + kn; ++k) s = fma(DPT_LA(r, k), c[k], s);
            c[r] = c[r] - s;
        }
    };
    auto solve_l = [&](int r0, int n) {
        for (int i = r0; i < r0 + n; ++i)
            for (int k = i + 1; k < r0 + n; ++k) c[k] = fma(-DPT_LA(k, i), c[i], c[k]);
    };
    auto solve_u = [&](int r0, int n) {
        for (int i = r0 + n - 1; i >= r0; --i) {
            const double bb = c[i] * (1.0 / DPT_LA(i, i));
            c[i] = bb;
            for (int k = r0; k < i; ++k) c[k] = fma(-DPT_LA(k, i), bb, c[k]);
        }
    };
    for (int col = 0; col < d; ++col) {
        for (int p = 0; p < d; ++p) c[p] = p == col ? 1.0 : 0.0;
        for (int j = 0; j < d; ++j) {
            const double t = c[j];
            c[j] = c[piv[j]];
            c[piv[j]] = t;
        }
        int kk = 0;  // L: full chunks from the top, then the remainders kUM/2 .. 1
        for (int q = 0; q < d / kUM; ++q) {
            if (kk > 0) upd(kk, kUM, 0, kk);
            solve_l(kk, kUM);
            kk += kUM;
        }
        for (int i = kUM >> 1; i > 0; i >>= 1)
            if (d & i) {
                if (kk > 0) upd(kk, i, 0, kk);
                solve_l(kk, i);
                kk += i;
            }
        kk = d;  // U: the remainders 1 .. kUM/2 from the bottom, then full chunks upwards
        for (int i = 1; i < kUM; i <<= 1)
            if (d & i) {
                const int r0 = (d & ~(i - 1)) - i;
                if (d > kk) upd(r0, i, kk, d - kk);
                solve_u(r0, i);
                kk -= i;
            }
        for (int q = 0; q < d / kUM; ++q) {
            const int r0 = kk - kUM;
            if (d > kk) upd(r0, kUM, kk, d - kk);
            solve_u(r0, kUM);
            kk -= kUM;
        }
        for (int p = 0; p < d; ++p) ci[p * kMaxD + col] = c[p];
    }
#undef DPT_LA
}

// Entry (p, k) of cov_inv @ X^T for a context row x: with n >= 2 rows numpy runs dgemm (K = d: one fma
// chain from the first product); with a single row X^T is a vector and numpy runs dgemv_t over row p of
// cov_inv (gemv_t_sum's order over the d entries, the kernel width of output row p)
__host__ __device__ inline double linucb_m(const double* cp, const double* x, int d, int n, int p) {
    if (n == 1) return gemv_t_sum([&](int j) { return cp[j]; }, [&](int j) { return x[j]; }, d, gemv_t_cols(p, d));
    double acc = cp[0] * x[0];
    for (int j = 1; j < d; ++j) acc = fma(cp[j], x[j], acc);
    return acc;
}

// Entry j of arm @ cov_inv: numpy runs dgemv_n (dgemv_n_4.c).  Output rows in whole blocks of 4 take
// the columns in groups of 4, each group's sum contracted as the kernels' C expressions compile
// (fma(a3, x3, fma(a2, x2, fma(a0, x0, a1 x1)))) and added into y, then a pair (fma(a0, x0, a1 x1)) and
// a single product likewise; the d % 4 tail rows are one fma chain from 0.  ci has row stride kMaxD.
__host__ __device__ inline double linucb_w(const double* ci, const double* x, int d, int j) {
    auto a = [&](int p) { return ci[p * kMaxD + j]; };
    if (j >= (d & ~3)) {
        double s = a(0) * x[0];
        for (int p = 1; p < d; ++p) s = fma(a(p), x[p], s);
        return s;
    }
    double y = 0.0;
    int p = 0;
    for (; p + 4 <= d; p += 4)
        y = y + fma(a(p + 3), x[p + 3], fma(a(p + 2), x[p + 2], fma(a(p), x[p], a(p + 1) * x[p + 1])));
    if ((d - p) & 2) {
        y = y + fma(a(p), x[p], a(p + 1) * x[p + 1]);
        p += 2;
    }
    if ((d - p) & 1) y = y + a(p) * x[p];
    return y;
}

// One LinUCB decision from the n-transition context (arm indices act(k), rewards rew(k), time
// order).  arms (A, d) row-major.
template <class Act, class Rew>
__host__ __device__ int linucb_choose(Act act, Rew rew, int n, const double* arms, int A, int d, double c,
                                      double* values_out = nullptr, double* ci_out = nullptr) {
    // cov = I + X^T X (upper triangle, mirrored like numpy's syrk result)
    double cov[kMaxD * kMaxD];
    for (int p = 0; p < d; ++p)
        for (int q = p; q < d; ++q) cov[p * kMaxD + q] = 0.0;
    for (int ls = 0; ls < n;) {
        const int ml = syrk_block(ls, n);
        double acc[kMaxD * kMaxD];
        for (int p = 0; p < d; ++p)
            for (int q = p; q < d; ++q) acc[p * kMaxD + q] = 0.0;
        for (int k0 = ls; k0 < ls + ml; k0 += 8) {
            // the arm indices of 8 transitions loaded together, then the fma chains in order
            const int kn = min(8, ls + ml - k0);
            int ak[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) ak[t] = t < kn ? act(k0 + t) : 0;
            for (int t = 0; t < kn; ++t) {
                const double* x = arms + (size_t)ak[t] * d;
                for (int p = 0; p < d; ++p)
                    for (int q = p; q < d; ++q) acc[p * kMaxD + q] = fma(x[p], x[q], acc[p * kMaxD + q]);
            }
        }
        for (int p = 0; p < d; ++p)
            for (int q = p; q < d; ++q) cov[p * kMaxD + q] = cov[p * kMaxD + q] + acc[p * kMaxD + q];
        ls += ml;
    }
    for (int p = 0; p < d; ++p) {
        cov[p * kMaxD + p] = 1.0 + cov[p * kMaxD + p];
        for (int q = p + 1; q < d; ++q) {
            cov[p * kMaxD + q] = 0.0 + cov[p * kMaxD + q];
            cov[q * kMaxD + p] = cov[p * kMaxD + q];
        }
    }
    double ci[kMaxD * kMaxD];
    {
        int piv[kMaxD];
        double cs[kMaxD];
        linucb_inverse(cov, piv, cs, ci, d);
    }
    if (ci_out)
        for (int p = 0; p < d; ++p)
            for (int q = 0; q < d; ++q) ci_out[p * d + q] = ci[p * kMaxD + q];
    // theta = (cov_inv @ X^T) @ r
    double theta[kMaxD];
    for (int p = 0; p < d; ++p) {
        const double* cp = ci + p * kMaxD;
        auto mk = [&](int k) { return linucb_m(cp, arms + (size_t)act(k) * d, d, n, p); };
        theta[p] = gemv_t_sum(mk, rew, n, gemv_t_cols(p, d));
    }
    int best_k = 0;
    double best = -INFINITY;
    for (int k = 0; k < A; ++k) {
        const double* x = arms + (size_t)k * d;
        double tv = theta[0] * x[0];
        for (int p = 1; p < d; ++p) tv = fma(theta[p], x[p], tv);
        double qv = 0.0;
        for (int j = 0; j < d; ++j) {
            const double w = linucb_w(ci, x, d, j);
            qv = j == 0 ? w * x[0] : fma(w, x[j], qv);
        }
        const double v = tv + c * sqrt(qv);
        if (values_out) values_out[k] = v;
        if (v > best) { best = v; best_k = k; }
    }
    return best_k;
}

}  // namespace dpt
