// Shared device-side definitions for libdpt_hip.so (gfx950 / CDNA4 only).
//
// Compiled with -ffp-contract=off: every fused multiply-add below is an
// explicit fmaf()/__builtin_amdgcn_mfma_*, so the fp64 env arithmetic stays
// two-rounding (bit-exact to numpy) and the fp32 model arithmetic is exactly
// the order written here.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dpt_hip.h"

namespace dpt {

constexpr int kE = 32;          // n_embd (only size built; common_args.py:31 default)
constexpr int kFF = 4 * kE;     // GPT-2 inner dim
constexpr int kWave = 64;
constexpr int kMaxA = 32;       // action_dim limit of the selection / head tiles
constexpr int kMaxF = 64;       // token feature limit (2*sd + A + 1)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef double doublex2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------------------- error plumbing
void set_error(int code, const char* fmt, ...);
int check_hip(hipError_t e, const char* what);

// ----------------------------------------------------------------------------- model view
// Offsets (in floats) inside one transformer block of the packed blob, dpt_hip.h order.
struct LayerOff {
    static constexpr int ln1_g = 0;
    static constexpr int ln1_b = ln1_g + kE;
    static constexpr int attn_w = ln1_b + kE;
    static constexpr int attn_b = attn_w + kE * 3 * kE;
    static constexpr int proj_w = attn_b + 3 * kE;
    static constexpr int proj_b = proj_w + kE * kE;
    static constexpr int ln2_g = proj_b + kE;
    static constexpr int ln2_b = ln2_g + kE;
    static constexpr int fc_w = ln2_b + kE;
    static constexpr int fc_b = fc_w + kE * kFF;
    static constexpr int mp_w = fc_b + kFF;
    static constexpr int mp_b = mp_w + kFF * kE;
    static constexpr int size = mp_b + kE;  // 12,704 floats per block at E = 32
};
static_assert(LayerOff::size == 12704, "GPT-2 block parameter count at E=32");

// Device pointers into one packed weight blob (passed to kernels by value).
struct ModelView {
    const float* emb_w;   // [F][E]
    const float* emb_b;   // [E]
    const float* wpe;     // [n_positions][E]
    const float* layers;  // n_layer * LayerOff::size
    const float* lnf_g;
    const float* lnf_b;
    const float* head_w;  // [E][A]
    const float* head_b;  // [A]
    // every block's attention folded (L0Off, one block per layer): G = Wq Wk^T,
    // g0 = Wk bq, Wvp = Wv Wproj, bvp = bv Wproj + bproj
    const float* l0;
    int n_layer, sd, A, F, n_positions;
    // MLP products on fp16 two-part splits (dpt_mfma_fwd.h Split2): c_fc / mlp.c_proj
    // weights are packed x 2^mlp_ew and the activations split x 2^mlp_ex, powers of two
    // chosen at model creation from static bounds (mlp_scales), so nothing overflows fp16
    int mlp_ew, mlp_ex;
    // the same for the attention's dense products and scores: G and Wvp packed x 2^attn_ew,
    // ln_1 outputs y (keys) and attention outputs x 2^attn_ey, queries u x 2^attn_eq
    int attn_ew, attn_ey, attn_eq;
};

// ----------------------------------------------------------------------------- Philox4x32-10
struct U4 { uint32_t x, y, z, w; };

__host__ __device__ inline uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

// Philox4x32 with 10 rounds (Salmon et al., SC'11); key = seed, counter =
// (step lo, task lo, stream, task hi ^ step hi).
__host__ __device__ inline U4 philox(uint64_t seed, uint64_t step, int64_t task, uint32_t stream) {
    uint32_t c0 = (uint32_t)step, c1 = (uint32_t)task, c2 = stream;
    uint32_t c3 = (uint32_t)((uint64_t)task >> 32) ^ (uint32_t)(step >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, &hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, &hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return U4{c0, c1, c2, c3};
}

// 53-bit uniform in [0, 1) from two words (numpy's random_sample construction).
__host__ __device__ inline double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

__host__ __device__ inline double philox_uniform(uint64_t seed, uint64_t step, int64_t task, uint32_t stream) {
    U4 r = philox(seed, step, task, stream);
    return u53(r.x, r.y);
}

// Box-Muller standard normal from one Philox block (u1 in (0,1], u2 in [0,1)).
__device__ inline double philox_normal(uint64_t seed, uint64_t step, int64_t task, uint32_t stream) {
    U4 r = philox(seed, step, task, stream);
    double u1 = 1.0 - u53(r.x, r.y);
    double u2 = u53(r.z, r.w);
    return sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}

// ----------------------------------------------------------------------------- selection
// numpy pairwise float32 sum (numpy/_core/src/umath/loops_utils.h.src pairwise_sum):
// sequential from 0 below 8 elements, 8 running partials + fixed tree above.
// Element k is produced by elem(k) (recomputed, never stored: no scratch arrays).
template <class Elem>
__device__ inline float np_pairwise_sum_f32(Elem elem, int n) {
    if (n < 8) {
        float res = 0.f;
        for (int i = 0; i < n; ++i) res += elem(i);
        return res;
    }
    float r0 = elem(0), r1 = elem(1), r2 = elem(2), r3 = elem(3);
    float r4 = elem(4), r5 = elem(5), r6 = elem(6), r7 = elem(7);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
        r0 += elem(i); r1 += elem(i + 1); r2 += elem(i + 2); r3 += elem(i + 3);
        r4 += elem(i + 4); r5 += elem(i + 5); r6 += elem(i + 6); r7 += elem(i + 7);
    }
    float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res += elem(i);
    return res;
}

// Reference action choice (ctrls/ctrl_bandit.py:435-443, ctrls/ctrl_darkroom.py:48-62):
// greedy = first argmax of the fp32 logits; sampling = scipy softmax (fp32:
// max-shift, exp, pairwise sum, divide) then numpy RandomState.choice(A, p)
// with its uniform u: cdf = cumsum(float64(p)); cdf /= cdf[-1];
// idx = searchsorted(cdf, u, 'right').  Every intermediate is recomputed
// bit-identically instead of stored, so no per-lane arrays are needed.
__device__ inline int select_from_logits(const float* logits, int A, int sample, float temp, double u) {
    if (!sample) {
        int best = 0;
        float bv = logits[0];
        for (int k = 1; k < A; ++k) {
            if (logits[k] > bv) { bv = logits[k]; best = k; }
        }
        return best;
    }
    auto xk = [&](int k) { return (temp == 1.0f) ? logits[k] : logits[k] / temp; };
    float m = -INFINITY;
    for (int k = 0; k < A; ++k) m = fmaxf(m, xk(k));
    auto ek = [&](int k) { return expf(xk(k) - m); };
    const float s = np_pairwise_sum_f32(ek, A);
    double total = 0.0;
    for (int k = 0; k < A; ++k) total += (double)(ek(k) / s);
    double c = 0.0;
    int idx = 0;
    for (int k = 0; k < A; ++k) {
        c += (double)(ek(k) / s);
        idx += (c / total <= u) ? 1 : 0;
    }
    return idx < A ? idx : A - 1;
}

// Fixed-A twin of select_from_logits: same arithmetic, every intermediate in
// registers (each exp and quotient computed once).
template <int NA>
__device__ inline int select_fixed(const float (&lg)[NA], int sample, float temp, double u) {
    if (!sample) {
        int best = 0;
        float bv = lg[0];
#pragma unroll
        for (int k = 1; k < NA; ++k)
            if (lg[k] > bv) { bv = lg[k]; best = k; }
        return best;
    }
    float xk[NA], ek[NA];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        xk[k] = (temp == 1.0f) ? lg[k] : lg[k] / temp;
        m = fmaxf(m, xk[k]);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) ek[k] = expf(xk[k] - m);
    const float s = np_pairwise_sum_f32([&](int k) { return ek[k]; }, NA);
    double total = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) total += (double)(ek[k] / s);
    double c = 0.0;
    int idx = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        c += (double)(ek[k] / s);
        idx += (c / total <= u) ? 1 : 0;
    }
    return idx < NA ? idx : NA - 1;
}

// select_fixed split at its cdf: q[k] = c_k / total (the values select_fixed
// compares with u), so a caller that meets the same logits again selects with
// select_from_cdf alone -- bit-identical to select_fixed on those logits.
template <int NA>
__device__ inline void cdf_fixed(const float (&lg)[NA], float temp, double (&q)[NA]) {
    float xk[NA], ek[NA];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        xk[k] = (temp == 1.0f) ? lg[k] : lg[k] / temp;
        m = fmaxf(m, xk[k]);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) ek[k] = expf(xk[k] - m);
    const float s = np_pairwise_sum_f32([&](int k) { return ek[k]; }, NA);
    double total = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) total += (double)(ek[k] / s);
    double c = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        c += (double)(ek[k] / s);
        q[k] = c / total;
    }
}

template <int NA>
__device__ inline int select_from_cdf(const double* q, double u) {
    int idx = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) idx += (q[k] <= u) ? 1 : 0;
    return idx < NA ? idx : NA - 1;
}

// The same selection with a fp32 fast path.  cdf_fast is the cdf in fp32 (q_k = prefix_k(e) /
// sum(e), e_k = 2^((x_k - m) log2 e) on v_exp_f32); it is within about 1e-6 (absolute) of
// cdf_fixed's fp64 values (the fp32 quotients and exponentials differ by a few ulp, and a term's
// weight e_k / sum(e) shrinks faster than its argument's rounding grows).  Where every
// |q_k - u| exceeds kCdfMargin = 2^-15 the comparisons q_k <= u therefore agree with cdf_fixed's,
// and select_fast returns select_from_cdf's index without the fp64 work; otherwise (about 5e-4 of
// the draws, NaN logits included) it runs cdf_fixed itself.  Bit-identical to select_fixed.
constexpr float kCdfMargin = 1.0f / 32768.0f;
template <int NA>
__device__ inline void cdf_fast(const float (&lg)[NA], float temp, float (&q)[NA]) {
    float xk[NA], e[NA];
    float m = -INFINITY;
    // temp is uniform: a real branch, so the IEEE divisions (a dozen instructions each, on the
    // tail's serial chain) run only when temp != 1 (the empty asm keeps the compiler from
    // computing both sides and selecting)
    if (temp == 1.0f) {
#pragma unroll
        for (int k = 0; k < NA; ++k) xk[k] = lg[k];
    } else {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < NA; ++k) xk[k] = lg[k] / temp;
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) m = fmaxf(m, xk[k]);
#pragma unroll
    for (int k = 0; k < NA; ++k) e[k] = __builtin_amdgcn_exp2f((xk[k] - m) * 1.4426950408889634f);
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < NA; ++k) tot += e[k];
    const float r = __builtin_amdgcn_rcpf(tot);
    float c = 0.f;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        c += e[k];
        q[k] = c * r;
    }
}
template <int NA>
__device__ inline int select_fast(const float* q, const float (&lg)[NA], float temp, double u) {
    const float uf = (float)u;
    int idx = 0;
    bool safe = true;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        idx += (q[k] <= uf) ? 1 : 0;
        safe = safe && __builtin_fabsf(q[k] - uf) > kCdfMargin;  // false for NaN
    }
    if (safe) return idx < NA ? idx : NA - 1;
    double qe[NA];
    cdf_fixed<NA>(lg, temp, qe);
    return select_from_cdf<NA>(qe, u);
}
// select_fixed through the fast path (bit-identical)
template <int NA>
__device__ inline int select_fixed_fast(const float (&lg)[NA], int sample, float temp, double u) {
    if (!sample) return select_fixed<NA>(lg, 0, temp, u);
    float q[NA];
    cdf_fast<NA>(lg, temp, q);
    return select_fast<NA>(q, lg, temp, u);
}

// Every block's attention folded (ModelView::l0, one L0Off block per layer,
// derived at model creation by derive_l0_kernel): with y = LN1(h), q.k_s =
// y_s . u + (terms constant over the keys s) for u = Wk q = y G + g0, and
// sum_s P_s v_s = (sum_s P_s y_s) Wv + bv.  Used by the bandit rollout
// (dpt_decode.hip) and the MFMA window forwards (dpt_mfma_fwd.h).  All
// matrices [in][out], E x E.
// Dimensions of the generic-width training forward / backward (dpt_train.hip): layers, width,
// token features, actions, sequences, tokens per sequence, wpe rows.
struct TrDims {
    int L, E, F, A, B, T, npos;
    int fwd_only;  // DPT_TRAIN_FORWARD_ONLY: inference workspace (nothing saved for a backward)
    // dropout (dpt_hip.h dpt_train_desc): element kept iff its Philox word >= drop_thr, then
    // scaled by drop_scale; drop_thr == 0: no dropout
    uint32_t drop_thr;
    float drop_scale;
    uint64_t drop_seed;
    __host__ __device__ bool drop() const { return drop_thr != 0; }
    __host__ __device__ int R() const { return B * T; }
    __host__ __device__ int64_t layer_size() const { return 12ll * E * E + 13ll * E; }
};

struct L0Off {
    static constexpr int G = 0;                 // Wq Wk^T: u = xn G + g0 = Wk q
    static constexpr int g0 = G + kE * kE;      // Wk bq
    static constexpr int Wvp = g0 + kE;         // Wv Wproj
    static constexpr int bvp = Wvp + kE * kE;   // bv Wproj + bproj
    static constexpr int size = bvp + kE;
};

// Tasks the K/V workspace is laid out for: N rounded up to whole tiles of the
// largest decode tile (16), so the bandit rollout's tile-interleaved y rows of a
// partial last tile stay inside their block's slot (dpt_kvcache_numel).
__host__ __device__ inline int kv_tasks(int N) { return (N + 15) & ~15; }

// ----------------------------------------------------------------------------- env arithmetic
// envs/bandit_env.py:59: means[a] + np.random.normal(0, var) == means[a] + (0.0 + var*g).
__device__ inline double gaussian_reward(double mean, double var, double g) {
    double noise = __dadd_rn(0.0, __dmul_rn(var, g));
    return __dadd_rn(mean, noise);
}

}  // namespace dpt
