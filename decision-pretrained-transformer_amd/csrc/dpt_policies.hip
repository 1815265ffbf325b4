// Classical bandit baselines of the online/offline evaluation, fused with the
// env: ctrls/ctrl_bandit.py EmpMeanPolicy (:57-118), UCBPolicy (:318-380),
// ThompsonSamplingPolicy (:122-251), PessMeanPolicy (:255-314),
// LinUCBPolicy (:447-528) and OptPolicy (:22-38), each stepped inside
// evals/eval_bandit.py:56-103 deploy_online_vec.
//
// One 64-lane workgroup per task runs all H steps with the task's context in LDS.
// The reference recomputes every per-arm statistic from the whole context each
// step with numpy (fp64, pairwise summation); the kernel sums the per-arm reward
// lists in numpy's pairwise order each step, so means, bounds and therefore action
// indices are bit-identical to the reference for the same draws (LinUCB: the BLAS
// orders of dpt_linucb.h).
#include "dpt_common.h"
#include "dpt_linucb.h"

namespace dpt {

struct PolicyParams {
    int N, H, A, policy, online, type, sample, d, C, step0;
    const int32_t* ctx_actions;
    const double* ctx_rewards;
    int64_t first_task;
    double var, c, ts_std, ts_prior_mean, ts_prior_var;
    uint64_t seed;
    const double* means;
    const double* arms;
    const double* noise;
    const double* policy_noise;
    int32_t* actions_out;
    double* rewards_out;
    double* arm_value_out;
};

// ----------------------------------------------------------------------------- wave per task
// Each task gets a 64-lane workgroup and keeps its whole context in LDS (C + H <= 2048, so at most
// ~36 KB at kMaxA arms):
//  * per-arm sums: 8 lanes per arm (8 arms at a time), lane c runs numpy's pairwise chain c of
//    every 128-element leaf (r[c] += x[8t + c]); the 8 chains combine by a xor 1 / 2 / 4
//    butterfly, which is exactly ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)); the tail and
//    the recursive halving above 128 follow pairwise_sum, so every sum is bit-identical to
//    numpy's (loops_utils.h.src pairwise_sum);
//  * the lists are 8-element chunks of one pool, in arrival order (element j of arm a sits at
//    pool[tab[a][j / 8] * 8 + j % 8]): sum_a ceil(cnt_a / 8) <= cap / 8 + A chunks, instead of A
//    lists of full capacity;
//  * LinUCB: X^T X entries on d(d+1)/2 lanes, ci . x of every arm on d * A lanes (the per-k
//    factor m(k) of theta's dgemv_t depends on the arm index alone), theta's rows on d lanes,
//    the arm values on A lanes, all in the BLAS orders of dpt_linucb.h;
//  * selection, the env step and the appends on lane 0, which owns the step's outputs.
// Round 6 retired the round-4 lane-per-task kernel (one lane per task, lists in a global
// workspace): it only served contexts too large for LDS, which the C + H <= 2048 bound of the
// pairwise depth never produces.
constexpr int kPwLeaf = 128;  // numpy PW_BLOCKSIZE

struct WaveLds {
    // byte offsets into the dynamic LDS block of one task
    int pool, vals, pm, ps, mrow, arms, mv, cov, ci, theta, r, tab, cnt, freq, act, total;
    int cap8;
    __host__ __device__ static WaveLds make(int A, int cap, bool lin, int d) {
        WaveLds w{};
        const int cap8 = (cap + 7) / 8;
        w.cap8 = cap8;
        int o = 0;
        auto take = [&](int bytes) {
            const int at = o;
            o += (bytes + 15) & ~15;
            return at;
        };
        w.pool = lin ? 0 : take((cap8 + A) * 8 * 8);
        w.vals = take(kMaxA * 8);
        w.pm = take(kMaxA * 8);
        w.ps = take(kMaxA * 8);
        w.mrow = take(kMaxA * 8);
        w.arms = lin ? take(A * d * 8) : 0;
        w.mv = lin ? take(d * A * 8) : 0;
        w.cov = lin ? take(kMaxD * kMaxD * 8) : 0;
        w.ci = lin ? take(kMaxD * kMaxD * 8) : 0;
        w.theta = lin ? take(kMaxD * 8) : 0;
        w.r = lin ? take(cap * 8) : 0;
        w.tab = lin ? 0 : take(A * cap8 * 2);
        w.cnt = take(kMaxA * 4);
        w.freq = take(kMaxA * 4);
        w.act = lin ? take(cap) : 0;
        w.total = o;
        return w;
    }
};

// numpy pairwise_sum leaf [s, s + m) of arm a (s a multiple of 8), by the 8 lanes of a group:
// lane c holds chain c; every lane returns the leaf's sum
__device__ inline double pw_leaf8(const double* pool, const uint16_t* tab, int s, int m, int c) {
    auto at = [&](int j) { return pool[(int)tab[j >> 3] * 8 + (j & 7)]; };
    if (m < 8) {
        double res = 0.0;
        for (int i = 0; i < m; ++i) res += at(s + i);
        return res;
    }
    const int g = m >> 3;
    const uint16_t* tb = tab + (s >> 3);
    double r = pool[(int)tb[0] * 8 + c];
    for (int t = 1; t < g; ++t) r += pool[(int)tb[t] * 8 + c];
    // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) on every lane (fp addition is commutative)
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    for (int i = 8 * g; i < m; ++i) r += at(s + i);
    return r;
}

// pairwise_sum over [s, s + n): leaves of <= 128, halving at multiples of 8 (D levels: n < 128 * 2^D)
template <int D>
__device__ double pw_group(const double* pool, const uint16_t* tab, int s, int n, int c) {
    if constexpr (D == 0) {
        return pw_leaf8(pool, tab, s, n, c);
    } else {
        if (n <= kPwLeaf) return pw_leaf8(pool, tab, s, n, c);
        int h = n / 2;
        h -= h % 8;
        const double lo = pw_group<D - 1>(pool, tab, s, h, c);
        const double hi = pw_group<D - 1>(pool, tab, s + h, n - h, c);
        return lo + hi;
    }
}

template <bool LIN>
__global__ __launch_bounds__(64) void rollout_policy_wave_kernel(PolicyParams P) {
    extern __shared__ double wave_lds[];
    char* base = reinterpret_cast<char*>(wave_lds);
    const int A = P.A, d = P.d, cap = P.C + P.H;
    const WaveLds W = WaveLds::make(A, cap, LIN, d);
    double* vals = reinterpret_cast<double*>(base + W.vals);
    double* pm_s = reinterpret_cast<double*>(base + W.pm);
    double* ps_s = reinterpret_cast<double*>(base + W.ps);
    double* mrow = reinterpret_cast<double*>(base + W.mrow);
    int* cnt = reinterpret_cast<int*>(base + W.cnt);
    int* freq = reinterpret_cast<int*>(base + W.freq);
    double* pool = reinterpret_cast<double*>(base + W.pool);
    uint16_t* tab = reinterpret_cast<uint16_t*>(base + W.tab);
    double* arms = reinterpret_cast<double*>(base + W.arms);
    double* mv = reinterpret_cast<double*>(base + W.mv);
    double* cov = reinterpret_cast<double*>(base + W.cov);
    double* ci = reinterpret_cast<double*>(base + W.ci);
    double* theta = reinterpret_cast<double*>(base + W.theta);
    double* lr = reinterpret_cast<double*>(base + W.r);
    uint8_t* lact = reinterpret_cast<uint8_t*>(base + W.act);

    const int i = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t task = P.first_task + i;
    const int cap8 = W.cap8;
    for (int k = lane; k < A; k += 64) {
        mrow[k] = P.means[(size_t)i * A + k];
        cnt[k] = 0;
    }
    if constexpr (LIN)
        for (int t = lane; t < A * d; t += 64) arms[t] = P.arms[t];
    __syncthreads();
    int opt = 0;  // lane 0's copies: the optimal arm and the pool's next free chunk
    int nchunk = 0;
    if (lane == 0)
        for (int k = 1; k < A; ++k)
            if (mrow[k] > mrow[opt]) opt = k;
    // lane 0: one transition into the context (time order)
    auto append = [&](int a, double r, int n) {
        if constexpr (LIN) {
            lr[n] = r;
            lact[n] = (uint8_t)a;
        } else {
            const int k = cnt[a];
            uint16_t* ta = tab + a * cap8;
            if ((k & 7) == 0) ta[k >> 3] = (uint16_t)nchunk++;
            pool[(int)ta[k >> 3] * 8 + (k & 7)] = r;
        }
        cnt[a] += 1;
    };
    if (lane == 0)
        for (int c = 0; c < P.C; ++c)  // prefix context (set_batch_numpy_vec), time order
            append(P.ctx_actions[(size_t)i * P.C + c], P.ctx_rewards[(size_t)i * P.C + c], c);
    __syncthreads();
    const int grp = lane >> 3, c8 = lane & 7;
    for (int h = 0; h < P.H; ++h) {
        const int n = P.C + h;  // context length
        int a = 0;
        if constexpr (LIN) {
            if (n > 0) {
                // cov = I + X^T X: entry e = (p, q), p <= q, on lane e (dsyrk order, linucb_choose)
                const int ne = d * (d + 1) / 2;
                if (lane < ne) {
                    int p = 0, e = lane;
                    while (e >= d - p) {
                        e -= d - p;
                        ++p;
                    }
                    const int q = p + e;
                    double cv = 0.0;
                    for (int ls = 0; ls < n;) {
                        const int ml = syrk_block(ls, n);
                        double acc = 0.0;
                        int k = ls;
                        for (; k + 8 <= ls + ml; k += 8) {
                            double xp[8], xq[8];
#pragma unroll
                            for (int t = 0; t < 8; ++t) {
                                const int ak = lact[k + t];
                                xp[t] = arms[ak * d + p];
                                xq[t] = arms[ak * d + q];
                            }
#pragma unroll
                            for (int t = 0; t < 8; ++t) acc = fma(xp[t], xq[t], acc);
                        }
                        for (; k < ls + ml; ++k) {
                            const int ak = lact[k];
                            acc = fma(arms[ak * d + p], arms[ak * d + q], acc);
                        }
                        cv = cv + acc;
                        ls += ml;
                    }
                    cov[p * kMaxD + q] = p == q ? 1.0 + cv : 0.0 + cv;
                    if (p != q) cov[q * kMaxD + p] = 0.0 + cv;
                }
                __syncthreads();
                if (lane == 0) {  // np.linalg.inv (linucb_inverse): the LU in place in cov (no longer
                    // needed), pivots and the solve vector in LDS words LinUCB does not use otherwise
                    // (no private arrays: no scratch)
                    linucb_inverse(cov, freq, pm_s, ci, d);
                }
                __syncthreads();
                // m_p(arm) = ci[p] . x_arm (the dgemm entry of cov_inv @ X^T for a row of that arm)
                for (int t = lane; t < d * A; t += 64) {
                    const int p = t / A, k = t - p * A;
                    mv[t] = linucb_m(ci + p * kMaxD, arms + k * d, d, n, p);
                }
                __syncthreads();
                if (lane < d) {  // theta[p] = (cov_inv @ X^T)[p] @ r  (dgemv_t order)
                    const double* mp = mv + lane * A;
                    theta[lane] = gemv_t_sum([&](int k) { return mp[lact[k]]; }, [&](int k) { return lr[k]; }, n,
                                             gemv_t_cols(lane, d));
                }
                __syncthreads();
                for (int k = lane; k < A; k += 64) {
                    const double* x = arms + k * d;
                    double tv = theta[0] * x[0];
                    for (int p = 1; p < d; ++p) tv = fma(theta[p], x[p], tv);
                    double qv = 0.0;
                    for (int j = 0; j < d; ++j) {
                        const double w = linucb_w(ci, x, d, j);
                        qv = j == 0 ? w * x[0] : fma(w, x[j], qv);
                    }
                    vals[k] = tv + P.c * sqrt(qv);
                }
                __syncthreads();
            }
            if (lane == 0) {
                if (n == 0) {  // np.random.choice(np.arange(dim)) for an empty context
                    const double u = P.policy_noise ? P.policy_noise[(size_t)i]
                                                    : philox_uniform(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_POLICY);
                    a = min((int)(u * A), A - 1);
                } else {
                    double best = -INFINITY;
                    for (int k = 0; k < A; ++k)
                        if (vals[k] > best) {
                            best = vals[k];
                            a = k;
                        }
                }
            }
        } else if (P.policy != DPT_POLICY_OPT) {
            const bool ts = P.policy == DPT_POLICY_THOMPSON;
            // per-arm sums, 8 arms at a time (lanes of a group share the arm's control flow)
            for (int a0 = 0; a0 < A; a0 += 8) {
                const int k = a0 + grp;
                if (k < A) {
                    const int nk = cnt[k];
                    const double s = nk ? pw_group<5>(pool, tab + k * cap8, 0, nk, c8) : 0.0;
                    if (c8 == 0) {
                        const double bmean = ts ? (nk ? s / nk : 0.0) : s / fmax(1.0, (double)nk);
                        if (ts) {
                            const double variance = P.ts_std * P.ts_std, pv = P.ts_prior_var, pmu = P.ts_prior_mean;
                            double m_, s_;
                            if (nk > 0) {  // update_posterior_all (ctrl_bandit.py:218-226)
                                const double nn = (double)nk;
                                const double w = variance / (variance + nn * pv);
                                m_ = w * pmu + (1.0 - w) * bmean;
                                s_ = sqrt(1.0 / (1.0 / pv + nn / variance));
                            } else {
                                m_ = pmu;
                                s_ = sqrt(pv);
                            }
                            pm_s[k] = m_;
                            ps_s[k] = s_;
                            if (P.sample) {
                                const double g = P.policy_noise ? P.policy_noise[((size_t)h * P.N + i) * A + k]
                                                                : philox_normal(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_POLICY + k);
                                vals[k] = m_ + s_ * g;
                            }
                        } else {
                            double v = bmean;
                            if (P.policy != DPT_POLICY_EMP) {  // UCB / LCB bonus c / max(1, sqrt(n))
                                const double bon = P.c / fmax(1.0, sqrt((double)nk));
                                v = (P.policy == DPT_POLICY_UCB) ? v + bon : v - bon;
                            }
                            vals[k] = v;
                        }
                    }
                }
            }
            if (ts && !P.sample) {  // 100 posterior draws, most frequent argmax (ctrl_bandit.py:238-244)
                for (int k = lane; k < A; k += 64) freq[k] = 0;
                __syncthreads();
                for (int s = lane; s < 100; s += 64) {
                    double best = -INFINITY;
                    int am = 0;
                    for (int k = 0; k < A; ++k) {
                        const double g = P.policy_noise ? P.policy_noise[(((size_t)h * 100 + s) * P.N + i) * A + k]
                                                        : philox_normal(P.seed, ((uint64_t)P.step0 + h) * 128 + s, task,
                                                                        DPT_STREAM_POLICY + k);
                        const double v = pm_s[k] + ps_s[k] * g;
                        if (v > best) {
                            best = v;
                            am = k;
                        }
                    }
                    atomicAdd(&freq[am], 1);
                }
            }
            __syncthreads();
            if (lane == 0) {
                if (ts && !P.sample) {
                    for (int k = 1; k < A; ++k)
                        if (freq[k] > freq[a]) a = k;
                } else {
                    double best = -INFINITY;
                    for (int k = 0; k < A; ++k)
                        if (vals[k] > best) {
                            best = vals[k];
                            a = k;
                        }
                    int amin = 0;
                    for (int k = 1; k < A; ++k)
                        if (cnt[k] < cnt[amin]) amin = k;
                    // EmpMean(online) and UCB play an unseen arm first (ctrl_bandit.py:107-110, :373-375)
                    if (!ts && (P.policy == DPT_POLICY_UCB || (P.policy == DPT_POLICY_EMP && P.online)) && cnt[amin] == 0)
                        a = amin;
                }
            }
        } else {
            a = opt;
        }
        if (lane == 0) {
            // env step (BanditEnv.transit, envs/bandit_env.py:56-64)
            const double mean = mrow[a];
            double r;
            if (P.type == DPT_BANDIT_BERNOULLI) {
                const double ur = P.noise ? P.noise[(size_t)h * P.N + i]
                                          : philox_uniform(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_REWARD);
                r = (ur < mean) ? 1.0 : 0.0;
            } else {
                const double g = P.noise ? P.noise[(size_t)h * P.N + i]
                                         : philox_normal(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_REWARD);
                r = gaussian_reward(mean, P.var, g);
            }
            append(a, r, n);
            P.actions_out[(size_t)i * P.H + h] = a;
            P.rewards_out[(size_t)i * P.H + h] = r;
            P.arm_value_out[(size_t)i * P.H + h] = mean;
        }
        __syncthreads();
    }
}

int set_policy_wave(int on) {
    // DPT_TUNE_POLICY_WAVE: 1 is the only kernel (the lane-per-task form was retired in round 6)
    if (on != 1) return DPT_EUNSUPPORTED;
    return DPT_OK;
}

int launch_rollout_policy(const dpt_policy_rollout_args& a, hipStream_t st) {
    PolicyParams P;
    P.N = a.N; P.H = a.H; P.A = a.A; P.policy = a.policy; P.online = a.online; P.type = a.type;
    P.sample = a.sample; P.d = a.lin_d; P.C = a.C; P.step0 = a.step0; P.ctx_actions = a.ctx_actions; P.ctx_rewards = a.ctx_rewards;
    P.first_task = a.first_task; P.var = a.var; P.c = a.c;
    P.ts_std = a.ts_std; P.ts_prior_mean = a.ts_prior_mean; P.ts_prior_var = a.ts_prior_var; P.seed = a.seed;
    P.means = a.means; P.arms = a.arms; P.noise = a.noise; P.policy_noise = a.policy_noise;
    P.actions_out = a.actions_out; P.rewards_out = a.rewards_out; P.arm_value_out = a.arm_value_out;
    const bool lin = a.policy == DPT_POLICY_LINUCB;
    const size_t lds = (size_t)WaveLds::make(a.A, a.C + a.H, lin, a.lin_d).total;
    if (lds > 160 * 1024) {  // unreachable under dpt_rollout_policy's C + H <= 2048, A <= kMaxA
        set_error(DPT_EUNSUPPORTED, "policy context of %d steps x %d arms needs %zu B of LDS", a.C + a.H, a.A, lds);
        return DPT_EUNSUPPORTED;
    }
    const void* kern = lin ? reinterpret_cast<const void*>(rollout_policy_wave_kernel<true>)
                           : reinterpret_cast<const void*>(rollout_policy_wave_kernel<false>);
    if (lds > 64 * 1024) (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (lin)
        hipLaunchKernelGGL(rollout_policy_wave_kernel<true>, dim3(a.N), dim3(64), lds, st, P);
    else
        hipLaunchKernelGGL(rollout_policy_wave_kernel<false>, dim3(a.N), dim3(64), lds, st, P);
    return check_hip(hipGetLastError(), "rollout_policy_wave_kernel launch");
}

}  // namespace dpt
