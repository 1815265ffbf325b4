// Classical bandit baselines of the online/offline evaluation, fused with the
// env: ctrls/ctrl_bandit.py EmpMeanPolicy (:57-118), UCBPolicy (:318-380),
// ThompsonSamplingPolicy (:122-251), PessMeanPolicy (:255-314),
// LinUCBPolicy (:447-528) and OptPolicy (:22-38), each stepped inside
// evals/eval_bandit.py:56-103 deploy_online_vec.
//
// One lane per task runs all H steps.  The reference recomputes every
// per-arm statistic from the whole context each step with numpy (fp64,
// pairwise summation), so the per-arm reward lists are kept in a workspace laid
// out [arm][k][task] (lane-contiguous: coalesced) and summed with numpy's
// pairwise order each step: means, bounds and therefore action indices are
// bit-identical to the reference for the same draws (LinUCB excepted: its 2x2
// inverse is LAPACK's in the reference, closed-form here).
#include "dpt_common.h"

namespace dpt {

constexpr int kPolThreads = 128;

// numpy pairwise_sum for float64 over a strided sequence x[k*stride], k < n
// (loops_utils.h.src): blocks of <= 128 with 8 partials, recursive halving above.
__device__ double pw_block(const double* x, size_t stride, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += x[(size_t)i * stride];
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x[(size_t)j * stride];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += x[(size_t)(i + j) * stride];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x[(size_t)i * stride];
    return res;
}

__device__ double pw_sum(const double* x, size_t stride, int n) {
    // explicit recursion unrolled to depth 4 (n <= 2048)
    if (n <= 128) return pw_block(x, stride, n);
    int a = n / 2;
    a -= a % 8;
    auto lvl2 = [&](const double* y, int m) -> double {
        if (m <= 128) return pw_block(y, stride, m);
        int b = m / 2;
        b -= b % 8;
        auto lvl3 = [&](const double* z, int k) -> double {
            if (k <= 128) return pw_block(z, stride, k);
            int c = k / 2;
            c -= c % 8;
            auto lvl4 = [&](const double* w, int q) -> double {
                if (q <= 128) return pw_block(w, stride, q);
                int d = q / 2;
                d -= d % 8;
                return pw_block(w, stride, d) + pw_block(w + (size_t)d * stride, stride, q - d);
            };
            return lvl4(z, c) + lvl4(z + (size_t)c * stride, k - c);
        };
        return lvl3(y, b) + lvl3(y + (size_t)b * stride, m - b);
    };
    return lvl2(x, a) + lvl2(x + (size_t)a * stride, n - a);
}

constexpr int kMaxD = 8;  // LinUCB feature dimension (lin_d) supported

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
    double* lists;   // [A][H][N]
    int32_t* actions_out;
    double* rewards_out;
    double* arm_value_out;
};

__global__ __launch_bounds__(kPolThreads) void rollout_policy_kernel(PolicyParams P) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.N) return;
    const int A = P.A;
    const int64_t task = P.first_task + i;
    const double* mrow = P.means + (size_t)i * A;
    int cnt[kMaxA];
    for (int k = 0; k < A; ++k) cnt[k] = 0;
    // LinUCB running design: X^T X (d x d, d <= kMaxD, row-major) and X^T r
    double xtx[kMaxD * kMaxD], xtr[kMaxD];
    for (int k = 0; k < kMaxD * kMaxD; ++k) xtx[k] = 0.0;
    for (int k = 0; k < kMaxD; ++k) xtr[k] = 0.0;
    int opt = 0;
    for (int k = 1; k < A; ++k)
        if (mrow[k] > mrow[opt]) opt = k;
    const int L = P.C + P.H;                   // list capacity per arm
    const size_t lstride = (size_t)L * P.N;    // arm stride of the lists
    auto append = [&](int a, double r) {
        if (P.lists) P.lists[a * lstride + (size_t)cnt[a] * P.N + i] = r;
        ++cnt[a];
        if (P.policy == DPT_POLICY_LINUCB) {
            const double* x = P.arms + (size_t)a * P.d;
            for (int p = 0; p < P.d; ++p) {
                xtr[p] += x[p] * r;
                for (int q = 0; q < P.d; ++q) xtx[p * kMaxD + q] += x[p] * x[q];
            }
        }
    };
    for (int c = 0; c < P.C; ++c)  // prefix context (set_batch_numpy_vec), time order
        append(P.ctx_actions[(size_t)i * P.C + c], P.ctx_rewards[(size_t)i * P.C + c]);
    for (int h = 0; h < P.H; ++h) {
        int a = 0;
        if (P.policy == DPT_POLICY_OPT) {
            a = opt;
        } else if (P.policy == DPT_POLICY_LINUCB) {
            if (P.C + h == 0) {  // np.random.choice(np.arange(dim)) for an empty context
                const double u = P.policy_noise ? P.policy_noise[(size_t)i]
                                                : philox_uniform(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_POLICY);
                a = min((int)(u * A), A - 1);
            } else if (P.d <= 2) {  // closed-form 2 x 2 inverse
                const double c00 = 1.0 + xtx[0], c01 = xtx[1], c11 = 1.0 + xtx[kMaxD + 1];
                const double det = c00 * c11 - c01 * c01;
                const double i00 = c11 / det, i01 = -c01 / det, i11 = c00 / det;
                const double t0 = i00 * xtr[0] + i01 * xtr[1], t1 = i01 * xtr[0] + i11 * xtr[1];
                double best = -INFINITY;
                for (int k = 0; k < A; ++k) {
                    const double x0 = P.arms[k * P.d], x1 = P.d > 1 ? P.arms[k * P.d + 1] : 0.0;
                    const double q = x0 * (i00 * x0 + i01 * x1) + x1 * (i01 * x0 + i11 * x1);
                    const double v = (t0 * x0 + t1 * x1) + P.c * sqrt(q);
                    if (v > best) { best = v; a = k; }
                }
            } else {
                // cov_inv = inv(I + X^T X) by Gauss-Jordan (cov is symmetric positive definite, so no
                // pivoting), theta = cov_inv X^T r, value = theta . x + c sqrt(x cov_inv x)
                // (ctrls/ctrl_bandit.py:505-522; LAPACK's inverse rounds differently: equal up to
                // near-ties of the arm values)
                const int d = P.d;
                double m[kMaxD * kMaxD], inv[kMaxD * kMaxD];
                for (int p = 0; p < d; ++p)
                    for (int q = 0; q < d; ++q) {
                        m[p * kMaxD + q] = xtx[p * kMaxD + q] + (p == q ? 1.0 : 0.0);
                        inv[p * kMaxD + q] = p == q ? 1.0 : 0.0;
                    }
                for (int c = 0; c < d; ++c) {
                    const double piv = 1.0 / m[c * kMaxD + c];
                    for (int q = 0; q < d; ++q) {
                        m[c * kMaxD + q] *= piv;
                        inv[c * kMaxD + q] *= piv;
                    }
                    for (int p = 0; p < d; ++p) {
                        if (p == c) continue;
                        const double f = m[p * kMaxD + c];
                        for (int q = 0; q < d; ++q) {
                            m[p * kMaxD + q] -= f * m[c * kMaxD + q];
                            inv[p * kMaxD + q] -= f * inv[c * kMaxD + q];
                        }
                    }
                }
                double theta[kMaxD];
                for (int p = 0; p < d; ++p) {
                    double t = 0.0;
                    for (int q = 0; q < d; ++q) t += inv[p * kMaxD + q] * xtr[q];
                    theta[p] = t;
                }
                double best = -INFINITY;
                for (int k = 0; k < A; ++k) {
                    const double* x = P.arms + (size_t)k * d;
                    double tv = 0.0, qv = 0.0;
                    for (int p = 0; p < d; ++p) {
                        tv += theta[p] * x[p];
                        double s = 0.0;
                        for (int q = 0; q < d; ++q) s += inv[p * kMaxD + q] * x[q];
                        qv += x[p] * s;
                    }
                    const double v = tv + P.c * sqrt(qv);
                    if (v > best) { best = v; a = k; }
                }
            }
        } else {
            // per-arm sums over the context (numpy pairwise order, fp64)
            double bmean[kMaxA];
            for (int k = 0; k < A; ++k) {
                const double s = cnt[k] ? pw_sum(P.lists + k * lstride + i, P.N, cnt[k]) : 0.0;
                bmean[k] = (P.policy == DPT_POLICY_THOMPSON) ? (cnt[k] ? s / cnt[k] : 0.0) : s / fmax(1.0, (double)cnt[k]);
            }
            int amin = 0;
            for (int k = 1; k < A; ++k)
                if (cnt[k] < cnt[amin]) amin = k;
            if (P.policy == DPT_POLICY_THOMPSON) {
                const double variance = P.ts_std * P.ts_std, pv = P.ts_prior_var, pm = P.ts_prior_mean;
                double post_m[kMaxA], post_s[kMaxA];
                for (int k = 0; k < A; ++k) {
                    if (cnt[k] > 0) {  // update_posterior_all (ctrl_bandit.py:218-226)
                        const double n = (double)cnt[k];
                        const double w = variance / (variance + n * pv);
                        post_m[k] = w * pm + (1.0 - w) * bmean[k];
                        post_s[k] = sqrt(1.0 / (1.0 / pv + n / variance));
                    } else {
                        post_m[k] = pm;
                        post_s[k] = sqrt(pv);
                    }
                }
                if (P.sample) {  // values = normal(means, sqrt(variances)); argmax
                    double best = -INFINITY;
                    for (int k = 0; k < A; ++k) {
                        const double g = P.policy_noise ? P.policy_noise[((size_t)h * P.N + i) * A + k]
                                                        : philox_normal(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_POLICY + k);
                        const double v = post_m[k] + post_s[k] * g;
                        if (v > best) { best = v; a = k; }
                    }
                } else {  // 100 posterior draws, most frequent argmax (ctrl_bandit.py:238-244)
                    int freq[kMaxA];
                    for (int k = 0; k < A; ++k) freq[k] = 0;
                    for (int s = 0; s < 100; ++s) {
                        double best = -INFINITY;
                        int am = 0;
                        for (int k = 0; k < A; ++k) {
                            const double g = philox_normal(P.seed, ((uint64_t)P.step0 + h) * 128 + s, task, DPT_STREAM_POLICY + k);
                            const double v = post_m[k] + post_s[k] * g;
                            if (v > best) { best = v; am = k; }
                        }
                        ++freq[am];
                    }
                    for (int k = 1; k < A; ++k)
                        if (freq[k] > freq[a]) a = k;
                }
            } else {
                double best = -INFINITY;
                for (int k = 0; k < A; ++k) {
                    double v = bmean[k];
                    if (P.policy != DPT_POLICY_EMP) {  // UCB / LCB bonus c / max(1, sqrt(n))
                        const double bon = P.c / fmax(1.0, sqrt((double)cnt[k]));
                        v = (P.policy == DPT_POLICY_UCB) ? v + bon : v - bon;
                    }
                    if (v > best) { best = v; a = k; }
                }
                // EmpMean(online) and UCB play an unseen arm first (ctrl_bandit.py:107-110, :373-375)
                if ((P.policy == DPT_POLICY_UCB || (P.policy == DPT_POLICY_EMP && P.online)) && cnt[amin] == 0)
                    a = amin;
            }
        }
        // env step (BanditEnv.transit, envs/bandit_env.py:56-64)
        const double mean = mrow[a];
        double r;
        if (P.type == DPT_BANDIT_BERNOULLI) {
            const double ur = P.noise ? P.noise[(size_t)h * P.N + i] : philox_uniform(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_REWARD);
            r = (ur < mean) ? 1.0 : 0.0;
        } else {
            const double g = P.noise ? P.noise[(size_t)h * P.N + i] : philox_normal(P.seed, (uint64_t)P.step0 + h, task, DPT_STREAM_REWARD);
            r = gaussian_reward(mean, P.var, g);
        }
        append(a, r);
        P.actions_out[(size_t)i * P.H + h] = a;
        P.rewards_out[(size_t)i * P.H + h] = r;
        P.arm_value_out[(size_t)i * P.H + h] = mean;
    }
}

int launch_rollout_policy(const dpt_policy_rollout_args& a, hipStream_t st) {
    PolicyParams P;
    P.N = a.N; P.H = a.H; P.A = a.A; P.policy = a.policy; P.online = a.online; P.type = a.type;
    P.sample = a.sample; P.d = a.lin_d; P.C = a.C; P.step0 = a.step0; P.ctx_actions = a.ctx_actions; P.ctx_rewards = a.ctx_rewards;
    P.first_task = a.first_task; P.var = a.var; P.c = a.c;
    P.ts_std = a.ts_std; P.ts_prior_mean = a.ts_prior_mean; P.ts_prior_var = a.ts_prior_var; P.seed = a.seed;
    P.means = a.means; P.arms = a.arms; P.noise = a.noise; P.policy_noise = a.policy_noise; P.lists = a.workspace;
    P.actions_out = a.actions_out; P.rewards_out = a.rewards_out; P.arm_value_out = a.arm_value_out;
    hipLaunchKernelGGL(rollout_policy_kernel, dim3((a.N + kPolThreads - 1) / kPolThreads), dim3(kPolThreads), 0, st,
                       P);
    return check_hip(hipGetLastError(), "rollout_policy_kernel launch");
}

}  // namespace dpt
