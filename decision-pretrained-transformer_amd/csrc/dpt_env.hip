// Environment transitions, action selection and RNG draw kernels (gfx950).
//
// All of these are HBM/latency-trivial element-wise kernels: one lane per task,
// 256-thread workgroups, coalesced per-task rows.  They exist for the per-step
// ABI (generic controllers / envs driven from Python); the bandit hot loop runs
// fused inside rollout_bandit_kernel (dpt_decode.hip).
#include "dpt_common.h"

namespace dpt {

constexpr int kEnvThreads = 256;

__global__ void bandit_step_kernel(const double* __restrict__ means, int N, int A,
                                   const int32_t* __restrict__ action, int type, double var,
                                   const double* __restrict__ noise, uint64_t seed, uint64_t counter,
                                   int64_t first_task, double* __restrict__ reward,
                                   double* __restrict__ arm_value) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int a = action[i];
    const double mean = means[(size_t)i * A + a];
    const bool f32 = (type & DPT_BANDIT_F32) != 0;
    double r;
    if ((type & ~DPT_BANDIT_F32) == DPT_BANDIT_BERNOULLI) {
        const double u = noise ? noise[i] : philox_uniform(seed, counter, first_task + i, DPT_STREAM_REWARD);
        r = (u < mean) ? 1.0 : 0.0;
    } else {
        const double g = noise ? noise[i] : philox_normal(seed, counter, first_task + i, DPT_STREAM_REWARD);
        if (f32)  // torch: mean_rewards + randn * var, all fp32 (gpu_bandit_env.py:58-59)
            r = (double)__fadd_rn((float)mean, __fmul_rn((float)g, (float)var));
        else
            r = gaussian_reward(mean, var, g);
    }
    reward[i] = r;
    if (arm_value) arm_value[i] = mean;
}

// envs/darkroom_env.py:37-55 (+ :100-103 permuted): argmax -> move -> clip -> goal test.
__global__ void darkroom_step_kernel(const int32_t* __restrict__ state, const int32_t* __restrict__ action,
                                     const int32_t* __restrict__ goal, const int32_t* __restrict__ perm,
                                     int N, int dim, int32_t* __restrict__ next_state,
                                     int32_t* __restrict__ reward) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    int a = action[i];
    if (perm) a = perm[(size_t)i * 5 + a];
    int x = state[2 * i], y = state[2 * i + 1];
    x += (a == 0) - (a == 1);
    y += (a == 2) - (a == 3);
    x = min(max(x, 0), dim - 1);
    y = min(max(y, 0), dim - 1);
    next_state[2 * i] = x;
    next_state[2 * i + 1] = y;
    reward[i] = (x == goal[2 * i] && y == goal[2 * i + 1]) ? 1 : 0;
}

// envs/darkroom_env.py:69-82 (+ :105-111: index of the expert action inside perm).
__global__ void darkroom_opt_kernel(const int32_t* __restrict__ state, const int32_t* __restrict__ goal,
                                    const int32_t* __restrict__ perm, int N, int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int x = state[2 * i], y = state[2 * i + 1], gx = goal[2 * i], gy = goal[2 * i + 1];
    int a = x < gx ? 0 : x > gx ? 1 : y < gy ? 2 : y > gy ? 3 : 4;
    if (perm) {
        int k = 0;
        while (k < 5 && perm[(size_t)i * 5 + k] != a) ++k;
        a = k;
    }
    out[i] = a;
}

__global__ void select_kernel(const float* __restrict__ logits, int N, int A, int sample, float temp,
                              const double* __restrict__ uniforms, uint64_t seed, uint64_t counter,
                              int64_t first_task, int fast_path, int32_t* __restrict__ action) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double u = 0.0;
    if (sample) u = uniforms ? uniforms[i] : philox_uniform(seed, counter, first_task + i, DPT_STREAM_SELECT);
    const float* lp = logits + (size_t)i * A;
    auto fast = [&](auto na) {
        constexpr int NA = decltype(na)::value;
        float lg[NA];
#pragma unroll
        for (int k = 0; k < NA; ++k) lg[k] = lp[k];
        return select_fixed_fast<NA>(lg, sample, temp, u);
    };
    if (fast_path && A == 5) action[i] = fast(std::integral_constant<int, 5>{});
    else if (fast_path && A == 20) action[i] = fast(std::integral_constant<int, 20>{});
    else action[i] = select_from_logits(lp, A, sample, temp, u);
}

// Materialise the Philox draws the library uses (tests, data-generation replay).
__global__ void draw_kernel(int kind, uint64_t seed, uint64_t counter, int64_t first_task, int N,
                            uint32_t stream, double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    out[i] = kind == 0 ? philox_uniform(seed, counter, first_task + i, stream)
                       : philox_normal(seed, counter, first_task + i, stream);
}

// collect_data.py:23-53 rollin_bandit, all tasks x steps in parallel: given each
// task's behaviour policy p (the Dirichlet/point-mass mixture, drawn on the host)
// step h draws i ~ choice(A, p) (numpy legacy cdf/searchsorted semantics) and
// r = means[i] + (0.0 + var*g).  One lane per (task, step); rows are (N, H).
__global__ void rollin_bandit_kernel(const double* __restrict__ means, const double* __restrict__ probs, int N, int A,
                                     int H, int type, double var, const double* __restrict__ uniforms,
                                     const double* __restrict__ noise, uint64_t seed, int64_t first_task,
                                     int32_t* __restrict__ actions, double* __restrict__ rewards) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)N * H) return;
    const int i = (int)(gid / H), h = (int)(gid % H);
    const int64_t task = first_task + i;
    const double u = uniforms ? uniforms[(size_t)h * N + i] : philox_uniform(seed, h, task, DPT_STREAM_ROLLIN);
    const double* p = probs + (size_t)i * A;
    double total = 0.0;
    for (int k = 0; k < A; ++k) total += p[k];
    double c = 0.0;
    int a = 0;
    for (int k = 0; k < A; ++k) {
        c += p[k];
        a += (c / total <= u) ? 1 : 0;
    }
    a = a < A ? a : A - 1;
    const double mean = means[(size_t)i * A + a];
    double r;
    if (type == DPT_BANDIT_BERNOULLI) {
        const double ur = noise ? noise[(size_t)h * N + i] : philox_uniform(seed, h, task, DPT_STREAM_REWARD);
        r = (ur < mean) ? 1.0 : 0.0;
    } else {
        const double g = noise ? noise[(size_t)h * N + i] : philox_normal(seed, h, task, DPT_STREAM_REWARD);
        r = gaussian_reward(mean, var, g);
    }
    actions[gid] = a;
    rewards[gid] = r;
}

__device__ inline int philox_randint(uint64_t seed, uint64_t step, int64_t task, uint32_t stream, int word, int n) {
    U4 r = philox(seed, step, task, stream);
    const uint32_t w = word == 0 ? r.x : word == 1 ? r.y : word == 2 ? r.z : r.w;
    return (int)(((uint64_t)w * (uint64_t)n) >> 32);  // multiply-shift, bias < n / 2^32
}

__device__ inline void darkroom_move(int& x, int& y, int a, int dim) {
    x += (a == 0) - (a == 1);
    y += (a == 2) - (a == 3);
    x = min(max(x, 0), dim - 1);
    y = min(max(y, 0), dim - 1);
}

__device__ inline int darkroom_opt(int x, int y, int gx, int gy, const int32_t* perm) {
    int a = x < gx ? 0 : x > gx ? 1 : y < gy ? 2 : y > gy ? 3 : 4;
    if (perm) {
        int k = 0;
        while (k < 5 && perm[k] != a) ++k;
        a = k;
    }
    return a;
}

// collect_data.py:83-111 rollin_mdp + generate_mdp_histories_from_envs (:189-218).
// mode 0 ('uniform'): each step draws s ~ U{0..dim-1}^2, a ~ U{0..4} i.i.d.
// (one lane per (task, step)); mode 1 ('expert'): the expert walk from (0, 0)
// (one lane per task, sequential).  Injected states/actions (mode 0) replay a
// reference run.  Query state ~ U and its expert label are written per task.
__global__ void rollin_darkroom_kernel(const int32_t* __restrict__ goal, const int32_t* __restrict__ perm, int N, int H,
                                       int dim, int mode, const int32_t* __restrict__ states_in,
                                       const int32_t* __restrict__ actions_in, uint64_t seed, int64_t first_task,
                                       int32_t* __restrict__ states, int32_t* __restrict__ actions,
                                       int32_t* __restrict__ next_states, int32_t* __restrict__ rewards,
                                       int32_t* __restrict__ query, int32_t* __restrict__ opt_action) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = mode == 0 ? (int64_t)N * H : N;
    if (gid >= total) return;
    const int i = mode == 0 ? (int)(gid / H) : (int)gid;
    const int64_t task = first_task + i;
    const int gx = goal[2 * i], gy = goal[2 * i + 1];
    const int32_t* pm = perm ? perm + (size_t)i * 5 : nullptr;
    auto emit = [&](int h, int x, int y, int a) {
        const size_t o = (size_t)i * H + h;
        states[2 * o] = x;
        states[2 * o + 1] = y;
        actions[o] = a;
        const int ea = pm ? pm[a] : a;
        darkroom_move(x, y, ea, dim);
        next_states[2 * o] = x;
        next_states[2 * o + 1] = y;
        rewards[o] = (x == gx && y == gy) ? 1 : 0;
    };
    if (mode == 0) {
        const int h = (int)(gid % H);
        int x, y, a;
        if (states_in) {
            const size_t o = (size_t)i * H + h;
            x = states_in[2 * o];
            y = states_in[2 * o + 1];
            a = actions_in[o];
        } else {
            x = philox_randint(seed, h, task, DPT_STREAM_ROLLIN, 0, dim);
            y = philox_randint(seed, h, task, DPT_STREAM_ROLLIN, 1, dim);
            a = philox_randint(seed, h, task, DPT_STREAM_ROLLIN, 2, 5);
        }
        emit(h, x, y, a);
    } else {
        int x = 0, y = 0;
        for (int h = 0; h < H; ++h) {
            const int a = darkroom_opt(x, y, gx, gy, pm);
            emit(h, x, y, a);
            const int ea = pm ? pm[a] : a;
            darkroom_move(x, y, ea, dim);
        }
    }
    const bool lead = mode == 0 ? (gid % H == 0) : true;
    if (lead && query) {
        const int qx = philox_randint(seed, H, task, DPT_STREAM_ROLLIN, 0, dim);
        const int qy = philox_randint(seed, H, task, DPT_STREAM_ROLLIN, 1, dim);
        query[2 * i] = qx;
        query[2 * i + 1] = qy;
        if (opt_action) opt_action[i] = darkroom_opt(qx, qy, gx, gy, pm);
    }
}

static inline dim3 grid_for(int n) { return dim3((n + kEnvThreads - 1) / kEnvThreads); }
static inline dim3 grid_for64(int64_t n) { return dim3((unsigned)((n + kEnvThreads - 1) / kEnvThreads)); }

int launch_rollin_bandit(const double* means, const double* probs, int N, int A, int H, int type, double var,
                         const double* uniforms, const double* noise, uint64_t seed, int64_t first_task,
                         int32_t* actions, double* rewards, hipStream_t st) {
    hipLaunchKernelGGL(rollin_bandit_kernel, grid_for64((int64_t)N * H), dim3(kEnvThreads), 0, st, means, probs, N, A,
                       H, type, var, uniforms, noise, seed, first_task, actions, rewards);
    return check_hip(hipGetLastError(), "rollin_bandit_kernel launch");
}

int launch_rollin_darkroom(const int32_t* goal, const int32_t* perm, int N, int H, int dim, int mode,
                           const int32_t* states_in, const int32_t* actions_in, uint64_t seed, int64_t first_task,
                           int32_t* states, int32_t* actions, int32_t* next_states, int32_t* rewards, int32_t* query,
                           int32_t* opt_action, hipStream_t st) {
    const int64_t total = mode == 0 ? (int64_t)N * H : N;
    hipLaunchKernelGGL(rollin_darkroom_kernel, grid_for64(total), dim3(kEnvThreads), 0, st, goal, perm, N, H, dim,
                       mode, states_in, actions_in, seed, first_task, states, actions, next_states, rewards, query,
                       opt_action);
    return check_hip(hipGetLastError(), "rollin_darkroom_kernel launch");
}

int launch_bandit_step(const double* means, int N, int A, const int32_t* action, int type, double var,
                       const double* noise, uint64_t seed, uint64_t counter, int64_t first_task,
                       double* reward, double* arm_value, hipStream_t st) {
    hipLaunchKernelGGL(bandit_step_kernel, grid_for(N), dim3(kEnvThreads), 0, st, means, N, A, action, type,
                       var, noise, seed, counter, first_task, reward, arm_value);
    return check_hip(hipGetLastError(), "bandit_step_kernel launch");
}

int launch_darkroom_step(const int32_t* state, const int32_t* action, const int32_t* goal, const int32_t* perm,
                         int N, int dim, int32_t* next_state, int32_t* reward, hipStream_t st) {
    hipLaunchKernelGGL(darkroom_step_kernel, grid_for(N), dim3(kEnvThreads), 0, st, state, action, goal, perm, N,
                       dim, next_state, reward);
    return check_hip(hipGetLastError(), "darkroom_step_kernel launch");
}

int launch_darkroom_opt(const int32_t* state, const int32_t* goal, const int32_t* perm, int N, int32_t* out,
                        hipStream_t st) {
    hipLaunchKernelGGL(darkroom_opt_kernel, grid_for(N), dim3(kEnvThreads), 0, st, state, goal, perm, N, out);
    return check_hip(hipGetLastError(), "darkroom_opt_kernel launch");
}

static bool g_select_fast = true;  // DPT_TUNE_SELECT_FAST

int set_select_fast(int on) {
    if (on != 0 && on != 1) return DPT_EINVAL;
    g_select_fast = on == 1;
    return DPT_OK;
}

int launch_select(const float* logits, int N, int A, int sample, float temp, const double* uniforms,
                  uint64_t seed, uint64_t counter, int64_t first_task, int32_t* action, hipStream_t st) {
    hipLaunchKernelGGL(select_kernel, grid_for(N), dim3(kEnvThreads), 0, st, logits, N, A, sample, temp,
                       uniforms, seed, counter, first_task, g_select_fast ? 1 : 0, action);
    return check_hip(hipGetLastError(), "select_kernel launch");
}

int launch_draw(int kind, uint64_t seed, uint64_t counter, int64_t first_task, int N, uint32_t stream,
                double* out, hipStream_t st) {
    hipLaunchKernelGGL(draw_kernel, grid_for(N), dim3(kEnvThreads), 0, st, kind, seed, counter, first_task, N,
                       stream, out);
    return check_hip(hipGetLastError(), "draw_kernel launch");
}

}  // namespace dpt
