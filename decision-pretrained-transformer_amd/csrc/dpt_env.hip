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
    double r;
    if (type == DPT_BANDIT_BERNOULLI) {
        const double u = noise ? noise[i] : philox_uniform(seed, counter, first_task + i, DPT_STREAM_REWARD);
        r = (u < mean) ? 1.0 : 0.0;
    } else {
        const double g = noise ? noise[i] : philox_normal(seed, counter, first_task + i, DPT_STREAM_REWARD);
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
                              int64_t first_task, int32_t* __restrict__ action) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double u = 0.0;
    if (sample) u = uniforms ? uniforms[i] : philox_uniform(seed, counter, first_task + i, DPT_STREAM_SELECT);
    action[i] = select_from_logits(logits + (size_t)i * A, A, sample, temp, u);
}

// Materialise the Philox draws the library uses (tests, data-generation replay).
__global__ void draw_kernel(int kind, uint64_t seed, uint64_t counter, int64_t first_task, int N,
                            uint32_t stream, double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    out[i] = kind == 0 ? philox_uniform(seed, counter, first_task + i, stream)
                       : philox_normal(seed, counter, first_task + i, stream);
}

static inline dim3 grid_for(int n) { return dim3((n + kEnvThreads - 1) / kEnvThreads); }

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

int launch_select(const float* logits, int N, int A, int sample, float temp, const double* uniforms,
                  uint64_t seed, uint64_t counter, int64_t first_task, int32_t* action, hipStream_t st) {
    hipLaunchKernelGGL(select_kernel, grid_for(N), dim3(kEnvThreads), 0, st, logits, N, A, sample, temp,
                       uniforms, seed, counter, first_task, action);
    return check_hip(hipGetLastError(), "select_kernel launch");
}

int launch_draw(int kind, uint64_t seed, uint64_t counter, int64_t first_task, int N, uint32_t stream,
                double* out, hipStream_t st) {
    hipLaunchKernelGGL(draw_kernel, grid_for(N), dim3(kEnvThreads), 0, st, kind, seed, counter, first_task, N,
                       stream, out);
    return check_hip(hipGetLastError(), "draw_kernel launch");
}

}  // namespace dpt
