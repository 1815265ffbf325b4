// Regret statistics of the online bandit eval on device (evals/eval_bandit.py:169-178:
// diff = opt - lnr per step, cumsum over steps, mean and scipy.stats.sem over tasks).
//
// Two passes, each one launch of regret_partials_kernel + one of regret_finish_kernel:
//   DPT_REGRET_SUMS     out[0][h] = sum_t diff[t][h],  out[1][h] = sum_t cr[t][h]
//   DPT_REGRET_CENTRED  out[0][h] = sum_t (diff[t][h] - mean[0][h])^2,
//                       out[1][h] = sum_t (cr[t][h] - mean[1][h])^2
// with cr[t][h] = sum_{h' <= h} diff[t][h'] (the caller all-reduces the sums over
// ranks, divides, and runs the centred pass: scipy's two-pass form).  Fixed reduction
// order (a block's 16 tasks in wave order, then the blocks in index order), so the
// result is deterministic.  fp64 like numpy; HBM-trivial (one read of
// the (N, H) curves per pass).
#include "dpt_common.h"

namespace dpt {

constexpr int kStatWaves = 16;      // one task per wave, 16 tasks per block
constexpr int kStatThreads = kStatWaves * kWave;
constexpr int kStatMaxChunks = 16;  // H <= 1024: 64 steps per chunk, one step per lane

// partial[b][k][h] over the block's 16 tasks.  Lanes are steps (64 per chunk, coalesced
// row reads); a task's cumsum is an inclusive shuffle scan per chunk plus the carry of
// the chunks before it; each lane keeps its steps' moments in registers, then the 16
// waves are combined through LDS chunk by chunk, in wave order.
__global__ void __launch_bounds__(kStatThreads) regret_partials_kernel(
    const double* __restrict__ arm_value, const double* __restrict__ opt, int N, int H, int mode,
    const double* __restrict__ mean, double* __restrict__ partial) {
    __shared__ double red[kStatWaves][2][kWave];
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int nch = (H + kWave - 1) / kWave;
    const int t = blockIdx.x * kStatWaves + wave;
    double ad[kStatMaxChunks], ac[kStatMaxChunks];
#pragma unroll
    for (int k = 0; k < kStatMaxChunks; ++k) ad[k] = ac[k] = 0.0;
    if (t < N) {
        const double o = opt[t];
        const double* row = arm_value + (size_t)t * H;
        double carry = 0.0;
#pragma unroll
        for (int k = 0; k < kStatMaxChunks; ++k) {
            if (k >= nch) continue;  // (no break: the loop must stay unrolled, ad/ac in registers)
            const int h = k * kWave + lane;
            const double d = h < H ? o - row[h] : 0.0;
            double s = d;  // inclusive scan over the chunk's lanes
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const double up = __shfl_up(s, off);
                if (lane >= off) s += up;
            }
            const double cr = carry + s;
            carry = __shfl(cr, kWave - 1);
            if (h < H) {
                if (mode == DPT_REGRET_CENTRED) {
                    const double e = d - mean[h], f = cr - mean[H + h];
                    ad[k] = e * e;
                    ac[k] = f * f;
                } else {
                    ad[k] = d;
                    ac[k] = cr;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kStatMaxChunks; ++k) {
        if (k >= nch) continue;
        red[wave][0][lane] = ad[k];
        red[wave][1][lane] = ac[k];
        __syncthreads();
        if (threadIdx.x < 2 * kWave) {  // waves in order
            const int q = threadIdx.x / kWave, h = k * kWave + lane;
            double s = 0.0;
#pragma unroll
            for (int w = 0; w < kStatWaves; ++w) s += red[w][q][lane];
            if (h < H) partial[((size_t)blockIdx.x * 2 + q) * H + h] = s;
        }
        __syncthreads();
    }
}

// out[k][h] = sum of the blocks' partials: block (k, 64 steps), wave q of kFinWaves takes the
// partials b = q (mod kFinWaves) in kFinAcc interleaved accumulators (loads in flight), then
// the accumulators and the waves are added in a fixed order
constexpr int kFinWaves = 16;
constexpr int kFinAcc = 4;
__global__ void __launch_bounds__(kFinWaves * kWave) regret_finish_kernel(const double* __restrict__ partial,
                                                                           int nb, int H, double* __restrict__ out) {
    __shared__ double red[kFinWaves][kWave];
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int k = blockIdx.y, h = blockIdx.x * kWave + lane;
    double acc[kFinAcc];
#pragma unroll
    for (int a = 0; a < kFinAcc; ++a) acc[a] = 0.0;
    if (h < H) {
        for (int b0 = wave; b0 < nb; b0 += kFinWaves * kFinAcc) {
#pragma unroll
            for (int a = 0; a < kFinAcc; ++a) {
                const int b = b0 + a * kFinWaves;
                if (b < nb) acc[a] += partial[((size_t)b * 2 + k) * H + h];
            }
        }
    }
    double s = 0.0;
#pragma unroll
    for (int a = 0; a < kFinAcc; ++a) s += acc[a];
    red[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && h < H) {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < kFinWaves; ++q) t += red[q][lane];
        out[(size_t)k * H + h] = t;
    }
}

int regret_max_steps() { return kStatMaxChunks * kWave; }

int64_t regret_workspace_numel(int N, int H) {
    return (int64_t)((N + kStatWaves - 1) / kStatWaves) * 2 * H;
}

int launch_regret_moments(const double* arm_value, const double* opt, int N, int H, int mode, const double* mean,
                          double* workspace, double* out, hipStream_t st) {
    const int nblk = (N + kStatWaves - 1) / kStatWaves;
    hipLaunchKernelGGL(regret_partials_kernel, dim3(nblk), dim3(kStatThreads), 0, st, arm_value, opt, N, H, mode,
                       mean, workspace);
    if (int rc = check_hip(hipGetLastError(), "regret_partials_kernel launch")) return rc;
    hipLaunchKernelGGL(regret_finish_kernel, dim3((H + kWave - 1) / kWave, 2), dim3(kFinWaves * kWave), 0, st,
                       workspace, nblk, H, out);
    return check_hip(hipGetLastError(), "regret_finish_kernel launch");
}

}  // namespace dpt
