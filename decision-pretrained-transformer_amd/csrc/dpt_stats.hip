// Regret statistics of the online bandit eval on device (evals/eval_bandit.py:169-178:
// diff = opt - lnr per step, cumsum over steps, mean and scipy.stats.sem over tasks).
//
// Two passes, each one launch of regret_partials_kernel + one of regret_finish_kernel:
//   DPT_REGRET_SUMS     out[0][h] = sum_t diff[t][h],  out[1][h] = sum_t cr[t][h]
//   DPT_REGRET_CENTRED  out[0][h] = sum_t (diff[t][h] - mean[0][h])^2,
//                       out[1][h] = sum_t (cr[t][h] - mean[1][h])^2
// with cr[t][h] = sum_{h' <= h} diff[t][h'] (the caller all-reduces the sums over
// ranks, divides, and runs the centred pass: scipy's two-pass form).  Fixed reduction
// order (each wave's 4 tasks in order, then the waves in index order), so the result
// is deterministic.  fp64 like numpy; HBM-trivial (one read of
// the (N, H) curves per pass).
#include "dpt_common.h"

namespace dpt {

constexpr int kStatThreads = 256;   // 4 waves
constexpr int kStatWaves = kStatThreads / kWave;
constexpr int kStatTasks = 16;      // tasks per block (4 per wave)
constexpr int kStatMaxChunks = 16;  // H <= 1024: 64 steps per chunk, one step per lane

// partial[w][k][h] over the tasks of wave w (4 per wave, consecutive).  Lanes are steps (64 per chunk, coalesced row
// reads); a task's cumsum is an inclusive shuffle scan per chunk plus the carry of the
// chunks before it; each lane accumulates its steps' moments in registers.
__global__ void __launch_bounds__(kStatThreads) regret_partials_kernel(
    const double* __restrict__ arm_value, const double* __restrict__ opt, int N, int H, int mode,
    const double* __restrict__ mean, double* __restrict__ partial) {
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int nch = (H + kWave - 1) / kWave;
    double ad[kStatMaxChunks], ac[kStatMaxChunks];
#pragma unroll
    for (int k = 0; k < kStatMaxChunks; ++k) ad[k] = ac[k] = 0.0;
    for (int i = 0; i < kStatTasks / kStatWaves; ++i) {
        const int t = (blockIdx.x * kStatWaves + wave) * (kStatTasks / kStatWaves) + i;
        if (t >= N) break;
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
                    ad[k] += e * e;
                    ac[k] += f * f;
                } else {
                    ad[k] += d;
                    ac[k] += cr;
                }
            }
        }
    }
    const size_t w = (size_t)blockIdx.x * kStatWaves + wave;
#pragma unroll
    for (int k = 0; k < kStatMaxChunks; ++k) {
        const int h = k * kWave + lane;
        if (k < nch && h < H) {
            partial[(w * 2 + 0) * H + h] = ad[k];
            partial[(w * 2 + 1) * H + h] = ac[k];
        }
    }
}

// out[k][h] = sum of the waves' partials: block (k, 64 steps), wave q of kFinWaves takes the
// partials w = q (mod kFinWaves) in kFinAcc interleaved accumulators (loads in flight), then
// the accumulators and the waves are added in a fixed order
constexpr int kFinWaves = 8;
constexpr int kFinAcc = 8;
__global__ void __launch_bounds__(kFinWaves * kWave) regret_finish_kernel(const double* __restrict__ partial,
                                                                           int nw, int H, double* __restrict__ out) {
    __shared__ double red[kFinWaves][kWave];
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int k = blockIdx.y, h = blockIdx.x * kWave + lane;
    double acc[kFinAcc];
#pragma unroll
    for (int a = 0; a < kFinAcc; ++a) acc[a] = 0.0;
    if (h < H) {
        for (int w0 = wave; w0 < nw; w0 += kFinWaves * kFinAcc) {
#pragma unroll
            for (int a = 0; a < kFinAcc; ++a) {
                const int w = w0 + a * kFinWaves;
                if (w < nw) acc[a] += partial[((size_t)w * 2 + k) * H + h];
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
    return (int64_t)((N + kStatTasks - 1) / kStatTasks) * kStatWaves * 2 * H;
}

int launch_regret_moments(const double* arm_value, const double* opt, int N, int H, int mode, const double* mean,
                          double* workspace, double* out, hipStream_t st) {
    const int nblk = (N + kStatTasks - 1) / kStatTasks;
    hipLaunchKernelGGL(regret_partials_kernel, dim3(nblk), dim3(kStatThreads), 0, st, arm_value, opt, N, H, mode,
                       mean, workspace);
    if (int rc = check_hip(hipGetLastError(), "regret_partials_kernel launch")) return rc;
    hipLaunchKernelGGL(regret_finish_kernel, dim3((H + kWave - 1) / kWave, 2), dim3(kFinWaves * kWave), 0, st,
                       workspace, nblk * kStatWaves, H, out);
    return check_hip(hipGetLastError(), "regret_finish_kernel launch");
}

}  // namespace dpt
