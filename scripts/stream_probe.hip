// Streaming probe for the bandit rollout's read pattern (no compute): per step h and per
// block 1..3, every wave reads its task's cached y rows of positions < h exactly as
// attend_one<KV_SAME> does (lane (g, c): position base + 8 r + g, dims 4c..4c+3, 8 rows in
// flight, tile-interleaved [tile][position][task][32]), the first `pin` positions with the
// default cache policy and the rest non-temporal.  Measures the rate the rollout's stream can
// reach on this layout without its dense phases.  Built by scripts/stream_probe.py.
#include <hip/hip_runtime.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int R, bool SYNC, bool NT>
__device__ void probe(const float* __restrict__ y, int N, int H, int pin, int nblk, float* __restrict__ out) {
    const int tile0 = blockIdx.x * 8, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 3, c = lane & 7;
    const size_t lstride = (size_t)N * H * 32;
    float acc = 0.f;
    for (int h = 1; h < H; ++h) {
        for (int l = 0; l < nblk; ++l) {
            const float* yc = y + l * lstride + (size_t)tile0 * H * 32 + wave * 32;
            for (int base = 0; base < h; base += 8 * R) {
                floatx4 v[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int p = min(base + 8 * r + g, h - 1);
                    const floatx4* s = reinterpret_cast<const floatx4*>(yc + (size_t)p * 8 * 32) + c;
                    v[r] = (!NT || p < pin) ? *s : __builtin_nontemporal_load(s);
                }
#pragma unroll
                for (int r = 0; r < R; ++r) acc += (v[r].x + v[r].y) + (v[r].z + v[r].w);
            }
        }
        if (SYNC) __syncthreads();
    }
    if (acc == 12345.f) out[0] = acc;
}
#define PROBE(NAME, R, SYNC, NT)                                                                              \
    extern "C" __global__ __launch_bounds__(512) void NAME(const float* y, int N, int H, int pin, int nblk, float* out) { \
        probe<R, SYNC, NT>(y, N, H, pin, nblk, out);                                                         \
    }
PROBE(stream_probe, 8, true, true)
PROBE(stream_probe_r16, 16, true, true)
PROBE(stream_probe_r4, 4, true, true)
PROBE(stream_probe_nosync, 8, false, true)
PROBE(stream_probe_temporal, 8, true, false)
