// DPT policy forward on gfx950: KV-cache decode, teacher-forced window
// forward and the fused on-device bandit rollout.
//
// Reference arithmetic: models/net.py:41-60 (pack + embed_transition +
// GPT2Model + pred_actions) with transformers' GPT2Block (ln_1 -> c_attn ->
// causal SDPA, one head -> c_proj -> residual -> ln_2 -> c_fc -> gelu_new ->
// c_proj -> residual) and ln_f.
//
// Work decomposition (one workgroup = one tile of kTile = 16 tasks, 16 waves):
//  * dense projections (embed excluded): f32 MFMA 16x16x4, tasks are the M
//    rows, weights [in][out] are the B operand streamed from L2, one 16-column
//    tile per wave; every weight element is read once per workgroup per step;
//  * attention: one wave per task streams that task's K/V rows for positions
//    0..pos-1 from HBM (8 positions x 128 B per float4 wave-load = 1 KiB
//    coalesced), online softmax per lane-group of 8, combined across the 8
//    groups by a 3-step butterfly; the new position's K/V come from LDS;
//  * LayerNorm / gelu / residual: one half-wave per task in LDS.
// The rollout kernel keeps a tile resident for all H steps (tasks never
// interact, so no inter-workgroup synchronisation exists anywhere).
#include <stdarg.h>
#include <stdio.h>

#include <string>

#include "dpt_common.h"

namespace dpt {

constexpr int kTile = 16;
constexpr int kThreads = 1024;            // 16 waves
constexpr int kLdE = kE + 2;              // padded LDS row strides (conflict-free A reads)
constexpr int kLdFF = kFF + 2;
constexpr int kRows = 4;                  // K/V rows (of 8 positions) in flight per wave

struct DecodeSmem {
    float x[kTile][kE];          // residual stream of the current position
    float xn[kTile][kLdE];       // LayerNorm output (MFMA A operand)
    float q[kTile][kE];
    float kcur[kTile][kE];
    float vcur[kTile][kE];
    float o[kTile][kLdE];        // attention output (A operand of c_proj)
    float h[kTile][kLdFF];       // MLP hidden (A operand of mlp.c_proj)
    float part[4][kTile][kE];    // split-K partials of mlp.c_proj
    float logits[kTile][kMaxA];
    float tok[kTile][kMaxF];     // packed token features of the current position
    int action[kTile];
};

__device__ inline floatx4 mfma_tile(const float* A, int lda, const float* __restrict__ B, int ldb,
                                     int K, int lane) {
    // C[16x16] = A[16 x K] (LDS) * B[K x 16] (global, column offset folded into B).
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const int i = lane & 15, kq = lane >> 4;
    float b[32];
#pragma unroll 8
    for (int s = 0; s < K / 4; ++s) b[s] = __ldg(B + (size_t)(4 * s + kq) * ldb + i);
#pragma unroll 8
    for (int s = 0; s < K / 4; ++s) {
        float a = A[i * lda + 4 * s + kq];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[s], acc, 0, 0, 0);
    }
    return acc;
}

// LayerNorm of the tile's residual rows: one half-wave (32 lanes) per task.
__device__ inline void layer_norm_tile(DecodeSmem& S, const float* __restrict__ g,
                                       const float* __restrict__ b, int tid) {
    if (tid < kTile * kE) {
        const int t = tid >> 5, j = tid & 31;
        float v = S.x[t][j];
        float s = v;
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) s += __shfl_xor(s, off, 32);
        const float mean = s * (1.0f / kE);
        const float d = v - mean;
        float s2 = d * d;
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) s2 += __shfl_xor(s2, off, 32);
        const float rstd = 1.0f / sqrtf(s2 * (1.0f / kE) + 1e-5f);
        S.xn[t][j] = fmaf(d * rstd, g[j], b[j]);
    }
}

__device__ inline float gelu_new(float x) {
    // 0.5*x*(1 + tanh(sqrt(2/pi)*(x + 0.044715*x^3)))  (transformers/activations.py:65)
    const float k0 = 0.7978845608028654f;
    float inner = k0 * (x + 0.044715f * (x * x * x));
    return 0.5f * x * (1.0f + tanhf(inner));
}

// Flash-decoding attention of one task (one wave): positions 0..pos-1 from the
// cache (global), position pos from LDS.  Writes o = softmax(qK^T/sqrt(E)) V.
__device__ inline void attend_one(const float* __restrict__ kc, const float* __restrict__ vc, int pos,
                                  const float* q, const float* kcur, const float* vcur, float* o,
                                  int lane) {
    const int g = lane >> 3, c = lane & 7;
    const float scale = 0.17677669529663687f;  // 32 ** -0.5
    const float4 q4 = *reinterpret_cast<const float4*>(q + 4 * c);
    float m = -1e30f, l = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int base = 0; base < pos; base += 8 * kRows) {
        float4 kk[kRows], vv[kRows];
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            const int p = base + 8 * r + g;
            if (p < pos) {
                kk[r] = __ldg(reinterpret_cast<const float4*>(kc + (size_t)p * kE) + c);
                vv[r] = __ldg(reinterpret_cast<const float4*>(vc + (size_t)p * kE) + c);
            } else {
                kk[r] = make_float4(0.f, 0.f, 0.f, 0.f);
                vv[r] = kk[r];
            }
        }
        float s[kRows];
        float mx = -1e30f;
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            float d = q4.x * kk[r].x;
            d = fmaf(q4.y, kk[r].y, d);
            d = fmaf(q4.z, kk[r].z, d);
            d = fmaf(q4.w, kk[r].w, d);
            d += __shfl_xor(d, 1);
            d += __shfl_xor(d, 2);
            d += __shfl_xor(d, 4);
            const int p = base + 8 * r + g;
            s[r] = (p < pos) ? d * scale : -INFINITY;
            mx = fmaxf(mx, s[r]);
        }
        const float mn = fmaxf(m, mx);
        const float corr = expf(m - mn);
        l *= corr;
        acc.x *= corr; acc.y *= corr; acc.z *= corr; acc.w *= corr;
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            const float pr = expf(s[r] - mn);
            l += pr;
            acc.x = fmaf(pr, vv[r].x, acc.x);
            acc.y = fmaf(pr, vv[r].y, acc.y);
            acc.z = fmaf(pr, vv[r].z, acc.z);
            acc.w = fmaf(pr, vv[r].w, acc.w);
        }
        m = mn;
    }
    {   // the new position (group 0 only; all lanes run the shuffles)
        const float4 k4 = *reinterpret_cast<const float4*>(kcur + 4 * c);
        const float4 v4 = *reinterpret_cast<const float4*>(vcur + 4 * c);
        float d = q4.x * k4.x;
        d = fmaf(q4.y, k4.y, d);
        d = fmaf(q4.z, k4.z, d);
        d = fmaf(q4.w, k4.w, d);
        d += __shfl_xor(d, 1);
        d += __shfl_xor(d, 2);
        d += __shfl_xor(d, 4);
        if (g == 0) {
            const float sc = d * scale;
            const float mn = fmaxf(m, sc);
            const float corr = expf(m - mn);
            const float pr = expf(sc - mn);
            l = l * corr + pr;
            acc.x = fmaf(pr, v4.x, acc.x * corr);
            acc.y = fmaf(pr, v4.y, acc.y * corr);
            acc.z = fmaf(pr, v4.z, acc.z * corr);
            acc.w = fmaf(pr, v4.w, acc.w * corr);
            m = mn;
        }
    }
#pragma unroll
    for (int off = 8; off <= 32; off <<= 1) {
        const float mo = __shfl_xor(m, off);
        const float lo = __shfl_xor(l, off);
        const float ax = __shfl_xor(acc.x, off), ay = __shfl_xor(acc.y, off);
        const float az = __shfl_xor(acc.z, off), aw = __shfl_xor(acc.w, off);
        const float mn = fmaxf(m, mo);
        const float sa = expf(m - mn), sb = expf(mo - mn);
        l = l * sa + lo * sb;
        acc.x = acc.x * sa + ax * sb;
        acc.y = acc.y * sa + ay * sb;
        acc.z = acc.z * sa + az * sb;
        acc.w = acc.w * sa + aw * sb;
        m = mn;
    }
    if (lane < 8) {
        const float inv = 1.0f / l;
        o[4 * c + 0] = acc.x * inv;
        o[4 * c + 1] = acc.y * inv;
        o[4 * c + 2] = acc.z * inv;
        o[4 * c + 3] = acc.w * inv;
    }
}

// One decode position for the tile: S.tok -> ... -> S.logits.  K/V of `pos`
// are appended to the cache.  kv: [2][L][N][max_pos][E].
__device__ void decode_position(DecodeSmem& S, const ModelView& M, float* __restrict__ kv, int N,
                                int max_pos, int tile0, int pos) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t lstride = (size_t)N * max_pos * kE;            // one layer of K (or V)
    const size_t vhalf = (size_t)M.n_layer * lstride;

    // embed_transition + wpe (net.py:52-53; GPT2Model inputs_embeds + position_embeds)
    if (tid < kTile * kE) {
        const int t = tid >> 5, j = tid & 31;
        float acc = 0.f;
        for (int f = 0; f < M.F; ++f) acc = fmaf(S.tok[t][f], M.emb_w[f * kE + j], acc);
        S.x[t][j] = (acc + M.emb_b[j]) + M.wpe[(size_t)pos * kE + j];
    }
    __syncthreads();

    for (int li = 0; li < M.n_layer; ++li) {
        const float* W = M.layers + (size_t)li * LayerOff::size;
        layer_norm_tile(S, W + LayerOff::ln1_g, W + LayerOff::ln1_b, tid);
        __syncthreads();
        // c_attn: [16 x 32] x [32 x 96] -> q | k | v, one 16-column tile per wave
        if (wave < 6) {
            floatx4 acc = mfma_tile(&S.xn[0][0], kLdE, W + LayerOff::attn_w + wave * 16, 3 * kE, kE, lane);
            const int col = wave * 16 + (lane & 15);
            const float bias = W[LayerOff::attn_b + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = (lane >> 4) * 4 + r;
                const float v = acc[r] + bias;
                const int task = tile0 + t;
                if (col < kE) {
                    S.q[t][col] = v;
                } else if (col < 2 * kE) {
                    S.kcur[t][col - kE] = v;
                    if (task < N) kv[li * lstride + ((size_t)task * max_pos + pos) * kE + col - kE] = v;
                } else {
                    S.vcur[t][col - 2 * kE] = v;
                    if (task < N)
                        kv[vhalf + li * lstride + ((size_t)task * max_pos + pos) * kE + col - 2 * kE] = v;
                }
            }
        }
        __syncthreads();
        // causal self-attention, one wave per task
        {
            const int t = wave;
            const int task = tile0 + t;
            if (task < N) {
                const float* kc = kv + li * lstride + (size_t)task * max_pos * kE;
                const float* vc = kv + vhalf + li * lstride + (size_t)task * max_pos * kE;
                attend_one(kc, vc, pos, S.q[t], S.kcur[t], S.vcur[t], S.o[t], lane);
            }
        }
        __syncthreads();
        // c_proj + residual
        if (wave < 2) {
            floatx4 acc = mfma_tile(&S.o[0][0], kLdE, W + LayerOff::proj_w + wave * 16, kE, kE, lane);
            const int col = wave * 16 + (lane & 15);
            const float bias = W[LayerOff::proj_b + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = (lane >> 4) * 4 + r;
                S.x[t][col] = (acc[r] + bias) + S.x[t][col];
            }
        }
        __syncthreads();
        layer_norm_tile(S, W + LayerOff::ln2_g, W + LayerOff::ln2_b, tid);
        __syncthreads();
        // c_fc + gelu_new
        if (wave < 8) {
            floatx4 acc = mfma_tile(&S.xn[0][0], kLdE, W + LayerOff::fc_w + wave * 16, kFF, kE, lane);
            const int col = wave * 16 + (lane & 15);
            const float bias = W[LayerOff::fc_b + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = (lane >> 4) * 4 + r;
                S.h[t][col] = gelu_new(acc[r] + bias);
            }
        }
        __syncthreads();
        // mlp.c_proj: K = 128 split four ways over waves, partials reduced in order
        if (wave < 8) {
            const int ct = wave & 1, kc4 = wave >> 1;
            floatx4 acc = mfma_tile(&S.h[0][kc4 * 32], kLdFF,
                                    W + LayerOff::mp_w + (size_t)kc4 * 32 * kE + ct * 16, kE, 32, lane);
            const int col = ct * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) S.part[kc4][(lane >> 4) * 4 + r][col] = acc[r];
        }
        __syncthreads();
        if (tid < kTile * kE) {
            const int t = tid >> 5, j = tid & 31;
            const float ff = ((S.part[0][t][j] + S.part[1][t][j]) + (S.part[2][t][j] + S.part[3][t][j]));
            S.x[t][j] = S.x[t][j] + (ff + W[LayerOff::mp_b + j]);
        }
        __syncthreads();
    }
    layer_norm_tile(S, M.lnf_g, M.lnf_b, tid);
    __syncthreads();
    // pred_actions head: [16 x 32] x [32 x A]
    const int ntile = (M.A + 15) >> 4;
    if (wave < ntile) {
        // head_w is [E][A]; columns beyond A read a clamped column and are discarded
        const int i = lane & 15, kq = lane >> 4;
        const int col = wave * 16 + i;
        const int colc = col < M.A ? col : M.A - 1;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kE / 4; ++s) {
            float a = S.xn[i][4 * s + kq];
            float b = M.head_w[(4 * s + kq) * M.A + colc];
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
        if (col < M.A) {
            const float bias = M.head_b[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) S.logits[kq * 4 + r][col] = acc[r] + bias;
        }
    }
    __syncthreads();
}

// ----------------------------------------------------------------------------- kernels

// One decode position for all tasks; tokens (N, F) given.
__global__ __launch_bounds__(kThreads) void decode_step_kernel(ModelView M, float* kv, int N, int max_pos,
                                                               int pos, const float* __restrict__ token,
                                                               float* __restrict__ logits) {
    __shared__ DecodeSmem S;
    const int tile0 = blockIdx.x * kTile;
    const int tid = threadIdx.x;
    for (int i = tid; i < kTile * kMaxF; i += kThreads) {
        const int t = i / kMaxF, f = i % kMaxF;
        S.tok[t][f] = (tile0 + t < N && f < M.F) ? token[(size_t)(tile0 + t) * M.F + f] : 0.f;
    }
    __syncthreads();
    decode_position(S, M, kv, N, max_pos, tile0, pos);
    for (int i = tid; i < kTile * M.A; i += kThreads) {
        const int t = i / M.A, a = i % M.A;
        if (tile0 + t < N) logits[(size_t)(tile0 + t) * M.A + a] = S.logits[t][a];
    }
}

// Teacher-forced window forward (= Transformer.forward over query + C context
// rows): positions 0..C decoded in order through the workspace cache.
__global__ __launch_bounds__(kThreads) void window_decode_kernel(
    ModelView M, float* kv, int N, int C, const float* __restrict__ query, const float* __restrict__ cs,
    const float* __restrict__ ca, const float* __restrict__ cn, const float* __restrict__ cr, int out_mode,
    float* __restrict__ out) {
    __shared__ DecodeSmem S;
    const int tile0 = blockIdx.x * kTile;
    const int tid = threadIdx.x;
    const int sd = M.sd, A = M.A;
    const int T = C + 1;
    for (int pos = 0; pos < T; ++pos) {
        // token packing (models/net.py:42-51)
        for (int i = tid; i < kTile * kMaxF; i += kThreads) {
            const int t = i / kMaxF, f = i % kMaxF;
            const int task = tile0 + t;
            float v = 0.f;
            if (task < N && f < M.F) {
                if (pos == 0) {
                    v = (f < sd) ? query[(size_t)task * sd + f] : 0.f;
                } else {
                    const size_t row = (size_t)task * C + (pos - 1);
                    if (f < sd) v = cs[row * sd + f];
                    else if (f < sd + A) v = ca[row * A + (f - sd)];
                    else if (f < 2 * sd + A) v = cn[row * sd + (f - sd - A)];
                    else v = cr[row];
                }
            }
            S.tok[t][f] = v;
        }
        __syncthreads();
        decode_position(S, M, kv, N, T, tile0, pos);
        if (out_mode == 0 && pos == C) {
            for (int i = tid; i < kTile * A; i += kThreads) {
                const int t = i / A, a = i % A;
                if (tile0 + t < N) out[(size_t)(tile0 + t) * A + a] = S.logits[t][a];
            }
        } else if (out_mode == 1 && pos >= 1) {
            for (int i = tid; i < kTile * A; i += kThreads) {
                const int t = i / A, a = i % A;
                if (tile0 + t < N) out[((size_t)(tile0 + t) * C + (pos - 1)) * A + a] = S.logits[t][a];
            }
        }
        __syncthreads();
    }
}

struct BanditRolloutParams {
    int N, H, A, type, sample;
    int64_t first_task;
    double var;
    uint64_t seed;
    const double* means;
    const double* uniforms;
    const double* noise;
    float* kv;
    int32_t* actions_out;
    double* rewards_out;
    double* arm_value_out;
    float* logits_out;
};

// The bandit online loop (evals/eval_bandit.py:70-89) for one tile of tasks,
// all H steps: decode -> select -> env step -> append transition.
__global__ __launch_bounds__(kThreads) void rollout_bandit_kernel(ModelView M, BanditRolloutParams P) {
    __shared__ DecodeSmem S;
    const int tile0 = blockIdx.x * kTile;
    const int tid = threadIdx.x;
    const int A = P.A;
    // position 0: the query token [state=1, 0_A, 0, 0] (BanditEnv.state = [1], ctrl_bandit.py:426)
    for (int i = tid; i < kTile * kMaxF; i += kThreads) {
        const int t = i / kMaxF, f = i % kMaxF;
        S.tok[t][f] = (f == 0) ? 1.f : 0.f;
    }
    __syncthreads();
    for (int h = 0; h < P.H; ++h) {
        decode_position(S, M, P.kv, P.N, P.H, tile0, h);
        if (tid < kTile) {
            const int t = tid, task = tile0 + t;
            if (task < P.N) {
                const int64_t gtask = P.first_task + task;
                double u = 0.0;
                if (P.sample)
                    u = P.uniforms ? P.uniforms[(size_t)h * P.N + task]
                                   : philox_uniform(P.seed, h, gtask, DPT_STREAM_SELECT);
                const int a = select_from_logits(S.logits[t], A, P.sample, 1.0f, u);
                const double mean = P.means[(size_t)task * A + a];
                double r;
                if (P.type == DPT_BANDIT_BERNOULLI) {
                    const double ur = P.noise ? P.noise[(size_t)h * P.N + task]
                                              : philox_uniform(P.seed, h, gtask, DPT_STREAM_REWARD);
                    r = (ur < mean) ? 1.0 : 0.0;
                } else {
                    const double g = P.noise ? P.noise[(size_t)h * P.N + task]
                                             : philox_normal(P.seed, h, gtask, DPT_STREAM_REWARD);
                    r = gaussian_reward(mean, P.var, g);
                }
                P.actions_out[(size_t)task * P.H + h] = a;
                P.rewards_out[(size_t)task * P.H + h] = r;
                P.arm_value_out[(size_t)task * P.H + h] = mean;
                if (P.logits_out)
                    for (int k = 0; k < A; ++k) P.logits_out[((size_t)h * P.N + task) * A + k] = S.logits[t][k];
                // next token = transition h: [s=1, onehot(a), s'=1, float(r)] (eval_bandit.py:83-86)
                S.tok[t][0] = 1.f;
                for (int k = 0; k < A; ++k) S.tok[t][1 + k] = (k == a) ? 1.f : 0.f;
                S.tok[t][1 + A] = 1.f;
                S.tok[t][2 + A] = (float)r;
            }
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------------------- host side

ModelView make_view(const float* blob, const dpt_model_desc& d) {
    ModelView v;
    const int F = 2 * d.state_dim + d.action_dim + 1;
    size_t off = 0;
    v.emb_w = blob + off; off += (size_t)F * kE;
    v.emb_b = blob + off; off += kE;
    v.wpe = blob + off; off += (size_t)d.n_positions * kE;
    v.layers = blob + off; off += (size_t)d.n_layer * LayerOff::size;
    v.lnf_g = blob + off; off += kE;
    v.lnf_b = blob + off; off += kE;
    v.head_w = blob + off; off += (size_t)kE * d.action_dim;
    v.head_b = blob + off;
    v.n_layer = d.n_layer;
    v.sd = d.state_dim;
    v.A = d.action_dim;
    v.F = F;
    v.n_positions = d.n_positions;
    return v;
}

int64_t weights_numel(const dpt_model_desc& d) {
    const int F = 2 * d.state_dim + d.action_dim + 1;
    return (int64_t)F * kE + kE + (int64_t)d.n_positions * kE + (int64_t)d.n_layer * LayerOff::size + 2 * kE +
           (int64_t)kE * d.action_dim + d.action_dim;
}

int launch_decode_step(const ModelView& M, float* kv, int N, int max_pos, int pos, const float* token,
                       float* logits, hipStream_t st) {
    dim3 grid((N + kTile - 1) / kTile);
    hipLaunchKernelGGL(decode_step_kernel, grid, dim3(kThreads), 0, st, M, kv, N, max_pos, pos, token, logits);
    return check_hip(hipGetLastError(), "decode_step_kernel launch");
}

int launch_window_decode(const ModelView& M, float* kv, int N, int C, const float* q, const float* cs,
                         const float* ca, const float* cn, const float* cr, int out_mode, float* out,
                         hipStream_t st) {
    dim3 grid((N + kTile - 1) / kTile);
    hipLaunchKernelGGL(window_decode_kernel, grid, dim3(kThreads), 0, st, M, kv, N, C, q, cs, ca, cn, cr,
                       out_mode, out);
    return check_hip(hipGetLastError(), "window_decode_kernel launch");
}

int launch_rollout_bandit(const ModelView& M, const dpt_bandit_rollout_args& a, hipStream_t st) {
    BanditRolloutParams P;
    P.N = a.N; P.H = a.H; P.A = a.A; P.type = a.type; P.sample = a.sample;
    P.first_task = a.first_task; P.var = a.var; P.seed = a.seed;
    P.means = a.means; P.uniforms = a.uniforms; P.noise = a.noise; P.kv = a.kvcache;
    P.actions_out = a.actions_out; P.rewards_out = a.rewards_out; P.arm_value_out = a.arm_value_out;
    P.logits_out = a.logits_out;
    dim3 grid((a.N + kTile - 1) / kTile);
    hipLaunchKernelGGL(rollout_bandit_kernel, grid, dim3(kThreads), 0, st, M, P);
    return check_hip(hipGetLastError(), "rollout_bandit_kernel launch");
}

}  // namespace dpt
