// Fused DarkRoom in-context evaluation on gfx950: evals/eval_darkroom.py:20-84
// deploy_online_vec with DarkroomTransformerController (ctrls/ctrl_darkroom.py:23-66)
// and DarkroomEnvVec.deploy_eval (envs/darkroom_env.py:151-175), one launch.
//
// The query (current state) changes every step, so each step is a full causal
// forward over the window [query, context transitions...] (models/net.py:41-60);
// the prediction is the LAST position.  That is fp32-MFMA work: one workgroup
// owns one task for all Heps x horizon steps, and wave w owns the 16 tokens
// [16w, 16w+16) of the window (T <= 128).
//
// Dataflow is transposed (features x tokens): a wave keeps x^T of its 16
// tokens in registers as MFMA 16x16x4 C-layout fragments -- lane (g = l>>4,
// c = l&15) holds features 16*blk + 4g + r of token c, blk in {0,1}, r < 4.
// That is exactly the B-operand layout of the next product W^T x^T (k-step s
// reads feature 16*(s>>2) + 4g + (s&3)), so c_attn, attention, c_proj, c_fc,
// gelu and mlp.c_proj chain in registers; only K (token-major) and V
// (feature-major) go through LDS, because every later token reads them.
// Weights are the A operand, pre-packed per layer in fragment order
// (FragOff) so one 16-B load per lane feeds four MFMAs.
//
// Per step and layer: c_attn -> barrier -> causal flash attention (S^T = K Q^T
// in registers, online softmax per token column, O^T += V^T P^T) -> barrier ->
// c_proj, LayerNorm, MLP.  In the last layer only the wave that owns the last
// position continues past the K/V exchange (nothing else is read), then it
// applies ln_f + head, selects the action and steps the grid env.
#include "dpt_common.h"

namespace dpt {

constexpr int kDrWaves = 8;                 // token blocks per window
constexpr int kDrT = 16 * kDrWaves;         // max window (1 + R*horizon)
constexpr int kKStride = kE + 4;            // K[token][feature]
constexpr int kVStride = kDrT + 4;          // Vt[feature][token]
constexpr int kDrA = 5;                     // DarkRoom actions

// Fragment-packed weights of one block (floats), see pack_fragments_kernel.
struct FragOff {
    static constexpr int attn = 0;            // [6 ob][2 q][64 lanes][4]
    static constexpr int proj = attn + 3072;  // [2 ob][2 q][64][4]
    static constexpr int fc = proj + 1024;    // [8 ob][2 q][64][4]
    static constexpr int mp = fc + 4096;      // [2 ob][8 chunk][64][4]
    static constexpr int size = mp + 4096;    // 12,288
};

// A-operand fragment of W^T for a k=32 input (W is [in][out], Conv1D layout):
// lane l, k-step s reads W[16*(s>>2) + 4*(l>>4) + (s&3)][ob*16 + (l&15)].
__global__ void pack_fragments_kernel(ModelView M, float* __restrict__ frag) {
    const int total = M.n_layer * FragOff::size;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int layer = i / FragOff::size;
        int o = i % FragOff::size;
        const float* W = M.layers + (size_t)layer * LayerOff::size;
        const float* src;
        int n_out, in, out;
        if (o < FragOff::fc && o >= 0) {
            int base, width;
            if (o < FragOff::proj) { base = FragOff::attn; src = W + LayerOff::attn_w; width = 3 * kE; }
            else { base = FragOff::proj; src = W + LayerOff::proj_w; width = kE; }
            o -= base;
            const int s4 = o & 3, lane = (o >> 2) & 63, q = (o >> 8) & 1, ob = o >> 9;
            const int s = 4 * q + s4;
            in = 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3);
            out = ob * 16 + (lane & 15);
            n_out = width;
        } else if (o < FragOff::mp) {
            o -= FragOff::fc;
            src = W + LayerOff::fc_w;
            const int s4 = o & 3, lane = (o >> 2) & 63, q = (o >> 8) & 1, ob = o >> 9;
            const int s = 4 * q + s4;
            in = 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3);
            out = ob * 16 + (lane & 15);
            n_out = kFF;
        } else {
            // mlp.c_proj [128][32]: chunk j, step s reads hidden 16j + 4*(l>>4) + s
            o -= FragOff::mp;
            src = W + LayerOff::mp_w;
            const int s = o & 3, lane = (o >> 2) & 63, j = (o >> 8) & 7, ob = o >> 11;
            in = 16 * j + 4 * (lane >> 4) + s;
            out = ob * 16 + (lane & 15);
            n_out = kE;
        }
        frag[i] = src[(size_t)in * n_out + out];
    }
}

struct DrSmem {
    float K[kDrT][kKStride];
    float Vt[kE][kVStride];
    int2 ctx[kDrT];   // context transitions, oldest first: .x = x|y<<8|a<<16|r<<24, .y = nx|ny<<8
    int2 cur[kDrT];   // this episode's transitions
    int sx, sy, ret, pad;
};

__device__ inline floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ inline floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

__device__ inline void bar_lds_dr() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LayerNorm over the 32 features of each token column (eps 1e-5): a lane holds
// 8 of them; the other 24 live in lanes l^16, l^32, l^48.
__device__ inline void ln_cols(const float (&v)[8], float (&out)[8], const float* __restrict__ gam,
                               const float* __restrict__ bet, int g) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    const float mean = s * (1.0f / kE);
    float d[8], s2 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        d[k] = v[k] - mean;
        s2 += d[k] * d[k];
    }
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    const float rstd = 1.0f / sqrtf(s2 * (1.0f / kE) + 1e-5f);
    const floatx4 g0 = ld4(gam + 4 * g), g1 = ld4(gam + 16 + 4 * g);
    const floatx4 b0 = ld4(bet + 4 * g), b1 = ld4(bet + 16 + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        out[r] = fmaf(d[r] * rstd, g0[r], b0[r]);
        out[4 + r] = fmaf(d[4 + r] * rstd, g1[r], b1[r]);
    }
}

__device__ inline float gelu_fast(float x) {
    // gelu_new (transformers/activations.py:65) with tanh(z) = 1 - 2/(exp(2z)+1)
    const float z = 0.7978845608028654f * (x + 0.044715f * (x * x * x));
    const float t = 1.0f - 2.0f / (__expf(2.0f * z) + 1.0f);
    return 0.5f * x * (1.0f + t);
}

// out^T(ob) = bias + W^T xin^T for a k=32 input held as 8 C-layout values.
__device__ inline floatx4 proj32(const float* __restrict__ frag, int ob, int lane, const float (&xin)[8],
                                 floatx4 acc) {
    const floatx4 w0 = ld4(frag + ((ob * 2 + 0) * 64 + lane) * 4);
    const floatx4 w1 = ld4(frag + ((ob * 2 + 1) * 64 + lane) * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma4(w0[s], xin[s], acc);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma4(w1[s], xin[4 + s], acc);
    return acc;
}

__device__ inline int2 pack_tr(int x, int y, int a, int nx, int ny, int r) {
    return make_int2(x | (y << 8) | (a << 16) | (r << 24), nx | (ny << 8));
}

// Fixed-A twin of select_from_logits (dpt_common.h): same arithmetic, the
// logits stay in registers.
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

struct DarkroomParams {
    int N, Heps, horizon, R, dim, sample;
    int64_t first_task;
    uint64_t seed, counter;
    float temp;
    const int32_t* goals;
    const int32_t* perms;
    const double* uniforms;
    int32_t* returns_out;
    int32_t* actions_out;
    float* logits_out;
    const float* frag;
};

__global__ void __launch_bounds__(kDrWaves * 64, 4)
rollout_darkroom_kernel(ModelView M, DarkroomParams p) {
    __shared__ DrSmem S;
    const int task = blockIdx.x;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
    const int tok = wave * 16 + c;
    const int gx = p.goals[2 * task], gy = p.goals[2 * task + 1];
    int perm[kDrA];
#pragma unroll
    for (int k = 0; k < kDrA; ++k) perm[k] = p.perms ? p.perms[(size_t)task * kDrA + k] : k;
    const int steps_total = p.Heps * p.horizon;
    const float scale = 0.17677669529663687f;  // 1/sqrt(head_dim = 32)
    // position-0 embedding pieces: emb_b + wpe[0] and the state rows of emb_w
    const floatx4 eb0 = ld4(M.emb_b + 4 * g), eb1 = ld4(M.emb_b + 16 + 4 * g);

    for (int ep = 0; ep < p.Heps; ++ep) {
        const int nctx = min(ep, p.R) * p.horizon;
        const int T = 1 + nctx;
        const int nqb = (T + 15) >> 4;
        const int qlast = (T - 1) >> 4, clast = (T - 1) & 15;
        const bool active = wave < nqb;
        if (tid == 0) {
            S.sx = 0;
            S.sy = 0;
            S.ret = 0;
        }
        // context embeddings of this wave's tokens (fixed for the episode)
        float x0[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x0[k] = 0.f;
        if (active && tok >= 1 && tok < T) {
            const int2 tr = S.ctx[tok - 1];
            const float fv[6] = {(float)(tr.x & 255), (float)((tr.x >> 8) & 255), 1.0f,
                                (float)(tr.y & 255), (float)((tr.y >> 8) & 255), (float)((tr.x >> 24) & 255)};
            const int rows[6] = {0, 1, 2 + ((tr.x >> 16) & 255), 7, 8, 9};
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                const int d0 = 16 * blk + 4 * g;
                floatx4 acc = blk ? eb1 : eb0;
#pragma unroll
                for (int f = 0; f < 6; ++f) {
                    const floatx4 w = ld4(M.emb_w + rows[f] * kE + d0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[r] = fmaf(fv[f], w[r], acc[r]);
                }
                const floatx4 pe = ld4(M.wpe + (size_t)tok * kE + d0);
#pragma unroll
                for (int r = 0; r < 4; ++r) x0[blk * 4 + r] = acc[r] + pe[r];
            }
        }
        __syncthreads();

        for (int t = 0; t < p.horizon; ++t) {
            const int sx = S.sx, sy = S.sy;
            float x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = x0[k];
            if (tok == 0) {  // the query token [state, 0...] at position 0
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const int d0 = 16 * blk + 4 * g;
                    const floatx4 w0 = ld4(M.emb_w + 0 * kE + d0), w1 = ld4(M.emb_w + 1 * kE + d0);
                    const floatx4 pe = ld4(M.wpe + d0);
                    floatx4 acc = blk ? eb1 : eb0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        acc[r] = fmaf((float)sx, w0[r], acc[r]);
                        acc[r] = fmaf((float)sy, w1[r], acc[r]);
                        x[blk * 4 + r] = acc[r] + pe[r];
                    }
                }
            }

            for (int layer = 0; layer < M.n_layer; ++layer) {
                const bool last = layer == M.n_layer - 1;
                const float* W = M.layers + (size_t)layer * LayerOff::size;
                const float* F = p.frag + (size_t)layer * FragOff::size;
                float q[8];
                if (active) {
                    float xn[8];
                    ln_cols(x, xn, W + LayerOff::ln1_g, W + LayerOff::ln1_b, g);
                    // c_attn: Q stays in registers, K -> LDS token-major, V -> LDS feature-major
#pragma unroll
                    for (int ob = 0; ob < 6; ++ob) {
                        floatx4 acc = ld4(W + LayerOff::attn_b + ob * 16 + 4 * g);
                        acc = proj32(F + FragOff::attn, ob, lane, xn, acc);
                        if (ob < 2) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) q[ob * 4 + r] = acc[r];
                        } else if (ob < 4) {
                            *reinterpret_cast<floatx4*>(&S.K[tok][16 * (ob - 2) + 4 * g]) = acc;
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; ++r) S.Vt[16 * (ob - 4) + 4 * g + r][tok] = acc[r];
                        }
                    }
                }
                bar_lds_dr();
                const bool work = active && (!last || wave == qlast);
                if (work) {
                    // causal flash attention for this wave's query block
                    float m = -INFINITY, lsum = 0.f;
                    floatx4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
                    for (int kb = 0; kb <= wave; ++kb) {
                        const floatx4 k0 = ld4(&S.K[kb * 16 + c][4 * g]);
                        const floatx4 k1 = ld4(&S.K[kb * 16 + c][16 + 4 * g]);
                        floatx4 sc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int s = 0; s < 4; ++s) sc = mfma4(k0[s], q[s], sc);
#pragma unroll
                        for (int s = 0; s < 4; ++s) sc = mfma4(k1[s], q[4 + s], sc);
                        float sv[4];
                        float mt = -INFINITY;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            sv[r] = sc[r] * scale;
                            if (kb == wave && 4 * g + r > c) sv[r] = -INFINITY;
                            mt = fmaxf(mt, sv[r]);
                        }
                        mt = fmaxf(mt, __shfl_xor(mt, 16));
                        mt = fmaxf(mt, __shfl_xor(mt, 32));
                        const float mn = fmaxf(m, mt);
                        const float corr = __expf(m - mn);
                        float pr[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) pr[r] = __expf(sv[r] - mn);
                        lsum = lsum * corr + ((pr[0] + pr[1]) + (pr[2] + pr[3]));
                        m = mn;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            o0[r] *= corr;
                            o1[r] *= corr;
                        }
                        const floatx4 v0 = ld4(&S.Vt[c][kb * 16 + 4 * g]);
                        const floatx4 v1 = ld4(&S.Vt[16 + c][kb * 16 + 4 * g]);
#pragma unroll
                        for (int s = 0; s < 4; ++s) o0 = mfma4(v0[s], pr[s], o0);
#pragma unroll
                        for (int s = 0; s < 4; ++s) o1 = mfma4(v1[s], pr[s], o1);
                    }
                    lsum += __shfl_xor(lsum, 16);
                    lsum += __shfl_xor(lsum, 32);
                    const float inv = 1.0f / lsum;
                    float o[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        o[r] = o0[r] * inv;
                        o[4 + r] = o1[r] * inv;
                    }
                    // attn.c_proj + residual
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob) {
                        floatx4 acc = ld4(W + LayerOff::proj_b + ob * 16 + 4 * g);
                        acc = proj32(F + FragOff::proj, ob, lane, o, acc);
#pragma unroll
                        for (int r = 0; r < 4; ++r) x[ob * 4 + r] += acc[r];
                    }
                }
                if (!last) bar_lds_dr();  // every read of this layer's K/V is done
                if (work) {
                    float xn[8];
                    ln_cols(x, xn, W + LayerOff::ln2_g, W + LayerOff::ln2_b, g);
                    floatx4 y0 = ld4(W + LayerOff::mp_b + 4 * g), y1 = ld4(W + LayerOff::mp_b + 16 + 4 * g);
#pragma unroll 2
                    for (int j = 0; j < kFF / 16; ++j) {
                        floatx4 h = ld4(W + LayerOff::fc_b + j * 16 + 4 * g);
                        h = proj32(F + FragOff::fc, j, lane, xn, h);
#pragma unroll
                        for (int r = 0; r < 4; ++r) h[r] = gelu_fast(h[r]);
                        const floatx4 w0 = ld4(F + FragOff::mp + ((0 * 8 + j) * 64 + lane) * 4);
                        const floatx4 w1 = ld4(F + FragOff::mp + ((1 * 8 + j) * 64 + lane) * 4);
#pragma unroll
                        for (int s = 0; s < 4; ++s) y0 = mfma4(w0[s], h[s], y0);
#pragma unroll
                        for (int s = 0; s < 4; ++s) y1 = mfma4(w1[s], h[s], y1);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        x[r] += y0[r];
                        x[4 + r] += y1[r];
                    }
                }
            }

            // ln_f + head + selection + env step, by the wave holding position T-1
            if (wave == qlast) {
                float xf[8];
                ln_cols(x, xf, M.lnf_g, M.lnf_b, g);
                float lg[kDrA];
#pragma unroll
                for (int a = 0; a < kDrA; ++a) {
                    float part = 0.f;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int d = 16 * (k >> 2) + 4 * g + (k & 3);
                        part = fmaf(xf[k], M.head_w[d * kDrA + a], part);
                    }
                    part += __shfl_xor(part, 16);
                    part += __shfl_xor(part, 32);
                    lg[a] = part + M.head_b[a];
                }
                if (lane == clast) {
                    const int step = ep * p.horizon + t;
                    double u = 0.0;
                    if (p.sample)
                        u = p.uniforms ? p.uniforms[(size_t)step * p.N + task]
                                       : philox_uniform(p.seed, p.counter + step, p.first_task + task,
                                                        DPT_STREAM_SELECT);
                    const int a = select_fixed<kDrA>(lg, p.sample, p.temp, u);
                    int ea = a;
#pragma unroll
                    for (int k = 0; k < kDrA; ++k)
                        if (k == a) ea = perm[k];
                    int nx = sx + (ea == 0) - (ea == 1);
                    int ny = sy + (ea == 2) - (ea == 3);
                    nx = min(max(nx, 0), p.dim - 1);
                    ny = min(max(ny, 0), p.dim - 1);
                    const int r = (nx == gx && ny == gy) ? 1 : 0;
                    S.cur[t] = pack_tr(sx, sy, a, nx, ny, r);
                    S.sx = nx;
                    S.sy = ny;
                    S.ret += r;
                    if (p.actions_out) p.actions_out[(size_t)task * steps_total + step] = a;
                    if (p.logits_out) {
#pragma unroll
                        for (int k = 0; k < kDrA; ++k) p.logits_out[((size_t)step * p.N + task) * kDrA + k] = lg[k];
                    }
                }
            }
            bar_lds_dr();
        }

        // episode bookkeeping: returns, then shift-append the context (eval_darkroom.py:75-82)
        if (tid == 0) p.returns_out[(size_t)task * p.Heps + ep] = S.ret;
        const int R = p.R, H = p.horizon;
        int2 v = make_int2(0, 0);
        const bool mv = tid < R * H;
        if (mv) {
            if (ep < R) v = (tid >= ep * H && tid < (ep + 1) * H) ? S.cur[tid - ep * H] : S.ctx[tid];
            else v = tid < (R - 1) * H ? S.ctx[tid + H] : S.cur[tid - (R - 1) * H];
        }
        __syncthreads();
        if (mv) S.ctx[tid] = v;
        __syncthreads();
    }
}

int launch_pack_fragments(const ModelView& M, float* frag, hipStream_t st) {
    hipLaunchKernelGGL(pack_fragments_kernel, dim3(64), dim3(256), 0, st, M, frag);
    return check_hip(hipGetLastError(), "pack_fragments_kernel launch");
}

int64_t fragments_numel(int n_layer) { return (int64_t)n_layer * FragOff::size; }

int launch_rollout_darkroom(const ModelView& M, const float* frag, const dpt_darkroom_rollout_args& a,
                            hipStream_t st) {
    DarkroomParams p;
    p.N = a.N;
    p.Heps = a.Heps;
    p.horizon = a.horizon;
    p.R = a.ctx_episodes;
    p.dim = a.dim;
    p.sample = a.sample;
    p.first_task = a.first_task;
    p.seed = a.seed;
    p.counter = a.counter;
    p.temp = a.temp;
    p.goals = a.goals;
    p.perms = a.perms;
    p.uniforms = a.uniforms;
    p.returns_out = a.returns_out;
    p.actions_out = a.actions_out;
    p.logits_out = a.logits_out;
    p.frag = frag;
    hipLaunchKernelGGL(rollout_darkroom_kernel, dim3(a.N), dim3(kDrWaves * 64), 0, st, M, p);
    return check_hip(hipGetLastError(), "rollout_darkroom_kernel launch");
}

int darkroom_max_window() { return kDrT; }

}  // namespace dpt
