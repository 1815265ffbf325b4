// Training forward / backward of the DPT Transformer (models/net.py:9-60 with test=False:
// preds at every position; train.py:286-331 trains on preds[:, 1:] with CrossEntropyLoss(sum)
// and AdamW).  SURVEY.md 8(f) row 4.  Generic in the model width (any n_embd, FF = 4 n_embd,
// one head as net.py:29 forces) and the window, all fp32:
//
//   forward : embed_transition + wpe -> n_layer x [ln_1, c_attn, causal softmax(QK^T/sqrt(E)) V,
//             c_proj + residual, ln_2, c_fc, gelu_new, mlp.c_proj + residual] -> ln_f -> head,
//             saving what the backward needs (the residual stream, LayerNorm statistics, q/k/v,
//             the attention probabilities, the MLP pre-activations) in a caller workspace;
//   backward: dL/dpreds -> every parameter's gradient in the packed blob layout of dpt_hip.h,
//             with fixed-order (deterministic) reductions over the B*T rows.
//
// The kernels are plain row / element kernels: at the reference's widths (E = 32, FF = 128) a
// training step is dominated by launch count and the O(T^2) attention, not by dense products,
// and one code path serves every width (the fused rollout kernels are specialised for E = 32).
// The same forward serves dpt_forward_window for models of other widths (inference).
#include "dpt_common.h"

namespace dpt {

constexpr int kTrThreads = 256;
constexpr int kTrRowsPerChunk = 64;   // rows per partial of the weight-gradient reductions


// offsets of one layer in the packed blob (dpt_hip.h: [ln1 g b][c_attn W b][c_proj W b][ln2 g b][c_fc W b][mlp.c_proj W b])
struct TrLayer {
    int64_t ln1_g, ln1_b, attn_w, attn_b, proj_w, proj_b, ln2_g, ln2_b, fc_w, fc_b, mp_w, mp_b;
    __host__ __device__ static TrLayer make(int64_t base, int E) {
        TrLayer o;
        int64_t p = base;
        o.ln1_g = p; p += E;
        o.ln1_b = p; p += E;
        o.attn_w = p; p += 3ll * E * E;
        o.attn_b = p; p += 3 * E;
        o.proj_w = p; p += (int64_t)E * E;
        o.proj_b = p; p += E;
        o.ln2_g = p; p += E;
        o.ln2_b = p; p += E;
        o.fc_w = p; p += 4ll * E * E;
        o.fc_b = p; p += 4 * E;
        o.mp_w = p; p += 4ll * E * E;
        o.mp_b = p;
        return o;
    }
};

struct TrBlob {  // offsets of the model-level parameters
    int64_t emb_w, emb_b, wpe, layers, lnf_g, lnf_b, head_w, head_b, total;
    __host__ __device__ static TrBlob make(const TrDims& d) {
        TrBlob b;
        int64_t p = 0;
        b.emb_w = p; p += (int64_t)d.F * d.E;
        b.emb_b = p; p += d.E;
        b.wpe = p; p += (int64_t)d.npos * d.E;
        b.layers = p; p += d.L * d.layer_size();
        b.lnf_g = p; p += d.E;
        b.lnf_b = p; p += d.E;
        b.head_w = p; p += (int64_t)d.E * d.A;
        b.head_b = p; p += d.A;
        b.total = p;
        return b;
    }
};

// Workspace (floats): the forward's saved activations, then the backward's scratch.
struct TrWs {
    int64_t x, y1, st1, qkv, P, o, x2, y2, st2, hpre, yf, stf;  // x: [L+1][R][E]; per-layer arrays [L][...]
    int64_t dx, dx2, dqkv, dout, dh, dy, dS, part, total;
    __host__ __device__ static int64_t nchunks(const TrDims& d) { return (d.R() + kTrRowsPerChunk - 1) / kTrRowsPerChunk; }
    __host__ __device__ static int tpad(int T) { return (T + 3) & ~3; }
    __host__ __device__ static TrWs make(const TrDims& d) {
        TrWs w;
        // every array starts 16-B aligned (the matrix-core kernels read rows as float4); the
        // attention probabilities / score gradients have rows padded to a multiple of 4 (tpad)
        const int64_t R = d.R(), E = d.E, TT = (int64_t)d.B * d.T * tpad(d.T);
        // forward-only: one slot per per-layer array (x ping-pongs over two), no probabilities,
        // no backward scratch
        const int64_t L = d.fwd_only ? 1 : d.L;
        int64_t p = 0;
        w.x = p; p += (d.fwd_only ? 2 : L + 1) * R * E; p = (p + 3) & ~3ll;
        w.y1 = p; p += L * R * E; p = (p + 3) & ~3ll;
        w.st1 = p; p += L * R * 2; p = (p + 3) & ~3ll;
        w.qkv = p; p += L * R * 3 * E; p = (p + 3) & ~3ll;
        w.P = p; p += d.fwd_only ? 0 : L * TT; p = (p + 3) & ~3ll;
        w.o = p; p += L * R * E; p = (p + 3) & ~3ll;
        w.x2 = p; p += L * R * E; p = (p + 3) & ~3ll;
        w.y2 = p; p += L * R * E; p = (p + 3) & ~3ll;
        w.st2 = p; p += L * R * 2; p = (p + 3) & ~3ll;
        w.hpre = p; p += L * R * 4 * E; p = (p + 3) & ~3ll;
        w.yf = p; p += R * E; p = (p + 3) & ~3ll;
        w.stf = p; p += R * 2; p = (p + 3) & ~3ll;
        if (d.fwd_only) {
            w.dx = w.dx2 = w.dqkv = w.dout = w.dh = w.dy = w.dS = w.part = w.total = p;
            return w;
        }
        w.dx = p; p += R * E; p = (p + 3) & ~3ll;
        w.dx2 = p; p += R * E; p = (p + 3) & ~3ll;
        w.dqkv = p; p += R * 3 * E; p = (p + 3) & ~3ll;
        w.dout = p; p += R * E; p = (p + 3) & ~3ll;
        w.dh = p; p += R * 4 * E; p = (p + 3) & ~3ll;
        w.dy = p; p += R * E; p = (p + 3) & ~3ll;
        w.dS = p; p += TT; p = (p + 3) & ~3ll;
        const int64_t wmax = std::max<int64_t>(4 * E * E + 4 * E, (int64_t)(d.F + 1) * E);
        w.part = p; p += nchunks(d) * std::max<int64_t>(wmax, (int64_t)(E + 1) * d.A); p = (p + 3) & ~3ll;
        w.total = p;
        return w;
    }
};

__device__ inline float tr_gelu(float x) {  // gelu_new (transformers/activations.py:65), accurate tanhf
    return 0.5f * x * (1.0f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}
__device__ inline float tr_gelu_grad(float x) {
    const float c = 0.7978845608028654f, a = 0.044715f;
    const float th = tanhf(c * (x + a * x * x * x));
    return 0.5f * (1.0f + th) + 0.5f * x * (1.0f - th * th) * c * (1.0f + 3.0f * a * x * x);
}

// order this wave's LDS writes before its later LDS reads of other lanes' entries
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}
__device__ inline float wave_max(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    return v;
}

// x[r][e] = embed_transition(tok[r]) + wpe[t]   (models/net.py:52-54 + GPT2Model inputs_embeds + wpe)
__global__ void tr_embed(const float* __restrict__ tok, const float* __restrict__ blob, TrDims d, TrBlob b,
                         float* __restrict__ x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)d.R() * d.E) return;
    const int r = (int)(i / d.E), e = (int)(i % d.E), t = r % d.T;
    float acc = blob[b.emb_b + e];
    for (int f = 0; f < d.F; ++f) acc = fmaf(tok[(int64_t)r * d.F + f], blob[b.emb_w + (int64_t)f * d.E + e], acc);
    x[i] = acc + blob[b.wpe + (int64_t)t * d.E + e];
}

// dropout factor of element e of a site (dpt_hip.h dpt_train_desc): drop_scale when the element's
// Philox word clears the threshold, else 0.  Regenerated in the backward -- no mask is stored.
__device__ inline float tr_keep(const TrDims& d, int site, int64_t e) {
    const U4 r = philox(d.drop_seed, (uint64_t)site, e >> 2, DPT_STREAM_DROPOUT);
    const int k = (int)(e & 3);
    const uint32_t w = k == 0 ? r.x : k == 1 ? r.y : k == 2 ? r.z : r.w;
    return w >= d.drop_thr ? d.drop_scale : 0.0f;
}

// out[i] = (add ? add[i] : 0) + x[i] keep(site, i) over n elements: the dropout of the embedding
// (in place), the residual adds x + drop(y) after c_proj / mlp.c_proj, and the gradients through them.
// Launched in place (out == x, and out == add), so no pointer is __restrict__: each thread reads
// its own element before writing it.
__global__ void tr_dropout(const float* x, const float* add, int64_t n, TrDims d, int site, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = x[i] * tr_keep(d, site, i);
    out[i] = add ? add[i] + v : v;
}

// LayerNorm over E (eps 1e-5), one wave per row; saves (mean, rstd)
__global__ void tr_layernorm(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ bb,
                             int R, int E, float* __restrict__ y, float* __restrict__ st) {
    const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= R) return;
    const float* xr = x + (int64_t)row * E;
    float s = 0.f;
    for (int e = lane; e < E; e += 64) s += xr[e];
    const float mean = wave_sum(s) / E;
    float q = 0.f;
    for (int e = lane; e < E; e += 64) q += (xr[e] - mean) * (xr[e] - mean);
    const float rstd = 1.0f / sqrtf(wave_sum(q) / E + 1e-5f);
    for (int e = lane; e < E; e += 64) y[(int64_t)row * E + e] = (xr[e] - mean) * rstd * g[e] + bb[e];
    if (lane == 0) {
        st[2 * row] = mean;
        st[2 * row + 1] = rstd;
    }
}

// tr_layernorm for rows of E <= 256 floats (E % 4 == 0): LPR lanes per row (E / 4 rounded up to a
// power of two), 64 / LPR rows per wave, the row read once into registers (one float4 per lane) and
// reduced over its lane group by xor shuffles.  At E = 16 a wave normalises 16 rows where
// tr_layernorm normalises one with 16 of its 64 lanes (the inference forward's row count is tasks x
// window, so the kernel is latency-bound on the per-row reductions, not on its bytes)
template <int LPR>
__global__ void tr_layernorm_rows(const float* __restrict__ x, const float* __restrict__ g,
                                  const float* __restrict__ bb, int R, int E, float* __restrict__ y,
                                  float* __restrict__ st) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63, c = lane % LPR;
    const int64_t wrow = ((int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * RPW;
    if (wrow >= R) return;  // whole wave past the end: no shuffle partner is left waiting
    const int64_t row = wrow + lane / LPR;
    const bool live = row < R, act = live && c < (E >> 2);
    const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
    const floatx4 v = act ? reinterpret_cast<const floatx4*>(x + row * E)[c] : zero;
    float s = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
    for (int k = 1; k < LPR; k <<= 1) s += __shfl_xor(s, k, 64);
    const float mean = s / E;
    const floatx4 dv = act ? v - mean : zero;
    float q = (dv[0] * dv[0] + dv[1] * dv[1]) + (dv[2] * dv[2] + dv[3] * dv[3]);
#pragma unroll
    for (int k = 1; k < LPR; k <<= 1) q += __shfl_xor(q, k, 64);
    const float rstd = 1.0f / sqrtf(q / E + 1e-5f);
    if (act) {
        floatx4 out;
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r] = dv[r] * rstd * g[4 * c + r] + bb[4 * c + r];
        reinterpret_cast<floatx4*>(y + row * E)[c] = out;
    }
    if (live && c == 0) {
        st[2 * row] = mean;
        st[2 * row + 1] = rstd;
    }
}

// LayerNorm of R rows: the row-group kernel where E and the pointers allow float4 rows, else tr_layernorm
static void layernorm(const float* x, const float* g, const float* bb, int R, int E, float* y, float* st,
                      hipStream_t s) {
    const int wpb = kTrThreads / 64;
    if (E % 4 == 0 && E <= 256 && !(((uintptr_t)x | (uintptr_t)y) & 15)) {
        int lpr = 1;
        while (lpr < E / 4) lpr <<= 1;
        const unsigned blocks = (unsigned)((R + (int64_t)wpb * (64 / lpr) - 1) / ((int64_t)wpb * (64 / lpr)));
        switch (lpr) {
            case 1: hipLaunchKernelGGL(tr_layernorm_rows<1>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
            case 2: hipLaunchKernelGGL(tr_layernorm_rows<2>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
            case 4: hipLaunchKernelGGL(tr_layernorm_rows<4>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
            case 8: hipLaunchKernelGGL(tr_layernorm_rows<8>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
            case 16: hipLaunchKernelGGL(tr_layernorm_rows<16>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
            case 32: hipLaunchKernelGGL(tr_layernorm_rows<32>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
            default: hipLaunchKernelGGL(tr_layernorm_rows<64>, dim3(blocks), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st); return;
        }
    }
    hipLaunchKernelGGL(tr_layernorm, dim3((R + wpb - 1) / wpb), dim3(kTrThreads), 0, s, x, g, bb, R, E, y, st);
}

// Y[r][o] = bias[o] + sum_i act(X[r][i]) W[i][o] (+ res[r][o]); act = gelu_new when gelu != 0
__global__ void tr_linear(const float* __restrict__ X, const float* __restrict__ W, const float* __restrict__ bias,
                          const float* __restrict__ res, int R, int IN, int OUT, int gelu, float* __restrict__ Y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)R * OUT) return;
    const int r = (int)(i / OUT), o = (int)(i % OUT);
    const float* xr = X + (int64_t)r * IN;
    float acc = bias[o];
    for (int k = 0; k < IN; ++k) acc = fmaf(gelu ? tr_gelu(xr[k]) : xr[k], W[(int64_t)k * OUT + o], acc);
    Y[i] = res ? acc + res[i] : acc;
}

// causal single-head attention, one wave per (task, query t): P[b][t][j] = softmax_j(q_t k_j / sqrt(E)),
// j <= t, and o_t = sum_j P[b][t][j] keep(site, (b T + t) T + j) v_j (site < 0: no dropout; P is
// saved undropped).  qkv rows [q | k | v] (c_attn output).
__global__ void tr_attn_fwd(const float* __restrict__ qkv, TrDims d, int site, float* __restrict__ P,
                            float* __restrict__ O) {
    extern __shared__ float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * (blockDim.x / 64) + wave;
    if (row >= d.R()) return;
    const int E = d.E, T = d.T, b = row / T, t = row % T;
    float* pr = sm + (size_t)wave * (T + E);
    float* q = pr + T;
    const float* base = qkv + (int64_t)b * T * 3 * E;
    for (int e = lane; e < E; e += 64) q[e] = base[(int64_t)t * 3 * E + e];
    wave_lds_sync();
    const float scale = 1.0f / sqrtf((float)E);
    float m = -INFINITY;
    for (int j = lane; j <= t; j += 64) {
        const float* k = base + (int64_t)j * 3 * E + E;
        float s = 0.f;
        for (int e = 0; e < E; ++e) s = fmaf(q[e], k[e], s);
        s *= scale;
        pr[j] = s;
        m = fmaxf(m, s);
    }
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j <= t; j += 64) {
        const float p = expf(pr[j] - m);
        pr[j] = p;
        l += p;
    }
    const float inv = 1.0f / wave_sum(l);
    float* prow = P ? P + ((int64_t)b * T + t) * T : nullptr;  // saved for the backward unless forward-only
    const int64_t mrow = ((int64_t)b * T + t) * T;
    for (int j = lane; j <= t; j += 64) {
        const float p = pr[j] * inv;
        pr[j] = site >= 0 ? p * tr_keep(d, site, mrow + j) : p;
        if (prow) prow[j] = p;
    }
    wave_lds_sync();
    for (int e = lane; e < E; e += 64) {
        float acc = 0.f;
        for (int j = 0; j <= t; ++j) acc = fmaf(pr[j], base[(int64_t)j * 3 * E + 2 * E + e], acc);
        O[(int64_t)row * E + e] = acc;
    }
}

// ------------------------------------------------------------------------------ backward

// dX[r][i] = sum_o dY[r][o] W[i][o], times gelu'(hpre[r][i]) when hpre is given, plus add[r][i]
__global__ void tr_linear_bwd_data(const float* __restrict__ dY, const float* __restrict__ W, int R, int IN, int OUT,
                                   const float* __restrict__ hpre, const float* __restrict__ add,
                                   float* __restrict__ dX) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)R * IN) return;
    const int r = (int)(i / IN), k = (int)(i % IN);
    const float* dy = dY + (int64_t)r * OUT;
    const float* w = W + (int64_t)k * OUT;
    float acc = 0.f;
    for (int o = 0; o < OUT; ++o) acc = fmaf(dy[o], w[o], acc);
    if (hpre) acc *= tr_gelu_grad(hpre[i]);
    dX[i] = add ? acc + add[i] : acc;
}

// partial weight gradients over one chunk of rows: part[c][i][o] = sum_r act(X[r][i]) dY[r][o] for
// i < IN and part[c][IN][o] = sum_r dY[r][o] (the bias); act = gelu_new when gelu != 0.
// grid (chunks, ceil((IN+1)*OUT / threads)); X may be null for a bias-only reduction.
__global__ void tr_wgrad_part(const float* __restrict__ X, const float* __restrict__ dY, int R, int IN, int OUT,
                              int gelu, float* __restrict__ part) {
    const int c = blockIdx.x;
    const int k = blockIdx.y * blockDim.x + threadIdx.x;
    if (k >= (IN + 1) * OUT) return;
    const int i = k / OUT, o = k % OUT;
    const int r0 = c * kTrRowsPerChunk, r1 = min(R, r0 + kTrRowsPerChunk);
    float acc = 0.f;
    if (i < IN) {
        for (int r = r0; r < r1; ++r) {
            const float xv = X[(int64_t)r * IN + i];
            acc = fmaf(gelu ? tr_gelu(xv) : xv, dY[(int64_t)r * OUT + o], acc);
        }
    } else {
        for (int r = r0; r < r1; ++r) acc += dY[(int64_t)r * OUT + o];
    }
    part[(int64_t)c * (IN + 1) * OUT + k] = acc;
}

// dW (IN x OUT, the blob's [in][out] layout) and db (OUT) = the chunk partials summed in a fixed
// order: 64 columns per workgroup (one per lane, 256-B coalesced rows), kTrRedWaves waves each
// summing a contiguous run of chunks in chunk order (loads unrolled so several are in flight), the
// run sums then added in wave order through LDS.  The same order every launch: deterministic.
// (One thread per column over all chunks left ~17 workgroups per product serially reading ~500
// partials: 61 % of a T = 501 training step.)
constexpr int kTrRedWaves = 16;
__global__ __launch_bounds__(64 * kTrRedWaves) void tr_wgrad_reduce(const float* __restrict__ part, int nch, int IN,
                                                                    int OUT, float* __restrict__ dW,
                                                                    float* __restrict__ db) {
    __shared__ float runs[kTrRedWaves][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t K = (int64_t)(IN + 1) * OUT;
    const int64_t k = (int64_t)blockIdx.x * 64 + lane;
    const int c0 = (int)((int64_t)nch * w / kTrRedWaves), c1 = (int)((int64_t)nch * (w + 1) / kTrRedWaves);
    float acc = 0.f;
    if (k < K) {
#pragma unroll 8
        for (int c = c0; c < c1; ++c) acc += part[(int64_t)c * K + k];
    }
    runs[w][lane] = acc;
    __syncthreads();
    if (w != 0 || k >= K) return;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kTrRedWaves; ++j) s += runs[j][lane];
    if (k < (int64_t)IN * OUT) {
        if (dW) dW[k] = s;
    } else if (db) {
        db[k - (int64_t)IN * OUT] = s;
    }
}
static void reduce_parts(const float* part, int nch, int IN, int OUT, float* dW, float* db, hipStream_t st) {
    const unsigned blocks = (unsigned)(((int64_t)(IN + 1) * OUT + 63) / 64);
    hipLaunchKernelGGL(tr_wgrad_reduce, dim3(blocks), dim3(64 * kTrRedWaves), 0, st, part, nch, IN, OUT, dW, db);
}

// LayerNorm backward, one wave per row: n = (x - mean) rstd, dn = dy g,
// dx = rstd (dn - mean(dn) - n mean(dn n)) (+ add)
__global__ void tr_layernorm_bwd(const float* __restrict__ x, const float* __restrict__ st,
                                 const float* __restrict__ g, const float* __restrict__ dy, int R, int E,
                                 const float* __restrict__ add, float* __restrict__ dx) {
    const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= R) return;
    const float mean = st[2 * row], rstd = st[2 * row + 1];
    const float* xr = x + (int64_t)row * E;
    const float* dr = dy + (int64_t)row * E;
    float s1 = 0.f, s2 = 0.f;
    for (int e = lane; e < E; e += 64) {
        const float n = (xr[e] - mean) * rstd, dn = dr[e] * g[e];
        s1 += dn;
        s2 += dn * n;
    }
    s1 = wave_sum(s1) / E;
    s2 = wave_sum(s2) / E;
    for (int e = lane; e < E; e += 64) {
        const float n = (xr[e] - mean) * rstd, dn = dr[e] * g[e];
        const float v = rstd * (dn - s1 - n * s2);
        const int64_t i = (int64_t)row * E + e;
        dx[i] = add ? v + add[i] : v;
    }
}

// LayerNorm parameter gradients, chunk partials: part[c][0][e] = sum_r dy n, part[c][1][e] = sum_r dy
__global__ void tr_ln_param_part(const float* __restrict__ x, const float* __restrict__ st,
                                 const float* __restrict__ dy, int R, int E, float* __restrict__ part) {
    const int c = blockIdx.x, e = blockIdx.y * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int r0 = c * kTrRowsPerChunk, r1 = min(R, r0 + kTrRowsPerChunk);
    float sg = 0.f, sb = 0.f;
    for (int r = r0; r < r1; ++r) {
        const float n = (x[(int64_t)r * E + e] - st[2 * r]) * st[2 * r + 1];
        const float v = dy[(int64_t)r * E + e];
        sg = fmaf(v, n, sg);
        sb += v;
    }
    part[(int64_t)c * 2 * E + e] = sg;
    part[(int64_t)c * 2 * E + E + e] = sb;
}

// attention backward, one wave per (task, query t): D_t = sum_e dO_t O_t,
// dS[b][t][j] = P[b][t][j] (keep_tj dO_t . v_j - D_t) for j <= t (keep = 1 when site < 0; D_t stays
// dO_t . O_t since O was formed from the dropped probabilities)
__global__ void tr_attn_bwd_ds(const float* __restrict__ qkv, const float* __restrict__ P,
                               const float* __restrict__ O, const float* __restrict__ dO, TrDims d, int site,
                               float* __restrict__ dS) {
    extern __shared__ float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * (blockDim.x / 64) + wave;
    if (row >= d.R()) return;
    const int E = d.E, T = d.T, b = row / T, t = row % T;
    float* go = sm + (size_t)wave * E;
    float dd = 0.f;
    for (int e = lane; e < E; e += 64) {
        const float v = dO[(int64_t)row * E + e];
        go[e] = v;
        dd = fmaf(v, O[(int64_t)row * E + e], dd);
    }
    dd = wave_sum(dd);
    wave_lds_sync();
    const float* base = qkv + (int64_t)b * T * 3 * E;
    const int64_t pr = ((int64_t)b * T + t) * T;
    for (int j = lane; j <= t; j += 64) {
        const float* v = base + (int64_t)j * 3 * E + 2 * E;
        float dp = 0.f;
        for (int e = 0; e < E; ++e) dp = fmaf(go[e], v[e], dp);
        if (site >= 0) dp *= tr_keep(d, site, ((int64_t)b * T + t) * T + j);
        dS[pr + j] = P[pr + j] * (dp - dd);
    }
}

// dq_t = sum_{j <= t} dS[t][j] k_j / sqrt(E) into dqkv[r][0:E]; thread per (row, e)
__global__ void tr_attn_bwd_dq(const float* __restrict__ qkv, const float* __restrict__ dS, TrDims d,
                               float* __restrict__ dqkv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)d.R() * d.E) return;
    const int E = d.E, T = d.T, row = (int)(i / E), e = (int)(i % E), b = row / T, t = row % T;
    const float* base = qkv + (int64_t)b * T * 3 * E + E + e;
    const float* ds = dS + ((int64_t)b * T + t) * T;
    float acc = 0.f;
    for (int j = 0; j <= t; ++j) acc = fmaf(ds[j], base[(int64_t)j * 3 * E], acc);
    dqkv[(int64_t)row * 3 * E + e] = acc / sqrtf((float)E);
}

// dk_j = sum_{t >= j} dS[t][j] q_t / sqrt(E), dv_j = sum_{t >= j} P[t][j] keep_tj dO_t into dqkv[r][E:3E]
__global__ void tr_attn_bwd_dkv(const float* __restrict__ qkv, const float* __restrict__ P,
                                const float* __restrict__ dS, const float* __restrict__ dO, TrDims d, int site,
                                float* __restrict__ dqkv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)d.R() * d.E) return;
    const int E = d.E, T = d.T, row = (int)(i / E), e = (int)(i % E), b = row / T, j = row % T;
    const float* q = qkv + (int64_t)b * T * 3 * E + e;
    const float* go = dO + (int64_t)b * T * E + e;
    const int64_t col = (int64_t)b * T * T + j;
    float ak = 0.f, av = 0.f;
    for (int t = j; t < T; ++t) {
        ak = fmaf(dS[col + (int64_t)t * T], q[(int64_t)t * 3 * E], ak);
        const float pt = P[col + (int64_t)t * T];
        av = fmaf(site >= 0 ? pt * tr_keep(d, site, ((int64_t)b * T + t) * T + j) : pt, go[(int64_t)t * E], av);
    }
    dqkv[(int64_t)row * 3 * E + E + e] = ak / sqrtf((float)E);
    dqkv[(int64_t)row * 3 * E + 2 * E + e] = av;
}

// dwpe[t][e] = sum_b dx[b][t][e]
__global__ void tr_wpe_grad(const float* __restrict__ dx, TrDims d, float* __restrict__ dwpe) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)d.T * d.E) return;
    float acc = 0.f;
    for (int b = 0; b < d.B; ++b) acc += dx[(int64_t)b * d.T * d.E + i];
    dwpe[i] = acc;
}

// ------------------------------------------------------------------------------ matrix-core forms
// The row products and weight gradients of widths E in {16, 32, 64} (every dimension a multiple of
// 16) on v_mfma_f32_16x16x4_f32 (fp32 products and accumulation, like the row kernels above; a
// different but fixed summation order, so results stay deterministic).

// Y[r][n] = epi( sum_k act(X[r][k]) B[k][n] ), B = W ([K][N]) or, TRANS, W^T (W stored [N][K]).
// One wave = 16 rows x all N columns, 4 waves = 64 rows per workgroup; B is staged in LDS once
// per workgroup.  The k order inside a lane is permuted -- lane (row i, kq) holds
// k = kq (K/4) + s at step s, a contiguous run of its row -- and B is read at the same k.
// EPI: bit 0 + bias[n], bit 1 + res[r][n], bit 2 x gelu'(aux[r][n]); ACT: gelu_new on X.
// kMmLnIn: X's rows LayerNorm'd on load (the forward-only inference path: ln_1 -> c_attn, ln_2 -> c_fc,
// no y1 / y2 round trip), gamma = aux[k], beta = aux[K + k] (the blob's ln_g, ln_b pair)
constexpr int kMmBias = 1, kMmRes = 2, kMmGeluGrad = 4, kMmLnIn = 8;
// LDS row stride of B (floats): the four 16-lane groups of a B read hit rows KS apart, so pad
// N until two groups of one 32-lane half land 16 banks apart (2-way at worst when impossible)
__host__ __device__ constexpr int mm_ldb(int K, int N) {
    for (int p = 0; p < 32; ++p)
        if (((K / 4) * (N + p)) % 32 == 16) return N + p;
    return N + 1;
}
// NC < N (the decode-sized rows of the generic rollout): blockIdx.y takes columns [NC y, NC y + NC),
// and only that slice of B is staged, so R / 64 row blocks still fill the chip; every output's
// k order is unchanged (bit-identical to NC = N).
template <int K, int N, bool TRANS, bool ACT, int EPI, int NC = N>
__global__ __launch_bounds__(256) void tr_mm_rows(const float* __restrict__ X, const float* __restrict__ W,
                                                  const float* __restrict__ bias, const float* __restrict__ res,
                                                  const float* __restrict__ aux, int R, float* __restrict__ Y) {
    static_assert(K % 16 == 0 && N % 16 == 0 && NC % 16 == 0 && N % NC == 0, "K, N, NC multiples of 16");
    constexpr int KS = K / 4;  // k-steps
    constexpr int LDB = mm_ldb(K, NC);
    extern __shared__ float Bs[];  // [K][LDB]
    const int n0 = NC == N ? 0 : blockIdx.y * NC;
    if constexpr (TRANS) {
        for (int i = threadIdx.x; i < K * NC; i += blockDim.x) {
            const int k = i / NC, n = i % NC;
            Bs[k * LDB + n] = W[(int64_t)(n0 + n) * K + k];
        }
    } else {  // 16-B loads (NC % 16 == 0: a float4 never crosses a row)
        for (int i = threadIdx.x; i < K * NC / 4; i += blockDim.x) {
            const int k = 4 * i / NC, n = 4 * i % NC;
            const floatx4 v = *reinterpret_cast<const floatx4*>(W + (int64_t)k * N + n0 + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) Bs[k * LDB + n + r] = v[r];
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i16 = lane & 15, kq = lane >> 4;
    const int row0 = (blockIdx.x * (blockDim.x >> 6) + wave) * 16;
    const int row = min(row0 + i16, R - 1);  // rows past R compute garbage that is never stored
    float a[KS];
    const floatx4* xr = reinterpret_cast<const floatx4*>(X + (int64_t)row * K + kq * KS);
#pragma unroll
    for (int s4 = 0; s4 < KS / 4; ++s4) {
        const floatx4 v = xr[s4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[4 * s4 + q] = ACT ? tr_gelu(v[q]) : v[q];
    }
    if constexpr ((EPI & kMmLnIn) != 0) {
        // the row's K values sit on lanes i16 + 16 kq (kq < 4), K / 4 contiguous each; the sums take
        // tr_layernorm_rows' order (float4 partials, then a balanced pairwise tree in row order: in
        // lane, then across the kq lanes), so y is bit-identical to the separate LayerNorm
        static_assert(KS % 4 == 0 && ((KS / 4) & (KS / 4 - 1)) == 0, "K / 16 a power of two");
        constexpr int NCH = KS / 4;
        auto tree = [&](float (&p)[NCH]) {
#pragma unroll
            for (int w = 1; w < NCH; w <<= 1)
#pragma unroll
                for (int j = 0; j < NCH; j += 2 * w) p[j] += p[j + w];
            float t = p[0];
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            return t;
        };
        float p[NCH];
#pragma unroll
        for (int j = 0; j < NCH; ++j) p[j] = (a[4 * j] + a[4 * j + 1]) + (a[4 * j + 2] + a[4 * j + 3]);
        const float mean = tree(p) / K;
#pragma unroll
        for (int k = 0; k < KS; ++k) a[k] -= mean;
#pragma unroll
        for (int j = 0; j < NCH; ++j)
            p[j] = (a[4 * j] * a[4 * j] + a[4 * j + 1] * a[4 * j + 1]) + (a[4 * j + 2] * a[4 * j + 2] + a[4 * j + 3] * a[4 * j + 3]);
        const float rstd = 1.0f / sqrtf(tree(p) / K + 1e-5f);
#pragma unroll
        for (int k = 0; k < KS; ++k) a[k] = a[k] * rstd * aux[kq * KS + k] + aux[K + kq * KS + k];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NC / 16; ++c) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], Bs[(kq * KS + s) * LDB + 16 * c + i16], acc, 0, 0, 0);
        const int n = n0 + 16 * c + i16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int rr = row0 + 4 * kq + r;
            if (rr >= R) continue;
            const int64_t o = (int64_t)rr * N + n;
            float v = acc[r];
            if (EPI & kMmBias) v += bias[n];
            if (EPI & kMmRes) v += res[o];
            if constexpr ((EPI & kMmGeluGrad) != 0) v *= tr_gelu_grad(aux[o]);
            Y[o] = v;
        }
    }
}

// Weight-gradient partials of one chunk of kTrRowsPerChunk rows: part[c][i][o] = sum_r act(X[r][i])
// dY[r][o] (i < IN) and part[c][IN][o] = sum_r dY[r][o], summed over the chunks in a fixed order by
// tr_wgrad_reduce.  The chunk's rows are staged in LDS (zeros past R); each wave takes output
// tiles (IN / 16) x (OUT / 16) round robin, 16 MFMA k-steps of 4 rows each.
template <int IN, int OUT, bool ACT>
__global__ __launch_bounds__(256) void tr_wgrad_mfma(const float* __restrict__ X, const float* __restrict__ dY,
                                                     int R, float* __restrict__ part) {
    static_assert(IN % 16 == 0 && OUT % 16 == 0, "IN, OUT multiples of 16");
    constexpr int C = kTrRowsPerChunk;
    extern __shared__ float sm[];
    float* Xs = sm;            // [C][IN + 1]: padded rows (conflict-free column reads)
    float* Ds = sm + C * (IN + 1);  // [C][OUT]
    const int r0 = blockIdx.x * C;
    for (int i = threadIdx.x; i < C * IN; i += 256) {
        const int r = i / IN, k = i % IN;
        const float v = r0 + r < R ? X[(int64_t)(r0 + r) * IN + k] : 0.f;
        Xs[r * (IN + 1) + k] = ACT ? tr_gelu(v) : v;
    }
    for (int i = threadIdx.x; i < C * OUT; i += 256) {
        const int r = i / OUT;
        Ds[i] = r0 + r < R ? dY[(int64_t)r0 * OUT + i] : 0.f;
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i16 = lane & 15, kq = lane >> 4;
    float* pc = part + (int64_t)blockIdx.x * (IN + 1) * OUT;
    for (int t = wave; t < (IN / 16) * (OUT / 16); t += 4) {
        const int ti = t / (OUT / 16), to = t % (OUT / 16);
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < C / 4; ++s) {
            const int r = 4 * s + kq;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[r * (IN + 1) + 16 * ti + i16], Ds[r * OUT + 16 * to + i16], acc,
                                                       0, 0, 0);
        }
        // C layout: lane (o = i16, kq) holds rows i = 16 ti + 4 kq + r
#pragma unroll
        for (int r = 0; r < 4; ++r) pc[(16 * ti + 4 * kq + r) * OUT + 16 * to + i16] = acc[r];
    }
    // the bias row: sum over the chunk's rows in order, one thread per output column
    for (int o = threadIdx.x; o < OUT; o += 256) {
        float acc = 0.f;
        for (int r = 0; r < C; ++r) acc += Ds[r * OUT + o];
        pc[IN * OUT + o] = acc;
    }
}

// ---- causal attention on the matrix cores (one head of width E; qkv rows [q | k | v], row stride 3E).
// A wave owns 16 queries (or, dkv, 16 keys); products are 16 x 16 tiles of v_mfma_f32_16x16x4_f32 with
// the tokens of the wave on the lane index: S^T = K Q^T gives lane (query n, g) the keys 4g + r of a
// 16-key tile, which is exactly the B operand of O^T += V^T P^T over that tile (k-step r takes keys
// 4g' + r of lane group g').  Feature k order of the Q / K products permuted per lane (run g E/4 .. ).
__device__ inline float grp_max(float v) {
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
}
__device__ inline float grp_sum(float v) {
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}
// lane (token n, g): row tok of the [rows][3E] qkv block at column off, features g E/4 .. g E/4 + E/4 - 1
template <int E>
__device__ inline void frag_row(const float* __restrict__ base, int tok, int off, float (&f)[E / 4]) {
    const floatx4* r = reinterpret_cast<const floatx4*>(base + (int64_t)tok * 3 * E + off + (threadIdx.x & 63) / 16 * (E / 4));
#pragma unroll
    for (int j = 0; j < E / 16; ++j) {
        const floatx4 v = r[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) f[4 * j + q] = v[q];
    }
}
// 4 consecutive entries of a T-wide row starting at column c (c % 4 == 0): columns >= T are not
// touched (stores) or read as 0 (loads)
__device__ inline void row4_store(float* row, int c, int T, floatx4 v) {
    if (c + 3 < T) {
        *reinterpret_cast<floatx4*>(row + c) = v;
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (c + r < T) row[c + r] = v[r];
    }
}
__device__ inline floatx4 row4_load(const float* row, int c, int T) {
    if (c + 3 < T) return *reinterpret_cast<const floatx4*>(row + c);
    floatx4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = c + r < T ? row[c + r] : 0.f;
    return v;
}
template <int E>
__device__ inline floatx4 tile_dot(const float (&a)[E / 4], const float (&b)[E / 4]) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < E / 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
    return acc;
}

// forward: P (saved unless null; rows of keys <= query, zeros past the diagonal inside the diagonal
// tile) and O = softmax(Q K^T / sqrt(E)) V.  Two passes over the key tiles: the row max and sum,
// then the probabilities and O.  grid (B, ceil(T / 64)), 256 threads.
template <int E>
__global__ __launch_bounds__(256) void tr_attn_fwd_mfma(const float* __restrict__ qkv, TrDims d, float* __restrict__ P,
                                                        float* __restrict__ O) {
    const int T = d.T, TP = (T + 3) & ~3, b = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 15, g = lane >> 4;  // P / dS rows are TP floats (TrWs::tpad)
    const int q0 = blockIdx.y * 64 + wave * 16;
    if (q0 >= T) return;
    const float* base = qkv + (int64_t)b * T * 3 * E;
    const int qn = q0 + n, qc = min(qn, T - 1);
    float qf[E / 4];
    frag_row<E>(base, qc, 0, qf);
    const float scale = 1.0f / sqrtf((float)E);
    const int nkt = (min(q0 + 15, T - 1)) / 16 + 1;  // key tiles up to the diagonal
    auto scores = [&](int kt, float (&sv)[4]) {
        float kf[E / 4];
        frag_row<E>(base, min(16 * kt + n, T - 1), E, kf);
        const floatx4 acc = tile_dot<E>(kf, qf);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int key = 16 * kt + 4 * g + r;
            sv[r] = (key <= qn && key < T) ? acc[r] * scale : -INFINITY;
        }
    };
    float m = -INFINITY, l = 0.f;
    for (int kt = 0; kt < nkt; ++kt) {
        float sv[4];
        scores(kt, sv);
        const float mt = grp_max(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])));
        const float mn = fmaxf(m, mt);
        l = (m == -INFINITY ? 0.f : l * expf(m - mn));
#pragma unroll
        for (int r = 0; r < 4; ++r) l += expf(sv[r] - mn);
        m = mn;
    }
    const float inv = 1.0f / grp_sum(l);
    floatx4 o[E / 16];
#pragma unroll
    for (int ft = 0; ft < E / 16; ++ft) o[ft] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nkt; ++kt) {
        float sv[4];
        scores(kt, sv);
        floatx4 pv;
#pragma unroll
        for (int r = 0; r < 4; ++r) pv[r] = expf(sv[r] - m) * inv;
        if (P && qn < T) row4_store(P + ((int64_t)b * T + qn) * TP, 16 * kt + 4 * g, T, pv);
#pragma unroll
        for (int ft = 0; ft < E / 16; ++ft)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = base[(int64_t)min(16 * kt + 4 * g + r, T - 1) * 3 * E + 2 * E + 16 * ft + n];
                o[ft] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, pv[r], o[ft], 0, 0, 0);
            }
    }
    if (qn < T)
#pragma unroll
        for (int ft = 0; ft < E / 16; ++ft) *reinterpret_cast<floatx4*>(O + ((int64_t)b * T + qn) * E + 16 * ft + 4 * g) = o[ft];
}

// backward, per 16 queries: D = dO . O, dP = dO V^T, dS = P (dP - D) (stored for the dK pass), dQ =
// dS K / sqrt(E) into dqkv[:, 0:E].  grid (B, ceil(T / 64)).
template <int E>
__global__ __launch_bounds__(256) void tr_attn_bwd_dq_mfma(const float* __restrict__ qkv, const float* __restrict__ P,
                                                           const float* __restrict__ O, const float* __restrict__ dO,
                                                           TrDims d, float* __restrict__ dS,
                                                           float* __restrict__ dqkv) {
    const int T = d.T, TP = (T + 3) & ~3, b = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 15, g = lane >> 4;  // P / dS rows are TP floats (TrWs::tpad)
    const int q0 = blockIdx.y * 64 + wave * 16;
    if (q0 >= T) return;
    const float* base = qkv + (int64_t)b * T * 3 * E;
    const int qn = q0 + n, qc = min(qn, T - 1);
    const int64_t orow = ((int64_t)b * T + qc) * E + g * (E / 4);
    float df[E / 4], dd = 0.f;
#pragma unroll
    for (int s = 0; s < E / 4; ++s) {
        df[s] = dO[orow + s];
        dd = fmaf(df[s], O[orow + s], dd);
    }
    dd = grp_sum(dd);
    const float scale = 1.0f / sqrtf((float)E);
    const int nkt = (min(q0 + 15, T - 1)) / 16 + 1;
    floatx4 dq[E / 16];
#pragma unroll
    for (int ft = 0; ft < E / 16; ++ft) dq[ft] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nkt; ++kt) {
        float vf[E / 4];
        frag_row<E>(base, min(16 * kt + n, T - 1), 2 * E, vf);
        const floatx4 dp = tile_dot<E>(vf, df);  // lane (query n, g): dP[query][keys 16 kt + 4g + r]
        const floatx4 pv = row4_load(P + ((int64_t)b * T + qc) * TP, 16 * kt + 4 * g, T);  // 0 past T
        floatx4 ds;
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[r] = pv[r] * (dp[r] - dd);
        if (qn < T) row4_store(dS + ((int64_t)b * T + qn) * TP, 16 * kt + 4 * g, T, ds);
#pragma unroll
        for (int ft = 0; ft < E / 16; ++ft)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float kv = base[(int64_t)min(16 * kt + 4 * g + r, T - 1) * 3 * E + E + 16 * ft + n];
                dq[ft] = __builtin_amdgcn_mfma_f32_16x16x4f32(kv, ds[r], dq[ft], 0, 0, 0);
            }
    }
    if (qn < T)
#pragma unroll
        for (int ft = 0; ft < E / 16; ++ft)
            *reinterpret_cast<floatx4*>(dqkv + ((int64_t)b * T + qn) * 3 * E + 16 * ft + 4 * g) = dq[ft] * scale;
}

// backward, per 16 keys: dK = dS^T Q / sqrt(E), dV = P^T dO into dqkv[:, E:3E], over the query tiles
// from the key tile's own (causal) to the last.  grid (B, ceil(T / 64)).
template <int E>
__global__ __launch_bounds__(256) void tr_attn_bwd_dkv_mfma(const float* __restrict__ qkv, const float* __restrict__ P,
                                                            const float* __restrict__ dS, const float* __restrict__ dO,
                                                            TrDims d, float* __restrict__ dqkv) {
    const int T = d.T, TP = (T + 3) & ~3, b = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 15, g = lane >> 4;  // P / dS rows are TP floats (TrWs::tpad)
    const int k0 = blockIdx.y * 64 + wave * 16;
    if (k0 >= T) return;
    const float* base = qkv + (int64_t)b * T * 3 * E;
    const int kn = k0 + n;
    floatx4 dk[E / 16], dv[E / 16];
#pragma unroll
    for (int ft = 0; ft < E / 16; ++ft) dk[ft] = dv[ft] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int nqt = (T - 1) / 16 + 1;
    for (int qt = k0 / 16; qt < nqt; ++qt) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int q = 16 * qt + 4 * s + g;  // k-step s: queries 16 qt + 4 s + g'
            const bool live = q < T && kn < T;
            const int64_t prow = ((int64_t)b * T + min(q, T - 1)) * TP + min(kn, T - 1);
            const float dsv = live ? dS[prow] : 0.f, pvv = live ? P[prow] : 0.f;
#pragma unroll
            for (int ft = 0; ft < E / 16; ++ft) {
                const int64_t qrow = (int64_t)min(q, T - 1);
                const float qv = base[qrow * 3 * E + 16 * ft + n];
                const float gv = dO[((int64_t)b * T + qrow) * E + 16 * ft + n];
                dk[ft] = __builtin_amdgcn_mfma_f32_16x16x4f32(qv, dsv, dk[ft], 0, 0, 0);
                dv[ft] = __builtin_amdgcn_mfma_f32_16x16x4f32(gv, pvv, dv[ft], 0, 0, 0);
            }
        }
    }
    const float scale = 1.0f / sqrtf((float)E);
    if (kn < T)
#pragma unroll
        for (int ft = 0; ft < E / 16; ++ft) {
            float* row = dqkv + ((int64_t)b * T + kn) * 3 * E;
            *reinterpret_cast<floatx4*>(row + E + 16 * ft + 4 * g) = dk[ft] * scale;
            *reinterpret_cast<floatx4*>(row + 2 * E + 16 * ft + 4 * g) = dv[ft];
        }
}

// LayerNorm parameter partials of one chunk: part[c][0][e] = sum_r dy n, part[c][1][e] = sum_r dy
// with 256 / E row lanes per column, combined in a fixed order through LDS.
__global__ __launch_bounds__(256) void tr_ln_param_part2(const float* __restrict__ x, const float* __restrict__ st,
                                                         const float* __restrict__ dy, int R, int E,
                                                         float* __restrict__ part) {
    __shared__ float sg[256], sb[256];
    const int c = blockIdx.x, t = threadIdx.x, lanes = 256 / E;
    const int e = t % E, rl = t / E;
    const int r0 = c * kTrRowsPerChunk, r1 = min(R, r0 + kTrRowsPerChunk);
    float g = 0.f, b = 0.f;
    if (rl < lanes)
        for (int r = r0 + rl; r < r1; r += lanes) {
            const float n = (x[(int64_t)r * E + e] - st[2 * r]) * st[2 * r + 1];
            const float v = dy[(int64_t)r * E + e];
            g = fmaf(v, n, g);
            b += v;
        }
    sg[t] = g;
    sb[t] = b;
    __syncthreads();
    if (t < E) {
        float G = 0.f, Bb = 0.f;
        for (int k = 0; k < lanes; ++k) {
            G += sg[k * E + t];
            Bb += sb[k * E + t];
        }
        part[(int64_t)c * 2 * E + t] = G;
        part[(int64_t)c * 2 * E + E + t] = Bb;
    }
}

// ------------------------------------------------------------------------------ host side

static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kTrThreads - 1) / kTrThreads); }

static int launched(const char* what) { return check_hip(hipGetLastError(), what); }

int train_dims_check(const TrDims& d) {
    if (d.L < 1 || d.E < 1 || d.E > 1024 || d.F < 1 || d.A < 1 || d.B < 1 || d.T < 1 || d.T > d.npos ||
        (int64_t)d.B * d.T > (1ll << 26)) {
        set_error(DPT_EINVAL, "train dims: L=%d E=%d F=%d A=%d B=%d T=%d npos=%d", d.L, d.E, d.F, d.A, d.B, d.T,
                  d.npos);
        return DPT_EINVAL;
    }
    return DPT_OK;
}

int64_t train_workspace_numel(const TrDims& d) { return TrWs::make(d).total; }
int64_t train_blob_numel(const TrDims& d) { return TrBlob::make(d).total; }

static int wgrad(const float* X, const float* dY, int R, int IN, int OUT, int gelu, float* part, float* dW,
                 float* db, hipStream_t st) {
    const int nch = (R + kTrRowsPerChunk - 1) / kTrRowsPerChunk;
    hipLaunchKernelGGL(tr_wgrad_part, dim3(nch, blocks_for((int64_t)(IN + 1) * OUT)), dim3(kTrThreads), 0, st, X, dY,
                       R, IN, OUT, gelu, part);
    reduce_parts(part, nch, IN, OUT, dW, db, st);
    return launched("tr_wgrad");
}

static int ln_param_grad(const float* x, const float* stt, const float* dy, int R, int E, float* part, float* dg,
                         float* db, hipStream_t st) {
    const int nch = (R + kTrRowsPerChunk - 1) / kTrRowsPerChunk;
    if (E <= 256)  // 256 / E row lanes per column (fixed-order LDS combine)
        hipLaunchKernelGGL(tr_ln_param_part2, dim3(nch), dim3(256), 0, st, x, stt, dy, R, E, part);
    else
        hipLaunchKernelGGL(tr_ln_param_part, dim3(nch, blocks_for(E)), dim3(kTrThreads), 0, st, x, stt, dy, R, E, part);
    // the (2, E) partials reduce like a bias-only weight gradient: IN = 1, OUT = E, [sum dy n | sum dy]
    reduce_parts(part, nch, 1, E, dg, db, st);
    return launched("tr_ln_param");
}

// ---- matrix-core dispatch (widths 16, 32, 64; other widths keep the row kernels)
static bool mm_fast(int E) { return E == 16 || E == 32 || E == 64; }
enum MmKind { kMmQkv, kMmProj, kMmFc, kMmMp, kMmBdMp, kMmBdFc, kMmBdProj, kMmBdQkv, kMmU, kMmLnQkv, kMmLnFc };

template <class Kern>
static void allow_lds(Kern k, size_t bytes) {
    if (bytes > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
template <int K, int N, bool TRANS, bool ACT, int EPI>
static void launch_mm(const float* X, const float* W, const float* bias, const float* res, const float* aux, int R,
                      float* Y, hipStream_t st) {
    const size_t lds = sizeof(float) * K * mm_ldb(K, N);
    allow_lds(tr_mm_rows<K, N, TRANS, ACT, EPI>, lds);
    // 4 waves (64 rows) per workgroup (1-wave workgroups for the decode rows of the generic-width
    // rollout were measured 2x slower: each stages the whole weight matrix for 16 rows)
    hipLaunchKernelGGL((tr_mm_rows<K, N, TRANS, ACT, EPI>), dim3((R + 63) / 64), dim3(256), lds, st, X, W, bias, res,
                       aux, R, Y);
}
// the layer's row products: forward (qkv, c_proj + residual, c_fc, gelu -> mlp.c_proj + residual)
// and the backward data products (dh = dx W_mp^T x gelu'(hpre), dy2 = dh W_fc^T, dout = dx2 W_proj^T,
// dy1 = dqkv W_attn^T); W in the blob's [in][out] layout
template <int E>
static void mm_kind(int kind, const float* X, const float* W, const float* bias, const float* res, const float* aux,
                    int R, float* Y, hipStream_t st) {
    switch (kind) {
        case kMmQkv: launch_mm<E, 3 * E, false, false, kMmBias>(X, W, bias, res, aux, R, Y, st); break;
        case kMmProj: launch_mm<E, E, false, false, kMmBias | kMmRes>(X, W, bias, res, aux, R, Y, st); break;
        case kMmFc: launch_mm<E, 4 * E, false, false, kMmBias>(X, W, bias, res, aux, R, Y, st); break;
        case kMmMp: launch_mm<4 * E, E, false, true, kMmBias | kMmRes>(X, W, bias, res, aux, R, Y, st); break;
        case kMmBdMp: launch_mm<E, 4 * E, true, false, kMmGeluGrad>(X, W, bias, res, aux, R, Y, st); break;
        case kMmBdFc: launch_mm<4 * E, E, true, false, 0>(X, W, bias, res, aux, R, Y, st); break;
        case kMmBdProj: launch_mm<E, E, true, false, 0>(X, W, bias, res, aux, R, Y, st); break;
        case kMmBdQkv: launch_mm<3 * E, E, true, false, 0>(X, W, bias, res, aux, R, Y, st); break;
        case kMmU: launch_mm<E, E, false, false, kMmBias>(X, W, bias, res, aux, R, Y, st); break;
        // X = the residual stream, aux = ln_g (ln_b follows): ln_1 -> c_attn and ln_2 -> c_fc in one pass
        case kMmLnQkv: launch_mm<E, 3 * E, false, false, kMmBias | kMmLnIn>(X, W, bias, res, aux, R, Y, st); break;
        case kMmLnFc: launch_mm<E, 4 * E, false, false, kMmBias | kMmLnIn>(X, W, bias, res, aux, R, Y, st); break;
    }
}
static void mm(int E, int kind, const float* X, const float* W, const float* bias, const float* res, const float* aux,
               int R, float* Y, hipStream_t st) {
    if (E == 16) mm_kind<16>(kind, X, W, bias, res, aux, R, Y, st);
    else if (E == 32) mm_kind<32>(kind, X, W, bias, res, aux, R, Y, st);
    else mm_kind<64>(kind, X, W, bias, res, aux, R, Y, st);
}
// the decode-row products of the generic rollout (R = N tasks, a few thousand rows): columns split so
// that the R / 64 row blocks times N / NC column slices fill the chip, NC = max(16, N / 4)
template <int K, int N, bool ACT, int EPI>
static void launch_mm_dec(const float* X, const float* W, const float* bias, const float* res, int R, float* Y,
                          hipStream_t st, const float* aux = nullptr) {
    constexpr int NC = N / 4 > 16 ? N / 4 : 16;
    const size_t lds = sizeof(float) * K * mm_ldb(K, NC);
    allow_lds(tr_mm_rows<K, N, false, ACT, EPI, NC>, lds);
    hipLaunchKernelGGL((tr_mm_rows<K, N, false, ACT, EPI, NC>), dim3((R + 63) / 64, N / NC), dim3(256), lds, st, X, W,
                       bias, res, aux, R, Y);
}
// LayerNorm on load at the widths whose row splits into a power-of-two count of float4 chunks per lane
// (tr_layernorm_rows' summation tree without its idle lanes)
static bool mm_ln_in_ok(int E) { return E == 16 || E == 32 || E == 64 || E == 128; }
template <int E>
static void mm_dec_kind(int kind, const float* X, const float* W, const float* bias, const float* res, int R, float* Y,
                        hipStream_t st, const float* aux = nullptr) {
    if constexpr (E == 16 || E == 32 || E == 64 || E == 128)
        if (kind == kMmLnFc) return launch_mm_dec<E, 4 * E, false, kMmBias | kMmLnIn>(X, W, bias, res, R, Y, st, aux);
    switch (kind) {
        case kMmU: launch_mm_dec<E, E, false, kMmBias>(X, W, bias, res, R, Y, st); break;
        case kMmProj: launch_mm_dec<E, E, false, kMmBias | kMmRes>(X, W, bias, res, R, Y, st); break;
        case kMmFc: launch_mm_dec<E, 4 * E, false, kMmBias>(X, W, bias, res, R, Y, st); break;
        case kMmMp: launch_mm_dec<4 * E, E, true, kMmBias | kMmRes>(X, W, bias, res, R, Y, st); break;
    }
}
static bool mm_dec_fast(int E) { return E == 16 || E == 32 || E == 48 || E == 64 || E == 128; }
static void mm_dec(int E, int kind, const float* X, const float* W, const float* bias, const float* res, int R,
                   float* Y, hipStream_t st, const float* aux = nullptr) {
    if (E == 16) mm_dec_kind<16>(kind, X, W, bias, res, R, Y, st, aux);
    else if (E == 32) mm_dec_kind<32>(kind, X, W, bias, res, R, Y, st, aux);
    else if (E == 48) mm_dec_kind<48>(kind, X, W, bias, res, R, Y, st, aux);
    else if (E == 64) mm_dec_kind<64>(kind, X, W, bias, res, R, Y, st, aux);
    else mm_dec_kind<128>(kind, X, W, bias, res, R, Y, st, aux);
}

template <int IN, int OUT, bool ACT>
static void launch_wg(const float* X, const float* dY, int R, float* part, hipStream_t st) {
    const size_t lds = sizeof(float) * kTrRowsPerChunk * (IN + 1 + OUT);
    allow_lds(tr_wgrad_mfma<IN, OUT, ACT>, lds);
    hipLaunchKernelGGL((tr_wgrad_mfma<IN, OUT, ACT>), dim3((R + kTrRowsPerChunk - 1) / kTrRowsPerChunk), dim3(256), lds,
                       st, X, dY, R, part);
}
// weight gradients of the layer's products: in = gelu(hpre) / y2 / o / y1, dY = dx / dh / dx2 / dqkv
template <int E>
static void wg_kind(int kind, const float* X, const float* dY, int R, float* part, hipStream_t st) {
    switch (kind) {
        case kMmMp: launch_wg<4 * E, E, true>(X, dY, R, part, st); break;
        case kMmFc: launch_wg<E, 4 * E, false>(X, dY, R, part, st); break;
        case kMmProj: launch_wg<E, E, false>(X, dY, R, part, st); break;
        case kMmQkv: launch_wg<E, 3 * E, false>(X, dY, R, part, st); break;
    }
}
static int wgrad_fast(int E, int kind, const float* X, const float* dY, int R, int IN, int OUT, float* part, float* dW,
                      float* db, hipStream_t st) {
    if (E == 16) wg_kind<16>(kind, X, dY, R, part, st);
    else if (E == 32) wg_kind<32>(kind, X, dY, R, part, st);
    else wg_kind<64>(kind, X, dY, R, part, st);
    const int nch = (R + kTrRowsPerChunk - 1) / kTrRowsPerChunk;
    reduce_parts(part, nch, IN, OUT, dW, db, st);
    return launched("tr_wgrad_mfma");
}

template <int E>
static void attn_fwd_e(const float* qkv, const TrDims& d, float* P, float* O, hipStream_t st) {
    hipLaunchKernelGGL(tr_attn_fwd_mfma<E>, dim3(d.B, (d.T + 63) / 64), dim3(256), 0, st, qkv, d, P, O);
}
static void attn_fwd_fast(int E, const float* qkv, const TrDims& d, float* P, float* O, hipStream_t st) {
    if (E == 16) attn_fwd_e<16>(qkv, d, P, O, st);
    else if (E == 32) attn_fwd_e<32>(qkv, d, P, O, st);
    else attn_fwd_e<64>(qkv, d, P, O, st);
}
template <int E>
static void attn_bwd_e(const float* qkv, const float* P, const float* O, const float* dO, const TrDims& d, float* dS,
                       float* dqkv, hipStream_t st) {
    const dim3 grid(d.B, (d.T + 63) / 64);
    hipLaunchKernelGGL(tr_attn_bwd_dq_mfma<E>, grid, dim3(256), 0, st, qkv, P, O, dO, d, dS, dqkv);
    hipLaunchKernelGGL(tr_attn_bwd_dkv_mfma<E>, grid, dim3(256), 0, st, qkv, P, dS, dO, d, dqkv);
}
static void attn_bwd_fast(int E, const float* qkv, const float* P, const float* O, const float* dO, const TrDims& d,
                          float* dS, float* dqkv, hipStream_t st) {
    if (E == 16) attn_bwd_e<16>(qkv, P, O, dO, d, dS, dqkv, st);
    else if (E == 32) attn_bwd_e<32>(qkv, P, O, dO, d, dS, dqkv, st);
    else attn_bwd_e<64>(qkv, P, O, dO, d, dS, dqkv, st);
}

// DPT_TRAIN_LAST_ONLY: the last block for the last position of each sequence alone.  One wave per
// sequence: the causal row of query T-1 over all T keys (tr_attn_fwd's arithmetic for that row).
__global__ void tr_attn_last(const float* __restrict__ qkv, TrDims d, float* __restrict__ O) {
    extern __shared__ float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x / 64) + wave;
    if (b >= d.B) return;
    const int T = d.T, E = d.E;
    float* pr = sm + (size_t)wave * (T + E);
    float* q = pr + T;
    const float* base = qkv + (int64_t)b * T * 3 * E;
    for (int e = lane; e < E; e += 64) q[e] = base[(int64_t)(T - 1) * 3 * E + e];
    wave_lds_sync();
    const float scale = 1.0f / sqrtf((float)E);
    float m = -INFINITY;
    for (int j = lane; j < T; j += 64) {
        const float* k = base + (int64_t)j * 3 * E + E;
        float s = 0.f;
        for (int e = 0; e < E; ++e) s = fmaf(q[e], k[e], s);
        s *= scale;
        pr[j] = s;
        m = fmaxf(m, s);
    }
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j < T; j += 64) {
        const float p = expf(pr[j] - m);
        pr[j] = p;
        l += p;
    }
    const float inv = 1.0f / wave_sum(l);
    wave_lds_sync();
    for (int e = lane; e < E; e += 64) {
        float acc = 0.f;
        for (int j = 0; j < T; ++j) acc = fmaf(pr[j], base[(int64_t)j * 3 * E + 2 * E + e], acc);
        O[(int64_t)b * E + e] = acc * inv;
    }
}
// dst[b][c] = src[(b T + T - 1)][c] (gather), or the reverse (scatter into the sequences' last rows)
__global__ void tr_last_rows(const float* __restrict__ src, float* __restrict__ dst, int B, int T, int C, int scatter) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * C) return;
    const int64_t b = i / C, c = i % C, r = (b * T + T - 1) * C + c;
    if (scatter) dst[r] = src[i];
    else dst[i] = src[r];
}

int train_forward(const TrDims& d, const float* blob, const float* tok, float* ws, float* preds, hipStream_t st) {
    if (int rc = train_dims_check(d)) return rc;
    const TrBlob B = TrBlob::make(d);
    const TrWs W = TrWs::make(d);
    const int R = d.R(), E = d.E;
    const int64_t RE = (int64_t)R * E, TT = (int64_t)d.B * d.T * TrWs::tpad(d.T);
    const int rows_per_block = kTrThreads / 64;
    const size_t attn_lds = sizeof(float) * rows_per_block * (size_t)(d.T + E);
    if ((!mm_fast(E) || d.drop()) && attn_lds > 160 * 1024) {
        set_error(DPT_EUNSUPPORTED, "train forward: window T=%d too long for the attention kernel", d.T);
        return DPT_EUNSUPPORTED;
    }
    if (attn_lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)tr_attn_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)attn_lds);
    hipLaunchKernelGGL(tr_embed, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, tok, blob, d, B, ws + W.x);
    // dropout (GPT2Model in training mode): drop(x0) in place, the attention probabilities, and
    // c_proj / mlp.c_proj outputs before their residual adds -- on the row kernels, which take the
    // masks (the matrix-core forms fuse the residual add)
    const bool drop = d.drop();
    if (drop) hipLaunchKernelGGL(tr_dropout, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, ws + W.x, nullptr, RE, d, 0,
                                 ws + W.x);
    // slot of layer l's arrays: l, or 0 (x: l & 1) in the forward-only workspace
    auto xs = [&](int l) -> int64_t { return d.fwd_only ? (l & 1) : l; };
    // DPT_TRAIN_LAST_ONLY (fwd_only == 3, no dropout, T > 1): the last block after its keys and values
    // for the last position of each sequence alone, then ln_f and the head on those rows
    const bool last_only = d.fwd_only == 3 && !drop && d.T > 1;
    for (int l = 0; l < d.L; ++l) {
        const TrLayer P = TrLayer::make(B.layers + l * d.layer_size(), E);
        const int64_t sl = d.fwd_only ? 0 : l;
        if (last_only && l == d.L - 1) {
            const float* x = ws + W.x + xs(l) * RE;
            float* y1 = ws + W.y1;
            float* qkv = ws + W.qkv;
            if (mm_fast(E)) {  // ln_1 on load (kMmLnQkv)
                mm(E, kMmLnQkv, x, blob + P.attn_w, blob + P.attn_b, nullptr, blob + P.ln1_g, R, qkv, st);
            } else {
                layernorm(x, blob + P.ln1_g, blob + P.ln1_b, R, E, y1, ws + W.st1, st);
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(RE * 3)), dim3(kTrThreads), 0, st, y1, blob + P.attn_w,
                                   blob + P.attn_b, nullptr, R, E, 3 * E, 0, qkv);
            }
            const int Bn = d.B;
            const int64_t BE = (int64_t)Bn * E;
            float* ol = ws + W.o;         // [B][E]
            float* xl = ws + W.y2;        // [B][E]: the last rows of x
            float* x2l = ws + W.x2;       // [B][E]
            float* y2l = ws + W.y1;       // [B][E] (y1 is done with)
            float* hl = ws + W.hpre;      // [B][4E]
            float* xnl = ws + W.x + xs(l + 1) * RE;  // [B][E]
            float* pl = ws + W.hpre + 4 * BE;        // [B][A] (4E (R - B) >= A B for T > 1)
            const size_t lds = sizeof(float) * rows_per_block * (size_t)(d.T + E);
            if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)tr_attn_last, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(tr_attn_last, dim3((Bn + rows_per_block - 1) / rows_per_block), dim3(kTrThreads), lds, st,
                               qkv, d, ol);
            hipLaunchKernelGGL(tr_last_rows, dim3(blocks_for(BE)), dim3(kTrThreads), 0, st, x, xl, Bn, d.T, E, 0);
            if (mm_fast(E)) {
                mm(E, kMmProj, ol, blob + P.proj_w, blob + P.proj_b, xl, nullptr, Bn, x2l, st);
            } else {
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(BE)), dim3(kTrThreads), 0, st, ol, blob + P.proj_w,
                                   blob + P.proj_b, xl, Bn, E, E, 0, x2l);
            }
            if (mm_fast(E)) {  // ln_2 on load (kMmLnFc)
                mm(E, kMmLnFc, x2l, blob + P.fc_w, blob + P.fc_b, nullptr, blob + P.ln2_g, Bn, hl, st);
                mm(E, kMmMp, hl, blob + P.mp_w, blob + P.mp_b, x2l, nullptr, Bn, xnl, st);
            } else {
                layernorm(x2l, blob + P.ln2_g, blob + P.ln2_b, Bn, E, y2l, ws + W.st2, st);
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(BE * 4)), dim3(kTrThreads), 0, st, y2l, blob + P.fc_w,
                                   blob + P.fc_b, nullptr, Bn, E, 4 * E, 0, hl);
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(BE)), dim3(kTrThreads), 0, st, hl, blob + P.mp_w,
                                   blob + P.mp_b, x2l, Bn, 4 * E, E, 1, xnl);
            }
            layernorm(xnl, blob + B.lnf_g, blob + B.lnf_b, Bn, E, ws + W.yf, ws + W.stf, st);
            hipLaunchKernelGGL(tr_linear, dim3(blocks_for((int64_t)Bn * d.A)), dim3(kTrThreads), 0, st, ws + W.yf,
                               blob + B.head_w, blob + B.head_b, nullptr, Bn, E, d.A, 0, pl);
            hipLaunchKernelGGL(tr_last_rows, dim3(blocks_for((int64_t)Bn * d.A)), dim3(kTrThreads), 0, st, pl, preds, Bn,
                               d.T, d.A, 1);
            return launched("train forward (last position only)");
        }
        const float* x = ws + W.x + xs(l) * RE;
        float* y1 = ws + W.y1 + sl * RE;
        float* st1 = ws + W.st1 + sl * R * 2;
        float* qkv = ws + W.qkv + sl * RE * 3;
        float* Pm = d.fwd_only ? nullptr : ws + W.P + sl * TT;
        float* o = ws + W.o + sl * RE;
        float* x2 = ws + W.x2 + sl * RE;
        float* y2 = ws + W.y2 + sl * RE;
        float* st2 = ws + W.st2 + sl * R * 2;
        float* hpre = ws + W.hpre + sl * RE * 4;
        float* xn = ws + W.x + xs(l + 1) * RE;
        const bool fast = mm_fast(E) && !drop;
        // forward only (nothing saved for a backward): ln_1 / ln_2 applied as the products load their rows
        const bool ln_in = fast && d.fwd_only;
        if (!ln_in) layernorm(x, blob + P.ln1_g, blob + P.ln1_b, R, E, y1, st1, st);
        if (ln_in)
            mm(E, kMmLnQkv, x, blob + P.attn_w, blob + P.attn_b, nullptr, blob + P.ln1_g, R, qkv, st);
        else if (fast)
            mm(E, kMmQkv, y1, blob + P.attn_w, blob + P.attn_b, nullptr, nullptr, R, qkv, st);
        else
            hipLaunchKernelGGL(tr_linear, dim3(blocks_for(RE * 3)), dim3(kTrThreads), 0, st, y1, blob + P.attn_w,
                               blob + P.attn_b, nullptr, R, E, 3 * E, 0, qkv);
        if (fast)
            attn_fwd_fast(E, qkv, d, Pm, o, st);
        else
            hipLaunchKernelGGL(tr_attn_fwd, dim3((R + rows_per_block - 1) / rows_per_block), dim3(kTrThreads), attn_lds,
                               st, qkv, d, drop ? 1 + 3 * l : -1, Pm, o);
        if (fast)
            mm(E, kMmProj, o, blob + P.proj_w, blob + P.proj_b, x, nullptr, R, x2, st);
        else
            hipLaunchKernelGGL(tr_linear, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, o, blob + P.proj_w,
                               blob + P.proj_b, drop ? nullptr : x, R, E, E, 0, x2);
        if (drop)  // x2 = x + drop(o W_proj + b_proj)
            hipLaunchKernelGGL(tr_dropout, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, x2, x, RE, d, 2 + 3 * l, x2);
        if (!ln_in) layernorm(x2, blob + P.ln2_g, blob + P.ln2_b, R, E, y2, st2, st);
        if (ln_in) {
            mm(E, kMmLnFc, x2, blob + P.fc_w, blob + P.fc_b, nullptr, blob + P.ln2_g, R, hpre, st);
            mm(E, kMmMp, hpre, blob + P.mp_w, blob + P.mp_b, x2, nullptr, R, xn, st);
        } else if (fast) {
            mm(E, kMmFc, y2, blob + P.fc_w, blob + P.fc_b, nullptr, nullptr, R, hpre, st);
            mm(E, kMmMp, hpre, blob + P.mp_w, blob + P.mp_b, x2, nullptr, R, xn, st);
        } else {
            hipLaunchKernelGGL(tr_linear, dim3(blocks_for(RE * 4)), dim3(kTrThreads), 0, st, y2, blob + P.fc_w,
                               blob + P.fc_b, nullptr, R, E, 4 * E, 0, hpre);
            hipLaunchKernelGGL(tr_linear, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, hpre, blob + P.mp_w,
                               blob + P.mp_b, drop ? nullptr : x2, R, 4 * E, E, 1, xn);
            if (drop)  // x_{l+1} = x2 + drop(gelu(hpre) W_mp + b_mp)
                hipLaunchKernelGGL(tr_dropout, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, xn, x2, RE, d, 3 + 3 * l,
                                   xn);
        }
        if (int rc = launched("train forward layer")) return rc;
    }
    layernorm(ws + W.x + xs(d.L) * RE, blob + B.lnf_g, blob + B.lnf_b, R, E, ws + W.yf, ws + W.stf, st);
    hipLaunchKernelGGL(tr_linear, dim3(blocks_for((int64_t)R * d.A)), dim3(kTrThreads), 0, st, ws + W.yf,
                       blob + B.head_w, blob + B.head_b, nullptr, R, E, d.A, 0, preds);
    return launched("train forward head");
}

int train_backward(const TrDims& d, const float* blob, const float* tok, float* ws, const float* dpreds,
                   float* dblob, hipStream_t st) {
    if (int rc = train_dims_check(d)) return rc;
    const TrBlob B = TrBlob::make(d);
    const TrWs W = TrWs::make(d);
    const int R = d.R(), E = d.E;
    const int64_t RE = (int64_t)R * E, TT = (int64_t)d.B * d.T * TrWs::tpad(d.T);
    const int rows_per_block = kTrThreads / 64;
    const unsigned row_blocks = (R + rows_per_block - 1) / rows_per_block;
    float* part = ws + W.part;
    float* dx = ws + W.dx;
    float* dx2 = ws + W.dx2;
    float* dy = ws + W.dy;
    if (int rc = check_hip(hipMemsetAsync(dblob, 0, sizeof(float) * B.total, st), "dblob memset")) return rc;
    // head: preds = yf head_w + head_b
    if (int rc = wgrad(ws + W.yf, dpreds, R, E, d.A, 0, part, dblob + B.head_w, dblob + B.head_b, st)) return rc;
    hipLaunchKernelGGL(tr_linear_bwd_data, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dpreds, blob + B.head_w, R, E,
                       d.A, nullptr, nullptr, dy);
    // ln_f
    if (int rc = ln_param_grad(ws + W.x + d.L * RE, ws + W.stf, dy, R, E, part, dblob + B.lnf_g, dblob + B.lnf_b, st))
        return rc;
    hipLaunchKernelGGL(tr_layernorm_bwd, dim3(row_blocks), dim3(kTrThreads), 0, st, ws + W.x + d.L * RE, ws + W.stf,
                       blob + B.lnf_g, dy, R, E, nullptr, dx);
    const size_t ds_lds = sizeof(float) * rows_per_block * (size_t)E;
    const bool drop = d.drop();
    for (int l = d.L - 1; l >= 0; --l) {
        const TrLayer P = TrLayer::make(B.layers + l * d.layer_size(), E);
        const TrLayer G = TrLayer::make(B.layers + l * d.layer_size(), E);  // same offsets in dblob
        const float* x = ws + W.x + l * RE;
        const float* y1 = ws + W.y1 + l * RE;
        const float* st1 = ws + W.st1 + (int64_t)l * R * 2;
        const float* qkv = ws + W.qkv + l * RE * 3;
        const float* Pm = ws + W.P + l * TT;
        const float* o = ws + W.o + l * RE;
        const float* x2 = ws + W.x2 + l * RE;
        const float* y2 = ws + W.y2 + l * RE;
        const float* st2 = ws + W.st2 + (int64_t)l * R * 2;
        const float* hpre = ws + W.hpre + l * RE * 4;
        float* dh = ws + W.dh;
        float* dqkv = ws + W.dqkv;
        float* dout = ws + W.dout;
        float* dS = ws + W.dS;
        const bool fast = mm_fast(E) && !drop;
        // MLP: x_{l+1} = x2 + drop(gelu(hpre) W_mp + b_mp), hpre = y2 W_fc + b_fc; with dropout the
        // product's gradient dx keep (into dy, free until the LayerNorm input gradient below)
        const float* dmp = dx;
        if (drop) {
            hipLaunchKernelGGL(tr_dropout, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dx, nullptr, RE, d, 3 + 3 * l,
                               dy);
            dmp = dy;
        }
        if (fast) {
            if (int rc = wgrad_fast(E, kMmMp, hpre, dx, R, 4 * E, E, part, dblob + G.mp_w, dblob + G.mp_b, st)) return rc;
            mm(E, kMmBdMp, dx, blob + P.mp_w, nullptr, nullptr, hpre, R, dh, st);
            if (int rc = wgrad_fast(E, kMmFc, y2, dh, R, E, 4 * E, part, dblob + G.fc_w, dblob + G.fc_b, st)) return rc;
            mm(E, kMmBdFc, dh, blob + P.fc_w, nullptr, nullptr, nullptr, R, dy, st);
        } else {
            if (int rc = wgrad(hpre, dmp, R, 4 * E, E, 1, part, dblob + G.mp_w, dblob + G.mp_b, st)) return rc;
            hipLaunchKernelGGL(tr_linear_bwd_data, dim3(blocks_for(RE * 4)), dim3(kTrThreads), 0, st, dmp, blob + P.mp_w,
                               R, 4 * E, E, hpre, nullptr, dh);
            if (int rc = wgrad(y2, dh, R, E, 4 * E, 0, part, dblob + G.fc_w, dblob + G.fc_b, st)) return rc;
            hipLaunchKernelGGL(tr_linear_bwd_data, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dh, blob + P.fc_w, R,
                               E, 4 * E, nullptr, nullptr, dy);
        }
        if (int rc = ln_param_grad(x2, st2, dy, R, E, part, dblob + G.ln2_g, dblob + G.ln2_b, st)) return rc;
        hipLaunchKernelGGL(tr_layernorm_bwd, dim3(row_blocks), dim3(kTrThreads), 0, st, x2, st2, blob + P.ln2_g, dy, R, E,
                           dx, dx2);
        // attention: x2 = x + drop(o W_proj + b_proj)
        const float* dpj = dx2;
        if (drop) {
            hipLaunchKernelGGL(tr_dropout, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dx2, nullptr, RE, d, 2 + 3 * l,
                               dy);
            dpj = dy;
        }
        if (fast) {
            if (int rc = wgrad_fast(E, kMmProj, o, dx2, R, E, E, part, dblob + G.proj_w, dblob + G.proj_b, st)) return rc;
            mm(E, kMmBdProj, dx2, blob + P.proj_w, nullptr, nullptr, nullptr, R, dout, st);
        } else {
            if (int rc = wgrad(o, dpj, R, E, E, 0, part, dblob + G.proj_w, dblob + G.proj_b, st)) return rc;
            hipLaunchKernelGGL(tr_linear_bwd_data, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dpj, blob + P.proj_w,
                               R, E, E, nullptr, nullptr, dout);
        }
        if (fast) {
            attn_bwd_fast(E, qkv, Pm, o, dout, d, dS, dqkv, st);
        } else {
            const int site = drop ? 1 + 3 * l : -1;
            hipLaunchKernelGGL(tr_attn_bwd_ds, dim3(row_blocks), dim3(kTrThreads), ds_lds, st, qkv, Pm, o, dout, d, site,
                               dS);
            hipLaunchKernelGGL(tr_attn_bwd_dq, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, qkv, dS, d, dqkv);
            hipLaunchKernelGGL(tr_attn_bwd_dkv, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, qkv, Pm, dS, dout, d, site,
                               dqkv);
        }
        if (fast) {
            if (int rc = wgrad_fast(E, kMmQkv, y1, dqkv, R, E, 3 * E, part, dblob + G.attn_w, dblob + G.attn_b, st))
                return rc;
            mm(E, kMmBdQkv, dqkv, blob + P.attn_w, nullptr, nullptr, nullptr, R, dy, st);
        } else {
            if (int rc = wgrad(y1, dqkv, R, E, 3 * E, 0, part, dblob + G.attn_w, dblob + G.attn_b, st)) return rc;
            hipLaunchKernelGGL(tr_linear_bwd_data, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dqkv, blob + P.attn_w,
                               R, E, 3 * E, nullptr, nullptr, dy);
        }
        if (int rc = ln_param_grad(x, st1, dy, R, E, part, dblob + G.ln1_g, dblob + G.ln1_b, st)) return rc;
        hipLaunchKernelGGL(tr_layernorm_bwd, dim3(row_blocks), dim3(kTrThreads), 0, st, x, st1, blob + P.ln1_g, dy, R, E,
                           dx2, dx);
        if (int rc = launched("train backward layer")) return rc;
    }
    // embedding: x0 = drop(tok emb_w + emb_b + wpe[t])
    if (drop) hipLaunchKernelGGL(tr_dropout, dim3(blocks_for(RE)), dim3(kTrThreads), 0, st, dx, nullptr, RE, d, 0, dx);
    if (int rc = wgrad(tok, dx, R, d.F, E, 0, part, dblob + B.emb_w, dblob + B.emb_b, st)) return rc;
    hipLaunchKernelGGL(tr_wpe_grad, dim3(blocks_for((int64_t)d.T * E)), dim3(kTrThreads), 0, st, dx, d, dblob + B.wpe);
    return launched("train backward embed");
}

// ------------------------------------------------------------------------------ generic-width rollout
// The bandit online loop (evals/eval_bandit.py:56-103: decode -> select -> env step -> append the
// transition) at ANY width, for models the fused E = 32 kernel (dpt_decode.hip) is not built for.
// Exact K/V-cache decode: the bandit's query token sits at position 0 and never changes, and the
// prediction is read at the last position, so every earlier position's keys and values stay
// valid (causal attention) and a step computes the new token only.  The cache holds each block's
// LayerNorm output y instead of K and V (the folded attention, GenFold): half the bytes.  One pass per step over all N
// tasks: embed, then per layer the training forward's row kernels (or their matrix-core forms at
// widths 16 / 32 / 64) on N rows, the attention of the new token over the task's cache, ln_f and
// the head; then selection and the env step with the draws and arithmetic of the fused kernel.
// Folded attention (the fused kernels' algebra, dpt_decode.hip): with y_p = LN1(x_p) a block's keys
// and values are affine in y_p, so q . k_p = u . y_p + const (u = q W_k^T = y G + g0, G = W_q W_k^T,
// g0 = b_q W_k^T; the constant shifts every score of the row equally and cancels in the softmax) and
// sum_p P_p v_p = (sum_p P_p y_p) W_v + b_v, so c_proj takes the attention-weighted y on
// Wvp = W_v W_proj with bvp = b_v W_proj + b_proj.  The cache holds y alone: E floats per position
// and layer instead of K and V's 2E.  Per layer [G | Wvp | g0 | bvp], [in][out], fp64 sums.
struct GenFold {
    __host__ __device__ static int64_t size(int E) { return 2ll * E * E + 2 * E; }
};
__global__ void gen_fold_kernel(const float* __restrict__ blob, TrDims d, TrBlob b, float* __restrict__ fold) {
    const int E = d.E;
    const int64_t per = GenFold::size(E), total = (int64_t)d.L * per;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int l = (int)(i / per);
        const int64_t o = i % per;
        const TrLayer P = TrLayer::make(b.layers + l * d.layer_size(), E);
        const float* Wa = blob + P.attn_w;  // [E][3E]: columns q | k | v
        const float* ba = blob + P.attn_b;
        const float* Wp = blob + P.proj_w;  // [E][E]
        double acc = 0.0;
        if (o < (int64_t)E * E) {  // G[r][c] = sum_k Wq[r][k] Wk[c][k]
            const int r = (int)(o / E), c = (int)(o % E);
            for (int k = 0; k < E; ++k) acc += (double)Wa[(int64_t)r * 3 * E + k] * Wa[(int64_t)c * 3 * E + E + k];
        } else if (o < 2ll * E * E) {  // Wvp[r][c] = sum_k Wv[r][k] Wp[k][c]
            const int64_t oo = o - (int64_t)E * E;
            const int r = (int)(oo / E), c = (int)(oo % E);
            for (int k = 0; k < E; ++k) acc += (double)Wa[(int64_t)r * 3 * E + 2 * E + k] * Wp[(int64_t)k * E + c];
        } else if (o < 2ll * E * E + E) {  // g0[c] = sum_k bq[k] Wk[c][k]
            const int c = (int)(o - 2ll * E * E);
            for (int k = 0; k < E; ++k) acc += (double)ba[k] * Wa[(int64_t)c * 3 * E + E + k];
        } else {  // bvp[c] = sum_k bv[k] Wp[k][c] + bp[c]
            const int c = (int)(o - 2ll * E * E - E);
            for (int k = 0; k < E; ++k) acc += (double)ba[2 * E + k] * Wp[(int64_t)k * E + c];
            acc += blob[P.proj_b + c];
        }
        fold[i] = (float)acc;
    }
}

// Workspace (floats): the y cache [L][N][H][E], the folded weights, then per-step rows.
struct GenWs {
    int64_t Y, fold, x, x2, y, st, qkv, o, h, lg, tok, total;
    static GenWs make(const TrDims& d, int N, int H) {
        GenWs w;
        const int64_t E = d.E, n = N, cache = (int64_t)d.L * n * H * E;
        int64_t p = 0;
        auto take = [&](int64_t k) { const int64_t at = p; p += k; p = (p + 3) & ~3ll; return at; };
        w.Y = take(cache);
        w.fold = take((int64_t)d.L * GenFold::size(d.E));
        w.x = take(n * E);
        w.x2 = take(n * E);
        w.y = take(n * E);
        w.st = take(n * 2);
        w.qkv = take(n * 3 * E);
        w.o = take(n * E);
        w.h = take(n * 4 * E);
        w.lg = take(n * d.A);
        w.tok = take(n * d.F);
        w.total = p;
        return w;
    }
};

// x[n][e] = tok[n] emb_w + emb_b + wpe[pos]: the new token of every task (tr_embed's order)
__global__ void gen_embed(const float* __restrict__ tok, const float* __restrict__ blob, TrDims d, TrBlob b, int N,
                          int pos, float* __restrict__ x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)N * d.E) return;
    const int n = (int)(i / d.E), e = (int)(i % d.E);
    float acc = blob[b.emb_b + e];
    for (int f = 0; f < d.F; ++f) acc = fmaf(tok[(int64_t)n * d.F + f], blob[b.emb_w + (int64_t)f * d.E + e], acc);
    x[i] = acc + blob[b.wpe + (int64_t)pos * d.E + e];
}

// One wave per task: store the new token's key and value at position pos of the task's cache
// (rows [pos][E] of [N][H][E]) and attend over positions 0..pos -- tr_attn_fwd's arithmetic for the
// causal row of the new token (the new key and value are read from the qkv row itself).
__global__ void gen_attn_decode(const float* __restrict__ qkv, float* __restrict__ Kc, float* __restrict__ Vc, int E,
                                int N, int H, int pos, float* __restrict__ O) {
    extern __shared__ float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int task = blockIdx.x * (blockDim.x / 64) + wave;
    if (task >= N) return;
    float* pr = sm + (size_t)wave * (H + E);
    float* q = pr + H;
    const float* row = qkv + (int64_t)task * 3 * E;
    float* K = Kc + (int64_t)task * H * E;
    float* V = Vc + (int64_t)task * H * E;
    for (int e = lane; e < E; e += 64) {
        q[e] = row[e];
        K[(int64_t)pos * E + e] = row[E + e];
        V[(int64_t)pos * E + e] = row[2 * E + e];
    }
    wave_lds_sync();
    const float scale = 1.0f / sqrtf((float)E);
    float m = -INFINITY;
    for (int j = lane; j <= pos; j += 64) {
        const float* k = j == pos ? row + E : K + (int64_t)j * E;
        float s = 0.f;
        for (int e = 0; e < E; ++e) s = fmaf(q[e], k[e], s);
        s *= scale;
        pr[j] = s;
        m = fmaxf(m, s);
    }
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j <= pos; j += 64) {
        const float p = expf(pr[j] - m);
        pr[j] = p;
        l += p;
    }
    const float inv = 1.0f / wave_sum(l);
    for (int j = lane; j <= pos; j += 64) pr[j] *= inv;
    wave_lds_sync();
    for (int e = lane; e < E; e += 64) {
        float acc = 0.f;
        for (int j = 0; j < pos; ++j) acc = fmaf(pr[j], V[(int64_t)j * E + e], acc);
        acc = fmaf(pr[pos], row[2 * E + e], acc);
        O[(int64_t)task * E + e] = acc;
    }
}

// gen_attn_decode in the folded-attention form (GenFold): u scores the cached y rows (and the new
// position's own y, at yn), the output is the attention-weighted y (c_proj runs on Wvp)
__global__ void gen_attn_ydecode(const float* __restrict__ u, const float* __restrict__ yn, float* __restrict__ Yc,
                                 int E, int N, int H, int pos, float* __restrict__ O) {
    extern __shared__ float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int task = blockIdx.x * (blockDim.x / 64) + wave;
    if (task >= N) return;
    float* pr = sm + (size_t)wave * (H + E);
    float* q = pr + H;
    const float* row = yn + (int64_t)task * E;
    float* Y = Yc + (int64_t)task * H * E;
    for (int e = lane; e < E; e += 64) {
        q[e] = u[(int64_t)task * E + e];
        Y[(int64_t)pos * E + e] = row[e];
    }
    wave_lds_sync();
    const float scale = 1.0f / sqrtf((float)E);
    float m = -INFINITY;
    for (int j = lane; j <= pos; j += 64) {
        const float* k = j == pos ? row : Y + (int64_t)j * E;
        float s = 0.f;
        for (int e = 0; e < E; ++e) s = fmaf(q[e], k[e], s);
        s *= scale;
        pr[j] = s;
        m = fmaxf(m, s);
    }
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j <= pos; j += 64) {
        const float p = expf(pr[j] - m);
        pr[j] = p;
        l += p;
    }
    const float inv = 1.0f / wave_sum(l);
    for (int j = lane; j <= pos; j += 64) pr[j] *= inv;
    wave_lds_sync();
    for (int e = lane; e < E; e += 64) {
        float acc = 0.f;
        for (int j = 0; j < pos; ++j) acc = fmaf(pr[j], Y[(int64_t)j * E + e], acc);
        acc = fmaf(pr[pos], row[e], acc);
        O[(int64_t)task * E + e] = acc;
    }
}

// The same for E % 4 == 0, E <= 256, with the rows read as float4: LPK lanes per key (a power of
// two >= E / 4), 64 / LPK keys per wave-instruction, so every key row is one coalesced read.  Scores
// are 4-term partial dots summed over the key's lanes by xor shuffles; the values accumulate per
// lane group (keys kq, kq + KPW, ...) and the groups are summed at the end: a different fp32
// order than gen_attn_decode (and tr_attn_fwd), the same softmax.
template <int LPK>
__global__ void gen_attn_decode4(const float* __restrict__ qkv, float* __restrict__ Kc, float* __restrict__ Vc, int E,
                                 int N, int H, int pos, float* __restrict__ O) {
    constexpr int KPW = 64 / LPK;
    extern __shared__ float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int task = blockIdx.x * (blockDim.x / 64) + wave;
    if (task >= N) return;
    float* pr = sm + (size_t)wave * H;
    const int E4 = E >> 2, c = lane % LPK, kq = lane / LPK;
    const bool act = c < E4;
    const float* row = qkv + (int64_t)task * 3 * E;
    const floatx4* K4 = reinterpret_cast<const floatx4*>(Kc + (int64_t)task * H * E);
    const floatx4* V4 = reinterpret_cast<const floatx4*>(Vc + (int64_t)task * H * E);
    const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
    const floatx4 q = act ? reinterpret_cast<const floatx4*>(row)[c] : zero;
    const floatx4 kn = act ? reinterpret_cast<const floatx4*>(row + E)[c] : zero;
    const floatx4 vn = act ? reinterpret_cast<const floatx4*>(row + 2 * E)[c] : zero;
    if (kq == 0 && act) {
        reinterpret_cast<floatx4*>(Kc + (int64_t)task * H * E)[(int64_t)pos * E4 + c] = kn;
        reinterpret_cast<floatx4*>(Vc + (int64_t)task * H * E)[(int64_t)pos * E4 + c] = vn;
    }
    const float scale = 1.0f / sqrtf((float)E);
    float m = -INFINITY;
    for (int jb = 0; jb <= pos; jb += KPW) {
        const int j = jb + kq;
        floatx4 k = zero;
        if (act && j < pos) k = K4[(int64_t)j * E4 + c];
        else if (act && j == pos) k = kn;
        float d = fmaf(q[0], k[0], fmaf(q[1], k[1], fmaf(q[2], k[2], q[3] * k[3])));
#pragma unroll
        for (int x = 1; x < LPK; x <<= 1) d += __shfl_xor(d, x, 64);
        if (j <= pos) {
            d *= scale;
            if (c == 0) pr[j] = d;
            m = fmaxf(m, d);
        }
    }
    m = wave_max(m);
    wave_lds_sync();
    float l = 0.f;
    for (int j = lane; j <= pos; j += 64) {
        const float p = expf(pr[j] - m);
        pr[j] = p;
        l += p;
    }
    const float inv = 1.0f / wave_sum(l);
    wave_lds_sync();
    floatx4 acc = zero;
    for (int jb = 0; jb <= pos; jb += KPW) {
        const int j = jb + kq;
        if (!act || j > pos) continue;
        const floatx4 v = j == pos ? vn : V4[(int64_t)j * E4 + c];
        const float p = pr[j];
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaf(p, v[r], acc[r]);
    }
#pragma unroll
    for (int x = LPK; x < 64; x <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += __shfl_xor(acc[r], x, 64);
    if (kq == 0 && act) reinterpret_cast<floatx4*>(O + (int64_t)task * E)[c] = acc * inv;
}

// The folded-attention form of gen_attn_decode4 (GenFold), one pass over the y cache (flash decoding):
// lane group kq takes keys kq, kq + KPW, ... (LPK lanes per key, one float4 of the row each), kU keys
// of the group per iteration (kU rows in flight per lane), and keeps its own softmax state (m, l, acc)
// in the exp2 domain; the KPW groups are merged at the end by xor shuffles.  Each y row is read once
// (the two-pass form read it for the scores and again for the weighted sum).  No LDS.
template <int LPK>
__global__ void gen_attn_ydecode4(const float* __restrict__ u, const float* __restrict__ yn, float* __restrict__ Yc,
                                  int E, int N, int H, int pos, float* __restrict__ O) {
    constexpr int KPW = 64 / LPK, kU = 4;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int task = blockIdx.x * (blockDim.x / 64) + wave;
    if (task >= N) return;
    const int E4 = E >> 2, c = lane % LPK, kq = lane / LPK;
    const bool act = c < E4;
    const floatx4* Y4 = reinterpret_cast<const floatx4*>(Yc + (int64_t)task * H * E);
    const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
    const floatx4 q = act ? reinterpret_cast<const floatx4*>(u + (int64_t)task * E)[c] : zero;
    const floatx4 yv = act ? reinterpret_cast<const floatx4*>(yn + (int64_t)task * E)[c] : zero;
    if (kq == 0 && act) reinterpret_cast<floatx4*>(Yc + (int64_t)task * H * E)[(int64_t)pos * E4 + c] = yv;
    const float scale = 1.4426950408889634f / sqrtf((float)E);  // scores in the exp2 domain
    float m = -INFINITY, l = 0.f;
    floatx4 acc = zero;
    for (int jb = 0; jb <= pos; jb += KPW * kU) {
        floatx4 v[kU];
        float sc[kU];
#pragma unroll
        for (int t = 0; t < kU; ++t) {
            const int j = jb + t * KPW + kq;
            v[t] = zero;
            if (act && j < pos) v[t] = Y4[(int64_t)j * E4 + c];
            else if (act && j == pos) v[t] = yv;
        }
        float mn = m;
#pragma unroll
        for (int t = 0; t < kU; ++t) {
            const int j = jb + t * KPW + kq;
            float d = fmaf(q[0], v[t][0], fmaf(q[1], v[t][1], fmaf(q[2], v[t][2], q[3] * v[t][3])));
#pragma unroll
            for (int x = 1; x < LPK; x <<= 1) d += __shfl_xor(d, x, 64);
            sc[t] = j <= pos ? d * scale : -INFINITY;
            mn = fmaxf(mn, sc[t]);
        }
        if (mn == -INFINITY) continue;  // no key of this group in the chunk yet
        const float corr = exp2f(m - mn);  // 0 while m = -inf
        l *= corr;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] *= corr;
#pragma unroll
        for (int t = 0; t < kU; ++t) {
            const float p = exp2f(sc[t] - mn);
            l += p;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = fmaf(p, v[t][r], acc[r]);
        }
        m = mn;
    }
    // merge the KPW groups' states (every group but kq = 0 may be empty: m = -inf, l = 0)
#pragma unroll
    for (int x = LPK; x < 64; x <<= 1) {
        const float mo = __shfl_xor(m, x, 64), lo = __shfl_xor(l, x, 64);
        floatx4 ao;
#pragma unroll
        for (int r = 0; r < 4; ++r) ao[r] = __shfl_xor(acc[r], x, 64);
        const float mm = fmaxf(m, mo);
        const float ca = m == -INFINITY ? 0.f : exp2f(m - mm), cb = mo == -INFINITY ? 0.f : exp2f(mo - mm);
        l = l * ca + lo * cb;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = acc[r] * ca + ao[r] * cb;
        m = mm;
    }
    if (kq == 0 && act) reinterpret_cast<floatx4*>(O + (int64_t)task * E)[c] = acc * (1.0f / l);
}

struct GenEnv {
    int N, H, A, sd, type, sample;
    int64_t first_task;
    double var;
    uint64_t seed, counter;
    const double* means;
    const double* uniforms;
    const double* noise;
    int32_t* actions_out;
    double* rewards_out;
    double* arm_value_out;
    float* logits_out;
};

// the token rows: the query [1_sd, 0_A, 0_sd, 0] at step 0 (eval_bandit.py: query state ones)
__global__ void gen_query_token(int N, int F, int sd, float* __restrict__ tok) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)N * F) return;
    tok[i] = (int)(i % F) < sd ? 1.f : 0.f;
}

// selection and env step of step h for every task (the fused kernel's draws, select_from_logits
// and reward arithmetic), the outputs, and the next token [1_sd, onehot(a), 1_sd, float(r)]
// (eval_bandit.py:83-86)
__global__ void gen_select_env(const float* __restrict__ lg, GenEnv g, int h, float* __restrict__ tok) {
    const int task = blockIdx.x * blockDim.x + threadIdx.x;
    if (task >= g.N) return;
    const int64_t gtask = g.first_task + task;
    const uint64_t ctr = g.counter + (uint64_t)h;
    double u = 0.0;
    if (g.sample) u = g.uniforms ? g.uniforms[(size_t)h * g.N + task] : philox_uniform(g.seed, ctr, gtask, DPT_STREAM_SELECT);
    const float* l = lg + (int64_t)task * g.A;
    const int a = select_from_logits(l, g.A, g.sample, 1.0f, u);
    const double mean = g.means[(int64_t)task * g.A + a];
    double dr;
    if (g.noise) dr = g.noise[(size_t)h * g.N + task];
    else if (g.type == DPT_BANDIT_BERNOULLI) dr = philox_uniform(g.seed, ctr, gtask, DPT_STREAM_REWARD);
    else dr = philox_normal(g.seed, ctr, gtask, DPT_STREAM_REWARD);
    const double r = g.type == DPT_BANDIT_BERNOULLI ? (dr < mean ? 1.0 : 0.0) : gaussian_reward(mean, g.var, dr);
    const size_t o = (size_t)task * g.H + h;
    g.actions_out[o] = a;
    g.rewards_out[o] = r;
    g.arm_value_out[o] = mean;
    if (g.logits_out)
        for (int k = 0; k < g.A; ++k) g.logits_out[((size_t)h * g.N + task) * g.A + k] = l[k];
    const int F = 2 * g.sd + g.A + 1;
    float* t = tok + (int64_t)task * F;
    for (int k = 0; k < g.sd; ++k) t[k] = 1.f;
    for (int k = 0; k < g.A; ++k) t[g.sd + k] = k == a ? 1.f : 0.f;
    for (int k = 0; k < g.sd; ++k) t[g.sd + g.A + k] = 1.f;
    t[F - 1] = (float)r;
}

int64_t gen_rollout_workspace_numel(const TrDims& d, int N, int H) { return GenWs::make(d, N, H).total; }

int rollout_bandit_generic(const TrDims& d, const float* blob, const dpt_bandit_rollout_args& a, hipStream_t st) {
    if (int rc = train_dims_check(d)) return rc;
    if (a.A != d.A || d.F != 2 + a.A + 1 || a.H > d.npos || a.N < 1 || a.H < 1 ||
        (a.type != DPT_BANDIT_GAUSSIAN && a.type != DPT_BANDIT_BERNOULLI) || a.kvcache == nullptr || a.means == nullptr ||
        a.actions_out == nullptr || a.rewards_out == nullptr || a.arm_value_out == nullptr) {
        set_error(DPT_EINVAL, "generic bandit rollout: A=%d (model %d), state_dim must be 1, H=%d (n_positions %d), type=%d",
                  a.A, d.A, a.H, d.npos, a.type);
        return DPT_EINVAL;
    }
    const int N = a.N, H = a.H, E = d.E, L = d.L;
    const TrBlob B = TrBlob::make(d);
    const GenWs W = GenWs::make(d, N, H);
    float* ws = a.kvcache;
    const int rows_per_block = kTrThreads / 64;
    const unsigned row_blocks = (N + rows_per_block - 1) / rows_per_block;
    // the float4 attention for E % 4 == 0 up to 256 (LPK lanes per key), else the scalar one
    const int lpk = E % 4 ? 0 : E <= 16 ? 4 : E <= 32 ? 8 : E <= 64 ? 16 : E <= 128 ? 32 : E <= 256 ? 64 : 0;
    const void* attn_k = lpk == 4    ? (const void*)gen_attn_ydecode4<4>
                         : lpk == 8  ? (const void*)gen_attn_ydecode4<8>
                         : lpk == 16 ? (const void*)gen_attn_ydecode4<16>
                         : lpk == 32 ? (const void*)gen_attn_ydecode4<32>
                         : lpk == 64 ? (const void*)gen_attn_ydecode4<64>
                                     : (const void*)gen_attn_ydecode;
    const size_t attn_lds = lpk ? 0 : sizeof(float) * rows_per_block * (size_t)(H + E);  // (the float4 form: none)
    if (attn_lds > 160 * 1024) {
        set_error(DPT_EUNSUPPORTED, "generic bandit rollout: H=%d too long for the attention kernel", H);
        return DPT_EUNSUPPORTED;
    }
    if (attn_lds > 64 * 1024) (void)hipFuncSetAttribute(attn_k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)attn_lds);
    GenEnv g{N, H, a.A, 1, a.type, a.sample, a.first_task, a.var, a.seed, a.counter, a.means, a.uniforms, a.noise,
             a.actions_out, a.rewards_out, a.arm_value_out, a.logits_out};
    const bool fast = mm_dec_fast(E);  // the column-split matrix-core products (mm_dec)
    float* x = ws + W.x;
    float* x2 = ws + W.x2;
    float* y = ws + W.y;
    float* stt = ws + W.st;
    float* qkv = ws + W.qkv;
    float* o = ws + W.o;
    float* hb = ws + W.h;
    const int64_t NE = (int64_t)N * E, cache = (int64_t)N * H * E;
    hipLaunchKernelGGL(gen_query_token, dim3(blocks_for((int64_t)N * d.F)), dim3(kTrThreads), 0, st, N, d.F, 1,
                       ws + W.tok);
    hipLaunchKernelGGL(gen_fold_kernel, dim3(blocks_for((int64_t)L * GenFold::size(E))), dim3(kTrThreads), 0, st, blob, d,
                       B, ws + W.fold);
    for (int h = 0; h < H; ++h) {
        hipLaunchKernelGGL(gen_embed, dim3(blocks_for(NE)), dim3(kTrThreads), 0, st, ws + W.tok, blob, d, B, N, h, x);
        for (int l = 0; l < L; ++l) {
            const TrLayer P = TrLayer::make(B.layers + l * d.layer_size(), E);
            layernorm(x, blob + P.ln1_g, blob + P.ln1_b, N, E, y, stt, st);
            // u = y G + g0, the folded attention over the y cache, c_proj on Wvp (GenFold)
            const float* F = ws + W.fold + l * GenFold::size(E);
            const float *G = F, *Wvp = F + (int64_t)E * E, *g0 = F + 2ll * E * E, *bvp = g0 + E;
            float* uq = qkv;
            if (fast)
                mm_dec(E, kMmU, y, G, g0, nullptr, N, uq, st);
            else
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(NE)), dim3(kTrThreads), 0, st, y, G, g0, nullptr, N, E, E, 0,
                                   uq);
            float* Yc = ws + W.Y + l * cache;
            switch (lpk) {
                case 4: hipLaunchKernelGGL(gen_attn_ydecode4<4>, dim3(row_blocks), dim3(kTrThreads), attn_lds, st, uq, y, Yc, E, N, H, h, o); break;
                case 8: hipLaunchKernelGGL(gen_attn_ydecode4<8>, dim3(row_blocks), dim3(kTrThreads), attn_lds, st, uq, y, Yc, E, N, H, h, o); break;
                case 16: hipLaunchKernelGGL(gen_attn_ydecode4<16>, dim3(row_blocks), dim3(kTrThreads), attn_lds, st, uq, y, Yc, E, N, H, h, o); break;
                case 32: hipLaunchKernelGGL(gen_attn_ydecode4<32>, dim3(row_blocks), dim3(kTrThreads), attn_lds, st, uq, y, Yc, E, N, H, h, o); break;
                case 64: hipLaunchKernelGGL(gen_attn_ydecode4<64>, dim3(row_blocks), dim3(kTrThreads), attn_lds, st, uq, y, Yc, E, N, H, h, o); break;
                default: hipLaunchKernelGGL(gen_attn_ydecode, dim3(row_blocks), dim3(kTrThreads), attn_lds, st, uq, y, Yc, E, N, H, h, o);
            }
            if (fast)
                mm_dec(E, kMmProj, o, Wvp, bvp, x, N, x2, st);
            else
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(NE)), dim3(kTrThreads), 0, st, o, Wvp, bvp, x, N, E, E, 0, x2);
            if (fast && mm_ln_in_ok(E)) {  // ln_2 on load (bit-identical to the separate LayerNorm)
                mm_dec(E, kMmLnFc, x2, blob + P.fc_w, blob + P.fc_b, nullptr, N, hb, st, blob + P.ln2_g);
                mm_dec(E, kMmMp, hb, blob + P.mp_w, blob + P.mp_b, x2, N, x, st);
            } else if (fast) {
                layernorm(x2, blob + P.ln2_g, blob + P.ln2_b, N, E, y, stt, st);
                mm_dec(E, kMmFc, y, blob + P.fc_w, blob + P.fc_b, nullptr, N, hb, st);
                mm_dec(E, kMmMp, hb, blob + P.mp_w, blob + P.mp_b, x2, N, x, st);
            } else {
                layernorm(x2, blob + P.ln2_g, blob + P.ln2_b, N, E, y, stt, st);
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(NE * 4)), dim3(kTrThreads), 0, st, y, blob + P.fc_w,
                                   blob + P.fc_b, nullptr, N, E, 4 * E, 0, hb);
                hipLaunchKernelGGL(tr_linear, dim3(blocks_for(NE)), dim3(kTrThreads), 0, st, hb, blob + P.mp_w,
                                   blob + P.mp_b, x2, N, 4 * E, E, 1, x);
            }
        }
        layernorm(x, blob + B.lnf_g, blob + B.lnf_b, N, E, y, stt, st);
        hipLaunchKernelGGL(tr_linear, dim3(blocks_for((int64_t)N * d.A)), dim3(kTrThreads), 0, st, y, blob + B.head_w,
                           blob + B.head_b, nullptr, N, E, d.A, 0, ws + W.lg);
        hipLaunchKernelGGL(gen_select_env, dim3((N + 255) / 256), dim3(256), 0, st, ws + W.lg, g, h, ws + W.tok);
        if (int rc = launched("generic bandit rollout step")) return rc;
    }
    return DPT_OK;
}

}  // namespace dpt
