// Fused DarkRoom in-context evaluation on gfx950: evals/eval_darkroom.py:20-84
// deploy_online_vec with DarkroomTransformerController (ctrls/ctrl_darkroom.py:23-66)
// and DarkroomEnvVec.deploy_eval (envs/darkroom_env.py:151-175), one launch.
//
// The query (current state) changes every step, so each step is a full causal
// forward over the window [query, context transitions...] (models/net.py:41-60);
// the prediction is the LAST position.  That is matrix-core work: one workgroup
// owns one task for all Heps x horizon steps, and each wave owns two 16-token
// blocks of the window (4 waves for T <= 128, 8 for T <= 256, 16 for T <= 512: DrGeom).
//
// Dataflow is transposed (features x tokens): a wave keeps x^T of its 16
// tokens in registers as MFMA 16x16x4 C-layout fragments -- lane (g = l>>4,
// c = l&15) holds features 16*blk + 4g + r of token c, blk in {0,1}, r < 4.
// That is exactly the B-operand layout of the next product W^T x^T (k-step s
// reads feature 16*(s>>2) + 4g + (s&3)), so c_attn, attention, c_proj, c_fc,
// gelu and mlp.c_proj chain in registers; only K (token-major) and V
// (feature-major) go through LDS, because every later token reads them.
// Weights are the A operand, split into fp16 parts and pre-packed per layer in
// operand order (Frag3, pack_split_kernel) and read through one buffer
// descriptor; every product (dense and attention) runs as fp32-accurate fp16
// two-part split products on the fp16 matrix cores (dpt_mfma_fwd.h mfma_x3).
//
// Exact restructurings (same arithmetic up to fp32 summation order):
//  * layer 0: within an episode the context tokens' layer-0 keys/values are
//    fixed, so the causal softmax partial (m, l, o) of every token over keys
//    1..t is computed once per episode; a step only projects the queries and
//    the query token's key/value and merges key 0 into each partial;
//  * last layer: only position T-1 is read, so after the K/V exchange its
//    attention (one key tile per wave, flash-merged), c_proj and MLP (one
//    hidden chunk per wave) are spread over the waves, then ln_f + head +
//    selection + the grid step run on one wave.
#include "dpt_mfma_fwd.h"

// DPT_STAMPS (diagnostic build only): s_memtime at the barriers of a step,
// accumulated by workgroup 0 thread 0 (see scripts/dr_stamps.py for the slots).
#ifdef DPT_STAMPS
__device__ unsigned long long g_dr_stamps[32];
__device__ unsigned long long g_dr_last;
#define DR_STAMP(k)                                                           \
    do {                                                                      \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                            \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
            if (g_dr_last) g_dr_stamps[(k)] += t_ - g_dr_last;                \
            g_dr_last = t_;                                                   \
        }                                                                     \
    } while (0)
#else
#define DR_STAMP(k) \
    do {            \
    } while (0)
#endif

// wave 0's serial tail and thread 0's memo-hit chain at issue priority 3, ahead of the
// other workgroup's waves on the same SIMD (only issue order changes: bit-identical;
// -0.9 % at config 3)
#define DPT_TAIL_PRIO(p) __builtin_amdgcn_s_setprio(p)
// The wave that runs the step's serial tail (ln_f, head, selection, env step) and the memo-hit
// chain (on its lane 0, which keeps the episode's state and return in registers): the last MLP
// wave, whose blocks are the fewest (blocks_of_wave gives the last waves the middle block or none)
#ifndef DPT_TAIL_WAVE
#define DPT_TAIL_WAVE 3
#endif

namespace dpt {

constexpr int kDrA = 5;                     // DarkRoom actions
constexpr int kDrF = 10;                    // token features 2*sd + A + 1
#ifndef DPT_DR_MEMO_STATES
#define DPT_DR_MEMO_STATES 128
#endif
constexpr int kMemoStates = DPT_DR_MEMO_STATES;  // logits memo rows (grids up to 11 x 11)

// DPT_DR_EMB_GLOBAL: the token embedding (10 x 32 floats, read by the episode prologue and the table-free
// kernels' block-0 re-embedding) from global memory instead of the LDS parameter block (1.25 KB less LDS
// per workgroup)
#ifndef DPT_DR_EMB_GLOBAL
#define DPT_DR_EMB_GLOBAL 0
#endif
struct PTop {
    int lnf_g, lnf_b, head_w, head_b, emb_b, wpe0, emb_w, total;
    __host__ __device__ static PTop make(int L) {
        PTop t;
        int o = L * PL::size;
        t.lnf_g = o; o += kE;
        t.lnf_b = o; o += kE;
        t.head_w = o; o += kE * kDrA;
        t.head_b = o; o += 8;
        t.emb_b = o; o += kE;
        t.wpe0 = o; o += kE;
        t.emb_w = o; o += DPT_DR_EMB_GLOBAL ? 0 : kDrF * kE;
        t.total = o;
        return t;
    }
};

// Window geometry of the kernel built with NW waves: 2 NW blocks of 16 tokens (NW = 4: windows
// of up to 128 tokens, two workgroups per CU; NW = 8: up to 256, one per CU; NW = 16: up to 512,
// one per CU at 128 VGPRs per wave, workspace only).
template <int NW>
struct DrGeom {
    static constexpr int kWaves = NW, kBlk = 2 * NW, kT = 16 * kBlk;
    static constexpr int kWsPerTask = 3 * kBlk * 64 * 8;  // [x | u | layer-0 partial o] per task
};

// DPT_DR_WG3 (default): the 4-wave workspace kernel at three workgroups per CU (<= 168 VGPRs, and the
// score product's keys read from the values' token-major rows so that three workgroups' LDS fit the
// CU: 35.6 KB + the parameter block).  The rollout is latency-bound per workgroup, so a third task
// per CU is nearly free: config 3 235.8 -> 202.4 ms, bit-identical (A/B in one process per library).
#ifndef DPT_DR_WG3
#define DPT_DR_WG3 1
#endif
#ifndef DPT_DR_NW8_2
#define DPT_DR_NW8_2 1
#endif
#ifndef DPT_DR_WG3_N
#define DPT_DR_WG3_N 3
#endif
// 16-B multiple: the dynamic parameter block P follows it and is read with 16-B loads.
// kWs (a per-task workspace is given): the layer-0 partials live in the workspace and
// the freed LDS holds the values as split pair tiles (P V on mfma_x3);
// without one they stay here and the values are fp32.
template <bool kWs, int NW>
struct alignas(16) DrSmem {
    static constexpr int kFwdT = DrGeom<NW>::kT, kFwdBlocks = DrGeom<NW>::kBlk;
    // keys and values of the current layer (the 16-wave geometry reads the keys from the values'
    // rows: 512 tokens of both in LDS)
    KVBuf<kFwdT, kSplitKeys, kSplitKeys && kWs, kWs && (NW == 16 || (NW == 4 && DPT_DR_WG3) || (NW == 8 && DPT_DR_NW8_2))> kv;
    int2 ctx[kFwdT];   // context transitions, oldest first: .x = x|y<<8|a<<16|r<<24, .y = nx|ny<<8
    int2 cur[kFwdT];   // this episode's transitions
    // layer-0 episode cache: the causal softmax partial of every token over keys
    // 1..t, unnormalised o^T in C-layout per (block, lane), m and l per token
    float l0o[kWs ? 0 : kFwdBlocks][64][8];  // (none with the workspace: zero-length, clang extension)
    float l0m[kFwdT], l0l[kFwdT];
    float k0[kE], v0[kE];             // layer 0: key / value of the query token
    float ql[kE], xl[kE];             // last layer: q and residual of token T-1
    float part_o[kFwdBlocks][kE];      // last layer: per-key-tile attention partials
    float part_m[kFwdBlocks], part_l[kFwdBlocks];
    float tl_x[kFF / 32][kE];         // last layer (dr_tail_mlp): ln_2 output of token T-1, per MLP wave
    float tl_g[kFF / 32][32];         // last layer (dr_tail_mlp): the wave's gelu outputs
    float part_y[kFF / 32][kE];       // last layer: mlp.c_proj shares per MLP wave
    // per-episode logits memo, one row per grid state (dim * dim <= kMemoStates)
    // row s: the fp32 selection cdf q (cdf_fast: a hit selects by 5 compares) in [0, 5), the logits
    // in [kMemoLg, kMemoLg + 5); 48-B rows, read by three 16-B loads in one round trip.  (No separate
    // valid flag: an empty row holds q[0] = -1 and lg[0] = NaN, so a hit is decided by the row's
    // own values.)
    static constexpr int kMemoRow = 12, kMemoLg = 6;
    static_assert(kMemoLg >= kDrA && kMemoLg + kDrA <= kMemoRow, "memo row layout");
    alignas(16) float memo[kMemoStates][kMemoRow];
    double u_ep[kFwdT];                // this episode's selection uniforms, one per step
    alignas(16) float diag_bias[kDiagBiasFloats];  // the masked score tiles' additive rows (diag_bias_init)
    int sx, sy, nfwd, tnext;
};

__device__ inline int2 pack_tr(int x, int y, int a, int nx, int ny, int r) {
    return make_int2(x | (y << 8) | (a << 16) | (r << 24), nx | (ny << 8));
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
    int32_t* forwards_out;
    int memo;  // 1: reuse this episode's logits for a state already queried (see the kernel)
    const float* frag;
    float* ws;  // per task: layer-0 inputs x and queries u of the window, C-layout (l0_cache), or null
    const float* tab;  // per grid state: the query token's layer-0 input and LN1 output (state_tables), or null
};

// The per-task workspace: within an episode the context tokens' layer-0 inputs
// (embedding + wpe) and queries (u = LN1(x) G + g0) are fixed, so the episode
// prologue stores them and every step reloads them instead of re-embedding and
// re-projecting; only the query token (position 0) is recomputed.  Layout per task:
// [x | u | o][block][lane][8] fp32, each lane's 8 C-layout values contiguous (2 x 16 B);
// o is the layer-0 episode partial (the prologue's attention over keys 1..t).
// The workspace starts with the per-state table (kDrTab floats), then the task caches, at the
// stride of the launch's geometry (dpt_darkroom_workspace_numel_window).
// DPT_DR_L0LIN (default): layer 0's attention output enters c_proj linearly.  Per token t the
// merged output is o_t = (1 - a_t) o'_t + a_t v0 (o'_t: the episode's normalised partial over keys
// 1..t, v0: the query token's value, a_t = 1 / (1 + l_t 2^(m_t - s0_t)), s0_t = q_t . k0), so
//   x_t + c_proj(o_t) = A_t + a_t (V0 - C_t),  C_t = Wvp o'_t + bvp,  A_t = x_t + C_t,  V0 = Wvp v0 + bvp.
// The episode prologue stores A and C in the workspace (slots x and o), the state table holds V0, and a
// step's layer 0 is the score, one exp and one rcp per token and a packed sub + fma per value instead of
// the merge, the split of o and c_proj's six MFMAs.  Same algebra, other fp32 rounding.
#ifndef DPT_DR_L0LIN
#define DPT_DR_L0LIN 1
#endif
// per state: [x | y | V0][g][8] (the query token's layer-0 input, its LN1 output, Wvp y + bvp)
constexpr int kDrTabPerState = (DPT_DR_L0LIN ? 3 : 2) * 4 * 8;
constexpr int kDrTab = kMemoStates * kDrTabPerState;
constexpr int kDrMaxWaves = 16;
template <int NW>
__device__ inline float* l0_cache(const DarkroomParams& p, int task, int which, int blk) {
    return p.ws + kDrTab + (size_t)task * DrGeom<NW>::kWsPerTask +
           ((size_t)(which * DrGeom<NW>::kBlk + blk) * 64 + lane_id()) * 8;
}
__device__ inline void ws_store(float* d, const float (&v)[8]) {
    *reinterpret_cast<floatx4*>(d) = floatx4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<floatx4*>(d + 4) = floatx4{v[4], v[5], v[6], v[7]};
}
__device__ inline void ws_load(const float* d, float (&v)[8]) {
    const floatx4 a = *reinterpret_cast<const floatx4*>(d), b = *reinterpret_cast<const floatx4*>(d + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r] = a[r];
        v[4 + r] = b[r];
    }
}

// DPT_DR_L0LIN episode prologue: c = Wvp o' + bvp from attend's (o, l) (o / l = o' x 2^attn_ey), at true
// scale, and x += c (A); the token-0 column (no key in 1..0: l = 0) gets c = 0
template <int NB, int J0 = 0>
__device__ inline void l0_cproj(const float* W, const FragSrc3& f3, float (&o)[2][8], const float (&l)[2],
                                float (&x)[2][8], const int (&qb)[2], const ModelView& M) {
    const int lane = lane_id(), g = lane >> 4;
    const int vo = FragSrc3::lane_off();
    const Split2 w0 = f3.ld2(Frag3::proj, vo), w1 = f3.ld2(Frag3::proj + 1, vo);
    const floatx4 b0 = ld4(W + PL::proj_b + 4 * g), b1 = ld4(W + PL::proj_b + 16 + 4 * g);  // scaled (PL)
    const float down = exp2i(-(M.attn_ew + M.attn_ey));
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) {
        const Split2 os = split2(o[j], l[j] > 0.f ? __builtin_amdgcn_rcpf(l[j]) : 0.f);
        const floatx4 c0 = mfma_x3(w0, os, b0), c1 = mfma_x3(w1, os, b1);
        const bool tok0 = qb[j] == 0 && (lane & 15) == 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            o[j][r] = tok0 ? 0.f : c0[r] * down;
            o[j][4 + r] = tok0 ? 0.f : c1[r] * down;
            x[j][r] += o[j][r];
            x[j][4 + r] += o[j][4 + r];
        }
    }
}

// Token embeddings of block qb (embed_transition + wpe, models/net.py:52-54):
// the query [state, 0...] at position 0, context transitions after it, zeros
// past the window.
template <class Smem>
__device__ inline void embed_block(const Smem& S, const float* P, const PTop& pt, const float* embw, const float* wpe,
                                   int qb, int T, float (&x)[8]) {
    const int lane = lane_id(), g = lane >> 4, tok = qb * 16 + (lane & 15);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = 0.f;
    if (tok >= T) return;
    const int2 tr = tok >= 1 ? S.ctx[tok - 1] : make_int2(S.sx | (S.sy << 8), 0);
    const float fv[6] = {(float)(tr.x & 255), (float)((tr.x >> 8) & 255), tok >= 1 ? 1.0f : 0.0f,
                         (float)(tr.y & 255), (float)((tr.y >> 8) & 255), (float)((tr.x >> 24) & 255)};
    const int rows[6] = {0, 1, 2 + ((tr.x >> 16) & 255), 7, 8, 9};
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
        const int d0 = 16 * blk + 4 * g;
        floatx4 acc = ld4(P + pt.emb_b + d0);
#pragma unroll
        for (int f = 0; f < 6; ++f) {
            const floatx4 w = ld4(embw + rows[f] * kE + d0);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = fmaf(fv[f], w[r], acc[r]);
        }
        const floatx4 pe = tok == 0 ? ld4(P + pt.wpe0 + d0) : ld4(wpe + (size_t)tok * kE + d0);
#pragma unroll
        for (int r = 0; r < 4; ++r) x[blk * 4 + r] = acc[r] + pe[r];
    }
}

// The query token (position 0) is [state, 0...]: its layer-0 input x = emb(state) +
// wpe[0] and its LN1 output y (its key and value in the folded attention) depend on
// the grid state alone, so one table per launch replaces the per-step re-embedding,
// LayerNorm and LDS hand-off of wave 0 (and the barrier after it).  Block = one
// state; each lane computes exactly what embed_block / ln_cols compute for token 0
// in the rollout (same lane layout, same operation order: bit-identical), and
// lanes of column 0 store [x | y][g][8] for g = lane >> 4.
__global__ void __launch_bounds__(64) state_tables_kernel(ModelView M, int dim, float* __restrict__ tab) {
    __shared__ float sp[kE * (kDrF + 4)];
    float* emb_b = sp;
    float* wpe0 = sp + kE;
    float* g1 = sp + 2 * kE;
    float* b1 = sp + 3 * kE;
    float* emb_w = sp + 4 * kE;
    for (int i = threadIdx.x; i < kE; i += 64) {
        emb_b[i] = M.emb_b[i];
        wpe0[i] = M.wpe[i];
        g1[i] = M.layers[LayerOff::ln1_g + i];
        b1[i] = M.layers[LayerOff::ln1_b + i];
    }
    for (int i = threadIdx.x; i < kDrF * kE; i += 64) emb_w[i] = M.emb_w[i];
    __syncthreads();
    const int s = blockIdx.x, lane = lane_id(), g = lane >> 4;
    const float fv[6] = {(float)(s / dim), (float)(s % dim), 0.0f, 0.0f, 0.0f, 0.0f};
    const int rows[6] = {0, 1, 2, 7, 8, 9};
    float x[8], y[8];
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
        const int d0 = 16 * blk + 4 * g;
        floatx4 acc = ld4(emb_b + d0);
#pragma unroll
        for (int f = 0; f < 6; ++f) {
            const floatx4 w = ld4(emb_w + rows[f] * kE + d0);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = fmaf(fv[f], w[r], acc[r]);
        }
        const floatx4 pe = ld4(wpe0 + d0);
#pragma unroll
        for (int r = 0; r < 4; ++r) x[blk * 4 + r] = acc[r] + pe[r];
    }
    ln_cols(x, y, g1, b1);
    if ((lane & 15) == 0) {
        float* d = tab + (size_t)s * kDrTabPerState + g * 8;
        ws_store(d, x);
        ws_store(d + 32, y);
    }
#if DPT_DR_L0LIN
    // V0 = Wvp y + bvp (fp32 fma chain per feature), stored in the same [g][8] lane order
    __shared__ float ys[kE];
    if ((lane & 15) == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) ys[16 * (k >> 2) + 4 * g + (k & 3)] = y[k];
    }
    __syncthreads();
    if (lane < kE) {
        const float* F = M.l0;  // layer 0's folded attention
        float v = F[L0Off::bvp + lane];
        for (int k = 0; k < kE; ++k) v = fmaf(F[L0Off::Wvp + k * kE + lane], ys[k], v);
        const int gf = (lane & 15) >> 2, kk = 4 * (lane >> 4) + (lane & 3);
        tab[(size_t)s * kDrTabPerState + 64 + gf * 8 + kk] = v;
    }
#endif
}

// LDS stores of this wave visible to its own later loads (waits for them: no barrier, one wave)
__device__ inline void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Sum over the 32 lanes of each half of the wave (DPP within rows of 16, then the xor-16 partner);
// every lane of the half gets the same value
__device__ inline float dr_sum32(float d) {
#define DR_DPP(v, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xF, 0xF, false))
    d += DR_DPP(d, 0xB1);   // quad_perm xor 1
    d += DR_DPP(d, 0x4E);   // quad_perm xor 2
    d += DR_DPP(d, 0x141);  // row_half_mirror: the two quads of each 8
    d += DR_DPP(d, 0x140);  // row_mirror: the two 8s of each row of 16
#undef DR_DPP
    return sum_x16(d);      // the two rows of each 32
}

// The last layer of token T-1 after its attention partials: every product there has ONE column (the
// token), so on the matrix cores 15 of 16 columns are waste and each operand needs its fp16 split.
// They run instead as fp32 matrix-vector products on the VALU (fp32 FMA chains: as accurate as the
// reference's fp32 matmuls, not its summation order), spread over the four MLP waves:
//  dr_tail_mlp (wave w < 4, lane (f = lane & 31, half = lane >> 5)): merge the key-tile partials
//    (every wave, the same values), c_proj (Wvp) + residual and ln_2 for feature f, then hidden units
//    32 w .. 32 w + 31 of c_fc (unit 32 w + f, the half's 16 inputs, halves summed) + gelu_new, and
//    their share of mlp.c_proj into feature f (the half's 16 units, halves summed) -> part_y[w];
//  dr_tail_head (the tail wave, after a barrier): the four shares + residual, ln_f, head.
// Each lane's 48 weights (pack_tail_kernel): Wvp and c_fc loaded before the attention partials, mlp.c_proj
// after their barrier (dr_tail_ld_*).
constexpr int kDrTailWv = 0, kDrTailFc = 64 * 16, kDrTailMp = 64 * 16 + 4 * 64 * 16,
              kDrTailFloats = 64 * 16 + 2 * 4 * 64 * 16;
struct DrTailW {
    floatx4 wv[4], wf[4], wm[4];
};
// Wvp and c_fc, then mlp.c_proj (used after the merge, c_proj, ln_2 and c_fc)
__device__ inline void dr_tail_ld_early(const float* tw, int w, DrTailW& t) {
    const int lane = lane_id();
    const floatx4* wv4 = reinterpret_cast<const floatx4*>(tw + kDrTailWv) + lane * 4;
    const floatx4* wf4 = reinterpret_cast<const floatx4*>(tw + kDrTailFc) + (w * 64 + lane) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        t.wv[i] = wv4[i];
        t.wf[i] = wf4[i];
    }
}
__device__ inline void dr_tail_ld_late(const float* tw, int w, DrTailW& t) {
    const floatx4* wm4 = reinterpret_cast<const floatx4*>(tw + kDrTailMp) + (w * 64 + lane_id()) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) t.wm[i] = wm4[i];
}
// sum of the lane's 16 products with a 16-vector held as 4 floatx4 (two chains)
__device__ inline float dot16(const floatx4 (&w)[4], const floatx4 (&v)[4]) {
    float c0 = 0.f, c1 = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            c0 = fmaf(w[r][i], v[r][i], c0);
            c1 = fmaf(w[r][i + 1], v[r][i + 1], c1);
        }
    return c0 + c1;
}
// returns x1 (the residual after c_proj) for feature f
template <class Smem>
__device__ inline float dr_tail_mlp(Smem& S, const float* W, const DrTailW& t, int w, int nparts, const ModelView& M) {
    const int lane = lane_id(), f = lane & 31, hf = lane >> 5;
    // merge the key-tile partials (attend's convention: o / l is the output x 2^attn_ey); this lane's
    // 16 features 16 half .. 16 half + 15
    float mx = -INFINITY;
    for (int k = 0; k < nparts; ++k) mx = vmax2(mx, S.part_m[k]);
    float lsum = 0.f;
    floatx4 o[4] = {};
    for (int k = 0; k < nparts; ++k) {
        const float e = __builtin_amdgcn_exp2f(S.part_m[k] - mx);
        lsum += S.part_l[k] * e;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const floatx4 po = ld4(&S.part_o[k][16 * hf + 4 * r]);
#pragma unroll
            for (int i = 0; i < 4; ++i) o[r][i] = fmaf(po[i], e, o[r][i]);
        }
    }
    // c_proj (Wvp, the folded attention): y_f = bvp_f + sum_k Wvp[k][f] out_k
    const float inv = __builtin_amdgcn_rcpf(lsum) * exp2i(-M.attn_ey);
    const float y = sum_x32(dot16(t.wv, o)) * inv + W[PL::proj_b + f] * exp2i(-(M.attn_ew + M.attn_ey));  // bvp scaled (PL)
    const float x1 = S.xl[f] + y;
    // ln_2 (PL keeps its parameters at the c_fc split's scale 2^mlp_ex: exact powers of two)
    const float sx = exp2i(-M.mlp_ex);
    const float mean = dr_sum32(x1) * (1.0f / kE);
    const float d1 = x1 - mean;
    const float rs1 = __builtin_amdgcn_rsqf(dr_sum32(d1 * d1) * (1.0f / kE) + 1e-5f);
    const float xn = fmaf(d1 * rs1, W[PL::ln2_g + f] * sx, W[PL::ln2_b + f] * sx);
    // this half's 16 inputs of xn (features 16 half ..): from the lanes that hold them, via LDS
    float* xw = &S.tl_x[w][0];
    if (hf == 0) xw[f] = xn;
    lds_wave_sync();
    floatx4 xv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) xv[r] = ld4(xw + 16 * hf + 4 * r);
    // c_fc unit j = 32 w + f over the half's inputs, halves summed; gelu_new
    const float mdown = exp2i(-(M.mlp_ew + M.mlp_ex));  // fc_b, mp_b at the MLP product scale (PL)
    const float h = sum_x32(dot16(t.wf, xv)) + W[PL::fc_b + 32 * w + f] * mdown;
    const float g = gelu_fast(h);
    float* gw = &S.tl_g[w][0];
    if (hf == 0) gw[f] = g;
    lds_wave_sync();
    floatx4 gv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) gv[r] = ld4(gw + 16 * hf + 4 * r);
    // mlp.c_proj share of units 32 w + 16 half .. into feature f, halves summed
    const float ym = sum_x32(dot16(t.wm, gv));
    if (hf == 0) S.part_y[w][f] = ym;
    return x1;
}
// the tail wave: the four mlp.c_proj shares + bias + residual, ln_f, head -> logits on every lane
template <class Smem>
__device__ inline void dr_tail_head(const Smem& S, const float* P, const float* W, const PTop& pt, float x1,
                                    const ModelView& M, float (&lg)[kDrA]) {
    const int f = lane_id() & 31;
    const float mdown = exp2i(-(M.mlp_ew + M.mlp_ex));
    const float ym = (S.part_y[0][f] + S.part_y[1][f]) + (S.part_y[2][f] + S.part_y[3][f]);
    const float x2 = x1 + (ym + W[PL::mp_b + f] * mdown);
    const float meanf = dr_sum32(x2) * (1.0f / kE);
    const float d2 = x2 - meanf;
    const float rs2 = __builtin_amdgcn_rsqf(dr_sum32(d2 * d2) * (1.0f / kE) + 1e-5f);
    const float xf = fmaf(d2 * rs2, P[pt.lnf_g + f], P[pt.lnf_b + f]);
#pragma unroll
    for (int a = 0; a < kDrA; ++a) lg[a] = dr_sum32(xf * P[pt.head_w + a * kE + f]) + P[pt.head_b + a];
}

// The last block's fp32 matrix-vector weights in the lanes' order (dr_tail_mlp), after the fragments:
// [Wvp: lane (f, half) -> Wvp[16 half + i][f], i < 16]
// [c_fc: wave w, lane (f, half) -> W_fc[16 half + i][32 w + f], i < 16]
// [mlp.c_proj: wave w, lane (f, half) -> W_mp[32 w + 16 half + i][f], i < 16]
__global__ void pack_tail_kernel(ModelView M, float* __restrict__ out) {
    const int L = M.n_layer;
    const float* Wl = M.layers + (size_t)(L - 1) * LayerOff::size;
    const float* Fl = M.l0 + (size_t)(L - 1) * L0Off::size;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kDrTailFloats; i += gridDim.x * blockDim.x) {
        float v;
        if (i < kDrTailFc) {
            const int lane = i / 16, k = i % 16, f = lane & 31, hf = lane >> 5;
            v = Fl[L0Off::Wvp + (16 * hf + k) * kE + f];
        } else if (i < kDrTailMp) {
            const int o = i - kDrTailFc, w = o / 1024, lane = (o / 16) & 63, k = o % 16, f = lane & 31, hf = lane >> 5;
            v = Wl[LayerOff::fc_w + (16 * hf + k) * kFF + 32 * w + f];
        } else {
            const int o = i - kDrTailMp, w = o / 1024, lane = (o / 16) & 63, k = o % 16, f = lane & 31, hf = lane >> 5;
            v = Wl[LayerOff::mp_w + (32 * w + 16 * hf + k) * kE + f];
        }
        out[i] = v;
    }
}

// The window's last block (the longest causal row) alone on the last wave, the other blocks
// paired as blocks_of_wave does (waves w and nqb - 2 - w); with every slot taken (nqb = 2 NW) the
// plain pairing.  Which wave computes a block changes no result (-2.2 % at config 3: the 7 blocks
// of a 101-token window on 4 waves had wave 0 holding blocks 0 and 6 with the key-tile tail,
// wave 3 the single block 3).  Returns the wave's block count.
// DPT_DR_SHORT8 (experimental): windows of up to 128 tokens on the 8-wave geometry, one block per
// wave (two workgroups per CU) instead of the 4-wave one with two blocks per wave (three per CU)
#ifndef DPT_DR_SHORT8
#define DPT_DR_SHORT8 0
#endif
template <int NW>
__device__ inline int assign_blocks(int wave, int nqb, int (&qb)[2]) {
    if (DPT_DR_SHORT8 && NW == 8 && nqb <= NW) {
        qb[0] = wave;
        qb[1] = wave;
        return wave < nqb ? 1 : 0;
    }
    if (nqb < 2 * NW) {
        if (wave == NW - 1) {
            qb[0] = nqb - 1;
            qb[1] = nqb - 1;
            return 1;
        }
        return blocks_of_wave(wave, nqb - 1, qb);
    }
    return blocks_of_wave(wave, nqb, qb);
}

// Values fixed for a whole episode (the wave's blocks, their workspace addresses, the task) are
// re-derived inside each step from copies the compiler cannot see through: otherwise it hoists
// them out of the step loop, and at the 106-SGPR limit they live as spills in VGPR lanes, read back
// by v_readlane (a VALU instruction plus its hazard wait) at every use.  Recomputing them is a few
// scalar instructions.
#ifndef DPT_DR_OPAQUE
#define DPT_DR_OPAQUE 1
#endif
#define DR_OPQ(v) asm volatile("" : "+s"(v))
#ifndef DPT_DR_SEQ_BLOCKS
#define DPT_DR_SEQ_BLOCKS 0
#endif
#ifndef DPT_DR_SEQ4
#define DPT_DR_SEQ4 0
#endif
#ifndef DPT_DR_HIT_WAVE
#define DPT_DR_HIT_WAVE 1
#endif
// one phase over the wave's blocks inside the step: specialised on NBC when it is known at compile
// time (no-op for 0), else dispatched on the run-time count (DPT_BLOCKS)
// With kSeqBlocks (DPT_DR_SEQ_BLOCKS = 1; the 8- and 16-wave geometries, 128 VGPRs per wave) a
// two-block wave runs each phase for one block after the other (NB = 1 at slots J0 = 0 and 1): the
// same arithmetic per block, so the same results (tested bit-identical), with one block's products
// and split operands live at a time instead of two.  It cuts their scratch from 64 to 16 B/lane but
// is 3.7 % slower at window 201 and 6 % at 301 (profiles/r6/ab_seq_blocks.json): the two blocks'
// interleaved chains hide each other's latency, which the spills cost less than.  Off by default.
#define DR_BLOCKS(...)                                      \
    do {                                                    \
        if constexpr (NBC >= 0) {                           \
            if constexpr (NBC == 2 && kSeqBlocks) {         \
                {                                           \
                    constexpr int NB = 1, J0 = 0;           \
                    __VA_ARGS__;                            \
                }                                           \
                {                                           \
                    constexpr int NB = 1, J0 = 1;           \
                    __VA_ARGS__;                            \
                }                                           \
            } else if constexpr (NBC > 0) {                 \
                constexpr int NB = NBC, J0 = 0;             \
                __VA_ARGS__;                                \
            }                                               \
        } else {                                            \
            DPT_BLOCKS(nb, __VA_ARGS__);                    \
        }                                                   \
    } while (0)


// kTab: token 0's layer-0 input and LN1 output come from the per-state table (the workspace kernels
// on grids of <= kMemoStates cells); without it block 0 is re-embedded and normalised every step
template <bool kWs, int NW, bool kTab = kWs>
__global__ void __launch_bounds__(NW * 64, NW == 4 ? (kWs && DPT_DR_WG3 ? DPT_DR_WG3_N : 2) : (NW == 8 && kWs && DPT_DR_NW8_2 ? 4 : 1))
rollout_darkroom_kernel(ModelView M, DarkroomParams p) {
    static_assert(kWs || !kTab, "the state table lives in the workspace");
    constexpr bool kSeqBlocks = (DPT_DR_SEQ_BLOCKS && NW >= 8) || (DPT_DR_SEQ4 && NW == 4);  // DR_BLOCKS
    // with kSeqBlocks the last layer's fp32 tail weights load after the partials' barrier
    constexpr bool kTailLate = kSeqBlocks;
    __shared__ DrSmem<kWs, NW> S;
    constexpr bool kSplitV = decltype(S.kv)::kSplitV;
    extern __shared__ float P[];
    const int task = blockIdx.x;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int kTailWave = DPT_TAIL_WAVE, kTailTid = 64 * kTailWave;
    static_assert(kTailWave < NW, "the tail wave is a wave of the workgroup");
    const int steps_total = p.Heps * p.horizon;
    const float scale = 0.17677669529663687f;  // 1/sqrt(head_dim = 32)
    const int L = M.n_layer;
    const PTop pt = PTop::make(L);
    const FragSrc3 split0{__builtin_amdgcn_make_buffer_rsrc((void*)p.frag, (short)0, L * Frag3::bytes, 0x00020000), 0};
    load_layer_params(P, M, tid, blockDim.x);
    for (int i = tid; i < kE; i += blockDim.x) {
        P[pt.lnf_g + i] = M.lnf_g[i];
        P[pt.lnf_b + i] = M.lnf_b[i];
        P[pt.emb_b + i] = M.emb_b[i];
        P[pt.wpe0 + i] = M.wpe[i];
    }
    for (int i = tid; i < kE * kDrA; i += blockDim.x)  // transposed to [a][E] for 16-B reads
        P[pt.head_w + (i % kDrA) * kE + i / kDrA] = M.head_w[i];
    for (int i = tid; i < kDrA; i += blockDim.x) P[pt.head_b + i] = M.head_b[i];
    if constexpr (kSplitV) {  // finite values in tiles no episode has written yet (attend)
        uint4* vs = reinterpret_cast<uint4*>(&S.kv.VT[0][0][0]);
        for (int i = tid; i < (int)(sizeof(S.kv.VT) / 16); i += blockDim.x) vs[i] = uint4{0u, 0u, 0u, 0u};
        if constexpr (decltype(S.kv)::kKS) {  // the key tiles too: attend scores the tile past the diagonal
            uint4* ks = reinterpret_cast<uint4*>(&S.kv.KS[0][0][0]);
            for (int i = tid; i < (int)(sizeof(S.kv.KS) / 16); i += blockDim.x) ks[i] = uint4{0u, 0u, 0u, 0u};
        }
    }
    if (!DPT_DR_EMB_GLOBAL)
        for (int i = tid; i < kDrF * kE; i += blockDim.x) P[pt.emb_w + i] = M.emb_w[i];
    const float* embw = DPT_DR_EMB_GLOBAL ? M.emb_w : P + pt.emb_w;
    diag_bias_init(S.diag_bias, tid, blockDim.x);
    const float* diag_bias = S.diag_bias;

    // the task's goal and action permutation, once (wave-uniform: scalar registers), not
    // reloaded from memory on thread 0's serial select chain every step
    const int goal_x = p.goals[2 * task], goal_y = p.goals[2 * task + 1];
    // the action permutation packed 3 bits per action in one register (a shift and a mask per step
    // instead of five held values and a select chain)
    int perm_bits = 0;
#pragma unroll
    for (int k = 0; k < kDrA; ++k) perm_bits |= (p.perms ? p.perms[(size_t)task * kDrA + k] : k) << (3 * k);
    for (int ep = 0; ep < p.Heps; ++ep) {
        const int nctx = min(ep, p.R) * p.horizon;
        const int T = 1 + nctx;
        const int nqb = (T + 15) >> 4;
        int qb[2];
        const int nb = assign_blocks<NW>(wave, nqb, qb);
#if !DPT_DR_OPAQUE
        const int qlast = (T - 1) >> 4, clast = (T - 1) & 15;
        const bool own0 = nb > 0 && qb[0] == 0;
#endif
        if (tid == 0) {
            S.sx = 0;
            S.sy = 0;
            S.nfwd = 0;
        }
        // the tail thread's copy of the state and the episode's return (it runs every selection)
        int cur_x = 0, cur_y = 0, cur_ret = 0;
        // an opaque thread id for the episode's LDS initialisation: its addresses are recomputed per
        // episode instead of being hoisted out of the episode loop and spilled (128-VGPR geometries)
        int tid_p = tid;
        asm volatile("" : "+v"(tid_p));
        for (int i = tid_p; i < kMemoStates; i += blockDim.x) {
            S.memo[i][0] = -1.0f;
            S.memo[i][S.kMemoLg] = __builtin_nanf("");
        }
        // the episode's selection uniforms up front, one thread per step (off the serial
        // select chain of thread 0; ordered before their use by the barriers below)
        if (p.sample) {
            for (int t = tid_p; t < p.horizon; t += blockDim.x) {
                const int step = ep * p.horizon + t;
                S.u_ep[t] = p.uniforms ? p.uniforms[(size_t)step * p.N + task]
                                       : philox_uniform(p.seed, p.counter + step, p.first_task + task, DPT_STREAM_SELECT);
            }
        }
        __syncthreads();

        // layer-0 episode cache: causal partial over keys 1..t of every token (specialised on the
        // wave's block count in the workspace kernels, as the step's forward below)
        auto prologue = [&](auto nb_c) {
            constexpr int NBC = decltype(nb_c)::value;
            const int NBR = NBC >= 0 ? NBC : nb;
            float x[2][8], xn[2][8], q[2][8];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                if (j < NBR) embed_block(S, P, pt, embw, M.wpe, qb[j], T, x[j]);
            DR_BLOCKS((ln_n<NB, J0>(x, xn, P + PL::ln1_g, P + PL::ln1_b), u_proj_kv3_n<NB, J0>(P, split0, xn, q, S.kv, qb, M)));
            if constexpr (kWs) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (j >= NBR) break;
                    if (!(DPT_DR_L0LIN && kTab)) ws_store(l0_cache<NW>(p, task, 0, qb[j]), x[j]);
                    ws_store(l0_cache<NW>(p, task, 1, qb[j]), q[j]);
                }
            }
            bar_lds();
#if DPT_DR_L0LIN
            if constexpr (kTab) {
                // the partials through c_proj once per episode: C = Wvp o' + bvp, A = x + C (the token-0
                // column has no partial: C = 0 there, and its A comes from the state table)
                float o[2][8], l[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (j >= NBR) break;
                    float m;
                    attend(S.kv, q[j], qb[j], 1, scale, m, l[j], o[j], M, diag_bias);
                    const int lane = lane_id();
                    if (lane < 16) {
                        S.l0m[qb[j] * 16 + lane] = m;
                        S.l0l[qb[j] * 16 + lane] = l[j] * exp2i(-kPExp);
                    }
                }
                DR_BLOCKS(l0_cproj<NB, J0>(P, split0, o, l, x, qb, M));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (j >= NBR) break;
                    ws_store(l0_cache<NW>(p, task, 0, qb[j]), x[j]);
                    ws_store(l0_cache<NW>(p, task, 2, qb[j]), o[j]);
                }
                __syncthreads();
                return;
            }
#endif
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j >= NBR) break;
                float m, l, o[8];
                attend(S.kv, q[j], qb[j], 1, scale, m, l, o, M, diag_bias);
                // the partial at its true scale (attend's o, l carry 2^(attn_ey + kPExp), 2^kPExp)
                l *= exp2i(-kPExp);
                const float down = exp2i(-(M.attn_ey + kPExp));
#pragma unroll
                for (int k = 0; k < 8; ++k) o[k] *= down;
                const int lane = lane_id();
                if constexpr (kWs) {
                    ws_store(l0_cache<NW>(p, task, 2, qb[j]), o);
                } else {
                    *reinterpret_cast<floatx4*>(&S.l0o[qb[j]][lane][0]) = {o[0], o[1], o[2], o[3]};
                    *reinterpret_cast<floatx4*>(&S.l0o[qb[j]][lane][4]) = {o[4], o[5], o[6], o[7]};
                }
                if (lane < 16) {
                    S.l0m[qb[j] * 16 + lane] = m;
                    S.l0l[qb[j] * 16 + lane] = l;
                }
            }
            __syncthreads();
        };
        if constexpr (kWs) {
            if (nb == 2) prologue(std::integral_constant<int, 2>{});
            else if (nb == 1) prologue(std::integral_constant<int, 1>{});
            else prologue(std::integral_constant<int, 0>{});
        } else {
            prologue(std::integral_constant<int, -1>{});
        }

        // the policy's logits are a pure function of (window, query state) and the
        // window is fixed for the whole episode: a state queried before in this
        // episode reuses that forward's logits (bit-identical to re-running it)
        // q: the fp32 selection cdf of lg (cdf_fast) when sampling; select_fast(q, lg, u) equals
        // select_fixed(lg, u) bit for bit (the exact fp64 cdf decides within 2^-15 of an edge)
        // u: this step's selection uniform (S.u_ep[t] when sampling)
        auto finish_step = [&](const float (&lg)[kDrA], const float* q, int t, int sx, int sy, double u) {
            const int step = ep * p.horizon + t;
            const int a = p.sample ? select_fast<kDrA>(q, lg, p.temp, u) : select_fixed<kDrA>(lg, 0, p.temp, u);
            const int ea = (perm_bits >> (3 * a)) & 7;
            int nx = sx + (ea == 0) - (ea == 1);
            int ny = sy + (ea == 2) - (ea == 3);
            nx = min(max(nx, 0), p.dim - 1);
            ny = min(max(ny, 0), p.dim - 1);
            const int r = (nx == goal_x && ny == goal_y) ? 1 : 0;
            S.cur[t] = pack_tr(sx, sy, a, nx, ny, r);
            cur_x = nx;  // thread 0's registers; published to S.sx / S.sy before other threads read them
            cur_y = ny;
            cur_ret += r;
            if (p.actions_out) p.actions_out[(size_t)task * steps_total + step] = a;
            if (p.logits_out) {
#pragma unroll
                for (int k = 0; k < kDrA; ++k) p.logits_out[((size_t)step * p.N + task) * kDrA + k] = lg[k];
            }
        };
        for (int t = 0; t < p.horizon; ++t) {
            if (DPT_DR_HIT_WAVE && p.memo && p.sample) {
                // the tail wave runs consecutive steps whose state was already queried this episode
                // (a memo hit needs no forward) as one wave-uniform chain: lane k < 5 reads the row's
                // cdf value q_k (and lanes 6..10 its logits) in one LDS round trip, the five compares
                // of select_fast are one ballot, and the state, action, env step and return are
                // wave-uniform (scalar) values -- instead of thread 0 alone walking the row, the five
                // compares and the margin tests one dependent instruction after another.  The same
                // comparisons in fp32 and the same fp64 fallback (cdf_fixed within 2^-15 of an edge):
                // bit-identical to finish_step.  The other waves wait at one barrier.
                if (wave == kTailWave) {
                    DPT_TAIL_PRIO(3);
                    const int lane = lane_id();
                    int tt = t;
                    int cx = __builtin_amdgcn_readfirstlane(cur_x), cy = __builtin_amdgcn_readfirstlane(cur_y);
                    int cret = __builtin_amdgcn_readfirstlane(cur_ret);
                    while (tt < p.horizon) {
                        const int sidx = cx * p.dim + cy;
                        const float rv = lane < S.kMemoRow ? S.memo[sidx][lane] : 0.0f;
                        const double u = S.u_ep[tt];
                        const float q0 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, rv)));
                        if (!(q0 >= 0.0f)) break;  // no stored row: this state needs a forward
                        const float uf = (float)u;
                        const unsigned long long le = __builtin_amdgcn_ballot_w64(lane < kDrA && rv <= uf);
                        const unsigned long long unsafe =
                            __builtin_amdgcn_ballot_w64(lane < kDrA && !(__builtin_fabsf(rv - uf) > kCdfMargin));
                        int a = __builtin_popcountll(le);
                        a = a < kDrA ? a : kDrA - 1;
                        const int step = ep * p.horizon + tt;
                        if (unsafe) {  // within 2^-15 of an edge (or a NaN logit): the exact fp64 cdf
                            float lg[kDrA];
#pragma unroll
                            for (int k = 0; k < kDrA; ++k)
                                lg[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, rv), S.kMemoLg + k));
                            double qe[kDrA];
                            cdf_fixed<kDrA>(lg, p.temp, qe);
                            a = __builtin_amdgcn_readfirstlane(select_from_cdf<kDrA>(qe, u));
                        }
                        const int ea = (perm_bits >> (3 * a)) & 7;
                        int nx = cx + (ea == 0) - (ea == 1);
                        int ny = cy + (ea == 2) - (ea == 3);
                        nx = min(max(nx, 0), p.dim - 1);
                        ny = min(max(ny, 0), p.dim - 1);
                        const int r = (nx == goal_x && ny == goal_y) ? 1 : 0;
                        if (lane == 0) {
                            S.cur[tt] = pack_tr(cx, cy, a, nx, ny, r);
                            if (p.actions_out) p.actions_out[(size_t)task * steps_total + step] = a;
                        }
                        if (p.logits_out && lane >= S.kMemoLg && lane < S.kMemoLg + kDrA)
                            p.logits_out[((size_t)step * p.N + task) * kDrA + (lane - S.kMemoLg)] = rv;
                        cx = nx;
                        cy = ny;
                        cret += r;
                        ++tt;
                    }
                    cur_x = cx;
                    cur_y = cy;
                    cur_ret = cret;
                    if (lane == 0) {
                        S.sx = cx;
                        S.sy = cy;
                        S.tnext = tt;
                    }
                    DPT_TAIL_PRIO(0);
                }
                bar_lds();
                DR_STAMP(2 * L + 4);
                t = S.tnext;
                if (t >= p.horizon) break;
            } else if (p.memo) {
                // thread 0 runs consecutive steps whose state was already queried this
                // episode (a memo hit needs no forward); the other threads wait at one
                // barrier for the first state that needs one
                if (tid == kTailTid) {
                    DPT_TAIL_PRIO(3);  // the memo-hit chain is the workgroup's critical path
                    int tt = t;
                    while (tt < p.horizon) {
                        const int sidx = cur_x * p.dim + cur_y;
                        const floatx4* row = reinterpret_cast<const floatx4*>(&S.memo[sidx][0]);
                        const floatx4 r0 = row[0], r1 = row[1], r2 = row[2];
                        const double u = p.sample ? S.u_ep[tt] : 0.0;  // in the same LDS round trip
                        const float qv[kDrA] = {r0[0], r0[1], r0[2], r0[3], r1[0]};
                        const float lg[kDrA] = {r1[2], r1[3], r2[0], r2[1], r2[2]};
                        // a stored row: sampling reads its cdf (q[0] >= 0), greedy its logits
                        if (p.sample ? !(qv[0] >= 0.0f) : __builtin_isnan(lg[0])) break;
                        finish_step(lg, qv, tt, cur_x, cur_y, u);
                        ++tt;
                    }
                    S.sx = cur_x;
                    S.sy = cur_y;
                    S.tnext = tt;
                    DPT_TAIL_PRIO(0);
                }
                bar_lds();
                DR_STAMP(2 * L + 4);
                t = S.tnext;
                if (t >= p.horizon) break;
            }
#if DPT_DR_OPAQUE
            // per-step copies of the episode's block assignment (see DR_OPQ)
            int wv = wave, Tq = T, task_s = task;
            DR_OPQ(wv);
            DR_OPQ(Tq);
            DR_OPQ(task_s);
            const int nqb_s = (Tq + 15) >> 4;
            int qb[2];
            const int nb = assign_blocks<NW>(wv, nqb_s, qb);
            const bool own0 = nb > 0 && qb[0] == 0;
            const int qlast = (Tq - 1) >> 4, clast = (Tq - 1) & 15;
            const int task = task_s;
            const int T = Tq;
#endif
            // The window forward of this step, specialised on the wave's block count (2, 1 or 0):
            // one dispatch per step instead of a branch per phase, so no register copies merge the
            // two paths' activations after every phase
            auto forward = [&](auto nb_c) {
                // NBC = the wave's block count, or -1: taken at run time (each phase dispatches)
                constexpr int NBC = decltype(nb_c)::value;
                const int NBR = NBC >= 0 ? NBC : nb;
                float x[2][8];
                float q[2][8];
                const int sx = S.sx, sy = S.sy;
                if constexpr (kWs) {
                    // the context tokens' inputs and queries from the episode's workspace; token 0's
                    // input (the new query token) from the per-state table, or block 0 re-embedded
                    const bool col0 = (lane_id() & 15) == 0;
    #pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        if (j >= NBR) break;
                        ws_load(l0_cache<NW>(p, task, 1, qb[j]), q[j]);
                        if constexpr (kTab) {
                            ws_load(qb[j] == 0 && col0 ? p.tab + (size_t)(sx * p.dim + sy) * kDrTabPerState + 8 * (lane_id() >> 4)
                                                       : l0_cache<NW>(p, task, 0, qb[j]),
                                    x[j]);
                        } else {
                            if (qb[j] == 0) embed_block(S, P, pt, embw, M.wpe, 0, T, x[j]);
                            else ws_load(l0_cache<NW>(p, task, 0, qb[j]), x[j]);
                        }
                    }
                } else {
    #pragma unroll
                    for (int j = 0; j < 2; ++j)
                        if (j < NBR) embed_block(S, P, pt, embw, M.wpe, qb[j], T, x[j]);
                }

                // ---- layer 0: queries of the window (token 0's is never used: it has no
                // earlier key), the query token's key/value new
                {
                    if constexpr (!kTab) {
                        float xn[2][8];
                        if constexpr (kWs) {
                            if (own0) ln_n<1>(x, xn, P + PL::ln1_g, P + PL::ln1_b);
                        } else {
                            DR_BLOCKS(ln_n<NB, J0>(x, xn, P + PL::ln1_g, P + PL::ln1_b));
                        }
                        if (own0) {  // block 0: key/value (= y) of the query token (the merge below reads them)
                            const int lane = lane_id();
                            if ((lane & 15) == 0) {  // token 0's y (folded attention: key = value = y)
                                const float ydown = exp2i(-M.attn_ey);  // ln_1 returns y x 2^attn_ey (PL)
    #pragma unroll
                                for (int k = 0; k < 8; ++k) {
                                    const int d = 16 * (k >> 2) + 4 * (lane >> 4) + (k & 3);
                                    S.k0[d] = xn[0][k] * ydown;
                                    S.v0[d] = xn[0][k] * ydown;
                                }
                            }
                        }
                        // the queries after the store above: no branch between their MFMAs and the
                        // first reads of q (the wait states stay in one block: attend's note)
                        if constexpr (!kWs) DR_BLOCKS(u_proj3_n<NB, J0>(P, split0, xn, q, M));
                        bar_lds();
                    }
                    DR_STAMP(0);
#if DPT_DR_L0LIN
                    if (kTab && NBR > 0) {
                        // x = A + a (V0 - C) per token column (DPT_DR_L0LIN): x holds A, the workspace's o slot C
                        const int lane = lane_id(), g = lane >> 4;
                        const float* tr = p.tab + (size_t)(sx * p.dim + sy) * kDrTabPerState + 8 * g;
                        const floatx4 ka = ld4(tr + 32), kc = ld4(tr + 36);
                        const floatx4 va = ld4(tr + 64), vb = ld4(tr + 68);
                        float sd[2] = {0.f, 0.f};
    #pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if (j >= NBR) break;
    #pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                sd[j] = fmaf(q[j][r], ka[r], sd[j]);
                                sd[j] = fmaf(q[j][4 + r], kc[r], sd[j]);
                            }
                        }
                        if constexpr (NBC == 2) {
                            sum_cols2(sd[0], sd[1]);
                        } else {
    #pragma unroll
                            for (int j = 0; j < 2; ++j)
                                if (j < NBR) sd[j] = sum_cols(sd[j]);
                        }
    #pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if (j >= NBR) break;
                            const int tok = qb[j] * 16 + (lane & 15);
                            const float s0 = sd[j] * ((scale * 1.4426950408889634f) * exp2i(-M.attn_eq));
                            const float mt = S.l0m[tok], lt = S.l0l[tok];
                            // a = 1 / (1 + l 2^(m - s0)): 1 for the token-0 column (l = 0, m = -inf)
                            const float a = __builtin_amdgcn_rcpf(fmaf(lt, __builtin_amdgcn_exp2f(mt - s0), 1.0f));
                            const float* pc = l0_cache<NW>(p, task, 2, qb[j]);
                            const floatx4 ca = ld4(pc), cb = ld4(pc + 4);
                            const floatx2 a2 = {a, a};
    #pragma unroll
                            for (int r = 0; r < 4; r += 2) {
                                const floatx2 t0 = __builtin_elementwise_fma(
                                    a2, floatx2{va[r], va[r + 1]} - floatx2{ca[r], ca[r + 1]}, floatx2{x[j][r], x[j][r + 1]});
                                const floatx2 t1 = __builtin_elementwise_fma(
                                    a2, floatx2{vb[r], vb[r + 1]} - floatx2{cb[r], cb[r + 1]}, floatx2{x[j][4 + r], x[j][5 + r]});
                                x[j][r] = t0.x;
                                x[j][r + 1] = t0.y;
                                x[j][4 + r] = t1.x;
                                x[j][5 + r] = t1.y;
                            }
                        }
                        float xn[2][8];
                        DR_BLOCKS((ln_n<NB, J0>(x, xn, P + PL::ln2_g, P + PL::ln2_b),
                                   mlp3_n<NB, J0>(P, split0, xn, x, M.mlp_ew, M.mlp_ex)));
                    } else
#endif
                    if (NBR > 0) {
                        // merge key 0 into the cached partial of every token column
                        const int lane = lane_id(), g = lane >> 4;
                        floatx4 ka, kc, va, vb;
                        if constexpr (kTab) {
                            const float* y0 = p.tab + (size_t)(sx * p.dim + sy) * kDrTabPerState + 32 + 8 * g;
                            ka = ld4(y0);
                            kc = ld4(y0 + 4);
                            va = ka;
                            vb = kc;
                        } else {
                            ka = ld4(&S.k0[4 * g]);
                            kc = ld4(&S.k0[16 + 4 * g]);
                            va = ld4(&S.v0[4 * g]);
                            vb = ld4(&S.v0[16 + 4 * g]);
                        }
                        float o[2][8], sd[2] = {0.f, 0.f};
    #pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if (j >= NBR) break;
    #pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                sd[j] = fmaf(q[j][r], ka[r], sd[j]);
                                sd[j] = fmaf(q[j][4 + r], kc[r], sd[j]);
                            }
                        }
                        if constexpr (NBC == 2) {
                            sum_cols2(sd[0], sd[1]);
                        } else {
    #pragma unroll
                            for (int j = 0; j < 2; ++j)
                                if (j < NBR) sd[j] = sum_cols(sd[j]);
                        }
    #pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if (j >= NBR) break;
                            const int tok = qb[j] * 16 + (lane & 15);
                            const float sdot = sd[j];
                            // exp2 domain, as attend's m (q is at 2^attn_eq: u_proj3_w)
                            const float s0 = sdot * ((scale * 1.4426950408889634f) * exp2i(-M.attn_eq));
                            const float mt = S.l0m[tok], lt = S.l0l[tok];
                            const float mn = vmax2(mt, s0);
                            const float ea = __builtin_amdgcn_exp2f(mt - mn), eb = __builtin_amdgcn_exp2f(s0 - mn);
                            // 1 / l by v_rcp_f32 (1 ulp, attn_proj3_ol), with c_proj's split scale 2^attn_ey
                            const float inv = __builtin_amdgcn_rcpf(lt * ea + eb) * exp2i(M.attn_ey);
                            floatx4 oa, ob;
                            if constexpr (kWs) {
                                const float* po = l0_cache<NW>(p, task, 2, qb[j]);
                                oa = ld4(po);
                                ob = ld4(po + 4);
                            } else {
                                oa = ld4(&S.l0o[qb[j]][lane][0]);
                                ob = ld4(&S.l0o[qb[j]][lane][4]);
                            }
                            // on packed f32 ops (each half rounded as the scalar op)
                            const floatx2 e2a = {ea, ea}, e2b = {eb, eb}, iv = {inv, inv};
    #pragma unroll
                            for (int r = 0; r < 4; r += 2) {
                                const floatx2 t0 = (floatx2{oa[r], oa[r + 1]} * e2a + floatx2{va[r], va[r + 1]} * e2b) * iv;
                                const floatx2 t1 = (floatx2{ob[r], ob[r + 1]} * e2a + floatx2{vb[r], vb[r + 1]} * e2b) * iv;
                                o[j][r] = t0.x;
                                o[j][r + 1] = t0.y;
                                o[j][4 + r] = t1.x;
                                o[j][5 + r] = t1.y;
                            }
                        }
                        float xn[2][8];
                        // o is the attention output x 2^attn_ey already (the merge's inv)
    #ifndef DPT_DR_SKIP_MLP  // (timing-only diagnostic builds: DPT_DR_SKIP_* leave phases out; results wrong)
                        DR_BLOCKS((attn_proj3<NB, J0>(P, split0, o, x, M, 1.0f), ln_n<NB, J0>(x, xn, P + PL::ln2_g, P + PL::ln2_b),
                                       mlp3_n<NB, J0>(P, split0, xn, x, M.mlp_ew, M.mlp_ex)));
    #else
                        DR_BLOCKS(attn_proj3<NB, J0>(P, split0, o, x, M, 1.0f));
    #endif
                    }
                    DR_STAMP(1);
                }

// DPT_DR_TAIL_LD_EARLY: the MLP waves' 48 fp32 tail weights per lane issued before the last layer's
// attention partials (1, the default: no spill at the 168-VGPR bound, -0.8 % at config 3,
// profiles/r5e/ab_darkroom_tail_ld_early.json), at the start of the last layer (2: 128 B/lane of
// spill) or after the partials' barrier (0)
#ifndef DPT_DR_TAIL_LD_EARLY
#define DPT_DR_TAIL_LD_EARLY 1
#endif
                DrTailW tlw;  // the last block's fp32 tail weights (dr_tail_ld_*)
                for (int layer = 1; layer < L; ++layer) {
                    const bool last = layer == L - 1;
                    if (DPT_DR_TAIL_LD_EARLY == 2 && !kTailLate && last && wave < kFF / 32) {  // in flight across the last layer
                        const float* tw0 = p.frag + (size_t)L * (Frag3::bytes / 4);
                        dr_tail_ld_early(tw0, wave, tlw);
                        dr_tail_ld_late(tw0, wave, tlw);
                    }
                    auto& kv = S.kv;
                    const float* W = P + layer * PL::size;
                    float q[2][8];
                    {
                        float xn[2][8];
                        if (!last) {
                            DR_BLOCKS((ln_n<NB, J0>(x, xn, W + PL::ln1_g, W + PL::ln1_b),
                                           u_proj_kv3_n<NB, J0>(W, split0.layer(layer), xn, q, kv, qb, M)));
                        } else {
                            // the last layer needs q only for token T-1 (block qlast)
                            DR_BLOCKS((ln_n<NB, J0>(x, xn, W + PL::ln1_g, W + PL::ln1_b), kv_from_y<NB, J0>(kv, qb, xn, M)));
    #pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                if (j < NBR && qb[j] == qlast) {
                                    float xn1[2][8], q1[2][8];
    #pragma unroll
                                    for (int k = 0; k < 8; ++k) xn1[0][k] = xn[j][k];
                                    u_proj3_n<1>(W, split0.layer(layer), xn1, q1, M);
                                    const int lane = lane_id();
                                    if ((lane & 15) == clast) {
    #pragma unroll
                                        for (int k = 0; k < 8; ++k) {
                                            const int d = 16 * (k >> 2) + 4 * (lane >> 4) + (k & 3);
                                            S.ql[d] = q1[0][k];
                                            S.xl[d] = x[j][k];
                                        }
                                    }
                                }
                            }
                        }
                    }
                    bar_lds();
                    DR_STAMP(2 * layer);
                    if (last) break;
    #ifndef DPT_DR_SKIP_ATTN
                    if (NBR > 0) {
                        float o[2][8], l[2];
                        if constexpr (NBC == 2 && kSplitV) {  // the two blocks' l reduced together (sum_cols2)
    #pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                float m;
                                attend<decltype(S.kv), false>(kv, q[j], qb[j], 0, scale, m, l[j], o[j], M, diag_bias);
                            }
                            sum_cols2(l[0], l[1]);
                        } else {
    #pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                if (j >= NBR) break;
                                float m;
                                attend(kv, q[j], qb[j], 0, scale, m, l[j], o[j], M, diag_bias);
                            }
                        }
                        DR_BLOCKS(attn_proj3_ol<NB, J0>(W, split0.layer(layer), o, l, x, M));
                    }
    #endif
                    bar_lds();  // every read of this layer's K/V is done
                    DR_STAMP(2 * layer + 1);
    #ifndef DPT_DR_SKIP_MLP
                    {
                        float xn[2][8];
                        DR_BLOCKS((ln_n<NB, J0>(x, xn, W + PL::ln2_g, W + PL::ln2_b),
                                       mlp3_n<NB, J0>(W, split0.layer(layer), xn, x, M.mlp_ew, M.mlp_ex)));
                    }
    #endif
                }

                // ---- last layer for the one token T-1, spread over the waves.  Every
                // column of these MFMAs carries the same token (B operands broadcast).
                {
                    const float* W = P + (L - 1) * PL::size;
                    const auto& kv = S.kv;
                    // the fp32 tail weights of the last block (pack_tail_kernel): each MLP wave's 48 per
                    // lane, in flight across the attention partials and their barrier
                    constexpr int kMlpWaves = kFF / 32;
                    static_assert(kMlpWaves == 4 && NW >= kMlpWaves && kTailWave < kMlpWaves, "four MLP waves");
                    const float* tw = p.frag + (size_t)L * (Frag3::bytes / 4);
                    if (DPT_DR_TAIL_LD_EARLY == 1 && !kTailLate && wave < kMlpWaves) {  // in flight across the attention partials
                        dr_tail_ld_early(tw, wave, tlw);
                        dr_tail_ld_late(tw, wave, tlw);
                    }
                    // (1) the attention as flash partials (m, l, o), in attend's convention (exp2
                    // domain; l and o at 2^kPExp and 2^(attn_ey + kPExp), so o / l is the output at
                    // the c_proj split's scale): with split values key tiles 2 wave and 2 wave + 1
                    // (one pair, both products on mfma_x3), else key tiles wave and wave + NW
                    const int nparts = kSplitV ? (qlast >> 1) + 1 : qlast + 1;
                    // raw score product -> exp2-domain score
                    const float sl = scale * 1.4426950408889634f * exp2i(-(M.attn_ey + M.attn_eq));
                    if constexpr (kSplitV) {
                        const int lane = lane_id(), g = lane >> 4, c = lane & 15;
                        const int kb = 2 * wave;
                        if (kb <= qlast) {
                            const floatx4 qa = ld4(&S.ql[4 * g]), qc = ld4(&S.ql[16 + 4 * g]);
                            const float qv[8] = {qa[0], qa[1], qa[2], qa[3], qc[0], qc[1], qc[2], qc[3]};
                            const Split2 qs = split2(qv, 1.0f);  // the query (x 2^attn_eq), broadcast to every column
                            float sv[8];
    #pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const int kt = kb + h;
                                if (kt > qlast) {
    #pragma unroll
                                    for (int r = 0; r < 4; ++r) sv[4 * h + r] = -INFINITY;
                                    continue;
                                }
                                const floatx4 sc = mfma_x3(key_split(kv, kt, lane), qs, floatx4{0.f, 0.f, 0.f, 0.f});
    #pragma unroll
                                for (int r = 0; r < 4; ++r) sv[4 * h + r] = (kt * 16 + 4 * g + r <= T - 1) ? sc[r] : -INFINITY;
                            }
                            const float mt = max_cols(vmax8(sv)) * sl;
                            // P x 2^kPExp <= 2^kPExp (mt is the exact max): fp16 two-part as in attend
                            const float bm = (float)kPExp - mt;
                            float pr[8];
    #pragma unroll
                            for (int r = 0; r < 8; ++r) pr[r] = __builtin_amdgcn_exp2f(fmaf(sv[r], sl, bm));
                            float lt = ((pr[0] + pr[1]) + (pr[2] + pr[3])) + ((pr[4] + pr[5]) + (pr[6] + pr[7]));
                            lt = sum_cols(lt);
                            const Split2 ps = split2(pr, 1.0f);
                            const int pp = wave;
                            const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
                            const int vlo = vt_lane_off(lane);
                            const floatx4 o0 = mfma_x3(vt_split(kv, pp, 0, vlo), ps, zero);
                            const floatx4 o1 = mfma_x3(vt_split(kv, pp, 1, vlo), ps, zero);
                            if (c == 0) {
                                *reinterpret_cast<floatx4*>(&S.part_o[wave][4 * g]) = o0;
                                *reinterpret_cast<floatx4*>(&S.part_o[wave][16 + 4 * g]) = o1;
                            }
                            if (lane == 0) {
                                S.part_m[wave] = mt;
                                S.part_l[wave] = lt;
                            }
                        }
                    } else {
                        const int lane = lane_id(), g = lane >> 4, c = lane & 15;
                        const floatx4 qa = ld4(&S.ql[4 * g]), qc = ld4(&S.ql[16 + 4 * g]);
    #pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int kt = wave + NW * h;
                            if (kt > qlast) break;
                            // split key tile x the split query, broadcast to every column
                            const float qv[8] = {qa[0], qa[1], qa[2], qa[3], qc[0], qc[1], qc[2], qc[3]};
                            const Split2 ks = key_split(kv, kt, lane);
                            const floatx4 sc = mfma_x3(ks, split2(qv, 1.0f), floatx4{0.f, 0.f, 0.f, 0.f});
                            float sv[4], mt = -INFINITY;
    #pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                sv[r] = (kt * 16 + 4 * g + r <= T - 1) ? sc[r] * sl : -INFINITY;
                                mt = fmaxf(mt, sv[r]);
                            }
                            mt = max_cols(mt);
                            float pr[4];
    #pragma unroll
                            for (int r = 0; r < 4; ++r) pr[r] = __builtin_amdgcn_exp2f(sv[r] - mt);
                            float lt = (pr[0] + pr[1]) + (pr[2] + pr[3]);
                            lt = sum_cols(lt) * exp2i(kPExp);
                            const floatx4 v0 = ld4(&kv.Vt[c][kt * 16 + 4 * g]);
                            const floatx4 v1 = ld4(&kv.Vt[16 + c][kt * 16 + 4 * g]);
                            floatx4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
    #pragma unroll
                            for (int s4 = 0; s4 < 4; ++s4) o0 = mfma4(v0[s4], pr[s4], o0);
    #pragma unroll
                            for (int s4 = 0; s4 < 4; ++s4) o1 = mfma4(v1[s4], pr[s4], o1);
                            o0 = o0 * exp2i(kPExp);  // the values are y x 2^attn_ey already
                            o1 = o1 * exp2i(kPExp);
                            if (c == 0) {
                                *reinterpret_cast<floatx4*>(&S.part_o[kt][4 * g]) = o0;
                                *reinterpret_cast<floatx4*>(&S.part_o[kt][16 + 4 * g]) = o1;
                            }
                            if (lane == 0) {
                                S.part_m[kt] = mt;
                                S.part_l[kt] = lt;
                            }
                        }
                    }
                    bar_lds();
                    DR_STAMP(2 * L - 1);
                    // (2) the MLP waves: merge, c_proj, ln_2 and a quarter of the MLP of token T-1 as fp32
                    // matrix-vector products (dr_tail_mlp); (3) after a barrier the tail wave: ln_f, head,
                    // selection and the env step
                    float x1 = 0.f;
                    if (wave < kMlpWaves) {
                        if (!DPT_DR_TAIL_LD_EARLY || kTailLate) {  // (the 128-VGPR geometries: after the barrier)
                            dr_tail_ld_early(tw, wave, tlw);
                            dr_tail_ld_late(tw, wave, tlw);
                        }
    #ifndef DPT_DR_SKIP_TAIL
                        x1 = dr_tail_mlp(S, W, tlw, wave, nparts, M);
    #endif
                    }
                    bar_lds();
                    DR_STAMP(2 * L);
                    if (wave == kTailWave) {
                        // the step's serial tail: issue ahead of the other workgroup's waves on this SIMD
                        DPT_TAIL_PRIO(3);
                        const int lane = lane_id();
                        float lg[kDrA] = {};
    #ifndef DPT_DR_SKIP_TAIL
                        dr_tail_head(S, P, W, pt, x1, M, lg);
    #endif
                        DR_STAMP(2 * L + 2);
                        if (lane == 0) {
                            float q[kDrA] = {0.f, 0.f, 0.f, 0.f, 0.f};
                            if (p.sample) cdf_fast<kDrA>(lg, p.temp, q);
                            if (p.memo) {
                                const int sidx = sx * p.dim + sy;
    #pragma unroll
                                for (int k = 0; k < kDrA; ++k) {
                                    S.memo[sidx][S.kMemoLg + k] = lg[k];
                                    S.memo[sidx][k] = q[k];
                                }
                            }
                            S.nfwd += 1;
                            finish_step(lg, q, t, sx, sy, p.sample ? S.u_ep[t] : 0.0);
                            S.sx = cur_x;
                            S.sy = cur_y;
                        }
                        DR_STAMP(2 * L + 3);
                        DPT_TAIL_PRIO(0);
                    }
                }
            };
            // specialised on the wave's block count (DPT_DR_SPEC_NOWS = 0: the workspace-free kernels
            // dispatch per phase instead, the A/B and diagnostic form, scripts/dr_nows_check.py)
#ifndef DPT_DR_SPEC_NOWS
#define DPT_DR_SPEC_NOWS 1
#endif
            if constexpr (kWs || DPT_DR_SPEC_NOWS) {
                if (nb == 2) forward(std::integral_constant<int, 2>{});
                else if (nb == 1) forward(std::integral_constant<int, 1>{});
                else forward(std::integral_constant<int, 0>{});
            } else {
                forward(std::integral_constant<int, -1>{});
            }
            // the end of the step (with the memo, the barrier after the memo-hit chain at the top of
            // the loop would order the state and the partials as well, but dropping this one was
            // 1 % slower at config 3)
            bar_lds();
            DR_STAMP(2 * L + 1);
        }

        // episode bookkeeping: returns, then shift-append the context (eval_darkroom.py:75-82)
        if (tid == kTailTid) {
            p.returns_out[(size_t)task * p.Heps + ep] = cur_ret;
            if (p.forwards_out) p.forwards_out[(size_t)task * p.Heps + ep] = S.nfwd;
        }
        const int R = p.R, H = p.horizon;
        int2 v[2] = {make_int2(0, 0), make_int2(0, 0)};
        // an opaque thread id: the LDS addresses below are recomputed per episode, not hoisted out
        // of the episode loop and spilled (the 8- and 16-wave kernels sit at 128 VGPRs)
        int tid_e = tid;
        asm volatile("" : "+v"(tid_e));
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = tid_e + h * blockDim.x;
            if (i < R * H) {
                if (ep < R) v[h] = (i >= ep * H && i < (ep + 1) * H) ? S.cur[i - ep * H] : S.ctx[i];
                else v[h] = i < (R - 1) * H ? S.ctx[i + H] : S.cur[i - (R - 1) * H];
            }
        }
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = tid_e + h * blockDim.x;
            if (i < R * H) S.ctx[i] = v[h];
        }
        __syncthreads();
    }
}

// The model's fragment buffer: the fp16 two-part split weight tiles (Frag3) of every layer,
// W x 2^mlp_ew (c_fc, mlp.c_proj) or W x 2^attn_ew (G, Wvp).
__global__ void pack_split_kernel(ModelView M, unsigned short* __restrict__ out) {
    const int per_layer = Frag3::tiles * 64 * 8;
    const int total = M.n_layer * per_layer;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int layer = i / per_layer;
        const int o = i % per_layer;
        const int tile = o / 512, lane = (o >> 3) & 63, j = o & 7;
        const int g = lane >> 4, c = lane & 15;
        const float* W = M.layers + (size_t)layer * LayerOff::size;
        const float* F = M.l0 + (size_t)layer * L0Off::size;
        const int kin = 16 * (j >> 2) + 4 * g + (j & 3);
        float w;
        if (tile < Frag3::proj) w = F[L0Off::G + kin * kE + tile * 16 + c];
        else if (tile < Frag3::fc) w = F[L0Off::Wvp + kin * kE + (tile - Frag3::proj) * 16 + c];
        else if (tile < Frag3::mp) w = W[LayerOff::fc_w + kin * kFF + (tile - Frag3::fc) * 16 + c];
        else {
            const int ob = (tile - Frag3::mp) >> 2, pair = (tile - Frag3::mp) & 3;
            w = W[LayerOff::mp_w + (32 * pair + kin) * kE + ob * 16 + c];
        }
        unsigned short* d = out + (size_t)layer * (Frag3::bytes / 2) + ((size_t)tile * Frag3::parts * 64 + lane) * 8 + j;
        const int e = tile >= Frag3::fc ? M.mlp_ew : M.attn_ew;
        const float ws = w * __int_as_float((e + 127) << 23);
        const _Float16 h = (_Float16)ws;
        const _Float16 m = (_Float16)(ws - (float)h);
        d[0] = __builtin_bit_cast(unsigned short, h);
        d[64 * 8] = __builtin_bit_cast(unsigned short, m);
    }
}

int launch_pack_fragments(const ModelView& M, float* frag, hipStream_t st) {
    hipLaunchKernelGGL(pack_split_kernel, dim3(64), dim3(256), 0, st, M, reinterpret_cast<unsigned short*>(frag));
    if (int rc = check_hip(hipGetLastError(), "pack_split_kernel launch")) return rc;
    hipLaunchKernelGGL(pack_tail_kernel, dim3(36), dim3(256), 0, st, M, frag + (size_t)M.n_layer * (Frag3::bytes / 4));
    return check_hip(hipGetLastError(), "pack_tail_kernel launch");
}

// the split fragments of every layer, then the last layer's fp32 tail weights (pack_tail_kernel)
int64_t fragments_numel(int n_layer) { return (int64_t)n_layer * Frag3::bytes / 4 + kDrTailFloats; }

static bool g_darkroom_memo = true;  // DPT_TUNE_DARKROOM_MEMO

int set_darkroom_memo(int on) {
    if (on != 0 && on != 1) return DPT_EINVAL;
    g_darkroom_memo = on == 1;
    return DPT_OK;
}

template <bool kWs, int NW, bool kTab = kWs>
static int launch_darkroom_geom(const ModelView& M, const DarkroomParams& p, hipStream_t st) {
    const size_t dyn = sizeof(float) * (size_t)PTop::make(M.n_layer).total;
    if (dyn + sizeof(DrSmem<kWs, NW>) > 160 * 1024) {
        set_error(DPT_EUNSUPPORTED, "n_layer=%d: parameter block does not fit in LDS", M.n_layer);
        return DPT_EUNSUPPORTED;
    }
    const void* kern = reinterpret_cast<const void*>(rollout_darkroom_kernel<kWs, NW, kTab>);
    if (dyn > 64 * 1024) (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    hipLaunchKernelGGL((rollout_darkroom_kernel<kWs, NW, kTab>), dim3(p.N), dim3(NW * 64), dyn, st, M, p);
    return check_hip(hipGetLastError(), "rollout_darkroom_kernel launch");
}

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
    p.forwards_out = a.forwards_out;
    p.memo = g_darkroom_memo && a.dim * a.dim <= kMemoStates;
    p.frag = frag;
    // the workspace kernels take token 0's layer-0 input from the per-state table when the grid fits
    // it (dim * dim <= kMemoStates); a larger grid runs the workspace-free kernel up to 256 tokens and
    // the table-free workspace kernel above
    const bool tab_ok = a.dim * a.dim <= kMemoStates;
    const int64_t window0 = 1 + (int64_t)a.ctx_episodes * a.horizon;
    p.ws = tab_ok || window0 > DrGeom<8>::kT ? a.workspace : nullptr;
    p.tab = tab_ok ? p.ws : nullptr;
    if (M.n_layer < 2) {
        set_error(DPT_EUNSUPPORTED, "fused darkroom rollout needs n_layer >= 2 (got %d)", M.n_layer);
        return DPT_EUNSUPPORTED;
    }
    if (p.tab) {
        hipLaunchKernelGGL(state_tables_kernel, dim3(a.dim * a.dim), dim3(64), 0, st, M, a.dim, a.workspace);
        if (int rc = check_hip(hipGetLastError(), "state_tables_kernel launch")) return rc;
    }
    // the smallest geometry that holds the window: 4 waves (two workgroups per CU) up to 128
    // tokens, 8 waves (one per CU) up to 256, 16 waves (one per CU, four per SIMD at 128 VGPRs,
    // keys and values of 512 tokens in LDS) up to 512
    const int64_t window = 1 + (int64_t)a.ctx_episodes * a.horizon;
    const bool ws = p.ws != nullptr;
    if (window <= DrGeom<4>::kT) {
        if (DPT_DR_SHORT8 && ws && p.tab) return launch_darkroom_geom<true, 8>(M, p, st);
        return ws ? launch_darkroom_geom<true, 4>(M, p, st) : launch_darkroom_geom<false, 4>(M, p, st);
    }
    if (window <= DrGeom<8>::kT)
        return ws ? launch_darkroom_geom<true, 8>(M, p, st) : launch_darkroom_geom<false, 8>(M, p, st);
    if (!ws) {
        set_error(DPT_EUNSUPPORTED, "fused darkroom rollout: windows over %d tokens need the workspace",
                  DrGeom<8>::kT);
        return DPT_EUNSUPPORTED;
    }
    return p.tab ? launch_darkroom_geom<true, 16>(M, p, st) : launch_darkroom_geom<true, 16, false>(M, p, st);
}

int darkroom_max_window() { return DrGeom<kDrMaxWaves>::kT; }

// per task: the stride of the geometry that runs the window (launch_rollout_darkroom's choice)
int64_t darkroom_workspace_numel(int N, int64_t window) {
    const int64_t per = window <= DrGeom<4>::kT ? (DPT_DR_SHORT8 ? DrGeom<8>::kWsPerTask : DrGeom<4>::kWsPerTask)
                        : window <= DrGeom<8>::kT ? DrGeom<8>::kWsPerTask
                                                  : DrGeom<kDrMaxWaves>::kWsPerTask;
    return kDrTab + (int64_t)N * per;
}

}  // namespace dpt

#ifdef DPT_STAMPS
extern "C" int dpt_debug_dr_stamps(unsigned long long* out, int n, int reset) {
    if (reset) {
        unsigned long long z[32] = {0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dr_stamps), z, sizeof(z));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dr_last), z, sizeof(unsigned long long));
        return 0;
    }
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dr_stamps), sizeof(unsigned long long) * (n < 32 ? n : 32));
}
#endif
