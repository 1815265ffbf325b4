// DPT policy forward on gfx950: KV-cache decode, teacher-forced window
// forward and the fused on-device bandit rollout.
//
// Reference arithmetic: models/net.py:41-60 (pack + embed_transition +
// GPT2Model + pred_actions) with transformers' GPT2Block (ln_1 -> c_attn ->
// causal SDPA, one head -> c_proj -> residual -> ln_2 -> c_fc -> gelu_new ->
// c_proj -> residual) and ln_f.
//
// Work decomposition (one workgroup = one tile of TILE = 8 or 16 tasks, TILE waves;
// TILE = 8 puts two workgroups on a CU so one streams K/V while the other computes):
//  * dense projections: f32 MFMA 16x16x4, tasks are the M rows, weights
//    [in][out] are the B operand streamed from L2 (every weight element is
//    read once per workgroup per step); c_fc is computed transposed so its
//    accumulator feeds mlp.c_proj as the A operand with no LDS round trip;
//  * attention: one wave per task streams that task's K/V rows for positions
//    0..pos-1 from HBM (8 positions x 128 B per float4 wave-load = 1 KiB
//    coalesced), online softmax per lane-group of 8, combined across the 8
//    groups by a 3-step butterfly; the new position's K/V come from LDS;
//  * LayerNorm / gelu / residual: one half-wave per task in LDS.
// The bandit rollout (decode_position<TILE, true>) runs every block on folded
// attention weights (dpt_common.h L0Off): block 0 recomputes its inputs from
// 8-B token records, blocks >= 1 cache y = LN1(h) (128 B per position) as both
// key and value, the u = y G + g0 projection replaces c_attn, and c_proj +
// ln_2 run per task inside the attention wave (proj_ln_task).
// Small parameters (embedding, LayerNorm, biases, head) and the tile's bandit
// means live in LDS for the whole launch.  Phases inside one position are
// separated by LDS-only barriers (lgkmcnt + s_barrier: the K/V stores of the
// step stay in flight); one full __syncthreads per position orders those
// stores before the next position reads them.  The rollout kernel keeps a
// tile resident for all H steps (tasks never interact, so no inter-workgroup
// synchronisation exists anywhere).
#include "dpt_common.h"

// DPT_STAMPS (diagnostic build only, libdpt_hip_stamps.so): s_memtime after
// every barrier of decode_position, accumulated per phase by workgroup 0
// thread 0 into g_stamps; never part of the shipped library.
#ifdef DPT_STAMPS
__device__ unsigned long long g_stamps[64];
__device__ unsigned long long g_stamp_last;
#define DPT_STAMP(k)                                                          \
    do {                                                                      \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                            \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
            if (g_stamp_last) g_stamps[(k)] += t_ - g_stamp_last;             \
            g_stamp_last = t_;                                                \
        }                                                                     \
    } while (0)
#else
#define DPT_STAMP(k) \
    do {             \
    } while (0)
#endif

namespace dpt {

constexpr int kM = 16;                    // MFMA rows = task slots in LDS (TILE <= 16 are live)
constexpr int kLdE = kE + 2;              // padded LDS row strides (conflict-free A reads)
constexpr int kRows = 4;                  // K/V rows (of 8 positions) in flight per wave
#ifndef DPT_YROWS
#define DPT_YROWS 8
#endif
constexpr int kYRows = DPT_YROWS;         // y rows in flight per wave (rollout blocks >= 1; 8: -1.5 % vs 4)
constexpr int kChunks = kFF / 16;         // hidden-unit chunks of the fused c_fc -> mlp.c_proj
#ifndef DPT_DEFAULT_CACHE_BUDGET
#define DPT_DEFAULT_CACHE_BUDGET (224ll << 20)
#endif

// barrier for LDS hand-offs only: does not wait for outstanding global stores
__device__ inline void bar_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The token record (TokRec) of task tile0 + t at position p: [position][task in
// tile] at the start of the tile's block-0 K slot (max_pos x TILE x 16 B of its
// max_pos x TILE x 128 B).
__device__ inline float* tokrec(float* kv, int max_pos, int tile0, int p, int tile, int t) {
    return kv + (size_t)tile0 * max_pos * kE + ((size_t)p * tile + t) * 4;
}

// The rollout's K/V workspace holds whole tiles (kv_tasks, dpt_common.h): blocks
// l >= 1 keep their y rows tile-interleaved, [tile][position][task in tile][E], so
// a tile's 8 (16) attention waves streaming the same positions read one
// contiguous range (DRAM page locality: -1.4 % at config 2, -3.8 % on the linear
// config against per-task streams; bit-identical).

struct Smem {
    float x[kM][kE];             // residual stream of the current position
    float xn[kM][kLdE];          // LayerNorm output (MFMA operand)
    float q[kM][kE];
    float kcur[kM][kE];
    float vcur[kM][kE];
    float o[kM][kLdE];           // attention output (A operand of c_proj)
    float part[kChunks][kM][kE]; // mlp.c_proj partial sums, one per 16-unit hidden chunk
    float logits[kM][kMaxA];
    float tok[kM][kMaxF];        // packed token features of the current position
};
static_assert(sizeof(Smem) % 16 == 0, "parameter block must start 16-B aligned");
static_assert(sizeof(Smem::part) >= 8 * 8 * 64 * sizeof(float), "l0_tiles partials (8 waves x 8 tasks x kL0Part) live in part");

// Columns of l0_tiles' per-task constants (alpha, gamma, beta[0..A]): one or two
// 16-column MFMA tiles of the u phase.
__host__ __device__ constexpr int l0_cols(int A) { return A + 3 <= 16 ? 16 : 32; }

// Small parameters copied to LDS once per launch (offsets in floats).
struct PLay {
    static constexpr int ln1_g = 0, ln1_b = 32, attn_b = 64, proj_b = 160, ln2_g = 192, ln2_b = 224,
                         fc_b = 256, mp_b = 384, size = 416;
};
struct ParamLDS {
    int emb_w, emb_b, layers, lnf_g, lnf_b, head_w, head_b, total;
    __host__ __device__ static ParamLDS make(int F, int L, int A) {
        ParamLDS p;
        int o = 0;
        p.emb_w = o; o += F * kE;
        p.emb_b = o; o += kE;
        p.layers = o; o += L * PLay::size;
        p.lnf_g = o; o += kE;
        p.lnf_b = o; o += kE;
        p.head_w = o; o += kE * A;
        p.head_b = o; o += A;
        p.total = (o + 3) & ~3;
        return p;
    }
};

__host__ inline size_t decode_smem_bytes(const ModelView& M) {
    return sizeof(Smem) + sizeof(float) * (size_t)ParamLDS::make(M.F, M.n_layer, M.A).total;
}

// LDS block of the rollout after ParamLDS (offsets in floats): the embedding of
// every bandit token up to its reward term, base[k] = ((w_s + w_a=k) + w_s') + emb_b
// for k < A and base[A] = w_s + emb_b (the query token), then g0 and bvp of
// every layer (kE floats per layer each) and the folded matrices Wvp and G.
struct RolloutLDS {
    int means, base, g0, bvp, wvp, G, gx, gx0, total;
    // l0m: block 0 on the matrix cores (l0_tiles) -- its extra u-projection columns
    // gx [E][C] (alpha, gamma, beta[0..A] of l0_tiles as linear maps of xn) and gx0 [C],
    // C = l0_cols(A)
    __host__ __device__ static RolloutLDS make(int A, int L, bool with_G = true, bool l0m = false) {
        RolloutLDS r;
        r.means = 0;               // the tile's arm means, double [kM][A]
        r.base = 2 * kM * A;
        r.g0 = r.base + (A + 1) * kE;
        r.bvp = r.g0 + L * kE;
        r.wvp = r.bvp + L * kE;  // Wv Wproj of every layer (c_proj's B operand, read from LDS)
        r.G = r.wvp + L * kE * kE;  // Wq Wk^T of every layer (the u projection's B operand)
        r.gx = r.G + (with_G ? L * kE * kE : 0);
        r.gx0 = r.gx + kE * l0_cols(A);
        r.total = l0m ? r.gx0 + l0_cols(A) : r.gx;
        return r;
    }
};

__host__ inline size_t rollout_smem_bytes(const ModelView& M, bool with_G, bool l0m = false) {
    return decode_smem_bytes(M) + sizeof(float) * (size_t)RolloutLDS::make(M.A, M.n_layer, with_G, l0m).total;
}

template <int NT>
__device__ inline void load_params(float* P, const ParamLDS& pl, const ModelView& M) {
    const int tid = threadIdx.x;
    for (int i = tid; i < M.F * kE; i += NT) P[pl.emb_w + i] = M.emb_w[i];
    for (int i = tid; i < kE; i += NT) {
        P[pl.emb_b + i] = M.emb_b[i];
        P[pl.lnf_g + i] = M.lnf_g[i];
        P[pl.lnf_b + i] = M.lnf_b[i];
    }
    for (int i = tid; i < M.n_layer * PLay::size; i += NT) {
        const int l = i / PLay::size, k = i % PLay::size;
        const float* W = M.layers + (size_t)l * LayerOff::size;
        float v;
        if (k < PLay::ln1_b) v = W[LayerOff::ln1_g + k];
        else if (k < PLay::attn_b) v = W[LayerOff::ln1_b + k - PLay::ln1_b];
        else if (k < PLay::proj_b) v = W[LayerOff::attn_b + k - PLay::attn_b];
        else if (k < PLay::ln2_g) v = W[LayerOff::proj_b + k - PLay::proj_b];
        else if (k < PLay::ln2_b) v = W[LayerOff::ln2_g + k - PLay::ln2_g];
        else if (k < PLay::fc_b) v = W[LayerOff::ln2_b + k - PLay::ln2_b];
        else if (k < PLay::mp_b) v = W[LayerOff::fc_b + k - PLay::fc_b];
        else v = W[LayerOff::mp_b + k - PLay::mp_b];
        P[pl.layers + i] = v;
    }
    for (int i = tid; i < kE * M.A; i += NT) P[pl.head_w + i] = M.head_w[i];
    for (int i = tid; i < M.A; i += NT) P[pl.head_b + i] = M.head_b[i];
}

// Sum over the 8 lanes of an aligned lane group with DPP (VALU, no LDS
// round trip): xor 1 and xor 2 by quad_perm, then row_half_mirror pairs the two
// quads of the group.  Every lane of the group gets the same value, bit-identical
// to the xor-1/2/4 shuffle butterfly.
__device__ inline float dpp_sum8(float d) {
    d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0xB1, 0xF, 0xF, false));
    d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x4E, 0xF, 0xF, false));
    d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x141, 0xF, 0xF, false));
    return d;
}

// Sum over the 16 lanes of a DPP row: dpp_sum8, then row_mirror (lane i <-> 15-i)
// pairs the row's two 8-lane groups (every lane of a group holds its group sum,
// so this equals the xor-8 step).
__device__ inline float dpp_sum16(float d) {
    d = dpp_sum8(d);
    d += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x140, 0xF, 0xF, false));
    return d;
}

// lane i <- lane i ^ 8 (row_ror:8 within each 16-lane row)
__device__ inline float dpp_xor8(float d) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, d), 0x128, 0xF, 0xF, false));
}

// LayerNorm of one 32-wide row held by the 32 lanes of a half-wave: the two
// row sums are 16-lane DPP reductions plus one xor-16 exchange.
__device__ inline float ln_halfwave(float v, float g, float b, float* mean_out = nullptr, float* rstd_out = nullptr) {
    float s = dpp_sum16(v);
    s += __shfl_xor(s, 16, 32);
    const float mean = s * (1.0f / kE);
    const float d = v - mean;
    float s2 = dpp_sum16(d * d);
    s2 += __shfl_xor(s2, 16, 32);
    const float rstd = __builtin_amdgcn_rsqf(s2 * (1.0f / kE) + 1e-5f);
    if (mean_out) {
        *mean_out = mean;
        *rstd_out = rstd;
    }
    return fmaf(d * rstd, g, b);
}

__device__ inline float gelu_new(float x) {
    // 0.5*x*(1 + tanh(z)), z = sqrt(2/pi)*(x + 0.044715*x^3) (transformers/activations.py:65),
    // evaluated as x * sigmoid(2z) = x / (1 + 2^(-2z log2 e)) with v_exp_f32 / v_rcp_f32
    const float c1 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
    const float c2 = c1 * 0.044715f;
    const float e = __builtin_amdgcn_exp2f(x * fmaf(x * x, c2, c1));
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// Packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32): two lanes' worth of
// fp32 work per VALU instruction, each half rounded exactly like the scalar op.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline f2 splat2(float s) { return f2{s, s}; }
__device__ inline f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Calls f(integral_constant<R'>) for the smallest power of two R' <= R with
// 8 R' >= rem: the last, partial chunk of a stream runs only the rows it needs.
template <int R, class F>
__device__ inline void tail_rows(int rem, F&& f) {
    if constexpr (R == 1) {
        f(std::integral_constant<int, 1>{});
    } else {
        if (rem > 8 * (R / 2)) f(std::integral_constant<int, R>{});
        else tail_rows<R / 2>(rem, f);
    }
}

// Flash-decoding attention of one task (one wave): positions 0..pos-1 from the
// cache (global), position pos from LDS.  Writes o = softmax(qK^T/sqrt(E)) V.
// KV_SAME (the rollout's blocks >= 1): keys and values are one stream (the
// LayerNorm outputs y_p, see attend_l0 for the algebra), read once.
// Cached rows of positions < pin (wave-uniform, a multiple of 8 * NR) are read with
// the default cache policy, later ones non-temporally (see BanditRolloutParams::pin).
// Accumulators are packed pairs (lo = dims 4c, 4c+1; hi = 4c+2, 4c+3).
template <bool KV_SAME = false, int NR = kRows, int PS = kE>
__device__ __attribute__((always_inline)) inline float4 attend_one(const float* __restrict__ kc, const float* __restrict__ vc, int pos,
                                    const float* q, const float* kcur, const float* vcur, float* o,
                                    int lane, int pin = 0) {
    const int g = lane >> 3, c = lane & 7;
    const float scale = 0.17677669529663687f * 1.4426950408889634f;  // 32 ** -0.5 * log2(e): exp2 domain
    const floatx4 q4 = *reinterpret_cast<const floatx4*>(q + 4 * c);
    float m = -1e30f, l = 0.f;
    f2 alo = {0.f, 0.f}, ahi = {0.f, 0.f};
    // KV_SAME (the rollout's one y stream per task): a buffer descriptor on the task's stream base,
    // which is wave-uniform (read into SGPRs; readfirstlane returns int, so through unsigned first,
    // or a set bit 31 of the low word would sign-extend over the high word)
    __amdgpu_buffer_rsrc_t rs;
    if constexpr (KV_SAME) {
        const unsigned long long kb = reinterpret_cast<unsigned long long>(kc);
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)kb);
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(kb >> 32));
        const unsigned long long ku = (unsigned long long)lo | ((unsigned long long)hi << 32);
        rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ku), (short)0, 0x7fffffff, 0x00020000);
    }
    // one chunk of 8 * R positions; NT: non-temporal loads; FULL: every position of the chunk is
    // below pos (the whole chunks), so no row is predicated: the R loads issue back to back
    // without a branch and an EXEC mask per row
    auto chunk = [&](int base, auto ntc, auto nrc, auto fullc) {
        constexpr bool NT = decltype(ntc)::value;
        constexpr int R = decltype(nrc)::value;
        constexpr bool FULL = decltype(fullc)::value;
        floatx4 kk[R], vv[R];
        if constexpr (KV_SAME && !FULL) {
            // the partial last chunk: rows past pos re-read position pos - 1 (masked in the scores
            // below), so every load is unconditional and they issue back to back
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int pm = min(base + 8 * r + g, pos - 1);
                kk[r] = __builtin_bit_cast(floatx4,
                                           __builtin_amdgcn_raw_buffer_load_b128(rs, (pm * PS + 4 * c) * 4, 0, NT ? 2 : 0));
                vv[r] = kk[r];
            }
        } else if constexpr (FULL && KV_SAME) {
            // whole chunk: the lane's byte offset (its g rows and c float4s) in a VGPR that stays
            // fixed, the row base (base + 8 r positions) as the wave-uniform soffset: no 64-bit
            // address arithmetic per row
            const int voff = (g * PS + 4 * c) * 4;
            const int sbase = __builtin_amdgcn_readfirstlane(base * PS * 4);  // uniform: an SGPR offset
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int soff = sbase + 8 * r * PS * 4;
                kk[r] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, NT ? 2 : 0));
                vv[r] = kk[r];
            }
        } else
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int p = base + 8 * r + g;
            if (FULL || p < pos) {
                // non-temporal: each K/V row is read once per step by this CU only, so it
                // must not evict the weights every workgroup re-reads from L2
                const floatx4* ks = reinterpret_cast<const floatx4*>(kc + (size_t)p * PS) + c;
                kk[r] = NT ? __builtin_nontemporal_load(ks) : *ks;
                if (KV_SAME) {
                    vv[r] = kk[r];
                } else {
                    const floatx4* vs = reinterpret_cast<const floatx4*>(vc + (size_t)p * PS) + c;
                    vv[r] = NT ? __builtin_nontemporal_load(vs) : *vs;
                }
            } else {
                kk[r] = floatx4{0.f, 0.f, 0.f, 0.f};
                vv[r] = kk[r];
            }
        }
        float s[R];
        float mx = -1e30f;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float d = q4.x * kk[r].x;
            d = fmaf(q4.y, kk[r].y, d);
            d = fmaf(q4.z, kk[r].z, d);
            d = fmaf(q4.w, kk[r].w, d);
            d = dpp_sum8(d);
            const int p = base + 8 * r + g;
            s[r] = (FULL || p < pos) ? d * scale : -INFINITY;
            mx = fmaxf(mx, s[r]);
        }
        const float mn = fmaxf(m, mx);
        const float corr = __builtin_amdgcn_exp2f(m - mn);
        l *= corr;
        alo *= splat2(corr);
        ahi *= splat2(corr);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float pr = __builtin_amdgcn_exp2f(s[r] - mn);
            l += pr;
            alo = pk_fma(splat2(pr), vv[r].lo, alo);
            ahi = pk_fma(splat2(pr), vv[r].hi, ahi);
        }
        m = mn;
    };
    constexpr auto full = std::integral_constant<int, NR>{};
    int base = 0;
    // whole chunks; the pinned ones (default cache policy) first
#pragma unroll 1
    for (const int pe = min(pos, pin) & ~(8 * NR - 1); base < pe; base += 8 * NR)
        chunk(base, std::false_type{}, full, std::true_type{});
#pragma unroll 1
    for (const int pe = pos & ~(8 * NR - 1); base < pe; base += 8 * NR)
        chunk(base, std::true_type{}, full, std::true_type{});
    if (base < pos) {  // the partial last chunk, with only as many rows as it needs
        const bool pinned = base < pin;
        tail_rows<NR>(pos - base, [&](auto nrc) {
            if (pinned) chunk(base, std::false_type{}, nrc, std::false_type{});
            else chunk(base, std::true_type{}, nrc, std::false_type{});
        });
    }
    {   // the new position (group 0 only; all lanes run the shuffles)
        const floatx4 k4 = *reinterpret_cast<const floatx4*>(kcur + 4 * c);
        const floatx4 v4 = *reinterpret_cast<const floatx4*>(vcur + 4 * c);
        float d = q4.x * k4.x;
        d = fmaf(q4.y, k4.y, d);
        d = fmaf(q4.z, k4.z, d);
        d = fmaf(q4.w, k4.w, d);
        d = dpp_sum8(d);
        if (g == 0) {
            const float sc = d * scale;
            const float mn = fmaxf(m, sc);
            const float corr = __builtin_amdgcn_exp2f(m - mn);
            const float pr = __builtin_amdgcn_exp2f(sc - mn);
            l = l * corr + pr;
            alo = pk_fma(splat2(pr), v4.lo, alo * splat2(corr));
            ahi = pk_fma(splat2(pr), v4.hi, ahi * splat2(corr));
            m = mn;
        }
    }
#pragma unroll
    for (int off = 8; off <= 32; off <<= 1) {  // xor 8 by DPP (row_ror:8), 16 and 32 by ds_bpermute
        auto xch = [&](float v) { return off == 8 ? dpp_xor8(v) : __shfl_xor(v, off); };
        const float mo = xch(m);
        const float lo = xch(l);
        const f2 olo = {xch(alo.x), xch(alo.y)};
        const f2 ohi = {xch(ahi.x), xch(ahi.y)};
        const float mn = fmaxf(m, mo);
        const float sa = __builtin_amdgcn_exp2f(m - mn), sb = __builtin_amdgcn_exp2f(mo - mn);
        l = l * sa + lo * sb;
        alo = alo * splat2(sa) + olo * splat2(sb);
        ahi = ahi * splat2(sa) + ohi * splat2(sb);
        m = mn;
    }
    // every lane holds dims 4c..4c+3 of the result after the butterfly
    const float inv = 1.0f / l;
    alo *= splat2(inv);
    ahi *= splat2(inv);
    const float4 res = make_float4(alo.x, alo.y, ahi.x, ahi.y);
    if (o && lane < 8) *reinterpret_cast<float4*>(o + 4 * c) = res;
    return res;
}

// Block-0 attention of one bandit task (one wave) without a K/V cache.  Every
// bandit context token is [1, onehot(a), 1, r], so block 0's input at position p
// is x_p = fma(r_p, w_r, base[a_p]) + wpe[p], rebuilt from the token record
// (a_p, r_p, ...; TokRec) instead of streaming 256 B of K and V.  With y_p = LN1(x_p) =
// rstd_p d_p * g + b (d_p = x_p - mean_p):
//   q . k_p = y_p . (Wk q) + const = rstd_p d_p . (g * u) + const'   (u = Wk q)
//   sum_p P_p v_p = (sum_p P_p y_p) Wv + bv
// The constants shift every score alike and cancel in the softmax; Wv, bv are
// folded into c_proj (L0Off::Wvp, bvp).  Writes o = sum_p P_p y_p.  The current
// position's x is xcur (the residual row, before attention).  Scores are kept in
// the log2 domain (v_exp_f32).
// tok: the task's token records, TS float4 apart per position (tokrec)
template <int TS>
__device__ __attribute__((always_inline)) inline float4 attend_l0(const float4* __restrict__ tok, const float* __restrict__ wpe, int pos,
                                 const float* u, const float* xcur, const float* baseT, const float* wr,
                                 const float* lng, const float* lnb, float* o, int lane) {
    const int g = lane >> 3, c = lane & 7;
    const float scale2 = 0.17677669529663687f * 1.4426950408889634f;  // 32 ** -0.5 * log2(e)
    const floatx4 u4 = *reinterpret_cast<const floatx4*>(u + 4 * c);
    const floatx4 g4 = *reinterpret_cast<const floatx4*>(lng + 4 * c);
    const floatx4 gu = g4 * u4;
    const floatx4 wr4 = *reinterpret_cast<const floatx4*>(wr + 4 * c);
    const float* bT = baseT + 4 * c;
    // centred row, 1/std and log2-domain score of one position's x (8-lane group sums)
    auto row = [&](floatx4 x, floatx4& d, float& rstd, float& sc) {
        const float mean = dpp_sum8((x.x + x.y) + (x.z + x.w)) * (1.0f / kE);
        d.lo = x.lo - splat2(mean);
        d.hi = x.hi - splat2(mean);
        float vv = d.x * d.x;
        vv = fmaf(d.y, d.y, vv);
        vv = fmaf(d.z, d.z, vv);
        vv = fmaf(d.w, d.w, vv);
        float dg = d.x * gu.x;
        dg = fmaf(d.y, gu.y, dg);
        dg = fmaf(d.z, gu.z, dg);
        dg = fmaf(d.w, gu.w, dg);
        vv = dpp_sum8(vv);
        dg = dpp_sum8(dg);
        rstd = __builtin_amdgcn_rsqf(vv * (1.0f / kE) + 1e-5f);
        sc = (rstd * dg) * scale2;
    };
    float m = -1e30f, l = 0.f;
    f2 alo = {0.f, 0.f}, ahi = {0.f, 0.f};
    // one chunk of 8 * R positions
    // one chunk of 8 * R positions; the ln_1 statistics come with the token record
    auto chunk = [&](int base, auto nrc) {
        constexpr int R = decltype(nrc)::value;
        float4 tk[R];
        floatx4 wp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {  // past the end: re-read position pos-1, masked below
            const int p = min(base + 8 * r + g, pos - 1);
            tk[r] = tok[(size_t)p * TS];
            wp[r] = *reinterpret_cast<const floatx4*>(wpe + (size_t)p * kE + 4 * c);
        }
        floatx4 d[R];
        float s[R];
        float mx = -1e30f;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const floatx4 b4 = *reinterpret_cast<const floatx4*>(bT + __float_as_int(tk[r].x) * kE);
            const f2 rr = splat2(tk[r].y), mu = splat2(-tk[r].z);
            d[r].lo = (pk_fma(rr, wr4.lo, b4.lo) + wp[r].lo) + mu;
            d[r].hi = (pk_fma(rr, wr4.hi, b4.hi) + wp[r].hi) + mu;
            float dg = d[r].x * gu.x;
            dg = fmaf(d[r].y, gu.y, dg);
            dg = fmaf(d[r].z, gu.z, dg);
            dg = fmaf(d[r].w, gu.w, dg);
            dg = dpp_sum8(dg);
            s[r] = (base + 8 * r + g < pos) ? (tk[r].w * dg) * scale2 : -INFINITY;
            mx = fmaxf(mx, s[r]);
        }
        const float mn = fmaxf(m, mx);
        const float corr = __builtin_amdgcn_exp2f(m - mn);
        l *= corr;
        alo *= splat2(corr);
        ahi *= splat2(corr);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float pr = __builtin_amdgcn_exp2f(s[r] - mn);
            l += pr;
            const f2 w = splat2(pr * tk[r].w);
            alo = pk_fma(w, d[r].lo, alo);
            ahi = pk_fma(w, d[r].hi, ahi);
        }
        m = mn;
    };
    int base = 0;
#pragma unroll 1
    for (const int pe = pos & ~(8 * kRows - 1); base < pe; base += 8 * kRows)
        chunk(base, std::integral_constant<int, kRows>{});
    if (base < pos) tail_rows<kRows>(pos - base, [&](auto nrc) { chunk(base, nrc); });
    {   // the current position (group 0 merges it; all lanes run the group sums)
        floatx4 dc;
        float rc, sc;
        row(*reinterpret_cast<const floatx4*>(xcur + 4 * c), dc, rc, sc);
        if (g == 0) {
            const float mn = fmaxf(m, sc);
            const float corr = __builtin_amdgcn_exp2f(m - mn);
            const float pr = __builtin_amdgcn_exp2f(sc - mn);
            const f2 w = splat2(pr * rc);
            l = l * corr + pr;
            alo = pk_fma(w, dc.lo, alo * splat2(corr));
            ahi = pk_fma(w, dc.hi, ahi * splat2(corr));
            m = mn;
        }
    }
#pragma unroll
    for (int off = 8; off <= 32; off <<= 1) {  // xor 8 by DPP (row_ror:8), 16 and 32 by ds_bpermute
        auto xch = [&](float v) { return off == 8 ? dpp_xor8(v) : __shfl_xor(v, off); };
        const float mo = xch(m);
        const float lo = xch(l);
        const f2 olo = {xch(alo.x), xch(alo.y)};
        const f2 ohi = {xch(ahi.x), xch(ahi.y)};
        const float mn = fmaxf(m, mo);
        const float sa = __builtin_amdgcn_exp2f(m - mn), sb = __builtin_amdgcn_exp2f(mo - mn);
        l = l * sa + lo * sb;
        alo = alo * splat2(sa) + olo * splat2(sb);
        ahi = ahi * splat2(sa) + ohi * splat2(sb);
        m = mn;
    }
    // sum_p P_p y_p = g * (sum_p P_p rstd_p d_p) + b   (sum_p P_p = 1); every lane holds dims 4c..4c+3
    const f2 inv = splat2(1.0f / l);
    const floatx4 b4 = *reinterpret_cast<const floatx4*>(lnb + 4 * c);
    const f2 rlo = pk_fma(g4.lo, alo * inv, b4.lo), rhi = pk_fma(g4.hi, ahi * inv, b4.hi);
    const float4 res = make_float4(rlo.x, rlo.y, rhi.x, rhi.y);
    if (o && lane < 8) *reinterpret_cast<float4*>(o + 4 * c) = res;
    return res;
}

// Block-0 attention of a whole tile on the matrix cores (L0M: tile of 8 tasks, NA =
// A + 1 token kinds).  With TokRec (a_p, r_p, mean_p, rstd_p), gu = g * u and
// x_p = r_p w_r + base[a_p] + wpe[p] (attend_l0):
//   score_p = rstd_p ((x_p - mean_p) . gu) = rstd_p (r_p alpha + beta[a_p] + wpe[p] . gu - mean_p gamma)
//   sum_p w_p (x_p - mean_p) = (sum w r) w_r + sum_k (sum_{a_p = k} w_p) base[k] + sum_p w_p wpe[p] - (sum w mean) 1
// with alpha = w_r . gu, beta[k] = base[k] . gu, gamma = sum gu (per task and step: the
// u projection's extra columns, kept in S.vcur) and w_p = P_p rstd_p.  The only
// per-position vector terms involve wpe, which every task shares: the scores are one
// [16 positions x 32] x [32 x 16 tasks] MFMA product per 16-position tile and the
// weighted wpe sum one [32 x 16 positions] x [16 x 16 tasks] product; everything else
// is per-(position, task) scalar work, one element per lane and register.  Wave w
// takes the tiles w, w + 8, ...; its partial softmax state per task (m, l, the scalar
// sums, the arm sums and the wpe sum) goes to part[w][task][kL0Part] for l0_merge.
constexpr int kL0Part = 64;  // floats per (wave, task) partial of l0_tiles (36 + NA <= 64)

template <int NA, int TILE>
__device__ __attribute__((always_inline)) inline void l0_tiles(const float* __restrict__ rec_base,
                                                               int ntask, int pos, const float* __restrict__ wpe,
                                                               const float* q, const float* cst, const float* lng,
                                                               float* part, int wave, int lane) {
    const int n = lane & 15, j = lane >> 4;
    const bool tv = n < ntask;  // lanes of columns >= the tile's live tasks carry zeros
    const float scale2 = 0.17677669529663687f * 1.4426950408889634f;  // 32 ** -0.5 * log2(e)
    // B operand of the score product: gu[task n][dim 8j + s] (k-step s takes dims {8j + s})
    float gb[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) gb[s] = tv ? lng[8 * j + s] * q[n * kE + 8 * j + s] : 0.f;
    const float* cn = cst + (tv ? n : 0) * kE;
    const float alpha = cn[0], gamma = cn[1];
    // this lane's task's records, TILE float4 apart per position (tokrec)
    const float4* rec = reinterpret_cast<const float4*>(rec_base) + (tv ? n : 0);
    float m = -1e30f, l = 0.f, sr = 0.f, sm = 0.f;
    float W[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) W[k] = 0.f;
    floatx4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll 1
    for (int p0 = 16 * wave; p0 < pos; p0 += 16 * 8) {
        // every global load of the tile first (independent; consumed in issue order):
        // the score operand rows, the 4 token records, the wpe operand of the output product
        const float* wrow = wpe + (size_t)min(p0 + n, pos - 1) * kE + 8 * j;
        const floatx4 wa0 = *reinterpret_cast<const floatx4*>(wrow);
        const floatx4 wa1 = *reinterpret_cast<const floatx4*>(wrow + 4);
        float4 R[4];
        float wo0[4], wo1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) R[r] = rec[(size_t)min(p0 + 4 * j + r, pos - 1) * TILE];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* wr = wpe + (size_t)min(p0 + 4 * j + r, pos - 1) * kE + n;
            wo0[r] = wr[0];
            wo1[r] = wr[16];
        }
        __builtin_amdgcn_sched_barrier(0);
        // scores: D[position p0 + 4j + r][task n] = wpe[p] . gu_n (two chains of 4)
        floatx4 sa = {0.f, 0.f, 0.f, 0.f}, sb = sa;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            sa = __builtin_amdgcn_mfma_f32_16x16x4f32(wa0[s], gb[s], sa, 0, 0, 0);
            sb = __builtin_amdgcn_mfma_f32_16x16x4f32(wa1[s], gb[4 + s], sb, 0, 0, 0);
        }
        float beta[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) beta[r] = cn[2 + __float_as_int(R[r].x)];
        float sc[4];
        float mx = -1e30f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = p0 + 4 * j + r;
            float t = fmaf(R[r].y, alpha, beta[r]) + (sa[r] + sb[r]);
            t = fmaf(-R[r].z, gamma, t);
            sc[r] = (tv && p < pos) ? (R[r].w * t) * scale2 : -INFINITY;
            mx = fmaxf(mx, sc[r]);
        }
        // one running max per task: over the 4 lane groups holding its positions
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mn = fmaxf(m, mx);
        const float corr = __builtin_amdgcn_exp2f(m - mn);
        l *= corr;
        sr *= corr;
        sm *= corr;
#pragma unroll
        for (int k = 0; k < NA; ++k) W[k] *= corr;
        o0 *= corr;
        o1 *= corr;
        m = mn;
        float wv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float pr = __builtin_amdgcn_exp2f(sc[r] - mn);
            l += pr;
            const float w = pr * R[r].w;
            wv[r] = w;
            sr = fmaf(w, R[r].y, sr);
            sm = fmaf(w, R[r].z, sm);
            const int ak = __float_as_int(R[r].x);
#pragma unroll
            for (int k = 0; k < NA; ++k) W[k] += (ak == k) ? w : 0.f;
        }
        // D2[dim 16 dt + 4j + i][task n] += sum over the tile's positions of wpe[p][dim] w[p][n]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            o0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wo0[r], wv[r], o0, 0, 0, 0);
            o1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wo1[r], wv[r], o1, 0, 0, 0);
        }
    }
    // the scalar sums over the 4 lane groups of each task
    auto red = [](float v) {
        v += __shfl_xor(v, 16);
        return v + __shfl_xor(v, 32);
    };
    l = red(l);
    sr = red(sr);
    sm = red(sm);
#pragma unroll
    for (int k = 0; k < NA; ++k) W[k] = red(W[k]);
    if (n < 8) {
        float* pp = part + (wave * 8 + n) * kL0Part;
        *reinterpret_cast<floatx4*>(pp + 4 * j) = o0;
        *reinterpret_cast<floatx4*>(pp + 16 + 4 * j) = o1;
        if (j == 0) {
            pp[32] = m;
            pp[33] = l;
            pp[34] = sr;
            pp[35] = sm;
#pragma unroll
            for (int k = 0; k < NA; ++k) pp[36 + k] = W[k];
        }
    }
}

// Combines the 8 waves' l0_tiles partials of one task (one wave, lane (g, c) forms
// dims 4c..4c+3), adds the current position (its x is xcur) and returns
// o = g * (sum_p P_p rstd_p (x_p - mean_p)) + b, as attend_l0.
template <int NA>
__device__ __attribute__((always_inline)) inline float4 l0_merge(const float* part, int t, const float* u,
                                                                 const float* xcur, const float* baseT,
                                                                 const float* wr, const float* lng, const float* lnb,
                                                                 int lane) {
    const int g = lane >> 3, c = lane & 7;
    const float scale2 = 0.17677669529663687f * 1.4426950408889634f;
    float mw[8];
    float M = -1e30f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        mw[w] = part[(w * 8 + t) * kL0Part + 32];
        M = fmaxf(M, mw[w]);
    }
    float L = 0.f, SR = 0.f, SM = 0.f;
    float Wk[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) Wk[k] = 0.f;
    f2 olo = {0.f, 0.f}, ohi = {0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const float* pp = part + (w * 8 + t) * kL0Part;
        const float sw = __builtin_amdgcn_exp2f(mw[w] - M);
        L = fmaf(sw, pp[33], L);
        SR = fmaf(sw, pp[34], SR);
        SM = fmaf(sw, pp[35], SM);
#pragma unroll
        for (int k = 0; k < NA; ++k) Wk[k] = fmaf(sw, pp[36 + k], Wk[k]);
        const floatx4 o4 = *reinterpret_cast<const floatx4*>(pp + 4 * c);
        olo = pk_fma(splat2(sw), o4.lo, olo);
        ohi = pk_fma(splat2(sw), o4.hi, ohi);
    }
    // V = sum_p w_p (x_p - mean_p) over the cached positions, dims 4c..4c+3
    const floatx4 wr4 = *reinterpret_cast<const floatx4*>(wr + 4 * c);
    olo = pk_fma(splat2(SR), wr4.lo, olo);
    ohi = pk_fma(splat2(SR), wr4.hi, ohi);
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        const floatx4 b4 = *reinterpret_cast<const floatx4*>(baseT + k * kE + 4 * c);
        olo = pk_fma(splat2(Wk[k]), b4.lo, olo);
        ohi = pk_fma(splat2(Wk[k]), b4.hi, ohi);
    }
    olo -= splat2(SM);
    ohi -= splat2(SM);
    // the current position (every lane computes it; its group sums are 8-lane DPP)
    const floatx4 u4 = *reinterpret_cast<const floatx4*>(u + 4 * c);
    const floatx4 g4 = *reinterpret_cast<const floatx4*>(lng + 4 * c);
    const floatx4 gu = g4 * u4;
    const floatx4 x = *reinterpret_cast<const floatx4*>(xcur + 4 * c);
    const float mean = dpp_sum8((x.x + x.y) + (x.z + x.w)) * (1.0f / kE);
    floatx4 d;
    d.lo = x.lo - splat2(mean);
    d.hi = x.hi - splat2(mean);
    float vv = d.x * d.x;
    vv = fmaf(d.y, d.y, vv);
    vv = fmaf(d.z, d.z, vv);
    vv = fmaf(d.w, d.w, vv);
    float dg = d.x * gu.x;
    dg = fmaf(d.y, gu.y, dg);
    dg = fmaf(d.z, gu.z, dg);
    dg = fmaf(d.w, gu.w, dg);
    vv = dpp_sum8(vv);
    dg = dpp_sum8(dg);
    const float rc = __builtin_amdgcn_rsqf(vv * (1.0f / kE) + 1e-5f);
    const float sc = (rc * dg) * scale2;
    const float mn = fmaxf(M, sc);
    const float corr = __builtin_amdgcn_exp2f(M - mn);
    const float pr = __builtin_amdgcn_exp2f(sc - mn);
    L = L * corr + pr;
    const f2 wc = splat2(pr * rc);
    olo = pk_fma(wc, d.lo, olo * splat2(corr));
    ohi = pk_fma(wc, d.hi, ohi * splat2(corr));
    const f2 inv = splat2(1.0f / L);
    const floatx4 b4 = *reinterpret_cast<const floatx4*>(lnb + 4 * c);
    const f2 rlo = pk_fma(g4.lo, olo * inv, b4.lo), rhi = pk_fma(g4.hi, ohi * inv, b4.hi);
    (void)g;
    return make_float4(rlo.x, rlo.y, rhi.x, rhi.y);
}

// The rollout's c_proj + residual + ln_2 for one task inside its attention wave (no
// extra phase or barrier): lane (c = l & 7, g = l >> 3) holds attention dims
// o4 = o[4c..4c+3] and forms the partial outputs j = 4g..4g+3 over them from the
// folded Wvp ([k][j], LDS); an 8-lane DPP sum over c completes them.  Then
// x += out + bvp and LayerNorm ln_2 over the 32 j (groups g combined by xor 8 / 16
// / 32); lane c == 0 of each group writes x[4g..] and xn[4g..].
__device__ inline void proj_ln_task(float4 o4, const float* Wvp, const float* bvp, const float* lng,
                                    const float* lnb, float* xrow, float* xnrow, int lane) {
    const int c = lane & 7, g = lane >> 3;
    const float ov[4] = {o4.x, o4.y, o4.z, o4.w};
    f2 alo = {0.f, 0.f}, ahi = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const floatx4 w = *reinterpret_cast<const floatx4*>(Wvp + (4 * c + i) * kE + 4 * g);
        alo = pk_fma(splat2(ov[i]), w.lo, alo);
        ahi = pk_fma(splat2(ov[i]), w.hi, ahi);
    }
    float4 acc;
    acc.x = dpp_sum8(alo.x);
    acc.y = dpp_sum8(alo.y);
    acc.z = dpp_sum8(ahi.x);
    acc.w = dpp_sum8(ahi.y);
    const float4 bv = *reinterpret_cast<const float4*>(bvp + 4 * g);
    const float4 xv = *reinterpret_cast<const float4*>(xrow + 4 * g);
    const float x0 = (acc.x + bv.x) + xv.x, x1 = (acc.y + bv.y) + xv.y;
    const float x2 = (acc.z + bv.z) + xv.z, x3 = (acc.w + bv.w) + xv.w;
    auto sum_groups = [](float v) {  // over the 8 groups g: lanes l ^ 8, l ^ 16, l ^ 32
        v += dpp_xor8(v);
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        return v;
    };
    const float mean = sum_groups((x0 + x1) + (x2 + x3)) * (1.0f / kE);
    const float d0 = x0 - mean, d1 = x1 - mean, d2 = x2 - mean, d3 = x3 - mean;
    const float var = sum_groups((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3)) * (1.0f / kE);
    const float rstd = __builtin_amdgcn_rsqf(var + 1e-5f);
    if (c == 0) {
        const float4 gv = *reinterpret_cast<const float4*>(lng + 4 * g);
        const float4 bb = *reinterpret_cast<const float4*>(lnb + 4 * g);
        *reinterpret_cast<float4*>(xrow + 4 * g) = make_float4(x0, x1, x2, x3);
        // xn rows are padded to kLdE floats: 8-B aligned stores
        *reinterpret_cast<float2*>(xnrow + 4 * g) = make_float2(fmaf(d0 * rstd, gv.x, bb.x), fmaf(d1 * rstd, gv.y, bb.y));
        *reinterpret_cast<float2*>(xnrow + 4 * g + 2) =
            make_float2(fmaf(d2 * rstd, gv.z, bb.z), fmaf(d3 * rstd, gv.w, bb.w));
    }
}

template <int TILE>
__device__ inline void zero_smem(Smem& S) {
    float* p = reinterpret_cast<float*>(&S);
    for (int i = threadIdx.x; i < (int)(sizeof(Smem) / sizeof(float)); i += TILE * kWave) p[i] = 0.f;
}

// One decode position for a tile of TILE tasks: S.tok -> S.logits, appending
// K/V of `pos` to the cache kv[2][L][N][max_pos][E].  Per layer:
//   c_attn (MFMA) | attention (wave per task) | c_proj + residual + ln_2 (one wave,
//   in registers) | c_fc -> gelu -> mlp.c_proj (fused, 8 waves, split-K) |
//   split-K reduce + residual + next LayerNorm (half-wave per task)
// `wpe_j` is wpe[pos][tid & 31] (prefetched by the caller); P is the LDS
// parameter block.
// L0R (bandit rollout only): every block runs on folded weights (L0Off) without
// K/V.  Block 0 recomputes its inputs from the (a_p, r_p) token records held in
// layer 0's K slot (attend_l0); block l >= 1 caches y_p = LN1(h_p) (128 B per
// position, layer l's K slot) instead of K and V (256 B): q . k_p = y_p . u +
// const with u = Wk q = xn G + g0, and sum_p P_p v_p = (sum_p P_p y_p) Wv + bv, so
// the same y stream serves as keys and values.  D is the RolloutLDS block.
// L0M (bandit rollout, tile 8): block 0's attention on the matrix cores for NA = L0M
// token kinds (l0_tiles + l0_merge) instead of one wave per task (attend_l0).
template <int TILE, bool L0R = false, bool GL = false, int L0M = 0>
__device__ void decode_position(Smem& S, const float* P, const ParamLDS& pl, const ModelView& M,
                                float* __restrict__ kv, int N, int max_pos, int tile0, int pos, float wpe_j,
                                const float* D = nullptr, int pin = 0, int pin_x = 0) {
    constexpr int kProjWave = TILE - 1;  // a wave with no c_attn tile (TILE >= 8)
    // opaque copy of the thread id: every lane-derived address is recomputed per call
    // instead of being hoisted out of the caller's step loop (128-VGPR budget, no spills)
    int tid_ = threadIdx.x;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: addresses in SGPRs
    // one layer of K (or V); the rollout's task count is padded to whole tiles (kv_tasks)
    const size_t lstride = (size_t)(L0R ? kv_tasks(N) : N) * max_pos * kE;
    const size_t vhalf = (size_t)M.n_layer * lstride;
    const int i16 = lane & 15, kq = lane >> 4;

    // embed_transition + wpe (net.py:52-53; GPT2Model inputs_embeds + position_embeds) + ln_1 of block 0
    if (tid < TILE * 32) {
        const int t = tid >> 5, j = tid & 31;
        float acc = 0.f;
        for (int f = 0; f < M.F; ++f) acc = fmaf(S.tok[t][f], P[pl.emb_w + f * kE + j], acc);
        const float x = (acc + P[pl.emb_b + j]) + wpe_j;
        S.x[t][j] = x;
        float mean, rstd;
        S.xn[t][j] = ln_halfwave(x, P[pl.layers + PLay::ln1_g + j], P[pl.layers + PLay::ln1_b + j], &mean, &rstd);
        const int task = tile0 + t;
        if (L0R && j == 0 && task < N)  // the LayerNorm statistics of this position's TokRec
            *reinterpret_cast<float2*>(tokrec(kv, max_pos, tile0, pos, TILE, t) + 2) = make_float2(mean, rstd);
    }
    bar_lds();
    DPT_STAMP(0);

    // block l's y rows of positions < lpin(l) use the default cache policy (rollout_pin)
    auto lpin = [&](int l) { return pin + (l <= pin_x ? 8 * kYRows : 0); };
    for (int li = 0; li < M.n_layer; ++li) {
        asm volatile("" : "+v"(tid_));  // and per layer (see above)
        const int lane = tid_ & 63, i16 = lane & 15, kq = lane >> 4;
        const float* W = M.layers + (size_t)li * LayerOff::size;
        const float* PL = P + pl.layers + li * PLay::size;
        const bool l0 = L0R && li == 0;
        if (L0R) {
            // u = xn G + g0 (= Wk q), two 16-column tiles; no block stores K/V (block 0
            // keeps token records, blocks >= 1 their LayerNorm outputs y, stored below)
            if (wave < 2) {
                // G from LDS (GL: the rollout's LDS block has room for it) or from L2
                const float* B = GL ? D + RolloutLDS::make(M.A, M.n_layer).G + li * kE * kE + wave * 16
                                    : M.l0 + (size_t)li * L0Off::size + L0Off::G + wave * 16;
                float w[8];
#pragma unroll
                for (int s = 0; s < 8; ++s) w[s] = GL ? B[(4 * s + kq) * kE + i16] : __ldg(B + (4 * s + kq) * kE + i16);
                floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(S.xn[i16][4 * s + kq], w[s], acc, 0, 0, 0);
                const int col = wave * 16 + i16;
                const float bias = D[RolloutLDS::make(M.A, M.n_layer).g0 + li * kE + col];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = kq * 4 + r;
                    if (t < TILE) S.q[t][col] = acc[r] + bias;
                }
            } else if (L0M && li == 0 && wave < 2 + l0_cols(L0M - 1) / 16) {
                // l0_tiles' per-task constants (alpha, gamma, beta[k]) = xn gx + gx0 -> S.vcur
                constexpr int C = l0_cols(L0M - 1);
                const RolloutLDS rl = RolloutLDS::make(M.A, M.n_layer, GL, true);
                const int col = (wave - 2) * 16 + i16;
                floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(S.xn[i16][4 * s + kq], D[rl.gx + (4 * s + kq) * C + col],
                                                               acc, 0, 0, 0);
                const float bias = D[rl.gx0 + col];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = kq * 4 + r;
                    if (t < TILE) S.vcur[t][col] = acc[r] + bias;
                }
            }
        } else if (wave < 6) {
        // c_attn: [16 x 32] x [32 x 96] -> q | k | v, one 16-column tile per wave
            const float* B = W + LayerOff::attn_w + wave * 16;
            float w[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) w[s] = __ldg(B + (size_t)(4 * s + kq) * 3 * kE + i16);
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 8; ++s)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(S.xn[i16][4 * s + kq], w[s], acc, 0, 0, 0);
            const int col = wave * 16 + i16;
            const float bias = PL[PLay::attn_b + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = kq * 4 + r;
                const float v = acc[r] + bias;
                const int task = tile0 + t;
                if (t < TILE) {
                    if (col < kE) {
                        S.q[t][col] = v;
                    } else if (col < 2 * kE) {
                        S.kcur[t][col - kE] = v;
                        if (task < N)  // non-temporal like the stream that reads it back
                            __builtin_nontemporal_store(v, kv + li * lstride + ((size_t)task * max_pos + pos) * kE + col - kE);
                    } else {
                        S.vcur[t][col - 2 * kE] = v;
                        if (task < N)
                            __builtin_nontemporal_store(
                                v, kv + vhalf + li * lstride + ((size_t)task * max_pos + pos) * kE + col - 2 * kE);
                    }
                }
            }
        }
        bar_lds();
        DPT_STAMP(1);
        if constexpr (L0M > 0) {
            if (li == 0) {  // block 0: every wave takes a share of the tile's cached positions
                l0_tiles<L0M, TILE>(tokrec(kv, max_pos, tile0, 0, TILE, 0), min(TILE, N - tile0),
                              pos, M.wpe, &S.q[0][0], &S.vcur[0][0], PL + PLay::ln1_g,
                              &S.part[0][0][0], wave, lane);
                bar_lds();
            }
        }
        // the streaming phase yields issue slots to the other workgroup's latency-bound dense
        // phases (s_setprio; -0.5 % at config 2, -1 % on the linear config)
        if (L0R) __builtin_amdgcn_s_setprio(0);
        // causal self-attention, one wave per task
        if (wave < TILE) {
            const int task = tile0 + wave;
            if (task < N) {
                const float* kc = kv + li * lstride + (size_t)task * max_pos * kE;
                // the rollout's y rows are tile-interleaved: one position of the tile's tasks is
                // TILE adjacent rows
                const float* yc = kv + li * lstride + (size_t)tile0 * max_pos * kE + wave * kE;
                constexpr int YPS = TILE * kE;
                const float* vc = kv + vhalf + li * lstride + (size_t)task * max_pos * kE;
                if (L0R) {
                    const RolloutLDS rl = RolloutLDS::make(M.A, M.n_layer);
                    const float4 o4 =
                        (L0M > 0 && l0) ? l0_merge<(L0M > 0 ? L0M : 1)>(&S.part[0][0][0], wave, S.q[wave], S.x[wave], D + rl.base,
                                                             P + pl.emb_w + (2 + M.A) * kE, PL + PLay::ln1_g,
                                                             PL + PLay::ln1_b, lane)
                        : l0 ? attend_l0<TILE>(reinterpret_cast<const float4*>(tokrec(kv, max_pos, tile0, 0, TILE, wave)), M.wpe, pos, S.q[wave], S.x[wave],
                                       D + rl.base, P + pl.emb_w + (2 + M.A) * kE, PL + PLay::ln1_g,
                                       PL + PLay::ln1_b, nullptr, lane)
                           // scores y_p . u, output sum_p P_p y_p; y_pos is in S.kcur
                           : attend_one<true, kYRows, YPS>(yc, yc, pos, S.q[wave], S.kcur[wave], S.kcur[wave], nullptr,
                                                      lane, lpin(li));
                    // c_proj (folded Wvp) + residual + ln_2 of this task, in this wave
                    proj_ln_task(o4, D + rl.wvp + li * kE * kE, D + rl.bvp + li * kE, PL + PLay::ln2_g,
                                 PL + PLay::ln2_b, S.x[wave], S.xn[wave], lane);
                } else {
                    attend_one(kc, vc, pos, S.q[wave], S.kcur[wave], S.vcur[wave], S.o[wave], lane);
                }
            }
        }
        bar_lds();
        DPT_STAMP(2);
        if (L0R) __builtin_amdgcn_s_setprio(2);
        // c_proj + residual + ln_2, one wave: both 16-column tiles, rows reduced over 16 lanes
        // (the rollout did this per task in the attention phase)
        if (!L0R && wave == kProjWave) {
            const float* B = L0R ? D + RolloutLDS::make(M.A, M.n_layer).wvp + li * kE * kE : W + LayerOff::proj_w;
            float w0[8], w1[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                w0[s] = L0R ? B[(4 * s + kq) * kE + i16] : __ldg(B + (size_t)(4 * s + kq) * kE + i16);
                w1[s] = L0R ? B[(4 * s + kq) * kE + 16 + i16] : __ldg(B + (size_t)(4 * s + kq) * kE + 16 + i16);
            }
            floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const float a = S.o[i16][4 * s + kq];
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w0[s], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w1[s], a1, 0, 0, 0);
            }
            const int c0 = i16, c1 = 16 + i16;
            const float* pb = L0R ? D + RolloutLDS::make(M.A, M.n_layer).bvp + li * kE : PL + PLay::proj_b;
            const float b0 = pb[c0], b1 = pb[c1];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = kq * 4 + r;
                const float x0 = (a0[r] + b0) + S.x[t][c0];
                const float x1 = (a1[r] + b1) + S.x[t][c1];
                float s = x0 + x1;
                s = dpp_sum16(s);
                const float mean = s * (1.0f / kE);
                const float d0 = x0 - mean, d1 = x1 - mean;
                float s2 = d0 * d0 + d1 * d1;
                s2 = dpp_sum16(s2);
                const float rstd = __builtin_amdgcn_rsqf(s2 * (1.0f / kE) + 1e-5f);
                if (t < TILE) {
                    S.x[t][c0] = x0;
                    S.x[t][c1] = x1;
                    S.xn[t][c0] = fmaf(d0 * rstd, PL[PLay::ln2_g + c0], PL[PLay::ln2_b + c0]);
                    S.xn[t][c1] = fmaf(d1 * rstd, PL[PLay::ln2_g + c1], PL[PLay::ln2_b + c1]);
                }
            }
        }
        if (!L0R) bar_lds();
        DPT_STAMP(3);
        // c_fc (computed transposed: hidden units on the MFMA rows) -> gelu_new -> mlp.c_proj
        // partial over this wave's 16 hidden units; the accumulator is the A operand
        // of the second product directly (k order permuted, matched on the B side).
        if (wave < kChunks) {
            const float* W1 = W + LayerOff::fc_w + wave * 16;                          // [E][FF]
            const float* W2 = W + LayerOff::mp_w + (size_t)(wave * 16 + kq * 4) * kE;  // this lane group's rows
            float w1[8], w2a[4], w2b[4];
#pragma unroll
            for (int s = 0; s < 8; ++s) w1[s] = __ldg(W1 + (size_t)(4 * s + kq) * kFF + i16);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                w2a[s] = __ldg(W2 + (size_t)s * kE + i16);
                w2b[s] = __ldg(W2 + (size_t)s * kE + 16 + i16);
            }
            floatx4 ht = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 8; ++s)
                ht = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[s], S.xn[i16][4 * s + kq], ht, 0, 0, 0);
            // ht[r] = h^T[unit 16*wave + 4*kq + r][task i16]
            floatx4 p0 = {0.f, 0.f, 0.f, 0.f}, p1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float hv = gelu_new(ht[s] + PL[PLay::fc_b + wave * 16 + kq * 4 + s]);
                p0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv, w2a[s], p0, 0, 0, 0);
                p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hv, w2b[s], p1, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                S.part[wave][kq * 4 + r][i16] = p0[r];
                S.part[wave][kq * 4 + r][16 + i16] = p1[r];
            }
        }
        bar_lds();
        DPT_STAMP(4);
        // reduce the 8 partials in a fixed tree + bias + residual, then the next LayerNorm
        if (tid < TILE * 32) {
            const int t = tid >> 5, j = tid & 31;
            const float ff = ((S.part[0][t][j] + S.part[1][t][j]) + (S.part[2][t][j] + S.part[3][t][j])) +
                             ((S.part[4][t][j] + S.part[5][t][j]) + (S.part[6][t][j] + S.part[7][t][j]));
            const float x = S.x[t][j] + (ff + PL[PLay::mp_b + j]);
            S.x[t][j] = x;
            const bool last = li + 1 == M.n_layer;
            const float g = last ? P[pl.lnf_g + j] : PL[PLay::size + PLay::ln1_g + j];
            const float b = last ? P[pl.lnf_b + j] : PL[PLay::size + PLay::ln1_b + j];
            const float y = ln_halfwave(x, g, b);
            S.xn[t][j] = y;
            if (L0R && !last) {  // block li+1's y at `pos`: its K/V-cache row (128 B per half-wave)
                S.kcur[t][j] = y;
                const int task = tile0 + t;
                float* yd = kv + (li + 1) * lstride + ((size_t)tile0 * max_pos + (size_t)pos * TILE + t) * kE + j;
                if (task < N) {
                    if (pos < lpin(li + 1)) *yd = y;
                    else __builtin_nontemporal_store(y, yd);
                }
            }
        }
        bar_lds();
        DPT_STAMP(5);
    }
    // pred_actions head: [16 x 32] x [32 x A] (weights in LDS)
    const int ntile = (M.A + 15) >> 4;
    if (wave < ntile) {
        const int col = wave * 16 + i16;
        const int colc = col < M.A ? col : M.A - 1;  // columns beyond A are computed and discarded
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kE / 4; ++s)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(S.xn[i16][4 * s + kq], P[pl.head_w + (4 * s + kq) * M.A + colc],
                                                       acc, 0, 0, 0);
        if (col < M.A) {
            const float bias = P[pl.head_b + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) S.logits[kq * 4 + r][col] = acc[r] + bias;
        }
    }
    if (L0R && ntile == 1) {
        // the rollout selects on wave 0, which wrote every logit: a wave-local LDS hand-off
        // instead of a workgroup barrier (the other waves go on to the step's closing barrier)
        if (wave == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    } else {
        bar_lds();
    }
    DPT_STAMP(6);
}

// dynamic LDS: Smem followed by the parameter block
#define DPT_SMEM_SETUP(TILE_)                                                   \
    extern __shared__ __align__(16) unsigned char smem_raw[];                   \
    Smem& S = *reinterpret_cast<Smem*>(smem_raw);                               \
    float* P = reinterpret_cast<float*>(smem_raw + sizeof(Smem));               \
    const ParamLDS pl = ParamLDS::make(M.F, M.n_layer, M.A);                    \
    zero_smem<TILE_>(S);                                                        \
    load_params<TILE_ * 64>(P, pl, M);                                          \
    __syncthreads();

// ----------------------------------------------------------------------------- kernels

// One decode position for all tasks; tokens (N, F) given.
template <int TILE>
__global__ __launch_bounds__(TILE * 64, 4) void decode_step_kernel(ModelView M, float* kv, int N, int max_pos,
                                                                   int pos, const float* __restrict__ token,
                                                                   float* __restrict__ logits) {
    DPT_SMEM_SETUP(TILE)
    const int tile0 = blockIdx.x * TILE;
    const int tid = threadIdx.x;
    for (int i = tid; i < TILE * kMaxF; i += TILE * 64) {
        const int t = i / kMaxF, f = i % kMaxF;
        S.tok[t][f] = (tile0 + t < N && f < M.F) ? token[(size_t)(tile0 + t) * M.F + f] : 0.f;
    }
    const float wpe_j = M.wpe[(size_t)pos * kE + (tid & 31)];
    __syncthreads();
    decode_position<TILE>(S, P, pl, M, kv, N, max_pos, tile0, pos, wpe_j);
    for (int i = tid; i < TILE * M.A; i += TILE * 64) {
        const int t = i / M.A, a = i % M.A;
        if (tile0 + t < N) logits[(size_t)(tile0 + t) * M.A + a] = S.logits[t][a];
    }
}

// Teacher-forced window forward (= Transformer.forward over query + C context
// rows): positions 0..C decoded in order through the workspace cache; the next
// position's token features and wpe row are prefetched into registers.
template <int TILE>
__global__ __launch_bounds__(TILE * 64, 4) void window_decode_kernel(
    ModelView M, float* kv, int N, int C, const float* __restrict__ query, const float* __restrict__ cs,
    const float* __restrict__ ca, const float* __restrict__ cn, const float* __restrict__ cr, int out_mode,
    float* __restrict__ out) {
    DPT_SMEM_SETUP(TILE)
    const int tile0 = blockIdx.x * TILE;
    const int tid = threadIdx.x;
    const int sd = M.sd, A = M.A;
    const int T = C + 1;
    // this thread's token element: t = tid / kMaxF, f = tid % kMaxF (TILE * kMaxF == TILE * 64 threads)
    const int tt = tid / kMaxF, ff = tid % kMaxF;
    const int ttask = tile0 + tt;
    auto token_elem = [&](int pos) -> float {
        if (ttask >= N || ff >= M.F) return 0.f;
        if (pos == 0) return (ff < sd) ? query[(size_t)ttask * sd + ff] : 0.f;
        const size_t row = (size_t)ttask * C + (pos - 1);
        if (ff < sd) return cs[row * sd + ff];
        if (ff < sd + A) return ca[row * A + (ff - sd)];
        if (ff < 2 * sd + A) return cn[row * sd + (ff - sd - A)];
        return cr[row];
    };
    float tok_next = token_elem(0);
    float wpe_next = M.wpe[tid & 31];
    for (int pos = 0; pos < T; ++pos) {
        S.tok[tt][ff] = tok_next;  // packing (models/net.py:42-51)
        const float wpe_j = wpe_next;
        if (pos + 1 < T) {
            tok_next = token_elem(pos + 1);
            wpe_next = M.wpe[(size_t)(pos + 1) * kE + (tid & 31)];
        }
        bar_lds();
        decode_position<TILE>(S, P, pl, M, kv, N, T, tile0, pos, wpe_j);
        if (out_mode == 0 && pos == C) {
            for (int i = tid; i < TILE * A; i += TILE * 64) {
                const int t = i / A, a = i % A;
                if (tile0 + t < N) out[(size_t)(tile0 + t) * A + a] = S.logits[t][a];
            }
        } else if (out_mode == 1 && pos >= 1) {
            for (int i = tid; i < TILE * A; i += TILE * 64) {
                const int t = i / A, a = i % A;
                if (tile0 + t < N) out[((size_t)(tile0 + t) * C + (pos - 1)) * A + a] = S.logits[t][a];
            }
        }
        __syncthreads();  // K/V stores of `pos` visible before position pos+1 reads them
    }
}

// TokRec: the rollout's record of one bandit token, 16 B per position: (a_p as int
// bits, float(r_p)) written after the selection that chose them, (mean_p, rstd_p) of
// ln_1 of block 0 written by the embedding phase of position p.  Position 0 is the
// query: (A, 0).  Records are tile-interleaved like the y rows, at the start of the
// tile's block-0 K slot: [position][task in tile] (tokrec), so one position of a
// tile's tasks is 128 B (tile 8) or 256 B (tile 16) of adjacent records.
struct BanditRolloutParams {
    int N, H, A, type, sample, n_layer, tile;
    // y rows of positions < pin (+ 8 kYRows for blocks 1..pin_x) use the default cache
    // policy (Infinity-Cache resident), later ones non-temporal (rollout_pin)
    int pin, pin_x;
    int64_t first_task;
    double var;
    uint64_t seed, counter;
    const double* means;
    const double* uniforms;
    const double* noise;
    float* kv;
    int32_t* actions_out;
    double* rewards_out;
    double* arm_value_out;
    float* logits_out;
};

// Block 0's V slot (unused by the K/V-free block 0) holds the per-step draw pairs
// (u = selection uniform, g = reward normal or Bernoulli uniform), tile-interleaved
// like the records: [tile][step][task in tile], 16 B each.
__device__ inline double2* draw_pair(const BanditRolloutParams& Pr, int task, int h) {
    const size_t vhalf = (size_t)Pr.n_layer * kv_tasks(Pr.N) * Pr.H * kE;
    const int tile0 = task / Pr.tile * Pr.tile;
    return reinterpret_cast<double2*>(Pr.kv + vhalf + (size_t)tile0 * Pr.H * kE) + (size_t)h * Pr.tile + (task - tile0);
}

// Every draw of the rollout, one thread per (task, step), before the rollout
// launch: Philox by (step, global task, stream), or the caller's injected draws.
__global__ void rollout_draws_kernel(BanditRolloutParams Pr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Pr.N * Pr.H) return;
    const int task = (int)(i / Pr.H), h = (int)(i % Pr.H);
    const int64_t gtask = Pr.first_task + task;
    double u = 0.0, g;
    const uint64_t ctr = Pr.counter + (uint64_t)h;
    if (Pr.sample)
        u = Pr.uniforms ? Pr.uniforms[(size_t)h * Pr.N + task] : philox_uniform(Pr.seed, ctr, gtask, DPT_STREAM_SELECT);
    if (Pr.noise)
        g = Pr.noise[(size_t)h * Pr.N + task];
    else if (Pr.type == DPT_BANDIT_BERNOULLI)
        g = philox_uniform(Pr.seed, ctr, gtask, DPT_STREAM_REWARD);
    else
        g = philox_normal(Pr.seed, ctr, gtask, DPT_STREAM_REWARD);
    *draw_pair(Pr, task, h) = make_double2(u, g);
}

// select_from_logits with the logits in registers for the configured arm counts
// (5: the bandit configs, 20: the linear-bandit config).
__device__ inline int select_rollout(const float* logits, int A, int sample, double u) {
    auto fixed = [&](auto na) {
        constexpr int NA = decltype(na)::value;
        float lg[NA];
#pragma unroll
        for (int k = 0; k < NA; ++k) lg[k] = logits[k];
        return select_fixed_fast<NA>(lg, sample, 1.0f, u);
    };
    if (A == 5) return fixed(std::integral_constant<int, 5>{});
    if (A == 20) return fixed(std::integral_constant<int, 20>{});
    return select_from_logits(logits, A, sample, 1.0f, u);
}

// The bandit online loop (evals/eval_bandit.py:70-89) for one tile of tasks,
// all H steps: decode -> select -> env step -> append transition.
template <int TILE, bool GL, int L0M = 0>
__global__ __launch_bounds__(TILE * 64, 4) void rollout_bandit_kernel(ModelView M, BanditRolloutParams Pr) {
    DPT_SMEM_SETUP(TILE)
    const int tile0 = blockIdx.x * TILE;
    const int tid = threadIdx.x;
    const int A = Pr.A;
    // block 0 runs K/V-free (attend_l0 / l0_tiles): token embedding table and folded weights in LDS
    float* D = P + pl.total;
    const RolloutLDS rl = RolloutLDS::make(A, M.n_layer, GL, L0M > 0);
    double* means = reinterpret_cast<double*>(D + rl.means);
    for (int i = tid; i < TILE * A; i += TILE * 64) {
        const int t = i / A, k = i % A;
        means[i] = (tile0 + t < Pr.N) ? Pr.means[(size_t)(tile0 + t) * A + k] : 0.0;
    }
    for (int i = tid; i < (A + 1) * kE; i += TILE * 64) {
        const int k = i / kE, j = i % kE;
        const float* ew = P + pl.emb_w;
        // the embedding's own rounding order (decode_position: fmaf over features, + emb_b)
        const float acc = (k < A) ? (ew[j] + ew[(1 + k) * kE + j]) + ew[(1 + A) * kE + j] : ew[j];
        D[rl.base + i] = acc + P[pl.emb_b + j];
    }
    for (int i = tid; i < M.n_layer * kE; i += TILE * 64) {
        const int li = i / kE, j = i % kE;
        D[rl.g0 + i] = M.l0[(size_t)li * L0Off::size + L0Off::g0 + j];
        D[rl.bvp + i] = M.l0[(size_t)li * L0Off::size + L0Off::bvp + j];
    }
    for (int i = tid; i < M.n_layer * kE * kE; i += TILE * 64) {
        const int li = i / (kE * kE), j = i % (kE * kE);
        D[rl.wvp + i] = M.l0[(size_t)li * L0Off::size + L0Off::Wvp + j];
        if (GL) D[rl.G + i] = M.l0[(size_t)li * L0Off::size + L0Off::G + j];
    }
    if constexpr (L0M > 0) {
        // l0_tiles' constants as maps of xn: column c of gx is G v_c and gx0[c] = g0 . v_c for
        // v_0 = g * w_r (alpha), v_1 = g (gamma), v_{2+k} = g * base[k] (beta[k]); fp64 sums
        __syncthreads();  // base[] complete
        const float* g = P + pl.layers + PLay::ln1_g;
        const float* wr = P + pl.emb_w + (2 + A) * kE;
        auto v = [&](int c, int jj) -> double {
            if (c == 0) return (double)g[jj] * wr[jj];
            if (c == 1) return (double)g[jj];
            if (c < 2 + L0M) return (double)g[jj] * D[rl.base + (c - 2) * kE + jj];
            return 0.0;
        };
        const float* G0 = M.l0 + L0Off::G;
        const float* g00 = M.l0 + L0Off::g0;
        constexpr int C = l0_cols(L0M - 1);
        for (int i = tid; i < (kE + 1) * C; i += TILE * 64) {
            const int row = i / C, c = i % C;
            double acc = 0.0;
            for (int jj = 0; jj < kE; ++jj) acc += (row < kE ? (double)G0[row * kE + jj] : (double)g00[jj]) * v(c, jj);
            D[rl.gx + i] = (float)acc;  // row kE lands in gx0 (= gx + kE * C)
        }
    }
    // (a_p, r_p) of this thread's task's token record of position p (TokRec)
    auto tokrec_ar = [&](int p) {
        return reinterpret_cast<float2*>(tokrec(Pr.kv, Pr.H, tile0, p, TILE, tid));
    };
    // position 0: the query token [state=1, 0_A, 0, 0] (BanditEnv.state = [1], ctrl_bandit.py:426)
    if (tid < TILE) {
        S.tok[tid][0] = 1.f;
        if (tile0 + tid < Pr.N) *tokrec_ar(0) = make_float2(__int_as_float(A), 0.f);
    }
    // this thread's task's (u, g) draw pairs (rollout_draws_kernel), one per step, TILE apart
    const double2* draws = (tid < TILE && tile0 + tid < Pr.N) ? draw_pair(Pr, tile0 + tid, 0) : nullptr;
    float wpe_next = M.wpe[tid & 31];
    __syncthreads();
    for (int h = 0; h < Pr.H; ++h) {
        const float wpe_j = wpe_next;
        if (h + 1 < Pr.H) wpe_next = M.wpe[(size_t)(h + 1) * kE + (tid & 31)];
        // consumed after the forward; read once, so non-temporal (keeps the pinned rows resident)
        double2 dr = make_double2(0.0, 0.0);
        if (draws) {
            const doublex2 d2 = __builtin_nontemporal_load(reinterpret_cast<const doublex2*>(draws + (size_t)h * TILE));
            dr = make_double2(d2[0], d2[1]);
        }
        decode_position<TILE, true, GL, L0M>(S, P, pl, M, Pr.kv, Pr.N, Pr.H, tile0, h, wpe_j, D, Pr.pin, Pr.pin_x);
        // selection + env step; the outputs are stored after the barrier so that it
        // waits only for the y rows (issued phases earlier), not for these stores
        const int t = tid, task = tile0 + t;
        const bool live = tid < TILE && task < Pr.N;
        int a = 0;
        double mean = 0.0, r = 0.0;
        if (live) {
            a = select_rollout(S.logits[t], A, Pr.sample, dr.x);
            mean = means[t * A + a];
            r = (Pr.type == DPT_BANDIT_BERNOULLI) ? ((dr.y < mean) ? 1.0 : 0.0) : gaussian_reward(mean, Pr.var, dr.y);
            // next token = transition h: [s=1, onehot(a), s'=1, float(r)] (eval_bandit.py:83-86)
            S.tok[t][0] = 1.f;
            for (int k = 0; k < A; ++k) S.tok[t][1 + k] = (k == a) ? 1.f : 0.f;
            S.tok[t][1 + A] = 1.f;
            S.tok[t][2 + A] = (float)r;
        }
        __syncthreads();  // y rows of step h visible before step h+1 reads them
        if (live) {
            __builtin_nontemporal_store(a, Pr.actions_out + (size_t)task * Pr.H + h);
            __builtin_nontemporal_store(r, Pr.rewards_out + (size_t)task * Pr.H + h);
            __builtin_nontemporal_store(mean, Pr.arm_value_out + (size_t)task * Pr.H + h);
            if (Pr.logits_out)  // S.logits is next rewritten by step h+1's head phase
                for (int k = 0; k < A; ++k) Pr.logits_out[((size_t)h * Pr.N + task) * A + k] = S.logits[t][k];
            // first read from memory by step h+2 (positions < h+2), so it may land during step h+1
            if (h + 1 < Pr.H) *tokrec_ar(h + 1) = make_float2(__int_as_float(a), (float)r);
        }
        DPT_STAMP(7);
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
    v.l0 = nullptr;  // set by dpt_model_create once derived
    v.n_layer = d.n_layer;
    v.sd = d.state_dim;
    v.A = d.action_dim;
    v.F = F;
    v.n_positions = d.n_positions;
    v.mlp_ew = 0;  // set by dpt_model_create (mlp_scales)
    v.mlp_ex = 0;
    v.attn_ew = v.attn_ey = v.attn_eq = 0;
    return v;
}

// ModelView::l0 from every block's weights (fp64 sums, one rounding per
// element); workgroup li derives block li.
__global__ void derive_l0_kernel(ModelView M, float* __restrict__ l0_all) {
    const float* W = M.layers + (size_t)blockIdx.x * LayerOff::size;
    float* l0 = l0_all + (size_t)blockIdx.x * L0Off::size;
    const float* aw = W + LayerOff::attn_w;  // [E][3E]: q | k | v columns
    const float* ab = W + LayerOff::attn_b;
    const float* pw = W + LayerOff::proj_w;  // [E][E]
    for (int i = threadIdx.x; i < L0Off::size; i += blockDim.x) {
        double acc = 0.0;
        if (i < L0Off::g0) {  // G[m][n] = sum_j Wq[m][j] Wk[n][j]
            const int m = i / kE, n = i % kE;
            for (int j = 0; j < kE; ++j) acc += (double)aw[m * 3 * kE + j] * (double)aw[n * 3 * kE + kE + j];
        } else if (i < L0Off::Wvp) {  // g0[n] = sum_j Wk[n][j] bq[j]
            const int n = i - L0Off::g0;
            for (int j = 0; j < kE; ++j) acc += (double)aw[n * 3 * kE + kE + j] * (double)ab[j];
        } else if (i < L0Off::bvp) {  // Wvp[m][n] = sum_j Wv[m][j] Wproj[j][n]
            const int m = (i - L0Off::Wvp) / kE, n = (i - L0Off::Wvp) % kE;
            for (int j = 0; j < kE; ++j) acc += (double)aw[m * 3 * kE + 2 * kE + j] * (double)pw[j * kE + n];
        } else {  // bvp[n] = sum_j bv[j] Wproj[j][n] + bproj[n]
            const int n = i - L0Off::bvp;
            for (int j = 0; j < kE; ++j) acc += (double)ab[2 * kE + j] * (double)pw[j * kE + n];
            acc += (double)W[LayerOff::proj_b + n];
        }
        l0[i] = (float)acc;
    }
}

int64_t l0_numel(int n_layer) { return (int64_t)n_layer * L0Off::size; }

int launch_derive_l0(const ModelView& M, float* l0, hipStream_t st) {
    hipLaunchKernelGGL(derive_l0_kernel, dim3(M.n_layer), dim3(256), 0, st, M, l0);
    return check_hip(hipGetLastError(), "derive_l0_kernel launch");
}

int64_t weights_numel(const dpt_model_desc& d) {
    const int F = 2 * d.state_dim + d.action_dim + 1;
    return (int64_t)F * kE + kE + (int64_t)d.n_positions * kE + (int64_t)d.n_layer * LayerOff::size + 2 * kE +
           (int64_t)kE * d.action_dim + d.action_dim;
}

#ifdef DPT_STAMPS
extern "C" int dpt_debug_stamps(unsigned long long* out, int n, int reset) {
    if (reset) {
        unsigned long long z[64] = {0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_last), z, sizeof(unsigned long long));
        return 0;
    }
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * (n < 64 ? n : 64));
}
#endif

static int g_decode_tile = 8;  // tuning knob (dpt_tuning_set(DPT_TUNE_DECODE_TILE, 8|16))
static int64_t g_cache_budget = DPT_DEFAULT_CACHE_BUDGET;  // DPT_TUNE_CACHE_BUDGET
static bool g_block0_mfma = false;                         // DPT_TUNE_BLOCK0_MFMA

int set_block0_mfma(int on) {
    g_block0_mfma = on != 0;
    return DPT_OK;
}

int set_cache_budget(int64_t b) {
    if (b < 0) return DPT_EINVAL;
    g_cache_budget = b;
    return DPT_OK;
}

// The rollout re-reads every cached y row of a task at every later step, the
// earliest positions most often.  Rows of positions < pin are stored and read with
// the default policy and, while they fit the budget, stay in the Infinity Cache
// across steps; the rest stream non-temporally and do not displace them.  The
// budget is spent in whole stream chunks (8 kYRows positions of one block): every
// block gets `pin` positions and blocks 1..pin_x one chunk more.
static void rollout_pin(int N, int H, int n_layer, int* pin, int* pin_x) {
    constexpr int chunk = 8 * kYRows;
    const int64_t row = (int64_t)N * kE * sizeof(float);  // one position of one block, all tasks
    const int64_t nb = n_layer - 1;                          // blocks with a y cache
    *pin = 0;
    *pin_x = 0;
    if (nb <= 0 || row <= 0) return;
    const int64_t chunks = g_cache_budget / (row * chunk);
    *pin = (int)std::min<int64_t>((chunks / nb) * chunk, H);
    if (*pin < H) *pin_x = (int)(chunks % nb);
}

int set_decode_tile(int t) {
    if (t != 8 && t != 16) return DPT_EINVAL;
    g_decode_tile = t;
    return DPT_OK;
}

// the dynamic-LDS size must fit one CU
static int check_smem(const ModelView& M, size_t* bytes) {
    *bytes = decode_smem_bytes(M);
    if (*bytes > 160 * 1024) {
        set_error(DPT_EUNSUPPORTED, "decode LDS %zu B > 160 KiB (n_layer=%d, action_dim=%d)", *bytes, M.n_layer, M.A);
        return DPT_EUNSUPPORTED;
    }
    return DPT_OK;
}

template <int TILE>
static dim3 tiles(int n) { return dim3((n + TILE - 1) / TILE); }

// dynamic LDS beyond the default 64 KiB must be opted into per kernel
template <class K>
static void allow_smem(K kernel, size_t bytes) {
    if (bytes > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)bytes);
}

int launch_decode_step(const ModelView& M, float* kv, int N, int max_pos, int pos, const float* token,
                       float* logits, hipStream_t st) {
    size_t sm;
    if (int rc = check_smem(M, &sm)) return rc;
    allow_smem(decode_step_kernel<8>, sm);
    allow_smem(decode_step_kernel<16>, sm);
    if (g_decode_tile == 8)
        hipLaunchKernelGGL(decode_step_kernel<8>, tiles<8>(N), dim3(512), sm, st, M, kv, N, max_pos, pos, token, logits);
    else
        hipLaunchKernelGGL(decode_step_kernel<16>, tiles<16>(N), dim3(1024), sm, st, M, kv, N, max_pos, pos, token,
                           logits);
    return check_hip(hipGetLastError(), "decode_step_kernel launch");
}

int launch_window_decode(const ModelView& M, float* kv, int N, int C, const float* q, const float* cs,
                         const float* ca, const float* cn, const float* cr, int out_mode, float* out,
                         hipStream_t st) {
    size_t sm;
    if (int rc = check_smem(M, &sm)) return rc;
    allow_smem(window_decode_kernel<8>, sm);
    allow_smem(window_decode_kernel<16>, sm);
    if (g_decode_tile == 8)
        hipLaunchKernelGGL(window_decode_kernel<8>, tiles<8>(N), dim3(512), sm, st, M, kv, N, C, q, cs, ca, cn, cr,
                           out_mode, out);
    else
        hipLaunchKernelGGL(window_decode_kernel<16>, tiles<16>(N), dim3(1024), sm, st, M, kv, N, C, q, cs, ca, cn,
                           cr, out_mode, out);
    return check_hip(hipGetLastError(), "window_decode_kernel launch");
}

int launch_rollout_bandit(const ModelView& M, const dpt_bandit_rollout_args& a, hipStream_t st) {
    size_t sm;
    if (int rc = check_smem(M, &sm)) return rc;
    // G in LDS when the block still lets the tile's workgroups share a CU (two at
    // tile 8, one at tile 16); otherwise the u projection reads it from L2
    const size_t per_cu = 160 * 1024 / (g_decode_tile == 8 ? 2 : 1);
    // block 0 on the matrix cores (l0_tiles) for the 5-arm configs at tile 8
    // (A = 20 in this form spills at the 128-VGPR cap: its 21 arm sums; measured +17 %)
    const bool l0m = g_block0_mfma && g_decode_tile == 8 && a.A == 5;
    const bool gl = rollout_smem_bytes(M, true, l0m) <= per_cu;
    sm = rollout_smem_bytes(M, gl, l0m);
    if (sm > 160 * 1024) {
        set_error(DPT_EUNSUPPORTED, "rollout LDS %zu B > 160 KiB (n_layer=%d, action_dim=%d)", sm, M.n_layer, M.A);
        return DPT_EUNSUPPORTED;
    }
    if (!M.l0) {
        set_error(DPT_EINVAL, "model has no derived block-0 weights");
        return DPT_EINVAL;
    }
    BanditRolloutParams P;
    P.N = a.N; P.H = a.H; P.A = a.A; P.type = a.type; P.sample = a.sample;
    P.first_task = a.first_task; P.var = a.var; P.seed = a.seed; P.counter = a.counter;
    P.means = a.means; P.uniforms = a.uniforms; P.noise = a.noise; P.kv = a.kvcache;
    P.actions_out = a.actions_out; P.rewards_out = a.rewards_out; P.arm_value_out = a.arm_value_out;
    P.logits_out = a.logits_out;
    P.n_layer = M.n_layer;
    P.tile = g_decode_tile;
    rollout_pin(a.N, a.H, M.n_layer, &P.pin, &P.pin_x);
    const int64_t nd = (int64_t)a.N * a.H;
    hipLaunchKernelGGL(rollout_draws_kernel, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, st, P);
    auto launch = [&](auto kernel, int tile) {
        allow_smem(kernel, sm);
        hipLaunchKernelGGL(kernel, dim3((a.N + tile - 1) / tile), dim3(tile * 64), sm, st, M, P);
    };
    if (l0m)
        gl ? launch(rollout_bandit_kernel<8, true, 6>, 8) : launch(rollout_bandit_kernel<8, false, 6>, 8);
    else if (g_decode_tile == 8)
        gl ? launch(rollout_bandit_kernel<8, true>, 8) : launch(rollout_bandit_kernel<8, false>, 8);
    else
        gl ? launch(rollout_bandit_kernel<16, true>, 16) : launch(rollout_bandit_kernel<16, false>, 16);
    return check_hip(hipGetLastError(), "rollout_bandit_kernel launch");
}

}  // namespace dpt
