// Building blocks of the transposed-dataflow MFMA forward (gfx950), shared by
// the fused DarkRoom rollout (dpt_darkroom.hip) and the window prefill
// (dpt_prefill.hip).  A window of <= 128 tokens is cut into 16-token blocks; a
// wave holds x^T of its blocks in registers as v_mfma_f32_16x16x4_f32 C-layout
// fragments (lane (g = l>>4, c = l&15): features 16*blk + 4g + r of token c),
// which is exactly the B operand of the next product W^T x^T.  Weights are the
// A operand, split and pre-packed per layer in operand order (Frag3); only K
// (token-major) and V (feature-major) go through LDS.
#pragma once

#include "dpt_common.h"

namespace dpt {

constexpr int kFwdWaves = 4;                 // waves per workgroup
constexpr int kFwdBlocks = 8;                // 16-token blocks per window (two per wave)
constexpr int kFwdT = 16 * kFwdBlocks;        // max window
constexpr int kKStride = kE + 4;            // K[token][feature]
constexpr int kVStride = kFwdT + 4;          // Vt[feature][token] (128-token buffer)

// Small parameters copied to LDS once per launch (offsets in floats): per block
// [ln1_g ln1_b attn_b proj_b ln2_g ln2_b fc_b mp_b], then the model-level ones.
// (attn_b holds only the folded attention's g0: the unfolded c_attn bias had 3E entries)
struct PL {
    static constexpr int ln1_g = 0, ln1_b = 32, attn_b = 64, proj_b = 96, ln2_g = 128, ln2_b = 160,
                         fc_b = 192, mp_b = 320, size = 352;
};
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
// This workgroup's keys and values of the current layer, for windows of up to TMAX
// tokens.  Keys are either fp32 token-major (K) or, with SPLITK, the fp16 two-part A
// operand tiles of the score product (KS[block][part h|m][lane], y x 2^attn_ey, written
// once by the lane that computed the key: 2 KB per 16 keys, no split per read).  Values
// stay fp32 feature-major (Vt).
// With SPLITV (requires SPLITK) the values are kept as the fp16 two-part split of y x 2^attn_ey
// (the keys' split), token-major: VT[part h|m][key][kVTRow] (features 0..31, rows padded to 72 B).
// The writer lane holds two runs of 4 consecutive features of its token (C-layout) and
// stores each as one 8-B write; the A operand of O^T += V^T P^T over a pair of key tiles
// (element j of lane (g, c) = V[key 16 (2 pair + (j >> 2)) + 4g + (j & 3)][feature 16 half + c],
// the lane group's k order of P^T's C-layout over the two tiles) is read back transposed by
// two ds_read_b64_tr_b16 per part (vt_split).  With KEYS_VT (requires SPLITV) the score product's
// key tiles are read from the same rows too (key_split) and KS is not kept: half the LDS, for the
// 512-token windows; otherwise the keys keep their own pre-split tiles (one 16-B read per part).
constexpr int kVTRow = kE + 4;  // halves per VT row: 72 B (8-B aligned rows for the transposed read)
template <int TMAX, bool SPLITK = false, bool SPLITV = false, bool KEYS_VT = false>
struct KVBuf {
    static_assert(SPLITK || !SPLITV, "split values need split keys");
    static_assert(SPLITV || !KEYS_VT, "keys from VT need split values");
    static constexpr bool kSplitK = SPLITK, kSplitV = SPLITV, kKeysVT = KEYS_VT;
    static constexpr bool kKS = SPLITK && !KEYS_VT;
    float K[SPLITK ? 1 : TMAX][kKStride];
    halfx8 KS[kKS ? TMAX / 16 : 1][kKS ? 2 : 1][kKS ? 64 : 1];  // (16 B when unused)
    _Float16 VT[SPLITV ? 2 : 1][SPLITV ? TMAX : 1][SPLITV ? kVTRow : 8];
    float Vt[SPLITV ? 1 : kE][TMAX + 4];
};
constexpr bool kSplitKeys = true;  // scores on mfma_x3 (and, with SPLITV, P V too)

__device__ inline floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ inline floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

// Lane index the compiler cannot hoist: every helper derives its lane-dependent
// LDS addresses from this at its own start, so they are short-lived values
// instead of loop invariants spilled across the whole rollout.
__device__ inline int lane_id() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t & 63;
}

// ---- dense products on fp16 two-part splits ("x3"): v = h + m + O(2^-22 v) with
// h, m fp16 (11-bit significands; the residual is exact in fp32), and a K = 32 product
// is h_a h_b + h_a m_b + m_a h_b (exact fp16 products, fp32 accumulation) on three
// v_mfma_f32_16x16x32_f16: 48 matrix cycles per K = 32 tile instead of the 256 of eight
// v_mfma_f32_16x16x4_f32 (and half those of a bf16 three-part form).  The dropped terms are
// below 2^-21 of |a||b| per product; weights and activations are scaled by powers of
// two (ModelView mlp_* / attn_*) so their residuals stay normal fp16 numbers.  Every
// product of the forward runs this way (P V with P <= 2^8, see attend).
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
struct Split2 {
    halfx8 h, m;
};
__device__ inline Split2 split2(const float (&v)[8], float scale) {
    // m = f16(x - h) (x = v scale): x - h is exact in fp32, formed by one v_fma_mix_f32 per value
    // (the f32 value times 1 minus the f16 h, no conversion of h back to fp32), and the pair is
    // rounded to fp16 by one v_cvt_pk_f16_f32.  The same bits as v_fma_mix{lo,hi}_f16 (one fma
    // rounded once to fp16), but those write half a register and issue at about 9.7 cycles each
    // against 5.0 for v_fma_mix_f32 and 6.0 for the pack (scripts/valu_issue.hip,
    // profiles/r4c/valu_issue.json): -2.1 % at config 3.  (An opaque 1.0 multiplier keeps the fma
    // from folding into a plain subtraction, which would lose the mixed-precision form.)
    float one = 1.0f;
    asm volatile("" : "+s"(one));
    unsigned hh[4], mm[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const floatx2 x = floatx2{v[2 * p], v[2 * p + 1]} * floatx2{scale, scale};
        const halfx2 h = __builtin_convertvector(x, halfx2);
        const halfx2 m = __builtin_convertvector(
            floatx2{__builtin_fmaf(x.x, one, -(float)h.x), __builtin_fmaf(x.y, one, -(float)h.y)}, halfx2);
        hh[p] = __builtin_bit_cast(unsigned, h);
        mm[p] = __builtin_bit_cast(unsigned, m);
    }
    return Split2{__builtin_bit_cast(halfx8, uint4{hh[0], hh[1], hh[2], hh[3]}),
                  __builtin_bit_cast(halfx8, uint4{mm[0], mm[1], mm[2], mm[3]})};
}
__device__ inline floatx4 mfma_f16(const halfx8& a, const halfx8& b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ inline floatx4 mfma_x3(const Split2& a, const Split2& b, floatx4 acc) {
    acc = mfma_f16(a.h, b.m, acc);
    acc = mfma_f16(a.m, b.h, acc);
    return mfma_f16(a.h, b.h, acc);
}
// 2^e as a float (|e| < 127)
__device__ inline float exp2i(int e) { return __int_as_float((e + 127) << 23); }

// The split A operand of O^T += V^T P^T for key-tile pair pp and feature half `half` from the
// token-major VT image: per part two ds_read_b64_tr_b16 (T10: the 16-lane group g reads keys
// 16 (2 pp + t) + 4g + q, q < 4, at features 16 half + 0..15; lane c receives feature c, key q
// in element q).  `lo` = vt_lane_off() of the calling lane; EXEC must be all ones.
typedef short i16x4 __attribute__((__vector_size__(4 * sizeof(short))));
__device__ inline int vt_lane_off(int lane) {
    // lane 4q + p of group g supplies row 4g + q, columns 4p..4p+3
    return ((4 * (lane >> 4) + ((lane & 15) >> 2)) * kVTRow + 4 * (lane & 3)) * 2;  // bytes
}
template <class KV>
__device__ inline Split2 vt_split(const KV& S, int pp, int half, int lo) {
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    const char* base = reinterpret_cast<const char*>(&S.VT[0][0][0]) + lo + (32 * pp * kVTRow + 16 * half) * 2;
    constexpr int kPart = (int)sizeof(S.VT[0]), kTile = 16 * kVTRow * 2;
    auto rd = [&](int off) {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off));
    };
    const i16x4 h0 = rd(0), h1 = rd(kTile), m0 = rd(kPart), m1 = rd(kPart + kTile);
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 h = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    const i16x8 m = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
    return Split2{__builtin_bit_cast(halfx8, h), __builtin_bit_cast(halfx8, m)};
}
// The split A operand of the score product S^T = K Q^T for key tile kt: lane (g, c) holds the
// k-elements j of key 16 kt + c, features 16 (j >> 2) + 4g + (j & 3) (the writer's C-layout order).
// With KEYS_VT the keys are read from the token-major VT image (two 8-B runs of a row per part,
// one ds_read2_b64; rows 72 B apart put the 16 lanes of a group on distinct banks), otherwise
// from the pre-split key tiles KS.
template <class KV>
__device__ inline Split2 key_split(const KV& S, int kt, int lane) {
    if constexpr (KV::kKeysVT) {
        const int row = 16 * kt + (lane & 15), g = lane >> 4;
        const uint2* h = reinterpret_cast<const uint2*>(&S.VT[0][row][4 * g]);
        const uint2* m = reinterpret_cast<const uint2*>(&S.VT[1][row][4 * g]);
        const uint2 h0 = h[0], h1 = h[4], m0 = m[0], m1 = m[4];
        return Split2{__builtin_bit_cast(halfx8, uint4{h0.x, h0.y, h1.x, h1.y}),
                      __builtin_bit_cast(halfx8, uint4{m0.x, m0.y, m1.x, m1.y})};
    } else {
        return Split2{S.KS[kt][0][lane], S.KS[kt][1][lane]};
    }
}

// scale of the attention probabilities in P V (P <= 2^8, so P x 2^kPExp < 2^14)
constexpr int kPExp = 2;


// The split weight tiles of one block (the model's fragment buffer, per layer):
// [tile][part h|m][64 lanes][8 fp16], tile element (lane (g, c), j) = W[in][out] x 2^e
// with in = 16*(j>>2) + 4g + (j&3) (mp: hidden 32*pair + that) and out = 16*ob + c;
// e = mlp_ew for the MLP tiles (fc, mp), attn_ew for G and Wvp.
struct Frag3 {
    static constexpr int attn = 0;   // 2 tiles: G
    static constexpr int proj = 2;   // 2 tiles: Wvp
    static constexpr int fc = 4;     // 8 tiles: c_fc, output chunk ob
    static constexpr int mp = 12;    // [2 ob][4 pairs]: mlp.c_proj over hidden chunks 2p, 2p+1
    static constexpr int tiles = 20;
    static constexpr int parts = 2;
    static constexpr int bytes = tiles * parts * 64 * 16;  // 40,960 per layer
};
struct FragSrc3 {
    __amdgpu_buffer_rsrc_t r;
    int base;  // byte offset of this layer's tiles
    // the lane's byte offset inside a tile: a helper that loads several tiles computes it once
    // (three VALU instructions per load otherwise, from the opaque lane_id)
    __device__ static int lane_off() { return lane_id() * 16; }
    __device__ halfx8 ld1(int tile, int part, int vo) const {
        return __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(
                                              r, vo, base + (tile * Frag3::parts + part) * 1024, 0));
    }
    __device__ Split2 ld2(int tile, int vo) const { return Split2{ld1(tile, 0, vo), ld1(tile, 1, vo)}; }
    __device__ Split2 ld2(int tile) const { return ld2(tile, lane_off()); }
    __device__ FragSrc3 layer(int l) const { return FragSrc3{r, l * Frag3::bytes}; }
};

// Cross-lane-group reductions with the gfx950 VALU permutes instead of
// ds_bpermute: v_permlane16_swap / v_permlane32_swap applied to (v, v) return
// the lane's own value and its xor-16 / xor-32 partner (in an order that
// depends on the lane), so a symmetric op of the pair is the same on both.
__device__ inline float sum_x16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float sum_x32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// max of scores without fmaxf's NaN quieting: the compiler cannot see that an MFMA result is
// canonical, so every fmaxf operand got a canonicalising v_max_f32 x, x (184 of the C3 kernel's 281
// v_max).  llvm.maximum (IEEE 754-2019 maximum, NaN-propagating) needs no canonical inputs and
// lowers to gfx950's v_maximum3_f32; scores are finite or -inf, never NaN, so the value is the
// same.  (Inline-asm v_max3 is not an option: the hazard recognizer does not pad an asm read of
// an MFMA result, which read stale accumulators.)
__device__ inline float vmax2(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ inline float vmax3(float a, float b, float c) { return vmax2(vmax2(a, b), c); }
__device__ inline float vmax8(const float (&v)[8]) {
    return vmax2(vmax2(vmax2(v[0], v[1]), vmax2(v[2], v[3])), vmax2(vmax2(v[4], v[5]), vmax2(v[6], v[7])));
}
__device__ inline float max_x16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return vmax2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ inline float max_x32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return vmax2(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// sum / max over the 4 lane groups (the 4 feature slices of a token column)
__device__ inline float sum_cols(float v) { return sum_x32(sum_x16(v)); }
// sum_cols of two values at once (a wave's two blocks): the first swap exchanges a's odd rows with
// b's even rows, so one add leaves a's row-pair sums in rows 0 / 2 and b's in rows 1 / 3; the
// xor-32 exchange completes both totals (a's in rows 0 / 2, b's in 1 / 3) and a last xor-16
// exchange hands every lane both.  Three permlanes and two adds instead of four and four, and
// the same sums in the same order as sum_cols: bit-identical.
__device__ inline void sum_cols2(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    const float s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    const float u = __uint_as_float(t[0]) + __uint_as_float(t[1]);
    const auto w = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
    a = __uint_as_float(w[0]);
    b = __uint_as_float(w[1]);
}
__device__ inline float max_cols(float v) { return max_x32(max_x16(v)); }

__device__ inline void bar_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LayerNorm over the 32 features of each token column (eps 1e-5): a lane holds
// 8 of them; the other 24 live in lanes l^16, l^32, l^48.
__device__ inline void ln_cols(const float (&v)[8], float (&out)[8], const float* __restrict__ gam,
                               const float* __restrict__ bet) {
    // pairwise (packed) sums, rstd by v_rsq: fp32-accurate, not the reference's summation order
    typedef float fx2 __attribute__((ext_vector_type(2)));
    const int g = lane_id() >> 4;
    const fx2 v0 = {v[0], v[1]}, v1 = {v[2], v[3]}, v2 = {v[4], v[5]}, v3 = {v[6], v[7]};
    const fx2 sa = (v0 + v1) + (v2 + v3);
    const float mean = sum_cols(sa.x + sa.y) * (1.0f / kE);
    const fx2 mm = {mean, mean};
    const fx2 d0 = v0 - mm, d1 = v1 - mm, d2 = v2 - mm, d3 = v3 - mm;
    const fx2 qa = (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    const float rstd = __builtin_amdgcn_rsqf(sum_cols(qa.x + qa.y) * (1.0f / kE) + 1e-5f);
    const fx2 rr = {rstd, rstd};
    const floatx4 g0 = ld4(gam + 4 * g), g1 = ld4(gam + 16 + 4 * g);
    const floatx4 b0 = ld4(bet + 4 * g), b1 = ld4(bet + 16 + 4 * g);
    const fx2 o0 = __builtin_elementwise_fma(d0 * rr, fx2{g0[0], g0[1]}, fx2{b0[0], b0[1]});
    const fx2 o1 = __builtin_elementwise_fma(d1 * rr, fx2{g0[2], g0[3]}, fx2{b0[2], b0[3]});
    const fx2 o2 = __builtin_elementwise_fma(d2 * rr, fx2{g1[0], g1[1]}, fx2{b1[0], b1[1]});
    const fx2 o3 = __builtin_elementwise_fma(d3 * rr, fx2{g1[2], g1[3]}, fx2{b1[2], b1[3]});
    out[0] = o0.x; out[1] = o0.y; out[2] = o1.x; out[3] = o1.y;
    out[4] = o2.x; out[5] = o2.y; out[6] = o3.x; out[7] = o3.y;
}

// ln_cols of a wave's two blocks with their column reductions paired (sum_cols2): the same
// arithmetic, bit-identical, three permlanes per statistic for both blocks instead of four
__device__ inline void ln_cols2(const float (&v)[2][8], float (&out)[2][8], const float* __restrict__ gam,
                                const float* __restrict__ bet) {
    typedef float fx2 __attribute__((ext_vector_type(2)));
    const int g = lane_id() >> 4;
    fx2 d[2][4];
    float mean[2], var[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const fx2 v0 = {v[j][0], v[j][1]}, v1 = {v[j][2], v[j][3]}, v2 = {v[j][4], v[j][5]}, v3 = {v[j][6], v[j][7]};
        const fx2 sa = (v0 + v1) + (v2 + v3);
        mean[j] = sa.x + sa.y;
    }
    sum_cols2(mean[0], mean[1]);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const float mj = mean[j] * (1.0f / kE);
        const fx2 mm = {mj, mj};
        d[j][0] = fx2{v[j][0], v[j][1]} - mm;
        d[j][1] = fx2{v[j][2], v[j][3]} - mm;
        d[j][2] = fx2{v[j][4], v[j][5]} - mm;
        d[j][3] = fx2{v[j][6], v[j][7]} - mm;
        const fx2 qa = (d[j][0] * d[j][0] + d[j][1] * d[j][1]) + (d[j][2] * d[j][2] + d[j][3] * d[j][3]);
        var[j] = qa.x + qa.y;
    }
    sum_cols2(var[0], var[1]);
    const floatx4 g0 = ld4(gam + 4 * g), g1 = ld4(gam + 16 + 4 * g);
    const floatx4 b0 = ld4(bet + 4 * g), b1 = ld4(bet + 16 + 4 * g);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const float rstd = __builtin_amdgcn_rsqf(var[j] * (1.0f / kE) + 1e-5f);
        const fx2 rr = {rstd, rstd};
        const fx2 o0 = __builtin_elementwise_fma(d[j][0] * rr, fx2{g0[0], g0[1]}, fx2{b0[0], b0[1]});
        const fx2 o1 = __builtin_elementwise_fma(d[j][1] * rr, fx2{g0[2], g0[3]}, fx2{b0[2], b0[3]});
        const fx2 o2 = __builtin_elementwise_fma(d[j][2] * rr, fx2{g1[0], g1[1]}, fx2{b1[0], b1[1]});
        const fx2 o3 = __builtin_elementwise_fma(d[j][3] * rr, fx2{g1[2], g1[3]}, fx2{b1[2], b1[3]});
        out[j][0] = o0.x; out[j][1] = o0.y; out[j][2] = o1.x; out[j][3] = o1.y;
        out[j][4] = o2.x; out[j][5] = o2.y; out[j][6] = o3.x; out[j][7] = o3.y;
    }
}

// gelu_fast on a pair: the same operations in the same order on v_pk_{mul,fma,add}_f32 (each
// half rounded like the scalar op: bit-identical), with the two transcendentals per value
__device__ inline floatx2 gelu_fast2(floatx2 x) {
    const float c1 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
    const float c2 = c1 * 0.044715f;
    const floatx2 t = __builtin_elementwise_fma(x * x, floatx2{c2, c2}, floatx2{c1, c1}) * x;
    const floatx2 d = floatx2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + floatx2{1.0f, 1.0f};
    return x * floatx2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

__device__ inline float gelu_fast(float x) {
    // gelu_new (transformers/activations.py:65): 0.5x(1 + tanh(z)) = x * sigmoid(2z)
    // = x / (1 + 2^(x * (c1 + c2 x^2))), z = sqrt(2/pi)(x + 0.044715 x^3), log2(e) folded in
    const float c1 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
    const float c2 = c1 * 0.044715f;
    const float e = __builtin_amdgcn_exp2f(x * fmaf(x * x, c2, c1));
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// gelu_new of the c_fc output taken straight from its product accumulator, returned as the
// fp16 two-part split of mlp.c_proj's B operand.  With y = h 2^(ew+ex) (the accumulator, bias
// included) every scale is an exact power of two folded into a constant:
//   gelu(h) 2^ex = y / ((1 + 2^t) 2^ew),  t = h (c1 + c2 h^2) = y (c1' + c2' y^2),
//   c1' = c1 2^-(ew+ex), c2' = c2 2^-3(ew+ex)
// so the scale-down before gelu and the scale-up of split2 vanish.  fwd_scales keeps
// ew + ex >= -40, so c2' stays a normal fp32 number.
struct GeluSplit {
    float c1, c2, s;
    __device__ GeluSplit(int ew, int ex) {
        const float k1 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
        c1 = k1 * exp2i(-(ew + ex));
        c2 = (k1 * 0.044715f) * exp2i(-3 * (ew + ex));
        s = exp2i(ew);
    }
};
__device__ inline Split2 gelu_split(const floatx4& a, const floatx4& b, const GeluSplit& k) {
    // pairs on the packed f32 ops (v_pk_mul / v_pk_fma: two values per issue, each rounded like
    // the scalar op); hi from one v_cvt_pk_f16_f32 per pair, lo = f16(g - hi) by v_fma_mix_f32 and a
    // second pack, as split2
    float one = 1.0f;
    asm volatile("" : "+s"(one));
    const floatx2 c1 = {k.c1, k.c1}, c2 = {k.c2, k.c2}, sv = {k.s, k.s};
    unsigned hh[4], mm[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const floatx2 y = p < 2 ? floatx2{a[2 * p], a[2 * p + 1]} : floatx2{b[2 * p - 4], b[2 * p - 3]};
        const floatx2 t = __builtin_elementwise_fma(y * y, c2, c1) * y;
        const floatx2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
        const floatx2 d = __builtin_elementwise_fma(e, sv, sv);
        const floatx2 g = y * floatx2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
        const halfx2 h = __builtin_convertvector(g, halfx2);
        const halfx2 m = __builtin_convertvector(
            floatx2{__builtin_fmaf(g.x, one, -(float)h.x), __builtin_fmaf(g.y, one, -(float)h.y)}, halfx2);
        hh[p] = __builtin_bit_cast(unsigned, h);
        mm[p] = __builtin_bit_cast(unsigned, m);
    }
    return Split2{__builtin_bit_cast(halfx8, uint4{hh[0], hh[1], hh[2], hh[3]}),
                  __builtin_bit_cast(halfx8, uint4{mm[0], mm[1], mm[2], mm[3]})};
}

template <int NB, int J0 = 0>
__device__ inline void ln_n(const float (&x)[2][8], float (&xn)[2][8], const float* gam, const float* bet) {
    static_assert(NB == 1 || J0 == 0, "two blocks start at slot 0");
    if constexpr (NB == 2) {
        ln_cols2(x, xn, gam, bet);
    } else {
#pragma unroll
        for (int j = J0; j < J0 + NB; ++j) ln_cols(x[j], xn[j], gam, bet);
    }
}

// x += (a | b) x down, down an exact power of two: one packed fma per pair (the product is exact,
// so each result equals x + a down rounded once, as the separate multiply and add)
__device__ inline void resid_add(float (&x)[8], const floatx4& a, const floatx4& b, float down) {
    const floatx2 dd = {down, down};
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
        const floatx2 u = __builtin_elementwise_fma(floatx2{a[r], a[r + 1]}, dd, floatx2{x[r], x[r + 1]});
        const floatx2 v = __builtin_elementwise_fma(floatx2{b[r], b[r + 1]}, dd, floatx2{x[4 + r], x[5 + r]});
        x[r] = u.x;
        x[r + 1] = u.y;
        x[4 + r] = v.x;
        x[5 + r] = v.y;
    }
}

// x^T += MLP(xn^T) on fp16 two-part products (mfma_x3): c_fc per 16-unit chunk, mlp.c_proj
// per pair of chunks (its K = 32 input is the two chunks' gelu outputs, C-layout).  Products
// accumulate at scale 2^(mlp_ew + mlp_ex) (the biases enter scaled, exactly) and are scaled
// back by the exact power of two.
template <int NB, int J0 = 0>
__device__ inline void mlp3_n(const float* W, const FragSrc3& f3, const float (&xn)[2][8], float (&x)[2][8],
                              int ew, int ex) {
    const int g = lane_id() >> 4;
    const float down = exp2i(-(ew + ex));
    const GeluSplit gk(ew, ex);
    const floatx4 yb0 = ld4(W + PL::mp_b + 4 * g), yb1 = ld4(W + PL::mp_b + 16 + 4 * g);  // scaled (PL)
    floatx4 y0[2] = {yb0, yb0}, y1[2] = {yb1, yb1};
    // c_fc tiles one pair ahead (in flight across the pair's gelu + c_proj products; the first
    // pair's across the split of xn), the pair's c_proj tiles at its start (in flight across its
    // c_fc + gelu)
    const int vo = FragSrc3::lane_off();
    Split2 wf0 = f3.ld2(Frag3::fc, vo), wf1 = f3.ld2(Frag3::fc + 1, vo);
    Split2 xs[2];
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) xs[j] = split2(xn[j], 1.0f);  // xn = ln_2 output x 2^mlp_ex (PL)
#pragma unroll
    for (int p = 0; p < kFF / 32; ++p) {
        const Split2 w0 = f3.ld2(Frag3::mp + p, vo), w1 = f3.ld2(Frag3::mp + 4 + p, vo);
        Split2 gs[2];
        const floatx4 fb0 = ld4(W + PL::fc_b + 2 * p * 16 + 4 * g);
        const floatx4 fb1 = ld4(W + PL::fc_b + (2 * p + 1) * 16 + 4 * g);
#pragma unroll
        for (int j = J0; j < J0 + NB; ++j)
            gs[j] = gelu_split(mfma_x3(wf0, xs[j], fb0), mfma_x3(wf1, xs[j], fb1), gk);
        if (p + 1 < kFF / 32) {
            wf0 = f3.ld2(Frag3::fc + 2 * p + 2, vo);
            wf1 = f3.ld2(Frag3::fc + 2 * p + 3, vo);
        }
#pragma unroll
        for (int j = J0; j < J0 + NB; ++j) {
            y0[j] = mfma_x3(w0, gs[j], y0[j]);
            y1[j] = mfma_x3(w1, gs[j], y1[j]);
        }
    }
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) resid_add(x[j], y0[j], y1[j], down);
}

// u = xn G + g0 of the NB blocks (the folded c_attn: only its q part) on fp16 two-part
// products (mfma_x3) at scale 2^(attn_ew + attn_ey), returned at 2^attn_eq (the scale of the score
// product's split query, so attend splits it as it stands); xs = the blocks' LayerNorm outputs
// split at 2^attn_ey
template <int NB, int J0 = 0>
__device__ inline void u_proj3_w(const float* W, const Split2 (&wg)[2], const Split2 (&xs)[2], float (&q)[2][8],
                                 const ModelView& M) {
    const int g = lane_id() >> 4;
    const float down = exp2i(M.attn_eq - (M.attn_ew + M.attn_ey));
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
        const Split2& w = wg[ob];
        const floatx4 bias = ld4(W + PL::attn_b + ob * 16 + 4 * g);  // scaled (PL)
#pragma unroll
        for (int j = J0; j < J0 + NB; ++j) {
            const floatx4 acc = mfma_x3(w, xs[j], bias) * down;
#pragma unroll
            for (int r = 0; r < 4; ++r) q[j][ob * 4 + r] = acc[r];
        }
    }
}
// the G tiles of u = xn G + g0 (both 16-column tiles), issued ahead of the work that precedes the product
__device__ inline void ld_g(const FragSrc3& f3, Split2 (&wg)[2]) {
    const int vo = FragSrc3::lane_off();
    wg[0] = f3.ld2(Frag3::attn, vo);
    wg[1] = f3.ld2(Frag3::attn + 1, vo);
}
template <int NB, int J0 = 0>
__device__ inline void u_proj3_s(const float* W, const FragSrc3& f3, const Split2 (&xs)[2], float (&q)[2][8],
                                 const ModelView& M) {
    Split2 wg[2];
    ld_g(f3, wg);
    u_proj3_w<NB, J0>(W, wg, xs, q, M);
}
template <int NB, int J0 = 0>
__device__ inline void u_proj3_n(const float* W, const FragSrc3& f3, const float (&xn)[2][8], float (&q)[2][8],
                                 const ModelView& M) {
    Split2 xs[2];
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) xs[j] = split2(xn[j], 1.0f);  // xn = ln_1 output x 2^attn_ey (PL)
    u_proj3_s<NB, J0>(W, f3, xs, q, M);
}

// attn_proj on mfma_x3: x^T += Wvp^T o^T + bvp (o, a convex combination of the values y,
// shares their bound and scale)
template <int NB, int J0 = 0>
__device__ inline void attn_proj3_w(const float* W, const Split2& w0, const Split2& w1, const Split2 (&os)[2],
                                    float (&x)[2][8], const ModelView& M) {
    const int g = lane_id() >> 4;
    const float down = exp2i(-(M.attn_ew + M.attn_ey));
    const floatx4 b0 = ld4(W + PL::proj_b + 4 * g), b1 = ld4(W + PL::proj_b + 16 + 4 * g);  // scaled (PL)
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) resid_add(x[j], mfma_x3(w0, os[j], b0), mfma_x3(w1, os[j], b1), down);
}
template <int NB, int J0 = 0>
__device__ inline void attn_proj3_s(const float* W, const FragSrc3& f3, const Split2 (&os)[2], float (&x)[2][8],
                                    const ModelView& M) {
    const int vo = FragSrc3::lane_off();
    attn_proj3_w<NB, J0>(W, f3.ld2(Frag3::proj, vo), f3.ld2(Frag3::proj + 1, vo), os, x, M);
}
// (oscale: the split's scale, 2^attn_ey for an attention output at its true scale)
template <int NB, int J0 = 0>
__device__ inline void attn_proj3(const float* W, const FragSrc3& f3, const float (&o)[2][8], float (&x)[2][8],
                                  const ModelView& M, float oscale) {
    // the Wvp tiles ahead of the split
    const int vo = FragSrc3::lane_off();
    const Split2 w0 = f3.ld2(Frag3::proj, vo), w1 = f3.ld2(Frag3::proj + 1, vo);
    Split2 os[2];
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) os[j] = split2(o[j], oscale);
    attn_proj3_w<NB, J0>(W, w0, w1, os, x, M);
}
// the same from attend's unnormalised (o, l): o / l is the attention output x 2^attn_ey already,
// so the split takes 1 / l as its scale (one multiply per value; 1 / l by v_rcp_f32, 1 ulp, instead
// of the dozen instructions of an IEEE division: -1.1 % at config 3 with the two below)
template <int NB, int J0 = 0>
__device__ inline void attn_proj3_ol(const float* W, const FragSrc3& f3, const float (&o)[2][8], const float (&l)[2],
                                     float (&x)[2][8], const ModelView& M) {
    const int vo = FragSrc3::lane_off();
    const Split2 w0 = f3.ld2(Frag3::proj, vo), w1 = f3.ld2(Frag3::proj + 1, vo);
    Split2 os[2];
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) os[j] = split2(o[j], __builtin_amdgcn_rcpf(l[j]));
    attn_proj3_w<NB, J0>(W, w0, w1, os, x, M);
}

// Folded attention input of the NB blocks qb[]: keys and values are the
// LayerNorm output y itself (K <- y token-major, Vt <- y feature-major, the
// C-layout of xn is the layout c_attn's K / V tiles had).  With split keys the
// split of y at 2^attn_ey (xs, the lane's 8 values are its A-operand k-elements) is
// what goes to LDS.
template <int NB, int J0 = 0, class KV>
__device__ inline void kv_store(KV& S, const int (&qb)[2], const float (&xn)[2][8], const Split2 (&xs)[2]) {
    const int lane = lane_id(), g = lane >> 4;
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) {
        const int tok = qb[j] * 16 + (lane & 15);
        if constexpr (KV::kSplitK) {
            if constexpr (KV::kKS) {
                S.KS[qb[j]][0][lane] = xs[j].h;
                S.KS[qb[j]][1][lane] = xs[j].m;
            }
            if constexpr (KV::kSplitV) {
                // the same split parts, token-major: value k of lane (g, c) is feature
                // 16 (k >> 2) + 4g + (k & 3) of token 16 b + c, so each half of the lane's 8
                // values is 4 consecutive features: one 8-B store per part and half
                const uint4 hu = __builtin_bit_cast(uint4, xs[j].h), mu = __builtin_bit_cast(uint4, xs[j].m);
                _Float16* row = &S.VT[0][tok][4 * g];
                *reinterpret_cast<uint2*>(row) = uint2{hu.x, hu.y};
                *reinterpret_cast<uint2*>(row + 16) = uint2{hu.z, hu.w};
                _Float16* rowm = &S.VT[1][tok][4 * g];
                *reinterpret_cast<uint2*>(rowm) = uint2{mu.x, mu.y};
                *reinterpret_cast<uint2*>(rowm + 16) = uint2{mu.z, mu.w};
            }
        }
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
            if constexpr (!KV::kSplitK)
                *reinterpret_cast<floatx4*>(&S.K[tok][16 * blk + 4 * g]) =
                    floatx4{xn[j][4 * blk], xn[j][4 * blk + 1], xn[j][4 * blk + 2], xn[j][4 * blk + 3]};
            if constexpr (!KV::kSplitV)
#pragma unroll
                for (int r = 0; r < 4; ++r) S.Vt[16 * blk + 4 * g + r][tok] = xn[j][4 * blk + r];
        }
    }
}
template <int NB, int J0 = 0, class KV>
__device__ inline void kv_from_y(KV& S, const int (&qb)[2], const float (&xn)[2][8], const ModelView& M) {
    Split2 xs[2];
    if constexpr (KV::kSplitK) {
#pragma unroll
        for (int j = J0; j < J0 + NB; ++j) xs[j] = split2(xn[j], 1.0f);  // xn = ln_1 output x 2^attn_ey (PL)
    }
    kv_store<NB, J0>(S, qb, xn, xs);
}
// both of the above from one split of xn (the u projection's B operand and the keys / values
// are the same LayerNorm output at the same scale)
template <int NB, int J0 = 0, class KV>
__device__ inline void u_proj_kv3_n(const float* W, const FragSrc3& f3, const float (&xn)[2][8], float (&q)[2][8],
                                    KV& S, const int (&qb)[2], const ModelView& M) {
    // the G tiles first: their L2 latency runs under the split and the K/V stores
    Split2 wg[2];
    ld_g(f3, wg);
    Split2 xs[2];
#pragma unroll
    for (int j = J0; j < J0 + NB; ++j) xs[j] = split2(xn[j], 1.0f);  // xn = ln_1 output x 2^attn_ey (PL)
    kv_store<NB, J0>(S, qb, xn, xs);
    u_proj3_w<NB, J0>(W, wg, xs, q, M);
}

// Causal flash attention of query block qb over keys [key_lo, 16*qb + c] (key_lo <= 16):
// per token column a softmax reference m (-inf when no key; never more than
// kSlack below the column's max), l = 2^kPExp sum_s 2^(s-m) and the unnormalised o^T =
// 2^(attn_ey + kPExp) sum_s 2^(s-m) v_s (C-layout), all in the exp2 domain: s and m are the
// scores times log2(e) (folded into the scale), so each probability is one v_exp_f32.  o / l is
// the attention output at the scale of the c_proj product's B operand (attn_proj3_ol).
// kReduceL = false (split-value form): lsum is returned as this lane's partial, for a caller that
// reduces two blocks' columns at once (sum_cols2).  The split-value form needs diag_bias (the three
// additive rows of diag_bias_init in LDS).
template <class KV, bool kReduceL = true>
__device__ inline void attend(const KV& S, const float (&q)[8], int qb, int key_lo, float scale, float& m,
                              float& lsum, float (&o)[8], const ModelView& M, const float* diag_bias = nullptr) {
    // The running reference m of a token column moves only when a key tile holds a
    // score more than kSlack above it (always for the first tile with a key): the
    // probabilities are exp(s - m) <= e^kSlack, so the sums cannot overflow, and the
    // result sum_s e^(s-m) v / sum_s e^(s-m) is the same softmax for any reference.
    // Tiles that move nothing skip the cross-lane column max and the rescale of o
    // and lsum, which shortens the per-tile chain (the test is one wave vote).
    constexpr float kSlack = 32.f;
    const int lane = lane_id(), g = lane >> 4, c = lane & 15;
    // 1 / scale below without a division: the callers' scale is a constant, so 1 / (scale log2 e)
    // folds at compile time and the power of two is exact (the same bits as the division)
    const float inv_scale_c = 1.0f / (scale * 1.4426950408889634f);
    scale *= 1.4426950408889634f;  // log2(e): the exp2 domain
    // scores on fp16 two-part products: keys x 2^attn_ey, queries x 2^attn_eq (as given), and the
    // exact power of two folded into the 1/sqrt(d) scale
    const Split2 qs = split2(q, 1.0f);  // q x 2^attn_eq already (u_proj3_w)
    scale *= exp2i(-(M.attn_ey + M.attn_eq));
    if constexpr (KV::kSplitV) {
        // both products on mfma_x3, key tiles in pairs: per tile S^T = K Q^T, per pair
        // and feature half O^T += V^T P^T with K = the pair's 32 keys (P^T's C-layout of
        // the two tiles is the B operand as it stands).  An unpaired last tile reads the
        // pair's second tile from LDS with probability 0 (the rollout zeroes VS at launch,
        // so it holds finite values).  The softmax reference moves as in the per-tile
        // form below, one vote per pair, but with kSlackP = 8: P <= 2^8, so P x 2^kPExp
        // fits fp16, and o accumulates at scale 2^(attn_ey + kPExp).
        // Per score: the vote compares the raw products with a threshold kept in their units
        // (thr = (m + kSlackP) / scale, moved with m), and the probability is one fma into
        // the exponent, 2^(sc scale - m + kPExp) = P x 2^kPExp (bm = kPExp - m), so neither
        // the scaled score nor the P x 2^kPExp product is formed; masks only on the diagonal
        // tile and the tile holding key_lo.
        constexpr float kSlackP = 8.f;
        const float inv_scale = inv_scale_c * exp2i(M.attn_ey + M.attn_eq);
        const int vlo = vt_lane_off(lane);
        m = -INFINITY;
        lsum = 0.f;
        float thr = -INFINITY, bm = 0.f;  // bm = 0 while no key (not NaN)
        floatx4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
        // one pair of key tiles; MASKED only for the pair holding the diagonal tile (and the
        // pair holding key_lo): the others need neither the causal nor the key_lo test
        auto pair = [&](const int kb, auto masked) {
            float sv[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kt = kb + h;
                if constexpr (decltype(masked)::value) {
                    // Branch-free masked tile: the score product, then one additive row per tile
                    // (diag_bias_init: the causal 0 / -inf on the diagonal tile, zeros below it, -inf
                    // past it; the row is wave-uniform) and the key_lo select, all in the block of the
                    // MFMA.  A branch between an MFMA and the VALU reading its result leaves the wait
                    // states to hipcc's hazard recognizer across blocks, which (ROCm 7.2) can count
                    // too few there (scripts/isa_hazard_cfg.py).  Past the diagonal the keys are
                    // finite (zeroed at launch), so score + -inf = -inf, as the skipped tile had;
                    // below it score + 0 (bit-identical softmax).
                    const int row = kt < qb ? 1 : (kt == qb ? 0 : 2);
                    const floatx4 b = *reinterpret_cast<const floatx4*>(diag_bias + 256 * row + 4 * lane);
                    const floatx4 sc = mfma_x3(key_split(S, kt, lane), qs, floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        sv[4 * h + r] = sc[r] + b[r];
                        if (key_lo > 0 && kt * 16 + 4 * g + r < key_lo) sv[4 * h + r] = -INFINITY;
                    }
                    continue;
                }
                const floatx4 sc = mfma_x3(key_split(S, kt, lane), qs, floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
                for (int r = 0; r < 4; ++r) sv[4 * h + r] = sc[r];
            }
            const float mt = vmax8(sv);
            if (__builtin_amdgcn_ballot_w64(mt > thr)) {  // wave-uniform
                const float mn = vmax2(m, max_cols(mt * scale));
                const float corr = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m - mn);
                lsum *= corr;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    o0[r] *= corr;
                    o1[r] *= corr;
                }
                m = mn;
                thr = (mn + kSlackP) * inv_scale;
                bm = mn == -INFINITY ? 0.f : (float)kPExp - mn;
            }
            float pr[8];
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const floatx2 a2 = __builtin_elementwise_fma(floatx2{sv[r], sv[r + 1]}, floatx2{scale, scale},
                                                             floatx2{bm, bm});
                pr[r] = __builtin_amdgcn_exp2f(a2.x);
                pr[r + 1] = __builtin_amdgcn_exp2f(a2.y);
            }
            const floatx2 l2 = (floatx2{pr[0], pr[1]} + floatx2{pr[2], pr[3]}) +
                               (floatx2{pr[4], pr[5]} + floatx2{pr[6], pr[7]});
            lsum += l2.x + l2.y;
            const Split2 ps = split2(pr, 1.0f);
            const int pp = kb >> 1;
            o0 = mfma_x3(vt_split(S, pp, 0, vlo), ps, o0);
            o1 = mfma_x3(vt_split(S, pp, 1, vlo), ps, o1);
        };
        const int kb_last = qb & ~1;  // the pair holding the diagonal tile
        int kb = 0;
        if (key_lo > 0 && kb_last > 0) {
            pair(0, std::true_type{});
            kb = 2;
        }
        for (; kb < kb_last; kb += 2) pair(kb, std::false_type{});
        pair(kb_last, std::true_type{});
        if constexpr (kReduceL) lsum = sum_cols(lsum);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            o[r] = o0[r];
            o[4 + r] = o1[r];
        }
        return;
    }
    m = -INFINITY;
    lsum = 0.f;
    floatx4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb <= qb; ++kb) {
        // S^T = K Q^T on mfma_x3: the key tile is the A operand (lane (g, c): key
        // 16 kb + c, the lane group's 8 features), Q^T the B operand (q's C-layout)
        Split2 ks;
        if constexpr (KV::kSplitK) {
            ks = Split2{S.KS[kb][0][lane], S.KS[kb][1][lane]};
        } else {
            const floatx4 k0 = ld4(&S.K[kb * 16 + c][4 * g]);
            const floatx4 k1 = ld4(&S.K[kb * 16 + c][16 + 4 * g]);
            const float kv[8] = {k0[0], k0[1], k0[2], k0[3], k1[0], k1[1], k1[2], k1[3]};
            ks = split2(kv, 1.0f);  // y x 2^attn_ey already
        }
        const floatx4 sc = mfma_x3(ks, qs, floatx4{0.f, 0.f, 0.f, 0.f});
        float sv[4];
        float mt = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int key = kb * 16 + 4 * g + r;
            sv[r] = sc[r] * scale;
            if ((kb == qb && 4 * g + r > c) || key < key_lo) sv[r] = -INFINITY;
            mt = fmaxf(mt, sv[r]);
        }
        if (__builtin_amdgcn_ballot_w64(mt > m + kSlack)) {  // wave-uniform
            mt = max_cols(mt);
            const float mn = fmaxf(m, mt);
            const float corr = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m - mn);
            lsum *= corr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                o0[r] *= corr;
                o1[r] *= corr;
            }
            m = mn;
        }
        const float base = m == -INFINITY ? 0.f : m;  // no key yet: keep 0, not NaN
        float pr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = __builtin_amdgcn_exp2f(sv[r] - base);
        lsum += (pr[0] + pr[1]) + (pr[2] + pr[3]);
        const floatx4 v0 = ld4(&S.Vt[c][kb * 16 + 4 * g]);
        const floatx4 v1 = ld4(&S.Vt[16 + c][kb * 16 + 4 * g]);
#pragma unroll
        for (int s = 0; s < 4; ++s) o0 = mfma4(v0[s], pr[s], o0);
#pragma unroll
        for (int s = 0; s < 4; ++s) o1 = mfma4(v1[s], pr[s], o1);
    }
    // the split-value form's scales (exact powers of two)
    lsum = sum_cols(lsum) * exp2i(kPExp);
    const float up = exp2i(kPExp);  // the values are y x 2^attn_ey already
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        o[r] = o0[r] * up;
        o[4 + r] = o1[r] * up;
    }
}

// The masked score tiles' additive terms, three rows of 64 x 4 floats in LDS: row 0 the diagonal
// tile's causal mask (element r of lane (g, c) is key 4g + r of the tile against query c, -inf when
// 4g + r > c), row 1 zeros (a tile below the diagonal), row 2 -inf (a tile past it).
constexpr int kDiagBiasFloats = 3 * 64 * 4;
__device__ inline void diag_bias_init(float* b, int tid, int nthreads) {
    for (int i = tid; i < kDiagBiasFloats; i += nthreads) {
        const int row = i >> 8, lane = (i >> 2) & 63, r = i & 3;
        b[i] = row == 1 ? 0.0f : (row == 2 || 4 * (lane >> 4) + r > (lane & 15)) ? -INFINITY : 0.0f;
    }
}

// Blocks of wave w: pairs (w, nqb-1-w), so a wave's causal attention rows sum
// to the same length; the middle block of an odd count goes alone.  Returns
// the number of blocks (0, 1 or 2).
__device__ inline int blocks_of_wave(int w, int nqb, int (&qb)[2]) {
    qb[0] = w;
    qb[1] = nqb - 1 - w;
    if (w < nqb / 2) return 2;
    if ((nqb & 1) && w == nqb / 2) return 1;
    return 0;
}

// Copy the small per-layer parameters of n_layer blocks into LDS (layout PL;
// attention biases in the folded form: attn_b[0, E) = g0, proj_b = bvp).  The biases enter
// the split products' accumulators, so they are stored at those products' scales (exact
// powers of two): g0 and bvp x 2^(attn_ew + attn_ey), fc_b and mp_b x 2^(mlp_ew + mlp_ex).  The
// LayerNorm parameters carry the scale of the split that consumes their output (ln_1: y x
// 2^attn_ey, the keys, values and the u projection's B operand; ln_2: 2^mlp_ex, c_fc's B operand),
// so ln_cols returns the scaled value and the split multiplies by nothing: exact powers of two, the
// same bits as the scale applied after the LayerNorm.
__device__ inline void load_layer_params(float* P, const ModelView& M, int tid, int nthreads) {
    const float sa = exp2i(M.attn_ew + M.attn_ey), sm = exp2i(M.mlp_ew + M.mlp_ex);
    const float sy = exp2i(M.attn_ey), sx = exp2i(M.mlp_ex);
    for (int i = tid; i < M.n_layer * PL::size; i += nthreads) {
        const int l = i / PL::size, k = i % PL::size;
        const float* Wg = M.layers + (size_t)l * LayerOff::size;
        float v;
        if (k < PL::ln1_b) v = Wg[LayerOff::ln1_g + k] * sy;
        else if (k < PL::attn_b) v = Wg[LayerOff::ln1_b + k - PL::ln1_b] * sy;
        else if (k < PL::attn_b + kE) v = M.l0[(size_t)l * L0Off::size + L0Off::g0 + k - PL::attn_b] * sa;  // folded
        else if (k < PL::proj_b) v = 0.f;                                                                 // unused
        else if (k < PL::ln2_g) v = M.l0[(size_t)l * L0Off::size + L0Off::bvp + k - PL::proj_b] * sa;     // folded
        else if (k < PL::ln2_b) v = Wg[LayerOff::ln2_g + k - PL::ln2_g] * sx;
        else if (k < PL::fc_b) v = Wg[LayerOff::ln2_b + k - PL::ln2_b] * sx;
        else if (k < PL::mp_b) v = Wg[LayerOff::fc_b + k - PL::fc_b] * sm;
        else v = Wg[LayerOff::mp_b + k - PL::mp_b] * sm;
        P[i] = v;
    }
}

// One phase over the wave's blocks, dispatched on their count (uniform per wave).
#define DPT_BLOCKS(nb, ...)       \
    do {                          \
        if ((nb) == 2) {          \
            constexpr int NB = 2; \
            constexpr int J0 = 0; \
            (void)J0;             \
            __VA_ARGS__;          \
        } else if ((nb) == 1) {   \
            constexpr int NB = 1; \
            constexpr int J0 = 0; \
            (void)J0;             \
            __VA_ARGS__;          \
        }                         \
    } while (0)

}  // namespace dpt
