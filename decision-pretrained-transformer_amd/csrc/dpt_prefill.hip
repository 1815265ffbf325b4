// Window prefill on gfx950: Transformer.forward (models/net.py:41-60) for
// windows of T = 1 + C <= 128 tokens, all positions at once.
//
// One workgroup per sequence; each of its NW waves owns two 16-token blocks and
// runs the transposed-dataflow MFMA forward of dpt_mfma_fwd.h: token packing
// (net.py:42-54) + embed_transition + wpe, then per GPT-2 block ln_1 -> c_attn
// -> causal attention -> c_proj -> residual -> ln_2 -> c_fc -> gelu_new ->
// mlp.c_proj -> residual, then ln_f + pred_actions for the positions asked for
// (out_mode 0: the last one, test=True; out_mode 1: positions 1..C, test=False).
// NW = 4, 8, 16 waves cover windows of 128, 256, 512 tokens (16 waves: K and V
// of 512 tokens fill 140 KB of LDS, one workgroup per CU).  Longer windows go
// to window_decode_kernel (dpt_decode.hip).
#include "dpt_mfma_fwd.h"

namespace dpt {

// Model-level parameters in LDS after the per-layer blocks (offsets in floats).
struct PfTop {
    int lnf_g, lnf_b, head_w, head_b, emb_b, emb_w, total;
    __host__ __device__ static PfTop make(int L, int F, int A) {
        PfTop t;
        int o = L * PL::size;
        t.lnf_g = o; o += kE;
        t.lnf_b = o; o += kE;
        t.head_w = o; o += A * kE;  // transposed: [a][E]
        t.head_b = o; o += (A + 3) & ~3;
        t.emb_b = o; o += kE;
        t.emb_w = o; o += F * kE;
        t.total = o;
        return t;
    }
};

struct PrefillArgs {
    const float *query, *states, *actions, *next_states, *rewards;
    int N, C, out_mode;
    float* out;
    const float* frag;
};

// Feature f of token `tok` of sequence n (net.py:42-54): token 0 =
// [query, 0_A, 0_sd, 0], token 1+j = [s_j, a_j, s'_j, r_j].
__device__ inline float token_feature(const PrefillArgs& a, int sd, int A, int n, int tok, int f) {
    if (tok == 0) return f < sd ? a.query[(size_t)n * sd + f] : 0.f;
    const size_t j = (size_t)n * a.C + (tok - 1);
    if (f < sd) return a.states[j * sd + f];
    if (f < sd + A) return a.actions[j * A + (f - sd)];
    if (f < 2 * sd + A) return a.next_states[j * sd + (f - sd - A)];
    return a.rewards[j];
}

template <int NW>
__global__ void __launch_bounds__(NW * 64, (NW + 3) / 4)
prefill_kernel(ModelView M, PrefillArgs a) {
    __shared__ KVBuf<32 * NW> S;
    extern __shared__ float P[];
    const int n = blockIdx.x;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = M.n_layer, A = M.A, sd = M.sd, F = M.F;
    const int T = a.C + 1;
    const float scale = 0.17677669529663687f;  // 1/sqrt(head_dim = 32)
    const PfTop pt = PfTop::make(L, F, A);
    const FragSrc3 split0{__builtin_amdgcn_make_buffer_rsrc((void*)a.frag, (short)0, L * Frag3::bytes, 0x00020000), 0};
    load_layer_params(P, M, tid, blockDim.x);
    for (int i = tid; i < kE; i += blockDim.x) {
        P[pt.lnf_g + i] = M.lnf_g[i];
        P[pt.lnf_b + i] = M.lnf_b[i];
        P[pt.emb_b + i] = M.emb_b[i];
    }
    for (int i = tid; i < kE * A; i += blockDim.x) P[pt.head_w + (i % A) * kE + i / A] = M.head_w[i];
    for (int i = tid; i < A; i += blockDim.x) P[pt.head_b + i] = M.head_b[i];
    for (int i = tid; i < F * kE; i += blockDim.x) P[pt.emb_w + i] = M.emb_w[i];
    __syncthreads();

    const int nqb = (T + 15) >> 4;
    int qb[2];
    const int nb = blocks_of_wave(wave, nqb, qb);

    // embeddings
    float x[2][8];
    {
        const int lane = lane_id(), g = lane >> 4;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x[j][k] = 0.f;
            const int tok = qb[j] * 16 + (lane & 15);
            if (j >= nb || tok >= T) continue;
            floatx4 acc0 = ld4(P + pt.emb_b + 4 * g), acc1 = ld4(P + pt.emb_b + 16 + 4 * g);
            for (int f = 0; f < F; ++f) {
                const float v = token_feature(a, sd, A, n, tok, f);
                const floatx4 w0 = ld4(P + pt.emb_w + f * kE + 4 * g), w1 = ld4(P + pt.emb_w + f * kE + 16 + 4 * g);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc0[r] = fmaf(v, w0[r], acc0[r]);
                    acc1[r] = fmaf(v, w1[r], acc1[r]);
                }
            }
            const floatx4 p0 = ld4(M.wpe + (size_t)tok * kE + 4 * g), p1 = ld4(M.wpe + (size_t)tok * kE + 16 + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                x[j][r] = acc0[r] + p0[r];
                x[j][4 + r] = acc1[r] + p1[r];
            }
        }
    }

    for (int layer = 0; layer < L; ++layer) {
        const float* W = P + layer * PL::size;
        const FragSrc3 fs = split0.layer(layer);
        float q[2][8];
        {
            float xn[2][8];
            DPT_BLOCKS(nb, (ln_n<NB>(x, xn, W + PL::ln1_g, W + PL::ln1_b), u_proj3_n<NB>(W, fs, xn, q, M),
                            kv_from_y<NB>(S, qb, xn, M)));
        }
        bar_lds();
        if (nb > 0) {
            float o[2][8], l[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j >= nb) break;
                float m;
                attend(S, q[j], qb[j], 0, scale, m, l[j], o[j], M);
            }
            DPT_BLOCKS(nb, attn_proj3_ol<NB>(W, fs, o, l, x, M));
        }
        bar_lds();  // every read of this layer's K/V is done
        {
            float xn[2][8];
            DPT_BLOCKS(nb, (ln_n<NB>(x, xn, W + PL::ln2_g, W + PL::ln2_b), mlp3_n<NB>(W, fs, xn, x, M.mlp_ew, M.mlp_ex)));
        }
    }

    // ln_f + pred_actions for the positions asked for
    {
        const int lane = lane_id(), g = lane >> 4, c = lane & 15;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j >= nb) break;
            const int tok = qb[j] * 16 + c;
            const bool want = a.out_mode == 0 ? tok == T - 1 : (tok >= 1 && tok < T);
            // ln_f / head over every column keeps the permlane reductions uniform
            float xf[8];
            ln_cols(x[j], xf, P + pt.lnf_g, P + pt.lnf_b);
            for (int act = 0; act < A; ++act) {
                const floatx4 w0 = ld4(P + pt.head_w + act * kE + 4 * g);
                const floatx4 w1 = ld4(P + pt.head_w + act * kE + 16 + 4 * g);
                float part = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    part = fmaf(xf[r], w0[r], part);
                    part = fmaf(xf[4 + r], w1[r], part);
                }
                const float lg = sum_cols(part) + P[pt.head_b + act];
                if (want && g == 0) {
                    if (a.out_mode == 0) a.out[(size_t)n * A + act] = lg;
                    else a.out[((size_t)n * a.C + (tok - 1)) * A + act] = lg;
                }
            }
        }
    }
}

constexpr int kPrefillMaxT = 512;

// Largest window the prefill takes for this model (the parameter block must
// fit in LDS next to the K/V buffer); 0 if none.
int prefill_max_window(const ModelView& M) {
    const size_t dyn = sizeof(float) * (size_t)PfTop::make(M.n_layer, M.F, M.A).total;
    for (int t = kPrefillMaxT; t >= 128; t /= 2)
        if (dyn + sizeof(KVBuf<512>) * t / 512 + 64 <= 160 * 1024) return t;
    return 0;
}

template <int NW>
static int launch_nw(const ModelView& M, const PrefillArgs& a, size_t dyn, hipStream_t st) {
    if (dyn + sizeof(KVBuf<32 * NW>) > 160 * 1024) {
        set_error(DPT_EUNSUPPORTED, "prefill: parameter block does not fit in LDS");
        return DPT_EUNSUPPORTED;
    }
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(prefill_kernel<NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    hipLaunchKernelGGL(prefill_kernel<NW>, dim3(a.N), dim3(NW * 64), dyn, st, M, a);
    return check_hip(hipGetLastError(), "prefill_kernel launch");
}

int launch_prefill(const ModelView& M, const float* frag, const float* q, const float* cs, const float* ca,
                   const float* cn, const float* cr, int N, int C, int out_mode, float* out, hipStream_t st) {
    PrefillArgs a{q, cs, ca, cn, cr, N, C, out_mode, out, frag};
    const size_t dyn = sizeof(float) * (size_t)PfTop::make(M.n_layer, M.F, M.A).total;
    const int T = C + 1;
    if (T <= 128) return launch_nw<4>(M, a, dyn, st);
    if (T <= 256) return launch_nw<8>(M, a, dyn, st);
    return launch_nw<16>(M, a, dyn, st);
}

}  // namespace dpt
