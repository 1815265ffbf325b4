// extern "C" surface of libdpt_hip.so (declared in include/dpt_hip.h).
// Validates shapes on the host (a kernel is never launched on an argument the
// grid arithmetic does not cover), maps failures to DPT_E* codes and keeps a
// thread-local message for dpt_last_error().
#include <algorithm>
#include <cmath>
#include <vector>
#include <stdarg.h>
#include <stdio.h>

#include <string>

#include "dpt_common.h"

namespace dpt {

static thread_local std::string g_last_error;

void set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = std::string("dpt error ") + std::to_string(code) + ": " + buf;
}

int check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return DPT_OK;
    set_error(DPT_EHIP, "%s: %s", what, hipGetErrorString(e));
    return DPT_EHIP;
}

// declared in the kernel translation units
ModelView make_view(const float* blob, const dpt_model_desc& d);
int64_t weights_numel(const dpt_model_desc& d);
int launch_decode_step(const ModelView&, float*, int, int, int, const float*, float*, hipStream_t);
int launch_window_decode(const ModelView&, float*, int, int, const float*, const float*, const float*,
                         const float*, const float*, int, float*, hipStream_t);
int launch_rollout_bandit(const ModelView&, const dpt_bandit_rollout_args&, hipStream_t);
int launch_bandit_step(const double*, int, int, const int32_t*, int, double, const double*, uint64_t, uint64_t,
                       int64_t, double*, double*, hipStream_t);
int launch_darkroom_step(const int32_t*, const int32_t*, const int32_t*, const int32_t*, int, int, int32_t*,
                         int32_t*, hipStream_t);
int launch_darkroom_opt(const int32_t*, const int32_t*, const int32_t*, int, int32_t*, hipStream_t);
int launch_select(const float*, int, int, int, float, const double*, uint64_t, uint64_t, int64_t, int32_t*,
                  hipStream_t);
int launch_draw(int, uint64_t, uint64_t, int64_t, int, uint32_t, double*, hipStream_t);
int launch_rollin_bandit(const double*, const double*, int, int, int, int, double, const double*, const double*,
                         uint64_t, int64_t, int32_t*, double*, hipStream_t);
int launch_rollin_darkroom(const int32_t*, const int32_t*, int, int, int, int, const int32_t*, const int32_t*,
                           uint64_t, int64_t, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*,
                           hipStream_t);
int launch_rollout_policy(const dpt_policy_rollout_args&, hipStream_t);
int set_policy_wave(int on);
int launch_pack_fragments(const ModelView&, float*, hipStream_t);
int64_t fragments_numel(int n_layer);
int launch_derive_l0(const ModelView&, float*, hipStream_t);
int64_t l0_numel(int n_layer);
int launch_rollout_darkroom(const ModelView&, const float*, const dpt_darkroom_rollout_args&, hipStream_t);
int darkroom_max_window();
int64_t darkroom_workspace_numel(int N, int64_t window);
int prefill_max_window(const ModelView&);
int launch_prefill(const ModelView&, const float*, const float*, const float*, const float*, const float*,
                   const float*, int, int, int, float*, hipStream_t);
int set_decode_tile(int);
int set_darkroom_memo(int);
int set_cache_budget(int64_t);
int set_block0_mfma(int);
int set_select_fast(int);
int regret_max_steps();
int64_t regret_workspace_numel(int N, int H);
int launch_regret_moments(const double*, const double*, int, int, int, const double*, double*, double*, hipStream_t);
int train_forward(const TrDims&, const float*, const float*, float*, float*, hipStream_t);
int train_backward(const TrDims&, const float*, const float*, float*, const float*, float*, hipStream_t);
int64_t train_workspace_numel(const TrDims&);
int64_t train_blob_numel(const TrDims&);
int train_dims_check(const TrDims&);
int64_t gen_rollout_workspace_numel(const TrDims&, int, int);
int rollout_bandit_generic(const TrDims&, const float*, const dpt_bandit_rollout_args&, hipStream_t);

}  // namespace dpt

using namespace dpt;

struct dpt_model {
    dpt_model_desc desc;
    float* blob;
    float* frag;  // the blocks' weights split into fp16 parts in MFMA operand order, attention folded (dpt_mfma_fwd.h Frag3)
    float* l0;    // every block's attention folded (dpt_common.h L0Off)
    ModelView view;
};

#define REQUIRE(cond, ...)                         \
    do {                                           \
        if (!(cond)) {                             \
            set_error(DPT_EINVAL, __VA_ARGS__);    \
            return DPT_EINVAL;                     \
        }                                          \
    } while (0)

static hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Power-of-two scales of the fp16 two-part products (ModelView::mlp_ew / mlp_ex,
// dpt_mfma_fwd.h Split2), from static bounds over every layer: |W| of c_fc and
// mlp.c_proj, and the activations split -- ln_2 outputs (|(x - mean) rstd| <= sqrt(E - 1),
// then g, b) and gelu outputs (|gelu(h)| <= max(|h|, 0.17), |h| <= sum_i |Wfc[i][j]| B_x +
// |b_j|).  Scaled values stay below 2^14 (fp16 max 65504) and as large as that allows,
// so the residual parts of small values stay normal fp16 numbers.
// The attention's scales (attn_ew / attn_ey / attn_eq) likewise: |G| and |Wvp|; the
// ln_1 outputs y (keys; the attention outputs are convex combinations of them); the
// queries u = y G + g0 (|u_j| <= sum_i |G[i][j]| B_y + |g0_j|).  Needs ModelView::l0.
static int fwd_scales(ModelView& v, int n_layer) {
    std::vector<float> h((size_t)n_layer * LayerOff::size), f((size_t)n_layer * L0Off::size);
    int rc = check_hip(hipMemcpy(h.data(), v.layers, h.size() * sizeof(float), hipMemcpyDeviceToHost),
                       "layer weights to host");
    if (!rc) rc = check_hip(hipMemcpy(f.data(), v.l0, f.size() * sizeof(float), hipMemcpyDeviceToHost),
                            "folded attention to host");
    if (rc) return rc;
    double wmax = 0.0, amax = 1.0, gw = 0.0, ymax = 1.0, qmax = 1.0;
    for (int l = 0; l < n_layer; ++l) {
        const float* W = h.data() + (size_t)l * LayerOff::size;
        const float* F = f.data() + (size_t)l * L0Off::size;
        double g1 = 0.0, b1 = 0.0;
        for (int i = 0; i < kE; ++i) {
            g1 = std::max(g1, (double)std::fabs(W[LayerOff::ln1_g + i]));
            b1 = std::max(b1, (double)std::fabs(W[LayerOff::ln1_b + i]));
        }
        const double by = std::sqrt((double)(kE - 1)) * g1 + b1;
        ymax = std::max(ymax, by);
        for (int j = 0; j < kE; ++j) {
            double s = std::fabs(F[L0Off::g0 + j]);
            for (int i = 0; i < kE; ++i) {
                s += std::fabs(F[L0Off::G + i * kE + j]) * by;
                gw = std::max({gw, (double)std::fabs(F[L0Off::G + i * kE + j]),
                               (double)std::fabs(F[L0Off::Wvp + i * kE + j])});
            }
            qmax = std::max(qmax, s);
        }
        double gmax = 0.0, bmax = 0.0;
        for (int i = 0; i < kE; ++i) {
            gmax = std::max(gmax, (double)std::fabs(W[LayerOff::ln2_g + i]));
            bmax = std::max(bmax, (double)std::fabs(W[LayerOff::ln2_b + i]));
        }
        const double bx = std::sqrt((double)(kE - 1)) * gmax + bmax;
        double bh = 0.17;
        for (int j = 0; j < kFF; ++j) {
            double s = std::fabs(W[LayerOff::fc_b + j]);
            for (int i = 0; i < kE; ++i) s += std::fabs(W[LayerOff::fc_w + i * kFF + j]) * bx;
            bh = std::max(bh, s);
        }
        for (int i = 0; i < kE * kFF; ++i)
            wmax = std::max({wmax, (double)std::fabs(W[LayerOff::fc_w + i]), (double)std::fabs(W[LayerOff::mp_w + i])});
        amax = std::max({amax, bx, bh});
    }
    if (!std::isfinite(wmax) || !std::isfinite(amax) || !std::isfinite(gw) || !std::isfinite(qmax)) {
        set_error(DPT_EINVAL, "non-finite block weights");
        return DPT_EINVAL;
    }
    auto expo = [](double bound, int lo, int hi) {  // largest e with bound * 2^e <= 2^14
        int e = bound > 0.0 ? (int)std::floor(std::log2(16384.0 / bound)) : hi;
        return std::min(std::max(e, lo), hi);
    };
    v.mlp_ew = expo(wmax, -24, 12);
    v.mlp_ex = expo(amax, -24, 8);
    v.attn_ew = expo(gw, -24, 12);
    v.attn_ey = expo(ymax, -24, 8);
    v.attn_eq = expo(qmax, -24, 8);
    // gelu_split folds 2^-3(ew + ex) into a constant: keep it a normal fp32 number
    if (v.mlp_ew + v.mlp_ex < -40) {
        set_error(DPT_EUNSUPPORTED, "MLP weights/activations too large for the fp16 split products (bound 2^%d)",
                  -(v.mlp_ew + v.mlp_ex) + 28);
        return DPT_EUNSUPPORTED;
    }
    return DPT_OK;
}

static int validate_desc(const dpt_model_desc* d) {
    REQUIRE(d != nullptr, "null model desc");
    if (d->n_embd != kE) {
        set_error(DPT_EUNSUPPORTED, "n_embd=%d: only n_embd=%d is built", d->n_embd, kE);
        return DPT_EUNSUPPORTED;
    }
    REQUIRE(d->n_layer >= 1 && d->n_layer <= 64, "n_layer=%d out of range", d->n_layer);
    REQUIRE(d->state_dim >= 1 && d->action_dim >= 1 && d->action_dim <= kMaxA, "state_dim=%d action_dim=%d",
            d->state_dim, d->action_dim);
    REQUIRE(2 * d->state_dim + d->action_dim + 1 <= kMaxF, "token features exceed %d", kMaxF);
    REQUIRE(d->n_positions >= 1, "n_positions=%d", d->n_positions);
    return DPT_OK;
}

extern "C" {

int dpt_abi_version(void) { return DPT_ABI_VERSION; }

const char* dpt_last_error(void) { return g_last_error.c_str(); }

static bool g_prefill = true;  // DPT_TUNE_PREFILL

int dpt_tuning_set(int32_t key, int64_t value) {
    if (key == DPT_TUNE_DECODE_TILE) {
        REQUIRE(set_decode_tile((int)value) == DPT_OK, "decode tile %lld: 8 or 16", (long long)value);
        return DPT_OK;
    }
    if (key == DPT_TUNE_PREFILL) {
        REQUIRE(value == 0 || value == 1, "prefill %lld: 0 or 1", (long long)value);
        g_prefill = value == 1;
        return DPT_OK;
    }
    if (key == DPT_TUNE_DARKROOM_MEMO) {
        REQUIRE(set_darkroom_memo((int)value) == DPT_OK, "darkroom memo %lld: 0 or 1", (long long)value);
        return DPT_OK;
    }
    if (key == DPT_TUNE_CACHE_BUDGET) {
        REQUIRE(set_cache_budget(value) == DPT_OK, "cache budget %lld B: >= 0", (long long)value);
        return DPT_OK;
    }
    if (key == DPT_TUNE_SELECT_FAST) {
        REQUIRE(set_select_fast((int)value) == DPT_OK, "select fast path %lld: 0 or 1", (long long)value);
        return DPT_OK;
    }
    if (key == DPT_TUNE_POLICY_WAVE) {
        if (set_policy_wave((int)value) != DPT_OK) {
            set_error(DPT_EUNSUPPORTED, "policy kernel %lld: only 1 (the wave-per-task kernel; the lane kernel "
                      "was retired)", (long long)value);
            return DPT_EUNSUPPORTED;
        }
        return DPT_OK;
    }
    if (key == DPT_TUNE_BLOCK0_MFMA) {
        REQUIRE(value == 0 || value == 1, "block-0 MFMA %lld: 0 or 1", (long long)value);
        return set_block0_mfma((int)value);
    }
    set_error(DPT_EINVAL, "unknown tuning key %d", key);
    return DPT_EINVAL;
}

int dpt_device_count(int* count) {
    REQUIRE(count != nullptr, "null count");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return DPT_OK;
}

int dpt_weights_numel(const dpt_model_desc* d, int64_t* numel) {
    int rc = validate_desc(d);
    if (rc) return rc;
    REQUIRE(numel != nullptr, "null numel");
    *numel = weights_numel(*d);
    return DPT_OK;
}

int dpt_model_create(const dpt_model_desc* d, const float* packed, dpt_model** out) {
    int rc = validate_desc(d);
    if (rc) return rc;
    REQUIRE(packed != nullptr && out != nullptr, "null packed/out");
    const size_t bytes = (size_t)weights_numel(*d) * sizeof(float);
    float* blob = nullptr;
    if (hipMalloc(&blob, bytes) != hipSuccess) {
        set_error(DPT_ENOMEM, "hipMalloc(%zu) for the weight blob failed", bytes);
        return DPT_ENOMEM;
    }
    rc = check_hip(hipMemcpy(blob, packed, bytes, hipMemcpyDeviceToDevice), "weight blob copy");
    if (rc) {
        (void)hipFree(blob);
        return rc;
    }
    ModelView view = make_view(blob, *d);
    float* frag = nullptr;
    float* l0 = nullptr;
    const size_t frag_bytes = (size_t)fragments_numel(d->n_layer) * sizeof(float);
    const size_t l0_bytes = (size_t)l0_numel(d->n_layer) * sizeof(float);
    if (hipMalloc(&frag, frag_bytes) != hipSuccess || hipMalloc(&l0, l0_bytes) != hipSuccess) {
        (void)hipFree(blob);
        (void)hipFree(frag);
        set_error(DPT_ENOMEM, "hipMalloc(%zu + %zu) for the derived weights failed", frag_bytes, l0_bytes);
        return DPT_ENOMEM;
    }
    rc = launch_derive_l0(view, l0, nullptr);
    view.l0 = l0;  // the fragments pack the folded attention (dpt_mfma_fwd.h Frag3)
    if (!rc) rc = check_hip(hipDeviceSynchronize(), "attention folding");
    if (!rc) rc = fwd_scales(view, d->n_layer);  // the packing uses the scales
    if (!rc) rc = launch_pack_fragments(view, frag, nullptr);
    if (!rc) rc = check_hip(hipDeviceSynchronize(), "weight derivation");
    if (rc) {
        (void)hipFree(blob);
        (void)hipFree(frag);
        (void)hipFree(l0);
        return rc;
    }
    dpt_model* m = new dpt_model;
    m->desc = *d;
    m->blob = blob;
    m->frag = frag;
    m->l0 = l0;
    m->view = view;
    *out = m;
    return DPT_OK;
}

int dpt_model_free(dpt_model* m) {
    if (!m) return DPT_OK;
    int rc = check_hip(hipFree(m->blob), "hipFree weight blob");
    int rc2 = check_hip(hipFree(m->frag), "hipFree fragment weights");
    const int rc3 = check_hip(hipFree(m->l0), "hipFree folded attention weights");
    if (!rc2) rc2 = rc3;
    delete m;
    if (!rc) rc = rc2;
    return rc;
}

int dpt_kvcache_numel(const dpt_model* m, int32_t N, int32_t max_pos, int64_t* numel) {
    REQUIRE(m && numel, "null model/numel");
    REQUIRE(N >= 1 && max_pos >= 1, "N=%d max_pos=%d", N, max_pos);
    *numel = (int64_t)2 * m->desc.n_layer * kv_tasks(N) * (int64_t)max_pos * kE;  // whole tiles (dpt_decode.hip)
    return DPT_OK;
}

int dpt_prefill_max_window(const dpt_model* m, int32_t* out) {
    REQUIRE(m && out, "null model/out");
    *out = g_prefill ? prefill_max_window(m->view) : 0;
    return DPT_OK;
}

int dpt_forward_window(const dpt_model* m, const float* query, const float* states, const float* actions,
                       const float* next_states, const float* rewards, int32_t N, int32_t C, int32_t out_mode,
                       float* out, float* workspace, void* stream) {
    REQUIRE(m, "null model");
    REQUIRE(N >= 1 && C >= 0, "N=%d C=%d", N, C);
    REQUIRE(C + 1 <= m->desc.n_positions, "context length %d + query exceeds n_positions=%d", C,
            m->desc.n_positions);
    REQUIRE(out_mode == 0 || (out_mode == 1 && C >= 1), "out_mode=%d with C=%d", out_mode, C);
    REQUIRE(query && out, "null query/out");
    REQUIRE(C == 0 || (states && actions && next_states && rewards), "null context arrays with C=%d", C);
    if (g_prefill && C + 1 <= prefill_max_window(m->view))  // all positions at once (MFMA)
        return launch_prefill(m->view, m->frag, query, states, actions, next_states, rewards, N, C, out_mode, out,
                              S(stream));
    REQUIRE(workspace, "null workspace (needed for windows over %d tokens)", prefill_max_window(m->view));
    return launch_window_decode(m->view, workspace, N, C, query, states, actions, next_states, rewards, out_mode,
                                out, S(stream));
}

int dpt_decode_step(const dpt_model* m, float* kv, int32_t N, int32_t max_pos, int32_t pos, const float* token,
                    float* logits, void* stream) {
    REQUIRE(m && kv && token && logits, "null pointer");
    REQUIRE(N >= 1 && pos >= 0 && pos < max_pos, "N=%d pos=%d max_pos=%d", N, pos, max_pos);
    REQUIRE(pos < m->desc.n_positions, "pos=%d >= n_positions=%d", pos, m->desc.n_positions);
    return launch_decode_step(m->view, kv, N, max_pos, pos, token, logits, S(stream));
}

int dpt_select_action(const float* logits, int32_t N, int32_t A, int32_t sample, float temp,
                      const double* uniforms, uint64_t seed, uint64_t counter, int64_t first_task,
                      int32_t* action_out, void* stream) {
    REQUIRE(logits && action_out, "null pointer");
    REQUIRE(N >= 1 && A >= 1 && A <= kMaxA, "N=%d A=%d", N, A);
    REQUIRE(temp > 0.f, "temp=%g", (double)temp);
    return launch_select(logits, N, A, sample, temp, uniforms, seed, counter, first_task, action_out, S(stream));
}

int dpt_bandit_step(const double* means, int32_t N, int32_t A, const int32_t* action, int32_t type, double var,
                    const double* noise, uint64_t seed, uint64_t counter, int64_t first_task, double* reward_out,
                    double* arm_value_out, void* stream) {
    REQUIRE(means && action && reward_out, "null pointer");
    REQUIRE(N >= 1 && A >= 1, "N=%d A=%d", N, A);
    const int base = type & ~DPT_BANDIT_F32;
    if (base != DPT_BANDIT_GAUSSIAN && base != DPT_BANDIT_BERNOULLI) {
        set_error(DPT_EUNSUPPORTED, "bandit type %d", type);
        return DPT_EUNSUPPORTED;
    }
    return launch_bandit_step(means, N, A, action, type, var, noise, seed, counter, first_task, reward_out,
                              arm_value_out, S(stream));
}

int dpt_darkroom_step(const int32_t* state, const int32_t* action, const int32_t* goal, const int32_t* perm,
                      int32_t N, int32_t dim, int32_t* next_state, int32_t* reward, void* stream) {
    REQUIRE(state && action && goal && next_state && reward, "null pointer");
    REQUIRE(N >= 1 && dim >= 1, "N=%d dim=%d", N, dim);
    return launch_darkroom_step(state, action, goal, perm, N, dim, next_state, reward, S(stream));
}

int dpt_darkroom_opt_action(const int32_t* state, const int32_t* goal, const int32_t* perm, int32_t N,
                            int32_t* action_out, void* stream) {
    REQUIRE(state && goal && action_out, "null pointer");
    REQUIRE(N >= 1, "N=%d", N);
    return launch_darkroom_opt(state, goal, perm, N, action_out, S(stream));
}

int dpt_draw(int32_t kind, uint64_t seed, uint64_t counter, int64_t first_task, int32_t N, uint32_t stream_id,
             double* out, void* stream) {
    REQUIRE(out && N >= 1 && (kind == 0 || kind == 1), "kind=%d N=%d", kind, N);
    return launch_draw(kind, seed, counter, first_task, N, stream_id, out, S(stream));
}

int dpt_rollin_bandit(const double* means, const double* probs, int32_t N, int32_t A, int32_t H, int32_t type,
                      double var, const double* uniforms, const double* noise, uint64_t seed, int64_t first_task,
                      int32_t* actions_out, double* rewards_out, void* stream) {
    REQUIRE(means && probs && actions_out && rewards_out, "null pointer");
    REQUIRE(N >= 1 && A >= 1 && H >= 1, "N=%d A=%d H=%d", N, A, H);
    if (type != DPT_BANDIT_GAUSSIAN && type != DPT_BANDIT_BERNOULLI) {
        set_error(DPT_EUNSUPPORTED, "bandit type %d", type);
        return DPT_EUNSUPPORTED;
    }
    return launch_rollin_bandit(means, probs, N, A, H, type, var, uniforms, noise, seed, first_task, actions_out,
                                rewards_out, S(stream));
}

int dpt_rollin_darkroom(const int32_t* goal, const int32_t* perm, int32_t N, int32_t H, int32_t dim, int32_t mode,
                        const int32_t* states_in, const int32_t* actions_in, uint64_t seed, int64_t first_task,
                        int32_t* states_out, int32_t* actions_out, int32_t* next_states_out, int32_t* rewards_out,
                        int32_t* query_out, int32_t* opt_action_out, void* stream) {
    REQUIRE(goal && states_out && actions_out && next_states_out && rewards_out, "null pointer");
    REQUIRE(N >= 1 && H >= 1 && dim >= 1, "N=%d H=%d dim=%d", N, H, dim);
    if (mode != 0 && mode != 1) {
        set_error(DPT_EUNSUPPORTED, "rollin mode %d (0 uniform, 1 expert)", mode);
        return DPT_EUNSUPPORTED;
    }
    REQUIRE((states_in == nullptr) == (actions_in == nullptr), "inject states and actions together");
    REQUIRE(mode == 0 || states_in == nullptr, "injected draws only in uniform mode");
    return launch_rollin_darkroom(goal, perm, N, H, dim, mode, states_in, actions_in, seed, first_task, states_out,
                                  actions_out, next_states_out, rewards_out, query_out, opt_action_out, S(stream));
}

int dpt_policy_workspace_numel(int32_t N, int32_t A, int32_t H, int64_t* numel) {
    REQUIRE(numel && N >= 1 && A >= 1 && H >= 1, "N=%d A=%d H=%d", N, A, H);
    // 0 since round 6: the policy kernel keeps each task's context in LDS (the retired lane kernel
    // kept per-arm reward lists here)
    *numel = 0;
    return DPT_OK;
}

int dpt_rollout_policy(const dpt_policy_rollout_args* a, void* stream) {
    REQUIRE(a, "null args");
    REQUIRE(a->N >= 1 && a->H >= 1 && a->A >= 1 && a->A <= kMaxA, "N=%d H=%d A=%d", a->N, a->H, a->A);
    REQUIRE(a->C >= 0 && a->C + a->H <= 2048, "C+H=%d > 2048 (pairwise-sum depth)", a->C + a->H);
    REQUIRE(a->C == 0 || (a->ctx_actions && a->ctx_rewards), "null prefix context with C=%d", a->C);
    REQUIRE(a->means && a->actions_out && a->rewards_out && a->arm_value_out, "null pointer");
    REQUIRE(a->policy >= DPT_POLICY_OPT && a->policy <= DPT_POLICY_LINUCB, "policy=%d", a->policy);
    REQUIRE(a->policy != DPT_POLICY_LINUCB || (a->arms && a->lin_d >= 1 && a->lin_d <= 8), "LinUCB needs arms, d<=8");
    if (a->type != DPT_BANDIT_GAUSSIAN && a->type != DPT_BANDIT_BERNOULLI) {
        set_error(DPT_EUNSUPPORTED, "bandit type %d", a->type);
        return DPT_EUNSUPPORTED;
    }
    return launch_rollout_policy(*a, S(stream));
}

int dpt_regret_max_steps(int32_t* out) {
    REQUIRE(out, "null out");
    *out = regret_max_steps();
    return DPT_OK;
}

int dpt_regret_workspace_numel(int32_t N, int32_t H, int64_t* numel) {
    REQUIRE(numel && N >= 1 && H >= 1, "N=%d H=%d", N, H);
    *numel = regret_workspace_numel(N, H);
    return DPT_OK;
}

int dpt_regret_moments(const double* arm_value, const double* opt, int32_t N, int32_t H, int32_t mode,
                       const double* mean, double* workspace, double* out, void* stream) {
    REQUIRE(arm_value && opt && workspace && out, "null pointer");
    REQUIRE(N >= 1 && H >= 1 && H <= regret_max_steps(), "N=%d H=%d (H <= %d)", N, H, regret_max_steps());
    REQUIRE(mode == DPT_REGRET_SUMS || mode == DPT_REGRET_CENTRED, "mode=%d", mode);
    REQUIRE(mode == DPT_REGRET_SUMS || mean, "centred pass needs the mean");
    return launch_regret_moments(arm_value, opt, N, H, mode, mean, workspace, out, S(stream));
}

int dpt_rollout_bandit(const dpt_model* m, const dpt_bandit_rollout_args* a, void* stream) {
    REQUIRE(m && a, "null model/args");
    REQUIRE(a->N >= 1 && a->H >= 1, "N=%d H=%d", a->N, a->H);
    REQUIRE(a->A == m->desc.action_dim, "A=%d != model action_dim=%d", a->A, m->desc.action_dim);
    REQUIRE(m->desc.state_dim == 1, "bandit rollout needs state_dim=1 (got %d)", m->desc.state_dim);
    REQUIRE(a->H <= m->desc.n_positions, "H=%d exceeds n_positions=%d", a->H, m->desc.n_positions);
    REQUIRE(a->means && a->kvcache && a->actions_out && a->rewards_out && a->arm_value_out, "null output");
    if (a->type != DPT_BANDIT_GAUSSIAN && a->type != DPT_BANDIT_BERNOULLI) {
        set_error(DPT_EUNSUPPORTED, "bandit type %d", a->type);
        return DPT_EUNSUPPORTED;
    }
    return launch_rollout_bandit(m->view, *a, S(stream));
}

int dpt_darkroom_workspace_numel(int32_t N, int64_t* numel) {
    REQUIRE(numel && N >= 1, "N=%d", N);
    *numel = darkroom_workspace_numel(N, darkroom_max_window());
    return DPT_OK;
}

int dpt_darkroom_workspace_numel_window(int32_t N, int32_t window, int64_t* numel) {
    REQUIRE(numel && N >= 1 && window >= 1, "N=%d window=%d", N, window);
    *numel = darkroom_workspace_numel(N, window);
    return DPT_OK;
}

int dpt_rollout_darkroom(const dpt_model* m, const dpt_darkroom_rollout_args* a, void* stream) {
    REQUIRE(m && a, "null model/args");
    REQUIRE(a->N >= 1 && a->Heps >= 1 && a->horizon >= 1 && a->ctx_episodes >= 1,
            "N=%d Heps=%d horizon=%d ctx_episodes=%d", a->N, a->Heps, a->horizon, a->ctx_episodes);
    REQUIRE(a->dim >= 1 && a->dim <= 255, "dim=%d", a->dim);
    REQUIRE(a->goals && a->returns_out, "null goals/returns_out");
    REQUIRE(!a->sample || a->temp > 0.0f, "temp=%g", (double)a->temp);
    const int64_t window = 1 + (int64_t)a->ctx_episodes * a->horizon;
    REQUIRE(window <= m->desc.n_positions, "window %lld exceeds n_positions=%d", (long long)window,
            m->desc.n_positions);
    if (m->desc.state_dim != 2 || m->desc.action_dim != 5 || window > darkroom_max_window()) {
        set_error(DPT_EUNSUPPORTED, "fused darkroom rollout needs sd=2, A=5, window<=%d (sd=%d A=%d window=%lld)",
                  darkroom_max_window(), m->desc.state_dim, m->desc.action_dim, (long long)window);
        return DPT_EUNSUPPORTED;
    }
    return launch_rollout_darkroom(m->view, m->frag, *a, S(stream));
}

static int train_dims(const dpt_train_desc* d, TrDims& o) {
    REQUIRE(d != nullptr, "null train desc");
    REQUIRE(d->n_layer >= 1 && d->n_layer <= 64 && d->n_embd >= 1 && d->n_embd <= 1024 && d->state_dim >= 1 &&
                d->action_dim >= 1 && d->n_positions >= 1 && d->batch >= 1 && d->window >= 1 &&
                d->window <= d->n_positions,
            "train desc: n_layer=%d n_embd=%d sd=%d A=%d n_positions=%d batch=%d window=%d", d->n_layer, d->n_embd,
            d->state_dim, d->action_dim, d->n_positions, d->batch, d->window);
    REQUIRE((d->reserved & ~(DPT_TRAIN_FORWARD_ONLY | DPT_TRAIN_LAST_ONLY)) == 0 && d->reserved2 == 0,
            "train desc: unknown flags 0x%x", d->reserved);
    REQUIRE(!(d->reserved & DPT_TRAIN_LAST_ONLY) || ((d->reserved & DPT_TRAIN_FORWARD_ONLY) && d->dropout == 0.0f),
            "train desc: DPT_TRAIN_LAST_ONLY needs DPT_TRAIN_FORWARD_ONLY and no dropout");
    REQUIRE(d->dropout >= 0.0f && d->dropout < 1.0f, "train desc: dropout %g outside [0, 1)", (double)d->dropout);
    // fwd_only: 1 = forward-only workspace, 3 = that and preds at the last position only
    const int fo = (d->reserved & DPT_TRAIN_FORWARD_ONLY) ? ((d->reserved & DPT_TRAIN_LAST_ONLY) ? 3 : 1) : 0;
    o = TrDims{d->n_layer, d->n_embd, 2 * d->state_dim + d->action_dim + 1, d->action_dim, d->batch, d->window,
               d->n_positions, fo, 0u, 1.0f, d->dropout_seed};
    if (d->dropout > 0.0f) {  // keep iff word >= ceil(p 2^32): P(keep) = 1 - p to 2^-32
        const double t = std::ceil((double)d->dropout * 4294967296.0);
        o.drop_thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
        o.drop_scale = 1.0f / (1.0f - d->dropout);
    }
    return train_dims_check(o);
}

int dpt_train_blob_numel(const dpt_train_desc* d, int64_t* numel) {
    TrDims t;
    if (int rc = train_dims(d, t)) return rc;
    REQUIRE(numel, "null numel");
    *numel = train_blob_numel(t);
    return DPT_OK;
}

int dpt_train_workspace_numel(const dpt_train_desc* d, int64_t* numel) {
    TrDims t;
    if (int rc = train_dims(d, t)) return rc;
    REQUIRE(numel, "null numel");
    *numel = train_workspace_numel(t);
    return DPT_OK;
}

int dpt_train_forward(const dpt_train_desc* d, const float* blob, const float* tokens, float* ws, float* preds,
                      void* stream) {
    TrDims t;
    if (int rc = train_dims(d, t)) return rc;
    REQUIRE(blob && tokens && ws && preds, "null pointer");
    return train_forward(t, blob, tokens, ws, preds, S(stream));
}

int dpt_train_backward(const dpt_train_desc* d, const float* blob, const float* tokens, float* ws,
                       const float* dpreds, float* dblob, void* stream) {
    TrDims t;
    if (int rc = train_dims(d, t)) return rc;
    REQUIRE(blob && tokens && ws && dpreds && dblob, "null pointer");
    REQUIRE(!t.fwd_only, "train backward: the description is forward-only (DPT_TRAIN_FORWARD_ONLY)");
    return train_backward(t, blob, tokens, ws, dpreds, dblob, S(stream));
}

int dpt_rollout_bandit_generic_workspace_numel(const dpt_train_desc* d, int32_t N, int32_t H, int64_t* numel) {
    TrDims t;
    if (int rc = train_dims(d, t)) return rc;
    REQUIRE(numel, "null numel");
    REQUIRE(N >= 0 && H >= 0, "N=%d H=%d", N, H);
    *numel = gen_rollout_workspace_numel(t, N, H);
    return DPT_OK;
}

int dpt_rollout_bandit_generic(const dpt_train_desc* d, const float* blob, const dpt_bandit_rollout_args* a,
                               void* stream) {
    TrDims t;
    if (int rc = train_dims(d, t)) return rc;
    REQUIRE(blob && a, "null pointer");
    REQUIRE(!t.drop(), "generic bandit rollout: dropout must be 0 (an eval-mode forward)");
    if (a->N == 0 || a->H == 0) return DPT_OK;
    return rollout_bandit_generic(t, blob, *a, S(stream));
}

}  // extern "C"
