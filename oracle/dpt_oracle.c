/*
 * C restatement of the DPT bandit online rollout.  TEST / BASELINE INFRASTRUCTURE.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (oracle/build/libdpt_oracle.so).  It mirrors
 * oracle/dpt_oracle.py and is pinned to the reference's recorded rollouts itself
 * (tests/test_oracle_golden.py::test_c_bandit_oracle_matches_reference,
 * ::test_c_darkroom_oracle_matches_reference).  The fp32 bandit rollout is the CPU
 * timing baseline ("port"), the float64 one (dpt_oracle_bandit_rollout_f64) the
 * full-size checker of the GPU tests: the reference algorithm
 * (evals/eval_bandit.py:56-103 + ctrls/ctrl_bandit.py:422-444 + models/net.py:41-60)
 * recomputes the whole window at every step; recompute=0 switches to the
 * exact incremental (KV-cache) form of the same arithmetic.
 *
 * Weights use the packed blob layout of include/dpt_hip.h.  OpenMP over tasks.
 */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define E 32
#define FF 128
#define LSIZE 12704

typedef struct {
    const float *emb_w, *emb_b, *wpe, *layers, *lnf_g, *lnf_b, *head_w, *head_b;
    int L, sd, A, F;
} view_t;

static view_t make_view(const float* b, int L, int sd, int A, int npos) {
    view_t v;
    int F = 2 * sd + A + 1;
    size_t o = 0;
    v.emb_w = b + o; o += (size_t)F * E;
    v.emb_b = b + o; o += E;
    v.wpe = b + o; o += (size_t)npos * E;
    v.layers = b + o; o += (size_t)L * LSIZE;
    v.lnf_g = b + o; o += E;
    v.lnf_b = b + o; o += E;
    v.head_w = b + o; o += (size_t)E * A;
    v.head_b = b + o;
    v.L = L; v.sd = sd; v.A = A; v.F = F;
    return v;
}

static void layer_norm(const float* x, const float* g, const float* b, float* y) {
    float mean = 0.f, var = 0.f;
    for (int j = 0; j < E; ++j) mean += x[j];
    mean /= E;
    for (int j = 0; j < E; ++j) var += (x[j] - mean) * (x[j] - mean);
    var /= E;
    float rstd = 1.0f / sqrtf(var + 1e-5f);
    for (int j = 0; j < E; ++j) y[j] = (x[j] - mean) * rstd * g[j] + b[j];
}

static float gelu_new(float x) {
    return 0.5f * x * (1.0f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}

/* y[out] = b[out] + sum_k x[k] W[k][out]   (W stored [in][out]) */
static void linear(const float* x, int in, const float* W, const float* b, int out, float* y) {
    for (int o = 0; o < out; ++o) y[o] = b[o];
    for (int k = 0; k < in; ++k) {
        const float xk = x[k];
        const float* w = W + (size_t)k * out;
        for (int o = 0; o < out; ++o) y[o] += xk * w[o];
    }
}

/* one token at position p through all layers, attending to K/V rows 0..p (kc/vc per layer [T][E]) */
static void token_forward(const view_t* v, const float* tok, int p, float* kc, float* vc, int Tcap,
                          float* logits) {
    float x[E], xn[E], qkv[3 * E], o[E], t[E], h[FF], sc[1024];
    linear(tok, v->F, v->emb_w, v->emb_b, E, x);
    for (int j = 0; j < E; ++j) x[j] += v->wpe[(size_t)p * E + j];
    for (int l = 0; l < v->L; ++l) {
        const float* W = v->layers + (size_t)l * LSIZE;
        float* K = kc + (size_t)l * Tcap * E;
        float* V = vc + (size_t)l * Tcap * E;
        layer_norm(x, W + 0, W + 32, xn);
        linear(xn, E, W + 64, W + 3136, 3 * E, qkv);
        memcpy(K + (size_t)p * E, qkv + E, E * sizeof(float));
        memcpy(V + (size_t)p * E, qkv + 2 * E, E * sizeof(float));
        float m = -INFINITY, s = 0.f;
        for (int j = 0; j <= p; ++j) {
            float d = 0.f;
            for (int k = 0; k < E; ++k) d += qkv[k] * K[(size_t)j * E + k];
            sc[j] = d * 0.17677669529663687f;
            if (sc[j] > m) m = sc[j];
        }
        for (int k = 0; k < E; ++k) o[k] = 0.f;
        for (int j = 0; j <= p; ++j) {
            sc[j] = expf(sc[j] - m);
            s += sc[j];
        }
        for (int j = 0; j <= p; ++j) {
            const float pj = sc[j] / s;
            for (int k = 0; k < E; ++k) o[k] += pj * V[(size_t)j * E + k];
        }
        linear(o, E, W + 3232, W + 4256, E, t);
        for (int j = 0; j < E; ++j) x[j] += t[j];
        layer_norm(x, W + 4288, W + 4320, xn);
        linear(xn, E, W + 4352, W + 8448, FF, h);
        for (int j = 0; j < FF; ++j) h[j] = gelu_new(h[j]);
        linear(h, FF, W + 8576, W + 12672, E, t);
        for (int j = 0; j < E; ++j) x[j] += t[j];
    }
    layer_norm(x, v->lnf_g, v->lnf_b, xn);
    linear(xn, E, v->head_w, v->head_b, v->A, logits);
}

/* numpy's float32 sum along a contiguous axis (pairwise_sum, numpy/_core/src/umath/
 * loops_utils.h.src): sequential below 8 elements, else 8 running partials, a fixed tree and
 * the remainder (A <= 64 < 128, so no recursive halving) */
static float np_sum_f32(const float* x, int n) {
    if (n < 8) {
        float res = 0.f;
        for (int i = 0; i < n; ++i) res += x[i];
        return res;
    }
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = x[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += x[i + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x[i];
    return res;
}

/* ctrls/ctrl_bandit.py:435-443: greedy = first argmax of the fp32 logits; sampling =
 * scipy.special.softmax in float32 (max-shift, exp, numpy sum, divide) then numpy
 * RandomState.choice(A, p): cdf = cumsum(float64(p)) / last, idx = #(cdf <= u).
 * *margin (if non-NULL) = distance of u to the nearest interior cdf edge. */
static int select_action(const float* lg, int A, int sample, double u, double* margin) {
    int best = 0;
    if (margin) *margin = INFINITY;
    if (!sample) {
        for (int k = 1; k < A; ++k)
            if (lg[k] > lg[best]) best = k;
        return best;
    }
    float m = -INFINITY, e[64];
    for (int k = 0; k < A; ++k) m = lg[k] > m ? lg[k] : m;
    for (int k = 0; k < A; ++k) e[k] = expf(lg[k] - m);
    const float s = np_sum_f32(e, A);
    double c = 0.0, cdf[64];
    for (int k = 0; k < A; ++k) { c += (double)(e[k] / s); cdf[k] = c; }
    int idx = 0;
    for (int k = 0; k < A; ++k) {
        const double q = cdf[k] / c;
        idx += (q <= u);
        if (margin && k < A - 1 && fabs(q - u) < *margin) *margin = fabs(q - u);
    }
    return idx < A ? idx : A - 1;
}

/* Returns 0 on success.  u,g: (H,N) injected draws.  Outputs (N,H); logits (H,N,A) or NULL. */
int dpt_oracle_bandit_rollout(const float* blob, int L, int A, int npos, const double* means, int N, int H,
                              double var, const double* u, const double* g, int sample, int recompute,
                              int nthreads, int32_t* actions, double* rewards, double* arm_value,
                              float* logits_out) {
    if (A > 64 || H + 1 > 1024 || H > npos) return -1;
    view_t v = make_view(blob, L, 1, A, npos);
    const int F = v.F;
    int rc = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < N; ++i) {
        float* kc = (float*)malloc(sizeof(float) * (size_t)L * (H + 1) * E);
        float* vc = (float*)malloc(sizeof(float) * (size_t)L * (H + 1) * E);
        float* toks = (float*)calloc((size_t)(H + 1) * F, sizeof(float));
        float lg[64];
        toks[0] = 1.f; /* query token [1, 0...] */
        for (int h = 0; h < H; ++h) {
            if (recompute) {
                for (int p = 0; p <= h; ++p) token_forward(&v, toks + (size_t)p * F, p, kc, vc, H + 1, lg);
            } else {
                token_forward(&v, toks + (size_t)h * F, h, kc, vc, H + 1, lg);
            }
            if (logits_out)
                for (int k = 0; k < A; ++k) logits_out[((size_t)h * N + i) * A + k] = lg[k];
            int a = select_action(lg, A, sample, sample ? u[(size_t)h * N + i] : 0.0, NULL);
            double mean = means[(size_t)i * A + a];
            volatile double noise = 0.0 + var * g[(size_t)h * N + i];
            double r = mean + noise;
            actions[(size_t)i * H + h] = a;
            rewards[(size_t)i * H + h] = r;
            arm_value[(size_t)i * H + h] = mean;
            float* t = toks + (size_t)(h + 1) * F;
            t[0] = 1.f;
            t[1 + a] = 1.f;
            t[1 + A] = 1.f;
            t[2 + A] = (float)r;
        }
        free(kc);
        free(vc);
        free(toks);
    }
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * The same bandit rollout with the forward in float64 (the full-size checker of the GPU
 * tests, like oracle/dpt_oracle.py's default dtype): every position's embedding, LayerNorms,
 * projections, attention and MLP in double from the fp32 weights, the logits rounded to
 * float32 as models/net.py hands them to the controller (`.cpu().detach().numpy()` of a
 * float32 tensor), then the reference's float32 softmax and float64 choice (select_action).
 * Position p's keys/values depend only on tokens <= p, so the incremental decode below is
 * the same arithmetic as re-forwarding the window each step (recompute=1 does that; tested).
 * Outputs as dpt_oracle_bandit_rollout, plus margin (H,N): distance of u to the nearest
 * interior cdf edge (the caller's near-tie flag).
 * ------------------------------------------------------------------------------------------ */

static void layer_norm_d(const double* x, const float* g, const float* b, double* y);
static void linear_d(const double* x, int in, const float* W, const float* b, int out, double* y);

static void token_forward_d(const view_t* v, const float* tok, int p, double* kc, double* vc, int Tcap,
                            double* sc, double* logits) {
    double x[E], xn[E], qkv[3 * E], o[E], t[E], h[FF], tk[64];
    for (int k = 0; k < v->F; ++k) tk[k] = tok[k];
    linear_d(tk, v->F, v->emb_w, v->emb_b, E, x);
    for (int j = 0; j < E; ++j) x[j] += v->wpe[(size_t)p * E + j];
    for (int l = 0; l < v->L; ++l) {
        const float* W = v->layers + (size_t)l * LSIZE;
        double* K = kc + (size_t)l * Tcap * E;
        double* V = vc + (size_t)l * Tcap * E;
        layer_norm_d(x, W + 0, W + 32, xn);
        linear_d(xn, E, W + 64, W + 3136, 3 * E, qkv);
        memcpy(K + (size_t)p * E, qkv + E, E * sizeof(double));
        memcpy(V + (size_t)p * E, qkv + 2 * E, E * sizeof(double));
        double m = -INFINITY, s = 0.0;
        for (int j = 0; j <= p; ++j) {
            double d = 0.0;
            for (int k = 0; k < E; ++k) d += qkv[k] * K[(size_t)j * E + k];
            sc[j] = d / sqrt((double)E);
            if (sc[j] > m) m = sc[j];
        }
        for (int j = 0; j <= p; ++j) {
            sc[j] = exp(sc[j] - m);
            s += sc[j];
        }
        for (int k = 0; k < E; ++k) o[k] = 0.0;
        for (int j = 0; j <= p; ++j) {
            const double pj = sc[j] / s;
            for (int k = 0; k < E; ++k) o[k] += pj * V[(size_t)j * E + k];
        }
        linear_d(o, E, W + 3232, W + 4256, E, t);
        for (int j = 0; j < E; ++j) x[j] += t[j];
        layer_norm_d(x, W + 4288, W + 4320, xn);
        linear_d(xn, E, W + 4352, W + 8448, FF, h);
        for (int j = 0; j < FF; ++j)
            h[j] = 0.5 * h[j] * (1.0 + tanh(0.7978845608028654 * (h[j] + 0.044715 * h[j] * h[j] * h[j])));
        linear_d(h, FF, W + 8576, W + 12672, E, t);
        for (int j = 0; j < E; ++j) x[j] += t[j];
    }
    layer_norm_d(x, v->lnf_g, v->lnf_b, xn);
    linear_d(xn, E, v->head_w, v->head_b, v->A, logits);
}

int dpt_oracle_bandit_rollout_f64(const float* blob, int L, int A, int npos, const double* means, int N, int H,
                                  double var, const double* u, const double* g, int sample, int recompute,
                                  int nthreads, int32_t* actions, double* rewards, double* arm_value,
                                  float* logits_out, double* margin_out) {
    if (A > 64 || H > npos || H < 1) return -1;
    view_t v = make_view(blob, L, 1, A, npos);
    const int F = v.F;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < N; ++i) {
        double* kc = (double*)malloc(sizeof(double) * (size_t)L * (H + 1) * E);
        double* vc = (double*)malloc(sizeof(double) * (size_t)L * (H + 1) * E);
        double* sc = (double*)malloc(sizeof(double) * (size_t)(H + 1));
        float* toks = (float*)calloc((size_t)(H + 1) * F, sizeof(float));
        double lgd[64];
        float lg[64];
        toks[0] = 1.f; /* query token [1, 0...] */
        for (int h = 0; h < H; ++h) {
            for (int p = recompute ? 0 : h; p <= h; ++p) token_forward_d(&v, toks + (size_t)p * F, p, kc, vc, H + 1, sc, lgd);
            for (int k = 0; k < A; ++k) lg[k] = (float)lgd[k];
            if (logits_out)
                for (int k = 0; k < A; ++k) logits_out[((size_t)h * N + i) * A + k] = lg[k];
            double mg;
            int a = select_action(lg, A, sample, sample ? u[(size_t)h * N + i] : 0.0, &mg);
            if (margin_out) margin_out[(size_t)h * N + i] = mg;
            double mean = means[(size_t)i * A + a];
            volatile double noise = 0.0 + var * g[(size_t)h * N + i];
            double r = mean + noise;
            actions[(size_t)i * H + h] = a;
            rewards[(size_t)i * H + h] = r;
            arm_value[(size_t)i * H + h] = mean;
            float* t = toks + (size_t)(h + 1) * F;
            t[0] = 1.f;
            t[1 + a] = 1.f;
            t[1 + A] = 1.f;
            t[2 + A] = (float)r;
        }
        free(kc);
        free(vc);
        free(sc);
        free(toks);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * DarkRoom online evaluation (evals/eval_darkroom.py:20-84 deploy_online_vec with
 * DarkroomTransformerController, ctrls/ctrl_darkroom.py:23-66, and DarkroomEnvVec.deploy_eval,
 * envs/darkroom_env.py:151-175), in float64 like oracle/dpt_oracle.py's darkroom_online_rollout.
 * Episode e runs `horizon` steps from (0, 0); its window is [query = current state | the last
 * min(e, R) episodes' transitions in order] and every step's logits are the last position of a
 * full causal forward over that window (models/net.py:41-60).  memo=1 reuses a task's logits
 * for a state already queried in the same episode (the window is fixed within an episode, so
 * they are the same numbers); memo=0 re-forwards every step, the reference's algorithm.
 * ------------------------------------------------------------------------------------------ */

static void layer_norm_d(const double* x, const float* g, const float* b, double* y) {
    double mean = 0.0, var = 0.0;
    for (int j = 0; j < E; ++j) mean += x[j];
    mean /= E;
    for (int j = 0; j < E; ++j) var += (x[j] - mean) * (x[j] - mean);
    var /= E;
    const double rstd = 1.0 / sqrt(var + 1e-5);
    for (int j = 0; j < E; ++j) y[j] = (x[j] - mean) * rstd * g[j] + b[j];
}

static void linear_d(const double* x, int in, const float* W, const float* b, int out, double* y) {
    for (int o = 0; o < out; ++o) y[o] = b[o];
    for (int k = 0; k < in; ++k) {
        const double xk = x[k];
        const float* w = W + (size_t)k * out;
        for (int o = 0; o < out; ++o) y[o] += xk * (double)w[o];
    }
}

/* glibc libmvec's AVX2 exp (4 doubles, within 4 ulp; 1.1 ns per value against 6 ns for libm's
 * scalar exp here): the DarkRoom float64 forward's softmax and gelu_new run through it -- most
 * of that oracle's time was scalar libm calls.  Its float64 results move by ~1e-16 relative,
 * far below the 1e-5 logit bar they check (the recorded logits and rollouts stay equal). */
extern __m256d _ZGVdN4v_exp(__m256d);

static void vexp_d(double* x, int n) {
    int i = 0;
    for (; i + 4 <= n; i += 4) _mm256_storeu_pd(x + i, _ZGVdN4v_exp(_mm256_loadu_pd(x + i)));
    if (i < n) {
        double t[4] = {0.0, 0.0, 0.0, 0.0};
        memcpy(t, x + i, sizeof(double) * (size_t)(n - i));
        _mm256_storeu_pd(t, _ZGVdN4v_exp(_mm256_loadu_pd(t)));
        memcpy(x + i, t, sizeof(double) * (size_t)(n - i));
    }
}

/* gelu_new (activations.py:65) over n values (n a multiple of 4):
 * 0.5 x (1 + tanh(z)) = x / (1 + exp(-2z)), z = sqrt(2/pi) (x + 0.044715 x^3) */
static void vgelu_d(double* h, int n) {
    for (int i = 0; i < n; i += 4) {
        double t[4];
        for (int j = 0; j < 4; ++j) {
            const double x = h[i + j];
            t[j] = -2.0 * 0.7978845608028654 * (x + 0.044715 * x * x * x);
        }
        _mm256_storeu_pd(t, _ZGVdN4v_exp(_mm256_loadu_pd(t)));
        for (int j = 0; j < 4; ++j) h[i + j] = h[i + j] / (1.0 + t[j]);
    }
}

/* linear_d over 4 rows at once (x: [4][in], y: [4][out], out a multiple of 8): each output
 * keeps linear_d's order (bias, then += x[k]*w[k][o] for k ascending; separate multiply and
 * add, as -ffp-contract=off compiles linear_d), so the values are identical.  A 4-row x
 * 8-column block of y stays in registers over the whole k loop. */
static void linear_d4(const double* x, int in, const float* W, const float* b, int out, double* y) {
    for (int o0 = 0; o0 < out; o0 += 8) {
        const __m256d b0 = _mm256_cvtps_pd(_mm_loadu_ps(b + o0)), b1 = _mm256_cvtps_pd(_mm_loadu_ps(b + o0 + 4));
        __m256d a00 = b0, a01 = b1, a10 = b0, a11 = b1, a20 = b0, a21 = b1, a30 = b0, a31 = b1;
        for (int k = 0; k < in; ++k) {
            const float* w = W + (size_t)k * out + o0;
            const __m256d w0 = _mm256_cvtps_pd(_mm_loadu_ps(w)), w1 = _mm256_cvtps_pd(_mm_loadu_ps(w + 4));
            const __m256d x0 = _mm256_set1_pd(x[k]), x1 = _mm256_set1_pd(x[in + k]);
            const __m256d x2 = _mm256_set1_pd(x[2 * in + k]), x3 = _mm256_set1_pd(x[3 * in + k]);
            a00 = _mm256_add_pd(a00, _mm256_mul_pd(x0, w0));
            a01 = _mm256_add_pd(a01, _mm256_mul_pd(x0, w1));
            a10 = _mm256_add_pd(a10, _mm256_mul_pd(x1, w0));
            a11 = _mm256_add_pd(a11, _mm256_mul_pd(x1, w1));
            a20 = _mm256_add_pd(a20, _mm256_mul_pd(x2, w0));
            a21 = _mm256_add_pd(a21, _mm256_mul_pd(x2, w1));
            a30 = _mm256_add_pd(a30, _mm256_mul_pd(x3, w0));
            a31 = _mm256_add_pd(a31, _mm256_mul_pd(x3, w1));
        }
        _mm256_storeu_pd(y + o0, a00);
        _mm256_storeu_pd(y + o0 + 4, a01);
        _mm256_storeu_pd(y + out + o0, a10);
        _mm256_storeu_pd(y + out + o0 + 4, a11);
        _mm256_storeu_pd(y + 2 * out + o0, a20);
        _mm256_storeu_pd(y + 2 * out + o0 + 4, a21);
        _mm256_storeu_pd(y + 3 * out + o0, a30);
        _mm256_storeu_pd(y + 3 * out + o0 + 4, a31);
    }
}

/* rows [p0, p1) of y = linear(x): blocks of 4 through linear_d4, the rest one by one */
static void linear_rows_d(const double* x, int in, const float* W, const float* b, int out, double* y, int p0,
                          int p1) {
    int p = p0;
    for (; p + 4 <= p1; p += 4) linear_d4(x + (size_t)p * in, in, W, b, out, y + (size_t)p * out);
    for (; p < p1; ++p) linear_d(x + (size_t)p * in, in, W, b, out, y + (size_t)p * out);
}

/* causal forward over T packed tokens (T x F), logits of position T-1 (5 actions, double).
 * Buffers (Tmax = the caller's capacity, a multiple of 16): X, O [Tmax][E]; KT [E][Tmax] (keys
 * transposed, zero-filled: a query's scores over its keys are vector loops over the features,
 * each score summed over the features in order); V, Q [Tmax][E]; H [Tmax][FF]; sc [Tmax].  Every value is computed by the
 * same operations in the same order as the token-at-a-time form (per token: ln_1, c_attn,
 * causal softmax attention, c_proj, residual, ln_2, c_fc, gelu_new, mlp.c_proj, residual); the
 * per-token steps of a layer are independent once its keys and values exist, so they run
 * phase by phase over the tokens. */
static void window_forward_d(const view_t* v, const double* toks, int T, int Tmax, double* X, double* KT,
                             double* V, double* Q, double* O, double* H, double* sc, double* logits) {
    const int F = v->F;
    for (int p = 0; p < T; ++p) {
        double* x = X + (size_t)p * E;
        for (int o = 0; o < E; ++o) x[o] = v->emb_b[o];
        for (int k = 0; k < F; ++k) {
            const double t = toks[(size_t)p * F + k];
            if (t != 0.0)
                for (int o = 0; o < E; ++o) x[o] += t * (double)v->emb_w[(size_t)k * E + o];
        }
        for (int o = 0; o < E; ++o) x[o] += v->wpe[(size_t)p * E + o];
    }
    double xn[E];
    const double rs = sqrt((double)E);
    for (int l = 0; l < v->L; ++l) {
        const float* W = v->layers + (size_t)l * LSIZE;
        /* the last block: only position T-1 reaches the head */
        const int p0 = (l == v->L - 1) ? T - 1 : 0;
        /* ln_1 -> c_attn, 4 tokens at a time (O holds ln_1's output, H the qkv rows) */
        for (int p = 0; p < T; ++p) layer_norm_d(X + (size_t)p * E, W + 0, W + 32, O + (size_t)p * E);
        linear_rows_d(O, E, W + 64, W + 3136, 3 * E, H, 0, T);
        for (int p = 0; p < T; ++p) {
            const double* qkv = H + (size_t)p * 3 * E;
            memcpy(Q + (size_t)p * E, qkv, E * sizeof(double));
            for (int k = 0; k < E; ++k) KT[(size_t)k * Tmax + p] = qkv[E + k];
            memcpy(V + (size_t)p * E, qkv + 2 * E, E * sizeof(double));
        }
        for (int p = p0; p < T; ++p) {
            const double* q = Q + (size_t)p * E;
            double* o = O + (size_t)p * E;
            double m = -INFINITY, s = 0.0;
            /* 16 scores at a time, each summed over the features in order from 0.0 (KT's rows
             * are padded to a multiple of 16; scores past p are never read) */
            for (int j0 = 0; j0 <= p; j0 += 16) {
                __m256d s0 = _mm256_setzero_pd(), s1 = s0, s2 = s0, s3 = s0;
                for (int k = 0; k < E; ++k) {
                    const __m256d qk = _mm256_set1_pd(q[k]);
                    const double* kt = KT + (size_t)k * Tmax + j0;
                    s0 = _mm256_add_pd(s0, _mm256_mul_pd(qk, _mm256_loadu_pd(kt)));
                    s1 = _mm256_add_pd(s1, _mm256_mul_pd(qk, _mm256_loadu_pd(kt + 4)));
                    s2 = _mm256_add_pd(s2, _mm256_mul_pd(qk, _mm256_loadu_pd(kt + 8)));
                    s3 = _mm256_add_pd(s3, _mm256_mul_pd(qk, _mm256_loadu_pd(kt + 12)));
                }
                _mm256_storeu_pd(sc + j0, s0);
                _mm256_storeu_pd(sc + j0 + 4, s1);
                _mm256_storeu_pd(sc + j0 + 8, s2);
                _mm256_storeu_pd(sc + j0 + 12, s3);
            }
            for (int j = 0; j <= p; ++j) {
                sc[j] = sc[j] / rs;
                if (sc[j] > m) m = sc[j];
            }
            for (int j = 0; j <= p; ++j) sc[j] = sc[j] - m;
            vexp_d(sc, p + 1);
            for (int j = 0; j <= p; ++j) s += sc[j];
            /* o = sum_j (sc[j] / s) v_j in j order, the 32 features in 8 registers */
            __m256d o8[E / 4];
            for (int i = 0; i < E / 4; ++i) o8[i] = _mm256_setzero_pd();
            for (int j = 0; j <= p; ++j) {
                const __m256d pj = _mm256_set1_pd(sc[j] / s);
                const double* vj = V + (size_t)j * E;
                for (int i = 0; i < E / 4; ++i) o8[i] = _mm256_add_pd(o8[i], _mm256_mul_pd(pj, _mm256_loadu_pd(vj + 4 * i)));
            }
            for (int i = 0; i < E / 4; ++i) _mm256_storeu_pd(o + 4 * i, o8[i]);
        }
        /* c_proj + residual (Q reused for c_proj's output) */
        linear_rows_d(O, E, W + 3232, W + 4256, E, Q, p0, T);
        for (int p = p0; p < T; ++p)
            for (int j = 0; j < E; ++j) X[(size_t)p * E + j] += Q[(size_t)p * E + j];
        /* ln_2 -> c_fc -> gelu_new -> mlp.c_proj + residual */
        for (int p = p0; p < T; ++p) layer_norm_d(X + (size_t)p * E, W + 4288, W + 4320, O + (size_t)p * E);
        linear_rows_d(O, E, W + 4352, W + 8448, FF, H, p0, T);
        vgelu_d(H + (size_t)p0 * FF, (T - p0) * FF);
        linear_rows_d(H, FF, W + 8576, W + 12672, E, Q, p0, T);
        for (int p = p0; p < T; ++p)
            for (int j = 0; j < E; ++j) X[(size_t)p * E + j] += Q[(size_t)p * E + j];
    }
    layer_norm_d(X + (size_t)(T - 1) * E, v->lnf_g, v->lnf_b, xn);
    linear_d(xn, E, v->head_w, v->head_b, v->A, logits);
}

/* scipy.special.softmax on float32 logits (temp 1.0: x / 1.0 leaves them unchanged), then
 * numpy choice: cdf = cumsum(float64(p)) / last, idx = #(cdf <= u).  *margin = distance of u
 * to the nearest interior cdf edge (the caller flags near-ties). */
static int select_dr(const float* lg, int sample, double u, double* margin) {
    int best = 0;
    *margin = INFINITY;
    if (!sample) {
        for (int k = 1; k < 5; ++k)
            if (lg[k] > lg[best]) best = k;
        return best;
    }
    float m = lg[0], e[5], s = 0.f;
    for (int k = 1; k < 5; ++k) m = lg[k] > m ? lg[k] : m;
    for (int k = 0; k < 5; ++k) { e[k] = expf(lg[k] - m); s += e[k]; }
    double c = 0.0, cdf[5];
    for (int k = 0; k < 5; ++k) { c += (double)(e[k] / s); cdf[k] = c; }
    int idx = 0;
    for (int k = 0; k < 5; ++k) {
        cdf[k] /= c;
        idx += (cdf[k] <= u);
        if (k < 4 && fabs(cdf[k] - u) < *margin) *margin = fabs(cdf[k] - u);
    }
    return idx < 5 ? idx : 4;
}

/* envs/darkroom_env.py:37-55 (+ :100-103): perm, move, clip, reward iff next == goal */
static void dr_transit(int* x, int* y, int a, const int32_t* perm, const int32_t* goal, int dim, int* r) {
    if (perm) a = perm[a];
    *x += (a == 0) - (a == 1);
    *y += (a == 2) - (a == 3);
    *x = *x < 0 ? 0 : (*x > dim - 1 ? dim - 1 : *x);
    *y = *y < 0 ? 0 : (*y > dim - 1 ? dim - 1 : *y);
    *r = (*x == goal[0] && *y == goal[1]);
}

/* goals (N,2); perms (N,5) or NULL; u (Heps*horizon, N) or NULL (greedy).  Outputs: returns
 * (N,Heps); actions (N,Heps*horizon), logits (Heps*horizon,N,5), margin (Heps*horizon,N) or NULL. */
int dpt_oracle_darkroom_rollout(const float* blob, int L, int npos, const int32_t* goals, const int32_t* perms,
                                int N, int Heps, int horizon, int R, int dim, const double* u, int sample, int memo,
                                int nthreads, int32_t* returns, int32_t* actions, float* logits_out,
                                double* margin_out) {
    const int Tmax = 1 + R * horizon, F = 10, steps = Heps * horizon;
    if (Tmax > npos || dim * dim > 4096) return -1;
    const int Tpad = (Tmax + 15) & ~15; /* window_forward_d's buffer capacity */
    view_t v = make_view(blob, L, 2, 5, npos);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < N; ++i) {
        double* toks = (double*)calloc((size_t)Tmax * F, sizeof(double));
        double* hist = (double*)calloc((size_t)(R + 1) * horizon * F, sizeof(double)); /* ring of episodes */
        double* X = (double*)malloc(sizeof(double) * (size_t)Tpad * E);
        double* K = (double*)calloc((size_t)Tpad * E, sizeof(double));
        double* V = (double*)malloc(sizeof(double) * (size_t)Tpad * E);
        double* Q = (double*)malloc(sizeof(double) * (size_t)Tpad * E);
        double* Ob = (double*)malloc(sizeof(double) * (size_t)Tpad * E);
        double* Hb = (double*)malloc(sizeof(double) * (size_t)Tpad * FF);
        double* sc = (double*)malloc(sizeof(double) * (size_t)Tpad);
        float* memo_lg = (float*)malloc(sizeof(float) * (size_t)dim * dim * 5);
        char* seen = (char*)malloc((size_t)dim * dim);
        const int32_t* perm = perms ? perms + (size_t)i * 5 : NULL;
        const int32_t* goal = goals + (size_t)i * 2;
        int nep = 0; /* episodes stored in hist (<= R, oldest first) */
        for (int e = 0; e < Heps; ++e) {
            const int C = nep * horizon, T = 1 + C;
            memcpy(toks + F, hist, sizeof(double) * (size_t)C * F);
            memset(seen, 0, (size_t)dim * dim);
            double* cur = hist + (size_t)nep * horizon * F; /* this episode's slot */
            int x = 0, y = 0, ret = 0;
            for (int t = 0; t < horizon; ++t) {
                const int k = e * horizon + t, cell = x * dim + y;
                float lg[5];
                if (memo && seen[cell]) {
                    memcpy(lg, memo_lg + (size_t)cell * 5, sizeof lg);
                } else {
                    double lgd[5];
                    memset(toks, 0, sizeof(double) * F);
                    toks[0] = x;
                    toks[1] = y;
                    window_forward_d(&v, toks, T, Tpad, X, K, V, Q, Ob, Hb, sc, lgd);
                    for (int a = 0; a < 5; ++a) lg[a] = (float)lgd[a];
                    memcpy(memo_lg + (size_t)cell * 5, lg, sizeof lg);
                    seen[cell] = 1;
                }
                double mg;
                const int a = select_dr(lg, sample, sample ? u[(size_t)k * N + i] : 0.0, &mg);
                if (logits_out)
                    for (int j = 0; j < 5; ++j) logits_out[((size_t)k * N + i) * 5 + j] = lg[j];
                if (margin_out) margin_out[(size_t)k * N + i] = mg;
                if (actions) actions[(size_t)i * steps + k] = a;
                double* tk = cur + (size_t)t * F;
                memset(tk, 0, sizeof(double) * F);
                tk[0] = x;
                tk[1] = y;
                tk[2 + a] = 1.0;
                int r;
                dr_transit(&x, &y, a, perm, goal, dim, &r);
                tk[7] = x;
                tk[8] = y;
                tk[9] = r;
                ret += r;
            }
            returns[(size_t)i * Heps + e] = ret;
            if (nep < R) {
                ++nep;
            } else { /* shift-append (evals/eval_darkroom.py:75-82): drop the oldest episode */
                memmove(hist, hist + (size_t)horizon * F, sizeof(double) * (size_t)R * horizon * F);
            }
        }
        free(toks); free(hist); free(X); free(K); free(V); free(Q); free(Ob); free(Hb); free(sc); free(memo_lg);
        free(seen);
    }
    return 0;
}
