/*
 * C restatement of the DPT bandit online rollout.  TEST / BASELINE INFRASTRUCTURE.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (oracle/build/libdpt_oracle.so).  It mirrors
 * oracle/dpt_oracle.py (pinned to the reference's golden vectors) in fp32 and
 * is the CPU timing baseline ("port"): the reference algorithm
 * (evals/eval_bandit.py:56-103 + ctrls/ctrl_bandit.py:422-444 + models/net.py:41-60)
 * recomputes the whole window at every step; recompute=0 switches to the
 * exact incremental (KV-cache) form of the same arithmetic.
 *
 * Weights use the packed blob layout of include/dpt_hip.h.  OpenMP over tasks.
 */
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

static int select_action(const float* lg, int A, int sample, double u) {
    int best = 0;
    if (!sample) {
        for (int k = 1; k < A; ++k)
            if (lg[k] > lg[best]) best = k;
        return best;
    }
    float m = -INFINITY, e[64], s = 0.f;
    for (int k = 0; k < A; ++k) m = lg[k] > m ? lg[k] : m;
    for (int k = 0; k < A; ++k) { e[k] = expf(lg[k] - m); s += e[k]; }
    double c = 0.0, cdf[64];
    for (int k = 0; k < A; ++k) { c += (double)(e[k] / s); cdf[k] = c; }
    int idx = 0;
    for (int k = 0; k < A; ++k) idx += (cdf[k] / c <= u);
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
            int a = select_action(lg, A, sample, sample ? u[(size_t)h * N + i] : 0.0);
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
