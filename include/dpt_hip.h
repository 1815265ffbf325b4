/*
 * dpt_hip.h — C ABI of libdpt_hip.so, the MI355X (gfx950) implementation of the
 * DPT data-generation + in-context-evaluation hot path.
 *
 * Reference: titanium-47/decision-pretrained-transformer (pure Python).  The
 * reference has no FFI; its "plugin API" is three duck-typed Python protocols
 * (Env, Controller, model.forward).  Every entry point below names the reference
 * interface it replaces (path:line relative to the reference root).  The Python
 * shims in decision-pretrained-transformer_amd/ (envs/, ctrls/, evals/, models/)
 * keep the reference names and call these through ctypes.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer unless the name ends in _host.
 *    The caller (torch) allocates every tensor; the library allocates only the
 *    weight blob owned by an opaque dpt_model handle.
 *  - All launches are asynchronous on the given stream (hipStream_t passed as
 *    void* so this header needs no HIP include; NULL = default stream).
 *  - Return 0 (DPT_OK) or a negative DPT_E* code; dpt_last_error() returns a
 *    thread-local message for the last failing call on this thread.
 *  - Layouts are C-contiguous, row-major.  fp64 for everything the reference
 *    keeps in numpy float64 (means, rewards, arm values, uniforms, normals),
 *    fp32 for the model (the reference converts contexts with .float()).
 *  - Randomness: when an optional uniforms/normals pointer is NULL the library
 *    draws from Philox4x32-10 keyed by `seed` with counter
 *    (step, global task id, stream, 0); results therefore do not depend on how
 *    tasks are sharded over GPUs.  Passing explicit draws reproduces a
 *    reference run draw-for-draw (tests/golden).
 */
#ifndef DPT_HIP_H
#define DPT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 7 (round 6): dpt_policy_workspace_numel returns 0 and dpt_policy_rollout_args.workspace may be
 * NULL (each task's context lives in LDS); DPT_TUNE_POLICY_WAVE accepts only 1 */
#define DPT_ABI_VERSION 7

/* error codes (mapped to the reference's Python exceptions by dpt_hip/_lib.py) */
#define DPT_OK 0
#define DPT_EINVAL (-1)          /* bad shape / argument        -> ValueError            */
#define DPT_EEPISODE_ENDED (-2)  /* step past horizon           -> ValueError("Episode has already ended")
                                    envs/bandit_env.py:67-68, envs/darkroom_env.py:58-59 */
#define DPT_EHIP (-3)            /* HIP runtime error           -> RuntimeError          */
#define DPT_ENOMEM (-4)          /* device allocation failed    -> MemoryError           */
#define DPT_EUNSUPPORTED (-5)    /* configuration not built     -> NotImplementedError
                                    (envs/bandit_env.py:16,63 unknown bandit type)      */

/* bandit reward type, envs/bandit_env.py:57-63 / envs/gpu_bandit_env.py:57-62 */
#define DPT_BANDIT_GAUSSIAN 0
#define DPT_BANDIT_BERNOULLI 1
/* OR-ed into `type`: fp32 arithmetic, r = float(m) + float(g) * float(var) (two
 * roundings), the torch semantics of GPUBanditEnv.transit (gpu_bandit_env.py:58-59) */
#define DPT_BANDIT_F32 16

/* Philox stream ids (counter word 2) */
#define DPT_STREAM_SELECT 0
#define DPT_STREAM_REWARD 1
#define DPT_STREAM_ROLLIN 2
#define DPT_STREAM_DROPOUT 3 /* training dropout masks: counter (site, element / 4), word element % 4 */
#define DPT_STREAM_POLICY 16 /* + arm index: baseline-policy draws (Thompson posterior samples) */

int dpt_abi_version(void);
const char* dpt_last_error(void);
/* Process-wide tuning knobs (no effect on results beyond fp32 summation order):
 * DPT_TUNE_DECODE_TILE = tasks per workgroup of the decode kernels, 8 (default:
 * two workgroups per CU) or 16.
 * DPT_TUNE_PREFILL = 1 (default): dpt_forward_window runs windows of up to
 * dpt_prefill_max_window() tokens as one MFMA prefill; 0: always position by
 * position through the K/V workspace.
 * DPT_TUNE_DARKROOM_MEMO = 1 (default): dpt_rollout_darkroom runs one window
 * forward per distinct query state per episode (the window is fixed within an
 * episode, so a repeated state's logits are the same pure function of the same
 * inputs: results are bit-identical); 0: one forward per step.
 * DPT_TUNE_CACHE_BUDGET = bytes of the 256 MiB Infinity Cache that
 * dpt_rollout_bandit may fill with the cached rows of its earliest positions
 * (stored and streamed with the default cache policy, so they stay resident and
 * are re-read on-die every step; later positions stream non-temporally and do
 * not displace them).  0: every row non-temporal.  Cache policy only: results
 * are bit-identical for any value.
 * DPT_TUNE_BLOCK0_MFMA = 0 (default): dpt_rollout_bandit computes block 0's
 * attention with one wave per task on the vector ALUs; 1: for tiles of 8
 * five-arm tasks, on the matrix cores (the shared position-embedding terms as
 * MFMA products, the per-token terms as scalars).  Same algebra, different fp32
 * summation order; equal speed at config 2.
 * DPT_TUNE_SELECT_FAST = 1 (default): dpt_select_action decides 5- and 20-arm
 * samples on the fp32 cdf when the uniform is more than 2^-15 from every cdf
 * edge and runs the exact fp64 cdf otherwise (the rollouts always do); 0: the
 * fp64 cdf for every sample.  Bit-identical either way.
 * DPT_TUNE_POLICY_WAVE = 1 (the only value): dpt_rollout_policy runs one 64-lane
 * workgroup per task with the task's context in LDS (the per-arm pairwise sums
 * split over lanes in numpy's order); 0 returns DPT_EUNSUPPORTED since round 6
 * (the lane-per-task kernel was retired).  */
#define DPT_TUNE_DECODE_TILE 1
#define DPT_TUNE_PREFILL 2
#define DPT_TUNE_DARKROOM_MEMO 3
#define DPT_TUNE_CACHE_BUDGET 4
#define DPT_TUNE_BLOCK0_MFMA 5
#define DPT_TUNE_SELECT_FAST 6
#define DPT_TUNE_POLICY_WAVE 7
int dpt_tuning_set(int32_t key, int64_t value);
/* number of visible gfx950 devices (0 on a CPU-only host; never faults) */
int dpt_device_count(int* count_out_host);

/* ------------------------------------------------------------------ model
 * Replaces models/net.py:9-60 `Transformer` (+ transformers.GPT2Model with
 * n_head forced to 1, net.py:29).  The dpt_model handle and every entry point
 * that takes it (dpt_forward_window, dpt_decode_step, dpt_rollout_bandit,
 * dpt_rollout_darkroom) are built for n_embd == 32 (the reference default,
 * common_args.py:31); n_layer is free.  Any other width runs through the
 * width-generic dpt_train_forward / dpt_train_backward below (same blob layout),
 * which Transformer.forward uses for inference at such widths as well.
 *
 * Packed fp32 weight blob, in this order (all matrices stored [in][out]):
 *   emb_w [F][E]  emb_b [E]                 F = 2*state_dim + action_dim + 1
 *   wpe   [n_positions][E]                  n_positions = 4*(1+horizon) (net.py:26)
 *   per layer l < n_layer:
 *     ln1_g[E] ln1_b[E] attn_w[E][3E] attn_b[3E] proj_w[E][E] proj_b[E]
 *     ln2_g[E] ln2_b[E] fc_w[E][4E] fc_b[4E] mp_w[4E][E] mp_b[E]
 *   lnf_g[E] lnf_b[E]
 *   head_w[E][A]  head_b[A]
 * Conv1D weights are already [in][out]; nn.Linear weights (embed_transition,
 * pred_actions) are transposed by the packer.
 */
typedef struct dpt_model dpt_model;

typedef struct dpt_model_desc {
    int32_t n_layer;
    int32_t n_embd;      /* must be 32 for this handle (other widths: dpt_train_*) */
    int32_t state_dim;
    int32_t action_dim;  /* 1..32 */
    int32_t n_positions; /* rows of wpe */
    int32_t reserved[3];
} dpt_model_desc;

/* number of floats in the packed blob for `desc` */
int dpt_weights_numel(const dpt_model_desc* desc_host, int64_t* numel_out_host);
/* copies `packed` (device, dpt_weights_numel floats) into a blob owned by the handle */
int dpt_model_create(const dpt_model_desc* desc_host, const float* packed, dpt_model** out_host);
int dpt_model_free(dpt_model* model);

/* Full-window forward, replaces Transformer.forward (models/net.py:41-60)
 * including the token packing (net.py:42-54):
 *   token 0 = [query, 0_A, 0_sd, 0], token 1+j = [s_j, a_j, s'_j, r_j].
 * query (N,sd); states/next_states (N,C,sd); actions (N,C,A); rewards (N,C).
 * C may be 0 (the context pointers may then be NULL).  T = C+1 <= n_positions.
 * out_mode 0: out (N,A) = preds[:, -1]  (test=True)
 * out_mode 1: out (N,C,A) = preds[:, 1:] (test=False)                       */
int dpt_forward_window(const dpt_model* model, const float* query, const float* states,
                       const float* actions, const float* next_states, const float* rewards,
                       int32_t N, int32_t C, int32_t out_mode, float* out, float* workspace,
                       void* stream);
/* Windows of T = C + 1 <= dpt_prefill_max_window(model) tokens (512 for the
 * reference models) run as one MFMA prefill (all positions at once, one
 * workgroup per sequence) and `workspace` may be NULL.  Longer windows are
 * evaluated causally, position by position, through a K/V cache in
 * `workspace` (dpt_kvcache_numel(model, N, C + 1) floats); both are the full
 * causal forward (each row attends to rows <= itself).                        */
int dpt_prefill_max_window(const dpt_model* model, int32_t* tokens_out_host);

/* ------------------------------------------------------------------ KV-cache decode
 * Exact incremental form of the growing-window forward used by the bandit
 * online loop (evals/eval_bandit.py:70-89): the query token is identical at
 * every step, so positions 0..h-1 are unchanged between steps h-1 and h and
 * their keys/values can be cached.  dpt_kvcache_numel sizes the buffer for
 * [2][n_layer][N'][max_pos][E] floats, N' = N rounded up to a multiple of 16.
 * Only dpt_rollout_bandit lays it out with the padded N' stride (whole decode
 * tiles; its own per-position records); dpt_decode_step and the
 * long-window dpt_forward_window use [2][n_layer][N][max_pos][E] (V half at
 * n_layer*N*max_pos*E) and simply leave the padding unused.                   */
int dpt_kvcache_numel(const dpt_model* model, int32_t N, int32_t max_pos, int64_t* numel_out_host);
/* one decode position for all N tasks: token (N,F) packed features of position
 * `pos` (pos 0 is the query token), appends K/V at `pos`, logits (N,A) of it.  */
int dpt_decode_step(const dpt_model* model, float* kvcache, int32_t N, int32_t max_pos,
                    int32_t pos, const float* token, float* logits, void* stream);

/* ------------------------------------------------------------------ action selection
 * Replaces ctrls/ctrl_bandit.py:435-443 and ctrls/ctrl_darkroom.py:48-62:
 * sample=1: p = softmax_fp32(logits/temp) (scipy.special.softmax semantics,
 *   pairwise fp32 sum), i = #{k : cdf64_k <= u} with cdf64 = cumsum(fp64(p)) /
 *   cdf[-1] — numpy legacy RandomState.choice(A, p=p) given its uniform u.
 * sample=0: first argmax (np.argmax).
 * uniforms (N) or NULL -> Philox(seed, (counter, first_task+i, DPT_STREAM_SELECT)). */
int dpt_select_action(const float* logits, int32_t N, int32_t A, int32_t sample, float temp,
                      const double* uniforms, uint64_t seed, uint64_t counter, int64_t first_task,
                      int32_t* action_out, void* stream);

/* ------------------------------------------------------------------ environments
 * BanditEnvVec.step / GPUBanditEnv.transit (envs/bandit_env.py:56-74,
 * envs/gpu_bandit_env.py:53-74):
 *   gaussian : r = means[a] + (0.0 + var*g)   fp64, no contraction (bit-exact to numpy)
 *   bernoulli: r = (u < means[a]) ? 1 : 0      (torch.bernoulli)
 * arm_value_out (optional) = means[a]  (get_arm_value, envs/bandit_env.py:151-153).
 * noise (N) or NULL -> Philox(seed, (counter, first_task+i, DPT_STREAM_REWARD)).   */
int dpt_bandit_step(const double* means, int32_t N, int32_t A, const int32_t* action,
                    int32_t type, double var, const double* noise, uint64_t seed,
                    uint64_t counter, int64_t first_task, double* reward_out,
                    double* arm_value_out, void* stream);

/* DarkroomEnv(.Permuted).transit (envs/darkroom_env.py:37-55, :100-103): int32
 * states (N,2), action index (N), goal (N,2), perm (N,5) or NULL.  Bit-exact.   */
int dpt_darkroom_step(const int32_t* state, const int32_t* action, const int32_t* goal,
                      const int32_t* perm, int32_t N, int32_t dim, int32_t* next_state,
                      int32_t* reward, void* stream);
/* DarkroomEnv.opt_action (envs/darkroom_env.py:69-82, permuted :105-111) */
int dpt_darkroom_opt_action(const int32_t* state, const int32_t* goal, const int32_t* perm,
                            int32_t N, int32_t* action_out, void* stream);

/* Materialise the Philox draws the library would use: kind 0 = uniform [0,1),
 * kind 1 = standard normal; out[i] for global task first_task+i at `counter`. */
int dpt_draw(int32_t kind, uint64_t seed, uint64_t counter, int64_t first_task, int32_t N,
             uint32_t stream_id, double* out, void* stream);

/* ------------------------------------------------------------------ data generation
 * collect_data.py:23-53 rollin_bandit (+ generate_bandit_histories :158-182,
 * :221-225): for every task i and step h, i.i.d. arm ~ choice(A, probs[i])
 * (cdf/searchsorted semantics on the given fp64 behaviour policy, which the
 * host draws as (1-cov)*Dirichlet(1) + cov*e_rand, collect_data.py:30-36) and
 * r = means[i][arm] + (0.0 + var*g) (or Bernoulli).  uniforms/noise (H,N) or
 * NULL -> Philox streams DPT_STREAM_ROLLIN / DPT_STREAM_REWARD.
 * Outputs actions (N,H) int32, rewards (N,H) fp64.                         */
int dpt_rollin_bandit(const double* means, const double* probs, int32_t N, int32_t A, int32_t H,
                      int32_t type, double var, const double* uniforms, const double* noise,
                      uint64_t seed, int64_t first_task, int32_t* actions_out, double* rewards_out,
                      void* stream);

/* collect_data.py:83-111 rollin_mdp + :189-218: mode 0 'uniform' (i.i.d. state
 * ~ U{0..dim-1}^2 and action ~ U{0..4} per step; states_in (N,H,2) /
 * actions_in (N,H) inject them), mode 1 'expert' (greedy walk from (0,0)).
 * Outputs (N,H,2)/(N,H) int32; query_out (N,2) ~ U and opt_action_out (N) =
 * its expert label (optional).                                              */
int dpt_rollin_darkroom(const int32_t* goal, const int32_t* perm, int32_t N, int32_t H, int32_t dim,
                        int32_t mode, const int32_t* states_in, const int32_t* actions_in,
                        uint64_t seed, int64_t first_task, int32_t* states_out,
                        int32_t* actions_out, int32_t* next_states_out, int32_t* rewards_out,
                        int32_t* query_out, int32_t* opt_action_out, void* stream);

/* ------------------------------------------------------------------ fused rollouts
 * The whole online loop on device, one launch: replaces
 * evals/eval_bandit.py:56-103 (and the identical evals/eval_linear_bandit.py:54-97)
 * with BanditTransformerController (ctrls/ctrl_bandit.py:383-444) in the loop.
 * For h in [0,H): decode position h (query token at h=0, else transition h-1),
 * select a_h, step the env, append [1, onehot(a_h), 1, float(r_h)].           */
typedef struct dpt_bandit_rollout_args {
    int32_t N;            /* tasks on this device                         */
    int32_t H;            /* horizon (steps = positions)                  */
    int32_t A;            /* arms == model action_dim                     */
    int32_t type;         /* DPT_BANDIT_*                                 */
    int32_t sample;       /* 1: softmax sampling (eval online), 0: argmax */
    int32_t reserved0;
    int64_t first_task;   /* global id of task 0 (Philox counter)         */
    double var;           /* reward noise std (the reference's `var`)     */
    uint64_t seed;
    const double* means;  /* (N, A)                                       */
    const double* uniforms; /* (H, N) or NULL                             */
    const double* noise;    /* (H, N) or NULL (normals, or bernoulli uniforms) */
    float* kvcache;         /* dpt_kvcache_numel(model, N, H) floats: blocks
                             * 1..L-1 keep their ln_1 outputs y (tile-
                             * interleaved rows); block 0 is recomputed from
                             * the tokens, so its K slot holds the 16-B token
                             * records and its V slot the per-step draws     */
    int32_t* actions_out;   /* (N, H)                                       */
    double* rewards_out;    /* (N, H)                                       */
    double* arm_value_out;  /* (N, H)  = cum_means.T                         */
    float* logits_out;      /* (H, N, A) or NULL                             */
    uint64_t counter;       /* Philox counter of step 0: step h draws at
                             * counter + h, as the per-step path's selects
                             * (dpt_select_action) numbered from `counter` */
} dpt_bandit_rollout_args;

int dpt_rollout_bandit(const dpt_model* model, const dpt_bandit_rollout_args* args_host,
                       void* stream);

/* The classical comparison policies of the same online loop, fused with the env
 * (one lane per task, all H steps): replaces deploy_online_vec with
 *   DPT_POLICY_OPT      OptPolicy            ctrls/ctrl_bandit.py:22-38
 *   DPT_POLICY_EMP      EmpMeanPolicy        :57-118  (online flag: play unseen arms first)
 *   DPT_POLICY_UCB      UCBPolicy(c)         :318-380
 *   DPT_POLICY_THOMPSON ThompsonSampling     :122-251 (std, prior_mean, prior_var; sample 0 = 100-draw vote)
 *   DPT_POLICY_LCB      PessMeanPolicy(c)    :255-314
 *   DPT_POLICY_LINUCB   LinUCBPolicy(c)      :447-528 (arms (A, lin_d), lin_d <= 8)
 * Per-arm statistics are recomputed each step from the per-arm reward lists in
 * numpy's fp64 pairwise-summation order, as the reference does, so action
 * indices match it bit for bit given the same draws (LinUCB: numpy's BLAS/LAPACK
 * rounding order restated at every lin_d, csrc/dpt_linucb.h).  policy_noise:
 * Thompson (H,N,A) posterior normals (sample = 1) or (H,100,N,A) for the 100-draw vote
 * (sample = 0); LinUCB (N) uniforms for the empty-context arm.  */
#define DPT_POLICY_OPT 0
#define DPT_POLICY_EMP 1
#define DPT_POLICY_UCB 2
#define DPT_POLICY_THOMPSON 3
#define DPT_POLICY_LCB 4
#define DPT_POLICY_LINUCB 5

typedef struct dpt_policy_rollout_args {
    int32_t N, H, A, policy;
    int32_t online, type, sample, lin_d;
    int64_t first_task;
    double var;          /* env reward noise std */
    double c;            /* UCB / LCB / LinUCB constant */
    double ts_std, ts_prior_mean, ts_prior_var;
    uint64_t seed;
    const double* means;        /* (N, A) */
    const double* arms;         /* (A, lin_d) or NULL */
    const double* noise;        /* (H, N) or NULL */
    const double* policy_noise; /* see above, or NULL */
    double* workspace;          /* unused since round 6 (may be NULL): dpt_policy_workspace_numel = 0 */
    int32_t* actions_out;       /* (N, H) */
    double* rewards_out;        /* (N, H) */
    double* arm_value_out;      /* (N, H) */
    /* optional prefix context (set_batch_numpy_vec): C transitions per task,
     * replayed into the statistics before step 0 (offline eval: C = h, H = 1) */
    int32_t C;
    int32_t step0;              /* Philox step counter of step 0: step h draws at step0 + h, so a
                                 * per-step call (H = 1, step0 = h) draws what the fused launch
                                 * (step0 = 0) draws at step h */
    const int32_t* ctx_actions; /* (N, C) arm indices */
    const double* ctx_rewards;  /* (N, C) */
} dpt_policy_rollout_args;

int dpt_policy_workspace_numel(int32_t N, int32_t A, int32_t H, int64_t* numel_out_host);
int dpt_rollout_policy(const dpt_policy_rollout_args* args_host, void* stream);

/* DarkRoom in-context online evaluation, one launch: replaces
 * evals/eval_darkroom.py:20-84 deploy_online_vec with
 * DarkroomTransformerController (ctrls/ctrl_darkroom.py:23-66) and
 * DarkroomEnvVec.deploy_eval (envs/darkroom_env.py:151-175).  Episode e runs
 * `horizon` steps from (0,0); its context is episodes max(0,e-R)..e-1 in order
 * (R = ctx_episodes = H / horizon, shift-append :75-82), and every step is a
 * full forward over the window [query = current state, context...] with the
 * prediction at the last position.  Action a_t = select(logits, u_t) with
 * u_t = uniforms[(e*horizon+t)*N + i] or Philox(seed, counter + e*horizon + t,
 * first_task + i, DPT_STREAM_SELECT) -- the same draws as dpt_select_action.
 * Requires sd = 2, A = 5, 1 + R*horizon <= 512 and dim <= 255 (else
 * DPT_EUNSUPPORTED: use dpt_forward_window per step).  Windows of up to 128
 * tokens run 4 waves per task (two tasks per CU), up to 256 8 waves, up to
 * 512 16 waves (one task per CU; these need the workspace).                 */
typedef struct dpt_darkroom_rollout_args {
    int32_t N, Heps, horizon, ctx_episodes;
    int32_t dim, sample;
    int64_t first_task;
    uint64_t seed, counter;
    float temp;                 /* softmax temperature (1.0 in the reference) */
    int32_t reserved0;
    const int32_t* goals;       /* (N, 2) */
    const int32_t* perms;       /* (N, 5) action permutation or NULL */
    const double* uniforms;     /* (Heps*horizon, N) or NULL */
    int32_t* returns_out;       /* (N, Heps) sum of rewards per episode */
    int32_t* actions_out;       /* (N, Heps*horizon) or NULL */
    float* logits_out;          /* (Heps*horizon, N, 5) or NULL */
    int32_t* forwards_out;      /* (N, Heps) window forwards run per task and episode, or NULL */
    float* workspace;           /* dpt_darkroom_workspace_numel_window(N, 1 + R*horizon) floats
                                 * (dpt_darkroom_workspace_numel(N): enough for any window), or
                                 * NULL (windows up to 256 only): the context
                                 * tokens' layer-0 inputs, queries and attention partials, fixed
                                 * within an episode, are kept there instead of recomputed every
                                 * step (or kept in LDS: the partials) */
} dpt_darkroom_rollout_args;

int dpt_darkroom_workspace_numel(int32_t N, int64_t* numel_out_host);
int dpt_darkroom_workspace_numel_window(int32_t N, int32_t window, int64_t* numel_out_host);

int dpt_rollout_darkroom(const dpt_model* model, const dpt_darkroom_rollout_args* args_host,
                         void* stream);

/* Regret statistics of the online bandit eval: replaces evals/eval_bandit.py:169-178
 * (diff = opt - lnr per step, cumsum over steps, mean and scipy.stats.sem over
 * tasks) on device, in scipy's two-pass form so that ranks can all-reduce between
 * the passes.  With diff[t][h] = opt[t] - arm_value[t][h] and cr[t][h] its cumsum
 * over h, out (2, H) fp64 is
 *   DPT_REGRET_SUMS:    (sum_t diff[.][h], sum_t cr[.][h])                 (mean unused)
 *   DPT_REGRET_CENTRED: (sum_t (diff - mean[0][h])^2, sum_t (cr - mean[1][h])^2)
 * for a caller-supplied mean (2, H).  Fixed reduction order (deterministic).
 * arm_value (N, H) fp64 (dpt_rollout_bandit's arm_value_out), opt (N) fp64,
 * H <= dpt_regret_max_steps(), workspace dpt_regret_workspace_numel(N, H) doubles. */
#define DPT_REGRET_SUMS 0
#define DPT_REGRET_CENTRED 1
int dpt_regret_max_steps(int32_t* steps_out_host);
int dpt_regret_workspace_numel(int32_t N, int32_t H, int64_t* numel_out_host);
int dpt_regret_moments(const double* arm_value, const double* opt, int32_t N, int32_t H, int32_t mode,
                       const double* mean, double* workspace, double* out, void* stream);

/* ------------------------------------------------------------------ training
 * Replaces the autograd of Transformer.forward with test=False (models/net.py:41-60: preds at
 * positions 1..T-1) inside train.py:286-331 (CrossEntropyLoss(sum) over preds[:, 1:], AdamW).
 * Any n_embd (FF = 4 n_embd, one head as net.py:29 forces), fp32.  The weights are a packed
 * blob in the dpt_weights_numel layout with this desc's width (dpt_train_blob_numel floats);
 * tokens (batch, window, 2 sd + A + 1) are the packed sequences of net.py:42-54.
 * dpt_train_forward writes preds (batch, window, A) at EVERY position (position 0 included) and
 * keeps in `workspace` what the backward needs; dpt_train_backward takes dL/dpreds (batch,
 * window, A) -- zero at positions the loss does not use -- and writes every parameter's
 * gradient into dblob (same layout; wpe rows >= window are zero).  Reductions over the
 * batch * window rows run in a fixed order: the gradients are deterministic.               */
typedef struct dpt_train_desc {
    int32_t n_layer, n_embd, state_dim, action_dim, n_positions;
    int32_t batch, window;        /* sequences and tokens per sequence (1 + context length) */
    int32_t reserved;             /* flags: DPT_TRAIN_FORWARD_ONLY [| DPT_TRAIN_LAST_ONLY] or 0 */
    float dropout;                /* GPT2Config embd/attn/resid_pdrop (net.py:30-32), 0 <= p < 1 */
    int32_t reserved2;            /* 0 */
    uint64_t dropout_seed;        /* Philox key of this forward's masks (a fresh one per step) */
} dpt_train_desc;
/* Dropout (GPT2Model in training mode, p = dropout > 0): element e of a site is kept iff
 * word_e >= thr, thr = min(ceil(p 2^32), 2^32 - 1), word_e = component e % 4 of
 * Philox(dropout_seed, (site, e / 4, DPT_STREAM_DROPOUT)), and kept elements are scaled by
 * float(1 / (1 - p)).  Sites: 0 = the embedding sum x0 (B, T, E); per layer l, 1 + 3 l = the
 * attention probabilities (B, T, T) [element (b t + i) T + j], 2 + 3 l = c_proj's output,
 * 3 + 3 l = mlp.c_proj's output (B, T, E), each dropped before its residual add.  The backward
 * regenerates the same masks from the desc: pass the forward's desc unchanged.  p > 0 runs the
 * row kernels (no matrix-core forms).                                                       */
/* Inference through the training forward (no backward will follow): the workspace holds one
 * layer's activations and no attention probabilities or backward scratch
 * (dpt_train_workspace_numel sizes it by the flag); dpt_train_backward rejects the desc. */
#define DPT_TRAIN_FORWARD_ONLY 1
/* with DPT_TRAIN_FORWARD_ONLY and no dropout: preds only at the last position of each sequence
 * (models/net.py:56-58 test mode reads preds[:, -1]); the last block runs for that position alone
 * (its keys and values still cover the window) and the other rows of preds are left unwritten */
#define DPT_TRAIN_LAST_ONLY 2
int dpt_train_blob_numel(const dpt_train_desc* desc_host, int64_t* numel_out_host);
int dpt_train_workspace_numel(const dpt_train_desc* desc_host, int64_t* numel_out_host);
int dpt_train_forward(const dpt_train_desc* desc_host, const float* blob, const float* tokens, float* workspace,
                      float* preds, void* stream);
int dpt_train_backward(const dpt_train_desc* desc_host, const float* blob, const float* tokens, float* workspace,
                       const float* dpreds, float* dblob, void* stream);

/* The bandit online loop (evals/eval_bandit.py:56-103, as dpt_rollout_bandit) for models of ANY
 * width (state_dim 1, blob in the dpt_train_desc layout; desc batch / window unused, set 1, and
 * dropout 0): an exact K/V-cache decode, one step for all N tasks at a time (the training
 * forward's row kernels, or their matrix-core forms at widths 16 / 32 / 64, on N rows; the new
 * token's attention over the task's cache), then the fused kernel's selection, draws and env
 * step.  The cache holds each block's LayerNorm output y (the folded attention: u = y W_q W_k^T
 * scores the cached rows, c_proj runs on W_v W_proj), read once per step by a flash-decoding pass.
 * args->kvcache = dpt_rollout_bandit_generic_workspace_numel floats (the y cache
 * [n_layer][N][H][n_embd], the folded weights, per-step rows); the other fields as for
 * dpt_rollout_bandit.
 * Replaces the per-step path (Transformer.forward over the whole window every step) at widths
 * the fused kernel is not built for.                                                        */
int dpt_rollout_bandit_generic_workspace_numel(const dpt_train_desc* desc_host, int32_t N, int32_t H,
                                               int64_t* numel_out_host);
int dpt_rollout_bandit_generic(const dpt_train_desc* desc_host, const float* blob,
                               const dpt_bandit_rollout_args* args_host, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DPT_HIP_H */
