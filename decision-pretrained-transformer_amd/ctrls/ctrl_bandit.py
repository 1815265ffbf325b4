"""Bandit controllers — drop-in for the reference ctrls/ctrl_bandit.py.

``BanditTransformerController`` keeps the reference protocol (set_batch /
set_batch_numpy_vec / act / act_numpy_vec returning one-hot numpy actions) but
the context is uploaded once per ``set_batch`` (not per act), the forward is
the gfx950 window kernel and action selection is the ``dpt_select_action``
kernel (scipy-softmax + numpy-choice semantics on device).  Inside
``evals.eval_bandit.deploy_online_vec`` the controller is not stepped at all:
the whole loop runs as one fused kernel (dpt_rollout_bandit).
"""
import numpy as np
import torch

import dpt_hip

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


class Controller:
    """Controller protocol (ctrls/ctrl_bandit.py:11-19)."""

    def set_batch(self, batch):
        self.batch = batch

    def set_batch_numpy_vec(self, batch):
        self.set_batch(batch)

    def set_env(self, env):
        self.env = env


class OptPolicy(Controller):
    """Plays the optimal arm (ctrls/ctrl_bandit.py:22-38)."""

    def __init__(self, env, batch_size=1):
        super().__init__()
        self.env = env
        self.batch_size = batch_size

    def reset(self):
        return

    def act(self, x):
        return self.env.opt_a

    def act_numpy_vec(self, x):
        return np.stack([env.opt_a for env in self.env], axis=0)


class _SelectStream:
    def __init__(self):
        self.seed = None
        self.counter = 0

    def next(self):
        if self.seed is None:
            self.seed = dpt_hip.next_seed()
        c = self.counter
        self.counter += 1
        return self.seed, c


def _onehot(idx, n):
    out = np.zeros((len(idx), n))
    out[np.arange(len(idx)), idx] = 1.0
    return out


class BanditTransformerController(Controller):
    """DPT policy for bandits (ctrls/ctrl_bandit.py:383-444)."""

    def __init__(self, model, sample=False, batch_size=1):
        self.model = model
        self.du = model.config["action_dim"]
        self.dx = model.config["state_dim"]
        self.H = model.horizon
        self.sample = sample
        self.batch_size = batch_size
        self.zeros = torch.zeros(batch_size, self.dx ** 2 + self.du + 1, device=dpt_hip.device())
        self._stream = _SelectStream()
        self.uniforms = None  # optional injected draws: callable(counter) -> (batch,) array

    def set_env(self, env):
        return

    def set_batch_numpy_vec(self, batch):
        dev = dpt_hip.device()
        self.set_batch({k: torch.as_tensor(np.asarray(v), dtype=torch.float32, device=dev) for k, v in batch.items()})

    def _select(self, logits):
        seed, ctr = self._stream.next()
        u = self.uniforms(ctr) if (self.sample and self.uniforms is not None) else None
        return dpt_hip.select_action(logits, self.sample, 1.0, uniforms=u, seed=seed, counter=ctr).cpu().numpy()

    def act(self, x):
        self.batch["zeros"] = self.zeros[:1]
        self.batch["query_states"] = torch.as_tensor(np.asarray(x), dtype=torch.float32,
                                                     device=dpt_hip.device())[None, :]
        a = self.model(self.batch)
        i = self._select(a[:1])[0]
        out = np.zeros(self.du)
        out[i] = 1.0
        return out

    def act_numpy_vec(self, x):
        self.batch["zeros"] = self.zeros
        states = torch.as_tensor(np.array(x), dtype=torch.float32, device=dpt_hip.device())
        if self.batch_size == 1:
            states = states[None, :]
        self.batch["query_states"] = states.reshape(self.batch_size, -1)
        a = self.model(self.batch)
        return _onehot(self._select(a), self.du)


class GreedyOptPolicy(Controller):
    """Replays the best-rewarded context action (ctrls/ctrl_bandit.py:41-54); single env, host."""

    def __init__(self, env):
        super().__init__()
        self.env = env

    def reset(self):
        return

    def act(self, x):
        rewards = np.asarray(torch.as_tensor(self.batch["context_rewards"]).cpu()).flatten()
        i = np.argmax(rewards)
        self.a = np.asarray(torch.as_tensor(self.batch["context_actions"]).cpu())[0][i]
        return self.a


class _KernelPolicy(Controller):
    """A classical policy evaluated by the dpt_rollout_policy kernel.

    Per-step protocol: ``set_batch_numpy_vec(context)`` then ``act_numpy_vec`` runs the
    kernel for one step on that prefix context.  Inside deploy_online_vec the whole loop
    runs fused instead (evals.eval_bandit).  Both draw the policy's own randomness (Thompson
    posterior normals, LinUCB's first arm) from the controller's stream: step k of the
    stream is Philox counter k of one seed, so the per-step and fused loops act on the same
    draws.  ``policy_noise``, optional: callable(counter) -> that step's draws ((N, A)
    posterior normals, (100, N, A) for Thompson's sample=False vote, or (N,) uniforms for
    LinUCB's first arm), injected instead.
    """

    policy = None
    online = False
    sample = True
    const = 1.0

    def __init__(self, env, batch_size=1):
        super().__init__()
        self.env = env
        self.batch_size = batch_size
        self._stream = _SelectStream()
        self.policy_noise = None
        self.first_task = 0  # global id of task 0 (a shard's first task): Philox key

    def reset(self):
        return

    def kernel_kwargs(self):
        return dict(online=self.online, sample=self.sample, c=self.const)

    def _ctx(self):
        acts = np.asarray(self.batch["context_actions"])
        rews = np.asarray(self.batch["context_rewards"]).reshape(acts.shape[0], -1)
        return np.argmax(acts, axis=-1).astype(np.int32), rews.astype(np.float64)

    def act_numpy_vec(self, x):
        ca, cr = self._ctx()
        means = np.zeros((self.batch_size, self.dim_()))  # the one env step's reward is discarded
        seed, ctr = self._stream.next()
        pn = None if self.policy_noise is None else np.asarray(self.policy_noise(ctr), np.float64)
        out = dpt_hip.rollout_policy(self.policy, means, 1, 0.0, seed=seed, counter=ctr, first_task=self.first_task,
                                     policy_noise=pn, ctx_actions=ca if ca.shape[1] else None,
                                     ctx_rewards=cr if ca.shape[1] else None, **self.kernel_kwargs())
        a = out["actions"][:, 0].cpu().numpy()
        self.a = _onehot(a, self.dim_())
        return self.a

    def dim_(self):
        return self.env.dim


class EmpMeanPolicy(_KernelPolicy):
    """Empirical-mean arm; online: unseen arms first (ctrls/ctrl_bandit.py:57-118)."""

    policy = dpt_hip.POLICY_EMP

    def __init__(self, env, online=False, batch_size=1):
        super().__init__(env, batch_size)
        self.online = online


class UCBPolicy(_KernelPolicy):
    """mean + const / max(1, sqrt(n)); unseen arms first (ctrls/ctrl_bandit.py:318-380).
    (The reference's act_numpy_vec hard-codes 200 tasks at :374; here any batch works.)"""

    policy = dpt_hip.POLICY_UCB

    def __init__(self, env, const=1.0, batch_size=1):
        super().__init__(env, batch_size)
        self.const = const


class PessMeanPolicy(_KernelPolicy):
    """Lower confidence bound mean - const / max(1, sqrt(n)) (ctrls/ctrl_bandit.py:255-314)."""

    policy = dpt_hip.POLICY_LCB

    def __init__(self, env, const=1.0, batch_size=1):
        super().__init__(env, batch_size)
        self.const = const


class ThompsonSamplingPolicy(_KernelPolicy):
    """Gaussian-prior Thompson sampling (ctrls/ctrl_bandit.py:122-251); sample=False takes the
    most frequent argmax of 100 posterior draws."""

    policy = dpt_hip.POLICY_THOMPSON

    def __init__(self, env, std=.1, sample=False, prior_mean=.5, prior_var=1 / 12.0, warm_start=False,
                 batch_size=1):
        super().__init__(env, batch_size)
        self.std = std
        self.variance = std ** 2
        self.prior_mean = prior_mean
        self.prior_variance = prior_var
        self.sample = sample
        self.warm_start = warm_start

    def kernel_kwargs(self):
        return dict(sample=self.sample, ts_std=self.std, ts_prior_mean=self.prior_mean,
                    ts_prior_var=self.prior_variance)


class LinUCBPolicy(_KernelPolicy):
    """LinUCB over fixed arm features (ctrls/ctrl_bandit.py:447-528); lin_d <= 8."""

    policy = dpt_hip.POLICY_LINUCB

    def __init__(self, env, const=1.0, batch_size=1):
        super().__init__(env, batch_size)
        self.const = const
        self.arms = env.arms
        self.d = self.arms.shape[1]
        self.dim = env.dim

    def kernel_kwargs(self):
        return dict(c=self.const, arms=np.asarray(self.arms, np.float64))


KERNEL_POLICIES = (EmpMeanPolicy, UCBPolicy, PessMeanPolicy, ThompsonSamplingPolicy, LinUCBPolicy)
