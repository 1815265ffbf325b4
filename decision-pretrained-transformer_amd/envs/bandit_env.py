"""Bandit environments — drop-in for the reference envs/bandit_env.py.

Task sampling (``sample``, ``sample_linear``, ``LinearBanditEnv.means``) stays on
the host with numpy, exactly as the reference draws it (it is setup, not the
loop, and keeping numpy's calls keeps task sets identical for a given
``np.random.seed``).  Every transition is a gfx950 kernel
(``dpt_bandit_step``): r = means[a] + (0.0 + var*g) in fp64, bit-identical to
numpy's ``means[a] + np.random.normal(0, var)`` for the same g.  Noise comes
from Philox keyed by a seed drawn from numpy's global RNG, so
``np.random.seed`` still determines a run.
"""
import numpy as np
import torch

import dpt_hip
from envs.base_env import BaseEnv, spaces

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")

_TYPES = {"uniform": dpt_hip.BANDIT_GAUSSIAN, "bernoulli": dpt_hip.BANDIT_BERNOULLI}


def sample(dim, H, var, type="uniform"):
    """envs/bandit_env.py:10-18."""
    if type == "uniform":
        means = np.random.uniform(0, 1, dim)
    elif type == "bernoulli":
        means = np.random.beta(1, 1, dim)
    else:
        raise NotImplementedError
    return BanditEnv(means, H, var=var, type=type)


def sample_linear(arms, H, var):
    """envs/bandit_env.py:21-25."""
    lin_d = arms.shape[1]
    theta = np.random.normal(0, 1, lin_d) / np.sqrt(lin_d)
    return LinearBanditEnv(theta, arms, H, var=var)


class _Stream:
    """Philox (seed, counter) pair owned by an env: one counter tick per transition."""

    def __init__(self):
        self.seed = None
        self.counter = 0

    def next(self):
        if self.seed is None:
            self.seed = dpt_hip.next_seed()
        c = self.counter
        self.counter += 1
        return self.seed, c


def _device_rewards(means, action_idx, var, type_code, stream, first_task=0, noise=None):
    seed, ctr = stream.next()
    g = None if noise is None else np.asarray(noise(ctr), np.float64).reshape(-1)
    r, _ = dpt_hip.bandit_step(means, action_idx, var, type_code, noise=g, seed=seed, counter=ctr,
                               first_task=first_task)
    return r.cpu().numpy()


class BanditEnv(BaseEnv):
    def __init__(self, means, H, var=0.0, type="uniform"):
        opt_a_index = np.argmax(means)
        self.means = means
        self.opt_a_index = opt_a_index
        self.opt_a = np.zeros(means.shape)
        self.opt_a[opt_a_index] = 1.0
        self.dim = len(means)
        self.observation_space = spaces.Box(low=1, high=1, shape=(1,))
        self.action_space = spaces.Box(low=0, high=1, shape=(self.dim,))
        self.state = np.array([1])
        self.var = var
        self.dx = 1
        self.du = self.dim
        self.topk = False
        self.type = type
        if type not in _TYPES:
            raise NotImplementedError
        # envs/bandit_env.py:45-47 ("some naming issue here"): context horizon vs episode length 1
        self.H_context = H
        self.H = 1
        self._stream = _Stream()

    def get_arm_value(self, u):
        return np.sum(self.means * u)

    def reset(self):
        self.current_step = 0
        return self.state

    def transit(self, x, u):
        a = int(np.argmax(u))
        r = _device_rewards(np.asarray(self.means, np.float64)[None], [a], self.var, _TYPES[self.type],
                            self._stream)[0]
        return self.state.copy(), r

    def step(self, action):
        if self.current_step >= self.H:
            raise ValueError("Episode has already ended")
        _, r = self.transit(self.state, action)
        self.current_step += 1
        done = self.current_step >= self.H
        return self.state.copy(), r, done, {}

    def deploy_eval(self, ctrl):
        tmp = self.var
        self.var = 0.0
        res = self.deploy(ctrl)
        self.var = tmp
        return res


class BanditEnvVec(BaseEnv):
    """Vectorized bandit environment (envs/bandit_env.py:85-153): the N tasks' means
    live on the device as one (N, A) fp64 tensor; ``step`` is one kernel launch."""

    def __init__(self, envs):
        self._envs = envs
        self._num_envs = len(envs)
        self.dx = envs[0].dx
        self.du = envs[0].du
        self._means_d = None
        self._stream = _Stream()
        # optional injected draws: callable(step counter) -> (N,) standard normals (or uniforms,
        # bernoulli): the np.random.normal of BanditEnv.transit per env; default: Philox
        self.noise = None

    # ------------------------------------------------------------------ device state
    @property
    def means_device(self):
        if self._means_d is None:
            m = np.stack([np.asarray(e.means, np.float64) for e in self._envs])
            self._means_d = torch.from_numpy(m).to(dpt_hip.device())
        return self._means_d

    def _common(self, attr):
        vals = {getattr(e, attr) for e in self._envs}
        if len(vals) != 1:
            raise ValueError(f"BanditEnvVec: all envs must share `{attr}` (got {sorted(vals)})")
        return vals.pop()

    @property
    def var(self):
        return float(self._common("var"))

    @property
    def type_code(self):
        return _TYPES[self._common("type")]

    # ------------------------------------------------------------------ reference API
    def reset(self):
        return [env.reset() for env in self._envs]

    def step(self, actions):
        if any(env.current_step >= env.H for env in self._envs):
            raise ValueError("Episode has already ended")
        a = np.argmax(np.asarray(actions), axis=-1)
        rews = _device_rewards(self.means_device, a, self.var, self.type_code, self._stream, noise=self.noise)
        next_obs, dones = [], []
        for env in self._envs:
            env.current_step += 1
            next_obs.append(env.state.copy())
            dones.append(env.current_step >= env.H)
        return next_obs, list(rews), dones, {}

    @property
    def num_envs(self):
        return self._num_envs

    @property
    def envs(self):
        return self._envs

    def deploy_eval(self, ctrl):
        tmp = [env.var for env in self._envs]
        for env in self._envs:
            env.var = 0.0
        try:
            res = self.deploy(ctrl)
        finally:
            for env, var in zip(self._envs, tmp):
                env.var = var
        return res

    def deploy(self, ctrl):
        """envs/bandit_env.py:125-149 (one step per episode: H = 1)."""
        x = self.reset()
        xs, xps, us, rs = [], [], [], []
        done = False
        while not done:
            u = ctrl.act_numpy_vec(x)
            xs.append(x)
            us.append(u)
            x, r, done, _ = self.step(u)
            done = all(done)
            rs.append(r)
            xps.append(x)
        return np.concatenate(xs), np.concatenate(us), np.concatenate(xps), np.concatenate(rs)

    def get_arm_value(self, us):
        return np.array([np.sum(env.means * u) for env, u in zip(self._envs, us)])


class LinearBanditEnv(BanditEnv):
    """envs/bandit_env.py:158-197: means = arms @ theta (host numpy GEMV, as the reference)."""

    def __init__(self, theta, arms, H, var=0.0):
        self.theta = theta
        self.arms = arms
        means = arms @ theta
        super().__init__(means, H, var=var, type="uniform")
