"""GPUBanditEnv — drop-in for the reference envs/gpu_bandit_env.py:8-82.

N tasks on one device; fp32 means as in the reference (torch.rand /
Beta(1,1)), rewards from the gfx950 ``dpt_bandit_step`` kernel in its fp32
mode (r = m + g*var, two fp32 roundings: the torch expression of
gpu_bandit_env.py:58-59) or Bernoulli (u < m, torch.bernoulli).  Unlike the
reference, ``deploy`` works for n_envs > 1 (the reference loops
``while not done`` on a bool tensor, base_env.py:32, and raises).
"""
import torch

import dpt_hip
from envs.base_env import BaseEnv, spaces

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


class GPUBanditEnv(BaseEnv):
    def __init__(self, dims, n_envs, H, var=0.0, type="uniform", device=None):
        self.dims = dims
        self.dim = dims
        self.n_envs = n_envs
        self._device = device if device is not None else dpt_hip.device()
        if type == "uniform":
            self.means = torch.rand((n_envs, dims), device=self._device)
        elif type == "bernoulli":
            self.means = torch.distributions.Beta(1, 1).sample((n_envs, dims)).to(self._device)
        else:
            raise NotImplementedError
        opt_a_index = torch.argmax(self.means, dim=1)
        self.opt_a_index = opt_a_index
        self.opt_a = torch.zeros((n_envs, dims), device=self._device)
        self.opt_a[torch.arange(n_envs, device=self._device), opt_a_index] = 1.0
        self.H_context = H
        self.H = H
        self.var = var
        self.dx = 1
        self.du = dims
        self.topk = False
        self.type = type
        self.observation_space = spaces.Box(low=1, high=1, shape=(1,))
        self.action_space = spaces.Box(low=0, high=1, shape=(self.dims,))
        self.state = torch.ones((n_envs, 1), device=self._device)
        self.current_step = torch.zeros(n_envs, device=self._device)
        self._seed = None
        self._counter = 0
        # optional injected draws: callable(step counter) -> (n_envs,) standard normals (the
        # torch.randn of gpu_bandit_env.py:58) or, bernoulli, uniforms; default: Philox
        self.noise = None

    def get_arm_value(self, actions):
        return torch.sum(self.means * actions, dim=1)

    def reset(self):
        self.current_step = torch.zeros(self.n_envs, device=self._device)
        return self.state.detach()

    def transit(self, x, us):
        us = us.to(self._device) if us.device != self._device else us
        a = torch.argmax(us, dim=1).to(torch.int32)
        if self._seed is None:
            self._seed = dpt_hip.next_seed()
        code = (dpt_hip.BANDIT_GAUSSIAN if self.type == "uniform" else dpt_hip.BANDIT_BERNOULLI)
        g = None if self.noise is None else torch.as_tensor(self.noise(self._counter), dtype=torch.float64)
        r, _ = dpt_hip.bandit_step(self.means.double(), a, self.var, code | dpt_hip.BANDIT_F32, noise=g,
                                   seed=self._seed, counter=self._counter)
        self._counter += 1
        return self.state.detach(), r.float()

    def step(self, actions):
        if self.current_step.max() >= self.H:
            raise ValueError("Episode has already ended")
        _, r = self.transit(self.state, actions)
        self.current_step += 1
        done = self.current_step >= self.H
        return self.state.detach(), r.detach(), done, {}

    def deploy_eval(self, ctrl):
        tmp = self.var
        self.var = 0.0
        try:
            return self.deploy(ctrl)
        finally:
            self.var = tmp

    def deploy(self, ctrl):
        ob = self.reset()
        obs, acts, next_obs, rews = [], [], [], []
        done = torch.zeros(self.n_envs, dtype=torch.bool, device=self._device)
        while not bool(done.all()):
            act = ctrl.act(ob)
            obs.append(ob)
            acts.append(act)
            ob, rew, done, _ = self.step(act)
            rews.append(rew)
            next_obs.append(ob)
        return torch.stack(obs, 1), torch.stack(acts, 1), torch.stack(next_obs, 1), torch.stack(rews, 1)
