"""DarkRoom environments — drop-in for the reference envs/darkroom_env.py.

Transitions, rewards and the expert action are gfx950 integer kernels
(``dpt_darkroom_step`` / ``dpt_darkroom_opt_action``), bit-exact to the
reference on the exhaustive state x action x goal (x 120 permutations) table.
State/action sampling for data collection keeps numpy's draws (reference
collect_data.py uses the global numpy RNG).
"""
import itertools

import numpy as np
import torch

import dpt_hip
from envs.base_env import BaseEnv, spaces

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")

PERMUTATIONS = np.array(list(itertools.permutations(range(5))), dtype=np.int32)  # darkroom_env.py:97-99


class DarkroomEnv(BaseEnv):
    def __init__(self, dim, goal, horizon):
        self.dim = dim
        self.goal = np.array(goal)
        self.horizon = horizon
        self.state_dim = 2
        self.action_dim = 5
        self.observation_space = spaces.Box(low=0, high=dim - 1, shape=(self.state_dim,))
        self.action_space = spaces.Discrete(self.action_dim)
        self.perm = None

    def sample_state(self):
        return np.random.randint(0, self.dim, 2)

    def sample_action(self):
        i = np.random.randint(0, 5)
        a = np.zeros(self.action_space.n)
        a[i] = 1
        return a

    def reset(self):
        self.current_step = 0
        self.state = np.array([0, 0])
        return self.state

    def _perm_row(self):
        return None if self.perm is None else np.asarray(self.perm, np.int32)[None]

    def transit(self, state, action):
        a = int(np.argmax(action))
        assert a in np.arange(self.action_space.n)
        ns, r = dpt_hip.darkroom_step(np.asarray(state, np.int32)[None], [a],
                                      np.asarray(self.goal, np.int32)[None], self._perm_row(), self.dim)
        return ns.cpu().numpy()[0].astype(np.int64), int(r.cpu().numpy()[0])

    def step(self, action):
        if self.current_step >= self.horizon:
            raise ValueError("Episode has already ended")
        self.state, r = self.transit(self.state, action)
        self.current_step += 1
        done = self.current_step >= self.horizon
        return self.state.copy(), r, done, {}

    def get_obs(self):
        return self.state.copy()

    def opt_action(self, state):
        a = dpt_hip.darkroom_opt_action(np.asarray(state, np.int32)[None], np.asarray(self.goal, np.int32)[None],
                                        self._perm_row())
        zeros = np.zeros(self.action_space.n)
        zeros[int(a.cpu().numpy()[0])] = 1
        return zeros


class DarkroomEnvPermuted(DarkroomEnv):
    """Goal fixed at the bottom-right corner; actions permuted (envs/darkroom_env.py:85-111)."""

    def __init__(self, dim, perm_index, H):
        goal = np.array([dim - 1, dim - 1])
        super().__init__(dim, goal, H)
        self.perm_index = perm_index
        assert perm_index < 120
        self.perm = tuple(int(x) for x in PERMUTATIONS[perm_index])


class DarkroomEnvVec(BaseEnv):
    """Vectorized DarkRoom (envs/darkroom_env.py:114-175); goals / permutations live on the device."""

    def __init__(self, envs, first_task=0):
        self._envs = envs
        self._num_envs = len(envs)
        self._goals_d = None
        self._perms_d = None
        # global id of envs[0] when the tasks are sharded over ranks: the fused rollout
        # keys its Philox draws by global task id (dpt_hip.distributed)
        self.first_task = int(first_task)

    @property
    def goals_device(self):
        if self._goals_d is None:
            self._goals_d = torch.from_numpy(np.stack([np.asarray(e.goal, np.int32) for e in self._envs])).to(
                dpt_hip.device())
        return self._goals_d

    @property
    def perms_device(self):
        if self._perms_d is None and any(e.perm is not None for e in self._envs):
            rows = [np.asarray(e.perm if e.perm is not None else range(5), np.int32) for e in self._envs]
            self._perms_d = torch.from_numpy(np.stack(rows)).to(dpt_hip.device())
        return self._perms_d

    @property
    def dim(self):
        dims = {e.dim for e in self._envs}
        if len(dims) != 1:
            raise ValueError("DarkroomEnvVec: envs must share `dim`")
        return dims.pop()

    def reset(self):
        return [env.reset() for env in self._envs]

    def step(self, actions):
        if any(env.current_step >= env.horizon for env in self._envs):
            raise ValueError("Episode has already ended")
        a = np.argmax(np.asarray(actions), axis=-1)
        st = np.stack([np.asarray(e.state, np.int32) for e in self._envs])
        ns, r = dpt_hip.darkroom_step(st, a, self.goals_device, self.perms_device, self.dim)
        ns = ns.cpu().numpy().astype(np.int64)
        r = r.cpu().numpy()
        next_obs, rews, dones = [], [], []
        for i, env in enumerate(self._envs):
            env.state = ns[i]
            env.current_step += 1
            next_obs.append(ns[i].copy())
            rews.append(int(r[i]))
            dones.append(env.current_step >= env.horizon)
        return next_obs, rews, dones, {}

    @property
    def num_envs(self):
        return self._num_envs

    @property
    def envs(self):
        return self._envs

    @property
    def state_dim(self):
        return self._envs[0].state_dim

    @property
    def action_dim(self):
        return self._envs[0].action_dim

    def deploy(self, ctrl):
        """envs/darkroom_env.py:151-175: horizon steps, stacked along axis 1."""
        ob = self.reset()
        obs, acts, next_obs, rews = [], [], [], []
        done = False
        while not done:
            act = ctrl.act(ob)
            obs.append(ob)
            acts.append(act)
            ob, rew, done, _ = self.step(act)
            done = all(done)
            rews.append(rew)
            next_obs.append(ob)
        return (np.stack(obs, axis=1), np.stack(acts, axis=1), np.stack(next_obs, axis=1),
                np.stack(rews, axis=1))
