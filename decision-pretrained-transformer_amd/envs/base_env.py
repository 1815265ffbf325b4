"""BaseEnv — drop-in for the reference envs/base_env.py:8-48.

The reference derives from gym.Env only for its name; gym is not a dependency
here.  ``spaces`` provides the two attribute holders the reference touches
(gym.spaces.Box / Discrete: shape, low, high, n).
"""
import numpy as np
import torch

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


class Box:
    def __init__(self, low, high, shape):
        self.low, self.high, self.shape = low, high, tuple(shape)


class Discrete:
    def __init__(self, n):
        self.n = n


class spaces:  # noqa: N801 - mirrors gym.spaces
    Box = Box
    Discrete = Discrete


class BaseEnv:
    def reset(self):
        raise NotImplementedError

    def transit(self, state, action):
        raise NotImplementedError

    def step(self, action):
        raise NotImplementedError

    def render(self, mode="human"):
        pass

    def deploy_eval(self, ctrl):
        return self.deploy(ctrl)

    def deploy(self, ctrl):
        """Single-episode loop (envs/base_env.py:24-48): act -> step until done."""
        ob = self.reset()
        obs, acts, next_obs, rews = [], [], [], []
        done = False
        while not done:
            act = ctrl.act(ob)
            obs.append(ob)
            acts.append(act)
            ob, rew, done, _ = self.step(act)
            rews.append(rew)
            next_obs.append(ob)
        return np.array(obs), np.array(acts), np.array(next_obs), np.array(rews)
