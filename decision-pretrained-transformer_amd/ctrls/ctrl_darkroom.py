"""DarkRoom controllers — drop-in for the reference ctrls/ctrl_darkroom.py."""
import numpy as np
import torch

import dpt_hip
from ctrls.ctrl_bandit import Controller, _SelectStream

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


class DarkroomOptPolicy(Controller):
    """Expert policy (ctrls/ctrl_darkroom.py:10-20)."""

    def __init__(self, env):
        super().__init__()
        self.env = env
        self.goal = env.goal

    def reset(self):
        return

    def act(self, state):
        return self.env.opt_action(state)


class DarkroomTransformerController(Controller):
    """DPT policy for DarkRoom (ctrls/ctrl_darkroom.py:23-66): query = current state,
    softmax(logits / temp) sampling with temp = 1, or argmax."""

    def __init__(self, model, batch_size=1, sample=False):
        self.model = model
        self.state_dim = model.config["state_dim"]
        self.action_dim = model.config["action_dim"]
        self.horizon = model.horizon
        self.zeros = torch.zeros(batch_size, self.state_dim ** 2 + self.action_dim + 1, device=dpt_hip.device())
        self.sample = sample
        self.temp = 1.0
        self.batch_size = batch_size
        self._stream = _SelectStream()
        self.uniforms = None

    def select(self, logits, first_task=0):
        """Device action indices for (B, A) logits (ctrl_darkroom.py:48-59).  Philox draws are
        keyed by the global task id (``first_task`` + row), as in the fused rollout, so a
        sharded env's tasks draw the same uniforms on any rank layout."""
        seed, ctr = self._stream.next()
        u = self.uniforms(ctr) if (self.sample and self.uniforms is not None) else None
        return dpt_hip.select_action(logits, self.sample, self.temp, uniforms=u, seed=seed, counter=ctr,
                                     first_task=first_task)

    def act(self, state):
        self.batch["zeros"] = self.zeros
        states = torch.as_tensor(np.array(state), dtype=torch.float32, device=dpt_hip.device())
        if self.batch_size == 1:
            states = states[None, :]
        self.batch["query_states"] = states
        idx = self.select(self.model(self.batch)).cpu().numpy()
        actions = np.zeros((self.batch_size, self.action_dim))
        actions[np.arange(self.batch_size), idx] = 1.0
        if self.batch_size == 1:
            actions = actions[0]
        return actions
