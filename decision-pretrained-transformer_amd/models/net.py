"""DPT policy model — drop-in for the reference models/net.py:9-60 ``Transformer``.

Same constructor config dict, same parameter names (so reference checkpoints
load with ``load_state_dict`` unchanged), same ``forward(batch) -> logits``
contract.  The GPT-2 stack is NOT transformers.GPT2Model: parameters live in a
plain module tree with GPT-2's names, and ``forward`` runs the hand-written
gfx950 kernels of libdpt_hip.so (dpt_forward_window).  ``n_head`` is accepted
and ignored exactly as the reference ignores it (net.py:29 forces one head).
"""
import math
import random

import numpy as np
import torch
import torch.nn as nn

import dpt_hip

# models/net.py:4 calls transformers.set_seed(0) at import time; keep that side
# effect so scripts that rely on it (random init without a checkpoint) behave alike.
random.seed(0)
np.random.seed(0)
torch.manual_seed(0)

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")

VOCAB = 50257  # GPT2Config default; wte is unused with inputs_embeds but is part of the state_dict


class Conv1D(nn.Module):
    """GPT-2 Conv1D: y = x @ W + b with W stored [in][out] (transformers pytorch_utils.Conv1D)."""

    def __init__(self, nf, nx):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(nx, nf))
        self.bias = nn.Parameter(torch.zeros(nf))


class _Attn(nn.Module):
    def __init__(self, E):
        super().__init__()
        self.c_attn = Conv1D(3 * E, E)
        self.c_proj = Conv1D(E, E)


class _MLP(nn.Module):
    def __init__(self, E):
        super().__init__()
        self.c_fc = Conv1D(4 * E, E)
        self.c_proj = Conv1D(E, 4 * E)


class _Block(nn.Module):
    def __init__(self, E):
        super().__init__()
        self.ln_1 = nn.LayerNorm(E, eps=1e-5)
        self.attn = _Attn(E)
        self.ln_2 = nn.LayerNorm(E, eps=1e-5)
        self.mlp = _MLP(E)


class GPT2Stack(nn.Module):
    """Parameter container with GPT2Model's names (wte, wpe, h.{i}.*, ln_f)."""

    def __init__(self, n_positions, E, n_layer):
        super().__init__()
        self.wte = nn.Embedding(VOCAB, E)
        self.wpe = nn.Embedding(n_positions, E)
        self.h = nn.ModuleList([_Block(E) for _ in range(n_layer)])
        self.ln_f = nn.LayerNorm(E, eps=1e-5)


def _dropout_seed():
    """A fresh Philox seed for one dropout call, from the CUDA generator as the reference's dropout
    draws its masks: the seed mixes the generator's initial seed with its Philox offset, and the
    offset advances as a dropout kernel would advance it.  torch.manual_seed (which resets the
    offset) reproduces a run, no device synchronisation is needed, and the CPU stream -- the
    DataLoader shuffle (train.py:203,249) and the per-item context permutation (dataset.py:85) --
    never sees dropout, as in the reference."""
    dev = dpt_hip.device()
    g = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
    off = g.get_offset()
    g.set_offset(off + 4)
    z = (g.initial_seed() * 0x9E3779B97F4A7C15 + off + 1) & 0xFFFFFFFFFFFFFFFF  # splitmix64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (z ^ (z >> 31)) & ((1 << 62) - 1)


class Transformer(nn.Module):
    """Transformer class (models/net.py:9-60)."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.test = config["test"]
        self.horizon = self.config["horizon"]
        self.n_embd = self.config["n_embd"]
        self.n_layer = self.config["n_layer"]
        self.n_head = self.config["n_head"]
        self.state_dim = self.config["state_dim"]
        self.action_dim = self.config["action_dim"]
        self.dropout = self.config["dropout"]
        self.n_positions = 4 * (1 + self.horizon)

        self.transformer = GPT2Stack(self.n_positions, self.n_embd, self.n_layer)
        self.embed_transition = nn.Linear(2 * self.state_dim + self.action_dim + 1, self.n_embd)
        self.pred_actions = nn.Linear(self.n_embd, self.action_dim)
        self._init_gpt2()
        self._register_load_state_dict_pre_hook(self._drop_legacy_buffers)
        self._dev_model = None
        self._dev_sig = None

    # GPT2PreTrainedModel._init_weights: N(0, 0.02) weights, zero biases, LN (1, 0),
    # c_proj weights N(0, 0.02 / sqrt(2 * n_layer)).
    def _init_gpt2(self):
        std = 0.02
        with torch.no_grad():
            for mod in self.modules():
                if isinstance(mod, (nn.Linear, Conv1D)):
                    mod.weight.normal_(0.0, std)
                    mod.bias.zero_()
                elif isinstance(mod, nn.Embedding):
                    mod.weight.normal_(0.0, std)
                elif isinstance(mod, nn.LayerNorm):
                    mod.weight.fill_(1.0)
                    mod.bias.zero_()
            for blk in self.transformer.h:
                blk.attn.c_proj.weight.normal_(0.0, std / math.sqrt(2 * self.n_layer))
                blk.mlp.c_proj.weight.normal_(0.0, std / math.sqrt(2 * self.n_layer))

    @staticmethod
    def _drop_legacy_buffers(state_dict, prefix, *args):
        # transformers 4.5.1 (requirements.txt:1) saved the causal-mask buffers
        # attn.bias / attn.masked_bias in GPT-2 checkpoints; they carry no weights.
        for k in list(state_dict.keys()):
            if k.startswith(prefix) and (k.endswith(".attn.masked_bias") or k.endswith(".attn.bias")):
                del state_dict[k]

    # ------------------------------------------------------------------ device weights
    def device_model(self):
        """The packed-weight handle on the GPU, rebuilt whenever a parameter changed."""
        sig = tuple((id(p), p._version, p.data_ptr()) for p in self.parameters())
        if self._dev_model is None or sig != self._dev_sig:
            if self.n_embd != dpt_hip.E:
                raise NotImplementedError(f"n_embd={self.n_embd}: only {dpt_hip.E} is built")
            self._dev_model = dpt_hip.DeviceModel(self.state_dict(), self.n_layer, self.state_dim,
                                                  self.action_dim, self.n_positions, self.n_embd)
            self._dev_sig = sig
        return self._dev_model

    def _tokens(self, x):
        """The packed sequences of models/net.py:42-54: [query | 0_A | 0_sd | 0] then the context
        transitions [s, a, s', r] -> (B, T, 2 sd + A + 1) fp32 on the device."""
        dev = dpt_hip.device()
        q = x["query_states"].to(dev, torch.float32)
        B = q.shape[0]
        first = torch.cat([q, torch.zeros((B, self.action_dim + self.state_dim + 1), device=dev)], dim=1)[:, None]
        cs = x.get("context_states")
        if cs is None or cs.shape[1] == 0:
            return first.contiguous()
        C = cs.shape[1]
        ctx = torch.cat([cs.to(dev, torch.float32), x["context_actions"].to(dev, torch.float32),
                         x["context_next_states"].to(dev, torch.float32),
                         x["context_rewards"].to(dev, torch.float32).reshape(B, C, 1)], dim=2)
        return torch.cat([first, ctx], dim=1).contiguous()

    def _forward_generic(self, x):
        """The generic-width path (dpt_hip.train): preds at every position from
        dpt_train_forward, differentiable through dpt_train_backward (the HIP backward of the
        whole model).  Used when autograd needs the graph and for widths other than 32."""
        from dpt_hip import train as tr
        tok = self._tokens(x)
        grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        p, seed = 0.0, 0
        if self.training and self.dropout > 0:  # fresh masks per call (_dropout_seed)
            p, seed = float(self.dropout), _dropout_seed()
        # inference in test mode reads the last position only (LAST_ONLY: the last block for that row alone)
        flags = 0 if grad else tr.FORWARD_ONLY | (tr.LAST_ONLY if self.test and p == 0.0 else 0)
        dims = (self.n_layer, self.n_embd, self.state_dim, self.action_dim, self.n_positions, tok.shape[0],
                tok.shape[1], flags, p, seed)
        preds = tr.TransformerFunction.apply(tok, dims, *tr.param_list(self))
        return preds[:, -1, :] if self.test else preds[:, 1:, :]

    def forward(self, x):
        """models/net.py:41-60: pack [query | context] -> embed -> GPT-2 -> head;
        last position (test) or positions 1.. (train).

        When autograd would differentiate the call (training mode, grad enabled, trainable
        parameters: train.py:286-331) the forward and backward run through the HIP training
        kernels (dpt_hip.train.TransformerFunction): ``loss.backward()`` fills every
        parameter's ``.grad`` and the reference's AdamW step works unchanged.  Inference
        (eval.py:152 ``model.eval()``; train.py:265-278's test loss under ``torch.no_grad()``)
        takes the fused kernels at width 32 and the generic kernels at other widths.

        Dropout: the reference's GPT2Config applies embd/attn/resid dropout with p = ``dropout``
        (models/net.py:30-32) in training mode -- with or without grad (train.py:265-278's test
        loss runs in training mode).  Such calls take the training kernels with dropout: masks
        from Philox keyed by a seed taken per call from the CUDA generator (_dropout_seed;
        include/dpt_hip.h dpt_train_desc), the same distribution as torch's dropout, not its
        random stream."""
        if (self.training and (self.dropout > 0 or (torch.is_grad_enabled()
                                                    and any(p.requires_grad for p in self.parameters())))) \
                or self.n_embd != dpt_hip.E:
            return self._forward_generic(x)
        dm = self.device_model()
        query = x["query_states"]
        cs = x.get("context_states")
        C = 0 if cs is None else int(cs.shape[1])
        if C == 0:
            if not self.test:
                return torch.zeros((query.shape[0], 0, self.action_dim), device=dpt_hip.device())
            return dm.forward_window(query)
        cr = x["context_rewards"]
        return dm.forward_window(query, cs, x["context_actions"], x["context_next_states"],
                                 cr.reshape(cr.shape[0], C), out_mode=0 if self.test else 1)
