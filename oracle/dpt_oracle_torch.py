"""Float64 torch restatement of the reference Transformer forward, for gradients.

TEST INFRASTRUCTURE ONLY (like the rest of oracle/): tests/ use it as the checker of the
HIP training kernels (dpt_train_forward / dpt_train_backward); nothing in the product imports
it.  It is oracle/dpt_oracle.py's gpt2_hidden / transformer_forward written with torch ops so
that autograd gives the exact float64 gradient of train.py's loss:

* models/net.py:41-60 -- token packing, embed_transition, GPT2Model(inputs_embeds), pred_actions,
  preds[:, 1:] (test=False);
* transformers GPT2 block (modeling_gpt2.py:262-309): h += c_proj(softmax(QK^T/sqrt(E) + causal) V),
  h += W2 gelu_new(W1 ln_2(h) + b1) + b2, one head (net.py:29), LayerNorm eps 1e-5, then ln_f;
* train.py:296-309 -- CrossEntropyLoss(reduction='sum') of the preds against the optimal action
  repeated over the positions.

Pinned by tests/test_oracle_golden.py against tests/golden/train_grads.npz (gradients recorded
from the reference itself in float64).
"""
import math

import torch


def state_dict_params(w, n_layer, dtype=torch.float64):
    """Leaf tensors (requires_grad) of a reference state_dict, keyed by the reference names."""
    return {k: torch.tensor(v, dtype=dtype, requires_grad=True) for k, v in w.items() if not k.endswith("wte.weight")}


def gelu_new(x):
    """transformers/activations.py:65 NewGELUActivation."""
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def pack(batch, state_dim, action_dim, dtype=torch.float64):
    """models/net.py:42-54: [query | 0_A | 0_sd | 0] then [s, a, s', r] per transition."""
    t = lambda k: torch.as_tensor(batch[k], dtype=dtype)  # noqa: E731
    q = t("query_states")[:, None, :]
    z = torch.zeros((q.shape[0], 1, action_dim + state_dim + 1), dtype=dtype)
    first = torch.cat([q, z], dim=2)
    ctx = torch.cat([t("context_states"), t("context_actions"), t("context_next_states"),
                     t("context_rewards").reshape(q.shape[0], -1, 1)], dim=2)
    return torch.cat([first, ctx], dim=1)


def forward(P, seq, n_layer, drop=None):
    """Transformer.forward (models/net.py:52-60) on packed tokens -> preds at every position.

    drop (training-mode dropout, GPT2Config embd/attn/resid_pdrop, net.py:30-32): a callable
    site -> keep factors (0 or 1 / (1 - p)) shaped like the site's tensor, the masks the
    kernels drew (the caller regenerates them; include/dpt_hip.h dpt_train_desc names the sites):
    0 the embedding sum, 1 + 3 l the attention probabilities, 2 + 3 l / 3 + 3 l the c_proj /
    mlp.c_proj outputs before their residual adds (transformers GPT2Model / GPT2Attention /
    GPT2MLP dropout placement)."""
    E = P["transformer.wpe.weight"].shape[1]
    T = seq.shape[1]
    keep = (lambda site, v: v) if drop is None else (lambda site, v: v * drop(site))  # noqa: E731
    x = keep(0, seq @ P["embed_transition.weight"].t() + P["embed_transition.bias"] + P["transformer.wpe.weight"][:T])
    mask = torch.triu(torch.ones((T, T), dtype=torch.bool), 1)
    ln = lambda v, g, b: torch.nn.functional.layer_norm(v, (E,), g, b, 1e-5)  # noqa: E731
    for i in range(n_layer):
        p = f"transformer.h.{i}."
        h = ln(x, P[p + "ln_1.weight"], P[p + "ln_1.bias"])
        qkv = h @ P[p + "attn.c_attn.weight"] + P[p + "attn.c_attn.bias"]
        q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
        s = (q @ k.transpose(1, 2)) / math.sqrt(E)
        a = keep(1 + 3 * i, torch.softmax(s.masked_fill(mask, float("-inf")), dim=-1)) @ v
        x = x + keep(2 + 3 * i, a @ P[p + "attn.c_proj.weight"] + P[p + "attn.c_proj.bias"])
        h = ln(x, P[p + "ln_2.weight"], P[p + "ln_2.bias"])
        x = x + keep(3 + 3 * i, gelu_new(h @ P[p + "mlp.c_fc.weight"] + P[p + "mlp.c_fc.bias"])
                     @ P[p + "mlp.c_proj.weight"] + P[p + "mlp.c_proj.bias"])
    x = ln(x, P["transformer.ln_f.weight"], P["transformer.ln_f.bias"])
    return x @ P["pred_actions.weight"].t() + P["pred_actions.bias"]


def train_loss(P, batch, n_layer, state_dim, action_dim, drop=None):
    """train.py:296-309: CrossEntropyLoss(sum) of preds[:, 1:] against the repeated optimal action."""
    preds = forward(P, pack(batch, state_dim, action_dim), n_layer, drop)[:, 1:, :]
    true = torch.as_tensor(batch["optimal_actions"], dtype=preds.dtype)[:, None, :].expand_as(preds)
    loss = torch.nn.functional.cross_entropy(preds.reshape(-1, action_dim), true.reshape(-1, action_dim),
                                             reduction="sum")
    return loss, preds


def grads(w, batch, n_layer, state_dim, action_dim, drop=None):
    """(loss, preds, {name: float64 gradient}) of train.py's loss at the weights ``w``."""
    P = state_dict_params(w, n_layer)
    loss, preds = train_loss(P, batch, n_layer, state_dim, action_dim, drop)
    loss.backward()
    return loss.item(), preds.detach().numpy(), {k: v.grad.numpy() for k, v in P.items()}
