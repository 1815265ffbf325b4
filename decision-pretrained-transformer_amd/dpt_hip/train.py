"""Training forward / backward through libdpt_hip (dpt_train_forward / dpt_train_backward).

``TransformerFunction`` is the autograd node of ``models.net.Transformer.forward`` when autograd
needs it (train.py:286-331: ``loss.backward()`` then ``AdamW.step()``) and the forward of models
whose width the fused kernels are not built for (any ``n_embd``).  The parameters enter in the
packed blob order of include/dpt_hip.h; the gradients come back in that order and are mapped to
the reference's parameter shapes (nn.Linear weights are stored [out][in] by torch and [in][out]
in the blob).  Everything runs on the device; the library owns no memory here (the workspace
holding the forward's saved activations is a torch tensor kept on the autograd context).
"""
import ctypes

import torch

from . import _lib
from . import _p, _stream, device

GRAD_BACKWARD = "dpt_train_backward"


def param_list(model):
    """The Transformer's parameters in blob order (pack_weights): embed_transition, wpe, the
    blocks' [ln_1, c_attn, c_proj, ln_2, c_fc, mlp.c_proj] weight/bias pairs, ln_f, pred_actions."""
    t = model.transformer
    ps = [model.embed_transition.weight, model.embed_transition.bias, t.wpe.weight]
    for blk in t.h:
        ps += [blk.ln_1.weight, blk.ln_1.bias, blk.attn.c_attn.weight, blk.attn.c_attn.bias,
               blk.attn.c_proj.weight, blk.attn.c_proj.bias, blk.ln_2.weight, blk.ln_2.bias,
               blk.mlp.c_fc.weight, blk.mlp.c_fc.bias, blk.mlp.c_proj.weight, blk.mlp.c_proj.bias]
    ps += [t.ln_f.weight, t.ln_f.bias, model.pred_actions.weight, model.pred_actions.bias]
    return ps


def pack_params(params, dev=None):
    """Flatten the parameters (blob order) into one fp32 vector on ``dev`` (default: the
    parameters' own device).  The nn.Linear weights (the first and the second-to-last
    parameter) are stored [out][in] by torch and [in][out] in the blob.  Called on every
    training forward, so the common case (fp32, already on ``dev``) is one C++ flatten plus
    the two transposed copies."""
    n = len(params)
    dev = dev or params[0].device
    with torch.no_grad():
        if all(p.dtype == torch.float32 and p.device == dev for p in params):
            blob = torch._C._nn.flatten_dense_tensors([p.detach() for p in params])
        else:
            blob = torch.cat([p.detach().to(device=dev, dtype=torch.float32).reshape(-1) for p in params])
        off = 0
        for i, p in enumerate(params):
            k = p.numel()
            if i == 0 or i == n - 2:
                blob[off:off + k].view(p.shape[1], p.shape[0]).copy_(p.detach().t())
            off += k
    return blob


def _on_device(*tensors):
    """Every pointer handed to the library must be device memory (a host pointer would fault)."""
    for t in tensors:
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
            raise ValueError("dpt_hip.train: expected contiguous fp32 device tensors")


def unpack_grads(dblob, params):
    """Split a gradient blob into per-parameter gradients shaped like ``params`` (views of the
    blob; the two nn.Linear weights come back transposed to torch's [out][in])."""
    return _unpack(dblob, [p.shape for p in params], [p.dtype for p in params])


_META = {}


def _unpack(dblob, shapes, dtypes):
    key = tuple(shapes)
    metas = _META.get(key)
    if metas is None:  # shape templates for the C++ unflatten (no storage)
        metas = _META[key] = [torch.empty(sh, device="meta") for sh in shapes]
    total = sum(m.numel() for m in metas)
    if total != dblob.numel():
        raise ValueError(f"gradient blob {dblob.numel()} != parameters {total}")
    out = list(torch._C._nn.unflatten_dense_tensors(dblob, metas))
    n = len(shapes)
    off = 0
    for i, sh in enumerate(shapes):
        k = metas[i].numel()
        if i == 0 or i == n - 2:
            out[i] = dblob[off:off + k].view(sh[1], sh[0]).t()
        off += k
    return [g if dt == g.dtype else g.to(dt) for g, dt in zip(out, dtypes)]


FORWARD_ONLY = _lib.TRAIN_FORWARD_ONLY  # inference workspace, no backward


def desc(n_layer, n_embd, state_dim, action_dim, n_positions, batch, window, flags=0):
    return _lib.TrainDesc(n_layer, n_embd, state_dim, action_dim, n_positions, batch, window, flags)


def _numel(fn, d):
    n = ctypes.c_int64()
    _lib.call(fn, ctypes.byref(d), ctypes.byref(n))
    return n.value


def forward(d, blob, tokens):
    """preds (batch, window, A) at every position + the workspace the backward needs."""
    dev = device()
    _on_device(blob, tokens)
    if tokens.shape != (d.batch, d.window, 2 * d.state_dim + d.action_dim + 1):
        raise ValueError(f"tokens {tuple(tokens.shape)} do not match the description")
    ws = torch.empty(_numel("dpt_train_workspace_numel", d), dtype=torch.float32, device=dev)
    preds = torch.empty((d.batch, d.window, d.action_dim), dtype=torch.float32, device=dev)
    _lib.call("dpt_train_forward", ctypes.byref(d), _p(blob), _p(tokens), _p(ws), _p(preds), _stream())
    return preds, ws


def backward(d, blob, tokens, ws, dpreds):
    """dL/dblob (packed order) from dL/dpreds (batch, window, A)."""
    dblob = torch.empty(_numel("dpt_train_blob_numel", d), dtype=torch.float32, device=blob.device)
    dp = dpreds.to(torch.float32).contiguous()
    _on_device(blob, tokens, ws, dp)
    if dp.shape != (d.batch, d.window, d.action_dim):
        raise ValueError(f"dpreds {tuple(dp.shape)} do not match the description")
    _lib.call(GRAD_BACKWARD, ctypes.byref(d), _p(blob), _p(tokens), _p(ws), _p(dp), _p(dblob), _stream())
    return dblob


class TransformerFunction(torch.autograd.Function):
    """preds (B, T, A) = Transformer(tokens) at every position, with the HIP backward."""

    @staticmethod
    def forward(ctx, tokens, dims, *params):
        # dims[7] (optional) = FORWARD_ONLY when the caller runs without autograd (no_grad, or
        # no parameter requires grad): the forward-only workspace (one layer's activations, no
        # attention probabilities, no backward scratch) -- and nothing saved for a backward
        flags = dims[7] if len(dims) > 7 else 0
        need = any(ctx.needs_input_grad[2:]) and not flags & FORWARD_ONLY
        d = desc(*dims[:7], flags=0 if need else FORWARD_ONLY)
        dev = device()
        blob = pack_params(params, dev)
        if blob.numel() != _numel("dpt_train_blob_numel", d):
            raise ValueError("parameter shapes do not match the model description")
        tok = tokens.to(device=dev, dtype=torch.float32).contiguous()
        preds, ws = forward(d, blob, tok)
        if need:
            ctx.d, ctx.blob, ctx.tok, ctx.ws = d, blob, tok, ws
            ctx.params_meta = ([p.shape for p in params], [p.dtype for p in params], [p.device for p in params])
        # forward-only requested although a parameter requires grad: nothing is saved, so a
        # backward through this node must say so (not the retain_graph message below)
        ctx.forward_only = bool(flags & FORWARD_ONLY) and any(ctx.needs_input_grad[2:])
        return preds

    @staticmethod
    def backward(ctx, dpreds):
        if getattr(ctx, "forward_only", False):
            raise RuntimeError("dpt_hip.train: this forward ran with FORWARD_ONLY (no activations saved) while "
                               "parameters require grad; drop the FORWARD_ONLY flag to train through it")
        if getattr(ctx, "ws", None) is None:
            raise RuntimeError("dpt_hip.train: the saved activations were released by the first backward; "
                               "a second backward through the same graph (retain_graph=True) is not supported")
        dblob = backward(ctx.d, ctx.blob, ctx.tok, ctx.ws, dpreds)
        shapes, dtypes, devs = ctx.params_meta
        grads = [g if g.device == dv else g.to(dv) for g, dv in zip(_unpack(dblob, shapes, dtypes), devs)]
        ctx.ws = None  # the saved activations are not needed again
        return (None, None) + tuple(g if need else None for g, need in zip(grads, ctx.needs_input_grad[2:]))
