"""Host-side drop-in surface on CPU: filenames and CLI flags equal the reference's
(tests/golden/host_surface.json, recorded from the reference's utils.py / common_args.py)."""
import argparse
import json
import os

from conftest import GOLDEN


def surface():
    return json.load(open(os.path.join(GOLDEN, "host_surface.json")))


def test_filenames_match_reference():
    import utils
    for fn, args, expected in surface()["filenames"]:
        assert getattr(utils, fn)(*args) == expected, (fn, args)


def test_flag_defaults_match_reference():
    import common_args
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_train_args(p)
    common_args.add_eval_args(p)
    assert vars(p.parse_args(["--env", "bandit"])) == surface()["defaults"]


def test_run_scripts_parse():
    """The reference recipes' collect / eval command lines parse with our CLIs (run_bandit.sh:2,8)."""
    import common_args
    collect = "--env bandit --envs 100000 --H 500 --dim 5 --var 0.3 --cov 0.0 --envs_eval 200".split()
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    a = vars(p.parse_args(collect))
    assert a["H"] == 500 and a["envs_eval"] == 200
    ev = ("--env bandit --envs 100000 --H 500 --dim 5 --var 0.3 --cov 0.0 --lr 0.0001 --layer 4 --head 4 "
          "--shuffle --epoch 50 --n_eval 200 --seed 1").split()
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_eval_args(p)
    p.add_argument("--seed", type=int, default=0)
    a = vars(p.parse_args(ev))
    assert a["shuffle"] is True and a["layer"] == 4 and a["epoch"] == 50


def _tiny_transformer():
    from models.net import Transformer
    return Transformer(dict(horizon=4, state_dim=1, action_dim=5, n_layer=2, n_embd=32, n_head=1, dropout=0.0,
                            test=False))


def _tiny_batch():
    import torch
    return {"query_states": torch.ones(2, 1), "zeros": torch.zeros(2, 7), "context_states": torch.ones(2, 3, 1),
            "context_actions": torch.eye(5)[[0, 1, 2]].expand(2, 3, 5), "context_next_states": torch.ones(2, 3, 1),
            "context_rewards": torch.zeros(2, 3, 1)}


def test_training_forward_takes_the_hip_training_path():
    """train.py:286-331 (model in training mode, grad enabled) routes the forward through the HIP
    training kernels (dpt_hip.train.TransformerFunction, whose backward fills every parameter's
    .grad); on this CPU-only container that path refuses to run because there is no GPU."""
    import pytest
    m = _tiny_transformer()
    assert m.training
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m(_tiny_batch())


def test_train_blob_order_matches_pack_weights():
    """dpt_hip.train.pack_params (the device-side pack of the training path) lays the parameters
    out exactly as dpt_hip.pack_weights (the inference blob of include/dpt_hip.h), and
    unpack_grads inverts it shape for shape."""
    import torch
    import dpt_hip
    from dpt_hip import train as tr
    m = _tiny_transformer()
    ps = tr.param_list(m)
    sd = {k: v for k, v in m.state_dict().items() if not k.endswith("wte.weight")}
    assert torch.equal(tr.pack_params(ps), dpt_hip.pack_weights(sd, m.n_layer))
    assert len(ps) == len(sd) and sum(p.numel() for p in ps) == sum(v.numel() for v in sd.values())
    back = tr.unpack_grads(tr.pack_params(ps), ps)
    assert all(torch.equal(a, b) for a, b in zip(back, ps))


def test_training_mode_dropout_takes_the_training_kernels(monkeypatch):
    """GPT2Config applies dropout in training mode (models/net.py:30-32), with or without grad
    (train.py:265-278's test loss): such calls go to the training kernels (which implement it)
    with a fresh Philox seed per call (net._dropout_seed, from the CUDA generator: its
    seedability and that the CPU stream is untouched are GPU tests); eval mode ignores dropout."""
    import torch
    from dpt_hip import train as tr
    from models import net
    from models.net import Transformer
    m = Transformer(dict(horizon=4, state_dim=1, action_dim=5, n_layer=2, n_embd=32, n_head=1, dropout=0.1,
                         test=False))
    seen = []

    def fake_apply(tok, dims, *params):
        seen.append(dims)
        return torch.zeros((tok.shape[0], tok.shape[1], 5))
    monkeypatch.setattr(tr.TransformerFunction, "apply", fake_apply)
    monkeypatch.setattr(m, "_tokens", lambda x: torch.zeros((3, 9, 8)))
    seeds = iter([11, 12, 13])
    monkeypatch.setattr(net, "_dropout_seed", lambda: next(seeds))
    m(_tiny_batch())
    with torch.no_grad():
        m(_tiny_batch())
    m(_tiny_batch())
    assert [d[7] for d in seen] == [0, tr.FORWARD_ONLY, 0]
    assert all(abs(d[8] - 0.1) < 1e-12 for d in seen)
    assert [d[9] for d in seen] == [11, 12, 13]   # one seed per call
    m.eval()
    m.dropout = 0.1
    seen.clear()
    import pytest
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # eval mode: the fused inference path
        m(_tiny_batch())
    assert not seen


def test_train_desc_rejects_bad_dropout():
    """dpt_train_desc.dropout outside [0, 1) is an argument error (host-side check, no GPU)."""
    import ctypes
    import pytest
    from dpt_hip import _lib
    from dpt_hip import train as tr
    lib = _lib.load()
    n = ctypes.c_int64()
    for p in (1.0, -0.1, 1.5):
        d = tr.desc(2, 32, 1, 5, 40, 3, 9, dropout=p, seed=1)
        with pytest.raises(ValueError, match="dropout"):
            _lib.check(lib.dpt_train_blob_numel(ctypes.byref(d), ctypes.byref(n)))
    d = tr.desc(2, 32, 1, 5, 40, 3, 9, dropout=0.5, seed=1)
    _lib.check(lib.dpt_train_blob_numel(ctypes.byref(d), ctypes.byref(n)))
    assert n.value > 0


def test_generic_rollout_workspace_and_argument_checks():
    """dpt_rollout_bandit_generic_workspace_numel: the y cache [L][N][H][E], the folded attention
    weights [L][2E^2 + 2E] and the per-step rows (host-side, no GPU); a desc with dropout is rejected
    before any device work, and N = 0 is a no-op."""
    import ctypes
    import pytest
    from dpt_hip import _lib
    from dpt_hip import train as tr
    lib = _lib.load()
    L, E, A, N, H = 3, 48, 5, 10, 7
    d = tr.desc(L, E, 1, A, 4 * (1 + H), 1, 1)
    n = ctypes.c_int64()
    _lib.check(lib.dpt_rollout_bandit_generic_workspace_numel(ctypes.byref(d), N, H, ctypes.byref(n)))
    cache = L * N * H * E
    fold = L * (2 * E * E + 2 * E)
    rows = N * (4 * E + 2 + 3 * E + 4 * E + A + (2 + A + 1))  # x x2 y o, st, qkv, h, logits, token
    assert cache + fold + rows <= n.value <= cache + fold + rows + 4 * 13
    args = _lib.BanditRolloutArgs()
    args.N, args.H, args.A = 0, H, A
    _lib.check(lib.dpt_rollout_bandit_generic(ctypes.byref(d), ctypes.c_void_p(8), ctypes.byref(args), None))
    dd = tr.desc(L, E, 1, A, 4 * (1 + H), 1, 1, dropout=0.1, seed=3)
    args.N = N
    with pytest.raises(ValueError, match="dropout"):
        _lib.check(lib.dpt_rollout_bandit_generic(ctypes.byref(dd), ctypes.c_void_p(8), ctypes.byref(args), None))
