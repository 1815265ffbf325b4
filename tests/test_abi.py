"""CPU checks of the C-ABI library: it loads, exports every symbol include/dpt_hip.h
declares, the Python signature table matches the header, and host-side validation
maps to the reference's exception types.  No device work is launched."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "dpt_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(dpt_\w+)\s*\(", src, flags=re.M)))


def test_header_parses():
    fns = header_functions()
    for name in ("dpt_rollout_bandit", "dpt_forward_window", "dpt_decode_step", "dpt_select_action",
                 "dpt_bandit_step", "dpt_darkroom_step", "dpt_model_create", "dpt_last_error"):
        assert name in fns


def test_library_exports_every_header_symbol():
    from dpt_hip import _lib
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert set(header_functions()) == set(_lib.SIGNATURES), "ctypes table out of sync with dpt_hip.h"


def test_abi_version_and_validation():
    from dpt_hip import _lib
    lib = _lib.load()
    assert lib.dpt_abi_version() == _lib.ABI_VERSION
    d = _lib.ModelDesc(4, 32, 1, 5, 2004)
    n = ctypes.c_int64()
    assert lib.dpt_weights_numel(ctypes.byref(d), ctypes.byref(n)) == 0
    F = 2 * 1 + 5 + 1
    assert n.value == F * 32 + 32 + 2004 * 32 + 4 * 12704 + 64 + 32 * 5 + 5
    bad = _lib.ModelDesc(4, 64, 1, 5, 2004)
    with pytest.raises(NotImplementedError):
        _lib.check(lib.dpt_weights_numel(ctypes.byref(bad), ctypes.byref(n)))
    bad = _lib.ModelDesc(4, 32, 1, 99, 2004)
    with pytest.raises(ValueError):
        _lib.check(lib.dpt_weights_numel(ctypes.byref(bad), ctypes.byref(n)))
    assert b"action_dim" in lib.dpt_last_error()


def test_struct_layout_matches_header(tmp_path):
    """Every ctypes struct matches the C compiler's layout of include/dpt_hip.h field by field."""
    import shutil
    import subprocess

    from dpt_hip import _lib
    structs = {"dpt_model_desc": _lib.ModelDesc, "dpt_bandit_rollout_args": _lib.BanditRolloutArgs,
               "dpt_policy_rollout_args": _lib.PolicyRolloutArgs,
               "dpt_darkroom_rollout_args": _lib.DarkroomRolloutArgs, "dpt_train_desc": _lib.TrainDesc}
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "dpt_hip.h"', 'int main(void) {']
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                              text=True).stdout.splitlines())
    for cname, cls in structs.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert int(got[f"{cname} {fname}"]) == getattr(cls, fname).offset, (cname, fname)


def test_pack_weights_order():
    import numpy as np
    import torch

    import dpt_hip
    from conftest import golden
    g = golden("forward_bandit5.npz")
    w = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w/")}
    blob = dpt_hip.pack_weights(w, 4).numpy()
    emb = g["w/embed_transition.weight"]  # [E][F]
    assert np.array_equal(blob[:emb.size].reshape(emb.shape[1], 32), emb.T)
    head_b = g["w/pred_actions.bias"]
    assert np.array_equal(blob[-5:], head_b)
    off = emb.size + 32 + g["w/transformer.wpe.weight"].size
    assert np.array_equal(blob[off:off + 32], g["w/transformer.h.0.ln_1.weight"])
    assert np.array_equal(blob[off + 64:off + 64 + 3072].reshape(32, 96), g["w/transformer.h.0.attn.c_attn.weight"])


def test_product_path_has_no_oracle_import():
    """The shipped package must never import the test oracle."""
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), f


def test_header_constants_match_binding():
    """Every numeric #define DPT_* of include/dpt_hip.h has the same value in dpt_hip._lib
    (DPT_X -> X, or DPT_X itself for the error codes)."""
    from dpt_hip import _lib
    defs = dict(re.findall(r"^#define DPT_(\w+)\s+\(?(-?\d+)\)?", open(HEADER).read(), re.M))
    assert len(defs) >= 20
    for name, val in defs.items():
        if name == "HIP_H":
            continue
        py = getattr(_lib, "DPT_" + name, getattr(_lib, name, None))
        assert py is not None, name
        assert int(py) == int(val), (name, py, val)
