"""Shared test plumbing.

* registers the ``gpu`` marker (tests that need a real MI355X);
* puts the product source root (``decision-pretrained-transformer_amd/``, whose
  top-level modules keep the reference's names: envs, ctrls, evals, models ...)
  and the repo root (for ``oracle``) on ``sys.path``.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "decision-pretrained-transformer_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


@pytest.fixture
def load_golden():
    return golden
