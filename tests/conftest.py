"""Shared pytest setup.

* registers the `gpu` marker (tests that need a real MI355X; run with -m gpu);
* puts the product package directory (`understanding-hmc_amd/`) and the repo
  root (for `oracle/`, test infrastructure) on sys.path.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "understanding-hmc_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_golden(name):
    """Load a committed golden fixture (data only; produced by tests/golden/make_golden.py)."""
    path = os.path.join(GOLDEN, name)
    if name.endswith(".json"):
        with open(path) as f:
            return json.load(f)
    z = np.load(path, allow_pickle=False)
    out = {k: z[k] for k in z.files}
    if "meta" in out:
        out["meta"] = json.loads(str(out["meta"]))
    return out


@pytest.fixture
def golden():
    return load_golden
