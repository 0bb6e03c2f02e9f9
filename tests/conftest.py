import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
# the C restatement is built on demand (oracle/Makefile)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def unhex(xs):
    return np.array([float.fromhex(x) for x in xs], dtype=np.float64)


@pytest.fixture(scope="session")
def golden():
    return load_golden


def regen_window(case):
    """Re-create the exact DataFrames a span-level fixture was captured on."""
    from microrank_amd import synth

    p = dict(case["params"])
    ndf, adf = synth.window_dataframes(p.pop("n_ops"), p.pop("n_traces"), p.pop("seed"), **p)
    assert synth.frame_digest(ndf) == case["input_digest"]["normal"], "generator drifted (normal)"
    assert synth.frame_digest(adf) == case["input_digest"]["abnormal"], "generator drifted (abnormal)"
    return ndf, adf
