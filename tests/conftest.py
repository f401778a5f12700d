import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libsepvad.so")


CONFIGS = ("with_vad", "without_vad")
CASES = ("small", "ragged", "cfg")


def load_golden(cname, case):
    return dict(np.load(os.path.join(GOLDEN, f"golden_{cname}_{case}.npz")))


def config_of(cname):
    import sep_tfanet_vad_amd as pkg
    return pkg.CONFIG_WITH_VAD if cname == "with_vad" else pkg.CONFIG_WITHOUT_VAD


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def state_dicts():
    """Recipe weights (seed 1234) as float32 torch tensors, per config name."""
    import torch
    from sep_tfanet_vad_amd import synth
    out = {}
    for c in CONFIGS:
        out[c] = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(config_of(c), 1234).items()}
    return out
