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


def check_vad_labels(vad, v_ref, band=1e-4, flips_per=1e-4, where=""):
    """VAD labels (p >= 0.5, reference model/model.py:449) vs the reference probabilities: bit-exact wherever the
    reference is farther than `band` from the threshold; inside the band (where fp32 rounding of either side can move
    a probability across 0.5) the labels are counted, not skipped: at most one flip per 1/flips_per labels (and at
    least one allowed). Returns (labels, labels in the band, flips in the band); printed for the test log."""
    vad = np.asarray(vad)
    v_ref = np.asarray(v_ref)
    lab, lref = vad >= 0.5, v_ref >= 0.5
    near = np.abs(v_ref - 0.5) <= band
    far_flips = int((lab != lref)[~near].sum())
    near_flips = int((lab != lref)[near].sum())
    n, nb = lab.size, int(near.sum())
    allowed = int(n * flips_per)  # 0 below 10 000 labels: small tests must be bit-exact in the band too
    msg = f"{where} VAD labels: {n}, within {band:g} of 0.5: {nb}, flips there: {near_flips} (allowed {allowed})"
    print(msg)
    if os.environ.get("SEPVAD_VAD_LABEL_LOG"):  # archived per round under profiles/ (tools/gpu_round*.sh)
        with open(os.environ["SEPVAD_VAD_LABEL_LOG"], "a") as f:
            f.write(os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0] + ": " + msg + "\n")
    assert far_flips == 0, f"{msg}; flips outside the band: {far_flips}"
    assert near_flips <= allowed, msg
    return n, nb, near_flips
