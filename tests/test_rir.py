"""Image-method RIR generator (csrc/rir.hip, host) vs the reference's own generator: bit-exact against
the golden RIRs it produced (tests/golden/make_rir_golden.py) and, when the reference build is present
(oracle/_ref, built by oracle/Makefile), against it directly on randomised rooms. CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, REPO

import sys
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import make_rir_golden as mk  # noqa: E402


def _ours(room, src, mics, beta, orient, hp, dim, order, n, mtype):
    from sep_tfanet_vad_amd import rirgen
    kw = dict(betaCoeffs=beta) if len(beta) == 6 else dict(reverbTime=beta[0])
    return np.array(rirgen.generateRir(room, src, mics, soundVelocity=340, fs=16000, orientation=orient,
                                       isHighPassFilter=bool(hp), nDim=dim, nOrder=order, nSamples=n, micType=mtype,
                                       **kw))


def test_rir_matches_reference_goldens():
    g = np.load(os.path.join(GOLDEN, "golden_rir.npz"))
    for i, case in enumerate(mk.CASES):
        h = _ours(*case)
        assert h.shape == g[f"h{i}"].shape
        assert np.array_equal(h, g[f"h{i}"]), f"case {i}: max |diff| {np.abs(h - g[f'h{i}']).max()}"


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "librirgen_ref.so")),
                    reason="reference RIR build absent (oracle/Makefile needs /root/reference)")
def test_rir_matches_reference_build_random_rooms():
    lib = mk.ref_lib()
    rng = np.random.Generator(np.random.PCG64(77))
    for _ in range(6):
        room = rng.uniform([3, 3, 2.2], [8, 7, 3.5])
        src = rng.uniform(0.3, 1, 3) * (room - 0.6) + 0.3
        mics = [list(rng.uniform(0.3, 1, 3) * (room - 0.6) + 0.3) for _ in range(2)]
        t60 = float(rng.uniform(0.2, 0.6))  # create_data/data_conifg_wham.yaml:54-55
        case = (list(room), list(src), mics, [t60], [0.0, 0.0], 1, 3, -1, 1200, "o")
        assert np.array_equal(_ours(*case), mk.ref_rir(lib, *case))


def test_rir_api_errors_and_shapes():
    from sep_tfanet_vad_amd import rirgen
    with pytest.raises(ValueError):
        rirgen.generateRir([5, 4, 3], [1, 1, 1], [2, 2, 2])
    with pytest.raises(ValueError):
        rirgen.generateRir([5, 4, 3], [1, 1, 1], [2, 2, 2], reverbTime=0.3, betaCoeffs=[0.5] * 6)
    h = rirgen.generateRir([5, 4, 3], [1, 1, 1], [2, 2, 2], reverbTime=0.2, nSamples=300)
    assert isinstance(h, list) and len(h) == 300 and not isinstance(h[0], list)
    h = rirgen.generateRir([5, 4, 3], [1, 1, 1], [[2, 2, 2]], reverbTime=0.2)
    assert len(h) == 1 and len(h[0]) == int(0.2 * 16000)
