"""``pyrirgen.generateRir`` mirror (reference ``create_data/pyrirgen.pyx``) over the C-ABI image-method
generator ``sepvad_rir_generate`` (csrc/rir.hip; restates ``create_data/rirgen.cpp:115-351``).

Same keyword surface and errors: exactly one of ``reverbTime`` / ``betaCoeffs``; a single receiver
position (not a list of positions) returns one response; ``soundVelocity`` and ``fs`` pass through a C
``float`` in the reference's Cython signature, which is reproduced (``np.float32`` rounding)."""
from __future__ import annotations

import ctypes
from collections.abc import Iterable

import numpy as np

from . import native as _native


def generateRir(roomMeasures, sourcePosition, receiverPositions, *, reverbTime=None, betaCoeffs=None,  # noqa: N802,N803
                soundVelocity=340, fs=16000, orientation=(0.0, 0.0), isHighPassFilter=True, nDim=3,  # noqa: N803
                nOrder=-1, nSamples=-1, micType="o"):  # noqa: N803
    if not (reverbTime is None) != (betaCoeffs is None):
        raise ValueError("You provide either reverbTime or betaCoeffs.")
    beta = [reverbTime] if betaCoeffs is None else list(betaCoeffs)
    multiple = all(isinstance(e, Iterable) for e in receiverPositions)
    mics = np.ascontiguousarray(receiverPositions if multiple else [receiverPositions], dtype=np.float64)
    src = np.ascontiguousarray(sourcePosition, dtype=np.float64)
    room = np.ascontiguousarray(roomMeasures, dtype=np.float64)
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    orient = np.ascontiguousarray(orientation, dtype=np.float64)
    c, f = float(np.float32(soundVelocity)), float(np.float32(fs))
    lib = _native.load_library()
    dp = ctypes.POINTER(ctypes.c_double)

    def call(out, cap):
        return lib.sepvad_rir_generate(c, f, mics.ctypes.data_as(dp), len(mics), src.ctypes.data_as(dp),
                                       room.ctypes.data_as(dp), beta.ctypes.data_as(dp), len(beta),
                                       orient.ctypes.data_as(dp), int(bool(isHighPassFilter)), int(nDim),
                                       int(nOrder), int(nSamples), micType[0].encode(), out, cap)

    n = call(None, 0)
    if n < 0:
        raise RuntimeError(f"sepvad_rir_generate failed (status {n})")
    h = np.zeros((len(mics), n), dtype=np.float64)
    n2 = call(h.ctypes.data_as(dp), h.size)
    if n2 != n:
        raise RuntimeError(f"sepvad_rir_generate failed (status {n2})")
    return h.tolist() if multiple else h[0].tolist()
