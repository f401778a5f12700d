"""Golden RIRs from the REFERENCE's own generator (create_data/rirgen.cpp, compiled from /root/reference by
oracle/Makefile into oracle/_ref/librirgen_ref.so) -> tests/golden/golden_rir.npz (data only).

    make -C oracle && python tests/golden/make_rir_golden.py
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# (room, src, mics, beta, orientation, high_pass, dim, order, n_samples, mic_type) — c = 340, fs = 16000
CASES = [
    ([5.0, 4.0, 3.0], [1.0, 2.0, 1.5], [[2.0, 1.5, 1.2], [2.1, 1.5, 1.2]], [0.3], [0.0, 0.0], 1, 3, -1, 2048, "o"),
    ([6.5, 5.2, 2.9], [3.1, 0.7, 1.7], [[1.2, 4.0, 1.4]], [0.6], [0.0, 0.0], 1, 3, -1, 1500, "o"),
    ([4.0, 4.0, 2.5], [1.0, 1.0, 1.0], [[3.0, 3.0, 1.5]], [0.0], [0.0, 0.0], 1, 3, -1, 512, "o"),
    ([5.0, 4.0, 3.0], [1.0, 2.0, 1.5], [[2.0, 1.5, 1.2]], [0.9, 0.8, 0.7, 0.85, 0.6, 0.75], [0.3, 0.1], 0, 3, 5, -1, "c"),
    ([5.0, 4.0, 3.0], [1.0, 2.0, 1.5], [[2.0, 1.5, 1.2]], [0.5], [0.5, -0.2], 1, 2, -1, 1024, "h"),
]


def ref_lib():
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "librirgen_ref.so"))
    dp = ctypes.POINTER(ctypes.c_double)
    lib.ref_rir_generate.restype = ctypes.c_int
    lib.ref_rir_generate.argtypes = [ctypes.c_double, ctypes.c_double, dp, ctypes.c_int, dp, dp, dp, ctypes.c_int, dp,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char, dp,
                                     ctypes.c_longlong]
    return lib


def ref_rir(lib, room, src, mics, beta, orient, hp, dim, order, n, mtype, c=340.0, fs=16000.0):
    dp = ctypes.POINTER(ctypes.c_double)
    a = [np.ascontiguousarray(v, dtype=np.float64) for v in (mics, src, room, beta, orient)]
    cap = len(mics) * 200000
    out = np.zeros(cap)
    got = lib.ref_rir_generate(c, fs, a[0].ctypes.data_as(dp), len(mics), a[1].ctypes.data_as(dp),
                               a[2].ctypes.data_as(dp), a[3].ctypes.data_as(dp), len(beta), a[4].ctypes.data_as(dp),
                               hp, dim, order, n, mtype.encode(), out.ctypes.data_as(dp), cap)
    assert got > 0
    return out[:len(mics) * got].reshape(len(mics), got)


def main():
    lib = ref_lib()
    d = {}
    for i, case in enumerate(CASES):
        d[f"h{i}"] = ref_rir(lib, *case)
    np.savez_compressed(os.path.join(HERE, "golden_rir.npz"), **d)
    print({k: v.shape for k, v in d.items()})


if __name__ == "__main__":
    main()
