"""Phase breakdown of the role-specialised TCN (k_tcn_rs, tcn_rs.hip) from a SEPVAD_TCN_PROBE dump.

Stamps (wall clock, 100 MHz ticks), lane 0 of every wave, [grid][nblk][16 points][8 waves]:
  M waves 0-3: 0 block start, 1 conv1d GEMM done, 2 epilogue + res_out ring issued, 3 res_out GEMM done,
               4 raw row/column sums published, 5 moment record published + next ring issued, 6 x' update done
  V waves 4-7: 0 block start, 9 next parameters in LDS, 10 GN1 + halo polled, 11 depthwise conv done,
               12 GN2 + sums polled, gates done, 13 moments polled (wave 4)
usage: SEPVAD_TCN_PROBE=/tmp/p.bin python bench.py --steps 1 --warmup 1 --no-cpu-baseline
       python tools/rs_probe.py /tmp/p.bin
"""
import sys

import numpy as np


def main(path):
    raw = np.fromfile(path, dtype=np.int64)
    grid, nblk, G, T = (int(v) for v in raw[:4])
    st = raw[4:4 + grid * nblk * 16 * 8].astype(np.float64).reshape(grid, nblk, 16, 8) / 100.0  # us
    M, V = st[:, :, :, :4], st[:, :, :, 4:]
    ok = (M[:, :, [0, 1, 2, 3, 4, 5, 6], :] > 0).all(axis=(1, 2, 3))
    print(f"grid={grid} nblk={nblk} G={G} T={T}; workgroups with full stamps: {ok.sum()}")
    st, M, V = st[ok], M[ok], V[ok]
    blk = np.diff(M[:, :, 0, 0], axis=1)
    print(f"per block (median): {np.median(blk):.2f} us (p10 {np.percentile(blk, 10):.2f}, p90 {np.percentile(blk, 90):.2f});"
          f" launch span {M[:, -1, 6, :].max() - M[:, 0, 0, :].min():.1f} us")
    b1 = np.maximum(M[:, :, 2, :].max(axis=2), V[:, :, 9, :].max(axis=2))
    b3 = np.maximum(M[:, :, 4, :].max(axis=2), V[:, :, 12, :].max(axis=2))
    b4 = np.maximum(M[:, :, 5, :].max(axis=2), V[:, :, 13, 0])
    b0 = M[:, :, 6, :].max(axis=2)
    s0 = M[:, :, 0, :].min(axis=2)
    med = lambda a: f"{np.median(a):6.2f}"
    rows = [
        ("A  start -> B1 (latest arrival)", b1 - s0),
        ("   M conv1d GEMM", (M[:, :, 1, :] - M[:, :, 0, :]).mean(axis=2)),
        ("   M epilogue + res_out ring", (M[:, :, 2, :] - M[:, :, 1, :]).mean(axis=2)),
        ("   V next parameters", (V[:, :, 9, :] - V[:, :, 0, :]).mean(axis=2)),
        ("B  B1 -> B3 (latest arrival)", b3 - b1),
        ("   V GN1 + halo polls", (V[:, :, 10, :] - b1[:, :, None]).mean(axis=2)),
        ("   V depthwise conv (4 chunks)", (V[:, :, 11, :] - V[:, :, 10, :]).mean(axis=2)),
        ("   V GN2 + sums polls, gates", (V[:, :, 12, :] - V[:, :, 11, :]).mean(axis=2)),
        ("   M res_out GEMM (from B1)", (M[:, :, 3, :] - b1[:, :, None]).mean(axis=2)),
        ("   M raw sums", (M[:, :, 4, :] - M[:, :, 3, :]).mean(axis=2)),
        ("   M res_out end - V dwconv end", M[:, :, 3, :].max(axis=2) - V[:, :, 11, :].max(axis=2)),
        ("C  B3 -> B4 (latest arrival)", b4 - b3),
        ("   M gates + moments + ring", (M[:, :, 5, :] - b3[:, :, None]).mean(axis=2)),
        ("   V moments poll (wave 4)", V[:, :, 13, 0] - b3),
        ("D  B4 -> B0 (x' update)", b0 - b4),
    ]
    for name, a in rows:
        print(f"  {name:36s} median {med(a)}  p90 {np.percentile(a, 90):6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])


def detail(path):
    raw = np.fromfile(path, dtype=np.int64)
    grid, nblk, G, T = (int(v) for v in raw[:4])
    st = raw[4:4 + grid * nblk * 16 * 8].astype(np.float64).reshape(grid, nblk, 16, 8) / 100.0
    M, V = st[:, :, :, :4], st[:, :, :, 4:]
    med = lambda a: f"{np.median(a):6.2f}"
    s0 = M[:, :, 0, :].min(axis=2)
    print("  sub-phases, us from the block start (min over M waves), medians over workgroups and blocks:")
    for name, a in [("M G1 done", M[:, :, 1, :].max(axis=2)), ("M E1 done", M[:, :, 2, :].max(axis=2)),
                    ("V prm done", V[:, :, 9, :].max(axis=2)), ("V R1 gpoll returned", V[:, :, 7, :].max(axis=2)),
                    ("V R1 done (pflag)", V[:, :, 10, :].max(axis=2)), ("M ring issued", M[:, :, 7, :].max(axis=2)),
                    ("V chunk 0", V[:, :, 8, :].max(axis=2)), ("V chunk 1", V[:, :, 14, :].max(axis=2)),
                    ("V chunk 2", V[:, :, 15, :].max(axis=2)), ("V chunk 3 + GN2 pub", V[:, :, 11, :].max(axis=2)),
                    ("M G2 done", M[:, :, 3, :].max(axis=2)), ("M E2 done", M[:, :, 4, :].max(axis=2)),
                    ("V R23 gpoll returned", V[:, :, 6, :].max(axis=2)), ("V gates done", V[:, :, 12, :].max(axis=2)),
                    ("M after B3", M[:, :, 8, :].max(axis=2)), ("M MO done", M[:, :, 5, :].max(axis=2)),
                    ("V R4 gpoll returned", V[:, :, 5, 0]), ("V R4 done", V[:, :, 13, 0]),
                    ("M XU done", M[:, :, 6, :].max(axis=2))]:
        print(f"    {name:28s} {med(a - s0)}")
    # member skew: spread of block start over the G members of a group (consecutive workgroups b, b+8, ..)
    if grid % (8 * G) == 0:
        idx = np.arange(grid)
        grp = (idx >> 3) // G * 8 + (idx & 7)
        sk = []
        for gg in np.unique(grp):
            m = s0[grp == gg]
            sk.append(m.max(axis=0) - m.min(axis=0))
        print(f"  member skew of block start: median {np.median(sk):.2f} us, p90 {np.percentile(sk, 90):.2f}")


if __name__ == "__main__" and len(sys.argv) > 2:
    detail(sys.argv[1])
