"""Per-XCD view of a k_tcn phase probe (SEPVAD_TCN_PROBE dump, tools/tcn_probe.py format): workgroups grouped by
blockIdx % 8 (the workgroups of one XCD under round-robin dispatch), their per-block durations, block-0 start, last-block
end and the shader clock over blocks 0-1 (s_memtime / wall clock). Shows whether the launch's end waits for one slow XCD.
usage: python tools/r06_xcd.py probe.bin"""
import sys

import numpy as np


def main(path):
    raw = np.fromfile(path, dtype=np.int64)
    grid, nblk, G, T = (int(v) for v in raw[:4])
    full = raw[4:4 + grid * nblk * 16].astype(np.float64).reshape(grid, nblk, 16) / 100.0  # us
    st = full[:, :, :13]
    t0 = st[:, 0, 0].min()
    blk = st[:, 1:, 12] - st[:, 1:, 0]
    ent = full[:, 0, 15]
    clk = None
    if nblk > 5 and (full[:, 3:6, 15] > 0).all():
        c4, c5 = full[:, 4, 15] * 100.0, full[:, 5, 15] * 100.0
        clk = (c5 - c4) / (st[:, 2, 0] - st[:, 0, 0]) / 1e3
    print(f"grid {grid} nblk {nblk} G {G} T {T}")
    print("xcd  wgs  block0-start  last-end  block-median(us)  block-p90  clock(GHz)")
    for x in range(8):
        sel = np.arange(grid) % 8 == x
        c = f"{np.median(clk[sel]):.3f}" if clk is not None else "-"
        print(f"{x:3d} {sel.sum():4d} {np.median(st[sel, 0, 0] - t0):12.2f} {(st[sel, -1, 12] - t0).max():9.2f} "
              f"{np.median(blk[sel]):16.2f} {np.percentile(blk[sel], 90):10.2f}  {c}")
    ends = st[:, -1, 12] - t0
    print(f"last-block end: min {ends.min():.1f} median {np.median(ends):.1f} max {ends.max():.1f} us; "
          f"entry spread {ent.max() - ent.min():.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
