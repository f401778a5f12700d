"""Phase breakdown of the fused TCN from a SEPVAD_TCN_PROBE dump (wall clock, 100 MHz ticks).

usage: SEPVAD_TCN_PROBE=/tmp/p.bin python bench.py --steps 1 --warmup 1 --no-cpu-baseline
       python tools/tcn_probe.py /tmp/p.bin
"""
import os
import sys

import numpy as np

NAMES = ["conv1d GEMM", "epilogue+GN1 stats", "P1 publish+wait+halo", "dwconv+GN2 stats", "res_out GEMM",
         "P2 wait", "rowsum/colsum", "P3 publish+wait", "gates", "moments", "P4 publish+wait", "x' update"]
# sub-phase stamps currently placed in tcn_kernel.h: slot 13 after the residual-LN affines (x' update
# phase start), slot 14 after the next block's weight prefetch is issued
SUB = [(13, 11, "x': moments->affines"), (14, 13, "x': prefetch issue"), (12, 14, "x': update+barrier")]
if os.environ.get("TCN_SUB") == "1":  # library built with -DTCN_SUB=1: the stamps sit in the depthwise conv
    SUB = [(13, 3, "dw: GN1 affine"), (14, 13, "dw: rows (conv, PReLU, split stores)"), (4, 14, "dw: GN2 block sums")]
elif os.environ.get("TCN_SUB") == "2":  # in the conv1d epilogue
    SUB = [(13, 1, "epi: rows (PReLU, H stores, halo words)"), (14, 13, "epi: GN1 block sums"), (2, 14, "epi: GN1 words")]
elif os.environ.get("TCN_SUB") == "3":  # in the GN2 fold / row and frame sums
    SUB = [(13, 6, "rs: GN2 fold + rowsum words"), (14, 13, "rs: barrier"), (7, 14, "rs: frame sums + COL words")]


def main(path):
    raw = np.fromfile(path, dtype=np.int64)
    grid, nblk, G, T = (int(v) for v in raw[:4])
    full = raw[4:4 + grid * nblk * 16].astype(np.float64).reshape(grid, nblk, 16) / 100.0  # us
    keep = full[:, 0, 0] > 0  # (XCD-run launches: the blocks past a group's last member exit at once, no stamps)
    full = full[keep]
    st = full[:, :, :13]
    ok = (st > 0).all(axis=2)
    d = np.diff(st, axis=2)  # [grid, nblk, 12]
    print(f"grid={grid} nblk={nblk} G={G} T={T}; workgroups with full stamps: {ok.all(axis=1).sum()}")
    blk = (st[:, :, 12] - st[:, :, 0])
    print(f"per block (median over workgroups): {np.median(blk):.2f} us; first block start spread "
          f"{st[:, 0, 0].max() - st[:, 0, 0].min():.2f} us; launch span {st[:, -1, 12].max() - st[:, 0, 0].min():.1f} us")
    ent = full[:, 0, 15]
    if (ent > 0).all():
        print(f"kernel entry spread {ent.max() - ent.min():.2f} us; entry -> block 0 start: median "
              f"{np.median(st[:, 0, 0] - ent):.2f} max {(st[:, 0, 0] - ent).max():.2f} us")
        if nblk > 2 and (full[:, 1, 15] > 0).all() and (full[:, 2, 15] > 0).all():
            x1, x2 = full[:, 1, 15], full[:, 2, 15]  # after the XCD exchange; after the input statistics
            print(f"  prologue: first-touch loads + XCD exchange {np.median(x1 - ent):.2f}, record sums "
                  f"{np.median(x2 - x1):.2f}, input LN {np.median(st[:, 0, 0] - x2):.2f} us (medians)")
        if nblk > 7 and (full[:, 6, 15] > 0).all() and (full[:, 7, 15] > 0).all():
            x6, x7 = full[:, 6, 15], full[:, 7, 15]  # loads issued; LN records (and every earlier load) landed
            print(f"    entry -> loads issued {np.median(x6 - ent):.2f}, -> loads landed {np.median(x7 - x6):.2f} "
                  f"(max {(x7 - x6).max():.2f}), -> XCD exchange done {np.median(full[:, 1, 15] - x7):.2f} us")
    if nblk > 5 and (full[:, 3:6, 15] > 0).all() and (ent > 0).all():
        c3, c4, c5 = (full[:, k, 15] * 100.0 for k in (3, 4, 5))  # s_memtime ticks (undo the /100)
        wp = st[:, 0, 0] - ent
        wb = st[:, 2, 0] - st[:, 0, 0]
        print(f"shader clock: prologue {np.median((c4 - c3) / wp) / 1e3:.2f} GHz, blocks 0-1 "
              f"{np.median((c5 - c4) / wb) / 1e3:.2f} GHz")
    for i, n in enumerate(NAMES):
        v = d[:, 1:, i]  # skip block 0 (cold)
        print(f"  {n:24s} median {np.median(v):6.2f}  p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f} us")
    # per-wave stamps (lane 0 of each wave) after the wave-0 region: arrival spread at every phase point,
    # per-wave phase durations (which waves a barrier waits for)
    n0 = grid * nblk * 16
    if raw.size >= 4 + 9 * n0:
        W = raw[4 + n0: 4 + 9 * n0].astype(np.float64).reshape(grid, nblk, 16, 8)[keep] / 100.0
        Ws = W[:, 1:, :13, :]
        if (Ws > 0).all():
            print("  per-wave: phase                 spread-at-end  per-wave median durations w0..w7 (us)")
            dw = np.diff(Ws, axis=2)  # [grid, nblk-1, 12, 8]
            for i, n in enumerate(NAMES):
                spread = Ws[:, :, i + 1, :].max(axis=2) - Ws[:, :, i + 1, :].min(axis=2)
                med = np.median(dw[:, :, i, :], axis=(0, 1))
                print(f"    {n:24s} {np.median(spread):6.2f}   " + " ".join(f"{v:5.2f}" for v in med))
    # optional sub-phase stamps (slots 13..15) splitting one phase: (slot, previous stamp, label)
    for k, prev, label in SUB:
        v = full[:, 1:, k]
        if (v > 0).all():
            dv = v - full[:, 1:, prev]
            print(f"    {label:22s} median {np.median(dv):6.2f}  p90 {np.percentile(dv, 90):6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])

