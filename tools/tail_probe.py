"""Phase breakdown of k_istft_pair from a SEPVAD_TAIL_PROBE dump.

usage: SEPVAD_TAIL_PROBE=/tmp/t.bin python bench.py --steps 1 --warmup 1 --no-cpu-baseline
       python tools/tail_probe.py /tmp/t.bin [shader GHz, default 2.1]
slot 0: wall clock (100 MHz) at entry; slots 1..5: shader clock at entry, after the rows, after the VAD tail,
after the inverse transforms, after the overlap-add stores are issued.
"""
import sys

import numpy as np

NAMES = ["loads + X sigmoid(m) rows", "VAD tail", "side outputs + transforms", "overlap-add"]


def main(path, ghz=2.1):
    raw = np.fromfile(path, dtype=np.int64)
    gx, gy, ns = (int(v) for v in raw[:3])
    st = raw[3:3 + gx * gy * ns].reshape(gy * gx, ns).astype(np.float64)
    ok = (st[:, :6] != 0).all(axis=1)
    st = st[ok]
    print(f"grid {gx} x {gy}; workgroups with full stamps {ok.sum()}")
    ent = (st[:, 0] - st[:, 0].min()) / 100.0  # us
    dur = (st[:, 5] - st[:, 1]) / (ghz * 1e3)
    print(f"entry times: spread {ent.max():.1f} us; workgroup duration median {np.median(dur):.2f} "
          f"p90 {np.percentile(dur, 90):.2f} us; last exit ~ {np.max(ent + dur):.1f} us after first entry")
    hist, edges = np.histogram(ent, bins=8)
    print("entry histogram (us):", ", ".join(f"{edges[i]:.1f}:{hist[i]}" for i in range(8)))
    for i, n in enumerate(NAMES):
        d = (st[:, i + 2] - st[:, i + 1]) / (ghz * 1e3)
        print(f"  {n:28s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f} us")
    early = ent < np.median(ent)
    print(f"first-half entrants duration median {np.median(dur[early]):.2f} us, later {np.median(dur[~early]):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 2.1)
