"""Phase breakdown of k_istft_pair / k_stft_gate from a SEPVAD_TAIL_PROBE dump.

usage: SEPVAD_TAIL_PROBE=/tmp/t python bench.py --steps 1 --warmup 1 --no-cpu-baseline
       python tools/tail_probe.py /tmp/t.istft [shader GHz, default 2.1]   (and /tmp/t.stft)
slot 0: wall clock (100 MHz) at entry; slots 1..5: shader clock at entry and at the ends of the phases named
in NAMES (thread 0's view).
"""
import sys

import numpy as np

NAMES = {"istft": ["loads + X sigmoid(m) rows", "VAD tail", "side outputs + transforms", "overlap-add"],
         "stft": ["loads + transform (wave 0)", "split + dB (wave 0)", "barrier", "activity gate + records"],
         "head": ["x' loads + records", "GN affine + A (LDS)", "GEMM (wave 0)", "mask stores issued"],
         "tcnhead": ["P5 publish + poll", "records + GN + A (LDS)", "tiles (wave 0)", "tap sums + stores"],
         "vad1": ["loads + taps (FMA)", "lane reduction", "wave partials + barrier", "PReLU + features + records"]}


def main(path, ghz=2.1):
    names = NAMES[path.rsplit(".", 1)[-1]]
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
    for i, n in enumerate(names):
        d = (st[:, i + 2] - st[:, i + 1]) / (ghz * 1e3)
        print(f"  {n:28s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f} us")
    early = ent < np.median(ent)
    print(f"first-half entrants duration median {np.median(dur[early]):.2f} us, later {np.median(dur[~early]):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 2.1)
