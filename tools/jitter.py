"""k_tcn launch-to-launch spread vs the shader clock.
Runs R forwards of the bench workload (cfg 2) with SEPVAD_TCN_CLOCK=1; per launch: the span over all workgroups
(100 MHz wall clock), workgroup 0's span and its shader clock (s_memtime ticks / wall time).
usage: SEPVAD_TCN_CLOCK=1 python tools/jitter.py [R] > out.txt"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sep_tfanet_vad_amd as pkg  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402


def main(R=50):
    assert os.environ.get("SEPVAD_TCN_CLOCK") == "1", "run with SEPVAD_TCN_CLOCK=1"
    cfg = pkg.CONFIG_WITH_VAD
    net = pkg.SeparationModel(**cfg)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 1234).items()}, strict=True)
    net = net.eval().to("cuda")
    x = torch.from_numpy(synth.make_batch(64, 32000, 11)[0]).to("cuda")
    with torch.no_grad():
        for _ in range(R + 3):
            net(x)
    torch.cuda.synchronize()
    rec = net.native_handle("cuda").tcn_clock()[-R:]
    span, w0, mhz = rec[:, 0], rec[:, 1], rec[:, 2]
    print(f"{R} launches of k_tcn (cfg 2, B=64, T=126)")
    print(f"  span us: median {np.median(span):.1f}  min {span.min():.1f}  max {span.max():.1f}  std {span.std():.1f}")
    print(f"  shader clock MHz (workgroup 0): median {np.median(mhz):.0f}  min {mhz.min():.0f}  max {mhz.max():.0f}")
    c = np.corrcoef(span, 1.0 / mhz)[0, 1] if span.std() > 0 and mhz.std() > 0 else float("nan")
    print(f"  corr(span, 1/clock) = {c:.3f}")
    cyc = span * mhz  # span in shader cycles at workgroup 0's clock
    print(f"  span in shader cycles (M): median {np.median(cyc) / 1e6:.3f}  std/median {cyc.std() / np.median(cyc):.3f}"
          f"  (time std/median {span.std() / np.median(span):.3f})")
    print(f"SUMMARY span_us_median {np.median(span):.2f} mcycles_median {np.median(cyc) / 1e6:.4f} mhz_median {np.median(mhz):.0f}")
    print("  launch  span_us  wg0_us  MHz")
    for i, (a, b, m) in enumerate(rec):
        print(f"  {i:6d} {a:8.1f} {b:7.1f} {m:5.0f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
