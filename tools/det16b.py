"""k_tcn16 bring-up: block-level dumps (SEPVAD_TCN_DUMP_BLOCK) of k_tcn16 vs k_tcn and run to run.
usage: python tools/det16b.py B N blocks..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sep_tfanet_vad_amd as pkg  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402


def handle(t16):
    os.environ["SEPVAD_TCN16"] = str(t16)
    cfg = pkg.CONFIG_WITH_VAD
    net = pkg.SeparationModel(**cfg)
    sd = synth.make_state_dict(cfg, 1234)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return net.eval().to("cuda").native_handle("cuda")


B, N = int(sys.argv[1]), int(sys.argv[2])
blocks = [int(v) for v in sys.argv[3:]]
x = torch.from_numpy(synth.make_batch(B, N, 5000)[0]).cuda()
h16, h32 = handle(1), handle(0)
for blk in blocks:
    os.environ["SEPVAD_TCN_DUMP_BLOCK"] = str(blk)
    d0 = [t.clone() for t in h16.tcn_dump(x)]
    d1 = [t.clone() for t in h16.tcn_dump(x)]
    r = [t.clone() for t in h32.tcn_dump(x)]
    for name, a, b, c in zip(("input", "res", "att"), d0, d1, r):
        diff = (a - c).abs()
        bad = (diff > 1e-3 * c.abs().max()).nonzero()
        desc = ""
        if bad.shape[0]:
            desc = (f" bad utts {torch.unique(bad[:, 0]).tolist()[:12]} frames {torch.unique(bad[:, 2]).tolist()[:24]}"
                    f" nchan {torch.unique(bad[:, 1]).shape[0]}")
        print(f"block {blk} {name}: run-to-run {(a - b).abs().max().item():.2e}  vs k_tcn {diff.max().item():.2e}{desc}",
              flush=True)
