"""k_tcn16 bring-up: run-to-run determinism at B=64 (tcn_dump stages + outputs), k_tcn16 vs k_tcn difference.
usage (GPU box): python tools/det16.py"""
import os
import sys

import numpy as np
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
    net = net.eval().to("cuda")
    return net.native_handle("cuda")


B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 32000
x = torch.from_numpy(synth.make_batch(B, N, 5000)[0]).cuda()
h16 = handle(1)
h32 = handle(0)
runs = []
for k in range(4):
    d = [t.clone() for t in h16.tcn_dump(x)]
    o = h16.forward(x)
    torch.cuda.synchronize()
    runs.append((d, {kk: o[kk].clone() for kk in ("sep", "vad")}))
    print("run", k, "fused", h16.fused_status(), flush=True)
ref_d, ref_o = runs[0]
for k in range(1, len(runs)):
    d, o = runs[k]
    for name, a, b in zip(("tcn_in", "blk0_res", "blk0_att"), ref_d, d):
        diff = (a - b).abs()
        nz = (diff > 0).nonzero()
        print(f"run {k} {name}: maxdiff {diff.max().item():.3e} ndiff {nz.shape[0]}", flush=True)
        if nz.shape[0]:
            utt = torch.unique(nz[:, 0]).tolist()
            frames = torch.unique(nz[:, 2]).tolist()
            chans = torch.unique(nz[:, 1]).tolist()
            print("   utts", utt[:20], "frames", frames[:40], "nchan", len(chans), chans[:20])
    for kk in ("sep", "vad"):
        print(f"run {k} {kk}: maxdiff {(ref_o[kk] - o[kk]).abs().max().item():.3e}")
d32 = [t.clone() for t in h32.tcn_dump(x)]
o32 = h32.forward(x)
for name, a, b in zip(("tcn_in", "blk0_res", "blk0_att"), ref_d, d32):
    print(f"k_tcn16 vs k_tcn {name}: maxdiff {(a - b).abs().max().item():.3e} range {b.abs().max().item():.3e}")
for kk in ("sep", "vad"):
    print(f"k_tcn16 vs k_tcn {kk}: maxdiff {(ref_o[kk] - o32[kk]).abs().max().item():.3e}")
