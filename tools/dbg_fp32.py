"""Diagnostic: where the fused exact-fp32 TCN (k_tcn<PREC_F32>) departs from the multi-kernel fp32 schedule.

Prints, per configuration (shipped with_vad, and reduced stacks of 1 and 2 blocks), the masks' max difference
fused-fp32 vs multi-kernel-fp32 and fused-f16x3 vs multi-kernel-fp32, and the error's distribution over frame
position in a 32-frame slice, slice index and 32-bin tile. Not a test; run on the GPU box.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import sep_tfanet_vad_amd as pkg  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402

DEV = "cuda"


def masks(h, x, fused, prec):
    h.set_precision(prec)
    h.set_fused(fused)
    r = h.forward(x, return_aux=True)
    used = h.fused_status()
    return r["masks_b"].float().cpu().numpy(), r["sep"].cpu().numpy(), used


def report(tag, a, b):
    d = np.abs(a - b)  # [B, 514, T]
    T = d.shape[2]
    print(f"  {tag}: max {d.max():.3e} mean {d.mean():.3e}  frac>1e-3 {(d > 1e-3).mean():.4f}")
    fr = d.max(axis=(0, 1))
    pos = np.array([fr[t::32].max() if t < T else 0 for t in range(32)])
    print("    by frame%32:", " ".join(f"{v:.1e}" for v in pos))
    sl = np.array([fr[32 * s:32 * s + 32].max() for s in range((T + 31) // 32)])
    print("    by slice:", " ".join(f"{v:.1e}" for v in sl))
    bn = d.max(axis=(0, 2))
    tiles = np.array([bn[32 * k:32 * k + 32].max() for k in range((514 + 31) // 32)])
    print("    by 32-bin tile (spk0 0..8, spk1 ...):", " ".join(f"{v:.1e}" for v in tiles))
    print("    bin 256 / 513:", f"{bn[256]:.1e} {bn[513]:.1e}")


def main():
    x = torch.from_numpy(synth.make_batch(3, 32000, 515)[0]).to(DEV)
    for name, over in (("with_vad", {}), ("with_vad stack1 layer1", dict(stack=1, layer=1)),
                       ("with_vad stack1 layer2", dict(stack=1, layer=2)), ("without_vad", None)):
        cfg = dict(pkg.CONFIG_WITH_VAD if over is not None else pkg.CONFIG_WITHOUT_VAD)
        cfg.update(over or {})
        sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 1234).items()}
        net = pkg.SeparationModel(**cfg)
        net.load_state_dict(sd, strict=True)
        net = net.eval().to(DEV)
        net.native_precision = "fp32"
        h = net.native_handle(DEV)
        with torch.no_grad():
            mf, sf, uf = masks(h, x, True, "fp32")
            mm, sm, um = masks(h, x, False, "fp32")
            m3, s3, u3 = masks(h, x, True, "f16x3")
        print(f"{name}: fused fp32 used={uf} multi used={um} f16x3 used={u3}; sep fp32 fused-multi "
              f"{np.abs(sf - sm).max():.3e}, f16x3-multi {np.abs(s3 - sm).max():.3e}")
        report("fp32 fused vs fp32 multi", mf, mm)
        report("f16x3 fused vs fp32 multi", m3, mm)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
