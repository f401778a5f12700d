"""What precision the fp16x3 weight lo plane needs (design study for a narrower weight stream).

The fused TCN splits every pointwise weight (row-scaled by 2^-e, max |w| in [0.5, 1)) into fp16 hi + fp16 lo and
issues A_lo B_hi + A_hi B_lo + A_hi B_hi. This emulates narrower lo planes on the CPU: effective weights
(hi + q(lo)) / s in the oracle's conv1d / res_out (reg2 folded per column, as api.hip packs it), everything else
fp32, and compares sep / VAD against the fp64 oracle next to the fp32 oracle's own error.
usage: python tools/lo_plane_precision.py [B] [N]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import config_of  # noqa: E402
from oracle.torch_ref import OracleModel  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402


def quant(w, mode):
    """w [cout, cin] fp64 -> effective weights of the split `mode`."""
    mx = w.abs().amax(dim=1, keepdim=True)
    e = torch.frexp(mx)[1].to(torch.float64)
    s = torch.pow(2.0, -e)
    vs = (w * s).to(torch.float32)
    hi = vs.to(torch.float16).to(torch.float32)
    lo = vs - hi
    if mode == "f16":
        q = hi
    elif mode == "f16x3":
        q = hi + lo.to(torch.float16).to(torch.float32)
    elif mode.startswith("lo8"):
        sh = int(mode[3:] or 19)  # lo * 2^sh into e4m3 (|lo| <= 2^-12 -> <= 2^(sh-12) <= 448)
        l8 = (lo * 2.0 ** sh).to(torch.float8_e4m3fn).to(torch.float32) / 2.0 ** sh
        q = hi + l8.to(torch.float16).to(torch.float32)   # the MFMA's B_lo operand is fp16
    elif mode == "lo_i8":
        # lo as int8 steps of 2^-19 (row-scaled weights: |lo| <= 2^-12 -> |q| <= 128; the packer re-rounds hi when q
        # would be +128), widened exactly in fp16 by the 1024-magic-number trick
        q = torch.clamp(torch.round(lo * 2.0 ** 19), -128, 127)
        q = hi + (q / 2.0 ** 19).to(torch.float16).to(torch.float32)
    elif mode == "lo_bf16":
        q = hi + lo.to(torch.bfloat16).to(torch.float32)
    else:
        raise ValueError(mode)
    return q.to(torch.float64) / s


def run(mode, sd, x):
    om = OracleModel(config_of("with_vad"), sd, torch.float32)
    if mode != "fp32":
        for b in om.blocks:
            w1 = b["w1"].to(torch.float64)[:, :, 0]
            b["w1"] = quant(w1, mode).to(torch.float32)[:, :, None]
            g2 = b["g2"].to(torch.float64)
            w2f = b["w2"].to(torch.float64)[:, :, 0] * g2[None, :]
            b["w2"] = (quant(w2f, mode) / g2[None, :]).to(torch.float32)[:, :, None]
    return om(x)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 32000
    torch.set_num_threads(os.cpu_count() or 1)
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(config_of("with_vad"), 1234).items()}
    x, _ = synth.make_batch(B, N, 60_000 + B)
    x = torch.from_numpy(x)
    ref = OracleModel(config_of("with_vad"), sd, torch.float64)(x.to(torch.float64))
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["fp32", "f16x3", "lo8", "lo_i8", "lo_bf16", "f16"]
    erange = max(ref[2].real.abs().max().item(), ref[2].imag.abs().max().item())
    for mode in modes:
        sep, vad, est = run(mode, sd, x)
        err = (sep.double() - ref[0]).abs().max().item()
        flips = int(((vad >= 0.5) != (ref[1] >= 0.5)).sum())
        verr = (vad.double() - ref[1]).abs().max().item()
        eerr = (est.to(torch.complex128) - ref[2]).abs().max().item() / erange
        print(f"{mode:8s} sep max-abs vs fp64 {err:.3e}  est {eerr:.2e} of range  vad max-abs {verr:.3e}  "
              f"label flips {flips}/{vad.numel()}", flush=True)


if __name__ == "__main__":
    main()
