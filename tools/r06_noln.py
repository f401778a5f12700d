"""Diagnostics: one- vs two-slice vs multi-kernel on the no-LN (LD_ADD) and no-TF-attention configs."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import sep_tfanet_vad_amd as pkg  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402
from conftest import config_of  # noqa: E402


def run(net, x, slices=None, fused=True):
    if slices:
        os.environ["SEPVAD_TCN_SLICES"] = str(slices)
    h = net.native_handle("cuda")
    h.set_fused(fused)
    with torch.no_grad():
        out = net(x)
    st = h.fused_status()
    os.environ.pop("SEPVAD_TCN_SLICES", None)
    h.set_fused(True)
    return out, st, h.fused_slices()


for variant in ("no_ln", "no_tf_attention", "residual_no_tf"):
    cfg = dict(config_of("with_vad"))
    if variant == "no_ln":
        cfg.update(apply_recursive_ln=False, apply_residual_ln=False)
    elif variant == "no_tf_attention":
        cfg.update(tf_attention=False)
    else:
        cfg = dict(config_of("without_vad"), tf_attention=False)
    net = pkg.SeparationModel(**cfg)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 31).items()}, strict=True)
    net = net.eval().to("cuda")
    for N in (32000, 130816):
        x = torch.from_numpy(synth.make_batch(3, N, 606 + N)[0]).to("cuda")
        o1, st1, u1 = run(net, x, 1)
        o1b, _, _ = run(net, x, 1)
        o2, st2, u2 = run(net, x, 2)
        om, stm, _ = run(net, x, None, False)
        d = lambda a, b: max((a[i] - b[i]).abs().max().item() for i in range(2))
        print(variant, N, "slices", u1, u2, "status", st1, st2, stm, "nan1", torch.isnan(o1[0]).any().item(),
              "nan2", torch.isnan(o2[0]).any().item(), "1v1", d(o1, o1b), "1v2", d(o1, o2), "1vM", d(o1, om), "2vM", d(o2, om))
        if u2 == 2:
            per = (o1[0] - o2[0]).abs().amax(dim=(1, 2))
            print("   per-utterance 1v2:", [f"{v:.3g}" for v in per.tolist()])
