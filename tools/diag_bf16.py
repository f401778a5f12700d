"""Diagnostics: masks_b / sep / vad of the bf16 arm at cfg 2 shapes, saved to gpurun_out/diag_bf16_<tag>.npz, and a
comparison of two saved runs. usage: python tools/diag_bf16.py run <tag> | python tools/diag_bf16.py cmp <a> <b>"""
import sys
import numpy as np


def run(tag):
    import torch
    sys.path.insert(0, ".")
    sys.path.insert(0, "tests")
    from conftest import config_of
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(config_of("with_vad"), 1234).items()}
    net = pkg.SeparationModel(**config_of("with_vad"))
    net.load_state_dict(sd, strict=True)
    net = net.eval().to("cuda")
    x = torch.from_numpy(synth.make_batch(8, 32000, 1234)[0]).to("cuda")
    out = {}
    for prec in ("bf16", "f16"):
        net.native_precision = prec
        with torch.no_grad():
            s, v, _ = net(x)
        out[prec + "_sep"] = s.cpu().numpy(); out[prec + "_vad"] = v.cpu().numpy()
        out[prec + "_masks"] = net.masks_b.cpu().numpy()
    np.savez(f"gpurun_out/diag_bf16_{tag}.npz", **out)


def cmp(a, b):
    A = np.load(f"gpurun_out/diag_bf16_{a}.npz"); B = np.load(f"gpurun_out/diag_bf16_{b}.npz")
    for prec in ("bf16", "f16"):
        ma, mb = A[prec + "_masks"], B[prec + "_masks"]  # [B][514][T]
        d = np.abs(ma - mb)
        print(prec, "masks max diff", d.max(), "per speaker-bin block of 32:",
              [float(d[:, q * 257 + 32 * j: q * 257 + min(32 * j + 32, 257)].max()) for q in range(2) for j in range(9)])
        print(prec, "bin 256 diff", d[:, [256, 513]].max(), "frames with diff > 1e-2:", int((d.max(axis=1) > 1e-2).sum()))
        print(prec, "sep diff", np.abs(A[prec + "_sep"] - B[prec + "_sep"]).max(), "vad diff", np.abs(A[prec + "_vad"] - B[prec + "_vad"]).max())


if __name__ == "__main__":
    run(sys.argv[2]) if sys.argv[1] == "run" else cmp(sys.argv[2], sys.argv[3])
