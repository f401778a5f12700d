"""Digest of one forward's outputs (sep, vad, est) for bitwise A/B of library builds that claim equal bits.
usage: SEPVAD_LIB=var/lib_x.so python3 tools/bitwise_ab.py [B] [N]   -> prints "<lib> <sha256 of sep|vad|est>"
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 32000
    net = pkg.SeparationModel(**pkg.CONFIG_WITH_VAD)
    sd = synth.make_state_dict(pkg.CONFIG_WITH_VAD, 1234)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net = net.eval().to("cuda:0")
    x = torch.from_numpy(synth.make_batch(B, N, 99)[0]).to("cuda:0")
    with torch.no_grad():
        sep, vad, est = net(x)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (sep, vad, est):
        h.update(t.detach().cpu().contiguous().numpy().tobytes())
    print(os.path.basename(os.environ.get("SEPVAD_LIB", "libsepvad.so")), B, N, h.hexdigest()[:32])


if __name__ == "__main__":
    main()
