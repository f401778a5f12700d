"""Generate golden vectors by running the REFERENCE forward (run here, never on the GPU box).

    python tests/golden/make_golden.py

Imports ``/root/reference/model/model.py`` (and the streaming wrapper
``model/online_class_unknown_targets.py``) through two offline stand-ins:
  * ``tests/golden/_shim/torchaudio`` — torchaudio is not installed (reference model/model.py:5);
  * a stub ``turtle`` module — reference model/combined_loss.py:1 does ``from turtle import forward``
    (unused) and tkinter is absent.
Weights come from the PCG64 recipe ``synth.make_state_dict`` (the pretrained .pth files are absent,
reference .MISSING_LARGE_BLOBS:1-2) and are loaded ``strict=True`` into the reference model.
Inputs come from ``synth.make_batch``. Outputs are written as compressed .npz fixtures next to
this script. Only data (inputs and the reference's outputs) is written — no reference source.
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.path.insert(0, REPO)
import sep_tfanet_vad_amd as pkg  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402

SEED_W = 1234
CASES = [  # (name, B, N, base_seed)
    ("small", 2, 8000, 100),
    ("ragged", 1, 12345, 200),
    ("cfg", 1, 32000, 300),
]


def import_reference():
    sys.path.insert(0, os.path.join(HERE, "_shim"))
    sys.path.insert(0, REF)
    sys.modules.setdefault("turtle", types.SimpleNamespace(forward=None))
    import model.model as ref_model  # noqa: E402
    import model.online_class_unknown_targets as ref_online  # noqa: E402
    import model.pit_wrapper as ref_pit  # noqa: E402
    return ref_model, ref_online, ref_pit


def weights_sha(sd):
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v, dtype=np.float32).tobytes())
    return h.hexdigest()


def build(ref_model, cfg):
    net = ref_model.SeparationModel(**cfg)
    sd = synth.make_state_dict(cfg, SEED_W)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net.eval()
    return net, sd


def run_case(net, x, with_hooks=False, inference_kw=None):
    cap = {}
    hooks = []
    if with_hooks:
        hooks.append(net.TCN.LN.register_forward_hook(lambda m, i, o: cap.__setitem__("tcn_in", o.detach().clone())))
        hooks.append(net.TCN.TCN[0].register_forward_hook(lambda m, i, o: cap.__setitem__("blk0_res", o.detach().clone())))
        hooks.append(net.TCN.time_freq_attnetion[0].register_forward_hook(
            lambda m, i, o: cap.__setitem__("blk0_att", o.detach().clone())))
    with torch.no_grad():
        sep, vad, est = net(torch.from_numpy(x), inference_kw or {})
    for h in hooks:
        h.remove()
    out = dict(sep=sep.numpy(), vad=(vad.numpy() if torch.is_tensor(vad) else np.array(vad)),
               spectrum=net.spectrum.numpy(), masks_b=net.masks_b.numpy())
    out["est_re"] = est.real.numpy().astype(np.float32)
    out["est_im"] = est.imag.numpy().astype(np.float32)
    for k, v in cap.items():
        out[k] = v.numpy()
    return out


def main():
    ref_model, ref_online, ref_pit = import_reference()
    torch.set_num_threads(8)
    manifest = {}
    for cname, cfg in (("with_vad", pkg.CONFIG_WITH_VAD), ("without_vad", pkg.CONFIG_WITHOUT_VAD)):
        net, sd = build(ref_model, cfg)
        sha = weights_sha(sd)
        # the reference's own state_dict key contract (names + shapes), for the drop-in key test
        import json
        with open(os.path.join(HERE, f"state_dict_keys_{cname}.json"), "w") as f:
            json.dump([[k, list(v.shape)] for k, v in net.state_dict().items()], f)
        for case, B, N, seed in CASES:
            x, srcs = synth.make_batch(B, N, seed)
            out = run_case(net, x, with_hooks=(case == "small"))
            keep = dict(x=x, sources=srcs, sep=out["sep"], vad=out["vad"], spectrum=out["spectrum"],
                        masks_b=out["masks_b"])
            if case != "cfg":
                keep.update(est_re=out["est_re"], est_im=out["est_im"])
            if case == "small":
                keep.update(tcn_in=out["tcn_in"], blk0_res=out["blk0_res"], blk0_att=out["blk0_att"])
                # fp64 run of the same reference, for tolerance diagnosis
                net64 = ref_model.SeparationModel(**cfg).double()
                net64.load_state_dict({k: torch.from_numpy(v).double() for k, v in sd.items()}, strict=True)
                net64.eval()
                with torch.no_grad():
                    s64, v64, _ = net64(torch.from_numpy(x).double())
                keep.update(sep_f64=s64.numpy(), vad_f64=v64.numpy())
                # inference_kw path (model/model.py:444-457): smoothed VAD + masking of est
                ikw = dict(filter_signals_by_smo_vad=True, filter_signals_by_unsmo_vad=False,
                           length_smoothing_filter=3, threshold_activated_vad=0.5, return_smoothed_vad=True)
                o2 = run_case(net, x, inference_kw=ikw)
                keep.update(ikw_sep=o2["sep"], ikw_vad=o2["vad"])
            keep["weights_seed"] = np.array(SEED_W)
            keep["weights_sha256"] = np.array(sha)
            fn = os.path.join(HERE, f"golden_{cname}_{case}.npz")
            np.savez_compressed(fn, **keep)
            vad = out["vad"]
            margin = float(np.abs(vad - 0.5).min()) if vad.ndim else float("nan")
            manifest[f"{cname}_{case}"] = dict(B=B, N=N, seed=seed, vad_margin=margin, bytes=os.path.getsize(fn))
            print(cname, case, "vad margin", margin, "size", os.path.getsize(fn))

        # streaming wrapper golden (model/online_class_unknown_targets.py:72-105), 160 ms hop
        if cname == "with_vad":
            x, _ = synth.make_batch(2, 64000, 400)
            crit = ref_pit.PITLossWrapper(loss_func=torch.nn.L1Loss(), pit_from="pw_pt")
            with tempfile.TemporaryDirectory() as td:
                ons = ref_online.OnlineSaving(net, td, crit)
                ons.save_sec = 0.16
                ikw = dict(pkg.INFERENCE_KW_DEFAULTS)
                ons.calc_online(torch.from_numpy(x), "stream", 10 ** 6, ikw)  # sample_indx large: no wav writes
                online = ons.online_signal.numpy()
            fn = os.path.join(HERE, "golden_with_vad_stream.npz")
            np.savez_compressed(fn, x=x, online=online, save_sec=np.array(0.16), weights_seed=np.array(SEED_W))
            print("stream", online.shape, os.path.getsize(fn))

    # smoothing known-answer test (model/model.py:444-451), derived by hand and checked in tests
    np.savez_compressed(os.path.join(HERE, "golden_smoothing_kat.npz"),
                        vad=np.array([.9, .1, .7, .2, .3, .6, .55, .5], dtype=np.float32),
                        smoothed=np.array([1, 1, 0, 1, 1, 1, 1, 1], dtype=np.float32))
    import json
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
