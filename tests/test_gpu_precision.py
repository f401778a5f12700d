"""Reduced-precision arms (BASELINE cfg 2 "bf16", cfg 5 "fp16 vs fp32 sweep"): the pointwise GEMMs
(reference model/model.py:104,114,324) with fp16 or bf16 operands, one product, fp32 accumulation;
everything else fp32. They cannot meet the fp32 parity gate (the fp32 reference is itself
2.7e-5 from fp64), so this is a measured tolerance against the fp32 oracle (oracle/torch_ref.py):

* separated-waveform max-abs and RMS error,
* SI-SDR delta (model/combined_loss.py:16-56 via metrics.hip, PIT over the two speakers) of the HIP output
  against the clean sources vs the oracle's own SI-SDR — the metric string's "within 0.01 dB",
* VAD label flips (p >= 0.5, model/model.py:449) vs the oracle.

The measured numbers are written to gpurun_out/precision_<arm>_<cfg>.json (DESIGN.md §4 records them);
the gates below are the recorded tolerances with headroom.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import REPO, config_of

pytestmark = pytest.mark.gpu

DEV = "cuda"
# arm -> (sep max-abs, mean |SI-SDR delta| dB, max |SI-SDR delta| dB, VAD flip fraction). Measured on
# MI355X (r02b, cfg2 / cfg5): f16 1.1e-4 / 1.5e-4, 1.1e-4 dB, 4.1e-4 dB, 6 / 32256; bf16 8.7e-4 / 1.0e-3,
# 9.6e-4 dB, 3.9e-3 dB, 42 / 32256; f16x3 5.1e-6, 1.6e-7 dB, 9.5e-7 dB, 0. bf16 stays inside the metric
# string's 0.01 dB SI-SDR gate; only the fp32-equivalent arms meet the 1e-4 waveform gate.
# f16x3: the default int8 weight lo plane of the fused TCN (3 B per weight); f16x3-f16lo / -e4m3lo: the fp16 and e4m3
# lo planes (MI355X r03l, cfg2: sep 2.9e-6 / 3.0e-6 / 3.1e-6, 0 flips each; tools/lo_plane_precision.py emulates them).
GATES = {"f16": (5e-4, 1e-3, 5e-3, 1e-3), "bf16": (5e-3, 5e-3, 1e-2, 1e-2), "f16x3": (1e-4, 1e-4, 1e-3, 1e-4),
         "f16x3-e4m3lo": (1e-4, 1e-4, 1e-3, 1e-4), "f16x3-f16lo": (1e-4, 1e-4, 1e-3, 1e-4)}
# cfg 5: 128 utterances per GPU (1024 over 8); long: 16 s files (T = 1001, groups of 32 workgroups)
CFGS = {"cfg2": (64, 32000), "cfg5": (128, 32000), "long": (2, 256000)}


@pytest.fixture(scope="module")
def oracle_runs(state_dicts):
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    torch.set_num_threads(max(1, min(32, os.cpu_count() or 1)))
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    out = {}
    for name, (B, N) in CFGS.items():
        x, srcs = synth.make_batch(B, N, 60_000 + B)
        xt = torch.from_numpy(x)
        sep, vad, _ = om(xt)
        out[name] = (xt, torch.from_numpy(srcs), sep, vad)
    return out


@pytest.fixture(scope="module")
def net(state_dicts):
    import sep_tfanet_vad_amd as pkg
    m = pkg.SeparationModel(**config_of("with_vad"))
    m.load_state_dict(state_dicts["with_vad"], strict=True)
    return m.eval().to(DEV)


@pytest.mark.parametrize("cfg", list(CFGS))
@pytest.mark.parametrize("arm", ["f16", "bf16", "f16x3", "f16x3-e4m3lo", "f16x3-f16lo"])
def test_precision_arm_tolerance(arm, cfg, net, oracle_runs):
    from sep_tfanet_vad_amd.metrics import permutation_invariant_si_sdr
    x, srcs, s_ref, v_ref = oracle_runs[cfg]
    net.native_precision = arm.split("-")[0]
    net.native_weight_lo = arm.split("-")[1][:-2] if "-" in arm else "i8"
    try:
        with torch.no_grad():
            s, v, _ = net(x.to(DEV))
        assert net.native_handle(DEV).fused_status(), "the fused TCN did not run"
    finally:
        net.native_precision = "f16x3"
        net.native_weight_lo = "i8"
    err = (s.cpu() - s_ref).abs()
    tgt = srcs.to(DEV)
    sd_hip, _ = permutation_invariant_si_sdr(s, tgt)
    sd_ref, _ = permutation_invariant_si_sdr(s_ref.to(DEV), tgt)
    dsd = (sd_hip - sd_ref).abs().cpu()
    flips = int(((v.cpu() >= 0.5) != (v_ref >= 0.5)).sum())
    rec = dict(arm=arm, cfg=cfg, B=int(x.shape[0]), N=int(x.shape[1]), sep_maxabs=float(err.max()),
               sep_rms=float(err.pow(2).mean().sqrt()), sisdr_delta_mean=float(dsd.mean()),
               sisdr_delta_max=float(dsd.max()), sisdr_ref_mean=float(sd_ref.mean()), vad_flips=flips,
               vad_labels=int(v_ref.numel()), vad_prob_maxabs=float((v.cpu() - v_ref).abs().max()))
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"precision_{arm}_{cfg}.json"), "w") as f:
        json.dump(rec, f)
    print(json.dumps(rec))
    g = GATES[arm]
    assert np.isfinite(rec["sep_maxabs"])
    assert rec["sep_maxabs"] <= g[0], rec
    assert rec["sisdr_delta_mean"] <= g[1] and rec["sisdr_delta_max"] <= g[2], rec
    assert flips <= g[3] * rec["vad_labels"], rec
