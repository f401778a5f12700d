"""BASELINE configs beyond the headline one, as parity cases:
  cfg 4: 8 s reverberant mixtures (image-method RIRs, RT60 U[0.2, 0.6]) -> T = 251, 8 workgroups per group;
  cfg 5: GEMM precision sweep (fp32 MFMA vs fp16x3 split) against the fp32 oracle on cfg-2 inputs.
Both against oracle/torch_ref.py (fp32, CPU) at sizes it finishes in seconds."""
import numpy as np
import pytest
import torch

from conftest import check_vad_labels, config_of

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEP_TOL = 1e-4


def _net(cname, state_dicts, precision):
    import sep_tfanet_vad_amd as pkg
    net = pkg.SeparationModel(**config_of(cname))
    net.load_state_dict(state_dicts[cname], strict=True)
    net = net.eval().to(DEV)
    net.native_precision = precision
    return net


def _check(sep, vad, s_ref, v_ref):
    err = np.abs(sep - s_ref).max()
    assert err <= SEP_TOL, f"sep max-abs {err}"
    check_vad_labels(vad, v_ref)
    return err


def test_cfg4_reverberant_8s(state_dicts):
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    x, _ = synth.make_reverb_batch(2, 64000, 9100, rir_samples=4000)
    net = _net("with_vad", state_dicts, "f16x3")
    with torch.no_grad():
        sep, vad, _ = net(torch.from_numpy(x).to(DEV))
    assert net.native_handle(DEV).fused_status()  # T = 251 runs fused (G = 8)
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    s_ref, v_ref, _ = om(torch.from_numpy(x))
    _check(sep.cpu().numpy(), vad.cpu().numpy(), s_ref.numpy(), v_ref.numpy())


def test_cfg4_full_batch_sampled(state_dicts):
    """cfg 4 at its per-GPU batch (B = 64 reverberant 8 s mixtures, T = 251) in one forward, a sample of four
    utterances against the oracle (the oracle runs only those), and the batch-invariance of the sample."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    x, _ = synth.make_reverb_batch(64, 64000, 9200, rir_samples=4000)
    net = _net("with_vad", state_dicts, "f16x3")
    sub = [0, 21, 42, 63]
    with torch.no_grad():
        sep, vad, _ = net(torch.from_numpy(x).to(DEV))
        sep_s, vad_s, _ = net(torch.from_numpy(x[sub]).to(DEV))
    assert net.native_handle(DEV).fused_status()
    assert torch.equal(sep[sub], sep_s) and torch.equal(vad[sub], vad_s)
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    s_ref, v_ref, _ = om(torch.from_numpy(x[sub]))
    err = _check(sep_s.cpu().numpy(), vad_s.cpu().numpy(), s_ref.numpy(), v_ref.numpy())
    print(f"cfg4 B=64 sample: sep max-abs vs fp32 oracle {err:.2e}")


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_cfg5_precision_sweep(precision, state_dicts):
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    x, _ = synth.make_batch(4, 32000, 5150)
    net = _net("with_vad", state_dicts, precision)
    with torch.no_grad():
        sep, vad, _ = net(torch.from_numpy(x).to(DEV))
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    s_ref, v_ref, _ = om(torch.from_numpy(x))
    err = _check(sep.cpu().numpy(), vad.cpu().numpy(), s_ref.numpy(), v_ref.numpy())
    print(f"cfg5 {precision}: sep max-abs vs fp32 oracle {err:.2e}")


def test_distinct_stft_windows(state_dicts):
    """A checkpoint whose spec_input and spec_output windows differ (model/model.py:383-385,408-409): the
    spectrum / TCN input use spec_input's window, est and the output use spec_output's. The fused front end
    then runs two transforms per frame and keeps the dB spectrum for the side pass. vs the oracle."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    sd = dict(state_dicts["with_vad"])
    n = torch.arange(512, dtype=torch.float32)
    sd["spec_input.spec.window"] = 0.54 - 0.46 * torch.cos(2 * torch.pi * n / 512)  # periodic Hamming
    x, _ = synth.make_batch(3, 20000, 5170)
    net = _net("with_vad", {"with_vad": sd}, "f16x3")
    with torch.no_grad():
        sep, vad, _ = net(torch.from_numpy(x).to(DEV))
    om = OracleModel(config_of("with_vad"), sd, torch.float32)
    s_ref, v_ref, _ = om(torch.from_numpy(x))
    _check(sep.cpu().numpy(), vad.cpu().numpy(), s_ref.numpy(), v_ref.numpy())
    spec = net.spectrum.cpu().numpy()
    sref = om.spectrum.numpy() if hasattr(om, "spectrum") else None
    if sref is not None:
        X = torch.stft(torch.from_numpy(x), 512, 256, 512, sd["spec_input.spec.window"], center=True,
                       pad_mode="reflect", return_complex=True)
        ok = (X.abs() > 1e-2).numpy()
        assert np.abs(spec - sref)[ok].max() <= 1e-5 * np.abs(sref).max()
