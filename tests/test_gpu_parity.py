"""Parity of the HIP path (through the C ABI) with the reference's golden outputs and the oracle.

Gates: separated waveforms max-abs <= 1e-4 (fp32 path); thresholded VAD labels
bit-exact; SI-SDR within 0.01 dB. Kernel-level checks compare against plain PyTorch fp32 ops.
"""
import numpy as np
import pytest
import torch

from conftest import CASES, CONFIGS, config_of, load_golden

pytestmark = pytest.mark.gpu

SEP_TOL = 1e-4   # north_star: waveform max-abs
# VAD probabilities (the labels are compared bit-exact): the VAD head sees 10 log10 |X|^2 of near-silent
# bins, where any float32 FFT's rounding (~1e-7 of max |X|) moves the dB a lot; perturbing the reference
# STFT by 3e-8 max|X| already moves its own VAD probabilities by up to 6e-4 on the ragged golden
# (tests/test_oracle_golden.py::test_reference_vad_sensitivity), so 1e-3 is the honest bound.
VAD_PROB_TOL = 1e-3
DEV = "cuda"


_SD = {}


def _state_dict(cname):
    """Recipe weights (seed 1234) of config cname as float32 torch tensors (the oracle's copy)."""
    if cname not in _SD:
        from sep_tfanet_vad_amd import synth
        _SD[cname] = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(config_of(cname), 1234).items()}
    return _SD[cname]


def _model(cname, state_dicts):
    import sep_tfanet_vad_amd as pkg
    net = pkg.SeparationModel(**config_of(cname))
    net.load_state_dict(state_dicts[cname], strict=True)
    return net.eval().to(DEV)


@pytest.fixture(scope="module", params=["f16x3", "fp32"])
def models(request, state_dicts):
    out = {c: _model(c, state_dicts) for c in CONFIGS}
    for m in out.values():
        m.native_precision = request.param
    return out


def test_native_library_is_loaded():
    from sep_tfanet_vad_amd import native
    lib = native.load_library()
    assert lib.sepvad_abi_version() == 1
    assert torch.cuda.is_available()


@pytest.mark.parametrize("cname", CONFIGS)
@pytest.mark.parametrize("case", CASES)
def test_forward_matches_reference(cname, case, models):
    g = load_golden(cname, case)
    net = models[cname]
    x = torch.from_numpy(g["x"]).to(DEV)
    with torch.no_grad():
        sep, vad, est = net(x)
    torch.cuda.synchronize()
    sep, vad = sep.cpu().numpy(), vad.cpu().numpy()
    err = np.abs(sep - g["sep"]).max()
    assert err <= SEP_TOL, f"sep max-abs {err}"
    assert vad.shape == g["vad"].shape
    assert np.array_equal(vad >= 0.5, g["vad"] >= 0.5), "VAD labels differ"
    assert np.abs(vad - g["vad"]).max() <= VAD_PROB_TOL
    # side attributes and est (model/model.py:412,421,429,437), all errors collected, then gated at the tight bound
    # or at twice the reference's OWN float32 rounding noise (its fp32 golden vs the fp64 oracle on the same input),
    # whichever is larger: on the short ragged golden the reference's fp32 masks_b is 4.2e-4 and its est 1e-3 away
    # from fp64 (without_vad), so no fp32 implementation can meet a fixed 2e-4 there. Tight bounds: spectrum 1e-5
    # of its range on bins with |X| > 1e-3 max|X| (the dB of a bin moves by 8.7 |dX| / |X|), masks_b 2e-4,
    # mask_per_speaker 5e-5, est 1e-5 of its range.
    from oracle.torch_ref import OracleModel
    ref64 = OracleModel(config_of(cname), _state_dict(cname), torch.float64)
    _, _, e64 = ref64(torch.from_numpy(g["x"]))
    X = torch.stft(torch.from_numpy(g["x"]), 512, 256, 512, torch.hann_window(512), center=True, pad_mode="reflect",
                   return_complex=True)
    ok = (X.abs() > 1e-3 * X.abs().amax(dim=(1, 2), keepdim=True)).numpy()
    ok[:, 0, :] = True  # DC: exactly -100 dB times the gate in both
    mps = torch.sigmoid(torch.from_numpy(g["masks_b"])).reshape(net.mask_per_speaker.shape).numpy()
    rows = [("masks_b", net.masks_b.cpu().numpy(), g["masks_b"], ref64.masks_b.numpy(), None, 2e-4),
            ("spectrum", net.spectrum.cpu().numpy(), g["spectrum"], ref64.spectrum.numpy(), ok,
             1e-5 * np.abs(g["spectrum"]).max()),
            ("mask_per_speaker", net.mask_per_speaker.cpu().numpy(), mps, ref64.mask_per_speaker.numpy(), None, 5e-5)]
    if "est_re" in g:
        e = est.cpu()
        assert e.dtype == torch.complex64 and tuple(e.shape) == g["est_re"].shape
        ge = g["est_re"] + 1j * g["est_im"]
        rows.append(("est", e.numpy(), ge, e64.numpy(), None, 1e-5 * max(np.abs(g["est_re"]).max(), np.abs(g["est_im"]).max())))
    fails = []
    for name, ours, gold, f64, m, tight in rows:
        d_ours, d_ref = np.abs(ours - gold), np.abs(f64 - gold)
        if m is not None:
            d_ours, d_ref = d_ours[m], d_ref[m]
        err, noise = float(d_ours.max()), float(d_ref.max())
        if err > max(tight, 2.0 * noise):
            fails.append(f"{name}: {err:.3g} > max({tight:.3g}, 2 x reference fp32 noise {noise:.3g})")
    assert not fails, "; ".join(fails)


def test_strided_windows_match_contiguous(models):
    """forward on strided row views (streaming windows) == forward on their contiguous copies."""
    from sep_tfanet_vad_amd import synth
    full = torch.from_numpy(synth.make_batch(3, 40000, 950)[0]).to(DEV)
    win = full[:, 1000:1000 + 30000]
    assert not win.is_contiguous()
    net = models["with_vad"]
    with torch.no_grad():
        a, va, _ = net(win)
        b, vb, _ = net(win.contiguous())
    assert torch.equal(a, b) and torch.equal(va, vb)


@pytest.mark.parametrize("cname", CONFIGS)
def test_block_level_parity_vs_reference(cname, models):
    """Kernel-level localisation inside the fused TCN (sepvad_set_tcn_dump): TCN.LN output, block 0's
    DepthConv1d output and its TF_Attention output vs the reference module outputs captured by
    make_golden.py (tcn_in, blk0_res, blk0_att; model/model.py:333,144,207): max-abs within 1e-5 of each
    tensor's range (|values| reach 9: 1e-5 absolute is ~10 fp32 ulps there, and the TCN input inherits the
    dB amplification of tiny STFT bins, d dB = 8.7 |dX| / |X|)."""
    g = load_golden(cname, "small")
    h = models[cname].native_handle(DEV)
    if h.precision != "f16x3":
        pytest.skip("the block probe instantiates the fp16x3 kernel")
    tin, res, att = h.tcn_dump(torch.from_numpy(g["x"]).to(DEV))
    for name, v in (("tcn_in", tin), ("blk0_res", res), ("blk0_att", att)):
        err = np.abs(v.cpu().numpy() - g[name]).max()
        tol = 1e-5 * max(1.0, float(np.abs(g[name]).max()))
        assert err <= tol, f"{name}: max-abs {err} (tolerance {tol})"


@pytest.mark.parametrize("cname", CONFIGS)
def test_side_attributes_tight(cname, models):
    """self.spectrum on bins whose STFT magnitude exceeds 1e-2 (dB of tiny bins amplifies fp32 rounding:
    d dB = 8.7 |dX|/|X|) within 1e-5 of its range, self.masks_b within 2e-4, mask_per_speaker within 5e-5."""
    g = load_golden(cname, "cfg")
    net = models[cname]
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        net(x.to(DEV))
    X = torch.stft(x, 512, 256, 512, torch.hann_window(512), center=True, pad_mode="reflect", return_complex=True)
    ok = (X.abs() > 1e-2).numpy()
    ok[:, 0, :] = True  # DC: exactly -100 dB times the gate in both
    spec = net.spectrum.cpu().numpy()
    rng = np.abs(g["spectrum"]).max()
    e_spec = np.abs(spec - g["spectrum"])[ok].max()
    assert e_spec <= 1e-5 * rng, f"spectrum {e_spec} (range {rng})"
    e_mb = np.abs(net.masks_b.cpu().numpy() - g["masks_b"]).max()
    assert e_mb <= 2e-4, f"masks_b {e_mb}"
    mps = torch.sigmoid(torch.from_numpy(g["masks_b"])).reshape(net.mask_per_speaker.shape).numpy()
    e_m = np.abs(net.mask_per_speaker.cpu().numpy() - mps).max()
    assert e_m <= 5e-5, f"mask_per_speaker {e_m}"
