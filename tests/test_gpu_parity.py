"""Parity of the HIP path (through the C ABI) with the reference's golden outputs and the oracle.

Gates: separated waveforms max-abs <= 1e-4 (fp32 path); thresholded VAD labels
bit-exact; SI-SDR within 0.01 dB. Kernel-level checks compare against plain PyTorch fp32 ops.
"""
import os

import numpy as np
import pytest
import torch

from conftest import CASES, CONFIGS, check_vad_labels, config_of, load_golden

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


# f16x3 (default: int8 weight lo plane in the fused TCN), f16x3 with the fp16 / e4m3 lo planes, fp32 MFMA
@pytest.fixture(scope="module", params=["f16x3", "f16x3-f16lo", "f16x3-e4m3lo", "fp32"])
def models(request, state_dicts):
    out = {c: _model(c, state_dicts) for c in CONFIGS}
    for m in out.values():
        m.native_precision = request.param.split("-")[0]
        m.native_weight_lo = request.param.split("-")[1][:-2] if "-" in request.param else "i8"
    return out


def test_native_library_is_loaded():
    from sep_tfanet_vad_amd import native
    lib = native.load_library()
    assert lib.sepvad_abi_version() == 1
    if not os.environ.get("SEPVAD_LIB"):  # the tested binary is built from this tree's sources
        assert native.build_id() == native.tree_build_id(), (native.build_id(), native.tree_build_id())
    print(f"libsepvad build id {native.build_id()}")
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
        # the opt-in e4m3 weight lo plane (2^-16-relative weights) moves est by up to 1.4e-5 of its range: its gate is 2e-5
        rel = 2e-5 if net.native_weight_lo == "e4m3" else 1e-5
        rows.append(("est", e.numpy(), ge, e64.numpy(), None, rel * max(np.abs(g["est_re"]).max(), np.abs(g["est_im"]).max())))
    fails = []
    for name, ours, gold, f64, m, tight in rows:
        d_ours, d_ref = np.abs(ours - gold), np.abs(f64 - gold)
        if m is not None:
            d_ours, d_ref = d_ours[m], d_ref[m]
        err, noise = float(d_ours.max()), float(d_ref.max())
        if err > max(tight, 2.0 * noise):
            fails.append(f"{name}: {err:.3g} > max({tight:.3g}, 2 x reference fp32 noise {noise:.3g})")
    assert not fails, "; ".join(fails)


@pytest.mark.parametrize("cname", CONFIGS)
def test_inference_kw_smoothed_vad(cname, models):
    g = load_golden(cname, "small")
    ikw = dict(filter_signals_by_smo_vad=True, filter_signals_by_unsmo_vad=False, length_smoothing_filter=3,
               threshold_activated_vad=0.5, return_smoothed_vad=True)
    with torch.no_grad():
        sep, vad, _ = models[cname](torch.from_numpy(g["x"]).to(DEV), ikw)
    assert tuple(vad.shape) == g["ikw_vad"].shape  # [B, 2, 1, T]
    assert np.array_equal(vad.cpu().numpy(), g["ikw_vad"])
    assert np.abs(sep.cpu().numpy() - g["ikw_sep"]).max() <= SEP_TOL


def test_inference_kw_variants_vs_oracle(models, state_dicts):
    """unsmoothed-filter flag, threshold, length_smoothing_filter=5 (no effect) vs the oracle."""
    from oracle.torch_ref import OracleModel
    g = load_golden("with_vad", "small")
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"])
    x = torch.from_numpy(g["x"])
    for ikw in (dict(filter_signals_by_smo_vad=False, filter_signals_by_unsmo_vad=True, length_smoothing_filter=5,
                     threshold_activated_vad=0.4, return_smoothed_vad=False),
                dict(filter_signals_by_smo_vad=False, filter_signals_by_unsmo_vad=False, length_smoothing_filter=3,
                     threshold_activated_vad=0.6, return_smoothed_vad=True)):
        s_ref, v_ref, _ = om(x, ikw)
        with torch.no_grad():
            s, v, _ = models["with_vad"](x.to(DEV), ikw)
        assert tuple(v.shape) == tuple(v_ref.shape)
        assert np.abs(s.cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
        if ikw["return_smoothed_vad"]:
            assert np.array_equal(v.cpu().numpy(), v_ref.numpy())


def test_stft_kernel_vs_torch(models):
    """STFT kernel vs torch.stft (fp32, on the GPU) — the op torchaudio.Spectrogram runs."""
    h = models["with_vad"].native_handle(DEV)
    for N in (8000, 12345, 32000, 257):
        x = torch.rand(3, N, device=DEV) * 1.8 - 0.9
        X, spec = h.stft(x)
        win = torch.hann_window(512, device=DEV)
        Xr = torch.stft(x, 512, 256, 512, win, center=True, pad_mode="reflect", normalized=False, onesided=True,
                        return_complex=True)
        Xr[:, 0, :] = 0
        assert X.shape == Xr.shape
        assert (X - Xr).abs().max().item() <= 2e-5 * Xr.abs().max().item() + 1e-5
        sr = 10 * torch.log10(torch.clamp(Xr.abs() ** 2, min=1e-10))
        ok = Xr.abs() > 1e-2  # dB of tiny bins amplifies fp32 rounding (d dB = 8.7 |dX|/|X|)
        assert (spec - sr)[ok].abs().max().item() <= 2e-3


def test_istft_kernel_vs_torch(models):
    h = models["with_vad"].native_handle(DEV)
    for N in (8000, 12345, 32000):
        T = 1 + N // 256
        est = torch.randn(4, 257, T, device=DEV, dtype=torch.complex64)
        y = h.istft(est, N)
        win = torch.hann_window(512, device=DEV)
        yr = torch.istft(est, 512, 256, 512, win, center=True, normalized=False, onesided=True, length=N)
        assert (y - yr).abs().max().item() <= 1e-5 * max(1.0, yr.abs().max().item())


def test_stft_istft_round_trip(models):
    h = models["with_vad"].native_handle(DEV)
    x = torch.rand(2, 32000, device=DEV) * 1.8 - 0.9
    X, _ = h.stft(x)
    # DC was removed: the round trip reproduces x minus its per-frame DC contribution; compare with torch
    win = torch.hann_window(512, device=DEV)
    yr = torch.istft(X, 512, 256, 512, win, center=True, length=32000)
    y = h.istft(X, 32000)
    assert (y - yr).abs().max().item() <= 1e-5


PROD_N = (257, 8000, 12345, 32000, 261888)


@pytest.mark.parametrize("N", PROD_N)
def test_stft_gate_kernel_vs_torch(models, N):
    """The forward's own front end, k_stft_gate (sepvad_stft_gate_test), vs torch.stft + AmplitudeToDB
    (model/model.py:16-25,408-412): X within 2e-5 of its range, dB within 2e-3 on bins |X| > 1e-2 (d dB =
    8.7 |dX| / |X|), T = 2 .. 1024 frames."""
    h = models["with_vad"].native_handle(DEV)
    B = 3 if N <= 32000 else 1
    g = torch.Generator(device="cpu").manual_seed(N)
    x = (torch.rand(B, N, generator=g) * 1.8 - 0.9).to(DEV)
    X, db = h.stft_fused(x)
    win = torch.hann_window(512, device=DEV)
    Xr = torch.stft(x, 512, 256, 512, win, center=True, pad_mode="reflect", normalized=False, onesided=True,
                    return_complex=True)
    Xr[:, 0, :] = 0
    assert X.shape == Xr.shape and db.shape == Xr.shape
    assert (X - Xr).abs().max().item() <= 2e-5 * Xr.abs().max().item() + 1e-5
    sr = 10 * torch.log10(torch.clamp(Xr.abs() ** 2, min=1e-10))
    ok = Xr.abs() > 1e-2
    ok[:, 0, :] = True  # DC: -100 dB in both
    assert (db - sr)[ok].abs().max().item() <= 2e-3


@pytest.mark.parametrize("N", PROD_N)
def test_istft_pair_kernel_vs_torch(models, N):
    """The forward's own back end, k_istft_pair (sepvad_istft_pair_test): est = X sigmoid(m) per speaker within
    1e-6 of its range and y = torch.istft(est, length=N) within 1e-5 (model/model.py:429-460), X the DC-zeroed
    STFT of a real signal (as in the forward), pre-sigmoid masks in [-6, 6]."""
    h = models["with_vad"].native_handle(DEV)
    B = 2 if N <= 32000 else 1
    g = torch.Generator(device="cpu").manual_seed(7 + N)
    x = (torch.rand(B, N, generator=g) * 1.8 - 0.9).to(DEV)
    win = torch.hann_window(512, device=DEV)
    X = torch.stft(x, 512, 256, 512, win, center=True, pad_mode="reflect", return_complex=True)
    X[:, 0, :] = 0
    T = X.shape[-1]
    m = (torch.rand(B, 2, 257, T, generator=g) * 12 - 6).to(DEV)
    y, est = h.istft_pair(X, m, N)
    er = X[:, None] * torch.sigmoid(m)
    assert (est - er).abs().max().item() <= 1e-6 * er.abs().max().item()
    yr = torch.istft(er.reshape(B * 2, 257, T), 512, 256, 512, win, center=True, length=N).reshape(B, 2, N)
    assert (y - yr).abs().max().item() <= 1e-5 * max(1.0, yr.abs().max().item())


@pytest.mark.parametrize("cname", CONFIGS)
def test_full_batch_properties(cname, models, state_dicts):
    """BASELINE cfg shape B=64, N=32000: a sample of utterances vs the oracle, batch invariance
    (bitwise), determinism, and SI-SDR within 0.01 dB of the oracle against the clean sources."""
    from oracle.torch_ref import OracleModel, si_sdr
    from sep_tfanet_vad_amd import synth
    B, N = 64, 32000
    x, srcs = synth.make_batch(B, N, 5000)
    xd = torch.from_numpy(x).to(DEV)
    net = models[cname]
    with torch.no_grad():
        sep, vad, est = net(xd)
        sep2, vad2, _ = net(xd)
        sub = [0, 17, 63]
        sep_sub, vad_sub, _ = net(xd[sub])
    torch.cuda.synchronize()
    assert torch.equal(sep, sep2) and torch.equal(vad, vad2)           # deterministic
    assert torch.equal(sep[sub], sep_sub) and torch.equal(vad[sub], vad_sub)  # batch invariant
    om = OracleModel(config_of(cname), state_dicts[cname], torch.float32)
    s_ref, v_ref, _ = om(torch.from_numpy(x[sub]))
    assert np.abs(sep_sub.cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
    check_vad_labels(vad_sub.cpu().numpy(), v_ref.numpy(), where=f"B=64 {cname}")
    # SI-SDR (reference model/combined_loss.py:16-56) of each output vs the matching source
    tgt = torch.from_numpy(srcs[sub])
    d = (si_sdr(sep_sub.cpu(), tgt) - si_sdr(s_ref, tgt)).abs().max().item()
    assert d <= 0.01, f"SI-SDR differs by {d} dB"


def test_streams_and_devices_do_not_leak_state(models):
    """Two handles / back-to-back shapes: results depend only on the inputs."""
    g = load_golden("with_vad", "ragged")
    net = models["with_vad"]
    with torch.no_grad():
        a, _, _ = net(torch.from_numpy(g["x"]).to(DEV))
        net(torch.rand(5, 48000, device=DEV))  # grow the workspace
        b, _, _ = net(torch.from_numpy(g["x"]).to(DEV))
    assert torch.equal(a, b)


def test_batch_split_is_bitwise_identical(models):
    """sepvad_set_split: utterance chunks on concurrent internal streams give the same bits."""
    from sep_tfanet_vad_amd import synth
    x = torch.from_numpy(synth.make_batch(13, 20000, 900)[0]).to(DEV)
    net = models["with_vad"]
    h = net.native_handle(DEV)
    outs = []
    for n in (1, 2, 3, 4):
        h.set_split(n)
        with torch.no_grad():
            sep, vad, est = net(x)
        outs.append((sep.clone(), vad.clone(), est.clone(), net.masks_b.clone(), net.spectrum.clone()))
    h.set_split(1)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


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
