"""The fused persistent TCN (csrc/tcn_kernel.h, one launch for all 24 blocks) against the oracle, the
reference goldens and the multi-kernel schedule, over the group sizes it supports (G = ceil(T/32) =
1..32 workgroups per utterance: one-wave and LDS statistic finishes, one- and two-pass moment polls), batches larger than one resident wave of groups, and the fallback.

Tolerances: separated waveforms max-abs <= 1e-4 vs the reference/oracle (north_star); the two
schedules differ only in the order of fp32 partial sums, so the waveforms agree to 1e-5. The VAD
probabilities agree to 1e-4: the fused schedule computes the VAD conv1_1 as the output head's second GEMM (fp16x3
MFMA, channel sums in MFMA order), the other with k_vad1 (VALU, lane-tree order), and the VAD head
amplifies rounding (tests/test_oracle_golden.py::test_reference_vad_sensitivity).
"""
import numpy as np
import pytest
import torch

from conftest import CONFIGS, check_vad_labels, config_of, load_golden

pytestmark = pytest.mark.gpu

SEP_TOL = 1e-4
VAD_PROB_TOL = 1e-3  # VAD probabilities; labels bit-exact (see test_gpu_parity.VAD_PROB_TOL)
SCHED_TOL = 1e-5
VAD_SCHED_TOL = 1e-4
# the fused TCN's default int8 weight lo plane (include/sepvad.h SEPVAD_WLO_I8) vs its fp16 lo plane (the multi-kernel
# schedule's weights): different weights below 2^-20 of a row's largest, so the two fp32-equivalent results differ by
# up to about the fp32 reference's own distance from fp64 (2.7e-5 on the waveforms), not by summation
# order alone; VAD probabilities within the VAD head's own sensitivity (VAD_PROB_TOL)
LO8_TOL = 4e-5
DEV = "cuda"


@pytest.fixture(scope="module")
def nets(state_dicts):
    import sep_tfanet_vad_amd as pkg
    out = {}
    for c in CONFIGS:
        net = pkg.SeparationModel(**config_of(c))
        net.load_state_dict(state_dicts[c], strict=True)
        net = net.eval().to(DEV)
        net.native_precision = "f16x3"
        out[c] = net
    return out


def _run(net, x, fused, ikw=None, wlo="i8"):
    net.native_weight_lo = wlo
    h = net.native_handle(DEV)
    h.set_fused(fused)
    try:
        with torch.no_grad():
            sep, vad, est = net(x, ikw) if ikw is not None else net(x)
        used = h.fused_status()  # synchronises; raises if a hand-off wait gave up
    finally:
        h.set_fused(True)
        net.native_weight_lo = "i8"
    return sep, vad, est, used


def _check_schedules(net, x, sf, vf):
    """sf, vf: the fused TCN with the default int8 weight lo plane. The fused kernel with the fp16 lo plane (the
    multi-kernel schedule's weights) vs the multi-kernel schedule at SCHED_TOL; the int8 lo plane vs it at LO8_TOL."""
    s16, v16, _, used = _run(net, x, True, wlo="f16")
    assert used
    sm, vm, em, used_m = _run(net, x, False)
    assert not used_m
    assert (s16 - sm).abs().max().item() <= SCHED_TOL
    assert (v16 - vm).abs().max().item() <= VAD_SCHED_TOL
    assert (sf - s16).abs().max().item() <= LO8_TOL
    assert (vf - v16).abs().max().item() <= VAD_PROB_TOL
    return sm, vm, em


@pytest.mark.parametrize("cname", CONFIGS)
@pytest.mark.parametrize("case", ["small", "ragged", "cfg"])
def test_fused_matches_reference_goldens(cname, case, nets):
    g = load_golden(cname, case)
    sep, vad, _, used = _run(nets[cname], torch.from_numpy(g["x"]).to(DEV), True)
    assert used, "the fused TCN did not run"
    sep, vad = sep.cpu().numpy(), vad.cpu().numpy()
    assert np.abs(sep - g["sep"]).max() <= SEP_TOL
    assert np.array_equal(vad >= 0.5, g["vad"] >= 0.5)
    assert np.abs(vad - g["vad"]).max() <= VAD_PROB_TOL


@pytest.mark.parametrize("cname", CONFIGS)
@pytest.mark.parametrize("N", [300, 2000, 8000, 12345, 32000, 48000, 64000, 96000, 140000, 200000, 261888])
def test_fused_vs_multikernel_and_oracle(cname, N, nets, state_dicts):
    """G = 1, 1, 1, 2, 4, 6, 8, 12, 18, 25, 32 workgroups per utterance (T = 2 at the smallest) (G > 16: GroupNorm words finished
    from LDS; G > 23: the moment words polled in two passes; T = 1024 at the largest)."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    B = 3
    if N < 1000:  # too short for the gated synthetic sources (an all-silent mixture has no min-max scale)
        x = torch.rand(B, N, generator=torch.Generator().manual_seed(N)) * 1.8 - 0.9
    else:
        x = torch.from_numpy(synth.make_batch(B, N, 31 + N)[0])
    net = nets[cname]
    sf, vf, ef, used = _run(net, x.to(DEV), True)
    assert used
    sm, vm, em = _check_schedules(net, x.to(DEV), sf, vf)
    assert (ef - em).abs().max().item() <= 1e-3
    om = OracleModel(config_of(cname), state_dicts[cname], torch.float32)
    s_ref, v_ref, _ = om(x[:1])
    assert np.abs(sf[:1].cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
    check_vad_labels(vf[:1].cpu().numpy(), v_ref.numpy())


def test_persistent_groups_cover_large_batches(nets):
    """B above one resident wave of groups (64 groups of 4 at T=126): groups loop over utterances;
    results are bitwise independent of batch composition and deterministic."""
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    x = torch.from_numpy(synth.make_batch(150, 32000, 4242)[0]).to(DEV)
    a, va, _, used = _run(net, x, True)
    assert used
    b, vb, _, _ = _run(net, x, True)
    assert torch.equal(a, b) and torch.equal(va, vb)
    sub = [0, 63, 64, 127, 128, 149]
    c, vc, _, _ = _run(net, x[sub], True)
    assert torch.equal(a[sub], c) and torch.equal(va[sub], vc)
    _check_schedules(net, x[sub], c, vc)


def test_epoch_budget_small_stack(state_dicts, monkeypatch):
    """Hand-off epochs of one launch (api.hip enqueue_chunk): 1 + per utterance 4 per block + 1 for the output head's
    P5 round, below 2^12. A 2-block stack (layer 2, stack 1) with 8 groups per launch (SEPVAD_TCN_MAX_GROUPS) and
    SEPVAD_TCN_MAX_ITER unset: each group takes max_iter = 4094 // 9 = 454 utterances per launch, and the batch needs a
    second launch, whose tags the first would have repeated under the round-4 budget (4094 // 8 = 511 utterances:
    1 + 511 * 9 > 4095). Outputs equal the multi-kernel schedule's on every utterance."""
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    monkeypatch.delenv("SEPVAD_TCN_MAX_ITER", raising=False)
    cfg = dict(config_of("with_vad"), layer=2, stack=1)
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 77).items()}
    net = pkg.SeparationModel(**cfg)
    net.load_state_dict(sd, strict=True)
    net = net.eval().to(DEV)
    net.native_precision = "f16x3"
    B, N = 8 * 454 + 100, 2000  # T = 8: one workgroup per utterance
    x = torch.rand(B, N, generator=torch.Generator().manual_seed(5)) * 1.8 - 0.9
    monkeypatch.setenv("SEPVAD_TCN_MAX_GROUPS", "8")
    sf, vf, _, used = _run(net, x.to(DEV), True)
    assert used
    monkeypatch.delenv("SEPVAD_TCN_MAX_GROUPS")
    sm, vm, _, used_m = _run(net, x.to(DEV), False)
    assert not used_m
    assert (sf - sm).abs().max().item() <= LO8_TOL
    assert (vf - vm).abs().max().item() <= VAD_PROB_TOL


def _run_slices(net, x, slices, monkeypatch, prec="f16x3"):
    """One forward with the fused TCN forced to `slices` 32-frame slices per workgroup (SEPVAD_TCN_SLICES)."""
    monkeypatch.setenv("SEPVAD_TCN_SLICES", str(slices))
    net.native_precision = prec
    h = net.native_handle(DEV)
    try:
        with torch.no_grad():
            sep, vad, est = net(x)
        used = h.fused_slices()
    finally:
        monkeypatch.delenv("SEPVAD_TCN_SLICES")
        net.native_precision = "f16x3"
    return sep, vad, est, used


@pytest.mark.parametrize("cname", CONFIGS)
@pytest.mark.parametrize("N", [12345, 32000, 48000, 64000, 96000, 130816])
def test_two_slices_bitwise_equal_one_slice(cname, N, nets, monkeypatch):
    """Two-slice workgroups (tcn_kernel.h NSL = 2: 64 frames, one weight stream for both 32-frame tiles, the depthwise conv
    and res_out GEMM in two K halves) against one-slice workgroups: every member statistic is reduced in the one-slice
    order, so sep, vad and est are bitwise equal. G = 2, 4, 6, 8, 12, 16 members (T = 49 .. 512), both LN modes
    (recursive: config_with_vad, residual: config_without_vad)."""
    from sep_tfanet_vad_amd import synth
    x = torch.from_numpy(synth.make_batch(3, N, 900 + N)[0]).to(DEV)
    s1, v1, e1, u1 = _run_slices(nets[cname], x, 1, monkeypatch)
    s2, v2, e2, u2 = _run_slices(nets[cname], x, 2, monkeypatch)
    assert (u1, u2) == (1, 2)
    assert torch.equal(s1, s2) and torch.equal(v1, v2) and torch.equal(e1, e2)


@pytest.mark.parametrize("variant", ["no_tf_attention", "no_ln"])
@pytest.mark.parametrize("N", [32000, 130816])
def test_two_slices_bitwise_other_configs(variant, N, monkeypatch):
    """Two-slice vs one-slice workgroups on configurations the shipped configs do not reach: without
    TF-attention (model/model.py:345-346 skipped; the two-slice kernel keeps its gates in dead-H storage and skips the
    gating multiply) and with neither recursive nor residual LN (o = o + r, model/model.py:351-352: the LD_ADD
    instantiation) -- the reference constructor's defaults (model/model.py:362-366). Bitwise equal, and within the
    waveform gate of the fp32 oracle on utterance 0 (VAD labels bit-exact)."""
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    cfg = dict(config_of("with_vad"), tf_attention=False) if variant == "no_tf_attention" else \
        dict(config_of("with_vad"), apply_recursive_ln=False, apply_residual_ln=False)
    net = pkg.SeparationModel(**cfg)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 31).items()}, strict=True)
    net = net.eval().to(DEV)
    x = torch.from_numpy(synth.make_batch(3, N, 606 + N)[0]).to(DEV)
    s1, v1, e1, u1 = _run_slices(net, x, 1, monkeypatch)
    s2, v2, e2, u2 = _run_slices(net, x, 2, monkeypatch)
    assert (u1, u2) == (1, 2)
    assert torch.equal(s1, s2) and torch.equal(v1, v2) and torch.equal(e1, e2)
    from oracle.torch_ref import OracleModel
    om = OracleModel(cfg, {k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 31).items()}, torch.float32)
    s_ref, v_ref, _ = om(x[:1].cpu())
    assert np.abs(s1[:1].cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
    check_vad_labels(v1[:1].cpu().numpy(), v_ref.numpy())


@pytest.mark.parametrize("N", [32000, 130816])
def test_two_slices_int8_and_fp16_lo_planes_bitwise(N, nets, monkeypatch):
    """Two-slice workgroups stream the int8 lo plane's values as fp16 (api.hip twfq: no widening VALU beside the MFMAs);
    SEPVAD_TCN_WQ16=0 streams the int8 bytes and widens them in registers (exact). Same MFMA operands: equal bits."""
    from sep_tfanet_vad_amd import synth
    x = torch.from_numpy(synth.make_batch(3, N, 4242)[0]).to(DEV)
    net = nets["with_vad"]
    monkeypatch.setenv("SEPVAD_TCN_WQ16", "0")
    si, vi, ei, ui = _run_slices(net, x, 2, monkeypatch)
    monkeypatch.setenv("SEPVAD_TCN_WQ16", "1")
    sf, vf, ef, uf = _run_slices(net, x, 2, monkeypatch)
    assert (ui, uf) == (2, 2)
    assert torch.equal(si, sf) and torch.equal(vi, vf) and torch.equal(ei, ef)


@pytest.mark.parametrize("prec", ["bf16", "f16"])
def test_two_slices_reduced_precision_arms(prec, nets, monkeypatch):
    """The single-product arms (BASELINE cfg 2 bf16, cfg 5 fp16) on two-slice workgroups: bitwise the one-slice
    kernel's outputs."""
    from sep_tfanet_vad_amd import synth
    x = torch.from_numpy(synth.make_batch(4, 32000, 77)[0]).to(DEV)
    net = nets["with_vad"]
    s1, v1, _, u1 = _run_slices(net, x, 1, monkeypatch, prec)
    s2, v2, _, u2 = _run_slices(net, x, 2, monkeypatch, prec)
    assert (u1, u2) == (1, 2)
    assert torch.equal(s1, s2) and torch.equal(v1, v2)


def test_two_slices_chosen_past_one_round_and_repeatable(nets):
    """The launch takes two-slice workgroups once one-slice groups need more than one round of the chip (B = 128 at
    T = 126: 512 members on 256 CUs), one-slice below; the two-slice results are bitwise repeatable run to run and
    equal the one-slice results of the same utterances in a small batch (batch invariance across the two kernels)."""
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    h = net.native_handle(DEV)
    x = torch.from_numpy(synth.make_batch(128, 32000, 4343)[0]).to(DEV)
    outs = []
    for _ in range(3):
        with torch.no_grad():
            outs.append(net(x))
        assert h.fused_slices() == 2
    for o in outs[1:]:
        for a_, b_ in zip(outs[0], o):
            assert torch.equal(a_, b_)
    sub = [0, 1, 63, 64, 127]
    with torch.no_grad():
        small = net(x[sub])
    assert h.fused_slices() == 1
    for a_, b_ in zip(outs[0], small):
        assert torch.equal(a_[sub], b_)


def test_remainder_groups_span_xcds_bitwise(nets, monkeypatch):
    """All groups the chip holds: at T = 188 (G = 6, two-slice workgroups, 3 per group) the chip holds 85 groups; the
    kernel puts 80 of them on one XCD each and the remaining 5 on consecutive blocks (their hand-offs write through).
    Bitwise the outputs of the round-4 launch shape (SEPVAD_TCN_ALIGN8=1: 80 groups) and of a small batch of the same
    utterances (one-slice groups)."""
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    h = net.native_handle(DEV)
    x = torch.from_numpy(synth.make_batch(100, 48000, 5757)[0]).to(DEV)
    outs = {}
    for a8 in ("0", "1"):
        monkeypatch.setenv("SEPVAD_TCN_ALIGN8", a8)
        with torch.no_grad():
            outs[a8] = net(x)
        assert h.fused_slices() == 2
    monkeypatch.delenv("SEPVAD_TCN_ALIGN8")
    for a_, b_ in zip(outs["0"], outs["1"]):
        assert torch.equal(a_, b_)
    sub = [0, 84, 85, 99]  # group 0, the last remainder group, and the second round
    with torch.no_grad():
        small = net(x[sub])
    for a_, b_ in zip(outs["0"], small):
        assert torch.equal(a_[sub], b_)


def test_inference_kw_on_fused(nets):
    g = load_golden("with_vad", "small")
    ikw = dict(filter_signals_by_smo_vad=True, filter_signals_by_unsmo_vad=False, length_smoothing_filter=3,
               threshold_activated_vad=0.5, return_smoothed_vad=True)
    sep, vad, _, used = _run(nets["with_vad"], torch.from_numpy(g["x"]).to(DEV), True, ikw)
    assert used
    assert np.array_equal(vad.cpu().numpy(), g["ikw_vad"])
    assert np.abs(sep.cpu().numpy() - g["ikw_sep"]).max() <= SEP_TOL


def test_long_utterances_fall_back(nets):
    """T > 8192 (N >= 2097152, 131 s) does not fit one group of 256: the multi-kernel schedule runs."""
    x = torch.rand(1, 2097152, device=DEV) * 1.8 - 0.9
    _, _, _, used = _run(nets["with_vad"], x, True)
    assert not used


@pytest.mark.parametrize("N", [262144, 480000, 960000, 1048320, 2000000, 2096896])
def test_whole_file_forwards_stay_fused(N, nets, state_dicts):
    """only_inference.py:90-91 forwards a whole file (model/model.py:402-461 has no length limit): 16.4 s, 30 s, 60 s,
    65.5 s, 125 s and 131 s at 16 kHz are G = 33, 59, 118, 128, 245 and 256 workgroups per utterance -- groups that span
    XCDs (write-through hand-offs), the two-level P3 / P4 reductions (8 leaders), GN words two per thread above 128
    members; N = 2096896 is T = 8192, the largest fused utterance (N = 2097152, T = 8193, is
    test_long_utterances_fall_back). Fused vs the multi-kernel schedule and vs the oracle on utterance 0."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    x = torch.from_numpy(synth.make_batch(2, N, 5150 + N % 997)[0])
    sf, vf, _, used = _run(net, x.to(DEV), True)
    assert used, "the fused TCN did not run"
    _check_schedules(net, x.to(DEV), sf, vf)
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    s_ref, v_ref, _ = om(x[:1])
    assert np.abs(sf[:1].cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
    check_vad_labels(vf[:1].cpu().numpy(), v_ref.numpy())


@pytest.mark.parametrize("cname", CONFIGS)
def test_fp32_gemms_run_fused(cname, nets, state_dicts):
    """The exact-fp32 arm on the fused schedule (k_tcn<PREC_F32>: v_mfma_f32_32x32x2_f32 on fp32 operands, the fp32
    weights streamed, reference model/model.py:104,114,324): fused, within the fp32 gates of the oracle, and within
    SCHED_TOL of the multi-kernel fp32 schedule (the same fp32 products, summed in a different order)."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    net = nets[cname]
    net.native_precision = "fp32"
    try:
        x = torch.from_numpy(synth.make_batch(3, 32000, 515)[0])
        sf, vf, _, used = _run(net, x.to(DEV), True)
        assert used
        sm, vm, _, used_m = _run(net, x.to(DEV), False)
        assert not used_m
    finally:
        net.native_precision = "f16x3"
    assert (sf - sm).abs().max().item() <= SCHED_TOL
    assert (vf - vm).abs().max().item() <= VAD_SCHED_TOL
    om = OracleModel(config_of(cname), state_dicts[cname], torch.float32)
    s_ref, v_ref, _ = om(x[:2])
    assert np.abs(sf[:2].cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
    check_vad_labels(vf[:2].cpu().numpy(), v_ref.numpy())


@pytest.mark.parametrize("N", [261888, 960000])
def test_fp32_gemms_long_groups_fused(N, nets):
    """The exact-fp32 arm on whole files: G = 32 and 118 members take the long-group instantiation
    (k_tcn<PREC_F32, LG = true>: tree reductions, its own fp32 A-plane strides, VAD-tile placement and LN staging).
    Fused, and within SCHED_TOL of the multi-kernel fp32 schedule (same fp32 products, other summation order), VAD
    labels equal to the multi-kernel schedule's."""
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    net.native_precision = "fp32"
    try:
        x = torch.from_numpy(synth.make_batch(2, N, 717 + N % 991)[0]).to(DEV)
        sf, vf, _, used = _run(net, x, True)
        assert used, "the fused TCN did not run"
        sm, vm, _, used_m = _run(net, x, False)
        assert not used_m
    finally:
        net.native_precision = "f16x3"
    assert (sf - sm).abs().max().item() <= SCHED_TOL
    assert (vf - vm).abs().max().item() <= VAD_SCHED_TOL
    check_vad_labels(vf.cpu().numpy(), vm.cpu().numpy())


def test_handoff_protocols_bitwise_identical(nets):
    """Same-XCD groups keep hand-off bytes in L2 (plain stores); SEPVAD_TCN_XMODE=1 forces the
    write-through protocol everywhere. Only the transport differs, so the bits must not."""
    import os
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    x = torch.from_numpy(synth.make_batch(70, 32000, 777)[0]).to(DEV)
    a, va, _, _ = _run(net, x, True)
    os.environ["SEPVAD_TCN_XMODE"] = "1"
    try:
        b, vb, _, used = _run(net, x, True)
    finally:
        del os.environ["SEPVAD_TCN_XMODE"]
    assert used
    assert torch.equal(a, b) and torch.equal(va, vb)


def test_vad_taps_finished_in_istft(nets):
    """SEPVAD_VAD_FEAT=0: k_istft_pair finishes the VAD conv1_1 + BN_1 from the output head's tap products itself
    (k_vad_feat's arithmetic); same results as the k_vad_feat schedule up to fp32 rounding, reference-pinned."""
    import os
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    g = load_golden("with_vad", "cfg")
    x = torch.from_numpy(synth.make_batch(7, 100000, 515)[0]).to(DEV)
    a, va, ea, _ = _run(net, x, True)
    os.environ["SEPVAD_VAD_FEAT"] = "0"
    try:
        b, vb, eb, used = _run(net, x, True)
        sg, vg, _, _ = _run(net, torch.from_numpy(g["x"]).to(DEV), True)
    finally:
        del os.environ["SEPVAD_VAD_FEAT"]
    assert used
    assert (a - b).abs().max().item() <= 1e-6
    assert (va - vb).abs().max().item() <= 1e-5
    assert torch.equal(va >= 0.5, vb >= 0.5)
    assert np.abs(sg.cpu().numpy() - g["sep"]).max() <= SEP_TOL
    assert np.array_equal(vg.cpu().numpy() >= 0.5, g["vad"] >= 0.5)
    assert np.abs(vg.cpu().numpy() - g["vad"]).max() <= VAD_PROB_TOL


def test_vad_taps_in_istft_default_short_utterances(nets):
    """T <= 256 defaults to the in-k_istft_pair VAD features (SEPVAD_VAD_FEAT unset); they take k_vad_feat<4>'s items
    and summation order; the BN_1 affine rounds differently (the VAD probabilities move by fp32 rounding), the
    separated signals are unchanged."""
    import os
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    x = torch.from_numpy(synth.make_batch(9, 32000, 516)[0]).to(DEV)
    a, va, ea, _ = _run(net, x, True)
    os.environ["SEPVAD_VAD_FEAT"] = "1"
    try:
        b, vb, eb, _ = _run(net, x, True)
    finally:
        del os.environ["SEPVAD_VAD_FEAT"]
    assert (a - b).abs().max().item() <= 1e-6
    assert (va - vb).abs().max().item() <= 1e-5
    assert torch.equal(va >= 0.5, vb >= 0.5)
    assert (ea is None and eb is None) or (ea - eb).abs().max().item() <= 1e-6


def test_long_files_full_chip_groups(nets, state_dicts):
    """16 s files at B=8 (bench --workload long): 8 groups of 32 members fill the 256 CUs, each group on one
    XCD (the L2-resident hand-off protocol), at T = 1001 (two-pass moment polls, LDS GroupNorm finish)."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    net = nets["with_vad"]
    x = torch.from_numpy(synth.make_batch(8, 256000, 8080)[0])
    sf, vf, _, used = _run(net, x.to(DEV), True)
    assert used
    _check_schedules(net, x.to(DEV), sf, vf)
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    s_ref, v_ref, _ = om(x[:1])
    assert np.abs(sf[:1].cpu().numpy() - s_ref.numpy()).max() <= SEP_TOL
    check_vad_labels(vf[:1].cpu().numpy(), v_ref.numpy())


@pytest.mark.parametrize("cname,B,N,sub", [("with_vad", 70, 32000, [0, 64, 69]), ("without_vad", 66, 32000, [1, 65]),
                                            ("with_vad", 3, 256000, [2])])
def test_output_head_in_tcn_vs_oracle(cname, B, N, sub, nets, state_dicts):
    """The output head runs inside k_tcn after each utterance's last block (a second utterance per group when
    B > 64 groups; 32-member groups at 16 s): masks_b (pre-sigmoid, all 514 rows) against the fp32 oracle, with
    bin 256 of each speaker (fp32 VALU dot products, not MFMA) checked on its own, and the separated waveforms."""
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    net = nets[cname]
    x = torch.from_numpy(synth.make_batch(B, N, 4242 + N)[0])
    sf, vf, _, used = _run(net, x.to(DEV), True)
    assert used
    mb = net.masks_b.cpu().numpy()[sub]
    om = OracleModel(config_of(cname), state_dicts[cname], torch.float32)
    s_ref, v_ref, _ = om(x[sub])
    ref = om.masks_b.numpy()
    err = np.abs(mb - ref).max()
    err_ny = np.abs(mb[:, [256, 513]] - ref[:, [256, 513]]).max()
    print(f"masks_b max-abs vs oracle {err:.2e} (bin 256: {err_ny:.2e})")
    assert err <= 2e-4 and err_ny <= 2e-4
    assert np.abs(sf.cpu().numpy()[sub] - s_ref.numpy()).max() <= SEP_TOL
    if vf is not None and cname == "with_vad":
        check_vad_labels(vf.cpu().numpy()[sub], v_ref.numpy())
