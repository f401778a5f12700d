"""On-device SI-SDR family (csrc/metrics.hip via sepvad_si_sdr) vs the oracle restatement of the
reference's calc_sisdr (model/combined_loss.py:16-56) and its docstring known answer, plus the PIT and
SI-SDRi reductions of model/metric.py:145-160,258. The device computes the moments in double, the
reference in fp32 element-wise arithmetic: agreement to 1e-3 dB (the gate is 0.01 dB)."""
import itertools

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_DB = 1e-3


def _pit_ref(preds, target):
    """torchmetrics permutation_invariant_training(eval 'max') restated on the oracle's si_sdr (CPU)."""
    from oracle.torch_ref import si_sdr
    B, S, _ = preds.shape
    mtx = torch.empty(B, S, S)
    for t in range(S):
        for p in range(S):
            mtx[:, t, p] = si_sdr(preds[:, p], target[:, t])
    perms = list(itertools.permutations(range(S)))
    vals = torch.stack([mtx[:, torch.arange(S), torch.tensor(pm)].mean(-1) for pm in perms], -1)
    best, idx = vals.max(-1)
    return best, torch.tensor(perms)[idx]


def test_si_sdr_known_answer():
    from sep_tfanet_vad_amd import metrics
    preds = torch.tensor([2.5, 0.0, 2.0, 8.0], device=DEV)
    target = torch.tensor([3.0, -0.5, 2.0, 7.0], device=DEV)
    # model/combined_loss.py:31-33 docstring (torchmetrics' example, computed with zero_mean=False)
    v = metrics.scale_invariant_signal_distortion_ratio(preds, target, zero_mean=False).item()
    assert abs(v - 18.4030) < 1e-3


@pytest.mark.parametrize("N", [32000, 12345, 7])
@pytest.mark.parametrize("zero_mean", [True, False])
def test_si_sdr_vs_oracle(N, zero_mean):
    from oracle.torch_ref import si_sdr
    from sep_tfanet_vad_amd import metrics
    g = torch.Generator().manual_seed(N)
    t = torch.randn(4, 2, N, generator=g)
    p = 0.7 * t + 0.3 * torch.randn(4, 2, N, generator=g) + 0.1
    ref = si_sdr(p, t, zero_mean=zero_mean)
    got = metrics.calc_sisdr(p.to(DEV), t.to(DEV), zero_mean=zero_mean).cpu()
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= TOL_DB
    again = metrics.calc_sisdr(p.to(DEV), t.to(DEV), zero_mean=zero_mean).cpu()
    assert torch.equal(got, again)
    assert torch.equal(metrics.calc_sisdr_loss(p.to(DEV), t.to(DEV), zero_mean).cpu(), -got)


def test_pit_si_sdr_and_si_sdri_on_model_outputs(state_dicts):
    """PIT SI-SDR / SI-SDRi of the separated outputs of a B=6 forward vs the restated reductions."""
    import sep_tfanet_vad_amd as pkg
    from oracle.torch_ref import si_sdr
    from sep_tfanet_vad_amd import metrics, synth
    from conftest import config_of
    x, srcs = synth.make_batch(6, 16000, 321)
    net = pkg.SeparationModel(**config_of("with_vad"))
    net.load_state_dict(state_dicts["with_vad"], strict=True)
    net = net.eval().to(DEV)
    with torch.no_grad():
        sep, _, _ = net(torch.from_numpy(x).to(DEV))
    tgt = torch.from_numpy(srcs)
    best, perm = metrics.permutation_invariant_si_sdr(sep, tgt.to(DEV))
    rbest, rperm = _pit_ref(sep.cpu(), tgt)
    assert (best.cpu() - rbest).abs().max().item() <= TOL_DB
    margin = (best.cpu() - rbest).abs() < 0.05  # permutations are only comparable away from ties
    assert torch.equal(perm.cpu()[margin], rperm[margin])
    v = metrics.pit_si_sdr(sep, tgt.to(DEV)).item()
    assert abs(v - rbest.mean().item()) <= TOL_DB
    mix = torch.from_numpy(x)
    base = si_sdr(mix.unsqueeze(1).repeat(1, 2, 1), tgt).mean()
    vi = metrics.si_sdri(sep, tgt.to(DEV), mix.to(DEV)).item()
    assert abs(vi - (rbest.mean() - base).item()) <= 2 * TOL_DB


def test_metrics_reject_host_tensors():
    from sep_tfanet_vad_amd import metrics
    with pytest.raises(RuntimeError):
        metrics.calc_sisdr(torch.zeros(3, 100), torch.zeros(3, 100))


def test_metrics_match_reference_goldens():
    """Device calc_sisdr (both zero_mean branches) and Accuracy_Vad vs outputs of the reference itself
    (tests/golden/golden_metrics.npz, make_metric_golden.py). Accuracy_Vad thresholds preds in place
    like the reference (p > 0.5: exactly 0.5 is a 0)."""
    import os
    from conftest import GOLDEN
    from sep_tfanet_vad_amd import metrics
    g = np.load(os.path.join(GOLDEN, "golden_metrics.npz"))
    p, t = torch.from_numpy(g["sisdr_preds"]).to("cuda"), torch.from_numpy(g["sisdr_target"]).to("cuda")
    for zm in (0, 1):
        v = metrics.calc_sisdr(p, t, zero_mean=bool(zm)).cpu().numpy()
        assert np.abs(v - g[f"sisdr_zm{zm}"]).max() <= 1e-4  # fp32 reference vs moments in double
        e = metrics.calc_sisdr(torch.from_numpy(g["ex_preds"]).to("cuda"), torch.from_numpy(g["ex_target"]).to("cuda"),
                               zero_mean=bool(zm)).item()
        assert abs(e - float(g[f"ex_zm{zm}"])) <= 1e-5
    vp = torch.from_numpy(g["vad_preds"]).to("cuda")
    acc, acc0, acc1 = metrics.Accuracy_Vad()(vp, torch.from_numpy(g["vad_targets"]).to("cuda"), None)
    assert np.array_equal(vp.cpu().numpy(), g["vad_preds_after"])
    assert np.array_equal(np.array([acc.item(), acc0.item(), acc1.item()], np.float32), g["vad_acc"])
