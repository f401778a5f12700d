"""Streaming wrapper on the GPU (reference model/online_class_unknown_targets.py:72-105) through the
C ABI (sepvad_forward_strided, sepvad_pit_l1, sepvad_stream_append) vs the reference's output and
the CPU restatement oracle/stream_ref.py."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, config_of

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEP_TOL = 1e-4


@pytest.fixture(scope="module")
def net(state_dicts):
    import sep_tfanet_vad_amd as pkg
    m = pkg.SeparationModel(**config_of("with_vad"))
    m.load_state_dict(state_dicts["with_vad"], strict=True)
    return m.eval().to(DEV)


def _criterion():
    import sep_tfanet_vad_amd as pkg
    return pkg.PITLossWrapper(loss_func=torch.nn.L1Loss(), pit_from="pw_pt")


def test_online_matches_reference_golden(net, tmp_path):
    import sep_tfanet_vad_amd as pkg
    g = np.load(os.path.join(GOLDEN, "golden_with_vad_stream.npz"))
    ons = pkg.OnlineSaving(net, str(tmp_path), _criterion())
    ons.save_sec = float(g["save_sec"])
    ons.calc_online(torch.from_numpy(g["x"]).to(DEV), "stream", 10 ** 6, dict(pkg.INFERENCE_KW_DEFAULTS))
    online = ons.online_signal.cpu().numpy()
    assert online.shape == g["online"].shape      # 7 windows x 2560 samples
    assert np.abs(online - g["online"]).max() <= SEP_TOL
    assert ons.indx == 0                          # reset() after the loop
    assert not any(tmp_path.iterdir())            # sample_indx >= num_save_samples: no wav writes


def test_online_vs_oracle_other_hops_and_padding(net, state_dicts):
    """save_sec 1 (the reference default) and 0.5; a short input padded to 3 s; B=3."""
    import sep_tfanet_vad_amd as pkg
    from oracle.stream_ref import calc_online
    from oracle.torch_ref import OracleModel
    from sep_tfanet_vad_amd import synth
    om = OracleModel(config_of("with_vad"), state_dicts["with_vad"], torch.float32)
    for n, save_sec in ((56000, 1.0), (40000, 0.5), (30000, 1.0)):
        x = torch.from_numpy(synth.make_batch(3, n, 1234 + n)[0])
        ref = calc_online(om, x, save_sec=save_sec)
        ons = pkg.OnlineSaving(net, "/nonexistent", _criterion())
        ons.save_sec = save_sec
        ons.calc_online(x.to(DEV), "s", 10 ** 6, {})
        got = ons.online_signal.cpu()
        assert got.shape == ref.shape
        assert (got - ref).abs().max().item() <= SEP_TOL


def test_pit_l1_matches_oracle():
    from oracle.stream_ref import pit_l1_pw_pt
    from sep_tfanet_vad_amd import pit
    g = torch.Generator().manual_seed(5)
    for B, L, swap_frac in ((1, 777, 1.0), (4, 5000, 0.0), (3, 500, 0.34), (64, 45440, 0.25)):
        ref = torch.randn(B, 2, L, generator=g)
        est = ref + 0.3 * torch.randn(B, 2, L, generator=g)
        nsw = int(round(swap_frac * B))
        est[:nsw] = est[:nsw].flip(1)
        loss_r, bi_r = pit_l1_pw_pt(est, ref)
        loss, bi, pw = pit.pit_l1(est.to(DEV), ref.to(DEV))
        assert torch.equal(bi.cpu(), bi_r)
        assert abs(loss.item() - loss_r.item()) <= 1e-5 * abs(loss_r.item())


def test_pit_wrapper_api_and_reorder():
    import sep_tfanet_vad_amd as pkg
    crit = _criterion()
    ref = torch.randn(2, 2, 1000, device=DEV)
    est = ref.flip(1).clone()
    loss, bi = crit(est, ref, return_incides=True)
    assert bi.tolist() == [[1, 0], [1, 0]]
    loss2, reordered, bi2 = crit(est, ref, return_est=True, return_incides=True)
    assert torch.equal(reordered, ref) and torch.equal(bi2, bi) and loss2.item() == loss.item() == 0.0
    assert torch.equal(pkg.reorder_source_mse(est, bi), ref)
    with pytest.raises(NotImplementedError):
        pkg.PITLossWrapper(torch.nn.MSELoss(), pit_from="pw_pt")(est, ref)


def test_wav_outputs_written_for_first_samples(net, tmp_path):
    import sep_tfanet_vad_amd as pkg
    from scipy.io import wavfile
    from sep_tfanet_vad_amd import synth
    x = torch.from_numpy(synth.make_batch(1, 80000, 77)[0]).to(DEV)
    ons = pkg.OnlineSaving(net, str(tmp_path), _criterion())
    ons.calc_online(x, "utt", 0, {})
    assert (tmp_path / "utt" / "indx_0" / "output_1.wav").exists()
    assert (tmp_path / "utt" / "indx_2" / "mixed.wav").exists()
    sr, on0 = wavfile.read(str(tmp_path / "utt" / "online_signal0.wav"))
    assert sr == 16000 and np.array_equal(on0, ons.online_signal[0, 0].cpu().numpy())
