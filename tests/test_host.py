"""Host-side contract of the drop-in (no GPU): kwargs, state_dict keys, errors, C-ABI exports."""
import ctypes
import json
import os
import re

import pytest
import torch

from conftest import CONFIGS, GOLDEN, REPO, config_of


@pytest.mark.parametrize("cname", CONFIGS)
def test_state_dict_keys_match_reference(cname):
    import sep_tfanet_vad_amd as pkg
    ref = json.load(open(os.path.join(GOLDEN, f"state_dict_keys_{cname}.json")))
    net = pkg.SeparationModel(**config_of(cname))
    mine = {k: list(v.shape) for k, v in net.state_dict().items()}
    assert mine == {k: s for k, s in ref}
    assert len(mine) == (719 if cname == "with_vad" else 671)


@pytest.mark.parametrize("cname", CONFIGS)
def test_load_state_dict_strict(cname, state_dicts):
    import sep_tfanet_vad_amd as pkg
    net = pkg.SeparationModel(**config_of(cname))
    net.load_state_dict(state_dicts[cname], strict=True)
    net.eval()
    assert net.casual is False and net.n_fftBins_h == 257  # attributes set from kwargs


def test_param_spec_matches_module():
    import sep_tfanet_vad_amd as pkg
    for cname in CONFIGS:
        cfg = config_of(cname)
        net = pkg.SeparationModel(**cfg)
        spec = {n: tuple(s) for n, s, _ in pkg.param_spec(cfg)}
        assert spec == {k: tuple(v.shape) for k, v in net.state_dict().items()}


def test_forward_contract_errors():
    import sep_tfanet_vad_amd as pkg
    net = pkg.SeparationModel(**pkg.CONFIG_WITH_VAD)
    with pytest.raises(AssertionError):
        net(torch.zeros(1, 2, 8000))  # model/model.py:406
    with pytest.raises(RuntimeError, match="ROCm device"):
        net(torch.zeros(1, 8000))     # no CPU fallback


@pytest.mark.parametrize("bad", [dict(casual=True), dict(skip=True), dict(weight_norm=False),
                                 dict(num_spk=3), dict(n_fftBins=256, BN_dim=128, H_dim=256)])
def test_unsupported_configs_fail_loudly(bad):
    import sep_tfanet_vad_amd as pkg
    with pytest.raises(NotImplementedError):
        pkg.SeparationModel(**dict(pkg.CONFIG_WITH_VAD, **bad))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "sepvad.h")).read()
    return sorted(set(re.findall(r"\b(sepvad_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from sep_tfanet_vad_amd import native
    lib = native.load_library()
    syms = _header_symbols()
    assert set(syms) == set(native.EXPORTED_SYMBOLS)
    for s in syms:
        assert hasattr(lib, s), s
    assert lib.sepvad_abi_version() == 1


def test_library_rejects_bad_config_without_gpu():
    from sep_tfanet_vad_amd import native
    lib = native.load_library()
    c = native.make_config(dict(config_of("with_vad"), n_fftBins=1024, BN_dim=512, H_dim=1024))
    h = lib.sepvad_create(ctypes.byref(c), None, None, None, 0, 0)
    assert not h
    assert b"" != lib.sepvad_last_error()


def test_inference_kw_struct():
    from sep_tfanet_vad_amd import native
    assert native.make_kw({}) is None and native.make_kw(None) is None
    k = native.make_kw(dict(filter_signals_by_smo_vad=True, filter_signals_by_unsmo_vad=False,
                            length_smoothing_filter=5, threshold_activated_vad=0.3, return_smoothed_vad=True))
    assert k.enabled == 1 and k.filter_signals_by_smo_vad == 1 and abs(k.threshold_activated_vad - 0.3) < 1e-7
    with pytest.raises(KeyError):  # the reference indexes the keys directly
        native.make_kw({"threshold_activated_vad": 0.5})


def test_resample_filter_matches_restatement():
    """Host filter of sepvad_resample_filter vs the float64 restatement of torchaudio's kernel (no GPU)."""
    import numpy as np
    from oracle.prep_ref import sinc_kernel
    from sep_tfanet_vad_amd.inference import resample_filter
    for o, n in ((8000, 16000), (44100, 16000), (22050, 16000), (48000, 16000), (16000, 8000)):
        taps, info = resample_filter(o, n)
        k, width, oo, nn = sinc_kernel(o, n)
        assert info == (nn, 2 * width + oo, oo, width)
        assert np.abs(taps - k[:, 0, :].numpy()).max() <= 1e-7
