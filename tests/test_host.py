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


def test_library_is_built_from_this_tree():
    """The loaded library's source hash (sepvad_build_id) equals the hash of this tree's sources (buildid.py)."""
    from sep_tfanet_vad_amd import native
    if os.environ.get("SEPVAD_LIB"):
        pytest.skip("SEPVAD_LIB: an alternative build on purpose")
    assert native.build_id() == native.tree_build_id()


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


def test_e4m3_encoder_matches_torch():
    """The packer's e4m3 encoder (weight lo plane of the fused TCN, include/sepvad.h SEPVAD_WLO_E4M3) vs torch's
    float8_e4m3fn cast (OCP, round to nearest even): every finite magnitude class, ties, subnormals, saturation."""
    import numpy as np
    import torch
    from sep_tfanet_vad_amd import native
    lib = native.load_library()
    rng = np.random.default_rng(7)
    x = np.concatenate([
        rng.standard_normal(20000) * np.exp2(rng.uniform(-12, 9, 20000)),      # every binade of the range
        # all 256 codes' values and the midpoints between neighbouring codes (ties to even)
        torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).float().numpy(),
        np.array([0.0, -0.0, 2.0 ** -10, 3 * 2.0 ** -11, 2.0 ** -9 * 1.5, 440.0, 448.0, 449.0, 1e4, -1e4]),
    ]).astype(np.float32)
    codes = torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).float().numpy()
    fin = np.sort(np.unique(codes[np.isfinite(codes)]))
    x = np.concatenate([x, ((fin[1:] + fin[:-1]) / 2).astype(np.float32)])
    x = x[np.isfinite(x)]
    out = np.zeros(x.size, np.uint8)
    assert lib.sepvad_e4m3_encode(x.ctypes.data, out.ctypes.data, x.size) == 0
    got = torch.from_numpy(out).view(torch.float8_e4m3fn).float().numpy()
    want = torch.from_numpy(np.clip(x, -448, 448)).to(torch.float8_e4m3fn).float().numpy()
    assert np.array_equal(got, want)
    # the lo plane's range: |lo| <= 2^-12 of a row-scaled weight, stored * 2^19 -> <= 128, 4 significant bits
    lo = (rng.uniform(-1, 1, 4096) * 2.0 ** -12).astype(np.float32)
    assert lib.sepvad_e4m3_encode((lo * 2 ** 19).ctypes.data, out.ctypes.data, 4096) == 0
    back = torch.from_numpy(out[:4096].copy()).view(torch.float8_e4m3fn).float().numpy() / 2 ** 19
    assert np.all(np.abs(back - lo) <= np.abs(lo) * 2.0 ** -4 + 2.0 ** -29)


def test_unknown_weight_lo_is_rejected(monkeypatch):
    """SEPVAD_WLO is validated in both layers (the C library refuses the same values at sepvad_create)."""
    import sep_tfanet_vad_amd as pkg
    monkeypatch.setenv("SEPVAD_WLO", "int8")
    with pytest.raises(ValueError, match="SEPVAD_WLO"):
        pkg.SeparationModel(**pkg.CONFIG_WITH_VAD)
    monkeypatch.setenv("SEPVAD_WLO", "e4m3")
    assert pkg.SeparationModel(**pkg.CONFIG_WITH_VAD).native_weight_lo == "e4m3"
