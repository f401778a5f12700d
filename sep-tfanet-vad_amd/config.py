"""Architecture configuration and the state_dict key contract of Sep-TFAnet^VAD.

The constructor kwargs mirror ``SeparationModel.__init__`` defaults
(reference ``model/model.py:362-366``; note the reference's spelling ``casual``).
``param_spec`` enumerates every state_dict entry the reference model registers for a
given configuration (reference ``model/model.py:16-25,69-127,153-208,210-325,360-400``),
so the drop-in module can be loaded ``strict=True`` with a reference checkpoint.
"""
from __future__ import annotations

from collections import OrderedDict

# model/model.py:362-366
DEFAULTS = OrderedDict(
    n_fftBins=512, BN_dim=256, H_dim=512, layer=8, stack=3, kernel=3,
    num_spk=2, skip=False, dilated=True, casual=False, bool_drop=True,
    drop_value=0.1, weight_norm=False, final_vad=True, noisy_phase=False,
    activity_input_bool=False, tf_attention=False, apply_recursive_ln=False,
    apply_residual_ln=False, final_vad_masked_speakers=False,
)

# Inference options accepted by forward(x, inference_kw) (only_inference.py:102-108).
INFERENCE_KW_DEFAULTS = OrderedDict(
    filter_signals_by_smo_vad=False,
    filter_signals_by_unsmo_vad=False,
    length_smoothing_filter=3,
    threshold_activated_vad=0.5,
    return_smoothed_vad=False,
)

# The two configurations the reference ships (config_with_vad.json / config_without_vad.json, arch.args).
_SHIPPED_COMMON = dict(
    n_fftBins=512, BN_dim=256, H_dim=512, layer=8, stack=3, kernel=3, num_spk=2,
    skip=False, dilated=True, casual=False, bool_drop=True, drop_value=0.05,
    weight_norm=True, final_vad=True, final_vad_masked_speakers=False,
    noisy_phase=True, activity_input_bool=True, tf_attention=True,
)
CONFIG_WITH_VAD = dict(_SHIPPED_COMMON, apply_recursive_ln=True, apply_residual_ln=False)
CONFIG_WITHOUT_VAD = dict(_SHIPPED_COMMON, apply_recursive_ln=False, apply_residual_ln=True)


def merge_config(config: dict) -> dict:
    """Defaults updated by the caller's kwargs, like ``defaults.update(config)`` (model/model.py:370)."""
    cfg = dict(DEFAULTS)
    cfg.update(config)
    return cfg


def native_support_error(cfg: dict) -> str | None:
    """Return why the native MI355X path cannot run ``cfg`` (None if it can).

    The native path covers the weight-normed, non-causal, skip-free branch of the reference
    (the branch both shipped configs take, model/model.py:103-127,271-325).
    """
    if not cfg["weight_norm"]:
        return "weight_norm=False (the un-normed branch, model/model.py:77-101) is not built natively"
    if cfg["casual"]:
        return "casual=True (cumulative LN, model/model.py:27-66) is not built natively"
    if cfg["skip"]:
        return "skip=True (skip-connection sum, model/model.py:335-340) is not built natively"
    if not cfg["dilated"]:
        return "dilated=False is not built natively"
    if cfg["n_fftBins"] != 512:
        return "only n_fftBins=512 is built natively"
    if cfg["BN_dim"] != cfg["n_fftBins"] // 2:
        return "BN_dim must equal n_fftBins/2 (the TCN input is the 256 non-DC bins)"
    if cfg["H_dim"] != 2 * cfg["BN_dim"]:
        return "H_dim must be 2*BN_dim (depthwise multiplier 2, groups=BN_dim)"
    if cfg["kernel"] != 3:
        return "only kernel=3 is built natively"
    if cfg["num_spk"] != 2:
        return "only num_spk=2 is built natively"
    if cfg["apply_recursive_ln"] and cfg["apply_residual_ln"]:
        pass  # reference gives recursive precedence (model/model.py:347-350)
    return None


def dilations(cfg: dict) -> list[int]:
    """Per-block dilation of the weight-normed branch: i%4+1 (model/model.py:285-293)."""
    out = []
    for _ in range(cfg["stack"]):
        for i in range(cfg["layer"]):
            out.append(1 if i == 0 else (i % 4 + 1))
    return out


def param_spec(config: dict) -> list[tuple[str, tuple, str]]:
    """Ordered (name, shape, kind) for every state_dict entry of the weight-normed model.

    kinds: window, wn_g, wn_v, bias, conv_w, gn_w, gn_b, prelu.
    """
    cfg = merge_config(config)
    nfft = cfg["n_fftBins"]
    F = nfft // 2 + 1
    C, H = cfg["BN_dim"], cfg["H_dim"]
    nblk = cfg["layer"] * cfg["stack"]
    spec: list[tuple[str, tuple, str]] = []

    def wn_conv(prefix, cout, cin_per_group, k):
        spec.append((prefix + ".bias", (cout,), "bias"))
        spec.append((prefix + ".weight_g", (cout, 1, 1), "wn_g"))
        spec.append((prefix + ".weight_v", (cout, cin_per_group, k), "wn_v"))

    def gn(prefix, c):
        spec.append((prefix + ".weight", (c,), "gn_w"))
        spec.append((prefix + ".bias", (c,), "gn_b"))

    # model/model.py:383-387 (torchaudio transforms register their Hann window as a buffer)
    spec.append(("spec_input.spec.window", (nfft,), "window"))
    spec.append(("spec_output.window", (nfft,), "window"))
    spec.append(("inv_spec.window", (nfft,), "window"))
    # TCN (model/model.py:271-325)
    gn("TCN.LN", C)
    for i in range(nblk):
        p = f"TCN.TCN.{i}"
        wn_conv(p + ".conv1d", C, C, 1)
        wn_conv(p + ".dconv1d", H, 1, 3)
        wn_conv(p + ".res_out", C, H, 1)
        spec.append((p + ".nonlinearity1.weight", (1,), "prelu"))
        spec.append((p + ".nonlinearity2.weight", (1,), "prelu"))
        gn(p + ".reg1", C)
        gn(p + ".reg2", H)
    if cfg["tf_attention"]:
        for i in range(nblk):
            p = f"TCN.time_freq_attnetion.{i}"
            for ax in ("t", "f"):
                spec.append((f"{p}.conv1d_{ax}_1.weight", (1, 1, 3), "conv_w"))
                spec.append((f"{p}.conv1d_{ax}_1.bias", (1,), "bias"))
                spec.append((f"{p}.conv1d_{ax}_2.weight", (1, 1, 3), "conv_w"))
                spec.append((f"{p}.conv1d_{ax}_2.bias", (1,), "bias"))
            spec.append((f"{p}.prelu_t.weight", (1,), "prelu"))
            spec.append((f"{p}.prelu_f.weight", (1,), "prelu"))
    if cfg["apply_recursive_ln"]:
        for i in range(nblk):
            gn(f"TCN.ln_first_modules.{i}", C)
        for i in range(nblk):
            gn(f"TCN.ln_second_modules.{i}", C)
    if cfg["apply_residual_ln"]:
        for i in range(nblk):
            gn(f"TCN.ln_modules.{i}", C)
    spec.append(("TCN.output.0.weight", (1,), "prelu"))
    gn("TCN.output.1", C)
    wn_conv("TCN.output.2", F * cfg["num_spk"], C, 1)
    if cfg["final_vad"]:
        wn_conv("vad.common.conv1_1", 4, F, 5)
        spec.append(("vad.common.relu_1.weight", (1,), "prelu"))
        gn("vad.common.BN_1", 4)
        wn_conv("vad.output_layer_vad", 1, 4, 3)
    if cfg["activity_input_bool"]:
        spec.append(("activity_input.weight", (1, 1, 3, 3), "conv_w"))
        spec.append(("activity_input.bias", (1,), "bias"))
        spec.append(("prelu.weight", (1,), "prelu"))
    return spec


def frames(n_samples: int, nfft: int = 512) -> int:
    """STFT frame count with center=True: 1 + floor(N/hop) (torch.stft)."""
    return 1 + n_samples // (nfft // 2)
