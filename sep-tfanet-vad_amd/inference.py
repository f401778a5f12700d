"""``only_inference.py`` plumbing on the GPU (reference ``only_inference.py:27-136``).

    python -m sep_tfanet_vad_amd.inference -c config_with_vad.json -r model.pth -pm mix.wav \\
        [-sp results] [-o True] [-ps 32] [-ikw '{"return_smoothed_vad": true}']

What the reference CLI does, step by step, and where it lives here:

* checkpoint: ``torch.load(resume, map_location="cpu")['state_dict']`` + ``load_state_dict(strict=True)``
  (:57-61) -> ``load_checkpoint`` (``weights_only=True``: the published checkpoints were re-saved
  without the pickled ConfigParser, :37-56);
* input (:68-83): wav read, first channel of a multi-channel file, ``Resample(sr, 16000)`` when
  sr != 16 kHz, min-max normalisation to [-0.9, 0.9] -> ``prepare_input``: the resampler
  (``sepvad_resample``) and the normalisation (``sepvad_normalize``, bit-exact with the reference's
  float32 numpy expression) run on the device;
* streaming pass (:84-89) -> ``OnlineSaving`` (online.py) with the native ``PITLossWrapper``;
* full forward (:90-92) and the wav outputs (:94-95, ``Our_utils/utlis_inference.py:24-37``).

Deliberate differences: the model and input live on the ROCm device (the reference never
moves them); a non-16 kHz input is resampled and then normalised (the reference's resample branch hands
a tensor to ``torch.from_numpy`` at :82 and raises). Spectrogram/VAD plots are not produced
(visualisation is out of scope); ``save_vad`` writes the thresholded labels as ``.npy`` instead of PNGs.

VAD saving follows the reference's condition ``config.resume == "model_without_vad.pth"`` (:96), where
``config.resume`` is a ``pathlib.Path`` (parse_config.py:68-69) compared with a ``str``: never equal, so the
reference never saves the VAD; ``run(..., save_vad_output=True)`` opts in explicitly.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
from pathlib import Path

import numpy as np
import torch

from . import native as _native

DEFAULT_INFERENCE_KW = {
    "filter_signals_by_smo_vad": False,
    "filter_signals_by_unsmo_vad": False,
    "length_smoothing_filter": 3,
    "threshold_activated_vad": 0.5,
    "return_smoothed_vad": False,
}
NORM_SCRATCH_BYTES = 8192  # SEPVAD_NORM_SCRATCH_BYTES (include/sepvad.h)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def resample_filter(orig_freq: int, new_freq: int):
    """Host taps [phases, ntaps] and info (phases, ntaps, stride, width) of Resample(orig, new)."""
    lib = _native.load_library()
    info = (ctypes.c_int32 * 4)()
    _native._check(lib.sepvad_resample_filter(int(orig_freq), int(new_freq), None, 0, info), "sepvad_resample_filter")
    phases, ntaps = info[0], info[1]
    taps = np.empty(phases * ntaps, dtype=np.float32)
    _native._check(lib.sepvad_resample_filter(int(orig_freq), int(new_freq), taps.ctypes.data_as(ctypes.POINTER(
        ctypes.c_float)), taps.size, info), "sepvad_resample_filter")
    return taps.reshape(phases, ntaps), tuple(info)


def resample(x: torch.Tensor, orig_freq: int, new_freq: int = 16000) -> torch.Tensor:
    """torchaudio.transforms.Resample(orig_freq, new_freq)(x) for a 1-D device tensor."""
    lib = _native.load_library()
    if x.device.type != "cuda":
        raise RuntimeError("resample: input must be a ROCm device tensor")
    x = x.float().contiguous()
    taps, info = resample_filter(orig_freq, new_freq)
    phases, _, stride, _ = info
    ylen = int(np.ceil(phases * x.numel() / stride))
    y = torch.empty(ylen, dtype=torch.float32, device=x.device)
    t = torch.from_numpy(taps).to(x.device)
    cinfo = (ctypes.c_int32 * 4)(*info)  # host array read by the C entry point
    rc = lib.sepvad_resample(_native._ptr(x), x.numel(), _native._ptr(t), cinfo, _native._ptr(y), ylen,
                             _stream(x.device))
    _native._check(rc, "sepvad_resample")
    return y


def normalize(x: torch.Tensor) -> torch.Tensor:
    """1.8 * (x - min) / (max - min) - 0.9 (only_inference.py:81) on the device."""
    lib = _native.load_library()
    if x.device.type != "cuda":
        raise RuntimeError("normalize: input must be a ROCm device tensor")
    x = x.float().contiguous()
    y = torch.empty_like(x)
    scratch = torch.empty(NORM_SCRATCH_BYTES // 4, dtype=torch.float32, device=x.device)
    _native._check(lib.sepvad_normalize(_native._ptr(x), x.numel(), _native._ptr(y), _native._ptr(scratch),
                                        _stream(x.device)), "sepvad_normalize")
    return y


def prepare_input(samplerate: int, audio: np.ndarray, device="cuda") -> torch.Tensor:
    """only_inference.py:68-83: mono, resample to 16 kHz, normalise -> [1, N] float32 on `device`."""
    audio = np.array(audio, dtype=np.float32)
    if audio.ndim > 1:
        print("The audio is not mono, the first channel was chosen")
        if audio.shape[1] > audio.shape[0]:
            audio = audio[0]
        else:
            audio = audio[:, 0]
    x = torch.from_numpy(np.ascontiguousarray(audio)).to(device)
    if samplerate != 16000:
        print("The audio is not 16KHz, resmapling to 16KHz..")
        x = resample(x, samplerate, 16000)
    return normalize(x).unsqueeze(0)


def load_checkpoint(model, path: str):
    """only_inference.py:57-61 with a loader that executes nothing from the file."""
    checkpoint = torch.load(path, map_location="cpu", weights_only=True)
    state_dict = checkpoint["state_dict"] if "state_dict" in checkpoint else checkpoint
    model.load_state_dict(state_dict, strict=True)
    model.eval()
    return model


def save_audio(mix_waves, separated_signals, save_path, bit16):
    """Our_utils/utlis_inference.py:24-37 (16 -> float16 samples, as the reference writes them)."""
    from scipy.io.wavfile import write
    samplerate = 16000
    s1 = separated_signals[0, 0, :].cpu().detach().numpy()
    s2 = separated_signals[0, 1, :].cpu().detach().numpy()
    mix = mix_waves[0, :].cpu().detach().numpy()
    Path(save_path).mkdir(parents=True, exist_ok=True)
    dt = np.float16 if bit16 == 16 else np.float32
    write(os.path.join(save_path, "Mixed_0.wav"), samplerate, mix.astype(dt))
    write(os.path.join(save_path, "Speaker_0.wav"), samplerate, s1.astype(dt))
    write(os.path.join(save_path, "Speaker_1.wav"), samplerate, s2.astype(dt))


def save_vad(vad_output, save_path):
    """Our_utils/utlis_inference.py:39-46 without the plots: labels (p >= 0.5) per speaker as .npy."""
    Path(save_path).mkdir(parents=True, exist_ok=True)
    v = vad_output.cpu()
    for spk in range(v.shape[1]):
        np.save(os.path.join(save_path, f"estimated_vad_{spk}.npy"), (v[0, spk] >= 0.5).numpy().astype(np.int64))


def run(config_path, resume, path_mix, save_test_path, online=True, precision_save=32, inference_kw=None,
        device="cuda", save_vad_output=False):
    """only_inference.main (:27-97) for a config JSON (arch.args) and a checkpoint."""
    from scipy.io.wavfile import read
    from . import SeparationModel
    from .online import OnlineSaving
    from .pit import PITLossWrapper
    cfg = json.load(open(config_path))
    model = SeparationModel(**cfg["arch"]["args"])
    load_checkpoint(model, resume)
    model = model.to(device)
    ikw = dict(DEFAULT_INFERENCE_KW)
    ikw.update(inference_kw or {})
    samplerate, audio = read(path_mix)
    x = prepare_input(samplerate, audio, device)
    if online:
        crit = PITLossWrapper(loss_func=torch.nn.L1Loss(), pit_from="pw_pt")
        OnlineSaving(model, save_test_path, crit).calc_online(x, "online_results", 0, ikw)
    with torch.no_grad():
        out_separation, output_vad, _ = model(x, ikw)
    _ = model.mask_per_speaker  # the reference reads it for its mask plot (:92); plots are out of scope
    save_audio(x, out_separation, save_test_path, precision_save)
    # only_inference.py:96: Path(resume) == "model_without_vad.pth" is always False (Path vs str)
    if (save_vad_output or Path(resume) == "model_without_vad.pth") and isinstance(output_vad, torch.Tensor):
        save_vad(output_vad, save_test_path)
    return out_separation, output_vad


def main(argv=None):
    ap = argparse.ArgumentParser(description="Sep-TFAnet^VAD inference on MI355X")
    ap.add_argument("-c", "--config", default="config_without_vad.json", type=str)
    ap.add_argument("-r", "--resume", default="model_without_vad.pth", type=str)
    ap.add_argument("-d", "--device", default="0", type=str, help="ROCm device index")
    ap.add_argument("-sp", "--save_test_path", default="results_withoutvad", type=str)
    ap.add_argument("-o", "--online", default=True, type=bool)
    ap.add_argument("-ps", "--precision_save", default=32, choices=[16, 32], type=int)
    ap.add_argument("-pm", "--path_mix", type=str, required=True)
    ap.add_argument("-ikw", "--inference_kw", type=json.loads, default={})
    a = ap.parse_args(argv)
    run(a.config, a.resume, a.path_mix, a.save_test_path, a.online, a.precision_save, a.inference_kw,
        device=f"cuda:{a.device}")


if __name__ == "__main__":
    main()
