"""Seeded synthetic inputs and weights (no datasets or checkpoints are reachable offline).

* ``make_state_dict`` — a platform-independent NumPy PCG64 recipe that produces every
  state_dict entry of the reference model (key set: ``config.param_spec``). The pretrained
  ``model_with_vad.pth`` / ``model_without_vad.pth`` are absent from the reference tree
  (reference ``.MISSING_LARGE_BLOBS:1-2``).
* ``make_mixture`` — 2-speaker mixtures shaped like the reference's training data: two gated
  harmonic+coloured-noise sources at 0 dB SIR plus coloured noise at SNR ~ U[0,15] dB
  (reference ``create_data/data_conifg_wham.yaml:58-61``), min-max normalised to [-0.9, 0.9]
  like ``only_inference.py:81``.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .config import param_spec

FS = 16000


def hann_periodic(n: int) -> np.ndarray:
    """torch.hann_window(n) (periodic) in float32: 0.5 - 0.5 cos(2 pi k / n)."""
    k = np.arange(n, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)).astype(np.float32)


def make_state_dict(config: dict, seed: int = 1234) -> "OrderedDict[str, np.ndarray]":
    """Every state_dict tensor for ``config`` as float32 NumPy arrays, from PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, shape, kind in param_spec(config):
        if kind == "window":
            a = hann_periodic(shape[0])
        elif kind == "wn_v":
            a = rng.standard_normal(shape)
        elif kind == "wn_g":
            a = rng.uniform(0.7, 1.3, size=shape)
            if name == "vad.output_layer_vad.weight_g":
                # a sharp VAD output keeps the probabilities away from the 0.5 threshold, so the
                # thresholded labels have a margin well above the fp32 noise floor
                a = rng.uniform(4.0, 6.0, size=shape)
        elif kind == "bias":
            a = 0.1 * rng.standard_normal(shape)
        elif kind == "conv_w":
            fan_in = int(np.prod(shape[1:]))
            a = rng.standard_normal(shape) / np.sqrt(fan_in)
        elif kind == "gn_w":
            a = 1.0 + 0.1 * rng.standard_normal(shape)
        elif kind == "gn_b":
            a = 0.1 * rng.standard_normal(shape)
        elif kind == "prelu":
            a = rng.uniform(0.1, 0.35, size=shape)
        else:  # pragma: no cover
            raise ValueError(kind)
        out[name] = np.ascontiguousarray(a, dtype=np.float32)
    return out


def _ar1_noise(rng, n, rho):
    """y[i] = rho * y[i-1] + w[i] (AR(1) coloured noise)."""
    from scipy.signal import lfilter
    return lfilter([1.0], [1.0, -rho], rng.standard_normal(n))


def _source(rng, n, fs):
    """Harmonic voiced segments + AR(1)-coloured noise, gated on/off so VAD is non-trivial."""
    t = np.arange(n) / fs
    f0 = rng.uniform(90.0, 260.0)
    vib = 1.0 + 0.03 * np.sin(2 * np.pi * rng.uniform(2, 6) * t + rng.uniform(0, 2 * np.pi))
    phase = 2 * np.pi * np.cumsum(f0 * vib) / fs
    harm = np.zeros(n)
    for h in range(1, 12):
        harm += (rng.uniform(0.3, 1.0) / h) * np.sin(h * phase + rng.uniform(0, 2 * np.pi))
    noise = _ar1_noise(rng, n, rng.uniform(0.6, 0.95))
    sig = harm + 0.3 * noise / (np.std(noise) + 1e-9)
    gate = np.zeros(n)
    pos = int(rng.uniform(0, 0.2) * fs)
    while pos < n:
        on = int(rng.uniform(0.25, 1.2) * fs)
        off = int(rng.uniform(0.1, 0.6) * fs)
        gate[pos:pos + on] = 1.0
        pos += on + off
    ramp = np.convolve(gate, np.hanning(161) / np.hanning(161).sum(), mode="same")
    return sig * ramp


def make_mixture(n_samples: int, seed: int, fs: int = FS):
    """One normalised mixture and its two (equally scaled) sources, float32.

    Returns (mix[N], sources[2, N]).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    s1 = _source(rng, n_samples, fs)
    s2 = _source(rng, n_samples, fs)
    # SIR 0 dB
    s1 /= np.sqrt(np.mean(s1 ** 2)) + 1e-9
    s2 /= np.sqrt(np.mean(s2 ** 2)) + 1e-9
    speech = s1 + s2
    snr = rng.uniform(0.0, 15.0)
    noise = _ar1_noise(rng, n_samples, rng.uniform(0.3, 0.9))
    noise *= np.sqrt(np.mean(speech ** 2) / (np.mean(noise ** 2) * 10 ** (snr / 10)))
    mix = speech + noise
    lo, hi = mix.min(), mix.max()
    scale = 1.8 / (hi - lo)
    mix_n = scale * (mix - lo) - 0.9  # only_inference.py:81
    return mix_n.astype(np.float32), np.stack([scale * s1, scale * s2]).astype(np.float32)


def make_batch(batch: int, n_samples: int, base_seed: int = 2024):
    """[B, N] mixtures and [B, 2, N] sources; utterance b uses PCG64(base_seed + b)."""
    mixes, srcs = [], []
    for b in range(batch):
        m, s = make_mixture(n_samples, base_seed + b)
        mixes.append(m)
        srcs.append(s)
    return np.stack(mixes), np.stack(srcs)


def make_reverb_mixture(n_samples: int, seed: int, fs: int = FS, rt60=(0.2, 0.6), rir_samples: int | None = None):
    """BASELINE cfg 4 input: two sources convolved with image-method RIRs of a random shoebox room
    (RT60 ~ U[rt60], create_data/data_conifg_wham.yaml:54-55; generator: sepvad_rir_generate, the
    reference's rirgen restated) plus coloured noise at SNR ~ U[0,15] dB (WHAM! noise is not available
    offline), min-max normalised like only_inference.py:81.

    Returns (mix[N], direct-path sources[2, N]) in float32 (targets: anechoic RIRs, T60 = 0)."""
    from scipy.signal import fftconvolve
    from .rirgen import generateRir
    rng = np.random.Generator(np.random.PCG64(seed))
    room = rng.uniform([3.0, 3.0, 2.2], [8.0, 7.0, 3.5])
    mic = rng.uniform(0.2, 0.8, 3) * room
    t60 = float(rng.uniform(*rt60))
    n_rir = rir_samples or int(t60 * fs)
    rev, dry = [], []
    for _ in range(2):
        s = _source(rng, n_samples, fs)
        s /= np.sqrt(np.mean(s ** 2)) + 1e-9
        pos = rng.uniform(0.15, 0.85, 3) * room
        h = np.array(generateRir(list(room), list(pos), list(mic), reverbTime=t60, fs=fs, nSamples=n_rir))
        h0 = np.array(generateRir(list(room), list(pos), list(mic), reverbTime=0.0, fs=fs, nSamples=n_rir))
        rev.append(fftconvolve(s, h)[:n_samples])
        dry.append(fftconvolve(s, h0)[:n_samples])
    speech = rev[0] + rev[1]
    snr = rng.uniform(0.0, 15.0)
    noise = _ar1_noise(rng, n_samples, rng.uniform(0.3, 0.9))
    noise *= np.sqrt(np.mean(speech ** 2) / (np.mean(noise ** 2) * 10 ** (snr / 10)))
    mix = speech + noise
    lo, hi = mix.min(), mix.max()
    scale = 1.8 / (hi - lo)
    mix_n = scale * (mix - lo) - 0.9
    return mix_n.astype(np.float32), (scale * np.stack(dry)).astype(np.float32)


def make_reverb_batch(batch: int, n_samples: int, base_seed: int = 4096, **kw):
    """[B, N] reverberant mixtures and [B, 2, N] direct-path sources; utterance b uses PCG64(base_seed + b).
    RIRs are generated in parallel host threads (the C call releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=8) as ex:
        res = list(ex.map(lambda b: make_reverb_mixture(n_samples, base_seed + b, **kw), range(batch)))
    return np.stack([r[0] for r in res]), np.stack([r[1] for r in res])
