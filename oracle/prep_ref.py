"""ORACLE — test infrastructure only. Not part of the product path.

CPU restatement of the reference CLI's input preprocessing (``only_inference.py:68-83``):

* ``resample``: ``torchaudio.transforms.Resample(orig, new)`` with its defaults — the published
  algorithm of torchaudio's ``_get_sinc_resample_kernel`` / ``_apply_sinc_resample_kernel``
  (sinc_interp_hann, lowpass_filter_width=6, rolloff=0.99): pad (width, width + orig), conv1d with
  stride orig, interleave the phases, crop to ceil(new * len / orig). torchaudio is not installed in
  this image and the reference ships no resampled fixture, so this restatement is **parity unpinned**;
  it is written in float64 from the published algorithm and only bounds the device path.
* ``normalize``: the reference's float32 numpy expression, verbatim.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def sinc_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    g = math.gcd(orig_freq, new_freq)
    o, n = orig_freq // g, new_freq // g
    base = min(o, n) * rolloff
    width = math.ceil(lowpass_filter_width * o / base)
    idx = torch.arange(-width, width + o, dtype=torch.float64)[None, None] / o
    t = torch.arange(0, -n, -1, dtype=torch.float64)[:, None, None] / n + idx
    t *= base
    t = t.clamp(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    kernels = torch.where(t == 0, torch.tensor(1.0, dtype=torch.float64), t.sin() / t)
    kernels *= window * (base / o)
    return kernels, width, o, n


def resample(x: torch.Tensor, orig_freq: int, new_freq: int = 16000) -> torch.Tensor:
    k, width, o, n = sinc_kernel(orig_freq, new_freq)
    w = x.to(torch.float64).reshape(1, -1)
    length = w.shape[-1]
    w = torch.nn.functional.pad(w, (width, width + o))
    y = torch.nn.functional.conv1d(w[:, None], k, stride=o)
    y = y.transpose(1, 2).reshape(1, -1)
    target = int(math.ceil(n * length / o))
    return y[0, :target]


def normalize(audio: np.ndarray) -> np.ndarray:
    audio = np.asarray(audio, dtype=np.float32)
    return 1.8 * (audio - audio.min()) / (audio.max() - audio.min()) - 0.9
