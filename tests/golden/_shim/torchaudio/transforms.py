"""See package docstring. Spectrogram / InverseSpectrogram register ``window`` as a buffer
(so the reference state_dict carries spec_input.spec.window, spec_output.window,
inv_spec.window) and call torch.stft / torch.istft with torchaudio's defaults:
pad=0, normalized=False, center=True, pad_mode='reflect', onesided=True."""
import math

import torch
from torch import nn


class Spectrogram(nn.Module):
    def __init__(self, n_fft=400, win_length=None, hop_length=None, pad=0, window_fn=torch.hann_window,
                 power=2.0, normalized=False, wkwargs=None, center=True, pad_mode="reflect",
                 onesided=True, return_complex=None):
        super().__init__()
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        self.register_buffer("window", window_fn(self.win_length) if wkwargs is None
                             else window_fn(self.win_length, **wkwargs))
        self.pad, self.power, self.normalized = pad, power, normalized
        self.center, self.pad_mode, self.onesided = center, pad_mode, onesided

    def forward(self, waveform):
        if self.pad > 0:
            waveform = torch.nn.functional.pad(waveform, (self.pad, self.pad), "constant")
        shape = waveform.size()
        waveform = waveform.reshape(-1, shape[-1])
        spec = torch.stft(waveform, n_fft=self.n_fft, hop_length=self.hop_length,
                          win_length=self.win_length, window=self.window, center=self.center,
                          pad_mode=self.pad_mode, normalized=False, onesided=self.onesided,
                          return_complex=True)
        spec = spec.reshape(shape[:-1] + spec.shape[-2:])
        if self.normalized:
            spec = spec / self.window.pow(2.0).sum().sqrt()
        if self.power is not None:
            if self.power == 1.0:
                return spec.abs()
            return spec.abs().pow(self.power)
        return spec


class InverseSpectrogram(nn.Module):
    def __init__(self, n_fft=400, win_length=None, hop_length=None, pad=0, window_fn=torch.hann_window,
                 normalized=False, wkwargs=None, center=True, pad_mode="reflect", onesided=True):
        super().__init__()
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        self.register_buffer("window", window_fn(self.win_length) if wkwargs is None
                             else window_fn(self.win_length, **wkwargs))
        self.pad, self.normalized, self.center, self.onesided = pad, normalized, center, onesided

    def forward(self, spectrogram, length=None):
        if not spectrogram.is_complex():
            raise ValueError("Expected `spectrogram` to be complex dtype.")
        if self.normalized:
            spectrogram = spectrogram * self.window.pow(2.0).sum().sqrt()
        shape = spectrogram.size()
        spectrogram = spectrogram.reshape(-1, shape[-2], shape[-1])
        waveform = torch.istft(spectrogram, n_fft=self.n_fft, hop_length=self.hop_length,
                               win_length=self.win_length, window=self.window, center=self.center,
                               normalized=False, onesided=self.onesided,
                               length=length + 2 * self.pad if length is not None else None,
                               return_complex=False)
        if length is not None and self.pad > 0:
            waveform = waveform[:, self.pad:-self.pad]
        return waveform.reshape(shape[:-2] + waveform.shape[-1:])


class AmplitudeToDB(nn.Module):
    def __init__(self, stype="power", top_db=None):
        super().__init__()
        self.stype = stype
        self.top_db = top_db
        self.multiplier = 10.0 if stype == "power" else 20.0
        self.amin = 1e-10
        self.ref_value = 1.0
        self.db_multiplier = math.log10(max(self.amin, self.ref_value))

    def forward(self, x):
        x_db = self.multiplier * torch.log10(torch.clamp(x, min=self.amin))
        x_db = x_db - self.multiplier * self.db_multiplier
        if self.top_db is not None:
            shape = x_db.size()
            packed = 1 if x_db.dim() == 2 else shape[-3]
            x_db = x_db.reshape(-1, packed, shape[-2], shape[-1])
            x_db = torch.max(x_db, (x_db.amax(dim=(-3, -2, -1)) - self.top_db).view(-1, 1, 1, 1))
            x_db = x_db.reshape(shape)
        return x_db
