"""Separation quality metrics on the device, mirroring the reference's metric surface.

* ``calc_sisdr`` / ``calc_sisdr_loss`` (reference ``model/combined_loss.py:16-60``) and
  ``scale_invariant_signal_distortion_ratio`` (``model/metric.py:61-101``, the same formula):
  ``[..., time]`` -> ``[...]`` SI-SDR in dB, float32 epsilon, optional zero mean.
* ``pit_si_sdr`` (``model/metric.py:258``: torchmetrics ``PIT(scale_invariant_signal_distortion_ratio,
  'max')``): per utterance the best speaker permutation by mean SI-SDR, averaged over the batch.
  torchmetrics is not installed here; its published ``permutation_invariant_training`` (metric matrix
  [B, S, S] -> exhaustive permutations, eval 'max', mean over speakers; the Metric object averages over
  the batch) is restated; parity of that reduction is pinned by the oracle tests, not by torchmetrics.
* ``SI_SDRi`` / ``si_sdri`` (``model/metric.py:145-160``): ``pit_si_sdr(preds, target)`` minus the mean
  SI-SDR of the mixture against each target.
* ``Accuracy_Vad`` (``model/metric.py:163-177``): thresholded (``> 0.5``) VAD label accuracy, overall and per
  speaker; like the reference it thresholds ``preds`` in place (``k_vad_acc``, exact integer counts).

All inputs are ROCm tensors; the arithmetic runs in ``k_si_sdr`` (csrc/metrics.hip) through the C ABI
``sepvad_si_sdr``. There is no CPU fallback.
"""
from __future__ import annotations

import itertools

import torch

from . import native as _native


def _check_same_shape(preds, target):
    if preds.shape != target.shape:
        raise RuntimeError("Predictions and targets are expected to have the same shape, pred has shape of "
                           f"{preds.shape} and target has shape of {target.shape}")


def _rows(x: torch.Tensor) -> torch.Tensor:
    if x.device.type != "cuda":
        raise RuntimeError("sepvad metrics: inputs must be ROCm device tensors")
    return x.to(torch.float32).reshape(-1, x.shape[-1]).contiguous()


def _si_sdr_pairs(P, Tg, pidx=None, tidx=None, zero_mean=True):
    """SI-SDR of rows P[pidx[r]] vs Tg[tidx[r]] (2-D contiguous float32 device tensors)."""
    lib = _native.load_library()
    R = len(pidx) if pidx is not None else P.shape[0]
    out = torch.empty(R, device=P.device, dtype=torch.float32)
    pi = torch.as_tensor(pidx, dtype=torch.int32, device=P.device) if pidx is not None else None
    ti = torch.as_tensor(tidx, dtype=torch.int32, device=P.device) if tidx is not None else None
    stream = torch.cuda.current_stream(P.device).cuda_stream
    rc = lib.sepvad_si_sdr(_native._ptr(P), P.shape[1], _native._ptr(Tg), Tg.shape[1], P.shape[1], R,
                           _native._ptr(pi), _native._ptr(ti), int(bool(zero_mean)), _native._ptr(out), stream)
    _native._check(rc, "sepvad_si_sdr")
    return out


def scale_invariant_signal_distortion_ratio(preds: torch.Tensor, target: torch.Tensor, zero_mean: bool = True):
    """model/metric.py:61-101 (== model/combined_loss.py:16-56 calc_sisdr)."""
    _check_same_shape(preds, target)
    P, Tg = _rows(preds), _rows(target)
    return _si_sdr_pairs(P, Tg, zero_mean=zero_mean).reshape(preds.shape[:-1])


calc_sisdr = scale_invariant_signal_distortion_ratio


def calc_sisdr_loss(preds, target, zero_mean: bool = True):
    """model/combined_loss.py:58-60."""
    return -calc_sisdr(preds, target, zero_mean)


def permutation_invariant_si_sdr(preds: torch.Tensor, target: torch.Tensor, zero_mean: bool = True):
    """Per-utterance best permutation for [B, S, time] inputs.

    Returns (best_metric [B], best_perm [B, S] int64): metric matrix m[b, t, p] = SI-SDR(preds[b, p],
    target[b, t]); perm value = mean_t m[b, t, perm[t]]; the first maximum over permutations in
    itertools order (torchmetrics' exhaustive search)."""
    _check_same_shape(preds, target)
    B, S, N = preds.shape
    P, Tg = _rows(preds), _rows(target)
    pidx, tidx = [], []
    for b in range(B):
        for t in range(S):
            for p in range(S):
                pidx.append(b * S + p)
                tidx.append(b * S + t)
    mtx = _si_sdr_pairs(P, Tg, pidx, tidx, zero_mean).reshape(B, S, S)
    perms = torch.tensor(list(itertools.permutations(range(S))), device=preds.device)  # [P!, S]
    vals = mtx[:, torch.arange(S, device=preds.device), perms].mean(dim=-1)           # [B, P!]
    best, idx = vals.max(dim=-1)
    return best, perms[idx]


def pit_si_sdr(preds: torch.Tensor, target: torch.Tensor):
    """model/metric.py:258: mean over the batch of the best-permutation SI-SDR."""
    best, _ = permutation_invariant_si_sdr(preds, target, zero_mean=True)
    return best.mean()


class SI_SDRi(torch.nn.Module):
    """model/metric.py:145-160."""

    def forward(self, preds, target, mix):
        mix = mix.unsqueeze(dim=1).repeat(1, preds.shape[1], 1)
        si_sdr_mix_start = torch.mean(scale_invariant_signal_distortion_ratio(mix, target, zero_mean=True))
        return pit_si_sdr(preds, target) - si_sdr_mix_start


si_sdri = SI_SDRi()
si_sdri.__name__ = "si_sdri"


class Accuracy_Vad(torch.nn.Module):
    """model/metric.py:163-177: preds, targets [B, num_spk, T] -> (acc, acc0, acc1) 0-dim float32 tensors.
    preds is thresholded in place (> 0.5 -> 1, <= 0.5 -> 0), as the reference does."""

    def forward(self, preds, targets, batch_indices_vad=None):
        _check_same_shape(preds, targets)
        if preds.device.type != "cuda" or targets.device != preds.device:
            raise RuntimeError("sepvad metrics: inputs must be ROCm device tensors on one device")
        B, S, T = preds.shape
        work = preds if (preds.dtype == torch.float32 and preds.is_contiguous()) else preds.float().contiguous()
        tg = targets.to(torch.float32).contiguous()
        out = torch.empty(1 + S, device=preds.device, dtype=torch.float32)
        lib = _native.load_library()
        rc = lib.sepvad_vad_accuracy(_native._ptr(work), _native._ptr(tg), B, S, T, 1, _native._ptr(out),
                                     torch.cuda.current_stream(preds.device).cuda_stream)
        _native._check(rc, "sepvad_vad_accuracy")
        if work is not preds:
            preds.copy_(work)
        return out[0], out[1], out[2]
