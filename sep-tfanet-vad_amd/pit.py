"""Permutation-invariant L1 matching for the streaming wrapper, on the GPU.

Mirrors the part of the reference's ``PITLossWrapper`` (``model/pit_wrapper.py:7-362``) that the
streaming caller uses — ``PITLossWrapper(loss_func=torch.nn.L1Loss(), pit_from="pw_pt")`` called
with ``return_incides=True`` (``model/online_class_unknown_targets.py:87-91``,
``only_inference.py:84-89``) — and ``reorder_source_mse`` (``model/combined_loss.py:63-78``).
The pairwise losses, the permutation choice and the reordering run in ``libsepvad.so``
(``sepvad_pit_l1``, ``sepvad_stream_append``); there is no CPU path.

Reference semantics kept on purpose: ``nn.L1Loss()`` (reduction="mean") reduces over the batch as
well as the samples, so ``get_pw_losses`` (``pit_wrapper.py:172-177``) fills every batch row with the
same scalar and the chosen permutation is shared by the whole batch.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import native as _native

PIT_SCRATCH_BYTES = 16448  # SEPVAD_PIT_SCRATCH_BYTES (include/sepvad.h)
_scratch = {}


def _scratch_for(device):
    """Scratch of the current stream on `device` (one per stream: concurrent streams never share it)."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    buf = _scratch.pop(key, None)
    if buf is None:
        buf = torch.empty(PIT_SCRATCH_BYTES // 8, dtype=torch.float64, device=device)
        while len(_scratch) >= 32:  # bounded: drop the least recently used stream's scratch (its blocks return
            _scratch.pop(next(iter(_scratch)))  # to that stream's allocator pool, reused only in its order)
    _scratch[key] = buf  # most recently used last
    return buf


def _rows(t: torch.Tensor):
    """[B, 2, L] view with unit sample stride and a common speaker/batch row stride -> (ptr, ld)."""
    if t.dim() != 3 or t.shape[1] != 2:
        raise ValueError(f"expected [B, 2, L], got {tuple(t.shape)}")
    if t.stride(2) != 1 or t.stride(0) != 2 * t.stride(1):
        t = t.contiguous()
    return t, t.stride(1)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def pit_l1(est: torch.Tensor, ref: torch.Tensor):
    """(min loss [scalar], batch_indices [B, 2] int64, pairwise [2, 2]) on the device."""
    lib = _native.load_library()
    if est.device.type != "cuda" or ref.device != est.device:
        raise RuntimeError("pit_l1: est and ref must be on the same ROCm device")
    if est.shape != ref.shape:
        raise ValueError(f"pit_l1: shape mismatch {tuple(est.shape)} vs {tuple(ref.shape)}")
    est = est.float()
    ref = ref.float()
    est, eld = _rows(est)
    ref, rld = _rows(ref)
    B, _, L = est.shape
    dev = est.device
    perm = torch.empty(B, 2, dtype=torch.int64, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    pw = torch.empty(2, 2, dtype=torch.float32, device=dev)
    rc = lib.sepvad_pit_l1(_native._ptr(est), eld, _native._ptr(ref), rld, B, L, _native._ptr(_scratch_for(dev)),
                           _native._ptr(perm), _native._ptr(loss), _native._ptr(pw), _stream(dev))
    _native._check(rc, "sepvad_pit_l1")
    return loss, perm, pw


def pit_l1_sharded(est: torch.Tensor, ref: torch.Tensor, total_rows: int, group=None):
    """pit_l1 for a stream batch sharded over the ranks of `group` (total_rows streams over all ranks): the 4
    pairwise L1 sums of this rank's rows (sepvad_pit_l1_sums) are all-reduced (one 32-byte RCCL all-reduce,
    stream-ordered, no host sync), then every rank makes the batch-global choice of the unsharded call
    (sepvad_pit_l1_choose) with count = total_rows * L."""
    import torch.distributed as dist
    lib = _native.load_library()
    est, eld = _rows(est.float())
    ref, rld = _rows(ref.float())
    B, _, L = est.shape
    dev = est.device
    buf = torch.empty(4, dtype=torch.float64, device=dev)
    rc = lib.sepvad_pit_l1_sums(_native._ptr(est), eld, _native._ptr(ref), rld, B, L, _native._ptr(_scratch_for(dev)),
                                _native._ptr(buf), _stream(dev))
    _native._check(rc, "sepvad_pit_l1_sums")
    if dist.get_backend(group) == "gloo":  # (tests on a shared GPU: gloo reduces host tensors)
        hb = buf.cpu()
        dist.all_reduce(hb, op=dist.ReduceOp.SUM, group=group)
        buf.copy_(hb)
    else:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    count = float(total_rows) * float(L)
    perm = torch.empty(B, 2, dtype=torch.int64, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    pw = torch.empty(2, 2, dtype=torch.float32, device=dev)
    rc = lib.sepvad_pit_l1_choose(_native._ptr(buf), count, B, _native._ptr(perm), _native._ptr(loss), _native._ptr(pw),
                                  _stream(dev))
    _native._check(rc, "sepvad_pit_l1_choose")
    return loss, perm, pw


def stream_append(src: torch.Tensor, s0: int, H: int, perm, dst: torch.Tensor, d0: int):
    """dst[b, i, d0:d0+H] = src[b, perm[b, i], s0:s0+H] (perm None = identity), on the device."""
    lib = _native.load_library()
    src, sld = _rows(src)
    if dst.dim() != 3 or dst.stride(2) != 1 or dst.stride(0) != 2 * dst.stride(1):
        raise ValueError("stream_append: dst must be a [B, 2, L] buffer with unit sample stride")
    B = src.shape[0]
    if perm is not None:
        perm = perm.to(device=src.device, dtype=torch.int64).contiguous()
        if tuple(perm.shape) != (B, 2):
            raise ValueError("stream_append: perm must be [B, 2]")
    rc = lib.sepvad_stream_append(_native._ptr(src), sld, int(s0), B, int(H),
                                  _native._ptr(perm) if perm is not None else None,
                                  _native._ptr(dst), dst.stride(1), int(d0), _stream(src.device))
    _native._check(rc, "sepvad_stream_append")


def reorder_source_mse(preds: torch.Tensor, batch_indices: torch.Tensor) -> torch.Tensor:
    """Reference ``model/combined_loss.py:63-78``: out[b] = preds[b][batch_indices[b]] ([B, 2, L])."""
    out = torch.empty(preds.shape[0], 2, preds.shape[-1], dtype=torch.float32, device=preds.device)
    stream_append(preds, 0, preds.shape[-1], batch_indices, out, 0)
    return out


class PITLossWrapper(nn.Module):
    """``PITLossWrapper(loss_func, pit_from)`` (reference ``model/pit_wrapper.py:66-75``).

    Natively supported: ``loss_func`` an ``nn.L1Loss`` with reduction "mean", ``pit_from="pw_pt"``,
    two sources — the criterion the streaming wrapper is built with. Other combinations raise
    ``NotImplementedError`` (training losses are out of scope).
    """

    def __init__(self, loss_func, pit_from="pw_mtx", perm_reduce=None):
        super().__init__()
        self.loss_func = loss_func
        self.pit_from = pit_from
        self.perm_reduce = perm_reduce
        if self.pit_from not in ["pw_mtx", "pw_pt", "perm_avg"]:
            raise ValueError("Unsupported loss function type for now. Expected"
                             "one of [`pw_mtx`, `pw_pt`, `perm_avg`]")

    def _native_ok(self):
        return (self.pit_from == "pw_pt" and self.perm_reduce is None and isinstance(self.loss_func, nn.L1Loss)
                and self.loss_func.reduction == "mean")

    def forward(self, est_targets, targets, target_vad=0, return_est=False, return_incides=False,
                reduce_kwargs=None, **kwargs):
        n_src = targets.shape[1]
        assert n_src < 10, f"Expected source axis along dim 1, found {n_src}"
        if not self._native_ok() or n_src != 2 or kwargs:
            raise NotImplementedError("native PIT: only PITLossWrapper(nn.L1Loss(), pit_from='pw_pt') with 2 "
                                      "sources (the streaming wrapper's criterion) is built")
        mean_loss, batch_indices, _ = pit_l1(est_targets, targets)
        if not return_est and not return_incides:
            return mean_loss
        if not return_est and return_incides:
            return mean_loss, batch_indices
        reordered = reorder_source_mse(est_targets, batch_indices)
        if return_est and return_incides:
            return mean_loss, reordered, batch_indices
        return mean_loss, reordered
