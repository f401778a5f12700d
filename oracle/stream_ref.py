"""ORACLE — test infrastructure only. Not part of the product path.

CPU restatement of the reference streaming wrapper with unknown targets
(``model/online_class_unknown_targets.py:72-105``) and of the criterion it is built with,
``PITLossWrapper(nn.L1Loss(), pit_from="pw_pt")`` (``model/pit_wrapper.py:77-140,149-177,261-312``),
plus ``reorder_source_mse`` (``model/combined_loss.py:63-78``). Written as plain loops over windows
on top of any forward callable (the CPU restatement ``OracleModel`` in the tests).

Pinned by ``tests/golden/golden_with_vad_stream.npz``, produced by running the reference's own
``OnlineSaving.calc_online`` (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import numpy as np
import torch


def pit_l1_pw_pt(est, ref):
    """(min loss, batch_indices [B, 2]) — nn.L1Loss() reduces batch and samples, so pw is a scalar
    per (est, target) pair broadcast over the batch (pit_wrapper.py:172-177)."""
    B = est.shape[0]
    pw = torch.empty(B, 2, 2, dtype=est.dtype)
    for e in range(2):
        for t in range(2):
            pw[:, e, t] = torch.nn.functional.l1_loss(est[:, e], ref[:, t])
    pwl = pw.transpose(-1, -2)                                   # :289
    perms = [(0, 1), (1, 0)]
    loss_set = torch.stack([sum(pwl[:, i, p[i]] for i in range(2)) / 2 for p in perms], dim=1)  # :294-300
    min_loss, idx = torch.min(loss_set, dim=1)                   # :308
    batch_indices = torch.stack([torch.tensor(perms[int(m)]) for m in idx], dim=0)  # :311
    return min_loss.mean(), batch_indices


def reorder(preds, batch_indices):
    return torch.stack([torch.index_select(s, 0, b) for s, b in zip(preds, batch_indices)])


def calc_online(forward, x, save_sec=1.0, fs=16000, max_len=3, inference_kw=None):
    """Stitched online signal [B, 2, n*hop] of the reference loop (:72-97), wav writes omitted."""
    if x.shape[-1] < fs * max_len:
        x = torch.nn.functional.pad(x, (0, fs * max_len - x.shape[-1]))
    max_indx = np.floor(((x.shape[-1] - fs * max_len) / (fs * save_sec)))
    hop = int(np.floor(fs * save_sec))
    indx = 0
    online = None
    while indx <= max_indx:
        s = int(np.floor(fs * indx * save_sec))
        window = x[:, s: s + max_len * fs]
        pred, _, _ = forward(window, inference_kw)
        if indx == 0:
            online = pred[:, :, pred.shape[-1] - hop:]
        pred_sim = pred[:, :, - hop - online.shape[-1]: - hop]
        online_sim = online[:, :, - fs * max_len + hop:]
        _, bi = pit_l1_pw_pt(pred_sim, online_sim)
        pred = reorder(pred, bi)
        tail = pred[:, :, pred.shape[-1] - hop:]
        online = tail if indx == 0 else torch.cat((online, tail), dim=-1)
        indx += 1
    return online
