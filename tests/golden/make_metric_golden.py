"""Golden vectors of the reference's quality metrics (run here, never on the GPU box).

    python tests/golden/make_metric_golden.py

Imports the reference's ``model/combined_loss.py`` (``calc_sisdr``, :16-56) and ``model/metric.py``
(``Accuracy_Vad``, :163-177) through the same offline stand-ins as make_golden.py, plus a ``torchmetrics``
stand-in (absent here; metric.py:4-8,255-258 only bind / instantiate ``PIT`` at import, unused by these two functions).
Inputs are seeded; only inputs and the reference's outputs are written (golden_metrics.npz).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402
from sep_tfanet_vad_amd import synth  # noqa: E402


def main():
    import_reference()  # shims on sys.path, turtle stub, reference root importable
    class _PitStandIn:  # metric.py:255-258 instantiate PIT(...) at import; never called for these metrics
        def __init__(self, *args, **kwargs):
            pass
    sys.modules.setdefault("torchmetrics", types.SimpleNamespace(PIT=_PitStandIn, PermutationInvariantTraining=_PitStandIn))
    import model.combined_loss as ref_loss  # noqa: E402
    import model.metric as ref_metric  # noqa: E402
    rng = np.random.Generator(np.random.PCG64(777))
    _, srcs = synth.make_batch(4, 8000, 900)                    # [4, 2, 8000] clean sources
    tgt = srcs.astype(np.float32)
    noise = rng.standard_normal(tgt.shape).astype(np.float32)
    preds = (0.8 * tgt + 0.05 * noise + 0.01).astype(np.float32)  # non-zero mean: zero_mean matters
    preds[3, 1] = tgt[3, 0]                                       # a swapped speaker (low SI-SDR)
    out = dict(sisdr_preds=preds, sisdr_target=tgt)
    for zm in (True, False):
        out[f"sisdr_zm{int(zm)}"] = ref_loss.calc_sisdr(torch.from_numpy(preds), torch.from_numpy(tgt), zm).numpy()
    # the docstring's example (combined_loss.py:31-35 / metric.py): 18.4030 with zero_mean False
    ex_p, ex_t = np.array([2.5, 0.0, 2.0, 8.0], np.float32), np.array([3.0, -0.5, 2.0, 7.0], np.float32)
    out.update(ex_preds=ex_p, ex_target=ex_t)
    for zm in (True, False):
        out[f"ex_zm{int(zm)}"] = ref_loss.calc_sisdr(torch.from_numpy(ex_p), torch.from_numpy(ex_t), zm).numpy()
    # Accuracy_Vad (metric.py:163-177): threshold p > 0.5 (not >=), mutates preds in place
    vp = rng.random((3, 2, 50), dtype=np.float32)
    vp[0, 0, :5] = 0.5
    vp[1, 1, :3] = np.nextafter(np.float32(0.5), np.float32(1))
    vt = (rng.random((3, 2, 50)) > 0.5).astype(np.float32)
    pt = torch.from_numpy(vp.copy())
    acc, acc0, acc1 = ref_metric.Accuracy_Vad()(pt, torch.from_numpy(vt), None)
    out.update(vad_preds=vp, vad_targets=vt, vad_preds_after=pt.numpy(),
               vad_acc=np.array([acc.item(), acc0.item(), acc1.item()], np.float32))
    fn = os.path.join(HERE, "golden_metrics.npz")
    np.savez_compressed(fn, **out)
    print({k: v for k, v in out.items() if k.startswith(("ex_", "vad_acc"))}, os.path.getsize(fn))


if __name__ == "__main__":
    main()
