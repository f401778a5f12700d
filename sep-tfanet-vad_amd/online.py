"""Streaming separation with unknown targets — drop-in for the reference's ``OnlineSaving``
(``model/online_class_unknown_targets.py:8-105``), batched on the GPU.

The reference slides a fixed ``max_len`` (3 s) window over the input with hop ``save_sec``, runs a
full forward per window, matches the new window's speakers to the stitched output with
``PITLossWrapper(L1, "pw_pt")`` on the overlap, reorders, and appends the window's last hop. This
class keeps that algorithm, its attributes and its file outputs, and moves the data path onto the
device:

* all windows of all streams run as ONE forward (``sepvad_forward_windows``): window k of stream b is read at
  x + b * row + k * hop, no gather copy (``get_truncated_signal``, :39-41); only the PIT-L1 + append chain
  is sequential over windows; recordings longer than ``max_window_utts`` window-utterances run in window-major
  chunks of forwards (bounded workspace, same results);
* the stitched signal is one preallocated ``[B, 2, n_windows * hop]`` buffer; the reorder + append
  of each hop is one ``sepvad_stream_append`` launch (``reorder_source_mse`` + ``update_online_signal``,
  :28-37, :93-94); the permutation comes from ``sepvad_pit_l1`` and never leaves the device;
* the whole loop is stream-ordered with no host synchronisation (wav writes aside, which the
  reference does for the first ``num_save_samples`` calls only).

Window offsets use the reference's float expressions verbatim (``int(np.floor(fs * indx * save_sec))``)
so the same samples are selected for any ``save_sec``.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from . import pit as _pit


def _slice_bounds(length: int, start, stop):
    """Python slice semantics (negative indices, clamping) -> (begin, end)."""
    b, e, _ = slice(start, stop).indices(length)
    return b, max(b, e)


class OnlineSaving:
    def __init__(self, model, save_path, criterion_similarity=None) -> None:
        # attributes as in model/online_class_unknown_targets.py:9-22
        self.indx = 0
        self.fs = 16000
        self.max_len = 3
        self.save_sec = 1
        self.model = model
        self.save_path = save_path
        self.online_sisdr = []
        self.reference_sisdr = []
        self.num_save_samples = 30
        self.similarity = False
        self.one_forward = True  # all windows in one forward when possible (False: the reference's window loop)
        # window-utterances per forward_windows call: long recordings run in window-major chunks, so the
        # workspace (~2.5 MB per window-utterance at T = 188) stays bounded (cfg 3: 1 792 in one call)
        self.max_window_utts = 2048
        if criterion_similarity is not None:
            self.similarity = True
            self.criterion_similarity = criterion_similarity

    def reset(self):
        self.indx = 0

    def _hop(self) -> int:
        return int(np.floor(self.fs * self.save_sec))

    def update_online_signal(self, est_signals):
        """Reference :28-37 (stand-alone form; calc_online appends into a preallocated buffer)."""
        hop = self._hop()
        L = est_signals.shape[-1]
        if self.indx == 0:
            out = torch.empty(est_signals.shape[0], 2, hop, dtype=torch.float32, device=est_signals.device)
            _pit.stream_append(est_signals, L - hop, hop, None, out, 0)
        else:
            prev = self.online_signal
            n = prev.shape[-1]
            out = torch.empty(est_signals.shape[0], 2, n + hop, dtype=torch.float32, device=est_signals.device)
            _pit.stream_append(prev, 0, n, None, out, 0)
            _pit.stream_append(est_signals, L - hop, hop, None, out, n)
        self.online_signal = out

    def get_truncated_signal(self, full_signal_mix):
        s = int(np.floor(self.fs * self.indx * self.save_sec))
        return full_signal_mix[:, s: s + self.max_len * self.fs]

    def increase_indx(self):
        self.indx += 1

    def get_indx(self):
        return self.indx

    def save_audio(self, name_folder, separated_signals, mix):
        from scipy.io.wavfile import write
        separated_audio1 = separated_signals[0, 0, :].cpu().detach().numpy()
        separated_audio2 = separated_signals[0, 1, :].cpu().detach().numpy()
        mix_waves = mix[0, :].cpu().detach().numpy()
        d = Path(f"{self.save_path}/{name_folder}/indx_{self.indx}")
        d.mkdir(parents=True, exist_ok=True)
        write(str(d / "mixed.wav"), self.fs, mix_waves.astype(np.float32))
        write(str(d / "output_0.wav"), self.fs, separated_audio1.astype(np.float32))
        write(str(d / "output_1.wav"), self.fs, separated_audio2.astype(np.float32))

    def save_last_online_audio(self, name_folder, online_signal, mixed_signal_t):
        from scipy.io.wavfile import write
        online_signal = online_signal[0, :, :].cpu().detach().numpy()
        mixed_signal_t = mixed_signal_t[0, :].cpu().detach().numpy()
        d = Path(f"{self.save_path}/{name_folder}")
        d.mkdir(parents=True, exist_ok=True)
        write(str(d / "online_signal0.wav"), self.fs, online_signal[0].astype(np.float32))
        write(str(d / "online_signal1.wav"), self.fs, online_signal[1].astype(np.float32))
        write(str(d / "ref_mix.wav"), self.fs, mixed_signal_t.astype(np.float32))

    def n_windows(self, n_samples: int) -> int:
        """Windows calc_online runs for an input of n_samples (after the pad to max_len)."""
        n = max(n_samples, self.fs * self.max_len)
        return int(np.floor((n - self.fs * self.max_len) / (self.fs * self.save_sec))) + 1

    def _batched_ok(self, n_total: int, n_win: int, hop: int, save: bool) -> bool:
        """The one-forward path needs the native model, no per-window wav writes, and window offsets that
        are exactly k * hop (the reference's float expression floor(fs * k * save_sec), :39-41)."""
        if save or not self.one_forward or not hasattr(self.model, "native_handle"):
            return False
        return all(int(np.floor(self.fs * k * self.save_sec)) == k * hop for k in range(n_win))

    def calc_online(self, full_signal_mix, name_folder, sample_indx, inference_kw, process_group=None):
        """Reference :72-105. Leaves the stitched signal in ``self.online_signal`` ([B, 2, n*hop]).

        Every window of every stream runs in ONE forward (``sepvad_forward_windows``, window-major: window k of
        all streams is one contiguous block); only the PIT-L1 choice + append chain is sequential over windows
        (two small launches per window). With per-window wav writes (sample_indx < num_save_samples) or a
        non-native model the reference's window loop runs instead (same results). The model's side
        attributes are not updated by the one-forward path (the reference leaves the last window's there).

        process_group: streams sharded over ranks (bench.py cfg 3): the reference's PIT is batch-global
        (nn.L1Loss means over the batch, model/pit_wrapper.py:172-177), so each window's 4 pairwise L1 sums
        are all-reduced over the group (pit.pit_l1_sharded) and the sharded result equals the unsharded one.
        """
        win = self.fs * self.max_len
        if full_signal_mix.shape[-1] < win:
            full_signal_mix = torch.nn.functional.pad(full_signal_mix, (0, win - full_signal_mix.shape[-1]))
        max_indx = np.floor(((full_signal_mix.shape[-1] - win) / (self.fs * self.save_sec)))
        hop = self._hop()
        B = full_signal_mix.shape[0]
        n_win = int(max_indx) + 1
        dev = full_signal_mix.device
        buf = torch.empty(B, 2, n_win * hop, dtype=torch.float32, device=dev)
        filled = 0
        save = sample_indx < self.num_save_samples
        total_rows = B
        if process_group is not None:
            import torch.distributed as dist
            t = torch.tensor([B], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=process_group)
            total_rows = int(t.item())
        batched = self._batched_ok(full_signal_mix.shape[-1], n_win, hop, save)
        if batched:
            x = full_signal_mix.to(torch.float32)
            if x.stride(-1) != 1:
                x = x.contiguous()
            wchunk = max(1, int(self.max_window_utts) // max(1, B))
            k_base, sep_w = 0, None
        while self.indx <= max_indx:
            if batched:
                k = self.indx
                if sep_w is None or k >= k_base + sep_w.shape[0]:  # next window-major chunk, one forward
                    k_base, n = k, min(wchunk, n_win - k)
                    with torch.no_grad():
                        sep_w = self.model.native_handle(dev).forward_windows(x[:, k * hop:], n, hop, win, inference_kw)
                pred_separation = sep_w[k - k_base]
            else:
                truncated_signal_mix = self.get_truncated_signal(full_signal_mix)
                with torch.no_grad():
                    pred_separation, _, _ = self.model(truncated_signal_mix, inference_kw)
            L = pred_separation.shape[-1]
            # the reference seeds online_signal with the un-reordered last hop at indx 0 (:85-86)
            online = pred_separation[:, :, L - hop:] if self.indx == 0 else buf[:, :, :filled]
            n_on = online.shape[-1]
            pb, pe = _slice_bounds(L, -hop - n_on, -hop)                  # :87
            ob, oe = _slice_bounds(n_on, -win + hop, None)                # :88
            pred_sim = pred_separation[:, :, pb:pe]
            online_sim = online[:, :, ob:oe]
            if process_group is not None:
                _, batch_indices, _ = _pit.pit_l1_sharded(pred_sim, online_sim, total_rows, process_group)
            else:
                _, batch_indices = self.criterion_similarity(pred_sim, online_sim, return_incides=True)
            # reorder_source_mse + update_online_signal (:92-94) in one device launch
            d0 = 0 if self.indx == 0 else filled
            _pit.stream_append(pred_separation, L - hop, hop, batch_indices, buf, d0)
            filled = d0 + hop
            self.online_signal = buf[:, :, :filled]
            if save:
                self.save_audio(name_folder, _pit.reorder_source_mse(pred_separation, batch_indices),
                                truncated_signal_mix)
            self.increase_indx()
        mixed_signal_t = full_signal_mix[:, int(np.floor(self.fs * (self.max_len - self.save_sec))):
                                         int(np.floor(self.fs * (self.max_len + (self.indx - 1) * self.save_sec)))]
        if save:
            self.save_last_online_audio(name_folder, self.online_signal, mixed_signal_t)
        self.reset()
