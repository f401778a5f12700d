"""ctypes binding of ``libsepvad.so`` (C ABI declared in ``include/sepvad.h``).

This is the reference-side binding a Python caller of the boundary needs; ``model.py`` uses it to
keep the reference's ``SeparationModel`` surface. The library is built in-tree by
``__graft_entry__.build()`` (``make -C sep-tfanet-vad_amd/csrc``). There is no fallback: a missing
library, a CPU tensor or a non-zero status raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

# SEPVAD_LIB: an alternative build of the same library (A/B timing of kernel variants, tools/ab.sh)
LIB_PATH = os.environ.get("SEPVAD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsepvad.so")

SEPVAD_LN_PLAIN, SEPVAD_LN_RECURSIVE, SEPVAD_LN_RESIDUAL = 0, 1, 2
SEPVAD_PREC_FP32, SEPVAD_PREC_F16X3, SEPVAD_PREC_F16, SEPVAD_PREC_BF16 = 0, 1, 2, 3
# fp32 / f16x3: fp32-equivalent (parity path); f16 / bf16: reduced-precision arms (tolerance measured)
PRECISIONS = {"fp32": SEPVAD_PREC_FP32, "f16x3": SEPVAD_PREC_F16X3, "f16": SEPVAD_PREC_F16, "bf16": SEPVAD_PREC_BF16}
# storage of the f16x3 weight lo plane in the fused TCN (include/sepvad.h SEPVAD_WLO_*)
WEIGHT_LO = {"e4m3": 0, "f16": 1, "i8": 2}

EXPORTED_SYMBOLS = (
    "sepvad_create", "sepvad_reserve", "sepvad_set_precision", "sepvad_set_weight_lo", "sepvad_e4m3_encode",
    "sepvad_forward", "sepvad_forward_strided",
    "sepvad_forward_windows", "sepvad_pit_l1_sums", "sepvad_pit_l1_choose",
    "sepvad_set_split", "sepvad_set_fused", "sepvad_fused_status", "sepvad_side_outputs", "sepvad_set_tcn_dump",
    "sepvad_last_forward", "sepvad_side_outputs_of", "sepvad_release_stream", "sepvad_tcn_clock",
    "sepvad_stft_gate_test", "sepvad_istft_pair_test",
    "sepvad_stft", "sepvad_istft",
    "sepvad_pit_l1", "sepvad_stream_append",
    "sepvad_resample_filter", "sepvad_resample", "sepvad_normalize", "sepvad_si_sdr", "sepvad_vad_accuracy",
    "sepvad_rir_generate",
    "sepvad_set_timing", "sepvad_timing", "sepvad_destroy", "sepvad_last_error", "sepvad_abi_version",
    "sepvad_build_id",
)


def build_id() -> str:
    """Source hash the loaded library was built from (sepvad_build_id, include/sepvad.h)."""
    return load_library().sepvad_build_id().decode()


def tree_build_id() -> str:
    """The same hash computed from this tree's sources (buildid.py)."""
    from . import buildid
    return buildid.source_hash()


class SepVadConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_fft", "bn_dim", "h_dim", "layer", "stack", "num_spk", "tf_attention", "ln_mode",
        "final_vad", "final_vad_masked_speakers", "noisy_phase", "activity_input", "precision")]


class SepVadInferKw(ctypes.Structure):
    _fields_ = [("enabled", ctypes.c_int32), ("filter_signals_by_smo_vad", ctypes.c_int32),
                ("filter_signals_by_unsmo_vad", ctypes.c_int32), ("length_smoothing_filter", ctypes.c_int32),
                ("threshold_activated_vad", ctypes.c_float), ("return_smoothed_vad", ctypes.c_int32)]


class SepVadOutputs(ctypes.Structure):
    _fields_ = [("sep", ctypes.c_void_p), ("vad", ctypes.c_void_p), ("est", ctypes.c_void_p),
                ("spectrum", ctypes.c_void_p), ("masks_b", ctypes.c_void_p), ("mask", ctypes.c_void_p)]


_lib = None

# SEPVAD_CHECK=1: synchronise after every forward and raise if its fused TCN hand-offs gave up. Without it
# a give-up (which needs the chip to be shared with work that starves the launch's groups for ~1 s) is
# reported by the next forward on the same stream, or by Handle.fused_status().
CHECK_EACH_FORWARD = os.environ.get("SEPVAD_CHECK", "0") not in ("", "0")


def load_library(path: str = LIB_PATH):
    """Load libsepvad.so (after torch, so it binds to torch's HIP runtime) and declare signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libsepvad.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` or `make -C sep-tfanet-vad_amd/csrc`")
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    i32 = ctypes.c_int32
    lib.sepvad_create.restype = P
    lib.sepvad_create.argtypes = [ctypes.POINTER(SepVadConfig), ctypes.POINTER(P), ctypes.POINTER(ctypes.c_char_p),
                                  ctypes.POINTER(ctypes.c_int64), i32, i32]
    lib.sepvad_reserve.restype = i32
    lib.sepvad_reserve.argtypes = [P, i32, i32]
    lib.sepvad_set_precision.restype = i32
    lib.sepvad_set_precision.argtypes = [P, i32]
    lib.sepvad_set_weight_lo.restype = i32
    lib.sepvad_set_weight_lo.argtypes = [P, i32]
    lib.sepvad_e4m3_encode.restype = i32
    lib.sepvad_e4m3_encode.argtypes = [P, P, ctypes.c_int64]
    lib.sepvad_forward.restype = i32
    lib.sepvad_forward.argtypes = [P, P, i32, i32, ctypes.POINTER(SepVadOutputs), ctypes.POINTER(SepVadInferKw), P]
    lib.sepvad_forward_strided.restype = i32
    lib.sepvad_forward_strided.argtypes = [P, P, ctypes.c_int64, i32, i32, ctypes.POINTER(SepVadOutputs),
                                           ctypes.POINTER(SepVadInferKw), P]
    lib.sepvad_forward_windows.restype = i32
    lib.sepvad_forward_windows.argtypes = [P, P, ctypes.c_int64, i32, i32, ctypes.c_int64, i32,
                                           ctypes.POINTER(SepVadOutputs), ctypes.POINTER(SepVadInferKw), P]
    lib.sepvad_pit_l1_sums.restype = i32
    lib.sepvad_pit_l1_sums.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64, i32, ctypes.c_int64, P, P, P]
    lib.sepvad_pit_l1_choose.restype = i32
    lib.sepvad_pit_l1_choose.argtypes = [P, ctypes.c_double, i32, P, P, P, P]
    lib.sepvad_set_split.restype = i32
    lib.sepvad_set_split.argtypes = [P, i32]
    lib.sepvad_set_fused.restype = i32
    lib.sepvad_set_fused.argtypes = [P, i32]
    lib.sepvad_fused_status.restype = i32
    lib.sepvad_fused_status.argtypes = [P, ctypes.POINTER(i32)]
    lib.sepvad_set_tcn_dump.restype = i32
    lib.sepvad_set_tcn_dump.argtypes = [P, P]
    lib.sepvad_side_outputs.restype = i32
    lib.sepvad_side_outputs.argtypes = [P, ctypes.POINTER(SepVadOutputs), P]
    lib.sepvad_last_forward.restype = i32
    lib.sepvad_last_forward.argtypes = [P, P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(i32), ctypes.POINTER(i32)]
    lib.sepvad_side_outputs_of.restype = i32
    lib.sepvad_side_outputs_of.argtypes = [P, ctypes.POINTER(SepVadOutputs), P, ctypes.c_int64, i32, i32]
    lib.sepvad_release_stream.restype = i32
    lib.sepvad_release_stream.argtypes = [P, P]
    lib.sepvad_tcn_clock.restype = i32
    lib.sepvad_tcn_clock.argtypes = [P, P, i32, ctypes.POINTER(i32)]
    lib.sepvad_stft_gate_test.restype = i32
    lib.sepvad_stft_gate_test.argtypes = [P, P, i32, i32, P, P, P]
    lib.sepvad_istft_pair_test.restype = i32
    lib.sepvad_istft_pair_test.argtypes = [P, P, P, i32, i32, P, P, P]
    lib.sepvad_stft.restype = i32
    lib.sepvad_stft.argtypes = [P, P, i32, i32, P, P, P]
    lib.sepvad_istft.restype = i32
    lib.sepvad_istft.argtypes = [P, P, i32, i32, P, P]
    i64 = ctypes.c_int64
    lib.sepvad_pit_l1.restype = i32
    lib.sepvad_pit_l1.argtypes = [P, i64, P, i64, i32, i64, P, P, P, P, P]
    lib.sepvad_stream_append.restype = i32
    lib.sepvad_stream_append.argtypes = [P, i64, i64, i32, i64, P, P, i64, i64, P]
    lib.sepvad_resample_filter.restype = i32
    lib.sepvad_resample_filter.argtypes = [i32, i32, P, i32, P]
    lib.sepvad_resample.restype = i32
    lib.sepvad_resample.argtypes = [P, i64, P, P, P, i64, P]
    lib.sepvad_normalize.restype = i32
    lib.sepvad_normalize.argtypes = [P, i64, P, P, P]
    lib.sepvad_si_sdr.restype = i32
    lib.sepvad_si_sdr.argtypes = [P, i64, P, i64, i64, i32, P, P, i32, P, P]
    lib.sepvad_vad_accuracy.restype = i32
    lib.sepvad_vad_accuracy.argtypes = [P, P, i32, i32, i32, i32, P, P]
    dptr = ctypes.POINTER(ctypes.c_double)
    lib.sepvad_rir_generate.restype = i32
    lib.sepvad_rir_generate.argtypes = [ctypes.c_double, ctypes.c_double, dptr, i32, dptr, dptr, dptr, i32, dptr,
                                        i32, i32, i32, i32, ctypes.c_char, dptr, i64]
    lib.sepvad_set_timing.restype = i32
    lib.sepvad_set_timing.argtypes = [P, i32]
    lib.sepvad_timing.restype = i32
    lib.sepvad_timing.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double)]
    lib.sepvad_destroy.restype = None
    lib.sepvad_destroy.argtypes = [P]
    lib.sepvad_last_error.restype = ctypes.c_char_p
    lib.sepvad_last_error.argtypes = []
    lib.sepvad_abi_version.restype = i32
    lib.sepvad_abi_version.argtypes = []
    lib.sepvad_build_id.restype = ctypes.c_char_p
    lib.sepvad_build_id.argtypes = []
    _lib = lib
    return lib


def _check(rc, what):
    if rc != 0:
        msg = _lib.sepvad_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def make_config(cfg: dict, precision: str = "f16x3") -> SepVadConfig:
    c = SepVadConfig()
    c.n_fft, c.bn_dim, c.h_dim = cfg["n_fftBins"], cfg["BN_dim"], cfg["H_dim"]
    c.layer, c.stack, c.num_spk = cfg["layer"], cfg["stack"], cfg["num_spk"]
    c.tf_attention = int(bool(cfg["tf_attention"]))
    c.ln_mode = (SEPVAD_LN_RECURSIVE if cfg["apply_recursive_ln"] else
                 SEPVAD_LN_RESIDUAL if cfg["apply_residual_ln"] else SEPVAD_LN_PLAIN)
    c.final_vad = int(bool(cfg["final_vad"]))
    c.final_vad_masked_speakers = int(bool(cfg["final_vad_masked_speakers"]))
    c.noisy_phase = int(bool(cfg["noisy_phase"]))
    c.activity_input = int(bool(cfg["activity_input_bool"]))
    c.precision = PRECISIONS[precision]
    return c


def make_kw(inference_kw) -> SepVadInferKw | None:
    """inference_kw dict -> struct (None or {} == the reference's skipped branch, model/model.py:444)."""
    if not inference_kw:
        return None
    k = SepVadInferKw()
    k.enabled = 1
    # the reference indexes these keys directly (KeyError if absent) — keep that behaviour
    k.filter_signals_by_smo_vad = int(bool(inference_kw["filter_signals_by_smo_vad"]))
    k.filter_signals_by_unsmo_vad = int(bool(inference_kw["filter_signals_by_unsmo_vad"]))
    k.length_smoothing_filter = int(inference_kw["length_smoothing_filter"])
    k.threshold_activated_vad = float(inference_kw["threshold_activated_vad"])
    k.return_smoothed_vad = int(bool(inference_kw["return_smoothed_vad"]))
    return k


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class Handle:
    """Owns one ``sepvad_handle`` (device weights + workspace) for one device."""

    def __init__(self, cfg: dict, state_dict: dict, device, precision: str = "f16x3"):
        lib = load_library()
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("libsepvad needs a ROCm device")
        self.device = device
        self.index = device.index if device.index is not None else torch.cuda.current_device()
        self.cfg = dict(cfg)
        host = [(k, v.detach().to("cpu", torch.float32).contiguous()) for k, v in state_dict.items()
                if torch.is_floating_point(v)]
        n = len(host)
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for _, t in host])
        names = (ctypes.c_char_p * n)(*[k.encode() for k, _ in host])
        numels = (ctypes.c_int64 * n)(*[t.numel() for _, t in host])
        self._c = make_config(cfg, precision)
        self.precision = precision
        h = lib.sepvad_create(ctypes.byref(self._c), ptrs, names, numels, n, self.index)
        if not h:
            raise RuntimeError("sepvad_create failed: " + lib.sepvad_last_error().decode(errors="replace"))
        self._h = ctypes.c_void_p(h)
        self._lib = lib

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.sepvad_destroy(h)
            self._h = None

    @property
    def raw(self):
        return self._h

    def reserve(self, B: int, N: int):
        _check(self._lib.sepvad_reserve(self._h, B, N), "sepvad_reserve")

    def set_precision(self, precision: str):
        _check(self._lib.sepvad_set_precision(self._h, PRECISIONS[precision]), "sepvad_set_precision")
        self.precision = precision

    def set_weight_lo(self, mode: str):
        """Weight lo plane of the fused TCN's f16x3 GEMMs: "i8" (default) / "e4m3" (3 B per weight) or "f16"."""
        if mode not in WEIGHT_LO:
            raise ValueError(f"unknown weight lo-plane format {mode!r} (expected one of {sorted(WEIGHT_LO)})")
        _check(self._lib.sepvad_set_weight_lo(self._h, WEIGHT_LO[mode]), "sepvad_set_weight_lo")
        self.weight_lo = mode

    def set_split(self, nsplit: int):
        """Concurrent utterance chunks per forward (1..4; bitwise-identical results)."""
        _check(self._lib.sepvad_set_split(self._h, int(nsplit)), "sepvad_set_split")

    def set_fused(self, on: bool):
        """TCN schedule of later forwards: one persistent launch (default) or one launch per stage."""
        _check(self._lib.sepvad_set_fused(self._h, int(bool(on))), "sepvad_set_fused")

    def fused_status(self) -> bool:
        """Synchronise; True if the last forward ran the fused TCN. Raises if its hand-offs gave up."""
        used = ctypes.c_int32(0)
        _check(self._lib.sepvad_fused_status(self._h, ctypes.byref(used)), "sepvad_fused_status")
        return bool(used.value)

    def fused_slices(self) -> int:
        """Synchronise; the 32-frame slices per workgroup of the last forward's fused TCN (1 or 2; 0 = not fused).
        Raises if its hand-offs gave up."""
        used = ctypes.c_int32(0)
        _check(self._lib.sepvad_fused_status(self._h, ctypes.byref(used)), "sepvad_fused_status")
        return int(used.value)

    def set_timing(self, on: bool):
        _check(self._lib.sepvad_set_timing(self._h, int(on)), "sepvad_set_timing")

    def timing(self):
        ms = (ctypes.c_double * 2)()
        cnt = (ctypes.c_int32 * 2)()
        tot = ctypes.c_double()
        _check(self._lib.sepvad_timing(self._h, ms, cnt, ctypes.byref(tot)), "sepvad_timing")
        return dict(gemm_ms=ms[0], res_out_ms=ms[1], gemm_launches=cnt[0], res_out_launches=cnt[1], total_ms=tot.value)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def forward(self, x: torch.Tensor, inference_kw=None, return_aux: bool = False, outputs: dict | None = None):
        """One forward. Returns dict(sep, vad, est[, spectrum, masks_b, mask_per_speaker])."""
        if x.device.type != "cuda":
            raise RuntimeError("sepvad forward: input must be a ROCm device tensor")
        x = x.to(self.device, torch.float32)
        if x.stride(-1) != 1 or x.stride(0) < x.shape[-1]:
            x = x.contiguous()
        B, N = x.shape
        ldx = x.stride(0) if B > 1 else N  # strided row views (streaming windows) need no copy
        T = 1 + N // (self.cfg["n_fftBins"] // 2)
        F = self.cfg["n_fftBins"] // 2 + 1
        S = self.cfg["num_spk"]
        dev = self.device
        o = outputs or {}
        sep = o.get("sep") if o.get("sep") is not None else torch.empty(B, S, N, device=dev, dtype=torch.float32)
        has_vad = bool(self.cfg["final_vad"]) and (not self.cfg["final_vad_masked_speakers"] or self.cfg["noisy_phase"])
        vad = (o.get("vad") if o.get("vad") is not None else torch.empty(B, S, T, device=dev, dtype=torch.float32)) \
            if has_vad else None
        est = o.get("est") if o.get("est") is not None else torch.empty(B, S, F, T, device=dev, dtype=torch.complex64)
        spectrum = masks_b = mask = None
        if return_aux:
            spectrum = torch.empty(B, F, T, device=dev, dtype=torch.float32)
            masks_b = torch.empty(B, S * F, T, device=dev, dtype=torch.float32)
            mask = torch.empty(B, S, F, T, device=dev, dtype=torch.float32)
        outs = SepVadOutputs(_ptr(sep).value, _ptr(vad).value, _ptr(est).value, _ptr(spectrum).value,
                             _ptr(masks_b).value, _ptr(mask).value)
        kw = make_kw(inference_kw)
        stream = self._stream()
        rc = self._lib.sepvad_forward_strided(self._h, _ptr(x), ldx, B, N, ctypes.byref(outs),
                                              ctypes.byref(kw) if kw is not None else None, stream)
        _check(rc, "sepvad_forward")
        if CHECK_EACH_FORWARD:
            self.fused_status()  # synchronises; raises if this forward's fused TCN gave up
        if vad is None:
            vad_ret = 0  # model/model.py:427
        elif kw is not None and kw.return_smoothed_vad:
            vad_ret = vad.view(B, S, 1, T)  # model/model.py:456-457
        else:
            vad_ret = vad
        seq = ctypes.c_int64()
        lb, ln = ctypes.c_int32(), ctypes.c_int32()
        _check(self._lib.sepvad_last_forward(self._h, stream, ctypes.byref(seq), ctypes.byref(lb), ctypes.byref(ln)),
               "sepvad_last_forward")
        res = dict(sep=sep, vad=vad_ret, est=est, stream=stream.value or 0, B=B, T=T, N=N, seq=seq.value)
        if return_aux:
            res.update(spectrum=spectrum, masks_b=masks_b, mask_per_speaker=mask)
        return res

    def forward_windows(self, x: torch.Tensor, n_win: int, hop: int, N: int, inference_kw=None):
        """Every streaming window in ONE forward (sepvad_forward_windows): window k of row b of x [B, L]
        starts at sample k * hop; returns sep [n_win, B, num_spk, N] (window-major). No est is produced."""
        if x.device.type != "cuda" or x.dtype != torch.float32 or x.stride(-1) != 1:
            raise RuntimeError("forward_windows: x must be a float32 ROCm tensor with unit sample stride")
        B = x.shape[0]
        S = self.cfg["num_spk"]
        T = 1 + N // (self.cfg["n_fftBins"] // 2)
        sep = torch.empty(n_win, B, S, N, device=self.device, dtype=torch.float32)
        has_vad = bool(self.cfg["final_vad"]) and (not self.cfg["final_vad_masked_speakers"] or self.cfg["noisy_phase"])
        vad = torch.empty(n_win * B, S, T, device=self.device, dtype=torch.float32) if has_vad else None
        outs = SepVadOutputs(_ptr(sep).value, _ptr(vad).value, 0, 0, 0, 0)
        kw = make_kw(inference_kw)
        ld = x.stride(0) if B > 1 else x.shape[1]
        _check(self._lib.sepvad_forward_windows(self._h, _ptr(x), ld, B, n_win, hop, N, ctypes.byref(outs),
                                                ctypes.byref(kw) if kw is not None else None, self._stream()),
               "sepvad_forward_windows")
        if CHECK_EACH_FORWARD:
            self.fused_status()
        return sep

    def side_outputs(self, stream: int, B: int, T: int, want=("spectrum", "masks_b", "mask_per_speaker"),
                     seq: int | None = None, N: int | None = None):
        """The side attributes of forward `seq` (shape B x N) on `stream` (sepvad_side_outputs_of), materialised
        now on that stream: dict with the requested subset of spectrum [B,257,T], masks_b [B,514,T] and
        mask_per_speaker [B,2,257,T]. Raises RuntimeError if a later forward on that stream replaced its workspace
        (nothing is written then). Without seq: the last forward on the stream (sepvad_side_outputs).
        The tensors are safe to use on the caller's current stream (it waits for the copies)."""
        F = self.cfg["n_fftBins"] // 2 + 1
        S = self.cfg["num_spk"]
        cur = torch.cuda.current_stream(self.device)
        fwd = torch.cuda.ExternalStream(stream, device=self.device) if cur.cuda_stream != stream else cur
        res = {}
        with torch.cuda.stream(fwd):
            dev = self.device
            if "spectrum" in want:
                res["spectrum"] = torch.empty(B, F, T, device=dev, dtype=torch.float32)
            if "masks_b" in want:
                res["masks_b"] = torch.empty(B, S * F, T, device=dev, dtype=torch.float32)
            if "mask_per_speaker" in want:
                res["mask_per_speaker"] = torch.empty(B, S, F, T, device=dev, dtype=torch.float32)
            outs = SepVadOutputs(0, 0, 0, _ptr(res.get("spectrum")).value, _ptr(res.get("masks_b")).value,
                                 _ptr(res.get("mask_per_speaker")).value)
            if seq is None:
                rc = self._lib.sepvad_side_outputs(self._h, ctypes.byref(outs), ctypes.c_void_p(stream))
            else:
                rc = self._lib.sepvad_side_outputs_of(self._h, ctypes.byref(outs), ctypes.c_void_p(stream), seq, B, N)
            _check(rc, "sepvad_side_outputs")
        if fwd is not cur:  # the caller's stream waits for the copies; the allocator keeps the blocks until then
            cur.wait_stream(fwd)
            for t in res.values():
                t.record_stream(cur)
        return res

    def release_stream(self, stream: int | None = None):
        """Free the per-stream context (workspace, hand-off words) the handle keeps for `stream` (default: the
        current stream) after synchronising it (sepvad_release_stream)."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        _check(self._lib.sepvad_release_stream(self._h, ctypes.c_void_p(stream)), "sepvad_release_stream")

    def tcn_clock(self, max_records: int = 4096):
        """Per-launch k_tcn clock records (diagnostics; needs SEPVAD_TCN_CLOCK=1 when the forwards ran):
        numpy [n, 3] of (launch span us, workgroup 0 span us, workgroup 0 shader clock MHz), oldest first."""
        import numpy as np
        buf = (ctypes.c_uint64 * (8 * max_records))()
        n = ctypes.c_int32(0)
        _check(self._lib.sepvad_tcn_clock(self._h, buf, max_records, ctypes.byref(n)), "sepvad_tcn_clock")
        k = min(n.value, max_records)
        u = np.frombuffer(buf, dtype=np.uint64, count=8 * k).reshape(k, 8)
        span = (u[:, 1] - ~u[:, 0]).astype(np.float64) / 100.0  # the min start is stored as a max of complements
        r = u.astype(np.float64)
        w0 = (r[:, 3] - r[:, 2]) / 100.0
        mhz = (r[:, 5] - r[:, 4]) / np.maximum(w0, 1e-9)
        return np.stack([span, w0, mhz], axis=1)

    def tcn_dump(self, x: torch.Tensor):
        """Block-level parity probe (sepvad_set_tcn_dump): one forward of x with the fused TCN, returning
        (tcn_in, blk0_res, blk0_att) as [B, 256, T] like the reference module outputs."""
        B, N = x.shape
        T = 1 + N // 256
        Tp = (T + 63) // 64 * 64
        buf = torch.zeros(3, B, Tp, 256, device=self.device, dtype=torch.float32)
        _check(self._lib.sepvad_set_tcn_dump(self._h, _ptr(buf)), "sepvad_set_tcn_dump")
        try:
            self.forward(x)
            if not self.fused_status():
                raise RuntimeError("tcn_dump: the fused TCN did not run")
        finally:
            _check(self._lib.sepvad_set_tcn_dump(self._h, None), "sepvad_set_tcn_dump")
        v = buf[:, :, :T, :].permute(0, 1, 3, 2)
        return v[0], v[1], v[2]

    def stft(self, x: torch.Tensor):
        """STFT with DC zeroed and its dB spectrum (kernel-level test entry)."""
        x = x.to(self.device, torch.float32).contiguous()
        B, N = x.shape
        T = 1 + N // 256
        X = torch.empty(B, 257, T, device=self.device, dtype=torch.complex64)
        spec = torch.empty(B, 257, T, device=self.device, dtype=torch.float32)
        _check(self._lib.sepvad_stft(self._h, _ptr(x), B, N, _ptr(X), _ptr(spec), self._stream()), "sepvad_stft")
        return X, spec

    def stft_fused(self, x: torch.Tensor):
        """The forward's own front end (k_stft_gate, sepvad_stft_gate_test): (X [B, 257, T] complex64 with DC
        zeroed, its dB spectrum [B, 257, T]) from the frame-major workspace layout."""
        x = x.to(self.device, torch.float32).contiguous()
        B, N = x.shape
        T = 1 + N // 256
        Tp = (T + 63) // 64 * 64
        X = torch.zeros(B, Tp, 257, device=self.device, dtype=torch.complex64)
        db = torch.zeros(B, Tp, 260, device=self.device, dtype=torch.float32)
        _check(self._lib.sepvad_stft_gate_test(self._h, _ptr(x), B, N, _ptr(X), _ptr(db), self._stream()),
               "sepvad_stft_gate_test")
        return X[:, :T].transpose(1, 2), db[:, :T, :257].transpose(1, 2)

    def istft_pair(self, X: torch.Tensor, masks: torch.Tensor, N: int):
        """The forward's own back end (k_istft_pair, sepvad_istft_pair_test): for X [B, 257, T] complex and
        pre-sigmoid masks [B, 2, 257, T], est = X sigmoid(masks) [B, 2, 257, T] and y = istft(est, length=N)
        [B, 2, N]."""
        B, F, T = X.shape
        Tp = (T + 63) // 64 * 64
        Xf = torch.zeros(B, Tp, 257, device=self.device, dtype=torch.complex64)
        Xf[:, :T] = X.to(self.device, torch.complex64).transpose(1, 2)
        mf = torch.zeros(B, Tp, 576, device=self.device, dtype=torch.float32)
        mf[:, :T, :514] = masks.to(self.device, torch.float32).reshape(B, 514, T).transpose(1, 2)
        y = torch.empty(B, 2, N, device=self.device, dtype=torch.float32)
        est = torch.empty(B, 2, 257, T, device=self.device, dtype=torch.complex64)
        _check(self._lib.sepvad_istft_pair_test(self._h, _ptr(Xf), _ptr(mf), B, N, _ptr(y), _ptr(est), self._stream()),
               "sepvad_istft_pair_test")
        return y, est

    def istft(self, est: torch.Tensor, N: int):
        """torch.istft(center=True, length=N) of est [BS, 257, T] complex64 (kernel-level test entry)."""
        est = est.to(self.device, torch.complex64).contiguous()
        BS = est.shape[0]
        y = torch.empty(BS, N, device=self.device, dtype=torch.float32)
        _check(self._lib.sepvad_istft(self._h, _ptr(est), BS, N, _ptr(y), self._stream()), "sepvad_istft")
        return y
