"""ORACLE — test infrastructure only. Not part of the product path.

CPU restatement of the reference Sep-TFAnet^VAD forward (reference ``model/model.py:402-461``)
written functionally on torch CPU ops, for float32 or float64. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module, and
only as the checker / the timed CPU baseline — never as the thing shipped.

Parity of this restatement is pinned against golden vectors produced by the reference itself
(``tests/golden/make_golden.py`` imports ``/root/reference/model/model.py`` through an offline
torchaudio shim) — see ``tests/test_oracle_golden.py``.

The torchaudio semantics restated here (reference ``model/model.py:5,19-20,382-387``):
  Spectrogram(n_fft=512, hop=256, win=512, hann, power=None) ->
      torch.stft(center=True, pad_mode='reflect', normalized=False, onesided=True)
  InverseSpectrogram(...) -> torch.istft(center=True, normalized=False, onesided=True, length=N)
  AmplitudeToDB('power', top_db=None) -> 10*log10(clamp(x, 1e-10))
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPS_1E8 = 1e-8  # GroupNorm eps of TCN.LN, reg1, reg2, vad BN_1 (model/model.py:123-124,161,274)
EPS_DEF = 1e-5  # GroupNorm default eps of ln_first/second, ln_modules, TCN.output.1 (:314-319,323)


def _merge(config):
    from_defaults = dict(n_fftBins=512, BN_dim=256, H_dim=512, layer=8, stack=3, kernel=3,
                         num_spk=2, skip=False, dilated=True, casual=False, bool_drop=True,
                         drop_value=0.1, weight_norm=False, final_vad=True, noisy_phase=False,
                         activity_input_bool=False, tf_attention=False, apply_recursive_ln=False,
                         apply_residual_ln=False, final_vad_masked_speakers=False)
    from_defaults.update(config)
    return from_defaults


def wn_weight(sd, prefix, dtype):
    """torch.nn.utils.weight_norm: w = v * (g / ||v||), norm over all dims but 0 (model/model.py:7)."""
    g = sd[prefix + ".weight_g"].to(dtype)
    v = sd[prefix + ".weight_v"].to(dtype)
    norm = v.flatten(1).norm(dim=1).reshape(-1, *([1] * (v.dim() - 1)))
    return v * (g / norm)


def prelu(x, w):
    return torch.where(x >= 0, x, w * x)


def gn1(x, weight, bias, eps):
    """GroupNorm(1, C) on [B, C, T]."""
    return F.group_norm(x, 1, weight, bias, eps)


class OracleModel:
    """Callable CPU restatement: ``OracleModel(config, state_dict, dtype)(x, inference_kw)``.

    Returns (sep, vad, est) and sets ``spectrum``, ``masks_b``, ``mask_per_speaker`` like the
    reference (model/model.py:412,421,423,429).
    """

    def __init__(self, config: dict, state_dict: dict, dtype=torch.float32):
        self.cfg = _merge(config)
        self.dtype = dtype
        self.sd = {k: torch.as_tensor(v) for k, v in state_dict.items()}
        cfg = self.cfg
        self.nblk = cfg["layer"] * cfg["stack"]
        self.dil = [1 if i == 0 else i % 4 + 1 for _ in range(cfg["stack"]) for i in range(cfg["layer"])]
        d = dtype
        sd = self.sd
        # weight-norm folded once; the reference recomputes it in a pre-forward hook (numerically equal)
        self.blocks = []
        for i in range(self.nblk):
            p = f"TCN.TCN.{i}"
            self.blocks.append(dict(
                w1=wn_weight(sd, p + ".conv1d", d), b1=sd[p + ".conv1d.bias"].to(d),
                wd=wn_weight(sd, p + ".dconv1d", d), bd=sd[p + ".dconv1d.bias"].to(d),
                w2=wn_weight(sd, p + ".res_out", d), b2=sd[p + ".res_out.bias"].to(d),
                a1=sd[p + ".nonlinearity1.weight"].to(d), a2=sd[p + ".nonlinearity2.weight"].to(d),
                g1=sd[p + ".reg1.weight"].to(d), be1=sd[p + ".reg1.bias"].to(d),
                g2=sd[p + ".reg2.weight"].to(d), be2=sd[p + ".reg2.bias"].to(d),
            ))
        self.w_out = wn_weight(sd, "TCN.output.2", d)
        if cfg["final_vad"]:
            self.w_vad1 = wn_weight(sd, "vad.common.conv1_1", d)
            self.w_vad2 = wn_weight(sd, "vad.output_layer_vad", d)

    def _t(self, name):
        return self.sd[name].to(self.dtype)

    # ---- front end -------------------------------------------------------------------------
    def stft(self, x, window="spec_output.window"):
        """spec_output / spec_input (model/model.py:16-25,384-385,408-410), DC bin zeroed."""
        n_fft = self.cfg["n_fftBins"]
        win = self._t(window)
        X = torch.stft(x, n_fft, hop_length=n_fft // 2, win_length=n_fft, window=win, center=True,
                       pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
        X = X.clone()
        X[:, 0, :] = 0
        return X

    # ---- TCN (model/model.py:329-358) --------------------------------------------------------
    def depthconv(self, blk, o, dil):
        """DepthConv1d.forward with Dropout2d as identity (eval) (model/model.py:130-149)."""
        a = F.conv1d(o, blk["w1"], blk["b1"])
        h = gn1(prelu(a, blk["a1"]), blk["g1"], blk["be1"], EPS_1E8)
        d = F.conv1d(h, blk["wd"], blk["bd"], padding=dil, dilation=dil, groups=h.shape[1])
        g = gn1(prelu(d, blk["a2"]), blk["g2"], blk["be2"], EPS_1E8)
        return F.conv1d(g, blk["w2"], blk["b2"])

    def tf_attention(self, i, r):
        """TF_Attention.forward (model/model.py:197-208): sigmoid gates, rank-1 outer product."""
        p = f"TCN.time_freq_attnetion.{i}"
        t = self._t
        mt = r.mean(dim=1, keepdim=True)                          # [B,1,T]
        yt = F.conv1d(mt, t(p + ".conv1d_t_1.weight"), t(p + ".conv1d_t_1.bias"), padding=1)
        yt = F.conv1d(yt, t(p + ".conv1d_t_2.weight"), t(p + ".conv1d_t_2.bias"), padding=2, dilation=2)
        at = torch.sigmoid(prelu(yt, t(p + ".prelu_t.weight")))   # [B,1,T]
        mf = r.mean(dim=2, keepdim=True).transpose(1, 2)          # [B,1,C]
        yf = F.conv1d(mf, t(p + ".conv1d_f_1.weight"), t(p + ".conv1d_f_1.bias"), padding=1)
        yf = F.conv1d(yf, t(p + ".conv1d_f_2.weight"), t(p + ".conv1d_f_2.bias"), padding=2, dilation=2)
        af = torch.sigmoid(prelu(yf, t(p + ".prelu_f.weight"))).transpose(1, 2)  # [B,C,1]
        return r * torch.bmm(af, at)

    def tcn(self, s):
        cfg, t = self.cfg, self._t
        o = gn1(s, t("TCN.LN.weight"), t("TCN.LN.bias"), EPS_1E8)
        for i in range(self.nblk):
            r = self.depthconv(self.blocks[i], o, self.dil[i])
            if cfg["tf_attention"]:
                r = self.tf_attention(i, r)
            if cfg["apply_recursive_ln"]:
                u = gn1(o + r, t(f"TCN.ln_first_modules.{i}.weight"), t(f"TCN.ln_first_modules.{i}.bias"), EPS_DEF)
                o = gn1(o + u, t(f"TCN.ln_second_modules.{i}.weight"), t(f"TCN.ln_second_modules.{i}.bias"), EPS_DEF)
            elif cfg["apply_residual_ln"]:
                o = o + gn1(r, t(f"TCN.ln_modules.{i}.weight"), t(f"TCN.ln_modules.{i}.bias"), EPS_DEF)
            else:
                o = o + r
        o = prelu(o, t("TCN.output.0.weight"))
        o = gn1(o, t("TCN.output.1.weight"), t("TCN.output.1.bias"), EPS_DEF)
        return F.conv1d(o, self.w_out, t("TCN.output.2.bias"))

    def vad(self, m):
        """VAD.forward on one speaker's [B,257,T] (model/model.py:173-179)."""
        t = self._t
        y = F.conv1d(m, self.w_vad1, t("vad.common.conv1_1.bias"), padding=2)
        y = gn1(prelu(y, t("vad.common.relu_1.weight")), t("vad.common.BN_1.weight"), t("vad.common.BN_1.bias"), EPS_1E8)
        y = F.conv1d(y, self.w_vad2, t("vad.output_layer_vad.bias"), padding=1)
        return torch.sigmoid(y)

    # ---- forward (model/model.py:402-461) -------------------------------------------------------
    @torch.no_grad()
    def __call__(self, x, inference_kw=None):
        assert x.ndim == 2, "input tensor must be 2 dimensions (B, T)"
        cfg, t = self.cfg, self._t
        x = x.to(self.dtype)
        N = x.shape[-1]
        F_ = cfg["n_fftBins"] // 2 + 1
        ns = cfg["num_spk"]
        X = self.stft(x)                                          # stft_out [B,F,T] (model/model.py:408)
        Xin = X                                                   # stft (:409): the same unless the windows differ
        if not torch.equal(self._t("spec_input.spec.window"), self._t("spec_output.window")):
            Xin = self.stft(x, "spec_input.spec.window")
        power = Xin.abs() ** 2
        spec = 10.0 * torch.log10(torch.clamp(power, min=1e-10))
        if cfg["activity_input_bool"]:
            g = F.conv2d(spec.unsqueeze(1), t("activity_input.weight"), t("activity_input.bias"), padding=1)
            spec = spec * prelu(g.squeeze(1), t("prelu.weight"))
        self.spectrum = spec
        masks_b = self.tcn(spec[:, 1:])
        B, _, T = masks_b.shape
        self.masks_b = masks_b
        mps = masks_b.reshape(B, ns, F_, T)
        vad = 0
        if cfg["final_vad"] and not cfg["final_vad_masked_speakers"]:
            vad = torch.cat([self.vad(mps[:, s]) for s in range(ns)], dim=1)
        mask = torch.sigmoid(mps)
        self.mask_per_speaker = mask
        if cfg["noisy_phase"]:
            mag = X.abs().unsqueeze(1) * mask
            if cfg["final_vad"] and cfg["final_vad_masked_speakers"]:
                vad = torch.cat([self.vad(mag[:, s]) for s in range(ns)], dim=1)
            ctype = torch.complex64 if self.dtype == torch.float32 else torch.complex128
            est = mag.to(ctype) * torch.exp(1j * X.angle()).unsqueeze(1)
        else:
            est = X.unsqueeze(1) * mask
        if inference_kw and cfg["final_vad"]:
            # model/model.py:444-457: threshold, [1,0,1] smoothing (centre weight 0), edges copied
            thr = (vad.unsqueeze(2) >= inference_kw["threshold_activated_vad"]).to(self.dtype)  # [B,ns,1,T]
            k = torch.tensor([[[1.0, 0.0, 1.0]]], dtype=self.dtype)
            sm = torch.stack([F.conv1d(thr[:, s], k, padding=1) for s in range(ns)], dim=1)
            sm = torch.minimum(sm, torch.tensor(1.0, dtype=self.dtype))
            sm[..., [0, -1]] = thr[..., [0, -1]]
            if inference_kw["filter_signals_by_smo_vad"] or inference_kw["filter_signals_by_unsmo_vad"]:
                est = sm * est
            if inference_kw["return_smoothed_vad"]:
                vad = sm
        self.estimated_stfts = est
        n_fft = cfg["n_fftBins"]
        sep = torch.istft(est.reshape(-1, F_, T), n_fft, hop_length=n_fft // 2, win_length=n_fft,
                          window=t("inv_spec.window"), center=True, normalized=False, onesided=True,
                          length=N, return_complex=False).reshape(B, ns, N)
        return sep, vad, est

    # ---- intermediates for kernel-level checks -------------------------------------------------
    @torch.no_grad()
    def block_io(self, x, upto: int):
        """Return the TCN state ``o`` entering block ``upto`` (after LN and ``upto`` blocks)."""
        cfg, t = self.cfg, self._t
        X = self.stft(x.to(self.dtype))
        spec = 10.0 * torch.log10(torch.clamp(X.abs() ** 2, min=1e-10))
        if cfg["activity_input_bool"]:
            g = F.conv2d(spec.unsqueeze(1), t("activity_input.weight"), t("activity_input.bias"), padding=1)
            spec = spec * prelu(g.squeeze(1), t("prelu.weight"))
        o = gn1(spec[:, 1:], t("TCN.LN.weight"), t("TCN.LN.bias"), EPS_1E8)
        for i in range(upto):
            r = self.depthconv(self.blocks[i], o, self.dil[i])
            if cfg["tf_attention"]:
                r = self.tf_attention(i, r)
            if cfg["apply_recursive_ln"]:
                u = gn1(o + r, t(f"TCN.ln_first_modules.{i}.weight"), t(f"TCN.ln_first_modules.{i}.bias"), EPS_DEF)
                o = gn1(o + u, t(f"TCN.ln_second_modules.{i}.weight"), t(f"TCN.ln_second_modules.{i}.bias"), EPS_DEF)
            elif cfg["apply_residual_ln"]:
                o = o + gn1(r, t(f"TCN.ln_modules.{i}.weight"), t(f"TCN.ln_modules.{i}.bias"), EPS_DEF)
            else:
                o = o + r
        return o


def si_sdr(preds, target, zero_mean=True):
    """calc_sisdr (reference model/combined_loss.py:16-56): EPS = finfo(dtype).eps."""
    eps = torch.finfo(preds.dtype).eps
    if zero_mean:
        target = target - target.mean(dim=-1, keepdim=True)
        preds = preds - preds.mean(dim=-1, keepdim=True)
    alpha = ((preds * target).sum(-1, keepdim=True) + eps) / ((target ** 2).sum(-1, keepdim=True) + eps)
    ts = alpha * target
    noise = ts - preds
    return 10 * torch.log10(((ts ** 2).sum(-1) + eps) / ((noise ** 2).sum(-1) + eps))


def accuracy_vad(preds, targets):
    """Accuracy_Vad (reference model/metric.py:163-177) on numpy arrays [B, S, T]: labels = preds > 0.5
    (in the reference's order: > 0.5 -> 1, then <= 0.5 -> 0, NaN untouched); returns (labels, [acc, acc0, acc1])
    in float32 like torch's int64-sum / numel."""
    import numpy as np
    p = np.array(preds, dtype=np.float32, copy=True)
    p[p > 0.5] = 1
    p[p <= 0.5] = 0
    eq = p == targets
    n = np.float32(targets.size)
    accs = [np.float32(eq.sum()) / n] + [np.float32(eq[:, s].sum()) / np.float32(targets[:, s].size)
                                         for s in range(targets.shape[1])]
    return p, np.array(accs, dtype=np.float32)
