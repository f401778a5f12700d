// The forward's back end (model/model.py:160-179,429-460): k_istft_pair — VAD tail, est = X sigmoid(mask)
// [* smoothed VAD], torch.istft — for both speakers of a chunk of frames, with the inverse transforms as a
// register-resident four-step 16 x 16 FFT. Built with -fno-slp-vectorize (Makefile): hipcc's packing of the
// complex arithmetic into v_pk_* pairs adds register moves and pushed the kernel from 54 to 98 VGPRs.
#include "device_common.h"
#include "fft_common.h"

namespace sepvad {

// Inverse real 512-point transform of one est row (16 lanes per frame, c = lane & 15) as the 256-point
// complex inverse transform of z[m] = x[2m] + i x[2m+1] (as in k_istft): the split step produces this
// lane's column z[16 r + c] directly in registers; step 1 DFT over r; twiddle W256^(-c k1); XOR-swizzled
// transpose through the row (element (k1, n2) at 16 k1 + (n2 ^ k1): conflict-free both ways); step 2 DFT
// over n2 gives z[c + 16 k2]; the windowed, scaled time samples overwrite the row. The caller's row must be
// complete (barrier) on entry; the wave's other 48 lanes work on three other rows.
__device__ __forceinline__ void irfft512_col(float2* Y, float gain, const float2* tw, const float* win, int c) {
  float2 x[16];
  // three lane bases; every per-element address below is base + immediate (hipcc otherwise hoists ~50
  // computed addresses and spills them)
  const float2* Yc = Y + c;
  const float2* Ym = Y + (16 - c);
  const float2* twc = tw + c;
  // split step for the column's 16 inputs in the order of the first radix-4 pass (na, na + 4, na + 8,
  // na + 12), each group of four consumed by its dft4 at once (bounded register demand)
#pragma unroll
  for (int na = 0; na < 4; ++na) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int r = na + 4 * nb;
      const int k = c + 16 * r;  // 0..255
      const float2 y0 = Yc[16 * r], y1 = Ym[16 * (15 - r)];  // Y[k], Y[256 - k] (immediate offsets)
      float2 yk = make_float2(gain * y0.x, gain * y0.y), ym = make_float2(gain * y1.x, gain * y1.y);
      if (k == 0) { yk.y = 0.f; ym.y = 0.f; }  // c2r ignores Im of DC and Nyquist
      const float2 cym = conjf2(ym);
      const float2 E = make_float2(0.5f * (yk.x + cym.x), 0.5f * (yk.y + cym.y));
      const float2 Dd = csub(yk, cym);
      float2 w = twc[16 * r];
      w.y = -w.y;  // W512^{-k}
      const float2 Oo = cmul(make_float2(0.5f * Dd.x, 0.5f * Dd.y), w);
      x[r] = make_float2(E.x - Oo.y, E.y + Oo.x);  // E + i O
    }
    dft4<true>(x[na], x[na + 4], x[na + 8], x[na + 12]);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  dft16_tail<true>(x);  // A[k1] at slot d16(k1)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {  // W256^(-c k1) = conj(W512^(2 c k1))
    float2 w = twid<true>(tw, mul_late(c, 2 * k1));
    w.y = -w.y;
    x[d16(k1)] = cmul(x[d16(k1)], w);
    if (k1 % 4 == 3) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  wave_lds_sync();  // every lane's reads of the row done before the transpose overwrites it
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) Y[16 * k1 + xor_late(c, k1)] = x[d16(k1)];
  wave_lds_sync();
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) x[n2] = Y[16 * c + xor_late(c, n2)];  // row k1 = c of the transpose
  wave_lds_sync();
  dft16<true>(x);  // z[c + 16 k2] at slot d16(k2)
  __builtin_amdgcn_sched_barrier(0);
  float2* frc = Y + c;  // time samples 2m, 2m+1 (m = c + 16 k2) as one float2 per m
  const float2* winc = reinterpret_cast<const float2*>(win) + c;
  const float sc = 1.f / 256.f;  // 1/N of the 512-point c2r == 1/256 on the half-length transform
#pragma unroll
  for (int k2 = 0; k2 < 16; ++k2) {
    const float2 v = x[d16(k2)];
    const float2 wv = winc[16 * k2];
    frc[16 * k2] = make_float2(v.x * sc * wv.x, v.y * sc * wv.y);
    if (k2 % 4 == 3) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The forward's back end (est_mode 1): one workgroup (8 waves) per (utterance, chunk of IP_OWN frames) for
// BOTH speakers, so each X row is read once for the two masks. Frames [f0-1, f0+IP_OWN) of both speakers:
// 2 * IP_FR = 24 transforms, 3 rounds of 8 waves; owned output segments [f0, f0+IP_OWN) (+ segment T for
// the last chunk). The transforms run in place in the frames' own LDS rows (fft256_inplace), so the
// workgroup needs ~52 KB: three per CU, and at T = 126 the 64 x 12 workgroups of a B = 64 forward are all
// resident at once (one round). Overlap-add: one reciprocal window envelope per thread (its sample phase q
// is fixed across its segments), then products.
constexpr int IP_OWN = 11;
constexpr int IP_FR = IP_OWN + 1;
#ifndef ISTFT_WAVES
#define ISTFT_WAVES 6   // waves per SIMD the register budget must allow: 6 -> three 8-wave workgroups per CU
#endif
__global__ __launch_bounds__(512, ISTFT_WAVES) void k_istft_pair(IstftArgs a) {
  __shared__ float2 tw[256];
  __shared__ __attribute__((aligned(16))) float2 spec[2][IP_FR][NBIN + 1];  // (16-B aligned: float4 overlap-add reads)  // est of the computed frames; transformed in place
  __shared__ float yn[2][4][IP_FR + 6];   // GN'd VAD features, frames fbeg-3 .. fbeg+IP_FR+2
  __shared__ float vadv[2][IP_FR + 4];    // vad at frames fbeg-2 .. fbeg+IP_FR+1
  __shared__ float gain[2][IP_FR];
  __shared__ float vs[2][4], vh[2][4];
  __shared__ double dacc[4];
  __shared__ float vred[2 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x, f0 = blockIdx.y * IP_OWN;
  const int T = a.T;
  const int fbeg = f0 - 1;
  const bool vad = a.has_vad != 0;
  // give-up poisoning (sepvad_internal.h IstftArgs::gerr): NaN outputs for a forward whose fused TCN gave up
  const unsigned gev = a.gerr ? *a.gerr : 0u;
  const bool poison =
      gev != 0u && ((gev >> TCN_EPOCH_BITS) - a.gsalt_lo & ((1u << (32 - TCN_EPOCH_BITS)) - 1u)) < a.gsalt_n;
  const float qnan = __builtin_nanf("");
  // diagnostics: slot 0 wall clock at entry, slots 1.. shader clock at the phase ends
  unsigned long long* const pr = a.probe ? a.probe + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
  auto stamp = [&](int k) {
    if (pr && tid == 0) pr[k] = __builtin_amdgcn_s_memtime();
  };
  if (pr && tid == 0) pr[0] = wall_clock64();
  stamp(1);
  if (tid < 256) tw[tid] = a.tw[tid];

  // every input load first: X and both speakers' mask rows of the computed frames, the VAD features, the
  // BN_1 records and parameters (frames outside [0, T) load a clamped row)
  constexpr int NE = (IP_FR * NBIN + 511) / 512;
  float2 xr[NE];
  float mr[2][NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int i = min(tid + j * 512, IP_FR * NBIN - 1);
    const int fi = i / NBIN, k = i - fi * NBIN;
    const size_t row = (size_t)b * a.Tp + min(max(fbeg + fi, 0), T - 1);
    xr[j] = a.X[row * NBIN + k];
    mr[0][j] = a.masks[row * MOUT_PAD + k];
    mr[1][j] = a.masks[row * MOUT_PAD + NBIN + k];
  }
  constexpr int NQ = IP_FR + 6;
  // VAD conv1_1 from the output head's tap products (vP mode, model/model.py:158-160): y[t][o] = sum_k P[t-2+k][4k+o]
  // (zero outside [0, T)), v = PReLU(y + b1[o]) — k_vad_feat's arithmetic, expression for expression
  const bool taps = vad && a.vP != nullptr;
  auto tap_v = [&](const float* P, int i, int t, int o) {
    float y = 0.f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int tt = t - 2 + k;
      y += (i < 4 * T && tt >= 0 && tt < T) ? P[(size_t)tt * HEAD_VAD_N + 4 * k + o] : 0.f;
    }
    return prelu_f(y + a.vb1[o], a.valpha);
  };
  float yv = 0.f;
  if (vad && tid < 2 * 4 * NQ) {  // thread -> (speaker, feature o, frame q)
    const int sp = tid / (4 * NQ), o = (tid / NQ) % 4, q = tid % NQ;
    const int fc = min(max(fbeg - 3 + q, 0), T - 1);
    yv = taps ? tap_v(a.vP + ((size_t)b * 2 + sp) * a.Tp * HEAD_VAD_N, 4 * fc + o, fc, o)
              : a.vy[(((size_t)b * 2 + sp) * 4 + o) * a.Tp + fc];
  }
  if (taps) {  // BN_1 sums of the whole utterance: 256 threads per speaker, k_vad_feat's items and order
    const int sp = tid >> 8, t8 = tid & 255;
    const float* P = a.vP + ((size_t)b * 2 + sp) * a.Tp * HEAD_VAD_N;
    float st[2] = {0.f, 0.f};
    for (int it = 0; 256 * it < 4 * T; ++it) {
      const int i = t8 + 256 * it;
      const float v = tap_v(P, i, i >> 2, i & 3);
      if (i < 4 * T) { st[0] += v; st[1] += v * v; }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // as block_reduce_store<2> over each speaker's four waves
      const float ws = wave_sum(st[j]);
      if (lane == 0) vred[j * 16 + wave] = ws;
    }
  }

  // 1) X sigmoid(mask) of both speakers into the rows (frame-major, coalesced over bins); the VAD gain is
  // applied when the rows are read (gain * (X m), the same product order as est = X m gain); noisy-phase
  // synthesis (|X| m) e^{j angle X} == X m up to rounding (model/model.py:430-437)
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int i = tid + j * 512;
    if (i < IP_FR * NBIN) {
      const int fi = i / NBIN, k = i - fi * NBIN;
      const int f = fbeg + fi;
      const bool ok = f >= 0 && f < T;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const float m = ok ? sigmoid_f(mr[sp][j]) : 0.f;
        spec[sp][fi][k] = ok ? make_float2(xr[j].x * m, xr[j].y * m) : make_float2(0.f, 0.f);
      }
    }
  }
  stamp(2);

  // side outputs of the owned frames, bin-major [bs][k][f] (IP_OWN consecutive frames per bin): est from the
  // rows, sigmoid(mask) recomputed from the masks (read again: side path only)
  auto side_outputs = [&](bool unit_gain) {
    if (a.est_out && !a.mask_out && T % 2 == 0 && ((uintptr_t)a.est_out & 15) == 0) {
      // the forward's est alone (T even: a row starts 16-B aligned): two frames per 16-B store where the pair is aligned
      // (frames f0 + fo, f0 + fo + 1 with f0 + fo even), the odd one out alone -- half the store instructions of one
      // frame per lane (the store phase is issue-bound: every workgroup of the round stores at once)
      constexpr int NSL6 = (IP_OWN + 2) / 2;  // slots per (speaker, bin) row: 5 pairs and one single frame
      constexpr int NI6 = (2 * NBIN * NSL6 + 511) / 512;
      const int par = f0 & 1;
#pragma unroll
      for (int jj = 0; jj < NI6; ++jj) {
        const int i = tid + jj * 512;
        const int sp = i / (NBIN * NSL6), rem = i - sp * (NBIN * NSL6);
        const int k = rem / NSL6, sl = rem - k * NSL6;
        const int fo = par == 0 ? 2 * sl : (sl == 0 ? 0 : 2 * sl - 1);
        int n = par == 0 ? (fo + 1 < IP_OWN ? 2 : 1) : (sl == 0 ? 1 : 2);
        const int f = f0 + fo;
        if (i < 2 * NBIN * NSL6 && f < T) {
          if (f + 1 >= T) n = 1;
          const size_t o = (((size_t)b * 2 + sp) * NBIN + k) * T + f;
          const float2 e0 = spec[sp][fo + 1][k];
          const float g0 = unit_gain ? 1.f : gain[sp][fo + 1];
          const float2 v0 = poison ? make_float2(qnan, qnan) : make_float2(g0 * e0.x, g0 * e0.y);
          if (n == 2) {
            const float2 e1 = spec[sp][fo + 2][k];
            const float g1 = unit_gain ? 1.f : gain[sp][fo + 2];
            const float2 v1 = poison ? make_float2(qnan, qnan) : make_float2(g1 * e1.x, g1 * e1.y);
            st_out(reinterpret_cast<float4*>(a.est_out + o), make_float4(v0.x, v0.y, v1.x, v1.y));
          } else {
            st_out(a.est_out + o, v0);
          }
        }
      }
      return;
    }
    constexpr int NI = (2 * NBIN * IP_OWN + 511) / 512;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = tid + j * 512;
      const int sp = i / (NBIN * IP_OWN), rem = i - sp * (NBIN * IP_OWN);
      const int k = rem / IP_OWN, fo = rem - k * IP_OWN;
      const int f = f0 + fo;
      if (i < 2 * NBIN * IP_OWN && f < T) {
        const size_t o = (((size_t)b * 2 + sp) * NBIN + k) * T + f;
        if (a.est_out) {
          const float2 e = spec[sp][fo + 1][k];
          const float gg = unit_gain ? 1.f : gain[sp][fo + 1];
          st_out(a.est_out + o, poison ? make_float2(qnan, qnan) : make_float2(gg * e.x, gg * e.y));
        }
        if (a.mask_out)
          st_out(a.mask_out + o, poison ? qnan : sigmoid_f(a.masks[((size_t)b * a.Tp + f) * MOUT_PAD + sp * NBIN + k]));
      }
    }
  };
  // Without VAD filtering of the estimates the gain is 1 on every frame (est = X m): the side outputs go out now,
  // so their stores drain under the VAD tail and the transforms (the same values as after the tail: gain * e with
  // gain = 1 is e)
  const bool early = (a.est_out || a.mask_out) && !(vad && a.kw_enabled && a.filt);
  if (early) {
    lds_sync();  // every row of spec written
    side_outputs(true);
  }

  // 0) VAD tail (model/model.py:160-179,444-457) for the frames of both speakers
  if (vad) {
    float g = 0.f, be = 0.f;
    if (tid < 8) { g = a.vgn.g[tid & 3]; be = a.vgn.be[tid & 3]; }
    if (!a.vy_norm) {  // BN_1 = GroupNorm(1, 4) from k_vad1's records or the tap sums (else vy arrives normalised)
      if (taps) {
        lds_sync();  // vred complete
        if (tid < 4) {  // dacc[2 sp + j]: speaker sp's four wave totals in wave order (double)
          const int sp = tid >> 1, j = tid & 1;
          double s = 0.0;
          for (int i = 0; i < 4; ++i) s += vred[j * 16 + 4 * sp + i];
          dacc[tid] = s;
        }
      } else {
        reduce_records(rec_src(a.vgn, 2 * b, 2), rec_src(a.vgn, 2 * b + 1, 2), dacc);
      }
      lds_sync();
      if (tid < 8) {
        const int sp = tid >> 2, o = tid & 3;
        float mu, rs;
        gn_moments(dacc[2 * sp], dacc[2 * sp + 1], 4.0 * T, a.vgn.eps, mu, rs);
        vs[sp][o] = rs * g;
        vh[sp][o] = be - vs[sp][o] * mu;
      }
      lds_sync();
    }
    if (tid < 2 * 4 * NQ) {
      const int sp = tid / (4 * NQ), o = (tid / NQ) % 4, qq = tid % NQ;
      const int f = fbeg - 3 + qq;
      yn[sp][o][qq] = (f >= 0 && f < T) ? (a.vy_norm ? yv : fmaf(yv, vs[sp][o], vh[sp][o])) : 0.f;
    }
    lds_sync();
    if (tid < 2 * (IP_FR + 4)) {
      const int sp = tid / (IP_FR + 4), qq = tid % (IP_FR + 4);
      const int f = fbeg - 2 + qq;
      float z = a.b2;
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int k = 0; k < 3; ++k) z = fmaf(a.w2[o * 3 + k], yn[sp][o][qq + k], z);
      const float p = sigmoid_f(z);
      vadv[sp][qq] = (f >= 0 && f < T) ? p : 0.f;
      if (!a.kw_enabled && f >= f0 && f < f0 + IP_OWN && f < T) a.vad_out[((size_t)b * 2 + sp) * T + f] = poison ? qnan : p;
    }
    lds_sync();
    if (tid < 2 * IP_FR) {
      const int sp = tid / IP_FR, fi = tid % IP_FR;
      const int f = fbeg + fi;
      float gg = 1.f;
      if (a.kw_enabled && f >= 0 && f < T) {
        auto thr = [&](int ff) -> float {  // threshold of frame ff (0 outside [0,T): zero padding)
          if (ff < 0 || ff >= T) return 0.f;
          return vadv[sp][ff - (fbeg - 2)] >= a.thr ? 1.f : 0.f;
        };
        float smv = fminf(thr(f - 1) + thr(f + 1), 1.f);
        if (f == 0 || f == T - 1) smv = thr(f);
        if (a.filt) gg = smv;
        if (f >= f0 && f < f0 + IP_OWN)
          a.vad_out[((size_t)b * 2 + sp) * T + f] = poison ? qnan : (a.ret_smooth ? smv : vadv[sp][f - (fbeg - 2)]);
      }
      gain[sp][fi] = gg;
    }
  } else {
    if (tid < 2 * IP_FR) gain[tid / IP_FR][tid % IP_FR] = 1.f;
  }
  lds_sync();
  stamp(3);

  if ((a.est_out || a.mask_out) && !early) {  // after the VAD gains (filtered estimates)
    side_outputs(false);
    lds_sync();  // the transforms below overwrite the rows
  }
  // 2) inverse real FFT of every computed frame in its own row: 16 lanes per transform, transforms
  // 4 wave + lane / 16 (the 24 transforms on waves 0..5)
  static_assert(2 * IP_FR % 4 == 0, "whole waves of four transforms");
  if (wave < 2 * IP_FR / 4) {
    const int t = 4 * wave + (lane >> 4), sp = t / IP_FR, fi = t % IP_FR;
    irfft512_col(spec[sp][fi], gain[sp][fi], tw, a.window, lane & 15);
  }
  lds_sync();  // every frame's time samples in place for the overlap-add
  stamp(4);
  // 3) overlap-add of the owned segments, times the reciprocal window envelope (torch.istft)
  const int nseg = min(IP_OWN, T - f0) + ((f0 + IP_OWN >= T) ? 1 : 0);
  if (a.N % 4 == 0 && ((uintptr_t)a.y & 15) == 0) {
    // four consecutive samples per lane (16-B LDS reads and stores: a quarter of the store instructions), each sample's
    // arithmetic as below (the same bits)
    const int q4 = 4 * (tid & (HOP / 4 - 1));
    float inv_mid[4], inv_last[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float w0 = a.window[q4 + e], w1 = a.window[q4 + e + HOP];
      inv_mid[e] = 1.f / (w0 * w0 + w1 * w1);
      inv_last[e] = 1.f / (w1 * w1);
    }
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      float* yb = a.y + ((size_t)b * 2 + sp) * a.N;
      for (int i = tid; i < nseg * (HOP / 4); i += 512) {
        const int j = f0 + i / (HOP / 4);
        const int n = j * HOP + q4 - HOP;
        if (n < 0 || n >= a.N) continue;  // segment 0 lies in the centre padding
        const float4 cur = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(spec[sp][j - fbeg]) + q4);
        const float4 prv = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(spec[sp][j - 1 - fbeg]) + q4 + HOP);
        const float c4[4] = {cur.x, cur.y, cur.z, cur.w}, p4[4] = {prv.x, prv.y, prv.z, prv.w};
        float o4[4];
        if (j < T) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float num = 0.f;
            num += c4[e];
            num += p4[e];
            o4[e] = poison ? qnan : num * inv_mid[e];
          }
        } else {  // segment T: frame T - 1 only
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float num = 0.f;
            num += p4[e];
            o4[e] = poison ? qnan : num * inv_last[e];
          }
        }
        if (n + 3 < a.N) {
          st_out(reinterpret_cast<float4*>(yb + n), make_float4(o4[0], o4[1], o4[2], o4[3]));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < a.N) st_out(yb + n + e, o4[e]);
        }
      }
    }
    stamp(5);
    return;
  }
  const int q = tid & (HOP - 1);  // this thread's sample phase in every segment
  const float wq0 = a.window[q], wq1 = a.window[q + HOP];
  const float inv_mid = 1.f / (wq0 * wq0 + wq1 * wq1);  // segments 1..T-1: frame j and frame j-1
  const float inv_last = 1.f / (wq1 * wq1);             // segment T: frame T-1 only
#pragma unroll
  for (int sp = 0; sp < 2; ++sp) {
    float* yb = a.y + ((size_t)b * 2 + sp) * a.N;
    for (int i = tid; i < nseg * HOP; i += 512) {
      const int j = f0 + i / HOP;
      const int n = j * HOP + q - HOP;
      if (n < 0 || n >= a.N) continue;  // segment 0 lies in the centre padding
      float num = 0.f;
      if (j < T) num += reinterpret_cast<const float*>(spec[sp][j - fbeg])[q];  // frame j, first half
      num += reinterpret_cast<const float*>(spec[sp][j - 1 - fbeg])[q + HOP];    // frame j-1, second half
      st_out(yb + n, poison ? qnan : num * (j < T ? inv_mid : inv_last));
    }
  }
  stamp(5);
}

hipError_t launch_istft_pair(const IstftArgs& a, hipStream_t s) {
  if (a.S != 2 || a.BS % 2 || a.est_mode != 1) return hipErrorInvalidValue;
  dim3 grid(a.BS / 2, (a.T + IP_OWN - 1) / IP_OWN);
  hipLaunchKernelGGL(k_istft_pair, grid, dim3(512), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
