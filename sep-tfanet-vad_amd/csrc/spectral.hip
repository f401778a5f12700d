// Spectral front/back end and the VAD head (HBM-bound, LDS FFTs, no MFMA):
//   k_stft   reflect-padded periodic-Hann 512-point real STFT, hop 256, DC zeroed, and
//            10 log10(clamp(|X|^2, 1e-10))           (model/model.py:16-25,382-385,408-412)
//   k_vad    VAD head per speaker on the pre-sigmoid masks (or masked magnitudes), threshold and
//            [1,0,1] smoothing of the inference branch (model/model.py:153-179,424-427,444-457)
//   k_istft  est = X * sigmoid(mask) [* smoothed VAD], torch.istft(center=True, length=N)
//            (model/model.py:386-387,429-439,452-455,460)
//
// FFT: a 512-point real transform = one 256-point complex transform of z[m] = x[2m] + i x[2m+1]
// (radix-4 Stockham, 4 stages, one wave per transform in LDS) plus the split/merge twiddle step.
#include "device_common.h"

namespace sepvad {

constexpr int M256 = 256;
constexpr int FR_PER_WG = 16;   // STFT frames per workgroup
constexpr int IS_OWN = 15;      // iSTFT frames owned per workgroup (+1 halo frame computed)

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }

// 256-point complex FFT of buf0 (natural order in and out, result in buf0), one wave (64 lanes).
// tw: W_512^m = e^{-2 pi i m/512}, m in [0,512). INV: conjugate twiddles, no scaling.
template <bool INV>
__device__ inline void fft256_wave(float2* buf0, float2* buf1, const float2* tw, int lane) {
  float2* in = buf0;
  float2* out = buf1;
#pragma unroll
  for (int Ns = 1; Ns < M256; Ns *= 4) {
    const int j = lane;
    const int k = j & (Ns - 1);
    float2 v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = in[j + r * 64];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        float2 w = tw[2 * ((r * k * (64 / Ns)) & 255)];
        if (INV) w.y = -w.y;
        v[r] = cmul(v[r], w);
      }
    }
    const float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    const float2 a2 = cadd(v[1], v[3]);
    float2 a3 = csub(v[1], v[3]);
    a3 = INV ? make_float2(-a3.y, a3.x) : make_float2(a3.y, -a3.x);
    const int idxD = (j / Ns) * Ns * 4 + k;
    out[idxD] = cadd(a0, a2);
    out[idxD + Ns] = cadd(a1, a3);
    out[idxD + 2 * Ns] = csub(a0, a2);
    out[idxD + 3 * Ns] = csub(a1, a3);
    __syncthreads();
    float2* tmp = in; in = out; out = tmp;
  }
  // 4 stages: result back in buf0
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stft(StftArgs a) {
  __shared__ float2 tw[512];
  __shared__ float2 work[4][2][M256];
  __shared__ float2 Xs[FR_PER_WG][NBIN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x, f0 = blockIdx.y * FR_PER_WG;
  for (int i = tid; i < 512; i += 256) tw[i] = a.tw[i];
  __syncthreads();
  const float* xb = a.x + (size_t)b * a.N;
  const int N = a.N;
  for (int round = 0; round < FR_PER_WG / 4; ++round) {
    const int fi = round * 4 + wave;
    const int f = f0 + fi;
    const bool live = f < a.T;  // uniform per wave; all waves still run the FFT (barriers inside)
    // load z[m] = w[2m] x[2m] + i w[2m+1] x[2m+1] (reflect padding of 256 on both sides)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = lane + 64 * r;
      float2 z = make_float2(0.f, 0.f);
      if (live) {
        int s0 = f * HOP + 2 * m - HOP, s1 = s0 + 1;
        s0 = s0 < 0 ? -s0 : (s0 >= N ? 2 * (N - 1) - s0 : s0);
        s1 = s1 < 0 ? -s1 : (s1 >= N ? 2 * (N - 1) - s1 : s1);
        z = make_float2(a.window[2 * m] * xb[s0], a.window[2 * m + 1] * xb[s1]);
      }
      work[wave][0][m] = z;
    }
    __syncthreads();
    fft256_wave<false>(work[wave][0], work[wave][1], tw, lane);
    // split: X[k] = E[k] + W512^k O[k]
    const float2* Z = work[wave][0];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = lane + 64 * r;
      const float2 zk = Z[k], zm = conjf2(Z[(M256 - k) & 255]);
      const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y + zm.y));
      const float2 Dd = csub(zk, zm);
      const float2 O = make_float2(0.5f * Dd.y, -0.5f * Dd.x);
      float2 Xk = cadd(E, cmul(tw[k], O));
      if (k == 0) Xk = make_float2(0.f, 0.f);  // DC removed (model/model.py:24,410)
      Xs[fi][k] = Xk;
    }
    if (lane == 0) {
      const float2 z0 = Z[0];
      Xs[fi][256] = make_float2(z0.x - z0.y, 0.f);
    }
    __syncthreads();
  }
  // write [k][f] rows: 16 consecutive frames per bin
  for (int i = tid; i < NBIN * FR_PER_WG; i += 256) {
    const int k = i / FR_PER_WG, fi = i % FR_PER_WG;
    const int f = f0 + fi;
    if (f >= a.T) continue;
    const float2 X = Xs[fi][k];
    if (a.X) a.X[((size_t)b * NBIN + k) * a.Tp + f] = X;
    if (a.Xout) a.Xout[((size_t)b * NBIN + k) * a.T + f] = X;
    if (a.specdb || a.spec_out) {
      const float mag = hypotf(X.x, X.y);          // torch.abs(complex)
      const float pw = mag * mag;                    // torch.pow(., 2)
      const float db = 10.f * log10f(fmaxf(pw, 1e-10f));
      if (a.specdb) a.specdb[((size_t)b * NBIN + k) * a.Tp + f] = db;
      if (a.spec_out) a.spec_out[((size_t)b * NBIN + k) * a.T + f] = db;
    }
  }
}

hipError_t launch_stft(const StftArgs& a, hipStream_t s) {
  if (a.N <= HOP) return hipErrorInvalidValue;  // reflect pad needs N > 256 (torch.stft)
  dim3 grid(a.B, (a.T + FR_PER_WG - 1) / FR_PER_WG);
  hipLaunchKernelGGL(k_stft, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// VAD head: one workgroup per (utterance, speaker). LDS holds the conv1 accumulators for all T.
constexpr int VAD_CC = 16;  // channels staged per LDS chunk

__global__ __launch_bounds__(256) void k_vad(VadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int W = a.Tp + 4;
  const int Wy = a.Tp + 2;
  float* mch = smem;                 // [VAD_CC][Tp + 4] staged input rows, zero halo of 2
  float* y = mch + VAD_CC * W;       // [4][Tp + 2] conv1 -> PReLU -> GN, zero halo of 1
  float* pv = y + 4 * Wy;            // [Tp + 2] thresholds with zero halo
  __shared__ double red[16];
  const int tid = threadIdx.x;
  const int b = blockIdx.x >> 1, s = blockIdx.x & 1;
  const int T = a.T;
  const float* mrow = a.masks + ((size_t)b * 2 * NBIN + (size_t)s * NBIN) * a.Tp;
  const float2* Xb = a.X + (size_t)b * NBIN * a.Tp;

  for (int i = tid; i < 4 * Wy; i += 256) y[i] = 0.f;
  // conv1_1: 257 -> 4, k=5, pad 2, accumulated in LDS over channel chunks
  for (int cc0 = 0; cc0 < NBIN; cc0 += VAD_CC) {
    __syncthreads();
    for (int i = tid; i < VAD_CC * W; i += 256) {
      const int c = cc0 + i / W, t = i % W - 2;
      float v = 0.f;
      if (c < NBIN && t >= 0 && t < T) {
        v = mrow[(size_t)c * a.Tp + t];
        if (a.masked_speakers) {
          const float2 X = Xb[(size_t)c * a.Tp + t];
          v = hypotf(X.x, X.y) * sigmoid_f(v);
        }
      }
      mch[i] = v;
    }
    __syncthreads();
    const int ncc = min(VAD_CC, NBIN - cc0);
    for (int t = tid; t < T; t += 256) {
      float acc0 = y[0 * Wy + t + 1], acc1 = y[1 * Wy + t + 1], acc2 = y[2 * Wy + t + 1], acc3 = y[3 * Wy + t + 1];
      for (int c = 0; c < ncc; ++c) {
        const float* mr = mch + c * W + t;  // mr[k] = m[c][t + k - 2]
        const float* w0 = a.w1 + ((size_t)0 * NBIN + cc0 + c) * 5;
        const float* w1 = a.w1 + ((size_t)1 * NBIN + cc0 + c) * 5;
        const float* w2 = a.w1 + ((size_t)2 * NBIN + cc0 + c) * 5;
        const float* w3 = a.w1 + ((size_t)3 * NBIN + cc0 + c) * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const float m = mr[k];
          acc0 = fmaf(w0[k], m, acc0); acc1 = fmaf(w1[k], m, acc1);
          acc2 = fmaf(w2[k], m, acc2); acc3 = fmaf(w3[k], m, acc3);
        }
      }
      y[0 * Wy + t + 1] = acc0; y[1 * Wy + t + 1] = acc1; y[2 * Wy + t + 1] = acc2; y[3 * Wy + t + 1] = acc3;
    }
  }
  __syncthreads();
  // + bias, PReLU, GroupNorm(1,4) statistics over 4 x T
  double sm = 0.0, ssm = 0.0;
  for (int t = tid; t < T; t += 256) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const float v = prelu_f(y[o * Wy + t + 1] + a.b1[o], a.alpha);
      y[o * Wy + t + 1] = v;
      sm += v; ssm += (double)v * v;
    }
  }
  sm = block_sum(sm, red);
  ssm = block_sum(ssm, red);
  const double cnt = 4.0 * T;
  const double mu = sm / cnt;
  double var = ssm / cnt - mu * mu;
  if (var < 0.0) var = 0.0;
  const float muf = (float)mu, rs = (float)(1.0 / sqrt(var + 1e-8));
  for (int t = tid; t < T; t += 256) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const float sc = rs * a.g[o];
      const float sh = a.be[o] - sc * muf;
      float* p = &y[o * Wy + t + 1];
      *p = fmaf(*p, sc, sh);
    }
  }
  for (int i = tid; i < Wy; i += 256) pv[i] = 0.f;
  __syncthreads();
  // output_layer_vad: 4 -> 1, k=3, pad 1; sigmoid; threshold
  float* vo = a.vad_out + ((size_t)b * 2 + s) * T;
  float* go = a.gain + ((size_t)b * 2 + s) * a.Tp;
  for (int t = tid; t < T; t += 256) {
    float z = a.b2;
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int k = 0; k < 3; ++k) z = fmaf(a.w2[o * 3 + k], y[o * Wy + t + k], z);
    const float v = sigmoid_f(z);
    vo[t] = v;
    pv[t + 1] = v >= a.thr ? 1.f : 0.f;
  }
  if (!a.kw_enabled) {
    for (int t = tid; t < a.Tp; t += 256) go[t] = 1.f;
    return;
  }
  __syncthreads();
  // smoothing with taps [1,0,1], zero padding, min(.,1), first/last frame copied (model/model.py:445-451)
  for (int t = tid; t < a.Tp; t += 256) {
    float smv = 1.f;
    if (t < T) {
      smv = fminf(pv[t] + pv[t + 2], 1.f);
      if (t == 0 || t == T - 1) smv = pv[t + 1];
      if (a.ret_smooth) vo[t] = smv;
    }
    go[t] = a.filt ? smv : 1.f;
  }
}

hipError_t launch_vad(const VadArgs& a, hipStream_t s) {
  size_t lds = (size_t)(VAD_CC * (a.Tp + 4) + 5 * (a.Tp + 2)) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_vad, dim3(a.B * 2), dim3(256), lds, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// iSTFT: one workgroup per (utterance*speaker, chunk of IS_OWN frames). Computes frames
// [f0-1, f0+IS_OWN) (one halo frame), owns output hop-segments [f0, f0+IS_OWN) (+ segment T for
// the last chunk). Segment j = padded samples [256 j, 256 j + 256); output n = p - 256.
__global__ __launch_bounds__(256) void k_istft(IstftArgs a) {
  __shared__ float2 tw[512];
  __shared__ float2 work[4][2][M256];
  __shared__ float2 spec[IS_OWN + 1][NBIN + 1];  // est of computed frames
  __shared__ float fr[IS_OWN + 1][NFFT];          // windowed time frames
  __shared__ float win[NFFT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bs = blockIdx.x, f0 = blockIdx.y * IS_OWN;
  const int T = a.T;
  const int b = bs / a.S, s = bs % a.S;
  for (int i = tid; i < 512; i += 256) { tw[i] = a.tw[i]; win[i] = a.window[i]; }
  const int fbeg = f0 - 1;  // computed frame index fi -> f = fbeg + fi, fi in [0, IS_OWN]
  // 1) est for computed frames
  for (int i = tid; i < NBIN * (IS_OWN + 1); i += 256) {
    const int k = i / (IS_OWN + 1), fi = i % (IS_OWN + 1);
    const int f = fbeg + fi;
    float2 e = make_float2(0.f, 0.f);
    if (f >= 0 && f < T) {
      if (a.est_mode) {
        const float2 X = a.X[((size_t)b * NBIN + k) * a.Tp + f];
        const float mraw = a.masks[((size_t)b * a.S * NBIN + (size_t)s * NBIN + k) * a.Tp + f];
        const float m = sigmoid_f(mraw);
        if (a.noisy_phase) {
          const float mag = hypotf(X.x, X.y) * m;
          const float ph = atan2f(X.y, X.x);
          float sn, cs;
          sincosf(ph, &sn, &cs);
          e = make_float2(mag * cs, mag * sn);
        } else {
          e = make_float2(X.x * m, X.y * m);
        }
        if (a.gain) {
          const float g = a.gain[((size_t)b * a.S + s) * a.Tp + f];
          e = make_float2(g * e.x, g * e.y);
        }
        if (fi >= 1) {
          const size_t o = ((size_t)bs * NBIN + k) * T + f;
          if (a.est_out) a.est_out[o] = e;
          if (a.mask_out) a.mask_out[o] = m;
        }
      } else {
        e = a.est_in[((size_t)bs * NBIN + k) * T + f];
      }
    }
    spec[fi][k] = e;
  }
  __syncthreads();
  // 2) inverse real FFT per frame (4 waves x 4 rounds = 16 frames)
  for (int round = 0; round < (IS_OWN + 1) / 4; ++round) {
    const int fi = round * 4 + wave;
    const float2* Y = spec[fi];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = lane + 64 * r;  // 0..255
      float2 yk = Y[k], ym = Y[M256 - k];
      if (k == 0) { yk.y = 0.f; ym.y = 0.f; }  // c2r ignores Im of DC and Nyquist
      const float2 cym = conjf2(ym);
      const float2 E = make_float2(0.5f * (yk.x + cym.x), 0.5f * (yk.y + cym.y));
      const float2 Dd = csub(yk, cym);
      float2 w = tw[k];
      w.y = -w.y;  // W512^{-k}
      const float2 Oo = cmul(make_float2(0.5f * Dd.x, 0.5f * Dd.y), w);
      work[wave][0][k] = make_float2(E.x - Oo.y, E.y + Oo.x);  // E + i O
    }
    __syncthreads();
    fft256_wave<true>(work[wave][0], work[wave][1], tw, lane);
    const float2* z = work[wave][0];
    const float sc = 1.f / 256.f;  // 1/N of the 512-point c2r == 1/256 on the half-length transform
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = lane + 64 * r;
      const float2 v = z[m];
      fr[fi][2 * m] = v.x * sc * win[2 * m];
      fr[fi][2 * m + 1] = v.y * sc * win[2 * m + 1];
    }
    __syncthreads();
  }
  // 3) overlap-add of owned segments, divided by the window envelope
  const int nseg = min(IS_OWN, T - f0) + ((f0 + IS_OWN >= T) ? 1 : 0);
  float* yb = a.y + (size_t)bs * a.N;
  for (int i = tid; i < nseg * HOP; i += 256) {
    const int jj = i / HOP, q = i % HOP;
    const int j = f0 + jj;        // segment index
    const int n = j * HOP + q - HOP;  // output sample
    if (n < 0 || n >= a.N) continue;
    float num = 0.f, den = 0.f;
    if (j < T) {                  // frame j, first half
      const int fi = j - fbeg;
      num += fr[fi][q];
      den += win[q] * win[q];
    }
    if (j >= 1) {                 // frame j-1, second half
      const int fi = j - 1 - fbeg;
      num += fr[fi][q + HOP];
      den += win[q + HOP] * win[q + HOP];
    }
    yb[n] = num / den;
  }
}

hipError_t launch_istft(const IstftArgs& a, hipStream_t s) {
  dim3 grid(a.BS, (a.T + IS_OWN - 1) / IS_OWN);
  hipLaunchKernelGGL(k_istft, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
