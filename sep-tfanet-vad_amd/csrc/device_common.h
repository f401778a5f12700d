// Device helpers shared by the gfx950 kernels: deterministic reductions, PReLU/sigmoid, and the
// GroupNorm coefficient prologues of the normalize-on-load consumers.
//
// GroupNorm(1, C) is applied the way torch's CPU kernel applies it (fused per-channel affine):
//   scale[c] = rstd * gamma[c];  shift[c] = beta[c] - scale[c] * mean;  y = x * scale + shift.
#pragma once
#include <hip/hip_runtime.h>
#include "sepvad_internal.h"

namespace sepvad {

__device__ __forceinline__ float prelu_f(float x, float w) { return x > 0.f ? x : w * x; }
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

// Sum over the 64 lanes of a wave; callers use lane 0's value (fixed order => deterministic).
template <typename Tv>
__device__ __forceinline__ Tv wave_sum(Tv v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Deterministic block sum (blockDim a multiple of 64, <= 1024). `red` holds >= 16 doubles.
// Every thread returns the same value.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// (mean, rstd) from partial (sum, sumsq) records summed in record order; torch: biased variance,
// rstd = 1/sqrt(max(var,0)+eps).
__device__ __forceinline__ void slots_stats(const double* p, int n, int stride, double count, float eps,
                                            float& mean, float& rstd) {
  double s = 0.0, ss = 0.0;
  for (int i = 0; i < n; ++i) { s += p[(size_t)i * stride]; ss += p[(size_t)i * stride + 1]; }
  const double mu = s / count;
  double var = ss / count - mu * mu;
  if (var < 0.0) var = 0.0;
  mean = (float)mu;
  rstd = (float)(1.0 / sqrt(var + (double)eps));
}

// GN affine coefficients for channels [0, K) from slots (thread 0 finalizes, all threads fill).
__device__ inline void gn_coefs(const double* slots, int nslots, int stride, double count, float eps,
                                const float* g, const float* be, int K, float* s, float* h, float* bc) {
  if (threadIdx.x == 0) {
    float mu, rs;
    slots_stats(slots, nslots, stride, count, eps, mu, rs);
    bc[0] = mu; bc[1] = rs;
  }
  __syncthreads();
  const float mu = bc[0], rs = bc[1];
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float sc = rs * g[k];
    s[k] = sc;
    h[k] = be[k] - sc * mu;
  }
  __syncthreads();
}

// Recursive-LN coefficients (model/model.py:347-348) from the moment records of k_att_stats:
//   u = o + r', v = o + GN_a(u), o_new = GN_b(v);   record (per element, g = gamma_a[c], be = beta_a[c]):
//   0 Σo  1 Σo²  2 Σu  3 Σu²  4 Σbe·o  5 Σg·u  6 Σg·o·u  7 Σg·o  8 Σg·be·u  9 Σg²·u²  10 Σg²·u
// Σv and Σv² follow in closed form (v = (o+be) + ra·g·(u-μa)), so v is never materialized.
// Outputs c0 = sa, c1 = ha (GN_a), c2 = sb, c3 = hb (GN_b). All threads must call (barriers).
__device__ inline void recursive_coefs(const LoadSpec& ld, int b, int K, int T, float* c0, float* c1,
                                       float* c2, float* c3, double* red, float* bc) {
  const int tid = threadIdx.x;
  double gs = 0, bs = 0, bbs = 0, gbs = 0, ggs = 0;
  for (int k = tid; k < K; k += blockDim.x) {
    const double g = ld.g1[k], e = ld.be1[k];
    gs += g; bs += e; bbs += e * e; gbs += g * e; ggs += g * g;
  }
  gs = block_sum(gs, red); bs = block_sum(bs, red); bbs = block_sum(bbs, red);
  gbs = block_sum(gbs, red); ggs = block_sum(ggs, red);
  if (tid == 0) {
    const double* p = ld.slots + (size_t)b * ld.nslots * NMOM;
    double m[NMOM];
    for (int j = 0; j < NMOM; ++j) m[j] = 0.0;
    for (int i = 0; i < ld.nslots; ++i)
      for (int j = 0; j < NMOM; ++j) m[j] += p[(size_t)i * NMOM + j];
    const double n = (double)K * T, Tn = (double)T;
    const double mua = m[2] / n;
    double vara = m[3] / n - mua * mua;
    if (vara < 0.0) vara = 0.0;
    const float rsa = (float)(1.0 / sqrt(vara + (double)ld.eps1));
    const float mua_f = (float)mua;
    const double ra = rsa, mu = mua_f;
    const double sv = m[0] + ra * (m[5] - mu * Tn * gs) + Tn * bs;
    const double svv = m[1] + 2.0 * m[4] + Tn * bbs + 2.0 * ra * (m[6] - mu * m[7] + m[8] - mu * Tn * gbs) +
                       ra * ra * (m[9] - 2.0 * mu * m[10] + mu * mu * Tn * ggs);
    const double mub = sv / n;
    double varb = svv / n - mub * mub;
    if (varb < 0.0) varb = 0.0;
    bc[0] = mua_f; bc[1] = rsa;
    bc[2] = (float)mub; bc[3] = (float)(1.0 / sqrt(varb + (double)ld.eps2));
  }
  __syncthreads();
  const float mua = bc[0], rsa = bc[1], mub = bc[2], rsb = bc[3];
  for (int k = tid; k < K; k += blockDim.x) {
    const float sa = rsa * ld.g1[k];
    c0[k] = sa; c1[k] = ld.be1[k] - sa * mua;
    const float sb = rsb * ld.g2[k];
    c2[k] = sb; c3[k] = ld.be2[k] - sb * mub;
  }
  __syncthreads();
}

// Coefficients of the residual-stream transform for utterance b (modes GN/RECURSIVE/RESIDUAL).
__device__ inline void resid_coefs(const LoadSpec& ld, int b, int K, int T, float* c0, float* c1, float* c2,
                                   float* c3, double* red, float* bc) {
  if (ld.mode == LD_GN || ld.mode == LD_RESIDUAL) {
    gn_coefs(ld.slots + (size_t)b * ld.nslots * ld.sstride, ld.nslots, ld.sstride, (double)K * T, ld.eps1,
             ld.g1, ld.be1, K, c0, c1, bc);
  } else if (ld.mode == LD_RECURSIVE) {
    recursive_coefs(ld, b, K, T, c0, c1, c2, c3, red, bc);
  }
}

// x' for one element: o = X value, r = X2 value, g = a_f[k] * a_t[t] (1 when attention is off).
template <int MODE>
__device__ __forceinline__ float resid_apply(float o, float r, float g, int k, const float* c0, const float* c1,
                                             const float* c2, const float* c3) {
  if constexpr (MODE == LD_GN) {
    return fmaf(o, c0[k], c1[k]);
  } else if constexpr (MODE == LD_RECURSIVE) {
    const float u = o + r * g;
    const float v = o + fmaf(u, c0[k], c1[k]);
    return fmaf(v, c2[k], c3[k]);
  } else if constexpr (MODE == LD_RESIDUAL) {
    return o + fmaf(r * g, c0[k], c1[k]);
  } else if constexpr (MODE == LD_ADD) {
    return o + r * g;
  } else {
    return o;
  }
}

}  // namespace sepvad
