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

// Reduce NV per-thread float values over the block (deterministic: fixed shuffle tree, waves
// summed in order, in double) and store them to `out[0..NV)` from thread 0. One barrier.
// `lds` holds >= NV * 16 floats.
template <int NV>
__device__ __forceinline__ void block_reduce_store(float (&v)[NV], float* lds, double* out) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float s = wave_sum(v[j]);
    if (l == 0) lds[j * 16 + w] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += lds[threadIdx.x * 16 + i];
    out[threadIdx.x] = s;
  }
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


// ---- consumer-side statistics: partial records -> GroupNorm affine vectors in LDS --------------
// Records are loaded by all threads in parallel into LDS and summed in record order (fixed =>
// deterministic, identical in every consumer workgroup). All threads must call (barriers).

// Sum nrec records (stride rs, values at [off, off+nv)) into out[0..nv) (LDS). Thread (g, j) sums
// value j over records g, g+G, ... in order, then thread j sums the G partials in order.
// tmp: >= blockDim doubles of LDS.
__device__ inline void sum_records(const double* rec, int nrec, int rs, int off, int nv, double* tmp, double* out) {
  const int G = blockDim.x / nv;
  const int t = threadIdx.x;
  if (t < G * nv) {
    const int g = t / nv, j = t % nv;
    double s = 0.0;
    for (int r = g; r < nrec; r += G) s += rec[(size_t)r * rs + off + j];
    tmp[t] = s;
  }
  __syncthreads();
  if (t < nv) {
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += tmp[g * nv + t];
    out[t] = s;
  }
  __syncthreads();
}

// GroupNorm(1,K) affine (scale s[k], shift h[k]) of utterance b from its (sum, sumsq) records.
__device__ inline void gn_from_records(const GnSrc& src, int b, int K, int T, float* s, float* h, double* tmp,
                                       double* acc) {
  sum_records(src.rec + (size_t)b * src.nrec * src.rstride, src.nrec, src.rstride, src.roff, 2, tmp, acc);
  const double cnt = (double)K * T;
  const double mu = acc[0] / cnt;
  double var = acc[1] / cnt - mu * mu;
  if (var < 0.0) var = 0.0;
  const float muf = (float)mu, rs = (float)(1.0 / sqrt(var + (double)src.eps));
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float sc = rs * src.g[k];
    s[k] = sc;
    h[k] = src.be[k] - sc * muf;
  }
}

// Recursive-LN affine (GN_a: sa, ha; GN_b: sb, hb) of utterance b from the moment records
//   0 Σo  1 Σo²  2 Σu  3 Σu²  4 Σbe·o  5 Σg·u  6 Σg·o·u  7 Σg·o  8 Σg·be·u  9 Σg²·u²  10 Σg²·u
// (u = o + r', g = gamma_a[c], be = beta_a[c]); v = (o+be) + ra·g·(u-μa) gives Σv, Σv² in closed
// form, so neither u nor v is materialized. wsum = {Σg, Σbe, Σbe², Σg·be, Σg²} over channels (host).
__device__ inline void recursive_from_records(const LoadSpec& ld, int b, int K, int T, float* c0, float* c1,
                                              float* c2, float* c3, double* tmp, double* acc) {
  sum_records(ld.gn.rec + (size_t)b * ld.gn.nrec * NMOM, ld.gn.nrec, NMOM, 0, NMOM, tmp, acc);
  const double* m = acc;
  const double cnt = (double)K * T, Tn = (double)T;
  const double mua = m[2] / cnt;
  double vara = m[3] / cnt - mua * mua;
  if (vara < 0.0) vara = 0.0;
  const float rsa = (float)(1.0 / sqrt(vara + (double)ld.gn.eps));
  const float mua_f = (float)mua;
  const double ra = rsa, mu = mua_f;
  const double gs = ld.wsum[0], bs = ld.wsum[1], bbs = ld.wsum[2], gbs = ld.wsum[3], ggs = ld.wsum[4];
  const double sv = m[0] + ra * (m[5] - mu * Tn * gs) + Tn * bs;
  const double svv = m[1] + 2.0 * m[4] + Tn * bbs + 2.0 * ra * (m[6] - mu * m[7] + m[8] - mu * Tn * gbs) +
                     ra * ra * (m[9] - 2.0 * mu * m[10] + mu * mu * Tn * ggs);
  const double mub = sv / cnt;
  double varb = svv / cnt - mub * mub;
  if (varb < 0.0) varb = 0.0;
  const float mub_f = (float)mub, rsb = (float)(1.0 / sqrt(varb + (double)ld.eps2));
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float sa = rsa * ld.gn.g[k];
    c0[k] = sa; c1[k] = ld.gn.be[k] - sa * mua_f;
    const float sb = rsb * ld.g2[k];
    c2[k] = sb; c3[k] = ld.be2[k] - sb * mub_f;
  }
}

}  // namespace sepvad
