// Device helpers shared by the gfx950 kernels: deterministic wave/block reductions, PReLU,
// sigmoid, and the GroupNorm coefficient prologue used by every normalize-on-load consumer.
#pragma once
#include <hip/hip_runtime.h>
#include "sepvad_internal.h"

namespace sepvad {

__device__ __forceinline__ float prelu_f(float x, float w) { return x > 0.f ? x : w * x; }
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

// Sum over the 64 lanes of a wave; only lane 0's value is used by callers (fixed order).
template <typename Tv>
__device__ __forceinline__ Tv wave_sum(Tv v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Deterministic block sum (blockDim multiple of 64, <= 1024). `red` holds >= 16 doubles.
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

// (mean, rstd) of GroupNorm(1, ...) over `count` elements from partial (sum, sumsq) slots,
// summed in slot order. torch: var biased, rstd = 1/sqrt(max(var,0)+eps).
__device__ __forceinline__ void slots_stats(const double* slots, int nslots, double count, float eps,
                                            float& mean, float& rstd) {
  double s = 0.0, ss = 0.0;
  for (int i = 0; i < nslots; ++i) { s += slots[2 * i]; ss += slots[2 * i + 1]; }
  const double mu = s / count;
  double var = ss / count - mu * mu;
  if (var < 0.0) var = 0.0;
  mean = (float)mu;
  rstd = (float)(1.0 / sqrt(var + (double)eps));
}

// Loader coefficients for utterance b, written to LDS arrays c0..c3 (each >= K floats):
//   LD_GN / LD_RESIDUAL: x' = fma(x, c0, c1)         (torch GN: scale = rstd*gamma, bias = beta - scale*mean)
//   LD_RECURSIVE:        v = o + fma(u, c0, c1); x' = fma(v, c2, c3)
// Must be called by every thread of the block (contains barriers). `red`: >= 16 doubles of LDS,
// `bc`: >= 4 floats of LDS for broadcasts.
__device__ inline void loader_coefs(const LoadSpec& ld, int b, int K, int T, float* c0, float* c1,
                                    float* c2, float* c3, double* red, float* bc) {
  const int tid = threadIdx.x;
  if (ld.mode == LD_GN || ld.mode == LD_RESIDUAL) {
    if (tid == 0) {
      float mu, rs;
      slots_stats(ld.slots + (size_t)b * ld.nslots * 2, ld.nslots, (double)K * T, ld.eps1, mu, rs);
      bc[0] = mu; bc[1] = rs;
    }
    __syncthreads();
    const float mu = bc[0], rs = bc[1];
    for (int k = tid; k < K; k += blockDim.x) {
      const float s = rs * ld.g1[k];
      c0[k] = s;
      c1[k] = ld.be1[k] - s * mu;
    }
    __syncthreads();
  } else if (ld.mode == LD_RECURSIVE) {
    // Stats of u = o + r' (GN_a) and of v = o + GN_a(u) (GN_b) from per-channel moments
    // (model/model.py:347-348). Σ_t v and Σ_t v² are expanded per channel in double.
    const double* mom = ld.moments + (size_t)b * K * 5;
    double su = 0.0, suu = 0.0;
    for (int k = tid; k < K; k += blockDim.x) { su += mom[k * 5 + 2]; suu += mom[k * 5 + 3]; }
    su = block_sum(su, red);
    suu = block_sum(suu, red);
    const double cnt = (double)K * T;
    const double mua = su / cnt;
    double vara = suu / cnt - mua * mua;
    if (vara < 0.0) vara = 0.0;
    const float mua_f = (float)mua;
    const float rsa = (float)(1.0 / sqrt(vara + (double)ld.eps1));
    double sv = 0.0, svv = 0.0;
    for (int k = tid; k < K; k += blockDim.x) {
      const float sa = rsa * ld.g1[k];
      const float ha = ld.be1[k] - sa * mua_f;
      c0[k] = sa; c1[k] = ha;
      const double So = mom[k * 5 + 0], Soo = mom[k * 5 + 1], Su = mom[k * 5 + 2];
      const double Suu = mom[k * 5 + 3], Sou = mom[k * 5 + 4];
      const double a = sa, h = ha;
      sv += So + a * Su + (double)T * h;
      svv += Soo + a * a * Suu + (double)T * h * h + 2.0 * a * Sou + 2.0 * h * So + 2.0 * a * h * Su;
    }
    sv = block_sum(sv, red);
    svv = block_sum(svv, red);
    const double mub = sv / cnt;
    double varb = svv / cnt - mub * mub;
    if (varb < 0.0) varb = 0.0;
    const float mub_f = (float)mub;
    const float rsb = (float)(1.0 / sqrt(varb + (double)ld.eps2));
    for (int k = tid; k < K; k += blockDim.x) {
      const float sb = rsb * ld.g2[k];
      c2[k] = sb;
      c3[k] = ld.be2[k] - sb * mub_f;
    }
    __syncthreads();
  }
}

// Apply the loader transform to one element of channel k.
__device__ __forceinline__ float loader_apply(int mode, float x, float u, int k, const float* c0,
                                              const float* c1, const float* c2, const float* c3) {
  switch (mode) {
    case LD_GN: return fmaf(x, c0[k], c1[k]);
    case LD_RECURSIVE: { const float v = x + fmaf(u, c0[k], c1[k]); return fmaf(v, c2[k], c3[k]); }
    case LD_RESIDUAL: return x + fmaf(u, c0[k], c1[k]);
    case LD_ADD: return x + u;
    default: return x;
  }
}

}  // namespace sepvad
