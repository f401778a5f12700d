// Device helpers shared by the gfx950 kernels: deterministic reductions, PReLU/sigmoid, and the
// GroupNorm coefficient prologues of the normalize-on-load consumers.
//
// GroupNorm(1, C) is applied the way torch's CPU kernel applies it (fused per-channel affine):
//   scale[c] = rstd * gamma[c];  shift[c] = beta[c] - scale[c] * mean;  y = x * scale + shift.
#pragma once
#include <hip/hip_runtime.h>
#include "sepvad_internal.h"

namespace sepvad {

// Stores of the large inter-kernel buffers (X, S0, x', masks, est, sep): with SEPVAD_NT non-temporal, so the
// lines do not sit dirty in the XCD's L2 until the kernel boundary writes them back (A/B switch).
#ifndef SEPVAD_NT
#define SEPVAD_NT 0
#endif
__device__ __forceinline__ void st_out(float* p, float v) {
  if constexpr (SEPVAD_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ void st_out(float2* p, float2 v) {
  if constexpr (SEPVAD_NT) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(f2v{v.x, v.y}, reinterpret_cast<f2v*>(p));
  } else {
    *p = v;
  }
}

__device__ __forceinline__ void st_out(float4* p, float4 v) {
  if constexpr (SEPVAD_NT) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
  } else {
    *p = v;
  }
}

__device__ __forceinline__ float prelu_f(float x, float w) { return x > 0.f ? x : w * x; }

#ifndef SEPVAD_DB_FAST
#define SEPVAD_DB_FAST 1
#endif
// 10 log10(clamp(|X|^2, 1e-10)) of one STFT bin (AmplitudeToDB of the power spectrum, model/model.py:17-25). Fast
// form: |X|^2 as x^2 + y^2 and the logarithm through the hardware log2 (v_log_f32, ~1 ulp): within ~2e-5 dB of the
// hypot / log10 form; every dB of the forward and of the side attribute takes the same form.
__device__ __forceinline__ float power_db(float2 X) {
#if SEPVAD_DB_FAST
  return 3.01029995663981195f * __builtin_amdgcn_logf(fmaxf(fmaf(X.x, X.x, X.y * X.y), 1e-10f));
#else
  const float mag = hypotf(X.x, X.y);  // torch.abs(complex)
  return 10.f * log10f(fmaxf(mag * mag, 1e-10f));
#endif
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

// Workgroup barrier that orders LDS only. __syncthreads() carries a workgroup-scope fence, which hipcc
// lowers to s_waitcnt vmcnt(0) before s_barrier: every wave would first wait for all of its outstanding
// global stores (e.g. side outputs) to complete. Kernels whose threads never read each other's global
// writes within the launch synchronise with this instead.
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Orders this wave's LDS writes before its later LDS reads (for buffers that belong to one wave: no
// workgroup barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

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
  lds_sync();
  if (l == 0) red[w] = v;
  lds_sync();
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
  lds_sync();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += lds[threadIdx.x * 16 + i];
    out[threadIdx.x] = s;
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


// ---- consumer-side statistics: partial records -> GroupNorm affine vectors in LDS --------------
// Phase 1 (reduce_records, no barrier): thread j sums value j of the record sources over their
// records in record order (loads issued 16 at a time), so every consumer workgroup derives bitwise
// identical statistics. Phase 2 (after a barrier): per-channel affines from the sums, with
// gamma/beta prefetched into registers before phase 1 (ld_chan).

struct RecSrc {
  const double* p;  // first value of utterance b's first record
  int n, rs, nv;    // records, record stride (doubles), values per record used
};

__device__ __forceinline__ RecSrc rec_src(const GnSrc& s, int b, int nv) {
  return RecSrc{s.rec + (size_t)b * s.nrec * s.rstride + s.roff, s.nrec, s.rstride, nv};
}
__device__ __forceinline__ RecSrc rec_none() { return RecSrc{nullptr, 0, 0, 0}; }

// out[j] for j < s0.nv + s1.nv (<= blockDim): sums of value j over records (s0's values first).
__device__ inline void reduce_records(const RecSrc& s0, const RecSrc& s1, double* out) {
  const int j = threadIdx.x;
  if (j >= s0.nv + s1.nv) return;
  const bool f = j < s0.nv;
  const double* p = f ? s0.p + j : s1.p + (j - s0.nv);
  const int n = f ? s0.n : s1.n;
  const size_t rs = f ? s0.rs : s1.rs;
  double s = 0.0;
  int r = 0;
  for (; r + 16 <= n; r += 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = p[(r + u) * rs];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  for (; r + 4 <= n; r += 4) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[(r + u) * rs];
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u];
  }
  for (; r < n; ++r) s += p[r * rs];
  out[j] = s;
}

// Per-channel parameters of channels k = tid, tid + blockDim (K <= 2 * blockDim) into registers.
__device__ __forceinline__ void ld_chan(const float* p, int K, float (&r)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = threadIdx.x + q * blockDim.x;
    r[q] = k < K ? p[k] : 0.f;
  }
}

// Block reduction of NV per-thread floats through LDS (blockDim == 256, no shuffles): 16 threads
// per value sum 16 slots each, then thread j sums the 16 partials in double (fixed order =>
// deterministic) and stores out[j]. `lds` holds >= NV * 288 floats. Two barriers.
template <int NV>
__device__ inline void block_reduce_store_lds(float (&v)[NV], float* lds, double* out) {
  const int t = threadIdx.x;
  const int pos = (t >> 4) * 17 + (t & 15);  // rows of 16 padded to 17: conflict-free row sums
#pragma unroll
  for (int j = 0; j < NV; ++j) lds[j * 272 + pos] = v[j];
  lds_sync();
  if (t < NV * 16) {
    const int j = t >> 4, part = t & 15;
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) s += lds[j * 272 + part * 17 + u];
    lds[NV * 272 + t] = s;
  }
  lds_sync();
  if (t < NV) {
    double s = 0.0;
#pragma unroll
    for (int part = 0; part < 16; ++part) s += lds[NV * 272 + t * 16 + part];
    out[t] = s;
  }
}

// (mean, rstd) as torch computes GroupNorm(1, K) statistics: biased variance, 1/sqrt(var + eps).
__device__ __forceinline__ void gn_moments(double s, double ss, double cnt, float eps, float& mu, float& rstd) {
  const double m = s / cnt;
  double var = ss / cnt - m * m;
  if (var < 0.0) var = 0.0;
  mu = (float)m;
  rstd = (float)(1.0 / sqrt(var + (double)eps));
}

// The same from a precomputed inv = 1 / cnt, finished in float (torch's CPU GroupNorm computes rstd in
// float as well): no double division or square root on the persistent kernel's critical path. The sums
// stay double (E[x^2] - E[x]^2 cancels).
__device__ __forceinline__ void gn_moments_f(double s, double ss, double inv, float eps, float& mu, float& rstd) {
  const double m = s * inv;
  const double var = ss * inv - m * m;
  mu = (float)m;
  rstd = 1.f / sqrtf(fmaxf((float)var, 0.f) + eps);
}

// recursive_moments (below) with gn_moments_f
__device__ __forceinline__ void recursive_moments_f(const double* m, const double* wsum, float eps_a, float eps_b,
                                                    double inv, double Tn, float& mua_f, float& rsa, float& mub_f,
                                                    float& rsb) {
  gn_moments_f(m[2], m[3], inv, eps_a, mua_f, rsa);
  const double ra = rsa, mu = mua_f;
  const double gs = wsum[0], bs = wsum[1], bbs = wsum[2], gbs = wsum[3], ggs = wsum[4];
  const double sv = m[0] + ra * (m[5] - mu * Tn * gs) + Tn * bs;
  const double svv = m[1] + 2.0 * m[4] + Tn * bbs + 2.0 * ra * (m[6] - mu * m[7] + m[8] - mu * Tn * gbs) +
                     ra * ra * (m[9] - 2.0 * mu * m[10] + mu * mu * Tn * ggs);
  gn_moments_f(sv, svv, inv, eps_b, mub_f, rsb);
}

// GroupNorm affine from acc = {sum, sumsq}: s[k] = rstd*g[k], h[k] = be[k] - s[k]*mean.
__device__ __forceinline__ void gn_affine(const double* acc, int K, int T, float eps, const float (&g)[2],
                                          const float (&be)[2], float* s, float* h) {
  float mu, rs;
  gn_moments(acc[0], acc[1], (double)K * T, eps, mu, rs);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = threadIdx.x + q * blockDim.x;
    if (k < K) {
      const float sc = rs * g[q];
      s[k] = sc;
      h[k] = be[q] - sc * mu;
    }
  }
}

// Recursive-LN affines (GN_a: c0, c1; GN_b: c2, c3) from the moment sums
//   0 Σo  1 Σo²  2 Σu  3 Σu²  4 Σbe·o  5 Σg·u  6 Σg·o·u  7 Σg·o  8 Σg·be·u  9 Σg²·u²  10 Σg²·u
// (u = o + r', g = gamma_a[c], be = beta_a[c]); v = (o+be) + ra·g·(u-μa) gives Σv, Σv² in closed
// form, so neither u nor v is materialized. wsum = {Σg, Σbe, Σbe², Σg·be, Σg²} over channels (host).
// (mean, rstd) of GN_a and GN_b from the moment sums (the channel-independent part of recursive_affine).
__device__ __forceinline__ void recursive_moments(const double* m, const double* wsum, float eps_a, float eps_b,
                                                  int K, int T, float& mua_f, float& rsa, float& mub_f,
                                                  float& rsb) {
  const double cnt = (double)K * T, Tn = (double)T;
  gn_moments(m[2], m[3], cnt, eps_a, mua_f, rsa);
  const double ra = rsa, mu = mua_f;
  const double gs = wsum[0], bs = wsum[1], bbs = wsum[2], gbs = wsum[3], ggs = wsum[4];
  const double sv = m[0] + ra * (m[5] - mu * Tn * gs) + Tn * bs;
  const double svv = m[1] + 2.0 * m[4] + Tn * bbs + 2.0 * ra * (m[6] - mu * m[7] + m[8] - mu * Tn * gbs) +
                     ra * ra * (m[9] - 2.0 * mu * m[10] + mu * mu * Tn * ggs);
  gn_moments(sv, svv, cnt, eps_b, mub_f, rsb);
}

__device__ inline void recursive_affine(const double* m, const LoadSpec& ld, int K, int T, const float (&ga)[2],
                                        const float (&ba)[2], const float (&gb)[2], const float (&bb)[2], float* c0,
                                        float* c1, float* c2, float* c3) {
  float mua_f, rsa, mub_f, rsb;
  recursive_moments(m, ld.wsum, ld.gn.eps, ld.eps2, K, T, mua_f, rsa, mub_f, rsb);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = threadIdx.x + q * blockDim.x;
    if (k < K) {
      const float sa = rsa * ga[q];
      c0[k] = sa; c1[k] = ba[q] - sa * mua_f;
      const float sb = rsb * gb[q];
      c2[k] = sb; c3[k] = bb[q] - sb * mub_f;
    }
  }
}

// Single-source convenience form (one barrier inside; all threads must call).
__device__ inline void gn_from_records(const GnSrc& src, int b, int K, int T, float* s, float* h, double* acc) {
  float g[2], be[2];
  ld_chan(src.g, K, g);
  ld_chan(src.be, K, be);
  reduce_records(rec_src(src, b, 2), rec_none(), acc);
  __syncthreads();
  gn_affine(acc, K, T, src.eps, g, be, s, h);
}

}  // namespace sepvad
