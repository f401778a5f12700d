// Shared pieces of the LDS FFTs (spectral.hip, istft.hip): complex helpers, the W512 twiddle table access,
// the radix-4 Stockham stage and the one-wave 256-point transform.
#pragma once
#include "device_common.h"

namespace sepvad {

constexpr int M256 = 256;

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }

// One radix-4 Stockham stage (stride Ns) of a 256-point transform, one wave (lane = j).
// Twiddle W512^idx, idx in [0, 512). HALF: the table holds only W512^0..255 (W512^(x+256) = -W512^x).
template <bool HALF>
__device__ __forceinline__ float2 twid(const float2* tw, int idx) {
  if constexpr (HALF) {
    const float2 w = tw[idx & 255];
    return idx < 256 ? w : make_float2(-w.x, -w.y);
  } else {
    return tw[idx];
  }
}

template <bool INV, bool HALF = false>
__device__ __forceinline__ void fft_stage(const float2* in, float2* out, const float2* tw, int lane, int Ns) {
  const int j = lane;
  const int k = j & (Ns - 1);
  float2 v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = in[j + r * 64];
  if (Ns > 1) {
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      float2 w = twid<HALF>(tw, 2 * ((r * k * (64 / Ns)) & 255));  // W_256^(r k 64/Ns) = W_512^(2 ...)
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
}

// Orders this wave's LDS writes before its later LDS reads (the buffers of a transform belong to one
// wave: no workgroup barrier is needed between its stages).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// 256-point transform of one wave ping-ponging between its buffers b0 and b1 (4 stages: result back
// in b0); the caller's buffers must be complete for this wave (wave_lds_sync or a barrier) on entry.
template <bool INV, bool HALF = false>
__device__ inline void fft256(float2* b0, float2* b1, const float2* tw, int lane) {
  fft_stage<INV, HALF>(b0, b1, tw, lane, 1);
  wave_lds_sync();
  fft_stage<INV, HALF>(b1, b0, tw, lane, 4);
  wave_lds_sync();
  fft_stage<INV, HALF>(b0, b1, tw, lane, 16);
  wave_lds_sync();
  fft_stage<INV, HALF>(b1, b0, tw, lane, 64);
  wave_lds_sync();
}

}  // namespace sepvad
