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

// ------------------------------------------------------------------------------------------
// Register-resident 16-point DFTs for the four-step 256 = 16 x 16 transform (fft16x16_*: 16 lanes per
// transform, 4 transforms per wave, one XOR-swizzled LDS transpose in the frame's own row).
// dft4: X_k = sum_n v_n W4^(nk), W4 = -i (forward) or +i (inverse), in place.
template <bool INV>
__device__ __forceinline__ void dft4(float2& v0, float2& v1, float2& v2, float2& v3) {
  const float2 s0 = cadd(v0, v2), d0 = csub(v0, v2), s1 = cadd(v1, v3);
  float2 d1 = csub(v1, v3);
  d1 = INV ? make_float2(-d1.y, d1.x) : make_float2(d1.y, -d1.x);
  v0 = cadd(s0, s1);
  v1 = cadd(d0, d1);
  v2 = csub(s0, s1);
  v3 = csub(d0, d1);
}
// slot of output k of dft16 (n = na + 4 nb in, k = kb + 4 ka out; the 4 x 4 index transpose is a renaming)
__host__ __device__ constexpr int d16(int k) { return (k >> 2) + 4 * (k & 3); }
// W16^p (forward e^{-2 pi i p / 16}, inverse conjugate) for p = na kb in {1, 2, 3, 4, 6, 9}; float
// roundings of the same cosines as the W512 table (tw[32 p])
template <bool INV>
__device__ __forceinline__ float2 w16(int p) {
  constexpr float C1 = 0.9238795042037964f, S1 = 0.3826834261417389f, R = 0.7071067690849304f;
  float c = 1.f, sn = 0.f;  // sn = sin(2 pi p / 16)
  switch (p) {
    case 1: c = C1; sn = S1; break;
    case 2: c = R; sn = R; break;
    case 3: c = S1; sn = C1; break;
    case 6: c = -R; sn = R; break;
    case 9: c = -C1; sn = -S1; break;
    default: break;
  }
  return make_float2(c, INV ? sn : -sn);
}
// dft16 after its first radix-4 pass (slot na + 4 kb holds that pass's output kb of input group na)
template <bool INV>
__device__ __forceinline__ void dft16_tail(float2 (&x)[16]) {
#pragma unroll
  for (int na = 1; na < 4; ++na)
#pragma unroll
    for (int kb = 1; kb < 4; ++kb) {
      const int p = na * kb;
      float2& v = x[na + 4 * kb];
      if (p == 4) v = INV ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);  // W16^4 = -+i
      else v = cmul(v, w16<INV>(p));
    }
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) dft4<INV>(x[4 * kb], x[4 * kb + 1], x[4 * kb + 2], x[4 * kb + 3]);  // slot ka + 4 kb
}
// 16-point DFT in place: x[n] in, X[k] out at slot d16(k)
template <bool INV>
__device__ __forceinline__ void dft16(float2 (&x)[16]) {
#pragma unroll
  for (int na = 0; na < 4; ++na) dft4<INV>(x[na], x[na + 4], x[na + 8], x[na + 12]);  // slot na + 4 kb
  dft16_tail<INV>(x);
}

// c ^ k computed where it is used (volatile: hipcc would otherwise hoist the 32 swizzled addresses of the
// transpose and hold them all in registers)
__device__ __forceinline__ int xor_late(int c, int k) {
  int r;
  asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(c), "s"(k));
  return r;
}

__device__ __forceinline__ int mul_late(int c, int k) {
  int r;
  asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(c), "s"(k));
  return r;
}

}  // namespace sepvad
