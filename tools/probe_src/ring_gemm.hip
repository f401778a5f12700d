// Weight-stream microbenchmark for k_tcn's GEMM phases (diagnostics tool): one workgroup per CU
// runs 24 "blocks" of the two per-block GEMMs back to back — conv1d (K = 256, 16 steps) and res_out (K = 512,
// 32 steps), 32 frames x 256 output channels, fp16x3 (3 MFMAs per step on hi/lo planes) — with the weights
// streamed from L2 in k_tcn's fragment order through a register ring, A from LDS. Nothing else runs, so the
// time per block is the GEMM phases' floor for a given wave count and ring depth:
//   NW = 8 waves x 1 tile (32 channels) each, ring RD   (k_tcn today: RD = 8)
//   NW = 4 waves x 2 tiles each (one wave per SIMD: 512 registers per wave), ring RD
// usage: ./ring_gemm  -> one line per variant: us per block (median of 5 launches)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

constexpr int NBLK = 24, FR = 32, LDA = 520;             // A rows padded as k_tcn's d operand
constexpr size_t BLOCK_BYTES = (size_t)(256 * 256 + 256 * 512) * 4;  // hi + lo planes, fp16

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// One GEMM of NS K-steps for TL tiles of this wave; ring slot s % RD holds step s of every tile.
template <int NS, int TL, int RD>
__device__ __forceinline__ void gemm(f32x16v (&acc)[TL], const _Float16* Ahi, const _Float16* Alo,
                                     __amdgpu_buffer_rsrc_t w, const int (&vh)[TL], const int (&vl)[TL],
                                     u32x4v (&rh)[TL][RD], u32x4v (&rl)[TL][RD], int lane) {
  const int aoff = (lane & 31) * LDA + 8 * (lane >> 5);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int i = s % RD;
    const f16x8 ah = *reinterpret_cast<const f16x8*>(Ahi + aoff + 16 * s);
    const f16x8 al = *reinterpret_cast<const f16x8*>(Alo + aoff + 16 * s);
#pragma unroll
    for (int t = 0; t < TL; ++t) {
      const f16x8 bh = __builtin_bit_cast(f16x8, rh[t][i]), bl = __builtin_bit_cast(f16x8, rl[t][i]);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
      if (s + RD < NS) {
        rh[t][i] = __builtin_amdgcn_raw_buffer_load_b128(w, vh[t], (s + RD) * 1024, 0);
        rl[t][i] = __builtin_amdgcn_raw_buffer_load_b128(w, vl[t], (s + RD) * 1024, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NS, int TL, int RD>
__device__ __forceinline__ void fill(__amdgpu_buffer_rsrc_t w, const int (&vh)[TL], const int (&vl)[TL],
                                     u32x4v (&rh)[TL][RD], u32x4v (&rl)[TL][RD]) {
#pragma unroll
  for (int s = 0; s < RD; ++s)
#pragma unroll
    for (int t = 0; t < TL; ++t) {
      rh[t][s] = __builtin_amdgcn_raw_buffer_load_b128(w, vh[t], s * 1024, 0);
      rl[t][s] = __builtin_amdgcn_raw_buffer_load_b128(w, vl[t], s * 1024, 0);
    }
}

template <int NW, int RD>
__global__ __launch_bounds__(NW * 64) void k_ring(const _Float16* wts, float* out) {
  constexpr int TL = 8 / NW;  // 32-channel tiles per wave (8 tiles = 256 output channels)
  __shared__ _Float16 Ahi[FR * LDA], Alo[FR * LDA];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < FR * LDA; i += NW * 64) {
    Ahi[i] = (_Float16)(0.001f * (i % 97));
    Alo[i] = (_Float16)(1e-7f * (i % 13));
  }
  __syncthreads();
  f32x16v acc[TL];
#pragma unroll
  for (int t = 0; t < TL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  u32x4v rh[TL][RD], rl[TL][RD];
  for (int b = 0; b < NBLK; ++b) {
    const char* blk = reinterpret_cast<const char*>(wts) + b * BLOCK_BYTES;
    const __amdgpu_buffer_rsrc_t w = rsrc(blk);
    // fragment order as k_tcn: tile j's conv1d stream at j*16*1024 (hi), lo plane after all hi planes
    int v1h[TL], v1l[TL], v2h[TL], v2l[TL];
#pragma unroll
    for (int t = 0; t < TL; ++t) {
      const int j = wave * TL + t;
      v1h[t] = (j * 16 * 64 + lane) * 16;
      v1l[t] = v1h[t] + 256 * 256 * 2;
      v2h[t] = 2 * 256 * 256 * 2 + (j * 32 * 64 + lane) * 16;
      v2l[t] = v2h[t] + 256 * 512 * 2;
    }
    fill<16, TL, RD>(w, v1h, v1l, rh, rl);
    gemm<16, TL, RD>(acc, Ahi, Alo, w, v1h, v1l, rh, rl, lane);
    fill<32, TL, RD>(w, v2h, v2l, rh, rl);
    gemm<32, TL, RD>(acc, Ahi, Alo, w, v2h, v2l, rh, rl, lane);
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < TL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[t][r];
  out[blockIdx.x * NW * 64 + tid] = s;
}

template <int NW, int RD>
static void run(const _Float16* w, float* out, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<float> ms;
  for (int it = 0; it < 6; ++it) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_ring<NW, RD>), dim3(ncu), dim3(NW * 64), 0, 0, w, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t = 0.f;
    hipEventElapsedTime(&t, e0, e1);
    if (it > 0) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us_blk = ms[ms.size() / 2] * 1e3 / NBLK;
  printf("waves %d x %d tiles, ring %2d: %.2f us per block (GEMM phases only), %.1f GB/s per CU\n", NW, 8 / NW, RD,
         us_blk, BLOCK_BYTES / (us_blk * 1e-6) / 1e9);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  _Float16* w = nullptr;
  float* out = nullptr;
  if (hipMalloc(&w, BLOCK_BYTES * NBLK) != hipSuccess || hipMalloc(&out, (size_t)ncu * 512 * 4) != hipSuccess) return 1;
  hipMemset(w, 0, BLOCK_BYTES * NBLK);
  run<8, 4>(w, out, ncu);
  run<8, 8>(w, out, ncu);
  run<4, 8>(w, out, ncu);
  run<4, 16>(w, out, ncu);
  hipFree(w);
  hipFree(out);
  return 0;
}
