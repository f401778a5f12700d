// Check of k_vad1's lane reduction (permlane swaps + DPP): 64 lanes x 128 partials -> lane L holds the
// lane sums of outputs 2L, 2L+1. Prints the max error against the host sums (diagnostics tool).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <type_traits>

constexpr int NV = 128;
template <int MODE>
__global__ void k(const float* in, float* out) {
  const int lane = threadIdx.x;
  float acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = in[lane * NV + j];
#pragma unroll
  for (int j = 0; j < NV / 2; ++j) {
    float x = acc[j], y = acc[j + NV / 2];
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
    acc[j] = x + y;
  }
#pragma unroll
  for (int j = 0; j < NV / 4; ++j) {
    float x = acc[j], y = acc[j + NV / 4];
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
    acc[j] = x + y;
  }
  auto dpp_level = [&](auto CTRL, int msk, int n) {
    constexpr int C = decltype(CTRL)::value;
    const bool hi = (lane & msk) != 0;
#pragma unroll
    for (int j = 0; j < NV / 8; ++j) {
      if (j < n / 2) {
        const float send = hi ? acc[j] : acc[j + n / 2];
        const float keep = hi ? acc[j + n / 2] : acc[j];
        acc[j] = keep + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), C, 0xf, 0xf, false));
      }
    }
  };
  if (MODE == 0) {
    dpp_level(std::integral_constant<int, 0x140>{}, 8, NV / 4);
    dpp_level(std::integral_constant<int, 0x141>{}, 4, NV / 8);
    dpp_level(std::integral_constant<int, 0x4e>{}, 2, NV / 16);
    dpp_level(std::integral_constant<int, 0xb1>{}, 1, NV / 32);
  } else {
#pragma unroll
    for (int msk = 8, n = NV / 4; msk >= 1; msk >>= 1, n >>= 1) {
      const bool hi = (lane & msk) != 0;
#pragma unroll
      for (int j = 0; j < n / 2; ++j) {
        const float send = hi ? acc[j] : acc[j + n / 2];
        const float keep = hi ? acc[j + n / 2] : acc[j];
        acc[j] = keep + __shfl_xor(send, msk);
      }
    }
  }
  out[2 * lane] = acc[0];
  out[2 * lane + 1] = acc[1];
}

int main() {
  static float h[64 * NV], r[NV];
  for (int i = 0; i < 64 * NV; ++i) h[i] = (float)((i * 7919) % 1000) / 1000.f;
  float *din, *dout;
  if (hipMalloc(&din, sizeof(h)) != hipSuccess || hipMalloc(&dout, sizeof(r)) != hipSuccess) return 1;
  if (hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  for (int mode = 0; mode < 2; ++mode) {
  if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, din, dout);
  else hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, din, dout);
  if (hipMemcpy(r, dout, sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("mode %d\n", mode);
  double emax = 0;
  int bad = -1;
  for (int o = 0; o < NV; ++o) {
    double s = 0;
    for (int l = 0; l < 64; ++l) s += h[l * NV + o];
    const double e = std::fabs(s - r[o]);
    if (e > emax) { emax = e; bad = o; }
  }
  printf("max err %g at output %d (got %g)\n", emax, bad, bad >= 0 ? r[bad] : 0.f);
  for (int o = 0; o < 8; ++o) {
    double s = 0;
    for (int l = 0; l < 64; ++l) s += h[l * NV + o];
    printf("out %d: %g vs %g\n", o, r[o], s);
  }
  }
  return 0;
}
