// Lane-exchange semantics check on the GPU: v_permlane32_swap, v_permlane16_swap, DPP row_mirror /
// row_half_mirror. Prints, for each op, the source lane each output lane received (diagnostics tool).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  const unsigned a = l, b = 100 + l;
  const auto s32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  const auto s16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[0 * 64 + l] = s32[0];
  out[1 * 64 + l] = s32[1];
  out[2 * 64 + l] = s16[0];
  out[3 * 64 + l] = s16[1];
  out[4 * 64 + l] = __builtin_amdgcn_update_dpp(0, (int)a, 0x140, 0xf, 0xf, false);
  out[5 * 64 + l] = __builtin_amdgcn_update_dpp(0, (int)a, 0x141, 0xf, 0xf, false);
}

int main() {
  unsigned* d;
  unsigned h[6 * 64];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* names[6] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "row_mirror", "row_half_mirror"};
  for (int r = 0; r < 6; ++r) {
    printf("%-16s", names[r]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[r * 64 + l]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
