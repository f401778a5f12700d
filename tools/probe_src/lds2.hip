// Two workgroups per CU with > 64 KB of LDS each: does either ever see the other's LDS? Every workgroup fills its
// LDS with a pattern of its own, then re-checks it for a while; mismatches (and the first bad address) per workgroup.
// build: hipcc --offload-arch=gfx950 -O2 tools/probe_src/lds2.hip -o /tmp/lds2 ; run: /tmp/lds2 [bytes]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int N>
__global__ __launch_bounds__(256, 2) void k_lds(unsigned* out, int rounds) {
  __shared__ unsigned buf[N];
  const unsigned tag = (blockIdx.x + 1) << 20;
  for (int i = threadIdx.x; i < N; i += 256) buf[i] = tag ^ i;
  __syncthreads();
  unsigned bad = 0, first = 0xffffffffu;
  for (int r = 0; r < rounds; ++r) {
    for (int i = threadIdx.x; i < N; i += 256) {
      const unsigned v = buf[i];
      if (v != (tag ^ i)) { ++bad; if (first == 0xffffffffu) first = i; }
      buf[i] = tag ^ i;
    }
    __builtin_amdgcn_s_sleep(10);
  }
  __shared__ unsigned tot, fst;
  if (threadIdx.x == 0) { tot = 0; fst = 0xffffffffu; }
  __syncthreads();
  atomicAdd(&tot, bad);
  atomicMin(&fst, first);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = tot;
    out[3 * blockIdx.x + 1] = fst;
    out[3 * blockIdx.x + 2] = __builtin_amdgcn_s_getreg(63492);
  }
}

template <int N>
int run(int grid) {
  unsigned* d;
  hipMalloc(&d, grid * 3 * 4);
  hipMemset(d, 0, grid * 3 * 4);
  int nb = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_lds<N>, 256, 0);
  hipLaunchKernelGGL(k_lds<N>, dim3(grid), dim3(256), 0, 0, d, 2000);
  hipDeviceSynchronize();
  std::vector<unsigned> h(grid * 3);
  hipMemcpy(h.data(), d, grid * 12, hipMemcpyDeviceToHost);
  long bad = 0; int nbad = 0; unsigned first = 0xffffffffu;
  for (int b = 0; b < grid; ++b) { bad += h[3 * b]; if (h[3 * b]) { ++nbad; if (h[3 * b + 1] < first) first = h[3 * b + 1]; } }
  printf("LDS %6d B, %d per CU (occupancy API), grid %d: %ld mismatches in %d workgroups, lowest bad byte %u\n", N * 4, nb,
         grid, bad, nbad, first == 0xffffffffu ? 0u : first * 4);
  hipFree(d);
  return 0;
}

int main() {
  run<74016 / 4>(512);
  run<65536 / 4 - 64>(512);
  run<60000 / 4>(512);
  run<80000 / 4>(512);
  return 0;
}
