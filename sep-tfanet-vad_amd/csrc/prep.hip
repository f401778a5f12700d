// Input preprocessing of the reference CLI (only_inference.py:68-83), on the device:
//   k_resample    torchaudio.transforms.Resample(sr, 16000) (only_inference.py:76-79): polyphase
//                 windowed-sinc FIR, "sinc_interp_hann", lowpass_filter_width 6, rolloff 0.99
//                 (torchaudio defaults). y[new*n + j] = sum_i K[j][i] * xpad[orig*n + i] with
//                 xpad = x zero-padded by `width` on the left and `width + orig` on the right,
//                 output length ceil(new * len / orig). Filter taps come from sepvad_resample_filter
//                 (host, double precision, rounded to fp32).
//   k_minmax / k_normalize   1.8 * (a - min) / (max - min) - 0.9 (only_inference.py:81), evaluated in
//                 fp32 in numpy's operation order (mul, div, sub — no contraction), so it is bit-exact
//                 with the reference's float32 numpy expression.
#include "device_common.h"

namespace sepvad {

// taps are read through the L1/L2 (one phase row per output, shared by all lanes of that phase)
__global__ __launch_bounds__(256) void k_resample(ResampleArgs a) {
  const float* taps = a.taps;
  for (long long o = (long long)blockIdx.x * 256 + threadIdx.x; o < a.ylen; o += (long long)gridDim.x * 256) {
    const long long n = o / a.phases;
    const int j = (int)(o % a.phases);
    const long long base = n * a.stride - a.width;  // xpad index n*stride + i  ->  x index - width
    float acc = 0.f;
    for (int i = 0; i < a.ntaps; ++i) {
      const long long xi = base + i;
      const float v = (xi >= 0 && xi < a.n) ? a.x[xi] : 0.f;
      acc = fmaf(taps[j * a.ntaps + i], v, acc);
    }
    a.y[o] = acc;
  }
}

hipError_t launch_resample(const ResampleArgs& a, hipStream_t s) {
  if (a.n < 1 || a.ylen < 1 || a.phases < 1 || a.ntaps < 1) return hipErrorInvalidValue;
  const long long nb = (a.ylen + 255) / 256;
  const int grid = (int)(nb < 2048 ? nb : 2048);
  hipLaunchKernelGGL(k_resample, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

// per-block (min, max) partials -> the finalizer in k_normalize's every block (order-free: min/max
// are exact, so the result does not depend on the reduction order)
__global__ __launch_bounds__(256) void k_minmax(NormArgs a) {
  __shared__ float smin[256], smax[256];
  float mn = INFINITY, mx = -INFINITY;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (long long)gridDim.x * 256) {
    const float v = a.x[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.part[2 * blockIdx.x] = smin[0];
    a.part[2 * blockIdx.x + 1] = smax[0];
  }
}

__global__ __launch_bounds__(256) void k_normalize(NormArgs a, int nblk) {
  __shared__ float mm[2];
  if (threadIdx.x == 0) {
    float mn = INFINITY, mx = -INFINITY;
    for (int k = 0; k < nblk; ++k) {
      mn = fminf(mn, a.part[2 * k]);
      mx = fmaxf(mx, a.part[2 * k + 1]);
    }
    mm[0] = mn;
    mm[1] = mx;
  }
  __syncthreads();
  const float mn = mm[0];
  const float den = __fsub_rn(mm[1], mn);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (long long)gridDim.x * 256) {
    const float t1 = __fmul_rn(1.8f, __fsub_rn(a.x[i], mn));
    a.y[i] = __fsub_rn(__fdiv_rn(t1, den), 0.9f);
  }
}

hipError_t launch_normalize(const NormArgs& a, hipStream_t s) {
  if (a.n < 1) return hipErrorInvalidValue;
  const long long nb = (a.n + 255) / 256;
  const int grid = (int)(nb < NORM_MAX_BLOCKS ? nb : NORM_MAX_BLOCKS);
  hipLaunchKernelGGL(k_minmax, dim3(grid), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_normalize, dim3(grid), dim3(256), 0, s, a, grid);
  return hipGetLastError();
}

}  // namespace sepvad
