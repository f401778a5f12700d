// Scale-invariant SDR on the device (reference model/combined_loss.py:16-56 calc_sisdr, identical to
// model/metric.py:61-101 scale_invariant_signal_distortion_ratio): for each row pair r,
//   p = P[pidx[r]], t = Tg[tidx[r]] (rows of N samples; identity indices when null), optional zero mean,
//   alpha = (<p,t> + eps) / (<t,t> + eps), ts = alpha t, e = ts - p,
//   si_sdr = 10 log10((<ts,ts> + eps) / (<e,e> + eps)),  eps = float32 machine epsilon.
// One workgroup per pair streams both rows once (float4 loads) and accumulates the five moments
// {sum p, sum t, sum p^2, sum t^2, sum p t} in double; the zero-mean and scaled terms follow in closed
// form: <p',t'> = <p,t> - N mp mt, <t',t'> = <t,t> - N mt^2, <e,e> = alpha^2 <t',t'> - 2 alpha <p',t'> + <p',p'>.
// Fixed-order reductions: bitwise reproducible. HBM-bound (8 N bytes per pair).
#include "device_common.h"

namespace sepvad {

constexpr int SD_THREADS = 256;

__global__ __launch_bounds__(SD_THREADS) void k_si_sdr(SiSdrArgs a) {
  __shared__ double red[5 * 16];
  const int r = blockIdx.x;
  const long long pr = a.pidx ? a.pidx[r] : r, tr = a.tidx ? a.tidx[r] : r;
  const float* p = a.P + pr * a.p_ld;
  const float* t = a.Tg + tr * a.t_ld;
  const long long N = a.N;
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(t)) & 15) == 0;
  long long n0 = 0;
  if (vec) {
    const long long n4 = N / 4;
    const float4* p4 = reinterpret_cast<const float4*>(p);
    const float4* t4 = reinterpret_cast<const float4*>(t);
    for (long long i = threadIdx.x; i < n4; i += SD_THREADS) {
      const float4 a4 = p4[i], b4 = t4[i];
      const float pa[4] = {a4.x, a4.y, a4.z, a4.w}, ta[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double x = pa[k], y = ta[k];
        s[0] += x; s[1] += y; s[2] += x * x; s[3] += y * y; s[4] += x * y;
      }
    }
    n0 = n4 * 4;
  }
  for (long long i = n0 + threadIdx.x; i < N; i += SD_THREADS) {
    const double x = p[i], y = t[i];
    s[0] += x; s[1] += y; s[2] += x * x; s[3] += y * y; s[4] += x * y;
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    double v = wave_sum(s[k]);
    if (l == 0) red[k * 16 + w] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double m[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      double v = 0.0;
      for (int i = 0; i < SD_THREADS / 64; ++i) v += red[k * 16 + i];
      m[k] = v;
    }
    const double eps = 1.1920928955078125e-07;  // torch.finfo(torch.float32).eps
    const double Nd = (double)N;
    double pt = m[4], tt = m[3], pp = m[2];
    if (a.zero_mean) {
      const double mp = m[0] / Nd, mt = m[1] / Nd;
      pt -= Nd * mp * mt;
      tt -= Nd * mt * mt;
      pp -= Nd * mp * mp;
    }
    const double alpha = (pt + eps) / (tt + eps);
    const double sig = alpha * alpha * tt;
    double noise = sig - 2.0 * alpha * pt + pp;
    if (noise < 0.0) noise = 0.0;
    a.out[r] = (float)(10.0 * log10((sig + eps) / (noise + eps)));
  }
}

// VAD accuracy (reference model/metric.py:163-177 Accuracy_Vad): labels = preds > 0.5 (not >=; NaN kept),
// written back into preds as the reference's in-place masking does (when in_place), then the fraction of
// labels equal to the targets over everything and per speaker. One workgroup: integer counts, exact.
__global__ __launch_bounds__(1024) void k_vad_acc(VadAccArgs a) {
  __shared__ unsigned cnt[1024 / 64][VACC_MAX_S];
  unsigned c[VACC_MAX_S];
#pragma unroll
  for (int s = 0; s < VACC_MAX_S; ++s) c[s] = 0;
  const long long n = (long long)a.B * a.S * a.T;
  for (long long i = threadIdx.x; i < n; i += 1024) {
    const int s = (int)((i / a.T) % a.S);
    float p = a.preds[i];
    p = p > 0.5f ? 1.f : (p <= 0.5f ? 0.f : p);
    if (a.in_place) a.preds[i] = p;
    const unsigned hit = p == a.targets[i] ? 1u : 0u;
#pragma unroll
    for (int q = 0; q < VACC_MAX_S; ++q) c[q] += q == s ? hit : 0u;
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < VACC_MAX_S; ++q) {
    unsigned v = c[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (l == 0) cnt[w][q] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (int q = 0; q < a.S; ++q) {
      unsigned long long cq = 0;
      for (int ww = 0; ww < 1024 / 64; ++ww) cq += cnt[ww][q];
      tot += cq;
      a.out[1 + q] = (float)cq / (float)((long long)a.B * a.T);  // torch: int64 sum / int -> float32
    }
    a.out[0] = (float)tot / (float)n;
  }
}

hipError_t launch_vad_acc(const VadAccArgs& a, hipStream_t s) {
  if (a.B < 1 || a.S < 1 || a.S > VACC_MAX_S || a.T < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_vad_acc, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_si_sdr(const SiSdrArgs& a, hipStream_t s) {
  if (a.R < 1 || a.N < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_si_sdr, dim3(a.R), dim3(SD_THREADS), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
