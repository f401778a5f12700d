// TCN elementwise/reduction kernels (HBM/L2-bound; no MFMA):
//   k_gate      activity gate: Conv2d(1,1,3x3,pad 1) + PReLU, spectrum *= gate (model/model.py:414-419)
//               and the TCN.LN partial statistics of rows 1..256 (model/model.py:333,421)
//   k_dw        GN1 on load -> depthwise dilated conv 256->512 (k=3, groups=256) -> PReLU,
//               GN2 partial statistics (model/model.py:110-113,132-136)
//   k_att       TF_Attention gates from the res_out epilogue's partial means, rank-1 scaling,
//               then u = o + r' (recursive LN) with per-channel moments, or r' with stats
//               (residual LN) (model/model.py:182-208,345-352)
//   k_head_prep final o, PReLU of TCN.output.0 and GN statistics of TCN.output.1 (model/model.py:322-325)
#include "device_common.h"

namespace sepvad {

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gate(GateArgs a) {
  constexpr int R = GATE_ROWS;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int W = a.Tp + 2;
  float* tile = smem;                     // [R+2][Tp+2]
  __shared__ double red[16];
  const int b = blockIdx.x, r0 = blockIdx.y * R;
  const int tid = threadIdx.x;
  const float* sp = a.specdb + (size_t)b * NBIN * a.Tp;
  for (int i = tid; i < (R + 2) * W; i += blockDim.x) {
    const int rr = i / W, tt = i % W;
    const int f = r0 - 1 + rr, t = tt - 1;
    float v = 0.f;
    if (f >= 0 && f < NBIN && t >= 0 && t < a.T) v = sp[(size_t)f * a.Tp + t];
    tile[i] = v;
  }
  __syncthreads();
  float w[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) w[i] = a.w[i];
  const float bias = a.w[9], alpha = a.w[10];
  double s = 0.0, ss = 0.0;
  for (int i = tid; i < R * a.Tp; i += blockDim.x) {
    const int rr = i / a.Tp, t = i % a.Tp;
    const int f = r0 + rr;
    if (f >= NBIN) continue;
    const float x = tile[(rr + 1) * W + t + 1];
    float y = x;
    if (a.activity) {
      float g = bias;
#pragma unroll
      for (int di = 0; di < 3; ++di)
#pragma unroll
        for (int dj = 0; dj < 3; ++dj) g = fmaf(w[di * 3 + dj], tile[(rr + di) * W + t + dj], g);
      y = x * prelu_f(g, alpha);
    }
    if (f >= 1) a.S0[((size_t)b * CH + f - 1) * a.Tp + t] = y;
    if (t < a.T) {
      if (a.spec_side) a.spec_side[((size_t)b * NBIN + f) * a.T + t] = y;
      if (f >= 1) { s += y; ss += (double)y * y; }
    }
  }
  s = block_sum(s, red);
  ss = block_sum(ss, red);
  if (tid == 0) {
    double* o = a.out_slots + ((size_t)b * gate_tiles() + blockIdx.y) * 2;
    o[0] = s; o[1] = ss;
  }
}

hipError_t launch_gate(const GateArgs& a, hipStream_t s) {
  dim3 grid(a.B, gate_tiles());
  size_t lds = (size_t)(GATE_ROWS + 2) * (a.Tp + 2) * sizeof(float);
  hipLaunchKernelGGL(k_gate, grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
constexpr int DW_CH = 16;   // input channels per workgroup (-> 32 output channels)
constexpr int DW_HALO = 4;  // max dilation

__global__ __launch_bounds__(256) void k_dw(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int W = a.Tp + 2 * DW_HALO;
  float* h = smem;  // [DW_CH][W]
  __shared__ double red[16];
  __shared__ float bc[4];
  const int b = blockIdx.x, c0 = blockIdx.y * DW_CH;
  const int tid = threadIdx.x;
  if (tid == 0) {
    float mu, rs;
    slots_stats(a.slots + (size_t)b * a.nslots * 2, a.nslots, (double)CH * a.T, 1e-8f, mu, rs);
    bc[0] = mu; bc[1] = rs;
  }
  __syncthreads();
  const float mu = bc[0], rs = bc[1];
  for (int i = tid; i < DW_CH * W; i += blockDim.x) {
    const int c = i / W, tt = i % W, t = tt - DW_HALO;
    float v = 0.f;
    if (t >= 0 && t < a.T) {
      const float s = rs * a.g1[c0 + c];
      const float sh = a.be1[c0 + c] - s * mu;
      v = fmaf(a.A[((size_t)b * CH + c0 + c) * a.Tp + t], s, sh);
    }
    h[i] = v;
  }
  __syncthreads();
  const int d = a.dil;
  double s = 0.0, ss = 0.0;
  for (int i = tid; i < 2 * DW_CH * a.Tp; i += blockDim.x) {
    const int jj = i / a.Tp, t = i % a.Tp;
    const int j = 2 * c0 + jj, c = jj >> 1;
    const float* hr = h + c * W + DW_HALO + t;
    float v = a.bd[j];
    v = fmaf(a.wd[j * 3 + 0], hr[-d], v);
    v = fmaf(a.wd[j * 3 + 1], hr[0], v);
    v = fmaf(a.wd[j * 3 + 2], hr[d], v);
    v = prelu_f(v, a.alpha);
    a.D[((size_t)b * HID + j) * a.Tp + t] = v;
    if (t < a.T) { s += v; ss += (double)v * v; }
  }
  s = block_sum(s, red);
  ss = block_sum(ss, red);
  if (tid == 0) {
    double* o = a.out_slots + ((size_t)b * (CH / DW_CH) + blockIdx.y) * 2;
    o[0] = s; o[1] = ss;
  }
}

hipError_t launch_dw(const DwArgs& a, hipStream_t s) {
  if (a.dil < 1 || a.dil > DW_HALO) return hipErrorInvalidValue;
  dim3 grid(a.B, CH / DW_CH);
  size_t lds = (size_t)DW_CH * (a.Tp + 2 * DW_HALO) * sizeof(float);
  hipLaunchKernelGGL(k_dw, grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
constexpr int ATT_CH = 16;

__global__ __launch_bounds__(256) void k_att(AttArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // LDS: mc[Tp+8], y1[Tp+8], at[Tp], mf[ATT_CH+12], yf1[ATT_CH+12], af[ATT_CH]
  const int Wt = a.Tp + 8;
  float* mc = smem;
  float* y1 = mc + Wt;
  float* at = y1 + Wt;
  float* mf = at + a.Tp;
  float* yf1 = mf + (ATT_CH + 12);
  float* af = yf1 + (ATT_CH + 12);
  __shared__ double red[16];
  const int b = blockIdx.x, c0 = blockIdx.y * ATT_CH;
  const int tid = threadIdx.x;
  const int T = a.T;

  if (a.tf_att) {
    const float* p = a.attp;
    // time gate a_t: mean over channels (AdaptiveAvgPool2d((1,None))), conv d=1 -> conv d=2 -> PReLU -> sigmoid
    for (int i = tid; i < Wt; i += blockDim.x) {
      const int t = i - 4;
      float v = 0.f;
      if (t >= 0 && t < T) {
        float sacc = 0.f;
        for (int q = 0; q < a.mtiles; ++q) sacc += a.colsum[((size_t)b * a.mtiles + q) * a.Tp + t];
        v = sacc / (float)CH;
      }
      mc[i] = v;
    }
    __syncthreads();
    for (int i = tid; i < Wt; i += blockDim.x) {
      const int t = i - 4;
      float v = 0.f;
      if (t >= 0 && t < T) v = p[3] + p[0] * mc[i - 1] + p[1] * mc[i] + p[2] * mc[i + 1];
      y1[i] = v;
    }
    __syncthreads();
    for (int t = tid; t < a.Tp; t += blockDim.x) {
      const int i = t + 4;
      const float v = p[7] + p[4] * y1[i - 2] + p[5] * y1[i] + p[6] * y1[i + 2];
      at[t] = sigmoid_f(prelu_f(v, p[16]));
    }
    // frequency gate a_f for channels c0..c0+15 (needs means of c0-3 .. c0+18)
    for (int i = tid; i < ATT_CH + 12; i += blockDim.x) {
      const int c = c0 - 6 + i;
      float v = 0.f;
      if (c >= 0 && c < CH) {
        float sacc = 0.f;
        for (int q = 0; q < a.ntiles; ++q) sacc += a.rowsum[((size_t)b * a.ntiles + q) * CH + c];
        v = sacc / (float)T;
      }
      mf[i] = v;
    }
    __syncthreads();
    for (int i = tid; i < ATT_CH + 12; i += blockDim.x) {
      const int c = c0 - 6 + i;
      float v = 0.f;
      if (c >= 0 && c < CH && i >= 1 && i < ATT_CH + 11)
        v = p[11] + p[8] * mf[i - 1] + p[9] * mf[i] + p[10] * mf[i + 1];
      yf1[i] = v;
    }
    __syncthreads();
    for (int i = tid; i < ATT_CH; i += blockDim.x) {
      const int k = i + 6;
      const float v = p[15] + p[12] * yf1[k - 2] + p[13] * yf1[k] + p[14] * yf1[k + 2];
      af[i] = sigmoid_f(prelu_f(v, p[17]));
    }
    __syncthreads();
  }

  // main sweep: 16 channels x Tp, 16 threads per channel
  const int cg = tid >> 4, l16 = tid & 15;
  const int c = c0 + cg;
  const size_t rowoff = ((size_t)b * CH + c) * a.Tp;
  double So = 0, Soo = 0, Su = 0, Suu = 0, Sou = 0;
  const float afc = a.tf_att ? af[cg] : 1.f;
  for (int t = l16; t < a.Tp; t += 16) {
    const float r = a.R[rowoff + t];
    float rp = r;
    if (a.tf_att) rp = r * (afc * at[t]);  // attention_w = a_f @ a_t, then input * attention_w
    float u = rp;
    if (a.ln_mode == LD_RECURSIVE) {
      const float o = a.O[rowoff + t];
      u = o + rp;
      if (t < T) { So += o; Soo += (double)o * o; Su += u; Suu += (double)u * u; Sou += (double)o * u; }
    } else if (t < T) {
      Su += u; Suu += (double)u * u;
    }
    a.U[rowoff + t] = u;
  }
  // reduce within the 16-lane channel group
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    So += __shfl_xor(So, o); Soo += __shfl_xor(Soo, o); Su += __shfl_xor(Su, o);
    Suu += __shfl_xor(Suu, o); Sou += __shfl_xor(Sou, o);
  }
  if (a.ln_mode == LD_RECURSIVE) {
    if (l16 == 0) {
      double* m = a.moments + ((size_t)b * CH + c) * 5;
      m[0] = So; m[1] = Soo; m[2] = Su; m[3] = Suu; m[4] = Sou;
    }
  } else {
    // per-workgroup partial (sum, sumsq) of r' in channel order
    __shared__ double cs[2][ATT_CH];
    if (l16 == 0) { cs[0][cg] = Su; cs[1][cg] = Suu; }
    __syncthreads();
    if (tid == 0) {
      double s = 0, ss = 0;
      for (int i = 0; i < ATT_CH; ++i) { s += cs[0][i]; ss += cs[1][i]; }
      double* o = a.out_slots + ((size_t)b * (CH / ATT_CH) + blockIdx.y) * 2;
      o[0] = s; o[1] = ss;
    }
  }
  (void)red;
}

hipError_t launch_att(const AttArgs& a, hipStream_t s) {
  dim3 grid(a.B, CH / ATT_CH);
  size_t lds = (size_t)(2 * (a.Tp + 8) + a.Tp + 3 * (ATT_CH + 12)) * sizeof(float);
  hipLaunchKernelGGL(k_att, grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
constexpr int HP_CH = 16;

__global__ __launch_bounds__(256) void k_head_prep(HeadPrepArgs a) {
  __shared__ float cf[4][CH];
  __shared__ double red[16];
  __shared__ float bc[4];
  const int b = blockIdx.x, c0 = blockIdx.y * HP_CH;
  const int tid = threadIdx.x;
  loader_coefs(a.ld, b, CH, a.T, cf[0], cf[1], cf[2], cf[3], red, bc);
  double s = 0.0, ss = 0.0;
  for (int i = tid; i < HP_CH * a.Tp; i += blockDim.x) {
    const int c = c0 + i / a.Tp, t = i % a.Tp;
    const size_t off = ((size_t)b * CH + c) * a.Tp + t;
    const float x = a.ld.X[off];
    const float u = (a.ld.mode == LD_PLAIN || a.ld.mode == LD_GN) ? 0.f : a.ld.X2[off];
    const float o = loader_apply(a.ld.mode, x, u, c, cf[0], cf[1], cf[2], cf[3]);
    const float p = prelu_f(o, a.alpha);
    a.P[off] = p;
    if (t < a.T) { s += p; ss += (double)p * p; }
  }
  s = block_sum(s, red);
  ss = block_sum(ss, red);
  if (tid == 0) {
    double* o = a.out_slots + ((size_t)b * (CH / HP_CH) + blockIdx.y) * 2;
    o[0] = s; o[1] = ss;
  }
}

hipError_t launch_head_prep(const HeadPrepArgs& a, hipStream_t s) {
  dim3 grid(a.B, CH / HP_CH);
  hipLaunchKernelGGL(k_head_prep, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
