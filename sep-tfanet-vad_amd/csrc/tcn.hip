// TCN reduction kernels (HBM/L2-bound, no MFMA), channel-last [B][Tp][C]:
//   k_gate        activity gate: Conv2d(1,1,3x3,pad 1) on the dB spectrum + PReLU, spectrum *= gate
//                 (model/model.py:414-419); writes the TCN input (bins 1..256); TCN.LN statistics
//                 (model/model.py:333,421) records
//   k_dw_stats    d = PReLU(dconv(GN1(a))) (model/model.py:132-135), written once as the res_out
//                 GEMM operand (fp16 hi/lo split for PREC_F16X3, one fp16 / bf16 plane for F16 / BF16), and its statistics for reg2
//                 (model/model.py:136), which the res_out epilogue folds in
//   k_att_stats   TF_Attention gates a_t, a_f (model/model.py:197-205) from the res_out epilogue's partial
//                 means, and the moment records of the residual update (model/model.py:345-350)
//                 for the recursive/residual LN, without materializing u or v
//   k_head_stats  statistics of PReLU(o_final) (model/model.py:322-325) for TCN.output.1
// Workgroup = (utterance, a few frames), thread = channel: every row access is a coalesced 1 KB read.
// Each workgroup writes one partial record (deterministic, no atomics); consumers turn the records
// into GroupNorm affines in their prologues (device_common.h reduce_records + gn_affine / recursive_affine).
#include "device_common.h"

namespace sepvad {

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gate(GateArgs a) {
  constexpr int R = GATE_ROWS;
  __shared__ float S[R + 2][NBIN + 2];   // dB spectrum rows t0-1..t0+R, bins -1..257 (zero padded)
  __shared__ float G[R][NBIN + 1];       // gated spectrum
  __shared__ float red[2 * 16];
  const int b = blockIdx.x, t0 = blockIdx.y * R;
  const int tid = threadIdx.x;
  const int T = a.T;
  for (int i = tid; i < (R + 2) * (NBIN + 2); i += 256) {
    const int rr = i / (NBIN + 2), ff = i % (NBIN + 2);
    const int t = t0 - 1 + rr, f = ff - 1;
    float v = 0.f;
    if (t >= 0 && t < T && f >= 0 && f < NBIN) {
      if (a.X != nullptr) {  // side pass: the forward's dB spectrum, recomputed bitwise from the stored STFT
        const float2 Xk = a.X[((size_t)b * a.Tp + t) * NBIN + f];
        v = power_db(Xk);
      } else {
        v = a.specdb[((size_t)b * a.Tp + t) * SPEC_LD + f];
      }
    }
    S[rr][ff] = v;
  }
  lds_sync();
  float w[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) w[i] = a.w[i];
  const float bias = a.w[9], alpha = a.w[10];
  float st[2] = {0.f, 0.f};
  for (int i = tid; i < R * NBIN; i += 256) {
    const int ti = i / NBIN, f = i % NBIN;
    const int t = t0 + ti;
    const float x = S[ti + 1][f + 1];
    float y = x;
    if (a.activity) {
      // out[f][t] = b + sum_{i,j} w[i][j] s[f+i-1][t+j-1]  (weight [1,1,3(F),3(T)])
      float g = bias;
#pragma unroll
      for (int di = 0; di < 3; ++di)
#pragma unroll
        for (int dj = 0; dj < 3; ++dj) g = fmaf(w[di * 3 + dj], S[ti + dj][f + di], g);
      y = x * prelu_f(g, alpha);
    }
    G[ti][f] = y;
    if (a.S0 != nullptr && f >= 1) a.S0[((size_t)b * a.Tp + t) * CH + f - 1] = y;
    if (t < T && f >= 1) { st[0] += y; st[1] += y * y; }
  }
  const int nrec = a.Tp / R;
  if (a.out_rec != nullptr) block_reduce_store<2>(st, red, a.out_rec + ((size_t)b * nrec + blockIdx.y) * 2);
  else lds_sync();  // G complete (side-output pass: sepvad_side_outputs)
  if (a.spec_side) {  // self.spectrum, [B][257][T]: 16 consecutive frames per bin
    for (int i = tid; i < NBIN * R; i += 256) {
      const int f = i / R, ti = i % R, t = t0 + ti;
      if (t < T) a.spec_side[((size_t)b * NBIN + f) * T + t] = G[ti][f];
    }
  }
}

hipError_t launch_gate(const GateArgs& a, hipStream_t s) {
  if (a.Tp % GATE_ROWS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gate, dim3(a.B, a.Tp / GATE_ROWS), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dw_stats(DwStatsArgs a) {
  constexpr int R = STAT_ROWS;
  __shared__ float H[R + 8][CH];   // GN1(a) rows t0-dil .. t0+R+dil (zero outside [0,T))
  __shared__ float red[2 * 16];
  __shared__ float s1[CH], h1[CH];
  __shared__ double dacc[2];
  const int b = blockIdx.x, t0 = blockIdx.y * R;
  const int c = threadIdx.x;
  const int T = a.T, dl = a.dil;
  // issue the row loads first: their latency overlaps the record reduction below
  float raw[R + 8];
#pragma unroll
  for (int rr = 0; rr < R + 8; ++rr) {
    const int t = t0 - dl + rr;
    raw[rr] = (rr < R + 2 * dl && t >= 0 && t < T) ? a.A[((size_t)b * a.Tp + t) * CH + c] : 0.f;
  }
  float wv[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int j = 2 * c + q;
    wv[q][0] = a.wd[j * 3 + 0]; wv[q][1] = a.wd[j * 3 + 1]; wv[q][2] = a.wd[j * 3 + 2]; wv[q][3] = a.bd[j];
  }
  gn_from_records(a.gd1, b, CH, T, s1, h1, dacc);
  const float sc = s1[c], sh = h1[c];
#pragma unroll
  for (int rr = 0; rr < R + 8; ++rr) {
    const int t = t0 - dl + rr;
    if (rr < R + 2 * dl) H[rr][c] = (t >= 0 && t < T) ? fmaf(raw[rr], sc, sh) : 0.f;
  }
  // thread c owns input channel c -> output channels 2c, 2c+1 (groups=CH, multiplier 2); own column
  // only, so no barrier is needed between the H writes and reads
  float st[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int t = t0 + i;
    float v[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float x = wv[q][3];
      x = fmaf(wv[q][0], H[i][c], x);
      x = fmaf(wv[q][1], H[i + dl][c], x);
      x = fmaf(wv[q][2], H[i + 2 * dl][c], x);
      v[q] = t < T ? prelu_f(x, a.alpha) : 0.f;  // padding rows: zero operand rows for res_out
      st[0] += v[q]; st[1] += v[q] * v[q];
    }
    const size_t off = ((size_t)b * a.Tp + t) * HID + 2 * c;
    if (a.prec == PREC_F16X3) {
      const __half h0 = __float2half_rn(v[0]), h1v = __float2half_rn(v[1]);
      const __half l0 = __float2half_rn(v[0] - __half2float(h0)), l1 = __float2half_rn(v[1] - __half2float(h1v));
      *reinterpret_cast<__half2*>(a.Dhi + off) = __halves2half2(h0, h1v);
      *reinterpret_cast<__half2*>(a.Dlo + off) = __halves2half2(l0, l1);
    } else if (a.prec == PREC_F16) {
      *reinterpret_cast<__half2*>(a.Dhi + off) = __halves2half2(__float2half_rn(v[0]), __float2half_rn(v[1]));
    } else if (a.prec == PREC_BF16) {
      typedef __bf16 b2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<b2*>(a.Dhi + off) = b2{(__bf16)v[0], (__bf16)v[1]};
    } else {
      *reinterpret_cast<float2*>(a.D32 + off) = make_float2(v[0], v[1]);
    }
  }
  const int nrec = a.Tp / R;
  block_reduce_store<2>(st, red, a.out_rec + ((size_t)b * nrec + blockIdx.y) * 2);
}

hipError_t launch_dw_stats(const DwStatsArgs& a, hipStream_t s) {
  if (a.dil < 1 || a.dil > 4 || a.Tp % STAT_ROWS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_dw_stats, dim3(a.B, a.Tp / STAT_ROWS), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_att_stats(AttStatsArgs a) {
  constexpr int R = STAT_ROWS;
  __shared__ float mT[CH + 8], yf[CH + 8];
  __shared__ float mC[R + 8], yt[R + 8], ats[R];
  __shared__ float red[NMOM * 288];
  const int b = blockIdx.x, t0 = blockIdx.y * R;
  const int c = threadIdx.x;
  const int T = a.T;
  const bool rec = a.ln_mode == LD_RECURSIVE;
  // issue the row loads first: their latency overlaps the gate computation below
  float rv[R], ov[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int t = t0 + i;
    const size_t off = ((size_t)b * a.Tp + t) * CH + c;
    rv[i] = t < T ? a.R[off] : 0.f;
    ov[i] = (rec && t < T) ? a.O[off] : 0.f;
  }
  float afc = 1.f;
  if (a.tf_att) {
    const float* p = a.attp;
    // a_f: mean over frames (AdaptiveAvgPool2d((None,1))) -> conv(d=1) -> conv(d=2) -> PReLU -> sigmoid
    {
      float sacc = 0.f;
      for (int q = 0; q < a.ntiles; ++q) sacc += a.rowsum[((size_t)b * a.ntiles + q) * CH + c];
      mT[c + 4] = sacc / (float)T;
      if (c < 4) { mT[c] = 0.f; mT[CH + 4 + c] = 0.f; yf[c] = 0.f; yf[CH + 4 + c] = 0.f; }
    }
    // a_t rows t0-4 .. t0+R+4: mean over channels (AdaptiveAvgPool2d((1,None)))
    if (c < R + 8) {
      const int t = t0 - 4 + c;
      float v = 0.f;
      if (t >= 0 && t < T) {
        float sacc = 0.f;
        for (int q = 0; q < a.mtiles; ++q) sacc += a.colsum[((size_t)b * a.mtiles + q) * a.Tp + t];
        v = sacc / (float)CH;
      }
      mC[c] = v;
    }
    lds_sync();
    yf[c + 4] = p[11] + p[8] * mT[c + 3] + p[9] * mT[c + 4] + p[10] * mT[c + 5];
    if (c < R + 8) {
      const int t = t0 - 4 + c;
      float v = 0.f;
      if (t >= 0 && t < T && c >= 1 && c < R + 7) v = p[3] + p[0] * mC[c - 1] + p[1] * mC[c] + p[2] * mC[c + 1];
      yt[c] = v;
    }
    lds_sync();
    {
      const float v = p[15] + p[12] * yf[c + 2] + p[13] * yf[c + 4] + p[14] * yf[c + 6];
      afc = sigmoid_f(prelu_f(v, p[17]));
    }
    if (c < R) {
      const int k = c + 4;
      const float v = p[7] + p[4] * yt[k - 2] + p[5] * yt[k] + p[6] * yt[k + 2];
      ats[c] = sigmoid_f(prelu_f(v, p[16]));
    }
    lds_sync();
    if (blockIdx.y == 0) a.af[(size_t)b * CH + c] = afc;
    if (c < R) a.at[(size_t)b * a.Tp + t0 + c] = ats[c];
  }
  // moment record over this workgroup's frames (t < T), see device_common.h finalize_recursive
  const float g = rec ? a.ga[c] : 0.f, be = rec ? a.bea[c] : 0.f;
  float m[NMOM];
#pragma unroll
  for (int j = 0; j < NMOM; ++j) m[j] = 0.f;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int t = t0 + i;
    if (t >= T) break;
    const float r = rv[i];
    const float rp = a.tf_att ? r * (afc * ats[i]) : r;
    if (rec) {
      const float o = ov[i];
      const float u = o + rp;
      m[0] += o; m[1] += o * o; m[2] += u; m[3] += u * u; m[4] += be * o; m[5] += g * u;
      m[6] += g * o * u; m[7] += g * o; m[8] += g * be * u; m[9] += g * g * u * u; m[10] += g * g * u;
    } else {
      m[2] += rp; m[3] += rp * rp;
    }
  }
  const int nrec = a.Tp / R;
  block_reduce_store_lds<NMOM>(m, red, a.out_rec + ((size_t)b * nrec + blockIdx.y) * NMOM);
}

hipError_t launch_att_stats(const AttStatsArgs& a, hipStream_t s) {
  if (a.Tp % STAT_ROWS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_att_stats, dim3(a.B, a.Tp / STAT_ROWS), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_head_stats(HeadStatsArgs a) {
  constexpr int R = STAT_ROWS;
  __shared__ float red[2 * 16];
  __shared__ float cf[4][CH];
  __shared__ double dacc[NMOM];
  const int b = blockIdx.x, t0 = blockIdx.y * R;
  const int c = threadIdx.x;
  const LoadSpec& ld = a.ld;
  float ov[R], rv[R], gt[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int t = t0 + i;
    const size_t off = ((size_t)b * a.Tp + t) * CH + c;
    ov[i] = t < a.T ? ld.X[off] : 0.f;
    rv[i] = t < a.T ? ld.X2[off] : 0.f;
    gt[i] = (ld.at && t < a.T) ? ld.at[(size_t)b * a.Tp + t] : 1.f;
  }
  if (ld.mode == LD_RECURSIVE) {
    float ga[2], ba[2], gb[2], bb[2];
    ld_chan(ld.gn.g, CH, ga); ld_chan(ld.gn.be, CH, ba); ld_chan(ld.g2, CH, gb); ld_chan(ld.be2, CH, bb);
    reduce_records(rec_src(ld.gn, b, NMOM), rec_none(), dacc);
    lds_sync();
    recursive_affine(dacc, ld, CH, a.T, ga, ba, gb, bb, cf[0], cf[1], cf[2], cf[3]);
  } else if (ld.mode == LD_RESIDUAL) {
    gn_from_records(ld.gn, b, CH, a.T, cf[0], cf[1], dacc);
  }
  lds_sync();
  const float afc = ld.af ? ld.af[(size_t)b * CH + c] : 1.f;
  float st[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int t = t0 + i;
    if (t >= a.T) break;
    const float o = ov[i], r = rv[i];
    const float g = afc * gt[i];
    float x;
    if (ld.mode == LD_RECURSIVE) x = resid_apply<LD_RECURSIVE>(o, r, g, c, cf[0], cf[1], cf[2], cf[3]);
    else if (ld.mode == LD_RESIDUAL) x = resid_apply<LD_RESIDUAL>(o, r, g, c, cf[0], cf[1], cf[2], cf[3]);
    else x = resid_apply<LD_ADD>(o, r, g, c, cf[0], cf[1], cf[2], cf[3]);
    const float p = prelu_f(x, ld.alpha_h);
    st[0] += p; st[1] += p * p;
  }
  const int nrec = a.Tp / R;
  block_reduce_store<2>(st, red, a.out_rec + ((size_t)b * nrec + blockIdx.y) * 2);
}

// ------------------------------------------------------------------------------------------
// Side attributes of the last forward, materialised on first access (sepvad_side_outputs): the pre-sigmoid
// masks (self.masks_b, model/model.py:421) and their sigmoid (self.mask_per_speaker, :429), bin-major, from
// the frame-major head output still in the workspace. 16 frames per workgroup through an LDS transpose.
constexpr int SIDE_FR = 16;
__global__ __launch_bounds__(256) void k_mask_side(MaskSideArgs a) {
  __shared__ float tile[SIDE_FR][MOUT + 1];
  const int b = blockIdx.x, t0 = blockIdx.y * SIDE_FR, tid = threadIdx.x;
  const int nf = min(SIDE_FR, a.T - t0);
  for (int i = tid; i < SIDE_FR * MOUT; i += 256) {
    const int fi = i / MOUT, c = i - fi * MOUT;
    if (fi < nf) tile[fi][c] = a.masks[((size_t)b * a.Tp + t0 + fi) * MOUT_PAD + c];
  }
  lds_sync();
  for (int i = tid; i < MOUT * SIDE_FR; i += 256) {
    const int c = i / SIDE_FR, fi = i - c * SIDE_FR;
    if (fi >= nf) continue;
    const float v = tile[fi][c];
    const size_t o = ((size_t)b * MOUT + c) * a.T + t0 + fi;  // [B][514][T] == [B][2][257][T]
    if (a.masks_b) a.masks_b[o] = v;
    if (a.mask) a.mask[o] = sigmoid_f(v);
  }
}

hipError_t launch_mask_side(const MaskSideArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_mask_side, dim3(a.B, (a.T + SIDE_FR - 1) / SIDE_FR), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_head_stats(const HeadStatsArgs& a, hipStream_t s) {
  if (a.Tp % STAT_ROWS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_head_stats, dim3(a.B, a.Tp / STAT_ROWS), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
