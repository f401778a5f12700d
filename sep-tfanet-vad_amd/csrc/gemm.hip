// Pointwise (1x1 conv) GEMMs of the TCN, channel-last:  Y[t][m] = sum_k X'[t][k] * W[m][k] + bias[m]
//   DepthConv1d.conv1d  256->256  (reference model/model.py:104,132)   EP_PRELU_STATS
//   DepthConv1d.res_out 512->256  (model/model.py:114,144)             EP_BIAS_ATT, A operand LD_DW
//   TCN.output.2        256->514  (model/model.py:324,357)             EP_BIAS_OUT, A operand + head
// X' is produced while staging (normalize-on-load): the residual-stream update of the previous
// block (recursive / residual LN with the TF-attention gates folded in), the depthwise dilated
// conv + both GroupNorms for res_out, or PReLU + GroupNorm for the output head. None of those
// tensors is ever materialized except the block input o (written once, by m-tile 0).
//
// Arithmetic (GemmArgs::prec):
//   PREC_F16X3: fp32-equivalent GEMM on fp16 MFMA. x = x_hi + x_lo with x_hi = fp16(x),
//               x_lo = fp16(x - x_hi) (weights pre-scaled per row by 2^-e into [0.5,1));
//               acc += A_hi B_hi + A_hi B_lo + A_lo B_hi  on v_mfma_f32_32x32x16_f16, fp32 accumulate.
//               Products of fp16 are exact in fp32, so only the dropped lo*lo term (~2^-22 relative)
//               and fp32 accumulation remain: parity matches the fp32 path (tests/test_gpu_parity.py).
//   PREC_F32:   v_mfma_f32_32x32x2_f32 (exact fp32 fma chain), 1/16 of the f16 MFMA rate.
// Tile 64 frames x 64 channels, K chunk 64, 4 waves (2x2), one 32x32 accumulator per wave;
// single-buffered LDS with the next chunk prefetched into registers while the MFMAs run.
#include "device_common.h"

namespace sepvad {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BT = 64;        // frames per tile
constexpr int BMC = 64;       // output channels per tile
constexpr int BK = 64;        // K chunk
constexpr int LDH = BK + 8;   // halves per LDS row: 144 B = 9 x 16 B (odd) => conflict-free 16-B fragment reads
constexpr int LDF = BK + 1;   // floats per LDS row (fp32 path)
constexpr int KMAX = 512;
constexpr int DWROWS = BT + 8;  // LD_DW halo rows (dilation <= 4)
constexpr int NA = BT * BK / 4 / 256;          // float4 of the A chunk per thread (4)
constexpr int NDW = (DWROWS * BK / 2 / 4 + 255) / 256;  // float4 of the LD_DW halo chunk per thread (3)
constexpr int NWH = BMC * BK / 8 / 256;        // uint4 (8 halves) of each W split per thread (2)
constexpr int NWF = BMC * BK / 4 / 256;        // float4 of the fp32 W chunk per thread (4)

// Single-buffered LDS tiles; the next chunk is prefetched into registers during the MFMAs.
struct SmemF16 {
  __half Ahi[BT][LDH], Alo[BT][LDH], Bhi[BMC][LDH], Blo[BMC][LDH];
};
struct SmemF32 {
  float A[BT][LDF], B[BMC][LDF];
};

__device__ __forceinline__ void split4(const float4& v, uint2& hi, uint2& lo) {
  const __half h0 = __float2half_rn(v.x), h1 = __float2half_rn(v.y), h2 = __float2half_rn(v.z),
               h3 = __float2half_rn(v.w);
  const __half l0 = __float2half_rn(v.x - __half2float(h0)), l1 = __float2half_rn(v.y - __half2float(h1)),
               l2 = __float2half_rn(v.z - __half2float(h2)), l3 = __float2half_rn(v.w - __half2float(h3));
  __half2 a = __halves2half2(h0, h1), b = __halves2half2(h2, h3);
  __half2 c = __halves2half2(l0, l1), d = __halves2half2(l2, l3);
  hi = make_uint2(*reinterpret_cast<unsigned*>(&a), *reinterpret_cast<unsigned*>(&b));
  lo = make_uint2(*reinterpret_cast<unsigned*>(&c), *reinterpret_cast<unsigned*>(&d));
}

template <int PREC, int LM, int HEAD, int EP>
__global__ __launch_bounds__(256, 2) void k_gemm(GemmArgs a) {
  using Smem = typename std::conditional<PREC == PREC_F16X3, SmemF16, SmemF32>::type;
  __shared__ __attribute__((aligned(16))) Smem sm;
  constexpr bool NEED_C = (LM == LD_GN || LM == LD_RECURSIVE || LM == LD_RESIDUAL || LM == LD_DW);
  __shared__ float cf[4][NEED_C ? KMAX : 1];       // resid coefs / (LD_DW: s2,h2 over 512; s1,h1 over 256)
  __shared__ float hco[2][HEAD ? CH : 1];          // head GN_out affine
  __shared__ float afk[(LM == LD_RECURSIVE || LM == LD_RESIDUAL || LM == LD_ADD) ? KMAX : 1];
  __shared__ float atr[BT];
  __shared__ float wdl[LM == LD_DW ? HID * 4 : 1];  // dconv taps (3) + bias per output channel
  __shared__ float Hs[LM == LD_DW ? DWROWS : 1][LM == LD_DW ? BK / 2 + 1 : 1];
  __shared__ double dacc[16];
  __shared__ float epi[2][2][64];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int ntu = a.Tp / BT;
  const int b = blockIdx.x / ntu, rt = blockIdx.x % ntu;
  const int t0 = rt * BT;
  const int mt = blockIdx.y, m0 = mt * BMC;
  const int K = a.K, T = a.T, Tp = a.Tp;
  const LoadSpec& ld = a.ld;

  // ---------------- staging: global -> registers -> (transform) -> LDS ----------------
  float4 ro[LM == LD_DW ? NDW : NA], rr[NA];
  static_assert(NWH == 2, "W prefetch registers are named, not an array (keeps them out of scratch)");
  uint4 wh0, wh1, wl0, wl1;
  float4 wf[NWF];
  const size_t arow0 = (size_t)b * Tp + t0;

  auto gather = [&](int k0) {
    if constexpr (LM == LD_DW) {
      const int c0 = k0 >> 1;
#pragma unroll
      for (int i = 0; i < NDW; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 3, q = idx & 7;
        const int t = t0 - ld.dil + row;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < BT + 2 * ld.dil && t >= 0 && t < T)
          v = *reinterpret_cast<const float4*>(ld.X + ((size_t)b * Tp + t) * CH + c0 + 4 * q);
        ro[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        const size_t off = (arow0 + row) * K + k0 + c4;
        ro[i] = *reinterpret_cast<const float4*>(ld.X + off);
        if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL || LM == LD_ADD)
          rr[i] = *reinterpret_cast<const float4*>(ld.X2 + off);
      }
    }
    if constexpr (PREC == PREC_F16X3) {
      const int row = tid >> 3, q = tid & 7;
      const size_t o0 = (size_t)(m0 + row) * K + k0 + 8 * q, o1 = o0 + (size_t)32 * K;
      wh0 = *reinterpret_cast<const uint4*>(a.Whi + o0);
      wh1 = *reinterpret_cast<const uint4*>(a.Whi + o1);
      wl0 = *reinterpret_cast<const uint4*>(a.Wlo + o0);
      wl1 = *reinterpret_cast<const uint4*>(a.Wlo + o1);
    } else {
#pragma unroll
      for (int i = 0; i < NWF; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        wf[i] = *reinterpret_cast<const float4*>(a.W32 + (size_t)(m0 + row) * K + k0 + c4);
      }
    }
  };

  auto put_a = [&](int row, int col, const float4& v) {  // 4 consecutive k at (row, col)
    if constexpr (PREC == PREC_F16X3) {
      uint2 hi, lo;
      split4(v, hi, lo);
      *reinterpret_cast<uint2*>(&sm.Ahi[row][col]) = hi;
      *reinterpret_cast<uint2*>(&sm.Alo[row][col]) = lo;
    } else {
      sm.A[row][col + 0] = v.x; sm.A[row][col + 1] = v.y;
      sm.A[row][col + 2] = v.z; sm.A[row][col + 3] = v.w;
    }
  };

  auto head_apply = [&](float x, int k) -> float {
    if constexpr (HEAD) return fmaf(prelu_f(x, ld.alpha_h), hco[0][k], hco[1][k]);
    else return x;
  };

  auto stage = [&](int k0) {
    if constexpr (LM == LD_DW) {
      // 1) normalized a (GN1) of the halo rows into Hs[row][c_local], zero outside [0, T)
      const int c0 = k0 >> 1;
#pragma unroll
      for (int i = 0; i < NDW; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 3, q = idx & 7;
        if (row < BT + 2 * ld.dil) {
          const int t = t0 - ld.dil + row;
          const bool ok = t >= 0 && t < T;
          const int c = c0 + 4 * q;
          const float4 v = ro[i];
          Hs[row][4 * q + 0] = ok ? fmaf(v.x, cf[2][c + 0], cf[3][c + 0]) : 0.f;
          Hs[row][4 * q + 1] = ok ? fmaf(v.y, cf[2][c + 1], cf[3][c + 1]) : 0.f;
          Hs[row][4 * q + 2] = ok ? fmaf(v.z, cf[2][c + 2], cf[3][c + 2]) : 0.f;
          Hs[row][4 * q + 3] = ok ? fmaf(v.w, cf[2][c + 3], cf[3][c + 3]) : 0.f;
        }
      }
      __syncthreads();
      // 2) d = PReLU(dconv) for 64 rows x 64 output channels, then GN2 -> A tile
      const int row = tid >> 2, jg = (tid & 3) * 16;
      const int dl = ld.dil;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        float dv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int jl = jg + 4 * h + jj, j = k0 + jl, cl = jl >> 1;
          const float* w = &wdl[j * 4];
          float v = w[3];
          v = fmaf(w[0], Hs[row][cl], v);
          v = fmaf(w[1], Hs[row + dl][cl], v);
          v = fmaf(w[2], Hs[row + 2 * dl][cl], v);
          v = prelu_f(v, ld.alpha_d);
          dv[jj] = fmaf(v, cf[0][j], cf[1][j]);
        }
        put_a(row, jg + 4 * h, make_float4(dv[0], dv[1], dv[2], dv[3]));
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        const int k = k0 + c4;
        float4 v = ro[i];
        if constexpr (LM != LD_PLAIN) {
          float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
          float g0 = 1.f, g1 = 1.f, g2 = 1.f, g3 = 1.f;
          if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL || LM == LD_ADD) {
            r = rr[i];
            const float at = atr[row];
            g0 = afk[k] * at; g1 = afk[k + 1] * at; g2 = afk[k + 2] * at; g3 = afk[k + 3] * at;
          }
          v.x = resid_apply<LM>(v.x, r.x, g0, k + 0, cf[0], cf[1], cf[2], cf[3]);
          v.y = resid_apply<LM>(v.y, r.y, g1, k + 1, cf[0], cf[1], cf[2], cf[3]);
          v.z = resid_apply<LM>(v.z, r.z, g2, k + 2, cf[0], cf[1], cf[2], cf[3]);
          v.w = resid_apply<LM>(v.w, r.w, g3, k + 3, cf[0], cf[1], cf[2], cf[3]);
        }
        if (a.Xmat != nullptr && mt == 0)
          *reinterpret_cast<float4*>(a.Xmat + (arow0 + row) * K + k) = v;
        if constexpr (HEAD) {
          v.x = head_apply(v.x, k); v.y = head_apply(v.y, k + 1);
          v.z = head_apply(v.z, k + 2); v.w = head_apply(v.w, k + 3);
        }
        put_a(row, c4, v);
      }
    }
    if constexpr (PREC == PREC_F16X3) {
      const int row = tid >> 3, q = tid & 7;
      *reinterpret_cast<uint4*>(&sm.Bhi[row][8 * q]) = wh0;
      *reinterpret_cast<uint4*>(&sm.Bhi[row + 32][8 * q]) = wh1;
      *reinterpret_cast<uint4*>(&sm.Blo[row][8 * q]) = wl0;
      *reinterpret_cast<uint4*>(&sm.Blo[row + 32][8 * q]) = wl1;
    } else {
#pragma unroll
      for (int i = 0; i < NWF; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        sm.B[row][c4 + 0] = wf[i].x; sm.B[row][c4 + 1] = wf[i].y;
        sm.B[row][c4 + 2] = wf[i].z; sm.B[row][c4 + 3] = wf[i].w;
      }
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  const int nk = K / BK;
  gather(0);
  // ---------------- prologue (overlaps the first chunk's loads): GN affines -> LDS ----------------
  // all record / parameter loads are issued before the single reduction barrier
  {
    RecSrc s0 = rec_none(), s1 = rec_none();
    float p0[2], p1[2], p2[2], p3[2], p4[2], p5[2];
    if constexpr (LM == LD_GN || LM == LD_RESIDUAL) {
      s0 = rec_src(ld.gn, b, 2);
      ld_chan(ld.gn.g, K, p0); ld_chan(ld.gn.be, K, p1);
    }
    if constexpr (LM == LD_RECURSIVE) {
      s0 = rec_src(ld.gn, b, NMOM);
      ld_chan(ld.gn.g, K, p0); ld_chan(ld.gn.be, K, p1);
      ld_chan(ld.g2, K, p2); ld_chan(ld.be2, K, p3);
    }
    if constexpr (LM == LD_DW) {
      s0 = rec_src(ld.gd1, b, 2);  // GN1 (reg1) over a
      s1 = rec_src(ld.gn, b, 2);   // GN2 (reg2) over d
      ld_chan(ld.gd1.g, CH, p0); ld_chan(ld.gd1.be, CH, p1);
      ld_chan(ld.gn.g, HID, p2); ld_chan(ld.gn.be, HID, p3);
    }
    if constexpr (HEAD) {
      s1 = rec_src(ld.gh, b, 2);
      ld_chan(ld.gh.g, K, p4); ld_chan(ld.gh.be, K, p5);
    }
    reduce_records(s0, s1, dacc);
    if constexpr (LM == LD_DW) {
      for (int j = tid; j < HID; j += 256) {
        wdl[j * 4 + 0] = ld.wd[j * 3 + 0];
        wdl[j * 4 + 1] = ld.wd[j * 3 + 1];
        wdl[j * 4 + 2] = ld.wd[j * 3 + 2];
        wdl[j * 4 + 3] = ld.bd[j];
      }
    }
    if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL || LM == LD_ADD) {
      for (int k = tid; k < K; k += 256) afk[k] = ld.af ? ld.af[(size_t)b * K + k] : 1.f;
      if (tid < BT) atr[tid] = ld.at ? ld.at[(size_t)b * Tp + t0 + tid] : 1.f;
    }
    __syncthreads();
    if constexpr (LM == LD_GN || LM == LD_RESIDUAL) gn_affine(dacc, K, T, ld.gn.eps, p0, p1, cf[0], cf[1]);
    if constexpr (LM == LD_RECURSIVE) recursive_affine(dacc, ld, K, T, p0, p1, p2, p3, cf[0], cf[1], cf[2], cf[3]);
    if constexpr (LM == LD_DW) {
      gn_affine(dacc, CH, T, ld.gd1.eps, p0, p1, cf[2], cf[3]);
      gn_affine(dacc + 2, HID, T, ld.gn.eps, p2, p3, cf[0], cf[1]);
    }
    if constexpr (HEAD) gn_affine(dacc + s0.nv, K, T, ld.gh.eps, p4, p5, hco[0], hco[1]);
  }
  __syncthreads();

  stage(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gather((kt + 1) * BK);
    if constexpr (PREC == PREC_F16X3) {
      const int ar = wr * 32 + (lane & 31), br = wc * 32 + (lane & 31), kh = 8 * (lane >> 5);
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        const half8 ah = *reinterpret_cast<const half8*>(&sm.Ahi[ar][16 * s + kh]);
        const half8 al = *reinterpret_cast<const half8*>(&sm.Alo[ar][16 * s + kh]);
        const half8 bh = *reinterpret_cast<const half8*>(&sm.Bhi[br][16 * s + kh]);
        const half8 bl = *reinterpret_cast<const half8*>(&sm.Blo[br][16 * s + kh]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
      }
    } else {
      const float* Ab = &sm.A[wr * 32 + (lane & 31)][lane >> 5];
      const float* Bb = &sm.B[wc * 32 + (lane & 31)][lane >> 5];
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ab[kk], Bb[kk], acc, 0, 0, 0);
    }
    __syncthreads();
    if (kt + 1 < nk) {
      stage((kt + 1) * BK);
      __syncthreads();
    }
  }

  // ---------------- epilogue: lane = column m, registers = rows t ----------------
  const int col = lane & 31, half = lane >> 5;
  const int m = m0 + wc * 32 + col;
  const float ws = (PREC == PREC_F16X3) ? a.wscale[m] : 1.f;
  const float bias = a.bias[m];
  auto trow = [&](int r) { return t0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * half; };

  if constexpr (EP == EP_PRELU_STATS) {
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = trow(r);
      const float v = prelu_f(fmaf(acc[r], ws, bias), a.prelu);
      a.Y[((size_t)b * Tp + t) * a.ldy + m] = v;
      if (t < T) { s += v; ss += v * v; }
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    if (lane == 0) { epi[0][0][wave] = s; epi[0][1][wave] = ss; }
    __syncthreads();
    const int nslot = ntu * (a.M / BMC);
    if (tid == 0) {
      double S = 0.0, SS = 0.0;
      for (int w = 0; w < 4; ++w) { S += epi[0][0][w]; SS += epi[0][1][w]; }
      double* o = a.out_rec + ((size_t)b * nslot + rt * (a.M / BMC) + mt) * 2;
      o[0] = S; o[1] = SS;
    }
  } else if constexpr (EP == EP_BIAS_ATT) {
    float csum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = trow(r);
      const float v = fmaf(acc[r], ws, bias);
      a.Y[((size_t)b * Tp + t) * a.ldy + m] = v;
      if (t < T) csum += v;                       // partial mean over frames (per channel)
      float x = v;                                // partial mean over channels (per frame)
      x += __shfl_xor(x, 16); x += __shfl_xor(x, 8); x += __shfl_xor(x, 4);
      x += __shfl_xor(x, 2); x += __shfl_xor(x, 1);
      if (col == 0) epi[0][wc][wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * half] = x;
    }
    csum += __shfl_xor(csum, 32);
    if (half == 0) epi[1][wr][wc * 32 + col] = csum;
    __syncthreads();
    if (tid < 64) {
      a.colsum[((size_t)b * (a.M / BMC) + mt) * Tp + t0 + tid] = epi[0][0][tid] + epi[0][1][tid];
    } else if (tid < 128) {
      const int i = tid - 64;
      a.rowsum[((size_t)b * ntu + rt) * a.M + m0 + i] = epi[1][0][i] + epi[1][1][i];
    }
  } else {  // EP_BIAS_OUT
    float* tr = reinterpret_cast<float*>(&sm);  // [64 m][65] transpose staging for the freq-major copy
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = trow(r);
      const float v = fmaf(acc[r], ws, bias);
      if (m < a.Mreal) a.Y[((size_t)b * Tp + t) * a.ldy + m] = v;
      if (a.Yside) tr[(wc * 32 + col) * 65 + (t - t0)] = v;
    }
    if (a.Yside) {
      __syncthreads();
      for (int i = tid; i < BMC * BT; i += 256) {
        const int ml = i / BT, tl = i % BT;
        const int mm = m0 + ml, t = t0 + tl;
        if (mm < a.Mreal && t < T) a.Yside[((size_t)b * a.Mreal + mm) * T + t] = tr[ml * 65 + tl];
      }
    }
  }
}

template <int PREC, int EP>
static hipError_t dispatch_ld(const GemmArgs& a, dim3 grid, hipStream_t s) {
  const dim3 block(256);
  const int lm = a.ld.mode;
  if (a.ld.head) {
    if constexpr (EP == EP_BIAS_OUT) {
      switch (lm) {
        case LD_RECURSIVE: hipLaunchKernelGGL((k_gemm<PREC, LD_RECURSIVE, 1, EP>), grid, block, 0, s, a); break;
        case LD_RESIDUAL: hipLaunchKernelGGL((k_gemm<PREC, LD_RESIDUAL, 1, EP>), grid, block, 0, s, a); break;
        case LD_ADD: hipLaunchKernelGGL((k_gemm<PREC, LD_ADD, 1, EP>), grid, block, 0, s, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if constexpr (EP == EP_PRELU_STATS) {
    switch (lm) {
      case LD_GN: hipLaunchKernelGGL((k_gemm<PREC, LD_GN, 0, EP>), grid, block, 0, s, a); break;
      case LD_RECURSIVE: hipLaunchKernelGGL((k_gemm<PREC, LD_RECURSIVE, 0, EP>), grid, block, 0, s, a); break;
      case LD_RESIDUAL: hipLaunchKernelGGL((k_gemm<PREC, LD_RESIDUAL, 0, EP>), grid, block, 0, s, a); break;
      case LD_ADD: hipLaunchKernelGGL((k_gemm<PREC, LD_ADD, 0, EP>), grid, block, 0, s, a); break;
      default: return hipErrorInvalidValue;
    }
  } else if constexpr (EP == EP_BIAS_ATT) {
    if (lm != LD_DW) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_gemm<PREC, LD_DW, 0, EP>), grid, block, 0, s, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int PREC>
static hipError_t dispatch_ep(const GemmArgs& a, int ep, dim3 grid, hipStream_t s) {
  switch (ep) {
    case EP_PRELU_STATS: return dispatch_ld<PREC, EP_PRELU_STATS>(a, grid, s);
    case EP_BIAS_ATT: return dispatch_ld<PREC, EP_BIAS_ATT>(a, grid, s);
    case EP_BIAS_OUT: return dispatch_ld<PREC, EP_BIAS_OUT>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gemm(const GemmArgs& a, int ep, hipStream_t s) {
  if (a.M % BMC || a.K % BK || a.Tp % BT || a.K > KMAX) return hipErrorInvalidValue;
  if (a.ld.mode == LD_DW && (a.K != HID || a.ld.dil < 1 || a.ld.dil > 4)) return hipErrorInvalidValue;
  const dim3 grid(a.B * (a.Tp / BT), a.M / BMC);
  if (a.prec == PREC_F16X3) return dispatch_ep<PREC_F16X3>(a, ep, grid, s);
  return dispatch_ep<PREC_F32>(a, ep, grid, s);
}

}  // namespace sepvad
