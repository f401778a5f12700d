// Pointwise (1x1 conv) GEMMs of the TCN, channel-last:  Y[t][m] = sum_k X'[t][k] * W[m][k] + bias[m]
//   DepthConv1d.conv1d  256->256  (reference model/model.py:104,132)   EP_PRELU_STATS
//   DepthConv1d.res_out 512->256  (model/model.py:114,144)             EP_BIAS_ATT, A operand = d
//   TCN.output.2        256->514  (model/model.py:324,357)             EP_BIAS_OUT, A operand + head
// X' is produced while staging (normalize-on-load): the residual-stream update of the previous
// block (recursive / residual LN with the TF-attention gates folded in), or PReLU + GroupNorm for
// the output head. None of those tensors is ever materialized except the block input o (written
// once, by m-tile 0). For res_out the A operand d = PReLU(dconv(GN1(a))) is written by k_dw_stats
// (already split into fp16 hi/lo for PREC_F16X3) and its GroupNorm (reg2) is folded out of the
// operand entirely: GN2 is rstd*gamma[k]*(d - mu) + beta[k] per utterance, so
//   res_out(GN2(d))[m] = rstd * (sum_k W'[m][k] d[k] - mu * sum_k W'[m][k]) + bias[m] + sum_k W[m][k] beta[k]
// with W' = W * gamma (packed once on the host); the epilogue applies (mu, rstd) of the utterance.
//
// Arithmetic (GemmArgs::prec):
//   PREC_F16X3: fp32-equivalent GEMM on fp16 MFMA. x = x_hi + x_lo with x_hi = fp16(x),
//               x_lo = fp16(x - x_hi) (weights pre-scaled per row by 2^-e into [0.5,1));
//               acc += A_hi B_hi + A_hi B_lo + A_lo B_hi  on v_mfma_f32_32x32x16_f16, fp32 accumulate.
//               Products of fp16 are exact in fp32, so only the dropped lo*lo term (~2^-22 relative)
//               and fp32 accumulation remain: parity matches the fp32 path (tests/test_gpu_parity.py).
//   PREC_F32:   v_mfma_f32_32x32x2_f32 (exact fp32 fma chain), 1/16 of the f16 MFMA rate.
//   PREC_F16 / PREC_BF16: reduced-precision arms, one v_mfma_f32_32x32x16_{f16,bf16} per 16-deep step on the
//               hi plane only (operands rounded to fp16 / bf16, fp32 accumulation).
// Tile 64 frames x 64 channels, K chunk 64, 4 waves (2x2), one 32x32 accumulator per wave;
// single-buffered LDS fed from two register sets: chunk k+1 waits in registers to be staged while
// chunk k+2 is in flight during chunk k's MFMAs.
#include "device_common.h"

namespace sepvad {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs (HIP's uint4 wrapper can defeat SROA)

constexpr int BT = 64;        // frames per tile
constexpr int BMC = 64;       // output channels per tile
constexpr int BK = 64;        // K chunk
constexpr int LDH = BK + 8;   // halves per LDS row: 144 B = 9 x 16 B (odd) => conflict-free 16-B fragment reads
constexpr int LDF = BK + 1;   // floats per LDS row (fp32 path)
constexpr int KMAX = 512;
constexpr int NA = BT * BK / 4 / 256;          // float4 of the A chunk per thread (4)
constexpr int NWF = BMC * BK / 4 / 256;        // float4 of the fp32 W chunk per thread (4)
static_assert(BT * BK / 8 == 2 * 256 && BMC * BK / 8 == 2 * 256,
              "fp16 operand chunks are two uint4 per thread and plane (named registers, no scratch)");

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
  static_assert(LM != LD_SPLIT || PREC != PREC_F32, "pre-split operands are 16-bit planes");
  constexpr bool H16 = PREC != PREC_F32;     // 16-bit operand planes in LDS
  constexpr bool X3 = PREC == PREC_F16X3;    // ... with a lo plane
  using Smem = typename std::conditional<H16, SmemF16, SmemF32>::type;
  __shared__ __attribute__((aligned(16))) Smem sm;
  constexpr bool NEED_C = (LM == LD_GN || LM == LD_RECURSIVE || LM == LD_RESIDUAL);
  constexpr bool GATED = (LM == LD_RECURSIVE || LM == LD_RESIDUAL || LM == LD_ADD);
  __shared__ float cf[4][NEED_C ? KMAX : 1];       // residual-update affines
  __shared__ float hco[2][HEAD ? CH : 1];          // head GN_out affine
  __shared__ float afk[GATED ? KMAX : 1];
  __shared__ float atr[BT];
  __shared__ double dacc[16];
  __shared__ float epi[4][64];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int ntu = a.Tp / BT;
  const int b = blockIdx.x / ntu, rt = blockIdx.x % ntu;
  const int t0 = rt * BT;
  const int mt = blockIdx.y, m0 = mt * BMC;
  const int K = a.K, T = a.T, Tp = a.Tp;
  const LoadSpec& ld = a.ld;
  auto probe = [&](int slot) {
    if (a.probe != nullptr && tid == 0)
      a.probe[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * PROBE_SLOTS + slot] = wall_clock64();
  };
  probe(0);

  // ---------------- staging: global -> registers -> (transform) -> LDS ----------------
  // one chunk's operands in registers; two sets, so chunk k+2 is in flight while k+1 waits to be staged
  struct Regs {
    float4 ro[NA], rr[NA];
    u32x4 ah0, ah1, al0, al1;   // LD_SPLIT A chunk (rows tid/8 and tid/8 + 32)
    u32x4 wh0, wh1, wl0, wl1;   // F16X3 W chunk
    float4 wf[NWF];
  };
  const size_t arow0 = (size_t)b * Tp + t0;
  const int hrow = tid >> 3, hq = tid & 7;  // fp16 chunk mapping: row, 8-half group

  auto gather = [&](int k0, Regs& q) {
    if constexpr (LM == LD_SPLIT) {
      const size_t o0 = (arow0 + hrow) * K + k0 + 8 * hq, o1 = o0 + (size_t)32 * K;
      q.ah0 = *reinterpret_cast<const u32x4*>(ld.Xh + o0);
      q.ah1 = *reinterpret_cast<const u32x4*>(ld.Xh + o1);
      if constexpr (X3) {
        q.al0 = *reinterpret_cast<const u32x4*>(ld.Xl + o0);
        q.al1 = *reinterpret_cast<const u32x4*>(ld.Xl + o1);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        const size_t off = (arow0 + row) * K + k0 + c4;
        q.ro[i] = *reinterpret_cast<const float4*>(ld.X + off);
        if constexpr (GATED) q.rr[i] = *reinterpret_cast<const float4*>(ld.X2 + off);
      }
    }
    if constexpr (H16) {
      const size_t o0 = (size_t)(m0 + hrow) * K + k0 + 8 * hq, o1 = o0 + (size_t)32 * K;
      const __half* wp = PREC == PREC_BF16 ? a.Wbf : a.Whi;
      q.wh0 = *reinterpret_cast<const u32x4*>(wp + o0);
      q.wh1 = *reinterpret_cast<const u32x4*>(wp + o1);
      if constexpr (X3) {
        q.wl0 = *reinterpret_cast<const u32x4*>(a.Wlo + o0);
        q.wl1 = *reinterpret_cast<const u32x4*>(a.Wlo + o1);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NWF; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        q.wf[i] = *reinterpret_cast<const float4*>(a.W32 + (size_t)(m0 + row) * K + k0 + c4);
      }
    }
  };

  auto put_a = [&](int row, int col, const float4& v) {  // 4 consecutive k at (row, col)
    if constexpr (PREC == PREC_F16X3) {
      uint2 hi, lo;
      const float s = a.ascale;  // power-of-two range guard, undone exactly by wscale (api.hip)
      split4(make_float4(v.x * s, v.y * s, v.z * s, v.w * s), hi, lo);
      *reinterpret_cast<uint2*>(&sm.Ahi[row][col]) = hi;
      *reinterpret_cast<uint2*>(&sm.Alo[row][col]) = lo;
    } else if constexpr (PREC == PREC_F16) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const float s = a.ascale;
      *reinterpret_cast<h4*>(&sm.Ahi[row][col]) = h4{(_Float16)(v.x * s), (_Float16)(v.y * s), (_Float16)(v.z * s),
                                                      (_Float16)(v.w * s)};
    } else if constexpr (PREC == PREC_BF16) {
      typedef __bf16 b4 __attribute__((ext_vector_type(4)));
      const float s = a.ascale;  // bf16 has the fp32 range, but wscale carries the inverse of the scale
      *reinterpret_cast<b4*>(&sm.Ahi[row][col]) = b4{(__bf16)(v.x * s), (__bf16)(v.y * s), (__bf16)(v.z * s),
                                                     (__bf16)(v.w * s)};
    } else {
      sm.A[row][col + 0] = v.x; sm.A[row][col + 1] = v.y;
      sm.A[row][col + 2] = v.z; sm.A[row][col + 3] = v.w;
    }
  };

  auto head_apply = [&](float x, int k) -> float {
    if constexpr (HEAD) return fmaf(prelu_f(x, ld.alpha_h), hco[0][k], hco[1][k]);
    else return x;
  };

  auto stage = [&](int k0, const Regs& q) {
    if constexpr (LM == LD_SPLIT) {
      *reinterpret_cast<u32x4*>(&sm.Ahi[hrow][8 * hq]) = q.ah0;
      *reinterpret_cast<u32x4*>(&sm.Ahi[hrow + 32][8 * hq]) = q.ah1;
      if constexpr (X3) {
        *reinterpret_cast<u32x4*>(&sm.Alo[hrow][8 * hq]) = q.al0;
        *reinterpret_cast<u32x4*>(&sm.Alo[hrow + 32][8 * hq]) = q.al1;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        const int k = k0 + c4;
        float4 v = q.ro[i];
        if constexpr (LM != LD_PLAIN) {
          float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
          float g0 = 1.f, g1 = 1.f, g2 = 1.f, g3 = 1.f;
          if constexpr (GATED) {
            r = q.rr[i];
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
    if constexpr (H16) {
      *reinterpret_cast<u32x4*>(&sm.Bhi[hrow][8 * hq]) = q.wh0;
      *reinterpret_cast<u32x4*>(&sm.Bhi[hrow + 32][8 * hq]) = q.wh1;
      if constexpr (X3) {
        *reinterpret_cast<u32x4*>(&sm.Blo[hrow][8 * hq]) = q.wl0;
        *reinterpret_cast<u32x4*>(&sm.Blo[hrow + 32][8 * hq]) = q.wl1;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NWF; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx >> 4, c4 = (idx & 15) * 4;
        sm.B[row][c4 + 0] = q.wf[i].x; sm.B[row][c4 + 1] = q.wf[i].y;
        sm.B[row][c4 + 2] = q.wf[i].z; sm.B[row][c4 + 3] = q.wf[i].w;
      }
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  const int nk = K / BK;  // even (K is a multiple of 128)
  Regs q0, q1;
  gather(0, q0);
  gather(BK, q1);
  // ---------------- prologue (overlaps the first chunk's loads): GN affines -> LDS ----------------
  // all record / parameter loads are issued before the single reduction barrier
  // EP_BIAS_ATT fold: the (sum, sumsq) records of the operand's GroupNorm are loaded now (threads 0, 1)
  // and reduced in the epilogue, so their latency hides behind the main loop
  const bool fold = (EP == EP_BIAS_ATT) && a.fold.rec != nullptr;
  double fv[EP == EP_BIAS_ATT ? 16 : 1];
  const RecSrc fsrc = fold ? rec_src(a.fold, b, 2) : rec_none();
  if constexpr (EP == EP_BIAS_ATT) {
    if (fold && tid < 2) {
#pragma unroll
      for (int u = 0; u < 16; ++u) fv[u] = u < fsrc.n ? fsrc.p[tid + (size_t)u * fsrc.rs] : 0.0;
    }
  }
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
    if constexpr (HEAD) {
      s1 = rec_src(ld.gh, b, 2);
      ld_chan(ld.gh.g, K, p4); ld_chan(ld.gh.be, K, p5);
    }
    reduce_records(s0, s1, dacc);
    if constexpr (GATED) {
      for (int k = tid; k < K; k += 256) afk[k] = ld.af ? ld.af[(size_t)b * K + k] : 1.f;
      if (tid < BT) atr[tid] = ld.at ? ld.at[(size_t)b * Tp + t0 + tid] : 1.f;
    }
    __syncthreads();
    if constexpr (LM == LD_GN || LM == LD_RESIDUAL) gn_affine(dacc, K, T, ld.gn.eps, p0, p1, cf[0], cf[1]);
    if constexpr (LM == LD_RECURSIVE) recursive_affine(dacc, ld, K, T, p0, p1, p2, p3, cf[0], cf[1], cf[2], cf[3]);
    if constexpr (HEAD) gn_affine(dacc + s0.nv, K, T, ld.gh.eps, p4, p5, hco[0], hco[1]);
  }
  if constexpr (NEED_C || HEAD) __syncthreads();
  probe(1);

  auto mma = [&]() {
    if constexpr (PREC == PREC_F16 || PREC == PREC_BF16) {
      const int ar = wr * 32 + (lane & 31), br = wc * 32 + (lane & 31), kh = 8 * (lane >> 5);
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        const half8 ah = *reinterpret_cast<const half8*>(&sm.Ahi[ar][16 * s + kh]);
        const half8 bh = *reinterpret_cast<const half8*>(&sm.Bhi[br][16 * s + kh]);
        if constexpr (PREC == PREC_F16)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
        else
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah), __builtin_bit_cast(bf8, bh), acc,
                                                        0, 0, 0);
      }
    } else if constexpr (PREC == PREC_F16X3) {
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
  };

  stage(0, q0);
  __syncthreads();
  probe(2);
  // LDS holds chunk kt; q1 holds chunk kt+1; chunk kt+2 is loaded into q0 during the MFMAs
  for (int kt = 0; kt < nk; kt += 2) {
    if (kt + 2 < nk) gather((kt + 2) * BK, q0);
    mma();
    __syncthreads();
    stage((kt + 1) * BK, q1);
    __syncthreads();
    probe(3 + kt);
    if (kt + 3 < nk) gather((kt + 3) * BK, q1);
    mma();
    __syncthreads();
    if (kt + 2 < nk) {
      stage((kt + 2) * BK, q0);
      __syncthreads();
    }
    probe(4 + kt);
  }

  // ---------------- epilogue: lane = column m, registers = rows t ----------------
  // (the loop's last barrier guarantees every wave is done reading `sm`: it is reused below)
  const int col = lane & 31, half = lane >> 5;
  const int ml = wc * 32 + col, m = m0 + ml;
  const float ws = H16 ? a.wscale[m] : 1.f;
  const float bias = a.bias[m];
  auto tloc = [&](int r) { return wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * half; };

  if constexpr (EP == EP_PRELU_STATS) {
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = t0 + tloc(r);
      const float v = prelu_f(fmaf(acc[r], ws, bias), a.prelu);
      a.Y[((size_t)b * Tp + t) * a.ldy + m] = v;
      if (t < T) { s += v; ss += v * v; }
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    if (lane == 0) { epi[0][wave] = s; epi[1][wave] = ss; }
    __syncthreads();
    const int nslot = ntu * (a.M / BMC);
    if (tid == 0) {
      double S = 0.0, SS = 0.0;
      for (int w = 0; w < 4; ++w) { S += epi[0][w]; SS += epi[1][w]; }
      double* o = a.out_rec + ((size_t)b * nslot + rt * (a.M / BMC) + mt) * 2;
      o[0] = S; o[1] = SS;
    }
  } else if constexpr (EP == EP_BIAS_ATT) {
    // partial means for TF_Attention: over frames t < T per channel (rowsum) and over the tile's
    // channels per frame (colsum); the 64x64 tile goes through LDS for the channel direction
    float* ys = reinterpret_cast<float*>(&sm);  // [64 t][65]
    float fmu = 0.f, frs = 1.f;
    if (fold) {
      if (tid < 2) {
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) s += fv[u];  // records in order, as reduce_records sums them
        for (int r = 16; r < fsrc.n; ++r) s += fsrc.p[tid + (size_t)r * fsrc.rs];
        dacc[tid] = s;
      }
      __syncthreads();
      gn_moments(dacc[0], dacc[1], (double)a.foldK * T, a.fold.eps, fmu, frs);
    }
    const float fcm = fold ? fmu * a.foldc[m] : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int tl = tloc(r), t = t0 + tl;
      const float v = fold ? fmaf(frs, fmaf(acc[r], ws, -fcm), bias) : fmaf(acc[r], ws, bias);
      a.Y[((size_t)b * Tp + t) * a.ldy + m] = v;
      if (t < T) csum += v;
      ys[tl * 65 + ml] = v;
    }
    csum += __shfl_xor(csum, 32);
    __syncthreads();
    {
      const int row = tid & 63, part = tid >> 6;
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) p += ys[row * 65 + 16 * part + j];
      epi[part][row] = p;
    }
    if (half == 0) ys[64 * 65 + wr * 64 + ml] = csum;  // after the tile rows: [2 wr][64 m]
    __syncthreads();
    if (tid < 64) {
      a.colsum[((size_t)b * (a.M / BMC) + mt) * Tp + t0 + tid] = (epi[0][tid] + epi[1][tid]) + (epi[2][tid] + epi[3][tid]);
    } else if (tid < 128) {
      const int i = tid - 64;
      a.rowsum[((size_t)b * ntu + rt) * a.M + m0 + i] = ys[64 * 65 + i] + ys[64 * 65 + 64 + i];
    }
  } else {  // EP_BIAS_OUT
    float* tr = reinterpret_cast<float*>(&sm);  // [64 m][65] transpose staging for the freq-major copy
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int tl = tloc(r), t = t0 + tl;
      const float v = fmaf(acc[r], ws, bias);
      if (m < a.Mreal) a.Y[((size_t)b * Tp + t) * a.ldy + m] = v;
      if (a.Yside) tr[ml * 65 + tl] = v;
    }
    if (a.Yside) {
      __syncthreads();
      // all LDS reads first, then the stores (no per-element read -> wait -> store chain)
      constexpr int NI = BMC * BT / 256;
      float tv[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int i = tid + 256 * j;
        tv[j] = tr[(i / BT) * 65 + i % BT];
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int i = tid + 256 * j;
        const int mm = m0 + i / BT, t = t0 + i % BT;
        if (mm < a.Mreal && t < T) a.Yside[((size_t)b * a.Mreal + mm) * T + t] = tv[j];
      }
    }
  }
  if (a.probe != nullptr && tid == 0) {
    const size_t base = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * PROBE_SLOTS;
    a.probe[base + PROBE_SLOTS - 2] = wall_clock64();
    a.probe[base + PROBE_SLOTS - 1] = __smid();
  }
}

template <int PREC, int EP>
static hipError_t dispatch_ld(const GemmArgs& a, dim3 grid, hipStream_t s) {
  const dim3 block(256);
  const int lm = a.ld.mode;
  if (a.ld.head) {
    if constexpr (EP == EP_BIAS_OUT) {
      switch (lm) {
        case LD_PLAIN: hipLaunchKernelGGL((k_gemm<PREC, LD_PLAIN, 1, EP>), grid, block, 0, s, a); break;
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
    if (lm == LD_PLAIN) {
      hipLaunchKernelGGL((k_gemm<PREC, LD_PLAIN, 0, EP>), grid, block, 0, s, a);
    } else if (lm == LD_SPLIT) {
      if constexpr (PREC != PREC_F32) hipLaunchKernelGGL((k_gemm<PREC, LD_SPLIT, 0, EP>), grid, block, 0, s, a);
      else return hipErrorInvalidValue;
    } else {
      return hipErrorInvalidValue;
    }
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
  if (a.M % BMC || a.K % (2 * BK) || a.Tp % BT || a.K > KMAX) return hipErrorInvalidValue;
  const dim3 grid(a.B * (a.Tp / BT), a.M / BMC);
  switch (a.prec) {
    case PREC_F16X3: return dispatch_ep<PREC_F16X3>(a, ep, grid, s);
    case PREC_F16: return dispatch_ep<PREC_F16>(a, ep, grid, s);
    case PREC_BF16: return dispatch_ep<PREC_BF16>(a, ep, grid, s);
  }
  return dispatch_ep<PREC_F32>(a, ep, grid, s);
}

}  // namespace sepvad
