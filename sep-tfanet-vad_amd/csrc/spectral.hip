// Spectral front/back end and the VAD head (HBM-bound, LDS FFTs, no MFMA):
//   k_stft   reflect-padded periodic-Hann 512-point real STFT, hop 256, DC zeroed, and
//            10 log10(clamp(|X|^2, 1e-10))   (model/model.py:16-25,382-385,408-412); frame-major out
//   k_vad1   VAD conv1_1 (257->4, k=5, pad 2) + bias + PReLU on the pre-sigmoid masks (or the masked
//            magnitudes) with GroupNorm(1,4) partial statistics (model/model.py:158-161,173-176)
//   k_istft  GroupNorm + output_layer_vad + sigmoid, inference threshold/[1,0,1] smoothing
//            (model/model.py:176-178,444-457); est = X * sigmoid(mask) [* smoothed VAD]
//            (model/model.py:429-439,452-455); torch.istft(center=True, length=N) (model/model.py:460)
//
// FFT: a 512-point real transform = one 256-point complex transform of z[m] = x[2m] + i x[2m+1]
// (radix-4 Stockham, 4 stages, one wave per transform in LDS) plus the split/merge twiddle step.
#include <type_traits>

#include "device_common.h"
#include "fft_common.h"

namespace sepvad {

constexpr int FR_PER_WG = 16;   // STFT frames per workgroup (4 waves x 4 rounds)
constexpr int IS_OWN = 15;      // iSTFT frames owned per workgroup (+1 halo frame computed)
constexpr int IS_FR = IS_OWN + 1;

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stft(StftArgs a) {
  __shared__ float2 tw[512];
  __shared__ float2 work[4][2][M256];
  __shared__ float2 xt[FR_PER_WG][NBIN + 1];   // this block's frames, for the bin-major side outputs
  __shared__ float dt[FR_PER_WG][NBIN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x, f0 = blockIdx.y * FR_PER_WG;
  for (int i = tid; i < 512; i += 256) tw[i] = a.tw[i];
  const float* xb = a.x + (size_t)(b % a.nstr) * a.ldx + (size_t)(b / a.nstr) * a.hopw;
  const int N = a.N;
  constexpr int NR = FR_PER_WG / 4;
  // all of this wave's input samples first (frames f0 + 4 round + wave), so the loads of the four
  // transforms are in flight together; frames >= T load frame T-1's (in bounds, unused)
  float2 z[NR][4];
#pragma unroll
  for (int round = 0; round < NR; ++round) {
    const int f = min(f0 + round * 4 + wave, a.T - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = lane + 64 * r;
      int s0 = f * HOP + 2 * m - HOP, s1 = s0 + 1;  // reflect padding of 256 on both sides
      s0 = s0 < 0 ? -s0 : (s0 >= N ? 2 * (N - 1) - s0 : s0);
      s1 = s1 < 0 ? -s1 : (s1 >= N ? 2 * (N - 1) - s1 : s1);
      z[round][r] = make_float2(xb[s0], xb[s1]);
    }
  }
  lds_sync();  // twiddles
  const bool side = a.Xout != nullptr || a.spec_out != nullptr;
#pragma unroll
  for (int round = 0; round < NR; ++round) {
    const int fi = round * 4 + wave, f = f0 + fi;
    const bool live = f < a.T;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = lane + 64 * r;
      work[wave][0][m] = make_float2(a.window[2 * m] * z[round][r].x, a.window[2 * m + 1] * z[round][r].y);
    }
    wave_lds_sync();
    fft256<false>(work[wave][0], work[wave][1], tw, lane);
    const float2* Z = work[wave][0];
    const size_t row = (size_t)b * a.Tp + f;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int k = lane + 64 * r;
      if (k > 256) break;
      float2 Xk;
      if (k == 256) {
        Xk = make_float2(Z[0].x - Z[0].y, 0.f);       // Nyquist: E[0] - O[0]
      } else {
        const float2 zk = Z[k], zm = conjf2(Z[(M256 - k) & 255]);
        const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y + zm.y));
        const float2 Dd = csub(zk, zm);
        const float2 O = make_float2(0.5f * Dd.y, -0.5f * Dd.x);
        Xk = cadd(E, cmul(tw[k], O));
      }
      if (k == 0) Xk = make_float2(0.f, 0.f);       // DC removed (model/model.py:24,410)
      const float db = power_db(Xk);
      if (live) {
        if (a.X) a.X[row * NBIN + k] = Xk;
        if (a.specdb) a.specdb[row * SPEC_LD + k] = db;
      }
      if (side) { xt[fi][k] = Xk; dt[fi][k] = db; }
    }
    wave_lds_sync();  // this wave's next round overwrites work[wave]
  }
  // bin-major side outputs [B][NBIN][T]: runs of FR_PER_WG consecutive frames per bin
  if (side) {
    lds_sync();
    const int nf = min(FR_PER_WG, a.T - f0);
    for (int i = tid; i < NBIN * FR_PER_WG; i += 256) {
      const int k = i / FR_PER_WG, fi = i % FR_PER_WG;
      if (fi >= nf) continue;
      const size_t o = ((size_t)b * NBIN + k) * a.T + f0 + fi;
      if (a.Xout) a.Xout[o] = xt[fi][k];
      if (a.spec_out) a.spec_out[o] = dt[fi][k];
    }
  }
}

hipError_t launch_stft(const StftArgs& a, hipStream_t s) {
  if (a.N <= HOP) return hipErrorInvalidValue;  // reflect pad needs N > 256 (torch.stft)
  dim3 grid(a.B, (a.T + FR_PER_WG - 1) / FR_PER_WG);
  hipLaunchKernelGGL(k_stft, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// VAD conv1_1 for VAD_ROWS = 32 frames of one (utterance, speaker). Thread = input channel c (the
// 257th channel is folded in after the lane reduction): the thread's 20 taps stay in registers, its
// R + 4 input samples (one coalesced 1 KB row read per frame, every load in flight at once) form a
// register window, and it accumulates all R x 4 outputs. The 128 partial outputs are reduced over
// the wave by recursive halving (lane L ends with outputs 2L, 2L+1: 126 lane exchanges), then over
// the 4 waves through LDS in fixed order (deterministic).
__device__ __forceinline__ float vad_in(const Vad1Args& a, int b, int s, int t, int c) {
  const int tc = min(max(t, 0), a.T - 1);
  const size_t row = (size_t)b * a.Tp + tc;
  float v = a.masks[row * MOUT_PAD + s * NBIN + c];
  if (a.masked_speakers) {
    const float2 X = a.X[row * NBIN + c];
    v = hypotf(X.x, X.y) * sigmoid_f(v);
  }
  return (t >= 0 && t < a.T) ? v : 0.f;  // conv zero padding (padding 2)
}

__global__ __launch_bounds__(256) void k_vad1(Vad1Args a) {
  constexpr int R = VAD_ROWS;
  constexpr int NV = 4 * R;   // outputs of the block, index 4 i + o
  __shared__ float part[4][NV];
  __shared__ float red[2 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bs = blockIdx.x, b = bs >> 1, s = bs & 1;
  const int t0 = blockIdx.y * R;
  const int T = a.T;
  // diagnostics: slot 0 wall clock at entry, slots 1.. shader clock at the phase ends
  unsigned long long* const pr = a.probe ? a.probe + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
  auto stamp = [&](int k) {
    if (pr && tid == 0) pr[k] = __builtin_amdgcn_s_memtime();
  };
  if (pr && tid == 0) pr[0] = wall_clock64();
  stamp(1);
  float m[R + 4];
#pragma unroll
  for (int r = 0; r < R + 4; ++r) m[r] = vad_in(a, b, s, t0 - 2 + r, tid);
  float w[4][5];
#pragma unroll
  for (int o = 0; o < 4; ++o)
#pragma unroll
    for (int k = 0; k < 5; ++k) w[o][k] = a.w1[((size_t)o * NBIN + tid) * 5 + k];
  float acc[NV];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 5; ++k) v = fmaf(w[o][k], m[i + k], v);
      acc[4 * i + o] = v;
    }
  stamp(2);
  // recursive halving over the lanes: a lane whose bit msk is clear keeps the lower half of its outputs,
  // its partner (bit set, same higher bits) the upper half. Bits 32 / 16: one v_permlane32/16_swap per pair
  // (the swap hands each lane its partner's item of the kept half: kept = own + swapped, no selects);
  // bits 8, 4: DPP row_mirror / row_half_mirror partners (lane i <-> 15 - i / 7 - i: opposite bit, same
  // higher bits), bits 2, 1: DPP quad_perm xor. Same index mapping as an xor butterfly (lane L ends with
  // outputs 2L, 2L+1); cdna_hip_programming.md T12/T21.
  // (inline asm: with this hipcc the __builtin_amdgcn_permlane{16,32}_swap pair result came back as the
  // same register twice, x + x, tools/probe_src/halving.hip; "s_nop 1" covers the VALU-write -> permlane
  // hazard, cdna_hip_programming.md T21)
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
  dpp_level(std::integral_constant<int, 0x140>{}, 8, NV / 4);  // row_mirror
  dpp_level(std::integral_constant<int, 0x141>{}, 4, NV / 8);  // row_half_mirror
  dpp_level(std::integral_constant<int, 0x4e>{}, 2, NV / 16);  // quad_perm [2,3,0,1]
  dpp_level(std::integral_constant<int, 0xb1>{}, 1, NV / 32);  // quad_perm [1,0,3,2]
  // channel 256 (the Nyquist bin): lane L of wave 0 adds its contribution to outputs 2L, 2L+1
  if (wave == 0) {
    const int i = lane >> 1, o0 = 2 * (lane & 1);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float x = vad_in(a, b, s, t0 + i - 2 + k, NBIN - 1);
      acc[0] = fmaf(a.w1[((size_t)o0 * NBIN + NBIN - 1) * 5 + k], x, acc[0]);
      acc[1] = fmaf(a.w1[((size_t)(o0 + 1) * NBIN + NBIN - 1) * 5 + k], x, acc[1]);
    }
  }
  stamp(3);
  part[wave][2 * lane] = acc[0];
  part[wave][2 * lane + 1] = acc[1];
  lds_sync();
  stamp(4);
  float st[2] = {0.f, 0.f};
  if (tid < NV) {
    const int ii = tid >> 2, o = tid & 3;
    const int t = t0 + ii;
    const float y = ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid];
    const float v = prelu_f(y + a.b1[o], a.alpha);
    a.vy[(((size_t)b * 2 + s) * 4 + o) * a.Tp + t] = (t < T) ? v : 0.f;
    if (t < T) { st[0] = v; st[1] = v * v; }
  }
  const int nrec = a.Tp / R;
  block_reduce_store<2>(st, red, a.out_rec + ((size_t)bs * nrec + blockIdx.y) * 2);
  stamp(5);
}

// k_vad_feat: the VAD head's conv1_1 finished from the output head's tap products (k_tcn) (fused schedule), one workgroup per
// (utterance, speaker): y[t][o] = sum_k P[t - 2 + k][4 k + o] (zero outside [0, T)), v = PReLU(y + b1),
// BN_1 = GroupNorm(1, 4) over [4, T] (block sums in double, wave order), feat = v * s[o] + h[o] for
// k_istft_pair's VAD tail (model/model.py:158-176).
// NI items (t, o) per thread: 4 for T <= 256, 16 for T <= VF_ONE_T (longer utterances: k_vad_feat_rec).
template <int NI>
__global__ __launch_bounds__(256) void k_vad_feat(VadFeatArgs a) {
  __shared__ float red[2 * 16];
  __shared__ double dacc[2];
  __shared__ float vs[4], vh[4];
  const int tid = threadIdx.x, bs = blockIdx.x, T = a.T;
  const float* P = a.vP + (size_t)bs * a.Tp * HEAD_VAD_N;
  float v[NI], st[2] = {0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const int i = tid + 256 * it, t = i >> 2, o = i & 3;
    float y = 0.f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int tt = t - 2 + k;
      y += (i < 4 * T && tt >= 0 && tt < T) ? P[(size_t)tt * HEAD_VAD_N + 4 * k + o] : 0.f;
    }
    v[it] = prelu_f(y + a.b1[o], a.alpha);
    if (i < 4 * T) { st[0] += v[it]; st[1] += v[it] * v[it]; }
  }
  block_reduce_store<2>(st, red, dacc);
  lds_sync();
  if (tid < 4) {
    float mu, rs;
    gn_moments(dacc[0], dacc[1], 4.0 * T, a.eps, mu, rs);
    vs[tid] = rs * a.g[tid];
    vh[tid] = a.be[tid] - vs[tid] * mu;
  }
  lds_sync();
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const int i = tid + 256 * it, t = i >> 2, o = i & 3;
    if (i < 4 * T) a.feat[((size_t)bs * 4 + o) * a.Tp + t] = fmaf(v[it], vs[o], vh[o]);
  }
}

// k_vad_feat_rec: long utterances (T > VF_ONE_T). One workgroup per (utterance, speaker, VF_ROWS frames): the same
// conv1_1 + PReLU items as k_vad_feat, written un-normalised, and the chunk's BN_1 partial record {sum, sumsq} (wave
// sums, then the 4 wave totals in double in wave order); k_istft_pair sums the records in record order and applies BN_1
// (its vy_norm = 0 path). One workgroup per utterance and speaker took 35 us for two 60 s files (4 workgroups).
__global__ __launch_bounds__(256) void k_vad_feat_rec(VadFeatArgs a) {
  __shared__ float red[2 * 16];
  constexpr int NI = 4 * VF_ROWS / 256;
  const int tid = threadIdx.x, bs = blockIdx.x, T = a.T, t0 = blockIdx.y * VF_ROWS;
  const float* P = a.vP + (size_t)bs * a.Tp * HEAD_VAD_N;
  float st[2] = {0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const int i = tid + 256 * it, t = t0 + (i >> 2), o = i & 3;
    float y = 0.f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int tt = t - 2 + k;
      y += (t < T && tt >= 0 && tt < T) ? P[(size_t)tt * HEAD_VAD_N + 4 * k + o] : 0.f;
    }
    const float v = prelu_f(y + a.b1[o], a.alpha);
    if (t < a.Tp) a.feat[((size_t)bs * 4 + o) * a.Tp + t] = t < T ? v : 0.f;
    if (t < T) { st[0] += v; st[1] += v * v; }
  }
  block_reduce_store<2>(st, red, a.out_rec + ((size_t)bs * vf_nrec(a.Tp) + blockIdx.y) * 2);
}

hipError_t launch_vad_feat(const VadFeatArgs& a, hipStream_t s) {
  if (a.T < 1 || a.T > 8192) return hipErrorInvalidValue;
  if (a.T > VF_ONE_T) {
    if (a.out_rec == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_vad_feat_rec, dim3(a.B * 2, vf_nrec(a.Tp)), dim3(256), 0, s, a);
  } else if (a.T <= 256) {
    hipLaunchKernelGGL(k_vad_feat<4>, dim3(a.B * 2), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_vad_feat<16>, dim3(a.B * 2), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_vad1(const Vad1Args& a, hipStream_t s) {
  if (a.Tp % VAD_ROWS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_vad1, dim3(a.B * 2, a.Tp / VAD_ROWS), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// iSTFT: one workgroup (8 waves) per (utterance*speaker, chunk of IS_OWN frames). Computes frames
// [f0-1, f0+IS_OWN) (one halo frame) and owns output hop-segments [f0, f0+IS_OWN) (+ segment T for
// the last chunk). Segment j = padded samples [256 j, 256 j + 256); output n = p - 256.
// LDS <= 53 KB (three workgroups per CU): half twiddle table, the window read through the cache, and the
// mask side-output staging aliased onto the FFT work buffers (the two are live in different phases).
__global__ __launch_bounds__(512) void k_istft(IstftArgs a) {
  __shared__ float2 tw[256];
  __shared__ float2 spec[IS_FR][NBIN + 1];   // est of the computed frames; later their time samples
  __shared__ float2 work[8][M256];
  static_assert(IS_OWN * NBIN * sizeof(float) <= sizeof(work), "mask staging fits the work buffers");
  float (*mk)[NBIN] = reinterpret_cast<float (*)[NBIN]>(&work[0][0]);  // sigmoid(mask) of owned frame fo+1 at row fo
  const float* win = a.window;
  __shared__ float yn[4][IS_FR + 6];          // GN'd VAD features, frames fbeg-3 .. fbeg+IS_FR+2
  __shared__ float vadv[IS_FR + 4];           // vad at frames fbeg-2 .. fbeg+IS_FR+1
  __shared__ float gain[IS_FR];
  __shared__ float vs[4], vh[4];
  __shared__ double dacc[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bs = blockIdx.x, f0 = blockIdx.y * IS_OWN;
  const int T = a.T;
  const int b = bs / a.S, s = bs % a.S;
  const int fbeg = f0 - 1;
  if (tid < 256) tw[tid] = a.tw[tid];

  // Every input load of the block is issued up front (forward mode): the X / mask rows of the computed
  // frames into registers, the VAD features, then the BN_1 records. The block then waits once instead
  // of three dependent HBM round trips (records -> features -> rows). Frames outside [0, T) load a
  // clamped in-bounds row and are masked to zero on use.
  constexpr int NE = (IS_FR * NBIN + 511) / 512;
  float2 xr[NE];
  float mr[NE];
  float yv = 0.f;
  const bool fwd = a.est_mode != 0;
  const bool vad = fwd && a.has_vad;
  if (fwd) {
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int i = min(tid + j * 512, IS_FR * NBIN - 1);
      const int fi = i / NBIN, k = i - fi * NBIN;
      const int fc = min(max(fbeg + fi, 0), T - 1);
      const size_t row = (size_t)b * a.Tp + fc;
      xr[j] = a.X[row * NBIN + k];
      mr[j] = a.masks[row * MOUT_PAD + s * NBIN + k];
    }
    if (vad && tid < 4 * (IS_FR + 6)) {
      const int o = tid / (IS_FR + 6), q = tid % (IS_FR + 6);
      const int fc = min(max(fbeg - 3 + q, 0), T - 1);
      yv = a.vy[((size_t)bs * 4 + o) * a.Tp + fc];
    }
  }

  // 0) VAD tail for the frames this block needs
  if (vad) {
    gn_from_records(a.vgn, bs, 4, T, vs, vh, dacc);  // BN_1 = GroupNorm(1, 4, eps 1e-8)
    lds_sync();
    if (tid < 4 * (IS_FR + 6)) {
      const int o = tid / (IS_FR + 6), q = tid % (IS_FR + 6);
      const int f = fbeg - 3 + q;
      yn[o][q] = (f >= 0 && f < T) ? fmaf(yv, vs[o], vh[o]) : 0.f;
    }
    lds_sync();
    if (tid < IS_FR + 4) {
      const int f = fbeg - 2 + tid;
      float z = a.b2;
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int k = 0; k < 3; ++k) z = fmaf(a.w2[o * 3 + k], yn[o][tid + k], z);
      const float p = sigmoid_f(z);
      vadv[tid] = (f >= 0 && f < T) ? p : 0.f;
      if (!a.kw_enabled && f >= f0 && f < f0 + IS_OWN && f < T) a.vad_out[(size_t)bs * T + f] = p;
    }
    lds_sync();
    if (tid < IS_FR) {
      const int f = fbeg + tid;
      float g = 1.f;
      if (a.kw_enabled && f >= 0 && f < T) {
        auto thr = [&](int ff) -> float {  // threshold of frame ff (0 outside [0,T): zero padding)
          if (ff < 0 || ff >= T) return 0.f;
          return vadv[ff - (fbeg - 2)] >= a.thr ? 1.f : 0.f;
        };
        float smv = fminf(thr(f - 1) + thr(f + 1), 1.f);
        if (f == 0 || f == T - 1) smv = thr(f);
        if (a.filt) g = smv;
        if (f >= f0 && f < f0 + IS_OWN)
          a.vad_out[(size_t)bs * T + f] = a.ret_smooth ? smv : vadv[f - (fbeg - 2)];
      }
      gain[tid] = g;
    }
  } else {
    if (tid < IS_FR) gain[tid] = 1.f;
  }
  lds_sync();

  // 1) est for the computed frames (frame-major, coalesced over bins)
  if (fwd) {
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int i = tid + j * 512;
      if (i < IS_FR * NBIN) {
        const int fi = i / NBIN, k = i - fi * NBIN;
        const int f = fbeg + fi;
        const bool ok = f >= 0 && f < T;
        // noisy-phase synthesis (|X| m) e^{j angle X} == X m up to rounding (model/model.py:430-437)
        const float m = ok ? sigmoid_f(mr[j]) : 0.f;
        const float g = gain[fi];
        spec[fi][k] = ok ? make_float2(g * (xr[j].x * m), g * (xr[j].y * m)) : make_float2(0.f, 0.f);
        if (fi > 0) mk[fi - 1][k] = m;
      }
    }
  } else {
    for (int i = tid; i < IS_FR * NBIN; i += 512) {
      const int fi = i / NBIN, k = i % NBIN;
      const int f = fbeg + fi;
      float2 e = make_float2(0.f, 0.f);
      if (f >= 0 && f < T) e = a.est_in[((size_t)bs * NBIN + k) * T + f];
      spec[fi][k] = e;
      if (fi > 0) mk[fi - 1][k] = 0.f;
    }
  }
  lds_sync();
  // side outputs of the owned frames, bin-major [bs][k][f] (15 consecutive frames per bin)
  if (a.est_mode && (a.est_out || a.mask_out)) {
    // all LDS reads first, then the stores (no per-element read -> wait -> store chain)
    constexpr int NI = (NBIN * IS_OWN + 511) / 512;
    float2 ev[NI];
    float mv[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = min(tid + j * 512, NBIN * IS_OWN - 1);
      const int k = i / IS_OWN, fo = i - k * IS_OWN;
      ev[j] = spec[fo + 1][k];
      mv[j] = mk[fo][k];
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = tid + j * 512;
      const int k = i / IS_OWN, fo = i - k * IS_OWN;
      const int f = f0 + fo;
      if (i < NBIN * IS_OWN && f < T) {
        const size_t o = ((size_t)bs * NBIN + k) * T + f;
        if (a.est_out) a.est_out[o] = ev[j];
        if (a.mask_out) a.mask_out[o] = mv[j];
      }
    }
  }
  lds_sync();  // side outputs read spec rows that the transforms below overwrite
  // 2) inverse real FFT per frame: 8 waves x 2 rounds = 16 frames, each wave on its own rows (wave-local
  // ordering only)
  for (int round = 0; round < IS_FR / 8; ++round) {
    const int fi = round * 8 + wave;
    float2* Y = spec[fi];
    float2* w0 = work[wave];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = lane + 64 * r;  // 0..255
      float2 yk = Y[k], ym = Y[M256 - k];
      if (k == 0) { yk.y = 0.f; ym.y = 0.f; }  // c2r ignores Im of DC and Nyquist
      const float2 cym = conjf2(ym);
      const float2 E = make_float2(0.5f * (yk.x + cym.x), 0.5f * (yk.y + cym.y));
      const float2 Dd = csub(yk, cym);
      float2 w = tw[k];
      w.y = -w.y;  // W512^{-k}
      const float2 Oo = cmul(make_float2(0.5f * Dd.x, 0.5f * Dd.y), w);
      w0[k] = make_float2(E.x - Oo.y, E.y + Oo.x);  // E + i O
    }
    wave_lds_sync();
    // ping-pong with the (now consumed) spec row of this frame; result lands in w0
    fft256<true, true>(w0, Y, tw, lane);
    float* fr = reinterpret_cast<float*>(Y);  // time samples overwrite the frame's spectrum row
    const float sc = 1.f / 256.f;             // 1/N of the 512-point c2r == 1/256 on the half-length transform
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = lane + 64 * r;
      const float2 v = w0[m];
      fr[2 * m] = v.x * sc * win[2 * m];
      fr[2 * m + 1] = v.y * sc * win[2 * m + 1];
    }
    wave_lds_sync();
  }
  lds_sync();  // every frame's time samples in place for the overlap-add
  // 3) overlap-add of the owned segments, divided by the window envelope (torch.istft)
  const int nseg = min(IS_OWN, T - f0) + ((f0 + IS_OWN >= T) ? 1 : 0);
  float* yb = a.y + (size_t)bs * a.N;
  for (int i = tid; i < nseg * HOP; i += 512) {
    const int jj = i / HOP, q = i % HOP;
    const int j = f0 + jj;
    const int n = j * HOP + q - HOP;
    if (n < 0 || n >= a.N) continue;
    float num = 0.f, den = 0.f;
    if (j < T) {  // frame j, first half
      num += reinterpret_cast<const float*>(spec[j - fbeg])[q];
      den += win[q] * win[q];
    }
    if (j >= 1) {  // frame j-1, second half
      num += reinterpret_cast<const float*>(spec[j - 1 - fbeg])[q + HOP];
      den += win[q + HOP] * win[q + HOP];
    }
    yb[n] = num / den;
  }
}

hipError_t launch_istft(const IstftArgs& a, hipStream_t s) {
  dim3 grid(a.BS, (a.T + IS_OWN - 1) / IS_OWN);
  hipLaunchKernelGGL(k_istft, grid, dim3(512), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
