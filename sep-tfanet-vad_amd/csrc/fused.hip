// The whole TCN separator (24 x [DepthConv1d + TF_Attention + recursive/residual LN], reference
// model/model.py:103-149,182-208,271-357) as ONE persistent launch: k_tcn.
//
// Work split: an utterance of T frames is owned by a GROUP of G = ceil(T/32) workgroups; member g owns
// frames [32g, 32g+32) and ALL 256 channels of them, for every block. Inside a block every 1x1 conv is a
// row-local GEMM (frames x channels) and the depthwise conv needs `dil` halo frames, so the only
// cross-workgroup traffic of a block is four small hand-offs inside the group:
//   P1  after conv1d:     GroupNorm(reg1) partial sums + the raw conv1d output of the dil boundary frames
//   P2  after the dwconv: GroupNorm(reg2) partial sums (awaited only after the res_out GEMM main loop)
//   P3  after res_out:    per-channel sums over the member's frames (a_f) and per-frame channel sums (a_t)
//   P4  after the gates:  the moment record of the residual update (recursive / residual LN statistics)
// Everything else stays on the CU: the residual stream o lives in registers (the res_out accumulator
// layout), the GEMM A operands (x' for conv1d, d for res_out) live in LDS as fp16 hi/lo planes, the
// conv1d output lives in LDS, and the weights stream from L2 straight into registers in MFMA fragment
// order (packed on the host: one contiguous 1 KB per wave per 16-deep K step).
//
// Arithmetic: fp16x3 split (see gemm.hip): acc += A_lo B_hi + A_hi B_lo + A_hi B_hi on
// v_mfma_f32_32x32x16_f16, weights pre-scaled per row by 2^-e; reg2 folded into W2/epilogue as in
// the multi-kernel path. GroupNorm statistics: float partials per wave, double across waves and members,
// fixed order => bitwise reproducible and independent of placement and batch composition.
//
// Hand-off protocol (MI355X_MICROARCH.md visibility table, row "one lane of each storing workgroup";
// cdna_hip_programming.md Guideline 16 R1): wave 0 stores the payload write-through (sc1 buffer stores),
// drains (s_waitcnt vmcnt(0)), then lane 0 stores the epoch into the member's flag (agent-scope relaxed
// atomic store = sc1). Consumers: thread 0 polls the other members' flags (relaxed sc1 loads + s_sleep,
// bounded: a give-up sets *err and the kernel runs to completion instead of hanging), a workgroup barrier,
// then EVERY load of handed-off bytes is an sc1 buffer load. Payload slots are double-buffered by epoch
// parity: a member publishes epoch e+2 only after it has seen every member's epoch e+1 flag, and every
// member publishes e+1 only after it has read all epoch-e data.
//
// Residency: one 512-thread workgroup per CU (LDS ~114 KB), grid <= the occupancy-derived capacity, and a
// group's members are dealt to one XCD (blocks b, b+8, ... share an XCD under round-robin dispatch:
// speed only, never correctness). Groups loop over utterances (persistent), so any batch size runs.
#include "device_common.h"

namespace sepvad {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

constexpr int NTHR = 512;         // 8 waves; wave w owns output channels [32w, 32w+32) of both GEMMs
constexpr int LDX = CH + 8;       // x' row stride (halves): 132 dwords == 4 (mod 64) => conflict-free b128 reads
constexpr int LDD = HID + 8;      // d row stride (halves): 260 dwords == 4 (mod 64)
constexpr int HROW = FR + 8;      // conv1d output rows incl. 4 halo rows on each side
constexpr int PD = 8;             // weight K steps in flight per wave
constexpr int NS1 = CH / 16;      // conv1d K steps (256 / 16)
constexpr int NS2 = HID / 16;     // res_out K steps (512 / 16)

struct TcnSmem {
  _Float16 Ahi[FR * LDD];         // GEMM A operand, hi plane: x' [32][LDX] or d [32][LDD]
  _Float16 Alo[FR * LDD];         //                 lo plane
  float H[HROW * CH];             // conv1d output (raw, pre-GN1) rows -4..35; later r for the colsums
  float c[4][CH];                 // per-channel affines (GN1 / recursive-LN)
  float af[CH];                   // frequency gate a_f
  float vec[CH + 8];              // channel means / rowsum staging
  float yf[CH + 8];
  float mC[FR + 8], yt[FR + 8], at[FR];
  float cs[FR][8];                // per-frame channel partial sums (8 channel slices)
  float red[NMOM * 16];
  double dred[16];
  float prm[PB_SIZE];             // this block's parameter blob (PB_*)
};

// Wave-uniform copies (readfirstlane) of values loaded from the block-parameter table: the compiler cannot
// prove those loads uniform, and a buffer descriptor in VGPRs becomes a waterfall loop per access.
template <typename Tp>
__device__ __forceinline__ Tp* uni(Tp* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (Tp*)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float unif(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
}
// Buffer descriptor over a wave-uniform base. The base goes through readfirstlane: under SGPR pressure
// hipcc keeps uniform pointers in VGPRs, and a descriptor it cannot prove uniform turns every buffer
// access into a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uni(p)), (short)0, 0x7fffffff, 0x00020000);
}
// Write-through (sc1) stores / sc1 loads of hand-off payload, addressed as float offsets from the
// (wave-uniform) payload base: aux 16 = sc1 on gfx950.
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, int foff, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, foff * 4, 0, 16);
}
// Same-XCD groups: plain stores keep the line in the shared L2, where the consumers' sc1 loads (L1
// bypass) find it; the drain before the flag makes the stores complete at L2 first.
__device__ __forceinline__ void st_l2(__amdgpu_buffer_rsrc_t r, int foff, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, foff * 4, 0, 0);
}
__device__ __forceinline__ float4 ld_wt(__amdgpu_buffer_rsrc_t r, int foff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, foff * 4, 0, 16));
}
__device__ __forceinline__ float ld_wt1(__amdgpu_buffer_rsrc_t r, int foff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, foff * 4, 0, 16));
}
__device__ __forceinline__ double ld_wtd(__amdgpu_buffer_rsrc_t r, int foff) {  // foff even
  const unsigned lo = __builtin_amdgcn_raw_buffer_load_b32(r, foff * 4, 0, 16);
  const unsigned hi = __builtin_amdgcn_raw_buffer_load_b32(r, foff * 4 + 4, 0, 16);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// Sum over the group's members (in member order) of the double / float at float offset `off` of each
// member's slot of epoch e: all loads issued before the first add (one latency, not G).
template <typename Slot>
__device__ __forceinline__ double sum_members_d(__amdgpu_buffer_rsrc_t r, const Slot& slot, int G, unsigned e, int off) {
  double v[FG_MAX];
#pragma unroll
  for (int mm = 0; mm < FG_MAX; ++mm) v[mm] = mm < G ? ld_wtd(r, slot(mm, e) + off) : 0.0;
  double s = 0.0;
#pragma unroll
  for (int mm = 0; mm < FG_MAX; ++mm) if (mm < G) s += v[mm];
  return s;
}
template <typename Slot>
__device__ __forceinline__ float sum_members_f(__amdgpu_buffer_rsrc_t r, const Slot& slot, int G, unsigned e, int off) {
  float v[FG_MAX];
#pragma unroll
  for (int mm = 0; mm < FG_MAX; ++mm) v[mm] = mm < G ? ld_wt1(r, slot(mm, e) + off) : 0.f;
  float s = 0.f;
#pragma unroll
  for (int mm = 0; mm < FG_MAX; ++mm) if (mm < G) s += v[mm];
  return s;
}

__device__ __forceinline__ float4 dd_as_f4(double a, double b) {
  const unsigned long long x = __builtin_bit_cast(unsigned long long, a), y = __builtin_bit_cast(unsigned long long, b);
  return make_float4(__builtin_bit_cast(float, (unsigned)x), __builtin_bit_cast(float, (unsigned)(x >> 32)),
                     __builtin_bit_cast(float, (unsigned)y), __builtin_bit_cast(float, (unsigned)(y >> 32)));
}

// Group hand-off state of one workgroup (see the header comment).
struct Xchg {
  __amdgpu_buffer_rsrc_t pay; // payload slots [ngroups*G][2][FPAY]
  unsigned* flags;           // [ngroups*G][2]
  unsigned* err;
  int base, G, g;            // first member's index, members, own member index
  unsigned ep;               // epochs published so far
  bool failed;               // thread 0: a wait gave up (skip later waits)
  bool l2;                   // every member on this workgroup's XCD: payload and flags stay in its L2

  __device__ void store(int foff, float4 v) const {
    if (l2) st_l2(pay, foff, v);
    else st_wt(pay, foff, v);
  }
  __device__ int slot(int member, unsigned e) const { return ((base + member) * 2 + (int)(e & 1)) * FPAY; }
  // after wave 0 stored the payload of epoch ep+1 into slot(g, ep+1): drain, flag
  __device__ void publish(int wave, int lane) {
    ++ep;
    if (wave == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      unsigned* f = flags + (size_t)(base + g) * 2 + (ep & 1);
      if (lane == 0) {
        if (l2) *reinterpret_cast<volatile unsigned*>(f) = ep;
        else __hip_atomic_store(f, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // thread 0 waits for every other member's flag of epoch e; the caller then barriers
  __device__ void wait(unsigned e) {
    if (threadIdx.x != 0 || failed) return;
    // every member's flag loaded in one pass (independent loads in flight together), until all >= e
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int m = 0; m < FG_MAX; ++m) {
        if (m < G && m != g) {
          const unsigned* f = flags + (size_t)(base + m) * 2 + (e & 1);
          ok = (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= e) && ok;
        }
      }
      if (ok) return;
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 1023u) == 0 &&
          (spins > (1u << 22) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        failed = true;
        return;
      }
    }
  }
};

// conv1d / res_out GEMM of one wave: acc[32 frames x 32 channels] += A[32 x 16*NS] * W^T. A comes from
// LDS (hi/lo planes, row stride LDA); the W fragments stream from global (buffer loads over the
// fragment-ordered weight, this lane's bytes at voff + 1024 * step) with PD steps in flight in a
// static register ring; the first PD steps are already in (rh, rl) on entry.
template <int NS, int LDA>
__device__ __forceinline__ void wave_gemm(f32x16v& acc, const _Float16* Ahi, const _Float16* Alo,
                                          __amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int voff,
                                          u32x4v (&rh)[PD], u32x4v (&rl)[PD], int lane) {
  static_assert(NS % PD == 0 && NS > PD, "K steps");
  const int aoff = (lane & 31) * LDA + 8 * (lane >> 5);
  auto step = [&](int s, int i, bool pf) {
    const f16x8 ah = *reinterpret_cast<const f16x8*>(Ahi + aoff + 16 * s);
    const f16x8 al = *reinterpret_cast<const f16x8*>(Alo + aoff + 16 * s);
    const f16x8 bh = __builtin_bit_cast(f16x8, rh[i]);
    const f16x8 bl = __builtin_bit_cast(f16x8, rl[i]);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
    if (pf) {
      rh[i] = __builtin_amdgcn_raw_buffer_load_b128(wh, voff, (s + PD) * 1024, 0);
      rl[i] = __builtin_amdgcn_raw_buffer_load_b128(wl, voff, (s + PD) * 1024, 0);
    }
  };
#pragma unroll
  for (int s0 = 0; s0 < NS - PD; s0 += PD) {
#pragma unroll
    for (int i = 0; i < PD; ++i) step(s0 + i, i, true);
  }
#pragma unroll
  for (int i = 0; i < PD; ++i) step(NS - PD + i, i, false);
}

__device__ __forceinline__ void prefetch_w(__amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int voff,
                                           u32x4v (&rh)[PD], u32x4v (&rl)[PD]) {
#pragma unroll
  for (int s = 0; s < PD; ++s) {
    rh[s] = __builtin_amdgcn_raw_buffer_load_b128(wh, voff, s * 1024, 0);
    rl[s] = __builtin_amdgcn_raw_buffer_load_b128(wl, voff, s * 1024, 0);
  }
}

__device__ __forceinline__ void split_store(_Float16* hi, _Float16* lo, int idx, float v) {
  const _Float16 h = (_Float16)v;
  hi[idx] = h;
  lo[idx] = (_Float16)(v - (float)h);
}

// diagnostics (SEPVAD_TCN_PROBE): wave 0's wall clock at 13 phase points of every block of the first
// utterance each workgroup processes: probe[(blockIdx * nblk + block) * 16 + point]
#define TPROBE(k)                                                                                  \
  do {                                                                                             \
    if (a.probe != nullptr && tid == 0 && u == grp)                                                \
      a.probe[((size_t)blockIdx.x * a.nblk + bi) * 16 + (k)] = wall_clock64();                     \
  } while (0)

// DPP lane reductions (no LDS round trip, fixed order => deterministic). update_dpp with old = 0:
// lanes whose DPP source is out of range add 0.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// quad_perm [1,0,3,2], [2,3,0,1], row_shr:4, row_shr:8, row_bcast:15 => lane 31 holds the sum of lanes
// 0..31 and lane 63 the sum of lanes 32..63.
__device__ __forceinline__ float half_total(float v) {
  v += dpp_f<0xb1>(v);
  v += dpp_f<0x4e>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  v += dpp_f<0x142>(v);
  return v;
}
// Sum over the 64 lanes (+ row_bcast:31), returned wave-uniform (lane 63).
__device__ __forceinline__ float wave_total(float v) {
  v = half_total(v);
  v += dpp_f<0x143>(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
// Block sums of NV per-thread values (512 threads): waves by DPP, the 8 wave totals in double in wave
// order by thread j < NV into out[j]. One barrier; callers barrier again before reading `out`.
template <int NV>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* lds, double* out) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float t = wave_total(v[j]);
    if ((threadIdx.x & 63) == 0) lds[j * 8 + w] = t;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += lds[threadIdx.x * 8 + i];
    out[threadIdx.x] = t;
  }
}

template <int LM>
__global__ __launch_bounds__(NTHR) void k_tcn(TcnArgs a) {
  __shared__ __attribute__((aligned(16))) TcnSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = a.G;
  // block -> (group, member): members of a group on one XCD when the grid is a multiple of 8*G
  int grp, g;
  if (gridDim.x % (8 * G) == 0) {
    const int x = blockIdx.x & 7, idx = blockIdx.x >> 3;
    grp = (idx / G) * 8 + x;
    g = idx % G;
  } else {
    grp = blockIdx.x / G;
    g = blockIdx.x % G;
  }
  const int ngroups = gridDim.x / G;
  Xchg xc{rsrc_of(a.pay), a.flags, a.err, grp * G, G, g, 0u, false, false};
  const __amdgpu_buffer_rsrc_t pr = xc.pay;
  auto xslot = [&](int mm, unsigned e) { return xc.slot(mm, e); };
  // epoch 1: the members' XCD ids (write-through protocol); if the whole group shares one XCD, every later
  // hand-off keeps its bytes in that XCD's L2 (correct for any placement: checked, not assumed)
  {
    const unsigned xcc = __builtin_amdgcn_s_getreg(6164) & 0xfu;  // hwreg(HW_REG_XCC_ID, 0, 4)
    if (tid == 0) st_wt(pr, xc.slot(g, 1), make_float4(__builtin_bit_cast(float, xcc), 0.f, 0.f, 0.f));
    xc.publish(wave, lane);
    xc.wait(1);
    __syncthreads();
    if (tid == 0) {
      bool same = a.xmode == 0;
      for (int mm = 0; mm < G; ++mm) same = same && __builtin_bit_cast(unsigned, ld_wt1(pr, xc.slot(mm, 1))) == xcc;
      sm.red[0] = same ? 1.f : 0.f;
    }
    __syncthreads();
    xc.l2 = sm.red[0] != 0.f;
    __syncthreads();
  }
  const int T = a.T, Tp = a.Tp, t0 = g * FR;
  const int m = 32 * wave + (lane & 31);            // this lane's output channel in both GEMMs
  const int hl = lane >> 5;
  auto trow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * hl; };
  const bool tf = a.tf_att != 0;
  // byte offset of this lane's 16-B fragment within its wave's weight stream (step 0)
  const int voff1 = (wave * NS1 * 64 + lane) * 16, voff2 = (wave * NS2 * 64 + lane) * 16;

  for (int u = grp; u < a.B; u += ngroups) {
    // ---- TCN input: x'_0 = TCN.LN(S0) (model/model.py:333), own frames, into o and the LDS A operand
    float o[16];
    {
      float pg[2], pb[2];
      ld_chan(a.ln.g, CH, pg);
      ld_chan(a.ln.be, CH, pb);
      float raw[16];
      const float* S0u = a.S0 + ((size_t)u * Tp + t0) * CH;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = t0 + trow(r);
        raw[r] = t < T ? S0u[trow(r) * CH + m] : 0.f;
      }
      reduce_records(rec_src(a.ln, u, 2), rec_none(), sm.dred);
      __syncthreads();
      gn_affine(sm.dred, CH, T, a.ln.eps, pg, pb, sm.c[0], sm.c[1]);
      __syncthreads();
      const float s = sm.c[0][m], h = sm.c[1][m];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tl = trow(r);
        o[r] = (t0 + tl < T) ? fmaf(raw[r], s, h) : 0.f;
        split_store(sm.Ahi, sm.Alo, tl * LDX + m, o[r]);
      }
    }
    u32x4v rh[PD], rl[PD];
    prefetch_w(rsrc_of(a.wfrag), rsrc_of(a.wfrag + WF_W1L), voff1, rh, rl);
    __syncthreads();

    for (int bi = 0; bi < a.nblk; ++bi) {
      // Opaque per-iteration copies of the lane's row offset and channel: every per-row LDS address is then
      // base + immediate offset. Without this hipcc hoists the 16 row addresses of each array out of the
      // block loop as invariants, runs out of registers and spills them (scratch reloads on every row).
      int hl4o = 4 * hl, mo_ = 32 * wave + (lane & 31);
      asm volatile("" : "+v"(hl4o), "+v"(mo_));
      const int m = mo_;
      auto trow = [&](int r) { return (r & 3) + 8 * (r >> 2) + hl4o; };
      TPROBE(0);
      const __half* wb = a.wfrag + (size_t)bi * WF_BLOCK;
      const int li = bi % a.layer;
      const int dil = li == 0 ? 1 : (li % 4 + 1);   // model/model.py:285-295 (as api.hip packs it)
      const float* pm = sm.prm;
      // this block's parameters: loads issued now (behind the already-landed weight prefetch), stored
      // into LDS after the conv1d GEMM
      float4 pv[3];
      {
        const float4* src = reinterpret_cast<const float4*>(a.prm + (size_t)bi * PB_SIZE);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int idx = tid + k * NTHR;
          if (idx < PB_SIZE / 4) pv[k] = src[idx];
        }
      }
      // ================= conv1d 256->256 (model/model.py:132) + PReLU =================
      f32x16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      {
        wave_gemm<NS1, LDX>(acc, sm.Ahi, sm.Alo, rsrc_of(wb), rsrc_of(wb + WF_W1L), voff1, rh, rl, lane);
      TPROBE(1);
      }
      {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int idx = tid + k * NTHR;
          if (idx < PB_SIZE / 4) reinterpret_cast<float4*>(sm.prm)[idx] = pv[k];
        }
        __syncthreads();
        const float ws = pm[PB_WS1 + m], bias = pm[PB_B1 + m], a1 = pm[PB_A1];
        float st[2] = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tl = trow(r);
          float v = prelu_f(fmaf(acc[r], ws, bias), a1);
          v = (t0 + tl < T) ? v : 0.f;
          sm.H[(tl + 4) * CH + m] = v;
          st[0] += v; st[1] += v * v;
        }
        block_sums<2>(st, sm.red, sm.dred);  // barrier inside: H complete
      TPROBE(2);
      }
      // ---- P1: GN1 partial sums + boundary rows (first dil / last dil own frames) ----
      {
        const unsigned e = xc.ep + 1;
        const int dst = xc.slot(g, e);
        __syncthreads();
        if (wave == 0) {
          if (lane == 0) xc.store(dst + 0, dd_as_f4(sm.dred[0], sm.dred[1]));
          // rows 0..dil-1 -> [16, 16 + dil*256); rows 32-dil..31 -> [16 + 4*256, ...)
          for (int i = lane; i < 2 * dil * (CH / 4); i += 64) {
            const int j = i / (CH / 4), c4 = (i % (CH / 4)) * 4;
            const int tl = j < dil ? j : FR - 2 * dil + j;
            const int off = j < dil ? 16 + j * CH : 16 + 4 * CH + (j - dil) * CH;
            xc.store(dst + off + c4, *reinterpret_cast<const float4*>(&sm.H[(tl + 4) * CH + c4]));
          }
        }
        xc.publish(wave, lane);
        xc.wait(e);
        __syncthreads();
      TPROBE(3);
        // GN1 statistics over the group (members in order) -> affine
        float pg[2], pb[2];
        ld_chan(pm + PB_G1, CH, pg);
        ld_chan(pm + PB_BE1, CH, pb);
        if (tid < 2) {
          double s = 0.0;
          s = sum_members_d(pr, xslot, G, e, 2 * tid);
          sm.dred[8 + tid] = s;
        }
        // halo rows from the neighbours (raw conv1d outputs)
        for (int i = tid; i < 2 * dil * (CH / 4); i += NTHR) {
          const int j = i / (CH / 4), c4 = (i % (CH / 4)) * 4;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          int row;
          if (j < dil) {  // rows -dil..-1 = predecessor's last dil rows
            row = 4 - dil + j;
            if (g > 0) v = ld_wt(pr, xc.slot(g - 1, e) + 16 + 4 * CH + j * CH + c4);
          } else {        // rows 32..32+dil-1 = successor's first dil rows
            row = 4 + FR + (j - dil);
            if (g + 1 < G) v = ld_wt(pr, xc.slot(g + 1, e) + 16 + (j - dil) * CH + c4);
          }
          *reinterpret_cast<float4*>(&sm.H[row * CH + c4]) = v;
        }
        // res_out weights: in flight during the depthwise conv (issued after every load this phase
        // waits for: vmcnt retires in order, so nothing earlier waits behind the weight stream)
        prefetch_w(rsrc_of(wb + WF_W2H), rsrc_of(wb + WF_W2L), voff2, rh, rl);
        __syncthreads();
        gn_affine(sm.dred + 8, CH, T, 1e-8f, pg, pb, sm.c[0], sm.c[1]);
        __syncthreads();
      }
      // ================= depthwise conv (model/model.py:134-135): d = PReLU(dconv(GN1(h))) =================
      {
        const int c = tid & (CH - 1), rh0 = (tid >> 8) * (FR / 2);
        const float a2 = pm[PB_A2];
        const float sc = sm.c[0][c], sh = sm.c[1][c];
        float wv[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = 2 * c + q;
          wv[q][0] = pm[PB_WD + j * 3 + 0]; wv[q][1] = pm[PB_WD + j * 3 + 1]; wv[q][2] = pm[PB_WD + j * 3 + 2];
          wv[q][3] = pm[PB_BD + j];
        }
        auto hn = [&](int tl) -> float {  // GN1(h) at local frame tl (zero outside [0, T))
          const int t = t0 + tl;
          return (t >= 0 && t < T) ? fmaf(sm.H[(tl + 4) * CH + c], sc, sh) : 0.f;
        };
        float st[2] = {0.f, 0.f};
#pragma unroll 4
        for (int i = 0; i < FR / 2; ++i) {
          const int tl = rh0 + i;
          const float x0 = hn(tl - dil), x1 = hn(tl), x2 = hn(tl + dil);
          const bool valid = t0 + tl < T;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            float x = wv[q][3];
            x = fmaf(wv[q][0], x0, x);
            x = fmaf(wv[q][1], x1, x);
            x = fmaf(wv[q][2], x2, x);
            const float v = valid ? prelu_f(x, a2) : 0.f;
            st[0] += v; st[1] += v * v;
            split_store(sm.Ahi, sm.Alo, tl * LDD + 2 * c + q, v);
          }
        }
        block_sums<2>(st, sm.red, sm.dred);  // barrier inside: d complete in LDS
      TPROBE(4);
      }
      // ---- P2: GN2 partial sums (awaited after the res_out main loop) ----
      const unsigned e2 = xc.ep + 1;
      {
        __syncthreads();
        if (wave == 0 && lane == 0) xc.store(xc.slot(g, e2), dd_as_f4(sm.dred[0], sm.dred[1]));
        xc.publish(wave, lane);
      }
      // ================= res_out 512->256 (model/model.py:136,144) with reg2 folded =================
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      {
        wave_gemm<NS2, LDD>(acc, sm.Ahi, sm.Alo, rsrc_of(wb + WF_W2H), rsrc_of(wb + WF_W2L), voff2, rh, rl, lane);
      TPROBE(5);
      }
      xc.wait(e2);
      __syncthreads();  // also: every wave is done reading d from LDS
      TPROBE(6);
      if (tid < 2) {
        double s = 0.0;
        s = sum_members_d(pr, xslot, G, e2, 2 * tid);
        sm.dred[8 + tid] = s;
      }
      __syncthreads();
      f32x16v& rv = acc;  // r = res_out output, in place
      {
        float fmu, frs;
        gn_moments(sm.dred[8], sm.dred[9], (double)HID * T, 1e-8f, fmu, frs);
        const float ws = pm[PB_WS2 + m], bias = pm[PB_B2 + m], fcm = fmu * pm[PB_FC2 + m];
        float rsum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tl = trow(r);
          rv[r] = fmaf(frs, fmaf(rv[r], ws, -fcm), bias);
          const bool valid = t0 + tl < T;
          if (valid) rsum += rv[r];
          if (tf) {  // this frame's sum over the wave's 32 channels (lane 31: half 0 rows, lane 63: half 1)
            const float cs = half_total(valid ? rv[r] : 0.f);
            if ((lane & 31) == 31) sm.cs[tl][wave] = cs;
          }
        }
        if (tf) {
          rsum += __shfl_xor(rsum, 32);
          if (hl == 0) sm.vec[m] = rsum;
        }
      }
      // ---- TF_Attention (model/model.py:182-208): P3 = channel sums over own frames + per-frame sums ----
      if (tf) {
        __syncthreads();
        if (tid < FR) {
          float s = 0.f;
#pragma unroll
          for (int sl = 0; sl < 8; ++sl) s += sm.cs[tid][sl];
          sm.mC[tid] = s;   // staging (own frame channel sums)
        }
        __syncthreads();
      TPROBE(7);
        const unsigned e = xc.ep + 1;
        if (wave == 0) {
          const int dst = xc.slot(g, e);
          xc.store(dst + 4 * lane, *reinterpret_cast<const float4*>(&sm.vec[4 * lane]));     // [0, 256)
          if (lane < FR / 4) xc.store(dst + CH + 4 * lane, *reinterpret_cast<const float4*>(&sm.mC[4 * lane]));
        }
        xc.publish(wave, lane);
        xc.wait(e);
        __syncthreads();
      TPROBE(8);
        const float* p = pm + PB_ATT;
        // a_f: mean over frames -> conv(d=1) -> conv(d=2) -> PReLU -> sigmoid (over the channel axis)
        if (tid < CH) {
          float s = 0.f;
          s = sum_members_f(pr, xslot, G, e, tid);
          sm.vec[tid + 4] = s / (float)T;
          if (tid < 4) { sm.vec[tid] = 0.f; sm.vec[CH + 4 + tid] = 0.f; sm.yf[tid] = 0.f; sm.yf[CH + 4 + tid] = 0.f; }
        } else if (tid < CH + FR + 8) {
          // a_t inputs: channel means of frames t0-4 .. t0+35 (zero outside [0, T))
          const int i = tid - CH, tl = i - 4, t = t0 + tl;
          float v = 0.f;
          if (t >= 0 && t < T) {
            const int mm = tl < 0 ? g - 1 : (tl >= FR ? g + 1 : g);
            const int tj = tl < 0 ? tl + FR : (tl >= FR ? tl - FR : tl);
            v = ld_wt1(pr, xc.slot(mm, e) + CH + tj) / (float)CH;
          }
          sm.mC[i] = v;   // index i <-> frame t0 - 4 + i
        }
        __syncthreads();
        if (tid < CH) {
          sm.yf[tid + 4] = p[11] + p[8] * sm.vec[tid + 3] + p[9] * sm.vec[tid + 4] + p[10] * sm.vec[tid + 5];
        } else if (tid < CH + FR + 8) {
          const int i = tid - CH, t = t0 - 4 + i;
          float v = 0.f;
          if (t >= 0 && t < T && i >= 1 && i < FR + 7) v = p[3] + p[0] * sm.mC[i - 1] + p[1] * sm.mC[i] + p[2] * sm.mC[i + 1];
          sm.yt[i] = v;
        }
        __syncthreads();
        if (tid < CH) {
          const float v = p[15] + p[12] * sm.yf[tid + 2] + p[13] * sm.yf[tid + 4] + p[14] * sm.yf[tid + 6];
          sm.af[tid] = sigmoid_f(prelu_f(v, p[17]));
        } else if (tid < CH + FR) {
          const int tl = tid - CH, k = tl + 4;
          const float v = p[7] + p[4] * sm.yt[k - 2] + p[5] * sm.yt[k] + p[6] * sm.yt[k + 2];
          sm.at[tl] = sigmoid_f(prelu_f(v, p[16]));
        }
        __syncthreads();
      }
      TPROBE(9);
      // ---- residual update (model/model.py:345-352) ----
      const float afm = tf ? sm.af[m] : 1.f;
      if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL) {
        // moment record of u = o + r' (r' = r a_f a_t), see device_common.h recursive_affine
        const float ga = LM == LD_RECURSIVE ? pm[PB_LNAG + m] : 0.f, be = LM == LD_RECURSIVE ? pm[PB_LNAB + m] : 0.f;
        float mo[NMOM];
#pragma unroll
        for (int j = 0; j < NMOM; ++j) mo[j] = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tl = trow(r);
          const float vm = (t0 + tl < T) ? 1.f : 0.f;  // masked, not branched
          const float rp = vm * (tf ? rv[r] * (afm * sm.at[tl]) : rv[r]);
          if constexpr (LM == LD_RECURSIVE) {
            const float ov = vm * o[r], uv = ov + rp;
            mo[0] += ov; mo[1] += ov * ov; mo[2] += uv; mo[3] += uv * uv; mo[4] += be * ov; mo[5] += ga * uv;
            mo[6] += ga * ov * uv; mo[7] += ga * ov; mo[8] += ga * be * uv; mo[9] += ga * ga * uv * uv; mo[10] += ga * ga * uv;
          } else {
            mo[2] += rp; mo[3] += rp * rp;
          }
        }
        block_sums<NMOM>(mo, sm.red, sm.dred);
      TPROBE(10);
        // ---- P4 ----
        const unsigned e = xc.ep + 1;
        __syncthreads();
        if (wave == 0 && lane < 6) {
          const double d0 = sm.dred[2 * lane], d1 = 2 * lane + 1 < NMOM ? sm.dred[2 * lane + 1] : 0.0;
          xc.store(xc.slot(g, e) + 4 * lane, dd_as_f4(d0, d1));
        }
        xc.publish(wave, lane);
        xc.wait(e);
        __syncthreads();
      TPROBE(11);
        LoadSpec ld{};
        ld.gn.eps = 1e-5f; ld.eps2 = 1e-5f;
#pragma unroll
        for (int j = 0; j < 5; ++j) ld.wsum[j] = reinterpret_cast<const double*>(pm + PB_WSUM)[j];
        float pga[2], pba[2], pgb[2], pbb[2];
        ld_chan(pm + PB_LNAG, CH, pga); ld_chan(pm + PB_LNAB, CH, pba);
        if constexpr (LM == LD_RECURSIVE) { ld_chan(pm + PB_LNBG, CH, pgb); ld_chan(pm + PB_LNBB, CH, pbb); }
        if (tid < NMOM) {
          double s = 0.0;
          s = sum_members_d(pr, xslot, G, e, 2 * tid);
          sm.dred[tid] = s;
        }
        __syncthreads();
        if constexpr (LM == LD_RECURSIVE) {
          recursive_affine(sm.dred, ld, CH, T, pga, pba, pgb, pbb, sm.c[0], sm.c[1], sm.c[2], sm.c[3]);
        } else {
          gn_affine(sm.dred + 2, CH, T, 1e-5f, pga, pba, sm.c[0], sm.c[1]);
        }
        __syncthreads();
      }
      // next block's conv1d weights: in flight during the x' update
      if (bi + 1 < a.nblk) {
        const __half* wn = wb + WF_BLOCK;
        prefetch_w(rsrc_of(wn), rsrc_of(wn + WF_W1L), voff1, rh, rl);
      }
      // x' = next block input: o (registers) and the conv1d A operand (LDS)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tl = trow(r);
        const float gte = tf ? afm * sm.at[tl] : 1.f;
        const float x = resid_apply<LM>(o[r], rv[r], gte, m, sm.c[0], sm.c[1], sm.c[2], sm.c[3]);
        o[r] = (t0 + tl < T) ? x : 0.f;
        split_store(sm.Ahi, sm.Alo, tl * LDX + m, o[r]);
      }
      __syncthreads();
      TPROBE(12);
    }
    // ---- TCN output x' (head input) and the statistics of PReLU(x') for TCN.output.1 ----
    {
      float st[2] = {0.f, 0.f};
      float* Xu = a.Xfin + ((size_t)u * Tp + t0) * CH;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = t0 + trow(r);
        if (t < Tp) Xu[trow(r) * CH + m] = o[r];
        if (t < T) {
          const float pv = prelu_f(o[r], a.alpha_h);
          st[0] += pv; st[1] += pv * pv;
        }
      }
      block_sums<2>(st, sm.red, a.rec_head + ((size_t)u * G + g) * 2);
      __syncthreads();
    }
  }
}

hipError_t launch_tcn(const TcnArgs& a, int grid, hipStream_t s) {
  if (a.G < 1 || a.G > FG_MAX || a.G * FR < a.T || grid < a.G || grid % a.G) return hipErrorInvalidValue;
  switch (a.ln_mode) {
    case LD_RECURSIVE: hipLaunchKernelGGL(k_tcn<LD_RECURSIVE>, dim3(grid), dim3(NTHR), 0, s, a); break;
    case LD_RESIDUAL: hipLaunchKernelGGL(k_tcn<LD_RESIDUAL>, dim3(grid), dim3(NTHR), 0, s, a); break;
    case LD_ADD: hipLaunchKernelGGL(k_tcn<LD_ADD>, dim3(grid), dim3(NTHR), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int tcn_blocks_per_cu(int ln_mode) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
  switch (ln_mode) {
    case LD_RECURSIVE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn<LD_RECURSIVE>, NTHR, 0); break;
    case LD_RESIDUAL: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn<LD_RESIDUAL>, NTHR, 0); break;
    case LD_ADD: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn<LD_ADD>, NTHR, 0); break;
  }
  return e == hipSuccess ? nb : 0;
}

}  // namespace sepvad
