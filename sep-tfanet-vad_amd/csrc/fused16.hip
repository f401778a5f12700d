// k_tcn16: the whole TCN separator (24 x [DepthConv1d + TF_Attention + recursive/residual LN], reference
// model/model.py:103-149,182-208,271-357) as ONE persistent launch on 16-frame slices, TWO workgroups per CU.
//
// Why a second decomposition (DESIGN.md §4a "Round 4"): k_tcn (fused.hip) gives every CU one 32-frame slice and runs
// each block as one latency chain -- GEMM phases, elementwise phases and four cross-workgroup hand-offs strictly one
// after another, so the MFMA pipe idles through the hand-off waits and the VALU phases. Here a member owns 16 frames
// (G = ceil(T/16) members per utterance) and a workgroup is 4 waves with ~72 KB of LDS, so two independent members
// (two chains) share every CU: one's hand-off waits and elementwise phases overlap the other's GEMMs. At cfg 2
// (B = 64, T = 126) that is 512 members = two per CU, where k_tcn had one slice per CU and nothing to overlap.
//
// Work split inside a member: wave w owns output channels [64w, 64w+64) of both 1x1 convs as four 16-channel tiles of
// v_mfma_f32_16x16x32 (A = 16 frames x 32 K from LDS, B = 32 K x 16 channels streamed from L2 in fragment order);
// lane l holds frames 4(l>>4)..+3 of channels 64w + 16j + (l&15), j = 0..3, so the residual stream o is 16 registers.
// Everything else follows k_tcn: hand-offs P1 (GN1 sums + dil boundary rows), P2 (GN2 sums, polled inside the P3
// round), P3 (TF-attention row / column sums, raw accumulator, GN2 fold applied to the exchanged sums), P4 (the
// recursive-LN moment record); {tag, value} 8-byte words ("data is its own flag"), bounded polls, give-up reporting,
// fixed-order double statistics, the same slot layout (fused.hip GW_*: P3 clear of P1, P4 clear of P2).
//
// Arithmetic is k_tcn's (fp16x3 split with the int8 / e4m3 / fp16 weight lo plane, or single fp16 / bf16 products;
// fp32 accumulation; the GroupNorm finish in float from double sums); partial sums group differently (16-frame
// members, 4 channels per thread), so results equal k_tcn's to fp32 rounding, not bit for bit. Groups up to GMAX = 32
// members (T <= 512, 8.2 s at 16 kHz); longer utterances run k_tcn.
#include <type_traits>

#include "tcn_common.h"

namespace sepvad {
namespace t16 {

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int F = FR16;            // frames per member
constexpr int LDX = CH + 8;        // x' row stride (halves): 132 dwords == 4 (mod 64): conflict-free 16-row b128 reads
constexpr int LDD = HID + 8;       // d row stride (halves): 260 dwords == 4 (mod 64)
constexpr int HR = F + 8;          // conv1d output rows incl. 4 halo rows on each side
constexpr int NS1 = CH / 32;       // conv1d K steps of 32
constexpr int NS2 = HID / 32;      // res_out K steps of 32
constexpr int GMAX = FG16_MAX;     // members per group
// Workgroup geometry by wave count NWV (4 or 8): wave w owns output channels [CPW w, CPW w + CPW) as TPW tiles of 16
template <int NWV>
struct Geo {
  static constexpr int NW = NWV, NT = 64 * NWV;
  static constexpr int TPW = 16 / NWV;      // 16-channel tiles per wave
  static constexpr int CPW = 16 * TPW;      // channels per wave
  static constexpr int VPT = 4 * TPW;       // residual values per thread (4 frames x TPW channels)
  static constexpr int KH = 2048 / NT;      // P1 halo words per thread (2 x dil x 256 <= 2048)
  static constexpr int FPT = F * (CH / 2) / NT;  // depthwise frames per thread (input-channel pairs x frame slices)
  static constexpr int PCH = NWV == 4 ? 16 : 8;  // members' P3 row sums polled per pass
  static constexpr int WPE = NWV / 2;       // waves per SIMD at two workgroups per CU (launch bound)
};
// parameter blob staged in LDS: floats [0, PB_WD) (conv1d epilogue, GN1 affine) and [PB_WS2, PB_SIZE) (res_out
// epilogue, LN affines, attention taps, scalars); the depthwise weights (PB_WD .. PB_WS2) are read from global
constexpr int PS1 = PB_WD, PS2 = PB_SIZE - PB_WS2, PSTAGE = PS1 + PS2;
static_assert(PS1 % 4 == 0 && PS2 % 4 == 0 && (PB_WS2 - PS1) % 4 == 0, "float4 staging of the parameter blob");
static_assert((PB_WSUM - (PB_WS2 - PS1)) % 2 == 0, "8-byte alignment of the staged recursive-LN weight sums");

#ifndef TCN16_RD
#define TCN16_RD 2   // weight K steps (of 32) in flight per wave (4: 256 VGPRs + 6 spilled)
#endif

template <int NWV>
struct Smem {
  static constexpr int NW = NWV;
  _Float16 Ahi[F * LDD];           // GEMM A operand, hi plane: x' [16][LDX] or d [16][LDD]
  _Float16 Alo[F * LDD];           //                 lo plane
  float H[HR * CH];                // conv1d output (raw, pre-GN1) rows -4..19; the attention vectors alias it
  float prm[PSTAGE];               // this block's staged parameters (P() below)
  float af[CH];                    // frequency gate a_f
  float mC[F + 8], yt[F + 8], at[F];
  float gmom[4];                   // GN1 {mean, rstd}, GN2 {mean, rstd}
  float cs[F][NW];                 // per-frame channel partial sums per wave
  float csum[F];
  float red[NMOM * NW];
  unsigned gw[2 * NMOM * GMAX] __attribute__((aligned(8)));  // gathered statistic words of all members
  double dred[16];
};
static_assert(offsetof(Smem<4>, H) % 16 == 0 && offsetof(Smem<4>, prm) % 16 == 0 && sizeof(Smem<4>) <= 80 * 1024 &&
              offsetof(Smem<8>, H) % 16 == 0 && offsetof(Smem<8>, prm) % 16 == 0 && sizeof(Smem<8>) <= 80 * 1024,
              "alignment; two workgroups per CU (160 KB LDS)");

// A staged parameter (blob index i, PB_*)
template <class S>
__device__ __forceinline__ const float* P(const S& sm, int i) { return sm.prm + (i < PS1 ? i : i - (PB_WS2 - PS1)); }

// Weight-blob geometry per operand format: per (wave, K step) one contiguous chunk of SB bytes: the wave's TPW hi
// tiles (1 KB each), then its lo plane (fp16: TPW tiles; e4m3 / int8: TPW / 2 tile pairs of 1 KB).
template <int PRE, int LQ, int NWV>
struct Lay {
  static constexpr int TPW = Geo<NWV>::TPW, NW = NWV;
  static constexpr bool X3 = PRE == PREC_F16X3, L8 = LQ != 0;
  static constexpr int NLO = X3 ? (L8 ? TPW / 2 : TPW) : 0;
  static constexpr int NLO1 = NLO > 0 ? NLO : 1;
  static constexpr int SB = 1024 * TPW + 1024 * NLO;            // bytes per (wave, step)
  static constexpr size_t W1 = 0, W2 = (size_t)NW * NS1 * SB;   // byte offsets of the two GEMMs in a block
  static constexpr size_t BLOCK = (size_t)NW * (NS1 + NS2) * SB;  // bytes per block (the same for 4 and 8 waves)
};

// ring entry i <- K step s (the TPW hi tiles + the lo plane of step s)
template <int PRE, int LQ, int NWV, int RD>
__device__ __forceinline__ void ring_load(__amdgpu_buffer_rsrc_t w, int voff, u32x4v (&rh)[RD][Geo<NWV>::TPW],
                                          u32x4v (&rl)[RD][Lay<PRE, LQ, NWV>::NLO1], int i, int s) {
  using L = Lay<PRE, LQ, NWV>;
#pragma unroll
  for (int j = 0; j < L::TPW; ++j) rh[i][j] = __builtin_amdgcn_raw_buffer_load_b128(w, voff, s * L::SB + 1024 * j, 0);
#pragma unroll
  for (int p = 0; p < L::NLO; ++p)
    rl[i][p] = __builtin_amdgcn_raw_buffer_load_b128(w, voff, s * L::SB + 1024 * L::TPW + 1024 * p, 0);
}

// acc[j] (16 frames x channels 16j.. of the wave) += A[16 x 32 NS] . W^T on v_mfma_f32_16x16x32; A from LDS (row
// stride LDA halves), the weight steps stream through a static register ring of RD steps (the first RD already in)
template <int NS, int LDA, int PRE, int LQ, int NWV, int RD>
__device__ __forceinline__ void wave_gemm(f32x4v (&acc)[Geo<NWV>::TPW], const _Float16* Ahi, const _Float16* Alo,
                                          __amdgpu_buffer_rsrc_t w, int voff, u32x4v (&rh)[RD][Geo<NWV>::TPW],
                                          u32x4v (&rl)[RD][Lay<PRE, LQ, NWV>::NLO1], int lane) {
  using L = Lay<PRE, LQ, NWV>;
  constexpr int TP = L::TPW;
  constexpr bool X3 = L::X3, L8 = L::L8;
  static_assert(NS % RD == 0 && NS >= RD, "K steps");
  const int aoff = (lane & 15) * LDA + 8 * (lane >> 4);
  f16x8 aH[2], aL[2];
  aH[0] = *reinterpret_cast<const f16x8*>(Ahi + aoff);
  aL[0] = aH[0];
  if constexpr (X3) aL[0] = *reinterpret_cast<const f16x8*>(Alo + aoff);
  aH[1] = aL[1] = aH[0];
  auto step = [&](int s, int i, bool pf) {
    const int cur = s & 1, nxt = cur ^ 1;
    if (s + 1 < NS) {
      aH[nxt] = *reinterpret_cast<const f16x8*>(Ahi + aoff + 32 * (s + 1));
      if constexpr (X3) aL[nxt] = *reinterpret_cast<const f16x8*>(Alo + aoff + 32 * (s + 1));
    }
    const f16x8 ah = aH[cur], al = aL[cur];
    if constexpr (X3) {
      f16x8 bh[TP], bl[TP];
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        bh[j] = __builtin_bit_cast(f16x8, rh[i][j]);
        if constexpr (L8) bl[j] = lo8_widen<LQ>(rl[i][j >> 1], j & 1);
        else bl[j] = __builtin_bit_cast(f16x8, rl[i][j]);
      }
      // four independent accumulators between dependent MFMAs
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[j], 0, 0, 0);
    } else if constexpr (PRE == PREC_F16) {
#pragma unroll
      for (int j = 0; j < TP; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, __builtin_bit_cast(f16x8, rh[i][j]), acc[j], 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < TP; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, rh[i][j]),
                                                         acc[j], 0, 0, 0);
    }
    if (pf) ring_load<PRE, LQ, NWV, RD>(w, voff, rh, rl, i, s + RD);
    // pipeline shape of a step: the next step's A reads (DS), this step's MFMAs, then the ring refill (VMEM)
    if (s + 1 < NS) __builtin_amdgcn_sched_group_barrier(0x100, X3 ? 2 : 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, X3 ? 3 * TP : TP, 0);
    if (pf) __builtin_amdgcn_sched_group_barrier(0x020, TP + L::NLO, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int s0 = 0; s0 < NS - RD; s0 += RD) {
#pragma unroll
    for (int i = 0; i < RD; ++i) step(s0 + i, i, true);
  }
#pragma unroll
  for (int i = 0; i < RD; ++i) step(NS - RD + i, i, false);
}

// Block sums of NV per-thread floats (4 waves): waves by DPP, the wave totals in double in wave order by thread
// j < NV into out[j] (LDS or global). One barrier; callers barrier again before reading an LDS `out`.
template <int NV, int NW>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* lds, double* out) {
  const int w = threadIdx.x >> 6;
  float t[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    t[j] = half_total(v[j]);
    t[j] += dpp_f<0x143>(t[j]);
  }
  if ((threadIdx.x & 63) == 63) {
#pragma unroll
    for (int j = 0; j < NV; ++j) lds[j * NW + w] = t[j];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i) s += lds[threadIdx.x * NW + i];
    out[threadIdx.x] = s;
  }
}

// sum over the 16 lanes of a DPP row: lane 15 of the row holds it (the first four steps of half_total)
__device__ __forceinline__ float row_total(float v) {
  v += dpp_f<0xb1>(v);
  v += dpp_f<0x4e>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  return v;
}

// diagnostics (SEPVAD_TCN_PROBE, its own instantiation): wall clock at 13 phase points of every block of the first
// utterance each workgroup processes, as k_tcn's TPROBE (tools/tcn_probe.py): wave 0 at probe[(blockIdx * nblk + bi)
// * 16 + k], every wave at probe[grid * nblk * 16 + ((blockIdx * nblk + bi) * 16 + k) * 8 + wave]
#define T16P(k)                                                                                      \
  do {                                                                                               \
    if (PROBE && a.probe != nullptr && (threadIdx.x & 63) == 0 && u == grp) {                        \
      const unsigned long long _t = wall_clock64();                                                  \
      const size_t _i = ((size_t)blockIdx.x * a.nblk + bi) * 16 + (k);                               \
      if (threadIdx.x == 0) a.probe[_i] = _t;                                                        \
      a.probe[(size_t)gridDim.x * a.nblk * 16 + _i * 8 + (threadIdx.x >> 6)] = _t;                   \
    }                                                                                                \
  } while (0)

template <int LM, int PRE, int NWV, bool DUMP = false, int LQ = 0, bool PROBE = false>
__global__ __launch_bounds__(64 * NWV, NWV / 2) void k_tcn16(TcnArgs a) {
  using GE = Geo<NWV>;
  using L = Lay<PRE, LQ, NWV>;
  constexpr int NT = GE::NT, NW = GE::NW, TPW = GE::TPW, CPW = GE::CPW, VPT = GE::VPT, KH = GE::KH, FPT = GE::FPT;
  constexpr int PCH = GE::PCH;
  constexpr int RD = TCN16_RD;
  static_assert(FPT % RD == 0 && (2 * TPW) % RD == 0, "ring entries spread over the rows of the phases before the GEMMs");
  constexpr int RS = FPT / RD;       // depthwise frames per res_out ring entry
  constexpr int RX = 2 * TPW / RD;   // x' row pairs per conv1d ring entry
  __shared__ __attribute__((aligned(16))) Smem<NWV> sm;
  const int tid = threadIdx.x;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = a.G;
  int grp, g;  // members of a group on one XCD when the grid is a multiple of 8 G (speed only)
  if (a.xmode >= 2 && gridDim.x % (8 * G) == 0) {  // diagnostics: consecutive workgroups of an XCD in different groups
    const int x = blockIdx.x & 7, idx = blockIdx.x >> 3, gpx = gridDim.x / (8 * G);  // groups per XCD
    grp = (idx % gpx) * 8 + x;
    g = idx / gpx;
  } else if (gridDim.x % (8 * G) == 0) {
    const int x = blockIdx.x & 7, idx = blockIdx.x >> 3;
    grp = (idx / G) * 8 + x;
    g = idx % G;
  } else {
    grp = blockIdx.x / G;
    g = blockIdx.x % G;
  }
  const int ngroups = gridDim.x / G;
  u64* const gbase = a.gran + (size_t)grp * G * 2 * NGR;
  auto slot = [&](int mm, unsigned e) -> u64* { return gbase + ((size_t)mm * 2 + (e & 1)) * NGR; };
  unsigned ep = 1;  // epochs published so far; epoch 1 = XCD ids
  if (a.force_err && blockIdx.x == 0 && threadIdx.x == 0) giveup(a);
  if (PROBE && a.probe != nullptr && threadIdx.x == 0) {  // entry wall clock; HW_ID and XCC_ID (which CU / XCD)
    a.probe[(size_t)blockIdx.x * a.nblk * 16 + 15] = wall_clock64();
    a.probe[((size_t)blockIdx.x * a.nblk + a.nblk - 1) * 16 + 13] = __builtin_amdgcn_s_getreg(63492);  // hwreg(HW_REG_HW_ID)
    a.probe[((size_t)blockIdx.x * a.nblk + a.nblk - 1) * 16 + 14] = __builtin_amdgcn_s_getreg(6164) & 0xfu;
  }
  if (a.clk != nullptr && threadIdx.x == 0) {  // diagnostics (SEPVAD_TCN_CLOCK)
    const unsigned long long rt = wall_clock64();
    __hip_atomic_fetch_max(a.clk, ~rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) { a.clk[2] = rt; a.clk[4] = __builtin_amdgcn_s_memtime(); }
  }
  if (!a.tf_att) {  // no TF-attention: unit gates
    if (tid < CH) sm.af[tid] = 1.f;
    if (tid < F) sm.at[tid] = 1.f;
  }
  bool l2 = false;
  const int T = a.T, Tp = a.Tp, t0 = g * F;
  const bool tf = a.tf_att != 0;
  const int voff = (tid & 63) * 16;  // this lane's 16 bytes of a 1 KB wave fragment

  for (int u = grp; u < a.B; u += ngroups) {
    float o[VPT];  // o[4j + i]: frame 4(l>>4) + i, channel CPW wave + 16 j + (l & 15)
    u32x4v rh[RD][TPW], rl[RD][L::NLO1];
    {
      const int tidu = fresh_tid(wave_s);
      const int f0 = 4 * ((tidu & 63) >> 4), ch = CPW * wave_s + (tidu & 15);
      float raw[VPT], pg[TPW], pb[TPW], sx0;
      {
        const KArgs ka = kargs();
        const __amdgpu_buffer_rsrc_t s0r = rsrc_of(ka->S0 + ((size_t)u * Tp + t0) * CH);
        const __amdgpu_buffer_rsrc_t gr = rsrc_of(ka->ln.g), ber = rsrc_of(ka->ln.be);
        const __amdgpu_buffer_rsrc_t w1 = rsrc_of(reinterpret_cast<const char*>(ka->wfrag) + L::W1 + (size_t)wave_s * NS1 * L::SB);
        const int vo = (f0 * CH + ch) * 4;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)  // rows < G * 16 <= Tp: in bounds (masked below)
            raw[4 * j + i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s0r, vo, (i * CH + 16 * j) * 4, 0));
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          pg[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, (ch + 16 * j) * 4, 0, 0));
          pb[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ber, (ch + 16 * j) * 4, 0, 0));
        }
        sx0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc_of(ka->prm), 0, PB_SX * 4, 0));
#pragma unroll
        for (int i = 0; i < RD; ++i) ring_load<PRE, LQ, NWV, RD>(w1, voff, rh, rl, i, i);  // block-0 conv1d weights
        __builtin_amdgcn_sched_barrier(0);
      }
      reduce_records(rec_src(a.ln, u, 2), rec_none(), sm.dred);
      if (u == grp) {  // epoch 1: the members' XCD ids (write-through); one XCD => L2-resident hand-offs
        const unsigned xcc = __builtin_amdgcn_s_getreg(6164) & 0xfu;  // hwreg(HW_REG_XCC_ID, 0, 4)
        if (tid == 0) gput(slot(g, 1), a.tag0 + 1, xcc, false);
        const u64* p[1] = {tid < G ? slot(tid, 1) : nullptr};
        unsigned v[1];
        gpoll<1>(p, a.tag0 + 1, v, a);
        if (tid < G) sm.gw[tid] = v[0];
        __syncthreads();
        bool same = a.xmode == 0 || a.xmode == 2;
        for (int mm = 0; mm < G; ++mm) same = same && sm.gw[mm] == sm.gw[0];
        l2 = same;
      }
      __syncthreads();  // LN record sums (sm.dred) complete
      // x'_0 = TCN.LN(S0) (model/model.py:333): into o and the conv1d A operand (scaled by 2^-e, PB_SX)
      float mu, rs;
      gn_moments(sm.dred[0], sm.dred[1], (double)CH * T, a.ln.eps, mu, rs);
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const float sc = rs * pg[j], sh = pb[j] - sc * mu;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[4 * j + i] = fmaf(raw[4 * j + i], sc, sh) * (t0 + f0 + i < T ? 1.f : 0.f);
#pragma unroll
        for (int i = 0; i < 4; i += 2)
          split_store_rows_pk<PRE>(sm.Ahi, sm.Alo, (f0 + i) * LDX + ch + 16 * j, LDX,
                                   f32x2{o[4 * j + i], o[4 * j + i + 1]} * sx0, (tidu & 1) != 0);
      }
      if (float* dp = DUMP ? kargs()->dump : nullptr) {  // parity probe: TCN.LN output (model/model.py:333)
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[((size_t)u * Tp + t0 + f0 + i) * CH + ch + 16 * j] = o[4 * j + i];
      }
      __syncthreads();
    }
    for (int bi = 0; bi < a.nblk; ++bi) {
      // opaque per-iteration thread coordinates (fused.hip: keeps hipcc from hoisting per-row addresses)
      const int tido = fresh_tid(wave_s);
      const int tid = tido, lane = tid & 63, f0 = 4 * (lane >> 4), ch = CPW * wave_s + (lane & 15);
      const bool odd = (lane & 1) != 0;
      auto fm = [&](int i) { return t0 + f0 + i < T ? 1.f : 0.f; };  // own frame f0 + i valid
      const char* wb = reinterpret_cast<const char*>(a.wfrag) + (size_t)bi * L::BLOCK;
      const int li = bi % a.layer;
      const int dil = li == 0 ? 1 : (li % 4 + 1);  // model/model.py:285-295 (as api.hip packs it)
      // this block's staged parameters: loads now, LDS stores after the conv1d GEMM
      constexpr int NPV = (PSTAGE / 4 + NT - 1) / NT;
      u32x4v pv[NPV];
      {
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(uni(a.prm + (size_t)bi * PB_SIZE)), (short)0, PB_SIZE * 4, 0x00020000);
#pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int q = tid + k * NT;  // float4 index of the staged blob (past its end: the buffer reads 0)
          pv[k] = __builtin_amdgcn_raw_buffer_load_b128(pr, (q < PS1 / 4 ? q : q + (PB_WS2 - PS1) / 4) * 16, 0, 0);
        }
      }
      const float* pgl = a.prm + (size_t)bi * PB_SIZE;
      float ws1[TPW], b1[TPW];
#pragma unroll
      for (int j = 0; j < TPW; ++j) { ws1[j] = pgl[PB_WS1 + ch + 16 * j]; b1[j] = pgl[PB_B1 + ch + 16 * j]; }
      const float a1 = unif(pgl[PB_A1]);
      const unsigned e1 = ++ep, tag1 = a.tag0 + e1;
      T16P(0);
      if (DUMP && bi > 0 && bi == kargs()->dump_blk) {  // parity probe (SEPVAD_TCN_DUMP_BLOCK): this block's input
        if (float* dp = kargs()->dump) {
#pragma unroll
          for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) dp[((size_t)u * Tp + t0 + f0 + i) * CH + ch + 16 * j] = o[4 * j + i];
        }
      }
      // ================= conv1d 256->256 (model/model.py:132) + PReLU =================
      f32x4v acc[TPW];
#pragma unroll
      for (int j = 0; j < TPW; ++j) acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
      wave_gemm<NS1, LDX, PRE, LQ, NWV, RD>(acc, sm.Ahi, sm.Alo, rsrc_of(wb + L::W1 + (size_t)wave_s * NS1 * L::SB), voff, rh,
                                            rl, lane);
      T16P(1);
      // depthwise parameters of this thread's input-channel pair (not staged): in flight through the epilogue and P1
      // (4 waves; with 8 the registers are short, and they are loaded after the P1 round)
      const int c2 = 2 * (tid & (CH / 2 - 1)), fr0 = (tid >> 7) * FPT;
      f32x2 wv[2][3], bv[2];
      if constexpr (NWV == 4) dw_params2(pgl, c2, wv, bv);
      {
#pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int q = tid + k * NT;
          if (q < PSTAGE / 4) reinterpret_cast<u32x4v*>(sm.prm)[q] = pv[k];
        }
        u64* s1 = slot(g, e1);
        f32x2 s0 = {0.f, 0.f}, q0 = {0.f, 0.f};
        const float a1m1 = a1 - 1.f;
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const int c = ch + 16 * j;
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const f32x2 z = __builtin_elementwise_fma(f32x2{acc[j][i], acc[j][i + 1]}, f32x2{ws1[j], ws1[j]}, f32x2{b1[j], b1[j]});
            const f32x2 v = prelu2(z, a1m1) * f32x2{fm(i), fm(i + 1)};
            sm.H[(f0 + i + 4) * CH + c] = v.x;
            sm.H[(f0 + i + 5) * CH + c] = v.y;
            s0 += v;
            q0 = __builtin_elementwise_fma(v, v, q0);
            if (f0 == 0) {  // top boundary rows 0..dil-1
              if (i < dil) gputf(s1 + GW_TOP + i * CH + c, tag1, v.x, l2);
              if (i + 1 < dil) gputf(s1 + GW_TOP + (i + 1) * CH + c, tag1, v.y, l2);
            } else if (f0 == F - 4) {  // bottom boundary rows F-dil..F-1
              if (4 - i <= dil) gputf(s1 + GW_BOT + (i - (4 - dil)) * CH + c, tag1, v.x, l2);
              if (3 - i <= dil) gputf(s1 + GW_BOT + (i + 1 - (4 - dil)) * CH + c, tag1, v.y, l2);
            }
          }
        }
        float st[2] = {s0.x + s0.y, q0.x + q0.y};
        block_sums<2, NW>(st, sm.red, sm.dred);  // barrier inside: H and the staged blob complete
        if (tid < 2) gputd(s1 + GW_STAT + 2 * tid, tag1, sm.dred[tid], l2);
        tcn_delay(g);  // diagnostics (SEPVAD_TCN_DELAY)
        T16P(2);
      }
      // ---- consume P1: neighbours' boundary rows -> H halo; every member's GN1 sums ----
      {
        const u64* p[KH + 1];
        unsigned v[KH + 1];
        int hrow[KH], hcol[KH];
#pragma unroll
        for (int k = 0; k < KH; ++k) {
          const int i = tid + k * NT;
          p[k] = nullptr;
          hrow[k] = -1; hcol[k] = 0;
          if (i < 2 * dil * CH) {
            const int j = i / CH, c = i % CH;
            hcol[k] = c;
            if (j < dil) {  // frames -dil..-1: predecessor's last dil rows
              hrow[k] = 4 - dil + j;
              if (g > 0) p[k] = slot(g - 1, e1) + GW_BOT + j * CH + c;
            } else {        // frames F..F+dil-1: successor's first dil rows
              hrow[k] = 4 + F + (j - dil);
              if (g + 1 < G) p[k] = slot(g + 1, e1) + GW_TOP + (j - dil) * CH + c;
            }
          }
        }
        const int sk = tid - (NT - 4 * G);  // last 4G threads: GN1 words of member sk/4
        p[KH] = sk >= 0 ? slot(sk >> 2, e1) + GW_STAT + (sk & 3) : nullptr;
        gpoll<KH + 1>(p, tag1, v, a);
        T16P(3);
#pragma unroll
        for (int k = 0; k < KH; ++k)
          if (hrow[k] >= 0) sm.H[hrow[k] * CH + hcol[k]] = p[k] != nullptr ? __builtin_bit_cast(float, v[k]) : 0.f;
        if (G <= FG_WAVE) {
          if (wave_s == NW - 1) {  // the GN1 pollers' wave: moments before the barrier
            float mu, rs;
            member_moments_w(v[KH], 64 - 4 * G, G, a.inv_ch, 1e-8f, mu, rs);
            if (lane == 0) { sm.gmom[0] = mu; sm.gmom[1] = rs; }
          }
        } else if (sk >= 0) {
          sm.gw[sk] = v[KH];
        }
        __syncthreads();  // halo rows and the GN1 moments / words in LDS
      }
      // ================= depthwise conv (model/model.py:134-135): d = PReLU(dconv(GN1(h))) =================
      {
        if constexpr (NWV != 4) dw_params2(pgl, c2, wv, bv);
        float mu, rs;
        if (G <= FG_WAVE) {
          mu = sm.gmom[0]; rs = sm.gmom[1];
        } else {
          const double2 s = member_sums2(sm.gw, G, lane);
          gn_moments_f(s.x, s.y, a.inv_ch, 1e-8f, mu, rs);
        }
        const __amdgpu_buffer_rsrc_t w2 = rsrc_of(wb + L::W2 + (size_t)wave_s * NS2 * L::SB);
        const f32x2 sc2 = *reinterpret_cast<const f32x2*>(P(sm, PB_G1 + c2)) * rs;
        const f32x2 sh2 = *reinterpret_cast<const f32x2*>(P(sm, PB_BE1 + c2)) - sc2 * mu;
        const float a2m1 = *P(sm, PB_A2) - 1.f;
        f32x2 s0 = {0.f, 0.f}, s1 = {0.f, 0.f};
        // thread = input channels c2, c2+1 (hidden 2c2..2c2+3) x frames fr0..fr0+FPT-1; rows fr0-D .. fr0+FPT-1+D once
        // into registers (GN1 applied, zero outside [0, T)); H holds rows -4..F+3, so every load is in bounds
        auto rows = [&](auto DC) {
          constexpr int D = decltype(DC)::value;
          const float* hb = lds_base(sm.H + (fr0 - D + 4) * CH + c2);
          f32x2 hv[FPT + 2 * D];
#pragma unroll
          for (int i = 0; i < FPT + 2 * D; ++i) {
            const int t = t0 + fr0 - D + i;
            const float vm = (t >= 0 && t < T) ? 1.f : 0.f;
            hv[i] = __builtin_elementwise_fma(*reinterpret_cast<const f32x2*>(hb + i * CH), sc2, sh2) * vm;
          }
#pragma unroll
          for (int i = 0; i < FPT; ++i) {
            if (i % RS == 0) ring_load<PRE, LQ, NWV, RD>(w2, voff, rh, rl, i / RS, i / RS);  // res_out ring entry i/RS
            const int tl = fr0 + i;
            const float vo = t0 + tl < T ? 1.f : 0.f;
            f32x2 y[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              f32x2 x = __builtin_elementwise_fma(wv[q][0], hv[i], bv[q]);
              x = __builtin_elementwise_fma(wv[q][1], hv[i + D], x);
              x = __builtin_elementwise_fma(wv[q][2], hv[i + 2 * D], x);
              y[q] = prelu2(x, a2m1) * vo;
              s0 += y[q];
              s1 = __builtin_elementwise_fma(y[q], y[q], s1);
            }
            store_d4<PRE>(sm.Ahi + tl * LDD + 2 * c2, sm.Alo + tl * LDD + 2 * c2, y[0], y[1]);
          }
        };
        switch (dil) {
          case 1: rows(std::integral_constant<int, 1>{}); break;
          case 2: rows(std::integral_constant<int, 2>{}); break;
          case 3: rows(std::integral_constant<int, 3>{}); break;
          default: rows(std::integral_constant<int, 4>{}); break;
        }
        float st[2] = {s0.x + s0.y, s1.x + s1.y};
        block_sums<2, NW>(st, sm.red, sm.dred);  // barrier inside: d complete in LDS
        T16P(4);
      }
      // ---- P2 words: GN2 partial sums (awaited inside the P3 round) ----
      const unsigned e2 = ++ep, tag2 = a.tag0 + e2;
      if (tid < 2) gputd(slot(g, e2) + GW_STAT + 2 * tid, tag2, sm.dred[tid], l2);
      // ================= res_out 512->256 (model/model.py:136,144) with reg2 folded =================
#pragma unroll
      for (int j = 0; j < TPW; ++j) acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
      wave_gemm<NS2, LDD, PRE, LQ, NWV, RD>(acc, sm.Ahi, sm.Alo, rsrc_of(wb + L::W2 + (size_t)wave_s * NS2 * L::SB), voff, rh,
                                            rl, lane);
      T16P(5);
      // GN2 {mean, rstd} of the group (polled words in a wave's lanes, or in LDS)
      auto gn2_moments = [&](float& fmu, float& frs) {
        if (G <= FG_WAVE) {
          fmu = sm.gmom[2]; frs = sm.gmom[3];
        } else {
          const double2 sums = member_sums2(sm.gw, G, lane);
          gn_moments_f(sums.x, sums.y, a.inv_hid, *P(sm, PB_EPS2), fmu, frs);  // eps rescaled with d
        }
      };
      float* const vec = sm.H;            // attention vectors in the (dead) conv1d output rows
      float* const yf = sm.H + CH + 8;
      const unsigned e3 = tf ? ++ep : 0u, tag3 = a.tag0 + e3;
      if (!tf) {  // no TF-attention sums to exchange: the P2 round alone
        const u64* p[1] = {tid < 4 * G ? slot(tid >> 2, e2) + GW_STAT + (tid & 3) : nullptr};
        unsigned v[1];
        gpoll<1>(p, tag2, v, a);
        if (G <= FG_WAVE) {
          if (wave_s == 0) {
            float mu, rs;
            member_moments_w(v[0], 0, G, a.inv_hid, *P(sm, PB_EPS2), mu, rs);
            if (lane == 0) { sm.gmom[2] = mu; sm.gmom[3] = rs; }
          }
        } else if (tid < 4 * G) {
          sm.gw[tid] = v[0];
        }
        __syncthreads();
        float fmu, frs;
        gn2_moments(fmu, frs);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const int c = ch + 16 * j;
          const float ws = *P(sm, PB_WS2 + c), bias = *P(sm, PB_B2 + c), fcm = fmu * *P(sm, PB_FC2 + c);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(frs, fmaf(acc[j][i], ws, -fcm), bias);
        }
      } else {
        // ---- TF_Attention (model/model.py:182-208): P2 + P3 in one hand-off round; the row / column sums are taken on
        // the raw res_out accumulator and the GN2 fold (an affine per channel) is applied to the exchanged sums ----
        {
          float csr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < TPW; ++j) {
            const int c = ch + 16 * j;
            const float ws = *P(sm, PB_WS2 + c);
            float rsum = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              rsum += fm(i) * acc[j][i];
              csr[i] = fmaf(ws, acc[j][i], csr[i]);
            }
            rsum += __shfl_xor(rsum, 16);
            rsum += __shfl_xor(rsum, 32);
            if (lane < 16) gputf(slot(g, e3) + GW_ROW + c, tag3, rsum, l2);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) csr[i] = row_total(csr[i]);  // ws-weighted sum over the wave's channels
          if ((lane & 15) == 15) {
#pragma unroll
            for (int i = 0; i < 4; ++i) sm.cs[f0 + i][wave_s] = csr[i];
          }
        }
        __syncthreads();  // cs complete; every wave done reading d from LDS
        T16P(6);
        if (tid < F) {  // P3 words: per-frame raw channel sums (a_t)
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) s += sm.cs[tid][w];
          sm.csum[tid] = s;
          gputf(slot(g, e3) + GW_COL + tid, tag3, s, l2);
        }
        tcn_delay(g);  // diagnostics (SEPVAD_TCN_DELAY)
        T16P(7);
        {
          const u64* pp[PCH + 2];
          unsigned v[PCH + 2], tg[PCH + 2];
          const int mi = tid < 8 ? (tid < 4 ? tid : F + tid) : -1;  // a_t input index (frame t0 - 4 + mi)
          const u64* pat = nullptr;
          if (mi >= 0) {
            const int tl = mi - 4, t = t0 + tl;
            if (t >= 0 && t < T) pat = tl < 0 ? slot(g - 1, e3) + GW_COL + tl + F : slot(g + 1, e3) + GW_COL + tl - F;
          }
          float s = 0.f, vat = 0.f;
          unsigned vq = 0u;
          for (int c0 = 0; c0 < G; c0 += PCH) {  // thread tid < CH = channel tid: every member's row sum, member order
#pragma unroll
            for (int mm = 0; mm < PCH; ++mm) {
              pp[mm] = (tid < CH && c0 + mm < G) ? slot(c0 + mm, e3) + GW_ROW + tid : nullptr;
              tg[mm] = tag3;
            }
            pp[PCH] = (c0 == 0 && tid < 4 * G) ? slot(tid >> 2, e2) + GW_STAT + (tid & 3) : nullptr;  // GN2 words
            tg[PCH] = tag2;
            pp[PCH + 1] = c0 == 0 ? pat : nullptr;
            tg[PCH + 1] = tag3;
            gpollt<PCH + 2>(pp, tg, v, a);
#pragma unroll
            for (int mm = 0; mm < PCH; ++mm)
              if (c0 + mm < G) s += __builtin_bit_cast(float, v[mm]);
            if (c0 == 0) { vq = v[PCH]; vat = __builtin_bit_cast(float, v[PCH + 1]); }
          }
          if (G <= FG_WAVE) {
            if (wave_s == 0) {
              float mu, rs;
              member_moments_w(vq, 0, G, a.inv_hid, *P(sm, PB_EPS2), mu, rs);
              if (lane == 0) { sm.gmom[2] = mu; sm.gmom[3] = rs; }
            }
          } else if (tid < 4 * G) {
            sm.gw[tid] = vq;
          }
          __syncthreads();  // csum, the GN2 moments / words complete
          float fmu, frs;
          gn2_moments(fmu, frs);
          const float Tf = (float)T, sfc = *P(sm, PB_SFC2), sb = *P(sm, PB_SB2);
          // a_f input: channel means of r over the utterance (GN2 fold applied to the sums); thread tid < CH = channel
          if (tid < CH)
            vec[tid + 4] = (frs * (*P(sm, PB_WS2 + tid) * s - Tf * fmu * *P(sm, PB_FC2 + tid)) + Tf * *P(sm, PB_B2 + tid)) / Tf;
          if (tid < 4) { vec[tid] = 0.f; vec[CH + 4 + tid] = 0.f; yf[tid] = 0.f; yf[CH + 4 + tid] = 0.f; }
          if (mi >= 0) sm.mC[mi] = pat != nullptr ? (frs * (vat - fmu * sfc) + sb) / (float)CH : 0.f;
          if (tid >= 8 && tid < 8 + F) {
            const int tl = tid - 8;
            sm.mC[tl + 4] = (t0 + tl < T) ? (frs * (sm.csum[tl] - fmu * sfc) + sb) / (float)CH : 0.f;
          }
#pragma unroll
          for (int j = 0; j < TPW; ++j) {
            const int c = ch + 16 * j;
            const float ws = *P(sm, PB_WS2 + c), bias = *P(sm, PB_B2 + c), fcm = fmu * *P(sm, PB_FC2 + c);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(frs, fmaf(acc[j][i], ws, -fcm), bias);
          }
        }
        __syncthreads();
        T16P(8);
        const float* p = P(sm, PB_ATT);
        // a_f: mean over frames -> conv(d=1) -> conv(d=2) -> PReLU -> sigmoid (channel axis);
        // a_t: mean over channels -> conv(d=1) -> conv(d=2) -> PReLU -> sigmoid (frame axis)
        if (tid < CH) yf[tid + 4] = p[11] + p[8] * vec[tid + 3] + p[9] * vec[tid + 4] + p[10] * vec[tid + 5];
        if (tid < F + 8) {
          const int i = tid, t = t0 - 4 + i;
          float v = 0.f;
          if (t >= 0 && t < T && i >= 1 && i < F + 7) v = p[3] + p[0] * sm.mC[i - 1] + p[1] * sm.mC[i] + p[2] * sm.mC[i + 1];
          sm.yt[i] = v;
        }
        __syncthreads();
        if (tid < CH) {
          const float v = p[15] + p[12] * yf[tid + 2] + p[13] * yf[tid + 4] + p[14] * yf[tid + 6];
          sm.af[tid] = sigmoid_f(prelu_f(v, p[17]));
        }
        if (tid < F) {
          const int k = tid + 4;
          const float v = p[7] + p[4] * sm.yt[k - 2] + p[5] * sm.yt[k] + p[6] * sm.yt[k + 2];
          sm.at[tid] = sigmoid_f(prelu_f(v, p[16]));
        }
        __syncthreads();
      }
      T16P(9);
      // ---- residual update (model/model.py:345-352): r' = r a_f a_t in place ----
      if (DUMP && bi == kargs()->dump_blk) {  // parity probe: DepthConv1d output (model/model.py:144), before the gates
        if (float* dp = kargs()->dump) {
#pragma unroll
          for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) dp[((size_t)(kargs()->B + u) * Tp + t0 + f0 + i) * CH + ch + 16 * j] = acc[j][i];
        }
      }
      {
        float at4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) at4[i] = sm.at[f0 + i];
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const float afm = sm.af[ch + 16 * j];
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[j][i] = acc[j][i] * (at4[i] * afm);
        }
      }
      if (DUMP && bi == kargs()->dump_blk) {  // parity probe: TF_Attention output (model/model.py:207)
        if (float* dp = kargs()->dump) {
#pragma unroll
          for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) dp[((size_t)(2 * kargs()->B + u) * Tp + t0 + f0 + i) * CH + ch + 16 * j] = acc[j][i];
        }
      }
      float kc[TPW][4];  // per channel j: GN_a scale, shift, GN_b scale, shift
#pragma unroll
      for (int j = 0; j < TPW; ++j) kc[j][0] = kc[j][1] = kc[j][2] = kc[j][3] = 0.f;
      if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL) {
        // moment record of u = o + r' (device_common.h recursive_affine): per channel five sums over the thread's
        // four frames, then the channel weights
        float mo[NMOM];
#pragma unroll
        for (int k = 0; k < NMOM; ++k) mo[k] = 0.f;
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const int c = ch + 16 * j;
          float so = 0.f, soo = 0.f, su = 0.f, suu = 0.f, sou = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float vm = fm(i);
            const float rp = vm * acc[j][i];
            if constexpr (LM == LD_RECURSIVE) {
              const float ov = vm * o[4 * j + i], uv = ov + rp;
              so += ov; soo = fmaf(ov, ov, soo); su += uv; suu = fmaf(uv, uv, suu); sou = fmaf(ov, uv, sou);
            } else {
              su += rp; suu = fmaf(rp, rp, suu);
            }
          }
          mo[2] += su; mo[3] += suu;
          if constexpr (LM == LD_RECURSIVE) {
            const float ga = *P(sm, PB_LNAG + c), be = *P(sm, PB_LNAB + c);
            mo[0] += so; mo[1] += soo; mo[4] = fmaf(be, so, mo[4]); mo[5] = fmaf(ga, su, mo[5]); mo[6] = fmaf(ga, sou, mo[6]);
            mo[7] = fmaf(ga, so, mo[7]); mo[8] = fmaf(ga * be, su, mo[8]); mo[9] = fmaf(ga * ga, suu, mo[9]);
            mo[10] = fmaf(ga * ga, su, mo[10]);
          }
        }
        block_sums<NMOM, NW>(mo, sm.red, sm.dred);
        T16P(10);
        // ---- P4 words: the moment record (11 doubles); consume every member's ----
        const unsigned e4 = ++ep, tag4 = a.tag0 + e4;
        if (tid < NMOM) gputd(slot(g, e4) + GW_P4 + 2 * tid, tag4, sm.dred[tid], l2);
        {
          constexpr int NPW = (2 * NMOM * GMAX + NT - 1) / NT;  // words per thread
          const int nw = 2 * NMOM * G;
          const u64* pp[NPW];
          unsigned v[NPW];
#pragma unroll
          for (int j = 0; j < NPW; ++j) {
            const int k = tid + j * NT;
            pp[j] = k < nw ? slot(k / (2 * NMOM), e4) + GW_P4 + k % (2 * NMOM) : nullptr;
          }
          gpoll<NPW>(pp, tag4, v, a);
#pragma unroll
          for (int j = 0; j < NPW; ++j) {
            const int k = tid + j * NT;
            if (k < nw) sm.gw[k] = v[j];
          }
        }
        T16P(11);
        __syncthreads();  // every member's moment words in LDS
        // lane j < NMOM of every wave sums moment j over the members in member order; wave-uniform by readlane
        const double* gd = reinterpret_cast<const double*>(sm.gw);
        double sj = 0.0;
        {
          const int j = lane < NMOM ? lane : 0;
          for (int mm = 0; mm < G; ++mm) sj += gd[NMOM * mm + j];
        }
        double ms[NMOM];
#pragma unroll
        for (int j = 0; j < NMOM; ++j) ms[j] = readlane_d(sj, j);
        if constexpr (LM == LD_RECURSIVE) {
          float mua, rsa, mub, rsb;
          recursive_moments_f(ms, reinterpret_cast<const double*>(P(sm, PB_WSUM)), 1e-5f, 1e-5f, a.inv_ch, (double)T, mua,
                              rsa, mub, rsb);
#pragma unroll
          for (int j = 0; j < TPW; ++j) {
            const int c = ch + 16 * j;
            kc[j][0] = rsa * *P(sm, PB_LNAG + c); kc[j][1] = *P(sm, PB_LNAB + c) - kc[j][0] * mua;
            kc[j][2] = rsb * *P(sm, PB_LNBG + c); kc[j][3] = *P(sm, PB_LNBB + c) - kc[j][2] * mub;
          }
        } else {
          float mu, rs;
          gn_moments_f(ms[2], ms[3], a.inv_ch, 1e-5f, mu, rs);
#pragma unroll
          for (int j = 0; j < TPW; ++j) {
            const int c = ch + 16 * j;
            kc[j][0] = rs * *P(sm, PB_LNAG + c); kc[j][1] = *P(sm, PB_LNAB + c) - kc[j][0] * mu;
          }
        }
      }
      // x' = next block input: o (registers) and the conv1d A operand (LDS, scaled by the next block's 2^-e); the
      // next block's conv1d ring in flight meanwhile (the last block re-reads its own weights: in bounds)
      {
        const char* wn = bi + 1 < a.nblk ? wb + L::BLOCK : wb;
        const __amdgpu_buffer_rsrc_t w1n = rsrc_of(wn + L::W1 + (size_t)wave_s * NS1 * L::SB);
        const float sxn = *P(sm, PB_SXN);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const int r = 2 * j + i / 2;  // row-pair index 0..2 TPW - 1
            if (r % RX == 0) ring_load<PRE, LQ, NWV, RD>(w1n, voff, rh, rl, r / RX, r / RX);
            const f32x2 x = resid_apply2<LM>(f32x2{o[4 * j + i], o[4 * j + i + 1]}, f32x2{acc[j][i], acc[j][i + 1]}, kc[j]);
            const f32x2 ov = x * f32x2{fm(i), fm(i + 1)};
            o[4 * j + i] = ov.x; o[4 * j + i + 1] = ov.y;
            split_store_rows_pk<PRE>(sm.Ahi, sm.Alo, (f0 + i) * LDX + ch + 16 * j, LDX, ov * sxn, odd);
          }
        }
      }
      __syncthreads();
      T16P(12);
    }
    // ---- TCN output x' (head input) and the statistics of PReLU(x') for TCN.output.1 ----
    {
      const int tidt = fresh_tid(wave_s);
      const int f0 = 4 * ((tidt & 63) >> 4), ch = CPW * wave_s + (tidt & 15);
      float st[2] = {0.f, 0.f};
      float* Xu = a.Xfin + ((size_t)u * Tp + t0) * CH;
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = t0 + f0 + i;
          if (t < Tp) st_out(Xu + (f0 + i) * CH + ch + 16 * j, o[4 * j + i]);
          if (t < T) {
            const float pv = prelu_f(o[4 * j + i], a.alpha_h);
            st[0] += pv; st[1] += pv * pv;
          }
        }
      // k_head reads 32-frame slices: an odd group's last member also zeroes the 16 rows past its own (t >= T)
      if ((G & 1) && g == G - 1) {
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (t0 + F + f0 + i < Tp) st_out(Xu + (F + f0 + i) * CH + ch + 16 * j, 0.f);
      }
      block_sums<2, NW>(st, sm.red, a.rec_head + ((size_t)u * G + g) * 2);
      __syncthreads();
    }
  }
  if (unsigned long long* const ck = kargs()->clk; ck != nullptr && threadIdx.x == 0) {
    const unsigned long long rt = wall_clock64();
    if (blockIdx.x == 0) { ck[3] = rt; ck[5] = __builtin_amdgcn_s_memtime(); }
    __hip_atomic_fetch_max(ck + 1, rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// diagnostics (SEPVAD_TCN16_DYNLDS = bytes): unused dynamic LDS per workgroup, so fewer workgroups fit a CU (the
// capacity follows: hipOccupancy sees the same size)
inline size_t dyn_lds() {
  const char* v = getenv("SEPVAD_TCN16_DYNLDS");
  return v ? (size_t)atol(v) : 0;
}

template <int PRE, int LQ, int NWV>
hipError_t launch_pre(const TcnArgs& a, int grid, hipStream_t s) {
  const dim3 blk(64 * NWV);
  if (a.probe != nullptr && a.ln_mode == LD_RECURSIVE) {  // phase-stamp instantiation (SEPVAD_TCN_PROBE)
    hipLaunchKernelGGL((k_tcn16<LD_RECURSIVE, PRE, NWV, false, LQ, true>), dim3(grid), blk, dyn_lds(), s, a);
    return hipGetLastError();
  }
  if (a.dump != nullptr) {  // parity-probe instantiation
    switch (a.ln_mode) {
      case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn16<LD_RECURSIVE, PRE, NWV, true, LQ>), dim3(grid), blk, dyn_lds(), s, a); break;
      case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn16<LD_RESIDUAL, PRE, NWV, true, LQ>), dim3(grid), blk, dyn_lds(), s, a); break;
      case LD_ADD: hipLaunchKernelGGL((k_tcn16<LD_ADD, PRE, NWV, true, LQ>), dim3(grid), blk, dyn_lds(), s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (a.ln_mode) {
    case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn16<LD_RECURSIVE, PRE, NWV, false, LQ>), dim3(grid), blk, dyn_lds(), s, a); break;
    case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn16<LD_RESIDUAL, PRE, NWV, false, LQ>), dim3(grid), blk, dyn_lds(), s, a); break;
    case LD_ADD: hipLaunchKernelGGL((k_tcn16<LD_ADD, PRE, NWV, false, LQ>), dim3(grid), blk, dyn_lds(), s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int PRE, int LQ, int NWV>
int blocks_pre(int ln_mode) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
  const int nt = 64 * NWV;
  switch (ln_mode) {
    case LD_RECURSIVE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn16<LD_RECURSIVE, PRE, NWV, false, LQ>, nt, dyn_lds()); break;
    case LD_RESIDUAL: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn16<LD_RESIDUAL, PRE, NWV, false, LQ>, nt, dyn_lds()); break;
    case LD_ADD: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn16<LD_ADD, PRE, NWV, false, LQ>, nt, dyn_lds()); break;
  }
  return e == hipSuccess ? nb : 0;
}

template <int NWV>
hipError_t launch_w(const TcnArgs& a, int grid, hipStream_t s) {
  switch (a.prec) {
    case PREC_F16X3:
      switch (a.lo8) {
        case 0: return launch_pre<PREC_F16X3, 0, NWV>(a, grid, s);
        case 1: return launch_pre<PREC_F16X3, 1, NWV>(a, grid, s);
        case 2: return launch_pre<PREC_F16X3, 2, NWV>(a, grid, s);
      }
      return hipErrorInvalidValue;
    case PREC_F16: return launch_pre<PREC_F16, 0, NWV>(a, grid, s);
    case PREC_BF16: return launch_pre<PREC_BF16, 0, NWV>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

template <int NWV>
int blocks_w(int ln_mode, int prec, int lo) {
  switch (prec) {
    case PREC_F16X3:
      return lo == 1 ? blocks_pre<PREC_F16X3, 1, NWV>(ln_mode)
                     : (lo == 2 ? blocks_pre<PREC_F16X3, 2, NWV>(ln_mode) : blocks_pre<PREC_F16X3, 0, NWV>(ln_mode));
    case PREC_F16: return blocks_pre<PREC_F16, 0, NWV>(ln_mode);
    case PREC_BF16: return blocks_pre<PREC_BF16, 0, NWV>(ln_mode);
  }
  return 0;
}

}  // namespace t16

size_t tcn16_block_bytes(int prec, int lo) {
  // the same for 4 and 8 waves (every wave's chunks together are the block's weights)
  switch (prec) {
    case PREC_F16X3: return lo == 0 ? t16::Lay<PREC_F16X3, 0, 8>::BLOCK : t16::Lay<PREC_F16X3, 2, 8>::BLOCK;
    case PREC_F16: case PREC_BF16: return t16::Lay<PREC_F16, 0, 8>::BLOCK;
  }
  return 0;
}

hipError_t launch_tcn16(const TcnArgs& a, int grid, int nwaves, hipStream_t s) {
  if (a.G < 1 || a.G > FG16_MAX || a.G * FR16 < a.T || a.G * FR16 > a.Tp || grid < a.G || grid % a.G)
    return hipErrorInvalidValue;
  if (nwaves == 4) return t16::launch_w<4>(a, grid, s);
  if (nwaves == 8) return t16::launch_w<8>(a, grid, s);
  return hipErrorInvalidValue;
}

int tcn16_blocks_per_cu(int ln_mode, int prec, int lo, int nwaves) {
  return nwaves == 4 ? t16::blocks_w<4>(ln_mode, prec, lo) : (nwaves == 8 ? t16::blocks_w<8>(ln_mode, prec, lo) : 0);
}

}  // namespace sepvad
