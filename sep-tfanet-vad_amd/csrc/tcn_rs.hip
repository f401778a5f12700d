// k_tcn_rs: the whole TCN separator (24 x [DepthConv1d + TF_Attention + recursive/residual LN], reference
// model/model.py:103-149,182-208,271-357) as ONE persistent launch with ROLE-SPECIALISED waves.
//
// Same decomposition as k_tcn (fused.hip): an utterance of T frames is owned by a group of G = ceil(T/32)
// workgroups, member g owns frames [32g, 32g+32) and all 256 channels, the group exchanges GroupNorm / TF-attention
// statistics and the depthwise-conv halo rows through tagged 8-byte hand-off words. What differs is the division of
// labour inside the 512-thread workgroup: one wave of each role per SIMD,
//   M waves 0-3 (matrix): both 1x1-conv GEMMs, two 32x32 output tiles per wave (64 channels: each 1 KB weight
//       fragment is loaded once per CU and feeds two MFMA tiles through one A fragment), the GEMM epilogues, the
//       moment record and the residual update; they own the residual stream o in registers and issue the weight
//       stream (register ring) during the phases the V waves run;
//   V waves 4-7 (vector): the depthwise conv + PReLU + GroupNorm statistics, every hand-off poll, the TF-attention
//       gates and the GroupNorm/recursive-LN moments.
// The depthwise conv is produced in four channel chunks that the M waves consume as soon as each is in LDS (LDS
// flags): the res_out GEMM's MFMAs run beside the depthwise conv's VALU on the same SIMDs (separate pipes) instead
// of after it; polls are issued by waves that have no weight loads in flight (vmcnt retires in order); statistics
// are published by the last-arriving wave of a role (LDS counter) instead of behind a workgroup barrier; the
// GroupNorm(reg2) statistics and the TF-attention sums travel in ONE hand-off round (the sums are taken on the raw
// res_out accumulator and the GN2 fold is applied after the exchange: linearity). Four workgroup barriers per block.
//
// Arithmetic as k_tcn: fp16x3 split (acc += A_lo B_hi + A_hi B_lo + A_hi B_hi on v_mfma_f32_32x32x16_f16) or the
// single-plane fp16 / bf16 arms; GroupNorm statistics float per wave, double across waves and members in fixed
// order (bitwise reproducible, independent of placement and batch composition).
#include <type_traits>

#include "tcn_common.h"

namespace sepvad {
namespace {

constexpr int RS_NTHR = 512;
constexpr int RS_LDX = CH + 8;     // x' row stride (halves): 132 dwords == 4 (mod 64)
constexpr int RS_LDD = HID + 8;    // d row stride (halves): 260 dwords == 4 (mod 64)
constexpr int RS_HS = CH + 2;      // H row stride (floats): rows 8 apart land 16 banks apart (depthwise reads)
constexpr int RS_HROWS = FR + 8;   // H rows -4..35
#ifndef RS_NOG2
#define RS_NOG2 0                  // diagnostics: no res_out GEMM (wrong results; phase timing of the depthwise conv)
#endif
#ifndef RS_VPRIO
#define RS_VPRIO 0                 // A/B: V waves at s_setprio 1
#endif
#ifndef RS_G2NOMFMA
#define RS_G2NOMFMA 0              // diagnostics: res_out GEMM loads and waits without its MFMAs (wrong results)
#endif
#ifndef RS_G2NOLDS
#define RS_G2NOLDS 0               // diagnostics: res_out GEMM without its A fragment reads (wrong results)
#endif
#ifndef RS_DW_SCALAR
#define RS_DW_SCALAR 0             // A/B: the scalar depthwise conv
#endif
#ifndef RS_PD
#define RS_PD 8                    // weight K steps in flight per M wave (two tiles, hi/lo: 16 KB per CU per step)
#endif
constexpr int PD = RS_PD;
constexpr int NS1 = CH / 16;       // conv1d K steps
constexpr int NS2 = HID / 16;      // res_out K steps
constexpr int NCH = 4;             // depthwise chunks: V wave v, chunk j -> h channels 64v + 16j .. +15 (K steps 8v+2j, +1)
// hand-off word regions of one member slot (block parity p): slot = gbase + (member * 2 + p) * NGR
constexpr int Q_GN1 = 0;                 // GN1 {sum lo, hi, sumsq lo, hi}
constexpr int Q_TOP = 4;                 // conv1d output rows 0..dil-1        [dil][256]
constexpr int Q_BOT = 4 + 4 * CH;        // conv1d output rows 32-dil..31     [dil][256]
constexpr int Q_GN2 = 4 + 8 * CH;        // GN2 {sum lo, hi, sumsq lo, hi}
constexpr int Q_ROW = Q_GN2 + 4;         // raw res_out sums over own frames per channel [256]
constexpr int Q_COL = Q_ROW + CH;        // raw ws-weighted res_out sums over channels per frame [32]
constexpr int Q_MOM = Q_COL + FR;        // moment record, 11 doubles
constexpr int Q_XCD = Q_MOM + 2 * NMOM;  // XCD id (epoch 1)
static_assert(Q_XCD + 1 <= NGR, "hand-off slot size");

// physical LDS row of frame t in the GEMM A planes: rows 8 apart (one per depthwise frame group) are 16 banks apart
// for the depthwise conv's 32-bit stores, and every 16-lane group of the GEMM's b128 fragment reads still covers
// distinct bank quads
__device__ __forceinline__ int prow(int t) { return t ^ ((t & 8) >> 1); }

struct RsSmem {
  _Float16 Ahi[FR * RS_LDD];      // GEMM A operand, hi plane: x' [32][RS_LDX] or d [32][RS_LDD] (rows prow(t))
  _Float16 Alo[FR * RS_LDD];      //                 lo plane
  float H[RS_HROWS * RS_HS];      // conv1d output (raw, pre-GN1), rows -4..35 (halo rows from the neighbours)
  float prm[2][PB_SIZE];          // block parameter blobs, double-buffered (block bc in [bc & 1])
  float af[CH];                   // frequency gate a_f
  float at[FR];                   // time gate a_t
  float vecw[4][72];              // per V wave: channel means with a 3-channel halo (a_f taps)
  float yfw[4][72];
  float mC[FR + 8], yt[FR + 8];   // frame means with a 4-frame halo (a_t taps)
  float csp[FR][4];               // per M wave: raw per-frame channel sums
  float red1[4][2];               // per M wave: GN1 partial sums
  float vred[4][2];               // per V wave: GN2 partial sums
  float red4[4][12];              // per M wave: moment-record partial sums
  unsigned gw[FG_MAX * 2 * NMOM] __attribute__((aligned(8)));  // polled moment-record words (V wave 0)
  double dred[2];                 // TCN.LN record sums
  float scal[8];                  // 0,1: GN2 fold {mu, rstd}; 2..5: recursive/residual LN {mua, rsa, mub, rsb}
  unsigned flag[4] __attribute__((aligned(16)));  // per V wave: last depthwise chunk in LDS (monotonic id)
  unsigned cnt[4];                // last-arriver counters: 0 GN1 (M), 1 GN2 (V), 2 column sums (M), 3 moments (M)
  unsigned pflag[4] __attribute__((aligned(16)));  // per V wave: P1 polls done (block count + 1): the M waves then issue their ring
  unsigned l2;                    // hand-off stores stay in the XCD's L2 (whole group on one XCD)
};

template <int PRE>
struct RsLay {
  static constexpr size_t BLOCK = PRE == PREC_F16X3 ? WF_BLOCK : WS_BLOCK;
  static constexpr size_t W1L = PRE == PREC_F16X3 ? WF_W1L : 0;
  static constexpr size_t W2H = PRE == PREC_F16X3 ? WF_W2H : WS_W2, W2L = PRE == PREC_F16X3 ? WF_W2L : 0;
};

// res_out K step consumed i-th: chunk-major (the order the depthwise conv produces them)
__device__ __forceinline__ constexpr int ord2(int i) { return 8 * ((i % 8) / 2) + 2 * (i / 8) + (i % 2); }
__device__ __forceinline__ constexpr int ord1(int i) { return i; }

// Weight ring entry of consumed step i: the two tiles' fragments (hi, and lo for fp16x3)
template <int PRE, int NS, bool G2>
__device__ __forceinline__ void ring_load(__amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int vo0, int vo1,
                                          u32x4v (&rh)[PD][2], u32x4v (&rl)[PD][2], int i) {
  const int s = G2 ? ord2(i) : ord1(i);
  rh[i % PD][0] = __builtin_amdgcn_raw_buffer_load_b128(wh, vo0, s * 1024, 0);
  rh[i % PD][1] = __builtin_amdgcn_raw_buffer_load_b128(wh, vo1, s * 1024, 0);
  if constexpr (PRE == PREC_F16X3) {
    rl[i % PD][0] = __builtin_amdgcn_raw_buffer_load_b128(wl, vo0, s * 1024, 0);
    rl[i % PD][1] = __builtin_amdgcn_raw_buffer_load_b128(wl, vo1, s * 1024, 0);
  }
}

// One M wave's two tiles: c0/c1 [32 frames x 32 channels] += A[32 x 16 NS] W_q^T, the A fragment (LDS, physical
// rows prow) shared by both tiles, the weights from the register ring (first PD entries already issued). G2: the
// steps in ord2 order, each chunk of 8 awaited on the V waves' LDS flags (>= cid0 + chunk + 1).
template <int NS, int LDA, int PRE, bool G2>
__device__ __forceinline__ void mgemm(f32x16v& c0, f32x16v& c1, const _Float16* Ahi, const _Float16* Alo,
                                      __amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int vo0, int vo1,
                                      u32x4v (&rh)[PD][2], u32x4v (&rl)[PD][2], int lane, const unsigned* flag,
                                      unsigned cid0, const TcnArgs& a) {
  constexpr bool X3 = PRE == PREC_F16X3;
  const int aoff = prow(lane & 31) * LDA + 8 * (lane >> 5);
  auto wait_chunk = [&](int j) {
    if constexpr (G2) {
      const unsigned need = cid0 + (unsigned)j + 1u;
      unsigned spins = 0;
      for (;;) {
        const u32x4v f = *reinterpret_cast<const volatile u32x4v*>(flag);
        const unsigned m = min(min(f[0], f[1]), min(f[2], f[3]));
        if (m >= need) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > a.spin_limit) { giveup(a); break; }  // unreachable unless a V wave faulted: never hang
      }
    }
  };
  auto afrag = [&](int i, f16x8& h, f16x8& l) {
    const int s = G2 ? ord2(i) : ord1(i);
    h = *reinterpret_cast<const f16x8*>(Ahi + aoff + 16 * s);
    if constexpr (X3) l = *reinterpret_cast<const f16x8*>(Alo + aoff + 16 * s);
  };
  f16x8 ah, al = {};
  wait_chunk(0);
  afrag(0, ah, al);
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const bool chunk_edge = G2 && (i + 1) % 8 == 0 && i + 1 < NS;
    f16x8 nh = ah, nl = al;
    if (!(G2 && RS_G2NOLDS) && i + 1 < NS && !chunk_edge) afrag(i + 1, nh, nl);  // next step's A reads in flight
    const int e = i % PD;
    if constexpr (G2 && RS_G2NOMFMA) {  // diagnostics: the res_out step without its MFMAs
      asm volatile("" :: "v"(rh[e][0]), "v"(rh[e][1]), "v"(rl[e][0]), "v"(rl[e][1]), "v"(ah), "v"(al));
    } else if constexpr (X3) {
      const f16x8 b0h = __builtin_bit_cast(f16x8, rh[e][0]), b1h = __builtin_bit_cast(f16x8, rh[e][1]);
      const f16x8 b0l = __builtin_bit_cast(f16x8, rl[e][0]), b1l = __builtin_bit_cast(f16x8, rl[e][1]);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, b0h, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, b1h, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, b0l, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, b1l, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, b0h, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, b1h, c1, 0, 0, 0);
    } else if constexpr (PRE == PREC_F16) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, __builtin_bit_cast(f16x8, rh[e][0]), c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, __builtin_bit_cast(f16x8, rh[e][1]), c1, 0, 0, 0);
    } else {
      const bf16x8 a16 = __builtin_bit_cast(bf16x8, ah);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a16, __builtin_bit_cast(bf16x8, rh[e][0]), c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a16, __builtin_bit_cast(bf16x8, rh[e][1]), c1, 0, 0, 0);
    }
    if (i + PD < NS) ring_load<PRE, NS, G2>(wh, wl, vo0, vo1, rh, rl, i + PD);
    if (chunk_edge) {  // this step's MFMAs issued first, then the wait for the next chunk
      wait_chunk((i + 1) / 8);
      afrag(i + 1, nh, nl);
    }
    ah = nh; al = nl;
    __builtin_amdgcn_sched_barrier(0);  // program order per step (keeps the ring PD steps deep)
  }
}

// Sum of v over the 64 lanes in lane 63 (DPP row reductions + row_bcast:31; as wave_total without the readlane)
__device__ __forceinline__ float lane63_total(float v) {
  v = half_total(v);
  v += dpp_f<0x143>(v);
  return v;
}

// GroupNorm {mean, rstd} from the G members' statistic words {sum lo, hi, sumsq lo, hi}, polled one per lane: word k
// of 4G in lane k (w0) or lane k - 64 (w1); summed in member order (double), wave-uniform (readlane).
__device__ __forceinline__ void member_moments2(unsigned w0, unsigned w1, int G, double inv, float eps, float& mu,
                                                float& rs) {
  double s = 0.0, ss = 0.0;
  for (int mm = 0; mm < G; ++mm) {
    const int k = 4 * mm;
    unsigned a0, a1, b0, b1;
    if (k < 64) {
      a0 = __builtin_amdgcn_readlane(w0, k); a1 = __builtin_amdgcn_readlane(w0, k + 1);
      b0 = __builtin_amdgcn_readlane(w0, k + 2); b1 = __builtin_amdgcn_readlane(w0, k + 3);
    } else {
      a0 = __builtin_amdgcn_readlane(w1, k - 64); a1 = __builtin_amdgcn_readlane(w1, k - 63);
      b0 = __builtin_amdgcn_readlane(w1, k - 62); b1 = __builtin_amdgcn_readlane(w1, k - 61);
    }
    s += dword2(a0, a1);
    ss += dword2(b0, b1);
  }
  gn_moments_f(s, ss, inv, eps, mu, rs);
}

// This lane's id from v_mbcnt (volatile asm: never hoisted): every per-row address and mask derived from it inside a
// phase stays inside that phase; values derived once outside the block loop would stay live across it (hipcc hoists
// them, runs out of registers at 2 waves per SIMD and spills).
__device__ __forceinline__ int lane_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
#define MLANE                                                          \
  const int ln = lane_fresh();                                         \
  const int hl4 = 4 * (ln >> 5);                                       \
  auto trow = [hl4](int r) { return (r & 3) + 8 * (r >> 2) + hl4; };   \
  (void)trow
#define VOFF1A (((2 * mw) * NS1 * 64 + ln) * 16)
#define VOFF2A (((2 * mw) * NS2 * 64 + ln) * 16)

// diagnostics (SEPVAD_TCN_PROBE): lane 0 of every wave stamps the wall clock at phase point k of every block of the
// first utterance a workgroup processes: probe[((blockIdx * nblk + block) * 16 + k) * 8 + wave]
#define RPROBE(k)                                                                                          \
  do {                                                                                                     \
    if (a.probe != nullptr && lane == 0 && u == x.grp)                                                     \
      a.probe[(((size_t)blockIdx.x * a.nblk + bi) * 16 + (k)) * 8 + wave_s] = wall_clock64();             \
  } while (0)

// Per-workgroup constants, derived identically by both roles.
struct RsCtx {
  int G, grp, g, ngroups, T, Tp, t0;
  bool tf;
  u64* gbase;
  __device__ __forceinline__ u64* slot(int mm, int par) const { return gbase + ((size_t)mm * 2 + par) * NGR; }
};

// Tags of block bc's four hand-off rounds (the same epoch sequence in every member, both roles).
struct RsTags {
  unsigned t1, t2, t3, t4;
};
template <int LM>
__device__ __forceinline__ RsTags next_tags(unsigned& ep, bool tf, unsigned tag0) {
  RsTags t;
  t.t1 = tag0 + (++ep);                                   // P1: GN1 sums + halo rows
  t.t2 = tag0 + (++ep);                                   // P2: GN2 sums
  t.t3 = tf ? tag0 + (++ep) : tag0;                       // P3: raw row / column sums
  t.t4 = LM != LD_ADD ? tag0 + (++ep) : tag0;             // P4: moment record
  return t;
}

// ---------------------------------------------------------------------------------------------------------------
// M role (waves 0-3): residual stream, both GEMMs, their epilogues, the moment record, the x' update.
// Lane geometry: tiles q = 0, 1 -> channels 64 mw + 32 q + (lane & 31); accumulator row r -> frame trow(r).
// Workgroup barriers per utterance, in lockstep with v_role: 2 (prologue) + 4 per block + 2 (epilogue).
template <int LM, int PRE, bool DUMP>
__device__ __forceinline__ void m_role(const TcnArgs& a, RsSmem& sm, const RsCtx& x, int lane, int mw, int wave_s) {
  using WL = RsLay<PRE>;
  const int T = x.T, Tp = x.Tp, t0 = x.t0, g = x.g;
  float o[2][16];               // residual stream (both tiles)
  u32x4v rh[PD][2], rl[PD][2];  // weight ring
  f32x16v acc0, acc1;
  unsigned ep = 1, bc = 0;
  for (int u = x.grp; u < a.B; u += x.ngroups) {
    // ================= prologue: x'_0 = TCN.LN(S0) (model/model.py:333) =================
    float raw[2][16], pg[2], pb[2];
    {
      MLANE;
      const KArgs ka = kargs();
      const __amdgpu_buffer_rsrc_t s0r = rsrc_of(ka->S0 + ((size_t)u * Tp + t0) * CH);
      const __amdgpu_buffer_rsrc_t gr = rsrc_of(ka->ln.g), ber = rsrc_of(ka->ln.be);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = 64 * mw + 32 * q + (ln & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r)  // rows < G*32 <= Tp: in bounds (masked below)
          raw[q][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(s0r, (trow(r) * CH + c) * 4, 0, 0));
        pg[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, c * 4, 0, 0));
        pb[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ber, c * 4, 0, 0));
      }
      if (u == x.grp) {  // block-0 conv1d ring (later utterances: issued by the previous utterance's last block)
        const __amdgpu_buffer_rsrc_t w1h = rsrc_of(ka->wfrag), w1l = rsrc_of(ka->wfrag + WL::W1L);
#pragma unroll
        for (int i = 0; i < PD; ++i) ring_load<PRE, NS1, false>(w1h, w1l, VOFF1A, VOFF1A + NS1 * 1024, rh, rl, i);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (mw == 0 && lane < 2) {  // TCN.LN statistics: the k_stft_gate records of this utterance, record order
      const RecSrc rs = rec_src(a.ln, u, 2);
      double s = 0.0;
      for (int r = 0; r < rs.n; ++r) s += rs.p[(size_t)r * rs.rs + lane];
      sm.dred[lane] = s;
    }
    __syncthreads();  // (P1) LN sums, XCD check
    {
      MLANE;
      float mu, rs;
      gn_moments(sm.dred[0], sm.dred[1], (double)CH * T, a.ln.eps, mu, rs);
      const float sx0 = sm.prm[bc & 1][PB_SX];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = 64 * mw + 32 * q + (ln & 31);
        const float sc = rs * pg[q], sh = pb[q] - sc * mu;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tl = trow(r);
          o[q][r] = fmaf(raw[q][r], sc, sh) * (t0 + tl < T ? 1.f : 0.f);
          split_store<PRE>(sm.Ahi, sm.Alo, prow(tl) * RS_LDX + c, o[q][r] * sx0);  // x' * 2^-e (range guard)
        }
        if (float* dp = DUMP ? kargs()->dump : nullptr) {  // parity probe: TCN.LN output (model/model.py:333)
#pragma unroll
          for (int r = 0; r < 16; ++r) dp[((size_t)u * Tp + t0 + trow(r)) * CH + c] = o[q][r];
        }
      }
    }
    __syncthreads();  // (P2) x'_0 in LDS
    const bool l2 = sm.l2 != 0u;

    for (int bi = 0; bi < a.nblk; ++bi, ++bc) {
      const int par = bc & 1;
      const float* pm = sm.prm[par];
      const int li = bi % a.layer;
      const int dil = li == 0 ? 1 : (li % 4 + 1);  // model/model.py:285-295 (as api.hip packs it)
      const __half* wb = a.wfrag + (size_t)bi * WL::BLOCK;
      const RsTags tg = next_tags<LM>(ep, x.tf, a.tag0);
      u64* const own = x.slot(g, par);
      RPROBE(0);
      // ================= conv1d 256->256 (model/model.py:132) =================
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
      {
        MLANE;
        mgemm<NS1, RS_LDX, PRE, false>(acc0, acc1, sm.Ahi, sm.Alo, rsrc_of(wb), rsrc_of(wb + WL::W1L), VOFF1A,
                                       VOFF1A + NS1 * 1024, rh, rl, ln, sm.flag, 0u, a);
      }
      RPROBE(1);
      {  // epilogue: h = PReLU(W1 x' + b1) -> H (LDS), GN1 partial sums, boundary rows (P1)
        MLANE;
        const float a1 = pm[PB_A1];
        float st0 = 0.f, st1 = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int c = 64 * mw + 32 * q + (ln & 31);
          const float ws = pm[PB_WS1 + c], bias = pm[PB_B1 + c];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int tl = trow(r);
            float v = prelu_f(fmaf(q ? acc1[r] : acc0[r], ws, bias), a1);
            v = (t0 + tl < T) ? v : 0.f;
            sm.H[(tl + 4) * RS_HS + c] = v;
            st0 += v; st1 = fmaf(v, v, st1);
            if (r < 4 && hl4 == 0 && tl < dil) gputf(own + Q_TOP + tl * CH + c, tg.t1, v, l2);
            if (r >= 12 && hl4 == 4 && tl >= FR - dil) gputf(own + Q_BOT + (tl - (FR - dil)) * CH + c, tg.t1, v, l2);
          }
        }
        st0 = lane63_total(st0);
        st1 = lane63_total(st1);
        if (ln == 63) { sm.red1[mw][0] = st0; sm.red1[mw][1] = st1; }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        unsigned old = 0;
        if (ln == 0) old = __hip_atomic_fetch_add(&sm.cnt[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = __builtin_amdgcn_readlane(old, 0);
        if ((old & 3u) == 3u && ln < 2) {  // last M wave: the member's GN1 sums, wave order, double
          double s = 0.0;
#pragma unroll
          for (int m = 0; m < 4; ++m) s += (double)sm.red1[m][ln];
          gputd(own + Q_GN1 + 2 * ln, tg.t1, s, l2);
        }
      }
      RPROBE(2);
      __syncthreads();  // B1: H complete (the V waves' depthwise conv), next parameters in LDS
      // res_out weights: the first PD steps (chunk 0), issued once the V waves' P1 polls are done (a poll issued
      // behind 128 KB of weight loads waits for them in the CU's memory queue)
      {
        const unsigned need = bc + 1u;
        unsigned spins = 0;
        for (;;) {
          const u32x4v f = *reinterpret_cast<const volatile u32x4v*>(sm.pflag);
          if (min(min(f[0], f[1]), min(f[2], f[3])) >= need) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > a.spin_limit) { giveup(a); break; }
        }
        MLANE;
        const __amdgpu_buffer_rsrc_t w2h = rsrc_of(wb + WL::W2H), w2l = rsrc_of(wb + WL::W2L);
#pragma unroll
        for (int i = 0; i < PD; ++i) ring_load<PRE, NS2, true>(w2h, w2l, VOFF2A, VOFF2A + NS2 * 1024, rh, rl, i);
      }
      RPROBE(7);
      // ================= res_out 512->256 (model/model.py:136,144), beside the depthwise conv =================
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
      {
        MLANE;
#if RS_NOG2  // diagnostics only (wrong results): the M waves wait for the depthwise conv but run no res_out GEMM
        {
          const unsigned need = bc * NCH + NCH;
          for (;;) {
            const u32x4v f = *reinterpret_cast<const volatile u32x4v*>(sm.flag);
            if (min(min(f[0], f[1]), min(f[2], f[3])) >= need) break;
            __builtin_amdgcn_s_sleep(1);
          }
          (void)ln;
        }
#else
        mgemm<NS2, RS_LDD, PRE, true>(acc0, acc1, sm.Ahi, sm.Alo, rsrc_of(wb + WL::W2H), rsrc_of(wb + WL::W2L), VOFF2A,
                                      VOFF2A + NS2 * 1024, rh, rl, ln, sm.flag, bc * NCH, a);
#endif
      }
      RPROBE(3);
      // raw sums of the res_out accumulator (the GN2 fold is applied after the exchange, by linearity): per channel
      // over own frames (a_f) and ws-weighted per frame over channels (a_t) (P3)
      if (x.tf) {
        MLANE;
        float cv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) cv[r] = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int c = 64 * mw + 32 * q + (ln & 31);
          const float ws = pm[PB_WS2 + c];
          float rs = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = (t0 + trow(r) < T) ? (q ? acc1[r] : acc0[r]) : 0.f;
            rs += v;
            cv[r] = fmaf(ws, v, cv[r]);
          }
          rs += __shfl_xor(rs, 32);
          if (hl4 == 0) gputf(own + Q_ROW + c, tg.t3, rs, l2);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) cv[r] = half_total(cv[r]);  // lanes 31 / 63: the wave's 64 channels
        if ((ln & 31) == 31) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sm.csp[trow(r)][mw] = cv[r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        unsigned old = 0;
        if (ln == 0) old = __hip_atomic_fetch_add(&sm.cnt[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = __builtin_amdgcn_readlane(old, 0);
        if ((old & 3u) == 3u && ln < FR) {  // last M wave: the member's column sums, wave order
          const float s = ((sm.csp[ln][0] + sm.csp[ln][1]) + sm.csp[ln][2]) + sm.csp[ln][3];
          gputf(own + Q_COL + ln, tg.t3, s, l2);
        }
      }
      RPROBE(4);
      __syncthreads();  // B3: gates a_f / a_t and the GN2 fold in LDS
      RPROBE(8);
      // ================= r, gates, moment record (model/model.py:144,206-207,347-352) =================
      {
        MLANE;
        const float fmu = sm.scal[0], frs = sm.scal[1];
        float mo[NMOM];
#pragma unroll
        for (int j = 0; j < NMOM; ++j) mo[j] = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int c = 64 * mw + 32 * q + (ln & 31);
          const float ws = pm[PB_WS2 + c], bias = pm[PB_B2 + c], fcm = fmu * pm[PB_FC2 + c], afm = sm.af[c];
          f32x16v& rv = q ? acc1 : acc0;
#pragma unroll
          for (int r = 0; r < 16; ++r) rv[r] = fmaf(frs, fmaf(rv[r], ws, -fcm), bias);  // r (res_out, reg2 folded)
          if (bi == 0) {  // parity probe: DepthConv1d output of block 0 (model/model.py:144), before the gates
            if (float* dp = DUMP ? kargs()->dump : nullptr) {
#pragma unroll
              for (int r = 0; r < 16; ++r) dp[((size_t)(kargs()->B + u) * Tp + t0 + trow(r)) * CH + c] = rv[r];
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) rv[r] = rv[r] * (afm * sm.at[trow(r)]);  // r' = r a_f a_t
          if (bi == 0) {  // parity probe: TF_Attention output of block 0 (model/model.py:207)
            if (float* dp = DUMP ? kargs()->dump : nullptr) {
#pragma unroll
              for (int r = 0; r < 16; ++r) dp[((size_t)(2 * kargs()->B + u) * Tp + t0 + trow(r)) * CH + c] = rv[r];
            }
          }
          if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL) {
            // moment record of u = o + r' (device_common.h recursive_affine): 5 per-thread sums, channel weights once
            const float ga = LM == LD_RECURSIVE ? pm[PB_LNAG + c] : 0.f, be = LM == LD_RECURSIVE ? pm[PB_LNAB + c] : 0.f;
            float so = 0.f, soo = 0.f, su = 0.f, suu = 0.f, sou = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float vm = (t0 + trow(r) < T) ? 1.f : 0.f;
              const float rp = vm * rv[r];
              if constexpr (LM == LD_RECURSIVE) {
                const float ov = vm * o[q][r], uv = ov + rp;
                so += ov; soo = fmaf(ov, ov, soo); su += uv; suu = fmaf(uv, uv, suu); sou = fmaf(ov, uv, sou);
              } else {
                su += rp; suu = fmaf(rp, rp, suu);
              }
            }
            mo[2] += su; mo[3] += suu;
            if constexpr (LM == LD_RECURSIVE) {
              mo[0] += so; mo[1] += soo; mo[4] += be * so; mo[5] += ga * su; mo[6] += ga * sou; mo[7] += ga * so;
              mo[8] += ga * be * su; mo[9] += ga * ga * suu; mo[10] += ga * ga * su;
            }
          }
        }
        if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL) {
#pragma unroll
          for (int j = 0; j < NMOM; ++j) mo[j] = lane63_total(mo[j]);
          if (ln == 63) {
#pragma unroll
            for (int j = 0; j < NMOM; ++j) sm.red4[mw][j] = mo[j];
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          unsigned old = 0;
          if (ln == 0) old = __hip_atomic_fetch_add(&sm.cnt[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          old = __builtin_amdgcn_readlane(old, 0);
          if ((old & 3u) == 3u && ln < NMOM) {  // last M wave: the member's record (wave order, double) (P4)
            double s = 0.0;
#pragma unroll
            for (int m = 0; m < 4; ++m) s += (double)sm.red4[m][ln];
            gputd(own + Q_MOM + 2 * ln, tg.t4, s, l2);
          }
        }
      }
      RPROBE(5);
      __syncthreads();  // B4: residual-LN moments in LDS
      // next block's conv1d weights (the next utterance's block 0 after the last block): issued after the moment
      // polls, in flight through the x' update
      {
        MLANE;
        const __half* wn = bi + 1 < a.nblk ? wb + WL::BLOCK : a.wfrag;
        const __amdgpu_buffer_rsrc_t wnh = rsrc_of(wn), wnl = rsrc_of(wn + WL::W1L);
#pragma unroll
        for (int i = 0; i < PD; ++i) ring_load<PRE, NS1, false>(wnh, wnl, VOFF1A, VOFF1A + NS1 * 1024, rh, rl, i);
      }
      // ================= x' = next block input (model/model.py:347-352) into o and the conv1d A operand =========
      {
        MLANE;
        const float sxn = pm[PB_SXN];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int c = 64 * mw + 32 * q + (ln & 31);
          float kc[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (LM == LD_RECURSIVE) {
            kc[0] = sm.scal[3] * pm[PB_LNAG + c]; kc[1] = pm[PB_LNAB + c] - kc[0] * sm.scal[2];  // as recursive_affine
            kc[2] = sm.scal[5] * pm[PB_LNBG + c]; kc[3] = pm[PB_LNBB + c] - kc[2] * sm.scal[4];
          } else if constexpr (LM == LD_RESIDUAL) {
            kc[0] = sm.scal[3] * pm[PB_LNAG + c]; kc[1] = pm[PB_LNAB + c] - kc[0] * sm.scal[2];  // as gn_affine
          }
          const f32x16v& rv = q ? acc1 : acc0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int tl = trow(r);
            const float xv = resid_apply<LM>(o[q][r], rv[r], 1.f, 0, kc, kc + 1, kc + 2, kc + 3);
            o[q][r] = (t0 + tl < T) ? xv : 0.f;
            split_store<PRE>(sm.Ahi, sm.Alo, prow(tl) * RS_LDX + c, o[q][r] * sxn);
          }
        }
      }
      RPROBE(6);
      __syncthreads();  // B0: x' complete
    }
    // ---- TCN output x' (head input) and the statistics of PReLU(x') for TCN.output.1 ----
    {
      MLANE;
      float st0 = 0.f, st1 = 0.f;
      float* Xu = a.Xfin + ((size_t)u * Tp + t0) * CH;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = 64 * mw + 32 * q + (ln & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int t = t0 + trow(r);
          if (t < Tp) st_out(Xu + trow(r) * CH + c, o[q][r]);
          if (t < T) {
            const float pv = prelu_f(o[q][r], a.alpha_h);
            st0 += pv; st1 += pv * pv;
          }
        }
      }
      st0 = lane63_total(st0);
      st1 = lane63_total(st1);
      if (ln == 63) { sm.red1[mw][0] = st0; sm.red1[mw][1] = st1; }
    }
    __syncthreads();  // (E1)
    if (mw == 0 && lane < 2) {
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) s += (double)sm.red1[m][lane];
      a.rec_head[((size_t)u * x.G + g) * 2 + lane] = s;
    }
    __syncthreads();  // (E2) LDS free for the next utterance
  }
}

// ---------------------------------------------------------------------------------------------------------------
// One depthwise chunk of one lane: d = PReLU(dconv(GN1(h))) (model/model.py:134-135) for input channels c, c+1 (hidden
// 2c..2c+3) and frames 4f..4f+3, into the GEMM A planes; GN2 partial sums into s0/s1. MASK: zero padding of the
// normalised input outside the utterance and zero output rows past its end (members at the utterance edges).
template <int PRE, bool MASK>
__device__ __forceinline__ void dw_chunk(RsSmem& sm, const float* pm, int c, int f, int dil, float mu1, float rs1,
                                         float a2m1, int t0, int T, f32x2& s0, f32x2& s1) {
  const f32x2 g1 = *reinterpret_cast<const f32x2*>(pm + PB_G1 + c), be1 = *reinterpret_cast<const f32x2*>(pm + PB_BE1 + c);
  const f32x2 sc = g1 * rs1;
  const f32x2 sh = be1 - sc * mu1;
  f32x2 wv[2][3], bv[2];
  dw_params2(pm, c, wv, bv);
  const float* bl = lds_base(sm.H + (4 + 4 * f - dil) * RS_HS + c);
  const float* bm = lds_base(sm.H + (4 + 4 * f) * RS_HS + c);
  const float* br = lds_base(sm.H + (4 + 4 * f + dil) * RS_HS + c);
  f32x2 xv[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xv[i][0] = *reinterpret_cast<const f32x2*>(bl + i * RS_HS);
    xv[i][1] = *reinterpret_cast<const f32x2*>(bm + i * RS_HS);
    xv[i][2] = *reinterpret_cast<const f32x2*>(br + i * RS_HS);
  }
  const int pr = prow(4 * f);  // rows 4f..4f+3 stay consecutive under prow
  _Float16* const dh = sm.Ahi + pr * RS_LDD + 2 * c;
  _Float16* const dl = sm.Alo + pr * RS_LDD + 2 * c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = t0 + 4 * f + i;
    f32x2 h[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      h[k] = __builtin_elementwise_fma(xv[i][k], sc, sh);
      if constexpr (MASK) {
        const bool ok = (unsigned)(t + (k - 1) * dil) < (unsigned)T;
        h[k] = ok ? h[k] : f32x2{0.f, 0.f};
      }
    }
    f32x2 y[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      f32x2 x = __builtin_elementwise_fma(wv[q][0], h[0], bv[q]);
      x = __builtin_elementwise_fma(wv[q][1], h[1], x);
      x = __builtin_elementwise_fma(wv[q][2], h[2], x);
      f32x2 yy = prelu2(x, a2m1);
      if constexpr (MASK) yy = (unsigned)t < (unsigned)T ? yy : f32x2{0.f, 0.f};
      s0 += yy;
      s1 = __builtin_elementwise_fma(yy, yy, s1);
      y[q] = yy;
    }
    store_d4<PRE>(dh + i * RS_LDD, dl + i * RS_LDD, y[0], y[1]);
  }
}

// V role (waves 4-7): next block parameters, every hand-off poll, the depthwise conv, the gates and moments.
template <int LM, int PRE>
__device__ __forceinline__ void v_role(const TcnArgs& a, RsSmem& sm, const RsCtx& x, int lane, int v, int wave_s) {
  const int T = x.T, t0 = x.t0, g = x.g, G = x.G;
  unsigned ep = 1, bc = 0;
  for (int u = x.grp; u < a.B; u += x.ngroups) {
    if (u == x.grp && v == 0) {
      // the members' XCD ids (write-through, epoch 1); if the whole group shares one XCD, every later hand-off
      // keeps its words in that XCD's L2 (correct for any placement: checked, not assumed)
      const unsigned xcc = __builtin_amdgcn_s_getreg(6164) & 0xfu;  // hwreg(HW_REG_XCC_ID, 0, 4)
      if (lane == 0) gput(x.slot(g, 1) + Q_XCD, a.tag0 + 1, xcc, false);
      const u64* p[1] = {lane < G ? x.slot(lane, 1) + Q_XCD : nullptr};
      unsigned vv[1];
      gpoll<1>(p, a.tag0 + 1, vv, a);
      bool same = a.xmode == 0;
      const unsigned x0 = __builtin_amdgcn_readlane(vv[0], 0);
      for (int mm = 1; mm < G; ++mm) same = same && __builtin_amdgcn_readlane(vv[0], mm) == x0;
      if (lane == 0) sm.l2 = same ? 1u : 0u;
    }
    __syncthreads();  // (P1)
    __syncthreads();  // (P2)
    const bool l2 = sm.l2 != 0u;
    for (int bi = 0; bi < a.nblk; ++bi, ++bc) {
      const int par = bc & 1;
      const float* pm = sm.prm[par];
      const int li = bi % a.layer;
      const int dil = li == 0 ? 1 : (li % 4 + 1);
      const RsTags tg = next_tags<LM>(ep, x.tf, a.tag0);
      u64* const own = x.slot(g, par);
      RPROBE(0);
      {  // next block's parameter blob into the other buffer (the next utterance's block 0 after the last block)
        const int bn = bi + 1 < a.nblk ? bi + 1 : 0;
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(uni(a.prm + (size_t)bn * PB_SIZE)), (short)0, PB_SIZE * 4, 0x00020000);
        const int vt = v * 64 + lane;
        u32x4v pv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) pv[k] = __builtin_amdgcn_raw_buffer_load_b128(pr, (vt + k * 256) * 16, 0, 0);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const int idx = vt + k * 256;
          if (idx < PB_SIZE / 4) reinterpret_cast<u32x4v*>(sm.prm[par ^ 1])[idx] = pv[k];
        }
      }
      RPROBE(9);
      __syncthreads();  // B1
      // ---- P1 in one poll round: every member's GN1 words (each V wave polls them itself) and this lane's halo
      // rows: frames -dil..-1 from the predecessor (fg 0), 32..31+dil from the successor (fg 3), zero outside the
      // utterance, written into H rows that only this lane reads back ----
      const int ln = lane_fresh();              // (not hoisted out of the block loop, see lane_fresh)
      const int cl = ln & 15, fg = ln >> 4;     // depthwise lane geometry: channel in chunk, frame group
      float mu1, rs1;
      {
        const u64* p[18];
        int hrow[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int j = k >> 2, jj = k & 3, c = 64 * v + 16 * j + cl;
          p[k] = nullptr;
          hrow[k] = -1;
          if (jj < dil) {
            if (fg == 0) {
              hrow[k] = 4 - dil + jj;
              if (g > 0) p[k] = x.slot(g - 1, par) + Q_BOT + jj * CH + c;
            } else if (fg == 3) {
              hrow[k] = 4 + FR + jj;
              if (g + 1 < G) p[k] = x.slot(g + 1, par) + Q_TOP + jj * CH + c;
            }
          }
        }
        p[16] = ln < 4 * G ? x.slot(ln >> 2, par) + Q_GN1 + (ln & 3) : nullptr;
        p[17] = ln + 64 < 4 * G ? x.slot((ln + 64) >> 2, par) + Q_GN1 + (ln & 3) : nullptr;
        unsigned hv[18];
        gpoll<18>(p, tg.t1, hv, a);
        RPROBE(7);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int c = 64 * v + 16 * (k >> 2) + cl;
          if (hrow[k] >= 0) sm.H[hrow[k] * RS_HS + c] = p[k] != nullptr ? __builtin_bit_cast(float, hv[k]) : 0.f;
        }
        member_moments2(hv[16], hv[17], G, a.inv_ch, 1e-8f, mu1, rs1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ln == 0) *reinterpret_cast<volatile unsigned*>(&sm.pflag[v]) = bc + 1u;  // the M waves may issue their ring
      RPROBE(10);
      // ---- d = PReLU(dconv(GN1(h))) (model/model.py:134-135), chunk by chunk into the A planes ----
      {
        const unsigned cid0 = bc * NCH;
        float st0 = 0.f, st1 = 0.f;
#if RS_DW_SCALAR  // A/B: the first form (lane = channel x 8 frames, scalar VALU, the three taps read per frame)
        const float a2 = pm[PB_A2];
        const int lo = -t0, span = T;  // frame tl is inside the utterance iff (unsigned)(tl - lo) < span
#pragma unroll 1
        for (int j = 0; j < NCH; ++j) {
          const int c = 64 * v + 16 * j + cl;
          const float sc = rs1 * pm[PB_G1 + c], sh = pm[PB_BE1 + c] - sc * mu1;
          float wv[2][4];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            wv[q][0] = pm[PB_WD + (2 * c + q) * 3 + 0];
            wv[q][1] = pm[PB_WD + (2 * c + q) * 3 + 1];
            wv[q][2] = pm[PB_WD + (2 * c + q) * 3 + 2];
            wv[q][3] = pm[PB_BD + 2 * c + q];
          }
          const float* hc = sm.H + 4 * RS_HS + c;  // row 0 of channel c
          float xv[8][3];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int tl = 8 * fg + i;
            xv[i][0] = hc[(tl - dil) * RS_HS];
            xv[i][1] = hc[tl * RS_HS];
            xv[i][2] = hc[(tl + dil) * RS_HS];
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int tl = 8 * fg + i;
            const float h0 = (unsigned)(tl - dil - lo) < (unsigned)span ? fmaf(xv[i][0], sc, sh) : 0.f;
            const float h1 = (unsigned)(tl - lo) < (unsigned)span ? fmaf(xv[i][1], sc, sh) : 0.f;
            const float h2 = (unsigned)(tl + dil - lo) < (unsigned)span ? fmaf(xv[i][2], sc, sh) : 0.f;
            const bool vo = (unsigned)(tl - lo) < (unsigned)span;
            float dv[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              float xd = wv[q][3];
              xd = fmaf(wv[q][0], h0, xd);
              xd = fmaf(wv[q][1], h1, xd);
              xd = fmaf(wv[q][2], h2, xd);
              const float y = vo ? prelu_f(xd, a2) : 0.f;
              st0 += y; st1 = fmaf(y, y, st1);
              dv[q] = y;
            }
            split_store2<PRE>(sm.Ahi, sm.Alo, prow(tl) * RS_LDD + 2 * c, dv[0], dv[1]);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this chunk's d in LDS before its flag
          if (ln == 0) *reinterpret_cast<volatile unsigned*>(&sm.flag[v]) = cid0 + (unsigned)j + 1u;
          if (j == 0) RPROBE(8);
          if (j == 1) RPROBE(14);
          if (j == 2) RPROBE(15);
        }
#else
        // lane (p = ln & 7, f = ln >> 3): input channels c, c+1 (c = 64v + 16j + 2p) x frames 4f..4f+3, packed fp32
        // (v_pk_fma_f32 over the channel pair); members whose taps all lie inside the utterance skip the masks
        f32x2 s0v = {0.f, 0.f}, s1v = {0.f, 0.f};
        const float a2m1 = pm[PB_A2] - 1.f;
        const bool inner = t0 - dil >= 0 && t0 + FR + dil <= T;
        auto done = [&](int j) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this chunk's d in LDS before its flag
          if (ln == 0) *reinterpret_cast<volatile unsigned*>(&sm.flag[v]) = cid0 + (unsigned)j + 1u;
          if (j == 0) RPROBE(8);
          if (j == 1) RPROBE(14);
          if (j == 2) RPROBE(15);
        };
        if (inner) {
#pragma unroll 1
          for (int j = 0; j < NCH; ++j) {
            dw_chunk<PRE, false>(sm, pm, 64 * v + 16 * j + 2 * (ln & 7), ln >> 3, dil, mu1, rs1, a2m1, t0, T, s0v, s1v);
            done(j);
          }
        } else {
#pragma unroll 1
          for (int j = 0; j < NCH; ++j) {
            dw_chunk<PRE, true>(sm, pm, 64 * v + 16 * j + 2 * (ln & 7), ln >> 3, dil, mu1, rs1, a2m1, t0, T, s0v, s1v);
            done(j);
          }
        }
        st0 = s0v.x + s0v.y;
        st1 = s1v.x + s1v.y;
#endif
        // GN2 partial sums: the last V wave publishes the member's (wave order, double) (P2)
        st0 = lane63_total(st0);
        st1 = lane63_total(st1);
        if (ln == 63) { sm.vred[v][0] = st0; sm.vred[v][1] = st1; }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        unsigned old = 0;
        if (ln == 0) old = __hip_atomic_fetch_add(&sm.cnt[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = __builtin_amdgcn_readlane(old, 0);
        if ((old & 3u) == 3u && ln < 2) {
          double s = 0.0;
#pragma unroll
          for (int m = 0; m < 4; ++m) s += (double)sm.vred[m][ln];
          gputd(own + Q_GN2 + 2 * ln, tg.t2, s, l2);
        }
      }
      RPROBE(11);
      // ---- one hand-off round for GN2 and the TF-attention sums (P2 + P3) ----
      {
        const int lg = lane_fresh();
        const float* p = pm + PB_ATT;
        // this lane's words: GN2 (lg, lg + 64 of the 4G), row sums of channel 64v + lg and of halo channel ch
        // (lanes 0..5: 64v-3..64v-1, 64v+64..64v+66), the column sum of frame lg - 4 (wave 3, lanes 1..38)
        const int c = 64 * v + lg;
        const int ch = lg < 3 ? 64 * v - 3 + lg : 64 * v + 64 + (lg - 3);
        const bool hon = x.tf && lg < 6 && ch >= 0 && ch < CH;
        const int tl = lg - 4;  // lanes 4..35: own frames 0..31; lanes 1..3: -3..-1; lanes 36..38: 32..34
        const bool inr = x.tf && v == 3 && lg >= 1 && lg <= 38 && t0 + tl >= 0 && t0 + tl < T;
        float srow = 0.f, shal = 0.f, fmu = 0.f, frs = 0.f;
        unsigned cvw = 0u;
        for (int c0 = 0; c0 < G; c0 += FG_CHUNK) {
          const u64* pp[2 * FG_CHUNK + 3];
          unsigned vv[2 * FG_CHUNK + 3];
#pragma unroll
          for (int mm = 0; mm < FG_CHUNK; ++mm) {
            const bool on = c0 + mm < G;
            pp[mm] = (x.tf && on) ? x.slot(c0 + mm, par) + Q_ROW + c : nullptr;
            pp[FG_CHUNK + mm] = (hon && on) ? x.slot(c0 + mm, par) + Q_ROW + ch : nullptr;
          }
          pp[2 * FG_CHUNK] = (c0 == 0 && lg < 4 * G) ? x.slot(lg >> 2, par) + Q_GN2 + (lg & 3) : nullptr;
          pp[2 * FG_CHUNK + 1] = (c0 == 0 && lg + 64 < 4 * G) ? x.slot((lg + 64) >> 2, par) + Q_GN2 + (lg & 3) : nullptr;
          pp[2 * FG_CHUNK + 2] = nullptr;
          if (c0 == 0 && inr)
            pp[2 * FG_CHUNK + 2] = tl < 0 ? x.slot(g - 1, par) + Q_COL + tl + FR
                                          : (tl >= FR ? x.slot(g + 1, par) + Q_COL + tl - FR : own + Q_COL + tl);
          unsigned tt[2 * FG_CHUNK + 3];
#pragma unroll
          for (int k = 0; k < 2 * FG_CHUNK + 3; ++k) tt[k] = (k == 2 * FG_CHUNK || k == 2 * FG_CHUNK + 1) ? tg.t2 : tg.t3;
          gpollt<2 * FG_CHUNK + 3>(pp, tt, vv, a);
          if (c0 == 0) RPROBE(6);
#pragma unroll
          for (int mm = 0; mm < FG_CHUNK; ++mm)
            if (c0 + mm < G) { srow += __builtin_bit_cast(float, vv[mm]); shal += __builtin_bit_cast(float, vv[FG_CHUNK + mm]); }
          if (c0 == 0) {
            // GroupNorm(reg2) of d, folded into res_out (eps rescaled with d: api.hip range guard)
            member_moments2(vv[2 * FG_CHUNK], vv[2 * FG_CHUNK + 1], G, a.inv_hid, pm[PB_EPS2], fmu, frs);
            cvw = vv[2 * FG_CHUNK + 2];
          }
        }
        if (v == 0 && lg == 0) { sm.scal[0] = fmu; sm.scal[1] = frs; }
        if (x.tf) {
          const float Tf = (float)T;
          // a_f (model/model.py:198-203): channel means of r over the utterance, with a 3-channel halo per wave
          auto chan_mean = [&](int cc, float sum) {
            return (frs * (pm[PB_WS2 + cc] * sum - Tf * fmu * pm[PB_FC2 + cc]) + Tf * pm[PB_B2 + cc]) / Tf;
          };
          sm.vecw[v][lg + 3] = chan_mean(c, srow);
          if (lg < 6) sm.vecw[v][lg < 3 ? lg : lg + 64] = hon ? chan_mean(ch, shal) : 0.f;
          if (v == 3 && lg < FR + 8)
            sm.mC[lg] = inr ? (frs * (__builtin_bit_cast(float, cvw) - fmu * pm[PB_SFC2]) + pm[PB_SB2]) / (float)CH : 0.f;
          wave_lds_sync();
          {  // conv(d=1) over channels, zero outside [0, 256); index k <-> channel 64v - 3 + k
            auto yf = [&](int k) {
              const int cc = 64 * v - 3 + k;
              return (cc >= 0 && cc < CH) ? p[11] + p[8] * sm.vecw[v][k - 1] + p[9] * sm.vecw[v][k] + p[10] * sm.vecw[v][k + 1]
                                          : 0.f;
            };
            sm.yfw[v][lg + 1] = yf(lg + 1);
            if (lg < 4) sm.yfw[v][lg + 65] = yf(lg + 65);
          }
          if (v == 3 && lg < FR + 8) {  // a_t (model/model.py:199-202): conv(d=1) over frames
            const int t = t0 + lg - 4;
            float y = 0.f;
            if (t >= 0 && t < T && lg >= 1 && lg < FR + 7)
              y = p[3] + p[0] * sm.mC[lg - 1] + p[1] * sm.mC[lg] + p[2] * sm.mC[lg + 1];
            sm.yt[lg] = y;
          }
          wave_lds_sync();
          {
            const int k = lg + 3;
            const float y = p[15] + p[12] * sm.yfw[v][k - 2] + p[13] * sm.yfw[v][k] + p[14] * sm.yfw[v][k + 2];
            sm.af[64 * v + lg] = sigmoid_f(prelu_f(y, p[17]));
          }
          if (v == 3 && lg < FR) {
            const int k = lg + 4;
            const float y = p[7] + p[4] * sm.yt[k - 2] + p[5] * sm.yt[k] + p[6] * sm.yt[k + 2];
            sm.at[lg] = sigmoid_f(prelu_f(y, p[16]));
          }
        }
      }
      RPROBE(12);
      __syncthreads();  // B3
      // ---- P4: every member's moment record (22 words each) in one poll round, member order (double) ----
      if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL) {
        if (v == 0) {
          const int lp = lane_fresh();
          constexpr int NP = (FG_MAX * 2 * NMOM + 63) / 64;  // 11 words per lane at 32 members
          const u64* pp[NP];
          unsigned vv[NP];
#pragma unroll
          for (int i = 0; i < NP; ++i) {
            const int k = 64 * i + lp;
            pp[i] = k < 2 * NMOM * G ? x.slot(k / (2 * NMOM), par) + Q_MOM + k % (2 * NMOM) : nullptr;
          }
          gpoll<NP>(pp, tg.t4, vv, a);
          RPROBE(5);
#pragma unroll
          for (int i = 0; i < NP; ++i)
            if (64 * i + lp < 2 * NMOM * G) sm.gw[64 * i + lp] = vv[i];
          wave_lds_sync();
          const double* gd = reinterpret_cast<const double*>(sm.gw);
          double sj = 0.0;
          {
            const int j = lp < NMOM ? lp : 0;
            for (int mm = 0; mm < G; ++mm) sj += gd[NMOM * mm + j];
          }
          double ms[NMOM];
#pragma unroll
          for (int j = 0; j < NMOM; ++j) ms[j] = readlane_d(sj, j);
          float mua, rsa, mub = 0.f, rsb = 0.f;
          if constexpr (LM == LD_RECURSIVE) {
            recursive_moments_f(ms, reinterpret_cast<const double*>(pm + PB_WSUM), 1e-5f, 1e-5f, a.inv_ch, (double)T, mua,
                                rsa, mub, rsb);
          } else {
            gn_moments_f(ms[2], ms[3], a.inv_ch, 1e-5f, mua, rsa);
          }
          if (lp == 0) { sm.scal[2] = mua; sm.scal[3] = rsa; sm.scal[4] = mub; sm.scal[5] = rsb; }
        }
      }
      RPROBE(13);
      __syncthreads();  // B4
      __syncthreads();  // B0
    }
    __syncthreads();  // (E1)
    __syncthreads();  // (E2)
  }
}

template <int LM, int PRE, bool DUMP>
__global__ __launch_bounds__(RS_NTHR) void k_tcn_rs(TcnArgs a) {
  __shared__ __attribute__((aligned(16))) RsSmem sm;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  RsCtx x;
  x.G = a.G;
  // block -> (group, member): members of a group on one XCD when the grid is a multiple of 8*G (speed only)
  if (gridDim.x % (8 * x.G) == 0) {
    const int xi = blockIdx.x & 7, idx = blockIdx.x >> 3;
    x.grp = (idx / x.G) * 8 + xi;
    x.g = idx % x.G;
  } else {
    x.grp = blockIdx.x / x.G;
    x.g = blockIdx.x % x.G;
  }
  x.ngroups = gridDim.x / x.G;
  x.gbase = a.gran + (size_t)x.grp * x.G * 2 * NGR;
  x.T = a.T; x.Tp = a.Tp; x.t0 = x.g * FR;
  x.tf = a.tf_att != 0;
  if (a.force_err && blockIdx.x == 0 && tid == 0) giveup(a);  // diagnostics: report path only
  if (tid < 4) { sm.flag[tid] = 0u; sm.cnt[tid] = 0u; sm.pflag[tid] = 0u; }
  if (tid == 0) sm.l2 = 0u;
  if (!x.tf) {  // no TF-attention: unit gates
    if (tid < CH) sm.af[tid] = 1.f;
    if (tid < FR) sm.at[tid] = 1.f;
  }
  // first block's parameter blob (later blocks: loaded one block ahead by the V waves)
  for (int k = tid; k < PB_SIZE / 4; k += RS_NTHR)
    reinterpret_cast<float4*>(sm.prm[0])[k] = reinterpret_cast<const float4*>(a.prm)[k];
  if (RS_VPRIO && wave_s >= 4) __builtin_amdgcn_s_setprio(1);
  if (wave_s < 4) m_role<LM, PRE, DUMP>(a, sm, x, lane, wave_s, wave_s);
  else v_role<LM, PRE>(a, sm, x, lane, wave_s - 4, wave_s);
}
template <int PRE>
hipError_t launch_rs_pre(const TcnArgs& a, int grid, hipStream_t s) {
  if constexpr (PRE == PREC_F16X3) {
    if (a.dump != nullptr) {  // parity-probe instantiation (the probe code stays out of the production kernels)
      switch (a.ln_mode) {
        case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn_rs<LD_RECURSIVE, PRE, true>), dim3(grid), dim3(RS_NTHR), 0, s, a); break;
        case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn_rs<LD_RESIDUAL, PRE, true>), dim3(grid), dim3(RS_NTHR), 0, s, a); break;
        case LD_ADD: hipLaunchKernelGGL((k_tcn_rs<LD_ADD, PRE, true>), dim3(grid), dim3(RS_NTHR), 0, s, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  switch (a.ln_mode) {
    case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn_rs<LD_RECURSIVE, PRE, false>), dim3(grid), dim3(RS_NTHR), 0, s, a); break;
    case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn_rs<LD_RESIDUAL, PRE, false>), dim3(grid), dim3(RS_NTHR), 0, s, a); break;
    case LD_ADD: hipLaunchKernelGGL((k_tcn_rs<LD_ADD, PRE, false>), dim3(grid), dim3(RS_NTHR), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int PRE>
int rs_blocks_per_cu_pre(int ln_mode) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
  switch (ln_mode) {
    case LD_RECURSIVE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn_rs<LD_RECURSIVE, PRE, false>, RS_NTHR, 0); break;
    case LD_RESIDUAL: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn_rs<LD_RESIDUAL, PRE, false>, RS_NTHR, 0); break;
    case LD_ADD: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn_rs<LD_ADD, PRE, false>, RS_NTHR, 0); break;
  }
  return e == hipSuccess ? nb : 0;
}

}  // namespace

hipError_t launch_tcn_rs(const TcnArgs& a, int grid, hipStream_t s) {
  if (a.G < 1 || a.G > FG_MAX || a.G * FR < a.T || a.G * FR > a.Tp || grid < a.G || grid % a.G)
    return hipErrorInvalidValue;
  switch (a.prec) {
    case PREC_F16X3: return launch_rs_pre<PREC_F16X3>(a, grid, s);
    case PREC_F16: return launch_rs_pre<PREC_F16>(a, grid, s);
    case PREC_BF16: return launch_rs_pre<PREC_BF16>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

int tcn_rs_blocks_per_cu(int ln_mode, int prec) {
  switch (prec) {
    case PREC_F16X3: return rs_blocks_per_cu_pre<PREC_F16X3>(ln_mode);
    case PREC_F16: return rs_blocks_per_cu_pre<PREC_F16>(ln_mode);
    case PREC_BF16: return rs_blocks_per_cu_pre<PREC_BF16>(ln_mode);
  }
  return 0;
}

}  // namespace sepvad
