#pragma once
// The whole TCN separator (24 x [DepthConv1d + TF_Attention + recursive/residual LN], reference
// model/model.py:103-149,182-208,271-357) as ONE persistent launch: k_tcn.
//
// Work split: an utterance of T frames is cut into G = ceil(T/32) MEMBERS (32-frame slices). A workgroup owns NSL
// consecutive members (NSL = 1: 32 frames; NSL = 2: 64 frames, the two slices in lockstep sharing one weight stream)
// and ALL 256 channels of them, for every block; the G / NSL workgroups of an utterance form its GROUP. Inside a block
// every 1x1 conv is a row-local GEMM (frames x channels) and the depthwise conv needs `dil` halo frames, so the only
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
// Every statistic is published PER MEMBER (32-frame slice), reduced in registers and across the waves exactly as a
// one-slice workgroup reduces it, and summed over the members in member order: a two-slice workgroup gives the same
// bits as two one-slice workgroups (tests/test_gpu_fused.py), so the launch may pick either per batch.
//
// Arithmetic: fp16x3 split (see gemm.hip): acc += A_lo B_hi + A_hi B_lo + A_hi B_hi on
// v_mfma_f32_32x32x16_f16, weights pre-scaled per row by 2^-e; reg2 folded into W2/epilogue as in
// the multi-kernel path. GroupNorm statistics: float partials per wave, double across waves and members,
// fixed order => bitwise reproducible and independent of placement and batch composition.
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16 R2, "data is its own flag"): every handed-off
// 32-bit value travels as one 8-byte word {tag, value} written by a single 64-bit store, so a reader that
// sees the tag also sees the value (no payload/flag ordering, no drain before a flag). tag = launch salt
// << 12 | epoch (host: a fresh salt per launch, words zeroed once at create and when the salt wraps).
// Consumers poll exactly the words they need with agent-scope relaxed loads (L1 bypass), all words of a
// pass in flight together, bounded (a give-up sets *err and the kernel runs to completion instead of
// hanging). Stores: when all members of a group report the same XCD (HW_REG_XCC_ID, exchanged at epoch
// 1) plain stores suffice — the XCD's L2 is the coherence point — else agent-scope (sc1) write-through.
// Slots (one per member) are double-buffered by epoch parity. A member writes epoch e+2 only after it has polled
// epoch e+1 of every member, which each wrote after its epoch-e reads -- except where P2 is merged into the P3 round
// (no poll of its own): there the words of the epochs that could still be read are kept apart by offset (GW_* below).
//
// Residency: one 512-thread workgroup per CU (LDS ~140 KB one slice, ~159 KB two slices), grid <= the
// occupancy-derived capacity, and a group's workgroups are dealt to one XCD (blocks b, b+8, ... share an XCD under
// round-robin dispatch: speed only, never correctness). Groups loop over utterances (persistent), so any batch size
// runs.
#include <type_traits>

#include "tcn_common.h"

namespace sepvad {

// A/B switches (tools/build_variants.sh builds one library per setting; the losing alternatives of rounds 2-3 --
// scalar elementwise phases, separate P2 round, thread-finished GN moments, double GN finish, 11-term moments, burst
// ring prefetch, LDS epilogue parameters -- live in the git history)
#ifndef TCN_PRIO
// 1 (round 5): waves 4-7 at s_setprio 1 for the whole kernel (MI355X_MICROARCH.md "Static priority for the younger
// half"): they share each SIMD's MFMA pipe with waves 0-3 and, without it, finish every GEMM last (the barrier after
// the GEMM waits for them): k_tcn -2.4 % shader cycles at cfg 2, bitwise equal (profiles/r05_prio/). 0 = round 4.
#define TCN_PRIO 1
#endif
#ifndef TCN_FULLM
// 1 (round 6): row loops without the frame masks where a workgroup's frames are all inside [0, T) (a second copy of
// each loop, taken by a uniform branch); bitwise neutral; with it the two-slice kernels compile without spills
#define TCN_FULLM 1
#endif
#ifndef TCN_FULLDW
#define TCN_FULLDW 1  // TCN_FULLM for the depthwise conv too (a second copy of its 4 dilation variants)
#endif
#ifndef TCN_BSRED
// 1 (round 6): block_sums of more than 4 values (the moment record): reduce-scatters (rs16_wave) instead of DPP chains
#define TCN_BSRED 1
#endif
#ifndef TCN_RSRED
// 1 (round 6): row / frame sums: one reduce-scatter over the 32-lane halves (rs16_half) instead of 16 DPP chains of 5
// (the removal probe TCN_DIAG=3 put those chains at 2.9 % of k_tcn's cycles); with TCN_BSRED and TCN_FULLM cfg 2 +3 %,
// cfg 5 +7.8 % (profiles/r06w2/)
#define TCN_RSRED 1
#endif
#ifndef TCN_WPIPE
// 1 (round 6): the byte lo plane's widening one K step ahead (wave_gemm): -0.2 % k_tcn cycles at cfg 2, bitwise equal
// (profiles/r06a/cyc.txt)
#define TCN_WPIPE 1
#endif
#ifndef TCN_A1V
// 1 (round 6): conv1d PReLU slope a1 in a VGPR, not readfirstlane'd (hipcc hoisted that into the GEMM's first K step,
// whose vmcnt wait then also waited for the block-parameter loads): -0.5 % cycles, with TCN_WPIPE -0.7 %, bitwise equal
#define TCN_A1V 1
#endif
#ifndef TCN_PP
// 1 (round 6, measured, not kept): one-slice depthwise conv + res_out GEMM as a wave-role ping-pong. Waves 4-7 (s_setprio
// 1) compute the first K half of d (input channels 0..127) and start their res_out MFMAs on it while waves 0-3 compute the
// second half on the same SIMDs; waves 0-3 then run their whole K, waves 4-7 the second half. Hand-over by two LDS
// counters (no workgroup barrier); the same d, the same K order, the GN2 wave totals in the plain mapping's order: the
// same bits (digests equal at cfg 2 and cfg 5). Waves 0-3's half of d slows from 2.16 to 2.44 us beside the MFMAs and
// their 32 K steps still take 4.0 us, so the pair of phases shrinks by 0.2 us per block only, while the kernel spills 29
// VGPRs around its prologue and head: k_tcn +2.4 % cycles at cfg 2 (profiles/r06pp/).
#define TCN_PP 0
#endif
#ifndef TCN_SUB
#define TCN_SUB 0    // probe sub-stamps 13/14: 0 in the x' update, 1 in the depthwise conv (diagnostics)
#endif

constexpr int NTHR = 512;         // 8 waves; wave w owns output channels [32w, 32w+32) of both GEMMs
constexpr int LDX = CH + 8;       // x' row stride (halves): 132 dwords == 4 (mod 64) => conflict-free b128 reads
constexpr int LDD = HID + 8;      // d row stride (halves): 260 dwords == 4 (mod 64)
constexpr int HROW = FR + 8;      // conv1d output rows incl. 4 halo rows on each side
// PREC_F32 (exact fp32 GEMMs on v_mfma_f32_32x32x2_f32): the A operands are single fp32 planes in the same LDS, x'
// [32][LDXF] (= the hi plane's bytes) and d [32][LDDF] (within hi + lo), row strides == 4 (mod 64) dwords as above
constexpr int LDXF = CH + 4;
constexpr int LDDF = HID + 4;
#ifndef TCN_PD
#define TCN_PD 8     // weight K steps in flight per wave (4: +10 us; 16: spills at 2 waves per SIMD)
#endif
constexpr int PD = TCN_PD;        // weight K steps in flight per wave
#ifndef TCN_DIAG
#define TCN_DIAG 0   // diagnostics only (wrong results): 1 = GEMM ring refills skipped, 2 = GEMM MFMAs skipped,
                     // 3 = the frame sums' DPP reductions skipped (VALU-removal probe)
#endif
#ifndef TCN_AD
#define TCN_AD 1     // GEMM A-fragment LDS reads issued this many K steps ahead (2: no gain, profiles/r03h_ab_*)
#endif
#ifndef TCN_XPK
#define TCN_XPK 1    // x' update: lane pairs pack two channels per 32-bit LDS store (1) or 16-bit stores (0)
#endif
#ifndef TCN_PDQ
#define TCN_PDQ 8    // ... with the e4m3 lo plane (16 fits the registers, 238 VGPRs, but measured 4 % more cycles)
#endif
constexpr int NS1 = CH / 16;      // conv1d K steps (256 / 16)
constexpr int NS2 = HID / 16;     // res_out K steps (512 / 16)

// gathered words: 4 GN words per member, the flat moment records of up to FG_TREE members, a P4 tree leader's
// subgroup records (<= ceil(FG_MAX / 8) members)
constexpr int GW_WORDS = 4 * FG_MAX > 2 * NMOM * ((FG_MAX + 7) / 8) ? (4 * FG_MAX > 2 * NMOM * FG_TREE ? 4 * FG_MAX
                                                                                                   : 2 * NMOM * FG_TREE)
                                                                 : 2 * NMOM * ((FG_MAX + 7) / 8);
static_assert(GW_WORDS >= 2 * NMOM * FG_TREE && GW_WORDS >= 2 * NMOM * 8 && GW_WORDS >= FG_MAX, "gathered words");
static_assert(4 * FG_MAX <= 2 * NTHR, "GN words: at most two per thread");

struct TcnSmem {
  _Float16 Ahi[FR * LDD];         // GEMM A operand, hi plane: x' [32][LDX] or d [32][LDD]
  _Float16 Alo[FR * LDD];         //                 lo plane
  float H[HROW * CH];             // conv1d output (raw, pre-GN1) rows -4..35; later r for the colsums
  float c[4][CH];                 // per-channel affines (GN1 / recursive-LN)
  float af[CH];                   // frequency gate a_f
  float vec[CH + 8];              // channel means / rowsum staging
  float yf[CH + 8];
  float mC[FR + 8], yt[FR + 8], at[FR];
  float gmom[4];                  // GN1 {mean, rstd}, GN2 {mean, rstd}
  float cs[FR][8];                // per-frame channel partial sums (8 channel slices)
  float csum[FR];                 // own per-frame channel sums
  float red[NMOM * 16];
  unsigned gw[GW_WORDS] __attribute__((aligned(8)));  // gathered statistic words (GN words, moment records)
  double dred[16];
  float prm[PB_SIZE];             // this block's parameter blob (PB_*)
  float pps[16];                  // TCN_PP: the GN2 wave totals {sum [8], sumsq [8]}
  unsigned ppc[2];                // TCN_PP: waves done with K half 0 / 1 of d (4 per block)
};
static_assert(offsetof(TcnSmem, Alo) == offsetof(TcnSmem, Ahi) + sizeof(TcnSmem::Ahi) &&
              16 * FR * HEAD_VAD_N * 4 <= sizeof(TcnSmem::H) && 4 * FR * 32 * 2 <= FR * (LDD - LDX) &&
              2 * FR <= 4 * CH,
              "fused head: the waves' tap products in H, their VAD tiles in the A planes' unused row tails");
static_assert(offsetof(TcnSmem, at) % 8 == 0 && offsetof(TcnSmem, H) % 8 == 0 && offsetof(TcnSmem, prm) % 16 == 0,
              "packed (8-byte) reads of at / H / the parameter blob");

// Two-slice workgroups (64 frames): the A planes hold x' [64][LDX] or ONE K half of d [64][LDX] (the depthwise conv and
// the res_out GEMM run in two halves of 256 hidden channels), the conv1d output H [72][256] as before; the per-block
// vectors that live only from the res_out GEMM to the x' update (attention inputs, gates, frame sums) and the
// prologue's LN affine share H's storage once H is dead. 163 232 B of the 163 840 a workgroup may declare.
constexpr int FR2 = 2 * FR;
constexpr int GW2_WORDS = 2 * NMOM * FG_WAVE;  // P4 records of up to FG_WAVE members (>= the 4 G GN words)
struct TcnSmem2 {
  _Float16 Ahi[FR2 * LDX];
  _Float16 Alo[FR2 * LDX];
  union {
    float H[(FR2 + 8) * CH];      // conv1d output rows -4..67; the head's tap products [16][32][20] + VAD tiles [8][32][32]
    struct {                      // dead-H aliases (see above)
      float vec[CH + 8], yf[CH + 8];
      float mC[FR2 + 8], yt[FR2 + 8], at[FR2];
      float cs[FR2][8];
      float csum[FR2];
      float af[CH];
      float c[4][CH];
    };
  };
  float prm[PB_SIZE];
  float red[2 * NMOM * 8];
  unsigned gw[GW2_WORDS] __attribute__((aligned(8)));
  double dred[2 * NMOM];
  float gmom[4];
};
static_assert(sizeof(TcnSmem2) <= 163840 && offsetof(TcnSmem2, Alo) == offsetof(TcnSmem2, Ahi) + sizeof(TcnSmem2::Ahi),
              "two-slice LDS: one workgroup per CU");
static_assert(offsetof(TcnSmem2, at) % 8 == 0 && offsetof(TcnSmem2, H) % 16 == 0 && offsetof(TcnSmem2, prm) % 16 == 0 &&
              offsetof(TcnSmem2, gw) % 8 == 0 && offsetof(TcnSmem2, dred) % 8 == 0,
              "packed reads of at / H / the parameter blob; 8-byte gathered words");
static_assert(16 * FR * HEAD_VAD_N + 8 * FR * 32 <= (FR2 + 8) * CH && 4 * FG_WAVE <= GW2_WORDS && 2 * FR <= GW2_WORDS,
              "two-slice head: one slice's tap products and the waves' VAD tiles in H; bin 256 in gw");
template <int NSL> struct SmemOf { using type = TcnSmem; };
template <> struct SmemOf<2> { using type = TcnSmem2; };

// Weight-blob layout per operand format (api.hip init_fused): fp16x3 hi/lo planes, or one plane.
// PREC_F32: one fp32 plane per GEMM (WS32_*, in __half units of the blob pointer), 2 KB per wave per K step.
template <int PRE, int LQ = 0>
struct WLay {
  static constexpr bool L8 = LQ != 0;
  static constexpr bool X3 = PRE == PREC_F16X3;
  static constexpr bool F32 = PRE == PREC_F32;
  static constexpr size_t BLOCK = X3 ? (L8 ? WQ_BLOCK : WF_BLOCK) : (F32 ? WS32_BLOCK : WS_BLOCK);
  static constexpr size_t W1H = 0, W1L = X3 ? (L8 ? WQ_W1L : WF_W1L) : 0;
  static constexpr size_t W2H = X3 ? (L8 ? WQ_W2H : WF_W2H) : (F32 ? WS32_W2 : WS_W2), W2L = X3 ? (L8 ? WQ_W2L : WF_W2L) : W2H;
};
template <int PRE> constexpr int wstep_bytes() { return PRE == PREC_F32 ? 2048 : 1024; }  // per wave per K step

// conv1d / res_out GEMM of one wave: acc[t][32 frames x 32 channels] += A[32 t .. 32 t + 31][16*NS] * W^T for the NT
// 32-frame tiles of the workgroup (each weight fragment feeds all NT tiles). A comes from LDS (hi/lo planes, row stride
// LDA, tile t at row 32 t); the W fragments stream from global (buffer loads over the fragment-ordered weight, this
// lane's bytes at voff + 1024 * step, steps KS0 .. KS0 + NS - 1) with PD steps in flight in a static register ring; the
// first PD steps are already in (rh, rl) on entry.
// PRE: PREC_F16X3 = 3 fp16 products per step (hi/lo planes); PREC_F16 / PREC_BF16 = 1 product on the
// hi plane (fp16 or bf16 bits), no lo plane, half the weight stream.

// PREC_F32: eight v_mfma_f32_32x32x2_f32 per 16-deep step, MFMA j on the K pair (j, 8 + j) of the step (lane half h
// carries k = 8 h + j: the A reads are 8 consecutive floats per lane, the same element order as the fp16 fragments);
// the lane's 8 weight floats of a step are ring entries rh (0..3) and rl (4..7), loaded at voff and voffl = voff + 16.
template <int NS, int LDA, int RD, int NT, int KS0>
__device__ __forceinline__ void wave_gemm_f32(f32x16v (&acc)[NT], const float* Af, __amdgpu_buffer_rsrc_t wh,
                                              int voff, int voffl, u32x4v (&rh)[RD], u32x4v (&rl)[RD], int lane) {
  constexpr int SB = wstep_bytes<PREC_F32>();
  const int aoff = (lane & 31) * LDA + 8 * (lane >> 5);
  f32x4 a0[2][NT], a1[2][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    a0[0][t] = *reinterpret_cast<const f32x4*>(Af + aoff + t * FR * LDA);
    a1[0][t] = *reinterpret_cast<const f32x4*>(Af + aoff + t * FR * LDA + 4);
  }
  auto step = [&](int s, int i, bool pf) {
    const int cur = s & 1, nxt = cur ^ 1;
    if (s + 1 < NS) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        a0[nxt][t] = *reinterpret_cast<const f32x4*>(Af + aoff + t * FR * LDA + 16 * (s + 1));
        a1[nxt][t] = *reinterpret_cast<const f32x4*>(Af + aoff + t * FR * LDA + 16 * (s + 1) + 4);
      }
    }
    // (whole ring entries bit-cast: this hipcc's __builtin_bit_cast(float, v[j]) on a vector element reads element 0
    // for every j -- seen in the ISA as one B register for all four MFMAs)
    const f32x4 bh = __builtin_bit_cast(f32x4, rh[i]), bl = __builtin_bit_cast(f32x4, rl[i]);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[cur][t][j], bh[j], acc[t], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[cur][t][j], bl[j], acc[t], 0, 0, 0);
    }
    if (pf) {
      rh[i] = __builtin_amdgcn_raw_buffer_load_b128(wh, voff, (KS0 + s + RD) * SB, 0);
      rl[i] = __builtin_amdgcn_raw_buffer_load_b128(wh, voffl, (KS0 + s + RD) * SB, 0);
    }
    if (s + 1 < NS) __builtin_amdgcn_sched_group_barrier(0x100, 2 * NT, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 8 * NT, 0);
    if (pf) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
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

// CONT: the ring keeps streaming past the last step (steps KS0 + NS .. KS0 + NS + RD - 1 in flight on return, for a
// following call with KS0 + NS)
template <int NS, int LDA, int PRE, int RD = PD, int LQ = 0, int NT = 1, int KS0 = 0, bool CONT = false>
__device__ __forceinline__ void wave_gemm(f32x16v (&acc)[NT], const _Float16* Ahi, const _Float16* Alo,
                                          __amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int voff, int voffl,
                                          u32x4v (&rh)[RD], u32x4v (&rl)[RD], int lane) {
  static_assert(NS % RD == 0 && NS >= RD && KS0 % RD == 0, "K steps");
  if constexpr (PRE == PREC_F32) {
    (void)Alo; (void)wl;
    wave_gemm_f32<NS, LDA, RD, NT, KS0>(acc, reinterpret_cast<const float*>(Ahi), wh, voff, voffl, rh, rl, lane);
    return;
  } else {
  constexpr bool L8 = LQ != 0;
  static_assert(!L8 || (PRE == PREC_F16X3 && RD % 2 == 0), "byte lo plane: F16X3, K-step pairs");
  constexpr bool X3 = PRE == PREC_F16X3;
  const int aoff = (lane & 31) * LDA + 8 * (lane >> 5);
  // A fragments AD steps ahead: the LDS reads of step s+AD are in flight during steps s..s+AD-1 (AD = 2: a wave that
  // has the SIMD's matrix pipe to itself -- the other wave of the SIMD done with its GEMM -- issues a step every ~96
  // cycles, shorter than an LDS read under load)
  constexpr int AD = TCN_AD;
  static_assert(AD >= 1, "A-read depth");
  f16x8 aH[AD + 1][NT], aL[AD + 1][NT];
#pragma unroll
  for (int k = 0; k < AD; ++k) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      aH[k][t] = *reinterpret_cast<const f16x8*>(Ahi + aoff + t * FR * LDA + 16 * k);
      aL[k][t] = aH[k][t];
      if constexpr (X3) aL[k][t] = *reinterpret_cast<const f16x8*>(Alo + aoff + t * FR * LDA + 16 * k);
    }
  }
  // TCN_WPIPE (byte lo plane): the widened lo fragment of step s+1 computed during step s, so no VALU sits between a
  // step's first and second MFMA (the second one's B operand)
  constexpr bool WP = L8 && TCN_WPIPE;
  f16x8 blw;
  if constexpr (WP) blw = lo8_widen<LQ>(rl[0], 0);
  auto step = [&](int s, int i, bool pf) {
    const int cur = s % (AD + 1), nxt = (s + AD) % (AD + 1);
    if (s + AD < NS) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        aH[nxt][t] = *reinterpret_cast<const f16x8*>(Ahi + aoff + t * FR * LDA + 16 * (s + AD));
        if constexpr (X3) aL[nxt][t] = *reinterpret_cast<const f16x8*>(Alo + aoff + t * FR * LDA + 16 * (s + AD));
      }
    }
    if constexpr (TCN_DIAG == 2) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t][0] += (float)aH[cur][t][0] + (float)aL[cur][t][0] + __builtin_bit_cast(float, rh[i][0]) +
                     __builtin_bit_cast(float, rl[i][0]);
    } else if constexpr (X3) {
      const f16x8 bh = __builtin_bit_cast(f16x8, rh[i]);
      f16x8 bl;
      if constexpr (WP) bl = blw;
      else if constexpr (L8) bl = lo8_widen<LQ>(rl[i >> 1], i & 1);
      else bl = __builtin_bit_cast(f16x8, rl[i]);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f16x8 ah = aH[cur][t], al = aL[cur][t];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
      }
      if constexpr (WP) {
        if (s + 1 < NS) blw = lo8_widen<LQ>(rl[((i + 1) % RD) >> 1], (i + 1) & 1);
      }
    } else if constexpr (PRE == PREC_F16) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH[cur][t], __builtin_bit_cast(f16x8, rh[i]), acc[t], 0, 0, 0);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, aH[cur][t]),
                                                         __builtin_bit_cast(bf16x8, rh[i]), acc[t], 0, 0, 0);
    }
    // ring refill: hi entry i every step; the lo pair i/2 once both of its steps are consumed (odd i)
    if (TCN_DIAG == 1) pf = false;
    const bool pfl = pf && X3 && (!L8 || (i & 1));
    if (pf) rh[i] = __builtin_amdgcn_raw_buffer_load_b128(wh, voff, (KS0 + s + RD) * 1024, 0);
    if (pfl) {
      if constexpr (L8) rl[i >> 1] = __builtin_amdgcn_raw_buffer_load_b128(wl, voffl, ((KS0 + s + RD) >> 1) * 1024, 0);
      else rl[i] = __builtin_amdgcn_raw_buffer_load_b128(wl, voff, (KS0 + s + RD) * 1024, 0);
    }
    // pipeline shape of a step: step s+AD's A reads (DS), this step's MFMAs, then the ring refill (VMEM)
    if (s + AD < NS) __builtin_amdgcn_sched_group_barrier(0x100, (X3 ? 2 : 1) * NT, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, (X3 ? 3 : 1) * NT, 0);
    if (pfl) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
    else if (pf) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    // keep program order per step: the scheduler otherwise may sink the refill loads to their use and
    // collapse the ring to one step in flight (seen as s_waitcnt vmcnt(1) before every step)
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int s0 = 0; s0 < NS - RD; s0 += RD) {
#pragma unroll
    for (int i = 0; i < RD; ++i) step(s0 + i, i, true);
  }
#pragma unroll
  for (int i = 0; i < RD; ++i) step(NS - RD + i, i, CONT);
  }
}

template <int PRE, int RD = PD, int LQ = 0>
__device__ __forceinline__ void prefetch_w(__amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int voff, int voffl,
                                           u32x4v (&rh)[RD], u32x4v (&rl)[RD]) {
  constexpr bool L8 = LQ != 0;
#pragma unroll
  for (int s = 0; s < RD; ++s) {
    rh[s] = __builtin_amdgcn_raw_buffer_load_b128(wh, voff, s * wstep_bytes<PRE>(), 0);
    if constexpr (PRE == PREC_F32) {
      rl[s] = __builtin_amdgcn_raw_buffer_load_b128(wh, voffl, s * wstep_bytes<PRE>(), 0);
    } else if constexpr (L8) {
      if (s % 2 == 0) rl[s / 2] = __builtin_amdgcn_raw_buffer_load_b128(wl, voffl, (s / 2) * 1024, 0);
    } else if constexpr (PRE == PREC_F16X3) {
      rl[s] = __builtin_amdgcn_raw_buffer_load_b128(wl, voff, s * 1024, 0);
    }
  }
}

// Ring entry s <- K step sb + s (the burst above spread over a phase's rows: a CU's texture path takes one 1 KB wave
// load per ~16 clocks, so 8 waves issuing the whole ring at once stall ~1 us on issue)
template <int PRE, int RD, int LQ = 0>
__device__ __forceinline__ void prefetch_w1(__amdgpu_buffer_rsrc_t wh, __amdgpu_buffer_rsrc_t wl, int voff, int voffl,
                                            u32x4v (&rh)[RD], u32x4v (&rl)[RD], int s, int sb = 0) {
  constexpr bool L8 = LQ != 0;
  rh[s] = __builtin_amdgcn_raw_buffer_load_b128(wh, voff, (sb + s) * wstep_bytes<PRE>(), 0);
  if constexpr (PRE == PREC_F32) {
    rl[s] = __builtin_amdgcn_raw_buffer_load_b128(wh, voffl, (sb + s) * wstep_bytes<PRE>(), 0);
  } else if constexpr (L8) {
    if (s % 2 == 0) rl[s / 2] = __builtin_amdgcn_raw_buffer_load_b128(wl, voffl, ((sb + s) / 2) * 1024, 0);
  } else if constexpr (PRE == PREC_F16X3) {
    rl[s] = __builtin_amdgcn_raw_buffer_load_b128(wl, voff, (sb + s) * 1024, 0);
  }
}

// store_d4 (tcn_common.h) at element idx of the planes; PREC_F32: hidden 2c..2c+3 as one 16-byte store of 4 floats
template <int PRE>
__device__ __forceinline__ void store_d4i(_Float16* hi, _Float16* lo, int idx, f32x2 y0, f32x2 y1) {
  if constexpr (PRE == PREC_F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(hi) + idx) = f32x4{y0.x, y1.x, y0.y, y1.y};
  } else {
    store_d4<PRE>(hi + idx, lo + idx, y0, y1);
  }
}
// element e of an A plane as a plane pointer (fp32 planes count floats)
template <int PRE>
__device__ __forceinline__ _Float16* plane_at(_Float16* p, int e) {
  if constexpr (PRE == PREC_F32) return reinterpret_cast<_Float16*>(reinterpret_cast<float*>(p) + e);
  else return p + e;
}

// diagnostics (SEPVAD_TCN_PROBE): wave 0's wall clock at 13 phase points of every block of the first
// utterance each workgroup processes: probe[(blockIdx * nblk + block) * 16 + point]; and every wave's at the
// same points (lane 0 of each wave) after that region: probe[grid*nblk*16 + ((blockIdx*nblk + block)*16 + point)*8 + wave]
#ifdef TCN_MARK  // static census builds only (tools/isa_phases.py): an assembly comment at every phase point
#define TMARK(k) asm volatile(";;TMARK " #k)
#else
#define TMARK(k)
#endif
#define TPROBE(k)                                                                                  \
  do {                                                                                             \
    TMARK(k);                                                                                      \
    if (TP_ON && (tid & 63) == 0 && u == grp) {                                                   \
      const unsigned long long _t = wall_clock64();                                                \
      const size_t _i = ((size_t)blockIdx.x * a.nblk + bi) * 16 + (k);                            \
      if (tid == 0) a.probe[_i] = _t;                                                              \
      a.probe[(size_t)gridDim.x * a.nblk * 16 + _i * 8 + (tid >> 6)] = _t;                         \
    }                                                                                              \
  } while (0)

// Block sums of NV per-thread values (512 threads): waves by DPP, the 8 wave totals in double in wave
// order by thread j < NV into out[j]. One barrier; callers barrier again before reading `out`.
template <int NV>
__device__ __forceinline__ void block_sums(float (&v)[NV], float* lds, double* out, int tid) {
  // tid: the caller's recomputed thread id (tcn_common.h fresh_tid), so no value derived from threadIdx.x stays live
  // across the blocks (at 256 VGPRs hipcc spills such values to scratch and reloads them here behind vmcnt(0))
  const int w = tid >> 6;
  if constexpr (TCN_BSRED && NV > 4) {
    // wave totals by reduce-scatters of 16 values (rs16_wave: quad k of the wave holds value k), groups of 16
#pragma unroll
    for (int g0 = 0; g0 < NV; g0 += 16) {
      float x[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = g0 + j < NV ? v[g0 + j] : 0.f;
      const float tv = rs16_wave(x, tid & 63);
      const int j = g0 + ((tid & 63) >> 2);
      if ((tid & 3) == 0 && j < NV) lds[j * 8 + w] = tv;
    }
  } else {
  float t[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {  // independent DPP chains (interleaved by the scheduler); lane 63 = total
    t[j] = half_total(v[j]);
    t[j] += dpp_f<0x143>(t[j]);
  }
  if ((tid & 63) == 63) {  // one branch for all NV stores
#pragma unroll
    for (int j = 0; j < NV; ++j) lds[j * 8 + w] = t[j];
  }
  }
  __syncthreads();
  if (tid < NV) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += lds[tid * 8 + i];
    out[tid] = t;
  }
}

template <int LM, int PRE, bool DUMP = false, int LQ = 0, bool PROBE = false, bool LG = false, int NSL = 1>
__global__ __launch_bounds__(NTHR) void k_tcn(TcnArgs a) {
  // LG: groups above FG_WAVE members (long utterances). The short instantiation (G <= FG_WAVE, every batch of
  // utterances up to 16.4 s) compiles without the long groups' LDS word paths, wider polls and tree reductions:
  // they cost cfg 2 3.6 % of its k_tcn cycles as uniform branches (registers / SGPR spills, profiles/r04ab_*)
  static_assert(FG_TREE >= FG_WAVE, "tree reductions only in the long-group instantiation");
  // NSL: 32-frame slices (members) per workgroup. Two-slice workgroups serve short groups only (G even, <= FG_WAVE)
  static_assert(NSL == 1 || (NSL == 2 && !LG && !DUMP), "two-slice workgroups: short groups, no parity dumps");
  constexpr int FW = FR * NSL;  // frames of this workgroup
  // PREC_F32: exact fp32 GEMMs; the A planes hold fp32 rows (strides LDXF / LDDF floats), the weight stream 2 KB per wave
  // and K step (lane offsets voff and voff + 16)
  constexpr bool F32 = PRE == PREC_F32;
  static_assert(!F32 || (NSL == 1 && !DUMP), "fp32 GEMMs: one-slice workgroups");
  constexpr int LDXE = F32 ? LDXF : LDX, LDDE = F32 ? LDDF : LDD;  // A-plane row strides in elements
  constexpr int VB = F32 ? 32 : 16;                                // weight bytes per lane per K step
  using Smem = typename SmemOf<NSL>::type;
  // phase stamps only in the probe instantiation (SEPVAD_TCN_PROBE): none of their pointers or branches in production
  const bool TP_ON = PROBE && a.probe != nullptr;
  using WL = WLay<PRE, LQ>;
  constexpr bool L8 = LQ != 0;
  constexpr int RD = L8 ? TCN_PDQ : PD;  // weight K steps in flight per wave
  constexpr int RPI = RD / 8;            // ring entries issued per row of the phases before the GEMMs (8 row steps)
  static_assert(RD % 8 == 0 && RD <= 16, "ring depth: 8 or 16 K steps");
  __shared__ __attribute__((aligned(16))) Smem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const int G = a.G;        // members (32-frame slices) per utterance
  const int GW = G / NSL;   // workgroups per group
  if (TCN_PRIO && wave_s >= 4) __builtin_amdgcn_s_setprio(1);
  // block -> (group, workgroup g of the group): the groups of the first 8 * GW * floor(groups / 8) blocks each on one
  // XCD (blocks b, b + 8, ...: round-robin dispatch), the remaining groups (fewer than 8) on consecutive blocks, which
  // span XCDs (their hand-offs write through; speed only). Those take the highest group ids: with u = grp, grp +
  // groups, ... they never take an extra utterance.
  // RUN (a.run = R > 0, groups above 32 members, one slice): XCD runs -- member g on the blocks b with b % 8 = g / R,
  // so R consecutive members share an XCD (round-robin dispatch: speed only, never correctness; the hand-off store
  // types below are chosen from the members' XCD ids exchanged at epoch 1). A group spans 8 R blocks; the 8 R - G blocks
  // past its last member exit at once. Without runs a long group's consecutive members sit on consecutive XCDs and
  // every neighbour exchange (P1 halo rows, P3 frame sums) crosses XCDs.
  const int RUN = LG ? a.run : 0;
  int grp, g;
  if (RUN > 0) {
    const int S = 8 * RUN, bb = (int)blockIdx.x % S;
    grp = (int)blockIdx.x / S;
    g = (bb & 7) * RUN + (bb >> 3);
    if (g >= G) return;  // (before any publish or barrier: the whole workgroup leaves)
  } else {
    const int na = (int)(gridDim.x / (8 * GW)) * 8 * GW;  // blocks of the XCD-aligned groups
    if ((int)blockIdx.x < na) {
      const int x = blockIdx.x & 7, idx = blockIdx.x >> 3;
      grp = (idx / GW) * 8 + x;
      g = idx % GW;
    } else {
      grp = (int)blockIdx.x / GW;  // (na is a multiple of GW: group ids na / GW, ...)
      g = (int)blockIdx.x % GW;
    }
  }
  const int ngroups = gridDim.x / (RUN > 0 ? 8 * RUN : GW);
  const int m0 = NSL * g;  // this workgroup's first member: slice s is member m0 + s
  // hand-off slots of this group: member mm, epoch e -> NGR words; tags a.tag0 + epoch
  u64* const gbase = a.gran + (size_t)grp * G * 2 * NGR;
  auto slot = [&](int mm, unsigned e) -> u64* { return gbase + ((size_t)mm * 2 + (e & 1)) * NGR; };
  unsigned ep = 1;  // epochs published so far (identical sequence in every member); epoch 1 = XCD ids
  // epoch 1: the members' XCD ids (write-through); if the whole group shares one XCD, every later
  // hand-off keeps its words in that XCD's L2 (correct for any placement: checked, not assumed)
  if (TP_ON && tid == 0) {  // entry: wall clock, and the shader clock (s_memtime) when nblk > 5
    a.probe[(size_t)blockIdx.x * a.nblk * 16 + 15] = wall_clock64();
    if (a.nblk > 5) a.probe[((size_t)blockIdx.x * a.nblk + 3) * 16 + 15] = __builtin_amdgcn_s_memtime();
  }
  if (a.force_err && blockIdx.x == 0 && threadIdx.x == 0) giveup(a);  // diagnostics: report path only
  if (a.clk != nullptr && threadIdx.x == 0) {  // diagnostics (SEPVAD_TCN_CLOCK): launch span and shader clock
    const unsigned long long rt = wall_clock64();
    __hip_atomic_fetch_max(a.clk, ~rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) { a.clk[2] = rt; a.clk[4] = __builtin_amdgcn_s_memtime(); }
  }
  // epoch 1: this workgroup's XCD id for each of its members (write-through), polled in the first utterance's prologue
  if (tid < NSL && grp < a.B)
    gput(slot(m0 + tid, 1), a.tag0 + 1, __builtin_amdgcn_s_getreg(6164) & 0xfu, false);  // hwreg(HW_REG_XCC_ID, 0, 4)
  constexpr bool PP = TCN_PP && NSL == 1 && !F32;
  unsigned ppn = 0;  // TCN_PP: blocks run by this workgroup (the LDS counters' target is 4 ppn)
  if constexpr (PP) {
    if (tid < 2) sm.ppc[tid] = 0u;  // (the prologue's barriers order this before every use)
  }
  if (!a.tf_att) {  // no TF-attention: unit gates, so the gating multiply below is exact (two slices: not applied)
    if (tid < CH) sm.af[tid] = 1.f;
    if (tid < FW) sm.at[tid] = 1.f;
  }
  bool l2 = false;
  // groups above FG_TREE members reduce the P3 row sums and the P4 moment records in two levels: member g's words go
  // to leader g % 8 (above 32 members the group is dealt contiguously, so a leader's members share blockIdx % 8: one
  // XCD under round-robin dispatch, speed only), every member then polls the 8 leaders' partial sums -- 3 hand-off
  // round trips instead of G / 8 (P3) and a 176-word poll instead of 22 G words (P4). sl2: the member and its leader
  // share an XCD (checked at epoch 1); the leaders' partials stay in L2 only when the whole group does (l2)
  const bool tree = LG && G > FG_TREE;
  bool sl2 = false;
  // tree subgroups: leader k (k < nlead) is member lead_m(k); its subgroup is members sub_m(k, j), j < sub_n(k), in
  // member order: members k, k + 8, ... (no runs) or the run k R .. k R + R - 1 (runs: the run shares an XCD)
  const int nlead = RUN > 0 ? (G + RUN - 1) / RUN : 8;
  auto lead_m = [&](int k) { return RUN > 0 ? k * RUN : k; };
  auto sub_m = [&](int k, int j) { return RUN > 0 ? k * RUN + j : k + 8 * j; };
  auto sub_n = [&](int k) { return RUN > 0 ? min(RUN, G - k * RUN) : (G - k + 7) / 8; };
  const int myk = RUN > 0 ? g / RUN : g % 8;        // this member's subgroup
  const bool leader = RUN > 0 ? g % RUN == 0 : g < 8;
  // neighbour exchanges (P1 halo rows, P3 boundary frame sums) L2-only when the reading neighbour shares this XCD:
  // l2p for the words member g - 1 reads, l2n for member g + 1's (long groups; the short ones use l2)
  bool l2p = false, l2n = false;
  const int T = a.T, Tp = a.Tp, t0 = g * FW;
  const bool tf = a.tf_att != 0;
  // byte offset of this lane's 16-B fragment within its wave's weight stream (step 0)
  const int voff1 = (wave * NS1 * 64 + lane) * VB, voff2 = (wave * NS2 * 64 + lane) * VB;
  // ... and of its 16-B lo fragment pair (byte lo planes: one 1 KB wave load per two K steps), or (fp32) of its
  // second 16 bytes
  const int voff1l = F32 ? voff1 + 16 : (wave * (NS1 / 2) * 64 + lane) * 16;
  const int voff2l = F32 ? voff2 + 16 : (wave * (NS2 / 2) * 64 + lane) * 16;

  for (int u = grp; u < a.B; u += ngroups) {
    // opaque per-utterance copies (as in the block loop): keeps hipcc from hoisting and spilling the
    // per-row addresses of the prologue (their reloads waited on vmcnt(0) one by one)
    const int tidu = fresh_tid(wave_s);
    const int hl4u = 4 * ((tidu >> 5) & 1), mu_ = 32 * wave_s + (tidu & 31);
    // ---- TCN input: x'_0 = TCN.LN(S0) (model/model.py:333), own frames, into o and the LDS A operand.
    // The first-touch loads of the input (S0 rows, LN parameters, the LN records) are issued before
    // anything waits, so their latencies overlap.
    // Row r of a thread (r < 16 NSL): slice r / 16, its frame (r & 3) + 8 ((r & 15) / 4) + 4 (lane / 32): the
    // 32x32 MFMA accumulator layout of that slice's tile
    float o[16 * NSL];
    u32x4v rh[RD], rl[RD];
    {
    const int m = mu_, tid = tidu;
    auto trow = [&](int r) { return FR * (r >> 4) + (r & 3) + 8 * ((r & 15) >> 2) + hl4u; };
    float raw[16 * NSL], pg[2], pb[2], sx0;
    {
      // buffer loads off one lane offset, the row as a constant offset (flat loads here got a fresh address
      // pair per row and were serialized by s_waitcnt vmcnt(0) on register reuse, ~1.5 us each). All
      // descriptors first, then one batch of loads (the sched barrier keeps descriptor set-up, which may
      // reload spilled pointers and wait, from landing between the loads).
      const KArgs ka = kargs();
      const __amdgpu_buffer_rsrc_t s0r = rsrc_of(ka->S0 + ((size_t)u * Tp + t0) * CH);
      const __amdgpu_buffer_rsrc_t gr = rsrc_of(ka->ln.g), ber = rsrc_of(ka->ln.be);
      const __amdgpu_buffer_rsrc_t w1h = rsrc_of(ka->wfrag), w1l = rsrc_of(ka->wfrag + WL::W1L);
      const int vo = (hl4u * CH + m) * 4, co = (tid & (CH - 1)) * 4;
      const int voffu = (wave_s * NS1 * 64 + (tid & 63)) * VB;
      const int voffu_l = F32 ? voffu + 16 : (wave_s * (NS1 / 2) * 64 + (tid & 63)) * 16;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 16 * NSL; ++r)  // rows < G*32 <= Tp: in bounds (masked below)
        raw[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                               s0r, vo, ((r & 3) + 8 * ((r & 15) >> 2) + FR * (r >> 4)) * CH * 4, 0));
      // LN parameters of channel tid (threads tid < CH use them in gn_affine)
      pg[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, co, 0, 0));
      pb[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ber, co, 0, 0));
      pg[1] = pb[1] = 0.f;
      sx0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc_of(ka->prm), 0, PB_SX * 4, 0));
      prefetch_w<PRE, RD, LQ>(w1h, w1l, voffu, voffu_l, rh, rl);  // block-0 conv1d weights: in flight with the input rows
      __builtin_amdgcn_sched_barrier(0);
    }
    if (TP_ON && tid == 0 && u == grp && a.nblk > 7) a.probe[((size_t)blockIdx.x * a.nblk + 6) * 16 + 15] = wall_clock64();
    // TCN.LN records of utterance u (k_stft_gate: one per 16 frames): every value staged in LDS by one thread each (all
    // loads in flight at once), summed below in record order by threads j < 2 -- reduce_records' order, the same bits
    // (its batches of 16 dependent loads took ~6 us for the 236 records of a 60 s file). H is free until the blocks.
    double* const lnst = reinterpret_cast<double*>(sm.H);
    const RecSrc lnr = rec_src(a.ln, u, 2);
    static_assert(2 * (FG_MAX * FR / GATE_ROWS) * sizeof(double) <= sizeof(sm.H), "staged LN records in H");
    for (int i = tid; i < 2 * lnr.n; i += NTHR) lnst[i] = lnr.p[(size_t)(i >> 1) * lnr.rs + (i & 1)];
    if (TP_ON && tid == 0 && u == grp && a.nblk > 7) a.probe[((size_t)blockIdx.x * a.nblk + 7) * 16 + 15] = wall_clock64();
    if (u == grp) {
      // the members' XCD ids (write-through, epoch 1); if the whole group shares one XCD, every later
      // hand-off keeps its words in that XCD's L2 (correct for any placement: checked, not assumed)
      // (published at kernel entry, so its round trip overlaps the input loads)
      const u64* p[1] = {tid < G ? slot(tid, 1) : nullptr};
      unsigned v[1];
      gpoll<1>(p, a.tag0 + 1, v, a);
      if (tid < G) sm.gw[tid] = v[0];
      __syncthreads();
      // every member's id against member 0's (and, long groups, against its leader's) by the threads in parallel, then a
      // workgroup AND (a serial loop over the members in every thread took ~5 us at G = 118)
      int same_t = 1, sub_t = 1;
      for (int mm = tid; mm < G; mm += NTHR) {
        same_t &= sm.gw[mm] == sm.gw[0];
        if (LG) sub_t &= (RUN > 0 ? mm / RUN != myk : mm % 8 != myk) || sm.gw[mm] == sm.gw[lead_m(myk)];
      }
      const bool same = a.xmode == 0 && __syncthreads_and(same_t) != 0;
      const bool sub = a.xmode == 0 && (!LG || __syncthreads_and(sub_t) != 0);
      // wave-uniform (the words in LDS are the same for every lane): a per-lane flag in a VGPR made every hand-off
      // store a divergent branch, and at two slices hipcc spilled it and reloaded it behind vmcnt(0)
      l2 = __builtin_amdgcn_readfirstlane((int)same) != 0;
      sl2 = __builtin_amdgcn_readfirstlane((int)sub) != 0;
      if constexpr (LG) {
        const unsigned xg = sm.gw[g];
        l2p = l2 || (a.xmode == 0 && (g == 0 || sm.gw[g - 1] == xg));
        l2n = l2 || (a.xmode == 0 && (g + 1 >= G || sm.gw[g + 1] == xg));
      } else {
        l2p = l2n = l2;
      }
      if (TP_ON && tid == 0 && a.nblk > 1) a.probe[((size_t)blockIdx.x * a.nblk + 1) * 16 + 15] = wall_clock64();
    }
    __syncthreads();  // staged LN records complete
    if (tid < 2) sm.dred[tid] = seq_sum_lds(lnst + tid, 2, lnr.n);
    __syncthreads();  // LN record sums (sm.dred) complete (the LN affine below may overwrite H: two-slice sm.c)
    if (TP_ON && tid == 0 && u == grp && a.nblk > 2) a.probe[((size_t)blockIdx.x * a.nblk + 2) * 16 + 15] = wall_clock64();
    {  // gn_affine with this iteration's thread id (channel tid < CH)
      float mu, rs;
      gn_moments(sm.dred[0], sm.dred[1], (double)CH * T, a.ln.eps, mu, rs);
      if (tid < CH) {
        const float sc = rs * pg[0];
        sm.c[0][tid] = sc;
        sm.c[1][tid] = pb[0] - sc * mu;
      }
    }
    __syncthreads();
    {
      const float s = sm.c[0][m], h = sm.c[1][m];
#pragma unroll
      for (int r = 0; r < 16 * NSL; ++r) {
        const int tl = trow(r);
        o[r] = fmaf(raw[r], s, h) * (t0 + tl < T ? 1.f : 0.f);
        split_store<PRE>(sm.Ahi, sm.Alo, tl * LDXE + m, o[r] * sx0);  // x' * 2^-e (range guard, PB_SX)
      }
      if (float* dp = DUMP ? kargs()->dump : nullptr) {  // parity probe: TCN.LN output (model/model.py:333); pointer re-read
#pragma unroll                           // from the kernarg segment at use (no register held across the loop)
        for (int r = 0; r < 16; ++r) dp[((size_t)u * Tp + t0 + trow(r)) * CH + m] = o[r];
      }
    }
    __syncthreads();

    }
    for (int bi = 0; bi < a.nblk; ++bi) {
      // Opaque per-iteration copies of the lane's row offset and channel: every per-row LDS address is then
      // base + immediate offset. Without this hipcc hoists the 16 row addresses of each array out of the
      // block loop as invariants, runs out of registers and spills them (scratch reloads on every row).
      const int tido = fresh_tid(wave_s);
      const int hl4o = 4 * ((tido >> 5) & 1), mo_ = 32 * wave_s + (tido & 31);
      const int m = mo_, tid = tido, lane = tid & 63, hl = hl4o >> 2, wave = wave_s;
      auto trow = [&](int r) { return FR * (r >> 4) + (r & 3) + 8 * ((r & 15) >> 2) + hl4o; };
      TPROBE(0);
      if (DUMP && bi > 0 && bi == kargs()->dump_blk) {  // parity probe (SEPVAD_TCN_DUMP_BLOCK): this block's input
        if (float* dp = kargs()->dump) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dp[((size_t)u * Tp + t0 + trow(r)) * CH + m] = o[r];
        }
      }
      if (TP_ON && tid == 0 && u == grp && a.nblk > 5 && (bi == 0 || bi == 2))
        a.probe[((size_t)blockIdx.x * a.nblk + 4 + bi / 2) * 16 + 15] = __builtin_amdgcn_s_memtime();
      const __half* wb = a.wfrag + (size_t)bi * WL::BLOCK;
      // TCN_FULLM: the frame masks of the row loops (rows r, r + 1 of a lane's tile rows: pair p = r / 2 of 8 NSL) only
      // where a frame can be outside [0, T): none when every frame of the workgroup is inside (mpw = 0), the last two
      // pairs when only its last 8 frames can be out (mpw = 2: the other pairs hold frames <= FW - 9; T mod 32 >= 24,
      // e.g. T = 126, 188, 251), else all (a copy of each loop per case; the masks are 1 where skipped). The partial last
      // member set every group's pace (the masked loops: cfg 2 138.1k vs 145.8k utt/s, profiles/r06mp/). The depthwise
      // conv decides per wave (its 8 rows + halo).
      const int mpw = !TCN_FULLM ? 8 * NSL : (t0 + FW <= T ? 0 : (t0 + FW - 8 <= T ? 2 : 8 * NSL));
      auto by_mp = [&](auto&& f) {
        if (mpw == 0) f(std::integral_constant<int, 0>{});
        else if (mpw == 2) f(std::integral_constant<int, 2>{});
        else f(std::integral_constant<int, 8 * NSL>{});
      };
      const int li = bi % a.layer;
      const int dil = li == 0 ? 1 : (li % 4 + 1);   // model/model.py:285-295 (as api.hip packs it)
      const float* pm = sm.prm;
      // this block's parameters: loads issued now (behind the already-landed weight prefetch), stored
      // into LDS after the conv1d GEMM
      // Unconditional buffer loads (bytes past the blob read 0): a conditionally initialised array here was
      // promoted to LDS by hipcc (24 KB, a dispatch-packet read for the work-group size at kernel entry, and
      // a load -> vmcnt(0) -> ds_write chain at the start of every block).
      u32x4v pv[3];
      {
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(uni(a.prm + (size_t)bi * PB_SIZE)), (short)0, PB_SIZE * 4, 0x00020000);
#pragma unroll
        for (int k = 0; k < 3; ++k) pv[k] = __builtin_amdgcn_raw_buffer_load_b128(pr, (tid + k * NTHR) * 16, 0, 0);
      }
      // the epilogue's per-channel values straight into registers (no LDS round trip, no barrier)
      const float* pgl = a.prm + (size_t)bi * PB_SIZE;
      // (TCN_A1V: a1 kept in a VGPR -- its readfirstlane was hoisted into the GEMM's first K step, where the wait for it
      // (vmcnt) also waited for the parameter blob loads issued just before)
      const float ws1 = pgl[PB_WS1 + m], b1 = pgl[PB_B1 + m], a1 = TCN_A1V ? pgl[PB_A1] : unif(pgl[PB_A1]);
      const unsigned e1 = ++ep, tag1 = a.tag0 + e1;
      // ================= conv1d 256->256 (model/model.py:132) + PReLU =================
      f32x16v acc[NSL];
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[sl][r] = 0.f;
      {
        wave_gemm<NS1, LDXE, PRE, RD, LQ, NSL>(acc, sm.Ahi, sm.Alo, rsrc_of(wb), rsrc_of(wb + WL::W1L), voff1, voff1l, rh,
                                               rl, lane);
      TPROBE(1);
      }
      {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int idx = tid + k * NTHR;
          if (idx < PB_SIZE / 4) reinterpret_cast<u32x4v*>(sm.prm)[idx] = pv[k];
        }
        const float ws = ws1, bias = b1;  // block_sums' barrier below makes the blob visible to later phases
        float st[2 * NSL];
        // packed fp32 over row pairs (r, r+1) = frames (tl, tl+1); per slice its own sums (member statistics)
        auto epi_rows = [&](auto MPC) {
          constexpr int MP = decltype(MPC)::value;
          const float a1m1 = a1 - 1.f;
#pragma unroll
          for (int sl = 0; sl < NSL; ++sl) {
            f32x2 s0 = {0.f, 0.f}, q0 = {0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const int tl = trow(16 * sl + r);
              const f32x2 z = __builtin_elementwise_fma(f32x2{acc[sl][r], acc[sl][r + 1]}, f32x2{ws, ws}, f32x2{bias, bias});
              const f32x2 vm = 8 * sl + r / 2 < 8 * NSL - MP ? f32x2{1.f, 1.f}
                                                             : f32x2{t0 + tl < T ? 1.f : 0.f, t0 + tl + 1 < T ? 1.f : 0.f};
              const f32x2 v = prelu2(z, a1m1) * vm;
              sm.H[(tl + 4) * CH + m] = v.x;
              sm.H[(tl + 5) * CH + m] = v.y;
              s0 += v;
              q0 = __builtin_elementwise_fma(v, v, q0);
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const float ve = e ? v.y : v.x;
                // the workgroup's outer boundary rows only (the boundary between its own slices stays in H)
                if (sl == 0 && r + e < 4 && hl == 0 && tl + e < dil) gputf(slot(m0, e1) + GW_TOP + (tl + e) * CH + m, tag1, ve, l2p);
                if (sl == NSL - 1 && r + e >= 12 && hl == 1 && tl + e >= FW - dil)
                  gputf(slot(m0 + NSL - 1, e1) + GW_BOT + (tl + e - (FW - dil)) * CH + m, tag1, ve, l2n);
              }
            }
            st[2 * sl] = s0.x + s0.y;
            st[2 * sl + 1] = q0.x + q0.y;
          }
        };
        by_mp(epi_rows);
        if (TCN_SUB == 2) TPROBE(13);
        block_sums<2 * NSL>(st, sm.red, sm.dred, tid);  // barrier inside: H complete
        if (TCN_SUB == 2) TPROBE(14);
        if (tid < 2 * NSL) gputd(slot(m0 + (tid >> 1), e1) + GW_STAT + 2 * (tid & 1), tag1, sm.dred[tid], l2);
        tcn_delay(g);  // diagnostics (SEPVAD_TCN_DELAY): member 0 late to its P1 polls
      TPROBE(2);
      }
      // ---- consume P1: neighbours' boundary rows -> H halo; every member's GN1 sums ----
      {
        const u64* p[LG ? 6 : 5];
        unsigned v[LG ? 6 : 5];
        int hrow[4], hcol[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = tid + k * NTHR;
          p[k] = nullptr;
          hrow[k] = -1; hcol[k] = 0;
          if (i < 2 * dil * CH) {
            const int j = i / CH, c = i % CH;
            hcol[k] = c;
            if (j < dil) {          // frames -dil..-1: the preceding member's last dil rows
              hrow[k] = 4 - dil + j;
              if (g > 0) p[k] = slot(m0 - 1, e1) + GW_BOT + j * CH + c;
            } else {                // frames FW..FW+dil-1: the following member's first dil rows
              hrow[k] = 4 + FW + (j - dil);
              if (g + 1 < GW) p[k] = slot(m0 + NSL, e1) + GW_TOP + (j - dil) * CH + c;
            }
          }
        }
        // GN1 words of member sk/4: the last 4G threads up to 128 members; above, thread t takes words t and t + 512
        const int sk = !LG || 4 * G <= NTHR ? tid - (NTHR - 4 * G) : tid, sk2 = !LG || 4 * G <= NTHR ? -1 : tid + NTHR;
        p[4] = sk >= 0 ? slot(sk >> 2, e1) + GW_STAT + (sk & 3) : nullptr;
        if constexpr (LG) p[5] = sk2 >= 0 && sk2 < 4 * G ? slot(sk2 >> 2, e1) + GW_STAT + (sk2 & 3) : nullptr;
        gpoll<LG ? 6 : 5>(p, tag1, v, a);
      TPROBE(3);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (hrow[k] >= 0) sm.H[hrow[k] * CH + hcol[k]] = p[k] != nullptr ? __builtin_bit_cast(float, v[k]) : 0.f;
        if (!LG) {
          if (wave_s == NTHR / 64 - 1) {  // the GN1 pollers' wave: moments before the barrier
            float mu, rs;
            member_moments_w(v[4], 64 - 4 * G, G, a.inv_ch, 1e-8f, mu, rs);
            if (lane == 0) { sm.gmom[0] = mu; sm.gmom[1] = rs; }
          }
        } else {  // long utterances: the words span two waves or more, finished from LDS below
          if (sk >= 0) sm.gw[sk] = v[4];
          if constexpr (LG) if (p[5] != nullptr) sm.gw[sk2] = v[5];
        }
        __syncthreads();  // halo rows and every member's GN1 words in LDS
      }
      // ================= depthwise conv (model/model.py:134-135): d = PReLU(dconv(GN1(h))) =================
      // One pass of input-channel pairs c2, c2+1 (hidden 2c2..2c2+3) x frames fr0..fr0+7 per thread: d into the A
      // planes at column 2 c2 - acol0 (row stride LDA), its sums in (s0, s1); the res_out ring entries of K steps sb..
      // sb+RD-1 issued between the rows.
      const __amdgpu_buffer_rsrc_t w2h = rsrc_of(wb + WL::W2H), w2l = rsrc_of(wb + WL::W2L);
      float gmu, grs;  // GN1 {mean, rstd} of the group
      auto dwconv = [&](auto LDAC, int c2, int fr0, int acol0, int sb, f32x2& s0, f32x2& s1) {
        constexpr int LDA = decltype(LDAC)::value;
        const float a2 = pm[PB_A2];
        // GN1 affine of this thread's channels, computed in-thread from the group moments (no LDS round trip)
        const f32x2 sc2 = *reinterpret_cast<const f32x2*>(pm + PB_G1 + c2) * grs;
        const f32x2 sh2 = *reinterpret_cast<const f32x2*>(pm + PB_BE1 + c2) - sc2 * gmu;
        f32x2 wv[2][3], bv[2];
        dw_params2(pm, c2, wv, bv);
        const float a2m1 = a2 - 1.f;
        // rows fr0-D .. fr0+7+D of the pair once into registers (GN1 applied, zero outside [0, T)); H holds rows
        // -4..FW+3, so every load is in bounds and issued unconditionally
        auto rows = [&](auto DC, auto FULLC) {
          constexpr int D = decltype(DC)::value;
          constexpr bool FULL = decltype(FULLC)::value;
          const float* hb = lds_base(sm.H + (fr0 - D + 4) * CH + c2);
          f32x2 hv[FR / 4 + 2 * D];
#pragma unroll
          for (int i = 0; i < FR / 4 + 2 * D; ++i) {
            const int t = t0 + fr0 - D + i;
            const float vm = FULL || (t >= 0 && t < T) ? 1.f : 0.f;  // mask multiply (a select sinks each load into a branch)
            hv[i] = __builtin_elementwise_fma(*reinterpret_cast<const f32x2*>(hb + i * CH), sc2, sh2) * vm;
          }
#pragma unroll
          for (int i = 0; i < FR / 4; ++i) {
#pragma unroll
            for (int e = 0; e < RPI; ++e)  // res_out ring entries RPI i .. RPI i + RPI - 1
              prefetch_w1<PRE, RD, LQ>(w2h, w2l, voff2, voff2l, rh, rl, RPI * i + e, sb);
            const int tl = fr0 + i;
            const float vo = FULL || t0 + tl < T ? 1.f : 0.f;
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
            store_d4i<PRE>(sm.Ahi, sm.Alo, tl * LDA + 2 * c2 - acol0, y[0], y[1]);
          }
        };
        static_assert(RD == RPI * FR / 4, "RPI ring entries per frame of the packed depthwise conv");
        auto rows_d = [&](auto FULLC) {
#ifdef TCN_CENSUS_DIL  // static census builds only (tools/isa_phases.py): one dilation's code path, no switch
          rows(std::integral_constant<int, TCN_CENSUS_DIL>{}, FULLC);
          if (false)
#endif
          switch (dil) {
            case 1: rows(std::integral_constant<int, 1>{}, FULLC); break;
            case 2: rows(std::integral_constant<int, 2>{}, FULLC); break;
            case 3: rows(std::integral_constant<int, 3>{}, FULLC); break;
            default: rows(std::integral_constant<int, 4>{}, FULLC); break;
          }
        };
        // (per wave: the thread's 8 rows fr0 .. fr0 + 7 and their halo, wave-uniform in both layouts)
        const bool fullw = TCN_FULLDW && __builtin_amdgcn_readfirstlane((int)(TCN_FULLM && t0 + fr0 - 4 >= 0 && t0 + fr0 + FR / 4 + 4 <= T)) != 0;
        if (fullw) rows_d(std::true_type{});
        else rows_d(std::false_type{});
      };
      {
        if (!LG) {
          gmu = sm.gmom[0]; grs = sm.gmom[1];
        } else {  // long groups: member_sums2's fixed order (not member_moments_w's; each bitwise reproducible per G)
          const double2 acc = member_sums2(sm.gw, G, lane);
          gn_moments_f(acc.x, acc.y, a.inv_ch, 1e-8f, gmu, grs);
        }
      }
      // ---- P2 words: GN2 partial sums (awaited after the res_out main loop) ----
      const unsigned e2 = ++ep, tag2 = a.tag0 + e2;
      // TCN_PP hand-over: wait until the 4 waves of K half hh have stored their d rows (LDS counter; s_sleep between reads)
      auto pp_wait = [&](int hh) {
        if constexpr (PP) {
          while (__hip_atomic_load(&sm.ppc[hh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4u * ppn)
            __builtin_amdgcn_s_sleep(1);
          asm volatile("" ::: "memory");
        }
      };
      if constexpr (PP) {
        // waves 4-7 (the s_setprio 1 waves: they win the VALU while both compute d) take K half 0 = input channels
        // 0..127, waves 0-3 half 1; wave w's frames 8 (w & 3) .. + 7; vw = its wave in the plain mapping below
        ++ppn;
        const int hh = wave_s >= 4 ? 0 : 1, fq = wave_s & 3, vw = 2 * fq + hh;
        f32x2 s0 = {0.f, 0.f}, s1 = {0.f, 0.f};
        dwconv(std::integral_constant<int, LDDE>{}, 2 * (64 * hh + lane), fq * (FR / 4), 0, 0, s0, s1);
        // block_sums<2>'s wave totals (lane 63), at the plain mapping's wave index
        float t0v = half_total(s0.x + s0.y), t1v = half_total(s1.x + s1.y);
        t0v += dpp_f<0x143>(t0v);
        t1v += dpp_f<0x143>(t1v);
        if (lane == 63) { sm.pps[vw] = t0v; sm.pps[8 + vw] = t1v; }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's d rows and totals stored
        if (lane == 0) __hip_atomic_fetch_add(&sm.ppc[hh], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      TPROBE(4);
      } else if constexpr (NSL == 1) {
        if (TCN_SUB == 1) TPROBE(13);
        f32x2 s0 = {0.f, 0.f}, s1 = {0.f, 0.f};
        // thread = input channels c2, c2+1 (hidden 2c2..2c2+3) x frames fr0..fr0+7
        dwconv(std::integral_constant<int, LDDE>{}, 2 * (tid & (CH / 2 - 1)), (tid >> 7) * (FR / 4), 0, 0, s0, s1);
        float st[2] = {s0.x + s0.y, s1.x + s1.y};
        if (TCN_SUB == 1) TPROBE(14);
        block_sums<2>(st, sm.red, sm.dred, tid);  // barrier inside: d complete in LDS
      TPROBE(4);
        if (tid < 2) gputd(slot(g, e2) + GW_STAT + 2 * tid, tag2, sm.dred[tid], l2);
      }
      // ================= res_out 512->256 (model/model.py:136,144) with reg2 folded =================
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[sl][r] = 0.f;
      if constexpr (PP) {
        if (wave_s >= 4) {  // K half 0 as soon as its d is complete, then half 1
          pp_wait(0);
          wave_gemm<NS2 / 2, LDDE, PRE, RD, LQ, 1, 0, true>(acc, sm.Ahi, sm.Alo, w2h, w2l, voff2, voff2l, rh, rl, lane);
          pp_wait(1);
          wave_gemm<NS2 / 2, LDDE, PRE, RD, LQ, 1, NS2 / 2>(acc, plane_at<PRE>(sm.Ahi, HID / 2), plane_at<PRE>(sm.Alo, HID / 2),
                                                           w2h, w2l, voff2, voff2l, rh, rl, lane);
        } else {  // all of d, then the whole K; threads 0, 1 publish the GN2 words (block_sums<2>'s order and bits)
          pp_wait(1);
          pp_wait(0);
          if (tid < 2) {
            double t = 0.0;
#pragma unroll
            for (int i = 0; i < 8; ++i) t += sm.pps[tid * 8 + i];
            gputd(slot(g, e2) + GW_STAT + 2 * tid, tag2, t, l2);
          }
          wave_gemm<NS2, LDDE, PRE, RD, LQ>(acc, sm.Ahi, sm.Alo, w2h, w2l, voff2, voff2l, rh, rl, lane);
        }
      } else if constexpr (NSL == 1) {
        wave_gemm<NS2, LDDE, PRE, RD, LQ>(acc, sm.Ahi, sm.Alo, w2h, w2l, voff2, voff2l, rh, rl, lane);
      } else {
        // two K halves of 256 hidden channels each (input channels 0..127, then 128..255 of the depthwise conv) through
        // the same A planes. The member statistics of d: per half every wave's totals of the pass it ran, which is the
        // wave (2 (w' & 3) + half) of the one-slice mapping for slice w' / 4 (the same 64 channel pairs x 8 frames, the
        // same lane order), so the per-member doubles below are the one-slice workgroup's bits.
        auto d_half = [&](int h) {
          f32x2 s0 = {0.f, 0.f}, s1 = {0.f, 0.f};
          dwconv(std::integral_constant<int, LDX>{}, 128 * h + 2 * (tid & 63), (tid >> 6) * (FR / 4), 256 * h,
                 (NS2 / 2) * h, s0, s1);
          float t0v = half_total(s0.x + s0.y), t1v = half_total(s1.x + s1.y);
          t0v += dpp_f<0x143>(t0v);
          t1v += dpp_f<0x143>(t1v);
          if (lane == 63) {
            const int sl = wave_s >> 2, w = 2 * (wave_s & 3) + h;
            sm.red[(2 * sl) * 8 + w] = t0v;
            sm.red[(2 * sl + 1) * 8 + w] = t1v;
          }
          __syncthreads();  // this half of d complete in LDS
        };
        d_half(0);
      TPROBE(4);
        wave_gemm<NS2 / 2, LDX, PRE, RD, LQ, 2, 0>(acc, sm.Ahi, sm.Alo, w2h, w2l, voff2, voff2l, rh, rl, lane);
        __syncthreads();  // every wave done reading the first half of d
        d_half(1);
        if (tid < 4) {  // member (m0 + tid / 2)'s GN2 {sum, sumsq}: the 8 wave totals in one-slice wave order
          double t = 0.0;
#pragma unroll
          for (int i = 0; i < 8; ++i) t += sm.red[tid * 8 + i];
          gputd(slot(m0 + (tid >> 1), e2) + GW_STAT + 2 * (tid & 1), tag2, t, l2);
        }
        wave_gemm<NS2 / 2, LDX, PRE, RD, LQ, 2, NS2 / 2>(acc, sm.Ahi, sm.Alo, w2h, w2l, voff2, voff2l, rh, rl, lane);
      }
      TPROBE(5);
      f32x16v (&rv)[NSL] = acc;  // r = res_out output, in place
      const unsigned e3 = tf ? ++ep : 0u, tag3 = a.tag0 + e3;
      // GN2 {mean, rstd} of the group from the polled P2 words (a wave's lanes base.. or the words in LDS)
      auto gn2_moments = [&](float& fmu, float& frs) {
        if (!LG) {
          fmu = sm.gmom[2]; frs = sm.gmom[3];
        } else {
          const double2 sums = member_sums2(sm.gw, G, lane);
          gn_moments_f(sums.x, sums.y, a.inv_hid, pm[PB_EPS2], fmu, frs);  // eps rescaled with d
        }
      };
      if (!tf) {  // no TF-attention sums to exchange: the P2 round alone
        constexpr int NP2 = LG ? 2 : 1;
        const u64* p[NP2];
        unsigned v[NP2];
        p[0] = tid < 4 * G ? slot(tid >> 2, e2) + GW_STAT + (tid & 3) : nullptr;
        if constexpr (LG) p[1] = tid + NTHR < 4 * G ? slot((tid + NTHR) >> 2, e2) + GW_STAT + (tid & 3) : nullptr;
        gpoll<LG ? 2 : 1>(p, tag2, v, a);
        if (!LG) {
          if (wave_s == 0) {
            float mu, rs;
            member_moments_w(v[0], 0, G, a.inv_hid, pm[PB_EPS2], mu, rs);
            if (lane == 0) { sm.gmom[2] = mu; sm.gmom[3] = rs; }
          }
        } else {
          if (tid < 4 * G) sm.gw[tid] = v[0];
          if constexpr (LG) if (tid + NTHR < 4 * G) sm.gw[tid + NTHR] = v[NP2 - 1];
        }
        __syncthreads();
      TPROBE(6);
        float fmu, frs;
        gn2_moments(fmu, frs);
        const float ws = pm[PB_WS2 + m], bias = pm[PB_B2 + m], fcm = fmu * pm[PB_FC2 + m];
#pragma unroll
        for (int sl = 0; sl < NSL; ++sl)
#pragma unroll
          for (int r = 0; r < 16; ++r) rv[sl][r] = fmaf(frs, fmaf(rv[sl][r], ws, -fcm), bias);
      }
      // ---- TF_Attention (model/model.py:182-208) ----
      if (tf) {
        // P2 + P3 in ONE hand-off round: the row / column sums are taken on the raw res_out accumulator and the GN2 fold
        // (affine per channel) is applied to the exchanged sums, so they need not wait for the GN2 words
        {
          const float ws = pm[PB_WS2 + m];
#pragma unroll
          for (int sl = 0; sl < NSL; ++sl) {
            float rsum = 0.f, csr[16];
            by_mp([&](auto MPC) {
              constexpr int MP = decltype(MPC)::value;
              float rs = 0.f;
#pragma unroll
              for (int r = 0; r < 16; ++r)
                rs += 8 * sl + r / 2 < 8 * NSL - MP || t0 + trow(16 * sl + r) < T ? acc[sl][r] : 0.f;
              rsum = rs;
            });
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              if constexpr (TCN_RSRED) csr[r] = ws * acc[sl][r];
              else
              csr[r] = TCN_DIAG == 3 ? ws * acc[sl][r]  // (diagnostics: the 80 DPP adds per wave removed, wrong sums)
                                     : half_total(ws * acc[sl][r]);  // ws-weighted sum over the wave's 32 channels (lanes 31 / 63)
            }
            if constexpr (TCN_RSRED) {
              // ws-weighted sums over the wave's 32 channels of each frame by one reduce-scatter (lane L: row (L & 31) / 2
              // of its half), stored by the even lanes
              const float cv = rs16_half(csr, lane);
              if ((lane & 1) == 0) sm.cs[trow(16 * sl + ((lane & 31) >> 1))][wave] = cv;
              float ro = rsum;
              swap32(rsum, ro);  // (ro: the other half's frames; a + b == b + a, the bits of the __shfl_xor form)
              rsum += ro;
            } else {
            if ((lane & 31) == 31) {
#pragma unroll
              for (int r = 0; r < 16; ++r) sm.cs[trow(16 * sl + r)][wave] = csr[r];
            }
            rsum += __shfl_xor(rsum, 32);
            }
            if (hl == 0) gputf(slot(m0 + sl, e3) + GW_ROW + m, tag3, rsum, tree ? sl2 : l2);
          }
        }
        __syncthreads();  // cs complete; also: every wave is done reading d from LDS
      TPROBE(6);
        if (tid < FW) {  // P3 words: per-frame raw channel sums (a_t); the neighbours read the outer 4 frames each side
          float s = 0.f;
#pragma unroll
          for (int sl = 0; sl < 8; ++sl) s += sm.cs[tid][sl];
          sm.csum[tid] = s;
          // (only the outer 4 frames each side: the neighbours' a_t inputs; the own frames stay in LDS)
          if (tid < 4 || tid >= FW - 4) gputf(slot(m0 + tid / FR, e3) + GW_COL + tid % FR, tag3, s, tid < 4 ? l2p : l2n);
        }
        tcn_delay(g);  // diagnostics (SEPVAD_TCN_DELAY): member 0 late to its P2/P3 polls
      TPROBE(7);
        {
          const u64* pp[FG_CHUNK];
          unsigned v[FG_CHUNK], tg[FG_CHUNK];
          int mi = -1;  // a_t input index (frame t0 - 4 + mi) served by this thread
          const u64* pat = nullptr;
          if (tid >= CH && tid < CH + 8) {
            const int k = tid - CH;
            mi = k < 4 ? k : FW + k;             // 0..3 and FW+4..FW+7
            const int tl = mi - 4, t = t0 + tl;
            if (t >= 0 && t < T) pat = tl < 0 ? slot(m0 - 1, e3) + GW_COL + tl + FR : slot(m0 + NSL, e3) + GW_COL + tl - FW;
          }
          // threads 384..: GN2 words kq + 128 j (j < 8) of the 4G (wave 6 holds all of them for G <= 16; up to 256
          // members, 1024 words, in the first pass's free slots)
          const int kq = tid - (NTHR - 128);
          float s = 0.f, vat = 0.f;
          unsigned vq[FG_CHUNK] = {};
          if (tree) {
            // level 1 (the leaders): the row sums of their subgroup's members, member order, published for everyone
            if (leader) {
              constexpr int L1 = 16;  // subgroup members polled per pass (a subgroup has <= 16 up to 128 members)
              const int ns = sub_n(myk);
              float ss = 0.f;
              for (int j0 = 0; j0 < ns; j0 += L1) {
                const u64* p1[L1];
                unsigned v1[L1];
#pragma unroll
                for (int mm = 0; mm < L1; ++mm)
                  p1[mm] = (tid < CH && j0 + mm < ns) ? slot(sub_m(myk, j0 + mm), e3) + GW_ROW + tid : nullptr;
                gpoll<L1>(p1, tag3, v1, a);
#pragma unroll
                for (int mm = 0; mm < L1; ++mm)
                  if (j0 + mm < ns) ss += __builtin_bit_cast(float, v1[mm]);
              }
              if (tid < CH) gputf(slot(g, e3) + GW_SUB3 + tid, tag3, ss, l2);
            }
          }
          static_assert(FG_CHUNK == 8, "level 2 of the P3 tree polls the 8 leaders in one pass");
          // (a do-while: G >= 1, so no guard of the first pass -- hipcc kept that guard as a kernel-wide flag, spilled)
          int c0 = 0;
          do {  // (level 2: one pass over the 8 leaders)
#pragma unroll
            for (int mm = 0; mm < FG_CHUNK; ++mm) {
              pp[mm] = tree ? (tid < CH && mm < nlead ? slot(lead_m(mm), e3) + GW_SUB3 + tid : nullptr)
                            : ((tid < CH && c0 + mm < G) ? slot(c0 + mm, e3) + GW_ROW + tid : nullptr);
              tg[mm] = tag3;
            }
            if (c0 == 0 && mi >= 0) pp[0] = pat;
            if (c0 == 0 && kq >= 0) {
              if (!LG || G <= 32) {
                pp[0] = kq < 4 * G ? slot(kq >> 2, e2) + GW_STAT + (kq & 3) : nullptr;
                tg[0] = tag2;
              } else {
#pragma unroll
                for (int j = 0; j < FG_CHUNK; ++j) {
                  const int w = kq + 128 * j;
                  pp[j] = w < 4 * G ? slot(w >> 2, e2) + GW_STAT + (w & 3) : nullptr;
                  tg[j] = tag2;
                }
              }
            }
            gpollt<FG_CHUNK>(pp, tg, v, a);
            if (tid < CH) {
#pragma unroll
              for (int mm = 0; mm < FG_CHUNK; ++mm)
                if (tree ? mm < nlead : c0 + mm < G) s += __builtin_bit_cast(float, v[mm]);
            }
            if (c0 == 0) {
              vat = __builtin_bit_cast(float, v[0]);
#pragma unroll
              for (int j = 0; j < (LG ? FG_CHUNK : 1); ++j) vq[j] = v[j];
            }
            c0 += FG_CHUNK;
          } while (c0 < (tree ? 1 : G));
          if (!LG) {
            if (wave_s == 6) {
              float mu, rs;
              member_moments_w(vq[0], 0, G, a.inv_hid, pm[PB_EPS2], mu, rs);
              if (lane == 0) { sm.gmom[2] = mu; sm.gmom[3] = rs; }
            }
          } else if (kq >= 0) {
#pragma unroll
            for (int j = 0; j < FG_CHUNK; ++j)
              if (kq + 128 * j < 4 * G) sm.gw[kq + 128 * j] = vq[j];
          }
          __syncthreads();  // csum, the GN2 moments / words complete
          float fmu, frs;
          gn2_moments(fmu, frs);
          const float Tf = (float)T, sfc = pm[PB_SFC2], sb = pm[PB_SB2];
          if (tid < CH) {  // a_f input: channel means of r over the utterance (GN2 fold applied to the sums)
            sm.vec[tid + 4] = (frs * (pm[PB_WS2 + tid] * s - Tf * fmu * pm[PB_FC2 + tid]) + Tf * pm[PB_B2 + tid]) / Tf;
            if (tid < 4) { sm.vec[tid] = 0.f; sm.vec[CH + 4 + tid] = 0.f; sm.yf[tid] = 0.f; sm.yf[CH + 4 + tid] = 0.f; }
          } else if (mi >= 0) {
            sm.mC[mi] = pat != nullptr ? (frs * (vat - fmu * sfc) + sb) / (float)CH : 0.f;
          } else if (tid >= CH + 8 && tid < CH + 8 + FW) {
            const int tl = tid - CH - 8;
            sm.mC[tl + 4] = (t0 + tl < T) ? (frs * (sm.csum[tl] - fmu * sfc) + sb) / (float)CH : 0.f;
          }
          const float ws = pm[PB_WS2 + m], bias = pm[PB_B2 + m], fcm = fmu * pm[PB_FC2 + m];
#pragma unroll
          for (int sl = 0; sl < NSL; ++sl)
#pragma unroll
            for (int r = 0; r < 16; ++r) rv[sl][r] = fmaf(frs, fmaf(rv[sl][r], ws, -fcm), bias);
        }
        __syncthreads();
      TPROBE(8);
        const float* p = pm + PB_ATT;
        // a_f: mean over frames -> conv(d=1) -> conv(d=2) -> PReLU -> sigmoid (over the channel axis);
        // a_t: mean over channels -> conv(d=1) -> conv(d=2) -> PReLU -> sigmoid (over the frame axis)
        if (tid < CH) {
          sm.yf[tid + 4] = p[11] + p[8] * sm.vec[tid + 3] + p[9] * sm.vec[tid + 4] + p[10] * sm.vec[tid + 5];
        } else if (tid < CH + FW + 8) {
          const int i = tid - CH, t = t0 - 4 + i;
          float v = 0.f;
          if (t >= 0 && t < T && i >= 1 && i < FW + 7) v = p[3] + p[0] * sm.mC[i - 1] + p[1] * sm.mC[i] + p[2] * sm.mC[i + 1];
          sm.yt[i] = v;
        }
        __syncthreads();
        if (tid < CH) {
          const float v = p[15] + p[12] * sm.yf[tid + 2] + p[13] * sm.yf[tid + 4] + p[14] * sm.yf[tid + 6];
          sm.af[tid] = sigmoid_f(prelu_f(v, p[17]));
        } else if (tid < CH + FW) {
          const int tl = tid - CH, k = tl + 4;
          const float v = p[7] + p[4] * sm.yt[k - 2] + p[5] * sm.yt[k] + p[6] * sm.yt[k + 2];
          sm.at[tl] = sigmoid_f(prelu_f(v, p[16]));
        }
        __syncthreads();
      }
      TPROBE(9);
      // ---- residual update (model/model.py:345-352) ----
      // gate r in place once: r' = r a_f a_t (a_f = a_t = 1 without TF-attention, set at kernel start; the two-slice
      // workgroup keeps its gates in dead-H storage and skips the multiply instead)
      {
        if (bi == kargs()->dump_blk) {  // parity probe: DepthConv1d output of block 0 (model/model.py:144), before the gates
          if (float* dp = DUMP ? kargs()->dump : nullptr) {
#pragma unroll
            for (int r = 0; r < 16; ++r) dp[((size_t)(kargs()->B + u) * Tp + t0 + trow(r)) * CH + m] = rv[0][r];
          }
        }
        if (NSL == 1 || tf) {
          const float afm = sm.af[m];
#pragma unroll
          for (int r = 0; r < 16 * NSL; r += 2) {
            const f32x2 g2 = *reinterpret_cast<const f32x2*>(sm.at + trow(r)) * afm;  // frames trow(r), trow(r)+1
            f32x2 x = f32x2{rv[r >> 4][r & 15], rv[r >> 4][(r & 15) + 1]} * g2;
            // LD_ADD (x' = o + r'): the gated product's only use is that add, and hipcc contracted the pair into an FMA in
            // one of the one- / two-slice instantiations and not the other (1-ulp differences, tests/test_gpu_fused.py
            // test_two_slices_bitwise_other_configs); materialised, both round r' first as the other LN modes do
            if constexpr (LM == LD_ADD) asm volatile("" : "+v"(x));
            rv[r >> 4][r & 15] = x.x; rv[r >> 4][(r & 15) + 1] = x.y;
          }
        }
        if (bi == kargs()->dump_blk) {  // parity probe: TF_Attention output of block 0 (model/model.py:207)
          if (float* dp = DUMP ? kargs()->dump : nullptr) {
#pragma unroll
            for (int r = 0; r < 16; ++r) dp[((size_t)(2 * kargs()->B + u) * Tp + t0 + trow(r)) * CH + m] = rv[0][r];
          }
        }
      }
      float kc[4] = {0.f, 0.f, 0.f, 0.f};  // this channel's residual-LN affines (GN_a: 0, 1; GN_b: 2, 3)
      if constexpr (LM == LD_RECURSIVE || LM == LD_RESIDUAL) {
        // moment record of u = o + r' (r' = r a_f a_t) per member, see device_common.h recursive_affine: per-thread sums
        // over its 16 rows of the slice first, then the channel weights once
        const float ga = LM == LD_RECURSIVE ? pm[PB_LNAG + m] : 0.f, be = LM == LD_RECURSIVE ? pm[PB_LNAB + m] : 0.f;
        float mo[NSL * NMOM];
        auto mom_rows = [&](auto MPC) {
        constexpr int MP = decltype(MPC)::value;
#pragma unroll
        for (int sl = 0; sl < NSL; ++sl) {
          float so = 0.f, soo = 0.f, su = 0.f, suu = 0.f, sou = 0.f;
          {
            f32x2 so2 = {0.f, 0.f}, soo2 = so2, su2 = so2, suu2 = so2, sou2 = so2;
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const int tl = trow(16 * sl + r);
              const f32x2 vm = 8 * sl + r / 2 < 8 * NSL - MP ? f32x2{1.f, 1.f}  // masked, not branched
                                                             : f32x2{t0 + tl < T ? 1.f : 0.f, t0 + tl + 1 < T ? 1.f : 0.f};
              const f32x2 rp = vm * f32x2{rv[sl][r], rv[sl][r + 1]};
              if constexpr (LM == LD_RECURSIVE) {
                const f32x2 ov = vm * f32x2{o[16 * sl + r], o[16 * sl + r + 1]}, uv = ov + rp;
                so2 += ov; soo2 = __builtin_elementwise_fma(ov, ov, soo2); su2 += uv;
                suu2 = __builtin_elementwise_fma(uv, uv, suu2); sou2 = __builtin_elementwise_fma(ov, uv, sou2);
              } else {
                su2 += rp; suu2 = __builtin_elementwise_fma(rp, rp, suu2);
              }
            }
            so = so2.x + so2.y; soo = soo2.x + soo2.y; su = su2.x + su2.y; suu = suu2.x + suu2.y; sou = sou2.x + sou2.y;
          }
          float* const ms = mo + sl * NMOM;
#pragma unroll
          for (int j = 0; j < NMOM; ++j) ms[j] = 0.f;
          ms[2] = su; ms[3] = suu;
          if constexpr (LM == LD_RECURSIVE) {
            ms[0] = so; ms[1] = soo; ms[4] = be * so; ms[5] = ga * su; ms[6] = ga * sou; ms[7] = ga * so;
            ms[8] = ga * be * su; ms[9] = ga * ga * suu; ms[10] = ga * ga * su;
          }
        }
        };
        by_mp(mom_rows);
        block_sums<NSL * NMOM>(mo, sm.red, sm.dred, tid);
      TPROBE(10);
        // ---- P4 words: the moment record (11 doubles) of each member; consume every member's ----
        const unsigned e4 = ++ep, tag4 = a.tag0 + e4;
        if (tid < NSL * NMOM) gputd(slot(m0 + tid / NMOM, e4) + GW_P4 + 2 * (tid % NMOM), tag4, sm.dred[tid], tree ? sl2 : l2);
        if (tree) {
          // level 1 (the leaders): the records of their subgroup's members (<= 32: two words per thread), summed in member
          // order (double) by wave 0's lanes j < NMOM and published for everyone
          if (leader) {
            const int nsub = sub_n(myk), nw = 2 * NMOM * nsub;  // <= 704 words (32 members)
            const int k2 = tid + NTHR;
            const u64* pp[2] = {tid < nw ? slot(sub_m(myk, tid / (2 * NMOM)), e4) + GW_P4 + tid % (2 * NMOM) : nullptr,
                                k2 < nw ? slot(sub_m(myk, k2 / (2 * NMOM)), e4) + GW_P4 + k2 % (2 * NMOM) : nullptr};
            unsigned v[2];
            gpoll<2>(pp, tag4, v, a);
            if (tid < nw) sm.gw[tid] = v[0];
            if (k2 < nw) sm.gw[k2] = v[1];
            __syncthreads();
            if (wave_s == 0) {
              const double* gd = reinterpret_cast<const double*>(sm.gw);
              const int j = lane < NMOM ? lane : 0;
              const double sj = seq_sum_lds(gd + j, NMOM, nsub);
              if (lane < NMOM) gputd(slot(g, e4) + GW_SUB4 + 2 * lane, tag4, sj, l2);
            }
            __syncthreads();  // the leader's words read before the leaders' partials land in sm.gw
          }
          // level 2 (everyone): the leaders' partial records
          const int nw = 2 * NMOM * nlead;
          const u64* pp[1] = {tid < nw ? slot(lead_m(tid / (2 * NMOM)), e4) + GW_SUB4 + tid % (2 * NMOM) : nullptr};
          unsigned v[1];
          gpoll<1>(pp, tag4, v, a);
          if (tid < nw) sm.gw[tid] = v[0];
        } else {
          // word k % 22 of member k / 22: one word per thread up to 23 members; beyond, passes of up to four words in
          // flight per thread (32 members: 704 words, one pass)
          const int nw = 2 * NMOM * G;
          if (!LG || nw <= NTHR) {
            const u64* pp[1] = {tid < nw ? slot(tid / (2 * NMOM), e4) + GW_P4 + tid % (2 * NMOM) : nullptr};
            unsigned v[1];
            gpoll<1>(pp, tag4, v, a);
            if (tid < nw) sm.gw[tid] = v[0];
          } else for (int k0 = 0; k0 < nw; k0 += 4 * NTHR) {
            const u64* pp[4];
            unsigned v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int k = k0 + tid + j * NTHR;
              pp[j] = k < nw ? slot(k / (2 * NMOM), e4) + GW_P4 + k % (2 * NMOM) : nullptr;
            }
            gpoll<4>(pp, tag4, v, a);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int k = k0 + tid + j * NTHR;
              if (k < nw) sm.gw[k] = v[j];
            }
          }
        }
      TPROBE(11);
        __syncthreads();  // every member's moment words in LDS
        // GN_a / GN_b of this thread's channel m, in-thread (member order as before: no LDS round trip of
        // the sums or the affines, one barrier)
        // lane j < NMOM of every wave sums moment j over the members (one LDS load per member per wave),
        // then the 11 sums become wave-uniform by readlane
        const double* gd = reinterpret_cast<const double*>(sm.gw);
        const double sj = seq_sum_lds(gd + (lane < NMOM ? lane : 0), NMOM, tree ? nlead : G);  // members, or the 8
                                                                                              // leaders' partials
        double ms[NMOM];
#pragma unroll
        for (int j = 0; j < NMOM; ++j) ms[j] = readlane_d(sj, j);
        if constexpr (LM == LD_RECURSIVE) {
          float mua, rsa, mub, rsb;
          recursive_moments_f(ms, reinterpret_cast<const double*>(pm + PB_WSUM), 1e-5f, 1e-5f, a.inv_ch, (double)T, mua,
                              rsa, mub, rsb);
          kc[0] = rsa * pm[PB_LNAG + m]; kc[1] = pm[PB_LNAB + m] - kc[0] * mua;  // as recursive_affine
          kc[2] = rsb * pm[PB_LNBG + m]; kc[3] = pm[PB_LNBB + m] - kc[2] * mub;
        } else {
          float mu, rs;
          gn_moments_f(ms[2], ms[3], a.inv_ch, 1e-5f, mu, rs);  // as gn_affine
          kc[0] = rs * pm[PB_LNAG + m]; kc[1] = pm[PB_LNAB + m] - kc[0] * mu;
        }
      if (TCN_SUB == 0) TPROBE(13);
      }
      // next block's conv1d weights: in flight during the x' update; after the last block, the output head's first
      // row tile (speaker 0, tile hjl: the head's wave -> tile map) instead
      const bool lastb = bi + 1 == a.nblk;
      const int hjl = (wave_s + (blockIdx.x >> 3)) & 7;
      const __amdgpu_buffer_rsrc_t wnh = lastb ? rsrc_of(a.hwh) : rsrc_of(wb + WL::BLOCK);
      const __amdgpu_buffer_rsrc_t wnl = lastb ? rsrc_of(PRE == PREC_F16X3 ? a.hwl : a.hwh) : rsrc_of(wb + WL::BLOCK + WL::W1L);
      const int pvo = lastb ? (hjl * NS1 * 64 + lane) * VB : voff1;
      const int pvol = lastb ? (F32 ? pvo + 16 : (hjl * (NS1 / 2) * 64 + lane) * 16) : voff1l;
      if (TCN_SUB == 0) TPROBE(14);
      // x' = next block input: o (registers) and the conv1d A operand (LDS, scaled by the next block's 2^-e)
      {
        const float sxn = pm[PB_SXN];
        auto xup_rows = [&](auto MPC) {
        constexpr int MP = decltype(MPC)::value;
#pragma unroll
        for (int r = 0; r < 16 * NSL; r += 2) {
          const int pr = r / 2;  // row pair: the ring entries are spread over the first 8 (one slice) or all 16 pairs
          if (NSL == 1 || pr % 2 == 0) {
#pragma unroll
            for (int e = 0; e < RPI; ++e) prefetch_w1<PRE, RD, LQ>(wnh, wnl, pvo, pvol, rh, rl, RPI * (pr / NSL) + e);
          }
          const int tl = trow(r);
          const f32x2 x = resid_apply2<LM>(f32x2{o[r], o[r + 1]}, f32x2{rv[r >> 4][r & 15], rv[r >> 4][(r & 15) + 1]},
                                           kc);  // rv gated above
          const f32x2 vm = r / 2 < 8 * NSL - MP ? f32x2{1.f, 1.f}
                                                : f32x2{t0 + tl < T ? 1.f : 0.f, t0 + tl + 1 < T ? 1.f : 0.f};
          const f32x2 ov = x * vm;
          o[r] = ov.x; o[r + 1] = ov.y;
          if (TCN_XPK) split_store_rows_pk<PRE>(sm.Ahi, sm.Alo, tl * LDXE + m, LDXE, ov * sxn, (lane & 1) != 0);
          else split_store_rows<PRE>(sm.Ahi, sm.Alo, tl * LDXE + m, LDXE, ov * sxn);
        }
        };
        by_mp(xup_rows);
      }
      __syncthreads();
      TPROBE(12);
    }
    // ---- output head (model/model.py:322-325,357): masks = W_out GN_out(PReLU(x')) + b on this workgroup's slices,
    // and the VAD conv1_1 tap products of the masks (model/model.py:158-160), while x' is still in registers (o). The
    // statistics of PReLU(x') are one more hand-off round (P5). 16 row tiles of 32 on MFMA (speaker q's bins
    // 32 jl .. 32 jl + 31, jl < 8), two per wave, each weight fragment for all slices; bin 256 of each speaker (one
    // row) as fp32 VALU dot products.
    {
      const int tidh = fresh_tid(wave_s);
      const int hl4h = 4 * ((tidh >> 5) & 1), mh = 32 * wave_s + (tidh & 31);
      auto trow = [&](int r) { return FR * (r >> 4) + (r & 3) + 8 * ((r & 15) >> 2) + hl4h; };
      // diagnostics (SEPVAD_TAIL_PROBE, first utterance): slot 0 wall clock, 1.. shader clock at the phase ends
      unsigned long long* const hpr = a.hprobe != nullptr && u == grp ? a.hprobe + (size_t)blockIdx.x * 8 : nullptr;
      auto hstamp = [&](int k) {
        if (hpr != nullptr && tidh == 0) hpr[k] = __builtin_amdgcn_s_memtime();
      };
      if (hpr != nullptr && tidh == 0) hpr[0] = wall_clock64();
      hstamp(1);
      // the first tile's weights are in the ring since the last block's x' update (each next tile's are issued during
      // the current tile's epilogue)
      // (the weight copy keeps 9 row tiles per speaker: speaker q's tile jl is row tile HEAD_SPK / 32 * q + jl). The
      // wave -> tile map rotates with the workgroup's place on its XCD, so the XCD's CUs stream different tiles at a
      // time (speed only: every result is indexed by tile, not by wave)
      const int jl = (wave_s + (blockIdx.x >> 3)) & 7;
      const __amdgpu_buffer_rsrc_t wh = rsrc_of(a.hwh), wl = rsrc_of(PRE == PREC_F16X3 ? a.hwl : a.hwh);
      // P5: each member's record of PReLU(x') (sum, sumsq over its valid frames), every member's in member order
      {
        float st[2 * NSL];
#pragma unroll
        for (int k = 0; k < 2 * NSL; ++k) st[k] = 0.f;
#pragma unroll
        for (int r = 0; r < 16 * NSL; ++r) {
          if (t0 + trow(r) < T) {
            const float pv = prelu_f(o[r], a.alpha_h);
            st[2 * (r >> 4)] += pv; st[2 * (r >> 4) + 1] += pv * pv;
          }
        }
        block_sums<2 * NSL>(st, sm.red, sm.dred, tidh);
      }
      const unsigned e5 = ++ep, tag5 = a.tag0 + e5;  // (P4 is a full round before: no member still polls GW_STAT)
      if (tidh < 2 * NSL)  // (the thread's own sum)
        gputd(slot(m0 + (tidh >> 1), e5) + GW_STAT + 2 * (tidh & 1), tag5, sm.dred[tidh], l2);
      {
        constexpr int NP = LG ? 2 : 1;
        const u64* p[NP];
        unsigned v[NP];
        p[0] = tidh < 4 * G ? slot(tidh >> 2, e5) + GW_STAT + (tidh & 3) : nullptr;
        if constexpr (LG) p[NP - 1] = tidh + NTHR < 4 * G ? slot((tidh + NTHR) >> 2, e5) + GW_STAT + (tidh & 3) : nullptr;
        gpoll<NP>(p, tag5, v, a);
        if (tidh < 4 * G) sm.gw[tidh] = v[0];
        if constexpr (LG) if (tidh + NTHR < 4 * G) sm.gw[tidh + NTHR] = v[NP - 1];
      }
      hstamp(2);
      __syncthreads();
      if (tidh < 2) {  // GroupNorm statistics of PReLU(x') over the utterance: the members' records in member order
        const double* gd = reinterpret_cast<const double*>(sm.gw);
        sm.dred[8 + tidh] = seq_sum_lds(gd + tidh, 2, G);
      }
      __syncthreads();
      // A = GN_out(PReLU(x')) into LDS (scaled by hsx, undone by the weights' row scale)
      {
        float mu, rs;
        gn_moments_f(sm.dred[8], sm.dred[9], a.inv_ch, 1e-5f, mu, rs);
        const float sc = rs * a.hg[mh], sh = a.hbe[mh] - sc * mu;
#pragma unroll
        for (int r = 0; r < 16 * NSL; ++r)
          split_store<PRE>(sm.Ahi, sm.Alo, trow(r) * LDXE + mh, fmaf(prelu_f(o[r], a.alpha_h), sc, sh) * a.hsx);
      }
      __syncthreads();  // A complete
      hstamp(3);
      const bool vad = a.hvP != nullptr;
      // this wave's VAD tile: [32 frames][32 channels], 16-B granules XOR-swizzled by frame: one slice, in the unused
      // tail of the A planes (row stride LDD, only LDX in use); two slices, in H past one slice's tap products. The
      // waves' tap products [8][2][FR][20] of one slice in H (free now)
      // (fp32: the head's A fills the hi plane's bytes, the 8 tiles go to the lo plane)
      float* const vsc = F32 ? reinterpret_cast<float*>(sm.Alo) + wave_s * FR * 32
                             : (NSL == 1 ? reinterpret_cast<float*>((wave_s < 4 ? sm.Ahi : sm.Alo) + FR * LDX) + (wave_s & 3) * FR * 32
                                         : sm.H + 16 * FR * HEAD_VAD_N + wave_s * FR * 32);
      float* const Ps = sm.H;
      auto vidx = [](int t, int c) { return t * 32 + ((((c >> 2) ^ t) & 7) << 2) + (c & 3); };
      float* const nys = NSL == 1 ? &sm.c[0][0] : reinterpret_cast<float*>(sm.gw);  // [2][FR] bin 256 (free now)
      // slice by slice (two slices: the head's weights streamed once per slice; the head is a few % of the launch and
      // the one-tile loop keeps the registers of the one-slice kernel)
#pragma unroll 1
      for (int sl = 0; sl < NSL; ++sl) {
        // opaque per-slice lane values (as in the block loop): the per-row addresses are not hoisted across the slices
        const int tidh = fresh_tid(wave_s), lh = tidh & 63, hl4h = 4 * ((tidh >> 5) & 1);
        auto trow1 = [&](int r) { return (r & 3) + 8 * (r >> 2) + hl4h; };  // row r < 16 of one slice's tile
        auto tile_voff = [&](int q) { return ((q * (HEAD_SPK / 32) + jl) * NS1 * 64 + lh) * VB; };
        auto tile_voffl = [&](int q) { return F32 ? tile_voff(q) + 16 : ((q * (HEAD_SPK / 32) + jl) * (NS1 / 2) * 64 + lh) * 16; };
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int jt = q * (HEAD_SPK / 32) + jl;  // row tile of the weight copy
          f32x16v acc[1];
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[0][r] = 0.f;
          wave_gemm<NS1, LDXE, PRE, RD, LQ>(acc, plane_at<PRE>(sm.Ahi, FR * sl * LDXE), plane_at<PRE>(sm.Alo, FR * sl * LDXE),
                                            wh, wl, tile_voff(q), tile_voffl(q), rh, rl, lh);
          if (q == 0) prefetch_w<PRE, RD, LQ>(wh, wl, tile_voff(1), tile_voffl(1), rh, rl);
          else if (sl + 1 < NSL) prefetch_w<PRE, RD, LQ>(wh, wl, tile_voff(0), tile_voffl(0), rh, rl);
          f16x8 vb[2][2];
          if (vad && !F32) {
#pragma unroll
            for (int st = 0; st < 2; ++st) {
              vb[st][0] = *reinterpret_cast<const f16x8*>(a.hvwh + ((size_t)(2 * jl + st) * 64 + lh) * 8);
              vb[st][1] = *reinterpret_cast<const f16x8*>(a.hvwl + ((size_t)(2 * jl + st) * 64 + lh) * 8);
            }
          }
          const int c = 32 * jl + (lh & 31);  // speaker-local bin
          const float ws = a.hwscale[32 * jt + (lh & 31)], bias = a.hbias[32 * jt + (lh & 31)];
          float* const out = a.hmasks + ((size_t)u * Tp + t0 + FR * sl) * MOUT_PAD + q * NBIN + c;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            acc[0][r] = fmaf(acc[0][r], ws, bias);
            st_out(out + (size_t)trow1(r) * MOUT_PAD, acc[0][r]);
          }
          if (vad) {  // VAD conv1_1 tap products of the tile's 32 bins: P[t][n] = sum_c masks[t][c] Wv[c][n], fp16x3
#pragma unroll
            for (int r = 0; r < 16; ++r) vsc[vidx(trow1(r), lh & 31)] = acc[0][r] * a.hvsx;
            wave_lds_sync();
            f32x16v pv;
#pragma unroll
            for (int r = 0; r < 16; ++r) pv[r] = 0.f;
#pragma unroll
            for (int st = 0; st < 2; ++st) {
              const int tr = lh & 31, c0 = 16 * st + 8 * (lh >> 5);
              const f32x4 x0 = *reinterpret_cast<const f32x4*>(vsc + vidx(tr, c0));
              const f32x4 x1 = *reinterpret_cast<const f32x4*>(vsc + vidx(tr, c0 + 4));
              if constexpr (F32) {  // fp32 tap products (the K-pair convention of wave_gemm_f32), weights a.hvwf
                const float* wf = a.hvwf + ((size_t)(2 * jl + st) * 64 + lh) * 8;
                const f32x4 b0 = *reinterpret_cast<const f32x4*>(wf), b1 = *reinterpret_cast<const f32x4*>(wf + 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) pv = __builtin_amdgcn_mfma_f32_32x32x2f32(x0[j], b0[j], pv, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) pv = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[j], b1[j], pv, 0, 0, 0);
                continue;
              }
              f16x8 ah, al;
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float x = e < 4 ? x0[e] : x1[e - 4];
                const _Float16 hh = (_Float16)x;
                ah[e] = hh;
                al[e] = (_Float16)(x - (float)hh);
              }
              pv = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, vb[st][0], pv, 0, 0, 0);
              pv = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, vb[st][1], pv, 0, 0, 0);
              pv = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, vb[st][0], pv, 0, 0, 0);
            }
            wave_lds_sync();  // the tile's reads done before the wave's next tile overwrites it
            if ((lh & 31) < HEAD_VAD_N) {
#pragma unroll
              for (int r = 0; r < 16; ++r) Ps[((jl * 2 + q) * FR + trow1(r)) * HEAD_VAD_N + (lh & 31)] = pv[r];
            }
          }
        }
        if (sl + 1 == NSL) hstamp(4);
        // bin 256 of each speaker (one row, fp32 VALU) from A in LDS: thread -> (speaker, frame, 32-channel part),
        // channels in order, then the 8 parts by a fixed xor tree (while slower waves finish their tiles)
        {
          const int od = tidh >> 3, part = tidh & 7, qn = od >> 5, tn = od & 31;
          const _Float16* ah = sm.Ahi + (FR * sl + tn) * LDX + 32 * part;
          const _Float16* al = sm.Alo + (FR * sl + tn) * LDX + 32 * part;
          const f32x4* wq = reinterpret_cast<const f32x4*>(a.hnyw + qn * CH + 32 * part);
          float sn = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            // (read as the type split_store wrote: bf16 planes through __bf16, fp16 through _Float16)
            float xv[8];
            if constexpr (F32) {
              const float* af = reinterpret_cast<const float*>(sm.Ahi) + (FR * sl + tn) * LDXE + 32 * part + 8 * k;
              const f32x4 u0 = *reinterpret_cast<const f32x4*>(af), u1 = *reinterpret_cast<const f32x4*>(af + 4);
#pragma unroll
              for (int e = 0; e < 8; ++e) xv[e] = e < 4 ? u0[e] : u1[e - 4];
            } else if constexpr (PRE == PREC_BF16) {
              const bf16x8 bv = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(ah) + 8 * k);
#pragma unroll
              for (int e = 0; e < 8; ++e) xv[e] = (float)bv[e];
            } else {
              const f16x8 hv = *reinterpret_cast<const f16x8*>(ah + 8 * k);
              f16x8 lv = {};
              if constexpr (PRE == PREC_F16X3) lv = *reinterpret_cast<const f16x8*>(al + 8 * k);
#pragma unroll
              for (int e = 0; e < 8; ++e) xv[e] = PRE == PREC_F16X3 ? (float)hv[e] + (float)lv[e] : (float)hv[e];
            }
            const f32x4 w0 = wq[2 * k], w1 = wq[2 * k + 1];
#pragma unroll
            for (int e = 0; e < 8; ++e) sn = fmaf(xv[e], e < 4 ? w0[e] : w1[e - 4], sn);
          }
          sn += __shfl_xor(sn, 1);
          sn += __shfl_xor(sn, 2);
          sn += __shfl_xor(sn, 4);
          if (part == 0) nys[qn * FR + tn] = sn / a.hsx + a.hnyb[qn];  // (hsx: a power of two)
        }
        __syncthreads();  // bin 256 and every wave's tap products of this slice in LDS
        // the tap products: the tiles' in tile order, then bin 256's term (fp32)
        const int ts = t0 + FR * sl;  // the slice's first frame
        for (int i = tidh; i < (vad ? 2 * FR * HEAD_VAD_N : 2 * FR); i += NTHR) {
          const int per = vad ? FR * HEAD_VAD_N : FR;
          const int q = i >= per ? 1 : 0, ri = i - q * per;
          const int t = vad ? ri / HEAD_VAD_N : ri, n = vad ? ri - t * HEAD_VAD_N : 0;
          const float m = nys[q * FR + t];
          if (n == 0) st_out(a.hmasks + ((size_t)u * Tp + ts + t) * MOUT_PAD + q * NBIN + (NBIN - 1), m);
          if (vad) {
            float sum = 0.f;
#pragma unroll
            for (int w = 0; w < 8; ++w) sum += Ps[((w * 2 + q) * FR + t) * HEAD_VAD_N + n];  // tile order
            a.hvP[(((size_t)u * 2 + q) * Tp + ts) * HEAD_VAD_N + ri] = ts + t < T ? fmaf(m, a.hvny[n], sum * a.hvwscale[n]) : 0.f;
          }
        }
        if (sl + 1 == NSL) hstamp(5);
        __syncthreads();  // (the next slice's tiles / the next utterance's prologue rewrite the LDS)
      }
    }
  }
  // (the clock record pointer re-read from the kernarg segment: nothing held in registers across the blocks)
  if (unsigned long long* const ck = kargs()->clk; ck != nullptr && threadIdx.x == 0) {
    const unsigned long long rt = wall_clock64();
    if (blockIdx.x == 0) { ck[3] = rt; ck[5] = __builtin_amdgcn_s_memtime(); }
    __hip_atomic_fetch_max(ck + 1, rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// launchers of one (precision, lo-plane format): instantiated per translation unit by fused_inst.hip
template <int PRE, int LQ, bool LG>
static hipError_t launch_tcn_pre(const TcnArgs& a, int grid, hipStream_t s) {
  if constexpr (PRE == PREC_F16X3) {
    if (a.dump != nullptr) {  // parity-probe instantiation (the probe code stays out of the production kernels)
      switch (a.ln_mode) {
        case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn<LD_RECURSIVE, PRE, true, LQ, false, LG>), dim3(grid), dim3(NTHR), 0, s, a); break;
        case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn<LD_RESIDUAL, PRE, true, LQ, false, LG>), dim3(grid), dim3(NTHR), 0, s, a); break;
        case LD_ADD: hipLaunchKernelGGL((k_tcn<LD_ADD, PRE, true, LQ, false, LG>), dim3(grid), dim3(NTHR), 0, s, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  if (a.probe != nullptr && a.ln_mode == LD_RECURSIVE) {  // phase-stamp instantiation (SEPVAD_TCN_PROBE, recursive LN)
    hipLaunchKernelGGL((k_tcn<LD_RECURSIVE, PRE, false, LQ, true, LG>), dim3(grid), dim3(NTHR), 0, s, a);
    return hipGetLastError();
  }
  switch (a.ln_mode) {
    case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn<LD_RECURSIVE, PRE, false, LQ, false, LG>), dim3(grid), dim3(NTHR), 0, s, a); break;
    case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn<LD_RESIDUAL, PRE, false, LQ, false, LG>), dim3(grid), dim3(NTHR), 0, s, a); break;
    case LD_ADD: hipLaunchKernelGGL((k_tcn<LD_ADD, PRE, false, LQ, false, LG>), dim3(grid), dim3(NTHR), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// two-slice workgroups (short groups only; no parity-dump instantiation)
template <int PRE, int LQ>
static hipError_t launch_tcn2_pre(const TcnArgs& a, int grid, hipStream_t s) {
  if (a.dump != nullptr) return hipErrorInvalidValue;
  if (a.probe != nullptr && a.ln_mode == LD_RECURSIVE) {
    hipLaunchKernelGGL((k_tcn<LD_RECURSIVE, PRE, false, LQ, true, false, 2>), dim3(grid), dim3(NTHR), 0, s, a);
    return hipGetLastError();
  }
  switch (a.ln_mode) {
    case LD_RECURSIVE: hipLaunchKernelGGL((k_tcn<LD_RECURSIVE, PRE, false, LQ, false, false, 2>), dim3(grid), dim3(NTHR), 0, s, a); break;
    case LD_RESIDUAL: hipLaunchKernelGGL((k_tcn<LD_RESIDUAL, PRE, false, LQ, false, false, 2>), dim3(grid), dim3(NTHR), 0, s, a); break;
    case LD_ADD: hipLaunchKernelGGL((k_tcn<LD_ADD, PRE, false, LQ, false, false, 2>), dim3(grid), dim3(NTHR), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int PRE, int LQ>
static hipError_t launch_tcn_lg(const TcnArgs& a, int grid, hipStream_t s) {
  if constexpr (PRE != PREC_F32) {
    if (a.nsl == 2) return launch_tcn2_pre<PRE, LQ>(a, grid, s);
  }
  return a.G > FG_WAVE ? launch_tcn_pre<PRE, LQ, true>(a, grid, s) : launch_tcn_pre<PRE, LQ, false>(a, grid, s);
}

template <int PRE, int LQ, int NSL>
static int blocks_per_cu_pre(int ln_mode) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
  switch (ln_mode) {
    case LD_RECURSIVE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn<LD_RECURSIVE, PRE, false, LQ, false, false, NSL>, NTHR, 0); break;
    case LD_RESIDUAL: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn<LD_RESIDUAL, PRE, false, LQ, false, false, NSL>, NTHR, 0); break;
    case LD_ADD: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tcn<LD_ADD, PRE, false, LQ, false, false, NSL>, NTHR, 0); break;
  }
  if constexpr (NSL == 2) return e == hipSuccess ? nb : 0;
  int nl = 0;  // the long-group instantiation: the capacity is the smaller of the two (both 1 / CU by their LDS)
  hipError_t el = hipErrorInvalidValue;
  switch (ln_mode) {
    case LD_RECURSIVE: el = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nl, k_tcn<LD_RECURSIVE, PRE, false, LQ, false, true>, NTHR, 0); break;
    case LD_RESIDUAL: el = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nl, k_tcn<LD_RESIDUAL, PRE, false, LQ, false, true>, NTHR, 0); break;
    case LD_ADD: el = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nl, k_tcn<LD_ADD, PRE, false, LQ, false, true>, NTHR, 0); break;
  }
  return e == hipSuccess && el == hipSuccess ? (nb < nl ? nb : nl) : 0;
}

}  // namespace sepvad
