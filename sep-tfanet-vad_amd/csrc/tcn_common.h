// Device helpers of the persistent TCN kernel (tcn_kernel.h k_tcn):
// MFMA operand types, wave-uniform buffer descriptors, the tagged 8-byte hand-off words ("data is its own
// flag", cdna_hip_programming.md Guideline 16 R2) with bounded polls, DPP lane reductions and the fp16 hi/lo
// operand split.
#pragma once
#include <type_traits>

#include "device_common.h"

namespace sepvad {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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
typedef unsigned long long u64;
// ---- hand-off words: 8-byte {tag, value} granules (the data is its own flag) ----
// Same-XCD groups: plain stores keep the words in the XCD's shared L2; otherwise agent-scope (sc1)
// write-through stores. Consumers always load with agent-scope relaxed atomics (sc1: L1 bypass).
__device__ __forceinline__ void gput(u64* p, unsigned tag, unsigned v, bool l2) {
  const u64 w = ((u64)tag << 32) | v;
  if (l2) __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gputf(u64* p, unsigned tag, float v, bool l2) {
  gput(p, tag, __builtin_bit_cast(unsigned, v), l2);
}
__device__ __forceinline__ void gputd(u64* p, unsigned tag, double v, bool l2) {  // two consecutive words
  const u64 b = __builtin_bit_cast(u64, v);
  gput(p, tag, (unsigned)b, l2);
  gput(p + 1, tag, (unsigned)(b >> 32), l2);
}
__device__ __forceinline__ double dword2(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(double, ((u64)hi << 32) | lo);
}
#ifndef TCN_POLL_SERIAL
#define TCN_POLL_SERIAL 0
#endif
#ifndef TCN_POLL_SLEEP
#define TCN_POLL_SLEEP 1  // s_sleep between poll passes (units of 64 clocks; 0 = none)
#endif
// A bounded hand-off wait gave up: record this launch's tag0 in the device word and its host-mapped copy.
__device__ __forceinline__ void giveup(const TcnArgs& a) {
  __hip_atomic_store(a.err, a.tag0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.herr != nullptr) __hip_atomic_store(a.herr, a.tag0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Poll the N words p[k] (nullptr = none) until every tag equals tag[k]; values into v[k]. Every load of a pass is
// unconditional (a null word reads a valid dummy word instead and is ignored), so all N are in flight together: a
// load inside an exec-masked `if (p[k])` is waited for before the branch closes, which serialises the pass into N
// round trips. Bounded: gives up after a.spin_limit passes, or as soon as another workgroup of this launch gave up
// (the device word then holds this launch's tag0), and records the give-up in the device word and in its host-mapped
// copy; the launch then runs to completion with invalid outputs instead of hanging, and the host reports it
// (sepvad_forward / sepvad_fused_status; k_istft_pair writes NaN outputs). Words of earlier launches' give-ups hold
// other tags, so a give-up never leaks into a later launch.
template <int N>
__device__ __forceinline__ void gpollt(const u64* const (&p)[N], const unsigned (&tag)[N], unsigned (&v)[N],
                                       const TcnArgs& a) {
  // the word a null entry reads instead: an unused word past GW_SUB4 in slot pair blockIdx.x (gran holds a slot pair per
  // member, >= the grid), a line of this workgroup's own -- not one word for the whole launch, which every wave of
  // every CU read on every poll pass (a single hot L2 line)
  const u64* const dummy = a.gran + (size_t)blockIdx.x * 2 * NGR + 2 * NGR - 4;
  unsigned spins = 0;
  for (;;) {
    u64 x[N];
#if TCN_POLL_SERIAL  // A/B switch: the round-2 form (each load inside its own `if (p[k])`: one round trip per word)
#pragma unroll
    for (int k = 0; k < N; ++k) {
      x[k] = 0;
      if (p[k] != nullptr) x[k] = __hip_atomic_load(p[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    (void)dummy;
#else
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = __hip_atomic_load(p[k] != nullptr ? p[k] : dummy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      v[k] = (unsigned)x[k];
      ok = ok && (p[k] == nullptr || (unsigned)(x[k] >> 32) == tag[k]);
    }
    if (ok) return;
    if (TCN_POLL_SLEEP) __builtin_amdgcn_s_sleep(TCN_POLL_SLEEP);
    if ((++spins & 255u) == 0 &&
        (spins > a.spin_limit || __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.tag0)) {
      if (spins > a.spin_limit) {  // diagnostics: the first timed-out wait of the launch {tag, workgroup, word}
        int k0 = 0;
#pragma unroll
        for (int k = N - 1; k >= 0; --k)
          if (p[k] != nullptr && (unsigned)(x[k] >> 32) != tag[k]) k0 = k;
        unsigned z = 0;
        if (__hip_atomic_compare_exchange_strong(a.err + 1, &z, tag[k0], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          __hip_atomic_store(a.err + 2, blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err + 3, (unsigned)((p[k0] - a.gran) & 0xffffffffu), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      giveup(a);
      return;
    }
  }
}
template <int N>
__device__ __forceinline__ void gpoll(const u64* const (&p)[N], unsigned tag, unsigned (&v)[N], const TcnArgs& a) {
  unsigned tg[N];
#pragma unroll
  for (int k = 0; k < N; ++k) tg[k] = tag;
  gpollt<N>(p, tg, v, a);
}

// Weight lo plane of the fp16x3 split stored as bytes (sepvad_internal.h WQ_*), widened to fp16 in registers:
// L8 (F16X3 only): the lo plane is e4m3 (sepvad_internal.h WQ_*), one 1 KB wave load per two K steps at
// voffl + 1024 * pair into rl[i / 2], widened to fp16 in registers (v_cvt_scalef32_pk_f16_fp8, 4 per step,
// scale 2^-WQ_LO_SHIFT) right before the step's MFMAs: 3 bytes per weight instead of 4.
// LQ = 2: the lo bytes are int8 steps of 2^-WQ_LO_SHIFT (stored biased, q + 128): v_perm_b32 builds the fp16 values
// 1024 + byte (0x64XX), and one packed fma scales and unbiases them -- exact (every result is a multiple of 2^-19).
template <int LQ>
__device__ __forceinline__ f16x8 lo8_widen(u32x4v q, int half) {
  constexpr float sc = 1.0f / (float)(1 << WQ_LO_SHIFT);
  const unsigned d0 = half ? q[2] : q[0], d1 = half ? q[3] : q[1];
  if constexpr (LQ == 1) {
    const h16x2 c0 = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(d0, sc, false);
    const h16x2 c1 = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(d0, sc, true);
    const h16x2 c2 = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(d1, sc, false);
    const h16x2 c3 = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(d1, sc, true);
    return f16x8{c0[0], c0[1], c1[0], c1[1], c2[0], c2[1], c3[0], c3[1]};
  } else {
    // v_perm_b32(src0, src1, sel): selector byte k picks byte sel_k of {src0:src1} (0..3 = src1, 4..7 = src0)
    constexpr unsigned M = 0x64646464u;
    const h16x2 s2 = {(_Float16)sc, (_Float16)sc}, o2 = {(_Float16)(-1152.0f * sc), (_Float16)(-1152.0f * sc)};
    h16x2 c[4];
    c[0] = __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(M, d0, 0x07010700u));  // bytes 0, 1 -> 0x64b0, 0x64b1
    c[1] = __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(M, d0, 0x07030702u));  // bytes 2, 3
    c[2] = __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(M, d1, 0x07010700u));
    c[3] = __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(M, d1, 0x07030702u));
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = __builtin_elementwise_fma(c[k], s2, o2);
    return f16x8{c[0][0], c[0][1], c[1][0], c[1][1], c[2][0], c[2][1], c[3][0], c[3][1]};
  }
}

// Hand-off word layout of one slot (k_tcn and k_tcn16). With TF-attention a block publishes four epochs (P1, P2, P3, P4), so P1 and P3
// share a slot parity, as do P2 and P4. P2 is not polled on its own (its words ride in the P3 round), so a member can
// publish P3 while a slower member still polls its P1 words, and P4 while a slower member still polls its P2 words:
// P3's words never overlap P1's, and P4's never overlap P2's. Every other same-parity pair is separated by a round
// that every member polls, which each member enters only after its reads of the earlier epoch.
constexpr int GW_STAT = 0;          // P1/P2: {sum lo, sum hi, sumsq lo, sumsq hi}
constexpr int GW_TOP = 4;           // P1: rows 0..dil-1      [dil][256]
constexpr int GW_BOT = 4 + 4 * CH;  // P1: rows 32-dil..31  [dil][256]
constexpr int GW_ROW = GW_BOT + 4 * CH;  // P3: per-channel sums over own frames [256]
constexpr int GW_COL = GW_ROW + CH;      // P3: per-frame channel sums [32]
constexpr int GW_P4 = 4;                 // P4: the moment record, 11 doubles as 22 words (clear of P2's GW_STAT)
// Two-level reductions of large groups (k_tcn, G > FG_TREE): the leaders' partial P3 row sums and P4 records, past
// every P1 word (without TF-attention a block has three epochs, so P1 and P4 share a slot parity every other block)
constexpr int GW_SUB3 = GW_COL + FR;     // [256] a leader's partial row sums
constexpr int GW_SUB4 = GW_SUB3 + CH;    // [22] a leader's partial moment record
static_assert(GW_SUB4 + 2 * NMOM <= NGR - 4 && GW_P4 >= GW_STAT + 4,
              "granule slot size (the last 4 words unused: gpollt's dummy word) / P2-P4 separation");


// One GEMM operand value into LDS in the format PRE multiplies: fp16 hi/lo split (F16X3), fp16 (F16) or
// bf16 bits (BF16, round to nearest even) in the hi plane.
template <int PRE>
__device__ __forceinline__ void split_store(_Float16* hi, _Float16* lo, int idx, float v) {
  if constexpr (PRE == PREC_F16X3) {
    const _Float16 h = (_Float16)v;
    hi[idx] = h;
    lo[idx] = (_Float16)(v - (float)h);
  } else if constexpr (PRE == PREC_F16) {
    hi[idx] = (_Float16)v;
  } else if constexpr (PRE == PREC_F32) {  // one fp32 plane (idx in floats)
    reinterpret_cast<float*>(hi)[idx] = v;
  } else {
    reinterpret_cast<__bf16*>(hi)[idx] = (__bf16)v;
  }
}

// two adjacent values (idx even): one 32-bit LDS store per plane
template <int PRE>
__device__ __forceinline__ void split_store2(_Float16* hi, _Float16* lo, int idx, float v0, float v1) {
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  if constexpr (PRE == PREC_F16X3) {
    const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
    *reinterpret_cast<f16x2*>(hi + idx) = f16x2{h0, h1};
    *reinterpret_cast<f16x2*>(lo + idx) = f16x2{(_Float16)(v0 - (float)h0), (_Float16)(v1 - (float)h1)};
  } else if constexpr (PRE == PREC_F16) {
    *reinterpret_cast<f16x2*>(hi + idx) = f16x2{(_Float16)v0, (_Float16)v1};
  } else {
    *reinterpret_cast<bf16x2*>(hi + idx) = bf16x2{(__bf16)v0, (__bf16)v1};
  }
}

// ---- packed fp32 (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32: two channels per instruction) ----
typedef float f32x2 __attribute__((ext_vector_type(2)));
#ifndef TCN_MIX
#define TCN_MIX 1  // round 6: lo parts by v_fma_mix (bitwise equal, -0.5 % k_tcn cycles, profiles/r06mix/)
#endif
// The fp16 lo parts of a pair, (f16)(v - (float)h) with hb = the pair's hi halves, as two v_fma_mix (hi read as f16,
// the difference rounded to f16 once): v - h is exact in fp32 (h is v rounded to fp16), so the bits equal the
// convert / subtract / convert form, in 2 instructions instead of 5. Inline asm (no builtin); the closing s_nop 1 covers
// a DPP or permlane reader of the result (split_store_rows_pk).
__device__ __forceinline__ unsigned lo_pair_mix(f32x2 v, unsigned hb) {
  unsigned r;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\ts_nop 1"
      : "=&v"(r) : "v"(v.x), "v"(v.y), "v"(hb));
  return r;
}
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) float lds_f32;
// An LDS address the compiler must materialise in a VGPR: loads at constant distances from it then use the ds
// instruction's 16-bit offset field (the H planes sit above 64 KB of LDS, so a folded constant base would not fit
// and every load would get its own address add).
__device__ __forceinline__ const float* lds_base(const float* p) {
  unsigned a = (unsigned)(size_t)(const lds_f32*)p;
  asm volatile("" : "+v"(a));
  return (const float*)(const lds_f32*)(size_t)a;
}
// PReLU(x) = x > 0 ? x : a x, as x + (a - 1) min(x, 0) (a2m1 = a - 1): two v_min_f32 and one v_pk_fma_f32 per pair
__device__ __forceinline__ f32x2 prelu2(f32x2 x, float a2m1) {
  const f32x2 mn = {fminf(x.x, 0.f), fminf(x.y, 0.f)};
  return __builtin_elementwise_fma(mn, f32x2{a2m1, a2m1}, x);
}
// Depthwise outputs of two adjacent input channels c, c+1 at one frame: y0 = (d[2c], d[2c+2]), y1 = (d[2c+1], d[2c+3])
// (q = 0, 1 of each channel) -> hidden 2c..2c+3 as one 8-byte store per GEMM operand plane (PRE format as split_store)
template <int PRE>
__device__ __forceinline__ void store_d4(_Float16* hi, _Float16* lo, f32x2 y0, f32x2 y1) {
  const f32x2 a = {y0.x, y1.x}, b = {y0.y, y1.y};  // hidden 2c, 2c+1 | 2c+2, 2c+3
  if constexpr (PRE == PREC_F16X3) {
    const f16x2v ha = __builtin_convertvector(a, f16x2v), hb = __builtin_convertvector(b, f16x2v);
    *reinterpret_cast<u32x2v*>(hi) = u32x2v{__builtin_bit_cast(unsigned, ha), __builtin_bit_cast(unsigned, hb)};
    if constexpr (TCN_MIX) {
      *reinterpret_cast<u32x2v*>(lo) = u32x2v{lo_pair_mix(a, __builtin_bit_cast(unsigned, ha)),
                                              lo_pair_mix(b, __builtin_bit_cast(unsigned, hb))};
      return;
    }
    const f16x2v la = __builtin_convertvector(a - __builtin_convertvector(ha, f32x2), f16x2v);
    const f16x2v lb = __builtin_convertvector(b - __builtin_convertvector(hb, f32x2), f16x2v);
    *reinterpret_cast<u32x2v*>(lo) = u32x2v{__builtin_bit_cast(unsigned, la), __builtin_bit_cast(unsigned, lb)};
  } else if constexpr (PRE == PREC_F16) {
    const f16x2v ha = __builtin_convertvector(a, f16x2v), hb = __builtin_convertvector(b, f16x2v);
    *reinterpret_cast<u32x2v*>(hi) = u32x2v{__builtin_bit_cast(unsigned, ha), __builtin_bit_cast(unsigned, hb)};
  } else {
    const bf16x2v ha = __builtin_convertvector(a, bf16x2v), hb = __builtin_convertvector(b, bf16x2v);
    *reinterpret_cast<u32x2v*>(hi) = u32x2v{__builtin_bit_cast(unsigned, ha), __builtin_bit_cast(unsigned, hb)};
  }
}
// Two values of one channel at two frames (LDS rows idx and idx + ld) in the PRE format of split_store
template <int PRE>
__device__ __forceinline__ void split_store_rows(_Float16* hi, _Float16* lo, int idx, int ld, f32x2 v) {
  if constexpr (PRE == PREC_F16X3) {
    const f16x2v h = __builtin_convertvector(v, f16x2v);
    const f16x2v l = __builtin_convertvector(v - __builtin_convertvector(h, f32x2), f16x2v);
    hi[idx] = h.x; hi[idx + ld] = h.y;
    lo[idx] = l.x; lo[idx + ld] = l.y;
  } else if constexpr (PRE == PREC_F16) {
    const f16x2v h = __builtin_convertvector(v, f16x2v);
    hi[idx] = h.x; hi[idx + ld] = h.y;
  } else if constexpr (PRE == PREC_F32) {  // (idx, ld in floats)
    reinterpret_cast<float*>(hi)[idx] = v.x; reinterpret_cast<float*>(hi)[idx + ld] = v.y;
  } else {
    const bf16x2v h = __builtin_convertvector(v, bf16x2v);
    reinterpret_cast<__bf16*>(hi)[idx] = h.x; reinterpret_cast<__bf16*>(hi)[idx + ld] = h.y;
  }
}
// split_store_rows with the lane pair (2c, 2c+1) packing its two channels into 32-bit stores: the even lane writes
// channels (m, m+1) of frame tl, the odd lane channels (m-1, m) of frame tl+1, each taking the partner's 16-bit value
// through one DPP swap (quad_perm [1,0,3,2]) and one v_perm: half the LDS store instructions of split_store_rows.
// idx = the lane's element for frame tl (as split_store_rows); every lane of the wave must take part (DPP).
template <int PRE>
__device__ __forceinline__ void split_store_rows_pk(_Float16* hi, _Float16* lo, int idx, int ld, f32x2 v, bool odd) {
  if constexpr (PRE == PREC_F32) {  // 32-bit values already: plain stores (idx, ld in floats)
    split_store_rows<PRE>(hi, lo, idx, ld, v);
    return;
  }
  const unsigned sel = odd ? 0x03020706u : 0x05040100u;  // odd: {partner.y, own.y}; even: {own.x, partner.x}
  const int at = odd ? idx + ld - 1 : idx;                // 4-byte aligned (m - 1 even / m even)
  auto put = [&](_Float16* plane, unsigned own) {
    const unsigned nbr = (unsigned)__builtin_amdgcn_update_dpp(0, (int)own, 0xb1, 0xf, 0xf, false);
    *reinterpret_cast<unsigned*>(plane + at) = __builtin_amdgcn_perm(nbr, own, sel);
  };
  if constexpr (PRE == PREC_F16X3) {
    const f16x2v h = __builtin_convertvector(v, f16x2v);
    put(hi, __builtin_bit_cast(unsigned, h));
    if constexpr (TCN_MIX) {
      put(lo, lo_pair_mix(v, __builtin_bit_cast(unsigned, h)));
      return;
    }
    const f16x2v l = __builtin_convertvector(v - __builtin_convertvector(h, f32x2), f16x2v);
    put(lo, __builtin_bit_cast(unsigned, l));
  } else if constexpr (PRE == PREC_F16) {
    put(hi, __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2v)));
  } else {
    put(hi, __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2v)));
  }
}
// resid_apply (device_common.h) on two frames of one channel: kc = {GN_a scale, shift, GN_b scale, shift}
template <int MODE>
__device__ __forceinline__ f32x2 resid_apply2(f32x2 o, f32x2 r, const float (&kc)[4]) {
  const f32x2 k0 = {kc[0], kc[0]}, k1 = {kc[1], kc[1]};
  if constexpr (MODE == LD_GN) {
    return __builtin_elementwise_fma(o, k0, k1);
  } else if constexpr (MODE == LD_RECURSIVE) {
    const f32x2 v = o + __builtin_elementwise_fma(o + r, k0, k1);
    return __builtin_elementwise_fma(v, f32x2{kc[2], kc[2]}, f32x2{kc[3], kc[3]});
  } else if constexpr (MODE == LD_RESIDUAL) {
    return o + __builtin_elementwise_fma(r, k0, k1);
  } else if constexpr (MODE == LD_ADD) {
    return o + r;
  } else {
    return o;
  }
}
// Depthwise weights and bias of input channels c, c+1 (c even) from a parameter blob: wv[q][k] = (w[2c+q][k],
// w[2c+2+q][k]), bv[q] = (b[2c+q], b[2c+2+q]). Scalar float reads (merged into wide LDS reads by the compiler):
// pairs built from the elements of a u32x4 vector read miscompile on this toolchain (the packed FMA gets one element
// broadcast through op_sel_hi).
__device__ __forceinline__ void dw_params2(const float* pm, int c, f32x2 (&wv)[2][3], f32x2 (&bv)[2]) {
  const float* wp = pm + PB_WD + 6 * c;
  const float* bp = pm + PB_BD + 2 * c;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
#pragma unroll
    for (int k = 0; k < 3; ++k) wv[q][k] = f32x2{wp[3 * q + k], wp[6 + 3 * q + k]};
    bv[q] = f32x2{bp[q], bp[2 + q]};
  }
}

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
// Lane exchanges of the recursive-halving reductions (spectral.hip k_vad1): swap lanes L <-> L ^ 16 (v_permlane16_swap)
// or L <-> L ^ 32 (v_permlane32_swap) between two registers. Inline asm: this hipcc's builtin pair result came back as the
// same register twice (tools/probe_src/halving.hip); "s_nop 1" covers the VALU-write -> permlane hazard.
__device__ __forceinline__ void swap16(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void swap32(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}
// Reduce-scatter of 16 values per lane over each 32-lane half of the wave: returns, in lane L, the sum over the 32
// lanes of L's half of value (L & 31) >> 1 (lanes 2k and 2k + 1 both hold value k). Recursive halving (one
// v_permlane16_swap level, DPP row_mirror / row_half_mirror / quad_perm levels, a final pair add): 8 swaps + 8 + 4 x 3 +
// 2 x 3 + 3 + 1 VALU instead of 16 DPP chains of 5 (half_total). A fixed tree: deterministic.
__device__ __forceinline__ float rs16_half(float (&x)[16], int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = x[j], b = x[j + 8];
    swap16(a, b);  // bit 4 clear: keeps values 0..7 (own + partner's), set: 8..15
    x[j] = a + b;
  }
  auto level = [&](auto CTRL, int msk, int n) {
    constexpr int C = decltype(CTRL)::value;
    const bool hi = (lane & msk) != 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < n / 2) {
        const float send = hi ? x[j] : x[j + n / 2];
        const float keep = hi ? x[j + n / 2] : x[j];
        x[j] = keep + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), C, 0xf, 0xf, false));
      }
    }
  };
  level(std::integral_constant<int, 0x140>{}, 8, 8);  // row_mirror: lane i <-> 15 - i
  level(std::integral_constant<int, 0x141>{}, 4, 4);  // row_half_mirror: i <-> 7 - i
  level(std::integral_constant<int, 0x4e>{}, 2, 2);   // quad_perm [2,3,0,1]
  return x[0] + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x[0]), 0xb1, 0xf, 0xf, false));
}
// Reduce-scatter of 16 values per lane over all 64 lanes: returns, in lane L, the wave sum of value L >> 2 (the four
// lanes of a quad hold the same sum). Levels: v_permlane32_swap, v_permlane16_swap, DPP row_mirror, row_half_mirror,
// then two quad adds: 8 + 8 + 4 + 4 + 2 x 3 + 3 + 2 VALU instead of 16 chains of 6 DPP adds (half_total + row_bcast).
__device__ __forceinline__ float rs16_wave(float (&x)[16], int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = x[j], b = x[j + 8];
    swap32(a, b);  // lane bit 5 clear: keeps values 0..7, set: 8..15
    x[j] = a + b;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float a = x[j], b = x[j + 4];
    swap16(a, b);  // lane bit 4
    x[j] = a + b;
  }
  auto level = [&](auto CTRL, int msk, int n) {
    constexpr int C = decltype(CTRL)::value;
    const bool hi = (lane & msk) != 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < n / 2) {
        const float send = hi ? x[j] : x[j + n / 2];
        const float keep = hi ? x[j + n / 2] : x[j];
        x[j] = keep + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), C, 0xf, 0xf, false));
      }
    }
  };
  level(std::integral_constant<int, 0x140>{}, 8, 4);  // row_mirror (lane bit 3)
  level(std::integral_constant<int, 0x141>{}, 4, 2);  // row_half_mirror (lane bit 2)
  float v = x[0];
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4e, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xb1, 0xf, 0xf, false));
  return v;
}
// Sum over the 64 lanes (+ row_bcast:31), returned wave-uniform (lane 63).
__device__ __forceinline__ float wave_total(float v) {
  v = half_total(v);
  v += dpp_f<0x143>(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const u64 b = __builtin_bit_cast(u64, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((u64)hi << 32) | lo);
}
// This thread's workgroup-relative id, recomputed where it is needed: the wave index from a wave-uniform
// SGPR, the lane from v_mbcnt (volatile asm: never hoisted). Values derived from threadIdx.x before the
// utterance loop stay live across all of it; at 256 VGPRs hipcc spills them to scratch, and the first
// reloads of a launch (behind the scratch spill stores, vmcnt(0)) cost ~15 us of cold-start latency.
__device__ __forceinline__ int fresh_tid(int wave_s) {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return wave_s * 64 + l;
}

// The kernel arguments re-read from the kernarg segment (scalar loads through an opaque pointer) where
// the prologue uses them: pointers held in registers across the utterance loop end up in VGPRs and are
// spilled to scratch at this register pressure.
typedef const __attribute__((address_space(4))) TcnArgs* KArgs;
__device__ __forceinline__ KArgs kargs() {
  KArgs p = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// {sum, sumsq} over the G members' statistic words (member mm: doubles 2mm, 2mm+1 of gw), returned wave-uniform:
// lane l of half h (h = 0: sums, 1: sums of squares) adds members l, l + 32, ... in order, then a fixed xor tree over
// the half's 32 lanes; lanes 0 / 32 hold the results (a fixed order: bitwise reproducible). Large groups only (the
// polling wave finishes groups up to FG_WAVE in member order, member_moments_w).
__device__ __forceinline__ double2 member_sums2(const unsigned* gw, int G, int lane) {
  const double* gd = reinterpret_cast<const double*>(gw);
  const int h = lane >> 5, l = lane & 31;
  double s = 0.0;
  for (int mm = l; mm < G; mm += 32) s += gd[2 * mm + h];
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  return double2{readlane_d(s, 0), readlane_d(s, 32)};
}
// GroupNorm {mean, rstd} from the statistic words polled by one wave: lane base + 4 mm + {0, 1, 2, 3} holds
// member mm's {sum lo, sum hi, sumsq lo, sumsq hi}. Sums in member order, wave-uniform (readlane). This is NOT
// member_sums2's order (strided per-lane sums, then an xor tree): the two are different fixed orders, each chosen by
// its instantiation (groups up to FG_WAVE members here, the long-group instantiation LG there), and each is bitwise
// reproducible for a given G.
__device__ __forceinline__ void member_moments_w(unsigned w, int base, int G, double inv, float eps, float& mu, float& rs) {
  double s = 0.0, ss = 0.0;
  for (int mm = 0; mm < G; ++mm) {
    const int l = base + 4 * mm;
    const unsigned a0 = __builtin_amdgcn_readlane(w, l), a1 = __builtin_amdgcn_readlane(w, l + 1);
    const unsigned b0 = __builtin_amdgcn_readlane(w, l + 2), b1 = __builtin_amdgcn_readlane(w, l + 3);
    s += __builtin_bit_cast(double, ((u64)a1 << 32) | a0);
    ss += __builtin_bit_cast(double, ((u64)b1 << 32) | b0);
  }
  gn_moments_f(s, ss, inv, eps, mu, rs);
}

// p[0] + p[s] + ... + p[(n - 1) s] summed in index order (the order of the plain loop, so the same bits), the LDS
// loads issued 8 at a time: a runtime-count loop otherwise waits for each load before its add (a group of 118
// members' records took ~100 cycles per member).
__device__ __forceinline__ double seq_sum_lds(const double* p, int s, int n) {
  double acc = 0.0;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(k + u) * s];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; k < n; ++k) acc += p[k * s];
  return acc;
}

// Diagnostics (SEPVAD_TCN_DELAY = n): member 0 of every group sleeps n x ~8k cycles at the call sites (after a
// publish, before the matching polls), so the other members run ahead into the next epochs: the hand-off words of
// different epochs must not alias while a late member still polls them (tcn_kernel.h GW_*). 0 in production.
__device__ __forceinline__ void tcn_delay(int g) {
  const unsigned n = kargs()->dbg_delay;
  if (n != 0 && g == 0)
    for (unsigned k = 0; k < n; ++k) __builtin_amdgcn_s_sleep(127);
}

}  // namespace sepvad
