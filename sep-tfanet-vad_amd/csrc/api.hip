// C ABI of libsepvad.so (include/sepvad.h): weight folding/packing at create time and the
// stream-ordered launch sequence of one SeparationModel.forward (reference model/model.py:402-461).
//
// Per forward (B utterances, T frames, 24 blocks):
//   k_stft -> k_gate -> 24 x [ conv1d GEMM (loader: previous block's residual update)
//                              -> k_dw_stats (d, split) -> res_out GEMM (reg2 folded into W / epilogue)
//                              -> k_att_stats ]
//   -> k_head_stats -> output GEMM (loader: residual update, PReLU, GN) -> k_vad1 -> k_istft
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include "build/build_id.h"  // SEPVAD_BUILD_ID (Makefile: buildid.py)

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../../include/sepvad.h"
#include "sepvad_internal.h"

using namespace sepvad;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(SEPVAD_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));         \
  } while (0)

// Packed pointwise-conv weight: fp32 [M][K] and the fp16 split of the row-scaled copy.
struct PackedW {
  size_t w32 = 0, whi = 0, wlo = 0, scale = 0;
  size_t fhi = 0, flo = 0;  // fused-TCN copies in MFMA B-fragment order (see pack_pointwise)
  size_t wbf = 0, fbf = 0;  // bf16 bits of the row-scaled weight, row-major and in fragment order (PREC_BF16)
  size_t fl8 = 0;           // e4m3 lo plane in K-step-pair fragment order (bytes, stored in hblob; sepvad_internal.h WQ_*)
  size_t fi8 = 0;           // ... the same as int8 steps of 2^-WQ_LO_SHIFT, biased by 128
  size_t fq = 0;            // the int8 lo plane's values (q * 2^-WQ_LO_SHIFT, exact) as fp16 in flo's order (two slices)
  size_t ff32 = 0;          // the row-scaled fp32 weight in the same fragment order (float blob; fused PREC_F32)
};

struct BlockOff {
  PackedW w1, w2;
  size_t b1, g1, be1, wd, bd, b2, g2, be2, attp, lna_g, lna_b, lnb_g, lnb_b;
  size_t fc2;  // res_out with reg2 folded in: w2 = W*gamma2, b2 = bias + W*beta2, fc2[m] = sum_k w2[m][k]
  float a1, a2;
  int dil;
  double wsum[5];  // {Σγa, Σβa, Σβa², Σγa·βa, Σγa²} of ln_first (closed-form recursive-LN stats)
  float sx;        // 2^-ex: fp16 range scale of the conv1d A operand (x'), undone by w1.scale (range guard)
  float eps2;      // reg2 eps * 2^-2ed: d is produced scaled by 2^-ed (dconv weights/bias pre-scaled)
};

struct Workspace {
  int Bmax = 0, Tpmax = 0;
  char* base = nullptr;
  size_t bytes = 0;
  float2* X; float* specdb; float* S0; float* O[2]; float* A; float* R;
  float* masks; float* colsum; float* rowsum; float* at; float* af; float* vy; float* vad;
  float* vP;  // [B][2][Tp][HEAD_VAD_N] VAD conv1_1 tap products from k_tcn's output head (fused schedule)
  __half* Dhi; __half* Dlo; float* D32;  // res_out operand d (fp16 split planes, or fp32, same bytes)
  // partial records of the statistics producers (deterministic per-workgroup sums)
  double* rec_gate; double* rec_g1; double* rec_dw; double* rec_mom; double* rec_hs; double* rec_vad;
};

// The workspace slice of utterances [b0, b0 + Bc) at padded length Tp: every per-utterance array
// is utterance-major, so a chunk is a pointer offset (no copies).
Workspace ws_view(const Workspace& w, int b0, int Tp) {
  Workspace v = w;
  const size_t u = (size_t)b0 * Tp;
  v.X = w.X + u * NBIN; v.specdb = w.specdb + u * SPEC_LD; v.S0 = w.S0 + u * CH;
  v.O[0] = w.O[0] + u * CH; v.O[1] = w.O[1] + u * CH; v.A = w.A + u * CH; v.R = w.R + u * CH;
  v.masks = w.masks + u * MOUT_PAD;
  v.Dhi = w.Dhi + u * HID; v.Dlo = w.Dlo + u * HID; v.D32 = w.D32 + u * HID;
  v.colsum = w.colsum + u * (CH / TILE); v.rowsum = w.rowsum + (size_t)b0 * (Tp / TILE) * CH;
  v.at = w.at + u; v.af = w.af + (size_t)b0 * CH; v.vy = w.vy + u * 2 * 4; v.vad = w.vad + u * 2;
  v.vP = w.vP + u * 2 * HEAD_VAD_N;
  v.rec_gate = w.rec_gate + (size_t)b0 * (Tp / GATE_ROWS) * 2;
  v.rec_g1 = w.rec_g1 + (size_t)b0 * (Tp / TILE) * (CH / TILE) * 2;
  v.rec_dw = w.rec_dw + (size_t)b0 * (Tp / STAT_ROWS) * 2;
  v.rec_mom = w.rec_mom + (size_t)b0 * (Tp / STAT_ROWS) * NMOM;
  v.rec_hs = w.rec_hs + (size_t)b0 * (Tp / STAT_ROWS) * 2;
  v.rec_vad = w.rec_vad + (size_t)b0 * 2 * (Tp / VAD_ROWS) * 2;
  return v;
}

constexpr int MAX_SPLIT = 4;
constexpr int TCLK_RECS = 4096;  // SEPVAD_TCN_CLOCK records kept (ring)

// Per caller-stream state (include/sepvad.h: concurrent forwards on different streams of one handle are
// allowed): the workspace, the fused TCN's hand-off words, launch salt and give-up words. Weights are
// shared and read-only.
struct StreamCtx {
  void* stream = nullptr;
  Workspace ws;
  unsigned long long* tgran = nullptr;  // hand-off words [gran_slots][2][NGR]
  unsigned* terr = nullptr;             // device word: tag0 of the last launch whose hand-off wait gave up
  unsigned* herr = nullptr;             // host-mapped copy (pinned, written by the kernel)
  unsigned* herr_dev = nullptr;         // its device address
  unsigned reported = 0;                // last give-up word already returned to the caller
  unsigned pending = 0;                 // a give-up seen when the salt wrapped (words re-zeroed), not yet reported
  unsigned tsalt = 0;                   // launch counter (hand-off tag salt)
  int last_B = 0, last_N = 0;           // shape of the last forward on this stream (sepvad_side_outputs)
  long long seq = 0;                    // handle-wide id of the last forward on this stream (side outputs are tied to one)
  unsigned long long used = 0;          // LRU stamp (context cap, get_ctx)
};

}  // namespace

struct sepvad_model {
  SepVadConfig cfg{};
  int device = 0;
  int nblk = 0;
  int prec = PREC_F16X3;
  float* dparams = nullptr;   // packed fp32 weights (device)
  __half* dhalf = nullptr;    // packed fp16 split weights (device)
  std::vector<BlockOff> blk;
  size_t win_in = 0, win_out = 0, win_inv = 0, tw = 0;
  size_t ln_g = 0, ln_b = 0;
  PackedW wout;
  size_t out_g = 0, out_b = 0, bo = 0;
  // k_tcn's copy of the output head: speaker q's 257 rows at rows [288 q, 288 q + 257) (zero rows to 288); its MFMA
  // tiles are rows [288 q, 288 q + 256), bin 256 of each speaker is out_ny (fp32 [2][CH] + bias [2]); the VAD conv1_1
  // as a second GEMM on each masks tile (B[c][4 k + o] = w1[o][c][k], 20 of 32 columns, speaker-local channels
  // c < 256; vad_ny[4 k + o] = w1[o][256][k])
  PackedW wout_spk, vadw;
  size_t bo_spk = 0, out_nyw = 0, out_nyb = 0, vad_ny = 0;
  float vad_sx = 1.f;  // fp16 range scale of the VAD GEMM's A operand (undone by vadw.scale)
  float out_a = 0.f;
  size_t v_w1 = 0, v_b1 = 0, v_g = 0, v_b = 0, v_w2 = 0;
  float v_a = 0.f, v_b2 = 0.f;
  size_t gate = 0;
  bool same_stft_window = true;
  // batch split: utterance chunks of one forward run concurrently on internal streams (fork/join
  // on the caller's stream); the chunks' kernels fill each other's ramp/drain bubbles
  int split = 1;
  hipStream_t sub[MAX_SPLIT] = {};
  hipEvent_t fork = nullptr, join[MAX_SPLIT] = {};
  // fused persistent TCN (tcn_kernel.h): one launch for all blocks when the GEMMs are not fp32 and T <= 8192
  bool fused = true;
  int tcn_cap = 0;              // co-resident k_tcn workgroups (CUs x workgroups per CU), max over precisions
  int tcn_cap_p[4] = {};        // ... per operand precision (PREC_*)
  __half* twf = nullptr;        // [nblk][WF_BLOCK] fragment-ordered fp16 hi/lo weights (F16X3, SEPVAD_WLO_F16)
  __half* twq[3] = {};          // [nblk][WQ_BLOCK] fragment-ordered fp16 hi + byte lo weights: [1] e4m3, [2] int8
  __half* twfq = nullptr;       // [nblk][WF_BLOCK] as twf, the lo plane holding the int8 plane's values (two slices)
  int lo8 = 2;                  // k_tcn's weight lo plane: 0 fp16, 1 e4m3, 2 int8 (default); SEPVAD_WLO / sepvad_set_weight_lo
  int tcn_cap_q[3] = {};        // co-resident capacity of the byte-lo k_tcn variants
  int tcn2_cap_p[4] = {};       // ... of the two-slice (64-frame) k_tcn, per precision
  int tcn2_cap_q[3] = {};       // ... and per byte-lo variant
  int gran_slots = 0;           // member slot pairs of a context's hand-off words: max(capacity, 2 x two-slice capacity)
  __half* twf16 = nullptr;      // [nblk][WS_BLOCK] fragment-ordered fp16 weights (F16)
  __half* twbf = nullptr;       // [nblk][WS_BLOCK] fragment-ordered bf16 bits (BF16)
  float* twf32 = nullptr;       // [nblk][WS32_BLOCK / 2] fragment-ordered fp32 weights (F32)
  float* tprm = nullptr;        // [nblk][PB_SIZE] parameter blobs
  bool last_fused = false;
  float out_sx = 1.f;           // fp16 range scale of the head GEMM's A operand (undone by wout.scale)
  int last_nsl = 1;             // 32-frame slices per k_tcn workgroup of the last fused forward (1 or 2)
  float* tdump = nullptr;       // parity probe buffer of the fused TCN (sepvad_set_tcn_dump), caller-owned
  // caller-stream contexts (workspace, hand-off words, give-up words); `mu` serialises the host-side
  // enqueue of concurrent callers (the kernels of different streams still overlap on the device)
  std::vector<std::unique_ptr<StreamCtx>> ctx;
  std::mutex mu;
  unsigned long long use_clock = 0;  // LRU clock of the contexts (under mu)
  long long fwd_seq = 0;             // forwards enqueued on this handle (under mu): StreamCtx::seq
  int res_B = 0, res_N = 0;     // sepvad_reserve hint: every context's workspace is sized at least this
  unsigned long long* kprobe = nullptr;  // SEPVAD_TAIL_PROBE diagnostics: [workgroups][8]
  unsigned long long* tprobe = nullptr;  // SEPVAD_TCN_PROBE diagnostics: [tcn_cap][nblk][16]
  unsigned long long* tclk = nullptr;    // SEPVAD_TCN_CLOCK diagnostics: [TCLK_RECS][8] per-launch clock records
  long long tclk_n = 0;                  // k_tcn launches recorded so far
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev;
  double gemm_ms = 0.0, g2_ms = 0.0, total_ms = 0.0;
  int gemm_launches = 0, g2_launches = 0;
  // diagnostics: per-workgroup timestamps of one block's two GEMMs (env SEPVAD_PROBE_BLOCK=<i>,
  // written to SEPVAD_PROBE_OUT after each forward)
  int probe_blk = -1;
  unsigned long long* probe = nullptr;
  size_t probe_n = 0;

  const float* P(size_t off) const { return dparams + off; }
  const __half* H(size_t off) const { return dhalf + off; }
};

namespace {

struct TensorMap {
  std::unordered_map<std::string, std::pair<const float*, int64_t>> m;
  const float* get(const std::string& k, int64_t numel) const {
    auto it = m.find(k);
    if (it == m.end()) { g_err = "missing state_dict entry: " + k; return nullptr; }
    if (it->second.second != numel) {
      g_err = "state_dict entry " + k + " has " + std::to_string(it->second.second) +
              " elements, expected " + std::to_string(numel);
      return nullptr;
    }
    return it->second.first;
  }
};

struct Packer {
  std::vector<float> blob;
  std::vector<__half> hblob;
  size_t add(const float* p, size_t n) {
    size_t off = blob.size();
    blob.insert(blob.end(), p, p + n);
    while (blob.size() % 4) blob.push_back(0.f);  // 16-byte aligned arrays (float4 loads)
    return off;
  }
  size_t add(const std::vector<float>& v) { return add(v.data(), v.size()); }
  size_t addh(const std::vector<__half>& v) {
    size_t off = hblob.size();
    hblob.insert(hblob.end(), v.begin(), v.end());
    while (hblob.size() % 8) hblob.push_back(__float2half_rn(0.f));
    return off;
  }
};

// torch.nn.utils.weight_norm (dim=0): w = v * (g / ||v||_2 over all dims but 0).
std::vector<float> fold_wn(const float* g, const float* v, int cout, int rest) {
  std::vector<float> w((size_t)cout * rest);
  for (int o = 0; o < cout; ++o) {
    double s = 0.0;
    for (int i = 0; i < rest; ++i) s += (double)v[(size_t)o * rest + i] * v[(size_t)o * rest + i];
    const float nrm = (float)std::sqrt(s);
    const float scale = g[o] / nrm;
    for (int i = 0; i < rest; ++i) w[(size_t)o * rest + i] = v[(size_t)o * rest + i] * scale;
  }
  return w;
}

// float -> bf16 bits, round to nearest even (finite inputs: weights)
__half bf16_bits(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
  const unsigned short b = (unsigned short)u;
  __half h;
  std::memcpy(&h, &b, 2);
  return h;
}

// float -> e4m3fn (OCP FP8: 1-4-3, bias 7, max 448 = 0x7e, 0x7f NaN, no inf): round to nearest even, saturating.
// The gfx950 conversions (v_cvt_scalef32_pk_f16_fp8) read the same OCP format.
}  // namespace
uint8_t sepvad::e4m3_rn(float x) {
  if (std::isnan(x)) return 0x7f;
  const uint8_t sg = std::signbit(x) ? 0x80 : 0x00;
  const double a = std::fabs((double)x);
  if (a >= 448.0) return sg | 0x7e;
  if (a < std::ldexp(1.0, -6)) {                       // subnormal range: m * 2^-9, m = 0..8 (8 = smallest normal)
    const int m = (int)std::nearbyint(std::ldexp(a, 9));  // the default rounding mode: to nearest even
    return sg | (uint8_t)m;
  }
  int k = 0;
  (void)std::frexp(a, &k);                             // a = f * 2^k, f in [0.5, 1): exponent E = k - 1
  int E = k - 1;
  int q = (int)std::nearbyint(std::ldexp(a, 3 - E));   // 8..16
  if (q == 16) { q = 8; ++E; }
  if (E > 8 || (E == 8 && q > 14)) return sg | 0x7e;   // rounded past 448: saturate
  return sg | (uint8_t)(((E + 7) << 3) | (q - 8));
}
namespace {

// [cout][cin] fp32 -> zero-padded [mpad][cin] fp32 + the fp16 hi/lo split of each row scaled by
// 2^-e (e chosen so the row's max |w| lands in [0.5, 1)); scale[m] = 2^(e + col_e) undoes it exactly, and
// also the 2^-col_e the GEMM applies to its A operand before splitting it (range guard, see range_exp).
// int8 step of a lo residual (|lo| <= 2^-12 -> |q| <= 128; +128, a tie at half an ulp of hi, saturates to 127)
int lo_q(float lo) {
  const double q = std::nearbyint(std::ldexp((double)lo, WQ_LO_SHIFT));
  return (int)std::max(-128.0, std::min(127.0, q));
}

PackedW pack_pointwise(Packer& pk, const std::vector<float>& w, int cout, int cin, int mpad, int col_e = 0) {
  PackedW p;
  std::vector<float> w32((size_t)mpad * cin, 0.f), sc(mpad, 1.f);
  std::vector<__half> hi((size_t)mpad * cin), lo((size_t)mpad * cin), bf((size_t)mpad * cin);
  std::vector<float> lo32((size_t)mpad * cin);  // the exact fp32 residual (source of the e4m3 lo plane)
  std::vector<float> srow(mpad, 1.f);           // the row scale 2^-e
  for (int o = 0; o < mpad; ++o) {
    float mx = 0.f;
    if (o < cout)
      for (int i = 0; i < cin; ++i) mx = std::max(mx, std::fabs(w[(size_t)o * cin + i]));
    int e = 0;
    if (mx > 0.f) { (void)std::frexp(mx, &e); }  // mx = f * 2^e, f in [0.5, 1)
    const float s = std::ldexp(1.f, -e);
    srow[o] = s;
    sc[o] = std::ldexp(1.f, e + col_e);
    for (int i = 0; i < cin; ++i) {
      const float v = o < cout ? w[(size_t)o * cin + i] : 0.f;
      w32[(size_t)o * cin + i] = v;
      const float vs = v * s;
      const __half hh = __float2half_rn(vs);
      hi[(size_t)o * cin + i] = hh;
      lo32[(size_t)o * cin + i] = vs - __half2float(hh);
      lo[(size_t)o * cin + i] = __float2half_rn(lo32[(size_t)o * cin + i]);
      bf[(size_t)o * cin + i] = bf16_bits(vs);
    }
  }
  p.w32 = pk.add(w32);
  p.scale = pk.add(sc);
  p.whi = pk.addh(hi);
  p.wlo = pk.addh(lo);
  p.wbf = pk.addh(bf);
  // k_tcn streams each wave's 32 output rows as consecutive 1 KB fragments (v_mfma_f32_32x32x16_f16
  // B operand): [mpad/32 row tiles][cin/16 K steps][64 lanes][8 halves], lane l -> row 32*mt + (l & 31),
  // k = 16*s + 8*(l >> 5) + j.
  if (mpad % 32 == 0 && cin % 16 == 0) {
    std::vector<__half> fh((size_t)mpad * cin), fl((size_t)mpad * cin), fb((size_t)mpad * cin), fqv((size_t)mpad * cin);
    std::vector<float> ff((size_t)mpad * cin);
    size_t q = 0;
    for (int mt = 0; mt < mpad / 32; ++mt)
      for (int st = 0; st < cin / 16; ++st)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j, ++q) {
            const size_t src = (size_t)(32 * mt + (l & 31)) * cin + 16 * st + 8 * (l >> 5) + j;
            fh[q] = hi[src];
            fl[q] = lo[src];
            fb[q] = bf[src];
            fqv[q] = __float2half_rn(std::ldexp((float)lo_q(lo32[src]), -WQ_LO_SHIFT));  // exact in fp16
            // exact: a power-of-two row scale (PREC_F32: v_mfma_f32_32x32x2_f32 pairs k = 8 h + j, tcn_kernel.h)
            ff[q] = w32[src] * srow[src / cin];
          }
    p.ff32 = pk.add(ff);
    p.fhi = pk.addh(fh);
    p.flo = pk.addh(fl);
    p.fbf = pk.addh(fb);
    p.fq = pk.addh(fqv);
    // e4m3 lo plane: lane l, K-step pair pr -> 16 bytes: j = 0..7 of step 2 pr, then of step 2 pr + 1
    if ((cin / 16) % 2 == 0) {
      std::vector<uint8_t> f8((size_t)mpad * cin), i8((size_t)mpad * cin);
      size_t b = 0;
      for (int mt = 0; mt < mpad / 32; ++mt)
        for (int pr = 0; pr < cin / 32; ++pr)
          for (int l = 0; l < 64; ++l)
            for (int h = 0; h < 2; ++h)
              for (int j = 0; j < 8; ++j, ++b) {
                const size_t src = (size_t)(32 * mt + (l & 31)) * cin + 16 * (2 * pr + h) + 8 * (l >> 5) + j;
                f8[b] = e4m3_rn(lo32[src] * (float)(1 << WQ_LO_SHIFT));  // exact power-of-two scaling
                // int8: |lo| <= 2^-12 -> |q| <= 128; +128 (a tie at half an ulp of hi) saturates to 127
                i8[b] = (uint8_t)(lo_q(lo32[src]) + 128);
              }
      std::vector<__half> f8h(f8.size() / 2);
      std::memcpy(f8h.data(), f8.data(), f8.size());
      p.fl8 = pk.addh(f8h);
      std::memcpy(f8h.data(), i8.data(), i8.size());
      p.fi8 = pk.addh(f8h);
    }
  }
  return p;
}

// Range guard of the fp16 split: an fp16 plane holds |x| up to 65504, and the lo plane
// keeps full relative precision only for |x| >= 2^-3 (below that it becomes subnormal). Every A operand
// of the pointwise GEMMs is an affine image of GroupNorm-normalised data (x' = GN_b(..) or o + GN_c(..),
// d = PReLU(dconv(GN1(h))), the head's GN_out(PReLU(x'))), so its magnitude is fixed by the GN affines and
// weights, not by the utterance: |y_k| <~ |gamma_k| * NSIG + |beta_k| for normalised values within NSIG.
// Each operand is therefore scaled by a static power of two 2^-e that brings that bound into [0.5, 1)
// and the inverse is folded into the weights' per-row scale (or, for d, into the dconv weights, with the
// reg2 eps rescaled by 2^-2e): exact in fp32 arithmetic, bitwise neutral wherever nothing under- or
// overflowed, and it keeps weights scaled by 1e-3 or 1e3 at fp32-equivalent accuracy (tests).
constexpr double NSIG = 4.0;
double gn_bound(const float* g, const float* b, int n) {
  double m = 0.0;
  for (int k = 0; k < n; ++k) m = std::max(m, std::fabs((double)g[k]) * NSIG + std::fabs((double)b[k]));
  return m;
}
int range_exp(double bound) {
  if (!(bound > 0.0) || !std::isfinite(bound)) return 0;
  int e = 0;
  (void)std::frexp(bound, &e);  // bound = f * 2^e, f in [0.5, 1)
  return std::max(-60, std::min(60, e));
}

int ws_reserve(StreamCtx* c, int B, int N) {
  const int T = 1 + N / HOP;
  const int Tp = round_up(T, TILE);
  Workspace& w = c->ws;
  if (B <= w.Bmax && Tp <= w.Tpmax) return SEPVAD_OK;
  const int Bm = std::max(B, w.Bmax), Tm = std::max(Tp, w.Tpmax);
  if (w.base) { (void)hipFree(w.base); w.base = nullptr; w.Bmax = w.Tpmax = 0; }
  const size_t bt = (size_t)Bm * Tm;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) / 256 * 256; return o; };
  const size_t oX = take(bt * NBIN * 8), oSpec = take(bt * SPEC_LD * 4), oS0 = take(bt * CH * 4);
  const size_t oO0 = take(bt * CH * 4), oO1 = take(bt * CH * 4), oA = take(bt * CH * 4), oR = take(bt * CH * 4);
  const size_t oM = take(bt * MOUT_PAD * 4), oD = take(bt * HID * 4);
  const size_t oCs = take(bt * (CH / TILE) * 4), oRs = take((size_t)Bm * (Tm / TILE) * CH * 4);
  const size_t oAt = take(bt * 4), oAf = take((size_t)Bm * CH * 4), oVy = take(bt * 2 * 4 * 4), oV = take(bt * 2 * 4);
  const size_t oRg = take(bt / GATE_ROWS * 16 + 16), oR1 = take((size_t)Bm * (CH / TILE) * (Tm / TILE) * 16);
  const size_t oRd = take(bt / STAT_ROWS * 16 + 16), oRm = take(bt / STAT_ROWS * NMOM * 8 + 16);
  const size_t oRh = take(bt / STAT_ROWS * 16 + 16), oRv = take(bt * 2 / VAD_ROWS * 16 + 16);
  const size_t oVp = take(bt * 2 * HEAD_VAD_N * 4);
  char* base = nullptr;
  HIPCHK(hipMalloc(&base, off));
  // zeroed on the context's own stream, ahead of the forward that reserved it: a null-stream hipMemset is not
  // ordered with a non-blocking caller stream, and once zeroed the workspace of a concurrent forward's first launch
  // mid-run (tests/test_gpu_boundary.py::test_two_streams_concurrently_match_serial, round 4)
  HIPCHK(hipMemsetAsync(base, 0, off, (hipStream_t)c->stream));
  w.base = base; w.bytes = off; w.Bmax = Bm; w.Tpmax = Tm;
  w.X = (float2*)(base + oX); w.specdb = (float*)(base + oSpec); w.S0 = (float*)(base + oS0);
  w.O[0] = (float*)(base + oO0); w.O[1] = (float*)(base + oO1); w.A = (float*)(base + oA);
  w.R = (float*)(base + oR); w.masks = (float*)(base + oM);
  w.Dhi = (__half*)(base + oD); w.Dlo = w.Dhi + bt * HID; w.D32 = (float*)(base + oD);
  w.colsum = (float*)(base + oCs); w.rowsum = (float*)(base + oRs); w.at = (float*)(base + oAt);
  w.af = (float*)(base + oAf); w.vy = (float*)(base + oVy); w.vad = (float*)(base + oV);
  w.rec_gate = (double*)(base + oRg); w.rec_g1 = (double*)(base + oR1); w.rec_dw = (double*)(base + oRd);
  w.rec_mom = (double*)(base + oRm); w.rec_hs = (double*)(base + oRh); w.rec_vad = (double*)(base + oRv);
  w.vP = (float*)(base + oVp);
  return SEPVAD_OK;
}

// Restores the caller's current HIP device on scope exit (torch shares this runtime).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int ev_record(sepvad_model* h, hipStream_t s) {
  if (!h->timing) return 0;
  hipEvent_t e;
  HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventRecord(e, s));
  h->ev.push_back(e);
  return 0;
}

void set_weights(const sepvad_model* h, GemmArgs& g, const PackedW& w) {
  g.prec = h->prec;
  g.ascale = 1.f;
  g.W32 = h->P(w.w32);
  g.Whi = h->H(w.whi);
  g.Wlo = h->H(w.wlo);
  g.Wbf = h->H(w.wbf);
  g.wscale = h->P(w.scale);
}

// The residual-stream transform that turns (o_i, r_i) of block i into the next block input.
GnSrc gn_src(const double* rec, int nrec, int rstride, int roff, const float* g, const float* be, float eps) {
  GnSrc s;
  s.rec = rec; s.nrec = nrec; s.rstride = rstride; s.roff = roff; s.g = g; s.be = be; s.eps = eps;
  return s;
}

LoadSpec residual_spec(const sepvad_model* h, const Workspace& w, int i, const float* O, const float* R, int Tp) {
  LoadSpec ld{};
  ld.X = O; ld.X2 = R;
  if (h->cfg.tf_attention) { ld.at = w.at; ld.af = w.af; }
  const BlockOff& bo = h->blk[i];
  if (h->cfg.ln_mode == SEPVAD_LN_RECURSIVE) {
    ld.mode = LD_RECURSIVE;
    ld.gn = gn_src(w.rec_mom, Tp / STAT_ROWS, NMOM, 0, h->P(bo.lna_g), h->P(bo.lna_b), 1e-5f);
    ld.g2 = h->P(bo.lnb_g); ld.be2 = h->P(bo.lnb_b); ld.eps2 = 1e-5f;
    for (int j = 0; j < 5; ++j) ld.wsum[j] = bo.wsum[j];
  } else if (h->cfg.ln_mode == SEPVAD_LN_RESIDUAL) {
    ld.mode = LD_RESIDUAL;  // (Σr', Σr'²) at offsets 2, 3 of the moment record
    ld.gn = gn_src(w.rec_mom, Tp / STAT_ROWS, NMOM, 2, h->P(bo.lna_g), h->P(bo.lna_b), 1e-5f);
  } else {
    ld.mode = LD_ADD;
  }
  return ld;
}

// Weight/parameter blobs, hand-off buffers and residency capacity of the fused TCN (tcn_kernel.h):
// per block the fragment-ordered fp16 hi/lo weights (WF_*) and one float parameter blob (PB_*), both
// contiguous over blocks so the kernel addresses block i with uniform arithmetic (no pointer loads).
int init_fused(sepvad_model* h, const Packer& pk) {
  int ncu = 0, dev = h->device;
  HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int ln = h->cfg.ln_mode == SEPVAD_LN_RECURSIVE ? LD_RECURSIVE
                 : (h->cfg.ln_mode == SEPVAD_LN_RESIDUAL ? LD_RESIDUAL : LD_ADD);
  for (int p : {PREC_F16X3, PREC_F16, PREC_BF16, PREC_F32}) {
    // co-resident workgroups of the persistent TCN kernel that will run (both use one 512-thread workgroup per CU)
    h->tcn_cap_p[p] = ncu * tcn_blocks_per_cu(ln, p, 0, 1);
    h->tcn_cap = std::max(h->tcn_cap, h->tcn_cap_p[p]);
    h->tcn2_cap_p[p] = ncu * tcn_blocks_per_cu(ln, p, 0, 2);  // (0 for PREC_F32: one-slice only)
  }
  for (int q = 1; q <= 2; ++q) {
    h->tcn_cap_q[q] = ncu * tcn_blocks_per_cu(ln, PREC_F16X3, q, 1);
    h->tcn_cap = std::max(h->tcn_cap, h->tcn_cap_q[q]);
    h->tcn2_cap_q[q] = ncu * tcn_blocks_per_cu(ln, PREC_F16X3, q, 2);
  }
  if (h->tcn_cap < 1) { h->fused = false; return SEPVAD_OK; }
  // hand-off slots are per member: a two-slice workgroup publishes two members' words
  h->gran_slots = h->tcn_cap;
  for (int p : {PREC_F16X3, PREC_F16, PREC_BF16}) h->gran_slots = std::max(h->gran_slots, 2 * h->tcn2_cap_p[p]);
  for (int q = 1; q <= 2; ++q) h->gran_slots = std::max(h->gran_slots, 2 * h->tcn2_cap_q[q]);
  std::vector<__half> wf(WF_BLOCK * h->nblk), wfq(WF_BLOCK * h->nblk), ws16(WS_BLOCK * h->nblk), wsbf(WS_BLOCK * h->nblk), wq(WQ_BLOCK * h->nblk), wi(WQ_BLOCK * h->nblk);
  std::vector<float> pb((size_t)PB_SIZE * h->nblk, 0.f);
  std::vector<float> wf32(WS32_BLOCK / 2 * h->nblk);
  const bool rec = h->cfg.ln_mode == SEPVAD_LN_RECURSIVE, res = h->cfg.ln_mode == SEPVAD_LN_RESIDUAL;
  for (int i = 0; i < h->nblk; ++i) {
    const BlockOff& bo = h->blk[i];
    __half* w = wf.data() + WF_BLOCK * i;
    std::copy_n(pk.hblob.begin() + bo.w1.fhi, WF_W1L, w);
    std::copy_n(pk.hblob.begin() + bo.w1.flo, WF_W1L, w + WF_W1L);
    std::copy_n(pk.hblob.begin() + bo.w2.fhi, WF_W2L - WF_W2H, w + WF_W2H);
    std::copy_n(pk.hblob.begin() + bo.w2.flo, WF_W2L - WF_W2H, w + WF_W2L);
    __half* wqf = wfq.data() + WF_BLOCK * i;
    std::copy_n(w, WF_BLOCK, wqf);
    std::copy_n(pk.hblob.begin() + bo.w1.fq, WF_W1L, wqf + WF_W1L);
    std::copy_n(pk.hblob.begin() + bo.w2.fq, WF_W2L - WF_W2H, wqf + WF_W2L);
    __half* wqb = wq.data() + WQ_BLOCK * i;
    std::copy_n(pk.hblob.begin() + bo.w1.fhi, WQ_W1L, wqb);
    std::copy_n(pk.hblob.begin() + bo.w1.fl8, WQ_W2H - WQ_W1L, wqb + WQ_W1L);
    std::copy_n(pk.hblob.begin() + bo.w2.fhi, WQ_W2L - WQ_W2H, wqb + WQ_W2H);
    std::copy_n(pk.hblob.begin() + bo.w2.fl8, WQ_BLOCK - WQ_W2L, wqb + WQ_W2L);
    __half* wib = wi.data() + WQ_BLOCK * i;
    std::copy_n(pk.hblob.begin() + bo.w1.fhi, WQ_W1L, wib);
    std::copy_n(pk.hblob.begin() + bo.w1.fi8, WQ_W2H - WQ_W1L, wib + WQ_W1L);
    std::copy_n(pk.hblob.begin() + bo.w2.fhi, WQ_W2L - WQ_W2H, wib + WQ_W2H);
    std::copy_n(pk.hblob.begin() + bo.w2.fi8, WQ_BLOCK - WQ_W2L, wib + WQ_W2L);
    std::copy_n(pk.hblob.begin() + bo.w1.fhi, WS_W2, ws16.data() + WS_BLOCK * i);
    std::copy_n(pk.hblob.begin() + bo.w2.fhi, WS_BLOCK - WS_W2, ws16.data() + WS_BLOCK * i + WS_W2);
    std::copy_n(pk.hblob.begin() + bo.w1.fbf, WS_W2, wsbf.data() + WS_BLOCK * i);
    std::copy_n(pk.hblob.begin() + bo.w2.fbf, WS_BLOCK - WS_W2, wsbf.data() + WS_BLOCK * i + WS_W2);
    float* f32b = wf32.data() + WS32_BLOCK / 2 * i;
    std::copy_n(pk.blob.begin() + bo.w1.ff32, WS32_W2 / 2, f32b);
    std::copy_n(pk.blob.begin() + bo.w2.ff32, (WS32_BLOCK - WS32_W2) / 2, f32b + WS32_W2 / 2);
    float* q = pb.data() + (size_t)PB_SIZE * i;
    auto put = [&](int off, size_t src, int n) { std::copy_n(pk.blob.begin() + src, n, q + off); };
    put(PB_WS1, bo.w1.scale, CH); put(PB_B1, bo.b1, CH); put(PB_G1, bo.g1, CH); put(PB_BE1, bo.be1, CH);
    put(PB_WD, bo.wd, HID * 3); put(PB_BD, bo.bd, HID);
    put(PB_WS2, bo.w2.scale, CH); put(PB_B2, bo.b2, CH); put(PB_FC2, bo.fc2, CH);
    if (rec || res) { put(PB_LNAG, bo.lna_g, CH); put(PB_LNAB, bo.lna_b, CH); }
    if (rec) { put(PB_LNBG, bo.lnb_g, CH); put(PB_LNBB, bo.lnb_b, CH); }
    put(PB_ATT, bo.attp, 20);
    q[PB_A1] = bo.a1; q[PB_A2] = bo.a2;
    q[PB_SX] = bo.sx;
    q[PB_SXN] = i + 1 < h->nblk ? h->blk[i + 1].sx : 1.f;
    q[PB_EPS2] = bo.eps2;
    {
      double sf = 0.0, sb = 0.0;  // fixed order (bitwise reproducible)
      for (int k = 0; k < CH; ++k) { sf += pk.blob[bo.fc2 + k]; sb += pk.blob[bo.b2 + k]; }
      q[PB_SFC2] = (float)sf;
      q[PB_SB2] = (float)sb;
    }
    std::memcpy(q + PB_WSUM, bo.wsum, sizeof(bo.wsum));
    const int li = i % h->cfg.layer;
    if (bo.dil != (li == 0 ? 1 : (li % 4 + 1))) { g_err = "fused TCN: dilation schedule mismatch"; return SEPVAD_E_ARG; }
  }
  HIPCHK(hipMalloc(&h->twf, wf.size() * sizeof(__half)));
  HIPCHK(hipMemcpy(h->twf, wf.data(), wf.size() * sizeof(__half), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->twfq, wfq.size() * sizeof(__half)));
  HIPCHK(hipMemcpy(h->twfq, wfq.data(), wfq.size() * sizeof(__half), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->twq[1], wq.size() * sizeof(__half)));
  HIPCHK(hipMemcpy(h->twq[1], wq.data(), wq.size() * sizeof(__half), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->twq[2], wi.size() * sizeof(__half)));
  HIPCHK(hipMemcpy(h->twq[2], wi.data(), wi.size() * sizeof(__half), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->twf16, ws16.size() * sizeof(__half)));
  HIPCHK(hipMemcpy(h->twf16, ws16.data(), ws16.size() * sizeof(__half), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->twf32, wf32.size() * sizeof(float)));
  HIPCHK(hipMemcpy(h->twf32, wf32.data(), wf32.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->twbf, wsbf.size() * sizeof(__half)));
  HIPCHK(hipMemcpy(h->twbf, wsbf.data(), wsbf.size() * sizeof(__half), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&h->tprm, pb.size() * sizeof(float)));
  HIPCHK(hipMemcpy(h->tprm, pb.data(), pb.size() * sizeof(float), hipMemcpyHostToDevice));
  return SEPVAD_OK;
}

void free_ctx(StreamCtx* c) {
  if (c->ws.base) (void)hipFree(c->ws.base);
  if (c->tgran) (void)hipFree(c->tgran);
  if (c->terr) (void)hipFree(c->terr);
  if (c->herr) (void)hipHostFree(c->herr);
  delete c;
}

int env_int(const char* name, int dflt);
// The context of caller stream `stream` (created on first use; the caller holds h->mu).
int get_ctx(sepvad_model* h, void* stream, StreamCtx** out) {
  for (auto& c : h->ctx)
    if (c->stream == stream) { c->used = ++h->use_clock; *out = c.get(); return SEPVAD_OK; }
  // cap the per-stream contexts (each holds a workspace, hand-off words and pinned memory): evict the least
  // recently used one after draining the whole device (SEPVAD_MAX_STREAM_CTX, default 32; include/sepvad.h notes the
  // device-wide stall)
  const size_t cap = (size_t)std::max(1, env_int("SEPVAD_MAX_STREAM_CTX", 32));
  while (h->ctx.size() >= cap) {
    size_t lru = 0;
    for (size_t i = 1; i < h->ctx.size(); ++i)
      if (h->ctx[i]->used < h->ctx[lru]->used) lru = i;
    // every enqueued use of its buffers done: the whole device is drained, because the context's stream may already be
    // destroyed with work pending (an event recorded after every forward cost each forward 5.8 us of queue time,
    // profiles/r05_gap/; eviction is rare: more live streams than the cap)
    HIPCHK(hipDeviceSynchronize());
    free_ctx(h->ctx[lru].release());
    h->ctx.erase(h->ctx.begin() + lru);
  }
  std::unique_ptr<StreamCtx, void (*)(StreamCtx*)> c(new StreamCtx(), free_ctx);
  c->stream = stream;
  if (h->tcn_cap > 0) {
    const size_t gb = (size_t)h->gran_slots * 2 * NGR * sizeof(unsigned long long);
    HIPCHK(hipMalloc(&c->tgran, gb));
    HIPCHK(hipMemsetAsync(c->tgran, 0, gb, (hipStream_t)stream));  // (ordered before this stream's first launch)
  }
  HIPCHK(hipMalloc(&c->terr, 16));
  HIPCHK(hipMemsetAsync(c->terr, 0, 16, (hipStream_t)stream));
  HIPCHK(hipHostMalloc((void**)&c->herr, 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(c->herr, 0, 64);
  HIPCHK(hipHostGetDevicePointer((void**)&c->herr_dev, c->herr, 0));
  if (h->res_B > 0) {
    const int rc = ws_reserve(c.get(), h->res_B, h->res_N);
    if (rc) return rc;
  }
  c->used = ++h->use_clock;
  *out = c.get();
  h->ctx.emplace_back(c.release());
  return SEPVAD_OK;
}

// Give-up words written by k_tcn launches of this context that completed since the last check: report
// each once (the word holds the failing launch's salt, so a later give-up is a new value).
// n consecutive hand-off tag salts for the k_tcn launches of one forward chunk: never 0, and never wrapping inside
// the range (k_istft_pair poisons the outputs when the give-up word holds one of gsalt_lo .. gsalt_lo + n - 1). When
// the 20-bit salt would wrap, the stream is drained and the hand-off words, the device give-up word and its host copy
// restart from zero (a give-up not yet reported is kept in `pending`), so a reused salt never matches an old word.
int salt_reserve(sepvad_model* h, StreamCtx* c, hipStream_t s, unsigned n, unsigned* lo) {
  constexpr unsigned SMAX = (1u << (32 - TCN_EPOCH_BITS)) - 1;
  const unsigned wrap_at = (unsigned)std::max(2, std::min((int)SMAX, env_int("SEPVAD_TCN_SALT_MAX", (int)SMAX)));
  if (n > wrap_at) return fail(SEPVAD_E_ARG, "fused TCN: too many launches in one forward");
  if (c->tsalt + n > wrap_at) {
    HIPCHK(hipStreamSynchronize(s));
    const unsigned v = __atomic_load_n(c->herr, __ATOMIC_ACQUIRE);
    if (v != 0 && v != c->reported) c->pending = v;
    HIPCHK(hipMemsetAsync(c->tgran, 0, (size_t)h->gran_slots * 2 * NGR * sizeof(unsigned long long), s));
    HIPCHK(hipMemsetAsync(c->terr, 0, 16, s));
    __atomic_store_n(c->herr, 0u, __ATOMIC_RELEASE);
    c->reported = 0;
    c->tsalt = 0;
  }
  *lo = c->tsalt + 1;
  c->tsalt += n;
  return SEPVAD_OK;
}

int check_giveup(StreamCtx* c) {
  if (env_int("SEPVAD_GIVEUP_INFO", 0) && (c->pending != 0 || (c->herr[0] != 0 && c->herr[0] != c->reported))) {
    unsigned w[4] = {};  // diagnostics: {launch tag0, the timed-out wait's tag, its workgroup, its word index}
    if (hipMemcpy(w, c->terr, sizeof(w), hipMemcpyDeviceToHost) == hipSuccess)
      fprintf(stderr, "sepvad: give-up on stream %p: tag0 %#x, first timed-out wait: tag %#x (salt %u epoch %u) "
              "workgroup %u word %u (slot %u, offset %u)\n", c->stream, w[0], w[1], w[1] >> TCN_EPOCH_BITS,
              w[1] & ((1u << TCN_EPOCH_BITS) - 1), w[2], w[3], w[3] / NGR, w[3] % NGR);
    // reported: clear the diagnostic words (the first timed-out poller sets them by a compare-and-swap from 0), so a
    // later give-up on this context reports its own wait, not this one's
    // (synchronous, not on c->stream: a cached context's caller stream may already be destroyed)
    (void)hipMemset(c->terr + 1, 0, 3 * sizeof(unsigned));
  }
  if (c->pending != 0) {
    c->pending = 0;
    return fail(SEPVAD_E_HIP, "fused TCN: a group hand-off wait gave up in an earlier forward on this stream "
                              "(that forward's outputs are invalid)");
  }
  const unsigned v = __atomic_load_n(c->herr, __ATOMIC_ACQUIRE);
  if (v != 0 && v != c->reported) {
    c->reported = v;
    return fail(SEPVAD_E_HIP, "fused TCN: a group hand-off wait gave up in an earlier forward on this stream "
                              "(that forward's outputs are invalid)");
  }
  return SEPVAD_OK;
}

}  // namespace

extern "C" {

const char* sepvad_last_error(void) { return g_err.c_str(); }
int32_t sepvad_abi_version(void) { return SEPVAD_ABI_VERSION; }
const char* sepvad_build_id(void) { return SEPVAD_BUILD_ID; }

sepvad_handle sepvad_create(const SepVadConfig* cfg, const float* const* tensors, const char* const* names,
                            const int64_t* numels, int32_t n, int32_t device) {
  if (!cfg || !tensors || !names || !numels) { g_err = "null argument"; return nullptr; }
  const SepVadConfig& c = *cfg;
  if (c.n_fft != NFFT || c.bn_dim != CH || c.h_dim != HID || c.num_spk != 2 || c.layer < 1 || c.stack < 1 ||
      c.precision < SEPVAD_PREC_FP32 || c.precision > SEPVAD_PREC_BF16) {
    g_err = "unsupported configuration (native path: n_fft=512, BN_dim=256, H_dim=512, num_spk=2)";
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) { g_err = "invalid device"; return nullptr; }
  DeviceGuard dg(device);
  TensorMap tm;
  for (int i = 0; i < n; ++i) tm.m[names[i]] = {tensors[i], numels[i]};
  auto* h = new sepvad_model();
  h->cfg = c;
  h->device = device;
  h->nblk = c.layer * c.stack;
  h->prec = c.precision;  // SEPVAD_PREC_* == PREC_* (static_asserts below)
  Packer pk;
  bool ok = true;
  auto get = [&](const std::string& k, int64_t numel) -> const float* {
    const float* p = tm.get(k, numel);
    if (!p) ok = false;
    return p;
  };
#define BAIL() do { if (!ok) { delete h; return nullptr; } } while (0)
  // windows (model/model.py:383-387) and FFT twiddles
  const float* wi = get("spec_input.spec.window", NFFT);
  const float* wo = get("spec_output.window", NFFT);
  const float* wv = get("inv_spec.window", NFFT);
  BAIL();
  h->win_in = pk.add(wi, NFFT);
  h->win_out = pk.add(wo, NFFT);
  h->win_inv = pk.add(wv, NFFT);
  h->same_stft_window = std::memcmp(wi, wo, NFFT * sizeof(float)) == 0;
  {
    std::vector<float> tw(2 * NFFT);
    for (int m = 0; m < NFFT; ++m) {
      const double ang = -2.0 * M_PI * m / NFFT;
      tw[2 * m] = (float)std::cos(ang);
      tw[2 * m + 1] = (float)std::sin(ang);
    }
    h->tw = pk.add(tw);
  }
  double xbound = 0.0;  // range bound of the current block's x' (range guard)
  {
    const float* lg = get("TCN.LN.weight", CH);
    const float* lb = get("TCN.LN.bias", CH);
    BAIL();
    h->ln_g = pk.add(lg, CH);
    h->ln_b = pk.add(lb, CH);
    xbound = gn_bound(lg, lb, CH);  // x'_0 = TCN.LN(S0)
  }
  // blocks (model/model.py:285-295,103-127,182-195,310-319)
  for (int i = 0; i < h->nblk; ++i) {
    BlockOff bo{};
    const std::string p = "TCN.TCN." + std::to_string(i);
    const float* g1 = get(p + ".conv1d.weight_g", CH);
    const float* v1 = get(p + ".conv1d.weight_v", (int64_t)CH * CH);
    const float* gd = get(p + ".dconv1d.weight_g", HID);
    const float* vd = get(p + ".dconv1d.weight_v", (int64_t)HID * 3);
    const float* g2 = get(p + ".res_out.weight_g", CH);
    const float* v2 = get(p + ".res_out.weight_v", (int64_t)CH * HID);
    const float* b1 = get(p + ".conv1d.bias", CH);
    const float* bd = get(p + ".dconv1d.bias", HID);
    const float* b2 = get(p + ".res_out.bias", CH);
    const float* a1 = get(p + ".nonlinearity1.weight", 1);
    const float* a2 = get(p + ".nonlinearity2.weight", 1);
    const float* r1g = get(p + ".reg1.weight", CH);
    const float* r1b = get(p + ".reg1.bias", CH);
    const float* r2g = get(p + ".reg2.weight", HID);
    const float* r2b = get(p + ".reg2.bias", HID);
    BAIL();
    const int ex = range_exp(xbound);
    bo.sx = std::ldexp(1.f, -ex);
    bo.w1 = pack_pointwise(pk, fold_wn(g1, v1, CH, CH), CH, CH, CH, ex);
    bo.b1 = pk.add(b1, CH);
    bo.g1 = pk.add(r1g, CH);
    bo.be1 = pk.add(r1b, CH);
    {
      // d = PReLU(dconv(GN1(h))) produced pre-scaled by 2^-ed: dconv weights and bias scaled (exact), the
      // reg2 GroupNorm eps scaled by 2^-2ed so GN2(d) is unchanged (range guard)
      std::vector<float> wd = fold_wn(gd, vd, HID, 3), bds(bd, bd + HID);
      double dbound = 0.0;
      for (int j = 0; j < HID; ++j) {
        const int k = j / 2;  // groups = CH, depth multiplier 2 (model/model.py:110-113)
        const double nb = std::fabs((double)r1g[k]) * NSIG + std::fabs((double)r1b[k]);
        const double sw = std::fabs((double)wd[3 * j]) + std::fabs((double)wd[3 * j + 1]) + std::fabs((double)wd[3 * j + 2]);
        dbound = std::max(dbound, sw * nb + std::fabs((double)bd[j]));
      }
      dbound *= std::max(1.0, std::fabs((double)a2[0]));
      const int ed = range_exp(dbound);
      for (auto& v : wd) v = std::ldexp(v, -ed);
      for (auto& v : bds) v = std::ldexp(v, -ed);
      bo.wd = pk.add(wd);
      bo.bd = pk.add(bds);
      bo.eps2 = std::ldexp(1e-8f, -2 * ed);
    }
    {
      // reg2 (GroupNorm(1, H) of d, model/model.py:136) folded out of the res_out operand: see gemm.hip
      const std::vector<float> w2 = fold_wn(g2, v2, CH, HID);
      std::vector<float> w2g((size_t)CH * HID), cb(CH), fc(CH);
      for (int m = 0; m < CH; ++m) {
        double sb = b2[m], sg = 0.0;
        for (int k = 0; k < HID; ++k) {
          const float wg = w2[(size_t)m * HID + k] * r2g[k];
          w2g[(size_t)m * HID + k] = wg;
          sg += wg;
          sb += (double)w2[(size_t)m * HID + k] * r2b[k];
        }
        cb[m] = (float)sb;
        fc[m] = (float)sg;
      }
      bo.w2 = pack_pointwise(pk, w2g, CH, HID, CH);
      bo.b2 = pk.add(cb);
      bo.fc2 = pk.add(fc);
    }
    bo.g2 = pk.add(r2g, HID);
    bo.be2 = pk.add(r2b, HID);
    bo.a1 = a1[0];
    bo.a2 = a2[0];
    const int li = i % c.layer;
    bo.dil = li == 0 ? 1 : (li % 4 + 1);
    std::vector<float> attp(20, 0.f);
    if (c.tf_attention) {
      const std::string q = "TCN.time_freq_attnetion." + std::to_string(i);
      const char* convs[4] = {".conv1d_t_1", ".conv1d_t_2", ".conv1d_f_1", ".conv1d_f_2"};
      for (int j = 0; j < 4; ++j) {
        const float* w = get(q + convs[j] + ".weight", 3);
        const float* bb = get(q + convs[j] + ".bias", 1);
        BAIL();
        attp[4 * j + 0] = w[0]; attp[4 * j + 1] = w[1]; attp[4 * j + 2] = w[2]; attp[4 * j + 3] = bb[0];
      }
      const float* pt = get(q + ".prelu_t.weight", 1);
      const float* pf = get(q + ".prelu_f.weight", 1);
      BAIL();
      attp[16] = pt[0]; attp[17] = pf[0];
    }
    bo.attp = pk.add(attp);
    if (c.ln_mode == SEPVAD_LN_RECURSIVE) {
      const float* fa = get("TCN.ln_first_modules." + std::to_string(i) + ".weight", CH);
      const float* fb = get("TCN.ln_first_modules." + std::to_string(i) + ".bias", CH);
      const float* sa = get("TCN.ln_second_modules." + std::to_string(i) + ".weight", CH);
      const float* sb = get("TCN.ln_second_modules." + std::to_string(i) + ".bias", CH);
      BAIL();
      bo.lna_g = pk.add(fa, CH); bo.lna_b = pk.add(fb, CH);
      bo.lnb_g = pk.add(sa, CH); bo.lnb_b = pk.add(sb, CH);
      xbound = gn_bound(sa, sb, CH);  // next block's x' = GN_b(..)
      for (int j = 0; j < 5; ++j) bo.wsum[j] = 0.0;
      for (int k = 0; k < CH; ++k) {
        const double g = fa[k], e = fb[k];
        bo.wsum[0] += g; bo.wsum[1] += e; bo.wsum[2] += e * e; bo.wsum[3] += g * e; bo.wsum[4] += g * g;
      }
    } else if (c.ln_mode == SEPVAD_LN_RESIDUAL) {
      const float* fa = get("TCN.ln_modules." + std::to_string(i) + ".weight", CH);
      const float* fb = get("TCN.ln_modules." + std::to_string(i) + ".bias", CH);
      BAIL();
      bo.lna_g = pk.add(fa, CH); bo.lna_b = pk.add(fb, CH);
      xbound += gn_bound(fa, fb, CH);  // next block's x' = o + GN_c(..)
    } else {
      xbound = 0.0;  // plain residual add: no static bound, no scale
    }
    h->blk.push_back(bo);
  }
  // output head (model/model.py:322-325)
  {
    const float* oa = get("TCN.output.0.weight", 1);
    const float* og = get("TCN.output.1.weight", CH);
    const float* ob = get("TCN.output.1.bias", CH);
    const float* gg = get("TCN.output.2.weight_g", MOUT);
    const float* vv = get("TCN.output.2.weight_v", (int64_t)MOUT * CH);
    const float* bb = get("TCN.output.2.bias", MOUT);
    BAIL();
    h->out_a = oa[0];
    h->out_g = pk.add(og, CH);
    h->out_b = pk.add(ob, CH);
    const int eh = range_exp(gn_bound(og, ob, CH));  // head A operand = GN_out(PReLU(x'))
    h->out_sx = std::ldexp(1.f, -eh);
    const std::vector<float> wo = fold_wn(gg, vv, MOUT, CH);
    h->wout = pack_pointwise(pk, wo, MOUT, CH, MOUT_PAD, eh);
    std::vector<float> bpad(MOUT_PAD, 0.f);
    std::memcpy(bpad.data(), bb, MOUT * sizeof(float));
    h->bo = pk.add(bpad);
    std::vector<float> ws((size_t)MOUT_PAD * CH, 0.f), bs(MOUT_PAD, 0.f);
    for (int q = 0; q < 2; ++q)
      for (int i = 0; i < NBIN; ++i) {
        std::memcpy(&ws[((size_t)q * HEAD_SPK + i) * CH], &wo[((size_t)q * NBIN + i) * CH], CH * sizeof(float));
        bs[q * HEAD_SPK + i] = bb[q * NBIN + i];
      }
    h->wout_spk = pack_pointwise(pk, ws, MOUT_PAD, CH, MOUT_PAD, eh);
    h->bo_spk = pk.add(bs);
    std::vector<float> nyw((size_t)2 * CH), nyb(2);
    for (int q = 0; q < 2; ++q) {
      std::memcpy(&nyw[(size_t)q * CH], &wo[((size_t)q * NBIN + NBIN - 1) * CH], CH * sizeof(float));
      nyb[q] = bb[q * NBIN + NBIN - 1];
    }
    h->out_nyw = pk.add(nyw);
    h->out_nyb = pk.add(nyb);
  }
  // VAD head (model/model.py:153-171)
  if (c.final_vad) {
    const float* g1 = get("vad.common.conv1_1.weight_g", 4);
    const float* v1 = get("vad.common.conv1_1.weight_v", (int64_t)4 * NBIN * 5);
    const float* b1 = get("vad.common.conv1_1.bias", 4);
    const float* a = get("vad.common.relu_1.weight", 1);
    const float* gg = get("vad.common.BN_1.weight", 4);
    const float* gb = get("vad.common.BN_1.bias", 4);
    const float* g2 = get("vad.output_layer_vad.weight_g", 1);
    const float* v2 = get("vad.output_layer_vad.weight_v", 12);
    const float* b2 = get("vad.output_layer_vad.bias", 1);
    BAIL();
    const std::vector<float> w1 = fold_wn(g1, v1, 4, NBIN * 5);  // [o][c][k]
    h->v_w1 = pk.add(w1);
    std::vector<float> wv((size_t)32 * HEAD_SPK, 0.f);  // [4 k + o][speaker-local channel c]
    for (int o = 0; o < 4; ++o)
      for (int c2 = 0; c2 < NBIN; ++c2)
        for (int k = 0; k < 5; ++k) wv[(size_t)(4 * k + o) * HEAD_SPK + c2] = w1[((size_t)o * NBIN + c2) * 5 + k];
    // range guard of the VAD GEMM's A operand (the masks tile, fp16 split): |masks| <= max over rows of
    // sum_c |W| * bound(GN_out(..)) + |bias|; the tile is scaled by 2^-e on its way into the split and the
    // columns' scale carries 2^e back
    double mb = 0.0;
    {
      const std::vector<float> wo = fold_wn(get("TCN.output.2.weight_g", MOUT), get("TCN.output.2.weight_v", (int64_t)MOUT * CH), MOUT, CH);
      const float* ob2 = get("TCN.output.2.bias", MOUT);
      const double ab = gn_bound(get("TCN.output.1.weight", CH), get("TCN.output.1.bias", CH), CH);
      for (int r = 0; r < MOUT; ++r) {
        double sr = 0.0;
        for (int i = 0; i < CH; ++i) sr += std::fabs((double)wo[(size_t)r * CH + i]);
        mb = std::max(mb, sr * ab + std::fabs((double)ob2[r]));
      }
    }
    const int ev_ = range_exp(mb);
    h->vad_sx = std::ldexp(1.f, -ev_);
    h->vadw = pack_pointwise(pk, wv, HEAD_VAD_N, HEAD_SPK, 32, ev_);
    std::vector<float> vny(HEAD_VAD_N);
    for (int o = 0; o < 4; ++o)
      for (int k = 0; k < 5; ++k) vny[4 * k + o] = w1[((size_t)o * NBIN + NBIN - 1) * 5 + k];
    h->vad_ny = pk.add(vny);
    h->v_b1 = pk.add(b1, 4);
    h->v_a = a[0];
    h->v_g = pk.add(gg, 4);
    h->v_b = pk.add(gb, 4);
    h->v_w2 = pk.add(fold_wn(g2, v2, 1, 12));
    h->v_b2 = b2[0];
  }
  // activity gate (model/model.py:398-400)
  {
    std::vector<float> gw(12, 0.f);
    if (c.activity_input) {
      const float* w = get("activity_input.weight", 9);
      const float* bb = get("activity_input.bias", 1);
      const float* pa = get("prelu.weight", 1);
      BAIL();
      std::memcpy(gw.data(), w, 9 * sizeof(float));
      gw[9] = bb[0];
      gw[10] = pa[0];
    }
    h->gate = pk.add(gw);
  }
#undef BAIL
  h->split = 1;
  if (const char* sp = getenv("SEPVAD_SPLIT")) h->split = std::max(1, std::min(MAX_SPLIT, atoi(sp)));
  bool streams_ok = hipEventCreateWithFlags(&h->fork, hipEventDisableTiming) == hipSuccess;
  for (int k = 0; k < MAX_SPLIT && streams_ok; ++k)
    streams_ok = hipStreamCreateWithFlags(&h->sub[k], hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&h->join[k], hipEventDisableTiming) == hipSuccess;
  if (!streams_ok) {
    g_err = "creating the internal streams/events failed";
    sepvad_destroy(h);
    return nullptr;
  }
  if (hipMalloc(&h->dparams, pk.blob.size() * sizeof(float)) != hipSuccess ||
      hipMemcpy(h->dparams, pk.blob.data(), pk.blob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&h->dhalf, pk.hblob.size() * sizeof(__half)) != hipSuccess ||
      hipMemcpy(h->dhalf, pk.hblob.data(), pk.hblob.size() * sizeof(__half), hipMemcpyHostToDevice) != hipSuccess) {
    g_err = "device allocation/upload of the packed weights failed";
    sepvad_destroy(h);
    return nullptr;
  }
  if (const char* fz = getenv("SEPVAD_FUSED")) h->fused = atoi(fz) != 0;
  if (const char* wl = getenv("SEPVAD_WLO")) {  // "i8" (default) | "f16" | "e4m3"; anything else is an error
    if (std::strcmp(wl, "e4m3") == 0) h->lo8 = 1;
    else if (std::strcmp(wl, "f16") == 0) h->lo8 = 0;
    else if (std::strcmp(wl, "i8") == 0) h->lo8 = 2;
    else {
      g_err = std::string("SEPVAD_WLO: unknown weight lo-plane format '") + wl + "' (expected i8, f16 or e4m3)";
      sepvad_destroy(h);
      return nullptr;
    }
  }
  if (init_fused(h, pk) != SEPVAD_OK) {
    sepvad_destroy(h);
    return nullptr;
  }
  return h;
}

int32_t sepvad_reserve(sepvad_handle h, int32_t B, int32_t N) {
  if (!h || B < 1 || N <= HOP) return fail(SEPVAD_E_ARG, "sepvad_reserve: bad arguments");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  h->res_B = std::max(h->res_B, (int)B);
  h->res_N = std::max(h->res_N, (int)N);
  StreamCtx* c0 = nullptr;
  int rc = get_ctx(h, nullptr, &c0);  // the default stream's context exists from here on
  for (size_t i = 0; rc == SEPVAD_OK && i < h->ctx.size(); ++i) rc = ws_reserve(h->ctx[i].get(), h->res_B, h->res_N);
  return rc;
}

int32_t sepvad_set_precision(sepvad_handle h, int32_t precision) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  if (precision < SEPVAD_PREC_FP32 || precision > SEPVAD_PREC_BF16) return fail(SEPVAD_E_ARG, "unknown precision");
  h->prec = precision;
  return SEPVAD_OK;
}

int32_t sepvad_set_weight_lo(sepvad_handle h, int32_t mode) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  if (mode != SEPVAD_WLO_E4M3 && mode != SEPVAD_WLO_F16 && mode != SEPVAD_WLO_I8)
    return fail(SEPVAD_E_ARG, "unknown weight lo-plane format");
  h->lo8 = mode == SEPVAD_WLO_E4M3 ? 1 : (mode == SEPVAD_WLO_I8 ? 2 : 0);
  return SEPVAD_OK;
}

int32_t sepvad_e4m3_encode(const float* in, uint8_t* out, int64_t n) {
  if ((!in || !out) && n > 0) return fail(SEPVAD_E_ARG, "sepvad_e4m3_encode: null buffer");
  for (int64_t i = 0; i < n; ++i) out[i] = e4m3_rn(in[i]);
  return SEPVAD_OK;
}

int32_t sepvad_set_timing(sepvad_handle h, int32_t on) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  h->timing = on != 0;
  return SEPVAD_OK;
}

int32_t sepvad_timing(sepvad_handle h, double* gemm_ms, int32_t* gemm_launches, double* total_ms) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  if (gemm_ms) { gemm_ms[0] = h->gemm_ms; gemm_ms[1] = h->g2_ms; }
  if (gemm_launches) { gemm_launches[0] = h->gemm_launches; gemm_launches[1] = h->g2_launches; }
  if (total_ms) *total_ms = h->total_ms;
  return SEPVAD_OK;
}

}  // extern "C"

namespace {

// The fused TCN runs when the GEMMs are fp16x3, an utterance fits one group (T <= 32 * FG_MAX = 8192) and a group fits
// the co-resident capacity; otherwise the multi-kernel path below runs (same results within fp32 rounding).
static_assert(SEPVAD_PREC_FP32 == PREC_F32 && SEPVAD_PREC_F16X3 == PREC_F16X3 && SEPVAD_PREC_F16 == PREC_F16 &&
              SEPVAD_PREC_BF16 == PREC_BF16, "precision codes");

// co-resident k_tcn workgroups of the variant that will run (the e4m3-lo kernel is its own instantiation)
int tcn_cap_of(const sepvad_model* h) {
  return h->prec == PREC_F16X3 && h->lo8 ? h->tcn_cap_q[h->lo8] : h->tcn_cap_p[h->prec];
}

bool fused_ok(const sepvad_model* h, int T) {
  const int G = (T + FR - 1) / FR;
  return h->fused && G <= FG_MAX && tcn_cap_of(h) >= G;
}

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// Progress of concurrent fused launches (include/sepvad.h: concurrent forwards on different streams are allowed).
// A k_tcn group waits for all of its G members, and the grid is dealt in order, so a launch progresses as long as
// 8 G of its workgroups are resident (tcn_kernel.h header). Two launches that each need more than half the chip for
// that can each hold part of the CUs and wait on each other until the give-up bound. Such "big" launches (long
// utterances) are therefore ordered across streams, process-wide per device: each waits on the previous one's
// completion event (stream-ordered, no host sync). Launches of small groups need no ordering: any resident prefix
// of 8 G workgroups completes them, beside a big launch too, and they free their CUs.
int tcn2_cap_of(const sepvad_model* h) {
  return h->prec == PREC_F16X3 && h->lo8 ? h->tcn2_cap_q[h->lo8] : h->tcn2_cap_p[h->prec];
}
// Slices (32-frame members) per k_tcn workgroup for a batch of B utterances of G members: two (64 frames, tcn_kernel.h
// TcnSmem2) once one-slice workgroups would need more than one round of the chip (B * G > capacity), so every weight
// fragment a CU streams feeds 64 frames instead of 32; the two give the same bits, so the choice never changes a
// result. SEPVAD_TCN_SLICES = 1 | 2 forces one (2 where the two-slice kernel applies: G even, G <= FG_WAVE).
int tcn_slices(const sepvad_model* h, int B, int G) {
  const int cap2 = tcn2_cap_of(h);
  if (G % 2 || G > FG_WAVE || cap2 < G / 2) return 1;
  if (const int f = env_int("SEPVAD_TCN_SLICES", 0)) return f == 2 ? 2 : 1;
  const int per_round = std::max(1, tcn_cap_of(h) / G);  // utterances in one round of one-slice groups
  return B > per_round ? 2 : 1;
}
bool tcn_big(int cap, int gw) { return 8 * gw > cap / 2; }
// Runs `launch` (which enqueues one big k_tcn launch on s) behind the previous big launch of the device and records
// its completion as the next one's wait, all under one process-wide lock: two handles (or two threads) on the same
// device can then never both wait on the same predecessor and run their big launches side by side.
template <class F>
int tcn_launch_ordered(int device, hipStream_t s, F&& launch) {
  static std::mutex mu;
  static std::unordered_map<int, hipEvent_t> last;  // device -> the last big launch's completion
  std::lock_guard<std::mutex> lk(mu);
  hipEvent_t& e = last[device];
  if (e) HIPCHK(hipStreamWaitEvent(s, e, 0));
  if (const int rc = launch()) return rc;
  // a fresh event per launch: a wait already enqueued never sees a later record of the same event
  hipEvent_t n = nullptr;
  HIPCHK(hipEventCreateWithFlags(&n, hipEventDisableTiming));
  HIPCHK(hipEventRecord(n, s));
  if (e) HIPCHK(hipEventDestroy(e));  // (released once its waits have completed)
  e = n;
  return SEPVAD_OK;
}

// Per-forward timing state (sepvad_set_timing): HIP events around the GEMM launches of chunk 0.
struct TimingRec {
  std::vector<int> gemm_ev, g2_ev;
};

// Enqueues the forward of utterances [b0, b0 + B) on stream s (model/model.py:402-461).
// Input row mapping of one forward: utterance u reads x + (u % nstr) * ldx + (u / nstr) * hopw (nstr = 0:
// plain batch, every row at u * ldx).
struct XMap {
  int nstr = 0;
  long long hopw = 0;
};

// Diagnostics (SEPVAD_TAIL_PROBE=<prefix>): per-workgroup phase stamps of a tail kernel, dumped synchronously
// to <prefix>.<kernel> as {grid x, grid y, 8} + [workgroups][8] (tools/tail_probe.py). Inactive otherwise.
struct TailProbe {
  static constexpr size_t N = 8192 * 8;
  sepvad_model* h;
  hipStream_t s;
  std::string path;
  unsigned long long* buf = nullptr;
  TailProbe(sepvad_model* h_, hipStream_t s_, const char* kernel) : h(h_), s(s_) {
    const char* pre = getenv("SEPVAD_TAIL_PROBE");
    if (!pre) return;
    path = std::string(pre) + "." + kernel;
    if (!h->kprobe && hipMalloc(&h->kprobe, N * sizeof(unsigned long long)) != hipSuccess) return;
    if (hipMemsetAsync(h->kprobe, 0, N * sizeof(unsigned long long), s) != hipSuccess) return;
    buf = h->kprobe;
  }
  hipError_t dump(long long gx, long long gy) {
    if (!buf) return hipSuccess;
    std::vector<unsigned long long> hp((size_t)std::min<long long>(gx * gy * 8, (long long)N));
    hipError_t e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipMemcpy(hp.data(), buf, hp.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    if (FILE* f = fopen(path.c_str(), "wb")) {
      const long long hdr[3] = {gx, gy, 8};
      fwrite(hdr, sizeof(hdr), 1, f);
      fwrite(hp.data(), sizeof(unsigned long long), hp.size(), f);
      fclose(f);
    }
    return hipSuccess;
  }
};

// Host-side trace ranges (roctx: `rocprofv3 --marker-trace`), one per forward and per stage of its enqueue,
// so a host timeline shows where the forward's launch time goes; no-ops without a tool attached.
struct TraceRange {
  explicit TraceRange(const char* n) { roctxRangePushA(n); }
  void next(const char* n) {
    roctxRangePop();
    roctxRangePushA(n);
  }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

int enqueue_chunk(sepvad_model* h, StreamCtx* cx, const float* x, int ldx, int b0, int B, int N,
                  const SepVadOutputs* out, const SepVadInferKw* kw, hipStream_t s, TimingRec* tr,
                  const XMap& xm) {
  const int T = 1 + N / HOP;
  const int Tp = round_up(T, TILE);
  const SepVadConfig& c = h->cfg;
  const Workspace w = ws_view(cx->ws, b0, Tp);
  const int ntu = Tp / TILE;
  x += (size_t)b0 * ldx;
  const size_t u2 = (size_t)b0 * 2;
  auto ev = [&]() -> int { return tr ? ev_record(h, s) : 0; };
  const size_t g1_grid = (size_t)B * ntu * (CH / TILE);
  const bool probing = tr && h->probe && h->probe_blk >= 0;

  TraceRange stage("sepvad::stft_gate");
  // 1+2. STFT (spec_output for est; spec_input for the spectrum: one transform when the windows are equal)
  // fused with the activity gate, the TCN input and the TCN.LN statistics (k_stft_gate)
  {
    StftArgs sa{};
    sa.B = B; sa.N = N; sa.ldx = ldx; sa.T = T; sa.Tp = Tp; sa.x = x; sa.tw = (const float2*)h->P(h->tw);
    sa.nstr = xm.nstr > 0 ? xm.nstr : B; sa.hopw = xm.nstr > 0 ? xm.hopw : 0;
    sa.window = h->P(h->win_out);
    sa.window_db = h->same_stft_window ? sa.window : h->P(h->win_in);
    sa.X = w.X;
    sa.specdb = h->same_stft_window ? nullptr : w.specdb;
    sa.activity = c.activity_input; sa.gate_w = h->P(h->gate);
    sa.S0 = w.S0; sa.gate_rec = w.rec_gate;
    TailProbe tp(h, s, "stft");
    sa.probe = tp.buf;
    HIPCHK(launch_stft_gate(sa, s));
    HIPCHK(tp.dump(B, Tp / (2 * GATE_ROWS)));  // k_stft_gate's grid (32 own frames)
    if (out->spectrum) {  // eager side output (Handle.forward(return_aux=True))
      GateArgs ga{};
      ga.B = B; ga.T = T; ga.Tp = Tp; ga.activity = c.activity_input;
      ga.X = h->same_stft_window ? w.X : nullptr; ga.specdb = w.specdb; ga.w = h->P(h->gate);
      ga.S0 = nullptr; ga.out_rec = nullptr;
      ga.spec_side = out->spectrum + (size_t)b0 * NBIN * T;
      HIPCHK(launch_gate(ga, s));
    }
  }
  // 3+4. TCN + output head
  stage.next("sepvad::tcn_head");
  const int G = (T + FR - 1) / FR;
  const bool use_fused = fused_ok(h, T);
  unsigned gsalt_lo = 0, gsalt_n = 0;  // salts of this chunk's k_tcn launches (give-up poisoning, k_istft_pair)
  h->last_fused = use_fused;
  const bool has_vad = c.final_vad && (!c.final_vad_masked_speakers || c.noisy_phase);
  // the VAD conv1_1 as the output head's second GEMM (raw masks in; the masked-speakers variant reads |X| too)
  const bool vad_in_head = use_fused && has_vad && !c.final_vad_masked_speakers;
  if (use_fused) {
    // persistent launches of the whole TCN (tcn_kernel.h), the output head inside them
    const int nsl = h->tdump ? 1 : tcn_slices(h, B, G);  // (the parity-dump instantiation is one-slice only)
    const int cap = nsl == 2 ? tcn2_cap_of(h) : tcn_cap_of(h);
    h->last_nsl = nsl;
    const int Gt = G / nsl;  // workgroups per utterance
    TcnArgs ta{};
    ta.T = T; ta.Tp = Tp; ta.G = G; ta.nsl = nsl; ta.nblk = h->nblk; ta.layer = c.layer;
    if (const int nb = env_int("SEPVAD_TCN_NBLK", 0); nb > 0 && nb < h->nblk) ta.nblk = nb;  // diagnostics: truncated stack
    ta.ln_mode = c.ln_mode == SEPVAD_LN_RECURSIVE ? LD_RECURSIVE : (c.ln_mode == SEPVAD_LN_RESIDUAL ? LD_RESIDUAL : LD_ADD);
    ta.tf_att = c.tf_attention;
    ta.prec = h->prec;
    ta.lo8 = h->prec == PREC_F16X3 ? h->lo8 : 0;
    ta.wfrag = h->prec == PREC_F16X3 ? (ta.lo8 ? h->twq[ta.lo8] : h->twf)
                                     : (h->prec == PREC_F16 ? h->twf16
                                                            : (h->prec == PREC_F32 ? reinterpret_cast<const __half*>(h->twf32) : h->twbf));
    ta.prm = h->tprm;
    ta.inv_ch = 1.0 / ((double)CH * T);
    ta.inv_hid = 1.0 / ((double)HID * T);
    ta.alpha_h = h->out_a;
    ta.gran = cx->tgran; ta.err = cx->terr; ta.herr = cx->herr_dev;
    ta.xmode = env_int("SEPVAD_TCN_XMODE", 0);
    auto launch_t = [&](const TcnArgs& t, int grid) { return launch_tcn(t, grid, s); };
    ta.spin_limit = (unsigned)env_int("SEPVAD_TCN_SPIN_LIMIT", 1 << 20);
    ta.force_err = env_int("SEPVAD_TCN_FORCE_GIVEUP", 0);
    ta.dbg_delay = (unsigned)std::max(0, env_int("SEPVAD_TCN_DELAY", 0));
    ta.dump_blk = std::max(0, std::min(h->nblk - 1, env_int("SEPVAD_TCN_DUMP_BLOCK", 0)));
    // every group the chip holds (the kernel puts the groups of 8 * Gt * floor(groups / 8) blocks on one XCD each and the
    // rest, fewer than 8, on consecutive blocks; SEPVAD_TCN_ALIGN8=1: whole multiples of 8 groups only, as in round 4)
    int ngroups = std::min(B, cap / Gt);
    if (ngroups >= 8 && env_int("SEPVAD_TCN_ALIGN8", 0)) ngroups -= ngroups % 8;
    // the output head, inside k_tcn after each utterance's last block (its lo plane in the blocks' format)
    ta.hg = h->P(h->out_g); ta.hbe = h->P(h->out_b); ta.hsx = h->out_sx;
    ta.hwh = h->prec == PREC_F32 ? reinterpret_cast<const __half*>(h->P(h->wout_spk.ff32))
                                 : h->H(h->prec == PREC_BF16 ? h->wout_spk.fbf : h->wout_spk.fhi);
    ta.hwl = h->H(ta.lo8 == 2 ? h->wout_spk.fi8 : (ta.lo8 == 1 ? h->wout_spk.fl8 : h->wout_spk.flo));
    // two slices, int8 lo plane: the same lo values streamed as fp16 (no widening VALU beside the MFMAs; at two slices
    // the weight stream is not the bound). Bitwise equal to the int8 kernel: its widening is exact (tcn_common.h
    // lo8_widen), so both feed the MFMAs the same fp16 operands. SEPVAD_TCN_WQ16=0: the int8 kernel.
    // SEPVAD_TCN_WQ16=2: one-slice launches too (A/B)
    const int wq16 = env_int("SEPVAD_TCN_WQ16", 1);
    if (ta.lo8 == 2 && ((nsl == 2 && wq16 >= 1 && h->tcn2_cap_p[PREC_F16X3] >= cap) ||
                        (nsl == 1 && wq16 >= 2 && h->tcn_cap_p[PREC_F16X3] >= cap))) {
      ta.lo8 = 0;
      ta.wfrag = h->twfq;
      ta.hwl = h->H(h->wout_spk.fq);
    }
    ta.hwscale = h->P(h->wout_spk.scale); ta.hbias = h->P(h->bo_spk);
    ta.hnyw = h->P(h->out_nyw); ta.hnyb = h->P(h->out_nyb);
    if (vad_in_head) {
      ta.hvwh = h->H(h->vadw.fhi); ta.hvwl = h->H(h->vadw.flo); ta.hvwscale = h->P(h->vadw.scale);
      ta.hvwf = h->P(h->vadw.ff32);
      ta.hvny = h->P(h->vad_ny);
      ta.hvsx = h->vad_sx;
    }
    // diagnostics (SEPVAD_TCN_MAX_GROUPS): fewer groups per launch, so each loops over more utterances (tests reach
    // the epoch budget below with small batches)
    if (const int mg = env_int("SEPVAD_TCN_MAX_GROUPS", 0); mg > 0 && mg < ngroups) ngroups = mg;
    // groups above 32 members (whole files, one slice): XCD runs (tcn_kernel.h RUN: R = ceil(G / 8) consecutive members
    // per XCD, a group on 8 R blocks), where that costs this batch no group of the round; SEPVAD_TCN_RUNS=0: off
    ta.run = 0;
    if (nsl == 1 && G > 32 && env_int("SEPVAD_TCN_RUNS", 1)) {
      const int R = (G + 7) / 8;
      if (std::min(B, cap / (8 * R)) >= ngroups) ta.run = R;
    }
    const int gstride = ta.run ? 8 * ta.run : Gt;  // blocks per group
    // epochs per launch and group (tcn_kernel.h): 1 (XCD ids) + per utterance 4 per block with TF-attention (P1..P4;
    // 3 without) + 1 for the output head (P5). The tag is salt << TCN_EPOCH_BITS | epoch, so the last epoch of a
    // launch must stay below 2^TCN_EPOCH_BITS: an epoch carried into the salt bits would repeat the next launch's tags
    // (SEPVAD_TCN_MAX_ITER lowers it: tests force several launches per forward)
    const int ep_utt = 4 * h->nblk + 1;
    int max_iter = ((1 << TCN_EPOCH_BITS) - 2) / ep_utt;
    if (const int mi = env_int("SEPVAD_TCN_MAX_ITER", 0)) max_iter = std::min(max_iter, mi);
    if (max_iter < 1) return fail(SEPVAD_E_ARG, "fused TCN: too many blocks");
    if (1 + (long long)max_iter * ep_utt >= (1 << TCN_EPOCH_BITS)) return fail(SEPVAD_E_ARG, "fused TCN: epoch budget");
    const int per_launch = max_iter * ngroups;
    const char* probe_path = getenv("SEPVAD_TCN_PROBE");
    const size_t probe_n = (size_t)h->tcn_cap * h->nblk * 16 * 9;  // wave-0 region + per-wave region
    // this chunk's launch salts, reserved as one range (salt_reserve: never 0, no wrap inside the range)
    const bool warm = probe_path && env_int("SEPVAD_TCN_PROBE_WARM", 0);
    {
      const int rc = salt_reserve(h, cx, s, (unsigned)((B + per_launch - 1) / per_launch + (warm ? 1 : 0)), &gsalt_lo);
      if (rc) return rc;
    }
    gsalt_n = 0;
    for (int u0 = 0; u0 < B; u0 += per_launch) {
      const int Bl = std::min(per_launch, B - u0);
      const int ng = std::min(ngroups, Bl);
      const int ngl = ng;
      ta.tag0 = (gsalt_lo + gsalt_n++) << TCN_EPOCH_BITS;
      ta.B = Bl;
      ta.S0 = w.S0 + (size_t)u0 * Tp * CH;
      ta.ln = gn_src(w.rec_gate + (size_t)u0 * (Tp / GATE_ROWS) * 2, Tp / GATE_ROWS, 2, 0, h->P(h->ln_g), h->P(h->ln_b), 1e-8f);
      ta.hmasks = w.masks + (size_t)u0 * Tp * MOUT_PAD;
      ta.hvP = vad_in_head ? w.vP + (size_t)u0 * 2 * Tp * HEAD_VAD_N : nullptr;
      ta.probe = nullptr;
      ta.dump = (h->tdump && u0 == 0 && Bl == B) ? h->tdump : nullptr;
      if (probe_path && u0 == 0) {
        if (!h->tprobe) HIPCHK(hipMalloc(&h->tprobe, probe_n * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(h->tprobe, 0, probe_n * sizeof(unsigned long long), s));
        ta.probe = h->tprobe;
        if (warm) {  // diagnostics: an unprobed launch first (warm caches)
          TcnArgs tw = ta;
          tw.probe = nullptr;
          HIPCHK(launch_t(tw, ngl * gstride));
          ta.tag0 = (gsalt_lo + gsalt_n++) << TCN_EPOCH_BITS;
        }
      }
      ta.clk = nullptr;
      if (env_int("SEPVAD_TCN_CLOCK", 0)) {  // diagnostics: per-launch span and shader clock (sepvad_tcn_clock)
        if (!h->tclk) {
          HIPCHK(hipMalloc(&h->tclk, (size_t)TCLK_RECS * 8 * sizeof(unsigned long long)));
          HIPCHK(hipMemset(h->tclk, 0, (size_t)TCLK_RECS * 8 * sizeof(unsigned long long)));
        }
        ta.clk = h->tclk + (size_t)(h->tclk_n++ % TCLK_RECS) * 8;
        HIPCHK(hipMemsetAsync(ta.clk, 0, 8 * sizeof(unsigned long long), s));
      }
      if (env_int("SEPVAD_TCN_INFO", 0))  // diagnostics: the persistent launch's shape
        fprintf(stderr, "sepvad: k_tcn grid=%d G=%d slices=%d groups=%d B=%d capacity=%d run=%d\n", ngl * gstride, G, nsl, ngl,
                Bl, cap, ta.run);
      const bool big = tcn_big(cap, gstride) && !env_int("SEPVAD_TCN_NO_ORDER", 0);
      TailProbe thp(h, s, "tcnhead");
      ta.hprobe = u0 == 0 ? thp.buf : nullptr;
      auto run = [&]() -> int {
        if (ev()) return SEPVAD_E_HIP;
        HIPCHK(launch_t(ta, ngl * gstride));
        if (ev()) return SEPVAD_E_HIP;
        return SEPVAD_OK;
      };
      if (const int rc = big ? tcn_launch_ordered(h->device, s, run) : run()) return rc;
      if (ta.hprobe) HIPCHK(thp.dump(ngl * gstride, 1));
      if (tr) {
        tr->gemm_ev.push_back((int)h->ev.size() - 2);
        tr->g2_ev.push_back((int)h->ev.size() - 2);
      }
      if (ta.probe) {  // diagnostics only: synchronous dump {grid, nblk, G, T} + stamps
        std::vector<unsigned long long> hp(probe_n);
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemcpy(hp.data(), h->tprobe, probe_n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(probe_path, "wb")) {
          const long long hdr[4] = {(long long)ngl * gstride, h->nblk, Gt, T};
          fwrite(hdr, sizeof(hdr), 1, f);
          const size_t n0 = (size_t)ngl * gstride * h->nblk * 16;
          fwrite(hp.data(), sizeof(unsigned long long), n0, f);
          fwrite(hp.data() + n0, sizeof(unsigned long long), n0 * 8, f);  // per-wave stamps (kernel layout)
          fclose(f);
        }
      }
    }
    // the eager masks_b copy if asked
    if (out->masks_b) {
      MaskSideArgs m{};
      m.B = B; m.T = T; m.Tp = Tp; m.masks = w.masks; m.masks_b = out->masks_b + (size_t)b0 * MOUT * T;
      HIPCHK(launch_mask_side(m, s));
    }
  } else {
    // 3. TCN blocks
    int cur = 0;  // w.O[cur] holds the current block input o once the conv1d GEMM materialized it
    for (int i = 0; i < h->nblk; ++i) {
      const BlockOff& bo = h->blk[i];
      const int nxt = (i == 0) ? 0 : (cur ^ 1);
      GemmArgs g{};
      g.B = B; g.T = T; g.Tp = Tp; g.M = CH; g.Mreal = CH; g.K = CH; g.ldy = CH;
      set_weights(h, g, bo.w1);
      g.ascale = bo.sx;
      g.bias = h->P(bo.b1); g.prelu = bo.a1;
      if (i == 0) {
        g.ld.mode = LD_GN; g.ld.X = w.S0;   // TCN.LN (model/model.py:333)
        g.ld.gn = gn_src(w.rec_gate, Tp / GATE_ROWS, 2, 0, h->P(h->ln_g), h->P(h->ln_b), 1e-8f);
      } else {
        g.ld = residual_spec(h, w, i - 1, w.O[cur], w.R, Tp);
      }
      g.Xmat = w.O[nxt];
      g.Y = w.A;
      g.out_rec = w.rec_g1;
      if (probing && i == h->probe_blk) g.probe = h->probe;
      if (ev()) return SEPVAD_E_HIP;
      HIPCHK(launch_gemm(g, EP_PRELU_STATS, s));
      if (ev()) return SEPVAD_E_HIP;
      if (tr) tr->gemm_ev.push_back((int)h->ev.size() - 2);
      cur = nxt;

      DwStatsArgs d{};
      d.B = B; d.T = T; d.Tp = Tp; d.dil = bo.dil; d.A = w.A;
      const GnSrc gn1 = gn_src(w.rec_g1, ntu * (CH / TILE), 2, 0, h->P(bo.g1), h->P(bo.be1), 1e-8f);
      d.gd1 = gn1; d.wd = h->P(bo.wd); d.bd = h->P(bo.bd); d.alpha = bo.a2;
      d.prec = h->prec; d.Dhi = w.Dhi; d.Dlo = w.Dlo; d.D32 = w.D32;
      d.out_rec = w.rec_dw;
      HIPCHK(launch_dw_stats(d, s));

      GemmArgs g2{};
      g2.B = B; g2.T = T; g2.Tp = Tp; g2.M = CH; g2.Mreal = CH; g2.K = HID; g2.ldy = CH;
      set_weights(h, g2, bo.w2);
      g2.bias = h->P(bo.b2);
      if (h->prec != PREC_F32) {
        g2.ld.mode = LD_SPLIT; g2.ld.Xh = w.Dhi; g2.ld.Xl = w.Dlo;
      } else {
        g2.ld.mode = LD_PLAIN; g2.ld.X = w.D32;
      }
      g2.fold = gn_src(w.rec_dw, Tp / STAT_ROWS, 2, 0, nullptr, nullptr, bo.eps2);  // d pre-scaled (range guard)
      g2.foldK = HID; g2.foldc = h->P(bo.fc2);
      g2.Y = w.R; g2.colsum = w.colsum; g2.rowsum = w.rowsum;
      if (probing && i == h->probe_blk) g2.probe = h->probe + g1_grid * PROBE_SLOTS;
      if (ev()) return SEPVAD_E_HIP;
      HIPCHK(launch_gemm(g2, EP_BIAS_ATT, s));
      if (ev()) return SEPVAD_E_HIP;
      if (tr) {
        tr->gemm_ev.push_back((int)h->ev.size() - 2);
        tr->g2_ev.push_back((int)h->ev.size() - 2);
      }

      AttStatsArgs at{};
      at.B = B; at.T = T; at.Tp = Tp; at.mtiles = CH / TILE; at.ntiles = ntu; at.tf_att = c.tf_attention;
      at.ln_mode = c.ln_mode == SEPVAD_LN_RECURSIVE ? LD_RECURSIVE : (c.ln_mode == SEPVAD_LN_RESIDUAL ? LD_RESIDUAL : LD_ADD);
      at.R = w.R; at.O = w.O[cur]; at.colsum = w.colsum; at.rowsum = w.rowsum; at.attp = h->P(bo.attp);
      if (c.ln_mode == SEPVAD_LN_RECURSIVE) { at.ga = h->P(bo.lna_g); at.bea = h->P(bo.lna_b); }
      at.at = w.at; at.af = w.af; at.out_rec = w.rec_mom;
      HIPCHK(launch_att_stats(at, s));
    }
    // 4. output head: PReLU -> GN(1e-5) -> 1x1 256->514 (model/model.py:322-325,357)
    {
      HeadStatsArgs hs{};
      hs.B = B; hs.T = T; hs.Tp = Tp;
      hs.ld = residual_spec(h, w, h->nblk - 1, w.O[cur], w.R, Tp);
      hs.ld.alpha_h = h->out_a;
      hs.out_rec = w.rec_hs;
      HIPCHK(launch_head_stats(hs, s));
      GemmArgs g{};
      g.B = B; g.T = T; g.Tp = Tp; g.M = MOUT_PAD; g.Mreal = MOUT; g.K = CH; g.ldy = MOUT_PAD;
      set_weights(h, g, h->wout);
      g.ascale = h->out_sx;
      g.bias = h->P(h->bo);
      g.ld = residual_spec(h, w, h->nblk - 1, w.O[cur], w.R, Tp);
      g.ld.head = 1; g.ld.alpha_h = h->out_a;
      g.ld.gh = gn_src(w.rec_hs, Tp / STAT_ROWS, 2, 0, h->P(h->out_g), h->P(h->out_b), 1e-5f);
      g.Y = w.masks; g.Yside = out->masks_b ? out->masks_b + (size_t)b0 * MOUT * T : nullptr;
      if (ev()) return SEPVAD_E_HIP;
      HIPCHK(launch_gemm(g, EP_BIAS_OUT, s));
      if (ev()) return SEPVAD_E_HIP;
      if (tr) tr->gemm_ev.push_back((int)h->ev.size() - 2);
    }
  }
  stage.next("sepvad::vad");
  // 5. VAD conv1_1 (model/model.py:424-427,434-436): finished from the output head's tap products (k_vad_feat,
  // BN_1-normalised features), or the whole conv on the masks (k_vad1 + records)
  const bool kw_on = kw && kw->enabled && c.final_vad;
  // SEPVAD_VAD_FEAT=0: the tap sums finished inside k_istft_pair (one launch fewer, k_vad_feat<4>'s items and order;
  // the BN_1 affine rounds differently: VAD probabilities equal to fp32 rounding), 1: k_vad_feat. Default: inside k_istft_pair for T <= 256, where every k_istft_pair workgroup's
  // whole-utterance BN_1 sums are 2 items per thread (cfg 2: +0.4 %, 152.4k vs 151.9k utt/s interleaved,
  // profiles/r06pv/vadfeat_lines.txt; round 2 had measured equal, profiles/r02av_ab_vadfeat.txt); longer utterances
  // keep k_vad_feat (each of the T / 11 workgroups would sum all 4 T items).
  const bool vad_taps_in_istft = vad_in_head && !env_int("SEPVAD_VAD_FEAT", T > 256 ? 1 : 0);
  if (vad_in_head && !vad_taps_in_istft) {
    VadFeatArgs vf{};
    vf.B = B; vf.T = T; vf.Tp = Tp; vf.vP = w.vP;
    vf.b1 = h->P(h->v_b1); vf.alpha = h->v_a;
    vf.g = h->P(h->v_g); vf.be = h->P(h->v_b); vf.eps = 1e-8f;
    vf.feat = w.vy;
    vf.out_rec = T > VF_ONE_T ? w.rec_vad : nullptr;  // long utterances: partial records, BN_1 in k_istft_pair
    HIPCHK(launch_vad_feat(vf, s));
  }
  if (has_vad && !vad_in_head) {
    Vad1Args v{};
    v.B = B; v.T = T; v.Tp = Tp; v.masked_speakers = c.final_vad_masked_speakers;
    v.masks = w.masks; v.X = w.X;
    v.w1 = h->P(h->v_w1); v.b1 = h->P(h->v_b1); v.alpha = h->v_a;
    v.vy = w.vy; v.out_rec = w.rec_vad;
    TailProbe tp(h, s, "vad1");
    v.probe = tp.buf;
    HIPCHK(launch_vad1(v, s));
    HIPCHK(tp.dump(B * 2, Tp / VAD_ROWS));
  }
  stage.next("sepvad::istft");
  // 6. VAD tail + est = X * sigmoid(mask) [* smoothed VAD] -> iSTFT (model/model.py:429-460)
  {
    IstftArgs is{};
    is.BS = B * 2; is.S = 2; is.N = N; is.T = T; is.Tp = Tp; is.est_mode = 1;
    is.X = w.X; is.masks = w.masks;
    is.window = h->P(h->win_inv); is.tw = (const float2*)h->P(h->tw);
    is.has_vad = has_vad;
    if (has_vad) {
      is.kw_enabled = kw_on;
      is.filt = kw_on && (kw->filter_signals_by_smo_vad || kw->filter_signals_by_unsmo_vad);
      is.ret_smooth = kw_on && kw->return_smoothed_vad;
      is.thr = kw_on ? kw->threshold_activated_vad : 0.5f;
      is.vy = w.vy; is.w2 = h->P(h->v_w2); is.b2 = h->v_b2;
      is.vy_norm = vad_in_head && !vad_taps_in_istft && T <= VF_ONE_T;
      if (vad_taps_in_istft) {
        is.vP = w.vP; is.vb1 = h->P(h->v_b1); is.valpha = h->v_a; is.vy = nullptr;
      }
      is.vgn = gn_src(w.rec_vad, vad_in_head ? vf_nrec(Tp) : Tp / VAD_ROWS, 2, 0, h->P(h->v_g), h->P(h->v_b), 1e-8f);
      is.vad_out = out->vad ? out->vad + u2 * T : w.vad;
    }
    is.est_out = out->est ? (float2*)out->est + u2 * NBIN * T : nullptr;
    is.mask_out = out->mask ? out->mask + u2 * NBIN * T : nullptr;
    is.y = out->sep + u2 * N;
    if (use_fused && gsalt_n > 0) { is.gerr = cx->terr; is.gsalt_lo = gsalt_lo; is.gsalt_n = gsalt_n; }
    TailProbe tp(h, s, "istft");
    is.probe = tp.buf;
    HIPCHK(launch_istft_pair(is, s));
    HIPCHK(tp.dump(B, (T + 10) / 11));  // k_istft_pair's grid (IP_OWN = 11)
  }
  return SEPVAD_OK;
}

int forward_impl(sepvad_model* h, const float* x, int ldx, int B, int N, const SepVadOutputs* out,
                 const SepVadInferKw* kw, hipStream_t s, const XMap& xm = XMap()) {
  const int T = 1 + N / HOP;
  const int Tp = round_up(T, TILE);
  StreamCtx* cx = nullptr;
  int rc = get_ctx(h, (void*)s, &cx);
  if (rc) return rc;
  rc = check_giveup(cx);  // an earlier forward on this stream whose k_tcn gave up: report it now
  if (rc) return rc;
  rc = ws_reserve(cx, B, N);
  if (rc) return rc;
  cx->last_B = B;
  cx->last_N = N;
  cx->seq = ++h->fwd_seq;
  for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
  h->ev.clear();
  // diagnostics probe (single chunk only)
  h->probe_blk = -1;
  if (const char* pb = getenv("SEPVAD_PROBE_BLOCK")) {
    const size_t need = 2 * (size_t)B * (Tp / TILE) * (CH / TILE) * PROBE_SLOTS;
    if (need > h->probe_n) {
      if (h->probe) (void)hipFree(h->probe);
      h->probe = nullptr;
      h->probe_n = 0;
      HIPCHK(hipMalloc(&h->probe, need * sizeof(unsigned long long)));
      h->probe_n = need;
    }
    HIPCHK(hipMemsetAsync(h->probe, 0, need * sizeof(unsigned long long), s));
    h->probe_blk = atoi(pb);
  }
  const int nsplit = (h->probe_blk >= 0 || h->timing || fused_ok(h, T) || xm.nstr > 0) ? 1
                                                                                       : std::max(1, std::min(h->split, B));
  TimingRec tr;
  if (nsplit == 1) {
    if (ev_record(h, s)) return SEPVAD_E_HIP;
    rc = enqueue_chunk(h, cx, x, ldx, 0, B, N, out, kw, s, h->timing || h->probe_blk >= 0 ? &tr : nullptr, xm);
    if (rc) return rc;
    if (ev_record(h, s)) return SEPVAD_E_HIP;
  } else {
    // fork: every internal stream waits for the caller's stream; join: the caller waits for all
    HIPCHK(hipEventRecord(h->fork, s));
    int b0 = 0;
    for (int k = 0; k < nsplit; ++k) {
      const int bc = B / nsplit + (k < B % nsplit ? 1 : 0);
      HIPCHK(hipStreamWaitEvent(h->sub[k], h->fork, 0));
      rc = enqueue_chunk(h, cx, x, ldx, b0, bc, N, out, kw, h->sub[k], nullptr, xm);
      HIPCHK(hipEventRecord(h->join[k], h->sub[k]));
      HIPCHK(hipStreamWaitEvent(s, h->join[k], 0));
      if (rc) return rc;
      b0 += bc;
    }
  }
  if (h->timing) {
    HIPCHK(hipEventSynchronize(h->ev.back()));
    h->gemm_ms = h->g2_ms = 0.0;
    for (int k : tr.gemm_ev) { float ms; HIPCHK(hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1])); h->gemm_ms += ms; }
    for (int k : tr.g2_ev) { float ms; HIPCHK(hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1])); h->g2_ms += ms; }
    float tot; HIPCHK(hipEventElapsedTime(&tot, h->ev.front(), h->ev.back()));
    h->total_ms = tot;
    h->gemm_launches = (int)tr.gemm_ev.size();
    h->g2_launches = (int)tr.g2_ev.size();
  }
  if (h->probe && h->probe_blk >= 0) {
    const char* path = getenv("SEPVAD_PROBE_OUT");
    const size_t g1_grid = (size_t)B * (Tp / TILE) * (CH / TILE);
    std::vector<unsigned long long> hp(2 * g1_grid * PROBE_SLOTS);
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(hp.data(), h->probe, hp.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (path) {
      if (FILE* f = fopen(path, "wb")) {
        const long long hdr[4] = {(long long)g1_grid, PROBE_SLOTS, B, Tp};
        fwrite(hdr, sizeof(hdr), 1, f);
        fwrite(hp.data(), sizeof(unsigned long long), hp.size(), f);
        fclose(f);
      }
    }
  }
  return SEPVAD_OK;
}

}  // namespace

extern "C" {

int32_t sepvad_forward(sepvad_handle h, const float* x, int32_t B, int32_t N, const SepVadOutputs* out,
                       const SepVadInferKw* kw, void* stream) {
  return sepvad_forward_strided(h, x, N, B, N, out, kw, stream);
}

int32_t sepvad_forward_strided(sepvad_handle h, const float* x, int64_t ldx, int32_t B, int32_t N,
                               const SepVadOutputs* out, const SepVadInferKw* kw, void* stream) {
  if (!h || !x || !out || !out->sep) return fail(SEPVAD_E_ARG, "sepvad_forward: null argument");
  if (B < 1) return fail(SEPVAD_E_SHAPE, "sepvad_forward: B must be >= 1");
  if (N <= HOP) return fail(SEPVAD_E_SHAPE, "sepvad_forward: N must exceed 256 (reflect padding of the STFT)");
  if (ldx < N || ldx > INT32_MAX) return fail(SEPVAD_E_SHAPE, "sepvad_forward: row stride must be >= N");
  TraceRange trace("sepvad_forward");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  return forward_impl(h, x, (int)ldx, B, N, out, kw, (hipStream_t)stream);
}

int32_t sepvad_forward_windows(sepvad_handle h, const float* x, int64_t ld_stream, int32_t n_streams, int32_t n_win,
                               int64_t hop, int32_t N, const SepVadOutputs* out, const SepVadInferKw* kw,
                               void* stream) {
  if (!h || !x || !out || !out->sep) return fail(SEPVAD_E_ARG, "sepvad_forward_windows: null argument");
  if (n_streams < 1 || n_win < 1 || hop < 0 || (long long)n_streams * n_win > INT32_MAX)
    return fail(SEPVAD_E_SHAPE, "sepvad_forward_windows: bad window counts");
  if (N <= HOP) return fail(SEPVAD_E_SHAPE, "sepvad_forward_windows: N must exceed 256");
  if ((long long)(n_win - 1) * hop + N > ld_stream || ld_stream > INT32_MAX)
    return fail(SEPVAD_E_SHAPE, "sepvad_forward_windows: windows exceed the stream rows");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  XMap xm;
  xm.nstr = n_streams;
  xm.hopw = hop;
  return forward_impl(h, x, (int)ld_stream, n_streams * n_win, N, out, kw, (hipStream_t)stream, xm);
}

int32_t sepvad_set_split(sepvad_handle h, int32_t nsplit) {
  if (!h || nsplit < 1 || nsplit > MAX_SPLIT) return fail(SEPVAD_E_ARG, "sepvad_set_split: 1 <= n <= 4");
  h->split = nsplit;
  return SEPVAD_OK;
}
int32_t sepvad_set_fused(sepvad_handle h, int32_t on) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  h->fused = on != 0;
  return SEPVAD_OK;
}

int32_t sepvad_set_tcn_dump(sepvad_handle h, float* dump) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  std::lock_guard<std::mutex> lk(h->mu);
  h->tdump = dump;
  return SEPVAD_OK;
}

int32_t sepvad_fused_status(sepvad_handle h, int32_t* used) {
  if (!h) return fail(SEPVAD_E_ARG, "null handle");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  if (used) *used = h->last_fused ? h->last_nsl : 0;
  HIPCHK(hipDeviceSynchronize());
  int rc = SEPVAD_OK;
  for (auto& c : h->ctx) {
    const int r = check_giveup(c.get());
    if (r && rc == SEPVAD_OK) rc = r;
  }
  return rc;
}

int32_t sepvad_tcn_clock(sepvad_handle h, uint64_t* out, int32_t max_records, int32_t* n) {
  if (!h || !n || (max_records > 0 && !out)) return fail(SEPVAD_E_ARG, "sepvad_tcn_clock: null argument");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  HIPCHK(hipDeviceSynchronize());
  const long long have = std::min<long long>(h->tclk_n, TCLK_RECS);
  const int k = (int)std::min<long long>(have, std::max(0, max_records));
  *n = (int)have;
  if (k > 0) {  // the last k records, oldest first
    std::vector<unsigned long long> all((size_t)TCLK_RECS * 8);
    HIPCHK(hipMemcpy(all.data(), h->tclk, all.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int i = 0; i < k; ++i) {
      const long long r = (h->tclk_n - k + i) % TCLK_RECS;
      for (int j = 0; j < 8; ++j) out[(size_t)i * 8 + j] = all[(size_t)r * 8 + j];
    }
  }
  return SEPVAD_OK;
}

int32_t sepvad_last_forward(sepvad_handle h, void* stream, int64_t* seq, int32_t* B, int32_t* N) {
  if (!h || !seq || !B || !N) return fail(SEPVAD_E_ARG, "sepvad_last_forward: null argument");
  std::lock_guard<std::mutex> lk(h->mu);
  for (auto& c : h->ctx)
    if (c->stream == stream) {
      *seq = c->seq; *B = c->last_B; *N = c->last_N;
      return SEPVAD_OK;
    }
  return fail(SEPVAD_E_ARG, "sepvad_last_forward: no forward has run on this stream");
}

int32_t sepvad_release_stream(sepvad_handle h, void* stream) {
  if (!h) return fail(SEPVAD_E_ARG, "sepvad_release_stream: null handle");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  for (size_t i = 0; i < h->ctx.size(); ++i)
    if (h->ctx[i]->stream == stream) {
      HIPCHK(hipStreamSynchronize((hipStream_t)stream));
      free_ctx(h->ctx[i].release());
      h->ctx.erase(h->ctx.begin() + i);
      return SEPVAD_OK;
    }
  return SEPVAD_OK;  // nothing held for this stream
}

}  // extern "C"

namespace {
// sepvad_side_outputs with h->mu held by the caller (so a check of the forward's identity and the copies it guards
// are one critical section: no forward can be enqueued on the stream in between)
int side_outputs_locked(sepvad_model* h, const SepVadOutputs* out, void* stream);
}  // namespace

extern "C" {

int32_t sepvad_side_outputs_of(sepvad_handle h, const SepVadOutputs* out, void* stream, int64_t seq, int32_t Bx,
                               int32_t Nx) {
  if (!h || !out) return fail(SEPVAD_E_ARG, "sepvad_side_outputs_of: null argument");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  StreamCtx* cx = nullptr;
  for (auto& c : h->ctx)
    if (c->stream == stream) cx = c.get();
  // seq is handle-wide (never reused by a context that was evicted and recreated)
  if (!cx || cx->seq != seq || cx->last_B != Bx || cx->last_N != Nx)
    return fail(SEPVAD_E_ARG, "side outputs: a later forward on the same stream has replaced the workspace of the "
                              "forward that produced them (read them before the next forward on that stream)");
  return side_outputs_locked(h, out, stream);
}

int32_t sepvad_side_outputs(sepvad_handle h, const SepVadOutputs* out, void* stream) {
  if (!h || !out) return fail(SEPVAD_E_ARG, "sepvad_side_outputs: null argument");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  return side_outputs_locked(h, out, stream);
}

}  // extern "C"

namespace {
int side_outputs_locked(sepvad_model* h, const SepVadOutputs* out, void* stream) {
  StreamCtx* cx = nullptr;
  for (auto& c : h->ctx)
    if (c->stream == stream) cx = c.get();
  if (!cx || cx->last_B < 1) return fail(SEPVAD_E_ARG, "sepvad_side_outputs: no forward has run on this stream");
  const int B = cx->last_B, N = cx->last_N, T = 1 + N / HOP, Tp = round_up(T, TILE);
  const hipStream_t s = (hipStream_t)stream;
  const Workspace w = ws_view(cx->ws, 0, Tp);
  if (out->spectrum) {  // the gated dB spectrum, recomputed from the dB spectrum (same arithmetic as k_gate)
    GateArgs ga{};
    ga.B = B; ga.T = T; ga.Tp = Tp; ga.activity = h->cfg.activity_input;
    ga.X = h->same_stft_window ? w.X : nullptr;  // the dB spectrum from the stored STFT (or specdb)
    ga.specdb = w.specdb; ga.w = h->P(h->gate); ga.S0 = nullptr; ga.out_rec = nullptr;
    ga.spec_side = out->spectrum;
    HIPCHK(launch_gate(ga, s));
  }
  if (out->masks_b || out->mask) {
    MaskSideArgs m{};
    m.B = B; m.T = T; m.Tp = Tp; m.masks = w.masks; m.masks_b = out->masks_b; m.mask = out->mask;
    HIPCHK(launch_mask_side(m, s));
  }
  return SEPVAD_OK;
}
}  // namespace

extern "C" {

int32_t sepvad_stft_gate_test(sepvad_handle h, const float* x, int32_t B, int32_t N, void* X_fm, float* db_fm,
                              void* stream) {
  if (!h || !x || !X_fm || !db_fm || B < 1 || N <= HOP) return fail(SEPVAD_E_ARG, "sepvad_stft_gate_test: bad arguments");
  DeviceGuard dg(h->device);
  std::lock_guard<std::mutex> lk(h->mu);
  StreamCtx* cx = nullptr;
  int rc = get_ctx(h, stream, &cx);
  if (rc) return rc;
  rc = ws_reserve(cx, B, N);  // S0 and the TCN.LN records land in this stream's workspace
  if (rc) return rc;
  const int T = 1 + N / HOP, Tp = round_up(T, TILE);
  const Workspace w = ws_view(cx->ws, 0, Tp);
  StftArgs sa{};
  sa.B = B; sa.N = N; sa.ldx = N; sa.T = T; sa.Tp = Tp; sa.x = x; sa.tw = (const float2*)h->P(h->tw);
  sa.nstr = B; sa.hopw = 0;
  sa.window = h->P(h->win_out);
  sa.window_db = h->same_stft_window ? sa.window : h->P(h->win_in);
  sa.X = (float2*)X_fm; sa.specdb = db_fm; sa.db_out = 1;
  sa.activity = h->cfg.activity_input; sa.gate_w = h->P(h->gate);
  sa.S0 = w.S0; sa.gate_rec = w.rec_gate;
  HIPCHK(launch_stft_gate(sa, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_istft_pair_test(sepvad_handle h, const void* X_fm, const float* masks_fm, int32_t B, int32_t N, float* y,
                               void* est, void* stream) {
  if (!h || !X_fm || !masks_fm || !y || B < 1 || N <= HOP) return fail(SEPVAD_E_ARG, "sepvad_istft_pair_test: bad arguments");
  DeviceGuard dg(h->device);
  const int T = 1 + N / HOP, Tp = round_up(T, TILE);
  IstftArgs is{};
  is.BS = B * 2; is.S = 2; is.N = N; is.T = T; is.Tp = Tp; is.est_mode = 1;
  is.X = (const float2*)X_fm; is.masks = masks_fm;
  is.window = h->P(h->win_inv); is.tw = (const float2*)h->P(h->tw);
  is.has_vad = 0;
  is.est_out = (float2*)est; is.y = y;
  HIPCHK(launch_istft_pair(is, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_stft(sepvad_handle h, const float* x, int32_t B, int32_t N, void* X, float* spec, void* stream) {
  if (!h || !x || B < 1 || N <= HOP) return fail(SEPVAD_E_ARG, "sepvad_stft: bad arguments");
  DeviceGuard dg(h->device);
  const int T = 1 + N / HOP;
  StftArgs sa{};
  sa.B = B; sa.N = N; sa.ldx = N; sa.T = T; sa.Tp = round_up(T, TILE); sa.x = x; sa.nstr = B; sa.hopw = 0;
  sa.window = h->P(h->win_out); sa.tw = (const float2*)h->P(h->tw);
  sa.Xout = (float2*)X; sa.spec_out = h->same_stft_window ? spec : nullptr;
  HIPCHK(launch_stft(sa, (hipStream_t)stream));
  if (!h->same_stft_window && spec) {
    sa.window = h->P(h->win_in); sa.Xout = nullptr; sa.spec_out = spec;
    HIPCHK(launch_stft(sa, (hipStream_t)stream));
  }
  return SEPVAD_OK;
}

int32_t sepvad_istft(sepvad_handle h, const void* est, int32_t BS, int32_t N, float* y, void* stream) {
  if (!h || !est || !y || BS < 1 || N <= HOP) return fail(SEPVAD_E_ARG, "sepvad_istft: bad arguments");
  DeviceGuard dg(h->device);
  const int T = 1 + N / HOP;
  IstftArgs is{};
  is.BS = BS; is.S = 1; is.N = N; is.T = T; is.Tp = round_up(T, TILE); is.est_mode = 0;
  is.est_in = (const float2*)est; is.window = h->P(h->win_inv); is.tw = (const float2*)h->P(h->tw); is.y = y;
  HIPCHK(launch_istft(is, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_pit_l1(const float* est, int64_t est_ld, const float* ref, int64_t ref_ld, int32_t B, int64_t L,
                      void* scratch, int64_t* perm_out, float* loss_out, float* pw_out, void* stream) {
  if (!est || !ref || !scratch || B < 1 || L < 1 || est_ld < L || ref_ld < L)
    return fail(SEPVAD_E_ARG, "sepvad_pit_l1: bad arguments");
  PitArgs a{};
  a.B = B; a.L = L; a.est = est; a.est_ld = est_ld; a.ref = ref; a.ref_ld = ref_ld;
  a.nblk = (int)std::min<long long>(PIT_MAX_BLOCKS, std::max<long long>(1, ((long long)B * L + 8191) / 8192));
  static_assert((PIT_MAX_BLOCKS + 1) * 4 * sizeof(double) <= SEPVAD_PIT_SCRATCH_BYTES, "scratch size");
  a.partial = (double*)scratch;
  a.perm_out = (long long*)perm_out; a.loss_out = loss_out; a.pw_out = pw_out;
  HIPCHK(launch_pit_l1(a, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_pit_l1_sums(const float* est, int64_t est_ld, const float* ref, int64_t ref_ld, int32_t B, int64_t L,
                           void* scratch, double* sums, void* stream) {
  if (!est || !ref || !scratch || !sums || B < 1 || L < 1 || est_ld < L || ref_ld < L)
    return fail(SEPVAD_E_ARG, "sepvad_pit_l1_sums: bad arguments");
  PitArgs a{};
  a.B = B; a.L = L; a.est = est; a.est_ld = est_ld; a.ref = ref; a.ref_ld = ref_ld;
  a.nblk = (int)std::min<long long>(PIT_MAX_BLOCKS, std::max<long long>(1, ((long long)B * L + 8191) / 8192));
  a.partial = (double*)scratch;
  HIPCHK(launch_pit_l1_sums(a, sums, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_pit_l1_choose(const double* sums, double count, int32_t B, int64_t* perm_out, float* loss_out,
                             float* pw_out, void* stream) {
  if (!sums || B < 1 || !(count > 0.0)) return fail(SEPVAD_E_ARG, "sepvad_pit_l1_choose: bad arguments");
  PitArgs a{};
  a.B = B; a.perm_out = (long long*)perm_out; a.loss_out = loss_out; a.pw_out = pw_out;
  HIPCHK(launch_pit_l1_choose(a, sums, count, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_stream_append(const float* src, int64_t src_ld, int64_t s0, int32_t B, int64_t H,
                             const int64_t* perm, float* dst, int64_t dst_ld, int64_t d0, void* stream) {
  if (!src || !dst || B < 1 || H < 1 || s0 < 0 || d0 < 0 || s0 + H > src_ld || d0 + H > dst_ld)
    return fail(SEPVAD_E_ARG, "sepvad_stream_append: bad arguments");
  AppendArgs a{};
  a.B = B; a.H = H; a.src = src; a.src_ld = src_ld; a.s0 = s0; a.perm = (const long long*)perm;
  a.dst = dst; a.dst_ld = dst_ld; a.d0 = d0;
  HIPCHK(launch_stream_append(a, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_resample_filter(int32_t orig_freq, int32_t new_freq, float* taps, int32_t cap, int32_t* info) {
  if (orig_freq < 1 || new_freq < 1 || !info) return fail(SEPVAD_E_ARG, "sepvad_resample_filter: bad arguments");
  // torchaudio.functional.functional._get_sinc_resample_kernel, sinc_interp_hann, width 6, rolloff 0.99
  const int g = std::gcd(orig_freq, new_freq);
  const int o = orig_freq / g, nw = new_freq / g;
  const double lpw = 6.0, base = std::min(o, nw) * 0.99;
  const int width = (int)std::ceil(lpw * o / base);
  const int ntaps = 2 * width + o;
  info[0] = nw; info[1] = ntaps; info[2] = o; info[3] = width;
  if ((long long)nw * ntaps > (1 << 22)) return fail(SEPVAD_E_ARG, "sepvad_resample_filter: ratio too large");
  if (!taps) return SEPVAD_OK;  // size query
  if (cap < nw * ntaps) return fail(SEPVAD_E_ARG, "sepvad_resample_filter: taps capacity too small");
  for (int j = 0; j < nw; ++j) {
    for (int i = 0; i < ntaps; ++i) {
      double t = -(double)j / nw + (double)(i - width) / o;
      t *= base;
      t = std::min(lpw, std::max(-lpw, t));
      const double c = std::cos(t * M_PI / lpw / 2.0);
      const double win = c * c;
      t *= M_PI;
      const double k = (t == 0.0) ? 1.0 : std::sin(t) / t;
      taps[j * ntaps + i] = (float)(k * win * (base / o));
    }
  }
  return SEPVAD_OK;
}

int32_t sepvad_resample(const float* x, int64_t n, const float* taps, const int32_t* info, float* y, int64_t ylen,
                        void* stream) {
  if (!x || !taps || !info || !y || n < 1 || ylen < 1) return fail(SEPVAD_E_ARG, "sepvad_resample: bad arguments");
  ResampleArgs a{};
  a.x = x; a.n = n; a.taps = taps; a.phases = info[0]; a.ntaps = info[1]; a.stride = info[2]; a.width = info[3];
  a.y = y; a.ylen = ylen;
  const long long full = (long long)std::ceil((double)a.phases * (double)n / (double)a.stride);
  if (ylen > full) return fail(SEPVAD_E_ARG, "sepvad_resample: ylen exceeds ceil(new * n / orig)");
  HIPCHK(launch_resample(a, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_si_sdr(const float* P, int64_t p_ld, const float* Tg, int64_t t_ld, int64_t N, int32_t R,
                      const int32_t* pidx, const int32_t* tidx, int32_t zero_mean, float* out, void* stream) {
  if (!P || !Tg || !out || N < 1 || R < 1 || p_ld < N || t_ld < N) return fail(SEPVAD_E_ARG, "sepvad_si_sdr: bad arguments");
  SiSdrArgs a{};
  a.P = P; a.p_ld = p_ld; a.Tg = Tg; a.t_ld = t_ld; a.N = N; a.R = R; a.pidx = pidx; a.tidx = tidx;
  a.zero_mean = zero_mean; a.out = out;
  HIPCHK(launch_si_sdr(a, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_vad_accuracy(float* preds, const float* targets, int32_t B, int32_t S, int32_t T, int32_t in_place,
                            float* out, void* stream) {
  if (!preds || !targets || !out || B < 1 || S < 1 || S > VACC_MAX_S || T < 1)
    return fail(SEPVAD_E_ARG, "sepvad_vad_accuracy: bad arguments");
  VadAccArgs a{};
  a.preds = preds; a.targets = targets; a.B = B; a.S = S; a.T = T; a.in_place = in_place; a.out = out;
  HIPCHK(launch_vad_acc(a, (hipStream_t)stream));
  return SEPVAD_OK;
}

int32_t sepvad_normalize(const float* x, int64_t n, float* y, void* scratch, void* stream) {
  if (!x || !y || !scratch || n < 1) return fail(SEPVAD_E_ARG, "sepvad_normalize: bad arguments");
  static_assert(NORM_MAX_BLOCKS * 2 * sizeof(float) <= SEPVAD_NORM_SCRATCH_BYTES, "scratch size");
  NormArgs a{};
  a.x = x; a.n = n; a.y = y; a.part = (float*)scratch;
  HIPCHK(launch_normalize(a, (hipStream_t)stream));
  return SEPVAD_OK;
}

void sepvad_destroy(sepvad_handle h) {
  if (!h) return;
  DeviceGuard dg(h->device);
  for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
  if (h->probe) (void)hipFree(h->probe);
  for (int k = 0; k < MAX_SPLIT; ++k) {
    if (h->sub[k]) (void)hipStreamDestroy(h->sub[k]);
    if (h->join[k]) (void)hipEventDestroy(h->join[k]);
  }
  if (h->fork) (void)hipEventDestroy(h->fork);
  for (auto& c : h->ctx) free_ctx(c.release());
  if (h->twf) (void)hipFree(h->twf);
  if (h->twfq) (void)hipFree(h->twfq);
  for (__half* q : h->twq)
    if (q) (void)hipFree(q);
  if (h->twf16) (void)hipFree(h->twf16);
  if (h->twbf) (void)hipFree(h->twbf);
  if (h->twf32) (void)hipFree(h->twf32);
  if (h->tprm) (void)hipFree(h->tprm);
  if (h->tprobe) (void)hipFree(h->tprobe);
  if (h->tclk) (void)hipFree(h->tclk);
  if (h->kprobe) (void)hipFree(h->kprobe);
  if (h->dparams) (void)hipFree(h->dparams);
  if (h->dhalf) (void)hipFree(h->dhalf);
  delete h;
}

}  // extern "C"
