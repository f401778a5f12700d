// Internal declarations shared by the kernel translation units and the C-ABI layer.
// Layout conventions (see DESIGN.md "Data layout in HBM"):
//   * TCN activations are channel-last per utterance: [B][Tp][C], Tp = roundup(T, 64); rows
//     t >= T are padding that is never reduced over nor used as conv context (zero-padding is
//     applied explicitly), so a GEMM tile of 64 rows never straddles two utterances;
//   * spectra are frame-major: X [B][Tp][257] complex (float2), specdb [B][Tp][SPEC_LD];
//   * GroupNorm statistics travel as deterministic per-workgroup partial records in double
//     (never float atomics), so results are bitwise reproducible run to run and shard to shard.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>

namespace sepvad {

constexpr int NFFT = 512;   // n_fftBins (model/model.py:362)
constexpr int HOP = 256;    // n_fftBins/2 (model/model.py:378)
constexpr int NBIN = 257;   // n_fftBins/2+1
constexpr int CH = 256;     // BN_dim == TCN input channels (non-DC bins)
constexpr int HID = 512;    // H_dim (depthwise multiplier 2)
constexpr int TILE = 64;    // GEMM tile edge; Tp is a multiple of TILE
constexpr int MOUT = 2 * NBIN;  // 514 output-head rows (2 speakers x 257 bins)
constexpr int MOUT_PAD = 576;   // padded to a multiple of 64 (also the row stride of `masks`)
constexpr int HEAD_SPK = MOUT_PAD / 2;  // the output head's per-speaker row block (257 rows + zero rows)
constexpr int HEAD_VAD_N = 20;          // VAD conv1_1 tap products per frame: 5 taps x 4 outputs
constexpr int SPEC_LD = 260;    // row stride of the frame-major dB spectrum
constexpr int STAT_ROWS = 8;    // rows (frames) per workgroup of the stats kernels
constexpr int PROBE_SLOTS = 16;  // per-workgroup timestamps of a probed GEMM launch
constexpr int NMOM = 11;        // moment record of k_att_stats (see device_common.h)

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// GEMM arithmetic. F32 and F16X3 are fp32-equivalent (parity path); F16 and BF16 are the reduced-
// precision arms (one fp16 / bf16 product per MAC, fp32 accumulation; BASELINE cfg 2 bf16, cfg 5 fp16).
enum Precision { PREC_F32 = 0, PREC_F16X3 = 1, PREC_F16 = 2, PREC_BF16 = 3 };

// Residual-stream transform applied to the GEMM A operand as it is staged (normalize-on-load).
enum LoadMode {
  LD_PLAIN = 0,      // x
  LD_GN = 1,         // GroupNorm(1,K)(x)                              (stats: slots)
  LD_RECURSIVE = 2,  // GN_b(o + GN_a(o + r'))   model/model.py:347-348 (stats: moment records)
  LD_RESIDUAL = 3,   // o + GN_c(r')             model/model.py:349-350 (stats of r': records)
  LD_ADD = 4,        // o + r'                   model/model.py:351-352
  LD_SPLIT = 5       // A already split into fp16 hi/lo planes (d from k_dw_stats; res_out operand)
};
// r' = r * (a_f[c] * a_t[t])  (TF_Attention, model/model.py:206-207), or r when tf_attention is off.

enum EpiMode {
  EP_PRELU_STATS = 0,  // + bias, PReLU, store, GN partial stats       (DepthConv1d.conv1d)
  EP_BIAS_ATT = 1,     // + bias, store, channel/time partial sums      (DepthConv1d.res_out -> TF_Attention)
  EP_BIAS_OUT = 2      // + bias, store columns < Mreal, optional freq-major copy  (TCN.output.2)
};

// GroupNorm statistics source: partial records [B][nrec][rstride] written by a producer kernel
// ((sum, sumsq) at [roff, roff+1]); every consumer turns them into the affine in its prologue.
struct GnSrc {
  const double* rec; int nrec, rstride, roff;
  const float* g; const float* be; float eps;
};

struct LoadSpec {
  int mode;
  const float* X;        // [B][Tp][K]  o (or x)
  const float* X2;       // [B][Tp][K]  r (res_out output) for RECURSIVE/RESIDUAL/ADD
  const float* at;       // [B][Tp] time gate  (nullable => 1)
  const float* af;       // [B][K]  freq gate  (nullable => 1)
  const __half* Xh;      // LD_SPLIT: [B][Tp][K] fp16 hi plane
  const __half* Xl;      // LD_SPLIT: [B][Tp][K] fp16 lo plane
  GnSrc gn;              // LD_GN: GN; LD_RESIDUAL: GN_c of r'; LD_RECURSIVE: GN_a (moment records)
  const float* g2; const float* be2; float eps2;   // GN_b (recursive)
  double wsum[5];                                  // recursive: {Σg, Σbe, Σbe², Σg·be, Σg²} of GN_a
  // head: x' = GN_out(PReLU(transform(x)))  (model/model.py:322-325)
  int head;
  float alpha_h;
  GnSrc gh;
};

struct GemmArgs {
  int B, T, Tp, M, Mreal, K, ldy;
  int prec;
  const float* W32;                        // [M][K] fp32 (PREC_F32)
  const __half* Whi; const __half* Wlo;    // [M][K] fp16 split of (w * 2^-e_m)  (PREC_F16X3; F16 uses Whi)
  const __half* Wbf;                       // [M][K] bf16 bits of (w * 2^-e_m)  (PREC_BF16)
  const float* wscale;                     // [M] 2^e_m (F16X3)
  const float* bias;                       // [M]
  float prelu;
  float ascale;         // F16X3: power-of-two scale of the A operand before the fp16 split (range guard;
                        // undone exactly by wscale, which carries the inverse)
  LoadSpec ld;
  float* Xmat;          // nullable: transformed A operand x' written once (by m-tile 0), [B][Tp][K]
  float* Y;             // [B][Tp][ldy]
  float* Yside;         // nullable [B][Mreal][T] (freq-major copy: self.masks_b)
  double* out_rec;      // EP_PRELU_STATS: [B][(Tp/64)*(M/64)][2] partial (sum, sumsq)
  float* colsum;        // EP_BIAS_ATT: [B][M/64][Tp]   partial sums over channels
  float* rowsum;        // EP_BIAS_ATT: [B][Tp/64][M]   partial sums over frames
  // EP_BIAS_ATT: GroupNorm of the A operand folded out of the GEMM (gamma pre-multiplied into W):
  // y = rstd * (acc - mu * foldc[m]) + bias[m]  with (mu, rstd) of `fold` over foldK x T values
  GnSrc fold;
  int foldK;
  const float* foldc;   // [M] sum_k W'[m][k]
  unsigned long long* probe;  // diagnostics (SEPVAD_PROBE_BLOCK): [grid][PROBE_SLOTS] wall-clock stamps
};

struct DwStatsArgs {     // d = PReLU(dconv(GN1(a))) (the res_out A operand) + its statistics for GN2 (reg2)
  int B, T, Tp, dil, prec;
  const float* A;        // [B][Tp][CH]
  GnSrc gd1;             // GN1 (reg1) of a
  const float* wd; const float* bd; float alpha;
  __half* Dhi; __half* Dlo;  // PREC_F16X3: [B][Tp][HID] split of d (rows >= T zero)
  float* D32;            // PREC_F32: [B][Tp][HID] d
  double* out_rec;       // [B][Tp/STAT_ROWS][2]
};

struct AttStatsArgs {    // TF-attention gates + the moment records of the residual update
  int B, T, Tp, mtiles, ntiles, tf_att, ln_mode;
  const float* R;        // [B][Tp][CH]
  const float* O;        // [B][Tp][CH]
  const float* colsum;   // [B][mtiles][Tp]
  const float* rowsum;   // [B][ntiles][CH]
  const float* attp;     // t1w[3] t1b t2w[3] t2b f1w[3] f1b f2w[3] f2b ; [16] prelu_t, [17] prelu_f
  const float* ga; const float* bea;  // GN_a (recursive) affine: weights of the moment record
  float* at;             // [B][Tp]
  float* af;             // [B][CH]
  double* out_rec;       // [B][Tp/STAT_ROWS][NMOM]
};

struct HeadStatsArgs {   // statistics of PReLU(o_final) for TCN.output.1
  int B, T, Tp;
  LoadSpec ld;
  double* out_rec;       // [B][Tp/STAT_ROWS][2]
};

struct GateArgs {
  int B, T, Tp, activity;
  const float* specdb;   // [B][Tp][SPEC_LD] (used when X is null)
  const float2* X;       // nullable [B][Tp][NBIN]: the dB spectrum recomputed from the stored STFT (side pass)
  const float* w;        // activity_input.weight [9] ; bias at w[9]; prelu at w[10]
  float* S0;             // [B][Tp][CH] gated bins 1..256 (nullable: side-output pass)
  float* spec_side;      // nullable [B][NBIN][T] (self.spectrum)
  double* out_rec;       // [B][Tp/GATE_ROWS][2] (nullable: side-output pass)
};
constexpr int GATE_ROWS = 16;

struct StftArgs {
  int B, N, ldx, T, Tp;
  int nstr;              // utterance u reads x + (u % nstr) * ldx + (u / nstr) * hopw: nstr = B, hopw = 0 for a
  long long hopw;        // plain batch; streaming windows: u = window * nstr + stream (sepvad_forward_windows)
  const float* x;        // [B][ldx] (row stride ldx >= N: streaming windows are strided views)
  const float* window;   // [512]
  const float2* tw;      // [512] e^{-2 pi i m / 512}
  float2* X;             // nullable [B][Tp][NBIN]
  float2* Xout;          // nullable [B][NBIN][T] (debug entry)
  float* specdb;         // nullable [B][Tp][SPEC_LD]
  float* spec_out;       // nullable [B][NBIN][T] (debug entry)
  // fused STFT + activity gate (k_stft_gate, the forward): window_db != window only when the checkpoint's
  // spec_input and spec_output windows differ (then specdb keeps the dB spectrum for the side pass)
  const float* window_db;
  int activity;
  const float* gate_w;   // activity_input.weight [9], bias [9], prelu [10]
  float* S0;             // [B][Tp][CH] gated bins 1..256 (TCN input)
  double* gate_rec;      // [B][Tp/GATE_ROWS][2] TCN.LN partial statistics
  int db_out;            // k_stft_gate: also store the dB spectrum (specdb) when the windows are equal (test entry)
  unsigned long long* probe;  // nullable diagnostics (SEPVAD_TAIL_PROBE): [workgroups][8] phase stamps
};
hipError_t launch_stft_gate(const StftArgs& a, hipStream_t s);

constexpr int VAD_ROWS = 32;
struct Vad1Args {        // VAD conv1_1 (257->4, k=5) + bias + PReLU and GN(1,4) partial stats
  int B, T, Tp, masked_speakers;
  const float* masks;    // [B][Tp][MOUT_PAD] pre-sigmoid
  const float2* X;       // [B][Tp][NBIN]
  const float* w1;       // [4][257][5]
  const float* b1;       // [4]
  float alpha;
  float* vy;             // [B][2][4][Tp]
  double* out_rec;       // [B*2][Tp/VAD_ROWS][2]
  unsigned long long* probe;  // nullable diagnostics (SEPVAD_TAIL_PROBE): [workgroups][8] phase stamps
};

struct VadFeatArgs {     // k_vad_feat: conv1_1 finish + BN_1 from the output head's tap products
  int B, T, Tp;
  const float* vP;       // [B][2][Tp][HEAD_VAD_N]
  const float* b1; float alpha;       // conv1_1 bias [4], relu_1 PReLU
  const float* g; const float* be; float eps;  // BN_1 affine, eps
  float* feat;           // [B][2][4][Tp] normalised features (the k_istft VAD tail's input)
  double* out_rec;       // T > VF_ONE_T: [B*2][vf_nrec(Tp)][2] BN_1 partial records; feat is then un-normalised
};
// k_vad_feat finishes BN_1 itself up to VF_ONE_T frames (one workgroup per utterance and speaker); longer utterances run
// k_vad_feat_rec (one workgroup per VF_ROWS frames, partial records, BN_1 applied by k_istft_pair)
constexpr int VF_ONE_T = 1024, VF_ROWS = 128;
__host__ __device__ inline int vf_nrec(int Tp) { return (Tp + VF_ROWS - 1) / VF_ROWS; }
hipError_t launch_vad_feat(const VadFeatArgs& a, hipStream_t s);

struct IstftArgs {
  int BS, S, N, T, Tp, est_mode;  // est_mode 1: forward (mask X, VAD); 0: est given (debug entry)
  const float2* X;       // [B][Tp][NBIN]
  const float* masks;    // [B][Tp][MOUT_PAD] pre-sigmoid
  const float2* est_in;  // [BS][NBIN][T] (est_mode 0)
  const float* window;   // [512]
  const float2* tw;      // [512]
  // VAD tail (model/model.py:160-179,444-457); has_vad = 0 -> no VAD, gain 1
  int has_vad, kw_enabled, filt, ret_smooth;
  float thr;
  const float* vy;       // [B][S][4][Tp] PReLU(conv1_1) output (k_vad1), or BN_1-normalised (vy_norm)
  int vy_norm;           // vy already normalised (k_vad_feat): no BN_1 records
  const float* vP;       // nullable: the output head's conv1_1 tap products [B][2][Tp][HEAD_VAD_N]; the workgroup finishes
                         // conv1_1 + PReLU + BN_1 itself (k_vad_feat's arithmetic, no vy / records)
  const float* vb1; float valpha;     // conv1_1 bias [4], relu_1 PReLU (vP mode)
  GnSrc vgn;             // BN_1 = GroupNorm(1, 4) over [4, T] per (utterance, speaker); rec [B*S][..]
  const float* w2; float b2;          // output_layer_vad [4][3], bias
  float* vad_out;        // [B][S][T]
  float2* est_out;       // nullable [BS][NBIN][T]
  float* mask_out;       // nullable [BS][NBIN][T]
  float* y;              // [BS][N]
  unsigned long long* probe;  // nullable diagnostics (SEPVAD_TAIL_PROBE): [workgroups][8] phase stamps
  // give-up poisoning (fused TCN): when the stream context's give-up word (tag0 of a k_tcn launch whose bounded
  // hand-off wait gave up) names one of this forward's launches (salts gsalt_lo .. gsalt_lo + gsalt_n - 1, modulo the
  // salt width), every output of the launch (sep, vad, est, mask) is written as NaN: no invalid output is returned
  // as a valid one, stream-ordered, no host synchronisation. gerr nullable (no fused TCN in this forward).
  const unsigned* gerr;
  unsigned gsalt_lo, gsalt_n;
};

// streaming wrapper (stream.hip)
constexpr int PIT_MAX_BLOCKS = 512;
struct PitArgs {
  int B, nblk;
  long long L;                 // compared samples per (utterance, speaker)
  const float* est; long long est_ld;   // [B][2][est_ld], region starts at est
  const float* ref; long long ref_ld;   // [B][2][ref_ld]
  double* partial;             // [nblk][4]
  long long* perm_out;         // nullable [B][2] (torch.long batch_indices)
  float* loss_out;             // nullable scalar: min permutation loss
  float* pw_out;               // nullable [2][2] pairwise losses [est][target]
};
struct AppendArgs {
  int B;
  long long H;                 // samples per speaker row to move
  const float* src; long long src_ld, s0;
  const long long* perm;       // nullable [B][2]
  float* dst; long long dst_ld, d0;
};
hipError_t launch_pit_l1(const PitArgs& a, hipStream_t s);
hipError_t launch_pit_l1_sums(const PitArgs& a, double* sums, hipStream_t s);     // partials -> sums[4] (fixed order)
hipError_t launch_pit_l1_choose(const PitArgs& a, const double* sums, double count, hipStream_t s);
hipError_t launch_stream_append(const AppendArgs& a, hipStream_t s);

// input preprocessing (prep.hip)
constexpr int NORM_MAX_BLOCKS = 1024;
struct ResampleArgs {
  const float* x; long long n;   // input samples
  const float* taps;             // [phases][ntaps] device
  int phases, ntaps, stride, width;
  float* y; long long ylen;
};
struct NormArgs {
  const float* x; long long n;
  float* y;
  float* part;                   // [NORM_MAX_BLOCKS][2] scratch
};
hipError_t launch_resample(const ResampleArgs& a, hipStream_t s);

// quality metrics (metrics.hip)
struct SiSdrArgs {
  const float* P; long long p_ld;
  const float* Tg; long long t_ld;
  long long N; int R;
  const int* pidx; const int* tidx;
  int zero_mean;
  float* out;
};
hipError_t launch_si_sdr(const SiSdrArgs& a, hipStream_t s);
constexpr int VACC_MAX_S = 8;
struct VadAccArgs {
  float* preds; const float* targets;   // [B][S][T]
  int B, S, T, in_place;
  float* out;                           // [1 + S]: overall, per speaker
};
hipError_t launch_vad_acc(const VadAccArgs& a, hipStream_t s);
hipError_t launch_normalize(const NormArgs& a, hipStream_t s);

// ---- fused persistent TCN (tcn_kernel.h; dispatch fused.hip, instantiations fused_inst.hip) ----
constexpr int FR = 32;          // frames per workgroup
#ifndef SEPVAD_FG_MAX
#define SEPVAD_FG_MAX 256
#endif
constexpr int FG_MAX = SEPVAD_FG_MAX;  // workgroups per utterance (T <= 8192: 131 s at 16 kHz in one fused forward; groups
                                // above 32 members span XCDs and hand off through write-through words)
constexpr int FG_CHUNK = 8;     // members polled / summed per pass (register budget of the polls)
constexpr int FG_WAVE = 16;     // groups up to this size keep the GN1/GN2 words in one wave (readlane finish)
constexpr int NGR = 2624;       // 8-byte {tag, value} hand-off words per slot (P1 rows, P3 sums, tree partials: GW_*)
#ifndef SEPVAD_FG_TREE
#define SEPVAD_FG_TREE 16
#endif
constexpr int FG_TREE = SEPVAD_FG_TREE;     // groups above this many members reduce P3 / P4 in two levels (8 leaders)
constexpr int TCN_EPOCH_BITS = 12;  // tag = launch salt << 12 | epoch; epochs per launch < 4096
// Per-block parameter blob of the fused TCN (floats; staged into LDS once per block):
constexpr int PB_WS1 = 0, PB_B1 = 256, PB_G1 = 512, PB_BE1 = 768;   // conv1d row scales, bias; reg1 affine
constexpr int PB_WD = 1024, PB_BD = 2560;                          // depthwise [512][3], bias [512]
constexpr int PB_WS2 = 3072, PB_B2 = 3328, PB_FC2 = 3584;          // res_out row scales, folded bias, sum_k W'
constexpr int PB_LNAG = 3840, PB_LNAB = 4096, PB_LNBG = 4352, PB_LNBB = 4608;  // ln_first / ln_second (or ln_modules)
constexpr int PB_ATT = 4864;                                       // TF_Attention taps [20] (see AttStatsArgs)
constexpr int PB_A1 = 4884, PB_A2 = 4885;                          // PReLU slopes
constexpr int PB_SX = 4886, PB_SXN = 4887;                         // fp16 range scale of this / the next block's x'
constexpr int PB_WSUM = 4888;                                      // 5 doubles (8-byte aligned)
constexpr int PB_EPS2 = 4898;                                      // reg2 eps, rescaled with d (see api.hip range guard)
constexpr int PB_SFC2 = 4899, PB_SB2 = 4900;                       // sum_c fc2[c], sum_c b2[c] (frame means of r)
constexpr int PB_SIZE = 4904;                                      // multiple of 4 (float4 staging)
// fp16 hi/lo weights of one block in MFMA fragment order: conv1d hi | lo (256x256) | res_out hi | lo (256x512)
constexpr size_t WF_W1L = 65536, WF_W2H = 131072, WF_W2L = 262144, WF_BLOCK = 393216;  // halves
// single-plane (PREC_F16 / PREC_BF16) blobs: conv1d (256x256) | res_out (256x512)
constexpr size_t WS_W2 = 65536, WS_BLOCK = 196608;  // halves
// fused TCN, PREC_F32: conv1d (256x256) | res_out (256x512) as fp32 fragments (8 floats per lane per K step), in
// __half units of the blob pointer
constexpr size_t WS32_W2 = 2 * 65536, WS32_BLOCK = 2 * 196608;
// F16X3 with an e4m3 lo plane (k_tcn default, SEPVAD_WLO_E4M3): conv1d hi (256x256 halves) | conv1d lo (256x256
// bytes) | res_out hi (256x512 halves) | res_out lo (bytes). A lo byte is e4m3fn(lo * 2^WQ_LO_SHIFT): |lo| <= 2^-12 of
// the row-scaled weight, so the stored value is <= 2^7 (e4m3 max 448) and keeps 4 significant bits down to 2^-25.
// Lo fragment order: [row tile][K-step PAIR][64 lanes][16 bytes: 8 of step 2p, 8 of step 2p+1] (one 1 KB wave load
// per two K steps; the hi plane keeps one per step).
constexpr size_t WQ_W1L = 65536, WQ_W2H = 98304, WQ_W2L = 229376, WQ_BLOCK = 294912;  // halves
constexpr int WQ_LO_SHIFT = 19;
struct TcnArgs {
  int B, T, Tp, G, nblk, layer, ln_mode, tf_att, prec;
  int nsl;               // 32-frame slices (members) per workgroup: 1, or 2 (64 frames, G even and <= FG_WAVE)
  int run;               // > 0: XCD runs of `run` = ceil(G / 8) consecutive members (G > 32, one slice), 8 run blocks per group
  int lo8;               // F16X3 weight lo plane: 0 fp16 (WF_* layout), 1 e4m3, 2 int8 (WQ_* layout)
  const __half* wfrag;   // [nblk][WF_BLOCK | WQ_BLOCK] (F16X3) or [nblk][WS_BLOCK] (F16 / BF16 bits) fragment-ordered weights
  const float* prm;      // [nblk][PB_SIZE] parameter blobs
  const float* S0;       // [B][Tp][CH] TCN input (gated spectrum bins 1..256)
  GnSrc ln;              // TCN.LN statistics records (k_gate) + affine
  float alpha_h;         // TCN.output.0 PReLU
  unsigned long long* gran;  // hand-off words [grid * nsl][2][NGR] (one slot pair per member)
  unsigned tag0;         // launch salt << TCN_EPOCH_BITS (tags of this launch: tag0 + epoch, epoch >= 1)
  unsigned* err;         // device word: tag0 of the last launch on this stream context whose hand-off wait gave up
  unsigned* herr;        // host-mapped (pinned) copy of the same word, read by the host without a sync
  unsigned spin_limit;   // poll passes before a wait gives up (default 1 << 20)
  int force_err;         // diagnostics (SEPVAD_TCN_FORCE_GIVEUP): report a give-up without one happening
  double inv_ch, inv_hid;  // 1 / (CH * T), 1 / (HID * T): GroupNorm counts
  int xmode;             // hand-off protocol: 0 = L2-resident when a group shares one XCD, else write-through;
                         // 1 = always write-through (tests)
  unsigned long long* probe;  // diagnostics: [grid][nblk][16] phase timestamps (nullable)
  unsigned long long* clk;    // diagnostics (SEPVAD_TCN_CLOCK), nullable: this launch's record {~min start, max end
                              // (100 MHz wall clock), workgroup 0: start, end wall clock, start, end shader clock}
  float* dump;           // parity probe (sepvad_set_tcn_dump), nullable: [3][B][Tp][CH] = TCN.LN output x'_0,
                         // block 0's res_out output r and its TF-attention output r * a_f * a_t
  unsigned dbg_delay;    // diagnostics (SEPVAD_TCN_DELAY): member 0 of each group sleeps before its polls (0: off)
  int dump_blk;          // parity probe: the block whose input (dump slot 0 when > 0), r and r a_f a_t are dumped
  // output head after each utterance's last block (model/model.py:322-325,357): PReLU -> GroupNorm(1e-5) -> 1x1
  // 256 -> 514 on the member's slice, and the VAD conv1_1 tap products of the masks (model/model.py:158-160)
  float* hmasks;         // [B][Tp][MOUT_PAD] pre-sigmoid masks, speaker q's bins at [q * 257, q * 257 + 257)
  const float* hg; const float* hbe;  // TCN.output.1 affine
  float hsx;             // range scale of the head's A operand (undone by hwscale)
  const __half* hwh; const __half* hwl;  // speaker-padded rows (288 per speaker), fragment order, the blocks' lo format
  const float* hwscale; const float* hbias;  // [MOUT_PAD]
  const float* hnyw; const float* hnyb;  // bin 256 of each speaker (fp32 VALU): weights [2][CH], bias [2]
  // VAD conv1_1 as a second GEMM on each masks tile (nullable hvP: off): hvP[b][s][t][4 k + o] =
  // sum_c masks[t][s 257 + c] w1[o][c][k], zero for t >= T; B planes in fragment order, per-column scale; bin 256's
  // term w1[o][256][k] (hvny[4 k + o]) in fp32
  const __half* hvwh; const __half* hvwl; const float* hvwscale; const float* hvny;
  const float* hvwf;     // PREC_F32: the VAD conv1_1 weights as fp32 fragments (the order of hvwh)
  float hvsx;            // range scale of the masks tile as the VAD GEMM's A operand (undone by hvwscale)
  float* hvP;            // nullable [B][2][Tp][HEAD_VAD_N]
  unsigned long long* hprobe;  // nullable diagnostics (SEPVAD_TAIL_PROBE): [grid][8] fused-head phase stamps
};
hipError_t launch_tcn(const TcnArgs& a, int grid, hipStream_t s);
int tcn_blocks_per_cu(int ln_mode, int prec, int lo, int nsl = 1);
// host: float -> e4m3fn (OCP FP8, bias 7, max 448, no inf), round to nearest even, saturating
uint8_t e4m3_rn(float x);

hipError_t launch_gemm(const GemmArgs& a, int ep, hipStream_t s);
hipError_t launch_dw_stats(const DwStatsArgs& a, hipStream_t s);
hipError_t launch_att_stats(const AttStatsArgs& a, hipStream_t s);
hipError_t launch_head_stats(const HeadStatsArgs& a, hipStream_t s);
hipError_t launch_gate(const GateArgs& a, hipStream_t s);
struct MaskSideArgs {    // bin-major copies of the head output (side attributes, materialised on access)
  int B, T, Tp;
  const float* masks;    // [B][Tp][MOUT_PAD] pre-sigmoid
  float* masks_b;        // nullable [B][MOUT][T]
  float* mask;           // nullable [B][MOUT][T] sigmoid
};
hipError_t launch_mask_side(const MaskSideArgs& a, hipStream_t s);
hipError_t launch_stft(const StftArgs& a, hipStream_t s);
hipError_t launch_vad1(const Vad1Args& a, hipStream_t s);
hipError_t launch_istft(const IstftArgs& a, hipStream_t s);
hipError_t launch_istft_pair(const IstftArgs& a, hipStream_t s);  // the forward (est_mode 1, S = 2)

}  // namespace sepvad
