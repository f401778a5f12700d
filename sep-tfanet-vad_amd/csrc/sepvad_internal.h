// Internal declarations shared by the kernel translation units and the C-ABI layer.
// Layout conventions (see DESIGN.md "Data layout in HBM"):
//   * every per-utterance activation is channel-major [B][rows][Tp], Tp = roundup(T, 64); columns
//     t >= T are padding whose contents are never reduced over nor used as conv context;
//   * complex spectra are interleaved float2 [B][257][Tp];
//   * GroupNorm statistics travel as deterministic per-workgroup partial slots
//     [B][nslots][2] (sum, sumsq) in double, or per-channel moments [B][C][5] — never atomics,
//     so results are bitwise reproducible run to run and shard to shard.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sepvad {

constexpr int NFFT = 512;   // n_fftBins (model/model.py:362)
constexpr int HOP = 256;    // n_fftBins/2 (model/model.py:378)
constexpr int NBIN = 257;   // n_fftBins/2+1
constexpr int CH = 256;     // BN_dim == TCN input channels (non-DC bins)
constexpr int HID = 512;    // H_dim (depthwise multiplier 2)
constexpr int TILE = 64;    // GEMM tile edge; Tp is a multiple of TILE
constexpr int MOUT_PAD = 576;  // 2*257 = 514 output-head rows padded to a multiple of 64

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// Loader transform applied to the GEMM B operand as it is staged (normalize-on-load).
enum LoadMode {
  LD_PLAIN = 0,      // x
  LD_GN = 1,         // GroupNorm(1,K)(x)                       (stats from slots)
  LD_RECURSIVE = 2,  // GN_b(o + GN_a(u))   model/model.py:347-348 (stats from moments)
  LD_RESIDUAL = 3,   // o + GN_c(u)         model/model.py:349-350 (stats of u from slots)
  LD_ADD = 4         // o + u               model/model.py:351-352
};
// GEMM epilogue.
enum EpiMode {
  EP_PRELU_STATS = 0,  // + bias, PReLU, store, GN partial stats       (DepthConv1d.conv1d)
  EP_BIAS_ATT = 1,     // + bias, store, column/row partial sums        (DepthConv1d.res_out -> TF_Attention)
  EP_BIAS_OUT = 2      // + bias, store rows < Mreal (+ optional de-padded copy)  (TCN.output.2)
};

// Parameters of a GN-style loader transform (shared by the GEMM loader and head_prep).
struct LoadSpec {
  int mode;
  const float* X;        // [B][K][Tp]  o (or x)
  const float* X2;       // [B][K][Tp]  u (RECURSIVE/RESIDUAL/ADD)
  const float* g1; const float* be1; float eps1;  // GN (LD_GN), GN_a (RECURSIVE), GN_c (RESIDUAL)
  const float* g2; const float* be2; float eps2;  // GN_b (RECURSIVE)
  const double* slots; int nslots;                // [B][nslots][2]
  const double* moments;                          // [B][K][5]: S_o, S_oo, S_u, S_uu, S_ou
};

struct GemmArgs {
  int B, T, Tp, M, Mreal, K;
  const float* WT;     // [K][M] (M padded to a multiple of 64)
  const float* bias;   // [M]
  float prelu;
  LoadSpec ld;
  float* Xmat;         // nullable: transformed B operand written once (by m-tile 0)
  float* Y;            // [B][Mreal][Tp]
  float* Yside;        // nullable [B][Mreal][T]
  double* out_slots;   // EP_PRELU_STATS [B][(M/64)*(Tp/64)][2]
  float* colsum;       // EP_BIAS_ATT [B][M/64][Tp]
  float* rowsum;       // EP_BIAS_ATT [B][Tp/64][M]
};

struct DwArgs {
  int B, T, Tp, dil;
  const float* A;                 // [B][CH][Tp] PReLU(conv1d) output (pre-GN1)
  const double* slots; int nslots;
  const float* g1; const float* be1;  // reg1
  const float* wd; const float* bd;   // [HID][3], [HID]
  float alpha;                        // nonlinearity2
  float* D;                           // [B][HID][Tp]
  double* out_slots;                  // [B][CH/16][2]
};

struct AttArgs {
  int B, T, Tp, mtiles, ntiles, tf_att, ln_mode;
  const float* R;        // [B][CH][Tp] res_out output
  const float* O;        // [B][CH][Tp] block input o
  const float* colsum;   // [B][mtiles][Tp]
  const float* rowsum;   // [B][ntiles][CH]
  const float* attp;     // 16 floats: t1w[3] t1b t2w[3] t2b f1w[3] f1b f2w[3] f2b ; prelu_t, prelu_f at [16],[17]
  float* U;              // [B][CH][Tp]
  double* moments;       // [B][CH][5]   (recursive)
  double* out_slots;     // [B][CH/16][2] (residual: sum/sumsq of r')
};

struct HeadPrepArgs {
  int B, T, Tp;
  LoadSpec ld;           // final block's o_new transform
  float alpha;           // TCN.output.0 PReLU
  float* P;              // [B][CH][Tp]
  double* out_slots;     // [B][CH/16][2]
};

struct GateArgs {
  int B, T, Tp, activity;
  const float* specdb;   // [B][NBIN][Tp] 10log10(clamp(|X|^2,1e-10)), DC row = -100
  const float* w;        // activity_input.weight [9] ; bias at w[9]; prelu at w[10]
  float* S0;             // [B][CH][Tp] gated rows 1..256
  float* spec_side;      // nullable [B][NBIN][T]
  double* out_slots;     // [B][gate_tiles][2]
};

constexpr int GATE_ROWS = 16;
__host__ __device__ constexpr int gate_tiles() { return (NBIN + GATE_ROWS - 1) / GATE_ROWS; }

struct StftArgs {
  int B, N, T, Tp;
  const float* x;        // [B][N]
  const float* window;   // [512]
  const float2* tw;      // [512] e^{-2 pi i m / 512}
  float2* X;             // [B][NBIN][Tp]  (workspace) or nullable
  float2* Xout;          // nullable [B][NBIN][T] (debug entry)
  float* specdb;         // nullable [B][NBIN][Tp]
  float* spec_out;       // nullable [B][NBIN][T]
};

struct VadArgs {
  int B, T, Tp, masked_speakers, noisy_phase;
  const float* masks;    // [B][2*NBIN][Tp] pre-sigmoid
  const float2* X;       // [B][NBIN][Tp]
  const float* w1;       // [4][257][5]
  const float* b1;       // [4]
  float alpha;           // relu_1
  const float* g;        // BN_1 weight [4]
  const float* be;       // BN_1 bias [4]
  const float* w2;       // [4][3]
  float b2;
  int kw_enabled, filt, ret_smooth;
  float thr;
  float* vad_out;        // [B][2][T]
  float* gain;           // [B][2][Tp]
};

struct IstftArgs {
  int BS, S, N, T, Tp, noisy_phase, est_mode;  // est_mode 1: apply mask to X (forward); 0: est given
  const float2* X;       // [B][NBIN][Tp]  (est_mode 1)
  const float* masks;    // [B][S*NBIN][Tp] pre-sigmoid (est_mode 1)
  const float* gain;     // nullable [B][S][Tp]
  const float2* est_in;  // [BS][NBIN][T] (est_mode 0)
  const float* window;   // [512]
  const float2* tw;      // [512]
  float2* est_out;       // nullable [BS][NBIN][T]
  float* mask_out;       // nullable [BS][NBIN][T]
  float* y;              // [BS][N]
};

hipError_t launch_gemm(const GemmArgs& a, int ep, hipStream_t s);
hipError_t launch_dw(const DwArgs& a, hipStream_t s);
hipError_t launch_att(const AttArgs& a, hipStream_t s);
hipError_t launch_head_prep(const HeadPrepArgs& a, hipStream_t s);
hipError_t launch_gate(const GateArgs& a, hipStream_t s);
hipError_t launch_stft(const StftArgs& a, hipStream_t s);
hipError_t launch_vad(const VadArgs& a, hipStream_t s);
hipError_t launch_istft(const IstftArgs& a, hipStream_t s);

}  // namespace sepvad
