// The forward's front end in one launch (model/model.py:16-25,408-419,421): k_stft_gate — reflect-padded
// periodic-Hann 512-point real STFT (hop 256, DC zeroed) of SG_OWN own frames plus one halo frame either
// side, X stored frame-major for the iSTFT, 10 log10(clamp(|X|^2, 1e-10)) kept in LDS (written to HBM only
// when the spec_input and spec_output windows differ), then the activity gate 3x3 conv + PReLU + multiply
// (k_gate's arithmetic), the TCN input S0 and the TCN.LN partial records.
// Transforms: register-resident four-step 16 x 16 FFT, 16 lanes per frame, the 34 frames of a workgroup on
// 9 waves in one round; one workgroup per CU (LDS ~114 KB), and at B = 64, T = 126 the 256 workgroups are
// one round. The TCN.LN records stay per GATE_ROWS = 16 rows (two per workgroup: k_tcn's layout). Built
// with -fno-slp-vectorize (Makefile), as istft.hip.
#include "device_common.h"
#include "fft_common.h"

namespace sepvad {

constexpr int SG_OWN = 2 * GATE_ROWS;         // own frames per workgroup (two TCN.LN records)
constexpr int SG_FR = SG_OWN + 2;             // transforms per workgroup
constexpr int SG_WAVES = (SG_FR + 3) / 4;     // 4 transforms per wave
constexpr int SG_THREADS = 64 * SG_WAVES;

// Forward real 512-point transform of frame samples xs[0..511] (reflect-padded, windowed on load) as the
// 256-point complex transform of z[m] = x[2m] + i x[2m+1]: lane c loads its column z[16 n1 + c], step 1 DFT
// over n1, twiddle W256^(c k1), XOR-swizzled transpose through `row`, step 2 DFT over n2 -> Z[c + 16 k2],
// written to `row` in natural order for the split step (the caller syncs the wave before reading it).
__device__ __forceinline__ void rfft512_col(const float* xb, int s0base, int N, const float* win, float2* row,
                                            const float2* tw, int c) {
  float2 x[16];
  // samples by buffer loads off one descriptor (32-bit offsets: one register per address), all 32 in
  // flight at once; the window (LDS) applied after
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xb), (short)0, N * 4, 0x00020000);
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    const int m = 16 * n1 + c;
    int s0 = s0base + 2 * m, s1 = s0 + 1;  // reflect padding of 256 on both sides
    s0 = s0 < 0 ? -s0 : (s0 >= N ? 2 * (N - 1) - s0 : s0);
    s1 = s1 < 0 ? -s1 : (s1 >= N ? 2 * (N - 1) - s1 : s1);
    x[n1] = make_float2(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, s0 * 4, 0, 0)),
                        __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, s1 * 4, 0, 0)));
  }
  const float2* winc = reinterpret_cast<const float2*>(win) + c;
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    const float2 w = winc[16 * n1];
    x[n1] = make_float2(w.x * x[n1].x, w.y * x[n1].y);
  }
  dft16<false>(x);  // A[k1] at slot d16(k1)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {  // W256^(c k1) = W512^(2 c k1)
    x[d16(k1)] = cmul(x[d16(k1)], twid<true>(tw, mul_late(c, 2 * k1)));
    if (k1 % 4 == 3) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) row[16 * k1 + xor_late(c, k1)] = x[d16(k1)];
  wave_lds_sync();
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) x[n2] = row[16 * c + xor_late(c, n2)];  // row k1 = c of the transpose
  wave_lds_sync();  // every lane's reads done before the natural-order writes below
  dft16<false>(x);  // Z[c + 16 k2] at slot d16(k2)
  float2* rc = row + c;
#pragma unroll
  for (int k2 = 0; k2 < 16; ++k2) rc[16 * k2] = x[d16(k2)];
}

__global__ __launch_bounds__(SG_THREADS) void k_stft_gate(StftArgs a) {
  __shared__ float2 tw[256];
  __shared__ float2 rows[4 * SG_WAVES][M256];  // per transform: transpose, then Z in natural order
  __shared__ float S[SG_FR][NBIN + 2];         // dB of frames f0-1 .. f0+SG_OWN (zero outside [0, T)), bins -1 .. 257
  __shared__ float red[4 * 16];
  __shared__ float2 wins[2][M256];             // a.window, a.window_db (as sample pairs)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x, f0 = blockIdx.y * SG_OWN;
  const int T = a.T, N = a.N;
  const bool two = a.window_db != a.window;  // rare: distinct spec_input / spec_output windows
  if (tid < 256) {
    tw[tid] = a.tw[tid];
    wins[0][tid] = reinterpret_cast<const float2*>(a.window)[tid];
    if (two) wins[1][tid] = reinterpret_cast<const float2*>(a.window_db)[tid];
  }
  for (int i = tid; i < SG_FR; i += SG_THREADS) { S[i][0] = 0.f; S[i][NBIN + 1] = 0.f; }
  const float* xb = a.x + (size_t)(b % a.nstr) * a.ldx + (size_t)(b / a.nstr) * a.hopw;
  const int c = lane & 15, fi = 4 * wave + (lane >> 4), f = f0 - 1 + fi;
  const bool live = fi < SG_FR && f >= 0 && f < T;
  const bool own = live && fi >= 1 && fi <= SG_OWN;
  float2* row = rows[fi];
  // diagnostics: slot 0 wall clock at entry, slots 1.. shader clock at the phase ends
  unsigned long long* const pr = a.probe ? a.probe + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
  auto stamp = [&](int k) {
    if (pr && tid == 0) pr[k] = __builtin_amdgcn_s_memtime();
  };
  if (pr && tid == 0) pr[0] = wall_clock64();
  stamp(1);
  lds_sync();  // twiddles
  // one transform pass per window: X (and the dB unless the windows differ) from a.window, the dB from
  // a.window_db in a second pass when they differ (a called lambda, not a loop: no values held across passes)
  auto pass = [&](const float* win, bool store_x, bool store_db) {
    if (fi < SG_FR) {
      // frames outside [0, T) transform frame 0 / T-1 (in bounds, unused)
      const int fc = min(max(f, 0), T - 1);
      rfft512_col(xb, fc * HOP - HOP, N, win, row, tw, c);
      wave_lds_sync();
      if (store_x) stamp(2);
      // split step: X[k] = E + W512^k O, k = c + 16 r, then the Nyquist bin on lane c = 0
      const size_t xrow = (size_t)b * a.Tp + f;
      auto emit = [&](int k, float2 Xk) {
        if (k == 0) Xk = make_float2(0.f, 0.f);  // DC removed (model/model.py:24,410)
        const float db = power_db(Xk);
        if (store_x && own) st_out(a.X + xrow * NBIN + k, Xk);
        if (store_db) {
          S[fi][k + 1] = live ? db : 0.f;
          if ((two || a.db_out) && own) a.specdb[xrow * SPEC_LD + k] = db;
        }
      };
      const float2* rc = row + c;
      const float2* rm = row + (M256 - 240 - c);  // row[(256 - k) & 255] = rm[16 (15 - r)] for k = c + 16 r > 0
      const float2* twc = tw + c;
#pragma unroll 4
      for (int r = 0; r < 16; ++r) {
        const int k = c + 16 * r;
        const float2 zk = rc[16 * r], zm = conjf2(k == 0 ? row[0] : rm[16 * (15 - r)]);
        const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y + zm.y));
        const float2 Dd = csub(zk, zm);
        const float2 O = make_float2(0.5f * Dd.y, -0.5f * Dd.x);
        emit(k, cadd(E, cmul(twc[16 * r], O)));
      }
      if (c == 0) {
        const float2 z0 = row[0];
        emit(M256, make_float2(z0.x - z0.y, 0.f));  // Nyquist: E[0] - O[0]
      }
    }
  };
  pass(reinterpret_cast<const float*>(wins[0]), true, !two);
  if (two) {
    lds_sync();  // (the second pass reuses the rows)
    pass(reinterpret_cast<const float*>(wins[1]), false, true);
  }
  stamp(3);
  lds_sync();
  stamp(4);
  // activity gate over the own frames (k_gate's arithmetic, model/model.py:414-419)
  float w[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) w[i] = a.gate_w[i];
  const float bias = a.gate_w[9], alpha = a.gate_w[10];
  // thread -> (bin f = 1 + (tid & 255), half h = tid >> 8): rows [16h, 16h + 16) of bin f with the 3 x 3
  // window sliding down a register copy of its three S columns (k_gate's fma order); bin 0 (DC) is only a
  // neighbour, never an output
  float st[4] = {0.f, 0.f, 0.f, 0.f};  // {sum, sumsq} of rows [0, 16) and [16, 32): two records
  if (tid < 2 * CH) {
    const int f = 1 + (tid & (CH - 1)), h = tid >> 8, r0 = h * GATE_ROWS;
    float col[3][GATE_ROWS + 2];  // S[r0 + j][f + di]: bins f - 1 + di of frames f0 - 1 + r0 + j
#pragma unroll
    for (int j = 0; j < GATE_ROWS + 2; ++j)
#pragma unroll
      for (int di = 0; di < 3; ++di) col[di][j] = S[r0 + j][f + di];
    float s1 = 0.f, s2 = 0.f;
    float* s0p = a.S0 + ((size_t)b * a.Tp + f0 + r0) * CH + f - 1;
#pragma unroll
    for (int r = 0; r < GATE_ROWS; ++r) {
      const float x = col[1][r + 1];
      float y = x;
      if (a.activity) {
        float g = bias;
#pragma unroll
        for (int di = 0; di < 3; ++di)
#pragma unroll
          for (int dj = 0; dj < 3; ++dj) g = fmaf(w[di * 3 + dj], col[di][r + dj], g);
        y = x * prelu_f(g, alpha);
      }
      st_out(s0p + (size_t)r * CH, y);
      if (f0 + r0 + r < T) { s1 += y; s2 += y * y; }
    }
    st[0] = h == 0 ? s1 : 0.f;
    st[1] = h == 0 ? s2 : 0.f;
    st[2] = h == 1 ? s1 : 0.f;
    st[3] = h == 1 ? s2 : 0.f;
  }
  block_reduce_store<4>(st, red, a.gate_rec + ((size_t)b * (a.Tp / GATE_ROWS) + 2 * blockIdx.y) * 2);
  stamp(5);
}

hipError_t launch_stft_gate(const StftArgs& a, hipStream_t s) {
  if (a.N <= HOP || a.Tp % SG_OWN) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stft_gate, dim3(a.B, a.Tp / SG_OWN), dim3(SG_THREADS), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
