/*
 * sepvad.h — C ABI of libsepvad.so, the MI355X (gfx950) Sep-TFAnet^VAD forward path.
 *
 * The reference has no native interface: its hot path is the PyTorch module
 * `SeparationModel` (reference model/model.py:360-461) called as
 *     model = SeparationModel(**config["arch"]["args"])      (parse_config.py:99-103)
 *     model.load_state_dict(ckpt["state_dict"], strict=True)  (only_inference.py:57-61)
 *     sep, vad, est = model(x, inference_kw)                  (only_inference.py:90-91,
 *                                                               model/online_class_unknown_targets.py:84)
 * Each entry point below replaces one of those steps; the Python host
 * (sep-tfanet-vad_amd/model.py, native.py) binds them with ctypes. Plain pointers and sizes
 * only; no torch types cross this boundary. All device pointers are HIP device memory on
 * the handle's device; calls are ordered on the caller's hipStream_t.
 *
 * Errors: functions return SEPVAD_OK (0) or a negative status; sepvad_last_error() gives a
 * thread-local message. The Python host turns a non-zero status into RuntimeError.
 */
#ifndef SEPVAD_H
#define SEPVAD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEPVAD_ABI_VERSION 1

enum {
  SEPVAD_OK = 0,
  SEPVAD_E_ARG = -1,      /* invalid argument / unsupported configuration */
  SEPVAD_E_WEIGHTS = -2,  /* missing or mis-shaped state_dict entry */
  SEPVAD_E_HIP = -3,      /* a HIP runtime call failed */
  SEPVAD_E_SHAPE = -4     /* B/N outside what the handle supports */
};

/* TCN residual mode (model/model.py:347-352). */
enum { SEPVAD_LN_PLAIN = 0, SEPVAD_LN_RECURSIVE = 1, SEPVAD_LN_RESIDUAL = 2 };

/* Arithmetic of the pointwise (1x1) GEMMs (reference model/model.py:104,114,324). FP32 and F16X3 meet the
 * fp32 parity gates (max-abs <= 1e-4):
 *   FP32:  v_mfma_f32_32x32x2_f32 (exact fp32 fma chain);
 *   F16X3: fp32-equivalent split: x = hi + lo (fp16 each), acc += hi*hi + hi*lo + lo*hi on
 *          v_mfma_f32_32x32x16_f16 with fp32 accumulation (default; 16x the fp32 MFMA rate per pass).
 * F16 and BF16 are the reduced-precision arms (BASELINE cfg 2 "bf16", cfg 5 "fp16 vs fp32"): operands
 * rounded to fp16 / bf16, one v_mfma_f32_32x32x16_{f16,bf16} product, fp32 accumulation; everything outside
 * the GEMMs stays fp32. Their tolerance vs fp32 is measured, not gated. */
enum { SEPVAD_PREC_FP32 = 0, SEPVAD_PREC_F16X3 = 1, SEPVAD_PREC_F16 = 2, SEPVAD_PREC_BF16 = 3 };
/* Storage of the weight lo plane of F16X3 in the fused TCN (the 1x1 convs of model/model.py:104,114); the row-scaled
 * weight w*2^-e = hi + lo with hi fp16 and |lo| <= 2^-12:
 *   I8 (default): lo as int8 steps of 2^-19 (biased by 128), widened exactly to fp16 in registers by v_perm_b32 + one
 *          packed fp16 fma: 3 bytes per weight streamed instead of 4, absolute lo error <= 2^-20 of the row's largest
 *          weight. k_tcn -1.8 % shader cycles at cfg 2; every parity gate at its fp16-lo bound.
 *   F16:   lo as fp16 (rounds 1-2; 4 bytes per weight).
 *   E4M3:  lo as OCP e4m3 (scaled by 2^19), widened by v_cvt_scalef32_pk_f16_fp8: 3 bytes per weight, the cheapest
 *          widening (k_tcn -4.0 %), but 4 significant bits of lo move masks / est by up to 1.4e-5 of their range
 *          (others: below 1e-5), so it is opt-in. tools/lo_plane_precision.py emulates the formats on the CPU.
 * Waveforms stay within 3.1e-6 of the oracle with 0 VAD label flips in all three (tests/test_gpu_precision.py).
 * The multi-kernel schedule and the head always use F16. Environment override at create time: SEPVAD_WLO=f16|e4m3|i8. */
enum { SEPVAD_WLO_E4M3 = 0, SEPVAD_WLO_F16 = 1, SEPVAD_WLO_I8 = 2 };

/* SeparationModel kwargs that change the computation (model/model.py:362-366). */
typedef struct SepVadConfig {
  int32_t n_fft;                      /* n_fftBins; 512 */
  int32_t bn_dim;                     /* BN_dim; must be n_fft/2 */
  int32_t h_dim;                      /* H_dim; must be 2*bn_dim */
  int32_t layer;                      /* blocks per stack */
  int32_t stack;                      /* stacks; blocks = layer*stack */
  int32_t num_spk;                    /* 2 */
  int32_t tf_attention;               /* TF_Attention after every block */
  int32_t ln_mode;                    /* SEPVAD_LN_* */
  int32_t final_vad;                  /* VAD head present */
  int32_t final_vad_masked_speakers;  /* VAD on masked magnitudes instead of pre-sigmoid masks */
  int32_t noisy_phase;                /* est = (|X| m) e^{j angle X} instead of X m */
  int32_t activity_input;             /* 3x3 activity gate on the dB spectrum */
  int32_t precision;                  /* SEPVAD_PREC_* */
} SepVadConfig;

/* forward()'s inference_kw (only_inference.py:102-108; model/model.py:444-457). */
typedef struct SepVadInferKw {
  int32_t enabled;                    /* 0 == empty dict: the branch is skipped */
  int32_t filter_signals_by_smo_vad;
  int32_t filter_signals_by_unsmo_vad;
  int32_t length_smoothing_filter;    /* accepted, no effect on the math (reference overrides the taps) */
  float threshold_activated_vad;
  int32_t return_smoothed_vad;
} SepVadInferKw;

/* Caller-owned outputs of one forward (device pointers). T = 1 + N / (n_fft/2). */
typedef struct SepVadOutputs {
  float* sep;       /* [B, num_spk, N] f32, required                                        */
  float* vad;       /* [B, num_spk, T] f32 (probabilities, or {0,1} when smoothed); NULL if !final_vad */
  void* est;        /* [B, num_spk, n_fft/2+1, T] complex64 (re,im interleaved); nullable  */
  float* spectrum;  /* [B, n_fft/2+1, T] gated dB spectrum (self.spectrum); nullable         */
  float* masks_b;   /* [B, num_spk*(n_fft/2+1), T] pre-sigmoid masks (self.masks_b); nullable */
  float* mask;      /* [B, num_spk, n_fft/2+1, T] post-sigmoid (self.mask_per_speaker); nullable */
} SepVadOutputs;

typedef struct sepvad_model* sepvad_handle;

/* Replaces SeparationModel(**args) + load_state_dict(strict=True) (model/model.py:361-400,
 * only_inference.py:57-61). `tensors[i]` is a HOST float32 array of `numels[i]` elements named
 * `names[i]` (reference state_dict keys). Folds weight-norm (w = v * (g/||v||)) once, packs the
 * weights for the kernels and uploads them to `device`. Returns NULL on error. */
sepvad_handle sepvad_create(const SepVadConfig* cfg, const float* const* tensors,
                            const char* const* names, const int64_t* numels, int32_t n,
                            int32_t device);

/* Pre-size the workspace for up to B utterances of N samples (so forward never allocates). */
int32_t sepvad_reserve(sepvad_handle h, int32_t B, int32_t N);

/* Switch the GEMM arithmetic of later forwards (SEPVAD_PREC_*); weights for both are resident. */
int32_t sepvad_set_precision(sepvad_handle h, int32_t precision);

/* Weight lo-plane format of the fused TCN for later F16X3 forwards (SEPVAD_WLO_*); all three are resident. */
int32_t sepvad_set_weight_lo(sepvad_handle h, int32_t mode);

/* HOST function: the packer's float -> OCP e4m3fn encoder (round to nearest even, saturating at 448), as used
 * for the weight lo plane; out[i] = e4m3(in[i]). Lets the host-side quantisation be checked without a GPU. */
int32_t sepvad_e4m3_encode(const float* in, uint8_t* out, int64_t n);

/* Replaces SeparationModel.forward(x, inference_kw) (model/model.py:402-461).
 * x: device [B, N] f32. kw may be NULL (== empty dict). Stream-ordered on `stream`
 * (a hipStream_t; NULL = default stream). */
int32_t sepvad_forward(sepvad_handle h, const float* x, int32_t B, int32_t N,
                       const SepVadOutputs* out, const SepVadInferKw* kw, void* stream);

/* Same as sepvad_forward with a row stride: utterance b starts at x + b * ldx (ldx >= N).
 * The streaming wrapper passes its overlapping windows this way (window k of stream b is
 * x + b * N_total + k * hop, model/online_class_unknown_targets.py:39-41) without a gather copy. */
int32_t sepvad_forward_strided(sepvad_handle h, const float* x, int64_t ldx, int32_t B, int32_t N,
                               const SepVadOutputs* out, const SepVadInferKw* kw, void* stream);

/* Replaces the window loop of OnlineSaving.calc_online (model/online_class_unknown_targets.py:80-97) as ONE
 * forward: n_win windows of N samples for each of n_streams signals, window k of stream b starting at
 * x + b * ld_stream + k * hop (no gather copy); utterance u = k * n_streams + b of the outputs (so window k of
 * every stream is a contiguous [n_streams, ...] block). Requires (n_win - 1) * hop + N <= ld_stream. */
int32_t sepvad_forward_windows(sepvad_handle h, const float* x, int64_t ld_stream, int32_t n_streams, int32_t n_win,
                               int64_t hop, int32_t N, const SepVadOutputs* out, const SepVadInferKw* kw,
                               void* stream);

/* Split each forward's batch into n (1..4) utterance chunks that run concurrently on internal
 * streams forked from / joined to the caller's stream (results are bitwise identical for any n:
 * every reduction is per utterance). Default 1, or the SEPVAD_SPLIT environment variable. */
int32_t sepvad_set_split(sepvad_handle h, int32_t nsplit);

/* Select the TCN schedule of later forwards: 1 (default, or env SEPVAD_FUSED) = the whole separator stack
 * as one persistent launch when the GEMMs are F16X3 / F16 / BF16 and T <= 8192 (groups of ceil(T/32) <= 256 workgroups per
 * utterance); 0 = one launch per stage (4 per block). Both meet the same parity gates. */
int32_t sepvad_set_fused(sepvad_handle h, int32_t on);
/* Synchronises the device and reports the schedule of the last forward and the persistent launch's
 * health: *used = 0 if it ran one launch per stage, else the 32-frame slices per workgroup of its persistent launch
 * (1, or 2 when the batch needs more than one round of one-slice workgroups; both give the same bits); returns
 * SEPVAD_OK, or SEPVAD_E_HIP if a group hand-off gave up (a bounded wait timed out; outputs of that forward are
 * invalid). */
int32_t sepvad_fused_status(sepvad_handle h, int32_t* used);

/* The side attributes of the LAST forward on `stream` (self.spectrum, self.masks_b, self.mask_per_speaker,
 * reference model/model.py:412-429), materialised from that stream's workspace: `out->spectrum`, `out->masks_b`
 * and `out->mask` (each nullable; the other members are ignored) receive exactly the values the forward would
 * have written to them. Valid until the next forward on the same stream. The Python host calls this when
 * one of the attributes is first read, so a forward whose side attributes nobody reads does not pay for
 * their bin-major copies. SEPVAD_E_ARG if no forward ran on `stream`. */
int32_t sepvad_side_outputs(sepvad_handle h, const SepVadOutputs* out, void* stream);

/* The forward that sepvad_side_outputs would read: *seq = forwards enqueued so far on `stream` (a per-stream
 * sequence id), *B / *N = its shape. SEPVAD_E_ARG if no forward ran on `stream`. */
int32_t sepvad_last_forward(sepvad_handle h, void* stream, int64_t* seq, int32_t* B, int32_t* N);

/* sepvad_side_outputs of ONE forward: fails with SEPVAD_E_ARG (no write) unless forward `seq` of shape (B, N)
 * (from sepvad_last_forward right after it) is still the last forward on `stream`, so a later forward of another
 * shape can never be copied into buffers sized for this one (the reference's attributes belong to the forward that
 * set them, model/model.py:412-429). */
int32_t sepvad_side_outputs_of(sepvad_handle h, const SepVadOutputs* out, void* stream, int64_t seq, int32_t B,
                               int32_t N);

/* Diagnostics: with SEPVAD_TCN_CLOCK=1 in the environment every k_tcn launch records {~(min start), max end (100 MHz
 * wall clock over all workgroups), workgroup 0: start / end wall clock, start / end shader clock (s_memtime), 0, 0}.
 * Synchronises the device and copies the last min(max_records, recorded) records, oldest first, as 8 uint64 each;
 * *n = records available (at most 4096). */
int32_t sepvad_tcn_clock(sepvad_handle h, uint64_t* out, int32_t max_records, int32_t* n);

/* Synchronises `stream` and frees the per-stream context (workspace, hand-off words, pinned give-up word) the handle
 * holds for it. Contexts are otherwise kept (at most SEPVAD_MAX_STREAM_CTX = 32 per handle by default, the least
 * recently used evicted after a device-wide sync -- the host waits until every stream on the device is idle, other
 * handles' and the application's work included -- because its stream may already be destroyed with work pending). */
int32_t sepvad_release_stream(sepvad_handle h, void* stream);

/* Kernel-level test entries of the forward's own front and back end (the fused schedule's k_stft_gate and
 * k_istft_pair), in the frame-major layouts the forward's workspace holds (Tp = roundup(T, 64), T = 1 + N / 256):
 * sepvad_stft_gate_test: X_fm [B][Tp][257] complex (DC zeroed) and db_fm [B][Tp][260] = 10 log10(clamp(|X|^2, 1e-10))
 * of x [B][N] (model/model.py:16-25,408-412; the activity gate's outputs go to the stream's workspace).
 * sepvad_istft_pair_test: est[b][s] = X_fm[b] * sigmoid(masks_fm[b][:, 257 s + k]) and y[b][s] = torch.istft(est,
 * center=True, length=N) (model/model.py:429-460, no VAD gain), y [B][2][N], est (nullable) [B][2][257][T] complex,
 * masks_fm [B][Tp][576]. Tests only. */
int32_t sepvad_stft_gate_test(sepvad_handle h, const float* x, int32_t B, int32_t N, void* X_fm, float* db_fm,
                              void* stream);
int32_t sepvad_istft_pair_test(sepvad_handle h, const void* X_fm, const float* masks_fm, int32_t B, int32_t N, float* y,
                               void* est, void* stream);

/* Block-level parity probe of the fused TCN: while `dump` (device, >= 3 * B * roundup(T, 64) * 256 floats) is
 * set, forwards that run the fused TCN in one launch write dump[0] = TCN.LN output x'_0 (model/model.py:333),
 * dump[1] = block 0's DepthConv1d output (:144) and dump[2] = block 0's TF_Attention output (:207), each
 * [B][roundup(T, 64)][256] channel-last. NULL disables. F16X3 arithmetic only (a separate instantiation of the
 * kernel); tests only (the reference golden's tcn_in, blk0_res, blk0_att). */
int32_t sepvad_set_tcn_dump(sepvad_handle h, float* dump);

/* Front-end / back-end stages alone, for kernel-level parity tests:
 * STFT with DC zeroed (model/model.py:16-25,408-410) -> X [B, n_fft/2+1, T] complex64, and
 * 10 log10(clamp(|X|^2, 1e-10)) (model/model.py:411-412) -> spec [B, n_fft/2+1, T] (nullable). */
int32_t sepvad_stft(sepvad_handle h, const float* x, int32_t B, int32_t N, void* X, float* spec,
                    void* stream);
/* torch.istft(center=True, length=N) of est [B*S, n_fft/2+1, T] complex64 (model/model.py:460). */
int32_t sepvad_istft(sepvad_handle h, const void* est, int32_t BS, int32_t N, float* y, void* stream);

/* ---- streaming wrapper (model/online_class_unknown_targets.py:72-105) -------------------------
 * Signals are [B, 2, ld] f32 device arrays (speaker rows of stride ld).
 *
 * Replaces PITLossWrapper(nn.L1Loss(), pit_from="pw_pt")(est, ref, return_incides=True)
 * (model/pit_wrapper.py:77-140,149-177,261-312) on est[..., 0:L] vs ref[..., 0:L]: pairwise L1
 * means over batch and samples (nn.L1Loss reduces the batch too, so the permutation is shared by
 * the whole batch), loss set over the 2 permutations, first minimum. Writes perm_out [B, 2] int64
 * (batch_indices), loss_out (min loss) and pw_out [2, 2] (pairwise losses), each nullable.
 * scratch: device buffer of at least SEPVAD_PIT_SCRATCH_BYTES. Deterministic. */
#define SEPVAD_PIT_SCRATCH_BYTES 16448
int32_t sepvad_pit_l1(const float* est, int64_t est_ld, const float* ref, int64_t ref_ld, int32_t B, int64_t L,
                      void* scratch, int64_t* perm_out, float* loss_out, float* pw_out, void* stream);
/* The same in two steps, for a stream batch sharded over ranks (nn.L1Loss means over the WHOLE batch,
 * model/pit_wrapper.py:172-177): sepvad_pit_l1_sums writes this device's 4 pairwise L1 sums (double,
 * fixed order) to sums[4] (device); the caller all-reduces them over the ranks (RCCL, 32 bytes); then
 * sepvad_pit_l1_choose turns sums / count (count = total rows x L over all ranks) into the permutation
 * for this device's B rows, the loss and the pairwise means, exactly as sepvad_pit_l1 does. */
int32_t sepvad_pit_l1_sums(const float* est, int64_t est_ld, const float* ref, int64_t ref_ld, int32_t B, int64_t L,
                           void* scratch, double* sums, void* stream);
int32_t sepvad_pit_l1_choose(const double* sums, double count, int32_t B, int64_t* perm_out, float* loss_out,
                             float* pw_out, void* stream);

/* Replaces reorder_source_mse(preds, batch_indices) (model/combined_loss.py:63-78) fused with
 * OnlineSaving.update_online_signal (online_class_unknown_targets.py:28-37):
 * dst[b, i, d0 + n] = src[b, perm[b, i], s0 + n] for n < H (perm NULL = identity). */
int32_t sepvad_stream_append(const float* src, int64_t src_ld, int64_t s0, int32_t B, int64_t H,
                             const int64_t* perm, float* dst, int64_t dst_ld, int64_t d0, void* stream);

/* ---- quality metrics (model/combined_loss.py:16-56 calc_sisdr == model/metric.py:61-101
 * scale_invariant_signal_distortion_ratio; PIT over it: metric.py:258 pit_si_sdr) --------------------
 * out[r] = SI-SDR(P[pidx[r]], Tg[tidx[r]]) in dB for r < R: rows of N samples with row strides p_ld / t_ld,
 * pidx / tidx nullable (identity). eps = float32 epsilon; zero_mean as the reference's flag. Moments in
 * double, fixed-order reductions (bitwise reproducible). Device pointers, stream-ordered. */
int32_t sepvad_si_sdr(const float* P, int64_t p_ld, const float* Tg, int64_t t_ld, int64_t N, int32_t R,
                      const int32_t* pidx, const int32_t* tidx, int32_t zero_mean, float* out, void* stream);

/* Replaces Accuracy_Vad()(preds, targets, _) (model/metric.py:163-177): labels = preds > 0.5 (NaN kept),
 * written back into preds when in_place (the reference masks its argument in place); out[0] = fraction of
 * labels equal to targets over [B, S, T], out[1 + s] = the same for speaker s (S <= 8). Device pointers,
 * contiguous [B][S][T] f32, stream-ordered; integer counts (exact). */
int32_t sepvad_vad_accuracy(float* preds, const float* targets, int32_t B, int32_t S, int32_t T, int32_t in_place,
                            float* out, void* stream);

/* ---- synthetic reverberant mixtures (BASELINE cfg 4): image-method room impulse responses --------
 * Replaces pyrirgen.generateRir / gen_rir (create_data/rirgen.cpp:115-351, create_data/pyrirgen.pyx)
 * as create_data/create_simulation_data.py:284-289 calls it. HOST function, double precision:
 * c sound speed (m/s), fs (Hz), mics [n_mics][3] and src [3] positions (m), room [3] dimensions (m),
 * beta: n_beta = 1 -> T60 (s; 0 = anechoic) or n_beta = 6 -> reflection coefficients, orientation [2]
 * (azimuth, elevation; nullable = 0), high_pass 1/0, n_dim 2/3, order (-1 = all), n_samples (-1 = T60 fs),
 * mic_type 'o','s','c','h','b'. Writes out [n_mics][n_samples] (cap doubles) and returns n_samples;
 * out NULL = size query. Negative status on bad arguments. */
int32_t sepvad_rir_generate(double c, double fs, const double* mics, int32_t n_mics, const double* src,
                            const double* room, const double* beta, int32_t n_beta, const double* orientation,
                            int32_t high_pass, int32_t n_dim, int32_t order, int32_t n_samples, char mic_type,
                            double* out, int64_t cap);

/* ---- input preprocessing of the reference CLI (only_inference.py:68-83) ---------------------
 * Windowed-sinc resampling filter of torchaudio.transforms.Resample(orig_freq, new_freq) with its
 * defaults (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99), host-side, double precision
 * rounded to float: taps [phases][ntaps] into `taps` (capacity `cap` floats); info receives
 * {phases, ntaps, stride, width}. Returns SEPVAD_E_ARG if cap is too small. */
int32_t sepvad_resample_filter(int32_t orig_freq, int32_t new_freq, float* taps, int32_t cap, int32_t* info);

/* Polyphase FIR on the device: y [ylen] = resample(x [n]) with ylen = ceil(new * n / orig) (reduced
 * by the gcd) and taps (device) from sepvad_resample_filter. */
int32_t sepvad_resample(const float* x, int64_t n, const float* taps, const int32_t* info, float* y, int64_t ylen,
                        void* stream);

/* y = 1.8 * (x - min x) / (max x - min x) - 0.9 over n samples (only_inference.py:81), fp32 in the
 * reference's numpy operation order (bit-exact). scratch: SEPVAD_NORM_SCRATCH_BYTES device bytes. */
#define SEPVAD_NORM_SCRATCH_BYTES 8192
int32_t sepvad_normalize(const float* x, int64_t n, float* y, void* scratch, void* stream);

/* Seconds of the last forward's dominant-kernel launches measured with HIP events
 * (enabled by sepvad_set_timing(h, 1)); see bench.py. */
int32_t sepvad_set_timing(sepvad_handle h, int32_t on);
int32_t sepvad_timing(sepvad_handle h, double* gemm_ms, int32_t* gemm_launches, double* total_ms);

void sepvad_destroy(sepvad_handle h);
const char* sepvad_last_error(void);
int32_t sepvad_abi_version(void);
/* Source hash of this build: the first 16 hex digits of sha256 over include/sepvad.h and the library's sources
 * (sep-tfanet-vad_amd/buildid.py, computed at build time). A static string; tests compare it with the hash of the
 * tree they run in. No reference equivalent (build provenance). */
const char* sepvad_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* SEPVAD_H */
