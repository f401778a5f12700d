// Streaming-wrapper kernels (reference model/online_class_unknown_targets.py:72-105):
//   k_pit_l1_partial / k_pit_l1_sums / k_pit_l1_choose  PITLossWrapper(nn.L1Loss(), pit_from="pw_pt") with
//       return_incides=True (model/pit_wrapper.py:77-140,149-177,261-312): pairwise L1 losses between
//       the new window's overlap region and the stitched signal's tail. nn.L1Loss() reduces over the
//       batch AND the samples, so every pairwise loss is one scalar shared by the whole batch and the
//       chosen permutation is batch-global (exactly as the reference computes it).
//   k_stream_append  reorder_source_mse (model/combined_loss.py:63-78) fused with
//       OnlineSaving.update_online_signal (online_class_unknown_targets.py:28-37): the reordered last
//       hop of every window lands in its slot of the preallocated stitched signal (no torch.cat).
// Layouts: signals are [B][2][ld] fp32 (speaker rows with stride ld). HBM-bound, no MFMA.
// Reductions are deterministic: fixed per-block ranges, per-block partials in double, summed in
// block order by k_pit_l1_sums; a sharded stream batch all-reduces those 4 sums before k_pit_l1_choose.
#include "device_common.h"

namespace sepvad {

constexpr int PIT_THREADS = 256;

// partial[blk][4] = sums over this block's (b, n) range of |est[b][e][n] - ref[b][t][n]|, (e, t) in
// {(0,0), (0,1), (1,0), (1,1)} (pw_losses[:, est_idx, target_idx], model/pit_wrapper.py:172-177)
__global__ __launch_bounds__(PIT_THREADS) void k_pit_l1_partial(PitArgs a) {
  __shared__ float red[4 * 16];
  const long long total = (long long)a.B * a.L;
  const long long per = (total + gridDim.x - 1) / gridDim.x;
  const long long beg = per * blockIdx.x;
  const long long end = min(total, beg + per);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // fp32 per thread over a short strided range, then double across the block. (b, n) of element i advance by
  // PIT_THREADS per step with a carry into b (one 64-bit division per thread, not one per element: the per-element
  // i / L, i % L made the kernel VALU-bound)
  long long i = beg + threadIdx.x;
  long long b = i / a.L, n = i - b * a.L;
  for (; i < end; i += PIT_THREADS) {
    const float* e = a.est + (size_t)b * 2 * a.est_ld + n;
    const float* r = a.ref + (size_t)b * 2 * a.ref_ld + n;
    const float e0 = e[0], e1 = e[a.est_ld], r0 = r[0], r1 = r[a.ref_ld];
    acc[0] += fabsf(e0 - r0);
    acc[1] += fabsf(e0 - r1);
    acc[2] += fabsf(e1 - r0);
    acc[3] += fabsf(e1 - r1);
    n += PIT_THREADS;
    while (n >= a.L) { n -= a.L; ++b; }
  }
  block_reduce_store<4>(acc, red, a.partial + (size_t)blockIdx.x * 4);
}

// The pairwise L1 sums of this launch's rows: block partials summed in block order (sums[4], double). The partials are
// staged in LDS by all threads (every load in flight at once), then thread j < 4 adds value j of the blocks in block
// order, loads 8 at a time -- the same order and bits as one thread walking the partials (which took ~66 us for the
// 512 blocks of a 16 k-sample overlap: one dependent global load per add).
__device__ __forceinline__ void pit_block_sums(const PitArgs& a, int nblk, double* part, double* sums) {
  for (int i = threadIdx.x; i < nblk * 4; i += 256) part[i] = a.partial[i];
  __syncthreads();
  if (threadIdx.x >= 4) return;
  const int j = threadIdx.x;
  double pw = 0.0;
  int k = 0;
  for (; k + 8 <= nblk; k += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(k + u) * 4 + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) pw += v[u];
  }
  for (; k < nblk; ++k) pw += part[k * 4 + j];
  sums[j] = pw;
}

__global__ __launch_bounds__(256) void k_pit_l1_sums(PitArgs a, int nblk, double* sums) {
  __shared__ double part[PIT_MAX_BLOCKS * 4];
  pit_block_sums(a, nblk, part, sums);
}

// One block: pairwise means from the sums (of this device's rows, or all-reduced over the ranks of a
// sharded stream batch: nn.L1Loss means over the WHOLE batch, model/pit_wrapper.py:172-177), the permutation
// loss set (einsum over one-hot perms / n_src, :289-300), torch.min's first-minimum choice (:308), the
// indices (:311) for this device's a.B rows.
__device__ __forceinline__ void pit_choose(const PitArgs& a, const double* sums, double cnt) {
  // every thread makes the same choice from the same sums; the per-row indices are written by all threads
  double pw[4];
  for (int j = 0; j < 4; ++j) pw[j] = sums[j];
  float m[4];
  for (int j = 0; j < 4; ++j) m[j] = (float)(pw[j] / cnt);
  // pwl = pw^T (targets x estimates); perms (0,1), (1,0)
  const float loss_id = (m[0] + m[3]) / 2.f;    // pwl[0][0] + pwl[1][1]
  const float loss_sw = (m[2] + m[1]) / 2.f;    // pwl[0][1] + pwl[1][0] = pw[1][0] + pw[0][1]
  const bool swap = loss_sw < loss_id;          // ties keep the first permutation
  if (a.perm_out) {
    for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
      a.perm_out[2 * b] = swap ? 1 : 0;
      a.perm_out[2 * b + 1] = swap ? 0 : 1;
    }
  }
  if (threadIdx.x != 0) return;
  if (a.loss_out) *a.loss_out = swap ? loss_sw : loss_id;
  if (a.pw_out)
    for (int j = 0; j < 4; ++j) a.pw_out[j] = m[j];
}

__global__ __launch_bounds__(256) void k_pit_l1_choose(PitArgs a, const double* sums, double cnt) {
  pit_choose(a, sums, cnt);
}

// An unsharded batch: the block sums and the choice in one launch (the sums through LDS; also written to `sums`)
__global__ __launch_bounds__(256) void k_pit_l1_sums_choose(PitArgs a, int nblk, double* sums, double cnt) {
  __shared__ double part[PIT_MAX_BLOCKS * 4];
  __shared__ double tot[4];
  pit_block_sums(a, nblk, part, tot);
  __syncthreads();
  if (threadIdx.x < 4) sums[threadIdx.x] = tot[threadIdx.x];
  pit_choose(a, tot, cnt);
}

hipError_t launch_pit_l1_sums(const PitArgs& a, double* sums, hipStream_t s) {
  if (a.B < 1 || a.L < 1 || a.nblk < 1 || a.nblk > PIT_MAX_BLOCKS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pit_l1_partial, dim3(a.nblk), dim3(PIT_THREADS), 0, s, a);
  hipLaunchKernelGGL(k_pit_l1_sums, dim3(1), dim3(256), 0, s, a, a.nblk, sums);
  return hipGetLastError();
}

hipError_t launch_pit_l1_choose(const PitArgs& a, const double* sums, double count, hipStream_t s) {
  hipLaunchKernelGGL(k_pit_l1_choose, dim3(1), dim3(256), 0, s, a, sums, count);
  return hipGetLastError();
}

hipError_t launch_pit_l1(const PitArgs& a, hipStream_t s) {
  // the sums live in the scratch right after the block partials
  double* sums = a.partial + (size_t)PIT_MAX_BLOCKS * 4;
  if (a.B < 1 || a.L < 1 || a.nblk < 1 || a.nblk > PIT_MAX_BLOCKS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pit_l1_partial, dim3(a.nblk), dim3(PIT_THREADS), 0, s, a);
  hipLaunchKernelGGL(k_pit_l1_sums_choose, dim3(1), dim3(256), 0, s, a, a.nblk, sums, (double)a.B * (double)a.L);
  return hipGetLastError();
}

// dst[b][i][d0 + n] = src[b][perm[b][i]][s0 + n], n < H  (perm null = identity)
__global__ __launch_bounds__(256) void k_stream_append(AppendArgs a) {
  const long long total = (long long)a.B * 2 * a.H;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long n = i % a.H, bi = i / a.H;
    const int b = (int)(bi >> 1), s = (int)(bi & 1);
    const int ps = a.perm ? (int)a.perm[2 * b + s] : s;
    a.dst[((size_t)b * 2 + s) * a.dst_ld + a.d0 + n] = a.src[((size_t)b * 2 + ps) * a.src_ld + a.s0 + n];
  }
}

hipError_t launch_stream_append(const AppendArgs& a, hipStream_t s) {
  if (a.B < 1 || a.H < 1) return hipErrorInvalidValue;
  const long long total = (long long)a.B * 2 * a.H;
  const long long nb = (total + 255) / 256;
  const int grid = (int)(nb < 4096 ? nb : 4096);
  hipLaunchKernelGGL(k_stream_append, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sepvad
