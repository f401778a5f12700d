// The fused persistent TCN (k_tcn, tcn_kernel.h): launch and occupancy dispatch by (precision, weight lo-plane format).
// Each (precision, lo format) pair is instantiated in its own object (fused_inst.hip compiled once per pair, see the
// Makefile), so the ~80 kernel instantiations build in parallel.
#include "sepvad_internal.h"

namespace sepvad {

#ifdef TCN_ONE  // resource checks only (tools): the production kernels of both widths, nothing launchable
}  // namespace sepvad
#include "tcn_kernel.h"
namespace sepvad {
template __global__ void k_tcn<LD_RECURSIVE, PREC_F16X3, false, 2, false, false, 2>(TcnArgs);
template __global__ void k_tcn<LD_RECURSIVE, PREC_F16X3, false, 2, false, false, 1>(TcnArgs);
template __global__ void k_tcn<LD_RECURSIVE, PREC_F16X3, false, 0, false, false, 2>(TcnArgs);
template __global__ void k_tcn<LD_RECURSIVE, PREC_F32, false, 0, false, false, 1>(TcnArgs);
#else
// defined in fused_inst.hip, one explicit specialisation per object
template <int PRE, int LQ> hipError_t launch_tcn_combo(const TcnArgs& a, int grid, hipStream_t s);
template <int PRE, int LQ> int tcn_bpc_combo(int ln_mode, int nsl);

hipError_t launch_tcn(const TcnArgs& a, int grid, hipStream_t s) {
  if (a.nsl != 1 && a.nsl != 2) return hipErrorInvalidValue;
  const int gw = a.run > 0 ? 8 * a.run : a.G / a.nsl;  // blocks per group
  if (a.G < 1 || a.G > FG_MAX || a.G * FR < a.T || a.G * FR > a.Tp || a.G % a.nsl || grid < gw || grid % gw ||
      (a.nsl == 2 && a.G > FG_WAVE) || (a.run > 0 && (a.nsl != 1 || a.G <= 32 || a.run != (a.G + 7) / 8)))
    return hipErrorInvalidValue;
  switch (a.prec) {
    case PREC_F16X3:
      switch (a.lo8) {
        case 0: return launch_tcn_combo<PREC_F16X3, 0>(a, grid, s);
        case 1: return launch_tcn_combo<PREC_F16X3, 1>(a, grid, s);
        case 2: return launch_tcn_combo<PREC_F16X3, 2>(a, grid, s);
      }
      return hipErrorInvalidValue;
    case PREC_F16: return launch_tcn_combo<PREC_F16, 0>(a, grid, s);
    case PREC_BF16: return launch_tcn_combo<PREC_BF16, 0>(a, grid, s);
    case PREC_F32: return a.nsl == 1 ? launch_tcn_combo<PREC_F32, 0>(a, grid, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

int tcn_blocks_per_cu(int ln_mode, int prec, int lo, int nsl) {
  switch (prec) {
    case PREC_F16X3:
      return lo == 1 ? tcn_bpc_combo<PREC_F16X3, 1>(ln_mode, nsl)
                     : (lo == 2 ? tcn_bpc_combo<PREC_F16X3, 2>(ln_mode, nsl) : tcn_bpc_combo<PREC_F16X3, 0>(ln_mode, nsl));
    case PREC_F16: return tcn_bpc_combo<PREC_F16, 0>(ln_mode, nsl);
    case PREC_BF16: return tcn_bpc_combo<PREC_BF16, 0>(ln_mode, nsl);
    case PREC_F32: return nsl == 1 ? tcn_bpc_combo<PREC_F32, 0>(ln_mode, 1) : 0;
  }
  return 0;
}
#endif  // TCN_ONE

}  // namespace sepvad
