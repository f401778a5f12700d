// One (precision, weight lo-plane format) pair of the fused TCN: every k_tcn instantiation it launches and its
// occupancy query. Compiled once per pair with -DFI_PRE=<Precision> -DFI_LQ=<lo format> (Makefile).
#include "tcn_kernel.h"

#if !defined(FI_PRE) || !defined(FI_LQ)
#error "fused_inst.hip: build with -DFI_PRE and -DFI_LQ"
#endif

namespace sepvad {

template <int PRE, int LQ> hipError_t launch_tcn_combo(const TcnArgs& a, int grid, hipStream_t s);
template <int PRE, int LQ> int tcn_bpc_combo(int ln_mode, int nsl);

template <>
hipError_t launch_tcn_combo<FI_PRE, FI_LQ>(const TcnArgs& a, int grid, hipStream_t s) {
  return launch_tcn_lg<FI_PRE, FI_LQ>(a, grid, s);
}

template <>
int tcn_bpc_combo<FI_PRE, FI_LQ>(int ln_mode, int nsl) {
  if constexpr (FI_PRE != PREC_F32) {
    if (nsl == 2) return blocks_per_cu_pre<FI_PRE, FI_LQ, 2>(ln_mode);
  }
  return nsl == 1 ? blocks_per_cu_pre<FI_PRE, FI_LQ, 1>(ln_mode) : 0;
}

}  // namespace sepvad
