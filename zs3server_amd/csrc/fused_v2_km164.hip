// fused_v2_km164.hip — RS(16+4) encode variants (diagnostics build only; fused_v2_km.hpp).
#include "fused_v2_km.hpp"

namespace zs3k {

#if ZS3_DIAG
bool launch_ehx_km_16_4(int v, const EncArgs& a, hipStream_t s) { return launch_ehx_km<16, 4>(v, a, s); }
#endif

}  // namespace zs3k
