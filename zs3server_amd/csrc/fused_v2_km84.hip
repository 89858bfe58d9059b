// fused_v2_km84.hip — RS(8+4) encode variants (diagnostics build only; fused_v2_km.hpp).
#include "fused_v2_km.hpp"

namespace zs3k {

#if ZS3_DIAG
bool launch_ehx_km_8_4(int v, const EncArgs& a, hipStream_t s) { return launch_ehx_km<8, 4>(v, a, s); }
#endif

}  // namespace zs3k
