// fused_v2_km42.hip — RS(4+2) encode variants (diagnostics build only; fused_v2_km.hpp).
#include "fused_v2_km.hpp"

namespace zs3k {

#if ZS3_DIAG
bool launch_ehx_km_4_2(int v, const EncArgs& a, hipStream_t s) { return launch_ehx_km<4, 2>(v, a, s); }
#endif

}  // namespace zs3k
