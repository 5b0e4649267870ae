// gemm_tile_p0.hip — the tiled GEMM kernels of arithmetic 0 (gemm_tile.h: exact fp32),
// one translation unit per arithmetic so the library builds them in parallel.
#include "gemm_tile.h"

namespace alignn {
template void gemm_tiled_launch<0>(const GemmParams&, int, int, bool, bool, dim3, int, bool, hipStream_t);
}  // namespace alignn
