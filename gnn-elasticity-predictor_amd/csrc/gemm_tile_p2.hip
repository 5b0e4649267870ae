// gemm_tile_p2.hip — the tiled GEMM kernels of arithmetic 2 (gemm_tile.h: bf16 inputs through bf16
// LDS images), one translation unit per arithmetic so the library builds them in parallel.
#include "gemm_tile.h"

namespace alignn {
template void gemm_tiled_launch<2>(const GemmParams&, int, int, bool, bool, dim3, int, bool, hipStream_t);
}  // namespace alignn
