// gemm_tile_p1.hip — the tiled GEMM kernels of arithmetic 1 (gemm_tile.h: bf16 inputs),
// one translation unit per arithmetic so the library builds them in parallel.
#include "gemm_tile.h"

namespace alignn {
template void gemm_tiled_launch<1>(const GemmParams&, int, int, bool, bool, dim3, int, bool, hipStream_t);
}  // namespace alignn
