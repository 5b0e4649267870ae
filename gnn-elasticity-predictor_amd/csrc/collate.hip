// collate.hip — batch assembly from a dataset resident in HBM.
//
// Replaces PyG's Collater / Batch.from_data_list over the reference's per-sample
// `.pt` loads (train.py:132): the whole dataset lives in HBM as flat per-field arrays with per-graph
// row ranges, and a batch is a set of segmented copies.  Index fields (edge_index, lg_edge_index:
// two rows each) get the per-graph increment added — the caller passes PyG's increments, including
// the lg_edge_index-by-num_nodes rule, so the batch is bit-identical to PyG's.
#include <cstring>

#include "common.h"

namespace alignn {

// Up to kCopyMany device-to-device copies in one launch (re-binding a captured step to a new batch:
// the batch's fields and its device cache, FusedTrainer._rebind).  The list travels as a kernel
// argument, so the launch needs no upload.  Workgroups stride over the concatenated 16-byte units.
constexpr int kCopyMany = 32;
struct CopyList {
  const unsigned char* src[kCopyMany];
  unsigned char* dst[kCopyMany];
  int64_t units[kCopyMany + 1];  // exclusive prefix sums of 16-byte units per copy (last one may be partial)
  int64_t bytes[kCopyMany];
  int32_t n;
  int32_t pad_;
};

__global__ __launch_bounds__(256) void copy_many_kernel(CopyList L) {
  const int64_t total = L.units[L.n];
  int c = 0;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    while (u >= L.units[c + 1]) ++c;  // units ascend along a thread's grid-stride walk
    const int64_t o = (u - L.units[c]) * 16;
    const int64_t left = L.bytes[c] - o;
    if (left >= 16) {
      *reinterpret_cast<uint4*>(L.dst[c] + o) = *reinterpret_cast<const uint4*>(L.src[c] + o);
    } else {  // the copy's last, partial unit: 4-byte words
      for (int64_t w = 0; w < left; w += 4)
        *reinterpret_cast<uint32_t*>(L.dst[c] + o + w) = *reinterpret_cast<const uint32_t*>(L.src[c] + o + w);
    }
  }
}

// grid (chunks, G): graph g's segment [src_start[g], +count[g]) * width -> [dst_start[g], ...)
__global__ void collate_rows_kernel(const float* __restrict__ src, int64_t width, const int64_t* __restrict__ src_start,
                                    const int64_t* __restrict__ dst_start, const int64_t* __restrict__ count,
                                    float* __restrict__ dst) {
  const int g = blockIdx.y;
  const int64_t n = count[g] * width;
  const float* s = src + src_start[g] * width;
  float* d = dst + dst_start[g] * width;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

// Two-row int64 index field: row r of graph g's segment, plus add[g].
__global__ void collate_index_kernel(const int64_t* __restrict__ src, int64_t src_ld,
                                     const int64_t* __restrict__ src_start, const int64_t* __restrict__ dst_start,
                                     const int64_t* __restrict__ count, const int64_t* __restrict__ add,
                                     int64_t* __restrict__ dst, int64_t dst_ld) {
  const int g = blockIdx.y;
  const int64_t n = count[g];
  const int64_t a = add[g];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    dst[dst_start[g] + i] = src[src_start[g] + i] + a;
    dst[dst_ld + dst_start[g] + i] = src[src_ld + src_start[g] + i] + a;
  }
}

// batch vector: nodes of graph g get g
__global__ void collate_batchvec_kernel(const int64_t* __restrict__ dst_start, const int64_t* __restrict__ count,
                                        int64_t* __restrict__ batch) {
  const int g = blockIdx.y;
  const int64_t n = count[g];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    batch[dst_start[g] + i] = g;
}

// Rows with PtGraphDataset.__getitem__'s per-sample transform fused into the copy
// (train.py:137-154 node-dim select / pad / truncate, :200-216 z-scoring): a destination row is the
// source row's first copy_w values, zero-padded to dst_w; with statistics, every value becomes
// (v - mean[k]) / std[k] (fp32, correctly rounded as the reference's tensor ops), k = the column
// (by_row = 0: node features) or the element's index inside the graph's segment (by_row = 1:
// global_x, one value per row, standardized per position).
__global__ void collate_rows_std_kernel(const float* __restrict__ src, int64_t src_w,
                                        const int64_t* __restrict__ src_start, const int64_t* __restrict__ dst_start,
                                        const int64_t* __restrict__ count, float* __restrict__ dst, int64_t dst_w,
                                        int64_t copy_w, const float* __restrict__ mean, const float* __restrict__ stdv,
                                        int by_row) {
  const int g = blockIdx.y;
  const int64_t n = count[g] * dst_w;
  const float* s = src + src_start[g] * src_w;
  float* d = dst + dst_start[g] * dst_w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / dst_w, c = i - r * dst_w;
    float v = c < copy_w ? s[r * src_w + c] : 0.f;
    if (mean) {
      const int64_t k = by_row ? i : c;
      v = (v - mean[k]) / stdv[k];
    }
    d[i] = v;
  }
}

// ok[g] = 0 when graph g's segment of a float field holds a NaN or an infinity (PtGraphDataset._is_valid,
// train.py:174-182).  ok is preset to 1 by the caller; fields are checked one launch each.
__global__ void segment_finite_kernel(const float* __restrict__ src, int64_t width, const int64_t* __restrict__ start,
                                      const int64_t* __restrict__ count, int32_t* __restrict__ ok) {
  const int g = blockIdx.y;
  const int64_t n = count[g] * width;
  const float* s = src + start[g] * width;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(s[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) ok[g] = 0;
}

// Per-graph fp64 sums for the feature statistics (train.py:1337-1352): for graph j of the selection,
// part[j][k] = sum over its rows of v and of v^2 (by_row = 0: k = column, rows summed in order;
// by_row = 1: k = the element's index in the segment, one value each).  Block (j, column chunk).
__global__ void seg_stats_f64_kernel(const float* __restrict__ src, int64_t width, const int64_t* __restrict__ start,
                                     const int64_t* __restrict__ count, int64_t K, int by_row,
                                     double* __restrict__ psum, double* __restrict__ psq) {
  const int64_t j = blockIdx.y;
  const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (k >= K) return;
  const float* s = src + start[j] * width;
  double a = 0.0, q = 0.0;
  if (by_row) {
    if (k < count[j] * width) {
      a = (double)s[k];
      q = a * a;
    }
  } else {
    for (int64_t r = 0; r < count[j]; ++r) {
      const double v = (double)s[r * width + k];
      a += v;
      q += v * v;
    }
  }
  psum[j * K + k] = a;
  psq[j * K + k] = q;
}

// sum[k] = sum_j part[j][k] in selection order (the reference's running per-graph accumulation)
__global__ void stats_reduce_f64_kernel(const double* __restrict__ psum, const double* __restrict__ psq, int64_t J,
                                        int64_t K, double* __restrict__ sum, double* __restrict__ sq) {
  const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (k >= K) return;
  double a = 0.0, q = 0.0;
  for (int64_t j = 0; j < J; ++j) {
    a += psum[j * K + k];
    q += psq[j * K + k];
  }
  sum[k] = a;
  sq[k] = q;
}

// The inert "ghost" graph that pads a batch to a fixed capacity (store.BatchCapacity): ghost edge j
// (j < count) of a two-row int64 index field runs base + (j + 1) % mod -> base + j % mod, i.e. a ring
// over `mod` ghost nodes (in-degree ceil(count / mod)).
__global__ void ghost_edges_kernel(int64_t* __restrict__ dst, int64_t ld, int64_t start, int64_t count, int64_t base,
                                   int64_t mod) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < count; j += (int64_t)gridDim.x * blockDim.x) {
    dst[start + j] = base + (j + 1) % mod;
    dst[ld + start + j] = base + j % mod;
  }
}

static dim3 seg_grid(int64_t max_count_elems, int G) {
  int64_t chunks = (max_count_elems + 1023) / 1024;
  if (chunks < 1) chunks = 1;
  if (chunks > 64) chunks = 64;
  return dim3((unsigned)chunks, (unsigned)G);
}

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_collate_rows_f32(int32_t G, const float* src, int64_t width, const int64_t* src_start,
                                       const int64_t* dst_start, const int64_t* count, int64_t max_count,
                                       float* dst, void* stream) {
  if (G < 0 || width < 0 || max_count < 0) return ALIGNN_E_BAD_SHAPE;
  if (G == 0 || width == 0 || max_count == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(collate_rows_kernel, seg_grid(max_count * width, G), dim3(256), 0, s, src, width, src_start,
                     dst_start, count, dst);
  ALIGNN_LAUNCH_CHECK("collate_rows_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_collate_index_i64(int32_t G, const int64_t* src, int64_t src_ld, const int64_t* src_start,
                                        const int64_t* dst_start, const int64_t* count, const int64_t* add,
                                        int64_t max_count, int64_t* dst, int64_t dst_ld, void* stream) {
  if (G < 0 || max_count < 0) return ALIGNN_E_BAD_SHAPE;
  if (G == 0 || max_count == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(collate_index_kernel, seg_grid(max_count, G), dim3(256), 0, s, src, src_ld, src_start, dst_start,
                     count, add, dst, dst_ld);
  ALIGNN_LAUNCH_CHECK("collate_index_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_collate_batchvec(int32_t G, const int64_t* dst_start, const int64_t* count, int64_t max_count,
                                       int64_t* batch, void* stream) {
  if (G < 0 || max_count < 0) return ALIGNN_E_BAD_SHAPE;
  if (G == 0 || max_count == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(collate_batchvec_kernel, seg_grid(max_count, G), dim3(256), 0, s, dst_start, count, batch);
  ALIGNN_LAUNCH_CHECK("collate_batchvec_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_copy_many(int32_t n, const void* const* src, void* const* dst, const int64_t* bytes, void* stream) {
  if (n < 0 || n > kCopyMany || (n > 0 && (!src || !dst || !bytes))) {
    set_error("copy_many: 0..%d copies, host arrays of pointers and sizes", kCopyMany);
    return ALIGNN_E_BAD_SHAPE;
  }
  CopyList L;
  memset(&L, 0, sizeof L);  // defined padding bytes (plan.hip scans recorded struct words)
  L.n = n;
  for (int i = 0; i < n; ++i) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(src[i]), b = reinterpret_cast<uintptr_t>(dst[i]);
    if (bytes[i] < 0 || bytes[i] % 4 || (bytes[i] && (!src[i] || !dst[i] || (a & 15) || (b & 15)))) {
      set_error("copy_many: copy %d needs 16-byte aligned pointers and a multiple of 4 bytes", i);
      return ALIGNN_E_BAD_SHAPE;
    }
    L.src[i] = static_cast<const unsigned char*>(src[i]);
    L.dst[i] = static_cast<unsigned char*>(dst[i]);
    L.bytes[i] = bytes[i];
    L.units[i + 1] = L.units[i] + (bytes[i] + 15) / 16;
  }
  if (L.units[n] == 0) return ALIGNN_OK;
  const int64_t blocks = std::min<int64_t>((L.units[n] + 255) / 256, 2048);
  launch(copy_many_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), L);
  ALIGNN_LAUNCH_CHECK("copy_many_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_collate_rows_std_f32(int32_t G, const float* src, int64_t src_width, const int64_t* src_start,
                                           const int64_t* dst_start, const int64_t* count, int64_t max_count,
                                           float* dst, int64_t dst_width, int64_t copy_width, const float* mean,
                                           const float* stdv, int32_t by_row, void* stream) {
  if (G < 0 || src_width < 0 || dst_width < 0 || max_count < 0 || copy_width < 0 || copy_width > src_width ||
      copy_width > dst_width || (!mean) != (!stdv)) {
    set_error("collate_rows_std: 0 <= copy_width <= min(src_width, dst_width); mean and std both or neither");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (G == 0 || dst_width == 0 || max_count == 0) return ALIGNN_OK;
  launch(collate_rows_std_kernel, seg_grid(max_count * dst_width, G), dim3(256), 0,
         reinterpret_cast<hipStream_t>(stream), src, src_width, src_start, dst_start, count, dst, dst_width,
         copy_width, mean, stdv, (int)by_row);
  ALIGNN_LAUNCH_CHECK("collate_rows_std_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_segment_finite_f32(int32_t G, const float* src, int64_t width, const int64_t* start,
                                         const int64_t* count, int64_t max_count, int32_t* ok, void* stream) {
  if (G < 0 || width < 0 || max_count < 0) return ALIGNN_E_BAD_SHAPE;
  if (G == 0 || width == 0 || max_count == 0) return ALIGNN_OK;
  launch(segment_finite_kernel, seg_grid(max_count * width, G), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
         src, width, start, count, ok);
  ALIGNN_LAUNCH_CHECK("segment_finite_kernel");
  return ALIGNN_OK;
}

extern "C" int64_t alignn_feature_stats_workspace(int32_t J, int64_t K) {
  if (J < 0 || K < 0) return -1;
  return 2 * (int64_t)J * K;
}

extern "C" int alignn_feature_stats_f64(int32_t J, const float* src, int64_t width, const int64_t* start,
                                        const int64_t* count, int64_t K, int32_t by_row, double* sum, double* sq,
                                        double* workspace, int64_t workspace_elems, void* stream) {
  if (J < 0 || width <= 0 || K < 0 || (!by_row && K > width) || workspace_elems < 2 * (int64_t)J * K) {
    set_error("feature_stats: K <= width (columns) and a workspace of 2 J K doubles");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (K == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  double* psum = workspace;
  double* psq = workspace + (int64_t)J * K;
  if (J > 0) {
    launch(seg_stats_f64_kernel, dim3((unsigned)((K + 255) / 256), (unsigned)J), dim3(256), 0, s, src, width, start,
           count, K, (int)by_row, psum, psq);
    ALIGNN_LAUNCH_CHECK("seg_stats_f64_kernel");
  }
  launch(stats_reduce_f64_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, psum, psq, (int64_t)J, K, sum,
         sq);
  ALIGNN_LAUNCH_CHECK("stats_reduce_f64_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_ghost_edges_i64(int64_t* dst, int64_t ld, int64_t start, int64_t count, int64_t base,
                                      int64_t mod, void* stream) {
  if (count < 0 || start < 0 || base < 0 || (count > 0 && mod <= 0)) {
    set_error("ghost_edges: count >= 0, start >= 0, base >= 0 and mod > 0");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (count == 0) return ALIGNN_OK;
  const int64_t blocks = std::min<int64_t>((count + 255) / 256, 1024);
  launch(ghost_edges_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), dst, ld,
         start, count, base, mod);
  ALIGNN_LAUNCH_CHECK("ghost_edges_kernel");
  return ALIGNN_OK;
}
