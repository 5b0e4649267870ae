// graph.hip — CSR neighbour lists from PyG edge_index, built on the device once per batch.
//
// Replaces the index bookkeeping of PyG MessagePassing (collect: index_select by edge_index[0/1];
// aggregate: scatter by edge_index[1]) used by TransformerConv at train.py:315/:334.
//
// Deterministic counting sort: count (wave-aggregated int atomics) -> exclusive scan (one block) ->
// fill with per-key cursors (wave-aggregated int atomics, arbitrary order) -> per-segment rank sort by original position,
// so every segment lists its edges in ascending original order regardless of atomic timing.
#include "common.h"

namespace alignn {

// Keys of neighbouring edges often repeat (a line graph in target order lists the same few source
// bonds for every bond leaving one atom), and same-address atomics from one wave serialise in L2:
// the source-side CSR of the B = 32 line graph took 43 us (count) + 52 us (fill) with per-lane
// atomics.  Each wave therefore groups its lanes by key (readfirstlane + ballot over the lanes still
// pending, one round per distinct key) and one lane per group does the atomic for the whole group.

// Mask of the active lanes whose key equals this lane's: one readfirstlane + ballot round per
// distinct key among the lanes still pending.  Only the masks leave the loop; the atomics and the
// broadcast of their results run after it, where every active lane has converged again.
__device__ __forceinline__ uint64_t key_group(int32_t k) {
  uint64_t mine = 0;
  bool pending = true;
  while (pending) {
    const int32_t kl = __builtin_amdgcn_readfirstlane(k);
    const uint64_t same = __ballot(k == kl);
    if (k == kl) {
      mine = same;
      pending = false;
    }
  }
  return mine;
}

template <typename K>
__global__ void csr_count(const K* __restrict__ keys, int64_t m, int64_t n, int32_t* __restrict__ cnt,
                          int32_t* __restrict__ err) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k64 = (int64_t)keys[e];
    if (k64 < 0 || k64 >= n) {
      atomicOr(err, 1);
      continue;
    }
    const uint64_t same = key_group((int32_t)k64);
    if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)same) - 1) atomicAdd(&cnt[k64], __popcll(same));
  }
}

// Single-block exclusive scan of cnt[0..n) -> off[0..n]; cursor[i] = off[i].
__global__ __launch_bounds__(1024) void csr_scan(const int32_t* __restrict__ cnt, int64_t n, int32_t* __restrict__ off,
                                                 int32_t* __restrict__ cursor) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t b = t * chunk, e = min(n, b + chunk);
  int32_t s = 0;
  for (int64_t i = b; i < e; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan over 1024 partials
  for (int o = 1; o < 1024; o <<= 1) {
    int32_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int32_t run = t ? part[t - 1] : 0;
  for (int64_t i = b; i < e; ++i) {
    off[i] = run;
    cursor[i] = run;
    run += cnt[i];
  }
  if (t == 1023) off[n] = part[1023];
}

// Positions within a key's segment come out in arbitrary order (csr_sort_segments restores the
// original order); one atomic per (wave, key) group as in csr_count.
template <typename K>
__global__ void csr_fill(const K* __restrict__ keys, int64_t m, int64_t n, int32_t* __restrict__ cursor,
                         int32_t* __restrict__ perm) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k64 = (int64_t)keys[e];
    if (k64 < 0 || k64 >= n) continue;
    const uint64_t same = key_group((int32_t)k64);
    const int leader = __ffsll((unsigned long long)same) - 1;
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(&cursor[k64], __popcll(same));
    base = __shfl(base, leader);   // the leader is one of the lanes active here
    perm[base + __popcll(same & below)] = (int32_t)e;
  }
}

// One wave per segment: rank each element by counting the smaller ones (values are distinct
// edge ids), then scatter to its rank.  Segments up to 1024 are staged in LDS.
__global__ __launch_bounds__(256) void csr_sort_segments(const int32_t* __restrict__ off, int64_t n,
                                                         int32_t* __restrict__ perm) {
  __shared__ int32_t buf[4][1024];
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int64_t seg = blockIdx.x * 4 + wave;
  if (seg >= n) return;
  const int32_t b = off[seg], e = off[seg + 1], len = e - b;
  if (len <= 1) return;
  if (len <= 1024) {
    int32_t* s = buf[wave];
    for (int i = lane; i < len; i += 64) s[i] = perm[b + i];
    __threadfence_block();
    // ranks are read from the LDS copy, so writing perm in place is race-free
    for (int i = lane; i < len; i += 64) {
      const int32_t v = s[i];
      int32_t r = 0;
      for (int j = 0; j < len; ++j) r += s[j] < v;
      perm[b + r] = v;
    }
  } else if (lane == 0) {
    // Pathological segment (> 1024 in-edges; the reference's shapes peak at 132):
    // single-lane insertion sort — correct, slow, never on the measured path.
    for (int32_t i = b + 1; i < e; ++i) {
      int32_t v = perm[i], j = i - 1;
      while (j >= b && perm[j] > v) {
        perm[j + 1] = perm[j];
        --j;
      }
      perm[j + 1] = v;
    }
  }
}

// Per position p (target-sorted): src_at[p] = src[perm[p]], dst_at[p] = dst[perm[p]].
// Positions past off[n] exist only when some index was out of range (err flag set): mark them -1.
__global__ void csr_endpoints(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, const int32_t* __restrict__ perm,
                              const int32_t* __restrict__ off, int64_t n, int64_t m, int32_t* __restrict__ src_at,
                              int32_t* __restrict__ dst_at) {
  const int64_t valid = off[n];
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < m; p += (int64_t)gridDim.x * blockDim.x) {
    if (p >= valid) {
      src_at[p] = -1;
      dst_at[p] = -1;
      continue;
    }
    int32_t e = perm[p];
    src_at[p] = (int32_t)src[e];
    dst_at[p] = (int32_t)dst[e];
  }
}

__global__ void gather_rows_kernel(const float* __restrict__ in, int64_t ld_in, const int32_t* __restrict__ idx,
                                   int64_t rows, int64_t cols, float* __restrict__ out, int64_t ld_out) {
  const int64_t total = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i / cols, c = i % cols;
    out[r * ld_out + c] = in[(int64_t)idx[r] * ld_in + c];
  }
}

__global__ void scatter_rows_kernel(const float* __restrict__ in, int64_t ld_in, const int32_t* __restrict__ idx,
                                    int64_t rows, int64_t cols, float* __restrict__ out, int64_t ld_out, int acc) {
  const int64_t total = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i / cols, c = i % cols;
    float* o = out + (int64_t)idx[r] * ld_out + c;
    const float v = in[r * ld_in + c];
    *o = acc ? *o + v : v;
  }
}

// The same two row moves with one wave per row and 16-byte accesses (rows of 4-float multiples at
// 16-byte aligned addresses): no 64-bit divide per element — the element loops above are
// instruction-bound at C3 (a 16k x 256 gather: 27 us for 33 MB).
template <bool SCATTER>
__global__ __launch_bounds__(256) void move_rows4_kernel(const float4* __restrict__ in, int64_t ld_in4,
                                                         const int32_t* __restrict__ idx, int64_t rows, int cols4,
                                                         float4* __restrict__ out, int64_t ld_out4, int acc) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave_id(); r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t j = idx[r];
    const float4* src = in + (SCATTER ? r : j) * ld_in4;
    float4* dst = out + (SCATTER ? j : r) * ld_out4;
    for (int c = lane; c < cols4; c += 64) {
      float4 v = src[c];
      if (SCATTER && acc) {
        const float4 o = dst[c];
        v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
      }
      dst[c] = v;
    }
  }
}

static bool rows4_ok(const float* in, int64_t ld_in, const float* out, int64_t ld_out, int64_t cols) {
  return cols % 4 == 0 && ld_in % 4 == 0 && ld_out % 4 == 0 && cols / 4 <= (1 << 30) &&
         ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
}

static int grid_for(int64_t work, int block = 256, int64_t cap = 8192) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <typename K>
static int build_csr(const K* keys, int64_t m, int64_t n, int32_t* off, int32_t* perm, int32_t* ws, int32_t* err,
                     hipStream_t s) {
  int32_t* cnt = ws;
  int32_t* cursor = ws + n;
  hipError_t he = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (size_t)n, s);
  if (he != hipSuccess) return hip_status(he, "hipMemsetAsync");
  if (m > 0) {
    launch(csr_count<K>, dim3(grid_for(m)), dim3(256), 0, s, keys, m, n, cnt, err);
    ALIGNN_LAUNCH_CHECK("csr_count");
  }
  launch(csr_scan, dim3(1), dim3(1024), 0, s, cnt, n, off, cursor);
  ALIGNN_LAUNCH_CHECK("csr_scan");
  if (m > 0) {
    launch(csr_fill<K>, dim3(grid_for(m)), dim3(256), 0, s, keys, m, n, cursor, perm);
    ALIGNN_LAUNCH_CHECK("csr_fill");
    launch(csr_sort_segments, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, off, n, perm);
    ALIGNN_LAUNCH_CHECK("csr_sort_segments");
  }
  return ALIGNN_OK;
}


// -------------------------------------------------------------------------------------------
// Attention work lists on the device (ops.schedule_lists restated without the host round trip of
// the in-degrees): every target with in-edges, longest in-edge list first within each of `xcds`
// contiguous id ranges holding equal numbers of edges (ties in ascending id), the ranges interleaved
// in chunks of `chunk` items, then the targets without in-edges in ascending id — the host lists
// exactly.  One workgroup of four waves (it runs on the loader stream beside a step, where a small
// workgroup is easier to place than a 16-wave one): pass 1 histograms (range, degree) in LDS;
// pass 2 walks each range in id order, 256 targets at a time, and places each at its stable rank (rank among equal
// in-degrees within its wave from a ballot per distinct degree, plus the counts of the earlier waves
// of the block and of the earlier blocks).  The order matters for speed, not results: targets of one
// degree adjacent in id share their sources' rows in L2.  Needs every in-degree <= thr (the caller's
// host bound: no heavy list); a larger one sets bit 2 of *err.
// -------------------------------------------------------------------------------------------
constexpr int SCHED_MAX_THR = 512;
constexpr int SCHED_MAX_XCDS = 8;
constexpr int SCHED_WAVES = 4;

__global__ __launch_bounds__(256) void schedule_build_kernel(const int32_t* __restrict__ off, int64_t n, int thr,
                                                              int xcds, int chunk, int32_t* __restrict__ light,
                                                              int32_t* __restrict__ err) {
  __shared__ int32_t cur[SCHED_MAX_XCDS][SCHED_MAX_THR + 1];   // histogram, then bucket cursors
  __shared__ int32_t wcnt[SCHED_WAVES][SCHED_MAX_THR + 1];     // one block of 256: per-wave counts by degree
  __shared__ int64_t bounds[SCHED_MAX_XCDS + 1];
  __shared__ int32_t cnt[SCHED_MAX_XCDS];
  __shared__ int32_t nlit_s, zbase;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint64_t below = (1ull << lane) - 1;
  for (int i = t; i < SCHED_MAX_XCDS * (SCHED_MAX_THR + 1); i += blockDim.x) (&cur[0][0])[i] = 0;
  const int64_t tot = off[n];
  // range x covers ids [bounds[x], bounds[x+1]): bounds[x] = first id whose inclusive edge count
  // exceeds tot * x / xcds (numpy searchsorted(cumsum(deg), tot * x // xcds, 'right'))
  if (t <= xcds) {
    int64_t b;
    if (t == 0) b = 0;
    else if (t == xcds) b = n;
    else {
      const int64_t target = tot * t / xcds;
      int64_t lo = 0, hi = n;        // first i in [0, n) with off[i + 1] > target
      while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if ((int64_t)off[mid + 1] > target) hi = mid;
        else lo = mid + 1;
      }
      b = lo;
    }
    bounds[t] = b;
  }
  if (t == 0) { nlit_s = 0; zbase = 0; }
  __syncthreads();
  auto range_of = [&](int64_t i) {
    int r = 0;
    for (int x = 1; x < xcds; ++x) r += bounds[x] <= i;
    return r;
  };
  int mylit = 0;
  for (int64_t i = t; i < n; i += blockDim.x) {
    const int d = off[i + 1] - off[i];
    if (d > thr) {
      atomicOr(err, 2);
      continue;
    }
    if (d > 0) {
      atomicAdd(&cur[range_of(i)][d], 1);
      ++mylit;
    }
  }
  atomicAdd(&nlit_s, mylit);
  __syncthreads();
  const int64_t nlit = nlit_s;
  // fewer targets with in-edges than ranges: one range over all ids (the host rule: len(lit) > xcds)
  const bool ranged = nlit > xcds;
  if (!ranged) {
    for (int d = t; d <= thr; d += blockDim.x) {
      int32_t s = 0;
      for (int x = 0; x < xcds; ++x) s += cur[x][d];
      for (int x = 1; x < xcds; ++x) cur[x][d] = 0;
      cur[0][d] = s;
    }
    __syncthreads();
  }
  // per range: exclusive starts over degrees in descending order
  if (t < xcds) {
    int32_t run = 0;
    for (int d = thr; d >= 1; --d) {
      const int32_t c = cur[t][d];
      cur[t][d] = run;
      run += c;
    }
    cnt[t] = run;
  }
  __syncthreads();
  const int c = chunk < 1 ? 1 : chunk;
  const int nr = ranged ? xcds : 1;
  for (int r = 0; r < nr; ++r) {
    const int64_t b0 = ranged ? bounds[r] : 0, b1 = ranged ? bounds[r + 1] : n;
    for (int64_t c0 = b0; c0 < b1; c0 += blockDim.x) {
      for (int i = t; i < SCHED_WAVES * (thr + 1); i += blockDim.x) wcnt[i / (thr + 1)][i % (thr + 1)] = 0;
      __syncthreads();
      const int64_t i = c0 + t;
      int d = 0;
      if (i < b1) {
        d = off[i + 1] - off[i];
        if (d > thr) d = 0;
      }
      int rank = 0;
      if (d > 0) {
        const uint64_t same = key_group(d);
        rank = __popcll(same & below);
        if (lane == __ffsll((unsigned long long)same) - 1) wcnt[w][d] = __popcll(same);
      }
      __syncthreads();
      if (d > 0) {
        int32_t pre = 0;
        for (int w2 = 0; w2 < w; ++w2) pre += wcnt[w2][d];
        const int64_t k = (int64_t)cur[r][d] + pre + rank;   // stable rank within range r
        const int64_t j = k / c;                              // round
        int64_t pos = k % c;
        for (int x = 0; x < xcds; ++x) {
          const int64_t cx = cnt[x];
          pos += min(cx, j * c);                              // every range's items of earlier rounds
          if (x < r) pos += min((int64_t)c, max((int64_t)0, cx - j * c));   // earlier ranges, this round
        }
        light[pos] = (int32_t)i;
      }
      __syncthreads();
      for (int dd = t + 1; dd <= thr; dd += blockDim.x) {
        int32_t s = 0;
        for (int w2 = 0; w2 < SCHED_WAVES; ++w2) s += wcnt[w2][dd];
        cur[r][dd] += s;
      }
      __syncthreads();
    }
  }
  // targets without in-edges, ascending id, after every listed target — and any target whose
  // in-degree exceeds the threshold the caller promised (err bit 2): it still gets its place (the
  // single-wave kernels walk a segment of any length), so the list stays a permutation of the n
  // targets and no entry is left unwritten for the attention kernels to read as a node id
  for (int64_t c0 = 0; c0 < n; c0 += blockDim.x) {
    const int64_t i = c0 + t;
    const bool z = i < n && (off[i + 1] == off[i] || off[i + 1] - off[i] > thr);
    const uint64_t zm = __ballot(z);
    if (lane == 0) wcnt[w][0] = __popcll(zm);
    __syncthreads();
    if (z) {
      int32_t pre = zbase;
      for (int w2 = 0; w2 < w; ++w2) pre += wcnt[w2][0];
      light[nlit + pre + __popcll(zm & below)] = (int32_t)i;
    }
    __syncthreads();
    if (t == 0) {
      int32_t s = 0;
      for (int w2 = 0; w2 < SCHED_WAVES; ++w2) s += wcnt[w2][0];
      zbase += s;
    }
    __syncthreads();
  }
}
}  // namespace alignn

using namespace alignn;

extern "C" int alignn_graph_prep(const int64_t* edge_index, int64_t m, int64_t n, int32_t* off_dst, int32_t* perm_dst,
                                 int32_t* src_at, int32_t* dst_at, int32_t* off_src, int32_t* pos_src,
                                 int32_t* workspace, int32_t* err_flag, void* stream) {
  if (m < 0 || n < 0 || m > 0x7fffffffLL || n > 0x7ffffffeLL) {
    set_error("graph_prep: bad sizes m=%lld n=%lld", (long long)m, (long long)n);
    return ALIGNN_E_BAD_SHAPE;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t* src = edge_index;
  const int64_t* dst = edge_index + m;
  int rc = build_csr<int64_t>(dst, m, n, off_dst, perm_dst, workspace, err_flag, s);
  if (rc) return rc;
  if (m > 0) {
    launch(csr_endpoints, dim3(grid_for(m)), dim3(256), 0, s, src, dst, perm_dst, off_dst, n, m, src_at, dst_at);
    ALIGNN_LAUNCH_CHECK("csr_endpoints");
  }
  // Source-side CSR over target-sorted positions: keys = src_at.
  return build_csr<int32_t>(src_at, m, n, off_src, pos_src, workspace, err_flag, s);
}

extern "C" int alignn_gather_rows_f32(const float* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols,
                                      float* out, int64_t ld_out, void* stream) {
  if (rows < 0 || cols < 0) return ALIGNN_E_BAD_SHAPE;
  if (rows == 0 || cols == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows4_ok(in, ld_in, out, ld_out, cols)) {
    launch(move_rows4_kernel<false>, dim3(grid_for(rows, 4)), dim3(256), 0, s, reinterpret_cast<const float4*>(in),
           ld_in / 4, idx, rows, (int)(cols / 4), reinterpret_cast<float4*>(out), ld_out / 4, 0);
    ALIGNN_LAUNCH_CHECK("move_rows4_kernel");
    return ALIGNN_OK;
  }
  launch(gather_rows_kernel, dim3(grid_for(rows * cols)), dim3(256), 0, s, in, ld_in, idx, rows, cols,
                     out, ld_out);
  ALIGNN_LAUNCH_CHECK("gather_rows_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_scatter_rows_f32(const float* in, int64_t ld_in, const int32_t* idx, int64_t rows, int64_t cols,
                                       float* out, int64_t ld_out, int32_t accumulate, void* stream) {
  if (rows < 0 || cols < 0) return ALIGNN_E_BAD_SHAPE;
  if (rows == 0 || cols == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows4_ok(in, ld_in, out, ld_out, cols)) {
    launch(move_rows4_kernel<true>, dim3(grid_for(rows, 4)), dim3(256), 0, s, reinterpret_cast<const float4*>(in),
           ld_in / 4, idx, rows, (int)(cols / 4), reinterpret_cast<float4*>(out), ld_out / 4, accumulate);
    ALIGNN_LAUNCH_CHECK("move_rows4_kernel");
    return ALIGNN_OK;
  }
  launch(scatter_rows_kernel, dim3(grid_for(rows * cols)), dim3(256), 0, s, in, ld_in, idx, rows, cols,
                     out, ld_out, accumulate);
  ALIGNN_LAUNCH_CHECK("scatter_rows_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_schedule_build(const int32_t* off_dst, int64_t n, int32_t heavy_threshold, int32_t xcds,
                                     int32_t chunk, int32_t* light, int32_t* err_flag, void* stream) {
  if (n < 0 || n > 0x7ffffffeLL || heavy_threshold < 1 || heavy_threshold > SCHED_MAX_THR || xcds < 1 ||
      xcds > SCHED_MAX_XCDS || chunk < 1) {
    set_error("schedule_build: bad arguments n=%lld threshold=%d xcds=%d chunk=%d", (long long)n, heavy_threshold,
              xcds, chunk);
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(schedule_build_kernel, dim3(1), dim3(64 * SCHED_WAVES), 0, s, off_dst, n, (int)heavy_threshold, (int)xcds, (int)chunk,
         light, err_flag);
  ALIGNN_LAUNCH_CHECK("schedule_build_kernel");
  return ALIGNN_OK;
}
