// lgconv.hip — attention kernels, version 3: one single-wave workgroup per target segment.
//
// Same contract and arithmetic as tconv.hip's fwd2 / bwd_dst2 (PyG 2.7.0 TransformerConv message +
// utils.softmax + aggregate; callers train.py:315 and :334), for D = 256 (four
// features per lane, lane l holds features 4l..4l+3, so head h owns lanes [16h/(H/4)...]) with
// materialised edge features F and no dF output (the deferred angle-encoder backward).  What
// changes is the schedule and the instruction stream:
//
//  * Work items are target segments in the order of the schedule's list, one per workgroup of ONE
//    wave.  The hardware dispatcher starts a wave as soon as any wave slot frees, so the list order
//    (descending in-degree = longest-processing-time first, ops.GraphCSR) is a dynamic LPT
//    schedule: on the B = 32 line graph (2,580 targets, in-degrees 11..132, 1,260 of them 132) the
//    makespan is ~one 132-edge segment, where four-target workgroups ran ~1.3 rounds.
//  * Edges are processed in groups of G = 4 (edge j of a group <-> 16-lane row j after the
//    transpose reduction, as in fwd2/bwd2).  NR groups are in flight: with NR = 2 the loads of
//    group g + 2 are issued as soon as group g's registers are consumed and have one whole group of
//    compute to land.
//  * Branch-free tails: edge indices past the segment end are clamped to its last edge (valid
//    rows, masked out of the arithmetic), so every group issues the same 12 loads.
//  * No SGPR spills: per-edge addresses are formed from scalar-loaded indices in a few SGPRs; the
//    uniform per-target values (score offsets, softmax stats) are kept row-replicated in VGPRs.
//  * Per-(edge, head) dropout multipliers: lanes < G*H hash (t, h) with the same counter hash as
//    fwd2/bwd2 (bitwise the same masks), every lane fetches its row's H values by ds_bpermute.
//  * XF (the line graph's edge features recomputed, not streamed): the edge features of the line
//    convs are the angle encoder's hidden layer f_t = relu(W1 x_t + b1) of 11 raw inputs
//    (train.py:358-364, :553-556).  Instead of reading the [T, 256] rows the angle encoder's first
//    Linear wrote (82-86 % of these kernels' HBM bytes), each group loads its 4 edges' raw inputs (48 B
//    each) and recomputes its lanes' 4 x 4 features on the matrix cores: v_mfma_f32_4x4x1f32 with
//    A = x[edge lane & 3][k] and B = W1[4 lane + m][k] leaves h[edge r][4 lane + m] in register r —
//    a k-ordered chain of fused multiply-adds, bitwise linear_smallk's fmaf chain (skinny.hip;
//    tools/probe/mfma441.hip: 0 mismatches in 204,800), then + b1, ReLU (and the bf16 rounding of
//    the bf16-storage path), exactly as linear_smallk stores them.  W1 stays in registers (44 per
//    lane); the matrix cores are otherwise idle in these kernels.
#include "common.h"
#include "vec.h"

namespace alignn {
namespace lg3 {

constexpr int G = 4;      // edges per group (one per 16-lane row)
constexpr int D = 256;    // hidden size of this kernel family (64 lanes x 4 features)
constexpr int VPL = 4;

// One edge's rows as 128-bit register tuples (k, v, f): as float[4] arrays the loop-carried copies
// of the two-group ring were not coalesced (v_mov at the latch, each waiting for its load).
typedef float f4 __attribute__((ext_vector_type(4)));
struct Edge {
  f4 k, v, f;
};
__device__ __forceinline__ f4 ld4(const float* __restrict__ p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ float dot4(const float (&a)[VPL], f4 b) {
  return fmaf(a[3], b.w, fmaf(a[2], b.z, fmaf(a[1], b.y, a[0] * b.x)));
}

// Packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of fp32 FMAs per instruction, the
// vector fp32 peak).  Every element goes through the same fmaf / multiply, in the same order, as
// the scalar code (a per-head pair of dot4 chains; axpy over feature pairs), so results are bitwise
// those of the scalar loops.  Node vectors of two heads h, h+1 sit interleaved in LDS so that one
// 16-byte read gives (v_h[i], v_h+1[i], v_h[i+1], v_h+1[i+1]).
#ifndef ALIGNN_LG3_PK
#define ALIGNN_LG3_PK 1
#endif
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void axpy_pk(float (&acc)[VPL], float a, f4 x) {
  const f2 aa = {a, a};
  f2 lo = {acc[0], acc[1]}, hi = {acc[2], acc[3]};
  lo = __builtin_elementwise_fma(aa, f2{x.x, x.y}, lo);
  hi = __builtin_elementwise_fma(aa, f2{x.z, x.w}, hi);
  acc[0] = lo.x; acc[1] = lo.y; acc[2] = hi.x; acc[3] = hi.y;
}
__device__ __forceinline__ void scale_pk(float (&acc)[VPL], float a) {
  const f2 aa = {a, a};
  f2 lo = f2{acc[0], acc[1]} * aa, hi = f2{acc[2], acc[3]} * aa;
  acc[0] = lo.x; acc[1] = lo.y; acc[2] = hi.x; acc[3] = hi.y;
}
// LDS slot of feature i (of this lane's four) of head h's node vector, paired layout (H even)
__device__ __forceinline__ int pk_slot(int h, int i, int lane) {
  return (((h >> 1) * 2 + (i >> 1)) * 64 + lane) * 4 + (i & 1) * 2 + (h & 1);
}
// (dot4(v_h, f) , dot4(v_h+1, f)) for the head pair whose interleaved vectors start at `pair`,
// then fmaf(mk, qk, .) per head
__device__ __forceinline__ f2 dot4_pair(const float* pair, int lane, f4 f, f2 mk, float qk) {
  const f4 A = *reinterpret_cast<const f4*>(pair + lane * 4);
  const f4 B = *reinterpret_cast<const f4*>(pair + (64 + lane) * 4);
  f2 acc = f2{A.x, A.y} * f2{f.x, f.x};
  acc = __builtin_elementwise_fma(f2{A.z, A.w}, f2{f.y, f.y}, acc);
  acc = __builtin_elementwise_fma(f2{B.x, B.y}, f2{f.z, f.z}, acc);
  acc = __builtin_elementwise_fma(f2{B.z, B.w}, f2{f.w, f.w}, acc);
  return __builtin_elementwise_fma(mk, f2{qk, qk}, acc);
}

// bf16 storage (config C3, the reference's autocast: Linear outputs in bf16, train.py:632-636): the
// gathered K/V rows and the streamed edge-feature rows are bf16 in HBM (four per lane = one 8-byte
// load per row), widened to fp32 where a group is consumed; all arithmetic stays fp32.
typedef unsigned u2v __attribute__((ext_vector_type(2)));
struct EdgeH {
  u2v k, v, f;
};
__device__ __forceinline__ f4 widen(u2v u) {  // bf16 -> fp32 is exact: the bf16 bits become the top half
  f4 r;
  r.x = __builtin_bit_cast(float, u.x << 16);
  r.y = __builtin_bit_cast(float, u.x & 0xffff0000u);
  r.z = __builtin_bit_cast(float, u.y << 16);
  r.w = __builtin_bit_cast(float, u.y & 0xffff0000u);
  return r;
}
template <bool BF> struct RingT { using type = Edge; };
template <> struct RingT<true> { using type = EdgeH; };
// A group's rows as fp32 where it is consumed (widening at the consumer keeps the loads' wait there)
template <bool BF, bool XF = false>
__device__ __forceinline__ void to_f32(const typename RingT<BF>::type (&r)[G], Edge (&e)[G]) {
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if constexpr (BF) {
      e[j].k = widen(r[j].k);
      e[j].v = widen(r[j].v);
      if constexpr (!XF) e[j].f = widen(r[j].f);
    } else if constexpr (XF) {
      e[j].k = r[j].k;
      e[j].v = r[j].v;
    } else {
      e[j] = r[j];
    }
  }
}

// XF: the raw angle inputs of the lane's edge (group edge lane & 3), 12 floats (11 used + pad)
constexpr int KX = 11;    // raw angle inputs per triplet (lg_edge_attr width, SURVEY §8: F_a = 11)
constexpr int KXP = 12;   // row of the cache's padded copy (48 B: three 16-byte loads)
struct XRow {
  f4 a, b, c;
};
// The angle encoder's weights of this lane's four features (registers for the whole kernel)
struct W1Regs {
  float w[VPL][KX];
  float b[VPL];
};
__device__ __forceinline__ void load_w1(const float* __restrict__ W1, const float* __restrict__ b1, int j0, W1Regs& W) {
#pragma unroll
  for (int m = 0; m < VPL; ++m) {
#pragma unroll
    for (int k = 0; k < KX; ++k) W.w[m][k] = W1[(j0 + m) * KX + k];
    W.b[m] = b1[j0 + m];
  }
}
// f rows of the group's four edges for this lane's four features: relu(W1 x + b1) on the matrix
// cores (see the header), rounded to bf16 and widened back on the bf16-storage path (BF)
typedef float v4f __attribute__((ext_vector_type(4)));
template <bool BF>
__device__ __forceinline__ void angle_rows(const XRow& xr, const W1Regs& W, Edge (&e)[G]) {
  // the row's 12th float (padding) is loaded with the others but unused: this use keeps its register
  // allocated until here — else the allocator reuses it while the load is in flight, and the write
  // after write waits with vmcnt(0) for every load issued, the next group's prefetch included
  asm volatile("" ::"v"(xr.c.w));
  const float xs[KXP] = {xr.a.x, xr.a.y, xr.a.z, xr.a.w, xr.b.x, xr.b.y, xr.b.z, xr.b.w, xr.c.x, xr.c.y, xr.c.z, xr.c.w};
  v4f acc[VPL];
#pragma unroll
  for (int m = 0; m < VPL; ++m) {
    acc[m] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KX; ++k) acc[m] = __builtin_amdgcn_mfma_f32_4x4x1f32(xs[k], W.w[m][k], acc[m], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    float f[VPL];
#pragma unroll
    for (int m = 0; m < VPL; ++m) {
      f[m] = fmaxf(acc[m][j] + W.b[m], 0.f);
      if constexpr (BF) f[m] = (float)(__bf16)f[m];
    }
    e[j].f = f4{f[0], f[1], f[2], f[3]};
  }
}

struct Params {
  int64_t n, m;
  const int32_t* off;
  const int32_t* src_at;
  const int32_t* items;   // work list: target ids (one wave each), n_items entries
  int64_t n_items;
  const float* QKV; int64_t ldq;  // Q at col 0, K at D, V at 2D
  const float* U;                 // [n, H, D]
  const float* Vd;                // [n, H, D] (backward)
  const float* wbar;              // [D] or null
  const float* F; int64_t ldf;    // edge-feature rows, row of edge position t is t
  // bf16 storage (BF kernels): K|V rows [n, ldkv] (K at col 0, V at D) and edge-feature rows (ldf)
  const uint16_t* KV16; int64_t ldkv; const uint16_t* F16;
  // XF: raw angle inputs [m, ldx = 12] (target-sorted, 11 used), W1 [256, 11], b1 [256]
  const float* X; int64_t ldx; const float* W1; const float* b1;
  // forward outputs
  float* aggV; float* S; float* sumA; float* mstat; float* den;
  // backward inputs / outputs
  const float* dout; const float* outp; const float* mstat_in; const float* den_in;
  float* dq; int64_t lddq; float* Sz; float* sigz; float* dz_e; float* alpha_e;
  DropParams drop;
};

// The group's four source ids.  One scalar load of src_at[t0..t0+3] when that lies inside the array:
// entries past the segment's last edge are the next segment's sources — valid rows, and those edges
// are masked out of the arithmetic.  Loading them one by one, clamped, compiled to four dependent
// s_load / s_waitcnt round trips per group on the wave's critical path.
typedef int i4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void group_src(const Params& p, int32_t t0, int32_t last, int32_t (&s)[G]) {
  if ((int64_t)t0 + G <= p.m) {
    const i4u v = *((const __attribute__((address_space(4))) i4u*)(p.src_at + t0));
    s[0] = v.x; s[1] = v.y; s[2] = v.z; s[3] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j) s[j] = sld(p.src_at, min(t0 + j, last));
  }
}

// Loads of one group: edges t0..t0+3, clamped to `last` (the segment's last edge position).
template <bool BF, bool XF = false>
__device__ __forceinline__ void load_group(typename RingT<BF>::type (&r)[G], XRow& xr, const Params& p, int32_t t0,
                                           int32_t last, int j0) {
  int32_t sg[G];
  group_src(p, t0, last, sg);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int32_t t = min(t0 + j, last);
    const int64_t s = (int64_t)uni(sg[j]);
    if constexpr (BF) {
      const uint16_t* kv = p.KV16 + s * p.ldkv + j0;
      r[j].k = *reinterpret_cast<const u2v*>(kv);
      r[j].v = *reinterpret_cast<const u2v*>(kv + D);
      if constexpr (!XF) r[j].f = *reinterpret_cast<const u2v*>(p.F16 + (int64_t)t * p.ldf + j0);
    } else {
      const float* kv = p.QKV + s * p.ldq + D + j0;
      r[j].k = ld4(kv);
      r[j].v = ld4(kv + D);
      if constexpr (!XF) r[j].f = ld4(p.F + (int64_t)t * p.ldf + j0);
    }
  }
  if constexpr (XF) {   // the raw inputs of edge t0 + (lane & 3) (clamped like the rows above)
    const float* row = p.X + (int64_t)min(t0 + (int32_t)(threadIdx.x & 3), last) * p.ldx;
    xr.a = ld4(row);
    xr.b = ld4(row + 4);
    xr.c = ld4(row + 8);
  }
  // Pin the loads here: without this the compiler sinks them to their first use (one iteration
  // later, right behind their wait), which removes the prefetch (seen in the ISA of the 2-group loop:
  // the loop head waited vmcnt(0) on the group whose loads had just been issued).
  asm volatile("" ::: "memory");
}

// Dropout multiplier of (edge t0 + row, head h) for every lane (row = lane >> 4): lanes < G*H hash
// (t0 + lane / H, lane % H) exactly as group_dropout in tconv.hip does, then a bpermute per head.
template <int H, bool DROP>
__device__ __forceinline__ void drop_muls(const DropParams& dp, int32_t t0, int lane, float (&mul)[H]) {
  if constexpr (!DROP) {
#pragma unroll
    for (int h = 0; h < H; ++h) mul[h] = 1.0f;
  } else {
    const int src = lane < G * H ? lane : 0;
    const float mine = dropout_mul(dp.seed, (uint64_t)(t0 + src / H) * H + (src % H), dp.thresh, dp.inv_keep);
    const int row = lane >> 4;
#pragma unroll
    for (int h = 0; h < H; ++h) mul[h] = __shfl(mine, row * H + h, 64);
  }
}

// Sum over the four 16-lane rows of a row-replicated value (every lane gets the sum).
__device__ __forceinline__ float rows_sum4(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(u_bits(x), u_bits(x), false, false);
  x = f_bits(r[0]) + f_bits(r[1]);
  r = __builtin_amdgcn_permlane16_swap(u_bits(x), u_bits(x), false, false);
  return f_bits(r[0]) + f_bits(r[1]);
}
__device__ __forceinline__ float rows_max4(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(u_bits(x), u_bits(x), false, false);
  x = fmaxf(f_bits(r[0]), f_bits(r[1]));
  r = __builtin_amdgcn_permlane16_swap(u_bits(x), u_bits(x), false, false);
  return fmaxf(f_bits(r[0]), f_bits(r[1]));
}

// Group maxima of four row-distributed per-head values (row j = edge j): the transpose-reduction
// pattern (two value pairs per lane swap) instead of four separate row reductions, which each copy
// their operand twice for the in-place swaps.  Head h's maximum over the four rows ends in row h;
// returned as wave-uniform values.  Exact (max).
__device__ __forceinline__ void group_max4(const float (&z)[4], float (&g)[4]) {
  auto a = __builtin_amdgcn_permlane32_swap(u_bits(z[0]), u_bits(z[2]), false, false);
  const float t0 = fmaxf(f_bits(a[0]), f_bits(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(u_bits(z[1]), u_bits(z[3]), false, false);
  const float t1 = fmaxf(f_bits(b[0]), f_bits(b[1]));
  auto c = __builtin_amdgcn_permlane16_swap(u_bits(t0), u_bits(t1), false, false);
  const float u = fmaxf(f_bits(c[0]), f_bits(c[1]));
#pragma unroll
  for (int h = 0; h < 4; ++h) g[h] = readlane_f(u, 16 * h);
}

// Transpose-reduction (tconv.hip reduce_rows): value r*(N/4)+i ends in row r of b[i].
template <int N>
__device__ __forceinline__ void reduce_rows(const float (&v)[N], float (&b)[N / 4]) {
  static_assert(N % 4 == 0, "reduce_rows: N must be a multiple of 4");
  float a[N / 2];
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(u_bits(v[i]), u_bits(v[i + N / 2]), false, false);
    a[i] = f_bits(r[0]) + f_bits(r[1]);
  }
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(u_bits(a[i]), u_bits(a[i + N / 4]), false, false);
    b[i] = row_sum16(f_bits(r[0]) + f_bits(r[1]));
  }
}

// Lane's own-head entry of a per-head array: a select chain over values laundered through an
// empty asm (vec.h pick_r).  A plain select chain is folded into a dynamically indexed access of
// the array, which the compiler promoted to LDS (ds_write + indexed ds_read + lgkmcnt(0) in the
// edge loop, 8 KB of LDS per wave in the forward).
template <int H>
__device__ __forceinline__ float own(const float (&e)[H], int hl) {
  return pick_r<H>(e, hl);
}

// Lane's own-head entry of per-head wave-uniform values, as sum_h e[h] * mk[h] (mk = the lane's
// one-hot head mask): exact for finite e (one product is e[hl] * 1, the others 0) and branch-free —
// own() over uniform values compiled to one exec-masked branch per head inside the edge loop.
template <int H>
__device__ __forceinline__ float sel_head(const float (&e)[H], const float (&mk)[H]) {
  float r = e[0] * mk[0];
#pragma unroll
  for (int h = 1; h < H; ++h) r = fmaf(e[h], mk[h], r);
  return r;
}

// Per-edge-head output rows [t, H] written by the first lanes of each 16-lane row.
template <int H>
__device__ __forceinline__ void store_edge_heads(float* __restrict__ out, int64_t t, int col, const float (&b)[H]) {
  if constexpr (H % 4 == 0) {
    if (col < H / 4) {
      float4 w;
      w.x = b[0]; w.y = b[1]; w.z = b[2]; w.w = b[3];
#pragma unroll
      for (int q = 1; q < H / 4; ++q)
        if (col == q) { w.x = b[4 * q]; w.y = b[4 * q + 1]; w.z = b[4 * q + 2]; w.w = b[4 * q + 3]; }
      *reinterpret_cast<float4*>(out + t * H + 4 * col) = w;
    }
  } else {
    if (col < H) out[t * H + col] = own<H>(b, col);
  }
}

#ifndef ALIGNN_LG3_WPE1
#define ALIGNN_LG3_WPE1 3
#endif
#ifndef ALIGNN_LG3_WPE2
#define ALIGNN_LG3_WPE2 2
#endif
// bf16 rows at C3 size (2,027,520 edges over 16,020 targets; tools/lgm_bench.py, variants built
// with these macros): one group in flight and more waves beat the four-group ring — forward
// 438 -> 391 us at 3 waves/SIMD, 377 us at 4; target-side backward 497 -> 478 us at 3 (at 4 its
// registers spill: 635 us).  The fp32 kernels keep two groups at 2 waves/SIMD (B = 32 sweeps).
#ifndef ALIGNN_LG3_WPE_BF_FWD
#define ALIGNN_LG3_WPE_BF_FWD 4
#endif
#ifndef ALIGNN_LG3_WPE_BF_BWD
#define ALIGNN_LG3_WPE_BF_BWD 3
#endif
// XF with bf16 K|V: the 44 W1 registers do not fit the 4 / 3 waves of the streamed-row kernels
#ifndef ALIGNN_LG3_WPE_BF_XF
#define ALIGNN_LG3_WPE_BF_XF 2
#endif
template <int NR, bool BF = false, bool FWD = true, bool XF = false>
struct Occ {
  static constexpr int wpe = XF ? (BF ? ALIGNN_LG3_WPE_BF_XF : 2)
                                : (BF && NR == 1 ? (FWD ? ALIGNN_LG3_WPE_BF_FWD : ALIGNN_LG3_WPE_BF_BWD)
                                                 : (NR == 1 ? ALIGNN_LG3_WPE1 : ALIGNN_LG3_WPE2));
};

// Four groups in flight (bf16 rows: a group's loads take half the registers of fp32, so four cost
// what two do in fp32): fixed register names r0..r3, each refilled four groups ahead right after it
// is consumed; an exit check after every group (the loads already issued are simply not waited
// for), so a segment runs no fully masked groups beyond its last.  ra arrives holding group 0.
#define ALIGNN_LG3_RING4_BODY(LOAD, GRP)                                                   \
  do {                                                                                   \
    R r1[G], r2[G], r3[G];                                                               \
    LOAD(r1, beg + G);                                                                   \
    LOAD(r2, beg + 2 * G);                                                               \
    LOAD(r3, beg + 3 * G);                                                               \
    for (int32_t tb = beg;; tb += 4 * G) {                                               \
      GRP(ra, tb);                                                                       \
      LOAD(ra, tb + 4 * G);                                                              \
      if (tb + G >= end) break;                                                          \
      GRP(r1, tb + G);                                                                   \
      LOAD(r1, tb + 5 * G);                                                              \
      if (tb + 2 * G >= end) break;                                                      \
      GRP(r2, tb + 2 * G);                                                               \
      LOAD(r2, tb + 6 * G);                                                              \
      if (tb + 3 * G >= end) break;                                                      \
      GRP(r3, tb + 3 * G);                                                               \
      LOAD(r3, tb + 7 * G);                                                              \
      if (tb + 4 * G >= end) break;                                                      \
    }                                                                                    \
  } while (0)

// =============================================================================================
// Forward: aggV = sum alpha' V_src, S[h] = sum alpha'_h f_t (normalised), sumA, mstat, den
// =============================================================================================
template <int H, int NR, bool DROP>
__device__ __forceinline__ void fwd_group(const Params& p, const Edge (&r)[G], const float* uv, int32_t tb,
                                          int32_t end, int lane, int hl, int j0, float scale, const float (&q)[VPL],
                                          const float (&mk)[H], const float (&c)[H], float (&m)[H],
                                          float (&s_row)[H], float (&sa_row)[H], float (&accS)[H][VPL],
                                          float (&accV)[VPL]) {
  constexpr int RS = 64 * VPL;
  const int row = lane >> 4;
  asm volatile("" ::: "memory");  // keep the u reads in the loop (re-read from LDS, not held in VGPRs)
  float b[H];
  {
    float ps[G * H], qk[G];
#pragma unroll
    for (int j = 0; j < G; ++j) qk[j] = dot4(q, r[j].k);
    if constexpr (ALIGNN_LG3_PK && H % 2 == 0) {
#pragma unroll
      for (int hp = 0; hp < H / 2; ++hp) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const f2 v = dot4_pair(uv + hp * 2 * RS, lane, r[j].f, f2{mk[2 * hp], mk[2 * hp + 1]}, qk[j]);
          ps[j * H + 2 * hp] = v.x;
          ps[j * H + 2 * hp + 1] = v.y;
        }
      }
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float u[VPL];
        vload(uv + h * RS + j0, u);
#pragma unroll
        for (int j = 0; j < G; ++j) ps[j * H + h] = fmaf(mk[h], qk[j], dot4(u, r[j].f));
      }
    }
    reduce_rows<G * H>(ps, b);  // row j: b[h] = score partial of (edge tb + j, head h)
  }
  const bool rv = tb + row < end;
  float mul[H];
  drop_muls<H, DROP>(p.drop, tb, lane, mul);
  float z[H];
  bool grow = false;
  float mn[H];
  if constexpr (ALIGNN_LG3_PK && H == 4) {
    float gm[4];
#pragma unroll
    for (int h = 0; h < H; ++h) z[h] = rv ? (b[h] + c[h]) * scale : -INFINITY;
    group_max4(z, gm);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      mn[h] = fmaxf(m[h], gm[h]);
      grow |= mn[h] != m[h];
    }
  } else {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      z[h] = rv ? (b[h] + c[h]) * scale : -INFINITY;
      mn[h] = fmaxf(m[h], rows_max4(z[h]));
      grow |= mn[h] != m[h];
    }
  }
  if (grow) {  // wave-uniform: rescale only when some running maximum moved
    float corr[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      corr[h] = __expf(m[h] - mn[h]);
      m[h] = mn[h];
      s_row[h] *= corr[h];
      sa_row[h] *= corr[h];
      if constexpr (ALIGNN_LG3_PK) {
        scale_pk(accS[h], corr[h]);
      } else {
#pragma unroll
        for (int i = 0; i < VPL; ++i) accS[h][i] *= corr[h];
      }
    }
    const float cl = ALIGNN_LG3_PK ? sel_head<H>(corr, mk) : own<H>(corr, hl);
    if constexpr (ALIGNN_LG3_PK) {
      scale_pk(accV, cl);
    } else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) accV[i] *= cl;
    }
  }
  float ed[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float ex = __expf(z[h] - m[h]);  // 0 on rows past the segment end
    s_row[h] += ex;
    ed[h] = ex * mul[h];
    sa_row[h] += ed[h];
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    float e[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      e[h] = readlane_f(ed[h], 16 * j);
      if constexpr (ALIGNN_LG3_PK) {
        axpy_pk(accS[h], e[h], r[j].f);
      } else {
#pragma unroll
        for (int i = 0; i < VPL; ++i) accS[h][i] = fmaf(e[h], r[j].f[i], accS[h][i]);
      }
    }
    const float el = ALIGNN_LG3_PK ? sel_head<H>(e, mk) : own<H>(e, hl);
    if constexpr (ALIGNN_LG3_PK) {
      axpy_pk(accV, el, r[j].v);
    } else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) accV[i] = fmaf(el, r[j].v[i], accV[i]);
    }
  }
}

template <int H, int NR, bool DROP, bool BF, bool XF>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(Occ<NR, BF, true, XF>::wpe,
                                                                    Occ<NR, BF, true, XF>::wpe)))
void lg3_fwd_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  constexpr int C = D / H;
  constexpr int RS = 64 * VPL;
  __shared__ float uv[H * RS];  // u[h] of this wave's target
  const int lane = threadIdx.x;
  const int j0 = lane * VPL;
  const int hl = j0 / C;
  const float scale = 1.0f / sqrtf((float)C);
  const int64_t d = (int64_t)uni(sld(p.items, (int64_t)blockIdx.x));
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));

  float mk[H];
#pragma unroll
  for (int h = 0; h < H; ++h) mk[h] = (h == hl) ? 1.0f : 0.0f;
  float accS[H][VPL], accV[VPL], m[H], s_row[H], sa_row[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    m[h] = -INFINITY;
    s_row[h] = 0.f;
    sa_row[h] = 0.f;
    vzero(accS[h]);
  }
  vzero(accV);

  if (beg < end) {
    float q[VPL], c[H];
    vload(p.QKV + d * p.ldq + j0, q);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float t[VPL];
      vload(p.U + (d * H + h) * D + j0, t);
      if constexpr (ALIGNN_LG3_PK && H % 2 == 0) {
#pragma unroll
        for (int i = 0; i < VPL; ++i) uv[pk_slot(h, i, lane)] = t[i];
      } else {
        vstore(uv + h * RS + j0, t);
      }
    }
#pragma unroll
    for (int h = 0; h < H; ++h) c[h] = 0.f;
    if (p.wbar) {
      float wb[VPL];
      vload(p.wbar + j0, wb);
      const float part = vdot(wb, q);
#pragma unroll
      for (int h = 0; h < H; ++h) c[h] = (h == hl) ? part : 0.f;
      reduce_bcast<H>(c, lane);
    }
    W1Regs W;
    if constexpr (XF) load_w1(p.W1, p.b1, j0, W);
    __syncthreads();  // one wave: orders the LDS stores before the loop's reads
    // Loads are issued unconditionally (indices past the segment clamp to its last edge): a load
    // under a condition becomes a phi whose register copy waits for it at the join.
    const int32_t last = end - 1;
    using R = typename RingT<BF>::type;
    R ra[G];
    XRow xa;
    load_group<BF, XF>(ra, xa, p, beg, last, j0);
    auto grp = [&](const R (&r)[G], const XRow& xr, int32_t t) {
      Edge e[G];
      to_f32<BF, XF>(r, e);
      if constexpr (XF) angle_rows<BF>(xr, W, e);
      fwd_group<H, NR, DROP>(p, e, uv, t, end, lane, hl, j0, scale, q, mk, c, m, s_row, sa_row, accS, accV);
    };
    if constexpr (NR == 1) {
      for (int32_t tb = beg;; tb += G) {
        grp(ra, xa, tb);
        if (tb + G >= end) break;
        load_group<BF, XF>(ra, xa, p, tb + G, last, j0);
      }
    } else if constexpr (NR == 4) {
      static_assert(!XF, "the four-group ring streams the edge-feature rows");
      auto ld = [&](R (&r)[G], int32_t t) { load_group<BF>(r, xa, p, t, last, j0); };
      auto g4 = [&](const R (&r)[G], int32_t t) { grp(r, xa, t); };
      ALIGNN_LG3_RING4_BODY(ld, g4);
    } else {
      // one exit: pairs of groups (an odd count ends with a fully masked group, exactly 0)
      R rb[G];
      XRow xb;
      load_group<BF, XF>(rb, xb, p, beg + G, last, j0);
      const int32_t pairs = (end - beg + 2 * G - 1) / (2 * G);
      int32_t tb = beg;
      for (int32_t it = 0; it < pairs; ++it, tb += 2 * G) {
        grp(ra, xa, tb);
        load_group<BF, XF>(ra, xa, p, tb + 2 * G, last, j0);
        grp(rb, xb, tb + G);
        load_group<BF, XF>(rb, xb, p, tb + 3 * G, last, j0);
      }
    }
  }
  float inv[H], dn[H], sa[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    dn[h] = rows_sum4(s_row[h]) + 1e-16f;
    inv[h] = 1.0f / dn[h];
    sa[h] = rows_sum4(sa_row[h]);
  }
#pragma unroll
  for (int h = 0; h < H; ++h) {
    float o[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) o[i] = accS[h][i] * inv[h];
    vstore(p.S + (d * H + h) * D + j0, o);
  }
  {
    const float il = own<H>(inv, hl);
    float o[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) o[i] = accV[i] * il;
    vstore(p.aggV + d * D + j0, o);
  }
  if (lane < H) {
    p.sumA[d * H + lane] = own<H>(sa, lane) * own<H>(inv, lane);
    p.mstat[d * H + lane] = own<H>(m, lane);
    p.den[d * H + lane] = own<H>(dn, lane);
  }
}

// =============================================================================================
// Backward, target side: dq, Sz, sigz per target; dz_e, alpha_e per edge (no dF)
// =============================================================================================
template <int H, int NR, bool DROP>
__device__ __forceinline__ void bwd_group(const Params& p, const Edge (&r)[G], const float* uv, int32_t tb,
                                          int32_t end, int lane, int hl, int j0, float scale,
                                          const float (&q)[VPL], const float (&go)[VPL], const float (&mk)[H],
                                          const float (&c)[3 * H], const float (&mst)[H],
                                          const float (&inv_den)[H], float (&sgz_row)[H], float (&sz)[H][VPL],
                                          float (&dqa)[VPL]) {
  constexpr int RS = 64 * VPL;
  const int row = lane >> 4;
  asm volatile("" ::: "memory");  // keep the u / Vd reads in the loop
  float bs[H], bd[H];
  {
    float ps[G * H], pd[G * H];
    float qk[G], gv[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      qk[j] = dot4(q, r[j].k);
      gv[j] = dot4(go, r[j].v);
    }
    if constexpr (ALIGNN_LG3_PK && H % 2 == 0) {
#pragma unroll
      for (int hp = 0; hp < H / 2; ++hp) {
        const f2 mk2 = {mk[2 * hp], mk[2 * hp + 1]};
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const f2 a = dot4_pair(uv + hp * 2 * RS, lane, r[j].f, mk2, qk[j]);
          const f2 b = dot4_pair(uv + (H + 2 * hp) * RS, lane, r[j].f, mk2, gv[j]);
          ps[j * H + 2 * hp] = a.x;
          ps[j * H + 2 * hp + 1] = a.y;
          pd[j * H + 2 * hp] = b.x;
          pd[j * H + 2 * hp + 1] = b.y;
        }
      }
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float u[VPL], vd[VPL];
        vload(uv + h * RS + j0, u);
        vload(uv + (H + h) * RS + j0, vd);
#pragma unroll
        for (int j = 0; j < G; ++j) {
          ps[j * H + h] = fmaf(mk[h], qk[j], dot4(u, r[j].f));
          pd[j * H + h] = fmaf(mk[h], gv[j], dot4(vd, r[j].f));
        }
      }
    }
    reduce_rows<G * H>(ps, bs);
    reduce_rows<G * H>(pd, bd);
  }
  const bool rv = tb + row < end;
  float mul[H];
  drop_muls<H, DROP>(p.drop, tb, lane, mul);
  // row-distributed dz (= dL/dz / sqrt(C)) in bs, alpha' in bd
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float z = (bs[h] + c[h]) * scale;
    const float alpha = __expf(z - mst[h]) * inv_den[h];
    const float al = alpha * mul[h];
    const float dal = (bd[h] + c[H + h]) * mul[h];
    const float dz = alpha * (dal - c[2 * H + h]) * scale;
    bs[h] = rv ? dz : 0.f;
    bd[h] = rv ? al : 0.f;
    sgz_row[h] += bs[h];
  }
  {
    const int col = lane & 15;
    if (rv) {
      const int64_t t = (int64_t)(tb + row);
      store_edge_heads<H>(p.dz_e, t, col, bs);
      store_edge_heads<H>(p.alpha_e, t, col, bd);
    }
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    float e[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      e[h] = readlane_f(bs[h], 16 * j);
      if constexpr (ALIGNN_LG3_PK) {
        axpy_pk(sz[h], e[h], r[j].f);
      } else {
#pragma unroll
        for (int i = 0; i < VPL; ++i) sz[h][i] = fmaf(e[h], r[j].f[i], sz[h][i]);
      }
    }
    const float dzl = ALIGNN_LG3_PK ? sel_head<H>(e, mk) : own<H>(e, hl);
    if constexpr (ALIGNN_LG3_PK) {
      axpy_pk(dqa, dzl, r[j].k);
    } else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) dqa[i] = fmaf(dzl, r[j].k[i], dqa[i]);
    }
  }
}

template <int H, int NR, bool DROP, bool BF, bool XF>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(Occ<NR, BF, false, XF>::wpe,
                                                                    Occ<NR, BF, false, XF>::wpe)))
void lg3_bwd_dst_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  constexpr int C = D / H;
  constexpr int RS = 64 * VPL;
  __shared__ float uv[2 * H * RS];  // u[h] (h < H), Vd[h] (H + h) of this wave's target
  const int lane = threadIdx.x;
  const int j0 = lane * VPL;
  const int hl = j0 / C;
  const float scale = 1.0f / sqrtf((float)C);
  const int64_t d = (int64_t)uni(sld(p.items, (int64_t)blockIdx.x));
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));

  float mk[H];
#pragma unroll
  for (int h = 0; h < H; ++h) mk[h] = (h == hl) ? 1.0f : 0.0f;
  float sz[H][VPL], sgz_row[H], dqa[VPL];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    vzero(sz[h]);
    sgz_row[h] = 0.f;
  }
  vzero(dqa);

  if (beg < end) {
    float q[VPL], go[VPL], c[3 * H], mst[H], inv_den[H];
    {
      float op[VPL], wb[VPL];
      vload(p.QKV + d * p.ldq + j0, q);
      vload(p.dout + d * D + j0, go);
      vload(p.outp + d * D + j0, op);
      vzero(wb);
      if (p.wbar) vload(p.wbar + j0, wb);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float t[VPL], w[VPL];
        vload(p.U + (d * H + h) * D + j0, t);
        vload(p.Vd + (d * H + h) * D + j0, w);
        if constexpr (ALIGNN_LG3_PK && H % 2 == 0) {
#pragma unroll
          for (int i = 0; i < VPL; ++i) {
            uv[pk_slot(h, i, lane)] = t[i];
            uv[H * RS + pk_slot(h, i, lane)] = w[i];
          }
        } else {
          vstore(uv + h * RS + j0, t);
          vstore(uv + (H + h) * RS + j0, w);
        }
      }
      const float pc = vdot(wb, q), pc2 = vdot(wb, go), pdl = vdot(go, op);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        c[h] = (h == hl) ? pc : 0.f;
        c[H + h] = (h == hl) ? pc2 : 0.f;
        c[2 * H + h] = (h == hl) ? pdl : 0.f;
      }
      reduce_bcast<3 * H>(c, lane);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        mst[h] = readlane_f(p.mstat_in[d * H + (lane % H)], h);
        inv_den[h] = 1.0f / readlane_f(p.den_in[d * H + (lane % H)], h);
      }
    }
    W1Regs W;
    if constexpr (XF) load_w1(p.W1, p.b1, j0, W);
    __syncthreads();  // one wave: orders the LDS stores before the loop's reads
    const int32_t last = end - 1;  // unconditional loads, clamped indices (see lg3_fwd_kernel)
    using R = typename RingT<BF>::type;
    R ra[G];
    XRow xa;
    load_group<BF, XF>(ra, xa, p, beg, last, j0);
    auto grp = [&](const R (&r)[G], const XRow& xr, int32_t t) {
      Edge e[G];
      to_f32<BF, XF>(r, e);
      if constexpr (XF) angle_rows<BF>(xr, W, e);
      bwd_group<H, NR, DROP>(p, e, uv, t, end, lane, hl, j0, scale, q, go, mk, c, mst, inv_den, sgz_row, sz, dqa);
    };
    if constexpr (NR == 1) {
      for (int32_t tb = beg;; tb += G) {
        grp(ra, xa, tb);
        if (tb + G >= end) break;
        load_group<BF, XF>(ra, xa, p, tb + G, last, j0);
      }
    } else if constexpr (NR == 4) {
      static_assert(!XF, "the four-group ring streams the edge-feature rows");
      auto ld = [&](R (&r)[G], int32_t t) { load_group<BF>(r, xa, p, t, last, j0); };
      auto g4 = [&](const R (&r)[G], int32_t t) { grp(r, xa, t); };
      ALIGNN_LG3_RING4_BODY(ld, g4);
    } else {
      R rb[G];
      XRow xb;
      load_group<BF, XF>(rb, xb, p, beg + G, last, j0);
      const int32_t pairs = (end - beg + 2 * G - 1) / (2 * G);
      int32_t tb = beg;
      for (int32_t it = 0; it < pairs; ++it, tb += 2 * G) {
        grp(ra, xa, tb);
        load_group<BF, XF>(ra, xa, p, tb + 2 * G, last, j0);
        grp(rb, xb, tb + G);
        load_group<BF, XF>(rb, xb, p, tb + 3 * G, last, j0);
      }
    }
  }
  vstore(p.dq + d * p.lddq + j0, dqa);
#pragma unroll
  for (int h = 0; h < H; ++h) vstore(p.Sz + (d * H + h) * D + j0, sz[h]);
  float sg[H];
#pragma unroll
  for (int h = 0; h < H; ++h) sg[h] = rows_sum4(sgz_row[h]);
  if (lane < H) p.sigz[d * H + lane] = own<H>(sg, lane);
}

// ---------------------------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------------------------
// edge groups in flight per wave (1: 3 waves/SIMD, 2: 2 waves/SIMD)
#ifndef ALIGNN_LG3_NR_FWD
#define ALIGNN_LG3_NR_FWD 2
#endif
#ifndef ALIGNN_LG3_NR_BWD
#define ALIGNN_LG3_NR_BWD 2
#endif

// bf16 rows: groups in flight (1: measured best at C3 with Occ's wave counts; 4: the ring above)
#ifndef ALIGNN_LG3_NR_BF
#define ALIGNN_LG3_NR_BF 1
#endif
// XF: groups in flight (fp32 keeps the streamed-row kernels' 2; bf16 K|V: 1 or 2)
#ifndef ALIGNN_LG3_NR_BF_XF
#define ALIGNN_LG3_NR_BF_XF 1
#endif
template <int H, bool DROP, bool BF>
static void launch_fwd_h(const Params& p, hipStream_t s) {
  constexpr int NR = BF ? ALIGNN_LG3_NR_BF : ALIGNN_LG3_NR_FWD;
  launch((lg3_fwd_kernel<H, NR, DROP, BF, false>), dim3((unsigned)p.n_items), dim3(64), 0, s, p);
}
template <int H, bool DROP, bool BF>
static void launch_bwd_h(const Params& p, hipStream_t s) {
  constexpr int NR = BF ? ALIGNN_LG3_NR_BF : ALIGNN_LG3_NR_BWD;
  launch((lg3_bwd_dst_kernel<H, NR, DROP, BF, false>), dim3((unsigned)p.n_items), dim3(64), 0, s, p);
}
// XF (H = 4 only: the configuration of train.py's model, D = 256 / H = 4)
template <bool DROP, bool BF>
static void launch_fwd_x(const Params& p, hipStream_t s) {
  constexpr int NR = BF ? ALIGNN_LG3_NR_BF_XF : ALIGNN_LG3_NR_FWD;
  launch((lg3_fwd_kernel<4, NR, DROP, BF, true>), dim3((unsigned)p.n_items), dim3(64), 0, s, p);
}
// fp32 target-side backward with W1 in registers: two groups in flight spill (255 VGPRs), one fits
#ifndef ALIGNN_LG3_NR_BWD_XF
#define ALIGNN_LG3_NR_BWD_XF 1
#endif
template <bool DROP, bool BF>
static void launch_bwd_x(const Params& p, hipStream_t s) {
  constexpr int NR = BF ? ALIGNN_LG3_NR_BF_XF : ALIGNN_LG3_NR_BWD_XF;
  launch((lg3_bwd_dst_kernel<4, NR, DROP, BF, true>), dim3((unsigned)p.n_items), dim3(64), 0, s, p);
}

#define ALIGNN_LG3_DISPATCH_H(FN, H_, DROP_, BF_, ...)   \
  do {                                                   \
    if (H_ == 1) FN<1, DROP_, BF_>(__VA_ARGS__);         \
    else if (H_ == 2) FN<2, DROP_, BF_>(__VA_ARGS__);    \
    else FN<4, DROP_, BF_>(__VA_ARGS__);                 \
  } while (0)
#define ALIGNN_LG3_DISPATCH(FN, H_, DROP_, BF_, ...)                                        \
  do {                                                                                      \
    if (DROP_ && BF_) ALIGNN_LG3_DISPATCH_H(FN, H_, true, true, __VA_ARGS__);               \
    else if (DROP_) ALIGNN_LG3_DISPATCH_H(FN, H_, true, false, __VA_ARGS__);                \
    else if (BF_) ALIGNN_LG3_DISPATCH_H(FN, H_, false, true, __VA_ARGS__);                  \
    else ALIGNN_LG3_DISPATCH_H(FN, H_, false, false, __VA_ARGS__);                          \
  } while (0)

// fp32 -> bf16 (round to nearest even, v_cvt_pk_bf16_f32) of a [rows, cols] block, cols % 4 == 0;
// one thread per 4 columns.
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ src, int64_t lds, int64_t rows,
                                                        int64_t cols, uint16_t* __restrict__ dst, int64_t ldd) {
  const int64_t q = cols / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * q; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q, c = (i % q) * 4;
    const f4 v = ld4(src + r * lds + c);
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
    bf4 h;
    h.x = (__bf16)v.x; h.y = (__bf16)v.y; h.z = (__bf16)v.z; h.w = (__bf16)v.w;
    *reinterpret_cast<bf4*>(dst + r * ldd + c) = h;
  }
}

}  // namespace lg3

// The bf16 recompute kernels (matrix cores, lgmx.hip)
int lgm_fwd(int64_t n, int64_t m, const int32_t* off, const int32_t* src_at, const int32_t* items, int64_t n_items,
            const float* Q, int64_t ldq, const uint16_t* KV16, int64_t ldkv, const float* U, const float* wbar,
            const float* X, int64_t ldx, const float* W1, const float* b1, float* aggV, float* S, float* sumA,
            float* mstat, float* den, const DropParams& drop, hipStream_t s);
int lgm_bwd(int64_t n, int64_t m, const int32_t* off, const int32_t* src_at, const int32_t* items, int64_t n_items,
            const float* Q, int64_t ldq, const uint16_t* KV16, int64_t ldkv, const float* U, const float* Vd,
            const float* wbar, const float* X, int64_t ldx, const float* W1, const float* b1, const float* dout,
            const float* outp, const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz,
            float* dz_e, float* alpha_e, const DropParams& drop, hipStream_t s);

// Entry points used by tconv.hip's C ABI when the schedule asks for single-wave items
// (ALIGNN_SCHED_WAVE_ITEMS) and the call is in this family's domain (lg3_supported).
bool lg3_supported(int D, int H, const int32_t* feat_row, const float* F, const AlignnSchedule* sched) {
  // H = 8 spills at this register budget: it takes the compact-register kernels
  return D == lg3::D && (H == 1 || H == 2 || H == 4) && feat_row == nullptr && F != nullptr && sched != nullptr && (sched->flags & ALIGNN_SCHED_WAVE_ITEMS) && sched->n_heavy == 0 &&
         sched->light != nullptr;
}

int lg3_fwd(int64_t n, int64_t m, int H, const int32_t* off, const int32_t* src_at, const AlignnSchedule* sched,
            const float* QKV, int64_t ldq, const float* U, const float* wbar, const float* F, int64_t ldf,
            float* aggV, float* S, float* sumA, float* mstat, float* den, const DropParams& drop, hipStream_t s,
            const uint16_t* KV16 = nullptr, int64_t ldkv = 0, const uint16_t* F16 = nullptr) {
  lg3::Params p{};
  p.n = n; p.m = m; p.off = off; p.src_at = src_at; p.items = sched->light; p.n_items = sched->n_light;
  p.QKV = QKV; p.ldq = ldq; p.U = U; p.wbar = wbar; p.F = F; p.ldf = ldf;
  p.KV16 = KV16; p.ldkv = ldkv; p.F16 = F16;
  p.aggV = aggV; p.S = S; p.sumA = sumA; p.mstat = mstat; p.den = den;
  p.drop = drop;
  if (p.n_items <= 0) return ALIGNN_OK;
  ALIGNN_LG3_DISPATCH(lg3::launch_fwd_h, H, drop.active != 0, F16 != nullptr, p, s);
  ALIGNN_LAUNCH_CHECK("lg3_fwd_kernel");
  return ALIGNN_OK;
}

int lg3_bwd_dst(int64_t n, int64_t m, int H, const int32_t* off, const int32_t* src_at,
                const AlignnSchedule* sched, const float* QKV, int64_t ldq, const float* U, const float* Vd,
                const float* wbar, const float* F, int64_t ldf, const float* dout, const float* outp,
                const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e,
                float* alpha_e, const DropParams& drop, hipStream_t s, const uint16_t* KV16 = nullptr,
                int64_t ldkv = 0, const uint16_t* F16 = nullptr) {
  lg3::Params p{};
  p.n = n; p.m = m; p.off = off; p.src_at = src_at; p.items = sched->light; p.n_items = sched->n_light;
  p.QKV = QKV; p.ldq = ldq; p.U = U; p.Vd = Vd; p.wbar = wbar; p.F = F; p.ldf = ldf;
  p.KV16 = KV16; p.ldkv = ldkv; p.F16 = F16;
  p.dout = dout; p.outp = outp; p.mstat_in = mstat; p.den_in = den;
  p.dq = dq; p.lddq = lddq; p.Sz = Sz; p.sigz = sigz; p.dz_e = dz_e; p.alpha_e = alpha_e;
  p.drop = drop;
  if (p.n_items <= 0) return ALIGNN_OK;
  ALIGNN_LG3_DISPATCH(lg3::launch_bwd_h, H, drop.active != 0, F16 != nullptr, p, s);
  ALIGNN_LAUNCH_CHECK("lg3_bwd_dst_kernel");
  return ALIGNN_OK;
}

static bool aligned8(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 7u) == 0; }

// Shape checks of the bf16-storage entry points (host side, before any launch)
static int lg3_bf16_check(int64_t n, int32_t D, int32_t H, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                          const uint16_t* KV16, int64_t ldkv, const uint16_t* F16, int64_t ldf) {
  if (D != lg3::D || !(H == 1 || H == 2 || H == 4)) {
    set_error("lg bf16: needs hidden 256 and heads in {1, 2, 4} (got %d, %d)", (int)D, (int)H);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (!sched || !(sched->flags & ALIGNN_SCHED_WAVE_ITEMS) || sched->n_heavy != 0 || (n > 0 && !sched->light)) {
    set_error("lg bf16: needs an ALIGNN_SCHED_WAVE_ITEMS schedule listing every target (no heavy list)");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n > 0 && (!Q || !KV16 || !F16 || ldq < 3 * D || ldkv < 2 * D || ldf < D || ldkv % 4 || ldf % 4 ||
                !aligned8(KV16) || !aligned8(F16))) {
    set_error("lg bf16: Q (ldq >= 3D), K|V bf16 rows (ldkv >= 2D) and F bf16 rows (ldf >= D) with 8-byte aligned "
              "rows are required");
    return ALIGNN_E_BAD_SHAPE;
  }
  return ALIGNN_OK;
}

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_lg_fwd_bf16(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                  const int32_t* src_at, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                                  const uint16_t* KV16, int64_t ldkv, const float* U, const float* wbar,
                                  const uint16_t* F16, int64_t ldf, float* aggV, float* S, float* sumA, float* mstat,
                                  float* den, float drop_p, uint64_t seed, void* stream) {
  int rc = lg3_bf16_check(n, D, H, sched, Q, ldq, KV16, ldkv, F16, ldf);
  if (rc || n == 0) return rc;
  return lg3_fwd(n, m, H, off_dst, src_at, sched, Q, ldq, U, wbar, nullptr, ldf, aggV, S, sumA, mstat, den,
                 make_drop(drop_p, seed), reinterpret_cast<hipStream_t>(stream), KV16, ldkv, F16);
}

extern "C" int alignn_lg_bwd_dst_bf16(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                      const int32_t* src_at, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                                      const uint16_t* KV16, int64_t ldkv, const float* U, const float* Vd,
                                      const float* wbar, const uint16_t* F16, int64_t ldf, const float* dout,
                                      const float* outp, const float* mstat, const float* den, float* dq,
                                      int64_t lddq, float* Sz, float* sigz, float* dz_e, float* alpha_e, float drop_p,
                                      uint64_t seed, void* stream) {
  int rc = lg3_bf16_check(n, D, H, sched, Q, ldq, KV16, ldkv, F16, ldf);
  if (rc || n == 0) return rc;
  return lg3_bwd_dst(n, m, H, off_dst, src_at, sched, Q, ldq, U, Vd, wbar, nullptr, ldf, dout, outp, mstat, den, dq,
                     lddq, Sz, sigz, dz_e, alpha_e, make_drop(drop_p, seed), reinterpret_cast<hipStream_t>(stream),
                     KV16, ldkv, F16);
}

// Shape checks of the recompute (XF) entry points (host side, before any launch)
static int lgx_check(int64_t n, int32_t D, int32_t H, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                     const uint16_t* KV16, int64_t ldkv, const float* X, int64_t ldx, int32_t kin, const float* W1,
                     const float* b1) {
  if (D != lg3::D || H != 4 || kin != lg3::KX) {
    set_error("lg x: needs hidden 256, 4 heads and %d raw angle inputs (got %d, %d, %d)", lg3::KX, (int)D, (int)H,
              (int)kin);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (!sched || !(sched->flags & ALIGNN_SCHED_WAVE_ITEMS) || sched->n_heavy != 0 || (n > 0 && !sched->light)) {
    set_error("lg x: needs an ALIGNN_SCHED_WAVE_ITEMS schedule listing every target (no heavy list)");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n > 0 && (!Q || ldq < 3 * D || (KV16 && (ldkv < 2 * D || ldkv % 4 || !aligned8(KV16))))) {
    set_error("lg x: Q|K|V rows (ldq >= 3D) and, for bf16 storage, K|V bf16 rows (ldkv >= 2D, 8-byte aligned)");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n > 0 && (!X || ldx != lg3::KXP || (reinterpret_cast<uintptr_t>(X) & 15u) || !W1 || !b1)) {
    set_error("lg x: raw angle inputs as 16-byte aligned rows of %d floats (ldx = %lld), W1 [256, %d] and b1 required",
              lg3::KXP, (long long)ldx, lg3::KX);
    return ALIGNN_E_BAD_SHAPE;
  }
  return ALIGNN_OK;
}

extern "C" int alignn_lg_fwd_x(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                               const int32_t* src_at, const AlignnSchedule* sched, const float* QKV, int64_t ldq,
                               const uint16_t* KV16, int64_t ldkv, const float* U, const float* wbar, const float* X,
                               int64_t ldx, int32_t kin, const float* W1, const float* b1, float* aggV, float* S,
                               float* sumA, float* mstat, float* den, float drop_p, uint64_t seed, void* stream) {
  int rc = lgx_check(n, D, H, sched, QKV, ldq, KV16, ldkv, X, ldx, kin, W1, b1);
  if (rc || n == 0) return rc;
  lg3::Params p{};
  p.n = n; p.m = m; p.off = off_dst; p.src_at = src_at; p.items = sched->light; p.n_items = sched->n_light;
  p.QKV = QKV; p.ldq = ldq; p.U = U; p.wbar = wbar; p.KV16 = KV16; p.ldkv = ldkv;
  p.X = X; p.ldx = ldx; p.W1 = W1; p.b1 = b1;
  p.aggV = aggV; p.S = S; p.sumA = sumA; p.mstat = mstat; p.den = den;
  p.drop = make_drop(drop_p, seed);
  if (p.n_items <= 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (KV16)   // bf16 storage (config C3): the matrix-core kernels (lgmx.hip)
    return lgm_fwd(n, m, off_dst, src_at, p.items, p.n_items, QKV, ldq, KV16, ldkv, U, wbar, X, ldx, W1, b1, aggV, S,
                   sumA, mstat, den, p.drop, s);
  if (p.drop.active) lg3::launch_fwd_x<true, false>(p, s);
  else lg3::launch_fwd_x<false, false>(p, s);
  ALIGNN_LAUNCH_CHECK("lg3_fwd_kernel (x)");
  return ALIGNN_OK;
}

extern "C" int alignn_lg_bwd_dst_x(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                   const int32_t* src_at, const AlignnSchedule* sched, const float* QKV, int64_t ldq,
                                   const uint16_t* KV16, int64_t ldkv, const float* U, const float* Vd,
                                   const float* wbar, const float* X, int64_t ldx, int32_t kin, const float* W1,
                                   const float* b1, const float* dout, const float* outp, const float* mstat,
                                   const float* den, float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e,
                                   float* alpha_e, float drop_p, uint64_t seed, void* stream) {
  int rc = lgx_check(n, D, H, sched, QKV, ldq, KV16, ldkv, X, ldx, kin, W1, b1);
  if (rc || n == 0) return rc;
  lg3::Params p{};
  p.n = n; p.m = m; p.off = off_dst; p.src_at = src_at; p.items = sched->light; p.n_items = sched->n_light;
  p.QKV = QKV; p.ldq = ldq; p.U = U; p.Vd = Vd; p.wbar = wbar; p.KV16 = KV16; p.ldkv = ldkv;
  p.X = X; p.ldx = ldx; p.W1 = W1; p.b1 = b1;
  p.dout = dout; p.outp = outp; p.mstat_in = mstat; p.den_in = den;
  p.dq = dq; p.lddq = lddq; p.Sz = Sz; p.sigz = sigz; p.dz_e = dz_e; p.alpha_e = alpha_e;
  p.drop = make_drop(drop_p, seed);
  if (p.n_items <= 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (KV16)
    return lgm_bwd(n, m, off_dst, src_at, p.items, p.n_items, QKV, ldq, KV16, ldkv, U, Vd, wbar, X, ldx, W1, b1, dout,
                   outp, mstat, den, dq, lddq, Sz, sigz, dz_e, alpha_e, p.drop, s);
  if (p.drop.active) lg3::launch_bwd_x<true, false>(p, s);
  else lg3::launch_bwd_x<false, false>(p, s);
  ALIGNN_LAUNCH_CHECK("lg3_bwd_dst_kernel (x)");
  return ALIGNN_OK;
}

extern "C" int alignn_cast_bf16_f32(const float* src, int64_t lds, int64_t rows, int64_t cols, uint16_t* dst,
                                    int64_t ldd, void* stream) {
  if (rows < 0 || cols < 0 || cols % 4 || lds % 4 || ldd % 4 || lds < cols || ldd < cols ||
      (rows > 0 && cols > 0 && (!src || !dst || !aligned8(dst) || (reinterpret_cast<uintptr_t>(src) & 15u)))) {
    set_error("cast_bf16: cols and leading dimensions must be multiples of 4 with 16-byte aligned fp32 rows");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (rows == 0 || cols == 0) return ALIGNN_OK;
  const int64_t work = rows * (cols / 4);
  const unsigned blocks = (unsigned)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
  launch(lg3::cast_bf16_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), src, lds, rows,
         cols, dst, ldd);
  ALIGNN_LAUNCH_CHECK("cast_bf16_kernel");
  return ALIGNN_OK;
}
