// tconv.hip — fused TransformerConv attention over CSR segments (gfx950, wave64).
//
// Replaces PyG 2.7.0 TransformerConv.message + utils.softmax + aggregate('add'),
// called by EdgeUpdateBlock (train.py:315, line graph: nodes = bonds, edges = triplets) and
// NodeUpdateBlock (train.py:334, atom graph).  One wavefront owns one target segment and walks
// its in-edges with an online (running-max) softmax; VPL consecutive features per lane
// (D = 64*VPL, or fewer lanes active for D < 64).
//
// Edge-feature algebra: the reference projects every edge feature with lin_edge
// ([m, D] x [D, D]).  Here the score term <Q_dh, W_e,h f_t> is computed as <u_dh, f_t> with
// u_dh = M_h^T Q_dh (one n-row GEMM outside), and the message term sum_t alpha W_e,h f_t as
// M_h (sum_t alpha f_t) — so the per-edge work is D-wide dot products and axpys, and the m-row GEMM
// disappears.  M_h = W_e,h P and w̄ = W_e p fold the atom graph's edge_proj (P, p) in as well.
//
// Edge features are materialised rows F (the line graph: the angle encoder's hidden layer, its
// second Linear folded into M).  An in-kernel recompute of the hidden layer from the 11 raw angle
// inputs was measured slower (occupancy-bound) and removed in round 3.
#include "common.h"
#include "vec.h"

namespace alignn {

// ---------------------------------------------------------------------------------------------
// Work decomposition.  Work items: heavy target nodes (in-degree > threshold, one workgroup of
// four waves each; the waves take interleaved groups of PF edges and merge through LDS in fixed
// wave order), then light nodes four per workgroup (one wave each).  Heavy items come first so
// the long ones start early.  One workgroup per item.  Edges are processed in groups of PF: the
// operands of the next group are in flight while the current one computes, and the PF*H (or
// 2*PF*H) per-head dot products of a group are reduced across the wave together (reduce_bcast).
// ---------------------------------------------------------------------------------------------
#ifndef ALIGNN_PF
#define ALIGNN_PF 4
#endif
constexpr int PF = ALIGNN_PF;

struct Sched {
  const int32_t* light;
  int64_t n_light;
  const int32_t* heavy;
  int64_t n_heavy;
  __host__ __device__ int64_t items() const { return n_heavy + (n_light + 3) / 4; }
};

// The streamed edge rows of the _2 kernels.  FBF: the feature rows hold bf16 (config C3: the atom
// graph's edge features are the bond state as autocast casts it for edge_proj, train.py:325/:333
// under :632-636), widened exactly at use.  The feature row stays in its storage format (bf16
// pairs or fp32 bits) until the group is consumed, and nothing is computed from a row at its
// load: a value computed at the load (the bf16 widening) would put a wait for that load right
// behind it, and a value reaching a loop head through a phi makes the wait-count pass drain every
// load in flight (vmcnt(0)).  Lanes past D read column 0 (their q / u / Vd / dout are zero, so
// what they read never reaches a stored value) and callers clamp the edge index to the segment
// (rows past its end are masked out of the softmax and out of every store).
template <int VPL, bool FBF>
struct EdgeRow {
  float k[VPL], v[VPL];
  uint32_t fb[FBF ? (VPL + 1) / 2 : VPL];
  __device__ __forceinline__ void widen(float (&f)[VPL]) const {
#pragma unroll
    for (int i = 0; i < VPL; ++i)
      f[i] = FBF ? __builtin_bit_cast(float, (i & 1) ? (fb[i / 2] & 0xffff0000u) : (fb[i / 2] << 16))
                 : __builtin_bit_cast(float, fb[i]);
  }
};

template <int VPL, bool FBF>
__device__ __forceinline__ void load_row(EdgeRow<VPL, FBF>& e, const float* __restrict__ QKVR, int64_t ldq, int D,
                                         const float* __restrict__ F, int64_t ldf, int64_t src, int64_t row, int jc) {
  vload(QKVR + src * ldq + D + jc, e.k);
  vload(QKVR + src * ldq + 2 * D + jc, e.v);
  if constexpr (FBF) {
    const uint16_t* fp = reinterpret_cast<const uint16_t*>(F) + row * ldf + jc;
    if constexpr (VPL % 4 == 0) {
#pragma unroll
      for (int q = 0; q < VPL / 4; ++q) {
        const uint2 u = *reinterpret_cast<const uint2*>(fp + 4 * q);
        e.fb[2 * q] = u.x;
        e.fb[2 * q + 1] = u.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < (VPL + 1) / 2; ++i)
        e.fb[i] = (uint32_t)fp[2 * i] | (2 * i + 1 < VPL ? (uint32_t)fp[2 * i + 1] << 16 : 0u);
    }
  } else {
    float t[VPL];
    vload(F + row * ldf + jc, t);
#pragma unroll
    for (int i = 0; i < VPL; ++i) e.fb[i] = __builtin_bit_cast(uint32_t, t[i]);
  }
}

// Dropout multipliers of one edge group: lane l < PF*H evaluates the hash of (t0 + l/H, l%H);
// every lane then reads the PF*H values back as wave-uniform scalars.
template <int H>
__device__ __forceinline__ void group_dropout(const DropParams& dp, int32_t t0, int lane, float (&mul)[PF][H]) {
  float mine = 1.0f;
  if (dp.active && lane < PF * H)
    mine = dropout_mul(dp.seed, (uint64_t)(t0 + lane / H) * H + (lane % H), dp.thresh, dp.inv_keep);
#pragma unroll
  for (int j = 0; j < PF; ++j)
#pragma unroll
    for (int h = 0; h < H; ++h) mul[j][h] = dp.active ? readlane_f(mine, j * H + h) : 1.0f;
}

constexpr int cmax(int a, int b) { return a > b ? a : b; }

#ifdef ALIGNN_TCONV_WPE
#define TCONV_ATTR __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ALIGNN_TCONV_WPE, ALIGNN_TCONV_WPE)))
#else
#define TCONV_ATTR __launch_bounds__(256)
#endif
// waves per SIMD asked of the _2 kernels of up to 16 values per lane (0: the compiler's choice).
// Forward: 3 (168 registers, 4 spilled at bf16; C3 atom forward 354 -> 305 us, C2 59 -> 55 us:
// profiles/r06/ab_tconv_ring.txt)
#ifndef ALIGNN_TCONV2_WPE_FWD
#define ALIGNN_TCONV2_WPE_FWD 3
#endif
#ifndef ALIGNN_TCONV2_WPE_BWD
#define ALIGNN_TCONV2_WPE_BWD 0
#endif
#define TCONV2_ATTR_(W) __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((W) > 0 ? (W) : 1)))

// =============================================================================================
// Forward
// =============================================================================================
struct FwdParams {
  int64_t n, m;
  int D, pad_;
  const int32_t* off;
  const int32_t* src_at;
  const int32_t* feat_row;
  const float* QKVR; int64_t ldq;
  const float* U;
  const float* wbar;
  const float* F; int64_t ldf;
  float* aggV; float* S; float* sumA; float* mstat; float* den;
  DropParams drop;
  int fbf, pad3_;   // F holds bf16 elements (ldf in elements)
};

template <int VPL, int H>
constexpr int fwd_merge_floats() { return 4 * 64 * (3 * H + H * VPL + VPL); }

// =============================================================================================
// Backward, target side
// =============================================================================================
struct BwdDstParams {
  int64_t n, m;
  int D, pad_;
  const int32_t* off;
  const int32_t* src_at;
  const int32_t* feat_row;
  const float* QKVR; int64_t ldq;
  const float* U;
  const float* Vd;
  const float* wbar;
  const float* F; int64_t ldf;
  const float* dout;
  const float* outp;
  const float* mstat;
  const float* den;
  float* dq; int64_t lddq;
  float* Sz; float* sigz;
  float* dz_e; float* alpha_e;
  float* dF; int64_t lddf; int acc_dF, dfbf;   // dfbf: dF written as bf16 (acc_dF bit 0 clear)
  DropParams drop;
  int fbf, pad3_;   // F holds bf16 elements (ldf in elements)
};

template <int VPL, int H>
constexpr int bwd_merge_floats() {
  return 4 * 64 * (H + H * VPL + VPL);
}

// =============================================================================================
// The atom-graph (and general-shape) attention kernels: materialised edge features, per-(edge, head)
// softmax quantities kept small for more waves per SIMD on the latency-bound edge stream (the round-1
// broadcast-register variants and the in-kernel angle-encoder recompute were measured slower and
// removed in round 3):
//  * per-(edge, head) softmax quantities stay ROW-DISTRIBUTED — after the transpose-reduction
//    (reduce_rows) row j of value register h holds (edge j, head h) — so a group needs H registers
//    per quantity instead of PF*H broadcast copies; group max/sums over the PF rows are two xor-16/32
//    shuffles; single (edge, head) values are read back as scalars (v_readlane) where they scale a
//    feature vector;
//  * the node's per-head vectors (u, and Vd in the backward) are staged in LDS, one copy per wave,
//    and read one head at a time.
// The LDS of the node vectors and of the heavy-node merge alias (a barrier separates them).
// =============================================================================================

// Transpose-reduction without the broadcast: value r*(P/4)+i ends in row r of b[i] (P = N rounded up
// to a multiple of 4), replicated over the row's 16 lanes.
template <int N>
__device__ __forceinline__ void reduce_rows(const float (&v)[N], float (&b)[(N + 3) / 4]) {
  constexpr int P = (N + 3) / 4 * 4;
  float a[P / 2];
#pragma unroll
  for (int i = 0; i < P / 2; ++i) {
    const float x = i < N ? v[i] : 0.f;
    const float y = (i + P / 2) < N ? v[i + P / 2] : 0.f;
    const auto r = __builtin_amdgcn_permlane32_swap(u_bits(x), u_bits(y), false, false);
    a[i] = f_bits(r[0]) + f_bits(r[1]);
  }
#pragma unroll
  for (int i = 0; i < P / 4; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(u_bits(a[i]), u_bits(a[i + P / 4]), false, false);
    b[i] = row_sum16(f_bits(r[0]) + f_bits(r[1]));
  }
}

// Over the four rows of a row-replicated value (VALU lane swaps, no LDS crossbar):
// permlane32_swap(x, x) pairs lane l with l^32, permlane16_swap(x, x) row 2k with 2k+1.
__device__ __forceinline__ float rows_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(u_bits(x), u_bits(x), false, false);
  x = f_bits(r[0]) + f_bits(r[1]);
  r = __builtin_amdgcn_permlane16_swap(u_bits(x), u_bits(x), false, false);
  return f_bits(r[0]) + f_bits(r[1]);
}
__device__ __forceinline__ float rows_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(u_bits(x), u_bits(x), false, false);
  x = fmaxf(f_bits(r[0]), f_bits(r[1]));
  r = __builtin_amdgcn_permlane16_swap(u_bits(x), u_bits(x), false, false);
  return fmaxf(f_bits(r[0]), f_bits(r[1]));
}

template <int VPL, int H>
constexpr int fwd2_lds_floats() { return cmax(fwd_merge_floats<VPL, H>(), 4 * H * 64 * VPL); }

template <int VPL, int H, bool FBF>
__device__ __forceinline__ void fwd2_node(const FwdParams& p, float* smem, int64_t d, int wsub, int nw, bool heavy) {
  static_assert(PF == 4, "row-distributed layout assumes one edge per row");
  constexpr int NS = 3 * H + H * VPL + VPL;
  constexpr int RS = 64 * VPL;
  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int row = lane >> 4;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));
  float* uv = smem + wave * H * RS;  // this wave's copy of u[h]

  float accS[H][VPL], accV[VPL];
  float m[H], s[H], sa[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    m[h] = -INFINITY;
    s[h] = 0.f;
    sa[h] = 0.f;
    vzero(accS[h]);
  }
  vzero(accV);

  const int32_t first = beg + wsub * PF, stride = nw * PF;
  if (first < end) {
    const int jc = act ? j0 : 0;
    // The first group's rows go out with the node's own vectors (one round trip for both); the
    // next group is requested slot by slot as each row of the current one is consumed.
    EdgeRow<VPL, FBF> ring[PF];
    auto request = [&](int j, int32_t t0) {
      const int32_t t = min(t0 + j, end - 1);
      load_row<VPL, FBF>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, (int64_t)uni(sld(p.src_at, t)),
                         p.feat_row ? (int64_t)uni(sld(p.feat_row, t)) : t, jc);
    };
#pragma unroll
    for (int j = 0; j < PF; ++j) request(j, first);
    float q[VPL], wb[VPL];
    vzero(q);
    vzero(wb);
    if (act) {
      vload(p.QKVR + d * p.ldq + j0, q);
      if (p.wbar) vload(p.wbar + j0, wb);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float t[VPL];
        vload(p.U + (d * H + h) * D + j0, t);
        vstore(uv + h * RS + j0, t);
      }
    } else {
      // lanes past D: zeros, so their (otherwise uninitialised) LDS slots cannot put a NaN into
      // the cross-lane score reduction (0 * NaN)
      float z[VPL];
      vzero(z);
#pragma unroll
      for (int h = 0; h < H; ++h) vstore(uv + h * RS + j0, z);
    }
    float c[H];
#pragma unroll
    for (int h = 0; h < H; ++h) c[h] = 0.f;
    if (p.wbar) {
      const float part = vdot(wb, q);
#pragma unroll
      for (int h = 0; h < H; ++h) c[h] = (h == hl) ? part : 0.f;
      reduce_bcast<H>(c, lane);
    }
    // Straight-line control flow around the ring (the next group is requested unconditionally,
    // clamped to the segment): a conditional request would merge the ring's registers at the loop
    // head, and the copies of that merge wait for every load in flight.
    for (int32_t tb = first; tb < end; tb += stride) {
      asm volatile("" ::: "memory");  // keep the u reads in the loop (registers are the point)
      float f[PF][VPL];
#pragma unroll
      for (int j = 0; j < PF; ++j) ring[j].widen(f[j]);
      float pr[PF * H];
      {
        float qk[PF];
#pragma unroll
        for (int j = 0; j < PF; ++j) qk[j] = vdot(q, ring[j].k);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          float u[VPL];
          vload(uv + h * RS + j0, u);
#pragma unroll
          for (int j = 0; j < PF; ++j) pr[j * H + h] = vdot(u, f[j]) + ((h == hl) ? qk[j] : 0.f);
        }
      }
      float b[H];
      reduce_rows<PF * H>(pr, b);  // row j: b[h] = score partial of (edge tb + j, head h)
      const bool rv = tb + row < end;
      float mine = 1.0f;
      if (p.drop.active && lane < PF * H)
        mine = dropout_mul(p.drop.seed, (uint64_t)(tb + lane / H) * H + (lane % H), p.drop.thresh, p.drop.inv_keep);
      float corr[H];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float z = rv ? (b[h] + c[h]) * scale : -INFINITY;
        const float mn = fmaxf(m[h], rows_max(z));
        corr[h] = __expf(m[h] - mn);
        m[h] = mn;
        const float ex = __expf(z - mn);  // 0 on rows past the segment end
        const float mul = p.drop.active ? __shfl(mine, row * H + h, 64) : 1.0f;
        const float ed = ex * mul;
        s[h] = s[h] * corr[h] + rows_sum(ex);
        sa[h] = sa[h] * corr[h] + rows_sum(ed);
        b[h] = ed;  // row-distributed alpha' numerators
#pragma unroll
        for (int i = 0; i < VPL; ++i) accS[h][i] *= corr[h];
      }
      {
        const float cl = pick_r<H>(corr, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) accV[i] *= cl;
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        float e[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          e[h] = readlane_f(b[h], 16 * j);
#pragma unroll
          for (int i = 0; i < VPL; ++i) accS[h][i] = fmaf(e[h], f[j][i], accS[h][i]);
        }
        const float el = pick_r<H>(e, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) accV[i] = fmaf(el, ring[j].v[i], accV[i]);
        request(j, tb + stride);
      }
    }
  }

  if (heavy) {
    __syncthreads();  // every wave is done with its u copy (the merge buffer aliases it)
    float* my = smem + (wave * 64 + lane) * NS;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      my[h] = m[h];
      my[H + h] = s[h];
      my[2 * H + h] = sa[h];
#pragma unroll
      for (int i = 0; i < VPL; ++i) my[3 * H + h * VPL + i] = accS[h][i];
    }
#pragma unroll
    for (int i = 0; i < VPL; ++i) my[3 * H + H * VPL + i] = accV[i];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float mt = -INFINITY;
        for (int v = 0; v < 4; ++v) mt = fmaxf(mt, smem[(v * 64 + lane) * NS + h]);
        s[h] = 0.f;
        sa[h] = 0.f;
#pragma unroll
        for (int i = 0; i < VPL; ++i) accS[h][i] = 0.f;
        for (int v = 0; v < 4; ++v) {
          const float* o = smem + (v * 64 + lane) * NS;
          const float f = (o[h] == -INFINITY) ? 0.f : __expf(o[h] - mt);
          s[h] = fmaf(o[H + h], f, s[h]);
          sa[h] = fmaf(o[2 * H + h], f, sa[h]);
#pragma unroll
          for (int i = 0; i < VPL; ++i) accS[h][i] = fmaf(o[3 * H + h * VPL + i], f, accS[h][i]);
        }
        m[h] = mt;
      }
#pragma unroll
      for (int i = 0; i < VPL; ++i) accV[i] = 0.f;
      for (int v = 0; v < 4; ++v) {
        const float* o = smem + (v * 64 + lane) * NS;
        const float mh = o[hl];
        const float f = (mh == -INFINITY) ? 0.f : __expf(mh - pick_r<H>(m, hl));
#pragma unroll
        for (int i = 0; i < VPL; ++i) accV[i] = fmaf(o[3 * H + H * VPL + i], f, accV[i]);
      }
    }
  }

  if (!heavy || wave == 0) {
    float inv[H], dn[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      dn[h] = s[h] + 1e-16f;
      inv[h] = 1.0f / dn[h];
    }
    if (act) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float o[VPL];
#pragma unroll
        for (int i = 0; i < VPL; ++i) o[i] = accS[h][i] * inv[h];
        vstore(p.S + (d * H + h) * D + j0, o);
      }
      const float il = pick_r<H>(inv, hl);
      float o[VPL];
#pragma unroll
      for (int i = 0; i < VPL; ++i) o[i] = accV[i] * il;
      vstore(p.aggV + d * D + j0, o);
    }
    if (lane < H) {
      p.sumA[d * H + lane] = pick_r<H>(sa, lane) * pick_r<H>(inv, lane);
      p.mstat[d * H + lane] = pick_r<H>(m, lane);
      p.den[d * H + lane] = pick_r<H>(dn, lane);
    }
  }
  if (heavy) __syncthreads();  // merge buffer / u copies free for the next item
}

// FBF: bf16 edge-feature rows (a compile-time switch: the fp32 instantiation is unchanged)
template <int VPL, int H, bool FBF>
__global__ TCONV2_ATTR_(VPL * H <= 16 ? ALIGNN_TCONV2_WPE_FWD : 0) void tconv_fwd2_kernel(FwdParams p, Sched sc) {
  resolve_drop(p.drop);
  __shared__ float smem[fwd2_lds_floats<VPL, H>()];
  const int wave = wave_id();
  const int64_t items = sc.items();
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    if (it < sc.n_heavy) {
      fwd2_node<VPL, H, FBF>(p, smem, (int64_t)uni(sld(sc.heavy, it)), wave, 4, true);
    } else {
      const int64_t i = (it - sc.n_heavy) * 4 + wave;
      if (i < sc.n_light) fwd2_node<VPL, H, FBF>(p, smem, sc.light ? (int64_t)uni(sld(sc.light, i)) : i, 0, 1, false);
    }
  }
}

template <int VPL, int H>
constexpr int bwd2_lds_floats() { return cmax(bwd_merge_floats<VPL, H>(), 4 * 2 * H * 64 * VPL); }

// OLD: dF is accumulated into (acc_dF bit 0): its rows are prefetched with the edge rows (a
// compile-time switch, so the plain-write instantiation carries no conditional load)
template <int VPL, int H, bool FBF, bool OLD>
__device__ __forceinline__ void bwd2_node(const BwdDstParams& p, float* smem, int64_t d, int wsub, int nw, bool heavy) {
  static_assert(PF == 4, "row-distributed layout assumes one edge per row");
  constexpr int NS = H + H * VPL + VPL;
  constexpr int RS = 64 * VPL;
  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int row = lane >> 4;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));
  float* uv = smem + wave * 2 * H * RS;  // this wave's u[h] (h < H) and Vd[h] (H + h)
  const bool do_dF = p.dF != nullptr;

  float sz[H][VPL], sgz[H], dqa[VPL];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    vzero(sz[h]);
    sgz[h] = 0.f;
  }
  vzero(dqa);

  const int32_t first = beg + wsub * PF, stride = nw * PF;
  if (first < end) {
    const int jc = act ? j0 : 0;
    // the first group's rows go out with the node's own vectors (see fwd2_node)
    EdgeRow<VPL, FBF> ring[PF];
    int64_t rw[PF];
    float ob[OLD ? PF : 1][VPL];
    auto request = [&](int j, int32_t t0) {
      const int32_t t = min(t0 + j, end - 1);
      rw[j] = p.feat_row ? uni(sld(p.feat_row, t)) : t;
      load_row<VPL, FBF>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, (int64_t)uni(sld(p.src_at, t)), rw[j], jc);
      if constexpr (OLD) vload(p.dF + rw[j] * p.lddf + jc, ob[j]);
    };
#pragma unroll
    for (int j = 0; j < PF; ++j) request(j, first);
    float q[VPL], go[VPL];
    vzero(q);
    vzero(go);
    float c[3 * H];
    {
      float op[VPL], wb[VPL];
      vzero(op);
      vzero(wb);
      if (act) {
        vload(p.QKVR + d * p.ldq + j0, q);
        vload(p.dout + d * D + j0, go);
        vload(p.outp + d * D + j0, op);
        if (p.wbar) vload(p.wbar + j0, wb);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          float t[VPL];
          vload(p.U + (d * H + h) * D + j0, t);
          vstore(uv + h * RS + j0, t);
          vload(p.Vd + (d * H + h) * D + j0, t);
          vstore(uv + (H + h) * RS + j0, t);
        }
      } else {  // lanes past D: zeros (see tconv_fwd2)
        float z[VPL];
        vzero(z);
#pragma unroll
        for (int h = 0; h < 2 * H; ++h) vstore(uv + h * RS + j0, z);
      }
      const float pc = vdot(wb, q), pc2 = vdot(wb, go), pdl = vdot(go, op);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        c[h] = (h == hl) ? pc : 0.f;
        c[H + h] = (h == hl) ? pc2 : 0.f;
        c[2 * H + h] = (h == hl) ? pdl : 0.f;
      }
      reduce_bcast<3 * H>(c, lane);
    }
    float mst[H], inv_den[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      mst[h] = p.mstat[d * H + h];
      inv_den[h] = 1.0f / p.den[d * H + h];
    }
    for (int32_t tb = first; tb < end; tb += stride) {  // (straight-line around the ring: see fwd2_node)
      asm volatile("" ::: "memory");  // keep the u / Vd reads in the loop
      float f[PF][VPL];
#pragma unroll
      for (int j = 0; j < PF; ++j) ring[j].widen(f[j]);
      float bs[H], bd[H];
      {
        float ps[PF * H], pd[PF * H];
        float qk[PF], gv[PF];
#pragma unroll
        for (int j = 0; j < PF; ++j) {
          qk[j] = vdot(q, ring[j].k);
          gv[j] = vdot(go, ring[j].v);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
          float u[VPL], vd[VPL];
          vload(uv + h * RS + j0, u);
          vload(uv + (H + h) * RS + j0, vd);
#pragma unroll
          for (int j = 0; j < PF; ++j) {
            ps[j * H + h] = vdot(u, f[j]) + ((h == hl) ? qk[j] : 0.f);
            pd[j * H + h] = vdot(vd, f[j]) + ((h == hl) ? gv[j] : 0.f);
          }
        }
        reduce_rows<PF * H>(ps, bs);
        reduce_rows<PF * H>(pd, bd);
      }
      const bool rv = tb + row < end;
      float mine = 1.0f;
      if (p.drop.active && lane < PF * H)
        mine = dropout_mul(p.drop.seed, (uint64_t)(tb + lane / H) * H + (lane % H), p.drop.thresh, p.drop.inv_keep);
      // row-distributed dz (= dL/dz / sqrt(C)) in bs, alpha' in bd
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float mul = p.drop.active ? __shfl(mine, row * H + h, 64) : 1.0f;
        const float z = (bs[h] + c[h]) * scale;
        const float alpha = __expf(z - mst[h]) * inv_den[h];
        const float al = alpha * mul;
        const float dal = (bd[h] + c[H + h]) * mul;
        const float dz = alpha * (dal - c[2 * H + h]) * scale;
        bs[h] = rv ? dz : 0.f;
        bd[h] = rv ? al : 0.f;
        sgz[h] += rows_sum(bs[h]);
      }
      {
        const int col = lane & 15;
        if (col < H && rv) {
          const int64_t t = (int64_t)(tb + row);
          p.dz_e[t * H + col] = pick_r<H>(bs, col);
          p.alpha_e[t * H + col] = pick_r<H>(bd, col);
        }
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        float e[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          e[h] = readlane_f(bs[h], 16 * j);
#pragma unroll
          for (int i = 0; i < VPL; ++i) sz[h][i] = fmaf(e[h], f[j][i], sz[h][i]);
        }
        const float dzl = pick_r<H>(e, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) dqa[i] = fmaf(dzl, ring[j].k[i], dqa[i]);
      }
      if (do_dF) {
        // dF[row(t)] (+)= sum_h dz u_h + alpha' Vd_h, one edge at a time (u / Vd re-read from LDS
        // per edge: one edge's sum live instead of PF)
#pragma unroll
        for (int j = 0; j < PF; ++j) {
          float df[VPL];
          if constexpr (OLD) {
#pragma unroll
            for (int i = 0; i < VPL; ++i) df[i] = ob[j][i];
          } else {
            vzero(df);
          }
#pragma unroll
          for (int h = 0; h < H; ++h) {
            float u[VPL], vd[VPL];
            vload(uv + h * RS + j0, u);
            vload(uv + (H + h) * RS + j0, vd);
            const float ez = readlane_f(bs[h], 16 * j), ea = readlane_f(bd[h], 16 * j);
#pragma unroll
            for (int i = 0; i < VPL; ++i) df[i] = fmaf(ez, u[i], fmaf(ea, vd[i], df[i]));
          }
          if (tb + j < end && act) {
#pragma unroll
            for (int i = 0; i < VPL; ++i) df[i] = (p.acc_dF & 2) ? (f[j][i] > 0.f ? df[i] : 0.f) : df[i];
            if (p.dfbf) vstore_bf(reinterpret_cast<uint16_t*>(p.dF) + rw[j] * p.lddf + j0, df);
            else vstore(p.dF + rw[j] * p.lddf + j0, df);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < PF; ++j) request(j, tb + stride);
    }
  }
  if (heavy) {
    __syncthreads();  // u / Vd copies are dead before the merge buffer (aliased) is written
    float* my = smem + (wave * 64 + lane) * NS;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      my[h] = sgz[h];
#pragma unroll
      for (int i = 0; i < VPL; ++i) my[H + h * VPL + i] = sz[h][i];
    }
#pragma unroll
    for (int i = 0; i < VPL; ++i) my[H + H * VPL + i] = dqa[i];
    __syncthreads();
    if (wave == 0) {
      for (int v = 1; v < 4; ++v) {
        const float* o = smem + (v * 64 + lane) * NS;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          sgz[h] += o[h];
#pragma unroll
          for (int i = 0; i < VPL; ++i) sz[h][i] += o[H + h * VPL + i];
        }
#pragma unroll
        for (int i = 0; i < VPL; ++i) dqa[i] += o[H + H * VPL + i];
      }
    }
  }
  if (!heavy || wave == 0) {
    if (act) {
      vstore(p.dq + d * p.lddq + j0, dqa);
#pragma unroll
      for (int h = 0; h < H; ++h) vstore(p.Sz + (d * H + h) * D + j0, sz[h]);
    }
    if (lane < H) p.sigz[d * H + lane] = pick_r<H>(sgz, lane);
  }
  if (heavy) __syncthreads();
}

template <int VPL, int H, bool FBF, bool OLD>
__global__ TCONV2_ATTR_(VPL * H <= 16 ? ALIGNN_TCONV2_WPE_BWD : 0) void tconv_bwd_dst2_kernel(BwdDstParams p, Sched sc) {
  resolve_drop(p.drop);
  __shared__ float smem[bwd2_lds_floats<VPL, H>()];
  const int wave = wave_id();
  const int64_t items = sc.items();
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    if (it < sc.n_heavy) {
      bwd2_node<VPL, H, FBF, OLD>(p, smem, (int64_t)uni(sld(sc.heavy, it)), wave, 4, true);
    } else {
      const int64_t i = (it - sc.n_heavy) * 4 + wave;
      if (i < sc.n_light) bwd2_node<VPL, H, FBF, OLD>(p, smem, sc.light ? (int64_t)uni(sld(sc.light, i)) : i, 0, 1, false);
    }
  }
}

// =============================================================================================
// Backward, source side: dK, dV per source node over the by-source CSR (no atomics)
// =============================================================================================
struct BwdSrcParams {
  int64_t n, m;
  int D, pad_;
  const int32_t* off_src;
  const int32_t* pos_src;
  const int32_t* dst_at;
  const float* QKVR; int64_t ldq;
  const float* dout;
  const float* dz_e;
  const float* alpha_e;
  float* dKV; int64_t lddkv;
  const int32_t* dst_src;  // optional: dst_at[pos_src[i]] in by-source order (one index level less)
  // bf16 storage (tconv_bwd_src2_kernel<.., true>): the gathered target rows Q (ld ldq16) and dout
  // as bf16 copies, widened exactly at the load (autocast: Q is a bf16 Linear output)
  const uint16_t* Q16; int64_t ldq16; const uint16_t* dout16;
};

#ifndef ALIGNN_SRC_PF
#define ALIGNN_SRC_PF 16  // 4 -> 16: +1.2 % same-box (8: +0.6 %; 12, 3 waves/SIMD: -0.4 % vs 16; 24 drops to 1 wave/SIMD; v36, v41)
#endif
// edges in flight per wave: 2,580 line-graph sources give only ~2.5 waves per SIMD, so the
// memory-level parallelism has to come from each wave's own group depth
constexpr int SRC_PF = ALIGNN_SRC_PF;

template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_bwd_src_kernel(BwdSrcParams p) {
  constexpr int PF = SRC_PF;
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + wave_id();
  if (s >= p.n) return;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  float dk[VPL], dv[VPL];
  vzero(dk);
  vzero(dv);
  const int32_t beg = sld(p.off_src, s), end = sld(p.off_src, s + 1);
  if (act) {
    for (int32_t ib = beg; ib < end; ib += PF) {
      float qv[PF][VPL], gv[PF][VPL], dz[PF], al[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) {  // issue all loads of the group first
        vzero(qv[j]);
        vzero(gv[j]);
        dz[j] = 0.f;
        al[j] = 0.f;
        if (ib + j < end) {
          const int64_t pos = sld(p.pos_src, ib + j);
          const int64_t dd = sld(p.dst_at, pos);
          dz[j] = p.dz_e[pos * H + hl];
          al[j] = p.alpha_e[pos * H + hl];
          vload(p.QKVR + dd * p.ldq + j0, qv[j]);
          vload(p.dout + dd * D + j0, gv[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < PF; ++j)
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          dk[k] = fmaf(dz[j], qv[j][k], dk[k]);
          dv[k] = fmaf(al[j], gv[j][k], dv[k]);
        }
    }
    vstore(p.dKV + s * p.lddkv + j0, dk);
    vstore(p.dKV + s * p.lddkv + D + j0, dv);
  }
}

// Same sums, in the same order, over a by-source target list (dst_src): each edge's target and its
// position are two independent scalar loads instead of a dependent pair, the next group's indices are
// loaded while this group's rows are in flight, and tail edges are clamped to the source's last
// edge with their scalars zeroed (unconditional loads).  Bitwise equal to tconv_bwd_src_kernel.
template <int VPL, int H, bool QBF>
__device__ __forceinline__ void tconv_bwd_src2_body(const BwdSrcParams& p) {
  constexpr int PF = SRC_PF;
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + wave_id();
  if (s >= p.n) return;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  float dk[VPL], dv[VPL];
  vzero(dk);
  vzero(dv);
  const int32_t beg = uni(sld(p.off_src, s)), end = uni(sld(p.off_src, s + 1));
  if (act && beg < end) {
    const int32_t last = end - 1;
    int32_t pos[2][PF], dd[2][PF];
    auto indices = [&](int32_t (&po)[PF], int32_t (&d)[PF], int32_t ib) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int32_t i = min(ib + j, last);
        po[j] = uni(sld(p.pos_src, i));
        d[j] = uni(sld(p.dst_src, i));
      }
    };
    indices(pos[0], dd[0], beg);
    int cur = 0;
    for (int32_t ib = beg; ib < end; ib += PF) {
      float qv[PF][VPL], gv[PF][VPL], dz[PF], al[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int64_t po = pos[cur][j], d = dd[cur][j];
        dz[j] = p.dz_e[po * H + hl];
        al[j] = p.alpha_e[po * H + hl];
        if constexpr (QBF) {
          vload_bf(p.Q16 + d * p.ldq16 + j0, qv[j]);
          vload_bf(p.dout16 + d * D + j0, gv[j]);
        } else {
          vload(p.QKVR + d * p.ldq + j0, qv[j]);
          vload(p.dout + d * D + j0, gv[j]);
        }
      }
      if (ib + PF < end) indices(pos[cur ^ 1], dd[cur ^ 1], ib + PF);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const bool valid = ib + j < end;  // wave-uniform
        const float zj = valid ? dz[j] : 0.f, aj = valid ? al[j] : 0.f;
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          dk[k] = fmaf(zj, valid ? qv[j][k] : 0.f, dk[k]);
          dv[k] = fmaf(aj, valid ? gv[j][k] : 0.f, dv[k]);
        }
      }
      cur ^= 1;
    }
  }
  if (act) {
    vstore(p.dKV + s * p.lddkv + j0, dk);
    vstore(p.dKV + s * p.lddkv + D + j0, dv);
  }
}

template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_bwd_src2_kernel(BwdSrcParams p) {
  tconv_bwd_src2_body<VPL, H, false>(p);
}

// bf16 target rows (the gathered Q and dout rows are the kernel's traffic: half the bytes)
template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_bwd_src2_bf16_kernel(BwdSrcParams p) {
  tconv_bwd_src2_body<VPL, H, true>(p);
}
// bf16 target rows through buffer loads (the C3 line graph: 2,027,520 edges over 16,020 sources).
// Each edge's offsets are scalars (the instruction's SGPR offset) and the lane's part is one fixed
// VGPR offset, so a group holds nothing but its data: src2's flat loads formed a 64-bit VGPR address
// per load (240 VGPRs, 2 waves/SIMD).  Rows stay bf16 in registers until their FMAs; the sums run in
// src2's order (bitwise equal).  Offsets are 32-bit: the host takes this kernel only when every
// operand spans < 2 GB.
#ifndef ALIGNN_SRC3
#define ALIGNN_SRC3 1
#endif
#ifndef ALIGNN_SRC3_PF
#define ALIGNN_SRC3_PF 8   // C3 step: 8 edges per group (95 VGPRs, 5 waves/SIMD) 20,381-20,431 graphs/s, 16 (2 waves) 19,784-19,850
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n, 0x00020000);
}

#ifndef ALIGNN_SRC3_WPE
#define ALIGNN_SRC3_WPE 1  // minimum waves per SIMD asked of the register allocator (1: its own choice)
#endif
template <int VPL, int H>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VPL == 4 ? ALIGNN_SRC3_WPE : 1, 8)))
void tconv_bwd_src3_bf16_kernel(BwdSrcParams p) {
  static_assert(VPL % 4 == 0, "bwd_src3: four bf16 features per 8-byte load");
  constexpr int PF = ALIGNN_SRC3_PF;
  constexpr int NQ = VPL / 4;
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + wave_id();
  if (s >= p.n) return;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  float dk[VPL], dv[VPL];
  vzero(dk);
  vzero(dv);
  const int32_t beg = uni(sld(p.off_src, s)), end = uni(sld(p.off_src, s + 1));
  if (act && beg < end) {
    const __amdgpu_buffer_rsrc_t rq = buf_rsrc(p.Q16, p.n * p.ldq16 * 2), rg = buf_rsrc(p.dout16, p.n * D * 2);
    const __amdgpu_buffer_rsrc_t rz = buf_rsrc(p.dz_e, p.m * H * 4), ra = buf_rsrc(p.alpha_e, p.m * H * 4);
    const int vrow = j0 * 2, vh = hl * 4;
    const int32_t last = end - 1;
    int32_t pos[2][PF], dd[2][PF];
    auto indices = [&](int32_t (&po)[PF], int32_t (&d)[PF], int32_t ib) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int32_t i = min(ib + j, last);
        po[j] = uni(sld(p.pos_src, i));
        d[j] = uni(sld(p.dst_src, i));
      }
    };
    indices(pos[0], dd[0], beg);
    int cur = 0;
    for (int32_t ib = beg; ib < end; ib += PF) {
      u2 qr[PF][NQ], gr[PF][NQ];
      float dz[PF], al[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int po = pos[cur][j] * H * 4, d = dd[cur][j];
        dz[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rz, vh, po, 0));
        al[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, vh, po, 0));
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          qr[j][q] = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(rq, vrow + 8 * q, (int)(d * p.ldq16 * 2), 0));
          gr[j][q] = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(rg, vrow + 8 * q, d * D * 2, 0));
        }
      }
      if (ib + PF < end) indices(pos[cur ^ 1], dd[cur ^ 1], ib + PF);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const bool valid = ib + j < end;  // wave-uniform
        const float zj = valid ? dz[j] : 0.f, aj = valid ? al[j] : 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float qv[4] = {__builtin_bit_cast(float, qr[j][q].x << 16), __builtin_bit_cast(float, qr[j][q].x & 0xffff0000u),
                               __builtin_bit_cast(float, qr[j][q].y << 16), __builtin_bit_cast(float, qr[j][q].y & 0xffff0000u)};
          const float gv[4] = {__builtin_bit_cast(float, gr[j][q].x << 16), __builtin_bit_cast(float, gr[j][q].x & 0xffff0000u),
                               __builtin_bit_cast(float, gr[j][q].y << 16), __builtin_bit_cast(float, gr[j][q].y & 0xffff0000u)};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            dk[4 * q + k] = fmaf(zj, valid ? qv[k] : 0.f, dk[4 * q + k]);
            dv[4 * q + k] = fmaf(aj, valid ? gv[k] : 0.f, dv[4 * q + k]);
          }
        }
      }
      cur ^= 1;
    }
  }
  if (act) {
    vstore(p.dKV + s * p.lddkv + j0, dk);
    vstore(p.dKV + s * p.lddkv + D + j0, dv);
  }
}

// ---------------------------------------------------------------------------------------------
// Dispatch on (VPL, H)
// ---------------------------------------------------------------------------------------------

static int vpl_for(int D) {
  if (D <= 64) return 1;
  if (D == 128) return 2;
  if (D == 256) return 4;
  if (D == 512) return 8;
  return 0;
}

#define ALIGNN_DISPATCH_VH(VPL_, H_, FN, ...)                                        \
  do {                                                                               \
    if (VPL_ == 1 && H_ == 1) FN<1, 1>(__VA_ARGS__);                                 \
    else if (VPL_ == 1 && H_ == 2) FN<1, 2>(__VA_ARGS__);                            \
    else if (VPL_ == 1 && H_ == 4) FN<1, 4>(__VA_ARGS__);                            \
    else if (VPL_ == 2 && H_ == 1) FN<2, 1>(__VA_ARGS__);                            \
    else if (VPL_ == 2 && H_ == 2) FN<2, 2>(__VA_ARGS__);                            \
    else if (VPL_ == 2 && H_ == 4) FN<2, 4>(__VA_ARGS__);                            \
    else if (VPL_ == 4 && H_ == 1) FN<4, 1>(__VA_ARGS__);                            \
    else if (VPL_ == 4 && H_ == 2) FN<4, 2>(__VA_ARGS__);                            \
    else if (VPL_ == 4 && H_ == 4) FN<4, 4>(__VA_ARGS__);                            \
    else if (VPL_ == 4 && H_ == 8) FN<4, 8>(__VA_ARGS__);                            \
    else if (VPL_ == 8 && H_ == 4) FN<8, 4>(__VA_ARGS__);                            \
    else if (VPL_ == 8 && H_ == 8) FN<8, 8>(__VA_ARGS__);                            \
    else { set_error("tconv: unsupported D/H combination"); return ALIGNN_E_UNSUPPORTED; } \
  } while (0)

template <int VPL, int H>
static void launch_fwd(const FwdParams& p, const Sched& sc, hipStream_t s) {
  const int64_t items = sc.items();
  if (items <= 0) return;
  if (p.fbf) launch((tconv_fwd2_kernel<VPL, H, true>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
  else launch((tconv_fwd2_kernel<VPL, H, false>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
}

template <int VPL, int H>
static void launch_bwd_dst(const BwdDstParams& p, const Sched& sc, hipStream_t s) {
  const int64_t items = sc.items();
  if (items <= 0) return;
  const bool old = p.dF != nullptr && (p.acc_dF & 1);
  if (p.fbf) {
    if (old) launch((tconv_bwd_dst2_kernel<VPL, H, true, true>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
    else launch((tconv_bwd_dst2_kernel<VPL, H, true, false>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
  } else {
    if (old) launch((tconv_bwd_dst2_kernel<VPL, H, false, true>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
    else launch((tconv_bwd_dst2_kernel<VPL, H, false, false>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
  }
}

template <int VPL, int H>
static void launch_bwd_src(const BwdSrcParams& p, hipStream_t s) {
  if (p.Q16) {
    constexpr int64_t lim = int64_t(1) << 31;
    if constexpr (VPL % 4 == 0 && ALIGNN_SRC3) {
      if (p.n * p.ldq16 * 2 < lim && p.n * p.D * 2 < lim && p.m * H * 4 < lim) {
        launch((tconv_bwd_src3_bf16_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
        return;
      }
    }
    launch((tconv_bwd_src2_bf16_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
  }
  else if (p.dst_src) launch((tconv_bwd_src2_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
  else launch((tconv_bwd_src_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
}

static Sched make_sched(const AlignnSchedule* sc, int64_t n) {
  Sched r;
  if (sc && (sc->n_light + sc->n_heavy) > 0) {
    r.light = sc->light;
    r.n_light = sc->n_light;
    r.heavy = sc->heavy;
    r.n_heavy = sc->n_heavy;
  } else {
    r.light = nullptr;  // every node light, node = wave index
    r.n_light = n;
    r.heavy = nullptr;
    r.n_heavy = 0;
  }
  return r;
}

static int check_dims(int D, int H) {
  if (D <= 0 || H <= 0 || D % H != 0 || vpl_for(D) == 0) {
    set_error("tconv: unsupported hidden=%d heads=%d (hidden in {<=64,128,256,512}, divisible by heads)", D, H);
    return ALIGNN_E_UNSUPPORTED;
  }
  const int C = D / H;
  if (C < vpl_for(D)) {
    set_error("tconv: head dim %d smaller than values per lane", C);
    return ALIGNN_E_UNSUPPORTED;
  }
  return ALIGNN_OK;
}

// lgconv.hip: single-wave-item kernels (ALIGNN_SCHED_WAVE_ITEMS)
bool lg3_supported(int D, int H, const int32_t* feat_row, const float* F, const AlignnSchedule* sched);
int lg3_fwd(int64_t n, int64_t m, int H, const int32_t* off, const int32_t* src_at, const AlignnSchedule* sched,
            const float* QKV, int64_t ldq, const float* U, const float* wbar, const float* F, int64_t ldf,
            float* aggV, float* S, float* sumA, float* mstat, float* den, const DropParams& drop, hipStream_t s,
            const uint16_t* KV16 = nullptr, int64_t ldkv = 0, const uint16_t* F16 = nullptr);
int lg3_bwd_dst(int64_t n, int64_t m, int H, const int32_t* off, const int32_t* src_at,
                const AlignnSchedule* sched, const float* QKV, int64_t ldq, const float* U, const float* Vd,
                const float* wbar, const float* F, int64_t ldf, const float* dout, const float* outp,
                const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e,
                float* alpha_e, const DropParams& drop, hipStream_t s, const uint16_t* KV16 = nullptr,
                int64_t ldkv = 0, const uint16_t* F16 = nullptr);

}  // namespace alignn

using namespace alignn;

// bf16 feature rows: the light/heavy kernels only, rows 8-byte aligned for the 4-wide bf16 loads
static int check_fbf(const void* F, int64_t ldf, int32_t D, const char* what) {
  if ((D % 4) || (ldf % 4) || (reinterpret_cast<uintptr_t>(F) & 7)) {
    set_error("%s: bf16 edge-feature rows need D %% 4 == 0, ldf %% 4 == 0 and 8-byte alignment", what);
    return ALIGNN_E_BAD_SHAPE;
  }
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_fwd_ex(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                   const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                   const float* QKVR, int64_t ldq, const float* U, const float* wbar, const void* F,
                                   int64_t ldf, int32_t f_bf16, float* aggV, float* S, float* sumA, float* mstat,
                                   float* den, float drop_p, uint64_t seed, void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  if (F == nullptr) {
    set_error("tconv_fwd: edge features F are required");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (f_bf16 && (rc = check_fbf(F, ldf, D, "tconv_fwd"))) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* Ff = reinterpret_cast<const float*>(F);
  if (!f_bf16 && lg3_supported(D, H, feat_row, Ff, sched))
    return lg3_fwd(n, m, H, off_dst, src_at, sched, QKVR, ldq, U, wbar, Ff, ldf, aggV, S, sumA, mstat, den,
                   make_drop(drop_p, seed), s);
  FwdParams p{n, m, D, 0, off_dst, src_at, feat_row, QKVR, ldq, U, wbar, Ff, ldf, aggV, S, sumA, mstat, den,
              make_drop(drop_p, seed)};
  p.fbf = f_bf16 ? 1 : 0;
  const Sched sc = make_sched(sched, n);
  ALIGNN_DISPATCH_VH(vpl_for(D), H, launch_fwd, p, sc, s);
  ALIGNN_LAUNCH_CHECK("tconv_fwd2_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_fwd(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                const float* QKVR, int64_t ldq, const float* U, const float* wbar, const float* F,
                                int64_t ldf, float* aggV, float* S, float* sumA, float* mstat, float* den,
                                float drop_p, uint64_t seed, void* stream) {
  return alignn_tconv_fwd_ex(n, m, D, H, off_dst, src_at, feat_row, sched, QKVR, ldq, U, wbar, F, ldf, 0, aggV, S,
                             sumA, mstat, den, drop_p, seed, stream);
}

extern "C" int alignn_tconv_family(int32_t D, int32_t H, const int32_t* feat_row, const float* F,
                                   const AlignnSchedule* sched) {
  if (check_dims(D, H)) return 0;
  return lg3_supported(D, H, feat_row, F, sched) ? 3 : 2;
}

extern "C" int alignn_tconv_bwd_dst_ex(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                       const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                       const float* QKVR, int64_t ldq, const float* U, const float* Vd,
                                       const float* wbar, const void* F, int64_t ldf, int32_t f_bf16,
                                       const float* dout, const float* outp, const float* mstat, const float* den,
                                       float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e, float* alpha_e,
                                       float* dF, int64_t lddf, int32_t accumulate_dF, float drop_p, uint64_t seed,
                                       void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  if (F == nullptr) {
    set_error("tconv_bwd_dst: edge features F are required");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (f_bf16 && (rc = check_fbf(F, ldf, D, "tconv_bwd_dst"))) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* Ff = reinterpret_cast<const float*>(F);
  if (!f_bf16 && dF == nullptr && lg3_supported(D, H, feat_row, Ff, sched))
    return lg3_bwd_dst(n, m, H, off_dst, src_at, sched, QKVR, ldq, U, Vd, wbar, Ff, ldf, dout, outp, mstat, den, dq,
                       lddq, Sz, sigz, dz_e, alpha_e, make_drop(drop_p, seed), s);
  // accumulate_dF bit 2: dF is written as bf16 (the gradient of autocast's bf16 cast of the edge
  // features, train.py:325/:333 under :632-636); not with bit 0 (no bf16 read-modify-write)
  const int dfbf = (accumulate_dF >> 2) & 1;
  if (dfbf && (dF == nullptr || (accumulate_dF & 1) || lddf % 4 || (reinterpret_cast<uintptr_t>(dF) & 7))) {
    set_error("tconv_bwd_dst: a bf16 dF is write-only, 8-byte aligned rows (lddf %% 4 == 0)");
    return ALIGNN_E_BAD_SHAPE;
  }
  BwdDstParams p{n, m, D, 0, off_dst, src_at, feat_row, QKVR, ldq, U, Vd, wbar, Ff, ldf, dout, outp, mstat, den,
                 dq, lddq, Sz, sigz, dz_e, alpha_e, dF, lddf, accumulate_dF & 3, dfbf, make_drop(drop_p, seed)};
  p.fbf = f_bf16 ? 1 : 0;
  const Sched sc = make_sched(sched, n);
  ALIGNN_DISPATCH_VH(vpl_for(D), H, launch_bwd_dst, p, sc, s);
  ALIGNN_LAUNCH_CHECK("tconv_bwd_dst2_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_bwd_dst(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                    const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                    const float* QKVR, int64_t ldq, const float* U, const float* Vd,
                                    const float* wbar, const float* F, int64_t ldf, const float* dout,
                                    const float* outp, const float* mstat, const float* den, float* dq, int64_t lddq,
                                    float* Sz, float* sigz, float* dz_e, float* alpha_e, float* dF, int64_t lddf,
                                    int32_t accumulate_dF, float drop_p, uint64_t seed, void* stream) {
  return alignn_tconv_bwd_dst_ex(n, m, D, H, off_dst, src_at, feat_row, sched, QKVR, ldq, U, Vd, wbar, F, ldf, 0, dout,
                                 outp, mstat, den, dq, lddq, Sz, sigz, dz_e, alpha_e, dF, lddf, accumulate_dF, drop_p,
                                 seed, stream);
}

extern "C" int alignn_tconv_bwd_src(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_src,
                                    const int32_t* pos_src, const int32_t* dst_at, const float* QKVR, int64_t ldq,
                                    const float* dout, const float* dz_e, const float* alpha_e, float* dKV,
                                    int64_t lddkv, void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  BwdSrcParams p{n, m, D, 0, off_src, pos_src, dst_at, QKVR, ldq, dout, dz_e, alpha_e, dKV, lddkv, nullptr};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  ALIGNN_DISPATCH_VH(vpl, H, launch_bwd_src, p, s);
  ALIGNN_LAUNCH_CHECK("tconv_bwd_src_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_bwd_src_by(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_src,
                                       const int32_t* pos_src, const int32_t* dst_src, const float* QKVR,
                                       int64_t ldq, const float* dout, const float* dz_e, const float* alpha_e,
                                       float* dKV, int64_t lddkv, void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (!dst_src) {
    set_error("tconv_bwd_src_by: dst_src (dst_at[pos_src[i]]) is required");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n == 0) return ALIGNN_OK;
  BwdSrcParams p{n, m, D, 0, off_src, pos_src, nullptr, QKVR, ldq, dout, dz_e, alpha_e, dKV, lddkv, dst_src};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  ALIGNN_DISPATCH_VH(vpl, H, launch_bwd_src, p, s);
  ALIGNN_LAUNCH_CHECK("tconv_bwd_src2_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_bwd_src_by_bf16(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_src,
                                            const int32_t* pos_src, const int32_t* dst_src, const uint16_t* Q16,
                                            int64_t ldq16, const uint16_t* dout16, const float* dz_e,
                                            const float* alpha_e, float* dKV, int64_t lddkv, void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (!dst_src || !Q16 || !dout16) {
    set_error("tconv_bwd_src_by_bf16: dst_src, Q16 and dout16 are required");
    return ALIGNN_E_BAD_SHAPE;
  }
  if ((D % 4) || (ldq16 % 4) || (reinterpret_cast<uintptr_t>(Q16) & 7) || (reinterpret_cast<uintptr_t>(dout16) & 7)) {
    set_error("tconv_bwd_src_by_bf16: bf16 rows need D %% 4 == 0, ldq16 %% 4 == 0 and 8-byte alignment");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n == 0) return ALIGNN_OK;
  BwdSrcParams p{n, m, D, 0, off_src, pos_src, nullptr, nullptr, 0, nullptr, dz_e, alpha_e, dKV, lddkv, dst_src,
                 Q16, ldq16, dout16};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  ALIGNN_DISPATCH_VH(vpl, H, launch_bwd_src, p, s);
  ALIGNN_LAUNCH_CHECK("tconv_bwd_src2_bf16_kernel");
  return ALIGNN_OK;
}
