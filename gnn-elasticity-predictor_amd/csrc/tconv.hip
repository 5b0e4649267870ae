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
// Edge encoder (line graph): the edge features are the angle encoder's hidden layer
// f_t = relu(W1 x_t + b1) (train.py:353-356 first Linear+ReLU; its second Linear is folded into M).
// With KM > 0 the kernels recompute f_t from the raw angle features x_t (kin <= KM <= 16 floats per
// edge; W1/b1 staged in LDS) instead of reading a materialised [m, D] array, and the backward
// accumulates dW1 = sum_t (relu'(.) * g_t) x_t^T and db1 = sum_t relu'(.) * g_t directly (g_t = the
// gradient w.r.t. f_t), so the [m, D] hidden layer and its gradient never exist in HBM.
#include "common.h"
#include "vec.h"

namespace alignn {

// ---------------------------------------------------------------------------------------------
// Work decomposition.  Work items: heavy target nodes (in-degree > threshold, one workgroup of
// four waves each; the waves take interleaved groups of PF edges and merge through LDS in fixed
// wave order), then light nodes four per workgroup (one wave each).  Heavy items come first so
// the long ones start early.  Workgroups walk the item list with a grid stride (a bounded grid
// when per-workgroup gradient partials are produced).  Edges are processed in groups of PF: the
// operands of the next group are in flight while the current one computes, and the PF*H (or
// 2*PF*H) per-head dot products of a group are reduced across the wave together (reduce_bcast).
// ---------------------------------------------------------------------------------------------
#ifndef ALIGNN_PF
#define ALIGNN_PF 4
#endif
#ifndef ALIGNN_BWD_RING2
#define ALIGNN_BWD_RING2 0  // two groups in flight in bwd_dst: 245 VGPRs + SGPR spills, -1.4 % (v38_ab_bwd_dst_ring2_rejected.log)
#endif
constexpr int PF = ALIGNN_PF;

struct Sched {
  const int32_t* light;
  int64_t n_light;
  const int32_t* heavy;
  int64_t n_heavy;
  __host__ __device__ int64_t items() const { return n_heavy + (n_light + 3) / 4; }
};

struct EncParams {
  const float* x; int64_t ldx; int kin; int pad_;
  const float* w1;  // [D, kin] (nn.Linear weight)
  const float* b1;  // [D]
};

template <int VPL>
struct EdgeSlot {
  float k[VPL], v[VPL], f[VPL];
  float xr;  // KM > 0: lane (l & 15) holds x_t[l & 15]
};

template <int VPL, int KM>
__device__ __forceinline__ void load_edge(EdgeSlot<VPL>& e, const float* __restrict__ QKVR, int64_t ldq, int D,
                                          const float* __restrict__ F, int64_t ldf, const EncParams& en,
                                          int64_t src, int64_t row, int j0, bool act, int lane) {
  if (act) {
    vload(QKVR + src * ldq + D + j0, e.k);
    vload(QKVR + src * ldq + 2 * D + j0, e.v);
    if constexpr (KM == 0) vload(F + row * ldf + j0, e.f);
  }
  if constexpr (KM > 0) {
    const int c = lane & 15;
    e.xr = c < en.kin ? en.x[row * en.ldx + c] : 0.f;
  }
}

// Encoder weights in LDS: ew[k*D + j] = W1[j, k] (zero rows for kin <= k < KM), ew[KM*D + j] = b1[j].
template <int VPL, int KM>
__device__ __forceinline__ void stage_enc(float* ew, const EncParams& en, int D) {
  for (int i = threadIdx.x; i < (KM + 1) * D; i += blockDim.x) {
    const int k = i / D, j = i - k * D;
    float v;
    if (k < KM) v = k < en.kin ? en.w1[(int64_t)j * en.kin + k] : 0.f;
    else v = en.b1[j];
    ew[i] = v;
  }
  __syncthreads();
}

// f[j] = relu(b1 + W1 x_j) for the PF slots of a group (this lane's VPL features).
template <int VPL, int KM>
__device__ __forceinline__ void enc_group(const float* ew, int D, int j0, EdgeSlot<VPL> (&ring)[PF]) {
  float b[VPL];
  vload(ew + KM * D + j0, b);
#pragma unroll
  for (int j = 0; j < PF; ++j)
#pragma unroll
    for (int i = 0; i < VPL; ++i) ring[j].f[i] = b[i];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    float w[VPL];
    vload(ew + k * D + j0, w);
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const float xk = readlane_f(ring[j].xr, k);
#pragma unroll
      for (int i = 0; i < VPL; ++i) ring[j].f[i] = fmaf(xk, w[i], ring[j].f[i]);
    }
  }
#pragma unroll
  for (int j = 0; j < PF; ++j)
#pragma unroll
    for (int i = 0; i < VPL; ++i) ring[j].f[i] = fmaxf(ring[j].f[i], 0.f);
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
};

template <int VPL, int H>
constexpr int fwd_merge_floats() { return 4 * 64 * (3 * H + H * VPL + VPL); }

// One target node.  heavy: all four waves of the workgroup call this for the same d (wsub =
// wave, nw = 4) and merge; light: one wave (wsub = 0, nw = 1).
template <int VPL, int H, int KM>
__device__ __forceinline__ void fwd_node(const FwdParams& p, const EncParams& en, const float* ew, float* merge,
                                         int64_t d, int wsub, int nw, bool heavy) {
  constexpr int NS = 3 * H + H * VPL + VPL;  // per-lane merge state: m, s, sa, accS, accV
  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));

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
    float q[VPL], u[H][VPL];
    vzero(q);
#pragma unroll
    for (int h = 0; h < H; ++h) vzero(u[h]);
    if (act) {
      vload(p.QKVR + d * p.ldq + j0, q);
#pragma unroll
      for (int h = 0; h < H; ++h) vload(p.U + (d * H + h) * D + j0, u[h]);
    }
    float c[H];
#pragma unroll
    for (int h = 0; h < H; ++h) c[h] = 0.f;
    if (p.wbar) {
      float wb[VPL];
      vzero(wb);
      if (act) vload(p.wbar + j0, wb);
      const float part = vdot(wb, q);
#pragma unroll
      for (int h = 0; h < H; ++h) c[h] = (h == hl) ? part : 0.f;
      reduce_bcast<H>(c, lane);
    }
    EdgeSlot<VPL> ring[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      vzero(ring[j].k); vzero(ring[j].v); vzero(ring[j].f);
      ring[j].xr = 0.f;
      const int32_t t = first + j;
      if (t < end)
        load_edge<VPL, KM>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, en, (int64_t)uni(sld(p.src_at, t)),
                           p.feat_row ? (int64_t)uni(sld(p.feat_row, t)) : t, j0, act, lane);
    }
    for (int32_t tb = first; tb < end; tb += stride) {
      if constexpr (KM > 0) enc_group<VPL, KM>(ew, D, j0, ring);
      // all PF*H scores of the group in one reduction
      float pr[PF * H];
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const float qk = vdot(q, ring[j].k);
#pragma unroll
        for (int h = 0; h < H; ++h) pr[j * H + h] = vdot(u[h], ring[j].f) + ((h == hl) ? qk : 0.f);
      }
      reduce_bcast<PF * H>(pr, lane);
      float mul[PF][H];
      group_dropout<H>(p.drop, tb, lane, mul);
      // group-wise online softmax: one rescale per group
      float z[PF][H], corr[H];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        float mn = m[h];
#pragma unroll
        for (int j = 0; j < PF; ++j) {
          z[j][h] = (tb + j < end) ? (pr[j * H + h] + c[h]) * scale : -INFINITY;
          mn = fmaxf(mn, z[j][h]);
        }
        corr[h] = __expf(m[h] - mn);
        m[h] = mn;
        s[h] *= corr[h];
        sa[h] *= corr[h];
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
        float ed[H];
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const float ex = __expf(z[j][h] - m[h]);  // 0 for padded slots
          s[h] += ex;
          ed[h] = ex * mul[j][h];
          sa[h] += ed[h];
#pragma unroll
          for (int i = 0; i < VPL; ++i) accS[h][i] = fmaf(ed[h], ring[j].f[i], accS[h][i]);
        }
        const float el = pick_r<H>(ed, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) accV[i] = fmaf(el, ring[j].v[i], accV[i]);
        const int32_t tn = tb + stride + j;
        if (tn < end)
          load_edge<VPL, KM>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, en, (int64_t)uni(sld(p.src_at, tn)),
                             p.feat_row ? (int64_t)uni(sld(p.feat_row, tn)) : tn, j0, act, lane);
      }
    }
  }

  if (heavy) {
    // merge the four waves' states in wave order through LDS (wave 0 writes the node)
    float* my = merge + (wave * 64 + lane) * NS;
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
        for (int v = 0; v < 4; ++v) mt = fmaxf(mt, merge[(v * 64 + lane) * NS + h]);
        s[h] = 0.f;
        sa[h] = 0.f;
#pragma unroll
        for (int i = 0; i < VPL; ++i) accS[h][i] = 0.f;
        for (int v = 0; v < 4; ++v) {
          const float* o = merge + (v * 64 + lane) * NS;
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
        const float* o = merge + (v * 64 + lane) * NS;
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
  if (heavy) __syncthreads();  // merge buffer free for the next item
}

template <int VPL, int H, int KM>
__global__ TCONV_ATTR void tconv_fwd_kernel(FwdParams p, Sched sc, EncParams en) {
  resolve_drop(p.drop);
  constexpr int MERGE = fwd_merge_floats<VPL, H>();
  constexpr int ENCW = KM > 0 ? (KM + 1) * 64 * VPL : 0;
  __shared__ float smem[MERGE + ENCW];
  float* ew = smem + MERGE;
  const int wave = wave_id();
  const int64_t items = sc.items();
  bool staged = false;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    if constexpr (KM > 0) {
      // stage the encoder weights once, and only for items with edges (light lists end with the
      // in-degree-0 nodes, so an item whose first node is empty is empty)
      if (!staged) {
        bool need = it < sc.n_heavy;
        if (!need) {
          const int64_t i0 = (it - sc.n_heavy) * 4;
          const int64_t d0 = sc.light ? (int64_t)sc.light[i0] : i0;
          need = p.off[d0 + 1] > p.off[d0];
        }
        if (need) {
          stage_enc<VPL, KM>(ew, en, p.D);
          staged = true;
        }
      }
    }
    if (it < sc.n_heavy) {
      fwd_node<VPL, H, KM>(p, en, ew, smem, (int64_t)uni(sld(sc.heavy, it)), wave, 4, true);
    } else {
      const int64_t i = (it - sc.n_heavy) * 4 + wave;
      if (i < sc.n_light) fwd_node<VPL, H, KM>(p, en, ew, smem, sc.light ? (int64_t)uni(sld(sc.light, i)) : i, 0, 1, false);
    }
  }
}

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
  float* dF; int64_t lddf; int acc_dF, pad2_;
  DropParams drop;
};

template <int VPL, int H, int KM>
constexpr int bwd_merge_floats() {
  return cmax(4 * 64 * (H + H * VPL + VPL), KM > 0 ? (KM + 1) * 64 * VPL : 0);
}

template <int VPL, int KM>
struct EncAcc {
  float w[KM > 0 ? KM : 1][VPL];
  float b[VPL];
};

template <int VPL, int H, int KM>
__device__ __forceinline__ void bwd_dst_node(const BwdDstParams& p, const EncParams& en, const float* ew,
                                             float* merge, int64_t d, int wsub, int nw, bool heavy,
                                             EncAcc<VPL, KM>& ea) {
  constexpr int NS = H + H * VPL + VPL;  // per-lane merge state: sigz, Sz, dq
  const int lane = threadIdx.x & 63;
  const int wave = wave_id();
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));
  const bool do_dF = KM == 0 && p.dF != nullptr;

  float sz[H][VPL], sgz[H], dqa[VPL];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    vzero(sz[h]);
    sgz[h] = 0.f;
  }
  vzero(dqa);

  const int32_t first = beg + wsub * PF, stride = nw * PF;
  if (first < end) {
    float q[VPL], go[VPL], u[H][VPL], vd[H][VPL];
    vzero(q); vzero(go);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      vzero(u[h]);
      vzero(vd[h]);
    }
    float c[3 * H];  // c = <w̄_h, Q_h>, c2 = <w̄_h, dout_h>, delta = <dout_h, outp_h>
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
          vload(p.U + (d * H + h) * D + j0, u[h]);
          vload(p.Vd + (d * H + h) * D + j0, vd[h]);
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
    }
    float mst[H], inv_den[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      mst[h] = p.mstat[d * H + h];
      inv_den[h] = 1.0f / p.den[d * H + h];
    }

    EdgeSlot<VPL> ring[PF];
    float old[KM == 0 ? PF : 1][VPL];  // dF rows being accumulated (prefetched with the operands)
    int64_t rows[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      vzero(ring[j].k); vzero(ring[j].v); vzero(ring[j].f);
      ring[j].xr = 0.f;
      if constexpr (KM == 0) vzero(old[j]);
      const int32_t t = first + j;
      rows[j] = 0;
      if (t < end) {
        rows[j] = p.feat_row ? uni(sld(p.feat_row, t)) : t;
        load_edge<VPL, KM>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, en, (int64_t)uni(sld(p.src_at, t)), rows[j], j0, act, lane);
        if constexpr (KM == 0)
          if (act && do_dF && (p.acc_dF & 1)) vload(p.dF + rows[j] * p.lddf + j0, old[j]);
      }
    }
    for (int32_t tb = first; tb < end; tb += stride) {
      if constexpr (KM > 0) enc_group<VPL, KM>(ew, D, j0, ring);
      float pr[2 * PF * H];  // [score | d alpha'] per (edge, head)
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const float qk = vdot(q, ring[j].k), gv = vdot(go, ring[j].v);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          pr[j * H + h] = vdot(u[h], ring[j].f) + ((h == hl) ? qk : 0.f);
          pr[PF * H + j * H + h] = vdot(vd[h], ring[j].f) + ((h == hl) ? gv : 0.f);
        }
      }
      reduce_bcast<2 * PF * H>(pr, lane);
      float mul[PF][H];
      group_dropout<H>(p.drop, tb, lane, mul);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int32_t t = tb + j;
        if (t < end) {
          float dz[H], al[H];
#pragma unroll
          for (int h = 0; h < H; ++h) {
            const float z = (pr[j * H + h] + c[h]) * scale;
            const float alpha = __expf(z - mst[h]) * inv_den[h];
            al[h] = alpha * mul[j][h];                                          // alpha' (dropped)
            const float dal = (pr[PF * H + j * H + h] + c[H + h]) * mul[j][h];  // d alpha (pre-dropout)
            dz[h] = alpha * (dal - c[2 * H + h]) * scale;                       // dz / sqrt(C)
            sgz[h] += dz[h];
#pragma unroll
            for (int i = 0; i < VPL; ++i) sz[h][i] = fmaf(dz[h], ring[j].f[i], sz[h][i]);
          }
          const float dzl = pick_r<H>(dz, hl);
#pragma unroll
          for (int i = 0; i < VPL; ++i) dqa[i] = fmaf(dzl, ring[j].k[i], dqa[i]);
#ifndef ALIGNN_NO_ENC_ACC
          if constexpr (KM > 0) {
            // g = relu'(.) * sum_h (dz u + alpha' Vd); dW1 += g x^T, db1 += g
            float g[VPL];
#pragma unroll
            for (int i = 0; i < VPL; ++i) {
              float a = 0.f;
#pragma unroll
              for (int h = 0; h < H; ++h) a = fmaf(dz[h], u[h][i], fmaf(al[h], vd[h][i], a));
              g[i] = ring[j].f[i] > 0.f ? a : 0.f;
              ea.b[i] += g[i];
            }
#pragma unroll
            for (int k = 0; k < KM; ++k) {
              const float xk = readlane_f(ring[j].xr, k);
#pragma unroll
              for (int i = 0; i < VPL; ++i) ea.w[k][i] = fmaf(xk, g[i], ea.w[k][i]);
            }
          } else
#endif
          if constexpr (KM == 0) {
            if (do_dF && act) {
              float df[VPL];
#pragma unroll
              for (int i = 0; i < VPL; ++i) {
                float a = old[j][i];
#pragma unroll
                for (int h = 0; h < H; ++h) a = fmaf(dz[h], u[h][i], fmaf(al[h], vd[h][i], a));
                // bit 1: F is a ReLU output (angle-encoder hidden) -> apply its backward mask now
                df[i] = (p.acc_dF & 2) ? (ring[j].f[i] > 0.f ? a : 0.f) : a;
              }
              vstore(p.dF + rows[j] * p.lddf + j0, df);
            }
          }
          if (lane < H) {
            p.dz_e[(int64_t)t * H + lane] = pick_r<H>(dz, lane);
            p.alpha_e[(int64_t)t * H + lane] = pick_r<H>(al, lane);
          }
        }
        const int32_t tn = tb + stride + j;
        if (tn < end) {
          rows[j] = p.feat_row ? uni(sld(p.feat_row, tn)) : tn;
          load_edge<VPL, KM>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, en, (int64_t)uni(sld(p.src_at, tn)), rows[j], j0, act,
                             lane);
          if constexpr (KM == 0)
            if (act && do_dF && (p.acc_dF & 1)) vload(p.dF + rows[j] * p.lddf + j0, old[j]);
        }
      }
    }
  }
  if (heavy) {
    float* my = merge + (wave * 64 + lane) * NS;
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
        const float* o = merge + (v * 64 + lane) * NS;
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

// part (KM > 0): per-workgroup encoder-gradient partials, [gridDim.x][(KM+1)*D] (rows k < KM: dW1
// column k, row KM: db1), summed in fixed order by enc_grad_reduce.
template <int VPL, int H, int KM>
__global__ TCONV_ATTR void tconv_bwd_dst_kernel(BwdDstParams p, Sched sc, EncParams en,
                                                            float* __restrict__ part) {
  resolve_drop(p.drop);
  constexpr int MERGE = bwd_merge_floats<VPL, H, KM>();
  constexpr int ENCW = KM > 0 ? (KM + 1) * 64 * VPL : 0;
  __shared__ float smem[MERGE + ENCW];
  float* ew = smem + MERGE;
  if constexpr (KM > 0) stage_enc<VPL, KM>(ew, en, p.D);
  const int wave = wave_id();
  const int lane = threadIdx.x & 63;
  EncAcc<VPL, KM> ea;
  if constexpr (KM > 0) {
#pragma unroll
    for (int k = 0; k < KM; ++k) vzero(ea.w[k]);
    vzero(ea.b);
  }
  const int64_t items = sc.items();
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    if (it < sc.n_heavy) {
      bwd_dst_node<VPL, H, KM>(p, en, ew, smem, (int64_t)uni(sld(sc.heavy, it)), wave, 4, true, ea);
    } else {
      const int64_t i = (it - sc.n_heavy) * 4 + wave;
      if (i < sc.n_light)
        bwd_dst_node<VPL, H, KM>(p, en, ew, smem, sc.light ? (int64_t)uni(sld(sc.light, i)) : i, 0, 1, false, ea);
    }
  }
  if constexpr (KM > 0) {
    // fixed-order merge of the four waves' accumulators, then one partial row block per workgroup
    constexpr int RS = 64 * VPL;  // LDS row stride
    const int j0 = lane * VPL;
    __syncthreads();
    for (int w = 0; w < 4; ++w) {
      if (wave == w) {
#pragma unroll
        for (int k = 0; k <= KM; ++k) {
          const float* a = k < KM ? ea.w[k < KM ? k : 0] : ea.b;
#pragma unroll
          for (int i = 0; i < VPL; ++i) {
            float* r = smem + k * RS + j0 + i;
            *r = (w == 0 ? 0.f : *r) + a[i];
          }
        }
      }
      __syncthreads();
    }
    const int D = p.D;
    float* out = part + (int64_t)blockIdx.x * (KM + 1) * D;
    for (int i = threadIdx.x; i < (KM + 1) * D; i += blockDim.x) {
      const int k = i / D, j = i - k * D;
      out[i] = smem[k * RS + j];
    }
  }
}

// dW1[j, k] (+)= sum_g part[g][k*D + j] (k < kin), db1[j] (+)= sum_g part[g][KM*D + j].
// Grid: ceil((kin+1)*D / 64) blocks of 4 row-lanes x 64 outputs.
__global__ __launch_bounds__(1024) void enc_grad_reduce(const float* __restrict__ part, int G, int KM, int D, int kin,
                                                        float* __restrict__ dw1, float* __restrict__ db1, int acc) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + tx;
  const bool ok = c < (int64_t)(kin + 1) * D;
  const int k = ok ? (int)(c / D) : 0;
  const int j = (int)(c - (int64_t)k * D);
  const int kk = k < kin ? k : KM;
  const int64_t stride = (int64_t)(KM + 1) * D;
  const float* src = part + kk * D + j;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (ok) {
    int g = ty;
    for (; g + 48 < G; g += 64) {
      s0 += src[g * stride];
      s1 += src[(g + 16) * stride];
      s2 += src[(g + 32) * stride];
      s3 += src[(g + 48) * stride];
    }
    for (; g < G; g += 16) s0 += src[g * stride];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && ok) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][tx];
    float* dst = k < kin ? dw1 + (int64_t)j * kin + k : db1 + j;
    *dst = acc ? *dst + t : t;
  }
}

// =============================================================================================
// Version 2 kernels (schedule flag ALIGNN_SCHED_COMPACT_REGS; materialised edge features only).
//
// Same arithmetic as above with a smaller register footprint, for more waves per SIMD on the
// latency-bound edge stream:
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

template <int VPL, int H>
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
    float q[VPL];
    vzero(q);
    if (act) {
      vload(p.QKVR + d * p.ldq + j0, q);
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
      float wb[VPL];
      vzero(wb);
      if (act) vload(p.wbar + j0, wb);
      const float part = vdot(wb, q);
#pragma unroll
      for (int h = 0; h < H; ++h) c[h] = (h == hl) ? part : 0.f;
      reduce_bcast<H>(c, lane);
    }
    EdgeSlot<VPL> ring[PF];
    const EncParams no_enc{nullptr, 0, 0, 0, nullptr, nullptr};
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      vzero(ring[j].k); vzero(ring[j].v); vzero(ring[j].f);
      ring[j].xr = 0.f;
      const int32_t t = first + j;
      if (t < end)
        load_edge<VPL, 0>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, no_enc, (int64_t)uni(sld(p.src_at, t)),
                          p.feat_row ? (int64_t)uni(sld(p.feat_row, t)) : t, j0, act, lane);
    }
    for (int32_t tb = first; tb < end; tb += stride) {
      asm volatile("" ::: "memory");  // keep the u reads in the loop (registers are the point)
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
          for (int j = 0; j < PF; ++j) pr[j * H + h] = vdot(u, ring[j].f) + ((h == hl) ? qk[j] : 0.f);
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
          for (int i = 0; i < VPL; ++i) accS[h][i] = fmaf(e[h], ring[j].f[i], accS[h][i]);
        }
        const float el = pick_r<H>(e, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) accV[i] = fmaf(el, ring[j].v[i], accV[i]);
        const int32_t tn = tb + stride + j;
        if (tn < end)
          load_edge<VPL, 0>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, no_enc, (int64_t)uni(sld(p.src_at, tn)),
                            p.feat_row ? (int64_t)uni(sld(p.feat_row, tn)) : tn, j0, act, lane);
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

template <int VPL, int H>
__global__ TCONV_ATTR void tconv_fwd2_kernel(FwdParams p, Sched sc) {
  resolve_drop(p.drop);
  __shared__ float smem[fwd2_lds_floats<VPL, H>()];
  const int wave = wave_id();
  const int64_t items = sc.items();
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    if (it < sc.n_heavy) {
      fwd2_node<VPL, H>(p, smem, (int64_t)uni(sld(sc.heavy, it)), wave, 4, true);
    } else {
      const int64_t i = (it - sc.n_heavy) * 4 + wave;
      if (i < sc.n_light) fwd2_node<VPL, H>(p, smem, sc.light ? (int64_t)uni(sld(sc.light, i)) : i, 0, 1, false);
    }
  }
}

template <int VPL, int H>
constexpr int bwd2_lds_floats() { return cmax(bwd_merge_floats<VPL, H, 0>(), 4 * 2 * H * 64 * VPL); }

template <int VPL, int H>
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
    EdgeSlot<VPL> ring[PF];
    float old[PF][VPL];
    int64_t rows_[PF];
    const EncParams no_enc{nullptr, 0, 0, 0, nullptr, nullptr};
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      vzero(ring[j].k); vzero(ring[j].v); vzero(ring[j].f);
      ring[j].xr = 0.f;
      vzero(old[j]);
      const int32_t t = first + j;
      rows_[j] = 0;
      if (t < end) {
        rows_[j] = p.feat_row ? uni(sld(p.feat_row, t)) : t;
        load_edge<VPL, 0>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, no_enc, (int64_t)uni(sld(p.src_at, t)), rows_[j], j0, act,
                          lane);
        if (act && do_dF && (p.acc_dF & 1)) vload(p.dF + rows_[j] * p.lddf + j0, old[j]);
      }
    }
#if ALIGNN_BWD_RING2
    // second group in flight: its K/V/F rows load while the current group is processed
    EdgeSlot<VPL> ring2[PF];
    int64_t rows2[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      vzero(ring2[j].k); vzero(ring2[j].v); vzero(ring2[j].f);
      ring2[j].xr = 0.f;
      const int32_t t = first + stride + j;
      rows2[j] = 0;
      if (t < end) {
        rows2[j] = p.feat_row ? uni(sld(p.feat_row, t)) : t;
        load_edge<VPL, 0>(ring2[j], p.QKVR, p.ldq, D, p.F, p.ldf, no_enc, (int64_t)uni(sld(p.src_at, t)), rows2[j], j0,
                          act, lane);
      }
    }
#endif
    for (int32_t tb = first; tb < end; tb += stride) {
      asm volatile("" ::: "memory");  // keep the u / Vd reads in the loop
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
            ps[j * H + h] = vdot(u, ring[j].f) + ((h == hl) ? qk[j] : 0.f);
            pd[j * H + h] = vdot(vd, ring[j].f) + ((h == hl) ? gv[j] : 0.f);
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
          for (int i = 0; i < VPL; ++i) sz[h][i] = fmaf(e[h], ring[j].f[i], sz[h][i]);
        }
        const float dzl = pick_r<H>(e, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) dqa[i] = fmaf(dzl, ring[j].k[i], dqa[i]);
      }
      if (do_dF) {
        // dF[row(t)] (+)= sum_h dz u_h + alpha' Vd_h, one head at a time from LDS
#pragma unroll
        for (int h = 0; h < H; ++h) {
          float u[VPL], vd[VPL];
          vload(uv + h * RS + j0, u);
          vload(uv + (H + h) * RS + j0, vd);
#pragma unroll
          for (int j = 0; j < PF; ++j) {
            const float ez = readlane_f(bs[h], 16 * j), ea = readlane_f(bd[h], 16 * j);
#pragma unroll
            for (int i = 0; i < VPL; ++i) old[j][i] = fmaf(ez, u[i], fmaf(ea, vd[i], old[j][i]));
          }
        }
#pragma unroll
        for (int j = 0; j < PF; ++j) {
          if (tb + j < end && act) {
            float df[VPL];
#pragma unroll
            for (int i = 0; i < VPL; ++i) df[i] = (p.acc_dF & 2) ? (ring[j].f[i] > 0.f ? old[j][i] : 0.f) : old[j][i];
            vstore(p.dF + rows_[j] * p.lddf + j0, df);
          }
        }
      }
#if ALIGNN_BWD_RING2
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int32_t tn = tb + stride + j, tn2 = tn + stride;
        ring[j] = ring2[j];
        rows_[j] = rows2[j];
        vzero(old[j]);
        if (tn < end && act && do_dF && (p.acc_dF & 1)) vload(p.dF + rows_[j] * p.lddf + j0, old[j]);
        if (tn2 < end) {
          rows2[j] = p.feat_row ? uni(sld(p.feat_row, tn2)) : tn2;
          load_edge<VPL, 0>(ring2[j], p.QKVR, p.ldq, D, p.F, p.ldf, no_enc, (int64_t)uni(sld(p.src_at, tn2)),
                            rows2[j], j0, act, lane);
        }
      }
#else
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int32_t tn = tb + stride + j;
        vzero(old[j]);
        if (tn < end) {
          rows_[j] = p.feat_row ? uni(sld(p.feat_row, tn)) : tn;
          load_edge<VPL, 0>(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, no_enc, (int64_t)uni(sld(p.src_at, tn)), rows_[j], j0,
                            act, lane);
          if (act && do_dF && (p.acc_dF & 1)) vload(p.dF + rows_[j] * p.lddf + j0, old[j]);
        }
      }
#endif
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

template <int VPL, int H>
__global__ TCONV_ATTR void tconv_bwd_dst2_kernel(BwdDstParams p, Sched sc) {
  resolve_drop(p.drop);
  __shared__ float smem[bwd2_lds_floats<VPL, H>()];
  const int wave = wave_id();
  const int64_t items = sc.items();
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    if (it < sc.n_heavy) {
      bwd2_node<VPL, H>(p, smem, (int64_t)uni(sld(sc.heavy, it)), wave, 4, true);
    } else {
      const int64_t i = (it - sc.n_heavy) * 4 + wave;
      if (i < sc.n_light) bwd2_node<VPL, H>(p, smem, sc.light ? (int64_t)uni(sld(sc.light, i)) : i, 0, 1, false);
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
template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_bwd_src2_kernel(BwdSrcParams p) {
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
        vload(p.QKVR + d * p.ldq + j0, qv[j]);
        vload(p.dout + d * D + j0, gv[j]);
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

// ---------------------------------------------------------------------------------------------
// Dispatch on (VPL, H, KM)
// ---------------------------------------------------------------------------------------------

static int vpl_for(int D) {
  if (D <= 64) return 1;
  if (D == 128) return 2;
  if (D == 256) return 4;
  if (D == 512) return 8;
  return 0;
}

static int km_for(int kin) {
  if (kin <= 0) return 0;
  if (kin <= 8) return 8;
  if (kin <= 12) return 12;
  if (kin <= 16) return 16;
  return -1;
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

static int g_num_cus = 0;
static int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_num_cus = n;
  }
  return g_num_cus;
}

// Resident workgroups of a kernel on the whole device (bounded grid for the partial-producing
// backward: its partial count, hence the reduction order, is fixed per device and shape).
template <typename K>
static int64_t resident_wgs(K kernel) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
  return (int64_t)per_cu * num_cus();
}

template <int VPL, int H, int KM>
static int64_t bwd_grid_cap() {
  static int64_t cap = 0;
  if (cap == 0) cap = resident_wgs(tconv_bwd_dst_kernel<VPL, H, KM>);
  return cap;
}

template <int VPL, int H>
static void launch_fwd(const FwdParams& p, const Sched& sc, const EncParams& en, int km, hipStream_t s,
                       int flags = 0) {
  const int64_t items = sc.items();
  if (items == 0) return;
  const dim3 grid((unsigned)items), block(256);
  if (km == 0 && (flags & ALIGNN_SCHED_COMPACT_REGS)) {
    launch((tconv_fwd2_kernel<VPL, H>), grid, block, 0, s, p, sc);
    return;
  }
  switch (km) {
    case 0: launch((tconv_fwd_kernel<VPL, H, 0>), grid, block, 0, s, p, sc, en); break;
    case 8: launch((tconv_fwd_kernel<VPL, H, 8>), grid, block, 0, s, p, sc, en); break;
    case 12: launch((tconv_fwd_kernel<VPL, H, 12>), grid, block, 0, s, p, sc, en); break;
    default: launch((tconv_fwd_kernel<VPL, H, 16>), grid, block, 0, s, p, sc, en); break;
  }
}

template <int VPL, int H, int KM>
static int launch_bwd_dst_km(const BwdDstParams& p, const Sched& sc, const EncParams& en,
                             const AlignnEdgeEncoder* enc, hipStream_t s, int flags = 0) {
  const int64_t items = sc.items();
  if (KM == 0 && (flags & ALIGNN_SCHED_COMPACT_REGS)) {
    if (items > 0)
      launch((tconv_bwd_dst2_kernel<VPL, H>), dim3((unsigned)items), dim3(256), 0, s, p, sc);
    return ALIGNN_OK;
  }
  if (KM == 0) {
    if (items > 0)
      launch((tconv_bwd_dst_kernel<VPL, H, 0>), dim3((unsigned)items), dim3(256), 0, s, p, sc, en,
                         nullptr);
    return ALIGNN_OK;
  }
  const int64_t per = (int64_t)(KM + 1) * p.D;
  int64_t G = bwd_grid_cap<VPL, H, KM>();
  if (items < G) G = items;
  if (G < 1) G = 1;
  if (enc->workspace_elems / per < G) G = enc->workspace_elems / per;
  if (G < 1 || enc->workspace == nullptr) {
    set_error("tconv_bwd_dst: encoder workspace too small (%lld floats, need >= %lld)",
              (long long)enc->workspace_elems, (long long)per);
    return ALIGNN_E_WORKSPACE;
  }
  launch((tconv_bwd_dst_kernel<VPL, H, KM>), dim3((unsigned)G), dim3(256), 0, s, p, sc, en,
                     enc->workspace);
  const int64_t outs = (int64_t)(en.kin + 1) * p.D;
  launch(enc_grad_reduce, dim3((unsigned)((outs + 63) / 64)), dim3(1024), 0, s, enc->workspace, (int)G,
                     KM, p.D, en.kin, enc->dw1, enc->db1, enc->accumulate);
  return ALIGNN_OK;
}

template <int VPL, int H>
static int launch_bwd_dst(const BwdDstParams& p, const Sched& sc, const EncParams& en, const AlignnEdgeEncoder* enc,
                          int km, hipStream_t s, int flags) {
  switch (km) {
    case 0: return launch_bwd_dst_km<VPL, H, 0>(p, sc, en, enc, s, flags);
    case 8: return launch_bwd_dst_km<VPL, H, 8>(p, sc, en, enc, s);
    case 12: return launch_bwd_dst_km<VPL, H, 12>(p, sc, en, enc, s);
    default: return launch_bwd_dst_km<VPL, H, 16>(p, sc, en, enc, s);
  }
}

template <int VPL, int H>
static int64_t bwd_ws_elems(int km, int D) {
  switch (km) {
    case 0: return 0;
    case 8: return bwd_grid_cap<VPL, H, 8>() * 9 * D;
    case 12: return bwd_grid_cap<VPL, H, 12>() * 13 * D;
    default: return bwd_grid_cap<VPL, H, 16>() * 17 * D;
  }
}

template <int VPL, int H>
static void launch_bwd_src(const BwdSrcParams& p, hipStream_t s) {
  if (p.dst_src) launch((tconv_bwd_src2_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
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

// Validates the edge-feature source: exactly one of F (materialised rows) or enc (recomputed).
static int edge_source(const float* F, const AlignnEdgeEncoder* enc, EncParams& en, int& km) {
  en = EncParams{nullptr, 0, 0, 0, nullptr, nullptr};
  km = 0;
  if (enc) {
    km = km_for(enc->kin);
    if (km <= 0 || !enc->x || !enc->w1 || !enc->b1 || enc->ldx < enc->kin) {
      set_error("tconv: edge encoder needs 1 <= kin <= 16, x (ldx >= kin), w1 and b1 (kin=%d)", (int)enc->kin);
      return ALIGNN_E_BAD_SHAPE;
    }
    en = EncParams{enc->x, enc->ldx, enc->kin, 0, enc->w1, enc->b1};
    return ALIGNN_OK;
  }
  if (!F) {
    set_error("tconv: edge features F are required when no edge encoder is given");
    return ALIGNN_E_BAD_SHAPE;
  }
  return ALIGNN_OK;
}

// lgconv.hip: single-wave-item kernels (ALIGNN_SCHED_WAVE_ITEMS)
bool lg3_supported(int D, int H, const int32_t* feat_row, const AlignnEdgeEncoder* enc, const float* F,
                   const AlignnSchedule* sched);
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

extern "C" int alignn_tconv_fwd(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                const float* QKVR, int64_t ldq, const float* U, const float* wbar, const float* F,
                                int64_t ldf, const AlignnEdgeEncoder* enc, float* aggV, float* S, float* sumA,
                                float* mstat, float* den, float drop_p, uint64_t seed, void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  EncParams en;
  int km;
  if ((rc = edge_source(F, enc, en, km))) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (lg3_supported(D, H, feat_row, enc, F, sched))
    return lg3_fwd(n, m, H, off_dst, src_at, sched, QKVR, ldq, U, wbar, F, ldf, aggV, S, sumA, mstat, den,
                   make_drop(drop_p, seed), s);
  FwdParams p{n, m, D, 0, off_dst, src_at, feat_row, QKVR, ldq, U, wbar, F, ldf, aggV, S, sumA, mstat, den,
              make_drop(drop_p, seed)};
  const int vpl = vpl_for(D);
  const Sched sc = make_sched(sched, n);
  const int flags = sched ? sched->flags : 0;
  ALIGNN_DISPATCH_VH(vpl, H, launch_fwd, p, sc, en, km, s, flags);
  ALIGNN_LAUNCH_CHECK("tconv_fwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_family(int32_t D, int32_t H, const int32_t* feat_row, const AlignnEdgeEncoder* enc,
                                   const float* F, const AlignnSchedule* sched) {
  if (check_dims(D, H)) return 0;
  if (lg3_supported(D, H, feat_row, enc, F, sched)) return 3;
  return (enc == nullptr && sched && (sched->flags & ALIGNN_SCHED_COMPACT_REGS)) ? 2 : 1;
}

extern "C" int64_t alignn_tconv_bwd_workspace(int32_t D, int32_t H, int32_t kin) {
  if (check_dims(D, H)) return -1;
  const int km = km_for(kin);
  if (km < 0) return -1;
  const int vpl = vpl_for(D);
  int64_t r = -1;
#define ALIGNN_WS(V_, H_) r = bwd_ws_elems<V_, H_>(km, D)
  if (vpl == 1 && H == 1) ALIGNN_WS(1, 1);
  else if (vpl == 1 && H == 2) ALIGNN_WS(1, 2);
  else if (vpl == 1 && H == 4) ALIGNN_WS(1, 4);
  else if (vpl == 2 && H == 1) ALIGNN_WS(2, 1);
  else if (vpl == 2 && H == 2) ALIGNN_WS(2, 2);
  else if (vpl == 2 && H == 4) ALIGNN_WS(2, 4);
  else if (vpl == 4 && H == 1) ALIGNN_WS(4, 1);
  else if (vpl == 4 && H == 2) ALIGNN_WS(4, 2);
  else if (vpl == 4 && H == 4) ALIGNN_WS(4, 4);
  else if (vpl == 4 && H == 8) ALIGNN_WS(4, 8);
  else if (vpl == 8 && H == 4) ALIGNN_WS(8, 4);
  else if (vpl == 8 && H == 8) ALIGNN_WS(8, 8);
#undef ALIGNN_WS
  return r;
}

extern "C" int alignn_tconv_bwd_dst(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                    const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                    const float* QKVR, int64_t ldq, const float* U, const float* Vd,
                                    const float* wbar, const float* F, int64_t ldf, const AlignnEdgeEncoder* enc,
                                    const float* dout, const float* outp, const float* mstat, const float* den,
                                    float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e, float* alpha_e,
                                    float* dF, int64_t lddf, int32_t accumulate_dF, float drop_p, uint64_t seed,
                                    void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  EncParams en;
  int km;
  if ((rc = edge_source(F, enc, en, km))) return rc;
  if (enc && (!enc->dw1 || !enc->db1)) {
    set_error("tconv_bwd_dst: edge encoder gradients dw1/db1 are required");
    return ALIGNN_E_BAD_SHAPE;
  }
  const int flags = sched ? sched->flags : 0;
  if (dF == nullptr && lg3_supported(D, H, feat_row, enc, F, sched))
    return lg3_bwd_dst(n, m, H, off_dst, src_at, sched, QKVR, ldq, U, Vd, wbar, F, ldf, dout, outp, mstat, den, dq,
                       lddq, Sz, sigz, dz_e, alpha_e, make_drop(drop_p, seed), reinterpret_cast<hipStream_t>(stream));
  BwdDstParams p{n, m, D, 0, off_dst, src_at, feat_row, QKVR, ldq, U, Vd, wbar, F, ldf, dout, outp, mstat, den,
                 dq, lddq, Sz, sigz, dz_e, alpha_e, enc ? nullptr : dF, lddf, accumulate_dF, 0,
                 make_drop(drop_p, seed)};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  const Sched sc = make_sched(sched, n);
  int lrc = ALIGNN_OK;
#define ALIGNN_BWD(V_, H_) lrc = launch_bwd_dst<V_, H_>(p, sc, en, enc, km, s, flags)
  if (vpl == 1 && H == 1) ALIGNN_BWD(1, 1);
  else if (vpl == 1 && H == 2) ALIGNN_BWD(1, 2);
  else if (vpl == 1 && H == 4) ALIGNN_BWD(1, 4);
  else if (vpl == 2 && H == 1) ALIGNN_BWD(2, 1);
  else if (vpl == 2 && H == 2) ALIGNN_BWD(2, 2);
  else if (vpl == 2 && H == 4) ALIGNN_BWD(2, 4);
  else if (vpl == 4 && H == 1) ALIGNN_BWD(4, 1);
  else if (vpl == 4 && H == 2) ALIGNN_BWD(4, 2);
  else if (vpl == 4 && H == 4) ALIGNN_BWD(4, 4);
  else if (vpl == 4 && H == 8) ALIGNN_BWD(4, 8);
  else if (vpl == 8 && H == 4) ALIGNN_BWD(8, 4);
  else if (vpl == 8 && H == 8) ALIGNN_BWD(8, 8);
  else {
    set_error("tconv: unsupported D/H combination");
    return ALIGNN_E_UNSUPPORTED;
  }
#undef ALIGNN_BWD
  if (lrc) return lrc;
  ALIGNN_LAUNCH_CHECK("tconv_bwd_dst_kernel");
  return ALIGNN_OK;
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
