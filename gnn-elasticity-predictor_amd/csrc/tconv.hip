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
#include "common.h"
#include "vec.h"

namespace alignn {

struct FwdParams {
  int64_t n, m;
  int D;
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

// ---------------------------------------------------------------------------------------------
// Work decomposition.  Light target nodes (in-degree <= heavy threshold) get one wave each, four
// per workgroup; heavy nodes get a whole workgroup whose four waves take interleaved groups of PF
// edges and merge their partial states through LDS in fixed wave order (deterministic).  The
// node lists come from the caller (AlignnSchedule); without one every node is light.
// Edges are processed in groups of PF: the operands of the next group are in flight while the
// current one computes, and the PF*H (or 2*PF*H) per-head dot products of a group are reduced
// across the wave together (reduce_bcast: one transpose-reduction, then scalar broadcasts).
// ---------------------------------------------------------------------------------------------
constexpr int PF = 4;

template <int VPL>
struct EdgeSlot {
  float k[VPL], v[VPL], f[VPL];
};

template <int VPL>
__device__ __forceinline__ void load_edge(EdgeSlot<VPL>& e, const float* __restrict__ QKVR, int64_t ldq, int D,
                                          const float* __restrict__ F, int64_t ldf, int64_t src, int64_t row, int j0) {
  vload(QKVR + src * ldq + D + j0, e.k);
  vload(QKVR + src * ldq + 2 * D + j0, e.v);
  vload(F + row * ldf + j0, e.f);
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

// Wave offset inside a heavy node's workgroup (0 for light nodes): groups g = wsub, wsub+nw, ...
struct NodeWork {
  int64_t d;
  int wsub, nw;
  bool valid;
};

__device__ __forceinline__ NodeWork node_work(const int32_t* __restrict__ nodes, int64_t count, int heavy) {
  NodeWork w;
  const int wave = threadIdx.x >> 6;
  if (heavy) {
    w.valid = blockIdx.x < count;
    w.d = w.valid ? (int64_t)(nodes ? nodes[blockIdx.x] : blockIdx.x) : 0;
    w.wsub = wave;
    w.nw = 4;
  } else {
    const int64_t i = (int64_t)blockIdx.x * 4 + wave;
    w.valid = i < count;
    w.d = w.valid ? (int64_t)(nodes ? nodes[i] : i) : 0;
    w.wsub = 0;
    w.nw = 1;
  }
  return w;
}

template <int VPL, int H, bool HEAVY>
__global__ __launch_bounds__(256) void tconv_fwd_kernel(FwdParams p, const int32_t* __restrict__ nodes, int64_t count) {
  constexpr int NS = 3 * H + H * VPL + VPL;  // per-lane merge state: m, s, sa, accS, accV
  __shared__ float merge[HEAVY ? 4 * 64 * NS : 1];
  constexpr bool heavy = HEAVY;
  const int lane = threadIdx.x & 63;
  const NodeWork w = node_work(nodes, count, heavy);
  if (!heavy && !w.valid) return;  // wave-uniform
  const int64_t d = w.d;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);
  const int32_t beg = w.valid ? p.off[d] : 0, end = w.valid ? p.off[d + 1] : 0;

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

  const int32_t first = beg + w.wsub * PF, stride = w.nw * PF;
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
      const int32_t t = first + j;
      if (t < end && act)
        load_edge(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, (int64_t)p.src_at[t], p.feat_row ? (int64_t)p.feat_row[t] : t, j0);
    }
    for (int32_t tb = first; tb < end; tb += stride) {
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
        const float cl = pick<H>(corr, hl);
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
        const float el = pick<H>(ed, hl);
#pragma unroll
        for (int i = 0; i < VPL; ++i) accV[i] = fmaf(el, ring[j].v[i], accV[i]);
        const int32_t tn = tb + stride + j;
        if (tn < end && act)
          load_edge(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, (int64_t)p.src_at[tn],
                    p.feat_row ? (int64_t)p.feat_row[tn] : tn, j0);
      }
    }
  }

  if (heavy) {
    // merge the four waves' states in wave order through LDS (wave 0 writes the node)
    const int wave = threadIdx.x >> 6;
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
    if (wave != 0 || !w.valid) return;
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
      const float f = (mh == -INFINITY) ? 0.f : __expf(mh - pick<H>(m, hl));
#pragma unroll
      for (int i = 0; i < VPL; ++i) accV[i] = fmaf(o[3 * H + H * VPL + i], f, accV[i]);
    }
  }

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
    const float il = pick<H>(inv, hl);
    float o[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) o[i] = accV[i] * il;
    vstore(p.aggV + d * D + j0, o);
  }
  if (lane < H) {
    p.sumA[d * H + lane] = pick<H>(sa, lane) * pick<H>(inv, lane);
    p.mstat[d * H + lane] = pick<H>(m, lane);
    p.den[d * H + lane] = pick<H>(dn, lane);
  }
}

struct BwdDstParams {
  int64_t n, m;
  int D;
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
  float* dF; int64_t lddf; int acc_dF;
  DropParams drop;
};

template <int VPL, int H, bool HEAVY>
__global__ __launch_bounds__(256) void tconv_bwd_dst_kernel(BwdDstParams p, const int32_t* __restrict__ nodes,
                                                            int64_t count) {
  constexpr int NS = H + H * VPL + VPL;  // per-lane merge state: sigz, Sz, dq
  __shared__ float merge[HEAVY ? 4 * 64 * NS : 1];
  const int lane = threadIdx.x & 63;
  const NodeWork w = node_work(nodes, count, HEAVY);
  if (!HEAVY && !w.valid) return;
  const int64_t d = w.d;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);
  const int32_t beg = w.valid ? p.off[d] : 0, end = w.valid ? p.off[d + 1] : 0;

  float sz[H][VPL], sgz[H], dqa[VPL];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    vzero(sz[h]);
    sgz[h] = 0.f;
  }
  vzero(dqa);

  const int32_t first = beg + w.wsub * PF, stride = w.nw * PF;
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
    float old[PF][VPL];  // dF rows being accumulated (prefetched with the operands)
    int64_t rows[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      vzero(ring[j].k); vzero(ring[j].v); vzero(ring[j].f);
      vzero(old[j]);
      const int32_t t = first + j;
      rows[j] = 0;
      if (t < end) {
        rows[j] = p.feat_row ? p.feat_row[t] : t;
        if (act) {
          load_edge(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, (int64_t)p.src_at[t], rows[j], j0);
          if (p.dF && (p.acc_dF & 1)) vload(p.dF + rows[j] * p.lddf + j0, old[j]);
        }
      }
    }
    for (int32_t tb = first; tb < end; tb += stride) {
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
          const float dzl = pick<H>(dz, hl);
#pragma unroll
          for (int i = 0; i < VPL; ++i) dqa[i] = fmaf(dzl, ring[j].k[i], dqa[i]);
          if (p.dF && act) {
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
          if (lane < H) {
            p.dz_e[(int64_t)t * H + lane] = pick<H>(dz, lane);
            p.alpha_e[(int64_t)t * H + lane] = pick<H>(al, lane);
          }
        }
        const int32_t tn = tb + stride + j;
        if (tn < end) {
          rows[j] = p.feat_row ? p.feat_row[tn] : tn;
          if (act) {
            load_edge(ring[j], p.QKVR, p.ldq, D, p.F, p.ldf, (int64_t)p.src_at[tn], rows[j], j0);
            if (p.dF && (p.acc_dF & 1)) vload(p.dF + rows[j] * p.lddf + j0, old[j]);
          }
        }
      }
    }
  }
  if (HEAVY) {
    const int wave = threadIdx.x >> 6;
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
    if (wave != 0 || !w.valid) return;
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
  if (act) {
    vstore(p.dq + d * p.lddq + j0, dqa);
#pragma unroll
    for (int h = 0; h < H; ++h) vstore(p.Sz + (d * H + h) * D + j0, sz[h]);
  }
  if (lane < H) p.sigz[d * H + lane] = pick<H>(sgz, lane);
}

struct BwdSrcParams {
  int64_t n, m;
  int D;
  const int32_t* off_src;
  const int32_t* pos_src;
  const int32_t* dst_at;
  const float* QKVR; int64_t ldq;
  const float* dout;
  const float* dz_e;
  const float* alpha_e;
  float* dKV; int64_t lddkv;
};

template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_bwd_src_kernel(BwdSrcParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= p.n) return;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  float dk[VPL], dv[VPL];
  vzero(dk);
  vzero(dv);
  const int32_t beg = p.off_src[s], end = p.off_src[s + 1];
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
          const int64_t pos = p.pos_src[ib + j];
          const int64_t dd = p.dst_at[pos];
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

#define ALIGNN_DISPATCH(VPL_, H_, FN, ...)                                           \
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

struct Sched {
  const int32_t* light;
  int64_t n_light;
  const int32_t* heavy;
  int64_t n_heavy;
};

template <int VPL, int H>
static void launch_fwd(const FwdParams& p, const Sched& sc, hipStream_t s) {
  if (sc.n_light > 0)
    hipLaunchKernelGGL((tconv_fwd_kernel<VPL, H, false>), dim3((unsigned)((sc.n_light + 3) / 4)), dim3(256), 0, s, p,
                       sc.light, sc.n_light);
  if (sc.n_heavy > 0)
    hipLaunchKernelGGL((tconv_fwd_kernel<VPL, H, true>), dim3((unsigned)sc.n_heavy), dim3(256), 0, s, p, sc.heavy,
                       sc.n_heavy);
}
template <int VPL, int H>
static void launch_bwd_dst(const BwdDstParams& p, const Sched& sc, hipStream_t s) {
  if (sc.n_light > 0)
    hipLaunchKernelGGL((tconv_bwd_dst_kernel<VPL, H, false>), dim3((unsigned)((sc.n_light + 3) / 4)), dim3(256), 0, s,
                       p, sc.light, sc.n_light);
  if (sc.n_heavy > 0)
    hipLaunchKernelGGL((tconv_bwd_dst_kernel<VPL, H, true>), dim3((unsigned)sc.n_heavy), dim3(256), 0, s, p, sc.heavy,
                       sc.n_heavy);
}
template <int VPL, int H>
static void launch_bwd_src(const BwdSrcParams& p, hipStream_t s) {
  hipLaunchKernelGGL((tconv_bwd_src_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
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
  if (D <= 0 || H <= 0 || D % H != 0 || vpl_for(D) == 0 || (D < 64 && D % 1 != 0)) {
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

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_tconv_fwd(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                const float* QKVR, int64_t ldq,
                                const float* U, const float* wbar, const float* F, int64_t ldf, float* aggV,
                                float* S, float* sumA, float* mstat, float* den, float drop_p, uint64_t seed,
                                void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  FwdParams p{n, m, D, off_dst, src_at, feat_row, QKVR, ldq, U, wbar, F, ldf, aggV, S, sumA, mstat, den,
              make_drop(drop_p, seed)};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  const Sched sc = make_sched(sched, n);
  ALIGNN_DISPATCH(vpl, H, launch_fwd, p, sc, s);
  ALIGNN_LAUNCH_CHECK("tconv_fwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_bwd_dst(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                    const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                                    const float* QKVR, int64_t ldq,
                                    const float* U, const float* Vd, const float* wbar, const float* F, int64_t ldf,
                                    const float* dout, const float* outp, const float* mstat, const float* den,
                                    float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e, float* alpha_e,
                                    float* dF, int64_t lddf, int32_t accumulate_dF, float drop_p, uint64_t seed,
                                    void* stream) {
  int rc = check_dims(D, H);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  BwdDstParams p{n, m, D, off_dst, src_at, feat_row, QKVR, ldq, U, Vd, wbar, F, ldf, dout, outp, mstat, den,
                 dq, lddq, Sz, sigz, dz_e, alpha_e, dF, lddf, accumulate_dF, make_drop(drop_p, seed)};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  const Sched sc = make_sched(sched, n);
  ALIGNN_DISPATCH(vpl, H, launch_bwd_dst, p, sc, s);
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
  BwdSrcParams p{n, m, D, off_src, pos_src, dst_at, QKVR, ldq, dout, dz_e, alpha_e, dKV, lddkv};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vpl = vpl_for(D);
  ALIGNN_DISPATCH(vpl, H, launch_bwd_src, p, s);
  ALIGNN_LAUNCH_CHECK("tconv_bwd_src_kernel");
  return ALIGNN_OK;
}
