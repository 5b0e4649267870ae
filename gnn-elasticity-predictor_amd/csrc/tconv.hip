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

template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_fwd_kernel(FwdParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t d = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= p.n) return;  // wave-uniform
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);

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
    reduce_heads<H>(c, lane);
  }

  float m[H], s[H], sa[H], accS[H][VPL], accV[VPL];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    m[h] = -INFINITY;
    s[h] = 0.f;
    sa[h] = 0.f;
    vzero(accS[h]);
  }
  vzero(accV);

  const int32_t beg = p.off[d], end = p.off[d + 1];
  float k_c[VPL], v_c[VPL], f_c[VPL];
  vzero(k_c); vzero(v_c); vzero(f_c);
  if (beg < end && act) {
    const int64_t s0 = p.src_at[beg];
    const int64_t r0 = p.feat_row ? p.feat_row[beg] : beg;
    vload(p.QKVR + s0 * p.ldq + D + j0, k_c);
    vload(p.QKVR + s0 * p.ldq + 2 * D + j0, v_c);
    vload(p.F + r0 * p.ldf + j0, f_c);
  }
  for (int32_t t = beg; t < end; ++t) {
    float k_n[VPL], v_n[VPL], f_n[VPL];
    vzero(k_n); vzero(v_n); vzero(f_n);
    if (t + 1 < end && act) {
      const int64_t s1 = p.src_at[t + 1];
      const int64_t r1 = p.feat_row ? p.feat_row[t + 1] : (t + 1);
      vload(p.QKVR + s1 * p.ldq + D + j0, k_n);
      vload(p.QKVR + s1 * p.ldq + 2 * D + j0, v_n);
      vload(p.F + r1 * p.ldf + j0, f_n);
    }
    float pr[H];
#pragma unroll
    for (int h = 0; h < H; ++h) pr[h] = vdot(u[h], f_c);
    const float qk = vdot(q, k_c);
#pragma unroll
    for (int h = 0; h < H; ++h) pr[h] += (h == hl) ? qk : 0.f;
    reduce_heads<H>(pr, lane);
    float corr[H], ed[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float z = (pr[h] + c[h]) * scale;
      const float mn = fmaxf(m[h], z);
      corr[h] = __expf(m[h] - mn);
      const float e = __expf(z - mn);
      s[h] = fmaf(s[h], corr[h], e);
      m[h] = mn;
      ed[h] = p.drop.active ? e * dropout_mul(p.drop.seed, (uint64_t)t * H + h, p.drop.thresh, p.drop.inv_keep) : e;
      sa[h] = fmaf(sa[h], corr[h], ed[h]);
#pragma unroll
      for (int i = 0; i < VPL; ++i) accS[h][i] = fmaf(accS[h][i], corr[h], ed[h] * f_c[i]);
    }
    const float cl = pick<H>(corr, hl), el = pick<H>(ed, hl);
#pragma unroll
    for (int i = 0; i < VPL; ++i) accV[i] = fmaf(accV[i], cl, el * v_c[i]);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      k_c[i] = k_n[i];
      v_c[i] = v_n[i];
      f_c[i] = f_n[i];
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

template <int VPL, int H>
__global__ __launch_bounds__(256) void tconv_bwd_dst_kernel(BwdDstParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t d = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= p.n) return;
  const int D = p.D, C = D / H;
  const int j0 = lane * VPL;
  const bool act = j0 < D;
  const int hl = act ? j0 / C : 0;
  const float scale = 1.0f / sqrtf((float)C);

  float q[VPL], go[VPL], op[VPL], u[H][VPL], vd[H][VPL];
  vzero(q); vzero(go); vzero(op);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    vzero(u[h]);
    vzero(vd[h]);
  }
  if (act) {
    vload(p.QKVR + d * p.ldq + j0, q);
    vload(p.dout + d * D + j0, go);
    vload(p.outp + d * D + j0, op);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      vload(p.U + (d * H + h) * D + j0, u[h]);
      vload(p.Vd + (d * H + h) * D + j0, vd[h]);
    }
  }
  // per-head constants: c = <w̄_h, Q_h>, c2 = <w̄_h, dout_h>, delta = <dout_h, outp_h>
  float c[H], c2[H], delta[H];
  {
    float wb[VPL];
    vzero(wb);
    if (p.wbar && act) vload(p.wbar + j0, wb);
    const float pc = vdot(wb, q), pc2 = vdot(wb, go), pdl = vdot(go, op);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      c[h] = (h == hl) ? pc : 0.f;
      c2[h] = (h == hl) ? pc2 : 0.f;
      delta[h] = (h == hl) ? pdl : 0.f;
    }
    reduce_heads<H>(c, lane);
    reduce_heads<H>(c2, lane);
    reduce_heads<H>(delta, lane);
  }
  float mst[H], inv_den[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    mst[h] = p.mstat[d * H + h];
    inv_den[h] = 1.0f / p.den[d * H + h];
  }

  float sz[H][VPL], sgz[H], dqa[VPL];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    vzero(sz[h]);
    sgz[h] = 0.f;
  }
  vzero(dqa);

  const int32_t beg = p.off[d], end = p.off[d + 1];
  float k_c[VPL], v_c[VPL], f_c[VPL];
  vzero(k_c); vzero(v_c); vzero(f_c);
  int64_t row_c = 0;
  if (beg < end) {
    row_c = p.feat_row ? p.feat_row[beg] : beg;
    if (act) {
      const int64_t s0 = p.src_at[beg];
      vload(p.QKVR + s0 * p.ldq + D + j0, k_c);
      vload(p.QKVR + s0 * p.ldq + 2 * D + j0, v_c);
      vload(p.F + row_c * p.ldf + j0, f_c);
    }
  }
  for (int32_t t = beg; t < end; ++t) {
    float k_n[VPL], v_n[VPL], f_n[VPL];
    vzero(k_n); vzero(v_n); vzero(f_n);
    int64_t row_n = 0;
    if (t + 1 < end) {
      row_n = p.feat_row ? p.feat_row[t + 1] : (t + 1);
      if (act) {
        const int64_t s1 = p.src_at[t + 1];
        vload(p.QKVR + s1 * p.ldq + D + j0, k_n);
        vload(p.QKVR + s1 * p.ldq + 2 * D + j0, v_n);
        vload(p.F + row_n * p.ldf + j0, f_n);
      }
    }
    float pz[H], pg[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      pz[h] = vdot(u[h], f_c);
      pg[h] = vdot(vd[h], f_c);
    }
    const float qk = vdot(q, k_c), gv = vdot(go, v_c);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      pz[h] += (h == hl) ? qk : 0.f;
      pg[h] += (h == hl) ? gv : 0.f;
    }
    reduce_heads<H>(pz, lane);
    reduce_heads<H>(pg, lane);
    float dz[H], al[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float z = (pz[h] + c[h]) * scale;
      const float alpha = __expf(z - mst[h]) * inv_den[h];
      const float mul = p.drop.active ? dropout_mul(p.drop.seed, (uint64_t)t * H + h, p.drop.thresh, p.drop.inv_keep) : 1.f;
      al[h] = alpha * mul;                      // alpha' (dropped, used in the aggregation)
      const float dal = (pg[h] + c2[h]) * mul;  // d alpha (pre-dropout)
      dz[h] = alpha * (dal - delta[h]) * scale;  // dz * (1/sqrt(C)): every consumer wants it scaled
      sgz[h] += dz[h];
#pragma unroll
      for (int i = 0; i < VPL; ++i) sz[h][i] = fmaf(dz[h], f_c[i], sz[h][i]);
    }
    const float dzl = pick<H>(dz, hl);
#pragma unroll
    for (int i = 0; i < VPL; ++i) dqa[i] = fmaf(dzl, k_c[i], dqa[i]);
    if (p.dF && act) {
      float df[VPL];
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        float a = 0.f;
#pragma unroll
        for (int h = 0; h < H; ++h) a = fmaf(dz[h], u[h][i], fmaf(al[h], vd[h][i], a));
        df[i] = a;
      }
      float* dst = p.dF + row_c * p.lddf + j0;
      if (p.acc_dF) {
        float old[VPL];
        vload(dst, old);
#pragma unroll
        for (int i = 0; i < VPL; ++i) df[i] += old[i];
      }
      vstore(dst, df);
    }
    if (lane < H) {
      p.dz_e[(int64_t)t * H + lane] = pick<H>(dz, lane);
      p.alpha_e[(int64_t)t * H + lane] = pick<H>(al, lane);
    }
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      k_c[i] = k_n[i];
      v_c[i] = v_n[i];
      f_c[i] = f_n[i];
    }
    row_c = row_n;
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
    for (int32_t i = beg; i < end; ++i) {
      const int64_t pos = p.pos_src[i];
      const int64_t dd = p.dst_at[pos];
      const float dz = p.dz_e[pos * H + hl];
      const float al = p.alpha_e[pos * H + hl];
      float qv[VPL], gv[VPL];
      vload(p.QKVR + dd * p.ldq + j0, qv);
      vload(p.dout + dd * D + j0, gv);
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        dk[k] = fmaf(dz, qv[k], dk[k]);
        dv[k] = fmaf(al, gv[k], dv[k]);
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

template <int VPL, int H>
static void launch_fwd(const FwdParams& p, hipStream_t s) {
  hipLaunchKernelGGL((tconv_fwd_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
}
template <int VPL, int H>
static void launch_bwd_dst(const BwdDstParams& p, hipStream_t s) {
  hipLaunchKernelGGL((tconv_bwd_dst_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
}
template <int VPL, int H>
static void launch_bwd_src(const BwdSrcParams& p, hipStream_t s) {
  hipLaunchKernelGGL((tconv_bwd_src_kernel<VPL, H>), dim3((unsigned)((p.n + 3) / 4)), dim3(256), 0, s, p);
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
                                const int32_t* src_at, const int32_t* feat_row, const float* QKVR, int64_t ldq,
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
  ALIGNN_DISPATCH(vpl, H, launch_fwd, p, s);
  ALIGNN_LAUNCH_CHECK("tconv_fwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_tconv_bwd_dst(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                    const int32_t* src_at, const int32_t* feat_row, const float* QKVR, int64_t ldq,
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
  ALIGNN_DISPATCH(vpl, H, launch_bwd_dst, p, s);
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
