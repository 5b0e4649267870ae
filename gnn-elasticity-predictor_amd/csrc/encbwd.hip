// encbwd.hip — backward of the angle encoder's first Linear + ReLU (train.py:358-364), deferred to
// one pass after the last line-graph block.
//
// Each line-graph TransformerConv l reads the angle hidden layer f_t = relu(W1 x_t + b1) and
// contributes  g_{l,t} = sum_h dz_{l,t,h} u_{l,d,h} + alpha'_{l,t,h} Vd_{l,d,h}  to its gradient
// (d = target of edge t; u = M_h^T Q_h, Vd = M_h^T dout_h per target; dz, alpha' per edge — the
// edge-feature algebra of tconv.hip).  Accumulating g into a [T, D] array inside every layer's
// attention backward costs one read-modify-write of 2 x 259 MB per layer at B = 32.  Here the
// attention kernels only leave their per-edge scalars (dz, alpha': 2H floats per edge and layer)
// and this kernel forms, per edge,
//     dpre_t = relu'(W1 x_t + b1) * sum_{l,h} (dz u + alpha' Vd)       [D]
//     dW1 += dpre_t x_t^T,  db1 += dpre_t
// with the pre-activation recomputed from the kin raw inputs in the same fma order as the forward
// kernel (skinny.hip linear_smallk), so the ReLU mask is the forward's bit for bit.  Neither the
// [T, D] gradient nor a read of the [T, D] hidden layer exists.
//
// Layout: one wave walks chunks of EB_CHUNK consecutive target-sorted edges; lane j owns feature
// columns 4j..4j+3.  The per-target vectors of all (layer, head) pairs for the lane's columns stay
// in registers while the target does not change (2 x 16 x 4 floats); the per-edge scalars and
// x_t are wave-uniform scalar loads (prefetched one edge ahead).  dW1/db1 partials: registers per
// lane -> LDS merge of the 4 waves in wave order -> one partial per workgroup -> a second kernel
// sums the workgroup partials in workgroup order (deterministic: fixed grid, fixed orders).
#include "common.h"
#include "vec.h"

namespace alignn {

constexpr int EB_HL = 16;       // max H * L
constexpr int EB_CHUNK = 128;   // edges per wave work item
constexpr int EB_BLOCKS = 256;  // fixed grid: the partial-sum order does not depend on the device
constexpr int EB_LMAX = ALIGNN_ENCBWD_MAX_LAYERS;

struct EncBwdParams {
  int64_t n, T;
  int D, H, L, kin;
  const int32_t* dst_at;           // [T] target of each target-sorted edge
  const float* x; int64_t ldx;     // [T, kin] target-sorted raw angle inputs
  const float* w1;                 // [D, kin]
  const float* b1;                 // [D]
  const float* U[EB_LMAX];         // per layer [n, H, D]
  const float* Vd[EB_LMAX];        // per layer [n, H, D]
  const float* dz[EB_LMAX];        // per layer [T, H]
  const float* al[EB_LMAX];        // per layer [T, H]
  float* part;                     // [EB_BLOCKS, (kin + 1) * D]
};

template <int KM>
__global__ __launch_bounds__(256) void enc_bwd_kernel(EncBwdParams p) {
  __shared__ __attribute__((aligned(16))) float ew[(KM + 1) * 256];   // W1^T (zero rows k >= kin) | b1
  __shared__ __attribute__((aligned(16))) float red[256];
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int D = p.D, H = p.H, kin = p.kin;
  const int HL = H * p.L;
  const int j0 = 4 * lane;
  const bool act = j0 < D;
  for (int i = threadIdx.x; i < (KM + 1) * D; i += 256) {
    const int k = i / D, j = i - k * D;
    ew[k * 256 + j] = k < KM ? (k < kin ? p.w1[(int64_t)j * kin + k] : 0.f) : p.b1[j];
  }
  __syncthreads();

  float acc[KM][4], accb[4];
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[k][i] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) accb[i] = 0.f;

  float P[EB_HL][2][4];
  const int64_t nchunks = (p.T + EB_CHUNK - 1) / EB_CHUNK;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t ch = (int64_t)blockIdx.x * 4 + wave; ch < nchunks; ch += wstride) {
    const int64_t tb = ch * EB_CHUNK;
    const int64_t te = tb + EB_CHUNK < p.T ? tb + EB_CHUNK : p.T;
    int cur = -1;
    for (int64_t t = tb; t < te; ++t) {
      const int d = uni(sld(p.dst_at, t));
      if (d != cur) {
        cur = d;
#pragma unroll
        for (int q = 0; q < EB_HL; ++q) {
          if (q < HL && act) {
            const int l = q / H, h = q - (q / H) * H;
            vload(p.U[l] + ((int64_t)d * H + h) * D + j0, P[q][0]);
            vload(p.Vd[l] + ((int64_t)d * H + h) * D + j0, P[q][1]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) P[q][0][i] = P[q][1][i] = 0.f;
          }
        }
      }
      // g = sum over (layer, head) of dz u + alpha' Vd
      float g[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < EB_HL; ++q) {
        if (q < HL) {
          const int l = q / H, h = q - (q / H) * H;
          const float cz = sld(p.dz[l], t * H + h), ca = sld(p.al[l], t * H + h);
#pragma unroll
          for (int i = 0; i < 4; ++i) g[i] = fmaf(cz, P[q][0][i], fmaf(ca, P[q][1][i], g[i]));
        }
      }
      // pre-activation in linear_smallk's order: fma chain over k from 0, then + b1
      float xk[KM];
#pragma unroll
      for (int k = 0; k < KM; ++k) xk[k] = k < kin ? sld(p.x, t * p.ldx + k) : 0.f;
      float pre[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        float w[4];
        vload(ew + k * 256 + j0, w);
#pragma unroll
        for (int i = 0; i < 4; ++i) pre[i] = fmaf(xk[k], w[i], pre[i]);
      }
      float b[4];
      vload(ew + KM * 256 + j0, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dp = (pre[i] + b[i]) > 0.f ? g[i] : 0.f;
        accb[i] += dp;
#pragma unroll
        for (int k = 0; k < KM; ++k) acc[k][i] = fmaf(dp, xk[k], acc[k][i]);
      }
    }
  }

  // merge the 4 waves in wave order (red = w0 + w1 + w2 + w3), one partial row per workgroup
  float* part = p.part + (int64_t)blockIdx.x * (kin + 1) * D;
  auto merge_row = [&](const float (&v)[4], int k) {
    for (int w = 0; w < 4; ++w) {
      if (wave == w && act) {
        float o[4];
        if (w == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = v[i];
        } else {
          vload(red + j0, o);
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] += v[i];
        }
        if (w == 3) vstore(part + (int64_t)k * D + j0, o);
        else vstore(red + j0, o);
      }
      __syncthreads();
    }
  };
#pragma unroll
  for (int k = 0; k < KM; ++k)
    if (k < kin) merge_row(acc[k], k);
  merge_row(accb, kin);
}

// out (j, k): sum over workgroups b of part[b][k * D + j] in workgroup order (4 chains, fixed
// combine) -> dW1[j, k] (k < kin) or db1[j] (k == kin), written or accumulated.
__global__ __launch_bounds__(256) void enc_bwd_stage2(const float* __restrict__ part, int blocks, int D, int kin,
                                                      float* __restrict__ dW1, float* __restrict__ db1, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = (kin + 1) * D;
  if (i >= n) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = 0;
  for (; b + 3 < blocks; b += 4) {
    s0 += part[(int64_t)b * n + i];
    s1 += part[(int64_t)(b + 1) * n + i];
    s2 += part[(int64_t)(b + 2) * n + i];
    s3 += part[(int64_t)(b + 3) * n + i];
  }
  for (; b < blocks; ++b) s0 += part[(int64_t)b * n + i];
  const float t = (s0 + s1) + (s2 + s3);
  const int k = i / D, j = i - k * D;
  float* dst = k < kin ? dW1 + (int64_t)j * kin + k : db1 + j;
  *dst = accumulate ? *dst + t : t;
}

}  // namespace alignn

using namespace alignn;

extern "C" int64_t alignn_enc_bwd_workspace(int32_t D, int32_t kin) {
  if (D <= 0 || kin < 0) return -1;
  return (int64_t)EB_BLOCKS * (kin + 1) * D;
}

extern "C" int alignn_enc_bwd_f32(const AlignnEncBwdArgs* a, void* stream) {
  if (!a || a->n < 0 || a->T < 0 || a->D <= 0 || a->H <= 0 || a->L < 1 || a->kin < 0) {
    set_error("enc_bwd: bad shape");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (a->D > 256 || a->D % 4 != 0 || a->kin > 16 || a->H * a->L > EB_HL || a->L > EB_LMAX || a->ldx < a->kin) {
    set_error("enc_bwd: needs D <= 256 (multiple of 4), kin <= 16, H*L <= %d, L <= %d (D=%d kin=%d H=%d L=%d)", EB_HL,
              EB_LMAX, a->D, a->kin, a->H, a->L);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (!a->workspace || a->workspace_elems < (int64_t)EB_BLOCKS * (a->kin + 1) * a->D) {
    set_error("enc_bwd: needs %lld workspace floats", (long long)EB_BLOCKS * (a->kin + 1) * a->D);
    return ALIGNN_E_WORKSPACE;
  }
  EncBwdParams p;
  p.n = a->n; p.T = a->T; p.D = a->D; p.H = a->H; p.L = a->L; p.kin = a->kin;
  p.dst_at = a->dst_at; p.x = a->x; p.ldx = a->ldx; p.w1 = a->w1; p.b1 = a->b1;
  for (int l = 0; l < EB_LMAX; ++l) {
    const bool in = l < a->L;
    p.U[l] = in ? a->U[l] : nullptr;
    p.Vd[l] = in ? a->Vd[l] : nullptr;
    p.dz[l] = in ? a->dz[l] : nullptr;
    p.al[l] = in ? a->alpha[l] : nullptr;
    if (in && a->T > 0 && (!p.U[l] || !p.Vd[l] || !p.dz[l] || !p.al[l])) {
      set_error("enc_bwd: layer %d operand missing", l);
      return ALIGNN_E_BAD_SHAPE;
    }
  }
  p.part = a->workspace;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a->T > 0) {
    if (a->kin <= 8) launch(enc_bwd_kernel<8>, dim3(EB_BLOCKS), dim3(256), 0, s, p);
    else if (a->kin <= 12) launch(enc_bwd_kernel<12>, dim3(EB_BLOCKS), dim3(256), 0, s, p);
    else launch(enc_bwd_kernel<16>, dim3(EB_BLOCKS), dim3(256), 0, s, p);
    ALIGNN_LAUNCH_CHECK("enc_bwd_kernel");
  } else {
    const hipError_t e = hipMemsetAsync(a->workspace, 0, sizeof(float) * EB_BLOCKS * (a->kin + 1) * a->D, s);
    if (e != hipSuccess) return hip_status(e, "enc_bwd memset");
  }
  const int n = (a->kin + 1) * a->D;
  launch(enc_bwd_stage2, dim3((n + 255) / 256), dim3(256), 0, s, a->workspace, EB_BLOCKS, a->D, a->kin,
                     a->dW1, a->db1, (int)a->accumulate);
  ALIGNN_LAUNCH_CHECK("enc_bwd_stage2");
  return ALIGNN_OK;
}
