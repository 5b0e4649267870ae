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
// Layout: one workgroup per target segment (grid-strided over segments in a fixed order); thread j
// owns feature column j.  The segment's per-target vectors of all (layer, head) pairs stay in
// registers (2 x H*L floats per thread) and thread j keeps W1[j, :] and b1[j]; the segment's edges
// are staged in chunks of EB_CHUNK: their 2 x H*L per-edge scalars and kin raw inputs go to LDS with
// coalesced loads, and every thread walks the chunk reading them as LDS broadcasts — no dependent
// global load per edge (the previous one-wave-per-edge-stream form waited on scalar loads at every
// edge: 863 us at B = 32; profiles/r01/v13_sweep.log).  dW1/db1 partials: registers per thread,
// one partial row per workgroup, a second kernel sums the workgroup partials in workgroup order
// (deterministic: fixed grid, fixed orders).
#include <cstring>

#include "common.h"
#include "vec.h"

namespace alignn {

constexpr int EB_HL = 16;       // max H * L
constexpr int EB_CHUNK = 128;   // edges staged in LDS at a time
// fixed grid (the partial-sum order does not depend on the device): 4 workgroups per CU of an
// MI355X (22.5 KB LDS each), so segment-start loads of one hide behind the others' edge loops
#ifndef ALIGNN_EB_BLOCKS
#define ALIGNN_EB_BLOCKS 1024
#endif
constexpr int EB_BLOCKS = ALIGNN_EB_BLOCKS;
constexpr int EB_LMAX = ALIGNN_ENCBWD_MAX_LAYERS;

struct EncBwdParams {
  int64_t n, T;
  int D, H, L, kin;
  const int32_t* off_dst;          // [n + 1] target segments of the target-sorted edges
  const float* x; int64_t ldx;     // [T, kin] target-sorted raw angle inputs
  const float* w1;                 // [D, kin]
  const float* b1;                 // [D]
  const float* U[EB_LMAX];         // per layer [n, H, D]
  const float* Vd[EB_LMAX];        // per layer [n, H, D]
  const float* dz[EB_LMAX];        // per layer [T, H]
  const float* al[EB_LMAX];        // per layer [T, H]
  float* part;                     // [EB_BLOCKS, (kin + 1) * D]
};

template <int KM, int H>
__global__ __launch_bounds__(256) void enc_bwd_kernel(EncBwdParams p) {
  // per staged edge: [dz (HL) | alpha' (HL) | x (KM)]
  constexpr int ROW = 2 * EB_HL + KM;
  constexpr int LM = EB_HL / H < EB_LMAX ? EB_HL / H : EB_LMAX;  // layers that fit
  __shared__ __attribute__((aligned(16))) float es[EB_CHUNK * ROW];
  const int D = p.D, kin = p.kin, L = p.L;
  const int HL = H * L;
  const int j = threadIdx.x;
  const bool act = j < D;
  float w[KM], bj = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) w[k] = (act && k < kin) ? p.w1[(int64_t)j * kin + k] : 0.f;
  if (act) bj = p.b1[j];

  float acc[KM], accb = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) acc[k] = 0.f;
  // slots of (layer, head) pairs past H*L are never written: zero once (ordered by the first
  // chunk's barrier)
  for (int i = threadIdx.x; i < EB_CHUNK * ROW; i += 256) es[i] = 0.f;

  float Pu[EB_HL], Pv[EB_HL];
  for (int64_t d = blockIdx.x; d < p.n; d += gridDim.x) {
    const int64_t t0 = p.off_dst[d], t1 = p.off_dst[d + 1];
    if (t0 == t1) continue;
    // Every global load of a segment / chunk is issued before any of its values is used (one
    // memory round trip, not one per staging iteration): branch-free, absent layers and columns
    // read a valid row and are masked to 0 afterwards.
    const int jc = act ? j : 0;
#pragma unroll
    for (int q = 0; q < EB_HL; ++q) {
      const int l = q / H, h = q % H;   // constants: q unrolled, H a template parameter
      const int ls = l < L ? l : 0;
      const float u = p.U[ls][(d * H + h) * D + jc], v = p.Vd[ls][(d * H + h) * D + jc];
      Pu[q] = (q < HL && act) ? u : 0.f;
      Pv[q] = (q < HL && act) ? v : 0.f;
    }
    constexpr int PER_L = (EB_CHUNK * H + 255) / 256;   // per-layer scalars per thread
    constexpr int PER_X = (EB_CHUNK * KM + 255) / 256;  // raw-input values per thread
    for (int64_t tc = t0; tc < t1; tc += EB_CHUNK) {
      const int ne = (int)min<int64_t>(EB_CHUNK, t1 - tc);
      float vz[LM][PER_L], va[LM][PER_L], vx[PER_X];
      // per-edge scalars: layer l's [T, H] rows tc..tc+ne are contiguous
#pragma unroll
      for (int l = 0; l < LM; ++l) {
        const float* dz = p.dz[l < L ? l : 0] + tc * H;
        const float* al = p.al[l < L ? l : 0] + tc * H;
#pragma unroll
        for (int u = 0; u < PER_L; ++u) {
          const int i = threadIdx.x + 256 * u;
          const int ic = i < ne * H ? i : 0;
          vz[l][u] = dz[ic];
          va[l][u] = al[ic];
        }
      }
#pragma unroll
      for (int u = 0; u < PER_X; ++u) {
        const int i = threadIdx.x + 256 * u;
        const int e = i / KM, k = i % KM;
        vx[u] = (i < ne * KM && k < kin) ? p.x[(tc + e) * p.ldx + k] : 0.f;
      }
      __syncthreads();   // the previous chunk's readers are done with es
#pragma unroll
      for (int l = 0; l < LM; ++l) {
        if (l < L) {
#pragma unroll
          for (int u = 0; u < PER_L; ++u) {
            const int i = threadIdx.x + 256 * u;
            if (i < ne * H) {
              const int e = i / H, h = i % H;
              es[e * ROW + l * H + h] = vz[l][u];
              es[e * ROW + EB_HL + l * H + h] = va[l][u];
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PER_X; ++u) {
        const int i = threadIdx.x + 256 * u;
        if (i < ne * KM) es[(i / KM) * ROW + 2 * EB_HL + i % KM] = vx[u];
      }
      __syncthreads();
      if (act) {
        for (int e = 0; e < ne; ++e) {
          const float* r = es + e * ROW;
          // g = sum over (layer, head) of dz u + alpha' Vd
          // unconditional over all EB_HL slots: slots q >= HL are 0 in LDS and in Pu/Pv (a runtime
          // q < HL test here compiled to one LDS round trip and full wait per slot)
          float gq[4] = {0.f, 0.f, 0.f, 0.f};   // four independent chains
#pragma unroll
          for (int q = 0; q < EB_HL; ++q) gq[q & 3] = fmaf(r[q], Pu[q], fmaf(r[EB_HL + q], Pv[q], gq[q & 3]));
          const float g = (gq[0] + gq[1]) + (gq[2] + gq[3]);
          // pre-activation in linear_smallk's order: fma chain over k from 0, then + b1
          float pre = 0.f;
#pragma unroll
          for (int k = 0; k < KM; ++k) pre = fmaf(r[2 * EB_HL + k], w[k], pre);
          const float dp = (pre + bj) > 0.f ? g : 0.f;
          accb += dp;
#pragma unroll
          for (int k = 0; k < KM; ++k) acc[k] = fmaf(dp, r[2 * EB_HL + k], acc[k]);
        }
      }
    }
  }
  if (act) {
    float* part = p.part + (int64_t)blockIdx.x * (kin + 1) * D;
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < kin) part[(int64_t)k * D + j] = acc[k];
    part[(int64_t)kin * D + j] = accb;
  }
}

// out (j, k): sum over workgroups b of part[b][k * D + j] in workgroup order (4 chains, fixed
// combine) -> dW1[j, k] (k < kin) or db1[j] (k == kin), written or accumulated.
// Block: 16 row-lanes x 64 outputs; thread (ty, tx) keeps four chains over workgroups ty, ty+16,
// ty+32, ty+48 of every 64, then the 16 row-lanes are combined in lane order (fixed).
__global__ __launch_bounds__(1024) void enc_bwd_stage2(const float* __restrict__ part, int blocks, int D, int kin,
                                                       float* __restrict__ dW1, float* __restrict__ db1, int accumulate) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + tx;
  const int n = (kin + 1) * D;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n) {
    int b = ty;
    for (; b + 48 < blocks; b += 64) {
      s0 += part[(int64_t)b * n + i];
      s1 += part[(int64_t)(b + 16) * n + i];
      s2 += part[(int64_t)(b + 32) * n + i];
      s3 += part[(int64_t)(b + 48) * n + i];
    }
    for (; b < blocks; b += 16) s0 += part[(int64_t)b * n + i];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty != 0 || i >= n) return;
  float t = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) t += red[r][tx];
  const int k = i / D, j = i - k * D;
  float* dst = k < kin ? dW1 + (int64_t)j * kin + k : db1 + j;
  *dst = accumulate ? *dst + t : t;
}

// ---------------------------------------------------------------------------------------------
// bf16 storage (config C3, the reference's autocast, train.py:628-636): the same gradient on the
// matrix cores.  Under autocast the hidden layer f = relu(W1 x + b1) is a bf16 Linear output, its
// gradient reaches it through bf16 Linear backwards, ReLU's backward reads its own (bf16) output, and
// dW1 = dpre^T x is a bf16 product with fp32 accumulation.  Per target segment d and chunk of 32
// target-sorted edges, one wave per 64 feature columns (two 32-column tiles):
//     G    = [dz | alpha'] (32 edges x 32)  .  [U_d ; Vd_d] (32 x 32 columns)     (2 MFMA 32x32x16)
//     dpre = G * [f > 0]                     (f: the forward's bf16 hidden layer rows)
//     Z   += dpre^T . [x | 1] (32 columns x 32: kin inputs, a ones column for db1, zeros)  (2 MFMA)
// The G accumulator is the next product's A operand with no data movement: registers 8s..8s+7,
// rounded to bf16, are k-step s of dpre^T, whose k (edge) order is 16s + 8(j>>2) + 4h + (j&3) for
// element j of lane half h — the [x | 1] operand is loaded in that same edge order.  The 32 (layer,
// head) slots past H*L and the edges past a chunk's end are zeros.  Z partials per workgroup,
// reduced by enc_bwd_stage2 as in the fp32 kernel (fixed grid and orders: deterministic).  Memory
// bound: the f rows (T x D bf16) and U/Vd (once per target) dominate; 2.03 M triplets at B = 256
// take ~30 us of matrix-core time in all.
typedef float ebx16 __attribute__((ext_vector_type(16)));
typedef __bf16 ebh8 __attribute__((ext_vector_type(8)));
typedef uint32_t ebu4 __attribute__((ext_vector_type(4)));
// v where keep, else +0 — a bit mask, not a select: a select on a loaded value let the compiler sink
// the load into a branch (a branch and a full wait per element)
__device__ __forceinline__ float keep_if(float v, bool keep) {
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & (keep ? 0xffffffffu : 0u));
}
// fixed grid of the bf16 kernel: three workgroups per CU of an MI355X (its occupancy), all resident at
// once — a fourth, queued behind them, doubled the kernel's tail (partials: EBF_BLOCKS rows of the
// workspace, summed by enc_bwd_stage2 in workgroup order)
constexpr int EBF_BLOCKS = EB_BLOCKS < 768 ? EB_BLOCKS : 768;
constexpr int EBF_FP = 256 + 8;   // LDS row of a chunk's hidden-layer rows (bf16), padded
constexpr int EBF_XP = 17;        // LDS row of a chunk's raw inputs (kin <= 16 floats), padded

// The 32 k slots of the G product: k-step s (0: dz and U, 1: alpha' and Vd), element j of lane half hh
// is (layer j / (H/2), head hh (H/2) + j % (H/2)) — the layer depends on j only, so every per-layer
// pointer is wave-uniform (a per-lane choice of table entry compiled to vector loads of the table and
// a wait before every use).  Layers >= L: zeros (their table entries repeat layer 0, enc_bwd_params).
template <int H>
struct EbSlot {
  static constexpr int JPL = H / 2;   // j values per layer
  static __device__ __forceinline__ int layer(int j) { return j / JPL; }
  static __device__ __forceinline__ int head(int hh, int j) { return hh * JPL + j % JPL; }
};

// XF: no hidden-layer rows (the line convs recompute them on the matrix cores, lgmx.hip): the ReLU mask
// comes from the pre-activation recomputed here as the forward computes it — bf16(x) . bf16(W1)^T +
// bf16(b1) (autocast's operands for train.py:554 under :636; the bias enters as a ones column of x) on
// one v_mfma_f32_32x32x16_bf16 per 32 x 32 tile, laid out as the G tile (A: x of edge r, inputs 8 hh + j;
// B: W1 of column 64 w + 32 ct + r), then rounded to bf16 like the forward's f.  kin <= EB_XF_KMAX.
constexpr int EB_XF_KMAX = 12;
constexpr int EBF_BLOCKS_XF = EBF_BLOCKS;
template <int H, bool XF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void enc_bwd_bf16_kernel(EncBwdParams p, const uint16_t* __restrict__ F16, int64_t ldf) {
  constexpr int D = 256;
  __shared__ __attribute__((aligned(16))) uint16_t fs[XF ? 8 : 32 * EBF_FP];   // the chunk's f rows
  __shared__ float xs[32 * EBF_XP];                                            // the chunk's raw inputs
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int kin = p.kin;
  ebh8 W1B[2];   // XF: [W1 | b1] of this lane's two columns (bf16), inputs 8 hh .. 8 hh + 7
  if constexpr (XF) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int col = 64 * w + 32 * ct + r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * hh + j;
        W1B[ct][j] = (__bf16)(k < kin ? p.w1[col * kin + k] : (k == kin ? p.b1[col] : 0.f));
      }
    }
  }
  ebx16 Z[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int i = 0; i < 16; ++i) Z[ct][i] = 0.f;
  for (int64_t d = blockIdx.x; d < p.n; d += gridDim.x) {
    const int64_t t0 = p.off_dst[d], t1 = p.off_dst[d + 1];
    if (t0 == t1) continue;
    // B operands of G: slot q = 8 hh + j of k-step s (0: U, 1: Vd), column 64 w + 32 ct + r
    ebh8 PB[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = EbSlot<H>::layer(j);
        const float* base = (s ? p.Vd : p.U)[l < EB_LMAX ? l : 0];
        const bool ok = l < p.L;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {   // unconditional load (every table entry is a valid layer)
          const float v = base[(d * H + EbSlot<H>::head(hh, j)) * D + 64 * w + 32 * ct + r];
          PB[ct][s][j] = (__bf16)keep_if(v, ok);
        }
      }
    for (int64_t tc = t0; tc < t1; tc += 32) {
      const int ne = (int)min<int64_t>(32, t1 - tc);
      // stage the chunk's f rows (32 x 256 bf16: four 16-byte loads per thread, rows past the chunk
      // read a valid row and are never used) and raw inputs
      ebu4 fv[4];
      if constexpr (!XF) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = threadIdx.x + 256 * u, e = i >> 5, c8 = (i & 31) * 8;
          fv[u] = *reinterpret_cast<const ebu4*>(F16 + (tc + min(e, ne - 1)) * ldf + c8);
        }
      }
      float xv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = threadIdx.x + 256 * u, e = i >> 4, k = i & 15;
        const float v = p.x[(tc + min(e, ne - 1)) * p.ldx + min(k, kin - 1)];   // unconditional load
        xv[u] = keep_if(v, e < ne && k < kin);
      }
      // A operand of G: [dz | alpha'] of edge tc + r, slot 8 hh + j (k-step 0: dz, 1: alpha')
      const bool ev = r < ne;
      const int64_t te = tc + (ev ? r : 0);
      float sv[2][8];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int l = EbSlot<H>::layer(j);
          sv[s][j] = (s ? p.al : p.dz)[l < EB_LMAX ? l : 0][te * H + EbSlot<H>::head(hh, j)];
        }
      __syncthreads();   // the previous chunk's LDS readers are done
      if constexpr (!XF) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = threadIdx.x + 256 * u, e = i >> 5, c8 = (i & 31) * 8;
          *reinterpret_cast<ebu4*>(fs + e * EBF_FP + c8) = fv[u];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = threadIdx.x + 256 * u;
        xs[(i >> 4) * EBF_XP + (i & 15)] = xv[u];
      }
      __syncthreads();
      ebh8 XA;   // XF: x_aug of edge r (inputs 8 hh + j; the ones column at k = kin)
      if constexpr (XF) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * hh + j;
          const float v = xs[r * EBF_XP + (k < 16 ? k : 0)];   // unconditional read (zero past kin)
          XA[j] = (__bf16)(k < kin ? v : (k == kin ? 1.f : 0.f));
        }
      }
      ebh8 SA[2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) SA[s][j] = (__bf16)keep_if(sv[s][j], ev && EbSlot<H>::layer(j) < p.L);
      // B operand of Z: [x | 1 | 0] of edge 16 s + 8 (j>>2) + 4 hh + (j&3), input column r
      ebh8 XB[2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int e = 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3);
          const float v = xs[e * EBF_XP + (r & 15)];   // unconditional read
          const float one = (r == kin && e < ne) ? 1.f : 0.f;
          XB[s][j] = (__bf16)(keep_if(v, r < kin) + one);
        }
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        ebx16 G;
#pragma unroll
        for (int i = 0; i < 16; ++i) G[i] = 0.f;
        G = __builtin_amdgcn_mfma_f32_32x32x16_bf16(SA[0], PB[ct][0], G, 0, 0, 0);
        G = __builtin_amdgcn_mfma_f32_32x32x16_bf16(SA[1], PB[ct][1], G, 0, 0, 0);
        // ReLU backward from the bf16 output: register i is edge (i&3) + 8(i>>2) + 4 hh of the chunk
        // (edges past the chunk's end have zero G rows: their [dz | alpha'] rows are zero)
        const int col = 64 * w + 32 * ct + r;
        ebh8 GA[2];
        if constexpr (XF) {
          const ebx16 pre = __builtin_amdgcn_mfma_f32_32x32x16_bf16(XA, W1B[ct], ebx16{}, 0, 0, 0);
#pragma unroll
          for (int i = 0; i < 16; ++i) GA[i >> 3][i & 7] = (__bf16)((float)(__bf16)pre[i] > 0.f ? G[i] : 0.f);
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int e = (i & 3) + 8 * (i >> 2) + 4 * hh;
            const uint32_t fb = fs[e * EBF_FP + col];
            GA[i >> 3][i & 7] = (__bf16)(__builtin_bit_cast(float, fb << 16) > 0.f ? G[i] : 0.f);
          }
        }
        Z[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(GA[0], XB[0], Z[ct], 0, 0, 0);
        Z[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(GA[1], XB[1], Z[ct], 0, 0, 0);
      }
    }
  }
  // Z[ct] register i: feature column 64 w + 32 ct + (i&3) + 8(i>>2) + 4 hh, input column r
  if (r <= kin) {
    float* part = p.part + (int64_t)blockIdx.x * (kin + 1) * D + (int64_t)r * D;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i) part[64 * w + 32 * ct + (i & 3) + 8 * (i >> 2) + 4 * hh] = Z[ct][i];
  }
}

}  // namespace alignn

using namespace alignn;

extern "C" int64_t alignn_enc_bwd_workspace(int32_t D, int32_t kin) {
  if (D <= 0 || kin < 0) return -1;
  return (int64_t)EB_BLOCKS * (kin + 1) * D;
}

static int enc_bwd_params(const AlignnEncBwdArgs* a, EncBwdParams& p);
static int enc_bwd_stage2_launch(const AlignnEncBwdArgs* a, hipStream_t s, int blocks);

extern "C" int alignn_enc_bwd_bf16(const AlignnEncBwdArgs* a, const uint16_t* F16, int64_t ldf, void* stream) {
  EncBwdParams p;
  const int rc = enc_bwd_params(a, p);
  if (rc != ALIGNN_OK) return rc;
  if (a->D != 256 || a->kin < 1 || a->H < 2 || (!F16 && a->kin > EB_XF_KMAX) ||
      (a->T > 0 && F16 && (ldf < a->D || ldf % 8 != 0 || (reinterpret_cast<uintptr_t>(F16) & 15)))) {
    set_error("enc_bwd_bf16: needs D = 256, H >= 2, kin >= 1 and 16-byte aligned bf16 hidden-layer rows (ldf >= D, "
              "ldf %% 8 == 0) or none (kin <= %d; D=%d kin=%d ldf=%lld)", EB_XF_KMAX, a->D, a->kin, (long long)ldf);
    return ALIGNN_E_UNSUPPORTED;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a->T > 0) {
    if (F16) {
      switch (a->H) {
        case 2: launch(enc_bwd_bf16_kernel<2, false>, dim3(EBF_BLOCKS), dim3(256), 0, s, p, F16, ldf); break;
        case 4: launch(enc_bwd_bf16_kernel<4, false>, dim3(EBF_BLOCKS), dim3(256), 0, s, p, F16, ldf); break;
        default: launch(enc_bwd_bf16_kernel<8, false>, dim3(EBF_BLOCKS), dim3(256), 0, s, p, F16, ldf); break;
      }
    } else {   // the hidden layer recomputed (the line convs' XF path)
      switch (a->H) {
        case 2: launch(enc_bwd_bf16_kernel<2, true>, dim3(EBF_BLOCKS_XF), dim3(256), 0, s, p, F16, ldf); break;
        case 4: launch(enc_bwd_bf16_kernel<4, true>, dim3(EBF_BLOCKS_XF), dim3(256), 0, s, p, F16, ldf); break;
        default: launch(enc_bwd_bf16_kernel<8, true>, dim3(EBF_BLOCKS_XF), dim3(256), 0, s, p, F16, ldf); break;
      }
    }
    ALIGNN_LAUNCH_CHECK("enc_bwd_bf16_kernel");
  } else {
    const int rc2 = alignn_fill_f32(a->workspace, (int64_t)EBF_BLOCKS * (a->kin + 1) * a->D, 0.f, stream);
    if (rc2 != ALIGNN_OK) return rc2;
  }
  return enc_bwd_stage2_launch(a, s, F16 ? EBF_BLOCKS : EBF_BLOCKS_XF);
}

static int enc_bwd_params(const AlignnEncBwdArgs* a, EncBwdParams& p) {
  if (!a || a->n < 0 || a->T < 0 || a->D <= 0 || a->H <= 0 || a->L < 1 || a->kin < 0) {
    set_error("enc_bwd: bad shape");
    return ALIGNN_E_BAD_SHAPE;
  }
  const bool h_ok = a->H == 1 || a->H == 2 || a->H == 4 || a->H == 8;
  if (a->D > 256 || a->D % 4 != 0 || a->kin > 16 || !h_ok || a->H * a->L > EB_HL || a->L > EB_LMAX ||
      a->ldx < a->kin) {
    set_error("enc_bwd: needs D <= 256 (multiple of 4), kin <= 16, H in {1,2,4,8}, H*L <= %d, L <= %d "
              "(D=%d kin=%d H=%d L=%d)", EB_HL,
              EB_LMAX, a->D, a->kin, a->H, a->L);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (!a->workspace || a->workspace_elems < (int64_t)EB_BLOCKS * (a->kin + 1) * a->D) {
    set_error("enc_bwd: needs %lld workspace floats", (long long)EB_BLOCKS * (a->kin + 1) * a->D);
    return ALIGNN_E_WORKSPACE;
  }
  std::memset(&p, 0, sizeof p);  // defined padding bytes (plan.hip scans recorded struct words)
  p.n = a->n; p.T = a->T; p.D = a->D; p.H = a->H; p.L = a->L; p.kin = a->kin;
  p.off_dst = a->off_dst; p.x = a->x; p.ldx = a->ldx; p.w1 = a->w1; p.b1 = a->b1;
  for (int l = 0; l < EB_LMAX; ++l) {   // entries past L repeat layer 0 (read, never used)
    const int li = l < a->L ? l : 0;
    p.U[l] = a->U[li];
    p.Vd[l] = a->Vd[li];
    p.dz[l] = a->dz[li];
    p.al[l] = a->alpha[li];
    if (a->T > 0 && (!p.U[l] || !p.Vd[l] || !p.dz[l] || !p.al[l])) {
      set_error("enc_bwd: layer %d operand missing", li);
      return ALIGNN_E_BAD_SHAPE;
    }
  }
  p.part = a->workspace;
  if (a->T > 0 && !a->off_dst) {
    set_error("enc_bwd: off_dst missing");
    return ALIGNN_E_BAD_SHAPE;
  }
  return ALIGNN_OK;
}

static int enc_bwd_stage2_launch(const AlignnEncBwdArgs* a, hipStream_t s, int blocks) {
  const int n = (a->kin + 1) * a->D;
  launch(enc_bwd_stage2, dim3((n + 63) / 64), dim3(1024), 0, s, a->workspace, blocks, a->D, a->kin,
                     a->dW1, a->db1, (int)a->accumulate);
  ALIGNN_LAUNCH_CHECK("enc_bwd_stage2");
  return ALIGNN_OK;
}

extern "C" int alignn_enc_bwd_f32(const AlignnEncBwdArgs* a, void* stream) {
  EncBwdParams p;
  const int rc = enc_bwd_params(a, p);
  if (rc != ALIGNN_OK) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a->T > 0) {
    const int km = a->kin <= 8 ? 8 : a->kin <= 12 ? 12 : 16;
#define EB_LAUNCH_H(KM_)                                                                   \
  switch (a->H) {                                                                          \
    case 1: launch(enc_bwd_kernel<KM_, 1>, dim3(EB_BLOCKS), dim3(256), 0, s, p); break;    \
    case 2: launch(enc_bwd_kernel<KM_, 2>, dim3(EB_BLOCKS), dim3(256), 0, s, p); break;    \
    case 4: launch(enc_bwd_kernel<KM_, 4>, dim3(EB_BLOCKS), dim3(256), 0, s, p); break;    \
    default: launch(enc_bwd_kernel<KM_, 8>, dim3(EB_BLOCKS), dim3(256), 0, s, p); break;   \
  }
    if (km == 8) {
      EB_LAUNCH_H(8)
    } else if (km == 12) {
      EB_LAUNCH_H(12)
    } else {
      EB_LAUNCH_H(16)
    }
#undef EB_LAUNCH_H
    ALIGNN_LAUNCH_CHECK("enc_bwd_kernel");
  } else {
    const int rc2 = alignn_fill_f32(a->workspace, (int64_t)EB_BLOCKS * (a->kin + 1) * a->D, 0.f, stream);
    if (rc2 != ALIGNN_OK) return rc2;
  }
  return enc_bwd_stage2_launch(a, s, EB_BLOCKS);
}
