// rowops.hip — row-wise fused kernels: TransformerConv beta gate + LayerNorm + ReLU + dropout +
// residual (forward/backward), readout pooling/concat, dropout, hetero-Gaussian NLL, jitter.
#include <cstdarg>
#include <cstdio>

#include "common.h"
#include "vec.h"

namespace alignn {

static thread_local char g_err[512] = "";
thread_local const uint64_t* g_step_seed = nullptr;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hip_status(hipError_t e, const char* what) {
  set_error("%s: %s", what, hipGetErrorString(e));
  return ALIGNN_E_HIP;
}

static int grid_for(int64_t work, int block = 256, int64_t cap = 8192) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ---------------------------------------------------------------------------------------------
// Gate + LayerNorm + ReLU + dropout + residual.  One wave per row, VPL features per lane.
//   PyG TransformerConv (beta=True):  beta = sigmoid(lin_beta([o, r, o - r])); y = beta r + (1-beta) o
//   train.py:316-317 / :335-336:      x_new = x + dropout(relu(LayerNorm(y)))   (eps 1e-5)
// ---------------------------------------------------------------------------------------------
struct GateFwdParams {
  int64_t n;
  int D, pad_;
  const float* outp; const float* R; int64_t ldr;
  const float* wbeta;
  const float* X; int64_t ldx;
  const float* lnw; const float* lnb;
  float* Xn; int64_t ldxn;
  float* beta; float* mu; float* rstd;
  DropParams drop;
  const int32_t* orow;  // optional: row r of o is outp[orow[r]] (-1: o = 0) — compacted conv outputs
  // bf16 storage (the reference's autocast, train.py:632-636): R is the skip projection's bf16 output
  // (rbf); Xn16, if set, receives a bf16 copy of the new state (the next Linear's bf16 input)
  int rbf, pad2_;
  uint16_t* Xn16; int64_t ldxn16;
  float* xa;            // optional [#active, D]: row orow[r] (>= 0) also receives the new state's row r —
                        // the next line block's active-row gather, written here instead of by a launch
};

// IO: some operand is bf16 (bf16 storage); the fp32 instantiation carries no storage-type branches.
// RBF: R is bf16 (a template flag: no branch between the row's loads).  Every load of the row is
// issued at once and unconditionally (a row without an output row reads its residual row and zeroes
// o): one round trip per row.
template <int VPL, bool IO, bool RBF>
__global__ __launch_bounds__(256) void gate_ln_fwd_kernel(GateFwdParams p) {
  resolve_drop(p.drop);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= p.n) return;
  const int D = p.D, j0 = lane * VPL;
  const bool act = j0 < D;
  float o[VPL], r[VPL], w1[VPL], w2[VPL], w3[VPL], g[VPL], bb[VPL], x[VPL];
  vzero(o); vzero(r); vzero(w1); vzero(w2); vzero(w3);
  const int64_t orow = p.orow ? (int64_t)uni(sld(p.orow, row)) : row;
  if (act) {
    vload((orow >= 0 ? p.outp + orow * D : p.X + row * p.ldx) + j0, o);
    if constexpr (RBF) vload_bf(reinterpret_cast<const uint16_t*>(p.R) + row * p.ldr + j0, r);
    else vload(p.R + row * p.ldr + j0, r);
    vload(p.wbeta + j0, w1);
    vload(p.wbeta + D + j0, w2);
    vload(p.wbeta + 2 * D + j0, w3);
    // the LayerNorm parameters and the residual row with the rest: one round trip per row, not two
    vload(p.lnw + j0, g);
    vload(p.lnb + j0, bb);
    vload(p.X + row * p.ldx + j0, x);
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) o[i] = orow >= 0 ? o[i] : 0.f;
  float part = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) part += o[i] * w1[i] + r[i] * w2[i] + (o[i] - r[i]) * w3[i];
  const float logit = wave_sum(part);
  const float b = 1.0f / (1.0f + __expf(-logit));
  float y[VPL];
  float sy = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    y[i] = b * r[i] + (1.0f - b) * o[i];
    sy += y[i];
  }
  const float mean = wave_sum(sy) / (float)D;
  float sv = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float c = act ? (y[i] - mean) : 0.f;
    sv += c * c;
  }
  const float var = wave_sum(sv) / (float)D;
  const float rs = 1.0f / sqrtf(var + 1e-5f);
  if (act) {
    float out[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float a = fmaxf((y[i] - mean) * rs * g[i] + bb[i], 0.f);
      if (p.drop.active) a *= dropout_mul(p.drop.seed, (uint64_t)row * D + j0 + i, p.drop.thresh, p.drop.inv_keep);
      out[i] = x[i] + a;
    }
    vstore(p.Xn + row * p.ldxn + j0, out);
    if (IO && p.Xn16) vstore_bf(p.Xn16 + row * p.ldxn16 + j0, out);
    if (p.xa && orow >= 0) vstore(p.xa + orow * D + j0, out);
  }
  if (lane == 0) {
    p.beta[row] = b;
    p.mu[row] = mean;
    p.rstd[row] = rs;
  }
}

struct GateBwdParams {
  int64_t n;
  int D, pad_;
  const float* dXn; int64_t lddx;
  const float* outp; const float* R; int64_t ldr;
  const float* wbeta; const float* lnw; const float* lnb;
  const float* beta; const float* mu; const float* rstd;
  float* dout; float* dR; int64_t lddr;
  float* part;  // [workgroups][5*D]: one merged partial row per workgroup
  int nwaves, pad2_;
  DropParams drop;
  const int32_t* orow;  // optional: o and dout rows through this map (-1: o = 0, dout not written)
  const float* dX2;     // optional [n, D] addend: the incoming gradient is dXn + dX2, written back to dXn
  int rbf, drbf;        // bf16 storage: R read as bf16, dR written as bf16 (autocast: grad of a bf16 output)
  int x2bf;            // dX2 holds bf16 elements (the atom block's edge-feature gradient under autocast)
  int dxz;              // dXn holds no gradient yet: read as zero (with dX2: the sum is dX2, written to dXn)
};

// A row's operand as it lies in memory (bf16 pairs or fp32 bits), widened where it is used: a
// value computed at its load puts the wait for that load right behind it.
template <int VPL, bool BF>
struct RawRow {
  uint32_t u[BF ? (VPL + 1) / 2 : VPL];
  __device__ __forceinline__ void load(const void* base, int64_t idx) {
    if constexpr (BF) {
      const uint16_t* q = reinterpret_cast<const uint16_t*>(base) + idx;
      if constexpr (VPL % 4 == 0) {
#pragma unroll
        for (int k = 0; k < VPL / 4; ++k) {
          const uint2 t = *reinterpret_cast<const uint2*>(q + 4 * k);
          u[2 * k] = t.x;
          u[2 * k + 1] = t.y;
        }
      } else {
#pragma unroll
        for (int i = 0; i < (VPL + 1) / 2; ++i)
          u[i] = (uint32_t)q[2 * i] | (2 * i + 1 < VPL ? (uint32_t)q[2 * i + 1] << 16 : 0u);
      }
    } else {
      float t[VPL];
      vload(reinterpret_cast<const float*>(base) + idx, t);
#pragma unroll
      for (int i = 0; i < VPL; ++i) u[i] = __builtin_bit_cast(uint32_t, t[i]);
    }
  }
  __device__ __forceinline__ void widen(float (&f)[VPL], bool live) const {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const float v = BF ? __builtin_bit_cast(float, (i & 1) ? (u[i / 2] & 0xffff0000u) : (u[i / 2] << 16))
                         : __builtin_bit_cast(float, u[i]);
      f[i] = live ? v : 0.f;
    }
  }
};

// IO: some operand is bf16 (the bf16 stores take runtime flags); RBF: R is bf16; X2: an addend dX2
// (X2BF: bf16).  Rows r and r + nwaves are walked as a pair: both rows' loads are issued before
// either is computed (every load unconditional: the second row of the last pair is clamped to the
// first and its results dropped; a row without an output row, or a dXn read as zero, loads a valid
// row and zeroes it at use), then the two rows are computed in row order — the accumulations in the
// order of the one-row loop: bitwise its results.
template <int VPL, bool IO, bool RBF, bool X2, bool X2BF>
__global__ __launch_bounds__(256) void gate_ln_bwd_kernel(GateBwdParams p) {
  resolve_drop(p.drop);
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + wave_id();
  const int D = p.D, j0 = lane * VPL;
  const bool act = j0 < D;
  const int jc = act ? j0 : 0;
  float w1[VPL], w2[VPL], w3[VPL], g[VPL], bb[VPL];
  vzero(w1); vzero(w2); vzero(w3); vzero(g); vzero(bb);
  if (act) {
    vload(p.wbeta + j0, w1);
    vload(p.wbeta + D + j0, w2);
    vload(p.wbeta + 2 * D + j0, w3);
    vload(p.lnw + j0, g);
    vload(p.lnb + j0, bb);
  }
  float a_g[VPL], a_b[VPL], a_w1[VPL], a_w2[VPL], a_w3[VPL];
  vzero(a_g); vzero(a_b); vzero(a_w1); vzero(a_w2); vzero(a_w3);
  struct In {
    float o[VPL], gx[VPL];
    RawRow<VPL, RBF> r;
    RawRow<VPL, X2BF> x2;
    int64_t orow;
    float b, mean, rs;
  };
  auto issue = [&](In& t, int64_t row) {
    t.orow = p.orow ? (int64_t)uni(sld(p.orow, row)) : row;
    // (no output row: a valid address read instead — this row of dXn — and o zeroed at use)
    vload((t.orow >= 0 ? p.outp + t.orow * D : p.dXn + row * p.lddx) + jc, t.o);
    t.r.load(p.R, row * p.ldr + jc);
    vload(p.dXn + row * p.lddx + jc, t.gx);
    if constexpr (X2) t.x2.load(p.dX2, row * D + jc);
    t.b = p.beta[row];
    t.mean = p.mu[row];
    t.rs = p.rstd[row];
  };
  auto finish = [&](const In& t, int64_t row) {
    const int64_t orow = t.orow;
    float o[VPL], r[VPL], gx[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      o[i] = (act && orow >= 0) ? t.o[i] : 0.f;
      gx[i] = (act && !p.dxz) ? t.gx[i] : 0.f;
    }
    t.r.widen(r, act);
    if constexpr (X2) {   // one add per element, the sum kept as the residual's gradient
      float x2[VPL];
      t.x2.widen(x2, act);
#pragma unroll
      for (int i = 0; i < VPL; ++i) gx[i] += x2[i];
      if (act) vstore(const_cast<float*>(p.dXn) + row * p.lddx + j0, gx);
    }
    const float b = t.b, mean = t.mean, rs = t.rs;
    float yh[VPL], gyh[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const float y = b * r[i] + (1.0f - b) * o[i];
      yh[i] = act ? (y - mean) * rs : 0.f;
      const float ln = yh[i] * g[i] + bb[i];
      float ga = gx[i];
      if (p.drop.active && act)
        ga *= dropout_mul(p.drop.seed, (uint64_t)row * D + j0 + i, p.drop.thresh, p.drop.inv_keep);
      const float gl = (act && ln > 0.f) ? ga : 0.f;
      a_g[i] = fmaf(gl, yh[i], a_g[i]);
      a_b[i] += gl;
      gyh[i] = gl * g[i];
      s1 += gyh[i];
      s2 += gyh[i] * yh[i];
    }
    const float m1 = wave_sum(s1) / (float)D, m2 = wave_sum(s2) / (float)D;
    float dy[VPL];
    float sb = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      dy[i] = act ? rs * (gyh[i] - m1 - yh[i] * m2) : 0.f;
      sb += dy[i] * (r[i] - o[i]);
    }
    const float dbeta = wave_sum(sb);
    const float dl = dbeta * b * (1.0f - b);
    if (act) {
      float dov[VPL], drv[VPL];
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        dov[i] = (1.0f - b) * dy[i] + dl * (w1[i] + w3[i]);
        drv[i] = b * dy[i] + dl * (w2[i] - w3[i]);
        a_w1[i] = fmaf(dl, o[i], a_w1[i]);
        a_w2[i] = fmaf(dl, r[i], a_w2[i]);
        a_w3[i] = fmaf(dl, o[i] - r[i], a_w3[i]);
      }
      if (orow >= 0) vstore(p.dout + orow * D + j0, dov);
      if (IO && p.drbf) vstore_bf(reinterpret_cast<uint16_t*>(p.dR) + row * p.lddr + j0, drv);
      else vstore(p.dR + row * p.lddr + j0, drv);
    }
  };
  if (wid < p.nwaves) {
    In A, B;
    for (int64_t row = wid; row < p.n; row += 2 * (int64_t)p.nwaves) {
      const int64_t rb = row + p.nwaves;
      const bool two = rb < p.n;   // wave-uniform
      issue(A, row);
      issue(B, two ? rb : row);
      finish(A, row);
      if (two) finish(B, rb);
    }
  }
  // one partial row per workgroup: the 4 waves' sums merged in LDS in wave order (fixed)
  __shared__ __attribute__((aligned(16))) float red[3][5 * 64 * VPL];
  const int wave = wave_id();
  float* mine = wave > 0 ? red[wave - 1] : nullptr;
  if (wave > 0 && act) {
    vstore(mine + j0, a_w1);
    vstore(mine + D + j0, a_w2);
    vstore(mine + 2 * D + j0, a_w3);
    vstore(mine + 3 * D + j0, a_g);
    vstore(mine + 4 * D + j0, a_b);
  }
  __syncthreads();
  if (wave == 0 && act) {
    float* base = p.part + (int64_t)blockIdx.x * 5 * D;
    auto merge = [&](float (&a)[VPL], int q) {
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        float t[VPL];
        vload(red[w] + q * D + j0, t);
#pragma unroll
        for (int i = 0; i < VPL; ++i) a[i] += t[i];
      }
      vstore(base + q * D + j0, a);
    };
    merge(a_w1, 0);
    merge(a_w2, 1);
    merge(a_w3, 2);
    merge(a_g, 3);
    merge(a_b, 4);
  }
}

// out[c] += sum_w part[w*ld + c0 + c], c < n (same shape as colsum_stage2, strided rows)
__global__ __launch_bounds__(256) void gate_ln_slice_reduce(const float* __restrict__ part, int rows, int ld, int c0,
                                                            int n, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + tx;
  float s0 = 0.f;
  if (col < n)
    for (int r = ty; r < rows; r += 4) s0 += part[(int64_t)r * ld + c0 + col];
  red[ty][tx] = s0;
  __syncthreads();
  if (ty == 0 && col < n) out[col] += (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

template <int VPL>
static void launch_gate_fwd(const GateFwdParams& p, dim3 g, hipStream_t s, bool io, bool rbf) {
  if (!io) launch(gate_ln_fwd_kernel<VPL, false, false>, g, dim3(256), 0, s, p);
  else if (rbf) launch(gate_ln_fwd_kernel<VPL, true, true>, g, dim3(256), 0, s, p);
  else launch(gate_ln_fwd_kernel<VPL, true, false>, g, dim3(256), 0, s, p);
}

static int vpl_for(int D) {
  if (D <= 64) return 1;
  if (D == 128) return 2;
  if (D == 256) return 4;
  if (D == 512) return 8;
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Readout (train.py:562-573): feats[b] = dropout([mean_{i in graph b} h_i, global_x_b, sg_b])
// ---------------------------------------------------------------------------------------------
__global__ void readout_fwd_kernel(int64_t B, int D, const float* __restrict__ h, const int64_t* __restrict__ ptr,
                                   const float* __restrict__ gx, int gdim, const float* __restrict__ sg, int sgdim,
                                   float* __restrict__ feats, DropParams drop) {
  resolve_drop(drop);
  const int64_t b = blockIdx.x;
  const int W = D + gdim + sgdim;
  const int64_t s = ptr[b], e = ptr[b + 1];
  const float inv = 1.0f / (float)max((int64_t)1, e - s);
  for (int c = threadIdx.x; c < W; c += blockDim.x) {
    float v;
    if (c < D) {
      // eight rows' loads in flight, summed in row order (bitwise the one-row loop; the pass is a
      // chain of dependent round trips otherwise: 18 us for B = 32 graphs of 60 atoms)
      float acc = 0.f;
      int64_t i = s;
      for (; i + 8 <= e; i += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = h[(i + k) * D + c];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
      }
      for (; i < e; ++i) acc += h[i * D + c];
      v = acc * inv;
    } else if (c < D + gdim) {
      v = gx[b * gdim + (c - D)];
    } else {
      v = sg[b * sgdim + (c - D - gdim)];
    }
    if (drop.active) v *= dropout_mul(drop.seed, (uint64_t)b * W + c, drop.thresh, drop.inv_keep);
    feats[b * W + c] = v;
  }
}

__global__ void pool_bwd_kernel(int64_t N, int D, const float* __restrict__ dfeats, int64_t ldf,
                                const int64_t* __restrict__ ptr, const int64_t* __restrict__ batch,
                                float* __restrict__ dh, int acc, DropParams drop) {
  resolve_drop(drop);
  // one wave per node row (its graph and count loaded once, no per-element 64-bit divide); each
  // element's value as the element loop computed it
  const int lane = threadIdx.x & 63;
  for (int64_t node = (int64_t)blockIdx.x * 4 + wave_id(); node < N; node += (int64_t)gridDim.x * 4) {
    const int64_t b = batch[node];
    const float cnt = (float)max((int64_t)1, ptr[b + 1] - ptr[b]);
    for (int c = lane; c < D; c += 64) {
      float v = dfeats[b * ldf + c] / cnt;
      if (drop.active) v *= dropout_mul(drop.seed, (uint64_t)b * ldf + c, drop.thresh, drop.inv_keep);
      const int64_t i = node * D + c;
      dh[i] = acc ? dh[i] + v : v;
    }
  }
}

__global__ void dropout_kernel(int64_t rows, int64_t cols, const float* __restrict__ x, int64_t ldx, float* __restrict__ y,
                               int64_t ldy, const float* __restrict__ ref, int64_t ldr, DropParams drop) {
  resolve_drop(drop);
  const int64_t total = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols, c = i % cols;
    float v = x[r * ldx + c];
    if (drop.active) v *= dropout_mul(drop.seed, (uint64_t)i, drop.thresh, drop.inv_keep);
    if (ref) v = ref[r * ldr + c] > 0.f ? v : 0.f;
    y[r * ldy + c] = v;
  }
}

// Hetero NLL forward+gradient, single block (B*T is small).
__global__ __launch_bounds__(256) void hetero_nll_kernel(int64_t B, int T, const float* __restrict__ heads, int64_t ldh,
                                                         const float* __restrict__ y, const float* __restrict__ w,
                                                         const float* __restrict__ lm,
                                                         const float* __restrict__ ls, float floor, float l2,
                                                         float* __restrict__ loss, float* __restrict__ dh, int64_t lddh) {
  __shared__ float red[256];
  const int64_t total = B * T;
  const float inv = 1.0f / (float)total;
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < total; i += blockDim.x) {
    const int64_t b = i / T;
    const int t = (int)(i % T);
    const float mu = heads[b * ldh + t];
    const float lvr = heads[b * ldh + T + t];
    const float lv = fmaxf(lvr, floor);
    const float yz = (logf(y[b * T + t]) - lm[t]) / ls[t];
    const float var = expf(lv);
    const float diff = mu - yz;
    const float wb = w ? w[b] : 1.0f;  // KNN sample weight (train.py:660-674): scales the NLL term only
    acc += wb * (0.5f * (lv + diff * diff / var)) + l2 * (0.5f * lv) * (0.5f * lv);
    dh[b * lddh + t] = inv * wb * diff / var;
    const float dlv = inv * (wb * 0.5f * (1.0f - diff * diff / var) + l2 * 0.5f * lv);
    dh[b * lddh + T + t] = lvr >= floor ? dlv : 0.f;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0] * inv;
}

// The same loss as the reference's CUDA step computes it under autocast(bfloat16) (train.py:653-681,
// use_amp): the heads arrive as autocast's bf16 Linear outputs and every op keeps autocast's dtype —
// clamp, the target cast, ``mean - target`` and ``0.5 * logvar`` in bf16 (fp32 arithmetic rounded to
// bf16), exp / pow / div / the means in fp32 — and the backward rounds each gradient to the dtype of
// the tensor it belongs to.  The bf16 logvar receives three gradients (from ``0.5 * logvar``, from the
// promoted add, from exp), accumulated by autograd in bf16 in that order.  Unscaled (GradScaler's
// power-of-two scale commutes with every rounding here).  Gradients bitwise those of torch's autograd
// on the same bf16 heads (tests/test_gpu_x_round5.py).
__device__ __forceinline__ float bf16r(float x) { return (float)(__bf16)x; }

__global__ __launch_bounds__(256) void hetero_nll_amp_kernel(int64_t B, int T, const float* __restrict__ heads,
                                                             int64_t ldh, const float* __restrict__ y,
                                                             const float* __restrict__ w, const float* __restrict__ lm,
                                                             const float* __restrict__ ls, float floor, float l2,
                                                             float* __restrict__ loss, float* __restrict__ dh,
                                                             int64_t lddh) {
  __shared__ float red[2][256];
  const int64_t total = B * T;
  const float floor16 = bf16r(floor);                      // clamp's Scalar min as a bf16 value
  const float dnll = (1.0f / (float)B) / (float)T;         // mean().backward, then mean(dim=1).backward
  const float dP = (1.0f * l2) / (float)total;             // (l2 * mean(log_sigma^2)).backward
  float acc = 0.f, accp = 0.f;
  for (int64_t i = threadIdx.x; i < total; i += blockDim.x) {
    const int64_t b = i / T;
    const int t = (int)(i % T);
    const float mu = bf16r(heads[b * ldh + t]);
    const float lvr = bf16r(heads[b * ldh + T + t]);
    const float lc = (lvr != lvr) ? lvr : fmaxf(lvr, floor16);
    const float yt = bf16r((logf(y[b * T + t]) - lm[t]) / ls[t]);
    const float d = bf16r(mu - yt);
    const float p = d * d;
    const float var = expf(lc);
    const float q = p / var;
    float nll = 0.5f * (lc + q);
    const float ls16 = bf16r(0.5f * lc);
    if (w) nll = nll * w[b];
    acc += nll;
    accp += ls16 * ls16;
    const float ds = (w ? dnll * w[b] : dnll) * 0.5f;
    const float g1 = bf16r(ds);
    const float dp = ds / var;
    const float dvar = -ds * ((p / var) / var);
    const float g2 = bf16r(dvar * var);
    const float g3 = bf16r(bf16r(dP * (2.0f * ls16)) * 0.5f);
    dh[b * lddh + t] = bf16r(dp * (2.0f * d));
    dh[b * lddh + T + t] = lvr >= floor16 ? bf16r(bf16r(g3 + g1) + g2) : 0.f;
  }
  red[0][threadIdx.x] = acc;
  red[1][threadIdx.x] = accp;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0][0] / (float)total + l2 * (red[1][0] / (float)total);
}

// x + stdv * N(0, 1) of element i (Box-Muller over two counter hashes of (seed, i))
__device__ __forceinline__ float jittered(float x, float stdv, uint64_t seed, int64_t i) {
  const uint32_t a = hash_u32(seed, 2 * (uint64_t)i), b = hash_u32(seed, 2 * (uint64_t)i + 1);
  const float u1 = ((float)a + 1.0f) * 2.3283064e-10f;  // (0, 1]
  const float u2 = (float)b * 2.3283064e-10f;
  const float z = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
  return x + stdv * z;
}

__global__ void add_noise_kernel(int64_t n, float* __restrict__ x, float stdv, uint64_t seed, const uint64_t* sptr) {
  seed = mix_seed(seed, sptr);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = jittered(x[i], stdv, seed, i);
}

// Two jittered copies in one launch (the step's node and global features, train.py:650-652):
// dst_k[i] = src_k[i] + stdv * z_k(i), the same values as a copy followed by add_noise_kernel.
__global__ void noisy_copy2_kernel(int64_t n1, const float* __restrict__ s1, float* __restrict__ d1, uint64_t seed1,
                                   int64_t n2, const float* __restrict__ s2, float* __restrict__ d2, uint64_t seed2,
                                   float stdv, const uint64_t* sptr) {
  seed1 = mix_seed(seed1, sptr);
  seed2 = mix_seed(seed2, sptr);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1 + n2; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n1) d1[i] = jittered(s1[i], stdv, seed1, i);
    else d2[i - n1] = jittered(s2[i - n1], stdv, seed2, i - n1);
  }
}

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_version(void) { return ALIGNN_ABI_VERSION; }
extern "C" const char* alignn_last_error(void) { return g_err; }

extern "C" int alignn_gate_ln_fwd_ex2(int64_t n, int32_t D, const float* outp, const int32_t* outp_rows,
                                      const void* R, int64_t ldr, int32_t r_bf16, const float* wbeta, const float* X,
                                      int64_t ldx, const float* ln_w, const float* ln_b, float* Xnew, int64_t ldxn,
                                      uint16_t* Xnew16, int64_t ldxn16, float* Xa, float* beta, float* mu,
                                      float* rstd, float drop_p, uint64_t seed, void* stream) {
  const int vpl = vpl_for(D);
  if (!vpl) {
    set_error("gate_ln_fwd: unsupported hidden %d", D);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (Xa && !outp_rows) {
    set_error("gate_ln_fwd: the active-row copy Xa needs outp_rows");
    return ALIGNN_E_BAD_SHAPE;
  }
  if ((r_bf16 && (ldr % 4 || (reinterpret_cast<uintptr_t>(R) & 7))) ||
      (Xnew16 && (ldxn16 % 4 || (reinterpret_cast<uintptr_t>(Xnew16) & 7)))) {
    set_error("gate_ln_fwd: bf16 rows must be 8-byte aligned (leading dimension %% 4 == 0)");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n == 0) return ALIGNN_OK;
  GateFwdParams p{n, D, 0, outp, reinterpret_cast<const float*>(R), ldr, wbeta, X, ldx, ln_w, ln_b, Xnew, ldxn, beta,
                  mu, rstd, make_drop(drop_p, seed), outp_rows, r_bf16 ? 1 : 0, 0, Xnew16, ldxn16, Xa};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 g((unsigned)((n + 3) / 4));
  const bool io = r_bf16 || Xnew16;
  switch (vpl) {
    case 1: launch_gate_fwd<1>(p, g, s, io, r_bf16 != 0); break;
    case 2: launch_gate_fwd<2>(p, g, s, io, r_bf16 != 0); break;
    case 4: launch_gate_fwd<4>(p, g, s, io, r_bf16 != 0); break;
    default: launch_gate_fwd<8>(p, g, s, io, r_bf16 != 0); break;
  }
  ALIGNN_LAUNCH_CHECK("gate_ln_fwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_gate_ln_fwd_ex(int64_t n, int32_t D, const float* outp, const int32_t* outp_rows,
                                     const void* R, int64_t ldr, int32_t r_bf16, const float* wbeta, const float* X,
                                     int64_t ldx, const float* ln_w, const float* ln_b, float* Xnew, int64_t ldxn,
                                     uint16_t* Xnew16, int64_t ldxn16, float* beta, float* mu, float* rstd,
                                     float drop_p, uint64_t seed, void* stream) {
  return alignn_gate_ln_fwd_ex2(n, D, outp, outp_rows, R, ldr, r_bf16, wbeta, X, ldx, ln_w, ln_b, Xnew, ldxn, Xnew16,
                                ldxn16, nullptr, beta, mu, rstd, drop_p, seed, stream);
}

extern "C" int alignn_gate_ln_fwd_rows(int64_t n, int32_t D, const float* outp, const int32_t* outp_rows,
                                       const float* R, int64_t ldr, const float* wbeta, const float* X, int64_t ldx,
                                       const float* ln_w, const float* ln_b, float* Xnew, int64_t ldxn, float* beta,
                                       float* mu, float* rstd, float drop_p, uint64_t seed, void* stream) {
  return alignn_gate_ln_fwd_ex(n, D, outp, outp_rows, R, ldr, 0, wbeta, X, ldx, ln_w, ln_b, Xnew, ldxn, nullptr, 0,
                               beta, mu, rstd, drop_p, seed, stream);
}

extern "C" int alignn_gate_ln_fwd(int64_t n, int32_t D, const float* outp, const float* R, int64_t ldr,
                                  const float* wbeta, const float* X, int64_t ldx, const float* ln_w,
                                  const float* ln_b, float* Xnew, int64_t ldxn, float* beta, float* mu, float* rstd,
                                  float drop_p, uint64_t seed, void* stream) {
  return alignn_gate_ln_fwd_rows(n, D, outp, nullptr, R, ldr, wbeta, X, ldx, ln_w, ln_b, Xnew, ldxn, beta, mu, rstd,
                                 drop_p, seed, stream);
}

// Waves of the gate/LayerNorm backward (each walks n / waves rows; one partial row of parameter
// gradients per wave).
#ifndef ALIGNN_GATE_BWD_WAVES
#define ALIGNN_GATE_BWD_WAVES 4096  // 2048: +1.0 % (v18); 4096 once the parameter reduction left the main stream: +0.5 % (v43_ab_gate_waves_4096.log)
#endif

template <int VPL>
static void launch_gate_bwd(const GateBwdParams& p, dim3 g, hipStream_t s, bool io, bool rbf, bool x2, bool x2bf) {
  if (!io) {
    if (x2) launch(gate_ln_bwd_kernel<VPL, false, false, true, false>, g, dim3(256), 0, s, p);
    else launch(gate_ln_bwd_kernel<VPL, false, false, false, false>, g, dim3(256), 0, s, p);
  } else if (rbf) {
    if (x2bf) launch(gate_ln_bwd_kernel<VPL, true, true, true, true>, g, dim3(256), 0, s, p);
    else if (x2) launch(gate_ln_bwd_kernel<VPL, true, true, true, false>, g, dim3(256), 0, s, p);
    else launch(gate_ln_bwd_kernel<VPL, true, true, false, false>, g, dim3(256), 0, s, p);
  } else {
    if (x2bf) launch(gate_ln_bwd_kernel<VPL, true, false, true, true>, g, dim3(256), 0, s, p);
    else if (x2) launch(gate_ln_bwd_kernel<VPL, true, false, true, false>, g, dim3(256), 0, s, p);
    else launch(gate_ln_bwd_kernel<VPL, true, false, false, false>, g, dim3(256), 0, s, p);
  }
}

extern "C" int64_t alignn_gate_ln_bwd_workspace(int64_t n, int32_t D) {
  if (n < 0 || D <= 0) return -1;
  return std::max<int64_t>(1, std::min<int64_t>(ALIGNN_GATE_BWD_WAVES, n)) * 5 * D;
}

extern "C" int alignn_gate_ln_bwd_partials_ex(int64_t n, int32_t D, float* dXnew, int64_t lddx, const float* dX_add,
                                              const float* outp, const int32_t* outp_rows, const void* R, int64_t ldr,
                                              int32_t r_bf16, const float* wbeta, const float* ln_w, const float* ln_b,
                                              const float* beta, const float* mu, const float* rstd, float* dout,
                                              void* dR, int64_t lddr, int32_t dr_bf16, float* workspace, float drop_p,
                                              uint64_t seed, void* stream) {
  const int vpl = vpl_for(D);
  if (!vpl) {
    set_error("gate_ln_bwd: unsupported hidden %d", D);
    return ALIGNN_E_UNSUPPORTED;
  }
  // r_bf16 bit 0: R is bf16; bit 1: dX_add is bf16; bit 2: dXnew is read as zero (needs dX_add; the
  // incoming gradient is dX_add alone and is written to dXnew — no zero fill of dXnew beforehand)
  const int x2bf = (r_bf16 >> 1) & 1;
  const int dxz = (r_bf16 >> 2) & 1;
  r_bf16 &= 1;
  if (dxz && !dX_add) {
    set_error("gate_ln_bwd: a zero dXnew needs dX_add");
    return ALIGNN_E_BAD_SHAPE;
  }
  if ((r_bf16 && (ldr % 4 || (reinterpret_cast<uintptr_t>(R) & 7))) ||
      (dr_bf16 && (lddr % 4 || (reinterpret_cast<uintptr_t>(dR) & 7))) ||
      (x2bf && (!dX_add || D % 4 || (reinterpret_cast<uintptr_t>(dX_add) & 7)))) {
    set_error("gate_ln_bwd: bf16 rows must be 8-byte aligned (leading dimension %% 4 == 0)");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n == 0) return ALIGNN_OK;
  const int nwaves = (int)std::min<int64_t>(ALIGNN_GATE_BWD_WAVES, n);
  GateBwdParams p{n, D, 0, dXnew, lddx, outp, reinterpret_cast<const float*>(R), ldr, wbeta, ln_w, ln_b, beta, mu, rstd,
                  dout, reinterpret_cast<float*>(dR), lddr, workspace, nwaves, 0, make_drop(drop_p, seed), outp_rows,
                  dX_add, r_bf16 ? 1 : 0, dr_bf16 ? 1 : 0, x2bf, dxz};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 g((unsigned)((nwaves + 3) / 4));
  const bool io = r_bf16 || dr_bf16 || x2bf;
  switch (vpl) {
    case 1: launch_gate_bwd<1>(p, g, s, io, r_bf16 != 0, dX_add != nullptr, x2bf != 0); break;
    case 2: launch_gate_bwd<2>(p, g, s, io, r_bf16 != 0, dX_add != nullptr, x2bf != 0); break;
    case 4: launch_gate_bwd<4>(p, g, s, io, r_bf16 != 0, dX_add != nullptr, x2bf != 0); break;
    default: launch_gate_bwd<8>(p, g, s, io, r_bf16 != 0, dX_add != nullptr, x2bf != 0); break;
  }
  ALIGNN_LAUNCH_CHECK("gate_ln_bwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_gate_ln_bwd_partials_add(int64_t n, int32_t D, float* dXnew, int64_t lddx, const float* dX_add,
                                               const float* outp, const int32_t* outp_rows, const float* R, int64_t ldr,
                                               const float* wbeta, const float* ln_w, const float* ln_b,
                                               const float* beta, const float* mu, const float* rstd, float* dout,
                                               float* dR, int64_t lddr, float* workspace, float drop_p, uint64_t seed,
                                               void* stream) {
  return alignn_gate_ln_bwd_partials_ex(n, D, dXnew, lddx, dX_add, outp, outp_rows, R, ldr, 0, wbeta, ln_w, ln_b, beta,
                                        mu, rstd, dout, dR, lddr, 0, workspace, drop_p, seed, stream);
}

extern "C" int alignn_gate_ln_bwd_partials(int64_t n, int32_t D, const float* dXnew, int64_t lddx, const float* outp,
                                           const int32_t* outp_rows, const float* R, int64_t ldr, const float* wbeta,
                                           const float* ln_w, const float* ln_b, const float* beta, const float* mu,
                                           const float* rstd, float* dout, float* dR, int64_t lddr, float* workspace,
                                           float drop_p, uint64_t seed, void* stream) {
  return alignn_gate_ln_bwd_partials_add(n, D, const_cast<float*>(dXnew), lddx, nullptr, outp, outp_rows, R, ldr, wbeta,
                                         ln_w, ln_b, beta, mu, rstd, dout, dR, lddr, workspace, drop_p, seed, stream);
}

extern "C" int alignn_gate_ln_bwd_reduce(int64_t n, int32_t D, const float* workspace, float* d_wbeta, float* d_ln_w,
                                         float* d_ln_b, void* stream) {
  if (!vpl_for(D)) {
    set_error("gate_ln_bwd: unsupported hidden %d", D);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (n == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nwaves = (int)std::min<int64_t>(ALIGNN_GATE_BWD_WAVES, n);
  const int parts = (nwaves + 3) / 4;  // one partial row per workgroup of the partials kernel
  // d_wbeta[3D] | d_ln_w[D] | d_ln_b[D]: one 5D-wide fixed-order reduction when the three are
  // adjacent in memory (the flat gradient layout), else one per slice of the 5D-wide partial rows.
  const unsigned strips3 = (unsigned)((3 * D + 63) / 64), strips1 = (unsigned)((D + 63) / 64);
  if (d_ln_w == d_wbeta + 3 * D && d_ln_b == d_ln_w + D) {
    launch(colsum_stage2<0>, dim3(colsum_blocks(5 * D)), dim3(kColsumThreads), 0, s, workspace, parts,
           (int64_t)5 * D, d_wbeta, 1);
  } else {
    launch(gate_ln_slice_reduce, dim3(strips3), dim3(256), 0, s, workspace, parts, 5 * D, 0, 3 * D, d_wbeta);
    launch(gate_ln_slice_reduce, dim3(strips1), dim3(256), 0, s, workspace, parts, 5 * D, 3 * D, D, d_ln_w);
    launch(gate_ln_slice_reduce, dim3(strips1), dim3(256), 0, s, workspace, parts, 5 * D, 4 * D, D, d_ln_b);
  }
  ALIGNN_LAUNCH_CHECK("gate_ln param-grad reduction");
  return ALIGNN_OK;
}

extern "C" int alignn_gate_ln_bwd_rows(int64_t n, int32_t D, const float* dXnew, int64_t lddx, const float* outp,
                                       const int32_t* outp_rows, const float* R, int64_t ldr, const float* wbeta,
                                       const float* ln_w, const float* ln_b, const float* beta, const float* mu,
                                       const float* rstd, float* dout, float* dR, int64_t lddr, float* d_wbeta,
                                       float* d_ln_w, float* d_ln_b, float* workspace, float drop_p, uint64_t seed,
                                       void* stream) {
  int rc = alignn_gate_ln_bwd_partials(n, D, dXnew, lddx, outp, outp_rows, R, ldr, wbeta, ln_w, ln_b, beta, mu, rstd,
                                       dout, dR, lddr, workspace, drop_p, seed, stream);
  if (rc != ALIGNN_OK) return rc;
  return alignn_gate_ln_bwd_reduce(n, D, workspace, d_wbeta, d_ln_w, d_ln_b, stream);
}

extern "C" int alignn_gate_ln_bwd(int64_t n, int32_t D, const float* dXnew, int64_t lddx, const float* outp,
                                  const float* R, int64_t ldr, const float* wbeta, const float* ln_w, const float* ln_b,
                                  const float* beta, const float* mu, const float* rstd, float* dout, float* dR,
                                  int64_t lddr, float* d_wbeta, float* d_ln_w, float* d_ln_b, float* workspace,
                                  float drop_p, uint64_t seed, void* stream) {
  return alignn_gate_ln_bwd_rows(n, D, dXnew, lddx, outp, nullptr, R, ldr, wbeta, ln_w, ln_b, beta, mu, rstd, dout, dR,
                                 lddr, d_wbeta, d_ln_w, d_ln_b, workspace, drop_p, seed, stream);
}

extern "C" int alignn_readout_feats_fwd(int64_t B, int32_t D, const float* h, const int64_t* ptr, const float* global_x,
                                        int32_t gdim, const float* sg, int32_t sgdim, float* feats, float drop_p,
                                        uint64_t seed, void* stream) {
  if (B == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(readout_fwd_kernel, dim3((unsigned)B), dim3(256), 0, s, B, D, h, ptr, global_x, gdim, sg, sgdim,
                     feats, make_drop(drop_p, seed));
  ALIGNN_LAUNCH_CHECK("readout_fwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_readout_pool_bwd(int64_t B, int64_t N, int32_t D, const float* dfeats, int64_t ldf,
                                       const int64_t* ptr, const int64_t* batch, float* dh, int32_t accumulate,
                                       float drop_p, uint64_t seed, void* stream) {
  (void)B;
  if (N == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(pool_bwd_kernel, dim3(grid_for(N, 4)), dim3(256), 0, s, N, D, dfeats, ldf, ptr, batch, dh,
                     accumulate, make_drop(drop_p, seed));
  ALIGNN_LAUNCH_CHECK("pool_bwd_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_dropout_f32(int64_t rows, int64_t cols, const float* x, int64_t ldx, float* y, int64_t ldy,
                                  const float* relu_ref, int64_t ldr, float drop_p, uint64_t seed, void* stream) {
  if (rows * cols == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(dropout_kernel, dim3(grid_for(rows * cols)), dim3(256), 0, s, rows, cols, x, ldx, y, ldy, relu_ref,
                     ldr, make_drop(drop_p, seed));
  ALIGNN_LAUNCH_CHECK("dropout_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_hetero_nll(int64_t B, int32_t T, const float* heads, int64_t ldh, const float* y,
                                 const float* weights, const float* log_means, const float* log_stds, float floor,
                                 float l2, float* loss, float* dheads, int64_t lddh, void* stream) {
  if (B <= 0 || T <= 0) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(hetero_nll_kernel, dim3(1), dim3(256), 0, s, B, T, heads, ldh, y, weights, log_means, log_stds,
                     floor, l2, loss, dheads, lddh);
  ALIGNN_LAUNCH_CHECK("hetero_nll_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_hetero_nll_amp(int64_t B, int32_t T, const float* heads, int64_t ldh, const float* y,
                                     const float* weights, const float* log_means, const float* log_stds,
                                     float floor, float l2, float* loss, float* dheads, int64_t lddh, void* stream) {
  if (B <= 0 || T <= 0) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(hetero_nll_amp_kernel, dim3(1), dim3(256), 0, s, B, T, heads, ldh, y, weights, log_means, log_stds,
         floor, l2, loss, dheads, lddh);
  ALIGNN_LAUNCH_CHECK("hetero_nll_amp_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_add_noise_f32(int64_t n, float* x, float stdv, uint64_t seed, void* stream) {
  if (n == 0 || stdv == 0.f) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(add_noise_kernel, dim3(grid_for(n)), dim3(256), 0, s, n, x, stdv, seed, g_step_seed);
  ALIGNN_LAUNCH_CHECK("add_noise_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_noisy_copy2_f32(int64_t n1, const float* src1, float* dst1, uint64_t seed1, int64_t n2,
                                      const float* src2, float* dst2, uint64_t seed2, float stdv, void* stream) {
  if (n1 < 0 || n2 < 0) return ALIGNN_E_BAD_SHAPE;
  if (n1 + n2 == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(noisy_copy2_kernel, dim3(grid_for(n1 + n2)), dim3(256), 0, s, n1, src1, dst1, seed1, n2, src2, dst2, seed2,
         stdv, g_step_seed);
  ALIGNN_LAUNCH_CHECK("noisy_copy2_kernel");
  return ALIGNN_OK;
}

extern "C" void alignn_set_step_seed(const uint64_t* device_ptr) { alignn::g_step_seed = device_ptr; }
