// lgmx.hip — the line-graph attention of config C3 (bf16 storage, the reference's CUDA autocast,
// train.py:632-636) on the matrix cores, with the edge features recomputed from the 11 raw angle inputs.
//
// Semantics: PyG 2.7.0 TransformerConv message + utils.softmax + aggregate (callers
// train.py:315), in the engine's edge-feature algebra: per target d and head h the score of
// edge t = (s -> d) is  z = (<Q_d,h, K_s,h> + <u_d,h, f_t> + c_h) / sqrt(C)  with u_d,h = M_h^T Q_d,h and
// f_t = relu(W1 x_t + b1) the angle encoder's hidden layer (train.py:358-364, :553-556); the forward
// aggregates aggV = sum alpha' V_s and S_h = sum alpha'_h f_t, the target-side backward dz, alpha' per
// edge, dq = sum dz K_s and Sz_h = sum dz_h f_t.  Same contract as lgconv.hip's kernels (alignn_lg_fwd_x /
// alignn_lg_bwd_dst_x with bf16 K|V), which these replace at bf16.
//
// Layout: one workgroup of four waves per target (the schedule's list, descending in-degree: a dynamic
// LPT schedule); wave w owns features [64 w, 64 w + 64) — of f for the f-products (all four heads, a
// partial score summed over the waves through LDS) and of Q/K/V (= head w) for the gathered products.
// Edges go in pairs of 16-edge tiles.  Every product is a v_mfma_f32_16x16x32_bf16 (fp32 accumulation):
//   * f recomputed twice from the tile's raw inputs x (bf16, with a ones column carrying b1: autocast
//     rounds x, W1 and b1 to bf16 and accumulates in fp32 — train.py:554 under :636), as f^T = W1 x^T
//     (features on the rows: the score product sums over them) and f = x W1^T (edges on the rows: the
//     aggregation sums over them); each accumulator tile is the next product's operand as it lies
//     (cdna_hip_programming.md §3 'An accumulator tile as the next MFMA's operand');
//   * the score tile Z[edge][col] = f^T' U^T + K_g Q^blk, 16 columns = the four heads repeated, so the
//     score accumulator is directly the A operand (heads on the rows) of the aggregation;
//   * aggregation over 32 edges: S_h += alpha'^T f, aggV += alpha'^T V_g with the gathered V rows staged
//     in LDS and read transposed (ds_read_b64_tr_b16); alpha' enters as bf16 hi + lo parts (two
//     products), so the weights keep ~16 significant bits, as autocast keeps them in fp32.
// Softmax, its statistics and every accumulator are fp32; online softmax over the pairs.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "vec.h"

namespace alignn {
namespace lgm {

constexpr int D = 256;
constexpr int H = 4;
constexpr int KX = 11;    // raw angle inputs per triplet (lg_edge_attr width, SURVEY §8: F_a = 11)
constexpr int NT = 256;   // four waves
constexpr int LDV = 72;   // LDS image row (bf16): 64 features + 8 pad (144 B)
constexpr int IMG = 32 * LDV;

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

struct Params {
  int64_t n, m;
  const int32_t* off;
  const int32_t* src_at;
  const int32_t* items; int64_t n_items;
  const float* Q; int64_t ldq;            // fp32 Q rows (cols 0..D)
  const uint16_t* KV16; int64_t ldkv;     // bf16 K (col 0) | V (col D) rows
  const float* U; const float* Vd;        // [n, H, D]
  const float* wbar;                      // [D] or null
  const float* X; int64_t ldx;            // raw angle inputs [m, 12] (11 used), target-sorted
  const float* W1; const float* b1;       // [D, 11], [D]
  float* aggV; float* S; float* sumA; float* mstat; float* den;
  const float* dout; const float* outp; const float* mstat_in; const float* den_in;
  float* dq; int64_t lddq; float* Sz; float* sigz; float* dz_e; float* alpha_e;
  DropParams drop;
};

__device__ __forceinline__ f4 mma(const bf8& a, const bf8& b, const f4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ f4 ld4(const float* __restrict__ p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ bf8 pack8(const f4& a, const f4& b) {
  bf8 v;
  v[0] = (__bf16)a[0]; v[1] = (__bf16)a[1]; v[2] = (__bf16)a[2]; v[3] = (__bf16)a[3];
  v[4] = (__bf16)b[0]; v[5] = (__bf16)b[1]; v[6] = (__bf16)b[2]; v[7] = (__bf16)b[3];
  return v;
}
// relu(bf16(a | b)): autocast's order (the Linear's bf16 output, then ReLU), on the rounded bits — a
// bf16 orders as its int16 bits do on either side of zero, so one v_pk_max_i16 per two elements
__device__ __forceinline__ bf8 relu_pack8(const f4& a, const f4& b) {
  u4 v = __builtin_bit_cast(u4, pack8(a, b));
#pragma unroll
  for (int i = 0; i < 4; ++i) asm("v_pk_max_i16 %0, %1, 0" : "=v"(v[i]) : "v"(v[i]));
  return __builtin_bit_cast(bf8, v);
}
// v = hi + lo with hi = bf16(v), lo = bf16(v - hi): the A operand of an aggregation as two fragments
__device__ __forceinline__ void split8(const f4& a, const f4& b, bf8& hi, bf8& lo) {
  hi = pack8(a, b);
  f4 ra, rb;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ra[j] = a[j] - (float)hi[j];
    rb[j] = b[j] - (float)hi[4 + j];
  }
  lo = pack8(ra, rb);
}
__device__ __forceinline__ float pick4(const f4& v, int i) {
  float r = v[0];
  r = i == 1 ? v[1] : r;
  r = i == 2 ? v[2] : r;
  r = i == 3 ? v[3] : r;
  return r;
}
// sum / max over the four 16-lane rows (lanes c, c+16, c+32, c+48; every lane gets the result)
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

// A/B fragment of x_aug (lane (g, c): the edge's inputs k = 8 g .. 8 g + 7): g = 0 x[0..7]; g = 1 x[8..10]
// and 1 (the bias column, k = 11); g >= 2 zero.  As the B operand of W1 x^T and the A operand of x W1^T.
__device__ __forceinline__ bf8 x_frag(const Params& p, int32_t te, int g) {
  const float* row = p.X + __umul24((uint32_t)te, (uint32_t)p.ldx);   // m < 2^24 (lgm_check)
  const f4 a = ld4(row + (g == 0 ? 0 : 8));   // unconditional (every row has 12 floats)
  const f4 b = ld4(row + 4);
  const bool lo_on = g < 2, g0 = g == 0;
  const f4 lo = {lo_on ? a[0] : 0.f, lo_on ? a[1] : 0.f, lo_on ? a[2] : 0.f, g0 ? a[3] : (g == 1 ? 1.f : 0.f)};
  const f4 hi = g0 ? b : zero4();
  return pack8(lo, hi);
}
// W1_aug fragment of feature 64 w + 16 tau + c: k < 11 W1, k = 11 b1, else 0 (bf16: autocast's cast)
__device__ __forceinline__ bf8 w1_frag(const Params& p, int phi, int g) {
  bf8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g + j;
    const float x = k < KX ? p.W1[phi * KX + k] : (k == KX ? p.b1[phi] : 0.f);
    v[j] = (__bf16)x;
  }
  return v;
}
// B operand of an f-product over this wave's features for k-step s: lane (g, c) element j is
// P[d][c & 3][64 w + 32 s + 16 (j >> 2) + 4 g + (j & 3)] (the row order of two f^T accumulator tiles)
__device__ __forceinline__ bf8 u_frag(const float* __restrict__ P, int64_t d, int hc, int w, int s, int g) {
  const float* base = P + (d * H + hc) * D + 64 * w + 32 * s + 4 * g;
  return pack8(ld4(base), ld4(base + 16));
}
// B operand of a gathered product (head w only): lane (g, c) element j is row[64 w + 32 s + 8 g + j]
// in the columns of head w (c & 3 == w), else 0
__device__ __forceinline__ bf8 q_frag(const float* __restrict__ row, int w, int s, int g, bool on) {
  const float* base = row + 64 * w + 32 * s + 8 * g;
  f4 a = ld4(base), b = ld4(base + 4);
  if (!on) { a = zero4(); b = zero4(); }
  return pack8(a, b);
}
// A operand of a gathered product: lane (g, c) = the bf16 row's features 64 w + 32 s + 8 g .. + 7
__device__ __forceinline__ bf8 kv_frag(const uint16_t* __restrict__ row, int w, int s, int g) {
  return __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(row + 64 * w + 32 * s + 8 * g));
}
// LDS image row of pair edge e (tile e >> 4, edge e & 15): the k order of two accumulator tiles
__device__ __forceinline__ int img_row(int e) { return 8 * ((e & 15) >> 2) + 4 * (e >> 4) + (e & 3); }
// B operand from the image, read transposed: lane (g, i) gets image column 16 tau + i of rows 8 g .. 8 g + 7
__device__ __forceinline__ bf8 tr_frag(const __bf16* img, int tau, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int row = 8 * g + (li >> 2), col = 16 * tau + 4 * (li & 3);
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + row * LDV + col));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + (row + 4) * LDV + col));
  const s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf8, v);
}
// A operand from the image (row read): lane (g, c) = tile x's edge c, image columns 32 s + 8 g .. + 7
__device__ __forceinline__ bf8 row_frag(const __bf16* img, int x, int s, int g, int c) {
  const int row = img_row(16 * x + c);
  return __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(img + row * LDV + 32 * s + 8 * g));
}
// Dropout multipliers of the Z layout (lane (g, c) register r: edge t0 + 4 g + r, head c & 3): one
// hash per lane (edge t0 + lane / 4, head lane % 4 — the hash of every other kernel's mask of that
// (edge, head)), then a bpermute per register
template <bool DROP>
__device__ __forceinline__ f4 drop4(const DropParams& dp, int32_t t0, int lane, int g, int hc) {
  if constexpr (!DROP) {
    return f4{1.f, 1.f, 1.f, 1.f};
  } else {
    const float mine = dropout_mul(dp.seed, (uint64_t)(t0 + (lane >> 2)) * H + (lane & 3), dp.thresh, dp.inv_keep);
    f4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __shfl(mine, 16 * g + 4 * i + hc, 64);
    return r;
  }
}

// ---------------------------------------------------------------------------------------------
// Per-target edge stream.  The source ids of a 256-edge window of the segment are loaded once (lane l:
// window edges l, 64 + l, 128 + l, 192 + l) and handed out by bpermute, so a pair's gathers wait for
// one memory round trip, not two; the loads of pair p + 1 are issued before pair p is computed (two
// register sets).  Every load of the pair stream is unconditional, its index clamped into the segment
// (and the edge arrays): a value that comes from a load on one path of a branch and not on the other
// makes the compiler's wait at the join a full vmcnt(0) drain — every prefetched load of the next pair
// with it (that one branch, a direct src_at load for edges past 256, serialised the round-5 kernels'
// six gathers per pair).  A window past the first (segments longer than 256 edges, above the default
// heavy threshold) is loaded between pairs, and drained on its own path.
// ---------------------------------------------------------------------------------------------
struct Seg {
  int32_t beg, deg, wb;   // segment start and length; window base (a multiple of 256)
  int32_t s0, s1, s2, s3; // window edge wb + 64 u + lane's source (separate registers: an array
                          // indexed by a select becomes an LDS alloca)
};
// edge row of segment edge k, clamped into the segment and the edge arrays (m > 0)
__device__ __forceinline__ int32_t seg_edge(const Params& p, const Seg& sg, int32_t k) {
  return min(sg.beg + min(max(k, 0), max(sg.deg, 1) - 1), (int32_t)p.m - 1);
}
__device__ __forceinline__ void seg_window_load(const Params& p, Seg& sg, int32_t wb, int lane) {
  sg.wb = wb;
  sg.s0 = p.src_at[seg_edge(p, sg, wb + lane)];
  sg.s1 = p.src_at[seg_edge(p, sg, wb + 64 + lane)];
  sg.s2 = p.src_at[seg_edge(p, sg, wb + 128 + lane)];
  sg.s3 = p.src_at[seg_edge(p, sg, wb + 192 + lane)];
}
__device__ __forceinline__ void seg_load(const Params& p, Seg& sg, int32_t beg, int32_t end, int lane) {
  sg.beg = beg;
  sg.deg = end - beg;
  seg_window_load(p, sg, 0, lane);
}
// before the loads of pair pr (wave-uniform): move the window when pr starts a new 256-edge block.
// The rare path waits for its own loads (the asm uses them), so the join carries no pending load.
__device__ __forceinline__ void seg_advance(const Params& p, Seg& sg, int pr, int lane) {
  const int32_t wb = (32 * pr) & ~255;
  if (wb != sg.wb) {
    seg_window_load(p, sg, wb, lane);
    asm volatile("" : "+v"(sg.s0), "+v"(sg.s1), "+v"(sg.s2), "+v"(sg.s3));
  }
}
// One pair's loads: raw inputs (x_aug fragments), the gathered A-operand rows of both tiles (columns
// `gcol`: fwd K, bwd V) and the 32 rows staged into the LDS image (columns `rcol`: fwd V, bwd K)
struct PairIn {
  bf8 X[2];
  bf8 G[2][2];
  u4 R[4];
};
__device__ __forceinline__ void pair_load(const Params& p, const Seg& sg, int pr, PairIn& in, int gcol, int rcol,
                                          int w, int lane) {
  const int g = lane >> 4, c = lane & 15;
  const int32_t k0 = 32 * pr;
  // the pair's 32 edges lie in one 64-edge block of the window (k0 is 32-aligned)
  const int r = (k0 - sg.wb) >> 6;
  int32_t s0 = sg.s0, s1 = sg.s1, s2 = sg.s2, s3 = sg.s3;
  asm("" : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3));   // values, not a select of addresses (no alloca)
  int32_t blk = s0;
  blk = r == 1 ? s1 : blk;
  blk = r == 2 ? s2 : blk;
  blk = r == 3 ? s3 : blk;
  const int32_t last = max(sg.deg, 1) - 1;
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int32_t k = k0 + 16 * x + c;
    in.X[x] = x_frag(p, seg_edge(p, sg, k), g);
    const int32_t s = __shfl(blk, min(k, last) & 63, 64);
    const uint16_t* row = p.KV16 + (__umul24((uint32_t)s, (uint32_t)p.ldkv) + gcol);   // n ldkv < 2^31
    in.G[x][0] = kv_frag(row, w, 0, g);
    in.G[x][1] = kv_frag(row, w, 1, g);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = (lane >> 3) + 8 * u;
    const int32_t s = __shfl(blk, min(k0 + e, last) & 63, 64);
    in.R[u] = *reinterpret_cast<const u4*>(p.KV16 + (__umul24((uint32_t)s, (uint32_t)p.ldkv) + rcol + 64 * w +
                                                       8 * (lane & 7)));
  }
  asm volatile("" ::: "memory");   // keep the loads here (else they sink to their use, one pair later)
}
__device__ __forceinline__ void pair_stage(__bf16* img, const PairIn& in, int lane) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = (lane >> 3) + 8 * u;
    *reinterpret_cast<u4*>(img + img_row(e) * LDV + 8 * (lane & 7)) = in.R[u];
  }
}

// =============================================================================================
// Forward
// =============================================================================================
struct FwdState {
  f4 Sacc[4], Vacc[4];
  float m, den_l, sa_l;
};
// outputs of one target (lane (g, c): head c & 3 statistics; accumulator register r = head r)
__device__ __forceinline__ void fwd_out(const Params& p, const FwdState& st, int64_t d, int w, int lane) {
  const int g = lane >> 4, c = lane & 15;
  const float dn = rows_sum(st.den_l) + 1e-16f;
  const float inv = 1.0f / dn;
  const float sa = rows_sum(st.sa_l);
  const f4 iv = {readlane_f(inv, 0), readlane_f(inv, 1), readlane_f(inv, 2), readlane_f(inv, 3)};
  const float ig = pick4(iv, g);
#pragma unroll
  for (int t = 0; t < 4; ++t) p.S[(d * H + g) * D + 64 * w + 16 * t + c] = pick4(st.Sacc[t], g) * ig;
  f4 vv = st.Vacc[0];
  vv = g == 1 ? st.Vacc[1] : vv;
  vv = g == 2 ? st.Vacc[2] : vv;
  vv = g == 3 ? st.Vacc[3] : vv;
  p.aggV[d * D + 64 * w + 16 * g + c] = pick4(vv, w) * pick4(iv, w);
  if (w == 0 && lane < H) {
    p.sumA[d * H + lane] = sa * inv;
    p.mstat[d * H + lane] = st.m;
    p.den[d * H + lane] = dn;
  }
}
__device__ __forceinline__ void fwd_init(FwdState& st) {
#pragma unroll
  for (int i = 0; i < 4; ++i) { st.Sacc[i] = zero4(); st.Vacc[i] = zero4(); }
  st.m = -INFINITY;
  st.den_l = 0.f;
  st.sa_l = 0.f;
}


// W1 fragments of this wave: in registers, or in LDS (lane-linear 16-byte slots, the persistent kernel)
struct W1Regs {
  bf8 f[4];
  __device__ __forceinline__ bf8 get(int t, int) const { return f[t]; }
};
struct W1Lds {
  const u4* base;   // this wave's 4 x 64 slots
  __device__ __forceinline__ bf8 get(int t, int lane) const { return __builtin_bit_cast(bf8, base[64 * t + lane]); }
};

template <bool DROP, class W1S>
__device__ __forceinline__ void fwd_pair(const Params& p, const PairIn& in, int32_t tp, int32_t end, int buf,
                                         __bf16* img, float (*zb)[4][2][H][16], const W1S& W1f,
                                         const bf8 (&Uf)[2], const bf8 (&Qf)[2], float cadd, FwdState& st, int w,
                                         int lane) {
  const int g = lane >> 4, c = lane & 15, hc = c & 3;
  const float scale = 0.125f;   // 1 / sqrt(C), C = 64
  pair_stage(img, in, lane);    // V rows (head w's columns) for the transposed reads below
  // ---- partial scores of both tiles, and f with the edges on the rows (the aggregation's B operand)
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    f4 T[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) T[t] = mma(W1f.get(t, lane), in.X[x], zero4());
    f4 Zp = mma(relu_pack8(T[0], T[1]), Uf[0], zero4());
    Zp = mma(relu_pack8(T[2], T[3]), Uf[1], Zp);
    Zp = mma(in.G[x][0], Qf[0], Zp);
    Zp = mma(in.G[x][1], Qf[1], Zp);
#pragma unroll
    for (int r = 0; r < 4; ++r) Zp[r] += cadd;
    if (c < H) *reinterpret_cast<f4*>(&zb[buf][w][x][c][4 * g]) = Zp;
  }
  bf8 FB[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf8 Wt = W1f.get(t, lane);
    FB[t] = relu_pack8(mma(in.X[0], Wt, zero4()), mma(in.X[1], Wt, zero4()));
  }
  __syncthreads();
  f4 z[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    z[x] = *reinterpret_cast<const f4*>(&zb[buf][0][x][hc][4 * g]);
#pragma unroll
    for (int v = 1; v < 4; ++v) z[x] += *reinterpret_cast<const f4*>(&zb[buf][v][x][hc][4 * g]);
  }
  // ---- online softmax over the pair (lane (g, c): head c & 3, edges tp + 16 x + 4 g + r)
  float mt = -INFINITY;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = tp + 16 * x + 4 * g + r < end;
      z[x][r] = ok ? z[x][r] * scale : -INFINITY;
      mt = fmaxf(mt, z[x][r]);
    }
  mt = rows_max(mt);
  const float mn = fmaxf(st.m, mt);      // finite: the pair's first edge is valid
  const float corr = __expf(st.m - mn);  // 0 on the first pair (m = -inf)
  st.m = mn;
  f4 al[2];
  float ps = 0.f, as = 0.f;
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const f4 mul = drop4<DROP>(p.drop, tp + 16 * x, lane, g, hc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(z[x][r] - mn);   // 0 past the segment end
      ps += e;
      al[x][r] = e * mul[r];
      as += al[x][r];
    }
  }
  st.den_l = st.den_l * corr + ps;
  st.sa_l = st.sa_l * corr + as;
  const float c0 = readlane_f(corr, 0), c1 = readlane_f(corr, 1), c2 = readlane_f(corr, 2), c3 = readlane_f(corr, 3);
  if (c0 != 1.f || c1 != 1.f || c2 != 1.f || c3 != 1.f) {   // wave-uniform
    const f4 cv = {c0, c1, c2, c3};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st.Sacc[t] *= cv;
      st.Vacc[t] *= cv;
    }
  }
  bf8 AH, AL;
  split8(al[0], al[1], AH, AL);
  // ---- aggregation: S_h += alpha'^T f; aggV += alpha'^T V (head w's columns, the image read transposed)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    st.Sacc[t] = mma(AH, FB[t], st.Sacc[t]);
    st.Sacc[t] = mma(AL, FB[t], st.Sacc[t]);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf8 VB = tr_frag(img, t, lane);
    st.Vacc[t] = mma(AH, VB, st.Vacc[t]);
    st.Vacc[t] = mma(AL, VB, st.Vacc[t]);
  }
  asm volatile("" ::: "memory");
}

template <bool DROP>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void lgm_fwd_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  __shared__ __attribute__((aligned(16))) __bf16 imgs[4 * IMG];
  __shared__ __attribute__((aligned(16))) float zb[2][4][2][H][16];
  const int lane = threadIdx.x & 63, w = wave_id();
  const int g = lane >> 4, c = lane & 15, hc = c & 3;
  __bf16* img = imgs + w * IMG;
  const int64_t d = (int64_t)uni(sld(p.items, (int64_t)blockIdx.x));
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));

  FwdState st;
  fwd_init(st);

  if (beg < end) {
    Seg sg;
    seg_load(p, sg, beg, end, lane);
    W1Regs W1f;
    bf8 Uf[2], Qf[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) W1f.f[t] = w1_frag(p, 64 * w + 16 * t + c, g);
    const float* qrow = p.Q + d * p.ldq;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Uf[s] = u_frag(p.U, d, hc, w, s, g);
      Qf[s] = q_frag(qrow, w, s, g, hc == w);
    }
    float cw = 0.f;   // c_w = <wbar_w, Q_w> (the angle encoder's b2 folded through lin_edge)
    if (p.wbar) cw = wave_sum(p.wbar[64 * w + lane] * qrow[64 * w + lane]);
    const float cadd = hc == w ? cw : 0.f;
    const int np = (end - beg + 31) / 32;
    PairIn A, B;
    pair_load(p, sg, 0, A, 0, D, w, lane);
    for (int pr = 0; pr < np; pr += 2) {
      const int n1 = min(pr + 1, np - 1), n2 = min(pr + 2, np - 1);
      seg_advance(p, sg, n1, lane);
      pair_load(p, sg, n1, B, 0, D, w, lane);
      fwd_pair<DROP>(p, A, beg + 32 * pr, end, pr & 1, img, zb, W1f, Uf, Qf, cadd, st, w, lane);
      if (pr + 1 >= np) break;
      seg_advance(p, sg, n2, lane);
      pair_load(p, sg, n2, A, 0, D, w, lane);
      fwd_pair<DROP>(p, B, beg + 32 * (pr + 1), end, (pr + 1) & 1, img, zb, W1f, Uf, Qf, cadd, st, w, lane);
    }
  }
  fwd_out(p, st, d, w, lane);
}

// Persistent form: a grid of a few workgroups per CU walks the schedule's list (workgroup b takes items
// b, b + G, b + 2G, ...: the same XCD for every item of a block under round-robin placement, G % 8 == 0),
// and the loads run one unit (target, pair) ahead across target boundaries — the next target's source
// ids and constant fragments while the current target runs, its first pair's gathers during the current
// target's last pair — so no target waits for its own prologue.
struct FwdTgt {
  int64_t d;
  int32_t beg, end;
  Seg sg;
  bf8 Uf[2], Qf[2];
  float qv, wbv;   // this lane's element of Q_w and wbar_w (c_w is their wave sum)
};
__device__ __forceinline__ void fwd_tgt_load(const Params& p, int64_t item, FwdTgt& T, int w, int lane) {
  const int g = lane >> 4, c = lane & 15, hc = c & 3;
  T.d = (int64_t)uni(sld(p.items, item));
  T.beg = uni(sld(p.off, T.d));
  T.end = uni(sld(p.off, T.d + 1));
  seg_load(p, T.sg, T.beg, T.end, lane);   // (clamped: an empty segment reads a valid id)
  const float* qrow = p.Q + T.d * p.ldq;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    T.Uf[s] = u_frag(p.U, T.d, hc, w, s, g);
    T.Qf[s] = q_frag(qrow, w, s, g, hc == w);
  }
  T.qv = qrow[64 * w + lane];
  T.wbv = p.wbar ? p.wbar[64 * w + lane] : 0.f;
}

template <bool DROP>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void lgm_fwd_p_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  __shared__ __attribute__((aligned(16))) __bf16 imgs[4 * IMG];
  __shared__ __attribute__((aligned(16))) float zb[2][4][2][H][16];
  const int lane = threadIdx.x & 63, w = wave_id();
  const int g = lane >> 4, c = lane & 15, hc = c & 3;
  __shared__ u4 w1s[4][4 * 64];   // each wave's W1 fragments (16 KB: registers are the binding resource here)
  __bf16* img = imgs + w * IMG;
  int64_t it = blockIdx.x;
  if (it >= p.n_items) return;
  if (p.m == 0) {   // no edges: every target's outputs are the empty softmax's
    FwdState st;
    fwd_init(st);
    for (; it < p.n_items; it += gridDim.x) fwd_out(p, st, (int64_t)uni(sld(p.items, it)), w, lane);
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) w1s[w][64 * t + lane] = __builtin_bit_cast(u4, w1_frag(p, 64 * w + 16 * t + c, g));
  const W1Lds W1f{w1s[w]};   // read back by this wave only (LDS is in order within a wave)
  // The unit stream (target T, pair pr): each unit issues the next unit's loads — (T, pr + 1), or the
  // next target N's first pair — then computes its own.  An empty target is one unit with no compute.
  // Two register sets alternate (a copy of a loaded set would wait for its loads); every load is
  // unconditional: N past the list end is the list's last item again, its loads unused.
  FwdTgt T, N;
  fwd_tgt_load(p, it, T, w, lane);
  fwd_tgt_load(p, min<int64_t>(it + gridDim.x, p.n_items - 1), N, w, lane);
  PairIn A, B;
  pair_load(p, T.sg, 0, A, 0, D, w, lane);
  FwdState st;
  fwd_init(st);
  float cadd = wave_sum(T.wbv * T.qv);   // c_w = <wbar_w, Q_w> (wbv = 0 without wbar), head w's columns
  cadd = hc == w ? cadd : 0.f;
  int pr = 0, buf = 0;
  bool done = false;
  auto unit = [&](const PairIn& cur, PairIn& nxt) {
    const int np = (T.end - T.beg + 31) / 32;
    const bool last = pr + 1 >= max(np, 1);
    if (!last) {
      seg_advance(p, T.sg, pr + 1, lane);
      pair_load(p, T.sg, pr + 1, nxt, 0, D, w, lane);
    } else {
      pair_load(p, N.sg, 0, nxt, 0, D, w, lane);
    }
    if (np > 0) fwd_pair<DROP>(p, cur, T.beg + 32 * pr, T.end, buf, img, zb, W1f, T.Uf, T.Qf, cadd, st, w, lane);
    buf ^= 1;
    if (!last) {
      ++pr;
      return;
    }
    fwd_out(p, st, T.d, w, lane);
    it += gridDim.x;
    if (it >= p.n_items) {
      done = true;
      return;
    }
    T = N;
    fwd_tgt_load(p, min<int64_t>(it + gridDim.x, p.n_items - 1), N, w, lane);
    fwd_init(st);
    const float cw = wave_sum(T.wbv * T.qv);
    cadd = hc == w ? cw : 0.f;
    pr = 0;
  };
  while (true) {
    unit(A, B);
    if (done) break;
    unit(B, A);
    if (done) break;
  }
}

// =============================================================================================
// Target-side backward: dz, alpha' per edge; dq (the gathered part), Sz, sigz per target
// =============================================================================================
struct BwdConst {
  bf8 W1f[4], Uf[2], Qf[2], Vf[2], Of[2];
  float zadd, yadd, mst, invden, pdl;
};
struct BwdState {
  f4 Sacc[4], Qacc[4];
  float sg_l;
};

template <bool DROP>
__device__ __forceinline__ void bwd_pair(const Params& p, const PairIn& in, int32_t tp, int32_t end, int buf,
                                         __bf16* img, float (*zb)[4][2][2][H][16], const BwdConst& k, BwdState& st,
                                         int w, int lane) {
  const int g = lane >> 4, c = lane & 15, hc = c & 3;
  const float scale = 0.125f;
  // K rows (head w's columns) into the image: the A operand of the score (row reads) and the B operand
  // of dq (transposed reads)
  pair_stage(img, in, lane);
  asm volatile("" ::: "memory");
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    f4 T[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) T[t] = mma(k.W1f[t], in.X[x], zero4());
    const bf8 F0 = relu_pack8(T[0], T[1]), F1 = relu_pack8(T[2], T[3]);
    const bf8 K0 = row_frag(img, x, 0, g, c), K1 = row_frag(img, x, 1, g, c);
    f4 Zp = mma(F0, k.Uf[0], zero4());
    Zp = mma(F1, k.Uf[1], Zp);
    Zp = mma(K0, k.Qf[0], Zp);
    Zp = mma(K1, k.Qf[1], Zp);
    f4 Yp = mma(F0, k.Vf[0], zero4());
    Yp = mma(F1, k.Vf[1], Yp);
    Yp = mma(in.G[x][0], k.Of[0], Yp);
    Yp = mma(in.G[x][1], k.Of[1], Yp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Zp[r] += k.zadd;
      Yp[r] += k.yadd;
    }
    if (c < H) {
      *reinterpret_cast<f4*>(&zb[buf][w][0][x][c][4 * g]) = Zp;
      *reinterpret_cast<f4*>(&zb[buf][w][1][x][c][4 * g]) = Yp;
    }
  }
  bf8 FB[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    FB[t] = relu_pack8(mma(in.X[0], k.W1f[t], zero4()), mma(in.X[1], k.W1f[t], zero4()));
  __syncthreads();
  f4 dz[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    f4 z = *reinterpret_cast<const f4*>(&zb[buf][0][0][x][hc][4 * g]);
    f4 y = *reinterpret_cast<const f4*>(&zb[buf][0][1][x][hc][4 * g]);
#pragma unroll
    for (int v = 1; v < 4; ++v) {
      z += *reinterpret_cast<const f4*>(&zb[buf][v][0][x][hc][4 * g]);
      y += *reinterpret_cast<const f4*>(&zb[buf][v][1][x][hc][4 * g]);
    }
    const f4 mul = drop4<DROP>(p.drop, tp + 16 * x, lane, g, hc);
    f4 alp;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = tp + 16 * x + 4 * g + r < end;
      const float alpha = ok ? __expf(z[r] * scale - k.mst) * k.invden : 0.f;
      const float dal = y[r] * mul[r];
      dz[x][r] = alpha * (dal - k.pdl) * scale;
      alp[r] = alpha * mul[r];
      st.sg_l += dz[x][r];
    }
    if (w == 0 && c < H) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int32_t t = tp + 16 * x + 4 * g + r;
        if (t < end) {
          p.dz_e[(int64_t)t * H + c] = dz[x][r];
          p.alpha_e[(int64_t)t * H + c] = alp[r];
        }
      }
    }
  }
  bf8 AH, AL;
  split8(dz[0], dz[1], AH, AL);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    st.Sacc[t] = mma(AH, FB[t], st.Sacc[t]);
    st.Sacc[t] = mma(AL, FB[t], st.Sacc[t]);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf8 KB = tr_frag(img, t, lane);
    st.Qacc[t] = mma(AH, KB, st.Qacc[t]);
    st.Qacc[t] = mma(AL, KB, st.Qacc[t]);
  }
  asm volatile("" ::: "memory");
}

template <bool DROP>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void lgm_bwd_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  __shared__ __attribute__((aligned(16))) __bf16 imgs[4 * IMG];
  __shared__ __attribute__((aligned(16))) float zb[2][4][2][2][H][16];   // [buf][wave][Z|Y][tile][head][edge]
  __shared__ float cst[H];
  const int lane = threadIdx.x & 63, w = wave_id();
  const int g = lane >> 4, c = lane & 15, hc = c & 3;
  __bf16* img = imgs + w * IMG;
  const int64_t d = (int64_t)uni(sld(p.items, (int64_t)blockIdx.x));
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));

  BwdState st;
#pragma unroll
  for (int i = 0; i < 4; ++i) { st.Sacc[i] = zero4(); st.Qacc[i] = zero4(); }
  st.sg_l = 0.f;

  if (beg < end) {
    Seg sg;
    seg_load(p, sg, beg, end, lane);
    BwdConst k;
#pragma unroll
    for (int t = 0; t < 4; ++t) k.W1f[t] = w1_frag(p, 64 * w + 16 * t + c, g);
    const float* qrow = p.Q + d * p.ldq;
    const float* orow = p.dout + d * D;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      k.Uf[s] = u_frag(p.U, d, hc, w, s, g);
      k.Vf[s] = u_frag(p.Vd, d, hc, w, s, g);
      k.Qf[s] = q_frag(qrow, w, s, g, hc == w);
      k.Of[s] = q_frag(orow, w, s, g, hc == w);
    }
    // per head: c_h = <wbar_h, Q_h>, c2_h = <wbar_h, dout_h>, pdl_h = <dout_h, out_h> (softmax backward)
    float cw = 0.f, c2w = 0.f;
    const float ow = orow[64 * w + lane];
    if (p.wbar) {
      const float wb = p.wbar[64 * w + lane];
      cw = wave_sum(wb * qrow[64 * w + lane]);
      c2w = wave_sum(wb * ow);
    }
    const float pdw = wave_sum(ow * p.outp[d * D + 64 * w + lane]);
    if (lane == 0) cst[w] = pdw;
    k.zadd = hc == w ? cw : 0.f;
    k.yadd = hc == w ? c2w : 0.f;
    k.mst = p.mstat_in[d * H + hc];
    k.invden = 1.0f / p.den_in[d * H + hc];
    const int np = (end - beg + 31) / 32;
    PairIn A, B;
    pair_load(p, sg, 0, A, D, 0, w, lane);
    __syncthreads();
    k.pdl = cst[hc];
    for (int pr = 0; pr < np; pr += 2) {
      const int n1 = min(pr + 1, np - 1), n2 = min(pr + 2, np - 1);
      seg_advance(p, sg, n1, lane);
      pair_load(p, sg, n1, B, D, 0, w, lane);
      bwd_pair<DROP>(p, A, beg + 32 * pr, end, pr & 1, img, zb, k, st, w, lane);
      if (pr + 1 >= np) break;
      seg_advance(p, sg, n2, lane);
      pair_load(p, sg, n2, A, D, 0, w, lane);
      bwd_pair<DROP>(p, B, beg + 32 * (pr + 1), end, (pr + 1) & 1, img, zb, k, st, w, lane);
    }
  }
  const float sgt = rows_sum(st.sg_l);
#pragma unroll
  for (int t = 0; t < 4; ++t) p.Sz[(d * H + g) * D + 64 * w + 16 * t + c] = pick4(st.Sacc[t], g);
  {
    f4 vv = st.Qacc[0];
    vv = g == 1 ? st.Qacc[1] : vv;
    vv = g == 2 ? st.Qacc[2] : vv;
    vv = g == 3 ? st.Qacc[3] : vv;
    p.dq[d * p.lddq + 64 * w + 16 * g + c] = pick4(vv, w);
  }
  if (w == 0 && lane < H) p.sigz[d * H + lane] = sgt;
}

}  // namespace lgm

// Persistent grid: two workgroups per CU (the kernels' register budget: 2 waves per SIMD); a multiple
// of 8 so that every item of a workgroup lands on one XCD under round-robin placement.
static int lgm_persist_grid() {
  static int g = 0;
  if (g == 0) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t pr;
      if (hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0) cus = pr.multiProcessorCount;
    }
    g = (2 * cus + 7) / 8 * 8;
  }
  return g;
}
// ALIGNN_LGM_PERSIST=0: one workgroup per target instead (A/B measurements)
static bool lgm_persistent() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("ALIGNN_LGM_PERSIST");
    v = (e && *e) ? (std::atoi(e) != 0) : 1;
  }
  return v != 0;
}

// The kernels address rows with 24-bit products and 32-bit offsets (engine._angle_xf keeps larger
// batches on the streamed path)
static bool lgm_check(int64_t n, int64_t m, int64_t ldkv, int64_t ldx) {
  const int64_t lim = int64_t(1) << 24;
  return n < lim && m < lim && ldkv < lim && ldx < lim && n * ldkv < (int64_t(1) << 31) &&
         m * ldx < (int64_t(1) << 31);
}

// Entry points for lgconv.hip's C ABI (alignn_lg_fwd_x / alignn_lg_bwd_dst_x with bf16 K|V).
int lgm_fwd(int64_t n, int64_t m, const int32_t* off, const int32_t* src_at, const int32_t* items, int64_t n_items,
            const float* Q, int64_t ldq, const uint16_t* KV16, int64_t ldkv, const float* U, const float* wbar,
            const float* X, int64_t ldx, const float* W1, const float* b1, float* aggV, float* S, float* sumA,
            float* mstat, float* den, const DropParams& drop, hipStream_t s) {
  lgm::Params p{};
  p.n = n; p.m = m; p.off = off; p.src_at = src_at; p.items = items; p.n_items = n_items;
  p.Q = Q; p.ldq = ldq; p.KV16 = KV16; p.ldkv = ldkv; p.U = U; p.wbar = wbar;
  p.X = X; p.ldx = ldx; p.W1 = W1; p.b1 = b1;
  p.aggV = aggV; p.S = S; p.sumA = sumA; p.mstat = mstat; p.den = den;
  p.drop = drop;
  if (n_items <= 0) return ALIGNN_OK;
  if (!lgm_check(n, m, ldkv, ldx)) return ALIGNN_E_UNSUPPORTED;
  if (lgm_persistent()) {
    const unsigned grid = (unsigned)std::min<int64_t>(n_items, lgm_persist_grid());
    if (drop.active) launch(lgm::lgm_fwd_p_kernel<true>, dim3(grid), dim3(lgm::NT), 0, s, p);
    else launch(lgm::lgm_fwd_p_kernel<false>, dim3(grid), dim3(lgm::NT), 0, s, p);
  } else if (drop.active) {
    launch(lgm::lgm_fwd_kernel<true>, dim3((unsigned)n_items), dim3(lgm::NT), 0, s, p);
  } else {
    launch(lgm::lgm_fwd_kernel<false>, dim3((unsigned)n_items), dim3(lgm::NT), 0, s, p);
  }
  ALIGNN_LAUNCH_CHECK("lgm_fwd_kernel");
  return ALIGNN_OK;
}

int lgm_bwd(int64_t n, int64_t m, const int32_t* off, const int32_t* src_at, const int32_t* items, int64_t n_items,
            const float* Q, int64_t ldq, const uint16_t* KV16, int64_t ldkv, const float* U, const float* Vd,
            const float* wbar, const float* X, int64_t ldx, const float* W1, const float* b1, const float* dout,
            const float* outp, const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz,
            float* dz_e, float* alpha_e, const DropParams& drop, hipStream_t s) {
  lgm::Params p{};
  p.n = n; p.m = m; p.off = off; p.src_at = src_at; p.items = items; p.n_items = n_items;
  p.Q = Q; p.ldq = ldq; p.KV16 = KV16; p.ldkv = ldkv; p.U = U; p.Vd = Vd; p.wbar = wbar;
  p.X = X; p.ldx = ldx; p.W1 = W1; p.b1 = b1;
  p.dout = dout; p.outp = outp; p.mstat_in = mstat; p.den_in = den;
  p.dq = dq; p.lddq = lddq; p.Sz = Sz; p.sigz = sigz; p.dz_e = dz_e; p.alpha_e = alpha_e;
  p.drop = drop;
  if (n_items <= 0) return ALIGNN_OK;
  if (!lgm_check(n, m, ldkv, ldx)) return ALIGNN_E_UNSUPPORTED;
  if (drop.active) launch(lgm::lgm_bwd_kernel<true>, dim3((unsigned)n_items), dim3(lgm::NT), 0, s, p);
  else launch(lgm::lgm_bwd_kernel<false>, dim3((unsigned)n_items), dim3(lgm::NT), 0, s, p);
  ALIGNN_LAUNCH_CHECK("lgm_bwd_kernel");
  return ALIGNN_OK;
}

}  // namespace alignn
