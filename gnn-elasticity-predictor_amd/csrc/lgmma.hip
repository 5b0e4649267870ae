// lgmma.hip — the bf16-storage line-graph attention on the matrix cores (config C3).
//
// Same contract as lgconv.hip's bf16 kernels (PyG 2.7.0 TransformerConv message + utils.softmax +
// aggregate; callers train.py:315) for D = 256, H = 4 and bf16 K|V and edge-feature
// rows, but with the two GEMM-shaped parts of every 16-edge tile on the matrix cores instead of the
// VALU (which bounded lgconv.hip at ~70 vector instructions per edge):
//
//   scores   Z[e][h] = sum_k F[e][k] U[h][k] + sum_{k in head h} K_src(e)[k] q[k]
//            = [F | K] (16 x 512) . [U^T ; blockdiag(q)] (512 x 16, columns 4..15 zero):
//            16 x v_mfma_f32_16x16x32_bf16 per tile; the output lands as lane (g, r) = edges 4g..4g+3
//            of head r (r < 4), the layout the softmax and the next products read in place;
//   weighted sums  S[h][f] += sum_e a[e][h] F[e][f],  aggV[f] += sum_e a[e][h(f)] V_src(e)[f]:
//            per 4-edge group and 64-feature chunk one v_mfma_f32_4x4x4_16b_bf16 (16 blocks of
//            4 heads x 4 features x 4 edges, every block the same alpha); F and V reach the blocks
//            column-wise through ds_read_b64_tr_b16 from the tile's LDS image.
//
// Precision: the node vectors q and u = M_h^T q_h enter the matrix cores as bf16, as does alpha in
// the weighted sums (the reference's autocast holds q, the projected edge features and alpha in
// bf16 too, train.py:632-636); scores, softmax statistics and every accumulation are fp32.  Checked
// against the VALU kernels and the oracle within bf16 tolerances (tests/test_gpu_x_lgmma.py).
//
// Schedule: one single-wave workgroup per target segment (the lgconv.hip work list: descending
// in-degree, XCD-contiguous ranges), two waves per SIMD; the F, K, V rows of the next tile are in
// flight while one is computed; edge positions past the segment end are clamped to its last edge
// (valid rows, masked out of the softmax), so every tile issues the same loads.
#include "common.h"
#include "vec.h"

namespace alignn {
namespace lgm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

constexpr int D = 256, H = 4, TE = 16;   // C = D / H = 64 features per head
// LDS row pitch of a tile image, bf16 elements: 272 (544 B) puts rows 8 dwords apart modulo the 64
// banks, so a transposed read's eight rows per 32-lane half hit distinct banks
constexpr int LP = 272;
#ifndef LGM_WPE
#define LGM_WPE 2   // waves per SIMD the register budget is cut for (256 VGPR + AGPR per wave)
#endif

struct Params {
  int64_t n, m;
  const int32_t* off;
  const int32_t* src_at;
  const int32_t* items;
  int64_t n_items;
  const float* Q; int64_t ldq;        // fp32 Q rows (node vectors of the targets)
  const float* U;                     // [n, H, D]
  const float* wbar;                  // [D] or null
  const uint16_t* KV16; int64_t ldkv; // bf16 K | V rows
  const uint16_t* F16; int64_t ldf;   // bf16 edge-feature rows (target-sorted)
  float* aggV; float* S; float* sumA; float* mstat; float* den;
  // backward (target side)
  const float* Vd;                    // [n, H, D]
  const float* dout; const float* outp; const float* mstat_in; const float* den_in;
  float* dq; int64_t lddq; float* Sz; float* sigz; float* dz_e; float* alpha_e;
  DropParams drop;
};

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
}
__device__ __forceinline__ bf16x8 as_bf8(u4v u) { return __builtin_bit_cast(bf16x8, u); }

// One tile's rows in the 16x16x32 operand layout: lane (g, r) holds bf16 k = 32c + 8g .. +8 of edge
// row r, c = 0..7 (16-byte loads: per instruction 16 rows x 64 contiguous bytes)
struct Tile {
  u4v f[8], k[8], v[8];
};

__device__ __forceinline__ void load_tile(Tile& T, const Params& p, int32_t t0, int32_t last, int r, int g) {
  const int32_t t = min(t0 + r, last);
  // the tile's 16 source ids as scalar loads (lgkmcnt): a vector index load would make the K/V loads
  // wait on vmcnt, which counts every load issued before it — the tiles already in flight
  int32_t sid[TE];
#pragma unroll
  for (int j = 0; j < TE; ++j) sid[j] = uni(sld(p.src_at, (int64_t)min(t0 + j, last)));
  int32_t sv = sid[0];
#pragma unroll
  for (int j = 1; j < TE; ++j) sv = (r == j) ? sid[j] : sv;
  const int64_t s = (int64_t)sv;
  const uint16_t* fr = p.F16 + (int64_t)t * p.ldf + 8 * g;
  const uint16_t* kr = p.KV16 + s * p.ldkv + 8 * g;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    T.f[c] = *reinterpret_cast<const u4v*>(fr + 32 * c);
    T.k[c] = *reinterpret_cast<const u4v*>(kr + 32 * c);
    T.v[c] = *reinterpret_cast<const u4v*>(kr + D + 32 * c);
  }
  asm volatile("" ::: "memory");  // a prefetch: issued here, not sunk to its first use
}

// Transposed read (ds_read_b64_tr_b16) of rows 4G..4G+3, columns c0 + lane of a tile image: lane L
// receives column c0 + L of the four rows in its four elements.  Lane 4q + p of each 16-lane group
// supplies the address of row 4G + q, columns c0 + 16 (L >> 4) + 4p .. +3.
__device__ __forceinline__ s4v tr_read(const uint16_t* img, int G, int c0, int lane) {
  const int li = lane & 15;
  const uint16_t* a = img + (4 * G + (li >> 2)) * LP + c0 + 16 * (lane >> 4) + 4 * (li & 3);
  typedef short s4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(s4v, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(reinterpret_cast<uintptr_t>(a))));
}

template <bool DROP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LGM_WPE, LGM_WPE))) void lgm_fwd_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  __shared__ __attribute__((aligned(16))) uint16_t Fs[TE * LP];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[TE * LP];
  const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
  const float scale = 0.125f;   // 1 / sqrt(C)
  const int64_t d = (int64_t)uni(sld(p.items, (int64_t)blockIdx.x));
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));
  const bool hl = r < H;   // lanes holding a head's scores (column r of the score tile)

  // softmax state of head r (lanes r < 4, the same in every lane group g): running max, this lane's
  // partial sums of exp (its own 4 edges of every tile) and of exp x dropout multiplier
  float m = hl ? -INFINITY : 0.f, s_p = 0.f, sa_p = 0.f;
  // weighted sums, 4x4x4 block layout: accS[c4][h] = S_h[64 c4 + lane], accV[c4][h] likewise
  f4v accS[4], accV[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    accS[c] = f4v{0.f, 0.f, 0.f, 0.f};
    accV[c] = f4v{0.f, 0.f, 0.f, 0.f};
  }

  if (beg < end) {
    // B operands of the score product (bf16): Bu[c] = U[h = r][32c + 8g ..], Bq[c] = q[32c + 8g ..]
    // in column r = head of those features (c >> 1), zero elsewhere
    bf16x8 Bu[8], Bq[8];
    const float* Qd = p.Q + d * p.ldq;
    const float* Ud = p.U + (d * H + (r & 3)) * D;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int k0 = 32 * c + 8 * g;
      float u[8], q[8];
      vload<8>(Ud + k0, u);
      vload<8>(Qd + k0, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Bu[c][j] = (__bf16)(hl ? u[j] : 0.f);
        Bq[c][j] = (__bf16)(r == (c >> 1) ? q[j] : 0.f);
      }
    }
    // score offset of head r: wbar_h . q_h (the projected edge features' bias), fp32
    float cb = 0.f;
    if (p.wbar) {
      float wb[4], q4[4];
      vload<4>(p.wbar + 4 * lane, wb);
      vload<4>(Qd + 4 * lane, q4);
      const float part = row_sum16(vdot(wb, q4));          // lanes of group g: head g's sum
      cb = __shfl(part, 16 * (r & 3), 64);
    }
    const int32_t last = end - 1;
    // one tile: image for the transposed reads, scores, (the register set is free: `refill` issues the
    // loads of a later tile into it), online softmax, weighted sums
    auto tile = [&](Tile& T, int32_t t0, int32_t t_next) {
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the previous tile's transposed reads are done
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        *reinterpret_cast<u4v*>(Fs + r * LP + 32 * c + 8 * g) = T.f[c];
        *reinterpret_cast<u4v*>(Vs + r * LP + 32 * c + 8 * g) = T.v[c];
      }
      // scores of the 16 edges x 4 heads
      f4v z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        z4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(T.f[c]), Bu[c], z4, 0, 0, 0);
        z4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(T.k[c]), Bq[c], z4, 0, 0, 0);
      }
      load_tile(T, p, t_next, last, r, g);
      // online softmax (edges 4g + i of head r)
      float z[4], tmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = hl && (t0 + 4 * g + i < end);
        z[i] = ok ? (z4[i] + cb) * scale : -INFINITY;
        tmax = fmaxf(tmax, z[i]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax);
      if (__builtin_amdgcn_ballot_w64(mn != m)) {   // wave-uniform: rescale when a running max moved
        const float corr = __expf(m - mn);
        m = mn;
        s_p *= corr;
        sa_p *= corr;
        f4v cr;
#pragma unroll
        for (int h = 0; h < H; ++h) cr[h] = readlane_f(corr, h);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          accS[c] *= cr;
          accV[c] *= cr;
        }
      }
      float ed[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float ex = __expf(z[i] - m);   // 0 for masked entries
        s_p += ex;
        float mul = 1.0f;
        if constexpr (DROP) {
          if (hl) mul = dropout_mul(p.drop.seed, (uint64_t)(t0 + 4 * g + i) * H + r, p.drop.thresh, p.drop.inv_keep);
        }
        ed[i] = ex * mul;
        sa_p += ed[i];
      }
      // alpha of edge group G for the 4x4x4 blocks: lane (b, i) takes the row of head i from lane 16G + i
      const uint32_t e01 = pack_bf16(ed[0], ed[1]), e23 = pack_bf16(ed[2], ed[3]);
      s4v A[4];
#pragma unroll
      for (int G = 0; G < 4; ++G) {
        const int src = 16 * G + (lane & 3);
        const u2v a2 = {(uint32_t)__shfl((int)e01, src, 64), (uint32_t)__shfl((int)e23, src, 64)};
        A[G] = __builtin_bit_cast(s4v, a2);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the tile image is written (one wave)
      // transposed reads in batches of eight (one edge group: 4 chunks of F and of V), the next
      // group's batch issued before this group's products, so no product waits on a single read
      s4v rb[2][8];
      auto reads = [&](s4v (&b)[8], int G) {
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          b[c4] = tr_read(Fs, G, 64 * c4, lane);
          b[4 + c4] = tr_read(Vs, G, 64 * c4, lane);
        }
      };
      reads(rb[0], 0);
#pragma unroll
      for (int G = 0; G < 4; ++G) {
        if (G + 1 < 4) reads(rb[(G + 1) & 1], G + 1);
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          accS[c4] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(A[G], rb[G & 1][c4], accS[c4], 0, 0, 0);
          accV[c4] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(A[G], rb[G & 1][4 + c4], accV[c4], 0, 0, 0);
        }
      }
    };
    // one register set, refilled with the next tile's rows as soon as this tile's scores have consumed
    // it (the loads land during the softmax and the weighted sums; a second wave per SIMD covers the
    // rest: the kernel is held to 2 waves per SIMD, amdgpu_waves_per_eu).  Loads are unconditional,
    // clamped to the last edge: a conditional load leaves the compiler's wait counters unable to tell
    // which loads are outstanding, and it drains them all.
    Tile T;
    load_tile(T, p, beg, last, r, g);
    for (int32_t t0 = beg; t0 < end; t0 += TE) tile(T, t0, t0 + TE);
  }
  // per-head totals over the four lane groups
  float s = s_p + __shfl_xor(s_p, 16, 64);
  s += __shfl_xor(s, 32, 64);
  float sa = sa_p + __shfl_xor(sa_p, 16, 64);
  sa += __shfl_xor(sa, 32, 64);
  const float dn = s + 1e-16f;
  const float inv = 1.0f / dn;
  f4v iv;
#pragma unroll
  for (int h = 0; h < H; ++h) iv[h] = readlane_f(inv, h);
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) {
#pragma unroll
    for (int h = 0; h < H; ++h) p.S[(d * H + h) * D + 64 * c4 + lane] = accS[c4][h] * iv[h];
    p.aggV[d * D + 64 * c4 + lane] = accV[c4][c4] * iv[c4];
  }
  if (lane < H) {
    p.sumA[d * H + lane] = sa * inv;
    p.mstat[d * H + lane] = m;
    p.den[d * H + lane] = dn;
  }
}

// =============================================================================================
// Backward, target side (lgconv.hip lg3_bwd_dst's contract): per edge dz = alpha (dalpha' - c3) / sqrt(C)
// and alpha' = alpha x dropout; per target dq = sum dz k, Sz = sum dz f, sigz = sum dz.  Scores as in
// the forward plus P = [F | V] . [Vd^T ; blockdiag(dout)] (dalpha' numerators), the sums of dz as
// 4x4x4 products against the F and K tile images.
// =============================================================================================
#ifndef LGM_WPE_BWD
#define LGM_WPE_BWD 1
#endif
template <bool DROP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LGM_WPE_BWD, LGM_WPE_BWD)))
void lgm_bwd_dst_kernel(Params p) {
  if constexpr (DROP) resolve_drop(p.drop);
  __shared__ __attribute__((aligned(16))) uint16_t Fs[TE * LP];
  __shared__ __attribute__((aligned(16))) uint16_t Ks[TE * LP];
  const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
  const float scale = 0.125f;   // 1 / sqrt(C)
  const int64_t d = (int64_t)uni(sld(p.items, (int64_t)blockIdx.x));
  const int32_t beg = uni(sld(p.off, d)), end = uni(sld(p.off, d + 1));
  const bool hl = r < H;

  float sgz_p = 0.f;
  f4v accSz[4], accDq[4];   // 4x4x4 block layout: acc[c4][h] = value of head h at feature 64 c4 + lane
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    accSz[c] = f4v{0.f, 0.f, 0.f, 0.f};
    accDq[c] = f4v{0.f, 0.f, 0.f, 0.f};
  }

  if (beg < end) {
    bf16x8 Bu[8], Bq[8], Bvd[8], Bgo[8];
    const float* Qd = p.Q + d * p.ldq;
    const float* God = p.dout + d * D;
    const float* Ud = p.U + (d * H + (r & 3)) * D;
    const float* Vdd = p.Vd + (d * H + (r & 3)) * D;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int k0 = 32 * c + 8 * g;
      float u[8], q[8], vd[8], go[8];
      vload<8>(Ud + k0, u);
      vload<8>(Qd + k0, q);
      vload<8>(Vdd + k0, vd);
      vload<8>(God + k0, go);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Bu[c][j] = (__bf16)(hl ? u[j] : 0.f);
        Bq[c][j] = (__bf16)(r == (c >> 1) ? q[j] : 0.f);
        Bvd[c][j] = (__bf16)(hl ? vd[j] : 0.f);
        Bgo[c][j] = (__bf16)(r == (c >> 1) ? go[j] : 0.f);
      }
    }
    // per-head offsets (fp32): cb = wbar.q, c2 = wbar.dout, c3 = dout.outp (row sums of head g's 16 lanes)
    float cb = 0.f, c2 = 0.f, c3;
    {
      float q4[4], go4[4], op4[4];
      vload<4>(Qd + 4 * lane, q4);
      vload<4>(God + 4 * lane, go4);
      vload<4>(p.outp + d * D + 4 * lane, op4);
      if (p.wbar) {
        float wb[4];
        vload<4>(p.wbar + 4 * lane, wb);
        cb = __shfl(row_sum16(vdot(wb, q4)), 16 * (r & 3), 64);
        c2 = __shfl(row_sum16(vdot(wb, go4)), 16 * (r & 3), 64);
      }
      c3 = __shfl(row_sum16(vdot(go4, op4)), 16 * (r & 3), 64);
    }
    const float mst = hl ? p.mstat_in[d * H + r] : 0.f;
    const float inv_den = hl ? 1.0f / p.den_in[d * H + r] : 0.f;
    const int32_t last = end - 1;
    auto tile = [&](Tile& T, int32_t t0, int32_t t_next) {
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the previous tile's transposed reads are done
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        *reinterpret_cast<u4v*>(Fs + r * LP + 32 * c + 8 * g) = T.f[c];
        *reinterpret_cast<u4v*>(Ks + r * LP + 32 * c + 8 * g) = T.k[c];
      }
      f4v z4 = {0.f, 0.f, 0.f, 0.f}, p4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        z4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(T.f[c]), Bu[c], z4, 0, 0, 0);
        p4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(T.f[c]), Bvd[c], p4, 0, 0, 0);
        z4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(T.k[c]), Bq[c], z4, 0, 0, 0);
        p4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(T.v[c]), Bgo[c], p4, 0, 0, 0);
      }
      load_tile(T, p, t_next, last, r, g);
      float dz[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t e = t0 + 4 * g + i;
        const bool ok = hl && e < end;
        const float z = (z4[i] + cb) * scale;
        const float alpha = __expf(z - mst) * inv_den;
        float mul = 1.0f;
        if constexpr (DROP) {
          if (hl) mul = dropout_mul(p.drop.seed, (uint64_t)e * H + r, p.drop.thresh, p.drop.inv_keep);
        }
        const float al = alpha * mul;
        const float dal = (p4[i] + c2) * mul;
        dz[i] = ok ? alpha * (dal - c3) * scale : 0.f;
        if (ok) {
          p.dz_e[(int64_t)e * H + r] = dz[i];
          p.alpha_e[(int64_t)e * H + r] = al;
        }
        sgz_p += dz[i];
      }
      const uint32_t e01 = pack_bf16(dz[0], dz[1]), e23 = pack_bf16(dz[2], dz[3]);
      s4v A[4];
#pragma unroll
      for (int G = 0; G < 4; ++G) {
        const int src = 16 * G + (lane & 3);
        const u2v a2 = {(uint32_t)__shfl((int)e01, src, 64), (uint32_t)__shfl((int)e23, src, 64)};
        A[G] = __builtin_bit_cast(s4v, a2);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the tile images are written (one wave)
      s4v rb[2][8];
      auto reads = [&](s4v (&b)[8], int G) {
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          b[c4] = tr_read(Fs, G, 64 * c4, lane);
          b[4 + c4] = tr_read(Ks, G, 64 * c4, lane);
        }
      };
      reads(rb[0], 0);
#pragma unroll
      for (int G = 0; G < 4; ++G) {
        if (G + 1 < 4) reads(rb[(G + 1) & 1], G + 1);
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          accSz[c4] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(A[G], rb[G & 1][c4], accSz[c4], 0, 0, 0);
          accDq[c4] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(A[G], rb[G & 1][4 + c4], accDq[c4], 0, 0, 0);
        }
      }
    };
    Tile T;
    load_tile(T, p, beg, last, r, g);
    for (int32_t t0 = beg; t0 < end; t0 += TE) tile(T, t0, t0 + TE);
  }
  float sg = sgz_p + __shfl_xor(sgz_p, 16, 64);
  sg += __shfl_xor(sg, 32, 64);
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) {
#pragma unroll
    for (int h = 0; h < H; ++h) p.Sz[(d * H + h) * D + 64 * c4 + lane] = accSz[c4][h];
    p.dq[d * p.lddq + 64 * c4 + lane] = accDq[c4][c4];
  }
  if (lane < H) p.sigz[d * H + lane] = sg;
}

}  // namespace lgm

int lgm_bwd_dst(const lgm::Params& p, hipStream_t s) {
  if (p.n_items <= 0) return ALIGNN_OK;
  if (p.drop.active) launch(lgm::lgm_bwd_dst_kernel<true>, dim3((unsigned)p.n_items), dim3(64), 0, s, p);
  else launch(lgm::lgm_bwd_dst_kernel<false>, dim3((unsigned)p.n_items), dim3(64), 0, s, p);
  ALIGNN_LAUNCH_CHECK("lgm_bwd_dst_kernel");
  return ALIGNN_OK;
}

int lgm_fwd(const lgm::Params& p, hipStream_t s) {
  if (p.n_items <= 0) return ALIGNN_OK;
  if (p.drop.active) launch(lgm::lgm_fwd_kernel<true>, dim3((unsigned)p.n_items), dim3(64), 0, s, p);
  else launch(lgm::lgm_fwd_kernel<false>, dim3((unsigned)p.n_items), dim3(64), 0, s, p);
  ALIGNN_LAUNCH_CHECK("lgm_fwd_kernel");
  return ALIGNN_OK;
}

}  // namespace alignn

using namespace alignn;

static int lgm_check(int64_t n, int32_t D, int32_t H, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                     const uint16_t* KV16, int64_t ldkv, const float* U, const uint16_t* F16, int64_t ldf) {
  if (D != lgm::D || H != lgm::H) {
    set_error("lg mfma: needs hidden 256 and 4 heads (got %d, %d)", (int)D, (int)H);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (!sched || !(sched->flags & ALIGNN_SCHED_WAVE_ITEMS) || sched->n_heavy != 0 || (n > 0 && !sched->light)) {
    set_error("lg mfma: needs an ALIGNN_SCHED_WAVE_ITEMS schedule listing every target (no heavy list)");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (n > 0 && (!Q || !KV16 || !F16 || !U || ldq < 3 * D || ldkv < 2 * D || ldf < D || ldkv % 8 || ldf % 8 ||
                (reinterpret_cast<uintptr_t>(KV16) & 15) || (reinterpret_cast<uintptr_t>(F16) & 15) || ldq % 4 ||
                (reinterpret_cast<uintptr_t>(Q) & 15) || (reinterpret_cast<uintptr_t>(U) & 15))) {
    set_error("lg mfma: Q (ldq >= 3D), K|V bf16 rows (ldkv >= 2D) and F bf16 rows (ldf >= D), 16-byte aligned rows");
    return ALIGNN_E_BAD_SHAPE;
  }
  return ALIGNN_OK;
}

// Matrix-core form of alignn_lg_bwd_dst_bf16 (D = 256, H = 4; same arguments and outputs).
extern "C" int alignn_lg_bwd_dst_mfma(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                      const int32_t* src_at, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                                      const uint16_t* KV16, int64_t ldkv, const float* U, const float* Vd,
                                      const float* wbar, const uint16_t* F16, int64_t ldf, const float* dout,
                                      const float* outp, const float* mstat, const float* den, float* dq,
                                      int64_t lddq, float* Sz, float* sigz, float* dz_e, float* alpha_e, float drop_p,
                                      uint64_t seed, void* stream) {
  int rc = lgm_check(n, D, H, sched, Q, ldq, KV16, ldkv, U, F16, ldf);
  if (rc || n == 0) return rc;
  if (!Vd || !dout || !outp || !mstat || !den || !dq || !Sz || !sigz || !dz_e || !alpha_e ||
      (reinterpret_cast<uintptr_t>(Vd) & 15) || (reinterpret_cast<uintptr_t>(dout) & 15) ||
      (reinterpret_cast<uintptr_t>(outp) & 15)) {
    set_error("lg mfma bwd: Vd, dout, outp (16-byte aligned rows) and every output are required");
    return ALIGNN_E_BAD_SHAPE;
  }
  lgm::Params p{};
  p.n = n; p.m = m; p.off = off_dst; p.src_at = src_at; p.items = sched->light; p.n_items = sched->n_light;
  p.Q = Q; p.ldq = ldq; p.U = U; p.wbar = wbar; p.KV16 = KV16; p.ldkv = ldkv; p.F16 = F16; p.ldf = ldf;
  p.Vd = Vd; p.dout = dout; p.outp = outp; p.mstat_in = mstat; p.den_in = den;
  p.dq = dq; p.lddq = lddq; p.Sz = Sz; p.sigz = sigz; p.dz_e = dz_e; p.alpha_e = alpha_e;
  p.drop = make_drop(drop_p, seed);
  return lgm_bwd_dst(p, reinterpret_cast<hipStream_t>(stream));
}

// Matrix-core form of alignn_lg_fwd_bf16 (D = 256, H = 4; same arguments and outputs).
extern "C" int alignn_lg_fwd_mfma(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                                  const int32_t* src_at, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                                  const uint16_t* KV16, int64_t ldkv, const float* U, const float* wbar,
                                  const uint16_t* F16, int64_t ldf, float* aggV, float* S, float* sumA, float* mstat,
                                  float* den, float drop_p, uint64_t seed, void* stream) {
  int rc = lgm_check(n, D, H, sched, Q, ldq, KV16, ldkv, U, F16, ldf);
  if (rc) return rc;
  if (n == 0) return ALIGNN_OK;
  lgm::Params p{};
  p.n = n; p.m = m; p.off = off_dst; p.src_at = src_at; p.items = sched->light; p.n_items = sched->n_light;
  p.Q = Q; p.ldq = ldq; p.U = U; p.wbar = wbar; p.KV16 = KV16; p.ldkv = ldkv; p.F16 = F16; p.ldf = ldf;
  p.aggV = aggV; p.S = S; p.sumA = sumA; p.mstat = mstat; p.den = den;
  p.drop = make_drop(drop_p, seed);
  return lgm_fwd(p, reinterpret_cast<hipStream_t>(stream));
}
