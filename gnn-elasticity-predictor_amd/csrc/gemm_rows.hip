// gemm_rows.hip — row-streaming bf16 GEMM for the bond-level products of config C3 (every one of the
// batch's ~184k bonds times a 256-wide weight): C[M, N] = epi(alpha A W + beta C + bias), K <= 256,
// N a multiple of 256, M large.  Replaces the W-in-LDS streaming kernel (gemm.hip, bst) there.
//
// These products are HBM-bound (a 184,320 x 256 x 256 product is 24 GFLOP — 10 us of bf16 matrix
// cores — against 189-567 MB of A / C traffic, 24-71 us at 8 TB/s).  The streaming kernel it
// replaces keeps a 256-column W slice in 150 KB of LDS, so one 4-wave workgroup per CU: a single
// wave per SIMD, which exposes every LDS and global round trip (86-149 us for the product above).
// Here each of a workgroup's 8 waves holds ITS 32 columns of W in VGPRs — KT/16 MFMA B operands
// (bf16x8: 64 VGPRs at K = 256), loaded and rounded once — so the LDS holds only the streamed A
// bands (double-buffered bf16 [32][KT + 8]) and the waves' 32 x 36 epilogue tiles (72 KB), and the
// CU runs 8 waves (2 per SIMD) instead of 4.
//
// Work: a persistent grid of G workgroups (one per CU, a multiple of the batch x N / 256 work items:
// batch entry, 256-column slice); workgroup g serves item g % items and 32-row bands q, q + Q, ...
// (q = g / items, Q = G / items).  Two register sets hold the next two bands' A rows (16-byte loads, two bands in flight
// per CU); per band the set loaded two bands earlier is rounded to bf16 (RNE) into the other LDS
// image, and each wave runs KT/16 v_mfma_f32_32x32x16_bf16 (the A operand — band rows l32, k = 16 t
// + 8 h + j — read one slice ahead) and writes its 32 x 32 block through its LDS tile as 16-byte row
// segments: alpha acc, fma(beta, C, .), + bias (from an LDS copy), ReLU, mask — the order and k
// grouping of every GEMM path here (gemm_tile.h), so results are bitwise those of the tiled bf16
// kernels.  K < KT is zero-padded (the edge MLP's K = 36 runs as KT = 64).  Loads and stores are
// unconditional: rows past M are clamped for loads and dropped by the store descriptor.
#include "gemm_tile.h"

namespace alignn {
namespace rsk {

typedef float gf4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int NT = 512;      // threads: 8 waves x 32 columns
constexpr int NB = 256;      // columns per slice
constexpr int ROWS = 32;     // rows per band
constexpr int EPI_LD = 36;   // epilogue tile row stride (floats)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n, 0x00020000);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)bf_rne(a) | ((uint32_t)bf_rne(b) << 16);
}

// One band of A in registers: 16-byte chunks (four fp32 or eight bf16 values), PER per thread.
template <int KT, bool ABF>
struct Band {
  static constexpr int CH = ABF ? KT / 8 : KT / 4;   // chunks per row
  static constexpr int TOT = ROWS * CH;
  static constexpr int PER = (TOT + NT - 1) / NT;
  gf4 r[PER];

  __device__ __forceinline__ void load(const GemmParams& p, int64_t band) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = min((int)threadIdx.x + NT * i, TOT - 1);   // (KT = 64 bf16: half the threads repeat)
      const int64_t row = min(band * ROWS + idx / CH, p.M - 1);
      const int k = (idx % CH) * (ABF ? 8 : 4);
      const int kc = k < p.K ? k : 0;   // zero padding past K: a valid address, the value dropped at store
      r[i] = *reinterpret_cast<const gf4*>(eoff(p.A, row * p.sam + kc, ABF));
    }
    asm volatile("" ::: "memory");   // issued here, not sunk to the LDS store
  }
  // rounded to bf16 into the [ROWS][KT + 8] image
  __device__ __forceinline__ void store(__bf16* __restrict__ img, int K) const {
    constexpr int KP = KT + 8;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = (int)threadIdx.x + NT * i;
      if (TOT % NT != 0 && idx >= TOT) break;
      const int rr = idx / CH, k = (idx % CH) * (ABF ? 8 : 4);
      const bool live = k < K;
      if constexpr (ABF) {
        u32x4 u = __builtin_bit_cast(u32x4, r[i]);
        if (!live) u = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(img + rr * KP + k) = u;
      } else {
        const gf4 v = live ? r[i] : gf4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<u32x2*>(img + rr * KP + k) = u32x2{pack2(v.x, v.y), pack2(v.z, v.w)};
      }
    }
  }
};

// BKC: W given k-contiguous (W^T, sbk == 1, 16-byte aligned rows, K % 8 == 0): two 16-byte loads per
// operand; else element loads (W row-major: the wave's lanes read consecutive columns at each k).
template <int KT, bool ABF, bool CBF, bool BETA, bool MASK, bool BKC>
__global__ __launch_bounds__(NT, 1) void gemm_rows_kernel(GemmParams p, int nitems, int nsl, int64_t nbands) {
  static_assert(!(CBF && BETA), "bf16 C is write-only");
  constexpr int KP = KT + 8, T = KT / 16;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][ROWS * KP];
  __shared__ __attribute__((aligned(16))) float Lepi[NT / 64][ROWS * EPI_LD];
  __shared__ __attribute__((aligned(16))) float Lbias[NB];
  // work item (batch entry b, column slice z) = g % nitems; batched products (the per-head U / Vd
  // products, batch = heads) offset the operands per entry
  const int g = blockIdx.x;
  const int item = g % nitems, q = g / nitems, Q = gridDim.x / nitems;
  const int z = item % nsl, b = item / nsl;
  const int64_t n0 = (int64_t)z * NB;
  if (b > 0) {
    p.A = eoff(p.A, b * p.sab, ABF);
    p.B += b * p.sbb;
    p.C = const_cast<float*>(eoff(p.C, b * p.scb, CBF));
    if (p.bias) p.bias += b * p.sbias_b;
  }
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int l32 = lane & 31, h = lane >> 5;
  const bool has_bias = p.bias != nullptr;
  for (int i = threadIdx.x; i < NB; i += NT) Lbias[i] = has_bias ? p.bias[n0 + i] : 0.f;

  // this wave's W columns as MFMA B operands: column n0 + 32 wave + l32, k = 16 t + 8 h + e; loads
  // unconditional (indices clamped, values past K zeroed by select)
  const int64_t colw = n0 + 32 * wave;   // this wave's first column
  bf16x8 bw[T];
  {
    const int K = (int)p.K;
    const float* Bc = p.B + (colw + l32) * p.sbn;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int k0 = 16 * t + 8 * h;
      if constexpr (BKC) {
        const int kc = min(k0, K - 8);
        const gf4 x = *reinterpret_cast<const gf4*>(Bc + kc), y = *reinterpret_cast<const gf4*>(Bc + kc + 4);
        const bool live = k0 < K;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bw[t][e] = (__bf16)(live ? x[e] : 0.f);
          bw[t][4 + e] = (__bf16)(live ? y[e] : 0.f);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = Bc[(int64_t)min(k0 + e, K - 1) * p.sbk];
          bw[t][e] = (__bf16)(k0 + e < K ? v : 0.f);
        }
      }
      if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // <= four slices' loads in flight
    }
  }

  float* Cw = const_cast<float*>(eoff(p.C, colw, CBF));
  const int64_t cbytes = (p.M * p.scm - colw) * (CBF ? 2 : 4);
  const __amdgpu_buffer_rsrc_t cst = rsrc(Cw, cbytes);
  const __amdgpu_buffer_rsrc_t cld = rsrc(Cw, BETA ? cbytes : 0);
  const __amdgpu_buffer_rsrc_t cmk = rsrc(MASK ? p.mask + colw : Cw, MASK ? (p.M * p.smk_m - colw) * 4 : 0);
  float* Ls = Lepi[wave];
  const float* Lb = Lbias + 32 * wave;

  int64_t band = q;
  if (band >= nbands) return;   // workgroup-uniform, before any barrier
  Band<KT, ABF> r0, r1;
  r0.load(p, band);
  r1.load(p, min(band + Q, nbands - 1));
  r0.store(As[0], (int)p.K);
  r0.load(p, min(band + 2 * Q, nbands - 1));
  __syncthreads();

  // one band: MFMAs on image `cur`; the register set `nx` (band + Q, loaded two bands ago) into the
  // other image and reloaded with band + 3Q; the epilogue.  false: this was the workgroup's last band.
  auto step = [&](Band<KT, ABF>& nx, const __bf16* __restrict__ cur, __bf16* __restrict__ other) -> bool {
    const int64_t row0 = band * ROWS;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const __bf16* Al = cur + l32 * KP + 8 * h;
    bf16x8 a[2];
    a[0] = *reinterpret_cast<const bf16x8*>(Al);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (t + 1 < T) a[(t + 1) & 1] = *reinterpret_cast<const bf16x8*>(Al + 16 * (t + 1));
      __builtin_amdgcn_sched_barrier(0);   // the next slice's read ahead of this MFMA
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t & 1], bw[t], acc, 0, 0, 0);
    }
    // epilogue map: each pass writes whole row segments of the wave's 32 columns — fp32 C: 8 rows x
    // 8 lanes x 16 bytes (one 128-byte line per row), four passes; bf16 C: 16 rows x 4 lanes x 8
    // values, two passes.  The C / mask values (fp32 C only) are issued before the next band's loads
    // (a load issued after them would wait for them too: loads complete in order).
    constexpr int PASS = CBF ? 2 : 4, RPP = ROWS / PASS, LPR = 64 / RPP;   // rows per pass, lanes per row
    const int er = lane / LPR, ec = (lane % LPR) * (CBF ? 8 : 4);
    gf4 cv[BETA ? PASS : 1], mk[MASK ? PASS : 1];
#pragma unroll
    for (int ps = 0; ps < PASS; ++ps) {
      const int64_t row = row0 + RPP * ps + er;
      if constexpr (BETA)
        cv[ps] = __builtin_bit_cast(gf4, __builtin_amdgcn_raw_buffer_load_b128(cld, (int)((row * p.scm + ec) * 4), 0, 0));
      if constexpr (MASK)
        mk[ps] = __builtin_bit_cast(gf4, __builtin_amdgcn_raw_buffer_load_b128(cmk, (int)((row * p.smk_m + ec) * 4), 0, 0));
    }
    const int64_t b1 = band + Q;
    if (b1 < nbands) {   // workgroup-uniform
      nx.store(other, (int)p.K);
      nx.load(p, min(b1 + 2 * Q, nbands - 1));
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) Ls[((r & 3) + 8 * (r >> 2) + 4 * h) * EPI_LD + l32] = __fmul_rn(p.alpha, acc[r]);
    const gf4 zero = {0.f, 0.f, 0.f, 0.f};
    auto finish = [&](gf4 v, int c, int ps) -> gf4 {   // beta, bias, ReLU, mask of four values at column c
      if constexpr (BETA)
        v = gf4{fmaf(p.beta, cv[ps].x, v.x), fmaf(p.beta, cv[ps].y, v.y), fmaf(p.beta, cv[ps].z, v.z),
                fmaf(p.beta, cv[ps].w, v.w)};
      if (has_bias) {
        const gf4 bb = *reinterpret_cast<const gf4*>(Lb + c);
        v = gf4{__fadd_rn(v.x, bb.x), __fadd_rn(v.y, bb.y), __fadd_rn(v.z, bb.z), __fadd_rn(v.w, bb.w)};
      }
      v = p.relu ? __builtin_elementwise_max(v, zero) : v;
      if constexpr (MASK) {
        v.x = mk[ps].x > 0.f ? v.x : 0.f; v.y = mk[ps].y > 0.f ? v.y : 0.f;
        v.z = mk[ps].z > 0.f ? v.z : 0.f; v.w = mk[ps].w > 0.f ? v.w : 0.f;
      }
      return v;
    };
#pragma unroll
    for (int ps = 0; ps < PASS; ++ps) {
      const int rr = RPP * ps + er;
      const int off = (int)(((row0 + rr) * p.scm + ec) * (CBF ? 2 : 4));
      const gf4 v0 = finish(*reinterpret_cast<const gf4*>(Ls + rr * EPI_LD + ec), ec, ps);
      if constexpr (CBF) {
        const gf4 v1 = finish(*reinterpret_cast<const gf4*>(Ls + rr * EPI_LD + ec + 4), ec + 4, ps);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{pack2(v0.x, v0.y), pack2(v0.z, v0.w), pack2(v1.x, v1.y),
                                                     pack2(v1.z, v1.w)}, cst, off, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v0), cst, off, 0, 0);
      }
    }
    if (b1 >= nbands) return false;
    __syncthreads();   // the other image is complete; this one is free for the band after next
    band = b1;
    return true;
  };
  while (step(r1, As[0], As[1]) && step(r0, As[1], As[0])) {
  }
}

template <int KT, bool ABF, bool CBF, bool BKC>
static void launch_kt(const GemmParams& p, dim3 grid, int nslices, int nsl, int64_t nbands, hipStream_t s) {
  const bool beta = p.beta != 0.f, mask = p.mask != nullptr;
  if constexpr (CBF) {
    launch(gemm_rows_kernel<KT, ABF, true, false, false, BKC>, grid, dim3(NT), 0, s, p, nslices, nsl, nbands);
  } else {
    if (beta && mask) launch(gemm_rows_kernel<KT, ABF, false, true, true, BKC>, grid, dim3(NT), 0, s, p, nslices, nsl, nbands);
    else if (beta) launch(gemm_rows_kernel<KT, ABF, false, true, false, BKC>, grid, dim3(NT), 0, s, p, nslices, nsl, nbands);
    else if (mask) launch(gemm_rows_kernel<KT, ABF, false, false, true, BKC>, grid, dim3(NT), 0, s, p, nslices, nsl, nbands);
    else launch(gemm_rows_kernel<KT, ABF, false, false, false, BKC>, grid, dim3(NT), 0, s, p, nslices, nsl, nbands);
  }
}

template <int KT, bool BKC>
static void launch_k(const GemmParams& p, dim3 grid, int nslices, int nsl, int64_t nbands, hipStream_t s) {
  if (p.abf && p.cbf) launch_kt<KT, true, true, BKC>(p, grid, nslices, nsl, nbands, s);
  else if (p.abf) launch_kt<KT, true, false, BKC>(p, grid, nslices, nsl, nbands, s);
  else if (p.cbf) launch_kt<KT, false, true, BKC>(p, grid, nslices, nsl, nbands, s);
  else launch_kt<KT, false, false, BKC>(p, grid, nslices, nsl, nbands, s);
}

// ---------------------------------------------------------------------------------------------
// Per-head products with 64 output columns per head (config C3's outp_h += S_h M_h^T (+ sumA_h wbar_h)
// in the forward, dQ_h += Sz_h M_h^T (+ sigz_h wbar_h) in the backward: batch = H = 4 heads, K = 256,
// N = 64, A_h = S[:, h, :]): one workgroup's 256 output columns are the four heads' 64, wave w serving
// head w / 2, columns 32 (w % 2) ..; every head has its own A band, so the LDS holds the four heads'
// 32-row bands ([4][32][KT + 8] bf16, one image: the next band waits in registers), and the epilogue
// adds fma(rowscale[m, h], bias2[h, n], .) after beta (epilogue_value's order).  Same MFMA sequence
// per output as the tiled bf16 path: bitwise equal to it.
// ---------------------------------------------------------------------------------------------
constexpr int HH = 4, HN = 64;   // heads per workgroup, columns per head

template <int KT, bool ABF>
struct HeadBand {
  static constexpr int CH = ABF ? KT / 8 : KT / 4;   // 16-byte chunks per row
  static constexpr int TOT = HH * ROWS * CH;
  static constexpr int PER = TOT / NT;
  static_assert(TOT % NT == 0, "head band chunks");
  gf4 r[PER];
  __device__ __forceinline__ void load(const GemmParams& p, int64_t band) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int h = idx / (ROWS * CH), rem = idx % (ROWS * CH);
      const int64_t row = min(band * ROWS + rem / CH, p.M - 1);
      const int k = (rem % CH) * (ABF ? 8 : 4);
      const int kc = k < p.K ? k : 0;
      r[i] = *reinterpret_cast<const gf4*>(eoff(p.A, h * p.sab + row * p.sam + kc, ABF));
    }
    asm volatile("" ::: "memory");
  }
  __device__ __forceinline__ void store(__bf16* __restrict__ img, int K) const {
    constexpr int KP = KT + 8;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int h = idx / (ROWS * CH), rem = idx % (ROWS * CH);
      const int rr = rem / CH, k = (rem % CH) * (ABF ? 8 : 4);
      __bf16* d = img + (h * ROWS + rr) * KP + k;
      const bool live = k < K;
      if constexpr (ABF) {
        u32x4 u = __builtin_bit_cast(u32x4, r[i]);
        if (!live) u = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(d) = u;
      } else {
        const gf4 v = live ? r[i] : gf4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<u32x2*>(d) = u32x2{pack2(v.x, v.y), pack2(v.z, v.w)};
      }
    }
  }
};

template <int KT, bool ABF, bool BETA, bool RS, bool BKC>
__global__ __launch_bounds__(NT, 1) void gemm_heads_kernel(GemmParams p, int64_t nbands) {
  constexpr int KP = KT + 8, T = KT / 16;
  __shared__ __attribute__((aligned(16))) __bf16 As[HH * ROWS * KP];
  __shared__ __attribute__((aligned(16))) float Lepi[NT / 64][ROWS * EPI_LD];
  __shared__ __attribute__((aligned(16))) float Lb[HH * HN], Lb2[HH * HN];
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int l32 = lane & 31, h = lane >> 5;
  const int hw = wave >> 1, c0 = (wave & 1) * 32;   // this wave's head and first column in it
  const bool has_bias = p.bias != nullptr;
  for (int i = threadIdx.x; i < HH * HN; i += NT) {
    const int hh = i / HN, c = i % HN;
    Lb[i] = has_bias ? p.bias[hh * p.sbias_b + c] : 0.f;
    Lb2[i] = RS ? p.bias2[hh * p.sb2_b + c] : 0.f;
  }
  bf16x8 bw[T];
  {
    const int K = (int)p.K;
    const float* Bc = p.B + hw * p.sbb + (c0 + l32) * p.sbn;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int k0 = 16 * t + 8 * h;
      if constexpr (BKC) {
        const int kc = min(k0, K - 8);
        const gf4 x = *reinterpret_cast<const gf4*>(Bc + kc), y = *reinterpret_cast<const gf4*>(Bc + kc + 4);
        const bool live = k0 < K;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bw[t][e] = (__bf16)(live ? x[e] : 0.f);
          bw[t][4 + e] = (__bf16)(live ? y[e] : 0.f);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = Bc[(int64_t)min(k0 + e, K - 1) * p.sbk];
          bw[t][e] = (__bf16)(k0 + e < K ? v : 0.f);
        }
      }
      if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  float* Cw = p.C + hw * p.scb + c0;
  const int64_t cbytes = ((p.M - 1) * p.scm + HN - c0) * 4;   // this wave's columns of the M rows
  const __amdgpu_buffer_rsrc_t cst = rsrc(Cw, cbytes);
  const __amdgpu_buffer_rsrc_t cld = rsrc(Cw, BETA ? cbytes : 0);
  float* Ls = Lepi[wave];
  constexpr int PASS = 4, RPP = ROWS / PASS, LPR = 64 / RPP;   // fp32 C: 8 rows x 8 lanes x 16 bytes
  const int er = lane / LPR, ec = (lane % LPR) * 4;
  const float* rsp = RS ? p.rowscale + hw * p.srs_b : nullptr;

  int64_t band = blockIdx.x;
  const int64_t Q = gridDim.x;
  if (band >= nbands) return;   // workgroup-uniform
  HeadBand<KT, ABF> ld;
  ld.load(p, band);
  while (true) {
    const int64_t row0 = band * ROWS;
    __syncthreads();   // every wave done with the previous band's image
    ld.store(As, (int)p.K);
    __syncthreads();
    // this band's epilogue operands, then the next band's rows (loads complete in order: the
    // epilogue then waits for its own operands only)
    gf4 cv[BETA ? PASS : 1];
    float rsv[RS ? PASS : 1];
#pragma unroll
    for (int ps = 0; ps < PASS; ++ps) {
      const int64_t row = row0 + RPP * ps + er;
      if constexpr (BETA)
        cv[ps] = __builtin_bit_cast(gf4, __builtin_amdgcn_raw_buffer_load_b128(cld, (int)((row * p.scm + ec) * 4), 0, 0));
      if constexpr (RS) rsv[ps] = rsp[min(row, p.M - 1) * p.srs_m];
    }
    const int64_t b1 = band + Q;
    if (b1 < nbands) ld.load(p, b1);   // workgroup-uniform
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const __bf16* Al = As + (hw * ROWS + l32) * KP + 8 * h;
    bf16x8 a[2];
    a[0] = *reinterpret_cast<const bf16x8*>(Al);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (t + 1 < T) a[(t + 1) & 1] = *reinterpret_cast<const bf16x8*>(Al + 16 * (t + 1));
      __builtin_amdgcn_sched_barrier(0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t & 1], bw[t], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) Ls[((r & 3) + 8 * (r >> 2) + 4 * h) * EPI_LD + l32] = __fmul_rn(p.alpha, acc[r]);
    const gf4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ps = 0; ps < PASS; ++ps) {
      const int rr = RPP * ps + er;
      gf4 v = *reinterpret_cast<const gf4*>(Ls + rr * EPI_LD + ec);
      if constexpr (BETA)
        v = gf4{fmaf(p.beta, cv[ps].x, v.x), fmaf(p.beta, cv[ps].y, v.y), fmaf(p.beta, cv[ps].z, v.z),
                fmaf(p.beta, cv[ps].w, v.w)};
      const int cb = hw * HN + c0 + ec;
      if (has_bias) {
        const gf4 bb = *reinterpret_cast<const gf4*>(Lb + cb);
        v = gf4{__fadd_rn(v.x, bb.x), __fadd_rn(v.y, bb.y), __fadd_rn(v.z, bb.z), __fadd_rn(v.w, bb.w)};
      }
      if constexpr (RS) {
        const gf4 b2 = *reinterpret_cast<const gf4*>(Lb2 + cb);
        v = gf4{fmaf(rsv[ps], b2.x, v.x), fmaf(rsv[ps], b2.y, v.y), fmaf(rsv[ps], b2.z, v.z), fmaf(rsv[ps], b2.w, v.w)};
      }
      v = p.relu ? __builtin_elementwise_max(v, zero) : v;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), cst, (int)(((row0 + rr) * p.scm + ec) * 4), 0, 0);
    }
    if (b1 >= nbands) break;
    band = b1;
  }
}

template <int KT, bool ABF, bool BKC>
static void launch_heads_k(const GemmParams& p, dim3 grid, int64_t nbands, hipStream_t s) {
  const bool beta = p.beta != 0.f, rs = p.rowscale != nullptr;
  if (beta && rs) launch(gemm_heads_kernel<KT, ABF, true, true, BKC>, grid, dim3(NT), 0, s, p, nbands);
  else if (beta) launch(gemm_heads_kernel<KT, ABF, true, false, BKC>, grid, dim3(NT), 0, s, p, nbands);
  else if (rs) launch(gemm_heads_kernel<KT, ABF, false, true, BKC>, grid, dim3(NT), 0, s, p, nbands);
  else launch(gemm_heads_kernel<KT, ABF, false, false, BKC>, grid, dim3(NT), 0, s, p, nbands);
}

}  // namespace rsk

// Shapes (host check, gemm.hip rows_ok): bf16 arithmetic, K <= 256 (K % 4 == 0, % 8 for bf16 A),
// N % 256 == 0, batched without batch reduction (no mask then), no split / row scatter / rowscale / rowsum, A k-contiguous 16-byte rows,
// fp32 B, row-major C and mask with 32-bit byte offsets.
void gemm_rows_launch(const GemmParams& p, int cus, hipStream_t s) {
  const int nsl = (int)(p.N / rsk::NB);
  const int nslices = nsl * (int)p.batch;   // work items: (batch entry, column slice)
  const int64_t nbands = (p.M + rsk::ROWS - 1) / rsk::ROWS;
  const int64_t items = (int64_t)nslices * nbands;
  const int G = (int)(std::min<int64_t>((int64_t)cus, items) / nslices * nslices);
  const dim3 grid((unsigned)std::max(G, nslices));
  const bool bkc = p.sbk == 1 && p.vecB && p.K % 8 == 0;
  if (p.K <= 64) {
    if (bkc) rsk::launch_k<64, true>(p, grid, nslices, nsl, nbands, s);
    else rsk::launch_k<64, false>(p, grid, nslices, nsl, nbands, s);
  } else {
    if (bkc) rsk::launch_k<256, true>(p, grid, nslices, nsl, nbands, s);
    else rsk::launch_k<256, false>(p, grid, nslices, nsl, nbands, s);
  }
}

// The per-head form (host check, gemm.hip heads_ok): bf16 arithmetic, batch = 4 heads of N = 64
// columns, K <= 256 (K % 8), W k-contiguous (M_h^T: 16-byte loads), fp32 C with 16-byte rows per head,
// no mask / split / row scatter / rowsum; rowscale x bias2 and beta allowed.
void gemm_heads_launch(const GemmParams& p, int cus, hipStream_t s) {
  const int64_t nbands = (p.M + rsk::ROWS - 1) / rsk::ROWS;
  const dim3 grid((unsigned)std::min<int64_t>((int64_t)cus, nbands));
  if (p.abf) rsk::launch_heads_k<256, true, true>(p, grid, nbands, s);   // W k-contiguous (host check)
  else rsk::launch_heads_k<256, false, true>(p, grid, nbands, s);
}

}  // namespace alignn
