// FeatureL2Norm and FeatureCorrelation on gfx950.
//
// l2norm_rows: y = x / sqrt(sum_c x^2 + 1e-6) over the contiguous channel axis
//   of a channels-last feature map (lib/model.py:14-17), written as bf16 in the
//   [B, H*W, C] layout the correlation GEMM consumes (one pass, one wave/row);
//   optionally also y_lo = bf16(y - y_hi) (the fp32-accurate "bf16x3" mode:
//   A.B ~ Ahi.Bhi + Ahi.Blo + Alo.Bhi on three bf16 GEMMs, ~16 mantissa bits).
//
// corr_gemm: C[b] = A[amap[b]] . B[bmap[b]]^T, A:[M,K], B:[N,K] bf16 row-major,
//   fp32 accumulate, fp32 or bf16 output (lib/model.py:106-115, '4D' mode).
//   amap/bmap let the negative pairs of the weak loss (train.py:137, a roll of
//   the source batch) reuse the positive-pass features without a copy.
//   128x128 output tile per 4-wave workgroup, BK = 64, register-staged double
//   buffer, XOR-swizzled LDS rows (conflict-free ds_read_b128), XCD remap.
//   Optional fused epilogue: 4D max-pooling with stride=kernel=ks (relocalization,
//   lib/model.py:177-191) when the feature rows are ordered in ks x ks spatial
//   blocks: the full-resolution volume is never written.
#include "common.h"
#include <hip/hip_fp8.h>

namespace ncnet {

// ---------------------------------------------------------------------------
// OUT: 0 bf16 (+ optional lo half), 1 OCP fp8 e4m3 (scaled), 2 IEEE half
template <typename TIN, int OUT>
__global__ __launch_bounds__(256) void l2norm_rows_kernel(const TIN* __restrict__ x, void* __restrict__ yv,
                                                          float* __restrict__ inv_norm, int rows, int C,
                                                          float out_scale, bf16* __restrict__ ylo) {
  constexpr bool FP8 = OUT == 1;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TIN* xr = x + (size_t)row * C;
  float ss = 0.f;
  for (int c = lane * 8; c < C; c += 512) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = (c + e < C) ? (float)xr[c + e] : 0.f;
      ss += v * v;
    }
  }
  ss = wave_sum(ss);
  const float inv = 1.f / sqrtf(ss + 1e-6f);
  if (lane == 0 && inv_norm) inv_norm[row] = inv;
  if (FP8) {
    // OCP e4m3, scaled by out_scale (unit rows have |y| <= 1: the scale moves
    // the typical 1/sqrt(C) entries out of the subnormal range)
    const float s = inv * out_scale;
    uint8_t* yr = (uint8_t*)yv + (size_t)row * C;
    for (int c = lane * 8; c < C; c += 512) {
      if (c + 8 <= C) {
        uint32_t w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t v = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v |= (uint32_t)__hip_cvt_float_to_fp8((float)xr[c + 4 * h + e] * s, __HIP_SATFINITE, __HIP_E4M3) << (8 * e);
          w[h] = v;
        }
        *(uint2*)(yr + c) = make_uint2(w[0], w[1]);
      } else {
        for (int e = 0; c + e < C; ++e)
          yr[c + e] = (uint8_t)__hip_cvt_float_to_fp8((float)xr[c + e] * s, __HIP_SATFINITE, __HIP_E4M3);
      }
    }
    return;
  }
  if (OUT == 2) {
    uint16_t* hr = (uint16_t*)yv + (size_t)row * C;
    for (int c = lane * 8; c < C; c += 512) {
      if (c + 8 <= C) {
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = (uint32_t)f2s16<true>((float)xr[c + 2 * e] * inv) |
                 ((uint32_t)f2s16<true>((float)xr[c + 2 * e + 1] * inv) << 16);
        *(u32x4*)(hr + c) = o;
      } else {
        for (int e = 0; c + e < C; ++e) hr[c + e] = f2s16<true>((float)xr[c + e] * inv);
      }
    }
    return;
  }
  bf16* yr = (bf16*)yv + (size_t)row * C;
  bf16* lr = ylo ? ylo + (size_t)row * C : nullptr;
  for (int c = lane * 8; c < C; c += 512) {
    if (c + 8 <= C) {
      bf16x8 o, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (float)xr[c + e] * inv;
        o[e] = f2bf(v);
        lo[e] = f2bf(v - (float)o[e]);
      }
      *(bf16x8*)(yr + c) = o;
      if (lr) *(bf16x8*)(lr + c) = lo;
    } else {
      for (int e = 0; c + e < C; ++e) {
        const float v = (float)xr[c + e] * inv;
        yr[c + e] = f2bf(v);
        if (lr) lr[c + e] = f2bf(v - (float)yr[c + e]);
      }
    }
  }
}

// grad_x = inv * (g - y * sum_c(g*y)),  y = x*inv   (fe_finetune path)
__global__ __launch_bounds__(256) void l2norm_rows_bwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                              const float* __restrict__ inv_norm,
                                                              float* __restrict__ gx, int rows, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float inv = inv_norm[row];
  const float* xr = x + (size_t)row * C;
  const float* gr = g + (size_t)row * C;
  float dot = 0.f;
  for (int c = lane; c < C; c += 64) dot += gr[c] * xr[c] * inv;
  dot = wave_sum(dot);
  float* o = gx + (size_t)row * C;
  for (int c = lane; c < C; c += 64) o[c] = inv * (gr[c] - xr[c] * inv * dot);
}

// ---------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;

// LDS tile: [128 rows][128 B] = 64 bf16 k (or 128 fp8 k) per row, 8 x 16-B
// chunks, chunk position XOR-swizzled by (row & 7).
__device__ __forceinline__ uint32_t tile_off(int row, int chunk) { return (uint32_t)(row * 128 + ((chunk ^ (row & 7)) << 4)); }

struct GemmArgs {
  const void* A; const void* B; void* C;
  const int* amap; const int* bmap;
  int M, N, K;
  long long sA, sB, sC;   // batch strides (elements)
  float out_scale;        // fp8: 1 / (scale_A * scale_B)
  int tiles_m, tiles_n;
  // fused max-pool epilogue
  int pool_ks;           // 0 = plain store
  float* pool_val; uint8_t* pool_idx;
  int hA, wA, hB, wB;    // full-res feature grid (pooling only)
};

// plain / fused-pool epilogue of a wave's TM x TN 16 x 16 sub-tiles (below)
template <int TM, int TN, bool OUT_BF16, bool POOL, bool F16 = false>
__device__ __forceinline__ void corr_v2_epilogue(const f32x4 (&acc)[TM][TN], const GemmArgs& p, int b, int row0,
                                                 int col0, int lane);

// F16 (with !FP8): IEEE-half operands (f16 MFMA) and, with OUT_BF16, an IEEE-half output.
template <bool OUT_BF16, bool POOL, bool FP8, bool F16 = false>
__global__ __launch_bounds__(256, 2) void corr_gemm_kernel(GemmArgs p) {
  constexpr int EB = FP8 ? 1 : 2;            // bytes per element
  constexpr int KT = 128 / EB;               // k per 128-B LDS row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;                 // BM x BK
  char* Bs = smem + BM * 128;      // BN x 128 B

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % p.tiles_n; bid /= p.tiles_n;
  const int tm = bid % p.tiles_m;
  const int b = bid / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const char* A = (const char*)p.A + (size_t)(p.amap ? p.amap[b] : b) * p.sA * EB;
  const char* B = (const char*)p.B + (size_t)(p.bmap ? p.bmap[b] : b) * p.sB * EB;

  // staging: 1024 chunks per operand, 4 per thread
  u32x4 ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int c = threadIdx.x + m * 256;
      int row = c >> 3, ch = c & 7;
      int ga = m0 + row, gb = n0 + row, kk = k0 + ch * (16 / EB);
      ra[m] = (ga < p.M && kk < p.K) ? *(const u32x4*)(A + ((size_t)ga * p.K + kk) * EB) : u32x4{0u, 0u, 0u, 0u};
      rb[m] = (gb < p.N && kk < p.K) ? *(const u32x4*)(B + ((size_t)gb * p.K + kk) * EB) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int c = threadIdx.x + m * 256;
      int row = c >> 3, ch = c & 7;
      *(u32x4*)(As + tile_off(row, ch)) = ra[m];
      *(u32x4*)(Bs + tile_off(row, ch)) = rb[m];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto finish = [&]() {
    if (FP8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = acc[i][j] * p.out_scale;
    }
  };

  const int nk = (p.K + KT - 1) / KT;
  load(0);
  store();
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load((kt + 1) * KT);
    if (FP8) {
      // one K=128 MX-fp8 MFMA per sub-tile: lane group fq owns bytes 32fq..32fq+31
      i32x8 af[4], bfv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + fr;
        u32x4 lo = *(const u32x4*)(As + tile_off(r, 2 * fq)), hi = *(const u32x4*)(As + tile_off(r, 2 * fq + 1));
        af[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + fr;
        u32x4 lo = *(const u32x4*)(Bs + tile_off(r, 2 * fq)), hi = *(const u32x4*)(Bs + tile_off(r, 2 * fq + 1));
        bfv[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_fp8_k128(af[i], bfv[j], acc[i][j]);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[4], bfv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = lds_read16(As, tile_off(wm * 64 + i * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int j = 0; j < 4; ++j) bfv[j] = lds_read16(Bs, tile_off(wn * 64 + j * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = mfma16t<F16>(__builtin_bit_cast(u32x4, af[i]), __builtin_bit_cast(u32x4, bfv[j]), acc[i][j]);
      }
    }
    __syncthreads();
    if (more) store();
    __syncthreads();
  }

  finish();
  corr_v2_epilogue<4, 4, OUT_BF16, POOL, F16>(acc, p, b, m0 + wm * 64, n0 + wn * 64, lane);
}

// ===========================================================================
// corr_gemm_v2 (bf16, large grids: the InLoc volumes): the correlation GEMM
// fed by LDS-DMA through a 4-stage ring, as conv2d_nhwc_v2 (csrc/conv2d.hip):
// 256 x 128 tile, 8 waves of 64 x 64, BK = 32 (64-byte LDS rows, swizzled
// DMA source), one barrier per k-step with a compile-time vmcnt, global loads
// three k-steps ahead of the MFMAs (v1: register double buffer, the k-step's
// compute shorter than the load latency).  Rows past M / N read a 16-byte zero
// block.  Tile order: GM consecutive row tiles per column sweep, so the ~32
// workgroups an XCD runs at once share 4 A and 8 B tiles in its L2 instead of
// 1 A and 32 B.  Epilogues: plain fp32 / bf16 store, or the fused 2x2x2x2
// max-pool with packed argmax offsets, division-free and reduced through DPP
// quad moves, shared with v1 (the earlier epilogue with per-sub-tile integer
// divisions and ds_bpermute shuffles was ~1800 VALU per wave, more issue time
// than the tile's MFMAs at K = 1024: `profiles/r5/kernels/pmc_corr_3200*.md`).
// ===========================================================================
__device__ const uint4 g_corr_zero16 = {0u, 0u, 0u, 0u};

namespace cg2 {
constexpr int BM = 256, BN = 128, NW = 8, BK = 32, GM = 4;
constexpr int APW = BM / (16 * NW), BPW = BN / (16 * NW), PER = APW + BPW;
constexpr int STAGE = (BM + BN) * 64;
__device__ __forceinline__ int swz(int r) { return (r & 1) ^ ((r >> 1) & 2); }
__device__ __forceinline__ uint32_t roff(int row, int chunk) { return (uint32_t)(row * 64 + ((chunk ^ swz(row)) << 4)); }
}  // namespace cg2

template <int N>
__device__ __forceinline__ void cg2_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Epilogue of the v2 kernels for one wave's TM x TN 16 x 16 sub-tiles at
// (row0, col0): plain fp32 / bf16 store, or the fused 2x2x2x2 max-pool.
template <int TM, int TN, bool OUT_BF16, bool POOL, bool F16>
__device__ __forceinline__ void corr_v2_epilogue(const f32x4 (&acc)[TM][TN], const GemmArgs& p, int b, int row0,
                                                 int col0, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  if (!POOL) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gm = row0 + i * 16 + 4 * fq + r, gn = col0 + j * 16 + fr;
          if (gm < p.M && gn < p.N) {
            const size_t o = (size_t)b * p.sC + (size_t)gm * p.N + gn;
            if (OUT_BF16) ((uint16_t*)p.C)[o] = f2s16<F16>(acc[i][j][r]);
            else ((float*)p.C)[o] = acc[i][j][r];
          }
        }
  } else {
    // rows / columns in 2x2-block order: a lane's 4 accumulator rows are one A
    // block, the 4 columns of a B block sit in the lane quad fr&~3 .. fr|3.
    // Block index = pooled index (ba = ai * wA/2 + aj), so the pooled offset
    // is ba * nb + bb with no division.  Max first (quad max through DPP),
    // then the smallest packed offset code among the lanes / rows holding it:
    // the code is a bit-spread of r * 4 + (fr & 3), so its order is the
    // row-major tie order of the unfused pool.  M, N are multiples of 4: a
    // block is wholly inside or outside the volume.
    const size_t nb = (size_t)(p.hB >> 1) * (p.wB >> 1);
    const size_t vol = (size_t)(p.hA >> 1) * (p.wA >> 1) * nb;
    const int lcode = ((fr & 2) << 1) | (fr & 1);
    const bool lead = (fr & 3) == 0;
    size_t aoff[TM];
    bool aok[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int gm = row0 + i * 16 + 4 * fq;
      aok[i] = gm < p.M;
      aoff[i] = (size_t)b * vol + (size_t)(gm >> 2) * nb;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int gn = col0 + j * 16 + (fr & ~3);
      const bool bok = lead && gn < p.N;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const f32x4 v = acc[i][j];
        float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0xB1, 0xF, 0xF, false)));   // quad xor 1
        m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x4E, 0xF, 0xF, false)));   // quad xor 2
        int c = v[3] == m ? 0x50 : 0xFF;   // 0xFF: no element of this lane holds the quad max
        c = v[2] == m ? 0x40 : c;
        c = v[1] == m ? 0x10 : c;
        c = v[0] == m ? 0x00 : c;
        c |= lcode;
        c = min(c, __builtin_amdgcn_mov_dpp(c, 0xB1, 0xF, 0xF, false));
        c = min(c, __builtin_amdgcn_mov_dpp(c, 0x4E, 0xF, 0xF, false));
        if (c == 0xFF) c = 0;                // an all-NaN quad: offset 0, never an out-of-range code
        if (bok && aok[i]) {
          const size_t o = aoff[i] + (size_t)(gn >> 2);
          if (NCNET_OK(o < (size_t)(b + 1) * vol)) {
            p.pool_val[o] = m;
            p.pool_idx[o] = (uint8_t)c;
          }
        }
      }
    }
  }
}

template <bool OUT_BF16, bool POOL, int NS, bool F16 = false>
__global__ __launch_bounds__(512, NS <= 3 ? 2 : 1) void corr_gemm_v2_kernel(GemmArgs p) {
  constexpr int BM = cg2::BM, BN = cg2::BN, BK = cg2::BK, GM = cg2::GM;
  constexpr int APW = cg2::APW, BPW = cg2::BPW, PER = cg2::PER, STAGE = cg2::STAGE;
  using cg2::swz;
  using cg2::roff;
  constexpr int TM = 4, TN = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_b = p.tiles_m * p.tiles_n;
  const int b = bid / per_b;
  int t = bid - b * per_b;
  const int grp = t / (GM * p.tiles_n), first = grp * GM;
  const int gsz = min(GM, p.tiles_m - first);
  t -= grp * GM * p.tiles_n;
  const int tm = first + t % gsz, tn = t / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const bf16* A = (const bf16*)p.A + (size_t)(p.amap ? p.amap[b] : b) * p.sA;
  const bf16* B = (const bf16*)p.B + (size_t)(p.bmap ? p.bmap[b] : b) * p.sB;
  const bf16* zero = (const bf16*)&g_corr_zero16;
  const int pos = lane & 3;

  const bf16* a_ptr[APW];
  bool a_ok[APW];
#pragma unroll
  for (int m = 0; m < APW; ++m) {
    const int row = 16 * (wave * APW + m) + (lane >> 2);
    a_ok[m] = m0 + row < p.M;
    a_ptr[m] = A + (size_t)(a_ok[m] ? m0 + row : 0) * p.K + (pos ^ swz(row)) * 8;
  }
  const bf16* b_ptr[BPW];
  bool b_ok[BPW];
#pragma unroll
  for (int m = 0; m < BPW; ++m) {
    const int row = 16 * (wave * BPW + m) + (lane >> 2);
    b_ok[m] = n0 + row < p.N;
    b_ptr[m] = B + (size_t)(b_ok[m] ? n0 + row : 0) * p.K + (pos ^ swz(row)) * 8;
  }
  const int nk = p.K / BK;
  auto issue = [&](int ks, int buf) {
    char* sb = smem + buf * STAGE;
    const int kk = ks * BK;
#pragma unroll
    for (int m = 0; m < APW; ++m)
      __builtin_amdgcn_global_load_lds((const void*)(a_ok[m] ? a_ptr[m] + kk : zero),
                                       LDS_PTR(void, sb + (wave * APW + m) * 1024), 16, 0, 0);
#pragma unroll
    for (int m = 0; m < BPW; ++m)
      __builtin_amdgcn_global_load_lds((const void*)(b_ok[m] ? b_ptr[m] + kk : zero),
                                       LDS_PTR(void, sb + BM * 64 + (wave * BPW + m) * 1024), 16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
  const int fr = lane & 15, fq = lane >> 4;
  int buf = 0;
  for (int ks = 0; ks < nk; ++ks) {
    const int after = min(NS - 2, nk - 1 - ks);
    if (after >= 2) cg2_wait_barrier<2 * PER>();
    else if (after >= 1) cg2_wait_barrier<PER>();
    else cg2_wait_barrier<0>();
    if (ks + NS - 1 < nk) issue(ks + NS - 1, (buf + NS - 1) % NS);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 64;
    bf16x8 af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = lds_read16(As, roff(wm * 64 + i * 16 + fr, fq));
    bf16x8 bcur = lds_read16(Bs, roff(wn * 64 + fr, fq));
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bf16x8 bnext = bcur;
      if (j + 1 < TN) bnext = lds_read16(Bs, roff(wn * 64 + (j + 1) * 16 + fr, fq));
      __builtin_amdgcn_sched_barrier(0);   // keep the read ahead of these MFMAs (counted lgkmcnt)
#pragma unroll
      for (int i = 0; i < TM; ++i)
        acc[i][j] = mfma16t<F16>(__builtin_bit_cast(u32x4, af[i]), __builtin_bit_cast(u32x4, bcur), acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
      bcur = bnext;
    }
    buf = (buf + 1 == NS) ? 0 : buf + 1;
  }

  corr_v2_epilogue<TM, TN, OUT_BF16, POOL, F16>(acc, p, b, m0 + wm * 64, n0 + wn * 64, lane);
}


// ---------------------------------------------------------------------------
// corr_gemm_f8v2: the MX-fp8 (OCP e4m3) correlation GEMM on the same LDS-DMA
// ring: 256 x 128 tile, 8 waves of 64 x 64, one K = 128 stage (a 128-byte LDS
// row) per v_mfma_scale_f32_16x16x128_f8f6f4 k-step, 3 stages (144 KB, one
// workgroup per CU).  A lane's 32 operand bytes are two ds_read_b128 of
// chunks 2fq, 2fq + 1; chunk c of row r sits at 16-byte slot c ^ h(r),
// h(r) = bit1(r) | bit3(r) << 2 (searched offline: both reads conflict-free
// for all four ds_read_b128 lane groups; rows r, r+1 alternate 128-byte
// halves of the 256-byte bank period).  The DMA source is swizzled instead.
// ---------------------------------------------------------------------------
namespace cf2 {
constexpr int BM = 256, BN = 128, NW = 8, NS = 3, GM = 4;
constexpr int APW = BM / (8 * NW), BPW = BN / (8 * NW), PER = APW + BPW;   // 8 rows per DMA instruction
constexpr int STAGE = (BM + BN) * 128;
__device__ __forceinline__ int h(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ uint32_t roff(int row, int chunk) { return (uint32_t)(row * 128 + ((chunk ^ h(row)) << 4)); }
}  // namespace cf2

// Persistent: one workgroup per CU walks tiles lid = it * gridDim + r(blockIdx)
// (r = the XCD remap, so the tiles an XCD holds at once are neighbours), and
// the DMA ring runs across tile boundaries: the first NS - 1 stages of the
// next tile are in flight during the last k-steps and the epilogue of the
// current one.  With K = 1024 a tile is only 8 k-steps, so a per-tile ring
// fill (one workgroup per CU: nothing else hides it) cost as much as the
// MFMAs.  Every wave of a workgroup runs the same tile sequence (uniform exit).
__device__ __forceinline__ void cf2_tile(uint32_t lid, const GemmArgs& p, int& b, int& m0, int& n0) {
  const int per_b = p.tiles_m * p.tiles_n;
  b = (int)lid / per_b;
  int t = (int)lid - b * per_b;
  const int grp = t / (cf2::GM * p.tiles_n), first = grp * cf2::GM;
  const int gsz = min(cf2::GM, p.tiles_m - first);
  t -= grp * cf2::GM * p.tiles_n;
  m0 = (first + t % gsz) * cf2::BM;
  n0 = (t / gsz) * cf2::BN;
}

template <bool OUT_BF16, bool POOL>
__global__ __launch_bounds__(512, 1) void corr_gemm_f8v2_kernel(GemmArgs p, int total_tiles) {
  constexpr int BM = cf2::BM, NS = cf2::NS;
  constexpr int APW = cf2::APW, BPW = cf2::BPW, PER = cf2::PER, STAGE = cf2::STAGE;
  constexpr int TM = 4, TN = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const uint32_t G = gridDim.x, r0 = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = r0 < (uint32_t)total_tiles ? (int)((total_tiles - 1 - r0) / G) + 1 : 0;
  const int nk = p.K / 128;
  const int nsteps = ntiles * nk;
  const uint8_t* zero = (const uint8_t*)&g_corr_zero16;
  const int pos = lane & 7;

  // issue side: the tile whose stages are being fetched
  const uint8_t* a_ptr[APW];
  bool a_ok[APW];
  const uint8_t* b_ptr[BPW];
  bool b_ok[BPW];
  int is_tile = -1, is_ks = 0;
  auto issue_tile = [&](int it) {
    int b, m0, n0;
    cf2_tile(r0 + (uint32_t)it * G, p, b, m0, n0);
    const uint8_t* A = (const uint8_t*)p.A + (size_t)(p.amap ? p.amap[b] : b) * p.sA;
    const uint8_t* B = (const uint8_t*)p.B + (size_t)(p.bmap ? p.bmap[b] : b) * p.sB;
#pragma unroll
    for (int m = 0; m < APW; ++m) {
      const int row = 8 * (wave * APW + m) + (lane >> 3);
      a_ok[m] = m0 + row < p.M;
      a_ptr[m] = A + (size_t)(a_ok[m] ? m0 + row : 0) * p.K + (pos ^ cf2::h(row)) * 16;
    }
#pragma unroll
    for (int m = 0; m < BPW; ++m) {
      const int row = 8 * (wave * BPW + m) + (lane >> 3);
      b_ok[m] = n0 + row < p.N;
      b_ptr[m] = B + (size_t)(b_ok[m] ? n0 + row : 0) * p.K + (pos ^ cf2::h(row)) * 16;
    }
  };
  // fetch global step g (= the next unissued one) into ring slot buf
  auto issue = [&](int buf) {
    if (is_ks == 0) issue_tile(++is_tile);
    char* sb = smem + buf * STAGE;
    const int kk = is_ks * 128;
#pragma unroll
    for (int m = 0; m < APW; ++m)
      __builtin_amdgcn_global_load_lds((const void*)(a_ok[m] ? a_ptr[m] + kk : zero),
                                       LDS_PTR(void, sb + (wave * APW + m) * 1024), 16, 0, 0);
#pragma unroll
    for (int m = 0; m < BPW; ++m)
      __builtin_amdgcn_global_load_lds((const void*)(b_ok[m] ? b_ptr[m] + kk : zero),
                                       LDS_PTR(void, sb + BM * 128 + (wave * BPW + m) * 1024), 16, 0, 0);
    is_ks = (is_ks + 1 == nk) ? 0 : is_ks + 1;
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nsteps) issue(s);
  const int fr = lane & 15, fq = lane >> 4;
  int buf = 0, g = 0;
  for (int it = 0; it < ntiles; ++it) {
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < nk; ++ks, ++g) {
      // stage g landed (the one after it may still be in flight; a previous
      // tile's epilogue stores, issued later, make this wait conservative)
      if (g + 1 < nsteps) cg2_wait_barrier<PER>();
      else cg2_wait_barrier<0>();
      if (g + NS - 1 < nsteps) issue((buf + NS - 1) % NS);
      const char* As = smem + buf * STAGE;
      const char* Bs = As + BM * 128;
      auto frag = [&](const char* base, int r) {
        const u32x4 lo = *(const u32x4*)(base + cf2::roff(r, 2 * fq)), hi = *(const u32x4*)(base + cf2::roff(r, 2 * fq + 1));
        return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      };
      // column fragments stream one ahead of their MFMAs, so the matrix cores
      // start after the A fragments and the first B fragment have landed
      i32x8 af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag(As, wm * 64 + i * 16 + fr);
      i32x8 bcur = frag(Bs, wn * 64 + fr);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        i32x8 bnext = bcur;
        if (j + 1 < TN) bnext = frag(Bs, wn * 64 + (j + 1) * 16 + fr);
        __builtin_amdgcn_sched_barrier(0);   // keep the read ahead of these MFMAs (counted lgkmcnt)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma_fp8_k128(af[i], bcur, acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
        bcur = bnext;
      }
      buf = (buf + 1 == NS) ? 0 : buf + 1;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] * p.out_scale;
    int b, m0, n0;
    cf2_tile(r0 + (uint32_t)it * G, p, b, m0, n0);
    corr_v2_epilogue<TM, TN, OUT_BF16, POOL>(acc, p, b, m0 + wm * 64, n0 + wn * 64, lane);
  }
}

}  // namespace ncnet

using namespace ncnet;

// y dtype: bf16 (fp8_scale == 0; ylo: optional low half) or OCP fp8 e4m3 scaled by fp8_scale.
// y_f16: y is IEEE half (no lo half, no fp8).
extern "C" int ncnet_l2norm_rows(const void* x, int x_is_bf16, void* y, float* inv_norm, int rows, int C,
                                 float fp8_scale, void* ylo, int y_f16, hipStream_t stream) {
  bf16* lo = (bf16*)ylo;
  dim3 grid((unsigned)cdiv(rows, 4)), block(256);
  const bool f8 = fp8_scale != 0.f;
  if (y_f16 && (f8 || lo)) return -1;
#define L2N(TIN) do { \
    if (f8) hipLaunchKernelGGL((l2norm_rows_kernel<TIN, 1>), grid, block, 0, stream, (const TIN*)x, y, inv_norm, rows, C, fp8_scale, nullptr); \
    else if (y_f16) hipLaunchKernelGGL((l2norm_rows_kernel<TIN, 2>), grid, block, 0, stream, (const TIN*)x, y, inv_norm, rows, C, 1.f, nullptr); \
    else hipLaunchKernelGGL((l2norm_rows_kernel<TIN, 0>), grid, block, 0, stream, (const TIN*)x, y, inv_norm, rows, C, 1.f, lo); \
  } while (0)
  if (x_is_bf16) L2N(bf16); else L2N(float);
#undef L2N
  return (int)hipGetLastError();
}

extern "C" int ncnet_l2norm_rows_bwd(const float* x, const float* g, const float* inv_norm, float* gx, int rows, int C,
                                     hipStream_t stream) {
  dim3 grid((unsigned)cdiv(rows, 4)), block(256);
  hipLaunchKernelGGL(l2norm_rows_bwd_kernel, grid, block, 0, stream, x, g, inv_norm, gx, rows, C);
  return (int)hipGetLastError();
}

// v2 (LDS-DMA ring, 256 x 128 tiles; bf16 and MX-fp8) for GEMMs whose grid
// still gives >= 2 workgroups per CU (InLoc volumes); v1 for the small
// training GEMMs.  NCNET_CORR_V2=0 / 1 forces v1 / v2 (where legal: K % 32 ==
// 0 for bf16, K % 128 == 0 for fp8).
static bool use_v2(bool f8, int batch, int M, int N, int K) {
  if (K % (f8 ? 128 : cg2::BK) != 0) return false;
  const int force = tuning().corr_v2;
  if (force >= 0) return force == 1;
  return (long long)batch * cdiv(M, cg2::BM) * cdiv(N, cg2::BN) >= 512;
}

// ring depth: 4 stages (96 KB, one workgroup per CU) or 3 (72 KB, two per CU); NCNET_CORR_NS
static int cg2_stages() {
  return tuning().corr_ns == 4 ? 4 : 3;
}

// C[b] = A[amap[b]] . B[bmap[b]]^T ; out_bf16 selects the output dtype.
// fp8_out_scale != 0: A, B are OCP fp8 e4m3 and C = fp8_out_scale * (A . B^T).
// f16: A, B (and a 16-bit C) are IEEE half.
extern "C" int ncnet_corr_gemm(const void* A, const void* B, void* C, const int* amap, const int* bmap, int batch,
                               int M, int N, int K, long long sA, long long sB, long long sC, int out_bf16,
                               float fp8_out_scale, int f16, hipStream_t stream) {
  const bool f8 = fp8_out_scale != 0.f;
  if (f8 && f16) return -1;
  if (K % (f8 ? 16 : 8) != 0) return -1;
  GemmArgs p{};
  p.A = A; p.B = B; p.C = C; p.amap = amap; p.bmap = bmap;
  p.M = M; p.N = N; p.K = K; p.sA = sA; p.sB = sB; p.sC = sC;
  p.out_scale = fp8_out_scale;
  if (f8 && use_v2(f8, batch, M, N, K)) {
    p.tiles_m = cdiv(M, cf2::BM); p.tiles_n = cdiv(N, cf2::BN);
    const int tiles = batch * p.tiles_m * p.tiles_n;
    dim3 grid((unsigned)std::min(tiles, device_num_cus())), block(512);   // persistent
    const size_t lds = cf2::NS * cf2::STAGE;
    if (out_bf16) hipLaunchKernelGGL((corr_gemm_f8v2_kernel<true, false>), grid, block, lds, stream, p, tiles);
    else hipLaunchKernelGGL((corr_gemm_f8v2_kernel<false, false>), grid, block, lds, stream, p, tiles);
    return (int)hipGetLastError();
  }
  if (use_v2(f8, batch, M, N, K)) {
    p.tiles_m = cdiv(M, cg2::BM); p.tiles_n = cdiv(N, cg2::BN);
    dim3 grid((unsigned)(batch * p.tiles_m * p.tiles_n)), block(512);
#define CG2(OB, NSV, H) hipLaunchKernelGGL((corr_gemm_v2_kernel<OB, false, NSV, H>), grid, block, NSV * cg2::STAGE, stream, p)
    if (cg2_stages() == 3) {
      if (f16) { if (out_bf16) CG2(true, 3, true); else CG2(false, 3, true); }
      else { if (out_bf16) CG2(true, 3, false); else CG2(false, 3, false); }
    } else {
      if (f16) { if (out_bf16) CG2(true, 4, true); else CG2(false, 4, true); }
      else { if (out_bf16) CG2(true, 4, false); else CG2(false, 4, false); }
    }
#undef CG2
    return (int)hipGetLastError();
  }
  p.tiles_m = cdiv(M, BM); p.tiles_n = cdiv(N, BN);
  dim3 grid((unsigned)(batch * p.tiles_m * p.tiles_n)), block(256);
  size_t lds = (size_t)(BM + BN) * 128;
  if (f8) {
    if (out_bf16) hipLaunchKernelGGL((corr_gemm_kernel<true, false, true>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((corr_gemm_kernel<false, false, true>), grid, block, lds, stream, p);
  } else if (f16) {
    if (out_bf16) hipLaunchKernelGGL((corr_gemm_kernel<true, false, false, true>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((corr_gemm_kernel<false, false, false, true>), grid, block, lds, stream, p);
  } else {
    if (out_bf16) hipLaunchKernelGGL((corr_gemm_kernel<true, false, false>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((corr_gemm_kernel<false, false, false>), grid, block, lds, stream, p);
  }
  return (int)hipGetLastError();
}

// Fused correlation + 2x2x2x2 max-pool.  A rows / B rows must be in
// 2x2-block order (see ncnet_block_order_rows); hA, wA, hB, wB even.
extern "C" int ncnet_corr_gemm_pool2(const void* A, const void* B, float* pool_val, uint8_t* pool_idx, int batch,
                                     int hA, int wA, int hB, int wB, int K, long long sA, long long sB,
                                     float fp8_out_scale, int f16, hipStream_t stream) {
  const bool f8 = fp8_out_scale != 0.f;
  if (f8 && f16) return -1;
  if (K % (f8 ? 16 : 8) != 0 || (hA & 1) || (wA & 1) || (hB & 1) || (wB & 1)) return -1;
  GemmArgs p{};
  p.A = A; p.B = B; p.C = nullptr;
  p.M = hA * wA; p.N = hB * wB; p.K = K; p.sA = sA; p.sB = sB;
  p.out_scale = fp8_out_scale;
  p.pool_ks = 2; p.pool_val = pool_val; p.pool_idx = pool_idx;
  p.hA = hA; p.wA = wA; p.hB = hB; p.wB = wB;
  if (f8 && use_v2(f8, batch, p.M, p.N, K)) {
    p.tiles_m = cdiv(p.M, cf2::BM); p.tiles_n = cdiv(p.N, cf2::BN);
    const int tiles = batch * p.tiles_m * p.tiles_n;
    dim3 grid((unsigned)std::min(tiles, device_num_cus())), block(512);   // persistent
    hipLaunchKernelGGL((corr_gemm_f8v2_kernel<false, true>), grid, block, cf2::NS * cf2::STAGE, stream, p, tiles);
    return (int)hipGetLastError();
  }
  if (use_v2(f8, batch, p.M, p.N, K)) {
    p.tiles_m = cdiv(p.M, cg2::BM); p.tiles_n = cdiv(p.N, cg2::BN);
    dim3 grid((unsigned)(batch * p.tiles_m * p.tiles_n)), block(512);
    if (f16) {
      if (cg2_stages() == 3) hipLaunchKernelGGL((corr_gemm_v2_kernel<false, true, 3, true>), grid, block, 3 * cg2::STAGE, stream, p);
      else hipLaunchKernelGGL((corr_gemm_v2_kernel<false, true, 4, true>), grid, block, 4 * cg2::STAGE, stream, p);
    } else {
      if (cg2_stages() == 3) hipLaunchKernelGGL((corr_gemm_v2_kernel<false, true, 3>), grid, block, 3 * cg2::STAGE, stream, p);
      else hipLaunchKernelGGL((corr_gemm_v2_kernel<false, true, 4>), grid, block, 4 * cg2::STAGE, stream, p);
    }
    return (int)hipGetLastError();
  }
  p.tiles_m = cdiv(p.M, BM); p.tiles_n = cdiv(p.N, BN);
  dim3 grid((unsigned)(batch * p.tiles_m * p.tiles_n)), block(256);
  size_t lds = (size_t)(BM + BN) * 128;
  if (f8) hipLaunchKernelGGL((corr_gemm_kernel<false, true, true>), grid, block, lds, stream, p);
  else if (f16) hipLaunchKernelGGL((corr_gemm_kernel<false, true, false, true>), grid, block, lds, stream, p);
  else hipLaunchKernelGGL((corr_gemm_kernel<false, true, false>), grid, block, lds, stream, p);
  return (int)hipGetLastError();
}
