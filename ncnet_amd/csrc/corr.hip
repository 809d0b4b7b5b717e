// FeatureL2Norm and FeatureCorrelation on gfx950.
//
// l2norm_rows: y = x / sqrt(sum_c x^2 + 1e-6) over the contiguous channel axis
//   of a channels-last feature map (lib/model.py:14-17), written as bf16 in the
//   [B, H*W, C] layout the correlation GEMM consumes (one pass, one wave/row).
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

namespace ncnet {

// ---------------------------------------------------------------------------
template <typename TIN>
__global__ __launch_bounds__(256) void l2norm_rows_kernel(const TIN* __restrict__ x, bf16* __restrict__ y,
                                                          float* __restrict__ inv_norm, int rows, int C) {
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
  bf16* yr = y + (size_t)row * C;
  for (int c = lane * 8; c < C; c += 512) {
    if (c + 8 <= C) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf((float)xr[c + e] * inv);
      *(bf16x8*)(yr + c) = o;
    } else {
      for (int e = 0; c + e < C; ++e) yr[c + e] = f2bf((float)xr[c + e] * inv);
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

// LDS tile: [128 rows][64 k] bf16 = 128 B rows of 8 x 16-B chunks, chunk
// position XOR-swizzled by (row & 7).
__device__ __forceinline__ uint32_t tile_off(int row, int chunk) { return (uint32_t)(row * 128 + ((chunk ^ (row & 7)) << 4)); }

struct GemmArgs {
  const bf16* A; const bf16* B; void* C;
  const int* amap; const int* bmap;
  int M, N, K;
  long long sA, sB, sC;   // batch strides (elements)
  int tiles_m, tiles_n;
  // fused max-pool epilogue
  int pool_ks;           // 0 = plain store
  float* pool_val; uint8_t* pool_idx;
  int hA, wA, hB, wB;    // full-res feature grid (pooling only)
};

template <bool OUT_BF16, bool POOL>
__global__ __launch_bounds__(256, 2) void corr_gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;                 // BM x BK
  char* Bs = smem + BM * BK * 2;   // BN x BK

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % p.tiles_n; bid /= p.tiles_n;
  const int tm = bid % p.tiles_m;
  const int b = bid / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const bf16* A = p.A + (size_t)(p.amap ? p.amap[b] : b) * p.sA;
  const bf16* B = p.B + (size_t)(p.bmap ? p.bmap[b] : b) * p.sB;

  // staging: 1024 chunks per operand, 4 per thread
  u32x4 ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int c = threadIdx.x + m * 256;
      int row = c >> 3, ch = c & 7;
      int ga = m0 + row, gb = n0 + row, kk = k0 + ch * 8;
      ra[m] = (ga < p.M && kk < p.K) ? *(const u32x4*)(A + (size_t)ga * p.K + kk) : u32x4{0u, 0u, 0u, 0u};
      rb[m] = (gb < p.N && kk < p.K) ? *(const u32x4*)(B + (size_t)gb * p.K + kk) : u32x4{0u, 0u, 0u, 0u};
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

  const int nk = (p.K + BK - 1) / BK;
  load(0);
  store();
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load((kt + 1) * BK);
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
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfv[j], acc[i][j]);
    }
    __syncthreads();
    if (more) store();
    __syncthreads();
  }

  if (!POOL) {
    // D[row = 4fq + r][col = fr] of sub-tile (i,j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int gm = m0 + wm * 64 + i * 16 + 4 * fq + r, gn = n0 + wn * 64 + j * 16 + fr;
          if (gm < p.M && gn < p.N) {
            size_t o = (size_t)b * p.sC + (size_t)gm * p.N + gn;
            if (OUT_BF16) ((bf16*)p.C)[o] = f2bf(acc[i][j][r]);
            else ((float*)p.C)[o] = acc[i][j][r];
          }
        }
  } else {
    // Pooling epilogue for ks = 2: rows are ordered so that the 4 rows of a
    // 2x2 spatial block are consecutive (row = 4*blk + 2*dy + dx), same for
    // columns.  A lane's 4 accumulator rows (4fq..4fq+3) are exactly one A
    // block; the 4 columns of a B block live in lanes fr&~3 .. fr|3.
    // Reduce over the 4 rows in registers, then over 4 lanes with shuffles.
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float best = acc[i][j][0];
        int bidx = 0;  // (dyA*2+dxA)*4 + (dyB*2+dxB)
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (acc[i][j][r] > best) { best = acc[i][j][r]; bidx = r * 4; }
        bidx += (fr & 3);
        // butterfly over the 4 lanes of the B block (keep first max on ties)
#pragma unroll
        for (int o = 1; o < 4; o <<= 1) {
          float ob = __shfl_xor(best, o, 64);
          int oi = __shfl_xor(bidx, o, 64);
          bool take = (ob > best) || (ob == best && oi < bidx);
          best = take ? ob : best;
          bidx = take ? oi : bidx;
        }
        int gm = m0 + wm * 64 + i * 16 + 4 * fq;   // first row of the A block
        int gn = n0 + wn * 64 + j * 16 + (fr & ~3); // first col of the B block
        if ((fr & 3) == 0 && gm < p.M && gn < p.N) {
          int ba = gm >> 2, bb = gn >> 2;          // pooled A / B cell (block-major)
          int pa_w = p.wA >> 1, pb_w = p.wB >> 1;
          int ai = ba / pa_w, aj = ba - ai * pa_w;
          int bi = bb / pb_w, bj = bb - bi * pb_w;
          int ra_ = bidx >> 2, rb_ = bidx & 3;
          // offsets (di, dj, dk, dl) packed 2 bits each
          uint8_t code = (uint8_t)(((ra_ >> 1) << 6) | ((ra_ & 1) << 4) | ((rb_ >> 1) << 2) | (rb_ & 1));
          size_t o = (size_t)b * ((size_t)(p.hA >> 1) * pa_w * (p.hB >> 1) * pb_w) +
                     (((size_t)ai * pa_w + aj) * (p.hB >> 1) + bi) * pb_w + bj;
          p.pool_val[o] = best;
          p.pool_idx[o] = code;
        }
      }
  }
}

}  // namespace ncnet

using namespace ncnet;

extern "C" int ncnet_l2norm_rows(const void* x, int x_is_bf16, void* y, float* inv_norm, int rows, int C,
                                 hipStream_t stream) {
  dim3 grid((unsigned)cdiv(rows, 4)), block(256);
  if (x_is_bf16)
    hipLaunchKernelGGL((l2norm_rows_kernel<bf16>), grid, block, 0, stream, (const bf16*)x, (bf16*)y, inv_norm, rows, C);
  else
    hipLaunchKernelGGL((l2norm_rows_kernel<float>), grid, block, 0, stream, (const float*)x, (bf16*)y, inv_norm, rows, C);
  return (int)hipGetLastError();
}

extern "C" int ncnet_l2norm_rows_bwd(const float* x, const float* g, const float* inv_norm, float* gx, int rows, int C,
                                     hipStream_t stream) {
  dim3 grid((unsigned)cdiv(rows, 4)), block(256);
  hipLaunchKernelGGL(l2norm_rows_bwd_kernel, grid, block, 0, stream, x, g, inv_norm, gx, rows, C);
  return (int)hipGetLastError();
}

// C[b] = A[amap[b]] . B[bmap[b]]^T ; out_bf16 selects the output dtype.
extern "C" int ncnet_corr_gemm(const void* A, const void* B, void* C, const int* amap, const int* bmap, int batch,
                               int M, int N, int K, long long sA, long long sB, long long sC, int out_bf16,
                               hipStream_t stream) {
  if (K % 8 != 0) return -1;
  GemmArgs p{};
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.C = C; p.amap = amap; p.bmap = bmap;
  p.M = M; p.N = N; p.K = K; p.sA = sA; p.sB = sB; p.sC = sC;
  p.tiles_m = cdiv(M, BM); p.tiles_n = cdiv(N, BN);
  dim3 grid((unsigned)(batch * p.tiles_m * p.tiles_n)), block(256);
  size_t lds = (size_t)(BM + BN) * BK * 2;
  if (out_bf16) hipLaunchKernelGGL((corr_gemm_kernel<true, false>), grid, block, lds, stream, p);
  else hipLaunchKernelGGL((corr_gemm_kernel<false, false>), grid, block, lds, stream, p);
  return (int)hipGetLastError();
}

// Fused correlation + 2x2x2x2 max-pool.  A rows / B rows must be in
// 2x2-block order (see ncnet_block_order_rows); hA, wA, hB, wB even.
extern "C" int ncnet_corr_gemm_pool2(const void* A, const void* B, float* pool_val, uint8_t* pool_idx, int batch,
                                     int hA, int wA, int hB, int wB, int K, long long sA, long long sB,
                                     hipStream_t stream) {
  if (K % 8 != 0 || (hA & 1) || (wA & 1) || (hB & 1) || (wB & 1)) return -1;
  GemmArgs p{};
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.C = nullptr;
  p.M = hA * wA; p.N = hB * wB; p.K = K; p.sA = sA; p.sB = sB;
  p.tiles_m = cdiv(p.M, BM); p.tiles_n = cdiv(p.N, BN);
  p.pool_ks = 2; p.pool_val = pool_val; p.pool_idx = pool_idx;
  p.hA = hA; p.wA = wA; p.hB = hB; p.wB = wB;
  dim3 grid((unsigned)(batch * p.tiles_m * p.tiles_n)), block(256);
  size_t lds = (size_t)(BM + BN) * BK * 2;
  hipLaunchKernelGGL((corr_gemm_kernel<false, true>), grid, block, lds, stream, p);
  return (int)hipGetLastError();
}
