// Volume-level kernels on 1-channel correlation volumes, viewed as matrices
// [V, R = I*J (A positions), C = K*L (B positions)] of fp32.
//
//  * stats_rows / stats_cols: max, first-argmax and (optionally) sum exp(x-max)
//    (online softmax) or the plain sum (the weak loss's 'l1' normalisation)
//    per row / column in one pass.  Used by MutualMatching
//    (lib/model.py:163-166), the weak loss (train.py:125-134) and
//    corr_to_matches (lib/point_tnf.py:32-57).
//  * mm_apply: MutualMatching output c*((c/(maxB+eps))*(c/(maxA+eps))); can
//    also emit the bf16 NC input for BOTH symmetric branches (x and its A<->B
//    swap, lib/model.py:147) so no permuted copy is ever made.
//  * mm_bwd: gradient of MutualMatching including the max-routed terms.
//  * combine: y = z1 + z2^T (the symmetric-branch un-swap + add) and its
//    backward fused with the last Conv4d's ReLU mask.
//  * softmax_max_bwd: backward of the weak-loss score (closed form) for the
//    'softmax', 'l1' and None normalisations (train.py:111-116).
//  * maxpool4d: stride = kernel = ks 4D max pool + packed 2-bit offsets.
#include "common.h"

namespace ncnet {

struct Stat { float m; float s; int idx; };

// sum kind: 0 none, 1 sum exp(x - max) (online softmax), 2 plain sum
__device__ __forceinline__ Stat stat_merge(Stat a, Stat b, int want_sum) {
  Stat r;
  bool take_b = (b.m > a.m) || (b.m == a.m && b.idx < a.idx);
  r.m = take_b ? b.m : a.m;
  r.idx = take_b ? b.idx : a.idx;
  if (want_sum == 1) {
    float sa = (a.s == 0.f) ? 0.f : a.s * __expf(a.m - r.m);
    float sb = (b.s == 0.f) ? 0.f : b.s * __expf(b.m - r.m);
    r.s = sa + sb;
  } else if (want_sum == 2) {
    r.s = a.s + b.s;
  } else r.s = 0.f;
  return r;
}

__device__ __forceinline__ Stat stat_push(Stat a, float x, int idx, int want_sum) {
  if (want_sum == 2) a.s += x;
  if (x > a.m) {
    if (want_sum == 1) a.s = a.s * __expf(a.m - x) + 1.f;
    a.m = x; a.idx = idx;
  } else if (want_sum == 1) {
    a.s += __expf(x - a.m);
  }
  return a;
}

// One wave per row.
__global__ __launch_bounds__(256) void stats_rows_kernel(const float* __restrict__ x, float* __restrict__ mx,
                                                         int* __restrict__ arg, float* __restrict__ se,
                                                         long long rows, int C, int sum_kind) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * C;
  const int ws = se != nullptr ? sum_kind : 0;
  Stat st{-INFINITY, 0.f, 0x7fffffff};
  for (int c = lane; c < C; c += 64) st = stat_push(st, xr[c], c, ws);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Stat ot;
    ot.m = __shfl_xor(st.m, o, 64);
    ot.s = __shfl_xor(st.s, o, 64);
    ot.idx = __shfl_xor(st.idx, o, 64);
    st = stat_merge(st, ot, ws);
  }
  if (lane == 0) {
    mx[row] = st.m;
    if (arg) arg[row] = st.idx;
    if (ws) se[row] = st.s;
  }
}

// Block = 64 columns x 4 row-phases over the row range of chunk (blockIdx %
// nchunk).  nchunk == 1 writes the final stats; otherwise per-chunk partials
// (pm, pi, ps: [V][nchunk][C]) merged in row order by stats_cols_merge_kernel,
// so a short-and-wide volume (InLoc: V = 1, C = 7500) still fills the chip.
__global__ __launch_bounds__(256) void stats_cols_kernel(const float* __restrict__ x, float* __restrict__ mx,
                                                         int* __restrict__ arg, float* __restrict__ se,
                                                         int R, int C, int nchunk, int rpc, int sum_kind) {
  __shared__ float sm[4][64], ss[4][64];
  __shared__ int si[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ncb = (C + 63) / 64;
  const int chunk = blockIdx.x % nchunk, rest = blockIdx.x / nchunk;
  const int v = rest / ncb, cb = rest % ncb;
  const int c = cb * 64 + lane;
  const int ws = se != nullptr ? sum_kind : 0;
  const int r0 = chunk * rpc, r1 = min(R, r0 + rpc);
  Stat st{-INFINITY, 0.f, 0x7fffffff};
  if (c < C) {
    const float* xv = x + (size_t)v * R * C + c;
    for (int r = r0 + wave; r < r1; r += 4) st = stat_push(st, xv[(size_t)r * C], r, ws);
  }
  sm[wave][lane] = st.m; ss[wave][lane] = st.s; si[wave][lane] = st.idx;
  __syncthreads();
  if (wave == 0 && c < C) {
    Stat a{sm[0][lane], ss[0][lane], si[0][lane]};
#pragma unroll
    for (int w = 1; w < 4; ++w) a = stat_merge(a, Stat{sm[w][lane], ss[w][lane], si[w][lane]}, ws);
    const size_t o = ((size_t)v * nchunk + chunk) * C + c;
    mx[o] = a.m;
    if (arg) arg[o] = a.idx;
    if (ws) se[o] = a.s;
  }
}

__global__ __launch_bounds__(256) void stats_cols_merge_kernel(const float* __restrict__ pm, const int* __restrict__ pi,
                                                               const float* __restrict__ ps, float* __restrict__ mx,
                                                               int* __restrict__ arg, float* __restrict__ se, int V,
                                                               int C, int nchunk, int sum_kind) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)V * C) return;
  const int v = (int)(e / C), c = (int)(e % C);
  const int ws = se != nullptr ? sum_kind : 0;
  Stat a{-INFINITY, 0.f, 0x7fffffff};
  for (int k = 0; k < nchunk; ++k) {
    const size_t o = ((size_t)v * nchunk + k) * C + c;
    a = stat_merge(a, Stat{pm[o], ws ? ps[o] : 0.f, pi[o]}, ws);
  }
  mx[e] = a.m;
  if (arg) arg[e] = a.idx;
  if (ws) se[e] = a.s;
}

// ---------------------------------------------------------------------------
// stats2d: row AND column stats of [V, R, C] in ONE pass over the volume
// (MutualMatching needs both maxima, the bidirectional match extraction both
// softmax stats: two strided passes before, each at ~1 TB/s -- a wave per row
// with 4-byte loads, and 64-column blocks walking rows).  Block = a 64-row x
// 256-column tile, 4 waves x 16 rows, each lane 4 consecutive columns (one
// 16-byte load per row, all 16 rows issued before any use): per-lane column
// stats over the wave's rows are merged across the 4 waves in LDS into one
// column partial per tile; each row's 256-column partial is a wave reduction.
// Partials [V][tiles][n] are merged in tile order by stats2d_merge (ties keep
// the smallest index either way).  C % 4 != 0: four scalar loads per lane and row.
// ---------------------------------------------------------------------------
// RT: 64-row sub-tiles per block (the column stats run on in registers over
// all of them), so a tall volume leaves RT x fewer column partials for the
// merge (InLoc 3200 px: 118 -> 30 per column, the merge was 40 % of stats2d).
template <int WS, bool VEC, int RT>
__global__ __launch_bounds__(256) void stats2d_tile_kernel(const float* __restrict__ x, int R, int C, int nrt, int nct,
                                                           float* __restrict__ rpm, int* __restrict__ rpi,
                                                           float* __restrict__ rps, float* __restrict__ cpm,
                                                           int* __restrict__ cpi, float* __restrict__ cps) {
  __shared__ float sm[4][256], ss[4][256];
  __shared__ int si[4][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int b = blockIdx.x;
  const int ct = b % nct; b /= nct;
  const int rt = b % nrt;
  const int v = b / nrt;
  const int c0 = ct * 256 + lane * 4;
  const bool cok = c0 < C;
  const int nk = min(4, C - c0);                         // valid columns of this lane (C % 4 != 0: scalar loads)
  const float* xv = x + (size_t)v * R * C;
  Stat col[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) col[k] = Stat{-INFINITY, 0.f, 0x7fffffff};
  for (int st = 0; st < RT; ++st) {
    const int rbase = (rt * RT + st) * 64 + wave * 16;
    if (rbase >= R) break;                                 // wave-uniform
    float4 val[16];
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int r = rbase + rr;
      if constexpr (VEC) {
        val[rr] = (cok && r < R) ? *(const float4*)(xv + (size_t)r * C + c0) : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        const float* xr = xv + (size_t)(r < R ? r : 0) * C;
        val[rr] = float4{cok && r < R ? xr[c0] : 0.f, nk > 1 && r < R ? xr[c0 + 1] : 0.f,
                         nk > 2 && r < R ? xr[c0 + 2] : 0.f, nk > 3 && r < R ? xr[c0 + 3] : 0.f};
      }
    }
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int r = rbase + rr;
      if (r >= R) break;                                   // wave-uniform
      const float e[4] = {val[rr].x, val[rr].y, val[rr].z, val[rr].w};
      Stat rs{-INFINITY, 0.f, 0x7fffffff};
      if (cok) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (VEC || k < nk) {
            col[k] = stat_push(col[k], e[k], r, WS);
            rs = stat_push(rs, e[k], c0 + k, WS);
          }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        Stat ot;
        ot.m = __shfl_xor(rs.m, o, 64);
        ot.s = __shfl_xor(rs.s, o, 64);
        ot.idx = __shfl_xor(rs.idx, o, 64);
        rs = stat_merge(rs, ot, WS);
      }
      if (lane == 0) {
        const size_t o = ((size_t)v * nct + ct) * R + r;
        rpm[o] = rs.m; rpi[o] = rs.idx;
        if (WS) rps[o] = rs.s;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) { sm[wave][lane * 4 + k] = col[k].m; ss[wave][lane * 4 + k] = col[k].s; si[wave][lane * 4 + k] = col[k].idx; }
  __syncthreads();
  const int cc = threadIdx.x;                           // one column of the tile per thread
  const int c = ct * 256 + cc;
  if (c < C) {
    Stat a{sm[0][cc], ss[0][cc], si[0][cc]};
#pragma unroll
    for (int w = 1; w < 4; ++w) a = stat_merge(a, Stat{sm[w][cc], ss[w][cc], si[w][cc]}, WS);
    const size_t o = ((size_t)v * nrt + rt) * C + c;
    cpm[o] = a.m; cpi[o] = a.idx;
    if (WS) cps[o] = a.s;
  }
}

// merge [V][nt][n] partials -> [V][n]: 4 lanes per output (tiles t = q, q + 4,
// ...), then a 2-step lane shuffle (max / first argmax exact in any order)
template <int WS>
__global__ __launch_bounds__(256) void stats2d_merge_kernel(const float* __restrict__ pm, const int* __restrict__ pi,
                                                            const float* __restrict__ ps, float* __restrict__ mx,
                                                            int* __restrict__ arg, float* __restrict__ se, int V,
                                                            int n, int nt) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) >> 2;
  const int q = threadIdx.x & 3;
  const bool live = e < (long long)V * n;                // whole quads share `live` (4 | 256)
  const int v = live ? (int)(e / n) : 0, i = live ? (int)(e - (long long)v * n) : 0;
  Stat a{-INFINITY, 0.f, 0x7fffffff};
  if (live) {
    for (int t = q; t < nt; t += 4) {
      const size_t o = ((size_t)v * nt + t) * n + i;
      a = stat_merge(a, Stat{pm[o], WS ? ps[o] : 0.f, pi[o]}, WS);
    }
  }
#pragma unroll
  for (int o = 1; o < 4; o <<= 1) {
    Stat b;
    b.m = __shfl_xor(a.m, o, 64);
    b.s = __shfl_xor(a.s, o, 64);
    b.idx = __shfl_xor(a.idx, o, 64);
    a = stat_merge(a, b, WS);
  }
  if (!live || q != 0) return;
  mx[e] = a.m;
  if (arg) arg[e] = a.idx;
  if (WS && se) se[e] = a.s;
}

// ---------------------------------------------------------------------------
// match_candidates: the bidirectional match candidates of one volume
// [R = fs1*fs2 A cells, C = fs3*fs4 B cells] from its row / column stats, in
// one launch (lib/point_tnf.py:12-80 + eval_inloc.py:180-189): entry n < C is
// B cell n with its best A cell (column stats), entry C + m is A cell m with
// its best B cell (row stats); the 2-bit relocalization offsets of the matched
// cell are decoded (packed codes, k = 2), the cells mapped onto the [0, 1]
// linspace grids at full resolution and recentred to pixel centres.
// Outputs: m [N][5] = (xA, yA, xB, yB, score), sc [N] score, key [N] int64 =
// ((jA HA + iA) WB + jB) HB + iB (the lexicographic de-duplication key).
// Arithmetic mirrors the PyTorch ops it replaces (linspace's two-sided
// formula, recentre as mul -> div -> add with no contraction).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float lin01(int i, int n) {       // torch.linspace(0, 1, n)[i]
  const float step = __fdiv_rn(1.f, (float)(n - 1));
  return i < n / 2 ? __fmul_rn(step, (float)i) : __fsub_rn(1.f, __fmul_rn(step, (float)(n - i - 1)));
}
__device__ __forceinline__ float recentre(float y, int n) {
  return __fadd_rn(__fdiv_rn(__fmul_rn(y, (float)(n - 1)), (float)n), (float)(0.5 / (double)n));
}
__global__ __launch_bounds__(256) void match_candidates_kernel(const float* __restrict__ cmx, const float* __restrict__ cse,
                                                               const int* __restrict__ carg, const float* __restrict__ rmx,
                                                               const float* __restrict__ rse, const int* __restrict__ rarg,
                                                               const uint8_t* __restrict__ code, int fs1, int fs2, int fs3,
                                                               int fs4, int k, float* __restrict__ m, float* __restrict__ sc,
                                                               long long* __restrict__ key) {
  const int R = fs1 * fs2, C = fs3 * fs4;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= R + C) return;
  int a, b;
  float s;
  if (e < C) { b = e; a = carg[e]; s = cse ? __fdiv_rn(1.f, cse[e]) : cmx[e]; }
  else { a = e - C; b = rarg[a]; s = rse ? __fdiv_rn(1.f, rse[a]) : rmx[a]; }
  a = min(max(a, 0), R - 1);        // an all-NaN line leaves the argmax sentinel: keep the code read in range
  b = min(max(b, 0), C - 1);
  int iA = a / fs2, jA = a - (a / fs2) * fs2, iB = b / fs4, jB = b - (b / fs4) * fs4;
  if (code) {
    const int c = code[(size_t)a * C + b];
    iA = iA * k + ((c >> 6) & 3); jA = jA * k + ((c >> 4) & 3);
    iB = iB * k + ((c >> 2) & 3); jB = jB * k + (c & 3);
  }   // no offsets: the indices stay at pooled resolution on the k-times grid (point_tnf.corr_to_matches)
  const int HA = fs1 * k, WA = fs2 * k, HB = fs3 * k, WB = fs4 * k;
  m[(size_t)e * 5 + 0] = recentre(lin01(jA, WA), WA);
  m[(size_t)e * 5 + 1] = recentre(lin01(iA, HA), HA);
  m[(size_t)e * 5 + 2] = recentre(lin01(jB, WB), WB);
  m[(size_t)e * 5 + 3] = recentre(lin01(iB, HB), HB);
  m[(size_t)e * 5 + 4] = s;
  sc[e] = s;
  key[e] = (((long long)jA * HA + iA) * WB + jB) * HB + iB;
}

// ---------------------------------------------------------------------------
// MutualMatching apply, 64x64 tiles.  rmax: [V,R] (max over B for each A row),
// cmax: [V,C] (max over A for each B column).
//   out_f32 [V,R,C] (optional), out_x bf16 [V,R,C] at volume slot v (optional),
//   out_xt bf16 [V,C,R] at volume slot v (optional; A<->B swapped copy).
// F16: out_x / out_xt are IEEE half (the half_precision NC input).
// PAD (training NC input, csrc/conv1x.hip layout): out_x / out_xt are the
// zero-padded bf16 planes of conv1x16 / wgrad1x16 instead -- out_x [V*R][PPL]
// (plane (v, r) = the [K2, L2] row r), out_xt [V*C][PPL] (plane (v, c) = the
// [I2, J2] column c of the swapped branch) -- halos included: block (tr, tc)
// zeroes chunk tc of the halo of its 64 row planes and chunk tr of the halo of
// its 64 column planes, so no separate fill and pad passes are needed.
struct PadGeom { int K2, L2, I2, J2, P, LP, PPL; };

// position of halo element h of a padded [K2, L2] plane (rows of LP, P-wide
// margins, PPL - (K2 + 2P) LP tail elements)
__device__ __forceinline__ int halo_pos(int h, int K2, int L2, int P, int LP) {
  const int top = P * LP;
  if (h < top) return h;
  h -= top;
  const int mid = K2 * 2 * P;
  if (h < mid) {
    const int row = h / (2 * P), side = h - row * 2 * P;
    return (row + P) * LP + (side < P ? side : L2 + side);
  }
  return (K2 + P) * LP + (h - mid);   // bottom margin rows, then the tail
}

template <bool F16, bool PAD>
__global__ __launch_bounds__(256) void mm_apply_kernel(const float* __restrict__ c, const float* __restrict__ rmax,
                                                       const float* __restrict__ cmax, float* __restrict__ out_f32,
                                                       uint16_t* __restrict__ out_x, uint16_t* __restrict__ out_xt,
                                                       int R, int C, float eps, PadGeom pg) {
  __shared__ float tile[64][65];
  const int ntr = (R + 63) / 64, ntc = (C + 63) / 64;
  int b = blockIdx.x;
  const int tc = b % ntc; b /= ntc;
  const int tr = b % ntr; const int v = b / ntr;
  const int r0 = tr * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const size_t vb = (size_t)v * R * C;
  const int cc = c0 + tx;
  const float cm = (cc < C) ? cmax[(size_t)v * C + cc] + eps : 1.f;
  // padded position of this lane's column cc in a row plane (PAD)
  const int pcol = PAD ? (cc / pg.L2 + pg.P) * pg.LP + cc % pg.L2 + pg.P : 0;
  for (int rr = ty; rr < 64; rr += 4) {
    int r = r0 + rr;
    float o = 0.f;
    if (r < R && cc < C) {
      float x = c[vb + (size_t)r * C + cc];
      float ra = rmax[(size_t)v * R + r] + eps;
      o = x * ((x / ra) * (x / cm));
      if (out_f32) out_f32[vb + (size_t)r * C + cc] = o;
      if (out_x) {
        if constexpr (PAD) out_x[((size_t)v * R + r) * pg.PPL + pcol] = f2s16<F16>(o);
        else out_x[vb + (size_t)r * C + cc] = f2s16<F16>(o);
      }
    }
    tile[rr][tx] = o;
  }
  if (out_xt) {
    __syncthreads();
    // write transposed: row = c, col = r
    const int rw = r0 + tx;
    const int prow = PAD ? (rw / pg.J2 + pg.P) * pg.LP + rw % pg.J2 + pg.P : 0;
    for (int cl = ty; cl < 64; cl += 4) {
      int ccol = c0 + cl;
      if (ccol < C && rw < R) {
        if constexpr (PAD) out_xt[((size_t)v * C + ccol) * pg.PPL + prow] = f2s16<F16>(tile[tx][cl]);
        else out_xt[vb + (size_t)ccol * R + rw] = f2s16<F16>(tile[tx][cl]);
      }
    }
  }
  if constexpr (PAD) {
    const uint16_t zero = 0;
    if (out_x) {   // chunk tc of the halos of row planes r0 .. r0 + 63
      const int nh = pg.PPL - pg.K2 * pg.L2, ch = (nh + ntc - 1) / ntc;
      const int h0 = tc * ch, h1 = min(nh, h0 + ch);
      for (int e = threadIdx.x; e < 64 * (h1 - h0); e += 256) {
        const int rr = e / (h1 - h0), h = h0 + e - rr * (h1 - h0);
        if (r0 + rr < R) out_x[((size_t)v * R + r0 + rr) * pg.PPL + halo_pos(h, pg.K2, pg.L2, pg.P, pg.LP)] = zero;
      }
    }
    if (out_xt) {  // chunk tr of the halos of column planes c0 .. c0 + 63
      const int nh = pg.PPL - pg.I2 * pg.J2, ch = (nh + ntr - 1) / ntr;
      const int h0 = tr * ch, h1 = min(nh, h0 + ch);
      for (int e = threadIdx.x; e < 64 * (h1 - h0); e += 256) {
        const int cl = e / (h1 - h0), h = h0 + e - cl * (h1 - h0);
        if (c0 + cl < C) out_xt[((size_t)v * C + c0 + cl) * pg.PPL + halo_pos(h, pg.I2, pg.J2, pg.P, pg.LP)] = zero;
      }
    }
  }
}

// Row / column sums of g * out for the MutualMatching backward (out recomputed).
__global__ __launch_bounds__(256) void mm_bwd_rowsum_kernel(const float* __restrict__ c, const float* __restrict__ g,
                                                            const float* __restrict__ rmax, const float* __restrict__ cmax,
                                                            float* __restrict__ rsum, long long rows, int R, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int v = (int)(row / R);
  const float ra = rmax[row] + eps;
  const float* cr = c + row * C;
  const float* gr = g + row * C;
  const float* cmv = cmax + (size_t)v * C;
  float s = 0.f;
  for (int k = lane; k < C; k += 64) {
    float x = cr[k];
    s += gr[k] * (x * ((x / ra) * (x / (cmv[k] + eps))));
  }
  s = wave_sum(s);
  if (lane == 0) rsum[row] = s;
}

__global__ __launch_bounds__(256) void mm_bwd_colsum_kernel(const float* __restrict__ c, const float* __restrict__ g,
                                                            const float* __restrict__ rmax, const float* __restrict__ cmax,
                                                            float* __restrict__ csum, int R, int C, float eps) {
  __shared__ float sh[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ncb = (C + 63) / 64;
  const int v = blockIdx.x / ncb, cb = blockIdx.x % ncb;
  const int k = cb * 64 + lane;
  float s = 0.f;
  if (k < C) {
    const float cm = cmax[(size_t)v * C + k] + eps;
    const size_t vb = (size_t)v * R * C;
    for (int r = wave; r < R; r += 4) {
      float x = c[vb + (size_t)r * C + k];
      float ra = rmax[(size_t)v * R + r] + eps;
      s += g[vb + (size_t)r * C + k] * (x * ((x / ra) * (x / cm)));
    }
  }
  sh[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && k < C) csum[(size_t)v * C + k] = sh[0][lane] + sh[1][lane] + sh[2][lane] + sh[3][lane];
}

// Both sums of the MutualMatching backward in ONE pass over (c, g) (the
// separate row pass and the 64-column-block column pass read both volumes
// twice; the column pass, V * C / 64 blocks walking rows, was also a long
// tail on the critical path of the pipelined step).  Same 64 x 256 tiling as
// stats2d: row partials by wave reduction, column partials merged in LDS over
// the 4 waves; partials summed in tile order by sum_partials_kernel.
template <bool VEC>
__global__ __launch_bounds__(256) void mm_bwd_sums2d_kernel(const float* __restrict__ c, const float* __restrict__ g,
                                                            const float* __restrict__ rmax, const float* __restrict__ cmax,
                                                            int R, int C, int nrt, int nct, float* __restrict__ rp,
                                                            float* __restrict__ cp, float eps) {
  __shared__ float sh[4][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int b = blockIdx.x;
  const int ct = b % nct; b /= nct;
  const int rt = b % nrt;
  const int v = b / nrt;
  const int c0 = ct * 256 + lane * 4;
  const int nk = c0 < C ? min(4, C - c0) : 0;
  const int rbase = rt * 64 + wave * 16;
  const size_t vb = (size_t)v * R * C;
  float cm[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) cm[k] = k < nk ? cmax[(size_t)v * C + c0 + k] + eps : 1.f;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int rr = 0; rr < 16; ++rr) {
    const int r = rbase + rr;
    if (r >= R) break;                                   // wave-uniform
    const float ra = rmax[(size_t)v * R + r] + eps;
    const float* cr = c + vb + (size_t)r * C + c0;
    const float* gr = g + vb + (size_t)r * C + c0;
    float xv[4], gv[4];
    if constexpr (VEC) {
      const float4 x4 = nk ? *(const float4*)cr : float4{0.f, 0.f, 0.f, 0.f};
      const float4 g4 = nk ? *(const float4*)gr : float4{0.f, 0.f, 0.f, 0.f};
      xv[0] = x4.x; xv[1] = x4.y; xv[2] = x4.z; xv[3] = x4.w;
      gv[0] = g4.x; gv[1] = g4.y; gv[2] = g4.z; gv[3] = g4.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) { xv[k] = k < nk ? cr[k] : 0.f; gv[k] = k < nk ? gr[k] : 0.f; }
    }
    float rs = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = xv[k];
      const float t = k < nk ? gv[k] * (x * ((x / ra) * (x / cm[k]))) : 0.f;
      cs[k] += t;
      rs += t;
    }
    rs = wave_sum(rs);
    if (lane == 0) rp[((size_t)v * nct + ct) * R + r] = rs;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) sh[wave][lane * 4 + k] = cs[k];
  __syncthreads();
  const int cc = threadIdx.x, col = ct * 256 + cc;
  if (col < C) cp[((size_t)v * nrt + rt) * C + col] = sh[0][cc] + sh[1][cc] + sh[2][cc] + sh[3][cc];
}

// out [V][n] = sum over t of p [V][nt][n] (in t order)
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ p, float* __restrict__ out, int V,
                                                           int n, int nt) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)V * n) return;
  const int v = (int)(e / n), i = (int)(e - (long long)v * n);
  float s = 0.f;
  for (int t = 0; t < nt; ++t) s += p[((size_t)v * nt + t) * n + i];
  out[e] = s;
}

__global__ __launch_bounds__(256) void mm_bwd_apply_kernel(const float* __restrict__ c, const float* __restrict__ g,
                                                           const float* __restrict__ rmax, const int* __restrict__ rarg,
                                                           const float* __restrict__ rsum,
                                                           const float* __restrict__ cmax, const int* __restrict__ carg,
                                                           const float* __restrict__ csum, float* __restrict__ gc,
                                                           long long total, int R, int C, float eps) {
  long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int k = (int)(e % C);
  const long long row = e / C;     // v*R + r
  const int r = (int)(row % R);
  const int v = (int)(row / R);
  const float x = c[e];
  const float ra = rmax[row] + eps;
  const float cb = cmax[(size_t)v * C + k] + eps;
  float gr = g[e] * (3.f * x * x / (ra * cb));
  if (rarg[row] == k) gr -= rsum[row] / ra;
  if (carg[(size_t)v * C + k] == r) gr -= csum[(size_t)v * C + k] / cb;
  gc[e] = gr;
}

// ---------------------------------------------------------------------------
// combine: y[v] = z[v] + z[v+Vh]^T  (z second half stored as [C, R])
__global__ __launch_bounds__(256) void combine_fwd_kernel(const float* __restrict__ z, float* __restrict__ y,
                                                          int Vh, int R, int C) {
  __shared__ float tile[64][65];
  const int ntr = (R + 63) / 64, ntc = (C + 63) / 64;
  int b = blockIdx.x;
  const int tc = b % ntc; b /= ntc;
  const int tr = b % ntr; const int v = b / ntr;
  const int r0 = tr * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const float* z2 = z + (size_t)(v + Vh) * R * C;   // [C][R]
  // load z2 tile rows c0.., cols r0.. coalesced
  for (int cl = ty; cl < 64; cl += 4) {
    int cc = c0 + cl, rr = r0 + tx;
    tile[cl][tx] = (cc < C && rr < R) ? z2[(size_t)cc * R + rr] : 0.f;
  }
  __syncthreads();
  const float* z1 = z + (size_t)v * R * C;
  float* yv = y + (size_t)v * R * C;
  for (int rl = ty; rl < 64; rl += 4) {
    int rr = r0 + rl, cc = c0 + tx;
    if (rr < R && cc < C) yv[(size_t)rr * C + cc] = z1[(size_t)rr * C + cc] + tile[tx][rl];
  }
}

// gz[v] = g[v] * (z[v] > 0), gz[v+Vh] = g[v]^T * (z[v+Vh] > 0) as bf16; with
// gzl (bf16x3 training): also the residual gzl = bf16(value - gz).
__device__ __forceinline__ void put_split(bf16* __restrict__ gz, bf16* __restrict__ gzl, size_t o, float x) {
  const bf16 h = f2bf(x);
  gz[o] = h;
  if (gzl) gzl[o] = f2bf(x - bf2f(h));
}

__global__ __launch_bounds__(256) void combine_bwd_kernel(const float* __restrict__ g, const float* __restrict__ z,
                                                          bf16* __restrict__ gz, bf16* __restrict__ gzl, int Vh, int R,
                                                          int C) {
  __shared__ float tile[64][65];
  const int ntr = (R + 63) / 64, ntc = (C + 63) / 64;
  int b = blockIdx.x;
  const int tc = b % ntc; b /= ntc;
  const int tr = b % ntr; const int v = b / ntr;
  const int r0 = tr * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const size_t vb1 = (size_t)v * R * C, vb2 = (size_t)(v + Vh) * R * C;
  for (int rl = ty; rl < 64; rl += 4) {
    int rr = r0 + rl, cc = c0 + tx;
    float gv = 0.f;
    if (rr < R && cc < C) {
      gv = g[vb1 + (size_t)rr * C + cc];
      put_split(gz, gzl, vb1 + (size_t)rr * C + cc, z[vb1 + (size_t)rr * C + cc] > 0.f ? gv : 0.f);
    }
    tile[rl][tx] = gv;
  }
  __syncthreads();
  for (int cl = ty; cl < 64; cl += 4) {
    int cc = c0 + cl, rr = r0 + tx;
    if (cc < C && rr < R) {
      size_t o = vb2 + (size_t)cc * R + rr;
      put_split(gz, gzl, o, z[o] > 0.f ? tile[tx][cl] : 0.f);
    }
  }
}

// ---------------------------------------------------------------------------
// Weak-loss score backward (softmax normalisation):
//   s = max softmax = 1/sumexp; ds/dx_j = s (delta_{j,argmax} - softmax_j)
// g = wr[v] * ds_row/dx + wc[v] * ds_col/dx
// norm 1 'softmax': s = 1 / sum exp(x - max), ds/dx_j = s (delta_{j,argmax} - softmax_j)
// norm 2 'l1':      s = max / (sum + eps),     ds/dx_j = delta_{j,argmax} / D - max / D^2
// norm 0 None:      s = max,                   ds/dx_j = delta_{j,argmax}
// (rse / cse hold the row / column sum exp for 'softmax', the plain sum for 'l1')
__global__ __launch_bounds__(256) void softmax_max_bwd_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ rmax, const int* __restrict__ rarg,
                                                              const float* __restrict__ rse,
                                                              const float* __restrict__ cmax, const int* __restrict__ carg,
                                                              const float* __restrict__ cse,
                                                              const float* __restrict__ wr, const float* __restrict__ wc,
                                                              float* __restrict__ gx, long long total, int R, int C,
                                                              int norm, float eps, const float* __restrict__ gscale) {
  long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int k = (int)(e % C);
  const long long row = e / C;
  const int r = (int)(row % R);
  const int v = (int)(row / R);
  const size_t ci = (size_t)v * C + k;
  const float dr = (rarg[row] == k) ? 1.f : 0.f, dc = (carg[ci] == r) ? 1.f : 0.f;
  float gr;
  if (norm == 1) {
    const float xv = x[e];
    const float sr = 1.f / rse[row];
    const float sc = 1.f / cse[ci];
    const float pr = __expf(xv - rmax[row]) * sr;
    const float pc = __expf(xv - cmax[ci]) * sc;
    gr = wr[v] * sr * (dr - pr) + wc[v] * sc * (dc - pc);
  } else if (norm == 2) {
    const float ir = 1.f / (rse[row] + eps), ic = 1.f / (cse[ci] + eps);
    gr = wr[v] * ir * (dr - rmax[row] * ir) + wc[v] * ic * (dc - cmax[ci] * ic);
  } else {
    gr = wr[v] * dr + wc[v] * dc;
  }
  // gscale: the incoming gradient of the scalar score (autograd's g), read by
  // every lane from one address (no separate volume-sized multiply pass)
  gx[e] = gscale ? gr * gscale[0] : gr;
}

// Weak-loss score value from the row / column statistics, in one launch:
//   out = sum_{v,r} wr[v] s(rmax, rse) + sum_{v,c} wc[v] s(cmax, cse)
// with s = 1 / sum (norm 1 'softmax'), max / (sum + eps) (2 'l1'), max (0).
// One 1024-thread workgroup (V (R + C) is ~40 K terms at the training shape);
// replaces the reciprocal / multiply / two reductions / add of the PyTorch form.
__global__ __launch_bounds__(1024) void score_sum_kernel(const float* __restrict__ rmax, const float* __restrict__ rse,
                                                         const float* __restrict__ cmax, const float* __restrict__ cse,
                                                         const float* __restrict__ wr, const float* __restrict__ wc,
                                                         int V, int R, int C, int norm, float eps,
                                                         float* __restrict__ out) {
  __shared__ float part[16];
  float acc = 0.f;
  const long long nr = (long long)V * R, nc = (long long)V * C;
  for (long long e = threadIdx.x; e < nr + nc; e += 1024) {
    const bool row = e < nr;
    const long long i = row ? e : e - nr;
    const float mx = row ? rmax[i] : cmax[i];
    const float sm = row ? rse[i] : cse[i];
    const float w = row ? wr[i / R] : wc[i / C];
    const float sc = norm == 1 ? 1.f / sm : norm == 2 ? mx / (sm + eps) : mx;
    acc += w * sc;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < 16 ? part[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) out[0] = t;
  }
}

// ---------------------------------------------------------------------------
// 4D max pool, stride = kernel = ks (<= 4).  idx code: di<<6 | dj<<4 | dk<<2 | dl
template <typename T>
__global__ __launch_bounds__(256) void maxpool4d_kernel(const T* __restrict__ x, float* __restrict__ y,
                                                        uint8_t* __restrict__ code, int V, int I, int J, int K,
                                                        int L, int ks) {
  const int Io = I / ks, Jo = J / ks, Ko = K / ks, Lo = L / ks;
  long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  long long total = (long long)V * Io * Jo * Ko * Lo;
  if (e >= total) return;
  long long t = e;
  const int lo = (int)(t % Lo); t /= Lo;
  const int ko = (int)(t % Ko); t /= Ko;
  const int jo = (int)(t % Jo); t /= Jo;
  const int io = (int)(t % Io); const int v = (int)(t / Io);
  float best = -INFINITY;
  int bc = 0;
  for (int a = 0; a < ks; ++a)
    for (int b = 0; b < ks; ++b)
      for (int c = 0; c < ks; ++c)
        for (int d = 0; d < ks; ++d) {
          size_t o = ((((size_t)v * I + io * ks + a) * J + jo * ks + b) * K + ko * ks + c) * (size_t)L + lo * ks + d;
          float val = (float)x[o];
          if (val > best) { best = val; bc = (a << 6) | (b << 4) | (c << 2) | d; }
        }
  y[e] = best;
  code[e] = (uint8_t)bc;
}

// [V,R,C] -> [V,C,R] (bf16 or fp32), 64x64 tiles
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ x, T* __restrict__ y, int R, int C) {
  __shared__ T tile[64][65];
  const int ntr = (R + 63) / 64, ntc = (C + 63) / 64;
  int b = blockIdx.x;
  const int tc = b % ntc; b /= ntc;
  const int tr = b % ntr; const int v = b / ntr;
  const int r0 = tr * 64, c0 = tc * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const size_t vb = (size_t)v * R * C;
  for (int rl = ty; rl < 64; rl += 4) {
    int rr = r0 + rl, cc = c0 + tx;
    if (rr < R && cc < C) tile[rl][tx] = x[vb + (size_t)rr * C + cc];
  }
  __syncthreads();
  for (int cl = ty; cl < 64; cl += 4) {
    int cc = c0 + cl, rr = r0 + tx;
    if (cc < C && rr < R) y[vb + (size_t)cc * R + rr] = tile[tx][cl];
  }
}

}  // namespace ncnet

using namespace ncnet;

extern "C" int ncnet_pad_geom(int K, int L, int KS, int* lp, int* ppl);   // csrc/conv1x.hip
static unsigned tiles64(int V, int R, int C) { return (unsigned)((long long)V * cdiv(R, 64) * cdiv(C, 64)); }

// sum_kind: 1 sum exp(x - max), 2 plain sum (only when se != nullptr)
extern "C" int ncnet_stats_rows(const float* x, float* mx, int* arg, float* se, long long rows, int C, int sum_kind,
                                hipStream_t s) {
  hipLaunchKernelGGL(stats_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, mx, arg, se, rows, C,
                     sum_kind);
  return (int)hipGetLastError();
}
// work: nullptr (nchunk = 1) or 3 * V * nchunk * C floats of partials.
extern "C" int ncnet_stats_cols(const float* x, float* mx, int* arg, float* se, int V, int R, int C, float* work,
                                int nchunk, int sum_kind, hipStream_t s) {
  if (nchunk <= 1 || work == nullptr) {
    hipLaunchKernelGGL(stats_cols_kernel, dim3((unsigned)(V * cdiv(C, 64))), dim3(256), 0, s, x, mx, arg, se, R, C, 1, R, sum_kind);
    return (int)hipGetLastError();
  }
  const size_t n = (size_t)V * nchunk * C;
  float* pm = work; int* pi = (int*)(work + n); float* ps = work + 2 * n;
  const int rpc = cdiv(R, nchunk);
  hipLaunchKernelGGL(stats_cols_kernel, dim3((unsigned)(V * cdiv(C, 64) * nchunk)), dim3(256), 0, s, x, pm, pi,
                     se ? ps : nullptr, R, C, nchunk, rpc, sum_kind);
  hipLaunchKernelGGL(stats_cols_merge_kernel, dim3((unsigned)cdiv(V * C, 256)), dim3(256), 0, s, pm, pi,
                     se ? ps : nullptr, mx, arg, se, V, C, nchunk, sum_kind);
  return (int)hipGetLastError();
}
// stats2d: work = 3 * V * (nct * R + nrt * C) floats of partials (nrt = ceil(R / 64), nct = ceil(C / 256)).
// sum_kind 0: max / argmax only (rse, cse ignored).
extern "C" int ncnet_stats2d(const float* x, float* rmx, int* rarg, float* rse, float* cmx, int* carg, float* cse,
                             int V, int R, int C, float* work, int sum_kind, hipStream_t s) {
  const bool vec = C % 4 == 0;   // 16-byte rows: one float4 per lane and row; else four scalar loads
  // tall volumes: 64 rt-row blocks (rt x fewer column partials to merge;
  // tuning s2d_rt); the work buffer is sized for 64-row blocks (the bound)
  const int rt = R >= 1024 ? (tuning().s2d_rt >= 4 ? 4 : tuning().s2d_rt == 2 ? 2 : 1) : 1;
  const int nrt = cdiv(R, 64 * rt), nct = cdiv(C, 256);
  const size_t nr = (size_t)V * nct * R, nc = (size_t)V * nrt * C;
  float* rpm = work; int* rpi = (int*)(work + nr); float* rps = work + 2 * nr;
  float* cpm = work + 3 * nr; int* cpi = (int*)(cpm + nc); float* cps = cpm + 2 * nc;
  const dim3 grid((unsigned)((size_t)V * nrt * nct)), blk(256);
#define S2D_TILE(WSV, VECV) do { \
    if (rt == 4) hipLaunchKernelGGL((stats2d_tile_kernel<WSV, VECV, 4>), grid, blk, 0, s, x, R, C, nrt, nct, rpm, rpi, rps, cpm, cpi, cps); \
    else if (rt == 2) hipLaunchKernelGGL((stats2d_tile_kernel<WSV, VECV, 2>), grid, blk, 0, s, x, R, C, nrt, nct, rpm, rpi, rps, cpm, cpi, cps); \
    else hipLaunchKernelGGL((stats2d_tile_kernel<WSV, VECV, 1>), grid, blk, 0, s, x, R, C, nrt, nct, rpm, rpi, rps, cpm, cpi, cps); \
  } while (0)
#define S2D(WSV) do { \
    if (vec) S2D_TILE(WSV, true); \
    else S2D_TILE(WSV, false); \
    hipLaunchKernelGGL(stats2d_merge_kernel<WSV>, dim3((unsigned)cdiv(4 * V * R, 256)), blk, 0, s, rpm, rpi, rps, rmx, rarg, rse, V, R, nct); \
    hipLaunchKernelGGL(stats2d_merge_kernel<WSV>, dim3((unsigned)cdiv(4 * V * C, 256)), blk, 0, s, cpm, cpi, cps, cmx, carg, cse, V, C, nrt); \
  } while (0)
  if (sum_kind == 1) S2D(1); else if (sum_kind == 2) S2D(2); else S2D(0);
#undef S2D
#undef S2D_TILE
  return (int)hipGetLastError();
}
extern "C" int ncnet_match_candidates(const float* cmx, const float* cse, const int* carg, const float* rmx,
                                      const float* rse, const int* rarg, const uint8_t* code, int fs1, int fs2, int fs3,
                                      int fs4, int k, float* m, float* sc, long long* key, hipStream_t s) {
  const int n = fs1 * fs2 + fs3 * fs4;
  hipLaunchKernelGGL(match_candidates_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, cmx, cse, carg, rmx, rse,
                     rarg, code, fs1, fs2, fs3, fs4, k, m, sc, key);
  return (int)hipGetLastError();
}
// pad_ks > 0: out_x / out_xt are padded bf16 planes for kernel size pad_ks (I2 x J2 = R, K2 x L2 = C)
extern "C" int ncnet_mm_apply(const float* c, const float* rmax, const float* cmax, float* out_f32, void* out_x,
                              void* out_xt, int V, int R, int C, float eps, int x_f16, int pad_ks, int I2, int J2,
                              int K2, int L2, hipStream_t s) {
  PadGeom pg = {K2, L2, I2, J2, 0, 0, 0};
  if (pad_ks > 0) {
    if (x_f16 || I2 * J2 != R || K2 * L2 != C || I2 != K2 || J2 != L2) return -1;
    pg.P = pad_ks / 2;
    ncnet_pad_geom(K2, L2, pad_ks, &pg.LP, &pg.PPL);
    hipLaunchKernelGGL((mm_apply_kernel<false, true>), dim3(tiles64(V, R, C)), dim3(256), 0, s, c, rmax, cmax, out_f32,
                       (uint16_t*)out_x, (uint16_t*)out_xt, R, C, eps, pg);
  } else if (x_f16)
    hipLaunchKernelGGL((mm_apply_kernel<true, false>), dim3(tiles64(V, R, C)), dim3(256), 0, s, c, rmax, cmax, out_f32,
                       (uint16_t*)out_x, (uint16_t*)out_xt, R, C, eps, pg);
  else
    hipLaunchKernelGGL((mm_apply_kernel<false, false>), dim3(tiles64(V, R, C)), dim3(256), 0, s, c, rmax, cmax, out_f32,
                       (uint16_t*)out_x, (uint16_t*)out_xt, R, C, eps, pg);
  return (int)hipGetLastError();
}
// work: nullptr (separate row / column passes) or V * (ceil(C/256) * R + ceil(R/64) * C) floats (one pass)
extern "C" int ncnet_mm_bwd(const float* c, const float* g, const float* rmax, const int* rarg, const float* cmax,
                            const int* carg, float* rsum, float* csum, float* gc, int V, int R, int C, float eps,
                            float* work, hipStream_t s) {
  long long rows = (long long)V * R;
  if (work) {
    const int nrt = cdiv(R, 64), nct = cdiv(C, 256);
    float* rp = work;
    float* cp = work + (size_t)V * nct * R;
    const dim3 grid((unsigned)((size_t)V * nrt * nct));
    if (C % 4 == 0)
      hipLaunchKernelGGL((mm_bwd_sums2d_kernel<true>), grid, dim3(256), 0, s, c, g, rmax, cmax, R, C, nrt, nct, rp, cp, eps);
    else
      hipLaunchKernelGGL((mm_bwd_sums2d_kernel<false>), grid, dim3(256), 0, s, c, g, rmax, cmax, R, C, nrt, nct, rp, cp, eps);
    hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)cdiv(V * R, 256)), dim3(256), 0, s, rp, rsum, V, R, nct);
    hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)cdiv(V * C, 256)), dim3(256), 0, s, cp, csum, V, C, nrt);
  } else {
    hipLaunchKernelGGL(mm_bwd_rowsum_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, c, g, rmax, cmax, rsum,
                       rows, R, C, eps);
    hipLaunchKernelGGL(mm_bwd_colsum_kernel, dim3((unsigned)(V * cdiv(C, 64))), dim3(256), 0, s, c, g, rmax, cmax, csum,
                       R, C, eps);
  }
  long long total = rows * C;
  hipLaunchKernelGGL(mm_bwd_apply_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, c, g, rmax, rarg,
                     rsum, cmax, carg, csum, gc, total, R, C, eps);
  return (int)hipGetLastError();
}
extern "C" int ncnet_combine_fwd(const float* z, float* y, int Vh, int R, int C, hipStream_t s) {
  hipLaunchKernelGGL(combine_fwd_kernel, dim3(tiles64(Vh, R, C)), dim3(256), 0, s, z, y, Vh, R, C);
  return (int)hipGetLastError();
}
extern "C" int ncnet_combine_bwd(const float* g, const float* z, void* gz, void* gzl, int Vh, int R, int C,
                                 hipStream_t s) {
  hipLaunchKernelGGL(combine_bwd_kernel, dim3(tiles64(Vh, R, C)), dim3(256), 0, s, g, z, (bf16*)gz, (bf16*)gzl, Vh, R,
                     C);
  return (int)hipGetLastError();
}
extern "C" int ncnet_softmax_max_bwd(const float* x, const float* rmax, const int* rarg, const float* rse,
                                     const float* cmax, const int* carg, const float* cse, const float* wr,
                                     const float* wc, float* gx, int V, int R, int C, int norm, float eps,
                                     const float* gscale, hipStream_t s) {
  long long total = (long long)V * R * C;
  hipLaunchKernelGGL(softmax_max_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, rmax, rarg, rse,
                     cmax, carg, cse, wr, wc, gx, total, R, C, norm, eps, gscale);
  return (int)hipGetLastError();
}
extern "C" int ncnet_score_sum(const float* rmax, const float* rse, const float* cmax, const float* cse, const float* wr,
                               const float* wc, int V, int R, int C, int norm, float eps, float* out, hipStream_t s) {
  hipLaunchKernelGGL(score_sum_kernel, dim3(1), dim3(1024), 0, s, rmax, rse, cmax, cse, wr, wc, V, R, C, norm, eps, out);
  return (int)hipGetLastError();
}
extern "C" int ncnet_maxpool4d(const void* x, int x_is_bf16, float* y, uint8_t* code, int V, int I, int J, int K,
                               int L, int ks, hipStream_t s) {
  if (ks > 4 || ks < 1) return -1;
  long long total = (long long)V * (I / ks) * (J / ks) * (K / ks) * (L / ks);
  dim3 grid((unsigned)((total + 255) / 256));
  if (x_is_bf16) hipLaunchKernelGGL((maxpool4d_kernel<bf16>), grid, dim3(256), 0, s, (const bf16*)x, y, code, V, I, J, K, L, ks);
  else hipLaunchKernelGGL((maxpool4d_kernel<float>), grid, dim3(256), 0, s, (const float*)x, y, code, V, I, J, K, L, ks);
  return (int)hipGetLastError();
}
extern "C" int ncnet_transpose(const void* x, void* y, int elem_bytes, int V, int R, int C, hipStream_t s) {
  dim3 grid(tiles64(V, R, C));
  if (elem_bytes == 2) hipLaunchKernelGGL((transpose_kernel<bf16>), grid, dim3(256), 0, s, (const bf16*)x, (bf16*)y, R, C);
  else if (elem_bytes == 4) hipLaunchKernelGGL((transpose_kernel<float>), grid, dim3(256), 0, s, (const float*)x, (float*)y, R, C);
  else return -1;
  return (int)hipGetLastError();
}
