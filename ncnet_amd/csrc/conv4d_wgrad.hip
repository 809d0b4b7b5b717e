// Conv4d weight gradients on gfx950 MFMA.
//
//   dW[co,ci,di,dj,dk,dl] = sum_{v,i,j,k,l} X[v,i+di-P,j+dj-P,k+dk-P,l+dl-P,ci] * G[v,i,j,k,l,co]
//
// G is the gradient w.r.t. the conv's pre-activation (the ReLU mask is applied
// by the producer).  The reduction runs over ~25M voxels per step, so the grid
// is (KS*KS plane offsets (di,dj)) x NG groups; each workgroup keeps the
// (di,dj) slice of dW in accumulators while it walks its group's output tiles
// and writes one fp32 partial per group (summed by a tiny reduction).
//
//   wgrad16v2 (per (di,dj) plane offset, or plane-only for the ij-encoded
//     1-channel layers): per 32-voxel K chunk, the G^T operand is read once
//     (ds_read_b64_tr_b16) and reused by every tap; the X^T operand is the
//     staged plane read at the tap's shift, also through the transposing read
//     (each lane of the 16-lane group addresses its own voxel row, so arbitrary
//     shifts cost nothing).  Bias gradient is one extra MFMA with A = ones in
//     the (P,P) workgroups, which see every output tile exactly once.
//   wgrad16v3 (the 16 -> 16 training layers): sliding G-plane ring, below.
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace ncnet {

template <int B, int E, typename F>
__device__ __forceinline__ void wstatic_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    wstatic_for<B + 1, E>(f);
  }
}

struct WGeom {
  int V, I, J, K, L;
  int TK, TL, nkt, nlt;
  int PR, RS;          // staged X plane rows / row stride (wgrad16)
  int RW;              // staged row width (voxels, <= RS)
  int nitems, ipg;     // output tiles, tiles per group
  int dj_center;       // 0: all KS*KS (di, dj) offsets; 2: only (P, P) (plane-only:
                       // ij encoding or 16-channel input blocks, offsets in channels)
};

struct Item { int v, i, j, k0, l0; };
__device__ __forceinline__ Item decode_item(const WGeom& g, int it) {
  Item r;
  int lt = it % g.nlt; it /= g.nlt;
  int kt = it % g.nkt; it /= g.nkt;
  r.j = it % g.J; it /= g.J;
  r.i = it % g.I; r.v = it / g.I;
  r.k0 = kt * g.TK; r.l0 = lt * g.TL;
  return r;
}

// Advance a decoded item to item + 1 (same order as decode_item).
__device__ __forceinline__ void next_item(const WGeom& g, Item& r) {
  r.l0 += g.TL;
  if (r.l0 < g.nlt * g.TL) return;
  r.l0 = 0;
  r.k0 += g.TK;
  if (r.k0 < g.nkt * g.TK) return;
  r.k0 = 0;
  if (++r.j < g.J) return;
  r.j = 0;
  if (++r.i < g.I) return;
  r.i = 0;
  ++r.v;
}

__device__ __forceinline__ size_t plane_off(const WGeom& g, int v, int i, int j, int C) {
  return ((((size_t)v * g.I + i) * g.J + j) * (size_t)g.K * g.L) * C;
}

// ===========================================================================
// wgrad16v2: same math as wgrad16, restructured like conv16v2:
//  * 8 waves = 4 tap groups x 2 halves of the voxel K-chunks; each half writes
//    its own partial row (part is [2*ngroups, ...]), so no in-kernel reduction;
//  * X plane rows and G tile rows arrive by LDS-DMA (global_load_lds_dwordx4),
//    one wave-instruction per row (RS, TL <= 32 voxels): no staging VGPRs,
//    ~60 VGPRs, three workgroups per CU share the latency;
//  * halo / out-of-volume chunks are zeroed per item with ds_write.
// ===========================================================================
template <int KS>
__global__ __launch_bounds__(512, 2) void wgrad16v2_kernel(const bf16* __restrict__ X, const bf16* __restrict__ G,
                                                           float* __restrict__ part, float* __restrict__ partb,
                                                           WGeom g) {
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int TPW = (NT + 3) / 4;   // taps per tap-group
  constexpr int NW = 8;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nvox = g.TK * g.TL;
  const int nv32 = (nvox + 31) & ~31;
  const int plane_bytes = g.PR * g.RS * 32;
  char* plane = smem;
  char* gt = smem + plane_bytes;
  uint16_t* voff = (uint16_t*)(gt + nv32 * 32);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tg = wave & 3, half = wave >> 2;
  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int NDD = g.dj_center == 2 ? 1 : NT;
  const int dd = lb % NDD, grp = lb / NDD;
  const int di = g.dj_center == 2 ? P : dd / KS, dj = g.dj_center == 2 ? P : dd % KS;
  const bool center = (di == P && dj == P);

  for (int o = threadIdx.x * 16; o < plane_bytes + nv32 * 32; o += NW * 64 * 16)
    *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};   // tile padding voxels stay zero
  for (int e = threadIdx.x; e < nv32; e += NW * 64) {
    int kk = e / g.TL, ll = e - kk * g.TL;
    voff[e] = (uint16_t)((e < nvox) ? (kk * g.RS + ll) * 32 : 0);
  }

  uint32_t toffw[TPW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    int tap = min(tg + 4 * tt, NT - 1);
    int dk = tap / KS, dl = tap - dk * KS;
    toffw[tt] = (uint32_t)((dk * g.RS + dl) * 32);
  }
  f32x4 acc[TPW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int q = 0; q < 8; ++q) ones[q] = f2bf(1.f);

  const int it_lo = grp * g.ipg, it_hi = min(g.nitems, it_lo + g.ipg);
  const int nchunk = nv32 >> 5;
  const int c_lo = half ? (nchunk + 1) / 2 : 0, c_hi = half ? nchunk : (nchunk + 1) / 2;
  const int gq = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;

  __syncthreads();  // zero fill done before any DMA lands
  // items are consecutive: decode the first one, then step the (l, k, j, i, v)
  // tile counters instead of four runtime divisions (scalar unit) per item
  Item r = decode_item(g, it_lo);
  for (int it = it_lo; it < it_hi; ++it, next_item(g, r)) {
    const int ii = r.i + di - P, jj = r.j + dj - P;
    if (ii < 0 || ii >= g.I || jj < 0 || jj >= g.J) continue;   // uniform over the block
    // Stage X plane rows (corner (k0-P, l0-P)) and G tile rows (corner (k0, l0)):
    // in-volume 16-byte chunks by LDS-DMA, everything else of the row zeroed
    // with ds_write (tile positions differ per item, so no stale halo survives).
    const bf16* xp = X + plane_off(g, r.v, ii, jj, 16);
    const bf16* gp = G + plane_off(g, r.v, r.i, r.j, 16);
    const size_t ext = (size_t)g.V * g.I * g.J * g.K * g.L * 16;
    (void)ext;
    {
      const int ls = max(0, r.l0 - P), le = min(g.L, r.l0 - P + g.RW);
      const int c0 = 2 * (ls - (r.l0 - P)), c1 = c0 + 2 * (le - ls);
      for (int row = wave; row < g.PR; row += NW) {
        const int kg = r.k0 - P + row;
        const bool in_k = kg >= 0 && kg < g.K;
        if (in_k) {
          if (lane < c1 - c0 && NCNET_OK((size_t)(xp - X) + ((size_t)kg * g.L + ls) * 16 + lane * 8 + 8 <= ext) &&
              NCNET_OK(row * g.RS * 32 + c0 * 16 + lane * 16 + 16 <= g.PR * g.RS * 32))
            __builtin_amdgcn_global_load_lds((const void*)(xp + ((size_t)kg * g.L + ls) * 16 + lane * 8),
                                             LDS_PTR(void, plane + row * g.RS * 32 + c0 * 16), 16, 0, 0);
        }
        if (lane < 2 * g.RW && (!in_k || lane < c0 || lane >= c1))
          *(u32x4*)(plane + row * g.RS * 32 + lane * 16) = u32x4{0u, 0u, 0u, 0u};
      }
      const int tl = min(g.TL, g.L - r.l0), tk = min(g.TK, g.K - r.k0);
      for (int row = wave; row < g.TK; row += NW) {
        if (row < tk && lane < 2 * tl &&
            NCNET_OK((size_t)(gp - G) + ((size_t)(r.k0 + row) * g.L + r.l0) * 16 + lane * 8 + 8 <= ext))
          __builtin_amdgcn_global_load_lds((const void*)(gp + ((size_t)(r.k0 + row) * g.L + r.l0) * 16 + lane * 8),
                                           LDS_PTR(void, gt + row * g.TL * 32), 16, 0, 0);
        else if (lane < 2 * g.TL)
          *(u32x4*)(gt + row * g.TL * 32 + lane * 16) = u32x4{0u, 0u, 0u, 0u};
      }
    }
    __syncthreads();  // vmcnt(0) + barrier: plane and tile landed
    for (int c = c_lo; c < c_hi; ++c) {
      // k-slot -> voxel: each 32-lane half of a tr-read covers 8 consecutive
      // voxels (256 B, all 64 banks once); A and B use the same permutation.
      const int vb0 = c * 32 + gq * 4 + qq, vb1 = vb0 + 16;
      bf16x8 bfr = cat8(lds_read_tr16(gt, vb0 * 32 + pp * 8), lds_read_tr16(gt, vb1 * 32 + pp * 8));
      const uint32_t pa0 = voff[vb0] + pp * 8, pa1 = voff[vb1] + pp * 8;
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt) {
        if (tg + 4 * tt < NT) {
          bf16x8 afr = cat8(lds_read_tr16(plane, pa0 + toffw[tt]), lds_read_tr16(plane, pa1 + toffw[tt]));
          acc[tt] = mfma16(afr, bfr, acc[tt]);
        }
      }
      if (center && tg == 0) accb = mfma16(ones, bfr, accb);
    }
    __syncthreads();  // all reads done before the next DMA overwrites
  }

  float* pout = part + ((size_t)(grp * 2 + half) * NDD + dd) * NT * 256;
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    int tap = tg + 4 * tt;
    if (tap < NT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) pout[tap * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[tt][r];
    }
  }
  if (center && tg == 0 && lane < 16) partb[(grp * 2 + half) * 16 + lane] = accb[0];
}

// ===========================================================================
// wgrad16v3: sliding-window wgrad.  A workgroup owns one plane offset dj (or
// dj = P in dj-centre mode) and ALL KS offsets di, and walks X-plane columns
// (v, jj, tile) along ii.  X plane ii pairs with the G planes gi = ii - di + P
// (di = 0..KS-1), i.e. ii-P..ii+P: consecutive steps share KS-1 of them, so G
// tiles live in a ring of KS+1 LDS slots (one new tile per step streams in
// behind the compute) and each X-shift fragment read from LDS feeds KS MFMAs
// (one per di) instead of one: ~3x less LDS traffic per MFMA and ~KSx less
// global traffic than the per-(di,dj) kernels.
//   tiles: a contiguous range of VT (multiple of 64) voxels of the flattened
//   (k, l) plane, so every tile splits into an even number of 32-voxel chunks
//   (balanced halves); the X plane is staged full-width (L + KS - 1 <= 32) for
//   the rows the tile touches, at row stride RS = L + 8 (conflict-free wraps).
//   waves: 4 tap groups x 2 halves of the chunks; group g owns taps g, g+4, ..
//   for every di; the last tap NT-1 is split over groups 1..3 by di.
//   LDS: 2 X buffers + (KS+1) G slots + 1 zero slot (~110 KB: 1 WG/CU, 8 waves,
//   up to 256 VGPRs for the 6 x 5 accumulator tiles).
// part: [2*ngroups][NDD][NT][16 ci][16 co] (v2 layout), partb [2*ngroups][16].
// ===========================================================================
struct W3Geom {
  int V, I, J, K, L;
  int VT, ntl;         // voxels per tile (multiple of 64), tiles per plane
  int PR, RS, RW;      // staged X rows, row stride, row width (voxels)
  int ncols, cpg;      // X-plane columns (v, jj, tile); columns per group
  int flags;           // bit 0: s_setprio 1 for waves 4-7 (NCNET_WGRAD_FLAGS, tuning)
};

struct Col { int v, jj, a, nv, kf; };
__device__ __forceinline__ Col decode_col(const W3Geom& g, int c) {
  Col r;
  const int t = c % g.ntl; c /= g.ntl;
  r.jj = c % g.J; r.v = c / g.J;
  r.a = t * g.VT;
  r.nv = min(g.VT, g.K * g.L - r.a);
  r.kf = r.a / g.L;
  return r;
}

// NCH: 32-voxel chunks per half-tile (VT = 64 NCH), a compile-time constant so
// the chunk loop is branch-free and the fragment prefetch of chunk u + 1 needs
// no conservative LDS-counter drain at a control-flow merge.
template <int KS, int NCH>
__global__ __launch_bounds__(512, 1) void wgrad16v3_kernel(const bf16* __restrict__ X, const bf16* __restrict__ G,
                                                           float* __restrict__ part, float* __restrict__ partb,
                                                           W3Geom g) {
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int NS = KS + 1;             // G ring slots (+1 zero slot)
  constexpr int TPG = (NT - 1) / 4;      // regular taps per tap group
  constexpr int EXP = (KS + 2) / 3;      // di values of the last tap per group 1..3
  constexpr int NW = 8;
  constexpr int MAXC = NCH;              // voxel chunks per half (VT = 64 NCH <= 384)
  static_assert((NT - 1) % 4 == 0, "NT must be 1 mod 4");
  static_assert(NCH >= 1 && NCH <= 6, "1..6 chunks per half");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int xbytes = g.PR * g.RS * 32, gbytes = g.VT * 32;
  char* xbuf = smem;                      // [2][xbytes]
  char* gbuf = smem + 2 * xbytes;         // [NS + 1][gbytes]; slot NS stays zero (G planes outside the volume)

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform -> scalar branches
  const int tg = wave & 3, half = wave >> 2;
  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int NDJ = KS;
  const int djx = lb % NDJ, grp = lb / NDJ;
  const int dj = djx;
  const bool center_blk = (dj == P);
  const int NDD = NT;

  for (int o = threadIdx.x * 16; o < 2 * xbytes + (NS + 1) * gbytes; o += NW * 64 * 16)
    *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};
  uint32_t toff[TPG + 1];
#pragma unroll
  for (int m = 0; m <= TPG; ++m) {
    int tap = (m < TPG) ? tg + 4 * m : NT - 1;
    int dk = tap / KS, dl = tap - dk * KS;
    toff[m] = (uint32_t)((dk * g.RS + dl) * 32);
  }
  const int xdi_lo = tg == 0 ? KS : (tg - 1) * EXP, xdi_hi = tg == 0 ? KS : min(KS, tg * EXP);

  f32x4 acc[TPG][KS];
  f32x4 accx[EXP];
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < TPG; ++m)
#pragma unroll
    for (int d = 0; d < KS; ++d) acc[m][d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < EXP; ++e) accx[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const u32x4 ones = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};   // bf16 1.0 x 8

  const int c_lo = grp * g.cpg, c_hi = min(g.ncols, c_lo + g.cpg);
  constexpr int nch = NCH;                // chunks per half (VT multiple of 64)
  const int ch_lo = half * nch;
  const int gq = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const uint32_t ga_base = (ch_lo * 32 + gq * 4 + qq) * 32 + pp * 8;   // + u*1024 (+512 for the 2nd read)
  // per-lane X voxel addresses of this half's chunks for the current tile
  // (k-slot -> voxel: each 32-lane half of a tr-read covers 8 consecutive
  // voxels, i.e. 256 B or one 256-B jump across a row wrap: all banks once)
  uint32_t pav0[MAXC], pav1[MAXC];
  auto set_tile = [&](const Col& r) {
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
      const int e0 = (ch_lo + u) * 32 + gq * 4 + qq, e1 = e0 + 16;
      const int f0 = r.a + e0, f1 = r.a + e1;
      const int k0 = f0 / g.L, k1 = f1 / g.L;
      pav0[u] = (e0 < r.nv ? ((k0 - r.kf) * g.RS + f0 - k0 * g.L) * 32 : 0) + pp * 8;
      pav1[u] = (e1 < r.nv ? ((k1 - r.kf) * g.RS + f1 - k1 * g.L) * 32 : 0) + pp * 8;
    }
  };

  auto col_ok = [&](int c) {
    if (c >= c_hi) return true;   // end sentinel
    const int gj = decode_col(g, c).jj - dj + P;
    return gj >= 0 && gj < g.J;
  };
  auto next_col = [&](int c) {
    ++c;
    while (c < c_hi && !col_ok(c)) ++c;
    return c;
  };

  const size_t ext = (size_t)g.V * g.I * g.J * g.K * g.L * 16;
  (void)ext;
  // Stage the X rows kf-P .. kf-P+PR-1 of plane (ii, jj), full width, col 0 <-> l = -P.
  auto stage_x = [&](const Col& r, int ii, char* buf) {
    const bf16* xp = X + ((((size_t)r.v * g.I + ii) * g.J + r.jj) * (size_t)g.K * g.L) * 16;
    for (int row = wave; row < g.PR; row += NW) {
      const int kg = r.kf - P + row;
      const bool in_k = kg >= 0 && kg < g.K;
      if (in_k && lane < 2 * g.L && NCNET_OK((size_t)(xp - X) + (size_t)kg * g.L * 16 + lane * 8 + 8 <= ext) &&
          NCNET_OK(row * g.RS * 32 + P * 32 + lane * 16 + 16 <= g.PR * g.RS * 32))
        dma16_lds(xp + (size_t)kg * g.L * 16 + lane * 8, buf + row * g.RS * 32 + P * 32);
      if (lane < 2 * g.RW && (!in_k || lane < 2 * P || lane >= 2 * P + 2 * g.L))
        *(u32x4*)(buf + row * g.RS * 32 + lane * 16) = u32x4{0u, 0u, 0u, 0u};
    }
  };
  // Stage the tile's nv contiguous G voxels of plane (gi, gj); zero the rest of the slot.
  auto stage_g = [&](const Col& r, int gi, char* buf) {
    const int gj = r.jj - dj + P;
    const bf16* gp = G + ((((size_t)r.v * g.I + gi) * g.J + gj) * (size_t)g.K * g.L + r.a) * 16;
    for (int q = wave; q * 64 < 2 * g.VT; q += NW) {
      const int ci = q * 64 + lane;
      if (ci < 2 * r.nv && NCNET_OK((size_t)(gp - G) + ci * 8 + 8 <= ext))
        dma16_lds(gp + ci * 8, buf + q * 1024);
      else
        *(u32x4*)(buf + ci * 16) = u32x4{0u, 0u, 0u, 0u};
    }
  };

  int col = c_lo;
  while (col < c_hi && !col_ok(col)) col = next_col(col);
  // loaders: X (one plane per step), G (sequence over valid columns x gi)
  // the loaders keep their column decoded (three runtime divisions, all on the
  // scalar unit) and re-decode only when they move to the next column, not per step
  int xl_col = col, xl_ii = 0, xl_step = 0;
  int gl_col = col, gl_gi = 0, gl_seq = 0, gl_slot = 0;
  Col xl_r = decode_col(g, col), gl_r = xl_r;
  auto load_x_next = [&]() {
    if (xl_col >= c_hi) return;
    stage_x(xl_r, xl_ii, xbuf + (xl_step & 1) * xbytes);
    ++xl_step;
    if (++xl_ii == g.I) {
      xl_ii = 0;
      xl_col = next_col(xl_col);
      if (xl_col < c_hi) xl_r = decode_col(g, xl_col);
    }
  };
  auto load_g_upto = [&](int seq_max) {
    while (gl_col < c_hi && gl_seq <= seq_max) {
      stage_g(gl_r, gl_gi, gbuf + gl_slot * gbytes);
      ++gl_seq;
      if (++gl_slot == NS) gl_slot = 0;
      if (++gl_gi == g.I) {
        gl_gi = 0;
        gl_col = next_col(gl_col);
        if (gl_col < c_hi) gl_r = decode_col(g, gl_col);
      }
    }
  };

  // static priority for the second-dispatched half (waves 4-7 lose VALU
  // arbitration to the older half on every step otherwise); wave-uniform guard
  if ((g.flags & 1) && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  __syncthreads();   // zero fill before any DMA lands
  load_x_next();
  load_g_upto(NS - 2);
  int step = 0, base = 0;
  for (; col < c_hi; col = next_col(col), base += g.I) {
    set_tile(decode_col(g, col));
    for (int ii = 0; ii < g.I; ++ii, ++step) {
      asm_barrier_vm0();   // X[step] and the G tiles of this step landed; previous step's reads done
      load_x_next();
      load_g_upto(base + max(0, ii - P) + NS - 1);
      const char* xc = xbuf + (step & 1) * xbytes;
      // valid di: gi = ii - di + P in [0, I); invalid ones read the zero slot,
      // so every MFMA is issued unconditionally (<5% zero work at the I edges)
      const int di_lo = max(0, ii + P - g.I + 1), di_hi = min(KS - 1, ii + P);
      const int s0 = (base + ii + P) % NS;   // ring slot of G plane gi = ii + P (di = 0)
      uint32_t gslot[KS];
#pragma unroll
      for (int d = 0; d < KS; ++d) {
        const int sd = s0 - d < 0 ? s0 - d + NS : s0 - d;
        gslot[d] = (uint32_t)((d >= di_lo && d <= di_hi) ? sd : NS) * gbytes;
      }
      // software pipeline: the next chunk's G fragments and the next tap's X
      // fragment are in flight while the current MFMAs run
      // fragments held as u32 vectors (see cat4u in common.h)
      // ping-pong by chunk parity (compile-time after unrolling: no copies)
      u32x4 bfr[2][KS];
#pragma unroll
      for (int d = 0; d < KS; ++d)
        bfr[0][d] = cat4u(lds_read_tr16u(gbuf, gslot[d] + ga_base), lds_read_tr16u(gbuf, gslot[d] + ga_base + 512));
#pragma unroll
      for (int u = 0; u < MAXC; ++u) {
        if (u < nch) {
          const uint32_t pa0 = pav0[u], pa1 = pav1[u];
          u32x4 afr = cat4u(lds_read_tr16u(xc, pa0 + toff[0]), lds_read_tr16u(xc, pa1 + toff[0]));
          if (u + 1 < nch) {
            const uint32_t gn = ga_base + (u + 1) * 1024;
#pragma unroll
            for (int d = 0; d < KS; ++d)
              bfr[(u + 1) & 1][d] = cat4u(lds_read_tr16u(gbuf, gslot[d] + gn), lds_read_tr16u(gbuf, gslot[d] + gn + 512));
          }
#pragma unroll
          for (int m = 0; m < TPG; ++m) {
            // (m = TPG - 1: the last tap NT - 1, used by groups 1..3 only; group 0
            // reads it too, which keeps this loop free of a wave-uniform branch)
            const u32x4 afn = cat4u(lds_read_tr16u(xc, pa0 + toff[m + 1]), lds_read_tr16u(xc, pa1 + toff[m + 1]));
#pragma unroll
            for (int d = 0; d < KS; ++d) acc[m][d] = mfma16u(afr, bfr[u & 1][d], acc[m][d]);
            afr = afn;
          }
          // last tap (afr) x this group's di range: the G fragments of those di
          // are already in registers (bfr), selected by a wave-uniform branch
          // on the group so every fragment index stays compile-time
          wstatic_for<1, 4>([&](auto tc) {
            constexpr int TGC = decltype(tc)::value;
            if (tg == TGC) {
              wstatic_for<0, EXP>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                constexpr int d = (TGC - 1) * EXP + e;
                if constexpr (d < KS && d < TGC * EXP) accx[e] = mfma16u(afr, bfr[u & 1][d], accx[e]);
              });
            }
          });
          if (center_blk && tg == 0) accb = mfma16u(ones, bfr[u & 1][P], accb);
        }
      }
    }
  }

  // D[row = ci = 4(l>>4)+r][col = co = l&15]
  const int row = grp * 2 + half;
#pragma unroll
  for (int m = 0; m < TPG; ++m) {
    const int tap = tg + 4 * m;
#pragma unroll
    for (int d = 0; d < KS; ++d) {
      const int ddi = d * KS + dj;
      float* pout = part + (((size_t)row * NDD + ddi) * NT + tap) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) pout[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[m][d][r];
    }
  }
#pragma unroll
  for (int e = 0; e < EXP; ++e) {
    const int d = xdi_lo + e;
    if (d < xdi_hi) {
      const int ddi = d * KS + dj;
      float* pout = part + (((size_t)row * NDD + ddi) * NT + (NT - 1)) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) pout[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = accx[e][r];
    }
  }
  if (center_blk && tg == 0 && lane < 16) partb[row * 16 + lane] = accb[0];
}


// ===========================================================================
// wgrad16v4: wgrad16v3's decomposition (workgroup = one dj, all di, columns
// walked along ii, G tiles in a ring) at a compile-time (K, L) plane, rebuilt
// like conv16v4 for latency hiding:
//  * one X plane and one G tile per step, both DMA'd TWO steps ahead (3 X
//    buffers, G ring of 2P + 3 slots + a zero slot), every wave issuing a fixed
//    number of asm buffer-load->LDS DMAs per step (unowned rows / KiBs go to a
//    trash KiB) so each step's barrier waits with a compile-time vmcnt for
//    exactly the data it reads;
//  * buffer resources return zeros out of range: the X halo rows / columns and
//    the G voxels past the tile are written as zeros by the DMA itself (no
//    per-step ds_write zero fill);
//  * the tap group (wave & 3) is a template parameter of the whole loop, so
//    every X-fragment tap offset is a compile-time immediate of the transposed
//    read (no address VALU), and the X / G fragments of the next MFMA group are
//    in flight while the current one runs (sched_group_barrier).
// Same part / partb layout and grid as wgrad16v3.
// ===========================================================================
template <int KS, int K, int L>
struct W4C {
  static constexpr int P = KS / 2, NT = KS * KS, NW = 8;
  static constexpr int TPG = (NT - 1) / 4, EXP = (KS + 2) / 3;
  static constexpr int KL = K * L;
  static constexpr int NTL = (KL + 319) / 320;
  // VT: a multiple of 32 voxels (was 64): the two wave halves take NCH0 and
  // NCH1 32-voxel chunks (20 x 20 planes: 2 tiles of 224 = 4 + 3 chunks, 448
  // voxel slots for 400 voxels, where 64-voxel rounding gave 512)
  static constexpr int NC32 = (((KL + NTL - 1) / NTL) + 31) / 32;
  static constexpr int VT = NC32 * 32;
  static constexpr int NCH0 = (NC32 + 1) / 2, NCH1 = NC32 / 2;   // chunks of half 0 / half 1
  static constexpr int NCH = NCH0;                       // the larger
  static constexpr int RS = L + 8, RW = L + KS - 1;
  static constexpr int PR = (VT - 1) / L + 2 + KS - 1;   // staged X rows
  static constexpr int XB = PR * RS * 32, GB = VT * 32;
  static constexpr int NS = 2 * P + 3;                   // G ring slots (2 steps ahead)
  static constexpr int GOFF = 0, ZOFF = NS * GB, XOFF = ZOFF + GB, TRASH = XOFF + 3 * XB;
  static constexpr int LDS = TRASH + 1024;
  static constexpr int RPW = (PR + NW - 1) / NW;         // X rows per wave per step
  static constexpr int XI = (RW + 31) / 32;              // DMA wave-instructions per row (32 voxels each)
  static constexpr int GQ = GB / 1024;                   // 1-KiB G chunks per tile
  static constexpr int GPW = (GQ + NW - 1) / NW;         // G DMAs per wave per step
  static_assert((NT - 1) % 4 == 0, "NT must be 1 mod 4");
  static_assert(XI <= 2, "at most two DMA wave-instructions per staged row");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// 16-B-per-lane buffer load into LDS from asm (see dma16_lds in common.h):
// out-of-range offsets land as zeros.
typedef int i32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4v make_rsrc(const void* base, uint32_t nbytes) {
  const uint64_t b = (uint64_t)base;
  i32x4v r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(b >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)nbytes);
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void bdma16_lds(const i32x4v& rs, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds)
               : "memory", "m0");
}

template <int KS, int K, int L, int TG, int NCHH>
__device__ __forceinline__ void wgrad16v4_body(const bf16* __restrict__ X, const bf16* __restrict__ G,
                                               float* __restrict__ part, float* __restrict__ partb, const W3Geom& g,
                                               int wave, int half, int dj, int grp) {
  using C = W4C<KS, K, L>;
  constexpr int P = C::P, NT = C::NT, TPG = C::TPG, EXP = C::EXP, NS = C::NS, NW = C::NW;
  constexpr int NCH = NCHH;                              // this wave's chunks (its half's share)
  constexpr int RS = C::RS, PR = C::PR, XB = C::XB, GB = C::GB;
  constexpr int RPW = C::RPW, GPW = C::GPW, GQ = C::GQ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  const int lane = threadIdx.x & 63;
  const bool center_blk = dj == P;
  constexpr int XLO = TG == 0 ? KS : (TG - 1) * EXP;              // di range of the last tap (NT - 1)
  constexpr int XHI = TG == 0 ? KS : (TG * EXP < KS ? TG * EXP : KS);

  f32x4 acc[TPG][KS];
  f32x4 accx[EXP];
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < TPG; ++m)
#pragma unroll
    for (int d = 0; d < KS; ++d) acc[m][d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < EXP; ++e) accx[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  const u32x4 ones = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};   // bf16 1.0 x 8

  const int c_lo = grp * g.cpg, c_hi = min(g.ncols, c_lo + g.cpg);
  auto col_ok = [&](int c) { const int gj = (c / C::NTL) % g.J - dj + P; return gj >= 0 && gj < g.J; };
  auto next_col = [&](int c) { ++c; while (c < c_hi && !col_ok(c)) ++c; return c; };
  int c0 = c_lo;
  while (c0 < c_hi && !col_ok(c0)) ++c0;
  int nsteps = 0;                                     // valid columns x I
  for (int c = c0; c < c_hi; c = next_col(c)) nsteps += g.I;

  // ---- loaders ------------------------------------------------------------
  const int gq = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  // X: rows kf - P .. kf - P + PR - 1 of plane (v, ii, jj), col 0 <-> l = -P;
  // instruction h of a row covers its voxels 32 h .. 32 h + 31
  constexpr int XI = C::XI;
  uint32_t xvo[RPW][XI];
  auto set_xvo = [&](int kf) {
#pragma unroll
    for (int m = 0; m < RPW; ++m)
#pragma unroll
      for (int h = 0; h < XI; ++h) {
        const int r = wave + NW * m, kg = kf - P + r, c = (lane >> 1) + 32 * h, l = c - P;
        const bool ok = r < PR && kg >= 0 && kg < K && l >= 0 && l < L && c < C::RW;
        xvo[m][h] = ok ? (uint32_t)(((kg * L + l) * 16 + (lane & 1) * 8) * 2) : 0x7ffffff0u;
      }
  };
  // loader cursors keep their column decoded (a plane pointer at ii = 0 and the
  // plane stride): the runtime divisions run once per column, not per step
  const size_t pstride = (size_t)g.J * K * L * 16;       // elements between planes ii and ii + 1
  auto col_base = [&](int c, int jshift, int a) {
    const int v = (c / C::NTL) / g.J, jj = (c / C::NTL) % g.J;
    return (((size_t)v * g.I) * g.J + (jj + jshift)) * (size_t)K * L * 16 + (size_t)a * 16;
  };
  int xl_c = c0, xl_ii = 0, xl_n = 0;
  size_t xl_base = c0 < c_hi ? col_base(c0, 0, 0) : 0;
  set_xvo(((c0 % C::NTL) * C::VT) / L);
  auto issue_x = [&]() {
    const bool live = xl_n < nsteps;
    const bf16* xp = live ? X + xl_base + (size_t)xl_ii * pstride : X;
    const i32x4v rs = make_rsrc(xp, live ? (uint32_t)(K * L * 32) : 0u);
    const uint32_t xb = lds0 + C::XOFF + (uint32_t)((xl_n % 3) * XB);
#pragma unroll
    for (int m = 0; m < RPW; ++m) {
      const int r = wave + NW * m;
      // lanes past the row stride would overwrite the next row: off (count unchanged)
#pragma unroll
      for (int h = 0; h < XI; ++h)
        if (RS >= 32 * (h + 1) || (lane >> 1) + 32 * h < RS)
          bdma16_lds(rs, xvo[m][h], r < PR ? xb + (uint32_t)((r * RS + 32 * h) * 32) : lds0 + C::TRASH);
    }
    ++xl_n;
    if (++xl_ii == g.I) {
      xl_ii = 0;
      xl_c = next_col(xl_c);
      if (xl_c < c_hi) {
        set_xvo(((xl_c % C::NTL) * C::VT) / L);
        xl_base = col_base(xl_c, 0, 0);
      }
    }
  };
  // G: the tile's voxels a .. a + nv - 1 of plane (v, gi, jj - dj + P); ring slot = seq % NS
  int gl_c = c0, gl_gi = 0, gl_m = 0;
  int gl_nvb = 0;                                        // the tile's bytes (nv * 32)
  size_t gl_base = 0;
  auto set_gcol = [&](int c) {
    const int a = (c % C::NTL) * C::VT;
    gl_nvb = min(C::VT, K * L - a) * 32;
    gl_base = col_base(c, P - dj, a);
  };
  if (c0 < c_hi) set_gcol(c0);
  auto issue_g = [&]() {
    const bool live = gl_m < nsteps;
    const bf16* gp = live ? G + gl_base + (size_t)gl_gi * pstride : G;
    const i32x4v rs = make_rsrc(gp, live ? (uint32_t)gl_nvb : 0u);
    const uint32_t gb = lds0 + C::GOFF + (uint32_t)((gl_m % NS) * GB);
#pragma unroll
    for (int m = 0; m < GPW; ++m) {
      const int q = wave + NW * m;
      bdma16_lds(rs, (uint32_t)((q * 64 + lane) * 16), q < GQ ? gb + (uint32_t)(q * 1024) : lds0 + C::TRASH);
    }
    ++gl_m;
    if (++gl_gi == g.I) {
      gl_gi = 0;
      gl_c = next_col(gl_c);
      if (gl_c < c_hi) set_gcol(gl_c);
    }
  };

  // zero slot (G planes outside the volume), then the pipeline prologue:
  // G tiles 0 .. P-1, then steps "-2" and "-1" (X 0 / G P, X 1 / G P+1)
  for (int o = threadIdx.x * 16; o < GB; o += NW * 64 * 16) *(u32x4*)(smem + C::ZOFF + o) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  for (int i = 0; i < P; ++i) issue_g();
  issue_x(); issue_g();
  issue_x(); issue_g();

  // ---- compute ------------------------------------------------------------
  const int ch_lo = half * C::NCH0;
  const uint32_t ga_base = (uint32_t)((ch_lo * 32 + gq * 4 + qq) * 32 + pp * 8);
  uint32_t pav0[NCH], pav1[NCH];
  auto set_tile = [&](int c) {
    const int t = c % C::NTL, a = t * C::VT, nv = min(C::VT, K * L - a), kf = a / L;
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int e0 = (ch_lo + u) * 32 + gq * 4 + qq, e1 = e0 + 16;
      const int f0 = a + e0, f1 = a + e1;
      const int k0 = f0 / L, k1 = f1 / L;
      pav0[u] = (uint32_t)((e0 < nv ? ((k0 - kf) * RS + f0 - k0 * L) * 32 : 0) + pp * 8);
      pav1[u] = (uint32_t)((e1 < nv ? ((k1 - kf) * RS + f1 - k1 * L) * 32 : 0) + pp * 8);
    }
  };
  int cc = c0, ii = 0;
  if (cc < c_hi) set_tile(cc);
  for (int n = 0; n < nsteps; ++n) {
    // plane n and G tile n + P landed (issued two steps ago); only the previous
    // step's RPW + GPW DMAs may still be in flight; previous step's reads done
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(RPW * XI + GPW) : "memory");
    issue_x();
    issue_g();
    const uint32_t xb = (uint32_t)(C::XOFF + (n % 3) * XB);
    uint32_t xa0[NCH], xa1[NCH];
#pragma unroll
    for (int u = 0; u < NCH; ++u) { xa0[u] = pav0[u] + xb; xa1[u] = pav1[u] + xb; }
    uint32_t ga[KS];
#pragma unroll
    for (int d = 0; d < KS; ++d) {
      const int gi = ii - d + P;
      const int slot = (n - d + P) % NS;   // G sequence index n + P - d (same column when gi is valid)
      ga[d] = ((gi >= 0 && gi < g.I) ? (uint32_t)(C::GOFF + slot * GB) : (uint32_t)C::ZOFF) + ga_base;
    }
    // MFMA groups k = (u, m): m < TPG regular taps (x KS di), m == TPG the last
    // tap (this group's di range); fragments of group k + 1 read during k
    constexpr int NM = TPG + 1;
    constexpr int NKG = NCH * NM;
    u32x4 bfr[2][KS], afr[2];
    auto load_b = [&](auto uc, int d) {
      constexpr int u = decltype(uc)::value;
      bfr[u & 1][d] = cat4u(lds_read_tr16u(smem, ga[d] + u * 1024), lds_read_tr16u(smem, ga[d] + u * 1024 + 512));
    };
    auto load_a = [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int u = k / NM, m = k % NM;
      constexpr int tap = m < TPG ? TG + 4 * m : NT - 1;
      constexpr uint32_t to = (uint32_t)(((tap / KS) * RS + tap % KS) * 32);
      afr[k & 1] = cat4u(lds_read_tr16u(smem, xa0[u] + to), lds_read_tr16u(smem, xa1[u] + to));
    };
#pragma unroll
    for (int d = 0; d < KS; ++d) load_b(std::integral_constant<int, 0>{}, d);
    load_a(std::integral_constant<int, 0>{});
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * KS + 2, 0);
    wstatic_for<0, NKG>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int u = k / NM, m = k % NM;
      // reads issued in this group: the next group's X fragment, and (m < KS)
      // the G fragment d = m of the next chunk
      constexpr bool LA = k + 1 < NKG;
      constexpr bool LB = u + 1 < NCH && m < KS;
      if constexpr (LA) load_a(std::integral_constant<int, k + 1>{});
      if constexpr (LB) load_b(std::integral_constant<int, u + 1>{}, m);
      if constexpr (m < TPG) {
#pragma unroll
        for (int d = 0; d < KS; ++d) acc[m][d] = mfma16u(afr[k & 1], bfr[u & 1][d], acc[m][d]);
      } else {
        wstatic_for<XLO, XHI>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          accx[d - XLO] = mfma16u(afr[k & 1], bfr[u & 1][d], accx[d - XLO]);
        });
        if constexpr (TG == 0) {
          if (center_blk) accb = mfma16u(ones, bfr[u & 1][P], accb);
        }
      }
      constexpr int NR = (LA ? 2 : 0) + (LB ? 2 : 0);
      if constexpr (NR > 0) __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
      constexpr int NMF = m < TPG ? KS : (XHI - XLO);
      if constexpr (NMF > 0) __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
    });
    if (++ii == g.I) {
      ii = 0;
      cc = next_col(cc);
      if (cc < c_hi) set_tile(cc);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends

  // D[row = ci = 4(l>>4)+r][col = co = l&15]
  const int row = grp * 2 + half;
#pragma unroll
  for (int m = 0; m < TPG; ++m) {
    const int tap = TG + 4 * m;
#pragma unroll
    for (int d = 0; d < KS; ++d) {
      float* pout = part + (((size_t)row * NT + (d * KS + dj)) * NT + tap) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) pout[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[m][d][r];
    }
  }
#pragma unroll
  for (int e = 0; e < EXP; ++e) {
    const int d = XLO + e;
    if (d < XHI) {
      float* pout = part + (((size_t)row * NT + (d * KS + dj)) * NT + (NT - 1)) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) pout[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = accx[e][r];
    }
  }
  if (TG == 0 && center_blk && lane < 16) partb[row * 16 + lane] = accb[0];
}

// the body for this wave's half: one instantiation when both halves hold the
// same chunk count, two otherwise
template <int KS, int K, int L, int TG>
__device__ __forceinline__ void w4_half(const bf16* __restrict__ X, const bf16* __restrict__ G, float* __restrict__ part,
                                        float* __restrict__ partb, const W3Geom& g, int wave, int half, int dj, int grp) {
  using C = W4C<KS, K, L>;
  if constexpr (C::NCH0 == C::NCH1) {
    wgrad16v4_body<KS, K, L, TG, C::NCH0>(X, G, part, partb, g, wave, half, dj, grp);
  } else {
    if (half == 0) wgrad16v4_body<KS, K, L, TG, C::NCH0>(X, G, part, partb, g, wave, half, dj, grp);
    else wgrad16v4_body<KS, K, L, TG, C::NCH1>(X, G, part, partb, g, wave, half, dj, grp);
  }
}

template <int KS, int K, int L>
__global__ __launch_bounds__(512, 1) void wgrad16v4_kernel(const bf16* __restrict__ X, const bf16* __restrict__ G,
                                                           float* __restrict__ part, float* __restrict__ partb,
                                                           W3Geom g) {
#if defined(__HIP_DEVICE_COMPILE__)   // device-only body (asm DMA); the host pass keeps the stub
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = wave & 3, half = wave >> 2;
  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int dj = lb % KS, grp = lb / KS;
  switch (tg) {
    case 0: w4_half<KS, K, L, 0>(X, G, part, partb, g, wave, half, dj, grp); break;
    case 1: w4_half<KS, K, L, 1>(X, G, part, partb, g, wave, half, dj, grp); break;
    case 2: w4_half<KS, K, L, 2>(X, G, part, partb, g, wave, half, dj, grp); break;
    default: w4_half<KS, K, L, 3>(X, G, part, partb, g, wave, half, dj, grp); break;
  }
#endif
}

// ===========================================================================
// wgrad16p: plane-only weight gradient of the ij-encoded 1-channel layers
// (same math as wgrad16v2 with dj_center = 2) for whole-plane tiles
// (K, L <= 25), with the next item's X plane and G tiles streaming into the
// second of two LDS buffers while the current item is computed (v2 exposes the
// DMA latency of every item), and NGG G operands per X plane:
//   NGG = 2: the Cout = 1 layer, X = layer input, G = both groups of
//            ijpack(g, -1): every X fragment read feeds 2 MFMAs;
//   NGG = 1 with nsets = 2: the Cin = 1 layer, X = both groups of ijpack(x0)
//            (set = blockIdx-derived), G = the layer's output gradient.
// Tiles sit at fixed positions, so the zero halo is written once.
// part: [2 * ngroups][nsets * NGG][NT][16 ci][16 co]; partb [2 * ngroups][nsets * NGG][16].
// ===========================================================================
template <int KS, int NGG>
__global__ __launch_bounds__(512, 1) void wgrad16p_kernel(const bf16* __restrict__ X, const bf16* __restrict__ G,
                                                          float* __restrict__ part, float* __restrict__ partb, WGeom g,
                                                          long long xstride, long long gstride, int nsets) {
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int TPW = (NT + 3) / 4;
  constexpr int NW = 8;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nvox = g.K * g.L;
  const int nv32 = (nvox + 31) & ~31;
  const int xbytes = g.PR * g.RS * 32, gtb = nv32 * 32;
  const int bufbytes = xbytes + NGG * gtb;
  uint16_t* voff = (uint16_t*)(smem + 2 * bufbytes);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = wave & 3, half = wave >> 2;
  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int set = lb % nsets, grp = lb / nsets;
  const bf16* Xs = X + (size_t)set * xstride;

  for (int o = threadIdx.x * 16; o < 2 * bufbytes; o += NW * 64 * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};
  for (int e = threadIdx.x; e < nv32; e += NW * 64) {
    int kk = e / g.L, ll = e - kk * g.L;
    voff[e] = (uint16_t)((e < nvox) ? (kk * g.RS + ll) * 32 : 0);
  }
  uint32_t toffw[TPW];
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    int tap = min(tg + 4 * tt, NT - 1);
    int dk = tap / KS, dl = tap - dk * KS;
    toffw[tt] = (uint32_t)((dk * g.RS + dl) * 32);
  }
  f32x4 acc[NGG][TPW];
  f32x4 accb[NGG];
#pragma unroll
  for (int n = 0; n < NGG; ++n) {
    accb[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) acc[n][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int q = 0; q < 8; ++q) ones[q] = f2bf(1.f);

  const int it_lo = grp * g.ipg, it_hi = min(g.nitems, it_lo + g.ipg);
  const int nchunk = nv32 >> 5;
  const int c_lo = half ? (nchunk + 1) / 2 : 0, c_hi = half ? nchunk : (nchunk + 1) / 2;
  const int gq = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const size_t ext = (size_t)g.V * g.I * g.J * g.K * g.L * 16;
  (void)ext;

  // item = plane (v, i, j); X rows k = -P .. K+P-1 land at LDS row k + P, column P
  auto stage = [&](int it, char* buf) {
    const size_t po = (size_t)it * g.K * g.L * 16;
    for (int row = wave; row < g.K; row += NW) {
      if (lane < 2 * g.L && NCNET_OK(po + ((size_t)row * g.L) * 16 + lane * 8 + 8 <= ext))
        dma16_lds(Xs + po + (size_t)row * g.L * 16 + lane * 8, buf + ((row + P) * g.RS + P) * 32);
    }
#pragma unroll
    for (int n = 0; n < NGG; ++n) {
      const bf16* gp = G + (size_t)n * gstride + po;
      char* gb = buf + xbytes + n * gtb;
      for (int q = wave; q * 64 < 2 * nvox; q += NW) {
        const int ci = q * 64 + lane;
        if (ci < 2 * nvox && NCNET_OK(po + ci * 8 + 8 <= ext))
          dma16_lds(gp + ci * 8, gb + q * 1024);
      }
    }
  };

  __syncthreads();  // zero fill and voff done before any DMA lands
  if (it_lo < it_hi) stage(it_lo, smem);
  for (int it = it_lo; it < it_hi; ++it) {
    const int n0 = it - it_lo;
    asm_barrier_vm0();  // item it landed; item it-1's reads of the other buffer done
    if (it + 1 < it_hi) stage(it + 1, smem + ((n0 + 1) & 1) * bufbytes);
    const char* plane = smem + (n0 & 1) * bufbytes;
    const char* gt = plane + xbytes;
    for (int c = c_lo; c < c_hi; ++c) {
      const int vb0 = c * 32 + gq * 4 + qq, vb1 = vb0 + 16;
      bf16x8 bfr[NGG];
#pragma unroll
      for (int n = 0; n < NGG; ++n)
        bfr[n] = cat8(lds_read_tr16(gt + n * gtb, vb0 * 32 + pp * 8), lds_read_tr16(gt + n * gtb, vb1 * 32 + pp * 8));
      const uint32_t pa0 = voff[vb0] + pp * 8, pa1 = voff[vb1] + pp * 8;
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt) {
        if (tg + 4 * tt < NT) {
          bf16x8 afr = cat8(lds_read_tr16(plane, pa0 + toffw[tt]), lds_read_tr16(plane, pa1 + toffw[tt]));
#pragma unroll
          for (int n = 0; n < NGG; ++n) acc[n][tt] = mfma16(afr, bfr[n], acc[n][tt]);
        }
      }
      if (tg == 0) {
#pragma unroll
        for (int n = 0; n < NGG; ++n) accb[n] = mfma16(ones, bfr[n], accb[n]);
      }
    }
  }

  const int row = grp * 2 + half, nsl = nsets * NGG;
#pragma unroll
  for (int n = 0; n < NGG; ++n) {
    float* pout = part + ((size_t)row * nsl + set * NGG + n) * NT * 256;
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      int tap = tg + 4 * tt;
      if (tap < NT) {
#pragma unroll
        for (int r = 0; r < 4; ++r) pout[tap * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[n][tt][r];
      }
    }
    if (tg == 0 && lane < 16) partb[((size_t)row * nsl + set * NGG + n) * 16 + lane] = accb[n][0];
  }
}

}  // namespace ncnet

using namespace ncnet;

static void pick_tile_w(int K, int L, int& tk, int& tl) {
  tk = K <= 25 ? K : 25;
  tl = L <= 25 ? L : 25;
  while (tk * tl > 640) { if (tl > tk) --tl; else --tk; }
}

static WGeom make_wgeom(int V, int I, int J, int K, int L, int KS, int ngroups) {
  WGeom g;
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L;
  pick_tile_w(K, L, g.TK, g.TL);
  g.nkt = cdiv(K, g.TK); g.nlt = cdiv(L, g.TL);
  g.PR = g.TK + KS - 1; g.RS = g.TL + KS - 1; g.RW = g.RS;
  g.nitems = V * I * J * g.nkt * g.nlt;
  g.ipg = cdiv(g.nitems, ngroups);
  g.dj_center = 0;
  return g;
}

#define KS_DISPATCH(M, ...) \
  do { if (KS == 5) M(5, __VA_ARGS__); else if (KS == 3) M(3, __VA_ARGS__); \
       else if (KS == 7) M(7, __VA_ARGS__); else if (KS == 1) M(1, __VA_ARGS__); else return -2; } while (0)

// wgrad16v2.  part: [2 * ngroups][KS*KS (mode 0) or 1 (mode 2)][KS*KS][16 ci][16 co]
// fp32 (one row per voxel-chunk half); partb: [2 * ngroups][16].
extern "C" int ncnet_wgrad16(const void* X, const void* G, float* part, float* partb, int V, int I, int J, int K,
                             int L, int KS, int ngroups, int dj_center, hipStream_t stream) {
  WGeom g = make_wgeom(V, I, J, K, L, KS, ngroups);
  if (dj_center != 0 && dj_center != 2) return -3;
  g.dj_center = dj_center;
  int nv32 = (g.TK * g.TL + 31) & ~31;
  dim3 grid((unsigned)((dj_center == 2 ? 1 : KS * KS) * ngroups));
  const bf16* x = (const bf16*)X; const bf16* gg = (const bf16*)G;
  if (g.RW > 32 || g.TL > 32) return -1;   // one wave-instruction per staged row
  // row stride TL + 8: a row wrap inside an 8-voxel read group jumps 256 B
  // (bank period), keeping the transposed reads conflict-free
  g.RS = g.TL + ((KS - 1 + 7) / 8) * 8;
  if (g.PR * g.RS * 32 > 65535) return -1;  // 16-bit voxel offset table
  size_t lds = (size_t)g.PR * g.RS * 32 + (size_t)nv32 * 32 + (size_t)nv32 * 2;
  dim3 block(512);
#define WG2(KSV, _) hipLaunchKernelGGL((wgrad16v2_kernel<KSV>), grid, block, lds, stream, x, gg, part, partb, g)
  KS_DISPATCH(WG2, 0);
#undef WG2
  return (int)hipGetLastError();
}

// wgrad16p (plane-only, whole-plane tiles: K, L <= 25): X [nsets][V,I,J,K,L,16]
// (set stride xstride elements), G [NGG][...] (stride gstride); grid = ngroups * nsets.
extern "C" int ncnet_wgrad16p(const void* X, const void* G, float* part, float* partb, int V, int I, int J, int K,
                              int L, int KS, int ngroups, int nsets, int ngg, long long xstride, long long gstride,
                              hipStream_t stream) {
  if (K > 25 || L > 25) return -1;
  if (ngg != 1 && ngg != 2) return -3;
  WGeom g = make_wgeom(V, I, J, K, L, KS, ngroups);
  g.RS = L + ((KS - 1 + 7) / 8) * 8;        // row wrap jumps 256 B (conflict-free transposed reads)
  g.PR = K + KS - 1;
  if (L + KS - 1 > g.RS || g.PR * g.RS * 32 > 65535) return -1;
  const int nv32 = (K * L + 31) & ~31;
  const size_t buf = (size_t)g.PR * g.RS * 32 + (size_t)ngg * nv32 * 32;
  const size_t lds = 2 * buf + (size_t)nv32 * 2;
  if (lds > 160 * 1024) return -1;
  dim3 grid((unsigned)(ngroups * nsets)), block(512);
  const bf16* x = (const bf16*)X; const bf16* gg = (const bf16*)G;
#define WGP(KSV, _) do { if (ngg == 2) hipLaunchKernelGGL((wgrad16p_kernel<KSV, 2>), grid, block, lds, stream, x, gg, part, partb, g, xstride, gstride, nsets); \
                         else hipLaunchKernelGGL((wgrad16p_kernel<KSV, 1>), grid, block, lds, stream, x, gg, part, partb, g, xstride, gstride, nsets); } while (0)
  KS_DISPATCH(WGP, 0);
#undef WGP
  return (int)hipGetLastError();
}

template <int KS, int T>
static void w4_launch1(dim3 grid, dim3 block, hipStream_t stream, const bf16* x, const bf16* gg, float* part,
                       float* partb, const W3Geom& g) {
  using C = W4C<KS, T, T>;
  const size_t lds = (size_t)C::LDS;
  hipLaunchKernelGGL((wgrad16v4_kernel<KS, T, T>), grid, block, lds, stream, x, gg, part, partb, g);
}
static bool w4_launch(int KS, int K, dim3 grid, dim3 block, hipStream_t stream, const bf16* x, const bf16* gg,
                      float* part, float* partb, const W3Geom& g) {
  if (KS == 5 && K == 25) w4_launch1<5, 25>(grid, block, stream, x, gg, part, partb, g);
  else if (KS == 5 && K == 20) w4_launch1<5, 20>(grid, block, stream, x, gg, part, partb, g);
  else if (KS == 5 && K == 15) w4_launch1<5, 15>(grid, block, stream, x, gg, part, partb, g);
  else if (KS == 3 && K == 25) w4_launch1<3, 25>(grid, block, stream, x, gg, part, partb, g);
  else if (KS == 3 && K == 20) w4_launch1<3, 20>(grid, block, stream, x, gg, part, partb, g);
  else if (KS == 3 && K == 15) w4_launch1<3, 15>(grid, block, stream, x, gg, part, partb, g);
  else if (KS == 5 && K == 30) w4_launch1<5, 30>(grid, block, stream, x, gg, part, partb, g);   // rows of 34 voxels: 2 DMAs
  else if (KS == 3 && K == 30) w4_launch1<3, 30>(grid, block, stream, x, gg, part, partb, g);
  else return false;
  return true;
}

// v3: ngroups column groups per dj (grid = ngroups * KS).
// Tile rule (mirrored in ops/neigh_consensus.py wgrad_v3_groups):
// ntl = ceil(K*L / 320), VT = roundup(ceil(K*L / ntl), 64).
extern "C" int ncnet_wgrad16v3(const void* X, const void* G, float* part, float* partb, int V, int I, int J, int K,
                               int L, int KS, int ngroups, hipStream_t stream) {
  W3Geom g;
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L;
  const int KL = K * L;
  g.ntl = cdiv(KL, 320);
  g.VT = ((cdiv(KL, g.ntl) + 63) / 64) * 64;
  g.RW = L + KS - 1;
  g.RS = L + ((KS - 1 + 7) / 8) * 8;
  g.PR = (g.VT - 1) / L + 2 + KS - 1;
  g.ncols = V * J * g.ntl;
  g.cpg = cdiv(g.ncols, ngroups);
  g.flags = tuning().wgrad_flags;
  if (g.VT > 384) return -1;                // <= 6 chunks per half
  // the wgrad_v3 A/B switch selects the general kernel only where it can stage the
  // rows (RW <= 32); ops/neigh_consensus.py wgrad_v3_ntl mirrors the tile rule either way
  if (K == L && (!tuning().wgrad_v3 || g.RW > 32) &&
      w4_launch(KS, K, dim3((unsigned)(KS * ngroups)), dim3(512), stream, (const bf16*)X, (const bf16*)G, part,
                partb, g))
    return (int)hipGetLastError();   // compile-time planes of the training sizes (--image_size 240 / 320 / 400 / 480)
  if (g.RW > 32) return -1;                 // v3: one wave-instruction per staged row
  // wgrad16v3<5, NCH> spills at NCH 3, 4, 6 (256 VGPRs of accumulators and
  // double-buffered fragments): split the plane into more, smaller tiles until
  // the chunk count is 1, 2 or 5 (mirrored in ops/neigh_consensus.py wgrad_v3_ntl)
  if (KS == 5) {
    while (true) {
      const int nch = ((cdiv(KL, g.ntl) + 63) / 64);
      if (nch == 1 || nch == 2 || nch == 5) break;
      ++g.ntl;
    }
    g.VT = ((cdiv(KL, g.ntl) + 63) / 64) * 64;
    g.PR = (g.VT - 1) / L + 2 + KS - 1;
    g.ncols = V * J * g.ntl;
    g.cpg = cdiv(g.ncols, ngroups);
  }
  size_t lds = 2 * (size_t)g.PR * g.RS * 32 + (size_t)(KS + 2) * g.VT * 32;
  if (lds > 160 * 1024) return -1;
  dim3 grid((unsigned)(KS * ngroups)), block(512);
  const bf16* x = (const bf16*)X; const bf16* gg = (const bf16*)G;
  const int nch = g.VT / 64;
#define W3N(KSV, N) hipLaunchKernelGGL((wgrad16v3_kernel<KSV, N>), grid, block, lds, stream, x, gg, part, partb, g)
#define W3(KSV) do { switch (nch) { case 1: W3N(KSV, 1); break; case 2: W3N(KSV, 2); break; case 3: W3N(KSV, 3); break; \
                                    case 4: W3N(KSV, 4); break; case 5: W3N(KSV, 5); break; default: W3N(KSV, 6); } } while (0)
  if (KS == 5) {
    // only the spill-free chunk counts are instantiated (the tile rule above)
    switch (nch) { case 1: W3N(5, 1); break; case 2: W3N(5, 2); break; case 5: W3N(5, 5); break; default: return -3; }
  } else if (KS == 3) W3(3);
  else return -2;
#undef W3
#undef W3N
  return (int)hipGetLastError();
}
