// Conv4d forward (and transposed-conv data gradient) on gfx950 MFMA.
//
// Semantics: "same"-padded stride-1 4D cross-correlation (lib/conv4d.py:11-51)
//   Y[v,i,j,k,l,co] = sum_{di,dj,dk,dl,ci} X[v,i+di-P,j+dj-P,k+dk-P,l+dl-P,ci] W[co,ci,di,dj,dk,dl]
// computed as an implicit GEMM: M = output voxels, N = Cout, K = taps x Cin.
//
// Work decomposition (all three kernels): one workgroup owns one output tile
// (v, i, j, k0:k0+TK, l0:l0+TL) and streams the KS*KS input planes
// (i+di-P, j+dj-P, :, :) through a single LDS plane buffer, zero-padded by the
// halo, while the next plane is prefetched into registers (the reference's
// Python slice loop, lib/conv4d.py:39-48, moved inside one kernel).  Planes
// that fall outside the volume are skipped.  Bias + ReLU (forward) or the
// ReLU-mask of the previous layer (data-gradient) are fused in the epilogue.
//
//   Cin=16 -> Cout=16 : MFMA D[co][voxel], K = 2 taps x 16 ci (conv16v2 / v3).
//   The 1-channel layers run on the same kernels through the ij encoding
//   (csrc/jshift.hip): group-plane mode, in-plane (dk, dl) taps only.
//   Wider layers are channel blocks of 16 (ops/neigh_consensus.py).
#include "common.h"
#include <hip/hip_fp8.h>
#include <stdlib.h>
#include <type_traits>

namespace ncnet {

// EPI_F32X16: raw fp32 accumulators of the first nco channels, channel-planar
// [nco][V,I,J,K,L] (ij-encoded Cout=1 partials summed by ijsum, or the per
// input-block partials of a layer wider than 16 channels).
// EPI_BLK1: Cout = 1 layer in output-plane-block mode (conv16v2 only, below):
// the 16 MFMA rows are a 4 x 4 block of output (i, j) planes; fp32 single-channel
// output with bias (+ ReLU).
// EPI_X3 (flag, with EPI_BIAS_RELU / EPI_MASK / EPI_BLK1): fp32-accurate "bf16x3"
// layer -- the kernel runs three phases into the same accumulators,
// (X_hi, W_hi), (X_hi, W_lo), (X_lo, W_hi), with X_lo = X + g.xlo and the lo
// weight planes stored right after the hi ones; the bf16-block epilogues write
// the result split as hi = bf16(y) at Y and lo = bf16(y - hi) at Y + g.ylo.
enum Epi { EPI_NONE = 0, EPI_BIAS_RELU = 1, EPI_MASK = 2, EPI_F32X16 = 4, EPI_BLK1 = 8, EPI_X3 = 64 };

struct ConvGeom {
  int V, I, J, K, L;  // volume dims
  int TK, TL;         // output tile along k, l
  int nkt, nlt;       // tiles along k, l
  int PR, RS;         // staged plane rows / row stride (voxels)
  int RW;             // staged row width (voxels, <= RS)
    int nco;            // planar fp32 epilogue: output channels written (<= 16)
  float oscale;       // fp8 kernel: accumulator scale (1 / weight scale)
  int npg;            // > 0: "group planes" mode (v2 only): plane s is the (i, j)
  long long gstride;  //   plane of input group s at X + s * gstride, weights plane s
  int njb;            // output j-blocks per (v, i): J, or cdiv(J, R) (v3) / cdiv(J, tpw) (v2 group planes)
  int tpw;            // v2 group-plane mode: consecutive output j-tiles per workgroup (1 otherwise)
  int nt;             // v2 / v3 epilogues: non-temporal output stores (NCNET_NT_STORE)
  int nib;            // EPI_BLK1: 4-plane output blocks along i (njb: along j)
  int relu;           // EPI_BLK1: ReLU after the bias
  long long xlo;      // EPI_X3: element offset of X_lo from X
  long long ylo;      // EPI_X3: element offset of the lo output from Y
};

// Decode the workgroup's output tile.
struct TileId { int v, i, j, k0, l0; };
__device__ __forceinline__ TileId decode_tile(const ConvGeom& g) {
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  TileId t;
  int lt = bid % g.nlt; bid /= g.nlt;
  int kt = bid % g.nkt; bid /= g.nkt;
  t.j = (bid % g.njb) * g.tpw; bid /= g.njb;
  t.i = bid % g.I; t.v = bid / g.I;
  t.k0 = kt * g.TK; t.l0 = lt * g.TL;
  return t;
}

__device__ __forceinline__ size_t plane_offset(const ConvGeom& g, int v, int i, int j, int C) {
  return ((((size_t)v * g.I + i) * g.J + j) * (size_t)g.K * g.L) * C;
}

// Epilogue for a [16 co x 16 voxel] accumulator tile: lane holds co = 4(l>>4)+r
// of voxel (l & 15).
// nt: streaming (non-temporal) stores -- the volumes written here (0.1-1.6 GB)
// never stay in the 4 MB L2s, so a write-allocating store only evicts the
// operands the running kernel is still reading.
// This lane's 4 output-channel biases (rows 4 (lane >> 4) + r) for the bias +
// ReLU epilogues, read once before the store loop as 16 uniform scalar loads and
// a per-lane select.  A vector load used inside each conditional store block
// makes the waitcnt pass re-wait vmcnt(0) there -- stores count in vmcnt -- and
// serialises the epilogue (26-34 waits per kernel before, 1 after).
template <int EPI>
__device__ __forceinline__ f32x4 lane_bias4(const float* __restrict__ bias, int lane) {
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};
  if constexpr ((EPI & ~EPI_X3) == EPI_BIAS_RELU) {
    float bs[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) bs[c] = bias[c];
    const int gq = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = gq == 0 ? bs[r] : gq == 1 ? bs[4 + r] : gq == 2 ? bs[8 + r] : bs[12 + r];
  }
  return bv;
}

template <int EPI>
__device__ __forceinline__ void store16(const f32x4& acc, bf16* __restrict__ Y, const bf16* __restrict__ M,
                                        const float* __restrict__ bias, size_t vox_index, int co0, size_t nvox_all = 0,
                                        int nco = 16, bool nt = false, long long ylo = 0,
                                        const u32x2* mpre = nullptr, const f32x4* bpre = nullptr) {
  if (!NCNET_OK(vox_index < nvox_all && co0 >= 0 && co0 + 4 <= 16)) return;
  constexpr bool X3 = (EPI & EPI_X3) != 0;
  constexpr int E = EPI & ~EPI_X3;
  if (E == EPI_F32X16) {
    // channel-planar fp32 [nco][nvox_all] (only the channels a consumer reads):
    // 16 lanes write 16 consecutive voxels of one channel
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (co0 + r < nco) {
        float* dst = (float*)Y + (size_t)(co0 + r) * nvox_all + vox_index;
        if (nt) __builtin_nontemporal_store(acc[r], dst);
        else *dst = acc[r];
      }
    return;
  }
  float o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float x = acc[r];
    if (E == EPI_BIAS_RELU) x = fmaxf(x + (bpre ? (*bpre)[r] : bias[co0 + r]), 0.f);
    o[r] = x;
  }
  if (E == EPI_MASK) {
    // (X3: the mask is the hi part of the ReLU output -- bf16(y) > 0 iff y > 0)
    // mpre: the mask the caller fetched ahead (conv16v4), else loaded here
    const bf16x4 m = mpre ? __builtin_bit_cast(bf16x4, *mpre) : *(const bf16x4*)(M + vox_index * 16 + co0);
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = ((float)m[r] > 0.f) ? o[r] : 0.f;
  }
  bf16x4 out;
#pragma unroll
  for (int r = 0; r < 4; ++r) out[r] = f2bf(o[r]);
  if (nt) __builtin_nontemporal_store(__builtin_bit_cast(u32x2, out), (u32x2*)(Y + vox_index * 16 + co0));
  else *(bf16x4*)(Y + vox_index * 16 + co0) = out;
  if constexpr (X3) {
    bf16x4 lo;
#pragma unroll
    for (int r = 0; r < 4; ++r) lo[r] = f2bf(o[r] - bf2f(out[r]));
    bf16* yl = Y + ylo + vox_index * 16 + co0;
    if (nt) __builtin_nontemporal_store(__builtin_bit_cast(u32x2, lo), (u32x2*)yl);
    else *(bf16x4*)yl = lo;
  }
}

// ===========================================================================
// conv16v2_fwd: same math as conv16_fwd, restructured for occupancy and
// copy/compute overlap:
//  * 8 waves per workgroup, 5 voxel tiles per wave (20 accumulator VGPRs);
//  * planes and weights arrive by LDS-DMA (global_load_lds_dwordx4): one
//    wave-instruction per plane row (<= 32 voxels = 1 KiB), no staging VGPRs;
//  * plane rows at stride RS = TL + 8 voxels: a 16-voxel tile that wraps to
//    the next row jumps a whole 256-B bank period, so the ds_read_b128 lane
//    groups stay conflict-free;
//  * two plane buffers (plane s+1 streams in while plane s is computed) and
//    ONE weight buffer: the weights of plane s go to registers at the top of
//    the plane, a mid-plane s_barrier (no vmcnt drain, so the plane DMA keeps
//    flying) releases the buffer and plane s+1's weights stream in behind the
//    remaining tiles.  2 x 30.6 KB + 13 KB keeps two workgroups per CU.
//  * halo/out-of-volume voxels are zeroed once (fixed positions for the tile).
// Requires RW = TL + KS - 1 <= 32.  KS = 7 keeps its 25 weight fragments in
// registers at one workgroup per CU (256 VGPRs) instead of two.
// ===========================================================================
// CT > 0: the (k, l) planes are CT x CT and the tile is the whole plane, fixed
// at compile time (the Cout = 1 block layer at the 400 px training volume):
// plane geometry, tile decode and the per-tap LDS offsets fold into constants
// and instruction offsets instead of per-MFMA address VALU.
template <int KS, int EPI, bool MT, int CT = 0>
__global__ __launch_bounds__(512, KS >= 7 ? 1 : 2) void conv16v2_fwd_kernel(const bf16* __restrict__ X, const u32x4* __restrict__ Wp,
                                                              const float* __restrict__ bias,
                                                              const bf16* __restrict__ M, bf16* __restrict__ Y,
                                                              ConvGeom g_in) {
  ConvGeom g = g_in;
  if constexpr (CT > 0) {
    g.K = g.L = g.TK = g.TL = CT;
    g.nkt = g.nlt = 1;
    g.PR = g.RW = CT + KS - 1;
    g.RS = CT + ((KS - 1 + 7) / 8) * 8;
  }
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int NQ = (NT + 1) / 2;
  constexpr int NW = 8;
  constexpr int MAXT = 5;  // 16-voxel tiles per wave (TK*TL <= 640)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int plane_bytes = g.PR * g.RS * 32;
  char* wbuf = smem + 2 * plane_bytes;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr bool BLK = (EPI & ~EPI_X3) == EPI_BLK1;
  constexpr bool X3 = (EPI & EPI_X3) != 0;
  constexpr int PH = X3 ? 3 : 1;   // EPI_X3: phases (X_hi, W_hi), (X_hi, W_lo), (X_lo, W_hi)
  constexpr int SP = KS + 3;   // EPI_BLK1: input planes per block side (4 + KS - 1)
  TileId t;
  if (BLK) {
    uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
    const int lt = bid % g.nlt; bid /= g.nlt;
    const int kt = bid % g.nkt; bid /= g.nkt;
    t.j = (bid % g.njb) * 4; bid /= g.njb;
    t.i = (bid % g.nib) * 4; t.v = bid / g.nib;
    t.k0 = kt * g.TK; t.l0 = lt * g.TL;
  } else {
    t = decode_tile(g);
  }
  // plane-offset ranges; EPI_BLK1: absolute input plane ranges of the block
  // (i0 - P .. i0 + 3 + P clipped to the volume), every one feeding <= 16 rows
  const int di_lo = BLK ? max(0, t.i - P) : max(0, P - t.i);
  const int di_hi = BLK ? min(g.I, t.i + 4 + P) : min(KS, g.I + P - t.i);
  const int dj_lo = BLK ? max(0, t.j - P) : max(0, P - t.j);
  const int dj_hi = BLK ? min(g.J, t.j + 4 + P) : min(KS, g.J + P - t.j);
  const int ndj = dj_hi - dj_lo;
  const int nplanes1 = g.npg > 0 ? g.npg : (di_hi - di_lo) * ndj;   // planes of one phase
  const int nplanes = PH * nplanes1;
  const int nvox = g.TK * g.TL;
  const int ntile = (nvox + 15) >> 4;

  for (int o = threadIdx.x * 16; o < 2 * plane_bytes; o += NW * 64 * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};

  uint32_t vbase[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int vi = (wave + NW * tt) * 16 + (lane & 15);
    if (vi >= nvox) vi = 0;
    int kk = vi / g.TL, ll = vi - kk * g.TL;
    vbase[tt] = (uint32_t)((kk * g.RS + ll) * 32 + ((lane >> 4) & 1) * 16);
  }
  uint32_t toff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    int tap = 2 * q + (lane >> 5);
    if (tap >= NT) tap = NT - 1;
    int dk = tap / KS, dl = tap - dk * KS;
    toff[q] = (uint32_t)((dk * g.RS + dl) * 32);
  }
  // CT: per-lane bases of the two lane halves (taps 2q and 2q + 1: the next
  // voxel, or one row down with dl wrapped when 2q + 1 is a multiple of KS;
  // the padded last pair reads voxel + 1 of its row against zero weights), so
  // each tap's offset (2q's) is a compile-time ds_read immediate
  uint32_t c1[CT > 0 ? MAXT : 1], c2[CT > 0 ? MAXT : 1];
  if constexpr (CT > 0) {
    const uint32_t hh = (uint32_t)(lane >> 5);
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) {
      c1[tt] = vbase[tt] + hh * 32u;
      c2[tt] = vbase[tt] + hh * (uint32_t)((g.RS - KS + 1) * 32);
    }
  }
  f32x4 acc[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // in-volume column span of the staged rows (same for every plane)
  const int lstart = max(0, t.l0 - P), lend = min(g.L, t.l0 - P + g.RW);
  const int nchunk = 2 * (lend - lstart);
  const int col0 = lstart - (t.l0 - P);

  const size_t xext = g.npg > 0 ? (size_t)g.npg * g.gstride : (size_t)g.V * g.I * g.J * g.K * g.L * 16;
  (void)xext;
  // plane s of output j-tile t.j + jt (jt > 0 only in multi-tile group-plane mode)
  auto issue_x = [&](int jt, int s, char* buf) {
    const bf16* xb = X;
    if constexpr (X3) {
      const int ph = s / nplanes1;
      s -= ph * nplanes1;
      if (ph == 2) xb = X + g.xlo;
    }
    const bf16* xp;
    if (BLK) {
      xp = xb + plane_offset(g, t.v, di_lo + s / ndj, dj_lo + s % ndj, 16);
    } else if (g.npg > 0) {
      xp = xb + s * g.gstride + plane_offset(g, t.v, t.i, t.j + jt, 16);
    } else {
      const int di = di_lo + s / ndj, dj = dj_lo + s % ndj;
      xp = xb + plane_offset(g, t.v, t.i + di - P, t.j + jt + dj - P, 16);
    }
    for (int r = wave; r < g.PR; r += NW) {
      const int kg = t.k0 - P + r;
      if (kg >= 0 && kg < g.K && lane < nchunk) {
        const bf16* src = xp + ((size_t)kg * g.L + lstart) * 16 + lane * 8;
        if (NCNET_OK((size_t)(src - xb) + 8 <= xext) &&
            NCNET_OK((r * g.RS + col0) * 32 + lane * 16 + 16 <= plane_bytes))
          __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(void, buf + (r * g.RS + col0) * 32), 16, 0, 0);
      }
    }
  };
  const int nwp = BLK ? SP * SP : g.npg > 0 ? g.npg : NT;   // weight planes of one set
  auto issue_w = [&](int s) {
    int wset = 0;
    if constexpr (X3) {
      const int ph = s / nplanes1;
      s -= ph * nplanes1;
      wset = ph == 1 ? nwp : 0;   // phase 1 reads the lo weight planes
    }
    const int wplane = BLK ? (di_lo + s / ndj - (t.i - P)) * SP + dj_lo + s % ndj - (t.j - P)
                           : g.npg > 0 ? s : (di_lo + s / ndj) * KS + dj_lo + s % ndj;
    const u32x4* wp = Wp + (size_t)(wset + wplane) * (NQ * 64);
    if (NCNET_OK(wplane >= 0 && wplane < nwp))
      for (int q = wave; q < NQ; q += NW)
        __builtin_amdgcn_global_load_lds((const void*)(wp + q * 64 + lane), LDS_PTR(void, wbuf + q * 1024), 16, 0, 0);
  };

  const size_t nvox_all = (size_t)g.V * g.I * g.J * g.K * g.L;
  const f32x4 bv = lane_bias4<EPI>(bias, lane);
  auto store_tile = [&](int jt) {
    if constexpr (BLK) {
      // row co = 4 (lane >> 4) + r is output plane (i0 + (lane >> 4), j0 + r)
      const int oi = t.i + (lane >> 4);
      const float b0 = bias ? bias[0] : 0.f;
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) {
        int tile = wave + NW * tt;
        if (tile < ntile) {
          int vi = tile * 16 + (lane & 15);
          int kk = vi / g.TL, ll = vi - kk * g.TL;
          int kg = t.k0 + kk, lg = t.l0 + ll;
          if (vi < nvox && kg < g.K && lg < g.L && oi < g.I) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (t.j + r < g.J) {
                float x = acc[tt][r] + b0;
                if (g.relu) x = fmaxf(x, 0.f);
                const size_t o = plane_offset(g, t.v, oi, t.j + r, 1) + (size_t)kg * g.L + lg;
                if (NCNET_OK(o < nvox_all)) {
                  if (g.nt) __builtin_nontemporal_store(x, (float*)Y + o);
                  else ((float*)Y)[o] = x;
                }
              }
            }
          }
        }
      }
      return;
    }
    const size_t vbase_out = plane_offset(g, t.v, t.i, t.j + jt, 1);
    auto out_vox = [&](int tt, size_t& vox) -> bool {
      const int tile = wave + NW * tt;
      const int vi = tile * 16 + (lane & 15);
      const int kk = vi / g.TL, ll = vi - kk * g.TL;
      const int kg = t.k0 + kk, lg = t.l0 + ll;
      vox = vbase_out + (size_t)kg * g.L + lg;
      return tile < ntile && vi < nvox && kg < g.K && lg < g.L;
    };
    // ReLU-mask epilogue: all of the tile's mask loads before the first store
    constexpr bool MPF = (EPI & ~EPI_X3) == EPI_MASK;
    u32x2 mreg[MPF ? MAXT : 1];
    if constexpr (MPF) {
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) {
        size_t vox;
        if (!out_vox(tt, vox)) vox = 0;   // select, not a branch: one unconditional load each
        mreg[tt] = *(const u32x2*)(M + vox * 16 + 4 * (lane >> 4));
      }
    }
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) {
      size_t vox;
      if (out_vox(tt, vox)) {
        const u32x2* mp = nullptr;
        if constexpr (MPF) mp = &mreg[tt];
        store16<EPI>(acc[tt], Y, M, bias, vox, 4 * (lane >> 4), nvox_all, g.nco, g.nt, g.ylo, mp, &bv);
      }
    }
  };
  // MT (group-plane mode, tpw > 1): the workgroup computes ntl consecutive
  // output j-tiles with the same (k0, l0) -- so the zeroed halo is shared -- as
  // ONE plane stream: the DMA of the next tile's first plane is in flight while
  // the current tile finishes and stores, instead of every workgroup paying its
  // first plane's latency with nothing to overlap it.
  const int ntl = MT ? min(g.tpw, g.J - t.j) : 1;
  const int ntot = nplanes * ntl;

  __syncthreads();  // zero-fill complete before any DMA lands
  if (ntot > 0) { issue_x(0, 0, smem); issue_w(0); }
  int jt = 0, sp = 0;      // tile / plane of step s
  int njt = 0, nsp = 1;    // tile / plane of step s + 1
  if (nsp == nplanes) { nsp = 0; njt = 1; }
  for (int s = 0; s < ntot; ++s) {
    __syncthreads();  // drains this wave's DMA (vmcnt 0) and orders every wave's plane s + weights s
    char* cur = smem + (s & 1) * plane_bytes;
    if (s + 1 < ntot) issue_x(njt, nsp, smem + ((s + 1) & 1) * plane_bytes);
    bf16x8 wf[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) wf[q] = lds_read16(wbuf, (q * 64 + lane) * 16);
    // weights in registers in every wave -> release the weight buffer without
    // draining the in-flight plane DMA (plain s_barrier, LDS counter only)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + 1 < ntot) issue_w(nsp);
    // per-tile branches kept: the branch-free body needs 129 VGPRs (> 128,
    // one workgroup per CU instead of two: 6.4 -> 9.4 ms measured)
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) {
      if (wave + NW * tt < ntile) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          uint32_t a;
          if constexpr (CT > 0) {
            const uint32_t t0 = (uint32_t)((((2 * q) / KS) * g.RS + (2 * q) % KS) * 32);
            a = (((2 * q + 1) % KS == 0 && 2 * q + 1 < NT) ? c2[tt] : c1[tt]) + t0;
          } else {
            a = vbase[tt] + toff[q];
          }
          bf16x8 xf = lds_read16(cur, a);
          acc[tt] = mfma16(wf[q], xf, acc[tt]);
        }
      }
    }
    if (MT && sp == nplanes - 1) {
      store_tile(jt);
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    jt = njt; sp = nsp;
    if (++nsp == nplanes) { nsp = 0; ++njt; }
  }
  if (!MT || ntot == 0) store_tile(0);
}

// ===========================================================================
// conv16v3_fwd: 16 -> 16 (full (di, dj) plane sum) with the X operand reused
// from registers across output j-planes.
//
// conv16v2 reads one X fragment from LDS per MFMA (a ds_read_b128 = 4 LDS
// cycles per 16-cycle MFMA per SIMD: the LDS array is as busy as the matrix
// cores).  Here a workgroup owns R consecutive output planes (v, i, j0..j0+R-1)
// of one (k, l) tile.  Input plane (i+di-P, j') feeds output planes
// j = j' - dj + P for every dj, so each X fragment read from LDS is multiplied
// by up to KS weight fragments (one per dj) into KS different accumulator
// sets.  Per workgroup and di the R + KS - 1 input j-planes stream through two
// LDS buffers (LDS-DMA, one plane ahead) and the KS dj-slices of the di
// weights (KS x 13 KB for KS = 5) sit in LDS; LDS reads per MFMA drop from
// 1.2 to ~0.56 and each staged plane is used R_eff ~ 2.8 times instead of once.
//  * accumulators [R][MAXT] (100 VGPRs): the j' loop is unrolled at compile
//    time (static_for) so every accumulator index is static;
//  * weight slot dj of the next di is refilled as soon as its last consumer
//    plane (R - 1 + dj) has passed a barrier -- no stall between di steps;
//  * 8 waves x 5 voxel tiles, 1 workgroup per CU (128 KB LDS for KS = 5).
// Plane geometry (RS = TL + 8, halo zero-fill, row DMA) as conv16v2.
// ===========================================================================
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int KS, int R, int EPI>
__global__ __launch_bounds__(512, 1) void conv16v3_fwd_kernel(const bf16* __restrict__ X, const u32x4* __restrict__ Wp,
                                                              const float* __restrict__ bias,
                                                              const bf16* __restrict__ M, bf16* __restrict__ Y,
                                                              ConvGeom g) {
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int NQ = (NT + 1) / 2;
  constexpr int NW = 8;
  constexpr int MAXT = 5;
  constexpr int S = R + KS - 1;  // input j-planes per di

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int plane_bytes = g.PR * g.RS * 32;
  char* wbuf = smem + 2 * plane_bytes;  // [KS dj][NQ][64 lanes] x 16 B

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int lt = bid % g.nlt; bid /= g.nlt;
  const int kt = bid % g.nkt; bid /= g.nkt;
  const int jb = bid % g.njb; bid /= g.njb;
  const int ti = bid % g.I, tv = bid / g.I;
  const int k0 = kt * g.TK, l0 = lt * g.TL, j0 = jb * R;
  const int di_lo = max(0, P - ti), di_hi = min(KS, g.I + P - ti);
  const int nvox = g.TK * g.TL;
  const int ntile = (nvox + 15) >> 4;

  for (int o = threadIdx.x * 16; o < 2 * plane_bytes; o += NW * 64 * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};

  uint32_t vbase[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int vi = (wave + NW * tt) * 16 + (lane & 15);
    if (vi >= nvox) vi = 0;
    int kk = vi / g.TL, ll = vi - kk * g.TL;
    vbase[tt] = (uint32_t)((kk * g.RS + ll) * 32 + ((lane >> 4) & 1) * 16);
  }
  // tap-pair offsets without a per-lane table (13 VGPRs at KS = 5, which
  // pushed the <5, 5, *> bodies into scratch): tap 2q + h of lane half h sits
  // at the wave-uniform offset of tap 2q plus h x (one column or one row wrap)
  const uint32_t rs32 = (uint32_t)g.RS * 32u;
  const uint32_t hcol = (lane >> 5) ? 32u : 0u, hwrap = (lane >> 5) ? rs32 - (uint32_t)(KS - 1) * 32u : 0u;
  auto toff_q = [&](auto qc) -> uint32_t {
    constexpr int q = decltype(qc)::value;
    constexpr int ta = 2 * q, tb = (2 * q + 1 < NT) ? 2 * q + 1 : NT - 1;
    constexpr int dka = ta / KS, dla = ta % KS, dkb = tb / KS, dlb = tb % KS;
    const uint32_t base = (uint32_t)dka * rs32 + (uint32_t)dla * 32u;
    if constexpr (tb == ta) return base;                                  // padding tap: both halves alike
    else if constexpr (dkb == dka) { static_assert(dlb == dla + 1); return base + hcol; }
    else { static_assert(dkb == dka + 1 && dlb == 0 && dla == KS - 1); return base + hwrap; }
  };
  f32x4 acc[R][MAXT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) acc[r][tt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lstart = max(0, l0 - P), lend = min(g.L, l0 - P + g.RW);
  const int nchunk = 2 * (lend - lstart);
  const int col0 = lstart - (l0 - P);

  const size_t xext = (size_t)g.V * g.I * g.J * g.K * g.L * 16;
  (void)xext;
  auto issue_x = [&](int di, int jp, char* buf) {
    const bf16* xp = X + plane_offset(g, tv, ti + di - P, jp, 16);
    for (int r = wave; r < g.PR; r += NW) {
      const int kg = k0 - P + r;
      if (kg >= 0 && kg < g.K && lane < nchunk) {
        const bf16* src = xp + ((size_t)kg * g.L + lstart) * 16 + lane * 8;
        if (NCNET_OK(src >= X && (size_t)(src - X) + 8 <= xext) &&
            NCNET_OK((r * g.RS + col0) * 32 + lane * 16 + 16 <= plane_bytes))
          __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(void, buf + (r * g.RS + col0) * 32), 16, 0, 0);
      }
    }
  };
  auto issue_w = [&](int di, int dj) {
    const u32x4* wp = Wp + (size_t)(di * KS + dj) * (NQ * 64);
    if (NCNET_OK(di >= 0 && di < KS && dj >= 0 && dj < KS))
    for (int q = wave; q < NQ; q += NW)
      __builtin_amdgcn_global_load_lds((const void*)(wp + q * 64 + lane), LDS_PTR(void, wbuf + (dj * NQ + q) * 1024),
                                       16, 0, 0);
  };

  __syncthreads();  // zero-fill complete before any DMA lands
  for (int dj = 0; dj < KS; ++dj) issue_w(di_lo, dj);
  if (j0 - P >= 0 && j0 - P < g.J) issue_x(di_lo, j0 - P, smem);
  int n = 0;  // linear plane counter: buffer parity
  for (int di = di_lo; di < di_hi; ++di) {
    static_for<0, S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      __syncthreads();  // plane n (and weights issued earlier) landed; plane n-1 consumed
      char* cur = smem + (n & 1) * plane_bytes;
      {
        const int ndi = (s + 1 == S) ? di + 1 : di;
        const int njp = j0 - P + ((s + 1 == S) ? 0 : s + 1);
        if (ndi < di_hi && njp >= 0 && njp < g.J) issue_x(ndi, njp, smem + ((n + 1) & 1) * plane_bytes);
      }
      // weight slot dj is last read by plane R - 1 + dj: refill it for di + 1
      if constexpr (s >= R) {
        if (di + 1 < di_hi) issue_w(di + 1, s - R);
      }
      if constexpr (s == 0) {
        if (di > di_lo) issue_w(di, KS - 1);
      }
      const int jp = j0 - P + s;
      if (jp >= 0 && jp < g.J) {
        constexpr int dlo = (s - R + 1) > 0 ? (s - R + 1) : 0;
        constexpr int dhi = s < KS - 1 ? s : KS - 1;  // inclusive
        static_for<0, NQ>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          const uint32_t tq = toff_q(qc);
          bf16x8 a[KS];
          static_for<dlo, dhi + 1>([&](auto dc) {
            constexpr int dj = decltype(dc)::value;
            a[dj] = lds_read16(wbuf, ((dj * NQ + q) * 64 + lane) * 16);
          });
          // no per-tile validity branch: tiles past ntile read voxel 0 and are
          // never stored (a divergent branch here splits the block and
          // serialises every LDS read with its MFMAs)
#pragma unroll
          for (int tt = 0; tt < MAXT; ++tt) {
            const bf16x8 xf = lds_read16(cur, vbase[tt] + tq);
            static_for<dlo, dhi + 1>([&](auto dc) {
              constexpr int dj = decltype(dc)::value;
              acc[s - dj][tt] = mfma16(a[dj], xf, acc[s - dj][tt]);
            });
          }
        });
      }
      ++n;
    });
  }

  const size_t nvox_all = (size_t)g.V * g.I * g.J * g.K * g.L;
  const f32x4 bv = lane_bias4<EPI>(bias, lane);
  // data-gradient epilogue: every ReLU-mask load of the item issued before the
  // first store (as in conv16v4), not one load -> vmcnt(0) -> store per tile
  constexpr bool MPF = (EPI & ~EPI_X3) == EPI_MASK;
  u32x2 mreg[MPF ? R : 1][MPF ? MAXT : 1];
  auto out_vox = [&](int r, int tt, size_t& vox) -> bool {
    const int j = j0 + r;
    const int tile = wave + NW * tt;
    const int vi = tile * 16 + (lane & 15);
    const int kk = vi / g.TL, ll = vi - kk * g.TL;
    const int kg = k0 + kk, lg = l0 + ll;
    vox = plane_offset(g, tv, ti, j, 1) + (size_t)kg * g.L + lg;
    return j < g.J && tile < ntile && vi < nvox && kg < g.K && lg < g.L;
  };
  if constexpr (MPF) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) {
        size_t vox;
        mreg[r][tt] = out_vox(r, tt, vox) ? *(const u32x2*)(M + vox * 16 + 4 * (lane >> 4)) : u32x2{0u, 0u};
      }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) {
      size_t vox;
      if (out_vox(r, tt, vox)) {
        const u32x2* mp = nullptr;
        if constexpr (MPF) mp = &mreg[r][tt];
        store16<EPI>(acc[r][tt], Y, M, bias, vox, 4 * (lane >> 4), nvox_all, g.nco, g.nt, 0, mp, &bv);
      }
    }
  }
}

// ===========================================================================
// conv16v4_fwd: conv16v3 at a compile-time (TK, TL) tile (the 25 x 25 (k, l)
// planes of the training volume), rebuilt for latency hiding.  conv16v3's
// compiled body issued each fragment's ds_read right before its 3-5 MFMAs and
// waited lgkmcnt(0) in between (no read in flight while the matrix pipe ran),
// and drained every in-flight plane DMA at each step's barrier, so the short
// ramp steps of each di (1-2 dj slices) exposed a full plane load.  Here:
//  * fragments are software-pipelined in registers: the weight / X fragments of
//    K-step q + 1 are read while the MFMAs of q run (explicit double buffer);
//  * X fragment addresses are per-lane bases plus compile-time offsets (RS is
//    a constant): no address VALU in the loop; the two lane halves (taps 2q,
//    2q + 1) differ by one voxel or by one row wrap, two base sets cover both;
//  * three plane buffers, DMA two planes ahead, and a counted
//    `s_waitcnt vmcnt(N)` before each step's barrier waits for the plane (and
//    weights) that step reads but leaves the next plane's DMA in flight.  Every
//    wave issues a FIXED number of DMA instructions per plane and per weight
//    slot (rows / slots it does not own go to a trash KiB of LDS) so N is a
//    compile-time count; buffer-resource DMAs return zeros out of range, so the
//    halo is written by the DMA (no zero fill, no exec masks).
// LDS (KS = 5, 25 x 25): 65 KB weights + 3 x 30.6 KB planes + 1 KB = 156 KB.
// ===========================================================================
// does step s of a di issue a weight slot (slot s - R of di + 1, or slot KS - 1 of di at s = 0)?
__host__ __device__ constexpr bool v4_wstep(int s, int R) { return s == 0 || s >= R; }

template <int KS, int R, int EPI, int TK, int TL>
__global__ __launch_bounds__(512, 1) void conv16v4_fwd_kernel(const bf16* __restrict__ X, const u32x4* __restrict__ Wp,
                                                              const float* __restrict__ bias,
                                                              const bf16* __restrict__ M, bf16* __restrict__ Y,
                                                              ConvGeom g) {
#if defined(__HIP_DEVICE_COMPILE__)   // device-only body (buffer-resource builtins): the host pass keeps the stub
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int NQ = (NT + 1) / 2;
  constexpr int NW = 8;
  constexpr int NVOX = TK * TL;
  constexpr int NTILE = (NVOX + 15) / 16;
  constexpr int MAXT = (NTILE + NW - 1) / NW;
  // SPLIT (the 20 x 20 plane: 25 tiles over 8 waves): the one tile past
  // 8 x MT is not given whole to wave 0 (a 4th tile while the others hold 3,
  // i.e. 22 % idle MFMA time) but split by output plane: wave w < R computes
  // it for r = w only (one MFMA per K-step on the steps where dj = s - w is
  // a live tap), with its own accumulator and per-K-step weight reads
  constexpr bool SPLIT = NTILE % NW == 1 && NTILE > NW && R <= NW;
  constexpr int MT = SPLIT ? NTILE / NW : MAXT;   // whole tiles per wave
  constexpr int TS = NW * MT;                      // the split tile (SPLIT)
  constexpr int S = R + KS - 1;              // input j-planes per di
  constexpr int RS = TL + 8;                 // row stride (voxels): a wrapping tile jumps one 256-B bank period
  constexpr int PR = TK + KS - 1;            // staged rows
  constexpr int PLANE = PR * RS * 32;
  // LDS: weights first (so every fragment read is a base VGPR + a 16-bit
  // immediate: bases at 0 and 32 KiB), then the three plane buffers, then trash
  constexpr int WBYTES = KS * NQ * 1024;
  constexpr int XOFF = WBYTES;
  constexpr int TRASH = XOFF + 3 * PLANE;
  constexpr int RPW = (PR + NW - 1) / NW;    // row DMAs per wave per plane (fixed)
  constexpr int WPW = (NQ + NW - 1) / NW;    // weight DMAs per wave per slot (fixed)
  static_assert(TL + KS - 1 <= 32, "one LDS-DMA wave-instruction per staged row");
  static_assert(TRASH + 1024 <= 160 * 1024, "LDS");
  static_assert(S >= 2, "prologue emulates two steps");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int lt = bid % g.nlt; bid /= g.nlt;
  const int kt = bid % g.nkt; bid /= g.nkt;
  const int jb = bid % g.njb; bid /= g.njb;
  const int ti = bid % g.I, tv = bid / g.I;
  const int k0 = kt * TK, l0 = lt * TL, j0 = jb * R;
  const int di_lo = max(0, P - ti), di_hi = min(KS, g.I + P - ti);
  // EPI_X3: the di sweep runs once per phase, (X_hi, W_hi), (X_hi, W_lo),
  // (X_lo, W_hi), into the same accumulators; dv = phase * ndi + (di - di_lo)
  constexpr bool X3 = (EPI & EPI_X3) != 0;
  constexpr int PH = X3 ? 3 : 1;
  const int ndi = di_hi - di_lo;   // >= 1 (di = P is always valid)
  const int nd = PH * ndi;
  const int ntot = nd * S;

  // per-lane X addresses of the current plane buffer (advanced by one buffer per
  // step): c1 = half 1 on the next voxel (taps 2q, 2q + 1 in one row; also the
  // padded last pair, whose half-1 weights are zero: it reads voxel ll + 5 of
  // the same DMA-written row), c2 = half 1 one row down with dl wrapped
  // (2q + 1 a multiple of KS)
  uint32_t c1[MT], c2[MT];
  uint32_t c1s = 0, c2s = 0;                       // the split tile's bases (SPLIT)
  {
    const uint32_t hh = (uint32_t)(lane >> 5);
    auto bases = [&](int tile, uint32_t& a1, uint32_t& a2) {
      int vi = tile * 16 + (lane & 15);
      if (vi >= NVOX) vi = 0;
      const int kk = vi / TL, ll = vi - kk * TL;
      const uint32_t b0 = (uint32_t)(XOFF + (kk * RS + ll) * 32 + ((lane >> 4) & 1) * 16);
      a1 = b0 + hh * 32u;
      a2 = b0 + hh * (uint32_t)((RS - KS + 1) * 32);
    };
#pragma unroll
    for (int tt = 0; tt < MT; ++tt) bases(wave + NW * tt, c1[tt], c2[tt]);
    if constexpr (SPLIT) bases(TS, c1s, c2s);
  }
  f32x4 acc[R][MT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int tt = 0; tt < MT; ++tt) acc[r][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accs = {0.f, 0.f, 0.f, 0.f};               // split tile, output plane r = wave (SPLIT)

  // Plane DMA through a buffer resource over ONE (i, j) plane: every lane of a
  // row instruction writes its 16-B chunk (row voxel lane / 2 = l0 - P + lane / 2),
  // and a chunk outside the volume (halo column, halo row, or an invalid plane:
  // num_records 0) reads out of range and lands as ZERO -- the halo is rewritten
  // with zeros by the DMA itself, no zero fill, no per-lane exec masks.  Rows
  // r >= PR of the fixed RPW per wave go to a trash KiB.
  constexpr uint32_t OOB = 0x7ffffff0u;
  uint32_t xvo[RPW];
  uint32_t xld[RPW];
#pragma unroll
  for (int m = 0; m < RPW; ++m) {
    const int r = wave + NW * m;
    const int kg = k0 - P + r, lg = l0 - P + (lane >> 1);
    const bool ok = r < PR && kg >= 0 && kg < g.K && lg >= 0 && lg < g.L && (lane >> 1) < TL + KS - 1;
    xvo[m] = ok ? (uint32_t)(((kg * g.L + lg) * 16 + (lane & 1) * 8) * 2) : OOB;
    xld[m] = r < PR ? (uint32_t)(XOFF + r * RS * 32) : (uint32_t)TRASH;
  }
  const size_t plane_elems = (size_t)g.K * g.L * 16;
  auto issue_x = [&](int n) {
    int dq = n / S;
    const int s = n - dq * S;
    const int jp = j0 - P + s;
    const bool pv = n < ntot && jp >= 0 && jp < g.J;
    const bf16* xb = X;
    if constexpr (X3) {
      const int ph = dq / ndi;
      dq -= ph * ndi;
      if (ph == 2) xb = X + g.xlo;
    }
    const bf16* xp = pv ? xb + plane_offset(g, tv, ti + di_lo + dq - P, jp, 16) : X;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)xp, (short)0, pv ? (int)(plane_elems * 2) : 0, 0x00020000);
    const uint32_t boff = (uint32_t)((n % 3) * PLANE);
#pragma unroll
    for (int m = 0; m < RPW; ++m) {
      const uint32_t d = xld[m] == (uint32_t)TRASH ? (uint32_t)TRASH : xld[m] + boff;
      // a row instruction covers 32 voxels: with RS < 32 (planes narrower than
      // 25) the lanes past the row stride would overwrite the next row's first
      // voxels, so they stay off (the instruction, and the vmcnt count, remain)
      if (RS >= 32 || (lane >> 1) < RS)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, smem + d), 16, xvo[m], 0, 0, 0);
    }
  };
  // weight slot dj <- (di, dj) fragments of step dv; WPW DMAs per wave, always
  // (invalid -> trash).  X3: the lo weight set follows the hi one in Wp.
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, PH == 3 ? 2 * KS * KS * NQ * 1024 : KS * KS * NQ * 1024,
                                        0x00020000);
  auto issue_w = [&](int dv, int dj, bool valid) {
    int wplane;
    if constexpr (X3) {
      const int ph = dv / ndi;
      wplane = (ph == 1 ? KS * KS : 0) + (di_lo + dv - ph * ndi) * KS + dj;
    } else {
      wplane = (di_lo + dv) * KS + dj;
    }
#pragma unroll
    for (int m = 0; m < WPW; ++m) {
      const int q = wave + NW * m;
      const bool v = valid && q < NQ;
      const uint32_t d = v ? (uint32_t)((dj * NQ + q) * 1024) : (uint32_t)TRASH;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, LDS_PTR(void, smem + d), 16, (uint32_t)((q * 64 + lane) * 16),
                                               (uint32_t)(wplane * NQ * 1024), 0, 0);
    }
  };

  for (int dj = 0; dj < KS; ++dj) issue_w(0, dj, true);
  issue_x(0);
  issue_w(0, 0, false);   // step "-1" emulation: its weight slot (if any), then plane 1
  issue_x(1);
  static_assert(S - 1 >= R, "the emulated step issues a weight slot");

  const uint32_t wb = (uint32_t)lane * 16u;
  int n = 0;
  for (int dv = 0; dv < nd; ++dv) {
    static_for<0, S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      // DMAs younger than plane n: the previous step's weight slot (if any) and plane n + 1
      constexpr int YOUNGER = RPW + (v4_wstep(s == 0 ? S - 1 : s - 1, R) ? WPW : 0);
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(YOUNGER) : "memory");
      if constexpr (v4_wstep(s, R)) {
        if constexpr (s >= R) issue_w(dv + 1 < nd ? dv + 1 : dv, s - R, dv + 1 < nd);
        else issue_w(dv, KS - 1, dv > 0);
      }
      issue_x(n + 2);
      const int jp = j0 - P + s;
      if (jp >= 0 && jp < g.J) {
        constexpr int dlo = (s - R + 1) > 0 ? (s - R + 1) : 0;
        constexpr int dhi = s < KS - 1 ? s : KS - 1;  // inclusive
        // (q, tt) MFMA groups in order k = q * MT + tt; the weight fragments
        // of K-step q + 1 are read at group (q, 0) (double buffer), the X
        // fragment of group k + 2 at group k (three registers in rotation);
        // sched_group_barrier pins that order (the default scheduler sinks each
        // read to just before its MFMAs and waits lgkmcnt(0) there)
        constexpr int NDJ = dhi - dlo + 1;
        constexpr int NK = NQ * MT;
        bf16x8 A[2][KS], Xr[3];
        auto load_a = [&](auto qc) {
          constexpr int q = decltype(qc)::value;
          static_for<dlo, dhi + 1>([&](auto dc) {
            constexpr int dj = decltype(dc)::value;
            constexpr int o = (dj * NQ + q) * 1024;
            if constexpr (o < 32768) A[q & 1][dj] = *(const bf16x8*)(smem + wb + o);
            else A[q & 1][dj] = *(const bf16x8*)(smem + (wb + 32768u) + (o - 32768));
          });
        };
        auto load_x = [&](auto kc) {
          constexpr int k = decltype(kc)::value;
          constexpr int q = k / MT, tt = k % MT;
          constexpr int t0 = 2 * q;
          constexpr uint32_t T0 = (uint32_t)(((t0 / KS) * RS + t0 % KS) * 32);
          const uint32_t base = ((2 * q + 1) % KS == 0 && 2 * q + 1 < NT) ? c2[tt] : c1[tt];
          Xr[k % 3] = *(const bf16x8*)(smem + base + T0);
        };
        load_a(std::integral_constant<int, 0>{});
        load_x(std::integral_constant<int, 0>{});
        load_x(std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_group_barrier(0x100, NDJ + 2, 0);
        static_for<0, NK>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          constexpr int q = k / MT, tt = k % MT;
          constexpr bool LA = tt == 0 && q + 1 < NQ;
          constexpr bool LX = k + 2 < NK;
          if constexpr (LA) load_a(std::integral_constant<int, q + 1>{});
          if constexpr (LX) load_x(std::integral_constant<int, k + 2>{});
          static_for<dlo, dhi + 1>([&](auto dc) {
            constexpr int dj = decltype(dc)::value;
            acc[s - dj][tt] = mfma16(A[q & 1][dj], Xr[k % 3], acc[s - dj][tt]);
          });
          if constexpr (LA || LX) __builtin_amdgcn_sched_group_barrier(0x100, (LA ? NDJ : 0) + (LX ? 1 : 0), 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NDJ, 0);
        });
        if constexpr (SPLIT) {
          // the split tile for output plane r = wave: tap slot dj = s - wave,
          // one accumulation chain over the NQ K-steps (weights of slot dj and
          // the tile's X fragment read one K-step ahead)
          const int dj = s - wave;
          if (wave < R && dj >= 0 && dj < KS) {
            const uint32_t wdj = wb + (uint32_t)(dj * NQ * 1024);
            bf16x8 As[2], Xs[2];
            auto ld = [&](auto qc) {
              constexpr int q = decltype(qc)::value;
              constexpr int t0 = 2 * q;
              constexpr uint32_t T0 = (uint32_t)(((t0 / KS) * RS + t0 % KS) * 32);
              const uint32_t base = ((2 * q + 1) % KS == 0 && 2 * q + 1 < NT) ? c2s : c1s;
              As[q & 1] = *(const bf16x8*)(smem + wdj + q * 1024);
              Xs[q & 1] = *(const bf16x8*)(smem + base + T0);
            };
            ld(std::integral_constant<int, 0>{});
            static_for<0, NQ>([&](auto qc) {
              constexpr int q = decltype(qc)::value;
              if constexpr (q + 1 < NQ) ld(std::integral_constant<int, q + 1>{});
              accs = mfma16(As[q & 1], Xs[q & 1], accs);
            });
          }
        }
      }
      // advance the X addresses to the next step's buffer ((n + 1) % 3)
      {
        const uint32_t adv = (n % 3 == 2) ? (uint32_t)(-2 * PLANE) : (uint32_t)PLANE;
#pragma unroll
        for (int tt = 0; tt < MT; ++tt) { c1[tt] += adv; c2[tt] += adv; }
        if constexpr (SPLIT) { c1s += adv; c2s += adv; }
      }
      ++n;
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends

  const size_t nvox_all = (size_t)g.V * g.I * g.J * g.K * g.L;
  auto out_vox_t = [&](int r, int tile, size_t& vox) -> bool {
    const int j = j0 + r;
    const int vi = tile * 16 + (lane & 15);
    const int kk = vi / TL, ll = vi - kk * TL;
    const int kg = k0 + kk, lg = l0 + ll;
    const bool ok = j < g.J && tile < NTILE && vi < NVOX && kg < g.K && lg < g.L;
    vox = ok ? plane_offset(g, tv, ti, j, 1) + (size_t)kg * g.L + lg : 0;
    return ok;
  };
  auto out_vox = [&](int r, int tt, size_t& vox) -> bool { return out_vox_t(r, wave + NW * tt, vox); };
  // EPI_MASK: every ReLU-mask load of the item first (fixed count, out-of-range
  // voxels read voxel 0), then the stores: a load -> wait -> store sequence per
  // (r, tt) serialised 25 memory round trips (stores count in vmcnt here)
  constexpr bool MPF = (EPI & ~EPI_X3) == EPI_MASK;
  u32x2 mreg[MPF ? R : 1][MPF ? MT : 1];
  u32x2 mregs = {0u, 0u};
  const f32x4 bv = lane_bias4<EPI>(bias, lane);
  if constexpr (MPF) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int tt = 0; tt < MT; ++tt) {
        size_t vox;
        out_vox(r, tt, vox);
        mreg[r][tt] = *(const u32x2*)(M + vox * 16 + 4 * (lane >> 4));
      }
    if constexpr (SPLIT) {
      size_t vox;
      out_vox_t(wave < R ? wave : 0, TS, vox);
      mregs = *(const u32x2*)(M + vox * 16 + 4 * (lane >> 4));
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int tt = 0; tt < MT; ++tt) {
      size_t vox;
      if (out_vox(r, tt, vox)) {
        const u32x2* mp = nullptr;
        if constexpr (MPF) mp = &mreg[r][tt];
        store16<EPI>(acc[r][tt], Y, M, bias, vox, 4 * (lane >> 4), nvox_all, g.nco, g.nt, g.ylo, mp, &bv);
      }
    }
  }
  if constexpr (SPLIT) {
    size_t vox;
    if (wave < R && out_vox_t(wave, TS, vox)) {
      const u32x2* mp = nullptr;
      if constexpr (MPF) mp = &mregs;
      store16<EPI>(accs, Y, M, bias, vox, 4 * (lane >> 4), nvox_all, g.nco, g.nt, g.ylo, mp, &bv);
    }
  }
#endif
}

// ===========================================================================
// conv16f8_fwd: inference Conv4d 16 -> 16 on OCP fp8 e4m3 operands
// (v_mfma_f32_16x16x32_fp8_fp8, BASELINE config 5).  Same structure as
// conv16v2 (8 waves, LDS-DMA, double-buffered planes, single weight buffer with
// a mid-plane s_barrier, group-plane mode) with 16-byte voxels: every LDS,
// DMA and operand byte count halves (one ds_read_b64 per MFMA instead of a
// b128) and the weight fragments take 26 instead of 52 VGPRs.  The plane row
// stride is TL + 16 voxels so a wrapping 16-voxel tile still jumps one 256-B
// bank period.  Weights are pre-scaled by 1/oscale into the e4m3 range.
// Epilogues: EPI_BIAS_RELU -> fp8 [.., 16] (next layer's input),
//            EPI_F32X16   -> channel-planar fp32 partials (ijsum input).
// ===========================================================================
template <int KS, int EPI>
__global__ __launch_bounds__(512, KS >= 7 ? 1 : 2) void conv16f8_fwd_kernel(const uint8_t* __restrict__ X,
                                                              const uint8_t* __restrict__ Wp,
                                                              const float* __restrict__ bias, void* __restrict__ Y,
                                                              ConvGeom g) {
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int NQ = (NT + 1) / 2;
  constexpr int NW = 8;
  constexpr int MAXT = 5;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int plane_bytes = g.PR * g.RS * 16;
  char* wbuf = smem + 2 * plane_bytes;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const TileId t = decode_tile(g);
  const int di_lo = max(0, P - t.i), di_hi = min(KS, g.I + P - t.i);
  const int dj_lo = max(0, P - t.j), dj_hi = min(KS, g.J + P - t.j);
  const int ndj = dj_hi - dj_lo;
  const int nplanes = g.npg > 0 ? g.npg : (di_hi - di_lo) * ndj;
  const int nvox = g.TK * g.TL;
  const int ntile = (nvox + 15) >> 4;
  const bool full_wave = __builtin_amdgcn_readfirstlane(wave + NW * (MAXT - 1) < ntile);

  for (int o = threadIdx.x * 16; o < 2 * plane_bytes; o += NW * 64 * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};

  uint32_t vbase[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int vi = (wave + NW * tt) * 16 + (lane & 15);
    if (vi >= nvox) vi = 0;
    int kk = vi / g.TL, ll = vi - kk * g.TL;
    vbase[tt] = (uint32_t)((kk * g.RS + ll) * 16 + ((lane >> 4) & 1) * 8);
  }
  uint32_t toff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    int tap = 2 * q + (lane >> 5);
    if (tap >= NT) tap = NT - 1;
    int dk = tap / KS, dl = tap - dk * KS;
    toff[q] = (uint32_t)((dk * g.RS + dl) * 16);
  }
  f32x4 acc[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lstart = max(0, t.l0 - P), lend = min(g.L, t.l0 - P + g.RW);
  const int nvx = lend - lstart;          // 16-byte voxels per staged row (<= 32)
  const int col0 = lstart - (t.l0 - P);

  auto issue_x = [&](int s, char* buf) {
    const int di = di_lo + s / ndj, dj = dj_lo + s % ndj;
    const uint8_t* xp = g.npg > 0 ? X + s * g.gstride + plane_offset(g, t.v, t.i, t.j, 16)
                                  : X + plane_offset(g, t.v, t.i + di - P, t.j + dj - P, 16);
    for (int r = wave; r < g.PR; r += NW) {
      const int kg = t.k0 - P + r;
      if (kg >= 0 && kg < g.K && lane < nvx)
        __builtin_amdgcn_global_load_lds((const void*)(xp + ((size_t)kg * g.L + lstart + lane) * 16),
                                         LDS_PTR(void, buf + (r * g.RS + col0) * 16), 16, 0, 0);
    }
  };
  auto issue_w = [&](int s) {   // NQ * 512 B of fragments = NQ * 32 16-byte chunks
    const int di = di_lo + s / ndj, dj = dj_lo + s % ndj;
    const uint8_t* wp = Wp + (size_t)(g.npg > 0 ? s : di * KS + dj) * (NQ * 512);
    for (int c = wave * 64; c < NQ * 32; c += NW * 64)
      if (c + lane < NQ * 32)
        __builtin_amdgcn_global_load_lds((const void*)(wp + (size_t)(c + lane) * 16), LDS_PTR(void, wbuf + c * 16),
                                         16, 0, 0);
  };

  __syncthreads();
  if (nplanes > 0) { issue_x(0, smem); issue_w(0); }
  for (int s = 0; s < nplanes; ++s) {
    __syncthreads();
    char* cur = smem + (s & 1) * plane_bytes;
    if (s + 1 < nplanes) issue_x(s + 1, smem + ((s + 1) & 1) * plane_bytes);
    long wf[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) wf[q] = *(const long*)(wbuf + (q * 64 + lane) * 8);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + 1 < nplanes) issue_w(s + 1);
    auto tiles = [&](auto fullc) {   // branch-free body for full waves (see conv16v2)
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) {
        if (FULL || wave + NW * tt < ntile) {
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const long xf = *(const long*)(cur + vbase[tt] + toff[q]);
            acc[tt] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(wf[q], xf, acc[tt], 0, 0, 0);
          }
        }
      }
    };
    if (full_wave) tiles(std::true_type{}); else tiles(std::false_type{});
  }

  const size_t vbase_out = plane_offset(g, t.v, t.i, t.j, 1);
  const size_t nvox_all = (size_t)g.V * g.I * g.J * g.K * g.L;
  const int co0 = 4 * (lane >> 4);
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int tile = wave + NW * tt;
    if (tile < ntile) {
      int vi = tile * 16 + (lane & 15);
      int kk = vi / g.TL, ll = vi - kk * g.TL;
      int kg = t.k0 + kk, lg = t.l0 + ll;
      if (vi < nvox && kg < g.K && lg < g.L) {
        const size_t vox = vbase_out + (size_t)kg * g.L + lg;
        if (EPI == EPI_F32X16) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (co0 + r < g.nco) ((float*)Y)[(size_t)(co0 + r) * nvox_all + vox] = acc[tt][r] * g.oscale;
        } else {
          uint32_t packed = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = fmaxf(acc[tt][r] * g.oscale + bias[co0 + r], 0.f);
            packed |= (uint32_t)__hip_cvt_float_to_fp8(x, __HIP_SATFINITE, __HIP_E4M3) << (8 * r);
          }
          *(uint32_t*)((uint8_t*)Y + vox * 16 + co0) = packed;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Host launchers.
// ---------------------------------------------------------------------------
static ConvGeom make_geom(int V, int I, int J, int K, int L, int KS, int tk, int tl) {
  ConvGeom g;
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L;
  g.TK = tk; g.TL = tl;
  g.nkt = cdiv(K, tk); g.nlt = cdiv(L, tl);
  g.PR = tk + KS - 1;
  g.RW = tl + KS - 1;
  g.RS = g.RW;
  g.npg = 0; g.gstride = 0; g.nco = 16; g.oscale = 1.f;
  g.xlo = 0; g.ylo = 0;
  g.njb = J; g.tpw = 1;
  g.nib = I; g.relu = 0;
  // default on: conv16v3 5.51 -> 5.31 ms at 64 x 25^4 (profiles/r1s3_kbench_nt.json)
  g.nt = tuning().nt_store;
  return g;
}

}  // namespace ncnet

using namespace ncnet;

// conv16v4 at the compile-time tiles it is instantiated for: the
// --image_size 240 / 320 / 400 training planes (15, 20, 25: one whole-plane
// tile) and 480 (30 x 30: two 30 x 15 tiles) at KS 5 and KS 3.
template <int KS, int TK, int TL>
static void v4_launch1(int epi, dim3 grid, dim3 block, hipStream_t stream, const bf16* x, const u32x4* w,
                       const float* bias, const bf16* m, bf16* y, const ConvGeom& g) {
  constexpr int R = 5, NQ = (KS * KS + 1) / 2;
  const size_t lds = 3 * (size_t)(TK + KS - 1) * (TL + ((KS - 1 + 7) / 8) * 8) * 32 + (size_t)KS * NQ * 1024 + 1024;
  auto go = [&](auto ec) {
    constexpr int E = decltype(ec)::value;
    hipLaunchKernelGGL((conv16v4_fwd_kernel<KS, R, E, TK, TL>), grid, block, lds, stream, x, w, bias, m, y, g);
  };
  if (epi == EPI_BIAS_RELU) go(std::integral_constant<int, EPI_BIAS_RELU>{});
  else if (epi == EPI_MASK) go(std::integral_constant<int, EPI_MASK>{});
  else if (epi == (EPI_BIAS_RELU | EPI_X3)) go(std::integral_constant<int, EPI_BIAS_RELU | EPI_X3>{});
  else go(std::integral_constant<int, EPI_MASK | EPI_X3>{});
}
template <int KS>
static bool v4_launch_ks(int K, int L, int tk, int tl, int epi, dim3 grid, dim3 block, hipStream_t stream,
                         const bf16* x, const u32x4* w, const float* bias, const bf16* m, bf16* y, const ConvGeom& g) {
  if (K != L) return false;
  if (K == 25 && tk == 25 && tl == 25) v4_launch1<KS, 25, 25>(epi, grid, block, stream, x, w, bias, m, y, g);
  else if (K == 20 && tk == 20 && tl == 20) v4_launch1<KS, 20, 20>(epi, grid, block, stream, x, w, bias, m, y, g);
  else if (K == 15 && tk == 15 && tl == 15) v4_launch1<KS, 15, 15>(epi, grid, block, stream, x, w, bias, m, y, g);
  else if (K == 30 && tk == 30 && tl == 15) v4_launch1<KS, 30, 15>(epi, grid, block, stream, x, w, bias, m, y, g);
  else return false;
  return true;
}
static bool v4_launch(int KS, int K, int L, int tk, int tl, int epi, dim3 grid, dim3 block, hipStream_t stream,
                      const bf16* x, const u32x4* w, const float* bias, const bf16* m, bf16* y, const ConvGeom& g) {
  if (KS == 5) return v4_launch_ks<5>(K, L, tk, tl, epi, grid, block, stream, x, w, bias, m, y, g);
  if (KS == 3) return v4_launch_ks<3>(K, L, tk, tl, epi, grid, block, stream, x, w, bias, m, y, g);
  return false;
}

// Tile choice: the whole (k,l) plane when it fits (<= 25 x 25 output); planes
// up to 32 x 32 (--image_size 480: 30 x 30) split into two K x ceil(L / 2)
// tiles (a 25 x 25 tile on a 30 x 30 plane left 4 tiles of 2500 voxel slots
// for 900 voxels); else 25 x 25 tiles (InLoc-size planes).
static void pick_tile(int K, int L, int& tk, int& tl) {
  if (K > 25 || L > 25) {
    if (K <= 32 && L <= 32) { tk = K; tl = (L + 1) / 2; return; }
  }
  tk = K <= 25 ? K : 25;
  tl = L <= 25 ? L : 25;
  // keep TK*TL <= 640 (MAXT * 8 waves * 16 voxels)
  while (tk * tl > 640) { if (tl > tk) --tl; else --tk; }
}

// output j-tiles per workgroup of the group-plane conv
static int gp_tpw() { return tuning().gp_tpw; }

// KS = 5 and 3 are NC-Net's kernel sizes (lib/model.py:125-139 defaults, the
// InLoc and PF-Pascal checkpoints); 1 and 7 complete the general Conv4d.
#define KS_DISPATCH(M, ...) \
  do { if (KS == 5) M(5, __VA_ARGS__); else if (KS == 3) M(3, __VA_ARGS__); \
       else if (KS == 7) M(7, __VA_ARGS__); else if (KS == 1) M(1, __VA_ARGS__); else return -2; } while (0)

// X [V,I,J,K,L,16] (all KS*KS planes (i+di-P, j+dj-P)), or npg > 0: group-planes
// mode -- X holds npg input groups [npg][V,I,J,K,L,16] and
// Y = sum_s conv_(dk,dl)(X[s] plane (i,j), Wp plane s): the (di, dj) offsets
// live in the channels (ij encoding, csrc/jshift.hip) or s indexes 16-channel
// input blocks of a wider layer.
//
// epi | EPI_X3 (KS 3 / 5, epi 1 or 2): the bf16x3 layer, X_lo = X + xlo,
// Wp = [hi planes; lo planes], split output Y / Y + ylo (elements).
extern "C" int ncnet_conv16_fwd(const void* X, const void* Wp, const float* bias, const void* M, void* Y,
                                int V, int I, int J, int K, int L, int KS, int epi, int npg, int nco,
                                long long xlo, long long ylo, hipStream_t stream) {
  int tk, tl;
  pick_tile(K, L, tk, tl);
  ConvGeom g = make_geom(V, I, J, K, L, KS, tk, tl);
  g.npg = npg;
  g.gstride = (long long)V * I * J * K * L * 16;
  g.nco = nco;
  g.xlo = xlo; g.ylo = ylo;
  if (g.RW > 32) return -1;   // one LDS-DMA wave-instruction per staged row
  const bool x3 = (epi & EPI_X3) != 0;
  if (x3 && !((KS == 5 || KS == 3) && ((epi & ~EPI_X3) == EPI_BIAS_RELU || (epi & ~EPI_X3) == EPI_MASK))) return -2;
  // Row stride RS = TL + 8: a 16-voxel tile that wraps to the next row then
  // jumps 256 B (the full 64-bank period), so every ds_read_b128 lane group
  // stays conflict-free (a TL + KS - 1 stride cost ~1/3 extra LDS cycles).
  g.RS = tl + ((KS - 1 + 7) / 8) * 8;
  const int nq = (KS * KS + 1) / 2;
  const bf16* x = (const bf16*)X; const u32x4* w = (const u32x4*)Wp; const bf16* m = (const bf16*)M; bf16* y = (bf16*)Y;
  if (npg == 0 && (epi & ~EPI_X3) != EPI_NONE && (epi & ~EPI_X3) != EPI_F32X16 && (KS == 5 || KS == 3)) {
    // full (di, dj) sum: R = 5 output j-planes per workgroup, X reused across dj
    constexpr int R = 5;
    const int njb1 = g.njb;
    g.njb = cdiv(J, R);
    dim3 grid3((unsigned)(V * I * g.njb * g.nkt * g.nlt)), block3(512);
    if (!tuning().conv_v3 && v4_launch(KS, K, L, tk, tl, epi, grid3, block3, stream, x, w, bias, m, y, g))
      return (int)hipGetLastError();
    g.njb = njb1;
    if (x3) goto v2_x3;   // other shapes: the v2 kernel's phases
    g.njb = cdiv(J, R);
    size_t lds3 = 2 * (size_t)g.PR * g.RS * 32 + (size_t)KS * nq * 1024;
#define L16V3(KSV, EPIV) hipLaunchKernelGGL((conv16v3_fwd_kernel<KSV, R, EPIV>), grid3, block3, lds3, stream, x, w, bias, m, y, g)
    if (KS == 5) { if (epi == EPI_BIAS_RELU) L16V3(5, EPI_BIAS_RELU); else L16V3(5, EPI_MASK); }
    else { if (epi == EPI_BIAS_RELU) L16V3(3, EPI_BIAS_RELU); else L16V3(3, EPI_MASK); }
#undef L16V3
    return (int)hipGetLastError();
  }
v2_x3: {
  size_t lds2 = 2 * (size_t)g.PR * g.RS * 32 + (size_t)nq * 1024;
  // group planes: tpw consecutive output j-tiles per workgroup (NCNET_GP_TPW,
  // default 5): the next tile's first plane DMA overlaps the current epilogue
  const bool mt = npg > 0 && gp_tpw() > 1;
  if (mt) { g.tpw = gp_tpw(); g.njb = cdiv(J, g.tpw); }
  dim3 grid2((unsigned)(V * I * g.njb * g.nkt * g.nlt)), block2(512);
  if (x3) {
#define L16V2X(KSV, EPIV) do { if (mt) hipLaunchKernelGGL((conv16v2_fwd_kernel<KSV, EPIV, true>), grid2, block2, lds2, stream, x, w, bias, m, y, g); \
                               else hipLaunchKernelGGL((conv16v2_fwd_kernel<KSV, EPIV, false>), grid2, block2, lds2, stream, x, w, bias, m, y, g); } while (0)
    if (KS == 5) { if (epi == (EPI_BIAS_RELU | EPI_X3)) L16V2X(5, EPI_BIAS_RELU | EPI_X3); else L16V2X(5, EPI_MASK | EPI_X3); }
    else { if (epi == (EPI_BIAS_RELU | EPI_X3)) L16V2X(3, EPI_BIAS_RELU | EPI_X3); else L16V2X(3, EPI_MASK | EPI_X3); }
#undef L16V2X
    return (int)hipGetLastError();
  }
#define L16V2E(KSV, EPIV) do { if (mt) hipLaunchKernelGGL((conv16v2_fwd_kernel<KSV, EPIV, true>), grid2, block2, lds2, stream, x, w, bias, m, y, g); \
                               else hipLaunchKernelGGL((conv16v2_fwd_kernel<KSV, EPIV, false>), grid2, block2, lds2, stream, x, w, bias, m, y, g); } while (0)
#define L16V2(KSV, _) do { if (epi == EPI_BIAS_RELU) L16V2E(KSV, EPI_BIAS_RELU); else if (epi == EPI_MASK) L16V2E(KSV, EPI_MASK); \
                           else if (epi == EPI_F32X16) L16V2E(KSV, EPI_F32X16); else L16V2E(KSV, EPI_NONE); } while (0)
  KS_DISPATCH(L16V2, 0);
#undef L16V2
#undef L16V2E
  return (int)hipGetLastError();
}
}

// Cout = 1 layer (16 input channels) in output-plane-block mode: Y fp32
// [V,I,J,K,L] = act(bias + conv(X, W)); Wp [(KS+3)^2 relative planes][nq][64][8]
// (ops/packing.py blk_out_weights): the 16 MFMA rows are a 4 x 4 block of output
// planes, so every input plane staged in LDS feeds up to 16 output planes and
// no combo-planar partials (ij encoding + ijsum) round-trip HBM.
// xlo >= 0 ... any value with x3 != 0: the bf16x3 layer (X_lo = X + xlo, Wp = [hi; lo] planes).
extern "C" int ncnet_conv16_blk_fwd(const void* X, const void* Wp, const float* bias, float* Y, int V, int I, int J,
                                    int K, int L, int KS, int relu, int x3, long long xlo, hipStream_t stream) {
  int tk, tl;
  pick_tile(K, L, tk, tl);
  ConvGeom g = make_geom(V, I, J, K, L, KS, tk, tl);
  g.xlo = xlo;
  if (x3 && KS != 5 && KS != 3) return -2;
  if (g.RW > 32) return -1;
  g.RS = tl + ((KS - 1 + 7) / 8) * 8;
  g.nib = cdiv(I, 4); g.njb = cdiv(J, 4);
  g.relu = relu;
  const int nq = (KS * KS + 1) / 2;
  size_t lds2 = 2 * (size_t)g.PR * g.RS * 32 + (size_t)nq * 1024;
  dim3 grid((unsigned)(V * g.nib * g.njb * g.nkt * g.nlt)), block(512);
  const bf16* x = (const bf16*)X; const u32x4* w = (const u32x4*)Wp;
  if (KS == 5 && K == 25 && L == 25 && tk == 25 && tl == 25) {   // the 400 px training planes
    if (x3)
      hipLaunchKernelGGL((conv16v2_fwd_kernel<5, EPI_BLK1 | EPI_X3, false, 25>), grid, block, lds2, stream, x, w, bias,
                         nullptr, (bf16*)Y, g);
    else
      hipLaunchKernelGGL((conv16v2_fwd_kernel<5, EPI_BLK1, false, 25>), grid, block, lds2, stream, x, w, bias, nullptr,
                         (bf16*)Y, g);
    return (int)hipGetLastError();
  }
#define LBLK(KSV, _) hipLaunchKernelGGL((conv16v2_fwd_kernel<KSV, EPI_BLK1, false>), grid, block, lds2, stream, x, w, bias, nullptr, (bf16*)Y, g)
#define LBLKX(KSV) hipLaunchKernelGGL((conv16v2_fwd_kernel<KSV, EPI_BLK1 | EPI_X3, false>), grid, block, lds2, stream, x, w, bias, nullptr, (bf16*)Y, g)
  if (x3) {
    if (KS == 5) LBLKX(5); else LBLKX(3);
    return (int)hipGetLastError();
  }
#undef LBLKX
  KS_DISPATCH(LBLK, 0);
#undef LBLK
  return (int)hipGetLastError();
}

// fp8 (OCP e4m3) inference Conv4d 16 -> 16; epi 1 (fp8 out) or 4 (planar fp32), oscale = 1 / weight scale.
extern "C" int ncnet_conv16f8_fwd(const void* X, const void* Wp, const float* bias, void* Y, int V, int I, int J, int K,
                                  int L, int KS, int epi, int npg, int nco, float oscale, hipStream_t stream) {
  int tk, tl;
  pick_tile(K, L, tk, tl);
  ConvGeom g = make_geom(V, I, J, K, L, KS, tk, tl);
  g.npg = npg;
  g.gstride = (long long)V * I * J * K * L * 16;
  g.nco = nco;
  g.oscale = oscale;
  if (g.RW > 32) return -1;
  g.RS = tl + 16;                       // 16-byte voxels: a row wrap jumps 256 B
  const int nq = (KS * KS + 1) / 2;
  size_t lds = 2 * (size_t)g.PR * g.RS * 16 + (size_t)nq * 512;
  dim3 grid((unsigned)(V * I * J * g.nkt * g.nlt)), block(512);
  const uint8_t* x = (const uint8_t*)X; const uint8_t* w = (const uint8_t*)Wp;
#define LF8(KSV, _) do { if (epi == EPI_BIAS_RELU) hipLaunchKernelGGL((conv16f8_fwd_kernel<KSV, EPI_BIAS_RELU>), grid, block, lds, stream, x, w, bias, Y, g); \
                         else if (epi == EPI_F32X16) hipLaunchKernelGGL((conv16f8_fwd_kernel<KSV, EPI_F32X16>), grid, block, lds, stream, x, w, bias, Y, g); \
                         else return -2; } while (0)
  KS_DISPATCH(LF8, 0);
#undef LF8
  return (int)hipGetLastError();
}

// set_tuning binding: name -> previous value (INT32_MIN for an unknown name)
extern "C" int ncnet_set_tuning(const char* name, int value, int set) {
  int* p = tuning_slot(name);
  if (!p) return INT32_MIN;
  const int old = *p;
  if (set) *p = value;
  return old;
}
