// Conv4d layers with ONE input or ONE output channel on gfx950 MFMA, with the
// in-plane (dk, dl) shifts kept inside the workgroup ("kl" kernels).
//
// NC-Net's first layer is 1 -> 16 and its last 16 -> 1 (lib/model.py:130-139,
// reference NeighConsensus; lib/conv4d.py:11-51 for the Conv4d semantics).  A
// 1-channel operand wastes 15/16 of an MFMA unless some tap axis is moved into
// the channel axis.  The ij kernels (jshift.hip) do that through HBM: ijpack
// writes KS*KS shifted copies of the 1-channel volume (G x 16 channels) and
// the Cout = 1 layer writes KS*KS channel-planar fp32 partials that ijsum
// adds back -- at InLoc 3200 that is ~8 GB of partials per pass.  Here the
// shifts that live inside one (k, l) plane are resolved in LDS instead:
//
//  conv1to16_kl  (Cin = 1 -> 16: layer-1 forward, Cout=1 layer's data grad)
//    A workgroup owns an output tile (v, i, j, k0:k0+TK, l0:l0+TL).  The KS*KS
//    input plane tiles (i+di-P, j+dj-P) with their (dk, dl) halo sit in LDS
//    (1 channel, <= 42 KB); the implicit-GEMM K axis is the KS^4 taps, packed
//    densely 32 per MFMA (KS=5: 20 MFMAs per 16 voxels, KS=3: 3), each lane
//    gathering its 8 taps with 16-bit LDS reads through a per-tap offset table
//    (one ds_read_b128 of offsets per K step, shared by all voxel tiles).  No
//    shifted copy of the volume is ever written.
//
//  conv16to1_kl  (Cin = 16 -> 1: last layer forward)
//    z_q[k', l'] = sum_{di,dj,c} W[di,dj,q,c] h[i+di-P, j+dj-P, k', l', c]   for
//    every in-plane combo q = (dk, dl), then  y[k, l] = sum_q z_q[k+dk-P, l+dl-P].
//    The MFMA rows are the combos (16 per tile: 1 tile at KS=3, 2 at KS=5),
//    its K axis is (plane pair, channel) -- two input planes per MFMA, read
//    UNSHIFTED over the tile's halo-extended (TK+KS-1) x (TL+KS-1) region --
//    and the combo shift-sum runs on the accumulators parked in LDS.  Planes
//    stream through LDS by LDS-DMA, one pair ahead of the MFMAs.  Bias, ReLU
//    and (fp8 operands) the weight scale are fused; the output is the fp32
//    1-channel volume.  Operands: bf16 (v_mfma_f32_16x16x32_bf16) or OCP fp8
//    e4m3 (v_mfma_f32_16x16x32_fp8_fp8, same K layout, half the bytes).
#include "common.h"
#include <hip/hip_fp8.h>
#include <stdlib.h>
#include <algorithm>
#include <type_traits>

namespace ncnet {

struct KLGeom {
  int V, I, J, K, L;   // volume dims
  int TK, TL;          // output tile
  int nkt, nlt;        // tiles along k, l
  int PR, RW;          // staged (halo-extended) rows / row width = TK+KS-1 / TL+KS-1
  float oscale;        // accumulator scale (fp8 weights: 1 / weight scale)
};

struct KLTile { int v, i, j, k0, l0; };
__device__ __forceinline__ KLTile kl_tile(const KLGeom& g) {
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  KLTile t;
  int lt = bid % g.nlt; bid /= g.nlt;
  int kt = bid % g.nkt; bid /= g.nkt;
  t.j = bid % g.J; bid /= g.J;
  t.i = bid % g.I; t.v = bid / g.I;
  t.k0 = kt * g.TK; t.l0 = lt * g.TL;
  return t;
}

__device__ __forceinline__ size_t kl_plane(const KLGeom& g, int v, int i, int j) {
  return (((size_t)v * g.I + i) * g.J + j) * (size_t)g.K * g.L;
}

// ===========================================================================
// conv1to16_kl
//   X: [V,I,J,K,L] bf16 (1 channel);  Y: [V,I,J,K,L,16] bf16 (or fp8 when F8OUT)
//   Wp: [NS K-steps][64 lanes] x 16 B: lane l of step s holds
//       W[co = l&15][tap = 32s + 8(l>>4) + 0..7]  (tap = ((di*KS+dj)*KS+dk)*KS+dl,
//       zero past KS^4)
//   EPI_BIAS_RELU: y = relu(acc + b[co]);  EPI_MASK: y = acc * (M > 0)
// LDS: [KS*KS][PR*RW] bf16 plane tiles | [NS*32] u16 tap offsets | [NS*64] weight fragments
// ===========================================================================
enum KLEpi { KL_BIAS_RELU = 1, KL_MASK = 2 };

template <int KS, int EPI, bool F8OUT>
__global__ __launch_bounds__(512, 2) void conv1to16_kl_kernel(const bf16* __restrict__ X, const u32x4* __restrict__ Wp,
                                                              const float* __restrict__ bias,
                                                              const bf16* __restrict__ M, void* __restrict__ Y,
                                                              KLGeom g) {
  constexpr int P = KS / 2;
  constexpr int NC = KS * KS;             // planes = in-plane combos
  constexpr int NK = NC * NC;             // taps
  constexpr int NS = (NK + 31) / 32;      // K steps
  constexpr int NW = 8;
  constexpr int MAXT = 5;                 // 16-voxel tiles per wave (TK*TL <= 640)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int psz = g.PR * g.RW;
  bf16* xt = (bf16*)smem;
  const int xbytes = ((NC * psz * 2) + 15) & ~15;
  uint16_t* tab = (uint16_t*)(smem + xbytes);
  u32x4* wl = (u32x4*)(smem + xbytes + NS * 64);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const KLTile t = kl_tile(g);
  const int nvox = g.TK * g.TL;
  const int ntile = (nvox + 15) >> 4;
  const bool full_wave = __builtin_amdgcn_readfirstlane(wave + NW * (MAXT - 1) < ntile);

  // stage the KS*KS halo-extended plane tiles (zero outside the volume)
  const int total = NC * psz;
  for (int e = threadIdx.x; e < total; e += NW * 64) {
    const int p = e / psz, rem = e - p * psz;
    const int r = rem / g.RW, c = rem - r * g.RW;
    const int di = p / KS, dj = p - di * KS;
    const int ii = t.i + di - P, jj = t.j + dj - P, kg = t.k0 - P + r, lg = t.l0 - P + c;
    bf16 v = f2bf(0.f);
    if (ii >= 0 && ii < g.I && jj >= 0 && jj < g.J && kg >= 0 && kg < g.K && lg >= 0 && lg < g.L)
      v = X[kl_plane(g, t.v, ii, jj) + (size_t)kg * g.L + lg];
    xt[e] = v;
  }
  for (int k = threadIdx.x; k < NS * 32; k += NW * 64) {
    int off = 0;
    if (k < NK) {
      const int p = k / NC, q = k - p * NC, dk = q / KS, dl = q - dk * KS;
      off = p * psz + dk * g.RW + dl;
    }
    tab[k] = (uint16_t)off;
  }
  for (int k = threadIdx.x; k < NS * 64; k += NW * 64) wl[k] = Wp[k];
  __syncthreads();

  uint32_t vb[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int vi = (wave + NW * tt) * 16 + (lane & 15);
    if (vi >= nvox) vi = 0;
    const int kk = vi / g.TL, ll = vi - kk * g.TL;
    vb[tt] = (uint32_t)(kk * g.RW + ll);
  }
  f32x4 acc[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int grp = lane >> 4;
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const u32x4 a = wl[s * 64 + lane];
    const u32x4 o4 = *(const u32x4*)(tab + s * 32 + grp * 8);
    uint32_t off[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { off[2 * j] = o4[j] & 0xffffu; off[2 * j + 1] = o4[j] >> 16; }
    // branch-free body for full waves: the gathers of tile tt+1 overlap the MFMA of tile tt
    auto tiles = [&](auto fullc) {
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int tt = 0; tt < MAXT; ++tt) {
        if (FULL || wave + NW * tt < ntile) {
          const bf16* base = xt + vb[tt];
          bf16x8 b;
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = base[off[j]];
          acc[tt] = mfma16(__builtin_bit_cast(bf16x8, a), b, acc[tt]);
        }
      }
    };
    if (full_wave) tiles(std::true_type{}); else tiles(std::false_type{});
  }

  const size_t vbase_out = kl_plane(g, t.v, t.i, t.j);
  const int co0 = 4 * (lane >> 4);
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    const int tile = wave + NW * tt;
    if (tile >= ntile) continue;
    const int vi = tile * 16 + (lane & 15);
    const int kk = vi / g.TL, ll = vi - kk * g.TL;
    const int kg = t.k0 + kk, lg = t.l0 + ll;
    if (vi >= nvox || kg >= g.K || lg >= g.L) continue;
    const size_t vox = vbase_out + (size_t)kg * g.L + lg;
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = acc[tt][r];
    if (EPI == KL_BIAS_RELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r] + bias[co0 + r], 0.f);
    } else {
      const bf16x4 m = *(const bf16x4*)(M + vox * 16 + co0);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = ((float)m[r] > 0.f) ? o[r] : 0.f;
    }
    if (F8OUT) {
      uint32_t packed = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        packed |= (uint32_t)__hip_cvt_float_to_fp8(o[r], __HIP_SATFINITE, __HIP_E4M3) << (8 * r);
      *(uint32_t*)((uint8_t*)Y + vox * 16 + co0) = packed;
    } else {
      bf16x4 ob;
#pragma unroll
      for (int r = 0; r < 4; ++r) ob[r] = f2bf(o[r]);
      *(bf16x4*)((bf16*)Y + vox * 16 + co0) = ob;
    }
  }
}

// ===========================================================================
// conv16to1_kl
//   X: [V,I,J,K,L,16] bf16 or fp8 (F8);  Y: [V,I,J,K,L] fp32
//   Wp: [(KS*KS + 1) planes][NCT combo tiles][16 combos][16 ch] elements
//       (plane p = di*KS + dj; the extra plane is all zero: odd plane counts)
//   y = act(oscale * sum + b)
// LDS: 4 plane buffers [PR*RW][16 ch] (two pairs: current + next) | weights;
//      after the K loop the buffers hold z[NT combos][NEP ext voxels] fp32.
// ===========================================================================
template <int KS, bool F8, bool RELU>
__global__ __launch_bounds__(512, 1) void conv16to1_kl_kernel(const uint8_t* __restrict__ X,
                                                              const uint8_t* __restrict__ Wp,
                                                              const float* __restrict__ bias, float* __restrict__ Y,
                                                              KLGeom g) {
  constexpr int P = KS / 2;
  constexpr int NT = KS * KS;
  constexpr int NCT = (NT + 15) / 16;
  constexpr int NW = 8;
  constexpr int MAXT = 7;                 // 16-voxel ext tiles per wave (PR*RW <= 896)
  constexpr int ESZ = F8 ? 1 : 2;
  constexpr int ES = 16 * ESZ;            // bytes per voxel
  constexpr int HALF = 8 * ESZ;           // bytes of 8 channels

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ne = g.PR * g.RW;
  const int ntile = (ne + 15) >> 4;
  const int nep = ntile * 16;
  const int bufb = ne * ES;
  const int zbytes = NT * nep * 4;
  const int region = max(4 * bufb, zbytes);
  char* wl = smem + ((region + 15) & ~15);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const KLTile t = kl_tile(g);
  const int di_lo = max(0, P - t.i), di_hi = min(KS, g.I + P - t.i);
  const int dj_lo = max(0, P - t.j), dj_hi = min(KS, g.J + P - t.j);
  const int ndj = dj_hi - dj_lo;
  const int nplanes = (di_hi - di_lo) * ndj;
  const int npair = (nplanes + 1) >> 1;
  const bool full_wave = __builtin_amdgcn_readfirstlane(wave + NW * (MAXT - 1) < ntile);

  // zero the plane buffers (halo / out-of-volume voxels stay zero: fixed per tile)
  for (int o = threadIdx.x * 16; o < 4 * bufb; o += NW * 64 * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};
  const int wbytes = (NT + 1) * NCT * 256 * ESZ;
  for (int o = threadIdx.x * 16; o < wbytes; o += NW * 64 * 16) *(u32x4*)(wl + o) = *(const u32x4*)(Wp + o);

  const int lstart = max(0, t.l0 - P), lend = min(g.L, t.l0 - P + g.RW);
  const int nchunk = (lend - lstart) * ES / 16;
  const int col0 = lstart - (t.l0 - P);

  auto plane_of = [&](int s) { return (di_lo + s / ndj) * KS + dj_lo + s % ndj; };
  auto issue = [&](int s, char* buf) {
    const int p = plane_of(s), di = p / KS, dj = p - di * KS;
    const uint8_t* xp = X + kl_plane(g, t.v, t.i + di - P, t.j + dj - P) * ES;
    for (int r = wave; r < g.PR; r += NW) {
      const int kg = t.k0 - P + r;
      if (kg >= 0 && kg < g.K && lane < nchunk)
        __builtin_amdgcn_global_load_lds((const void*)(xp + ((size_t)kg * g.L + lstart) * ES + lane * 16),
                                         LDS_PTR(void, buf + (r * g.RW + col0) * ES), 16, 0, 0);
    }
  };
  auto issue_pair = [&](int q, char* pairbuf) {
    issue(2 * q, pairbuf);
    issue(2 * q + 1 < nplanes ? 2 * q + 1 : 2 * q, pairbuf + bufb);
  };

  uint32_t eoff[MAXT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    int e = (wave + NW * tt) * 16 + (lane & 15);
    if (e >= ne) e = ne - 1;
    eoff[tt] = (uint32_t)(e * ES + ((lane >> 4) & 1) * HALF) + (uint32_t)((lane >> 5) * bufb);
  }
  f32x4 acc[MAXT][NCT];
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[tt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();   // zero fill + weights complete before any DMA lands
  if (npair > 0) issue_pair(0, smem);
  for (int q = 0; q < npair; ++q) {
    __syncthreads();   // pair q landed (vmcnt drained per wave) and pair q-1 fully consumed
    char* cur = smem + (q & 1) * 2 * bufb;
    if (q + 1 < npair) issue_pair(q + 1, smem + ((q + 1) & 1) * 2 * bufb);
    const int pl = (lane >> 5) ? (2 * q + 1 < nplanes ? plane_of(2 * q + 1) : NT) : plane_of(2 * q);
    const uint32_t aoff = (uint32_t)((pl * NCT * 16 + (lane & 15)) * ES + ((lane >> 4) & 1) * HALF);
    if (F8) {
      long a[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) a[ct] = *(const long*)(wl + aoff + ct * 16 * ES);
      auto tiles = [&](auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
        for (int tt = 0; tt < MAXT; ++tt) {
          if (FULL || wave + NW * tt < ntile) {
            const long b = *(const long*)(cur + eoff[tt]);
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
              acc[tt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a[ct], b, acc[tt][ct], 0, 0, 0);
          }
        }
      };
      if (full_wave) tiles(std::true_type{}); else tiles(std::false_type{});
    } else {
      bf16x8 a[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) a[ct] = lds_read16(wl, aoff + ct * 16 * ES);
      auto tiles = [&](auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
        for (int tt = 0; tt < MAXT; ++tt) {
          if (FULL || wave + NW * tt < ntile) {
            const bf16x8 b = lds_read16(cur, eoff[tt]);
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) acc[tt][ct] = mfma16(a[ct], b, acc[tt][ct]);
          }
        }
      };
      if (full_wave) tiles(std::true_type{}); else tiles(std::false_type{});
    }
  }
  __syncthreads();   // every wave done reading the plane buffers

  // park the combo partials z[q][e] in LDS (16 lanes -> 16 consecutive floats)
  float* zl = (float*)smem;
#pragma unroll
  for (int tt = 0; tt < MAXT; ++tt) {
    const int tile = wave + NW * tt;
    if (tile >= ntile) continue;
    const int e = tile * 16 + (lane & 15);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = ct * 16 + 4 * (lane >> 4) + r;
        if (q < NT) zl[q * nep + e] = acc[tt][ct][r];
      }
  }
  __syncthreads();

  const float b0 = bias ? bias[0] : 0.f;
  const size_t vbase_out = kl_plane(g, t.v, t.i, t.j);
  for (int o = threadIdx.x; o < g.TK * g.TL; o += NW * 64) {
    const int kk = o / g.TL, ll = o - kk * g.TL;
    const int kg = t.k0 + kk, lg = t.l0 + ll;
    if (kg >= g.K || lg >= g.L) continue;
    float s = 0.f;
#pragma unroll
    for (int dk = 0; dk < KS; ++dk)
#pragma unroll
      for (int dl = 0; dl < KS; ++dl) s += zl[(dk * KS + dl) * nep + (kk + dk) * g.RW + ll + dl];
    float y = s * g.oscale + b0;
    if (RELU) y = fmaxf(y, 0.f);
    Y[vbase_out + (size_t)kg * g.L + lg] = y;
  }
}

// ---------------------------------------------------------------------------
// host-side tile choice
static void kl_tiles(KLGeom& g, int KS, int max_tl, int max_vox, int max_ext) {
  int nlt = cdiv(g.L, max_tl);
  g.TL = cdiv(g.L, nlt);
  g.RW = g.TL + KS - 1;
  int tk = g.K;
  while (tk > 1 && (tk * g.TL > max_vox || (tk + KS - 1) * g.RW > max_ext)) --tk;
  int nkt = cdiv(g.K, tk);
  g.TK = cdiv(g.K, nkt);
  g.PR = g.TK + KS - 1;
  g.nkt = cdiv(g.K, g.TK);
  g.nlt = cdiv(g.L, g.TL);
}

}  // namespace ncnet

using namespace ncnet;

// Tile geometry the bindings validate against (TK, TL) -- also used by tests.
extern "C" void ncnet_kl_tiles(int which, int K, int L, int KS, int F8, int* tk, int* tl) {
  KLGeom g{};
  g.K = K; g.L = L;
  if (which == 0) kl_tiles(g, KS, 32, 640, 1 << 30);
  else kl_tiles(g, KS, (F8 ? 64 : 32) - KS + 1, 1 << 30, 896);
  *tk = g.TK; *tl = g.TL;
}

// 1 -> 16.  epi 1: bias + ReLU, 2: ReLU mask M.  f8out: Y is fp8 e4m3.
extern "C" int ncnet_conv1to16_kl(const void* X, const void* Wp, const float* bias, const void* M, void* Y, int V, int I,
                                  int J, int K, int L, int KS, int epi, int f8out, hipStream_t stream) {
  if (KS != 3 && KS != 5) return -2;
  KLGeom g{};
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L; g.oscale = 1.f;
  kl_tiles(g, KS, 32, 640, 1 << 30);
  const int NC = KS * KS, NS = (NC * NC + 31) / 32;
  if (NC * g.PR * g.RW >= 65536) return -3;
  size_t lds = (((size_t)NC * g.PR * g.RW * 2 + 15) & ~(size_t)15) + NS * 64 + (size_t)NS * 64 * 16;
  dim3 grid((unsigned)((size_t)V * I * J * g.nkt * g.nlt)), block(512);
  const bf16* x = (const bf16*)X;
  const u32x4* w = (const u32x4*)Wp;
  const bf16* m = (const bf16*)M;
#define KL1(KSV, EPIV, F8V) \
  hipLaunchKernelGGL((conv1to16_kl_kernel<KSV, EPIV, F8V>), grid, block, lds, stream, x, w, bias, m, Y, g)
  if (KS == 5) {
    if (epi == KL_BIAS_RELU) { if (f8out) KL1(5, KL_BIAS_RELU, true); else KL1(5, KL_BIAS_RELU, false); }
    else if (epi == KL_MASK) KL1(5, KL_MASK, false);
    else return -4;
  } else {
    if (epi == KL_BIAS_RELU) { if (f8out) KL1(3, KL_BIAS_RELU, true); else KL1(3, KL_BIAS_RELU, false); }
    else if (epi == KL_MASK) KL1(3, KL_MASK, false);
    else return -4;
  }
#undef KL1
  return (int)hipGetLastError();
}

// 16 -> 1.  f8: X and Wp are fp8 e4m3 (oscale = 1 / weight scale), else bf16.
extern "C" int ncnet_conv16to1_kl(const void* X, const void* Wp, const float* bias, float* Y, int V, int I, int J,
                                  int K, int L, int KS, int relu, int f8, float oscale, hipStream_t stream) {
  if (KS != 3 && KS != 5) return -2;
  KLGeom g{};
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L; g.oscale = oscale;
  const int ES = f8 ? 16 : 32;
  kl_tiles(g, KS, 1024 / ES - KS + 1, 1 << 30, 896);
  const int NT = KS * KS, NCT = (NT + 15) / 16;
  const int ne = g.PR * g.RW, nep = cdiv(ne, 16) * 16;
  size_t region = std::max((size_t)4 * ne * ES, (size_t)NT * nep * 4);
  size_t lds = ((region + 15) & ~(size_t)15) + (size_t)(NT + 1) * NCT * 256 * (f8 ? 1 : 2);
  if (lds > 160 * 1024) return -3;
  dim3 grid((unsigned)((size_t)V * I * J * g.nkt * g.nlt)), block(512);
  const uint8_t* x = (const uint8_t*)X;
  const uint8_t* w = (const uint8_t*)Wp;
#define KLO(KSV, F8V, RV) hipLaunchKernelGGL((conv16to1_kl_kernel<KSV, F8V, RV>), grid, block, lds, stream, x, w, bias, Y, g)
  if (KS == 5) {
    if (f8) { if (relu) KLO(5, true, true); else KLO(5, true, false); }
    else { if (relu) KLO(5, false, true); else KLO(5, false, false); }
  } else {
    if (f8) { if (relu) KLO(3, true, true); else KLO(3, true, false); }
    else { if (relu) KLO(3, false, true); else KLO(3, false, false); }
  }
#undef KLO
  return (int)hipGetLastError();
}
