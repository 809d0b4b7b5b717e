// Cout = 1 Conv4d forward (the last NeighConsensus layer, 16 -> 1 channels,
// lib/model.py:130-139 / lib/conv4d.py:11-51) with the in-plane taps as the MFMA
// rows.
//
//   Y[v,i,j,k,l] = act(bias + sum_{di,dj} sum_{dk,dl,ci} W[ci,di,dj,dk,dl] X[v,i+di-P,j+dj-P,k+dk-P,l+dl-P,ci])
//
// The output-plane-block kernel (conv4d_fwd.hip EPI_BLK1) puts a 4 x 4 block
// of output planes on the 16 MFMA rows; an input plane feeds only the rows
// whose (di, dj) offset is inside the kernel, so 38 % of its MFMA rows are
// useful.  Here one MFMA (v_mfma_f32_32x32x16_bf16) is
//
//   Z_o[tap][c] += W[ci, di, dj, tap] (32 rows = the 25 (dk, dl) taps + 7 zero rows, K = 16 ci)
//                  x X_p[ci][c]       (32 columns = input voxels c of plane p = o + (di, dj) - P)
//
// -- every row is a real tap for every (input plane, output plane) pair, 76 %
// of the MFMA work useful (25 / 32 rows x 625 / 640 columns) -- and the in-plane
// shift is applied once per output plane at the end:
//
//   Y_o[k, l] = sum_{dk,dl} Z_o[(dk, dl)][(k + dk - P, l + dl - P)]   (zero outside the plane)
//
// through an fp32 staging copy of Z_o in LDS.
//
// Work: an item = an RI x RJ block of output planes (1 x 3 at the training
// plane: a 2 x 2 block needs 320 accumulator registers, past the 256 a wave
// can hold without AGPR <-> VGPR copies), whose (RI+KS-1) x (RJ+KS-1) window of
// input planes streams through LDS; a persistent workgroup (one per CU, 4
// waves = one per SIMD) walks items bid, bid + G, ...  The 640 columns
// are split over the waves (5 tiles of 32 each), and each wave DMAs only ITS
// 160 voxels of every plane into its own 6-slot ring (5 planes ahead), so the
// main loop has no workgroup barrier at all: a wave waits only for its own
// LDS-DMAs (counted vmcnt; a fixed count of DMA instructions per step, past the
// item's last plane they read zeros into the slot the step after next will
// overwrite anyway).  Accumulators: RI x RJ output planes x 5 tiles x 16
// (240 at 1 x 3).  The epilogue stages Z_o in LDS (two buffers, one barrier
// per output plane) and sums the shifted tap rows.
// Layouts: X bf16 [V,I,J,K,L,16]; Wt bf16 [KS*KS (di,dj)][64 lanes][8] =
// the A fragments (lane l: tap row l & 31, ci 8 (l >> 5) + e); Y fp32 [V,I,J,K,L].
#include "common.h"
#include <type_traits>

namespace ncnet {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int B, int E, typename F>
__device__ __forceinline__ void c1_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    c1_static_for<B + 1, E>(f);
  }
}

template <int KS, int K, int L, int RI, int RJ>
struct CT1 {
  static constexpr int P = KS / 2, NT = KS * KS, NW = 4;
  static constexpr int NV = K * L;                       // voxels per plane
  static constexpr int NCT = (NV + 31) / 32;             // 32-column tiles
  static constexpr int MT = (NCT + NW - 1) / NW;         // tiles per wave
  static constexpr int WV = MT * 32;                     // voxels per wave
  static constexpr int HB = WV * 16;                     // bytes of one channel half of a wave's slice
  static constexpr int SLOT = 2 * HB;                    // one plane slice (both halves)
  static constexpr int NSLOT = 6;                        // plane s + 5 in flight while s computes
  static constexpr int NDMA = SLOT / 1024;               // DMA wave-instructions per plane and wave
  static constexpr int WOFF = 0, WBYTES = NT * 1024;
  static constexpr int ROFF = WBYTES;                    // rings: [wave][slot][SLOT]
  static constexpr int ZCOLS = NW * WV;                  // staging row length (>= NV)
  static constexpr int ZPAD = 64;                        // floats before the staging rows (>= P K + P)
  static constexpr int LDS_RING = NW * NSLOT * SLOT;
  static constexpr int ZBUF = ZPAD + NT * ZCOLS;          // floats of one staging buffer (two)
  static constexpr int ZBYTES = 2 * ZBUF * 4;
  static constexpr int LDS = ROFF + (LDS_RING > ZBYTES ? LDS_RING : ZBYTES);
  static constexpr int WI = RI + KS - 1, WJ = RJ + KS - 1;   // input window (planes along i, j)
  static constexpr int NO = RI * RJ;                     // output planes per item
  static_assert(SLOT % 1024 == 0, "whole DMA instructions per slice");
  static_assert(NT <= 32, "taps fit the 32 MFMA rows");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(ZPAD >= P * L + P, "the gather's lowest tap offset stays inside the staging area");
};

// 16-B-per-lane buffer load into LDS (out-of-range offsets land as zeros),
// issued from asm so the compiler's waitcnt pass never drains it.
typedef int c1i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ c1i32x4 c1_rsrc(const void* base, uint32_t nbytes) {
  const uint64_t b = (uint64_t)base;
  c1i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(b >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)nbytes);
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void c1_dma(const c1i32x4& rs, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds)
               : "memory", "m0");
}

// DBG (scripts/probe/cout1_probe.hip only): 1 no epilogue, 2 no DMA waits,
// 4 no MFMAs -- timing decomposition, wrong results
template <int KS, int K, int L, int RI, int RJ, int DBG = 0>
__global__ __launch_bounds__(256, 1) void cout1_taps_fwd_kernel(const bf16* __restrict__ X, const u32x4* __restrict__ Wt,
                                                                const float* __restrict__ bias, float* __restrict__ Y,
                                                                int V, int I, int J, int relu) {
#if defined(__HIP_DEVICE_COMPILE__)
  using C = CT1<KS, K, L, RI, RJ>;
  constexpr int P = C::P, NW = C::NW, MT = C::MT, NV = C::NV, WI = C::WI, WJ = C::WJ, NO = C::NO;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // weights once per workgroup: NT KiB, wave w DMAs fragments w, w + 4, ...
  {
    const c1i32x4 rs = c1_rsrc(Wt, C::NT * 1024);
    for (int q = wave; q < C::NT; q += NW) c1_dma(rs, (uint32_t)((q * 64 + lane) * 16), lds0 + C::WOFF + q * 1024);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

  const int nbi = (I + RI - 1) / RI, nbj = (J + RJ - 1) / RJ;
  const int nitems = V * nbi * nbj;
  const uint32_t ring = lds0 + C::ROFF + (uint32_t)(wave * C::NSLOT * C::SLOT);
  // DMA instruction m of a plane slice: lanes q = 64 m + lane -> channel half
  // q / WV, voxel 160 wave + q % WV of the plane; LDS [half][voxel][16 B]
  uint32_t dvo[C::NDMA];
#pragma unroll
  for (int m = 0; m < C::NDMA; ++m) {
    const int q = 64 * m + lane, h = q / C::WV, vx = wave * C::WV + q % C::WV;
    dvo[m] = (uint32_t)(vx * 32 + h * 16);
  }
  const size_t plane_elems = (size_t)NV * 16;
  // B fragment of tile t: lane r + 32 h reads voxel 32 t + r, half h of the slice
  const uint32_t bbase = ring - lds0 + (uint32_t)((lane >> 5) * C::HB + (lane & 31) * 16);
  const uint32_t abase = (uint32_t)(C::WOFF + lane * 16);
  const float b0 = bias ? bias[0] : 0.f;

  // XCD-aware start: the workgroups of one XCD (blocks b, b + 8, ...) take
  // consecutive items, whose input windows overlap, so they share its L2
  for (int item = (int)xcd_remap(blockIdx.x, gridDim.x); item < nitems; item += gridDim.x) {
    const int bj = item % nbj, bi = (item / nbj) % nbi, v = item / (nbj * nbi);
    const int i0 = RI * bi, j0 = RJ * bj;
    const int na = min(RI, I - i0), nb = min(RJ, J - j0);
    const bf16* xv = X + (size_t)v * I * J * plane_elems;
    // the whole WIN x WIN window, unrolled: step s = window plane (s / WIN, s % WIN)
    // (input plane (i0 - P + pi, j0 - P + qj)); a plane outside the volume is
    // DMA'd as zeros (num_records 0) and contributes nothing, so the MFMAs of a
    // step -- the (a, b) outputs whose kernel window holds it -- are branch-free
    // (a per-step runtime branch around the accumulator updates made the
    // register allocator spill ~300 VGPRs).  Output planes past the volume (the
    // last block of an odd I or J) are computed and not stored.
    auto issue = [&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr int pi = s / WJ, qj = s % WJ;
      const int ii = i0 - P + pi, jj = j0 - P + qj;
      const bool live = s < WI * WJ && ii >= 0 && ii < I && jj >= 0 && jj < J;
      const bf16* xp = xv + ((size_t)(live ? ii : 0) * J + (live ? jj : 0)) * plane_elems;
      const c1i32x4 rs = c1_rsrc(xp, live ? (uint32_t)(NV * 32) : 0u);
      const uint32_t slot = ring + (uint32_t)((s % C::NSLOT) * C::SLOT);
#pragma unroll
      for (int m = 0; m < C::NDMA; ++m) c1_dma(rs, dvo[m], slot + m * 1024);
    };
    f32x16 acc[RI][RJ][MT];
#pragma unroll
    for (int a = 0; a < RI; ++a)
#pragma unroll
      for (int b = 0; b < RJ; ++b)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[a][b][t] = f32x16{};
    constexpr int NS = C::NSLOT, AHEAD = NS - 1;
    c1_static_for<0, AHEAD>([&](auto qc) { issue(qc); });
    // fragments of step s live in B[s & 1] / A[s & 1]; step s + 1's are read
    // while step s's MFMAs run (its plane landed: AHEAD - 1 steps of slack)
    bf16x8 B[2][MT], A[2][NO];
    auto load_frags = [&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr int pi = s / WJ, qj = s % WJ;
#pragma unroll
      for (int t = 0; t < MT; ++t)
        B[s & 1][t] = *(const bf16x8*)(smem + bbase + (uint32_t)((s % NS) * C::SLOT + t * 512));
      c1_static_for<0, NO>([&](auto oc) {
        constexpr int o = decltype(oc)::value, di = pi - o / RJ, dj = qj - o % RJ;
        if constexpr (di >= 0 && di < KS && dj >= 0 && dj < KS)
          A[s & 1][o] = *(const bf16x8*)(smem + abase + (uint32_t)((di * KS + dj) * 1024));
      });
    };
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((AHEAD - 1) * C::NDMA) : "memory");   // plane 0
    load_frags(std::integral_constant<int, 0>{});
    c1_static_for<0, WI * WJ>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr int pi = s / WJ, qj = s % WJ;
      issue(std::integral_constant<int, s + AHEAD>{});
      if constexpr (s + 1 < WI * WJ) {
        // this wave's slice of plane s + 1 has landed (s + 2 .. s + AHEAD may fly)
        if constexpr (!(DBG & 2)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((AHEAD - 1) * C::NDMA) : "memory");
        load_frags(std::integral_constant<int, s + 1>{});
      }
      c1_static_for<0, NO>([&](auto oc) {
        constexpr int o = decltype(oc)::value, a = o / RJ, b = o % RJ;
        constexpr int di = pi - a, dj = qj - b;
        if constexpr (di >= 0 && di < KS && dj >= 0 && dj < KS && !(DBG & 4)) {
#pragma unroll
          for (int t = 0; t < MT; ++t)
            acc[a][b][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s & 1][o], B[s & 1][t], acc[a][b][t], 0, 0, 0);
        }
      });
    });
    // ---- epilogue: per output plane, Z_o -> LDS staging [tap][col], shift-sum
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");   // every ring read and DMA done
    float* zs = (float*)(smem + C::ROFF) + C::ZPAD;
    // this thread's outputs o = tid + 256 m: per-tap validity as row / column
    // masks (1 / 0) and one staging base; tap (dk, dl) of output (k, l) reads
    // zs[tap][(k + dk - P) L + l + dl - P] = base + tap ZCOLS + dk L + dl - (P L + P)
    constexpr int NPT = (NV + NW * 64 - 1) / (NW * 64);   // outputs per thread
    float mk[NPT][KS], ml[NPT][KS];
    uint32_t zb[NPT];
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int o = threadIdx.x + NW * 64 * m, oc = o < NV ? o : 0;
      const int k = oc / L, l = oc - (oc / L) * L;
#pragma unroll
      for (int d = 0; d < KS; ++d) {
        mk[m][d] = (k + d - P >= 0 && k + d - P < K) ? 1.f : 0.f;
        ml[m][d] = (l + d - P >= 0 && l + d - P < L) ? 1.f : 0.f;
      }
      zb[m] = (uint32_t)(C::ROFF + (C::ZPAD + oc - (P * L + P)) * 4);
    }
    // two staging buffers: output plane o + 1 is written while o is gathered
    // (one barrier per plane instead of two, the writes beside the reads)
    auto write_z = [&](auto oc) {
      constexpr int o = decltype(oc)::value, a = o / RJ, b = o % RJ;
      float* z = zs + (o & 1) * C::ZBUF;
      // D row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5), col = lane & 31
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int col = wave * C::WV + t * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 13; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < C::NT) z[row * C::ZCOLS + col] = acc[a][b][t][r];
        }
      }
    };
    auto gather = [&](auto oc) {
      constexpr int o = decltype(oc)::value, a = o / RJ, b = o % RJ;
      float* yo = Y + (((size_t)v * I + i0 + a) * J + j0 + b) * NV;
      const uint32_t zo = (uint32_t)((o & 1) * C::ZBUF * 4);
#pragma unroll
      for (int m = 0; m < NPT; ++m) {
        const int oo = threadIdx.x + NW * 64 * m;
        float z[KS][KS];
        // all 25 reads first (immediate offsets on one base), then the sums
#pragma unroll
        for (int dk = 0; dk < KS; ++dk)
#pragma unroll
          for (int dl = 0; dl < KS; ++dl)
            z[dk][dl] = *(const float*)(smem + zb[m] + zo + (uint32_t)(((dk * KS + dl) * C::ZCOLS + dk * L + dl) * 4));
        float sum = b0;
#pragma unroll
        for (int dk = 0; dk < KS; ++dk) {
          float r = 0.f;
#pragma unroll
          for (int dl = 0; dl < KS; ++dl) r = fmaf(z[dk][dl], ml[m][dl], r);
          sum = fmaf(r, mk[m][dk], sum);
        }
        if (relu) sum = fmaxf(sum, 0.f);
        if (oo < NV) __builtin_nontemporal_store(sum, yo + oo);
      }
    };
    if constexpr (!(DBG & 1)) {
      write_z(std::integral_constant<int, 0>{});
      __syncthreads();
      c1_static_for<0, NO>([&](auto oc) {
        constexpr int o = decltype(oc)::value;
        const bool ok = o / RJ < na && o % RJ < nb;
        if constexpr (o + 1 < NO) {
          if ((o + 1) / RJ < na && (o + 1) % RJ < nb) write_z(std::integral_constant<int, o + 1>{});
        }
        if (ok) gather(oc);
        __syncthreads();
      });
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
#endif
}

}  // namespace ncnet

using namespace ncnet;

// output block per item: 1 x 3 planes along j (3 x 5 tiles x 16 = 240 accumulator
// registers, inside the 256 AGPRs: a 2 x 2 block's 320 made the compiler copy
// accumulators between the VGPR and AGPR halves ~2900 times per item)
#ifndef C1_RI
#define C1_RI 1
#define C1_RJ 3
#endif

// Y fp32 [V,I,J,K,L] = act(bias + conv(X, W)) for a 16 -> 1 layer; Wt: the tap-row
// A fragments (ops/packing.py cout1_taps_weights).  Returns -1 for shapes
// without an instantiation (the caller keeps the output-plane-block kernel).
extern "C" int ncnet_cout1_taps_fwd(const void* X, const void* Wt, const float* bias, float* Y, int V, int I, int J,
                                    int K, int L, int KS, int relu, hipStream_t s) {
  if (!(KS == 5 && K == 25 && L == 25)) return -1;
  constexpr int RI = C1_RI, RJ = C1_RJ;
  using C = CT1<5, 25, 25, RI, RJ>;
  const int nitems = V * ((I + RI - 1) / RI) * ((J + RJ - 1) / RJ);
  const int ncu = device_num_cus();
  const int grid = nitems < ncu ? nitems : ncu;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL((cout1_taps_fwd_kernel<5, 25, 25, RI, RJ>), dim3((unsigned)grid), dim3(256), (size_t)C::LDS, s,
                     (const bf16*)X, (const u32x4*)Wt, bias, Y, V, I, J, relu);
  return (int)hipGetLastError();
}
