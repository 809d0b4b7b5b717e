// Conv4d with a ONE-channel operand on gfx950 MFMA, without the ij packing.
//
// The 1 -> 16 convolutions of the NC-Net stack -- the first layer's forward
// (input = MutualMatching output) and the last (16 -> 1) layer's data gradient
// (input = the 1-channel output gradient, transposed flipped weights) -- were
// run as 16 -> 16 group-plane convs on an ij-packed copy of the 1-channel
// volume (csrc/jshift.hip): 16x the bytes of the volume written (1.6 GB at the
// training shape) and re-read.  Here the 1-channel planes are staged as they
// are, and the MFMA B operand (32 taps x 16 voxels) is gathered by the
// hardware-transposing LDS read ds_read_b64_tr_b16: each lane addresses four
// consecutive voxels of one tap row, so a fragment is any 32 (plane, tap) rows.
//
//  * input: zero-padded planes [N, PPL] bf16 (row stride LP = L + 2P, K + 2P
//    rows, PPL a multiple of 8); a voxel (k, l) of plane n sits at flattened
//    f = (k + P) LP + l + P and its tap (dk, dl) at f + (dk - P) LP + dl - P, so
//    every tap is a 1-D shift and the halo reads zeros;
//  * output voxels are 16-wide tiles of consecutive f (the 2P pad columns of
//    each row are computed and dropped: LP / L = 1.16x work);
//  * tr_b16 needs 8-byte-aligned rows: each staged plane is held as 4 copies
//    shifted by 0..3 elements (4 LDS-DMAs from the same global plane at
//    element offsets 0, -1, -2, -3, plus a bank-spreading shift; out-of-range
//    reads land as zeros) and a tap row reads the copy that re-aligns its shift;
//  * K = 32 per MFMA = the 25 (dk, dl) taps of one (di, dj) plane offset + 7
//    zero-weight rows; the B fragment of an input plane is shared by every
//    output plane it feeds (dj = 0..KS-1: up to KS MFMAs per 2 transposed reads);
//  * work item = (v, i, R consecutive output j-planes), 8 waves x MAXT tiles;
//    a step = one di: its R + KS - 1 input planes (j') land together in one
//    of two LDS slots, DMA'd one step ahead (the 25 taps of a single plane are
//    too little MFMA work to amortise a barrier);
//  * persistent workgroups (one per CU) walk items bid, bid + G, ...: the plane
//    DMA stream runs on across items, so the per-item prologue (weights, first
//    planes) and epilogue (stores) no longer idle the CU -- with ~0.4 ms of MFMA
//    work spread over 8000 items, one item per workgroup spent half its time
//    there.
// Reference semantics: lib/conv4d.py:11-51 (same-padded 4D cross-correlation),
// the first / last NeighConsensus layers of lib/model.py:130-139.
#include "common.h"
#include <algorithm>
#include <type_traits>

namespace ncnet {

template <int B, int E, typename F>
__device__ __forceinline__ void xstatic_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    xstatic_for<B + 1, E>(f);
  }
}

// EPI1X_X3 (| with either): the fp32-accurate bf16x3 layer of nc_precision='fp32'
// training: three phases per item, (X_hi, W_hi), (X_lo, W_hi), (X_hi, W_lo),
// into the same accumulators (X_lo = Xp + xlo, Wa = [hi set; lo set]); the
// epilogue splits the fp32 result into Y (hi) and Y + ylo (lo).
enum Epi1x { EPI1X_BIAS_RELU = 1, EPI1X_MASK = 2, EPI1X_X3 = 4 };

template <int KS, int K, int L>
struct C1X {
  static constexpr int P = KS / 2, NT = KS * KS, NW = 8;
  static constexpr int LP = L + 2 * P, KPR = K + 2 * P;
  static constexpr int PPL = (KPR * LP + 7) / 8 * 8;          // padded plane (elements)
  static constexpr int F0 = P * LP + P;                        // f of voxel (0, 0)
  static constexpr int FN = (K - 1 + P) * LP + (L - 1 + P) + 1;
  static constexpr int NTILE = (FN - F0 + 15) / 16;
  static constexpr int MAXT = (NTILE + NW - 1) / NW;
  // bytes per shifted copy: the plane + the largest shift (3 + 44), 16-B multiple
  static constexpr int COPYB = ((PPL + 3 + 44) * 2 + 15) / 16 * 16;
  // copy c holds element e at position e + c + DELTA(c): c re-aligns a tap row to
  // 8 bytes, DELTA (a multiple of 4) spreads the rows of one transposed read over
  // the LDS banks (exhaustive search over the KS = 5 tap rows: worst 2-way, mean
  // 1.75 dwords per bank, vs 4-way / 3.75 without)
  static constexpr int delta(int c) { return c == 0 ? 0 : c == 1 ? 12 : c == 2 ? 28 : 44; }
  static constexpr int SLOTB = 4 * COPYB;                      // one staged plane (4 copies)
  static constexpr int WOFF = 0, XOFF = NT * 1024;
  static constexpr int lds(int np, int d) { return XOFF + (d + 1) * np * SLOTB + 256; }   // + tail pad
  static_assert(NT <= 32, "one K fragment per plane offset");
  // reads for real voxels stay inside their copy; junk columns / tiles may read
  // past it into the next copy (finite data) or into the LDS tail pad
  static_assert(FN - 1 + P * LP + P + 3 + 44 < COPYB / 2, "real-voxel tap reads stay inside one copy");
  static constexpr int NCH = (COPYB + 1023) / 1024;           // DMA wave-instructions per copy (2 or 3)
  static_assert(COPYB > 1024 && COPYB <= 3072, "two or three DMA wave-instructions per copy");
};

// zero-padded planes (see the file comment): Y[n][(k+P)*LP + l + P] = X[n][k][l]
// for n in [0, N); the halo must be zero beforehand (hipMemsetAsync).
// TRANS: the planes of the A<->B-swapped volume of x [V, R = I*J, C = K*L]:
// output plane v*C + c holds x[v, :, c] as an [I, J] plane (I = K, J = L here).
template <typename T, bool TRANS>
__global__ __launch_bounds__(256) void pad_planes_kernel(const T* __restrict__ x, bf16* __restrict__ y, int V, int R,
                                                         int C, int I2, int J2, int LP, int PPL, int P) {
  if constexpr (!TRANS) {
    // one block per plane row-group: planes are rows of x ([V*R, C]), in-plane (k, l) = c
    const long long row = blockIdx.x;
    const T* xr = x + row * C;
    bf16* yr = y + row * PPL;
    for (int c = threadIdx.x; c < C; c += 256) {
      const int k = c / J2, l = c - k * J2;
      yr[(k + P) * LP + l + P] = (bf16)(float)xr[c];
    }
  } else {
    // 64 x 64 tile of x[v] ([R, C]) through LDS; output plane c, position r
    __shared__ float tile[64][65];
    const int ntc = (C + 63) / 64, ntr = (R + 63) / 64;
    int b = blockIdx.x;
    const int tc = b % ntc; b /= ntc;
    const int tr = b % ntr;
    const int v = b / ntr;
    const int c0 = tc * 64, r0 = tr * 64;
    const T* xv = x + (size_t)v * R * C;
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      const int r = r0 + rr, c = c0 + cc;
      tile[rr][cc] = (r < R && c < C) ? (float)xv[(size_t)r * C + c] : 0.f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int cc = e >> 6, rr = e & 63;
      const int r = r0 + rr, c = c0 + cc;
      if (r < R && c < C) {
        const int i = r / J2, j = r - i * J2;
        y[((size_t)v * C + c) * PPL + (i + P) * LP + j + P] = (bf16)tile[rr][cc];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// conv1x16: Y[v,i,j,k,l,co] = epi(sum_{di,dj,dk,dl} W[co][di,dj,dk,dl] X[v,i+di-P,j+dj-P,k+dk-P,l+dl-P])
// Xp: padded 1-channel planes [V*I*J][PPL]; Wa: A fragments [NT plane offsets][64 lanes][8] bf16
// (lane l: co = l & 15, K rows 8 (l >> 4) .. +7 = taps dk*KS+dl, >= NT zero);
// Y: bf16 [V,I,J,K,L,16]; EPI1X_BIAS_RELU (bias [16]) or EPI1X_MASK (M bf16 [V,I,J,K,L,16]: y *= M > 0).
// ---------------------------------------------------------------------------
template <int KS, int R, int EPI, int K, int L, int PD = 1>
__global__ __launch_bounds__(512, 1) void conv1x16_kernel(const bf16* __restrict__ Xp, const u32x4* __restrict__ Wa,
                                                          const float* __restrict__ bias, const bf16* __restrict__ M,
                                                          bf16* __restrict__ Y, int V, int I, int J, int nt_store,
                                                          long long xlo, long long ylo) {
#if defined(__HIP_DEVICE_COMPILE__)   // device-only body (asm DMA); the host pass keeps the stub
  using C = C1X<KS, K, L>;
  constexpr int P = C::P, NT = C::NT, NW = C::NW, LP = C::LP, PPL = C::PPL, MAXT = C::MAXT;
  constexpr bool X3 = (EPI & EPI1X_X3) != 0;
  constexpr int EP = EPI & ~EPI1X_X3;                 // EPI1X_BIAS_RELU or EPI1X_MASK
  constexpr int PH = X3 ? 3 : 1;                      // phases per item
  constexpr int SPI = KS * PH;                        // steps per item
  constexpr int XOFF = PH == 3 ? 2 * NT * 1024 : C::XOFF;   // both weight sets precede the planes
  constexpr int S = R + KS - 1;          // input j-planes per di = one step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int njb = (J + R - 1) / R;
  // persistent: items (v, i, j-block) bid, bid + G, ...; KS steps (di) per item,
  // the plane DMA stream runs on across items (the next item's first di lands
  // while the current item's last di computes and stores)
  const int nitems = V * I * njb;
  const int G = gridDim.x;
  const int bid = blockIdx.x;
  const int my_items = bid < nitems ? (nitems - 1 - bid) / G + 1 : 0;
  const int nsteps = my_items * SPI;

  // weights (one KiB per plane offset) by LDS-DMA, before the first plane
  for (int q = wave; q < (X3 ? 2 : 1) * NT; q += NW) dma16_lds(Wa + q * 64 + lane, smem + C::WOFF + q * 1024);

  // step n: item bid + G (n / KS), di = n % KS; its S planes -> ring slot n % 2;
  // a plane is 4 copies x NCH KiB-chunks; wave w DMAs chunks w, w + 8, ... of
  // each plane (NCH 2: copy w >> 1, half w & 1)
  constexpr int NCH = C::NCH, NJ = 4 * NCH, JPW = (NJ + NW - 1) / NW;
  uint32_t dvo[JPW], doff[JPW];
  bool jon[JPW];
#pragma unroll
  for (int m = 0; m < JPW; ++m) {
    const int jb = wave + NW * m, cpy = jb / NCH, prt = jb - cpy * NCH;
    dvo[m] = (uint32_t)((prt * 64 + lane) * 16 - 2 * (cpy + C::delta(cpy)));   // element e -> e + c + delta
    doff[m] = (uint32_t)(cpy * C::COPYB + prt * 1024);
    // the last KiB of a copy is partial: its lanes past the copy stay off
    // (exec never empty, so the instruction -- and the vmcnt count -- is fixed)
    jon[m] = jb < NJ && (prt < NCH - 1 || lane < C::COPYB / 16 - 64 * (NCH - 1));
  }
  // the item of a step as mixed-radix digits (jb, ti, tv) of it = (tv I + ti) njb + jb,
  // advanced by G per item with carries: no runtime-divisor division in the
  // step loop (they were ~2 scalar-ALU instructions per MFMA, PMC profiles/r5/)
  const int g_jb = G % njb, g_q = G / njb, g_ti = g_q % I, g_tv = g_q / I;
  auto advance = [&](int& jb, int& ti, int& tv) {
    jb += g_jb;
    int c = jb >= njb ? 1 : 0;
    jb -= c * njb;
    ti += g_ti + c;
    c = ti >= I ? 1 : 0;
    ti -= c * I;
    tv += g_tv + c;
  };
  auto issue = [&](int n, int jb, int ti, int tv) {
    const int di = (n % SPI) % KS;
    const int ii = ti + di - P;
    const bool iv = n < nsteps && ii >= 0 && ii < I;
    const bf16* xsrc = (X3 && (n % SPI) / KS == 1) ? Xp + xlo : Xp;        // phase 1 reads X_lo
    const bf16* xrow = xsrc + ((size_t)(tv * I + (iv ? ii : 0)) * J) * PPL;
    const uint32_t slot = lds0 + XOFF + (uint32_t)((n & 1) * S * C::SLOTB);
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const int jp = jb * R - P + u;
      const bool pv = iv && jp >= 0 && jp < J;
      const uint64_t pb = (uint64_t)(pv ? xrow + (size_t)jp * PPL : Xp);
      typedef int i32x4v __attribute__((ext_vector_type(4)));
      i32x4v rs;
      rs[0] = (int)(uint32_t)pb;
      rs[1] = (int)((uint32_t)(pb >> 32) & 0xffffu);
      rs[2] = pv ? PPL * 2 : 0;
      rs[3] = 0x00020000;
#pragma unroll
      for (int m = 0; m < JPW; ++m) {
        const uint32_t d = slot + (uint32_t)(u * C::SLOTB) + doff[m];
        if (jon[m])
          asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(dvo[m]), "s"(rs),
                       "s"(d)
                       : "memory", "m0");
      }
    }
  };
  int c_jb = bid % njb, c_ti = (bid / njb) % I, c_tv = (bid / njb) / I;   // item of the current step
  issue(0, c_jb, c_ti, c_tv);

  // per-lane transposed-read row offsets (h = 0, 1): K row kk = 8 g + 4 h + q of
  // lane (g = l >> 4, q = (l >> 2) & 3, p = l & 3): tap kk, 4 voxels from 4 p,
  // in the copy that re-aligns the tap's shift; + this wave's first tile
  uint32_t rowoff[2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kk = 8 * g + 4 * h + q;
      int t = 0, c = 0;
      if (kk < NT) {
        const int dk = kk / KS, dl = kk - dk * KS;
        t = (dk - P) * LP + (dl - P);
        c = (4 - ((C::F0 + t) & 3)) & 3;        // re-aligns element F0 + t (+ 16 w + 4 p) to 8 bytes
      }
      rowoff[h] = (uint32_t)(XOFF + c * C::COPYB + (C::F0 + 16 * wave + t + c + C::delta(c) + 4 * p) * 2);
    }
  }
  f32x4 acc[R][MAXT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int tt = 0; tt < MAXT; ++tt) acc[r][tt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const size_t KLs = (size_t)K * L;
  const int co0 = 4 * (lane >> 4);
  u32x2 mreg[EP == EPI1X_MASK ? R : 1][EP == EPI1X_MASK ? MAXT : 1];
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};   // this lane's 4 channels' bias, loaded once (not per store)
  if constexpr (EP == EPI1X_BIAS_RELU) bv = *(const f32x4*)(bias + co0);
  for (int n = 0; n < nsteps; ++n) {
    const int di = (n % SPI) % KS;
    const bool last = (n % SPI) == SPI - 1;             // the item's last step (last phase, di = KS - 1)
    const int wset = (X3 && (n % SPI) / KS == 2) ? NT : 0;   // phase 2 multiplies W_lo
    const int jb = c_jb, ti = c_ti, tv = c_tv;
    const int j0 = jb * R;
    int n_jb = c_jb, n_ti = c_ti, n_tv = c_tv;         // item of step n + 1
    if (last) advance(n_jb, n_ti, n_tv);
    // this step's planes landed (issued one step ago); the previous step's reads are done
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(n + 1, n_jb, n_ti, n_tv);
    if constexpr (EP == EPI1X_MASK) {
      // the item's last step: fetch the ReLU mask of its outputs now, so the
      // loads land under this step's MFMAs instead of stalling the epilogue
      // (issued after the DMA: in-order completion keeps the DMA count exact)
      if (last) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = j0 + r;
          const size_t pbase = (((size_t)tv * I + ti) * J + j) * KLs;
#pragma unroll
          for (int tt = 0; tt < MAXT; ++tt) {
            const int f = C::F0 + 16 * (wave + NW * tt) + (lane & 15);
            const int kp = f / LP, lp = f - kp * LP;
            const int k = kp - P, l = lp - P;
            // address select, not a branch: straight-line loads the waitcnt
            // pass can count past the epilogue's conditional stores
            const bool ok = j < J && f < C::FN && k >= 0 && k < K && l >= 0 && l < L;
            const size_t vox = ok ? pbase + (size_t)k * L + l : 0;
            mreg[r][tt] = *(const u32x2*)(M + vox * 16 + co0);
          }
        }
      }
    }
    const int ii = ti + di - P;
    if (ii >= 0 && ii < I) {
      bf16x8 A[KS];
#pragma unroll
      for (int dj = 0; dj < KS; ++dj) A[dj] = lds_read16(smem, C::WOFF + (wset + di * KS + dj) * 1024 + lane * 16);
      const uint32_t sb = (uint32_t)((n & 1) * S * C::SLOTB);
      xstatic_for<0, S>([&](auto sc) {
        constexpr int s = decltype(sc)::value;   // plane j' = j0 - P + s
        const int jp = j0 - P + s;
        if (jp >= 0 && jp < J) {
          constexpr int dlo = (s - R + 1) > 0 ? (s - R + 1) : 0;
          constexpr int dhi = s < KS - 1 ? s : KS - 1;   // inclusive
          constexpr int NDJ = dhi - dlo + 1;
          const uint32_t a0 = rowoff[0] + sb + s * C::SLOTB, a1 = rowoff[1] + sb + s * C::SLOTB;
          // B fragments read PD tiles ahead of their MFMAs (PD = 1: the round-4
          // schedule; 2: a deeper lookahead for the planes that feed only one or
          // two output planes, A/B via the c1x_pd tuning switch)
          u32x4 B[PD + 1];
          auto load_b = [&](auto tc) {
            constexpr int tt = decltype(tc)::value;
            B[tt % (PD + 1)] = cat4u(lds_read_tr16u(smem, a0 + tt * NW * 32), lds_read_tr16u(smem, a1 + tt * NW * 32));
          };
          xstatic_for<0, (PD < MAXT ? PD : MAXT)>([&](auto tc) { load_b(tc); });
          __builtin_amdgcn_sched_group_barrier(0x100, 2 * (PD < MAXT ? PD : MAXT), 0);
          xstatic_for<0, MAXT>([&](auto tc) {
            constexpr int tt = decltype(tc)::value;
            if constexpr (tt + PD < MAXT) load_b(std::integral_constant<int, tt + PD>{});
            xstatic_for<dlo, dhi + 1>([&](auto dc) {
              constexpr int dj = decltype(dc)::value;
              acc[s - dj][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  A[dj], __builtin_bit_cast(bf16x8, B[tt % (PD + 1)]), acc[s - dj][tt], 0, 0, 0);
            });
            if constexpr (tt + PD < MAXT) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NDJ, 0);
          });
        }
      });
    }
    if (last) {
      // item done: epilogue (stores are not waited for; the next item's planes are in flight)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int j = j0 + r;
        const size_t pbase = (((size_t)tv * I + ti) * J + j) * KLs;
#pragma unroll
        for (int tt = 0; tt < MAXT; ++tt) {
          const int f = C::F0 + 16 * (wave + NW * tt) + (lane & 15);
          const int kp = f / LP, lp = f - kp * LP;
          const int k = kp - P, l = lp - P;
          if (j < J && f < C::FN && k >= 0 && k < K && l >= 0 && l < L) {
            const size_t vox = pbase + (size_t)k * L + l;
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float x = acc[r][tt][q];
              if constexpr (EP == EPI1X_BIAS_RELU) x = fmaxf(x + bv[q], 0.f);
              o[q] = x;
            }
            if constexpr (EP == EPI1X_MASK) {
              const bf16x4 m = __builtin_bit_cast(bf16x4, mreg[r][tt]);
#pragma unroll
              for (int q = 0; q < 4; ++q) o[q] = ((float)m[q] > 0.f) ? o[q] : 0.f;
            }
            bf16x4 out;
#pragma unroll
            for (int q = 0; q < 4; ++q) out[q] = f2bf(o[q]);
            if (nt_store) __builtin_nontemporal_store(__builtin_bit_cast(u32x2, out), (u32x2*)(Y + vox * 16 + co0));
            else *(bf16x4*)(Y + vox * 16 + co0) = out;
            if constexpr (X3) {
              bf16x4 lo;
#pragma unroll
              for (int q = 0; q < 4; ++q) lo[q] = f2bf(o[q] - bf2f(out[q]));
              *(bf16x4*)(Y + ylo + vox * 16 + co0) = lo;
            }
          }
          acc[r][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    c_jb = n_jb; c_ti = n_ti; c_tv = n_tv;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
#endif
}

// ---------------------------------------------------------------------------
// wgrad1x16: weight gradient of a Conv4d whose one operand has ONE channel,
// straight from the padded 1-channel planes (no ij packing):
//
//   R[tap = (dk, dl)][combo = (di, dj)][c] =
//       sum_{o = (v, i, j)} sum_f D[o][f][c] * X1[(v, i+di-P, j+dj-P)][f + s(tap)]
//
// with D a 16-channel volume [V,I,J,K,L,16], X1 padded planes [V*I*J][PPL]
// (pad_planes), f = k*LP + l the padded-stride voxel index and s(tap) =
// dk*LP + dl.  Layer 1 (Cin = 1): D = gradient of its pre-activation, X1 = the
// NC input -> dW1[c][di,dj,dk,dl] = R; the Cout = 1 last layer: D = its input,
// X1 = the output gradient -> dW[0][c][t] = R[c][2P - t] (all four axes flipped).
//
// MFMA: rows = 16 combos (X1 planes of the 5 x 5 neighbourhood, two groups of
// 16: 25 valid), cols = the 16 channels, K = padded positions q = f + s:
//   A[combo][q] = X1[plane(combo)][q]     (ds_read_b64 x 2 at 16-B-aligned q:
//                                          independent of the tap -> reused by 13 taps)
//   B[q][c]     = D[q - s][c]             (ds_read_b64_tr_b16 from the staged D plane,
//                                          any voxel offset is 8-B aligned)
// so the in-plane tap shift moves into the D read and no shifted copies are
// needed.  K index k of a lane group g (= lane >> 4) maps to q0 + 4g + 16h + e
// (h = 0, 1; e = 0..3), which makes both the A reads and the transposed B reads
// of one instruction cover 256 contiguous / bank-distinct bytes.
//
// Work: a step = one output plane o = (v, i, j) in (v, i, j) order; a
// persistent workgroup (one per CU) owns a contiguous range of steps, D planes
// stream through two LDS buffers (read from HBM exactly once), X1 planes
// through a ring of KS rows x (KS + 1) column slots (each X1 plane is DMA'd by
// the KS rows i that use it: L2 traffic on 50 MB).  Wave w accumulates taps
// 13 (w & 1) .. +12 over the q chunks w >> 1, +4, ...; the 4 chunk-waves of a
// tap half are reduced through LDS atomics at the end into one partial per
// workgroup [G][NT][32 combos][16] (+ the bias sum of D on the ones-row MFMA).
// Reference: the autograd of lib/conv4d.py:11-51 for the first / last
// NeighConsensus layers (lib/model.py:130-139).
// ---------------------------------------------------------------------------
template <int KS, int K, int L>
struct W1X {
  static constexpr int P = KS / 2, NT = KS * KS, NW = 8;
  static constexpr int LP = L + 2 * P, PPL = ((K + 2 * P) * LP + 7) / 8 * 8;
  static constexpr int FV = (K - 1) * LP + L;                 // valid f in [0, FV)
  static constexpr int SMAX = (KS - 1) * LP + KS - 1;         // largest tap shift
  static constexpr int NQC = (FV + SMAX + 31) / 32;           // q chunks
  static constexpr int QN = NQC * 32;
  static constexpr int GM = (SMAX + 7) / 8 * 8;               // zero voxels before f = 0
  static constexpr int GBYTES = (GM + QN) * 32;               // one staged D plane
  static constexpr int XS = ((QN * 2 + 255) / 256) * 256 + 16;   // X1 slot stride: = 16 (mod 256) B
  static constexpr int NCOL = KS + 1;
  static constexpr int GOFF = 0, XOFF = 2 * GBYTES;
  static constexpr int LDS = XOFF + KS * NCOL * XS;
  static constexpr int NTW = (NT + 1) / 2;                    // taps per wave half
  static constexpr int NU = (NQC + 3) / 4;                    // chunks per wave (upper bound)
  static constexpr int NXD = (QN * 2 + 1023) / 1024;          // DMA wave-instructions per X1 plane (2 or 3)
  static constexpr int XDMAL = (QN * 2 - (NXD - 1) * 1024) / 16;   // lanes of an X1 plane's last DMA
  static_assert(QN * 2 > 1024 && QN * 2 <= 3072, "two or three DMA wave-instructions per X1 plane");
  static_assert(L * 32 % 16 == 0 && L * 2 <= 64, "one DMA wave-instruction per D row");
  static_assert(NT * 32 * 16 * 4 + 64 <= LDS, "reduction scratch fits the staging buffers");
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <int KS, int K, int L, bool BIAS>
__global__ __launch_bounds__(512, 1) void wgrad1x16_kernel(const bf16* __restrict__ D, const bf16* __restrict__ X1,
                                                           float* __restrict__ part, float* __restrict__ partb,
                                                           int V, int I, int J) {
#if defined(__HIP_DEVICE_COMPILE__)   // device-only body (asm DMA); the host pass keeps the stub
  using C = W1X<KS, K, L>;
  constexpr int P = C::P, NT = C::NT, NW = C::NW, LP = C::LP, PPL = C::PPL, NCOL = C::NCOL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int th = wave & 1, cq = wave >> 1;
  const int T = V * I * J;
  const int G = gridDim.x, bid = blockIdx.x;
  const int t0 = (int)((long long)bid * T / G), t1 = (int)((long long)(bid + 1) * T / G);

  // ---- DMA helpers (asm LDS-DMA; waited for by the vmcnt(0) barriers) ----
  auto dma_x = [&](int v, int i, int di, int jc, int half) {   // X1 plane (v, i+di-P, jc) -> its ring slot
    const int ip = i + di - P;
    const bool pv = ip >= 0 && ip < I && jc >= 0 && jc < J;
    const uint64_t pb = (uint64_t)(pv ? X1 + ((size_t)(v * I + ip) * J + jc) * PPL : X1);
    typedef int i32x4v __attribute__((ext_vector_type(4)));
    i32x4v rs;
    rs[0] = (int)(uint32_t)pb;
    rs[1] = (int)((uint32_t)(pb >> 32) & 0xffffu);
    rs[2] = pv ? PPL * 2 : 0;            // an absent plane reads as zeros
    rs[3] = 0x00020000;
    const uint32_t d = __builtin_amdgcn_readfirstlane(
        lds0 + (uint32_t)(C::XOFF + (di * NCOL + (jc + P + NCOL) % NCOL) * C::XS + half * 1024));
    const uint32_t vo = (uint32_t)(half * 1024 + lane * 16);
    if (half < C::NXD - 1 || lane < C::XDMAL)
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(vo), "s"(rs), "s"(d)
                   : "memory", "m0");
  };
  auto issue_g = [&](int t, int buf) {                          // D plane t (K rows of L voxels) -> buffer
    const bf16* src = D + (size_t)t * K * L * 16;
    for (int k = wave; k < K; k += NW) {
      const uint32_t d = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(C::GOFF + buf * C::GBYTES + (C::GM + k * LP) * 32));
      const bf16* a = src + (size_t)k * L * 16 + lane * 8;
      if (lane < L * 2)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(a), "s"(d) : "memory", "m0");
    }
  };
  auto issue_x_all = [&](int t) {                               // the KS x KS neighbourhood of step t
    const int vi = t / J, j = t - vi * J, v = vi / I, i = vi - v * I;
    for (int e = wave; e < C::NXD * NT; e += NW) {
      const int pl = e / C::NXD;
      dma_x(v, i, pl / KS, j - P + pl % KS, e - pl * C::NXD);
    }
  };
  auto issue_x_col = [&](int t) {                               // the new column j + P of step t
    const int vi = t / J, j = t - vi * J, v = vi / I, i = vi - v * I;
    for (int e = wave; e < C::NXD * KS; e += NW) dma_x(v, i, e / C::NXD, j + P, e % C::NXD);
  };

  // zero both D buffers once: margins, pad columns and the tail stay zero (the DMA writes rows only)
  for (int o = threadIdx.x * 16; o < 2 * C::GBYTES; o += 512 * 16) *(u32x4*)(smem + C::GOFF + o) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  if (t0 < t1) issue_g(t0, 0);

  f32x4 acc[C::NTW][2];
#pragma unroll
  for (int a = 0; a < C::NTW; ++a) acc[a][0] = acc[a][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb = {0.f, 0.f, 0.f, 0.f};
  const u32x4 ones = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};

  // lane constants: combo rows of the two groups, K group, transposed-read row/column
  const int kg = lane >> 4, li = lane & 15;
  const int c0 = (li < NT) ? li : 0, c1 = (16 + li < NT) ? 16 + li : (NT > 16 ? 16 : 0);   // rows >= NT repeat a valid combo
  const int di0 = c0 / KS, dj0 = c0 - di0 * KS, di1 = c1 / KS, dj1 = c1 - di1 * KS;
  const uint32_t gl = (uint32_t)((C::GM + 4 * kg + (li >> 2)) * 32 + 8 * (li & 3) + cq * 1024 - 32 * C::GM);

  // one body per wave (tap half TH, chunk residue CQ, both compile-time): a
  // (tap, chunk) pair whose positions q miss [s, s + FV) of that tap is never
  // issued (12 % of the MFMAs and transposed reads of a full 27-chunk sweep)
  auto body = [&](auto thc, auto cqc, uint32_t xa0, uint32_t xa1, uint32_t ga) {
    constexpr int TH = decltype(thc)::value, CQ = decltype(cqc)::value;
    xstatic_for<0, C::NU>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      constexpr int chunk = CQ + 4 * u;
      if constexpr (chunk < C::NQC) {
        constexpr bool TWO = NT > 16;     // a second 16-combo row group (KS 5: 25 combos; KS 3: 9)
        const u32x4 A0 = cat4u(*(const u32x2*)(smem + xa0 + 256 * u), *(const u32x2*)(smem + xa0 + 256 * u + 32));
        u32x4 A1 = A0;
        if constexpr (TWO) A1 = cat4u(*(const u32x2*)(smem + xa1 + 256 * u), *(const u32x2*)(smem + xa1 + 256 * u + 32));
        xstatic_for<0, C::NTW>([&](auto tc) {
          constexpr int tt = decltype(tc)::value;
          constexpr int tap = C::NTW * TH + tt;
          constexpr int s = (tap / KS) * LP + tap % KS;
          if constexpr (tap < NT && chunk >= s / 32 && chunk <= (s + C::FV - 1) / 32) {
            constexpr uint32_t off = 4096u * u + 32u * (C::GM - s);
            const u32x4 B = cat4u(lds_read_tr16u(smem, ga + off), lds_read_tr16u(smem, ga + off + 512));
            acc[tt][0] = mfma16u(A0, B, acc[tt][0]);
            if constexpr (TWO) acc[tt][1] = mfma16u(A1, B, acc[tt][1]);
            if constexpr (BIAS && TH == 0 && tt == 0) accb = mfma16u(ones, B, accb);
          }
        });
      }
    });
  };

  // the whole persistent loop per wave specialisation (one dispatch, so each
  // body's register allocation is its own)
  float* red = (float*)smem;                                  // [NT][32][16] + bias [16], over the drained buffers
  auto run = [&](auto thc, auto cqc) {
    constexpr int TH = decltype(thc)::value;
    for (int t = t0; t < t1; ++t) {
      const int n = t - t0;
      const int j = t % J;
      if (t == t0 || j == 0) {
        // a new (v, i) row: its whole X1 neighbourhood (the ring slots of the
        // previous row are free once every wave finished the previous step)
        asm_barrier_vm0();
        issue_x_all(t);
      }
      asm_barrier_vm0();               // this step's D plane and X1 planes landed; previous step's reads done
      if (t + 1 < t1) {
        issue_g(t + 1, (n + 1) & 1);
        if ((t + 1) % J != 0) issue_x_col(t + 1);
      }
      const int s0 = di0 * NCOL + (j + dj0 + NCOL) % NCOL, s1 = di1 * NCOL + (j + dj1 + NCOL) % NCOL;
      const uint32_t xa0 = (uint32_t)(C::XOFF + s0 * C::XS + 8 * kg + 64 * cq);
      const uint32_t xa1 = (uint32_t)(C::XOFF + s1 * C::XS + 8 * kg + 64 * cq);
      const uint32_t ga = (uint32_t)(C::GOFF + (n & 1) * C::GBYTES) + gl;
      body(thc, cqc, xa0, xa1, ga);
    }
    asm_barrier_vm0();
    // ---- reduce the 4 chunk-waves of each tap half, one partial per workgroup ----
    for (int o = threadIdx.x; o < NT * 512 + 16; o += 512) red[o] = 0.f;
    __syncthreads();
    xstatic_for<0, C::NTW>([&](auto tc) {
      constexpr int tt = decltype(tc)::value;
      constexpr int tap = C::NTW * TH + tt;
      if constexpr (tap < NT) {
#pragma unroll
        for (int grp = 0; grp < 2; ++grp)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            atomicAdd(&red[(tap * 32 + 16 * grp + 4 * kg + r) * 16 + li], acc[tt][grp][r]);
      }
    });
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  switch (wave) {
    case 0: run(I0{}, I0{}); break;
    case 1: run(I1{}, I0{}); break;
    case 2: run(I0{}, I1{}); break;
    case 3: run(I1{}, I1{}); break;
    case 4: run(I0{}, I2{}); break;
    case 5: run(I1{}, I2{}); break;
    case 6: run(I0{}, I3{}); break;
    default: run(I1{}, I3{}); break;
  }
  if (BIAS && th == 0 && lane < 16) atomicAdd(&red[NT * 512 + lane], accb[0]);
  __syncthreads();
  for (int o = threadIdx.x; o < NT * 512; o += 512) part[(size_t)bid * NT * 512 + o] = red[o];
  if (BIAS && threadIdx.x < 16) partb[(size_t)bid * 16 + threadIdx.x] = red[NT * 512 + threadIdx.x];
#endif
}

}  // namespace ncnet

using namespace ncnet;

// padded-plane geometry of a (K, L) plane for kernel size KS: {LP, PPL}
extern "C" int ncnet_pad_geom(int K, int L, int KS, int* lp, int* ppl) {
  const int P = KS / 2;
  *lp = L + 2 * P;
  *ppl = ((K + 2 * P) * (L + 2 * P) + 7) / 8 * 8;
  return 0;
}

// x: [V, R, C] fp32 or bf16 (x_is_bf16); planes of x (trans 0: N = V*R planes of
// [I2=K, J2=L]) or of its A<->B swap (trans 1: N = V*C planes of [I2=I, J2=J]) into y
// [N, PPL] bf16, whose halo the caller zeroed.
extern "C" int ncnet_pad_planes(const void* x, int x_is_bf16, void* y, int V, int R, int C, int I2, int J2, int KS,
                                int trans, hipStream_t s) {
  int LP, PPL;
  ncnet_pad_geom(I2, J2, KS, &LP, &PPL);
  const int P = KS / 2;
  bf16* yy = (bf16*)y;
  if (!trans) {
    dim3 grid((unsigned)((long long)V * R));
    if (x_is_bf16) hipLaunchKernelGGL((pad_planes_kernel<bf16, false>), grid, dim3(256), 0, s, (const bf16*)x, yy, V, R, C, I2, J2, LP, PPL, P);
    else hipLaunchKernelGGL((pad_planes_kernel<float, false>), grid, dim3(256), 0, s, (const float*)x, yy, V, R, C, I2, J2, LP, PPL, P);
  } else {
    dim3 grid((unsigned)((long long)V * cdiv(R, 64) * cdiv(C, 64)));
    if (x_is_bf16) hipLaunchKernelGGL((pad_planes_kernel<bf16, true>), grid, dim3(256), 0, s, (const bf16*)x, yy, V, R, C, I2, J2, LP, PPL, P);
    else hipLaunchKernelGGL((pad_planes_kernel<float, true>), grid, dim3(256), 0, s, (const float*)x, yy, V, R, C, I2, J2, LP, PPL, P);
  }
  return (int)hipGetLastError();
}

// conv1x16 / wgrad1x16 are instantiated for the training planes: KS 5 at 25 x 25
// (400 px), 20 x 20 (320 px) and 30 x 30 (480 px: three DMAs per staged copy,
// 3 output j-planes per item -- 1 in the bf16x3 mode -- to fit LDS), KS 3 at
// 25 x 25 (the IVD recipe, NC 3,3 / 16,1).  Mirrored in
// ops/neigh_consensus.py FAST1X_SHAPES.
template <int KS, int K, int L, int R, bool X3>
static void c1x_launch(int epi, int V, int I, int J, const bf16* x, const u32x4* w, const float* bias, const bf16* m,
                       bf16* y, int nt_store, long long xlo, long long ylo, hipStream_t s) {
  using C = C1X<KS, K, L>;
  const int nitems = V * I * cdiv(J, R);
  dim3 grid((unsigned)std::min(nitems, device_num_cus())), block(512);   // persistent: one workgroup per CU
  // X3: both weight sets ahead of the planes
  constexpr size_t lds = (size_t)C::lds(R + KS - 1, 1) + (X3 ? (size_t)C::NT * 1024 : 0);
  static_assert(lds <= 160 * 1024, "LDS");
  auto go = [&](auto ec) {
    constexpr int E = decltype(ec)::value;
    if constexpr (!X3 && KS == 5 && K == 25) {
      if (tuning().c1x_pd == 2) {
        hipLaunchKernelGGL((conv1x16_kernel<KS, R, E, K, L, 2>), grid, block, lds, s, x, w, bias, m, y, V, I, J,
                           nt_store, xlo, ylo);
        return;
      }
      if (tuning().c1x_pd == 3) {
        hipLaunchKernelGGL((conv1x16_kernel<KS, R, E, K, L, 3>), grid, block, lds, s, x, w, bias, m, y, V, I, J,
                           nt_store, xlo, ylo);
        return;
      }
    }
    hipLaunchKernelGGL((conv1x16_kernel<KS, R, E, K, L>), grid, block, lds, s, x, w, bias, m, y, V, I, J, nt_store, xlo,
                       ylo);
  };
  if constexpr (X3) {
    if ((epi & ~EPI1X_X3) == EPI1X_BIAS_RELU) go(std::integral_constant<int, EPI1X_BIAS_RELU | EPI1X_X3>{});
    else go(std::integral_constant<int, EPI1X_MASK | EPI1X_X3>{});
  } else {
    if (epi == EPI1X_BIAS_RELU) go(std::integral_constant<int, EPI1X_BIAS_RELU>{});
    else go(std::integral_constant<int, EPI1X_MASK>{});
  }
}

// returns -1 when the shape has no instantiation.  epi | 4 (EPI1X_X3): the
// bf16x3 layer (X_lo = Xp + xlo, Wa = [hi; lo] fragment sets, Y_lo = Y + ylo,
// elements); it runs 3 output j-planes per item (both weight sets in LDS).
extern "C" int ncnet_conv1x16(const void* Xp, const void* Wa, const float* bias, const void* M, void* Y, int V, int I,
                              int J, int K, int L, int KS, int epi, int nt_store, long long xlo, long long ylo,
                              hipStream_t s) {
  const int e = epi & ~EPI1X_X3;
  const bool x3 = (epi & EPI1X_X3) != 0;
  if (e != EPI1X_BIAS_RELU && e != EPI1X_MASK) return -3;
  const bf16* x = (const bf16*)Xp; const u32x4* w = (const u32x4*)Wa; const bf16* m = (const bf16*)M; bf16* y = (bf16*)Y;
  if (KS == 5 && K == 25 && L == 25) {
    if (x3) c1x_launch<5, 25, 25, 3, true>(epi, V, I, J, x, w, bias, m, y, 0, xlo, ylo, s);
    else c1x_launch<5, 25, 25, 5, false>(epi, V, I, J, x, w, bias, m, y, nt_store, 0, 0, s);
  } else if (KS == 5 && K == 20 && L == 20) {
    if (x3) c1x_launch<5, 20, 20, 3, true>(epi, V, I, J, x, w, bias, m, y, 0, xlo, ylo, s);
    else c1x_launch<5, 20, 20, 5, false>(epi, V, I, J, x, w, bias, m, y, nt_store, 0, 0, s);
  } else if (KS == 5 && K == 30 && L == 30) {
    if (x3) c1x_launch<5, 30, 30, 1, true>(epi, V, I, J, x, w, bias, m, y, 0, xlo, ylo, s);
    else c1x_launch<5, 30, 30, 3, false>(epi, V, I, J, x, w, bias, m, y, nt_store, 0, 0, s);
  } else if (KS == 3 && K == 25 && L == 25) {
    if (x3) c1x_launch<3, 25, 25, 3, true>(epi, V, I, J, x, w, bias, m, y, 0, xlo, ylo, s);
    else c1x_launch<3, 25, 25, 5, false>(epi, V, I, J, x, w, bias, m, y, nt_store, 0, 0, s);
  } else return -1;
  return (int)hipGetLastError();
}

template <int KS, int K, int L>
static void w1x_launch(int G, int V, int I, int J, const bf16* d, const bf16* x, float* part, float* partb,
                       hipStream_t s) {
  using C = W1X<KS, K, L>;
  if (partb)
    hipLaunchKernelGGL((wgrad1x16_kernel<KS, K, L, true>), dim3((unsigned)G), dim3(512), (size_t)C::LDS, s, d, x, part,
                       partb, V, I, J);
  else
    hipLaunchKernelGGL((wgrad1x16_kernel<KS, K, L, false>), dim3((unsigned)G), dim3(512), (size_t)C::LDS, s, d, x,
                       part, partb, V, I, J);
}

// wgrad1x16: D bf16 [V,I,J,K,L,16], X1 padded planes [V*I*J][PPL]; part fp32
// [G][KS*KS taps][32 combos][16] (one partial per workgroup, G <= the CU count),
// partb fp32 [G][16] (sum of D; null: none).  Returns -1 for shapes without an instantiation.
extern "C" int ncnet_wgrad1x16(const void* Dp, const void* X1p, float* part, float* partb, int G, int V, int I, int J,
                               int K, int L, int KS, hipStream_t s) {
  if (G < 1) return -2;
  const bf16* d = (const bf16*)Dp; const bf16* x = (const bf16*)X1p;
  if (KS == 5 && K == 25 && L == 25) w1x_launch<5, 25, 25>(G, V, I, J, d, x, part, partb, s);
  else if (KS == 5 && K == 20 && L == 20) w1x_launch<5, 20, 20>(G, V, I, J, d, x, part, partb, s);
  else if (KS == 5 && K == 30 && L == 30) w1x_launch<5, 30, 30>(G, V, I, J, d, x, part, partb, s);
  else if (KS == 3 && K == 25 && L == 25) w1x_launch<3, 25, 25>(G, V, I, J, d, x, part, partb, s);
  else return -1;
  return (int)hipGetLastError();
}
