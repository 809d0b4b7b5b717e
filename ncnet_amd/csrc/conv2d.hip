// NHWC implicit-GEMM 2D convolution with fused epilogues, for the frozen
// ResNet trunk (models/backbones.py FrozenResNetPlan).
//
//   Y[p, co] = act( sum_{dh,dw,ci} X[n, ho*s+dh-pad, wo*s+dw-pad, ci] * W[co, dh, dw, ci]
//                   + bias[co] (+ R[p, co]) ),      p = (n, ho, wo) row-major
//
// GEMM view: M = N*Ho*Wo pixels, N = Cout, K = KH*KW*Cin.  X, Y, R are
// channels-last (NHWC) bf16, W is [Cout][KH][KW][Cin] (a channels-last conv
// weight), bias fp32.  A k-step is one tap x 64 input channels, so the
// im2col gather is one 128-B row load per pixel (zero outside the image) and
// never materialised.  BM x BN output tile per 4-wave workgroup (BN = 128:
// 2x2 waves; BN = 64 for the 64-channel layers: 4x1 waves; BM = 64 for grids
// that would not fill the chip),
// v_mfma_f32_16x16x32_bf16, XOR-swizzled LDS rows, register double buffer,
// XCD-aware tile order.  The epilogue fuses bias, the bottleneck residual and
// ReLU, so a bottleneck is exactly four kernels and no elementwise passes
// (MIOpen: conv + separate bias pass + PyTorch ReLU / add passes).
// Requires Cin % 64 == 0 and Cout % 64 == 0 (every ResNet conv but the stem).
#include "common.h"
#include <stdlib.h>

namespace ncnet {

namespace cv {
constexpr int BK = 64;
// chunk ^ ((row >> 1) & 7): the 16 rows of a ds_read_b128 lane group land on 16
// distinct 16-B bank slots (chunk ^ (row & 7) put rows r and r + 8 on one slot)
__device__ __forceinline__ uint32_t toff(int row, int chunk) { return (uint32_t)(row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4)); }
}  // namespace cv

struct Conv2dArgs {
  const bf16* X; const bf16* W; const float* bias; const bf16* R; bf16* Y;
  int N, H, Wd, Cin, Cout, KH, KW, stride, pad, Ho, Wo;
  int M, tiles_m, tiles_n, relu;
  // conv2d_nhwc_v3 only: X pixel stride Cx and GEMM channels per tap Ck (Cin,
  // Cin for a plain conv; 2 Cin, 3 Cin for the bf16x3 split, see below)
  int Cx, Ck;
};

// Epilogue shared by both kernels, staged through LDS so the global writes
// (and the residual reads) are full 16-B-per-lane row segments: (acc + bias)
// -> 16-bit tile [BM][BN] in LDS (row = pixel), then + residual, ReLU, store.
// The staging rounds to the output type first, as the residual add did in
// bf16 (bit-for-bit the pre-F16 kernels for F16 = false).
template <int BM, int BN, int TM, int TN, int NT, bool F16>
__device__ __forceinline__ void conv2d_epilogue(const f32x4 (&acc)[TM][TN], const Conv2dArgs& p, char* smem, int m0,
                                                int n0, int wm, int wn, int fr, int fq) {
  constexpr int CPR = BN / 8;                     // 16-B chunks per tile row
  constexpr int NIT = (BM * CPR + NT - 1) / NT;   // chunks per thread
  const uint16_t* R = (const uint16_t*)p.R;
  uint16_t* Y = (uint16_t*)p.Y;
  uint16_t* Ts = (uint16_t*)smem;                 // BM * BN * 2 bytes (fits the operand buffers)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * TN * 16 + j * 16 + fr;
    const float b = p.bias[n0 + col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ts[(wm * TM * 16 + i * 16 + 4 * fq + r) * BN + col] = f2s16<F16>(acc[i][j][r] + b);
  }
  __syncthreads();
  // Residual: the chunks of the thread are loaded RB at a time ahead of their
  // stores.  Loaded inside the store loop, each load waited vmcnt(0) -- stores
  // count in vmcnt -- behind the previous chunk's store: NIT serialised memory
  // round trips per tile, which made the short-K residual 1x1 convs (K = 64 ...
  // 256) epilogue-bound.  (All NIT ahead: the scheduler hoists them over the
  // staging and the kernel doubles its VGPRs, halving the occupancy.)
  constexpr int RB = NIT < 4 ? NIT : 4;
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += RB) {
    u32x4 rv[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      rv[q] = u32x4{0u, 0u, 0u, 0u};
      const int c = (int)threadIdx.x + (i0 + q) * NT;
      const int row = c / CPR, cc = c - row * CPR;
      if (R && i0 + q < NIT && c < BM * CPR && m0 + row < p.M)
        rv[q] = *(const u32x4*)(R + (size_t)(m0 + row) * p.Cout + n0 + cc * 8);
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int c = (int)threadIdx.x + (i0 + q) * NT;
      const int row = c / CPR, cc = c - row * CPR;
      const int pix = m0 + row;
      if (i0 + q < NIT && c < BM * CPR && pix < p.M) {
        const u32x4 tv = *(const u32x4*)(Ts + row * BN + cc * 8);
        const size_t o = (size_t)pix * p.Cout + n0 + cc * 8;
        const u32x4 rvi = rv[q];
        u32x4 out;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t w = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v = s162f<F16>((uint16_t)(tv[e] >> (16 * h)));
            if (R) v = s162f<F16>(f2s16<F16>(v + s162f<F16>((uint16_t)(rvi[e] >> (16 * h)))));
            if (p.relu) v = fmaxf(v, 0.f);
            w |= (uint32_t)f2s16<F16>(v) << (16 * h);
          }
          out[e] = w;
        }
        *(u32x4*)(Y + o) = out;
      }
    }
  }
}

// BM x BN output tile: BM = 128, or 64 when the grid would not fill the chip
// (layer3 at the training size: 157 x 2 tiles of 128 on 256 CUs).
// F16: IEEE-half X / W / R / Y (f16 MFMA; the fp16 inference precision)
template <int BM, int BN, bool F16 = false>
__global__ __launch_bounds__(256, 2) void conv2d_nhwc_kernel(Conv2dArgs p) {
  using namespace cv;
  constexpr int WN = BN == 128 ? 2 : 1;          // waves along N
  constexpr int WMW = 4 / WN;                    // waves along M
  constexpr int TM = BM / WMW / 16;              // 16-row MFMA tiles per wave
  constexpr int TN = BN / WN / 16;               // 16-col MFMA tiles per wave (4)
  constexpr int ACH = BM * 8 / 256;              // A chunks per thread
  constexpr int BCH = BN * 8 / 256;              // B chunks per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;
  char* Bs = smem + BM * 128;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % p.tiles_n, tm = bid / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ch = threadIdx.x & 7;

  // this thread's ACH A rows (pixels): image base offset and top-left input coordinate
  int a_hi0[ACH], a_wi0[ACH];
  size_t a_base[ACH];
#pragma unroll
  for (int m = 0; m < ACH; ++m) {
    const int row = (threadIdx.x >> 3) + 32 * m;
    const int pix = m0 + row;
    if (pix < p.M) {
      const int wo = pix % p.Wo, t = pix / p.Wo, ho = t % p.Ho, n = t / p.Ho;
      a_hi0[m] = ho * p.stride - p.pad;
      a_wi0[m] = wo * p.stride - p.pad;
      a_base[m] = (size_t)n * p.H * p.Wd;
    } else {
      a_hi0[m] = -(1 << 28);   // never inside the image
      a_wi0[m] = 0;
      a_base[m] = 0;
    }
  }
  const int K = p.KH * p.KW * p.Cin;
  const int cpt = p.Cin / BK;                    // k-steps per tap
  const int nk = p.KH * p.KW * cpt;

  u32x4 ra[ACH], rb[BCH];
  auto load = [&](int ks) {
    const int tap = ks / cpt, c0 = (ks - tap * cpt) * BK;
    const int dh = tap / p.KW, dw = tap - dh * p.KW;
#pragma unroll
    for (int m = 0; m < ACH; ++m) {
      const int hi = a_hi0[m] + dh, wi = a_wi0[m] + dw;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (hi >= 0 && hi < p.H && wi >= 0 && wi < p.Wd)
        v = *(const u32x4*)(p.X + (a_base[m] + (size_t)hi * p.Wd + wi) * p.Cin + c0 + ch * 8);
      ra[m] = v;
    }
    const int kk = tap * p.Cin + c0 + ch * 8;
#pragma unroll
    for (int m = 0; m < BCH; ++m) {
      const int row = (threadIdx.x >> 3) + 32 * m;
      rb[m] = *(const u32x4*)(p.W + (size_t)(n0 + row) * K + kk);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int m = 0; m < ACH; ++m) *(u32x4*)(As + toff((threadIdx.x >> 3) + 32 * m, ch)) = ra[m];
#pragma unroll
    for (int m = 0; m < BCH; ++m) *(u32x4*)(Bs + toff((threadIdx.x >> 3) + 32 * m, ch)) = rb[m];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  store();
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) load(ks + 1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      bf16x8 af[TM], bfv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = lds_read16(As, toff(wm * TM * 16 + i * 16 + fr, kh * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j) bfv[j] = lds_read16(Bs, toff(wn * TN * 16 + j * 16 + fr, kh * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16t<F16>(__builtin_bit_cast(u32x4, af[i]), __builtin_bit_cast(u32x4, bfv[j]), acc[i][j]);
    }
    __syncthreads();
    if (more) store();
    __syncthreads();
  }

  // epilogue, staged through LDS so the global writes (and the residual
  // reads) are full 16-B-per-lane row segments: (acc + bias) -> bf16 tile
  // [BM][BN] in LDS (row = pixel), then + residual, ReLU, store.
  conv2d_epilogue<BM, BN, TM, TN, 256, F16>(acc, p, smem, m0, n0, wm, wn, fr, fq);
}


// ===========================================================================
// conv2d_nhwc_v2: the same implicit GEMM fed by LDS-DMA through a 4-stage
// ring (BK = 32 = one tap x 32 channels per stage), so global loads run three
// k-steps ahead of the MFMAs with no staging VGPRs and no LDS store
// instructions, and each k-step costs one barrier (v1: register double buffer,
// a load -> store -> barrier -> compute -> barrier sequence per k-step that
// leaves the matrix cores idle during the LDS stores).
//  * every wave issues exactly APW + BPW DMA wave-instructions per stage
//    (out-of-image im2col rows read a 16-byte zero block instead of being
//    masked), so the wait for stage ks is a compile-time vmcnt;
//  * 64-byte LDS rows, chunk c of row r at (c ^ swz(r)) with
//    swz(r) = (r & 1) ^ ((r >> 1) & 2): conflict-free for the ds_read_b128
//    lane groups of the 16x16x32 fragments (searched offline);
//  * the DMA source is swizzled instead of the destination (a DMA
//    instruction writes 1 KB contiguously).
// ===========================================================================
__device__ const uint4 g_zero16 = {0u, 0u, 0u, 0u};

namespace cv2 {
constexpr int BK = 32;
__device__ __forceinline__ int swz(int r) { return (r & 1) ^ ((r >> 1) & 2); }
__device__ __forceinline__ uint32_t roff(int row, int chunk) { return (uint32_t)(row * 64 + ((chunk ^ swz(row)) << 4)); }
}  // namespace cv2

template <int N>
__device__ __forceinline__ void c2_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// NW waves (4: 2x2 / 4x1 of 64x64 / 32x64; 8: 4x2 of 64x64 for the 256x128
// tile, 85 FLOP per L2 byte instead of 64; 8: 4x2 of 64x128 for the 256x256
// tile of the Cout = 256 layers, 128 FLOP per L2 byte: the im2col A rows are
// read once per pixel tile instead of once per 128-channel half), NSTG ring stages.
template <int BM, int BN, int NW, int NSTG, bool F16 = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void conv2d_nhwc_v2_kernel(Conv2dArgs p) {
  using namespace cv2;
  constexpr int NS = NSTG;
  constexpr int NT = NW * 64;
  constexpr int WN = BN >= 128 ? 2 : 1;
  constexpr int WMW = NW / WN;
  constexpr int TM = BM / WMW / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int APW = BM / (16 * NW);            // A DMA instructions (16 rows each) per wave per stage
  constexpr int BPW = BN / (16 * NW);
  static_assert(APW >= 1 && BPW >= 1 && TM >= 1, "tile / wave mismatch");
  constexpr int PER = APW + BPW;
  constexpr int STAGE = (BM + BN) * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % p.tiles_n, tm = bid / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int pos = lane & 3;

  // this lane's A rows (one per DMA instruction): image base and top-left input coordinate
  int a_hi0[APW], a_wi0[APW], a_chunk[APW];
  size_t a_base[APW];
#pragma unroll
  for (int m = 0; m < APW; ++m) {
    const int row = 16 * (wave * APW + m) + (lane >> 2);
    const int pix = m0 + row;
    a_chunk[m] = pos ^ swz(row);
    if (pix < p.M) {
      const int wo = pix % p.Wo, t = pix / p.Wo, ho = t % p.Ho, n = t / p.Ho;
      a_hi0[m] = ho * p.stride - p.pad;
      a_wi0[m] = wo * p.stride - p.pad;
      a_base[m] = (size_t)n * p.H * p.Wd;
    } else {
      a_hi0[m] = -(1 << 28);
      a_wi0[m] = 0;
      a_base[m] = 0;
    }
  }
  const bf16* b_ptr[BPW];
#pragma unroll
  for (int m = 0; m < BPW; ++m) {
    const int row = 16 * (wave * BPW + m) + (lane >> 2);
    b_ptr[m] = p.W + (size_t)(n0 + row) * (p.KH * p.KW * p.Cin) + (pos ^ swz(row)) * 8;
  }
  const int cpt = p.Cin / BK;
  const int nk = p.KH * p.KW * cpt;
  const bf16* zero = (const bf16*)&g_zero16;

  auto issue = [&](int ks, int buf) {
    const int tap = ks / cpt, c0 = (ks - tap * cpt) * BK;
    const int dh = tap / p.KW, dw = tap - dh * p.KW;
    char* sb = smem + buf * STAGE;
#pragma unroll
    for (int m = 0; m < APW; ++m) {
      const int hi = a_hi0[m] + dh, wi = a_wi0[m] + dw;
      const bool ok = hi >= 0 && hi < p.H && wi >= 0 && wi < p.Wd;
      const bf16* src = ok ? p.X + (a_base[m] + (size_t)hi * p.Wd + wi) * p.Cin + c0 + a_chunk[m] * 8 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(void, sb + (wave * APW + m) * 1024), 16, 0, 0);
    }
    const int kk = tap * p.Cin + c0;
#pragma unroll
    for (int m = 0; m < BPW; ++m)
      __builtin_amdgcn_global_load_lds((const void*)(b_ptr[m] + kk),
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
    // stage ks landed once at most the stages issued after it remain in flight
    const int after = min(NS - 2, nk - 1 - ks);
    if (NS >= 4 && after >= 2) c2_wait_barrier<2 * PER>();
    else if (after >= 1) c2_wait_barrier<PER>();
    else c2_wait_barrier<0>();
    if (ks + NS - 1 < nk) issue(ks + NS - 1, (buf + NS - 1) % NS);   // the buffer consumed at ks - 1
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 64;
    bf16x8 af[TM], bfv[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = lds_read16(As, roff(wm * TM * 16 + i * 16 + fr, fq));
#pragma unroll
    for (int j = 0; j < TN; ++j) bfv[j] = lds_read16(Bs, roff(wn * TN * 16 + j * 16 + fr, fq));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = mfma16t<F16>(__builtin_bit_cast(u32x4, af[i]), __builtin_bit_cast(u32x4, bfv[j]), acc[i][j]);
    buf = (buf + 1 == NS) ? 0 : buf + 1;
  }
  __syncthreads();   // all fragment reads done before the epilogue reuses the LDS

  conv2d_epilogue<BM, BN, TM, TN, NT, F16>(acc, p, smem, m0, n0, wm, wn, fr, fq);
}


// ===========================================================================
// conv2d_nhwc_v3: the implicit GEMM as ONE round of workgroups sized to the
// chip (layer 3 at the training size: M = 32 x 25 x 25 = 20,000 pixels, N =
// 256).  v1's 64 x 128 tiles give 626 workgroups = 1.22 rounds of two per CU
// and v2's 256 x 128 tiles 158, so either leaves up to half the chip idle for
// the last round; here the host picks BM = 16 TM rows so that
// ceil(tiles / CUs) x BM is smallest (BM = 80: 250 tiles of 80 x 256, one per
// CU).  BN = 64 TN covers all of N = 256 (TN = 4): per k-step an 80 x 256 tile
// reads 43 KB for 655 K MACs, 30 MAC per L2 byte.
//  * 8 waves = 2 K-groups x 4 N-groups: a ring stage holds BK = 64 (one tap x
//    64 input channels); K-group g runs the MFMAs of the stage's g-th 32-deep
//    half on its own accumulators (TM x TN tiles, 0.45 LDS reads per MFMA),
//    two waves per SIMD hide each other's fragment reads; the two partial sums
//    meet once, through LDS, in the epilogue;
//  * LDS-DMA ring of 3 stages, fixed DMA count per wave and stage (missing
//    rows go to a trash KiB, out-of-image im2col rows read a zero block), so
//    the wait for stage ks is a compile-time vmcnt; issued from asm (the
//    compiler never drains the ring in front of a fragment read);
//  * 128-B LDS rows, chunk c of row r at c ^ (r & 7) (v1's conflict-free
//    swizzle), applied to the DMA source (a DMA instruction writes 1 KiB
//    contiguously: 8 rows);
//  * epilogue: K-group 1 adds its accumulators through an fp32 LDS tile, then
//    bias -> 16-bit staging tile -> residual + ReLU with 16-B coalesced rows.
// Requires Cin % 64 == 0 and Cout % BN == 0.
// ===========================================================================
namespace cv3 {
constexpr int NS = 3;
// chunk ^ ((row >> 1) & 7): the 16 rows of a ds_read_b128 lane group land on 16
// distinct 16-B bank slots (chunk ^ (row & 7) put rows r and r + 8 on one slot)
__device__ __forceinline__ uint32_t toff(int row, int chunk) { return (uint32_t)(row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4)); }
template <int TM, int TN>
struct Geo {
  static constexpr int BM = 16 * TM, BN = 64 * TN;
  static constexpr int NIA = BM / 8, NIB = BN / 8, NI = NIA + NIB;
  static constexpr int PER = (NI + 7) / 8;              // DMA wave-instructions per wave per stage
  static constexpr int STAGE = (BM + BN) * 128;
  static constexpr int TRASH = NS * STAGE;
  static constexpr int PSTR = BN + 4;                    // fp32 row stride of the K-group sum tile
  static constexpr int EPI = BM * PSTR * 4 + BM * BN * 2;
  static constexpr int LDS = (TRASH + 1024) > EPI ? (TRASH + 1024) : EPI;
  static_assert(LDS <= 160 * 1024, "LDS");
};
}  // namespace cv3

template <int N>
__device__ __forceinline__ void c3_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// X3 (fp32-accurate "bf16x3" trunk, FrozenResNetPlan dtype float32): X, R, Y
// hold [hi | lo] bf16 channel pairs (Cx = 2 Cin), the GEMM runs Ck = 3 Cin
// channels per tap, channel c >= 2 Cin reading X channel c - 2 Cin (hi again),
// against W = [W_hi | W_hi | W_lo]: acc = X_hi W_hi + X_lo W_hi + X_hi W_lo
// (fp32 to ~2^-16 relative); the epilogue adds bias and the hi + lo residual
// in fp32 and writes the output split again.
template <int TM, int TN, bool F16 = false, bool X3 = false>
__global__ __launch_bounds__(512, 1) void conv2d_nhwc_v3_kernel(Conv2dArgs p) {
  using namespace cv3;
  using G = Geo<TM, TN>;
  constexpr int BM = G::BM, BN = G::BN, PER = G::PER;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kg = wave >> 2, wn = wave & 3;
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % p.tiles_n, tm = bid / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int K = p.KH * p.KW * p.Ck;

  // this lane's row of each of the wave's PER DMA instructions (instruction
  // j = wave + 8 m: A rows 8 j .. 8 j + 7, then B rows, then trash)
  int a_hi0[PER], a_wi0[PER];
  uint32_t a_pix[PER];            // n * H * W (image base, pixels)
  const bf16* b_src[PER];
  uint32_t dst[PER];
  int kind[PER];                  // 0 A, 1 B, 2 trash (wave-uniform)
  uint32_t coff[PER];             // this lane's source chunk offset (elements)
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int j = wave + 8 * m;
    const int sub = lane >> 3, pos = lane & 7;
    a_hi0[m] = -(1 << 28); a_wi0[m] = 0; a_pix[m] = 0; b_src[m] = p.W; coff[m] = 0;
    if (j < G::NIA) {
      kind[m] = 0;
      const int row = 8 * j + sub;
      const int pix = m0 + row;
      coff[m] = (uint32_t)((pos ^ ((row >> 1) & 7)) * 8);
      dst[m] = (uint32_t)(j * 1024);
      if (pix < p.M) {
        const int wo = pix % p.Wo, t = pix / p.Wo, ho = t % p.Ho, n = t / p.Ho;
        a_hi0[m] = ho * p.stride - p.pad;
        a_wi0[m] = wo * p.stride - p.pad;
        a_pix[m] = (uint32_t)(n * p.H * p.Wd);
      }
    } else if (j < G::NI) {
      kind[m] = 1;
      const int row = 8 * (j - G::NIA) + sub;
      b_src[m] = p.W + (size_t)(n0 + row) * K + (pos ^ ((row >> 1) & 7)) * 8;
      dst[m] = (uint32_t)(BM * 128 + (j - G::NIA) * 1024);
    } else {
      kind[m] = 2;
      dst[m] = (uint32_t)G::TRASH;
    }
  }
  const int cpt = p.Ck / 64;
  const int nk = p.KH * p.KW * cpt;
  const bf16* zero = (const bf16*)&g_zero16;

  auto issue = [&](int ks, int buf) {
    const int tap = ks / cpt, c0 = (ks - tap * cpt) * 64;
    const int cs = c0 >= p.Cx ? c0 - p.Cx : c0;      // X3: the W_lo third reads X_hi again
    const int dh = tap / p.KW, dw = tap - dh * p.KW;
    char* sb = smem + buf * G::STAGE;
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const bf16* src = zero;
      uint32_t d = dst[m];
      if (kind[m] == 0) {
        const int hi = a_hi0[m] + dh, wi = a_wi0[m] + dw;
        const bool ok = (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.Wd;
        const bf16* a = p.X + ((size_t)a_pix[m] + (size_t)(ok ? hi : 0) * p.Wd + (ok ? wi : 0)) * p.Cx + cs + coff[m];
        src = ok ? a : zero;
        d += buf * G::STAGE;
      } else if (kind[m] == 1) {
        src = b_src[m] + tap * p.Ck + c0;
        d += buf * G::STAGE;
      }
      dma16_lds(src, smem + d);
    }
    (void)sb;
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
  const int kc = kg * 4 + fq;      // this lane's 16-B chunk of the 64-deep stage
  int buf = 0;
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk) c3_wait_barrier<PER>();   // stage ks landed; ks + 1 may still fly
    else c3_wait_barrier<0>();
    if (ks + NS - 1 < nk) issue(ks + NS - 1, (buf + NS - 1) % NS);   // into the buffer consumed at ks - 1
    const char* As = smem + buf * G::STAGE;
    const char* Bs = As + BM * 128;
    bf16x8 af[TM], bfv[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = lds_read16(As, toff(i * 16 + fr, kc));
#pragma unroll
    for (int j = 0; j < TN; ++j) bfv[j] = lds_read16(Bs, toff(wn * TN * 16 + j * 16 + fr, kc));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = mfma16t<F16>(__builtin_bit_cast(u32x4, af[i]), __builtin_bit_cast(u32x4, bfv[j]), acc[i][j]);
    buf = (buf + 1 == NS) ? 0 : buf + 1;
  }
  __syncthreads();   // every fragment read done (and every DMA landed: the last wait was vmcnt(0))

  // K-group sum through LDS, then bias -> 16-bit staging tile [BM][BN]
  // (X3: the fp32 sum tile itself is the staging tile)
  float* P = (float*)smem;
  uint16_t* S = (uint16_t*)(smem + BM * G::PSTR * 4);
  if (kg == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) P[(i * 16 + 4 * fq + r) * G::PSTR + wn * TN * 16 + j * 16 + fr] = acc[i][j][r];
  }
  __syncthreads();
  if (kg == 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * TN * 16 + j * 16 + fr;
      const float b = p.bias[n0 + col];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + 4 * fq + r;
          const float v = acc[i][j][r] + P[row * G::PSTR + col] + b;
          if constexpr (X3) P[row * G::PSTR + col] = v;
          else S[row * BN + col] = f2s16<F16>(v);
        }
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  const uint16_t* R = (const uint16_t*)p.R;
  uint16_t* Y = (uint16_t*)p.Y;
  // residual loads RB at a time ahead of their stores (conv2d_epilogue)
  constexpr int NIT = (BM * CPR + 511) / 512;
  constexpr int RB = NIT < (X3 ? 2 : 4) ? NIT : (X3 ? 2 : 4);
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += RB) {
    u32x4 rh[RB], rl[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      rh[q] = rl[q] = u32x4{0u, 0u, 0u, 0u};
      const int c = (int)threadIdx.x + (i0 + q) * 512;
      const int row = c / CPR, cc = c - row * CPR;
      if (R && i0 + q < NIT && c < BM * CPR && m0 + row < p.M) {
        const size_t o = (size_t)(m0 + row) * (X3 ? 2 * p.Cout : p.Cout) + n0 + cc * 8;
        rh[q] = *(const u32x4*)(R + o);
        if constexpr (X3) rl[q] = *(const u32x4*)(R + o + p.Cout);
      }
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
    const int c = (int)threadIdx.x + (i0 + q) * 512;
    const int row = c / CPR, cc = c - row * CPR;
    const int pix = m0 + row;
    if (i0 + q >= NIT || c >= BM * CPR || pix >= p.M) continue;
    if constexpr (X3) {
      // 8 channels: fp32 sum (+ residual hi + lo), ReLU, split into hi / lo
      const f32x4 v0 = *(const f32x4*)(P + row * G::PSTR + cc * 8);
      const f32x4 v1 = *(const f32x4*)(P + row * G::PSTR + cc * 8 + 4);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const size_t o = (size_t)pix * (2 * p.Cout) + n0 + cc * 8;
      if (R) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] += s162f<false>((uint16_t)(rh[q][e >> 1] >> (16 * (e & 1)))) +
                  s162f<false>((uint16_t)(rl[q][e >> 1] >> (16 * (e & 1))));
      }
      u32x4 oh, ol;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t wh = 0, wl = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float x = v[2 * e + h];
          if (p.relu) x = fmaxf(x, 0.f);
          const uint16_t hb = f2s16<false>(x);
          wh |= (uint32_t)hb << (16 * h);
          wl |= (uint32_t)f2s16<false>(x - s162f<false>(hb)) << (16 * h);
        }
        oh[e] = wh; ol[e] = wl;
      }
      *(u32x4*)(Y + o) = oh;
      *(u32x4*)(Y + o + p.Cout) = ol;
    } else {
      const u32x4 tv = *(const u32x4*)(S + row * BN + cc * 8);
      const size_t o = (size_t)pix * p.Cout + n0 + cc * 8;
      const u32x4 rv = rh[q];
      u32x4 out;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t w = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v = s162f<F16>((uint16_t)(tv[e] >> (16 * h)));
          if (R) v = s162f<F16>(f2s16<F16>(v + s162f<F16>((uint16_t)(rv[e] >> (16 * h)))));
          if (p.relu) v = fmaxf(v, 0.f);
          w |= (uint32_t)f2s16<F16>(v) << (16 * h);
        }
        out[e] = w;
      }
      *(u32x4*)(Y + o) = out;
    }
    }
  }
}

static int c3_pick_tm(int M, int Cout, int Cin, int TN, int ncu, long long* cost);
// mode 0: bf16, 1: IEEE half, 2: bf16x3
template <int TM, int TN>
static void c3_launch1(int mode, dim3 g, dim3 b, hipStream_t stream, const Conv2dArgs& p) {
  const size_t lds = (size_t)cv3::Geo<TM, TN>::LDS;
  if (mode == 1) hipLaunchKernelGGL((conv2d_nhwc_v3_kernel<TM, TN, true, false>), g, b, lds, stream, p);
  else if (mode == 2) hipLaunchKernelGGL((conv2d_nhwc_v3_kernel<TM, TN, false, true>), g, b, lds, stream, p);
  else hipLaunchKernelGGL((conv2d_nhwc_v3_kernel<TM, TN, false, false>), g, b, lds, stream, p);
}
template <int TN>
static void c3_launch(int tm, int mode, dim3 g, dim3 b, hipStream_t stream, const Conv2dArgs& p) {
  if (tm == 3) c3_launch1<3, TN>(mode, g, b, stream, p);
  else if (tm == 4) c3_launch1<4, TN>(mode, g, b, stream, p);
  else if (tm == 5) c3_launch1<5, TN>(mode, g, b, stream, p);
  else c3_launch1<6, TN>(mode, g, b, stream, p);
}
// launch v3 with its tile choice; false when it does not apply
static bool c3_run(Conv2dArgs& p, int mode, hipStream_t stream) {
  const int TNv = (p.Cout % 256 == 0) ? 4 : (p.Cout % 128 == 0) ? 2 : 1;
  const int tm = c3_pick_tm(p.M, p.Cout, p.Ck, TNv, device_num_cus(), nullptr);
  if (!tm || p.Cx % 64) return false;
  p.tiles_n = p.Cout / (64 * TNv);
  p.tiles_m = cdiv(p.M, 16 * tm);
  dim3 g3((unsigned)(p.tiles_m * p.tiles_n)), b3(512);
  if (TNv == 4) c3_launch<4>(tm, mode, g3, b3, stream, p);
  else if (TNv == 2) c3_launch<2>(tm, mode, g3, b3, stream, p);
  else c3_launch<1>(tm, mode, g3, b3, stream, p);
  return true;
}

// v3 tile rows: BM = 16 TM minimising (rounds of one workgroup per CU) x BM,
// ties to the larger tile (fewer weight re-reads).  Returns TM, or 0 when v3
// does not apply (Cout % BN, Cin % 64).
static int c3_pick_tm(int M, int Cout, int Cin, int TN, int ncu, long long* cost) {
  if (Cin % 64 || Cout % (64 * TN)) return 0;
  const int tn = Cout / (64 * TN);
  int best = 0;
  long long bc = 0;
  for (int tm = 3; tm <= 6; ++tm) {
    const long long tiles = (long long)cdiv(M, 16 * tm) * tn;
    const long long c = ((tiles + ncu - 1) / ncu) * (long long)(16 * tm);
    if (!best || c < bc || (c == bc && tm > best)) { best = tm; bc = c; }
  }
  if (cost) *cost = bc;
  return best;
}

}  // namespace ncnet

using namespace ncnet;

// f16: X / W / R / Y are IEEE half (else bf16).
extern "C" int ncnet_conv2d_nhwc(const void* X, const void* W, const float* bias, const void* R, void* Y, int N, int H,
                                 int Wd, int Cin, int Cout, int KH, int KW, int stride, int pad, int relu, int f16,
                                 hipStream_t stream) {
  if (Cin % 64 || Cout % 64 || stride < 1) return -1;   // (v2 needs Cin % 32; both kernels share the check)
  Conv2dArgs p;
  p.X = (const bf16*)X; p.W = (const bf16*)W; p.bias = bias; p.R = (const bf16*)R; p.Y = (bf16*)Y;
  p.N = N; p.H = H; p.Wd = Wd; p.Cin = Cin; p.Cout = Cout; p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad;
  p.Ho = (H + 2 * pad - KH) / stride + 1;
  p.Wo = (Wd + 2 * pad - KW) / stride + 1;
  p.M = N * p.Ho * p.Wo;
  p.relu = relu;
  p.Cx = Cin; p.Ck = Cin;
  const int BN = (Cout % 128 == 0) ? 128 : 64;
  p.tiles_n = Cout / BN;
  // 128-row tiles unless that leaves fewer than two workgroups per CU
  const int BM = (cdiv(p.M, 128) * p.tiles_n < 512) ? 64 : 128;
  p.tiles_m = cdiv(p.M, BM);
  dim3 grid((unsigned)(p.tiles_m * p.tiles_n)), block(256);
  // Variant choice (measured per ResNet layer, scripts/conv_bench.py): the
  // 256 x 128 DMA-ring tile wins wherever it still gives >= 1.5 workgroups
  // per CU (3200-px InLoc layers 2-3: 3x3 convs 610-670 -> 760-790 TFLOP/s);
  // smaller grids and the 64-channel layers stay on the v1 kernel.
  // NCNET_CONV2D_VARIANT=1 / 2 forces v1 / the DMA ring (with 128-row tiles
  // unless NCNET_CONV2D_BIG is set or the grid is large).
  const int variant = tuning().conv2d_variant;
  // v3 (one round of chip-sized tiles) where measured faster (scripts/conv_bench.py,
  // profiles/r4/trunk): the N <= 256 convs with a deep K (layer-3 3x3 convs
  // at the training size: 48.7 -> 37.7 us, their reduce 1x1: 27.0 -> 21.9 us)
  const int t256 = cdiv(p.M, 256) * p.tiles_n;
  const bool big = BN == 128 && (variant == 0 ? t256 >= 384 : t256 >= 512);
  // (grids big enough for the 256 x 128 DMA-ring tile keep it: InLoc 3200 px
  // layer 3, 467 us v2 vs 707 us v3)
  const bool v3_auto = variant == 0 && tuning().conv2d_v3 && !big && Cout <= 256 && KH * KW * Cin >= 1024;
  if ((variant == 3 || v3_auto) && c3_run(p, f16 ? 1 : 0, stream)) return (int)hipGetLastError();
  // 256 x 256 tiles for Cout % 256 == 0 with a deep K (the layer-3 3x3 convs,
  // K = 2304: 447 -> 417 us, the stride-2 one 495 -> 447 us at the batch-256
  // training trunk, profiles/r6/kernels/conv_bench_400_n512_256tile.txt); the
  // short-K 1x1s (K <= 512) measured slower than the 256 x 128 tile.  Auto where
  // the grid still gives >= 3 workgroups per CU; forced by variant 4.
  const int t2562 = cdiv(p.M, 256) * (Cout / 256);
  const bool big2 = Cout % 256 == 0 && !f16 &&
                    ((variant == 0 && tuning().conv2d_256 && t2562 >= 768 && KH * KW * Cin >= 1024) || variant == 4);
  if (big2) {
    p.tiles_n = Cout / 256;
    p.tiles_m = cdiv(p.M, 256);
    dim3 g2((unsigned)(p.tiles_m * p.tiles_n)), b2(512);
    const size_t lds = (size_t)4 * (256 + 256) * 64;   // = the 256 x 256 16-bit epilogue tile
    hipLaunchKernelGGL((conv2d_nhwc_v2_kernel<256, 256, 8, 4>), g2, b2, lds, stream, p);
    return (int)hipGetLastError();
  }
  if (big && variant != 1) {
    p.tiles_m = cdiv(p.M, 256);
    dim3 g2((unsigned)(p.tiles_m * p.tiles_n)), b2(512);
    const size_t lds = (size_t)3 * (256 + BN) * 64;
    if (f16) hipLaunchKernelGGL((conv2d_nhwc_v2_kernel<256, 128, 8, 3, true>), g2, b2, lds, stream, p);
    else hipLaunchKernelGGL((conv2d_nhwc_v2_kernel<256, 128, 8, 3>), g2, b2, lds, stream, p);
    return (int)hipGetLastError();
  }
  if (variant == 2 && !f16) {
    const size_t lds = (size_t)4 * (BM + BN) * 64;
#define LC3(BMV, BNV) hipLaunchKernelGGL((conv2d_nhwc_v2_kernel<BMV, BNV, 4, 4>), grid, block, lds, stream, p)
    if (BM == 128) { if (BN == 128) LC3(128, 128); else LC3(128, 64); }
    else { if (BN == 128) LC3(64, 128); else LC3(64, 64); }
#undef LC3
    return (int)hipGetLastError();
  }
  const size_t lds = (size_t)(BM + BN) * 128;
#define LC2(BMV, BNV) do { if (f16) hipLaunchKernelGGL((conv2d_nhwc_kernel<BMV, BNV, true>), grid, block, lds, stream, p); \
                           else hipLaunchKernelGGL((conv2d_nhwc_kernel<BMV, BNV>), grid, block, lds, stream, p); } while (0)
  if (BM == 128) { if (BN == 128) LC2(128, 128); else LC2(128, 64); }
  else { if (BN == 128) LC2(64, 128); else LC2(64, 64); }
#undef LC2
  return (int)hipGetLastError();
}

// bf16x3 (fp32-accurate) conv: X [N,H,W,2 Cin] = [hi | lo] bf16 pairs, W [Cout][KH][KW][3 Cin]
// = [W_hi | W_hi | W_lo], R / Y [.., 2 Cout] pairs, bias fp32 (conv2d_nhwc_v3 X3).
extern "C" int ncnet_conv2d_nhwc_x3(const void* X, const void* W, const float* bias, const void* R, void* Y, int N,
                                    int H, int Wd, int Cin, int Cout, int KH, int KW, int stride, int pad, int relu,
                                    hipStream_t stream) {
  if (Cin % 64 || Cout % 64 || stride < 1) return -1;
  Conv2dArgs p;
  p.X = (const bf16*)X; p.W = (const bf16*)W; p.bias = bias; p.R = (const bf16*)R; p.Y = (bf16*)Y;
  p.N = N; p.H = H; p.Wd = Wd; p.Cin = Cin; p.Cout = Cout; p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad;
  p.Ho = (H + 2 * pad - KH) / stride + 1;
  p.Wo = (Wd + 2 * pad - KW) / stride + 1;
  p.M = N * p.Ho * p.Wo;
  p.relu = relu;
  p.Cx = 2 * Cin; p.Ck = 3 * Cin;
  if (!c3_run(p, 2, stream)) return -1;
  return (int)hipGetLastError();
}

