// j-offset <-> channel re-encoding for the 1-channel NC-Net layers.
//
// A Conv4d with one input (or one output) channel wastes 15/16 of an MFMA.
// Moving the kernel's j-offset (dj) into the channel axis turns it into a
// 16 -> 16 convolution whose kernel is non-zero only on the dj = P planes:
//
//   Cin = 1 :  X0s[v,i,j,k,l,c] = X0[v,i,j+(c-P),k,l]        (jpack, sgn = +1)
//              Y = conv16_{dj=P}(X0s, W1s),  W1s[co][c][di][P][dk][dl] = W1[co][0][di][c][dk][dl]
//   Cout = 1:  Z = conv16_{dj=P}(X2, Wz),    Wz[c][ci][di][P][dk][dl]  = W3[0][ci][di][c][dk][dl]
//              y[v,i,j,k,l] = sum_c Z[v,i,j+(c-P),k,l,c]      (jsum; its adjoint is jpack with sgn = -1)
//
// so forward, data-gradient and weight-gradient of those layers all run on the
// conv16 / wgrad16 MFMA kernels over KS planes instead of KS*KS.
//
// ij encoding (ijpack / ijsum): BOTH plane offsets (di, dj) go into channels,
// combo q = di*KS + dj, 16 combos per group, G = ceil(KS*KS/16) groups
// (KS=3: 1 group, 9/16 channels used; KS=5: 2 groups, 25/32):
//   S[g][v,i,j,k,l,c] = X[v, i+sgn*(di-P), j+sgn*(dj-P), k, l],  q = 16g + c
//   y[v,i,j,k,l]      = act(b + sum_q Z[g][v, i+sgn*(di-P), j+sgn*(dj-P), k, l, c])
// and the 1-channel layers become conv16 over G "group planes" with (dk, dl)
// taps only: 2.5x (KS=5) / 3x (KS=3) fewer MFMAs than the j encoding.
#include "common.h"
#include <hip/hip_fp8.h>
#include <stdlib.h>

namespace ncnet {

// S[v,i,j,k,l,c] = X[v,i,j+sgn*(c-P),k,l] for c < KS (zero outside the volume / for c >= KS).
template <typename T>
__global__ __launch_bounds__(256) void jpack_kernel(const T* __restrict__ X, bf16* __restrict__ S, long long nvox,
                                                    int J, int KL, int KS, int sgn) {
  // grid (planes, ceil(KL/256)): the plane index is block-uniform, so its
  // decomposition is scalar and no per-thread 64-bit division is needed
  const int kl = blockIdx.y * 256 + threadIdx.x;
  if (kl >= KL) return;
  const int P = KS / 2;
  const long long plane = blockIdx.x;      // (v*I + i)*J + j
  const int j = (int)(blockIdx.x % J);
  const long long e = plane * KL + kl;
  bf16x8 lo, hi;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    int jj = j + sgn * (c - P);
    float v = 0.f;
    if (c < KS && jj >= 0 && jj < J) v = (float)X[(plane + (jj - j)) * KL + kl];
    lo[c] = f2bf(v);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) hi[c] = f2bf(0.f);
  bf16x8* o = (bf16x8*)(S + e * 16);
  o[0] = lo;
  o[1] = hi;
}

// y[v,i,j,k,l] = act(bias + sum_{c<KS} Z8[c][v,i,j+sgn*(c-P),k,l]),  Z8 fp32 channel-planar [8][...]
// (sgn = +1: the Cout=1 forward; sgn = -1: adjoint of jpack(+1), the Cin=1 data gradient)
__global__ __launch_bounds__(256) void jsum_kernel(const float* __restrict__ Z8, const float* __restrict__ bias,
                                                   float* __restrict__ y, long long nvox, int J, int KL, int KS,
                                                   int relu, int sgn) {
  const int kl = blockIdx.y * 256 + threadIdx.x;
  if (kl >= KL) return;
  const int P = KS / 2;
  const int j = (int)(blockIdx.x % J);
  const long long e = (long long)blockIdx.x * KL + kl;
  float s = bias ? bias[0] : 0.f;
  for (int c = 0; c < KS; ++c) {
    int jj = j + sgn * (c - P);
    if (jj >= 0 && jj < J) s += Z8[(long long)c * nvox + e + (long long)(jj - j) * KL];
  }
  y[e] = relu ? fmaxf(s, 0.f) : s;
}

// ---------------------------------------------------------------------------
// F8OUT: S is OCP fp8 e4m3 [G][..][16] (inference path), else bf16.
template <typename T, int KS, bool F8OUT, bool NT = false>
__global__ __launch_bounds__(256) void ijpack_kernel(const T* __restrict__ X, void* __restrict__ S, long long nvox,
                                                     int I, int J, int KL, int sgn) {
  constexpr int P = KS / 2, NQ = KS * KS, G = (NQ + 15) / 16;
  const int kl = blockIdx.y * 256 + threadIdx.x;
  if (kl >= KL) return;
  const long long plane = blockIdx.x;       // (v*I + i)*J + j, block-uniform
  const int j = (int)(blockIdx.x % J);
  const int i = (int)((blockIdx.x / J) % I);
  const long long e = plane * KL + kl;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float vals[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int q = 16 * g + c;
      float v = 0.f;
      if (q < NQ) {
        const int ii = i + sgn * (q / KS - P), jj = j + sgn * (q % KS - P);
        if (ii >= 0 && ii < I && jj >= 0 && jj < J) v = (float)X[(plane + (long long)(ii - i) * J + (jj - j)) * KL + kl];
      }
      vals[c] = v;
    }
    if (F8OUT) {
      u32x4 o;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        uint32_t p = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          p |= (uint32_t)__hip_cvt_float_to_fp8(vals[4 * w + b], __HIP_SATFINITE, __HIP_E4M3) << (8 * b);
        o[w] = p;
      }
      *(u32x4*)((uint8_t*)S + ((long long)g * nvox + e) * 16) = o;
    } else {
      bf16x8 h[2];
#pragma unroll
      for (int c = 0; c < 16; ++c) h[c >> 3][c & 7] = f2bf(vals[c]);
      bf16x8* o = (bf16x8*)((bf16*)S + ((long long)g * nvox + e) * 16);
      if (NT) {   // streaming (non-temporal) stores: the 1.6 GB output never fits L2
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, h[0]), (u32x4*)o);
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, h[1]), (u32x4*)o + 1);
      } else {
        o[0] = h[0];
        o[1] = h[1];
      }
    }
  }
}

// ijpack v2 (bf16 output, opt-in NCNET_IJPACK_V=2): one thread per 16-byte
// output chunk (8 channels of one voxel), grid (plane, group), so every
// wave-store is 1 KB of contiguous bytes.  Measured SLOWER than v1 at the
// training shape (64 x 25^4, KS=5: 0.736 vs 0.571 ms, profiles/r1s3_kbench.json):
// each lane then issues 8 scalar 2-byte gathers per 16 bytes written instead of
// 16 per 32, and the lane pairs of one voxel read different planes.
template <typename T, int KS>
__global__ __launch_bounds__(256) void ijpack2_kernel(const T* __restrict__ X, bf16* __restrict__ S, long long nvox,
                                                      int I, int J, int KL, int sgn) {
  constexpr int P = KS / 2, NQ = KS * KS;
  const long long plane = blockIdx.x;       // (v*I + i)*J + j, block-uniform
  const int grp = blockIdx.y;
  const int j = (int)(blockIdx.x % J);
  const int i = (int)((blockIdx.x / J) % I);
  const T* xp = X + plane * KL;
  bf16* sp = S + ((long long)grp * nvox + plane * KL) * 16;
  for (int ch = threadIdx.x; ch < 2 * KL; ch += 256) {
    const int kl = ch >> 1, h = ch & 1;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = 16 * grp + 8 * h + e;
      float v = 0.f;
      if (q < NQ) {
        const int ii = i + sgn * (q / KS - P), jj = j + sgn * (q % KS - P);
        if (ii >= 0 && ii < I && jj >= 0 && jj < J) v = (float)xp[((ii - i) * J + (jj - j)) * KL + kl];
      }
      o[e] = f2bf(v);
    }
    *(bf16x8*)(sp + ch * 8) = o;
  }
}

// ijpack v3 (bf16 output, NCNET_IJPACK_V=3): a workgroup owns a range of KLT
// voxels of one output plane (v, i, j).  The KS*KS shifted source planes of
// that range are first staged in LDS with coalesced loads (one 1-channel row
// per combo), then every thread writes whole 16-byte chunks (8 channels of a
// voxel) read back from LDS: each wave-store is 1 KB of contiguous bytes.
template <typename T, int KS>
__global__ __launch_bounds__(256) void ijpack3_kernel(const T* __restrict__ X, bf16* __restrict__ S, long long nvox,
                                                      int I, int J, int KL, int KLT, int sgn) {
  constexpr int P = KS / 2, NQ = KS * KS, G = (NQ + 15) / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* src = (bf16*)smem;                   // [NQ][KLT]
  const long long plane = blockIdx.x;        // (v*I + i)*J + j, block-uniform
  const int j = (int)(blockIdx.x % J);
  const int i = (int)((blockIdx.x / J) % I);
  const int kl0 = blockIdx.y * KLT, n = min(KLT, KL - kl0);
  for (int q = 0; q < NQ; ++q) {
    const int ii = i + sgn * (q / KS - P), jj = j + sgn * (q % KS - P);
    const bool ok = ii >= 0 && ii < I && jj >= 0 && jj < J;   // uniform over the block
    const T* xp = X + (plane + (long long)(ii - i) * J + (jj - j)) * KL + kl0;
    for (int e = threadIdx.x; e < n; e += 256) src[q * KLT + e] = ok ? f2bf((float)xp[e]) : f2bf(0.f);
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    bf16* sp = S + ((long long)g * nvox + plane * KL + kl0) * 16;
    for (int ch = threadIdx.x; ch < 2 * n; ch += 256) {
      const int vox = ch >> 1, h = ch & 1;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = 16 * g + 8 * h + e;
        o[e] = q < NQ ? src[q * KLT + vox] : f2bf(0.f);
      }
      *(bf16x8*)(sp + ch * 8) = o;
    }
  }
}

// Z is channel-planar by combo: Z[q][voxel] (conv16 planar fp32 epilogue).
template <int KS>
__global__ __launch_bounds__(256) void ijsum_kernel(const float* __restrict__ Z, const float* __restrict__ bias,
                                                    float* __restrict__ y, long long nvox, int I, int J, int KL,
                                                    int relu, int sgn) {
  constexpr int P = KS / 2, NQ = KS * KS;
  const int kl = blockIdx.y * 256 + threadIdx.x;
  if (kl >= KL) return;
  const int j = (int)(blockIdx.x % J);
  const int i = (int)((blockIdx.x / J) % I);
  const long long e = (long long)blockIdx.x * KL + kl;
  float s = bias ? bias[0] : 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int ii = i + sgn * (q / KS - P), jj = j + sgn * (q % KS - P);
    if (ii >= 0 && ii < I && jj >= 0 && jj < J)
      s += Z[(long long)q * nvox + e + ((long long)(ii - i) * J + (jj - j)) * KL];
  }
  y[e] = relu ? fmaxf(s, 0.f) : s;
}

}  // namespace ncnet

using namespace ncnet;

extern "C" int ncnet_jpack(const void* X, int x_is_bf16, void* S, int V, int I, int J, int K, int L, int KS, int sgn,
                           hipStream_t stream) {
  if (KS > 8 || KS < 1) return -1;
  long long nvox = (long long)V * I * J * K * L;
  dim3 grid((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256));
  if (x_is_bf16)
    hipLaunchKernelGGL((jpack_kernel<bf16>), grid, dim3(256), 0, stream, (const bf16*)X, (bf16*)S, nvox, J, K * L, KS, sgn);
  else
    hipLaunchKernelGGL((jpack_kernel<float>), grid, dim3(256), 0, stream, (const float*)X, (bf16*)S, nvox, J, K * L, KS, sgn);
  return (int)hipGetLastError();
}

extern "C" int ncnet_jsum(const float* Z8, const float* bias, float* y, int V, int I, int J, int K, int L, int KS,
                          int relu, int sgn, hipStream_t stream) {
  if (KS > 8 || KS < 1) return -1;
  long long nvox = (long long)V * I * J * K * L;
  hipLaunchKernelGGL(jsum_kernel, dim3((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256)), dim3(256), 0, stream,
                     Z8, bias, y, nvox, J, K * L, KS, relu, sgn);
  return (int)hipGetLastError();
}

extern "C" int ncnet_ijpack(const void* X, int x_is_bf16, void* S, int V, int I, int J, int K, int L, int KS, int sgn,
                            int s_fp8, hipStream_t stream) {
  long long nvox = (long long)V * I * J * K * L;
  const char* ev = getenv("NCNET_IJPACK_V");
  if (!s_fp8 && !(ev && atoi(ev) >= 1 && atoi(ev) <= 3)) {   // default: v1 with non-temporal stores
    dim3 grid4((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256));
#define IJP4(T, KSV) hipLaunchKernelGGL((ijpack_kernel<T, KSV, false, true>), grid4, dim3(256), 0, stream, (const T*)X, S, nvox, I, J, K * L, sgn)
    if (KS == 5) { if (x_is_bf16) IJP4(bf16, 5); else IJP4(float, 5); }
    else if (KS == 3) { if (x_is_bf16) IJP4(bf16, 3); else IJP4(float, 3); }
    else return -1;
#undef IJP4
    return (int)hipGetLastError();
  }
  if (!s_fp8 && ev && atoi(ev) == 3) {
    const int KLT = min(K * L, 1024);
    dim3 grid3((unsigned)(V * I * J), (unsigned)((K * L + KLT - 1) / KLT));
    const size_t lds = (size_t)KS * KS * KLT * 2;
#define IJP3(T, KSV) hipLaunchKernelGGL((ijpack3_kernel<T, KSV>), grid3, dim3(256), lds, stream, (const T*)X, (bf16*)S, nvox, I, J, K * L, KLT, sgn)
    if (KS == 5) { if (x_is_bf16) IJP3(bf16, 5); else IJP3(float, 5); }
    else if (KS == 3) { if (x_is_bf16) IJP3(bf16, 3); else IJP3(float, 3); }
    else return -1;
#undef IJP3
    return (int)hipGetLastError();
  }
  if (!s_fp8 && ev && atoi(ev) == 2) {
    dim3 grid2((unsigned)(V * I * J), (unsigned)((KS * KS + 15) / 16));
#define IJP2(T, KSV) hipLaunchKernelGGL((ijpack2_kernel<T, KSV>), grid2, dim3(256), 0, stream, (const T*)X, (bf16*)S, nvox, I, J, K * L, sgn)
    if (KS == 5) { if (x_is_bf16) IJP2(bf16, 5); else IJP2(float, 5); }
    else if (KS == 3) { if (x_is_bf16) IJP2(bf16, 3); else IJP2(float, 3); }
    else return -1;
#undef IJP2
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256));
#define IJP(T, KSV) do { if (s_fp8) hipLaunchKernelGGL((ijpack_kernel<T, KSV, true>), grid, dim3(256), 0, stream, (const T*)X, S, nvox, I, J, K * L, sgn); \
                         else hipLaunchKernelGGL((ijpack_kernel<T, KSV, false>), grid, dim3(256), 0, stream, (const T*)X, S, nvox, I, J, K * L, sgn); } while (0)
  if (KS == 5) { if (x_is_bf16) IJP(bf16, 5); else IJP(float, 5); }
  else if (KS == 3) { if (x_is_bf16) IJP(bf16, 3); else IJP(float, 3); }
  else return -1;
#undef IJP
  return (int)hipGetLastError();
}

extern "C" int ncnet_ijsum(const float* Z, const float* bias, float* y, int V, int I, int J, int K, int L, int KS,
                           int relu, int sgn, hipStream_t stream) {
  long long nvox = (long long)V * I * J * K * L;
  dim3 grid((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256));
  if (KS == 5) hipLaunchKernelGGL((ijsum_kernel<5>), grid, dim3(256), 0, stream, Z, bias, y, nvox, I, J, K * L, relu, sgn);
  else if (KS == 3) hipLaunchKernelGGL((ijsum_kernel<3>), grid, dim3(256), 0, stream, Z, bias, y, nvox, I, J, K * L, relu, sgn);
  else return -1;
  return (int)hipGetLastError();
}
