// ij encoding of the 1-channel NC-Net layers (ijpack / ijsum).
//
// A Conv4d with one input (or one output) channel wastes 15/16 of an MFMA.
// Moving BOTH plane offsets (di, dj) into the channel axis turns it into a
// 16 -> 16 convolution over G "group planes" with in-plane (dk, dl) taps only:
// combo q = di*KS + dj, 16 combos per group, G = ceil(KS*KS/16) groups
// (KS=1: 1 group, 1/16 channels used; KS=3: 1, 9/16; KS=5: 2, 25/32; KS=7: 4, 49/64):
//   S[g][v,i,j,k,l,c] = X[v, i+sgn*(di-P), j+sgn*(dj-P), k, l],  q = 16g + c
//   y[v,i,j,k,l]      = act(b + sum_q Z[q][v, i+sgn*(di-P), j+sgn*(dj-P), k, l])
//   Cin = 1 :  Y = conv16_groups(ijpack(X, +1), W1 re-indexed by combo)
//   Cout = 1:  Z = conv16_groups(X2, Wz) as channel-planar fp32 partials, y = ijsum(Z, +1)
// and the adjoints: ijpack(g, -1) is the adjoint of ijsum(+1), ijsum(-1) of
// ijpack(+1), so forward, data gradient and weight gradient of those layers
// all run on the conv16 / wgrad16 MFMA kernels (lib/conv4d.py:11-51 semantics).
// The exact weight maps are verified on CPU (tests/test_kernel_emulation.py).
#include "common.h"
#include <hip/hip_fp8.h>
#include <stdlib.h>

namespace ncnet {

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
  if (!NCNET_OK(e < nvox)) return;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float vals[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int q = 16 * g + c;
      float v = 0.f;
      if (q < NQ) {
        const int ii = i + sgn * (q / KS - P), jj = j + sgn * (q % KS - P);
        const long long src = (plane + (long long)(ii - i) * J + (jj - j)) * KL + kl;
        if (ii >= 0 && ii < I && jj >= 0 && jj < J && NCNET_OK(src >= 0 && src < nvox)) v = (float)X[src];
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
    const long long src = e + ((long long)(ii - i) * J + (jj - j)) * KL;
    if (ii >= 0 && ii < I && jj >= 0 && jj < J && NCNET_OK(src >= 0 && src < nvox)) s += Z[(long long)q * nvox + src];
  }
  y[e] = relu ? fmaxf(s, 0.f) : s;
}

}  // namespace ncnet

using namespace ncnet;

#define KS_DISPATCH(M, ...) \
  do { if (KS == 5) M(5, __VA_ARGS__); else if (KS == 3) M(3, __VA_ARGS__); \
       else if (KS == 7) M(7, __VA_ARGS__); else if (KS == 1) M(1, __VA_ARGS__); else return -1; } while (0)

// S bf16 (non-temporal stores: the >= 1.6 GB output never stays in L2) or OCP fp8 e4m3 (inference).
extern "C" int ncnet_ijpack(const void* X, int x_is_bf16, void* S, int V, int I, int J, int K, int L, int KS, int sgn,
                            int s_fp8, hipStream_t stream) {
  long long nvox = (long long)V * I * J * K * L;
  dim3 grid((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256));
#define IJP(KSV, T) do { if (s_fp8) hipLaunchKernelGGL((ijpack_kernel<T, KSV, true>), grid, dim3(256), 0, stream, (const T*)X, S, nvox, I, J, K * L, sgn); \
                         else hipLaunchKernelGGL((ijpack_kernel<T, KSV, false, true>), grid, dim3(256), 0, stream, (const T*)X, S, nvox, I, J, K * L, sgn); } while (0)
  if (x_is_bf16) KS_DISPATCH(IJP, bf16); else KS_DISPATCH(IJP, float);
#undef IJP
  return (int)hipGetLastError();
}

extern "C" int ncnet_ijsum(const float* Z, const float* bias, float* y, int V, int I, int J, int K, int L, int KS,
                           int relu, int sgn, hipStream_t stream) {
  long long nvox = (long long)V * I * J * K * L;
  dim3 grid((unsigned)(V * I * J), (unsigned)((K * L + 255) / 256));
#define IJS(KSV, _) hipLaunchKernelGGL((ijsum_kernel<KSV>), grid, dim3(256), 0, stream, Z, bias, y, nvox, I, J, K * L, relu, sgn)
  KS_DISPATCH(IJS, 0);
#undef IJS
  return (int)hipGetLastError();
}
