// Backbone epilogues for the frozen-trunk execution plan (models/backbones.py
// FrozenResNetPlan).  MIOpen's bf16 NHWC convolutions add a bias in a separate
// pass and PyTorch then runs ReLU / residual add as further passes (~7 full
// activation round trips per bottleneck).  The plan routes 1x1 convolutions
// to hipBLASLt GEMMs (bias + ReLU in the GEMM epilogue, residual as the C
// operand) and finishes everything else with this single in-place pass:
//
//   Y[r, c] = act(Y[r, c] + b[c])          (bf16 rows of C channels, fp32 bias)
#include "common.h"

namespace ncnet {

// 8 channels (16 B) per thread; C % 8 == 0.  F16: Y is IEEE half.
template <bool RELU, bool F16>
__global__ __launch_bounds__(256) void bias_act_kernel(uint16_t* __restrict__ Y, const float* __restrict__ b,
                                                       long long n8, int C8) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n8) return;
  const int c0 = (int)(e % C8) * 8;
  u32x4 v = *(const u32x4*)(Y + e * 8);
  const f32x4 b0 = *(const f32x4*)(b + c0), b1 = *(const f32x4*)(b + c0 + 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 2 * q + h;
      float x = s162f<F16>((uint16_t)(v[q] >> (16 * h))) + (k < 4 ? b0[k] : b1[k - 4]);
      if (RELU) x = fmaxf(x, 0.f);
      w |= (uint32_t)f2s16<F16>(x) << (16 * h);
    }
    v[q] = w;
  }
  *(u32x4*)(Y + e * 8) = v;
}

// Stem finish: Y = act(maxpool_{k,s,p}(X) + b) in ONE pass over the stem conv
// output (NHWC, C % 8 == 0).  Equal to maxpool(act(X + b)) bit for bit:
// x -> round(act(x + b)) is monotonic per channel, so it commutes with max,
// and padded taps are skipped (MaxPool2d pads with -inf).  Replaces an
// in-place bias_act pass + PyTorch's max_pool2d (three full-size activation
// passes -> one read of the conv output; 2.9 -> ~0.4 ms per 11 images at 3200 px).
template <bool RELU, bool F16>
__global__ __launch_bounds__(256) void maxpool_bias_act_kernel(const uint16_t* __restrict__ X, uint16_t* __restrict__ Y,
                                                               const float* __restrict__ b, int N, int H, int W, int C8,
                                                               int Ho, int Wo, int k, int st, int pad) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)N * Ho * Wo * C8;
  if (e >= total) return;
  const int c8 = (int)(e % C8);
  long long r = e / C8;
  const int wo = (int)(r % Wo); r /= Wo;
  const int ho = (int)(r % Ho);
  const int n = (int)(r / Ho);
  float m[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) m[q] = -INFINITY;
  const int h0 = ho * st - pad, w0 = wo * st - pad;
  for (int dh = 0; dh < k; ++dh) {
    const int h = h0 + dh;
    if (h < 0 || h >= H) continue;
    for (int dw = 0; dw < k; ++dw) {
      const int w = w0 + dw;
      if (w < 0 || w >= W) continue;
      const u32x4 v = *(const u32x4*)(X + ((((size_t)n * H + h) * W + w) * C8 + c8) * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        m[2 * q] = fmaxf(m[2 * q], s162f<F16>((uint16_t)(v[q] & 0xffffu)));
        m[2 * q + 1] = fmaxf(m[2 * q + 1], s162f<F16>((uint16_t)(v[q] >> 16)));
      }
    }
  }
  const f32x4 b0 = *(const f32x4*)(b + c8 * 8), b1 = *(const f32x4*)(b + c8 * 8 + 4);
  u32x4 out;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t wv = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kk = 2 * q + h;
      float x = m[kk] + (kk < 4 ? b0[kk] : b1[kk - 4]);
      if (RELU) x = fmaxf(x, 0.f);
      wv |= (uint32_t)f2s16<F16>(x) << (16 * h);
    }
    out[q] = wv;
  }
  *(u32x4*)(Y + e * 8) = out;
}

// Sanitizer-tier self test: out[0] = 1 in release; in the debug build the
// check fails on purpose (n >= 0), prints its NCNET_CHECK line and out[0] = 0.
__global__ void debug_selftest_kernel(int* out, int n) {
  if (threadIdx.x == 0) out[0] = NCNET_OK(n < 0) ? 1 : 0;
}

}  // namespace ncnet

using namespace ncnet;

extern "C" int ncnet_debug_selftest(int* out, hipStream_t stream) {
  hipLaunchKernelGGL(debug_selftest_kernel, dim3(1), dim3(64), 0, stream, out, 1);
  return (int)hipGetLastError();
}

extern "C" int ncnet_bias_act(void* Y, const float* b, long long rows, int C, int relu, int f16, hipStream_t stream) {
  if (C % 8) return -1;
  const long long n8 = rows * (C / 8);
  if (n8 == 0) return 0;
  dim3 grid((unsigned)((n8 + 255) / 256)), block(256);
  uint16_t* y = (uint16_t*)Y;
  if (f16) {
    if (relu) hipLaunchKernelGGL((bias_act_kernel<true, true>), grid, block, 0, stream, y, b, n8, C / 8);
    else hipLaunchKernelGGL((bias_act_kernel<false, true>), grid, block, 0, stream, y, b, n8, C / 8);
  } else {
    if (relu) hipLaunchKernelGGL((bias_act_kernel<true, false>), grid, block, 0, stream, y, b, n8, C / 8);
    else hipLaunchKernelGGL((bias_act_kernel<false, false>), grid, block, 0, stream, y, b, n8, C / 8);
  }
  return (int)hipGetLastError();
}

// X [N, H, W, C] (NHWC, 16-bit), Y [N, Ho, Wo, C]; b fp32 [C]; C % 8 == 0.
extern "C" int ncnet_maxpool_bias_act(const void* X, void* Y, const float* b, int N, int H, int W, int C, int Ho,
                                      int Wo, int k, int stride, int pad, int relu, int f16, hipStream_t stream) {
  if (C % 8 || k < 1 || stride < 1 || pad < 0 || 2 * pad > k) return -1;
  const long long total = (long long)N * Ho * Wo * (C / 8);
  if (total == 0) return 0;
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  const uint16_t* x = (const uint16_t*)X; uint16_t* y = (uint16_t*)Y;
#define MPB(R, H) hipLaunchKernelGGL((maxpool_bias_act_kernel<R, H>), grid, block, 0, stream, x, y, b, N, H_, W, C / 8, Ho, \
                                     Wo, k, stride, pad)
  const int H_ = H;
  if (f16) { if (relu) MPB(true, true); else MPB(false, true); }
  else { if (relu) MPB(true, false); else MPB(false, false); }
#undef MPB
  return (int)hipGetLastError();
}
