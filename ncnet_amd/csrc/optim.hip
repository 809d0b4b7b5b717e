// Flat, guarded Adam for the trainable parameters (train.py:71).
//
// All trainable fp32 parameters, their gradients and the two Adam moments
// live in four flat device buffers (the parameters and gradients the model
// sees are views into them), so one step is three launches whatever the
// parameter count:
//
//   nonfinite_count  counts non-finite entries of the flat gradient (+ the
//                    loss-indicator slot that trails it) into one int;
//   adam_masked      the torch.optim.Adam update (L2 weight decay, bias
//                    correction from the device step counter) applied only
//                    when that count is 0 -- otherwise params, moments and
//                    step are left untouched and the gradient is zeroed;
//   adam_finalize    step += (count == 0), count = 0 (one lane).
//
// Nothing is read back to the host, so a skipped step costs no sync.  Under
// data parallelism the count runs AFTER the gradient all-reduce: a NaN on any
// rank reaches every rank's sum, so all ranks skip the same step.
#include "common.h"

namespace ncnet {

__global__ __launch_bounds__(256) void nonfinite_count_kernel(const float* __restrict__ g, long long n,
                                                              int* __restrict__ count) {
  int bad = 0;
  const long long n4 = n >> 2;
  const f32x4* g4 = (const f32x4*)g;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 x = g4[i];
#pragma unroll
    for (int r = 0; r < 4; ++r) bad += !__builtin_isfinite(x[r]);
  }
  for (long long i = (n4 << 2) + blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    bad += !__builtin_isfinite(g[i]);
  // wave reduce, then one atomic per wave that saw something
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(count, bad);
}

__global__ __launch_bounds__(256) void adam_masked_kernel(float* __restrict__ p, float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v, long long n,
                                                          const int* __restrict__ count,
                                                          const float* __restrict__ step, float lr, float b1,
                                                          float b2, float eps, float wd, float gscale) {
  const bool skip = *count != 0;
  // bias corrections in double, as torch computes them on the host
  const double t = (double)*step + 1.0;
  const float step_size = (float)((double)lr / (1.0 - pow((double)b1, t)));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, t));
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    if (skip) {
      g[i] = 0.f;
      continue;
    }
    float gi = g[i];
    if (gscale != 1.f) {   // data-parallel average folded in; keep the averaged gradient visible
      gi *= gscale;
      g[i] = gi;
    }
    const float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    // torch: exp_avg.lerp_(grad, 1 - beta1); exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    float mi = m[i] + (1.f - b1) * (gi - m[i]);
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi - step_size * (mi / denom);
  }
}

__global__ void adam_finalize_kernel(float* __restrict__ step, int* __restrict__ count,
                                     int* __restrict__ skipped) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (*count == 0) *step += 1.f;
    else *skipped += 1;
    *count = 0;
  }
}

}  // namespace ncnet

using namespace ncnet;

static int grid_for(long long n) {
  long long b = (n + 1023) / 1024;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

extern "C" int ncnet_nonfinite_count(const float* g, long long n, int* count, hipStream_t s) {
  hipLaunchKernelGGL(nonfinite_count_kernel, dim3(grid_for(n)), dim3(256), 0, s, g, n, count);
  return (int)hipGetLastError();
}

extern "C" int ncnet_adam_masked(float* p, float* g, float* m, float* v, long long n, const int* count,
                                 const float* step, float lr, float b1, float b2, float eps, float wd, float gscale,
                                 hipStream_t s) {
  hipLaunchKernelGGL(adam_masked_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, g, m, v, n, count, step, lr, b1, b2,
                     eps, wd, gscale);
  return (int)hipGetLastError();
}

extern "C" int ncnet_adam_finalize(float* step, int* count, int* skipped, hipStream_t s) {
  hipLaunchKernelGGL(adam_finalize_kernel, dim3(1), dim3(64), 0, s, step, count, skipped);
  return (int)hipGetLastError();
}
