// Training input preparation on the GPU: one launch turns a batch of decoded
// uint8 images of arbitrary sizes into the normalised float NCHW batch.
//
// Reference semantics: ImagePairDataset resizes every image to the output
// size with an identity AffineTnf under torch-0.3 grid_sample, i.e. bilinear
// sampling with align_corners=True (lib/im_pair_dataset.py:40,89,
// lib/transformation.py:44,63), then NormalizeImageDict divides by 255 and
// applies the ImageNet mean / std (lib/normalization.py:19-26).
//
// Layout: the DataLoader workers pack the decoded HWC uint8 pixels of all
// images of a batch into ONE byte buffer (one pinned host->device copy) with a
// table meta[b] = (byte offset, H, W).  One thread per output pixel reads its
// four HWC neighbours (3 contiguous bytes each) and writes the 3 normalised
// channels of out[b, :, y, x] (fp32, NCHW, what the trunk consumes).
#include "common.h"

namespace ncnet {

struct NormArgs { float m0, m1, m2, is0, is1, is2; };

__global__ __launch_bounds__(256) void resize_norm_u8_kernel(const uint8_t* __restrict__ src,
                                                             const long long* __restrict__ meta,
                                                             float* __restrict__ out, int oh, int ow,
                                                             NormArgs n) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= oh * ow) return;
  const long long off = meta[3 * b];
  const int H = (int)meta[3 * b + 1], W = (int)meta[3 * b + 2];
  const int oy = p / ow, ox = p - oy * ow;
  // align_corners=True: source coordinate = ((in - 1) / (out - 1)) * dst, in
  // fp32 and in this order, as ATen's upsample_bilinear2d
  const float ry = oh > 1 ? (float)(H - 1) / (float)(oh - 1) : 0.f;
  const float rx = ow > 1 ? (float)(W - 1) / (float)(ow - 1) : 0.f;
  const float sy = ry * (float)oy, sx = rx * (float)ox;
  const int y0 = min((int)sy, H - 1), x0 = min((int)sx, W - 1);
  const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
  const float fy = sy - (float)y0, fx = sx - (float)x0;
  if (!NCNET_OK(off >= 0 && H > 0 && W > 0 && (b == 0 || off >= meta[3 * (b - 1)]))) return;
  const uint8_t* im = src + off;
  const uint8_t* a = im + ((size_t)y0 * W + x0) * 3;
  const uint8_t* bb = im + ((size_t)y0 * W + x1) * 3;
  const uint8_t* c = im + ((size_t)y1 * W + x0) * 3;
  const uint8_t* d = im + ((size_t)y1 * W + x1) * 3;
  const float w00 = (1.f - fy) * (1.f - fx), w01 = (1.f - fy) * fx, w10 = fy * (1.f - fx), w11 = fy * fx;
  const float mean[3] = {n.m0, n.m1, n.m2}, istd[3] = {n.is0, n.is1, n.is2};
  float* o = out + (size_t)b * 3 * oh * ow + p;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float v = w00 * a[ch] + w01 * bb[ch] + w10 * c[ch] + w11 * d[ch];
    o[(size_t)ch * oh * ow] = (v * (1.f / 255.f) - mean[ch]) * istd[ch];
  }
}

}  // namespace ncnet

using namespace ncnet;

extern "C" int ncnet_resize_norm_u8(const void* src, const long long* meta, float* out, int B, int oh, int ow,
                                    const float* mean, const float* stdv, hipStream_t stream) {
  NormArgs n{mean[0], mean[1], mean[2], 1.f / stdv[0], 1.f / stdv[1], 1.f / stdv[2]};
  dim3 grid((unsigned)cdiv(oh * ow, 256), (unsigned)B);
  hipLaunchKernelGGL(resize_norm_u8_kernel, grid, dim3(256), 0, stream, (const uint8_t*)src, meta, out, oh, ow, n);
  return (int)hipGetLastError();
}
