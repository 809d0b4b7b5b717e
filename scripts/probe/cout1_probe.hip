// Timing decomposition of the tap-row Cout=1 kernel (csrc/cout1.hip) at the
// training shape, standalone (no torch):  hipcc -O3 --offload-arch=gfx950
// -I ncnet_amd/csrc scripts/probe/cout1_probe.hip -o /tmp/cout1_probe
// Prints ms per launch for DBG 0 (real), 1 (no epilogue), 2 (no DMA waits),
// 4 (no MFMAs), 5 (neither epilogue nor MFMAs).
#include "../../ncnet_amd/csrc/cout1.hip"
#include <cstdio>
#include <vector>

template <int DBG>
static float run(const bf16* x, const u32x4* w, float* y, int V, int reps) {
  using C = CT1<5, 25, 25, C1_RI, C1_RJ>;
  const int nitems = V * 25 * ((25 + C1_RJ - 1) / C1_RJ) / C1_RI;
  const int grid = nitems < 256 ? nitems : 256;
  auto go = [&] {
    hipLaunchKernelGGL((cout1_taps_fwd_kernel<5, 25, 25, C1_RI, C1_RJ, DBG>), dim3(grid), dim3(256), (size_t)C::LDS, 0,
                       x, w, nullptr, y, V, 25, 25, 1);
  };
  go();
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) go();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int V = 64;
  const size_t nx = (size_t)V * 25 * 25 * 625 * 16;
  std::vector<uint16_t> hx(nx), hw(25 * 64 * 8);
  uint32_t st = 12345;
  auto rnd = [&] { st = st * 1664525u + 1013904223u; return (st >> 9) & 0x7f; };
  for (auto& e : hx) e = (uint16_t)(0x3c00 | rnd());   // bf16 in [0.0078, 0.0156)
  for (auto& e : hw) e = (uint16_t)(0x3c00 | rnd());
  bf16* x; u32x4* w; float* y;
  hipMalloc(&x, nx * 2); hipMalloc(&w, hw.size() * 2); hipMalloc(&y, (size_t)V * 390625 * 4);
  hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  printf("real            %.3f ms\n", run<0>(x, w, y, V, 10));
  printf("no epilogue     %.3f ms\n", run<1>(x, w, y, V, 10));
  printf("no DMA waits    %.3f ms\n", run<2>(x, w, y, V, 10));
  printf("no MFMAs        %.3f ms\n", run<4>(x, w, y, V, 10));
  printf("no epi, no MFMA %.3f ms\n", run<5>(x, w, y, V, 10));
  printf("no epi, no wait %.3f ms\n", run<3>(x, w, y, V, 10));
  return 0;
}
