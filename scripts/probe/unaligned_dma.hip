// Probe: does buffer_load_dwordx4 ... lds (and global_load_lds_dwordx4) accept a
// 2-byte-aligned source offset on gfx950?  Writes 64 lanes x 16 B from src+2*shift.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint16_t* src, uint16_t* out, int shift) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const uint64_t b = (uint64_t)src;
  typedef int i32x4v __attribute__((ext_vector_type(4)));
  i32x4v r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(b >> 32) & 0xffffu));
  r[2] = 1 << 20;
  r[3] = 0x00020000;
  uint32_t voff = threadIdx.x * 16 + shift * 2;
  uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)sm;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds) : "memory", "m0");
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  for (int e = threadIdx.x; e < 512; e += 64) out[e] = ((uint16_t*)sm)[e];
}
int main() {
  uint16_t *s, *o, h[600];
  hipMalloc(&s, 1 << 20); hipMalloc(&o, 2048);
  for (int i = 0; i < 600; ++i) h[i] = (uint16_t)i;
  hipMemcpy(s, h, 1200, hipMemcpyHostToDevice);
  int bad = 0;
  for (int shift = 0; shift < 4; ++shift) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 1024, 0, s, o, shift);
    uint16_t r[512];
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    int nb = 0;
    for (int e = 0; e < 512; ++e) nb += r[e] != (uint16_t)(e + shift);
    printf("shift %d: %d mismatches (first %d %d %d %d)\n", shift, nb, r[0], r[1], r[2], r[3]);
    bad += nb;
  }
  printf(bad ? "UNALIGNED DMA: NOT OK\n" : "UNALIGNED DMA: OK\n");
  return 0;
}
