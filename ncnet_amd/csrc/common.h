// Shared definitions for the gfx950 (CDNA4 / MI355X) NC-Net kernels.
//
// Conventions used by every kernel in this directory:
//  * wave64; blocks are multiples of 64 lanes.
//  * bf16 operands are moved as 16-byte vectors (8 x bf16) everywhere the
//    layout allows it (global -> registers -> LDS -> MFMA fragments).
//  * MFMA shape is v_mfma_f32_16x16x32_bf16: lane l holds A[row l&15][k 8(l>>4)+j]
//    and B[k 8(l>>4)+j][col l&15], j = 0..7; D[row 4(l>>4)+r][col l&15], r = 0..3.
//  * Volumes are channels-last: [V, I, J, K, L, C] (C = 16 for the hidden
//    Conv4d activations, C = 1 for correlation volumes, which are then just
//    the matrix [V, I*J, K*L]).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// OCP fp8 e4m3 x fp8 e4m3 -> f32, 16x16x128, through the block-scaled MX form
// (2x the bf16 MFMA rate) with unit E8M0 scales (127 = 2^0) on both operands.
// Lane l holds A[row l&15][k = 32(l>>4) .. 32(l>>4)+31] (32 bytes, k in byte
// order) and B[k same][col l&15]; C/D as the bf16 16x16 form.
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma_fp8_k128(const i32x8& a, const i32x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// ds_read_b64_tr_b16: 16-lane group reads a [4 rows x 16 cols] bf16 block;
// lane 4q+p supplies the address of row q, columns 4p..4p+3 (8-byte aligned);
// lane i of the group receives column i of the 4 rows.
__device__ __forceinline__ bf16x4 lds_read_tr16(const char* lds_base, uint32_t byte_off) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds_base + byte_off));
  return __builtin_bit_cast(bf16x4, v);
}

__device__ __forceinline__ bf16x8 cat8(const bf16x4& lo, const bf16x4& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// The same fragments as 32-bit lanes: register copies / concatenations of
// bf16 vectors can be legalised element-wise (16-bit shifts + v_perm per
// element); moving them as u32 vectors keeps them plain VGPR moves.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 lds_read_tr16u(const char* lds_base, uint32_t byte_off) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds_base + byte_off));
  return __builtin_bit_cast(u32x2, v);
}
__device__ __forceinline__ u32x4 cat4u(const u32x2& lo, const u32x2& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
}
__device__ __forceinline__ f32x4 mfma16u(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                 0);
}

// IEEE half (f16) operands: v_mfma_f32_16x16x32_f16 has the bf16 form's
// fragment layout and rate with 3 more mantissa bits (the reference's
// half-precision InLoc path, eval_inloc.py:50).  Kernels templated on F16 move
// 16-bit operands as raw bits and pick the MFMA / the output rounding here.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma16h(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}
template <bool F16>
__device__ __forceinline__ f32x4 mfma16t(const u32x4& a, const u32x4& b, const f32x4& c) {
  if constexpr (F16) return mfma16h(a, b, c);
  else return mfma16u(a, b, c);
}
// 16-bit storage bits of x (round to nearest even): bf16, or IEEE half
template <bool F16>
__device__ __forceinline__ uint16_t f2s16(float x) {
  if constexpr (F16) return __builtin_bit_cast(uint16_t, (_Float16)x);
  else return __builtin_bit_cast(uint16_t, (__bf16)x);
}
template <bool F16>
__device__ __forceinline__ float s162f(uint16_t x) {
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, x);
  else return (float)__builtin_bit_cast(__bf16, x);
}

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4) issued from inline asm.
// The compiler's waitcnt pass cannot prove that an LDS-DMA misses a later
// ds_read_b64_tr_b16 (intrinsic reads carry no alias info), so with the builtin
// it drains EVERY in-flight DMA (s_waitcnt vmcnt(0)) before the first
// transposed read -- the next step's prefetch is serialised with the compute.
// Issued from asm the DMA is invisible to that pass; the kernel then owns the
// wait: `s_waitcnt vmcnt(..)` + s_barrier (asm_barrier_vm below) before reading
// what landed.  (Extra in-flight asm ops only make the compiler's own vmcnt
// waits stricter, never weaker: completion is in issue order.)  M0 is set here;
// kernels using this issue no other M0-based instruction.
__device__ __forceinline__ void dma16_lds(const void* gsrc, const void* lds_dst) {
  const uint32_t l = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst;
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(l) : "memory", "m0");
}
// Workgroup barrier that first waits for ALL of this wave's vector-memory ops
// (incl. asm LDS-DMAs) and LDS ops.
__device__ __forceinline__ void asm_barrier_vm0() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ bf16x8 lds_read16(const char* lds_base, uint32_t byte_off) {
  return *(const bf16x8*)(lds_base + byte_off);
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap of a linear block id: consecutive logical ids land
// on the same XCD (blocks are dealt round-robin over the 8 XCDs), so
// neighbouring output tiles that share input planes share an L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblocks) {
  const uint32_t nx = 8;
  if (nblocks < nx) return bid;
  uint32_t q = nblocks / nx, r = nblocks % nx;
  uint32_t x = bid % nx, k = bid / nx;
  uint32_t start = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return start + k;
}

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// CUs of the current device (persistent grids, tile picking), cached per device
static inline int device_num_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// Debug-build bounds checks (python -m ncnet_amd.build --debug -> _C_debug.so).
// NCNET_OK(cond) is `cond` in the debug build -- printing the failed condition
// with file:line and the block / thread, so the guarded access is skipped
// instead of faulting -- and `true` (compiled away) in release.  Used on every
// global-memory address a kernel forms from runtime geometry (LDS-DMA sources
// and destinations, gathers, stores); tests/conftest.py fails any GPU test
// whose output contains "NCNET_CHECK" when run with NCNET_EXT=debug.
#ifdef NCNET_DEBUG
__device__ __noinline__ bool ncnet_check_fail(const char* cond, const char* file, int line) {
  printf("NCNET_CHECK failed %s:%d: %s (block %d,%d,%d thread %d)\n", file, line, cond, (int)blockIdx.x,
         (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x);
  return false;
}
#define NCNET_OK(cond) ((cond) ? true : ncnet_check_fail(#cond, __FILE__, __LINE__))
#else
#define NCNET_OK(cond) true
#endif

// Launcher tuning switches -- A/B tests and scripts/kbench.py only.  ONE
// process-wide table with the defaults below; the Python side pushes
// ncnet_amd.config.RUNTIME's values (the NCNET_* environment, read once there)
// through the set_tuning binding when the extension loads (ops/_ext.py
// apply_tuning): no launcher reads the environment.
struct NcnetTuning {
  int nt_store;        // non-temporal Conv4d epilogue stores (1)
  int gp_tpw;          // output j-tiles per group-plane workgroup (5)
  int conv_v3;         // conv16v3 instead of conv16v4 at the compile-time planes (0)
  int wgrad_v3;        // wgrad16v3 instead of wgrad16v4 at the compile-time planes (0)
  int wgrad_flags;     // wgrad16v3 ablation flags (0)
  int conv2d_variant;  // 0 auto, 1 register-staged, 2 DMA ring
  int corr_v2;         // -1 auto, 0 / 1 force the correlation GEMM variant
  int corr_ns;         // 3 or 4 ring stages of corr_gemm_v2
  int conv2d_v3;       // chip-round v3 tiles where the auto rule picks them (1)
  int c1x_pd;          // conv1x16 transposed-read lookahead in tiles, 1, 2 or 3 (2)
  int conv2d_256;      // 256 x 256 trunk conv tiles for Cout = 256 where the grid is big enough (1)
  int s2d_rt;          // stats2d: 64-row sub-tiles per block for volumes of >= 1024 rows, 1, 2 or 4 (2)
};
__host__ inline NcnetTuning& tuning() {
  static NcnetTuning t = {1, 5, 0, 0, 0, 0, -1, 3, 1, 2, 1, 2};
  return t;
}
__host__ inline int* tuning_slot(const char* name) {
  NcnetTuning& t = tuning();
  if (!strcmp(name, "nt_store")) return &t.nt_store;
  if (!strcmp(name, "gp_tpw")) return &t.gp_tpw;
  if (!strcmp(name, "conv_v3")) return &t.conv_v3;
  if (!strcmp(name, "wgrad_v3")) return &t.wgrad_v3;
  if (!strcmp(name, "wgrad_flags")) return &t.wgrad_flags;
  if (!strcmp(name, "conv2d_variant")) return &t.conv2d_variant;
  if (!strcmp(name, "corr_v2")) return &t.corr_v2;
  if (!strcmp(name, "corr_ns")) return &t.corr_ns;
  if (!strcmp(name, "conv2d_v3")) return &t.conv2d_v3;
  if (!strcmp(name, "c1x_pd")) return &t.c1x_pd;
  if (!strcmp(name, "conv2d_256")) return &t.conv2d_256;
  if (!strcmp(name, "s2d_rt")) return &t.s2d_rt;
  return nullptr;
}
