// Fused NeighConsensus for the InLoc network (ncons_kernel_sizes 3,3 /
// ncons_channels 16,1; reference eval_inloc.py:50-57 with lib/model.py:122-153):
//
//   h = relu(conv4d_3(x0; W1) + b1)        1 -> 16 channels
//   y = relu(conv4d_3(h;  W2) + b2)        16 -> 1 channel
//
// in ONE kernel, per volume, with the 16-channel hidden activation never
// leaving LDS.  The layer-by-layer path writes h (1.8-3.6 GB at 3200 px), the
// ij-packed layer-1 input (1.8 GB) and 9 channel-planar fp32 partials of the
// last layer (4 GB) to HBM and reads them back; here HBM sees x0 once and y
// once.
//
// Work decomposition: a workgroup owns output rows [i0, i1), output planes
// j0 .. j0+R-1 and a (k, l) tile TK x TL, and STREAMS the volume along i:
//   for each hidden row ih (i0-1 .. i1), for each hidden plane j'' (j0-1 .. j0+R):
//     A  S tile: the ij-packed layer-1 input of plane (ih, j'') over the
//        (k, l) tile + 2-voxel halo -- channel c = (di1, dj1) holds
//        x0(ih+di1-1, j''+dj1-1, k, l) -- gathered from global (L1/L2-hot)
//        by a register prefetch issued one plane ahead, written as bf16x16.
//     B  layer 1: h(ih, j'') over the tile + 1-voxel halo = a 16 -> 16 plane
//        conv over the (dk, dl) taps of S (v_mfma_f32_16x16x32_bf16, A =
//        weights of 2 taps x 16 combos, B = S at the tap shift), + b1, ReLU,
//        zero outside the volume (layer 2's "same" padding), bf16 into LDS.
//     C  layer 2: z_q(ih, j'') for the 9 plane combos q = (di2, dj2) over the
//        tile (MFMA rows = combos, row 4 dj2 + di2, so a lane's 4 rows share
//        dj2 and the output plane; K = taps x 16 channels of h), accumulated
//        into an LDS ring of 3 output rows x R planes at
//        (ih - di2 + 1, j'' - dj2 + 1).
//   output row ih-1 is complete after hidden row ih: + b2, ReLU, store fp32.
// Every ring address (row slot, plane, voxel) is only ever touched by the
// lane that owns that voxel of the tile (static voxel -> wave/lane map, and
// distinct combos of one plane land on distinct ring addresses), so the ring
// needs no atomics and no barriers; two barriers per hidden plane order the
// S and h buffers.
#include "common.h"
#include <stdlib.h>

namespace ncnet {

struct NCFGeom {
  int V, I, J, K, L;
  int TK, TL, R, IR;        // tile, planes per workgroup, output rows per workgroup
  int nkt, nlt, njb, nib;
  int SRS, HRS;             // LDS row strides (voxels) of the S and h tiles
};

constexpr int NCF_NW = 8;          // waves per workgroup

// Output-ring plane stride (words): nvox rounded up to 16 mod 32.  The ring
// read-add-writes of one wave touch two planes at once (lane groups fq = 0, 1
// hold combo columns dj2 = 0, 1 of the same voxels): with the planes 16 banks
// apart the two 16-lane halves of a ds_read_b32 / ds_write_b32 never share a
// bank (a 300-voxel plane put 4 of them on the same banks).
__host__ __device__ constexpr int ncf_ring_stride(int nvox) { return nvox + ((16 - nvox % 32) + 32) % 32; }
constexpr int NCF_MAXT1 = 4;       // layer-1 tiles per wave: (TK+2)(TL+2) <= 512 voxels
constexpr int NCF_MAXT2 = 3;       // layer-2 tiles per wave: TK*TL <= 384 voxels

// F16: IEEE-half x0, weights and hidden activation (half_precision=True, as
// eval_inloc.py runs the reference: lib/model.py:265-267), f16 MFMA.
// CTK, CTL, CR: compile-time tile (k, l) and planes per workgroup for the
// InLoc shapes (0 = the runtime value of g): the tile counts, LDS row strides,
// tap offsets and ring indexing then fold into immediates -- the runtime
// geometry kept ~50 SGPRs live (spilled to VGPR lanes) and cost ~10 SALU per
// MFMA (profiles/r2_inloc/pmc_corr_ncfused_before.md).
template <bool F16, int CTK = 0, int CTL = 0, int CR = 0, int NW = 8>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 2 : 1) void nc_fused_k3_kernel(const bf16* __restrict__ X, const u32x4* __restrict__ W1p,
                                                             const float* __restrict__ b1,
                                                             const u32x4* __restrict__ W2p,
                                                             const float* __restrict__ b2, float* __restrict__ Y,
                                                             NCFGeom g) {
  constexpr int NQ = 5;            // tap pairs of the 3x3 (dk, dl) taps
  // NW = 8: two 512-thread workgroups per CU (<= 80 KB LDS each); NW = 16: one
  // 1024-thread workgroup per CU with up to 160 KB (a deeper output ring: more
  // planes per workgroup, less j halo) and half the tiles per wave per phase
  constexpr int MT1 = 32 / NW;                 // layer-1 tiles per wave: (TK+2)(TL+2) <= 512
  constexpr int MT2 = NW == 8 ? 3 : 2;         // layer-2 tiles per wave: TK*TL <= 16 NW MT2
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int TK = CTK ? CTK : g.TK, TL = CTL ? CTL : g.TL;
  const int GR = CR ? CR : g.R;                       // planes per workgroup (ring depth)
  const int SRS = CTL ? CTL + 10 : g.SRS, HRS = CTL ? CTL + 8 : g.HRS;
  const int SR = TK + 4, SW = TL + 4;        // S tile (layer-1 input): tile + 2 halo
  const int HR = TK + 2, HW = TL + 2;        // h tile (layer-2 input): tile + 1 halo
  char* S = smem;
  char* H = S + SR * SRS * 32;
  float* ring = (float*)(H + HR * HRS * 32);
  // ring + 64 trash words (one per lane), rounded to 16 B; then the weight fragments [2 layers][5 tap pairs][64 lanes]
  const int nvox = TK * TL;
  const int rps = ncf_ring_stride(nvox);
  u32x4* wl = (u32x4*)(ring + ((3 * GR * rps + 64 + 3) & ~3));

  // wave index made wave-uniform (an SGPR): the per-wave tile-count checks are
  // then scalar branches, not exec-mask save / restore sequences
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NW);   // static tile counts fold the per-wave checks
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int lt = bid % g.nlt; bid /= g.nlt;
  const int kt = bid % g.nkt; bid /= g.nkt;
  const int jb = bid % g.njb; bid /= g.njb;
  const int ib = bid % g.nib;
  const int v = bid / g.nib;
  const int k0 = kt * TK, l0 = lt * TL, j0 = jb * GR, i0 = ib * g.IR;
  const int i1 = min(g.I, i0 + g.IR);
  const int R = min(GR, g.J - j0);
  const size_t KL = (size_t)g.K * g.L;
  const int KLi = g.K * g.L;
  // this volume's x0 through a buffer resource: a lane whose S voxel lies
  // outside the (k, l) volume reads with an out-of-range offset and gets 0,
  // the plane offset is a scalar (one buffer_load_ushort per combo, no
  // per-lane address arithmetic); one volume < 2^31 bytes (host-checked)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X + (size_t)v * g.I * g.J * KL), (short)0, (int)((size_t)g.I * g.J * KL * 2), 0x00020000);

  // ---- static maps --------------------------------------------------------
  // the S voxel owned by this thread (phase A): (TK+4)(TL+4) <= 512
  int s_lds, s_goff;
  bool s_in;
  {
    const int e = threadIdx.x;
    const int r = e / SW, c = e - r * SW;
    const int kg = k0 - 2 + r, lg = l0 - 2 + c;
    // threads past the S tile write to column SW of row 0, a padding voxel no
    // layer-1 read touches (taps reach column TL + 3 < SW <= SRS - 1): the
    // S write is branch-free
    s_lds = (e < SR * SW) ? (r * SRS + c) * 32 : SW * 32;
    s_in = e < SR * SW && kg >= 0 && kg < g.K && lg >= 0 && lg < g.L;
    s_goff = s_in ? (kg * g.L + lg) * 2 : 0x7ffffff0;   // byte offset in the plane / out of range
  }
  // layer-1 tiles: h ext voxels e = tile*16 + (lane & 15) over HR x HW
  const int nt1 = (HR * HW + 15) >> 4;
  uint32_t b1off[MT1], h_wr[MT1];
  bool h_in[MT1];
  // tap-pair read bases: lane half hh = lane >> 5 reads tap 2q + hh, which is
  // the voxel after tap 2q (pairs 0, 2, 3), one row wrap after it (pair 1:
  // taps (0,2) -> (1,0)) or the same voxel (pair 4: the padding tap); with the
  // base per kind the tap offset of 2q is a compile-time immediate
  const uint32_t hh = (uint32_t)(lane >> 5);
#pragma unroll
  for (int t = 0; t < MT1; ++t) {
    int e = (wave + NW * t) * 16 + (lane & 15);
    const bool ok = e < HR * HW;
    if (!ok) e = 0;
    const int r = e / HW, c = e - r * HW;
    b1off[t] = (uint32_t)((r * SRS + c) * 32 + ((lane >> 4) & 1) * 16);
    // lanes past the h region write to column HW of row 0 (padding no layer-2
    // read touches: taps reach column TL + 1 < HW <= HRS - 1): branch-free
    h_wr[t] = (uint32_t)(((ok ? r * HRS + c : HW)) * 32 + 8 * (lane >> 4));
    const int kg = k0 - 1 + r, lg = l0 - 1 + c;
    h_in[t] = ok && kg >= 0 && kg < g.K && lg >= 0 && lg < g.L;
  }
  uint32_t a1c[MT1], a1w[MT1];
#pragma unroll
  for (int t = 0; t < MT1; ++t) { a1c[t] = b1off[t] + hh * 32u; a1w[t] = b1off[t] + hh * (uint32_t)(SRS - 2) * 32u; }
  // layer-2 tiles: output voxels vi = tile*16 + (lane & 15) over TK x TL
  const int nt2 = (nvox + 15) >> 4;
  uint32_t b2off[MT2];
  int vo[MT2];
#pragma unroll
  for (int t = 0; t < MT2; ++t) {
    int vi = (wave + NW * t) * 16 + (lane & 15);
    vo[t] = vi < nvox ? vi : -1;
    if (vi >= nvox) vi = 0;
    const int kk = vi / TL, ll = vi - kk * TL;
    b2off[t] = (uint32_t)((kk * HRS + ll) * 32 + ((lane >> 4) & 1) * 16);
  }
  uint32_t a2c[MT2], a2w[MT2];
#pragma unroll
  for (int t = 0; t < MT2; ++t) { a2c[t] = b2off[t] + hh * 32u; a2w[t] = b2off[t] + hh * (uint32_t)(HRS - 2) * 32u; }
  for (int o = threadIdx.x; o < NQ * 64; o += NW * 64) { wl[o] = W1p[o]; wl[NQ * 64 + o] = W2p[o]; }
  const int co0 = 4 * (lane >> 4);
  const int dj2 = lane >> 4;                 // layer-2 combo column of this lane's MFMA rows
  float bias1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias1[r] = b1[co0 + r];
  const float bias2 = b2[0];

  // zero the output ring (3 row slots x R planes x TK*TL)
  for (int o = threadIdx.x; o < 3 * GR * rps; o += NW * 64) ring[o] = 0.f;

  const int ih_lo = max(0, i0 - 1), ih_hi = min(g.I, i1 + 1);   // hidden rows [lo, hi)
  const int jh_lo = max(0, j0 - 1), jh_hi = min(g.J, j0 + R + 1); // hidden planes [lo, hi)
  const int nplane = jh_hi - jh_lo;
  const int nsteps = (ih_hi - ih_lo) * nplane;

  // ---- the S gather: 9 plane-shifted x0 values per S voxel ----------------
  // Loads land in a register set that is only read (packed into the S tile)
  // two planes later: the set of plane t+2 is issued right after plane t's
  // set was written out, so no plane waits for its own gather.
  // plane byte offsets: one multiply per gather, the 9 combos differ by constants
  const int pstride = KLi * 2, rstride = g.J * KLi * 2;
  // every load is issued (branch-free: a combo outside the volume gets the
  // scalar offset nrec, past the buffer's range -> 0: on gfx950 the raw-buffer
  // range check covers voffset + soffset, pinned by
  // tests/test_gpu_kernels.py::test_nc_fused_k3_last_volume_borders, which
  // places large non-zero data right after a single volume); a conditional load let
  // the compiler merge the loads of both gather paths behind a VGPR phi of
  // the offset, i.e. a readfirstlane waterfall loop around each load
  const int nrec = (int)((size_t)g.I * g.J * KL * 2);
  auto gather = [&](int ih, int jh, uint32_t (&raw)[9]) {
    const int base = (ih * g.J + jh) * pstride;
    const bool iok[3] = {ih >= 1, true, ih + 1 < g.I}, jok[3] = {jh >= 1, true, jh + 1 < g.J};   // wave-uniform
#pragma unroll
    for (int c = 0; c < 9; ++c) {
      const int di = c / 3, dj = c % 3;
      const int so = (iok[di] && jok[dj]) ? base + (di - 1) * rstride + (dj - 1) * pstride : nrec;
      raw[c] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(xr, s_goff, __builtin_amdgcn_readfirstlane(so), 0);
    }
  };
  // sliding gather: plane (ih, jh) shares its combo columns dj = 0, 1 with
  // columns dj = 1, 2 of plane (ih, jh - 1), still in the other register set
  // (`prev`, that plane is one step younger): only the 3 values of the new
  // column jh + 1 are loaded (was 9 buffer_load_ushort per S voxel per plane)
  auto gather_slide = [&](int ih, int jh, uint32_t (&raw)[9], const uint32_t (&prev)[9]) {
    const int base = (ih * g.J + jh) * pstride;
    const bool iok[3] = {ih >= 1, true, ih + 1 < g.I};
    const bool jok = jh + 1 < g.J;
    // loads first, register moves last: the two gather paths then end in
    // different instructions and are not tail-merged into one phi'd load
#pragma unroll
    for (int di = 0; di < 3; ++di) {
      const int so = (iok[di] && jok) ? base + (di - 1) * rstride + pstride : nrec;
      raw[di * 3 + 2] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(xr, s_goff, __builtin_amdgcn_readfirstlane(so), 0);
    }
#pragma unroll
    for (int di = 0; di < 3; ++di) {
      raw[di * 3 + 0] = prev[di * 3 + 1];
      raw[di * 3 + 1] = prev[di * 3 + 2];
    }
  };
  // B fragment of tap pair q for tile u (S: layer 1, H: layer 2)
  auto bread = [&](const char* buf, uint32_t c, uint32_t w, uint32_t z, int RS, int q) -> u32x4 {
    const uint32_t t0 = q == 0 ? 0u : q == 1 ? 64u : q == 2 ? (uint32_t)(RS + 1) * 32u : q == 3 ? (uint32_t)(2 * RS) * 32u
                                                                                    : (uint32_t)(2 * RS + 2) * 32u;
    const uint32_t base = q == 1 ? w : q == 4 ? z : c;
    return *(const u32x4*)(buf + base + t0);
  };
  auto write_s = [&](const uint32_t (&raw)[9]) {
    *(u32x4*)(S + s_lds) = u32x4{raw[0] | (raw[1] << 16), raw[2] | (raw[3] << 16), raw[4] | (raw[5] << 16),
                                 raw[6] | (raw[7] << 16)};
    *(u32x4*)(S + s_lds + 16) = u32x4{raw[8], 0u, 0u, 0u};
  };

  // output voxel (kg, lg) offsets of this lane's layer-2 tiles (-1: none / outside the volume)
  int yvox[MT2];
#pragma unroll
  for (int t = 0; t < MT2; ++t) {
    const int vv = vo[t] < 0 ? 0 : vo[t];
    const int kk = vv / TL, ll = vv - kk * TL;
    const int kg = k0 + kk, lg = l0 + ll;
    yvox[t] = (vo[t] >= 0 && kg < g.K && lg < g.L) ? kg * g.L + lg : -1;
  }
  // output row io -> Y (this wave's voxels; lane group lane >> 4 takes planes
  // p = lane >> 4, + 4, ...: all 64 lanes store, not 16)
  auto flush = [&](int io) {
    const int slot = io % 3;
    float* yrow = Y + (((size_t)v * g.I + io) * g.J + j0) * KL;
    const int pg = lane >> 4;
#pragma unroll
    for (int t = 0; t < MT2; ++t) {
      if (wave + NW * t >= nt2) continue;
      if (vo[t] < 0) continue;     // padding lanes of the last tile own no ring entry
      for (int p = pg; p < R; p += 4) {
        float* rp = ring + (slot * GR + p) * rps + vo[t];
        const float val = fmaxf(*rp + bias2, 0.f);
        if (yvox[t] >= 0) yrow[(size_t)p * KL + yvox[t]] = val;
        *rp = 0.f;
      }
    }
  };

  // hidden plane (ih, jh = jh_lo + pj); its gather registers are refilled with
  // the plane two steps ahead (gih, gpj), advanced incrementally (no divisions)
  int ih = ih_lo, pj = 0, gih = ih_lo, gpj = 0;
  int slot0 = (ih_lo + 1) % 3;         // ring slot of output row ih + 1 (row ih - r + 1 -> slot0 - r mod 3)
  auto advance = [&](int& a, int& b) {
    if (++b == nplane) { b = 0; ++a; }
  };
  auto step = [&](uint32_t (&raw)[9], const uint32_t (&other)[9]) {
    const int jh = jh_lo + pj;
    // no barrier here: every wave already passed the previous step's "h
    // complete" barrier, i.e. all layer-1 reads of S are done, and h is next
    // written only after the "S complete" barrier below, i.e. after all
    // layer-2 reads of the previous plane (ring entries are wave-private)
    write_s(raw);
    if (gih < ih_hi) {
      // `other` holds plane (gih, gpj - 1) when gpj >= 1 (same row, one plane back)
      if (gpj >= 1) gather_slide(gih, jh_lo + gpj, raw, other);
      else gather(gih, jh_lo + gpj, raw);
    }
    advance(gih, gpj);
    __syncthreads();                   // S complete
    // ---- B: layer 1 -> h (bf16, zero outside the volume) ----
    // K-step-major: each weight fragment is read from LDS once per plane and
    // feeds every tile of this wave (was: once per tile and K-step, i.e. an
    // LDS read of A beside every LDS read of B)
    f32x4 acc1[MT1];
#pragma unroll
    for (int u = 0; u < MT1; ++u) acc1[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const u32x4 a = wl[q * 64 + lane];
#pragma unroll
      for (int u = 0; u < MT1; ++u)
        if (wave + NW * u < nt1) acc1[u] = mfma16t<F16>(a, bread(S, a1c[u], a1w[u], b1off[u], SRS, q), acc1[u]);
    }
#pragma unroll
    for (int u = 0; u < MT1; ++u) {
      if (wave + NW * u >= nt1) continue;
      const f32x4 acc = acc1[u];
      // branch-free: bias + ReLU, packed conversion of channel pairs, then the
      // zero of voxels outside the volume as one select per packed dword
      float hv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) hv[r] = fmaxf(acc[r] + bias1[r], 0.f);
      u32x2 o;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        uint32_t pk;
        if constexpr (F16) {
          typedef _Float16 h2 __attribute__((ext_vector_type(2)));
          pk = __builtin_bit_cast(uint32_t, h2{(_Float16)hv[2 * r], (_Float16)hv[2 * r + 1]});
        } else {
          typedef __bf16 b2t __attribute__((ext_vector_type(2)));
          pk = __builtin_bit_cast(uint32_t, b2t{(__bf16)hv[2 * r], (__bf16)hv[2 * r + 1]});
        }
        o[r] = h_in[u] ? pk : 0u;
      }
      *(u32x2*)(H + h_wr[u]) = o;
    }
    __syncthreads();                   // h complete
    // ---- C: layer 2 combos -> ring ----
    const int p2 = jh - dj2 + 1 - j0;         // output plane of this lane's combos
    const bool p_ok = dj2 < 3 && p2 >= 0 && p2 < R;
    f32x4 acc2[MT2];
#pragma unroll
    for (int u = 0; u < MT2; ++u) acc2[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const u32x4 a = wl[(NQ + q) * 64 + lane];
#pragma unroll
      for (int u = 0; u < MT2; ++u)
        if (wave + NW * u < nt2) acc2[u] = mfma16t<F16>(a, bread(H, a2c[u], a2w[u], b2off[u], HRS, q), acc2[u]);
    }
#pragma unroll
    for (int u = 0; u < MT2; ++u) {
      if (wave + NW * u >= nt2) continue;
      const f32x4 acc = acc2[u];
      // MFMA row 4 * dj2 + di2 <-> combo (di2, dj2): this lane's rows r share
      // one output plane p2 and differ in the output row ih - r + 1 (uniform).
      // Lanes with no valid (voxel, plane) update a trash word past the ring
      // (never an entry another lane owns: the RMW would race): no exec-mask
      // branch around the update
      const bool lok = vo[u] >= 0 && p_ok;
      const int roff = p2 * rps + vo[u];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int io = ih - r + 1;
        if (io < i0 || io >= i1) continue;
        const int slot = r == 0 ? slot0 : r == 1 ? (slot0 == 0 ? 2 : slot0 - 1) : (slot0 == 2 ? 0 : slot0 + 1);   // io % 3
        float* rp = ring + (lok ? slot * GR * rps + roff : 3 * GR * rps + lane);   // trash: one word per lane
        // read-add-write (lane-private entries); the LDS float atomic
        // (ds_add_f32) measured 3.2x slower for the whole kernel
        *rp += lok ? acc[r] : 0.f;
      }
    }
    // hidden row ih done: output row ih - 1 has all three contributions
    if (pj + 1 == nplane && ih - 1 >= i0 && ih - 1 < i1) flush(ih - 1);
    if (++pj == nplane) { pj = 0; ++ih; slot0 = slot0 == 2 ? 0 : slot0 + 1; }
  };

  __syncthreads();                     // weights in LDS and the zeroed ring visible to every wave
  uint32_t rawA[9], rawB[9];
  gather(gih, jh_lo + gpj, rawA);
  advance(gih, gpj);
  if (gih < ih_hi) gather(gih, jh_lo + gpj, rawB);
  advance(gih, gpj);
  for (int t = 0; t < nsteps; t += 2) {
    step(rawA, rawB);
    if (t + 1 < nsteps) step(rawB, rawA);
  }
  // rows whose last contributing hidden row is past the volume / the segment
  for (int io = max(i0, ih_hi - 1); io < i1; ++io) flush(io);
}

// ===========================================================================
// nc_fused_k3_f8: the same fused stack on OCP e4m3 operands (BASELINE config
// 5, the all-fp8 InLoc pipeline).  Differences from nc_fused_k3:
//  * S and h voxels are 16 bytes (16 fp8 channels): half the LDS tiles;
//  * layer 1 / layer 2 per 16-voxel tile = ONE v_mfma_scale_f32_16x16x128_f8f6f4
//    (taps 0..7 x 16 channels: a lane's 32 operand bytes are taps 2fq, 2fq+1,
//    two ds_read_b128 at per-lane tap offsets) + one v_mfma_f32_16x16x32_fp8_fp8
//    for tap 8 (lane groups fq = 0, 1: channels 0-7 / 8-15; fq = 2, 3 carry
//    zero weights) instead of 5 bf16 MFMAs: 48 instead of 80 matrix cycles and
//    3 instead of 5 LDS reads per tile and layer;
//  * the weight fragments (20 VGPRs) stay in registers for the whole kernel;
//  * power-of-two scales: x0 * sx (x0 in [0, 1] after MutualMatching),
//    weights * sw (amax -> 240), h * sh (sh from the layer-1 output bound, host
//    side), undone in fp32 in the epilogues (inv1 = 1 / (sw1 sx), inv2 =
//    1 / (sw2 sh)).
// Row strides: a 16-voxel tile that wraps a row jumps 1 mod 16 voxels (one
// 256-B bank period + 1): SRS = TL + 18, HRS = TL + 16.
// ===========================================================================
struct NCF8Scales {
  float sx, inv1, sh, inv2;
};

// two floats -> e4m3 bytes 0-1 (HI = false) or 2-3 (HI = true) of `old`
template <bool HI>
__device__ __forceinline__ uint32_t f8x2(float a, float b, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, (int)old, HI);
}

template <int CTK = 0, int CTL = 0, int CR = 0>
__global__ __launch_bounds__(512, 4) void nc_fused_k3_f8_kernel(const bf16* __restrict__ X, const i32x8* __restrict__ W1a,
                                                                const long* __restrict__ W1b, const float* __restrict__ b1,
                                                                const i32x8* __restrict__ W2a, const long* __restrict__ W2b,
                                                                const float* __restrict__ b2, float* __restrict__ Y,
                                                                NCFGeom g, NCF8Scales sc) {
  constexpr int NW = 8, MT1 = 4, MT2 = 3;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int TK = CTK ? CTK : g.TK, TL = CTL ? CTL : g.TL;
  const int GR = CR ? CR : g.R;
  const int SRS = CTL ? CTL + 18 : g.SRS, HRS = CTL ? CTL + 16 : g.HRS;
  const int SR = TK + 4, SW = TL + 4;
  const int HR = TK + 2, HW = TL + 2;
  char* S = smem;
  char* H = S + SR * SRS * 16;
  float* ring = (float*)(H + HR * HRS * 16);
  const int nvox = TK * TL;
  const int rps = ncf_ring_stride(nvox);

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NW);
  uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int lt = bid % g.nlt; bid /= g.nlt;
  const int kt = bid % g.nkt; bid /= g.nkt;
  const int jb = bid % g.njb; bid /= g.njb;
  const int ib = bid % g.nib;
  const int v = bid / g.nib;
  const int k0 = kt * TK, l0 = lt * TL, j0 = jb * GR, i0 = ib * g.IR;
  const int i1 = min(g.I, i0 + g.IR);
  const int R = min(GR, g.J - j0);
  const size_t KL = (size_t)g.K * g.L;
  const int KLi = g.K * g.L;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X + (size_t)v * g.I * g.J * KL), (short)0, (int)((size_t)g.I * g.J * KL * 2), 0x00020000);

  // ---- static maps (as nc_fused_k3, 16-byte voxels) -------------------------
  int s_lds, s_goff;
  {
    const int e = threadIdx.x;
    const int r = e / SW, c = e - r * SW;
    const int kg = k0 - 2 + r, lg = l0 - 2 + c;
    const bool in = e < SR * SW && kg >= 0 && kg < g.K && lg >= 0 && lg < g.L;
    s_lds = (e < SR * SW) ? (r * SRS + c) * 16 : SW * 16;
    s_goff = in ? (kg * g.L + lg) * 2 : 0x7ffffff0;
  }
  const int fr = lane & 15, fq = lane >> 4;
  // per-lane tap offsets (voxels) of the MX fragment (taps 2fq, 2fq + 1) and of tap 8
  auto tapoff = [](int t, int rs) { return (t / 3) * rs + t % 3; };
  const int st0 = tapoff(2 * fq, SRS) * 16, st1 = tapoff(2 * fq + 1, SRS) * 16, st8 = tapoff(8, SRS) * 16 + 8 * (fq & 1);
  const int ht0 = tapoff(2 * fq, HRS) * 16, ht1 = tapoff(2 * fq + 1, HRS) * 16, ht8 = tapoff(8, HRS) * 16 + 8 * (fq & 1);
  const int nt1 = (HR * HW + 15) >> 4;
  uint32_t s1b[MT1], h_wr[MT1];
  bool h_in[MT1];
#pragma unroll
  for (int t = 0; t < MT1; ++t) {
    int e = (wave + NW * t) * 16 + fr;
    const bool ok = e < HR * HW;
    if (!ok) e = 0;
    const int r = e / HW, c = e - r * HW;
    s1b[t] = (uint32_t)((r * SRS + c) * 16);
    h_wr[t] = (uint32_t)((ok ? r * HRS + c : HW) * 16 + 4 * fq);
    const int kg = k0 - 1 + r, lg = l0 - 1 + c;
    h_in[t] = ok && kg >= 0 && kg < g.K && lg >= 0 && lg < g.L;
  }
  const int nt2 = (nvox + 15) >> 4;
  uint32_t h2b[MT2];
  int vo[MT2];
#pragma unroll
  for (int t = 0; t < MT2; ++t) {
    int vi = (wave + NW * t) * 16 + fr;
    vo[t] = vi < nvox ? vi : -1;
    if (vi >= nvox) vi = 0;
    const int kk = vi / TL, ll = vi - kk * TL;
    h2b[t] = (uint32_t)((kk * HRS + ll) * 16);
  }
  // weights: register-resident fragments (rows = output channels / layer-2 combos)
  const i32x8 w1a = W1a[lane], w2a = W2a[lane];
  const long w1b = W1b[lane], w2b = W2b[lane];
  const int co0 = 4 * fq;
  const int dj2 = fq;
  float bias1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias1[r] = b1[co0 + r];
  const float bias2 = b2[0];

  for (int o = threadIdx.x; o < 3 * GR * rps; o += NW * 64) ring[o] = 0.f;

  const int ih_lo = max(0, i0 - 1), ih_hi = min(g.I, i1 + 1);
  const int jh_lo = max(0, j0 - 1), jh_hi = min(g.J, j0 + R + 1);
  const int nplane = jh_hi - jh_lo;
  const int nsteps = (ih_hi - ih_lo) * nplane;

  const int pstride = KLi * 2, rstride = g.J * KLi * 2;
  const int nrec = (int)((size_t)g.I * g.J * KL * 2);
  auto gather = [&](int ih, int jh, uint32_t (&raw)[9]) {
    const int base = (ih * g.J + jh) * pstride;
    const bool iok[3] = {ih >= 1, true, ih + 1 < g.I}, jok[3] = {jh >= 1, true, jh + 1 < g.J};
#pragma unroll
    for (int c = 0; c < 9; ++c) {
      const int di = c / 3, dj = c % 3;
      const int so = (iok[di] && jok[dj]) ? base + (di - 1) * rstride + (dj - 1) * pstride : nrec;
      raw[c] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(xr, s_goff, __builtin_amdgcn_readfirstlane(so), 0);
    }
  };
  auto gather_slide = [&](int ih, int jh, uint32_t (&raw)[9], const uint32_t (&prev)[9]) {
    const int base = (ih * g.J + jh) * pstride;
    const bool iok[3] = {ih >= 1, true, ih + 1 < g.I};
    const bool jok = jh + 1 < g.J;
#pragma unroll
    for (int di = 0; di < 3; ++di) {
      const int so = (iok[di] && jok) ? base + (di - 1) * rstride + pstride : nrec;
      raw[di * 3 + 2] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(xr, s_goff, __builtin_amdgcn_readfirstlane(so), 0);
    }
#pragma unroll
    for (int di = 0; di < 3; ++di) {
      raw[di * 3 + 0] = prev[di * 3 + 1];
      raw[di * 3 + 1] = prev[di * 3 + 2];
    }
  };
  // S voxel: the 9 combos as e4m3 (x0 * sx, clamped), channels 9..15 zero
  auto write_s = [&](const uint32_t (&raw)[9]) {
    float f[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) f[c] = fminf(fmaxf(__uint_as_float(raw[c] << 16) * sc.sx, -448.f), 448.f);
    uint32_t w0 = f8x2<false>(f[0], f[1], 0u);
    w0 = f8x2<true>(f[2], f[3], w0);
    uint32_t w1 = f8x2<false>(f[4], f[5], 0u);
    w1 = f8x2<true>(f[6], f[7], w1);
    const uint32_t w2 = f8x2<false>(f[8], 0.f, 0u);
    *(u32x4*)(S + s_lds) = u32x4{w0, w1, w2, 0u};
  };
  auto frag = [&](const char* buf, uint32_t a0, uint32_t a1) -> i32x8 {
    const u32x4 lo = *(const u32x4*)(buf + a0), hi = *(const u32x4*)(buf + a1);
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };

  int yvox[MT2];
#pragma unroll
  for (int t = 0; t < MT2; ++t) {
    const int vv = vo[t] < 0 ? 0 : vo[t];
    const int kk = vv / TL, ll = vv - kk * TL;
    const int kg = k0 + kk, lg = l0 + ll;
    yvox[t] = (vo[t] >= 0 && kg < g.K && lg < g.L) ? kg * g.L + lg : -1;
  }
  auto flush = [&](int io) {
    const int slot = io % 3;
    float* yrow = Y + (((size_t)v * g.I + io) * g.J + j0) * KL;
    const int pg = lane >> 4;
#pragma unroll
    for (int t = 0; t < MT2; ++t) {
      if (wave + NW * t >= nt2) continue;
      if (vo[t] < 0) continue;
      for (int p = pg; p < R; p += 4) {
        float* rp = ring + (slot * GR + p) * rps + vo[t];
        const float val = fmaxf(*rp + bias2, 0.f);
        if (yvox[t] >= 0) yrow[(size_t)p * KL + yvox[t]] = val;
        *rp = 0.f;
      }
    }
  };

  int ih = ih_lo, pj = 0, gih = ih_lo, gpj = 0;
  int slot0 = (ih_lo + 1) % 3;
  auto advance = [&](int& a, int& b) {
    if (++b == nplane) { b = 0; ++a; }
  };
  auto step = [&](uint32_t (&raw)[9], const uint32_t (&other)[9]) {
    const int jh = jh_lo + pj;
    write_s(raw);
    if (gih < ih_hi) {
      if (gpj >= 1) gather_slide(gih, jh_lo + gpj, raw, other);
      else gather(gih, jh_lo + gpj, raw);
    }
    advance(gih, gpj);
    __syncthreads();                   // S complete
    // ---- layer 1 -> h (e4m3 h * sh, zero outside the volume) ----
#pragma unroll
    for (int u = 0; u < MT1; ++u) {
      if (wave + NW * u >= nt1) continue;
      const i32x8 bx = frag(S, s1b[u] + st0, s1b[u] + st1);
      const long b8 = *(const long*)(S + s1b[u] + st8);
      // two independent accumulators, summed by VALU: a 16x16x32 fp8 MFMA
      // reading the scaled MFMA's result as srcC read stale rows (no wait
      // states are inserted between the two MFMA kinds for that chain;
      // tests/test_gpu_kernels.py test_nc_fused_k3_f8_vs_quantized_oracle).
      // One tile at a time: all tiles' accumulators live at once spill at
      // the 128-VGPR budget of two workgroups per CU.
      const f32x4 a8 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(w1b, b8, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const f32x4 acc = mfma_fp8_k128(w1a, bx, f32x4{0.f, 0.f, 0.f, 0.f}) + a8;
      float hv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) hv[r] = fminf(fmaxf(acc[r] * sc.inv1 + bias1[r], 0.f) * sc.sh, 448.f);
      uint32_t pk = f8x2<false>(hv[0], hv[1], 0u);
      pk = f8x2<true>(hv[2], hv[3], pk);
      *(uint32_t*)(H + h_wr[u]) = h_in[u] ? pk : 0u;
    }
    __syncthreads();                   // h complete
    // ---- layer 2 combos -> ring ----
    const int p2 = jh - dj2 + 1 - j0;
    const bool p_ok = dj2 < 3 && p2 >= 0 && p2 < R;
#pragma unroll
    for (int u = 0; u < MT2; ++u) {
      if (wave + NW * u >= nt2) continue;
      const i32x8 bh = frag(H, h2b[u] + ht0, h2b[u] + ht1);
      const long b8 = *(const long*)(H + h2b[u] + ht8);
      const f32x4 a8 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(w2b, b8, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const f32x4 acc = mfma_fp8_k128(w2a, bh, f32x4{0.f, 0.f, 0.f, 0.f}) + a8;
      const bool lok = vo[u] >= 0 && p_ok;
      const int roff = p2 * rps + vo[u];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int io = ih - r + 1;
        if (io < i0 || io >= i1) continue;
        const int slot = r == 0 ? slot0 : r == 1 ? (slot0 == 0 ? 2 : slot0 - 1) : (slot0 == 2 ? 0 : slot0 + 1);
        float* rp = ring + (lok ? slot * GR * rps + roff : 3 * GR * rps + lane);
        *rp += lok ? acc[r] * sc.inv2 : 0.f;
      }
    }
    if (pj + 1 == nplane && ih - 1 >= i0 && ih - 1 < i1) flush(ih - 1);
    if (++pj == nplane) { pj = 0; ++ih; slot0 = slot0 == 2 ? 0 : slot0 + 1; }
  };

  __syncthreads();
  uint32_t rawA[9], rawB[9];
  gather(gih, jh_lo + gpj, rawA);
  advance(gih, gpj);
  if (gih < ih_hi) gather(gih, jh_lo + gpj, rawB);
  advance(gih, gpj);
  for (int t = 0; t < nsteps; t += 2) {
    step(rawA, rawB);
    if (t + 1 < nsteps) step(rawB, rawA);
  }
  for (int io = max(i0, ih_hi - 1); io < i1; ++io) flush(io);
}

}  // namespace ncnet

using namespace ncnet;

// x0 bf16 [V,I,J,K,L]; W1p / W2p bf16 [5][64][8] (pack_w16_planes of the ij layer weights);
// b1 fp32 [16], b2 fp32 [1]; y fp32 [V,I,J,K,L].
// f16: x0 / W1p / W2p are IEEE half (f16 MFMA, f16 hidden activation).
extern "C" int ncnet_nc_fused_k3(const void* X, const void* W1p, const float* b1, const void* W2p, const float* b2,
                                 float* Y, int V, int I, int J, int K, int L, int R, int IR, int TK, int TL, int f16,
                                 hipStream_t stream) {
  NCFGeom g{};
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L;
  g.TK = TK; g.TL = TL; g.R = R; g.IR = IR;
  g.nkt = cdiv(K, TK); g.nlt = cdiv(L, TL); g.njb = cdiv(J, R); g.nib = cdiv(I, IR);
  g.SRS = TL + 10;   // S rows: a layer-1 tile wrapping from column TL+1 to 0 jumps 9 voxels (one 256-B bank period + 1)
  g.HRS = TL + 8;    // h rows: a layer-2 tile wrapping from column TL-1 to 0 jumps 9 voxels
  if ((long long)I * J * K * L * 2 >= (1ll << 31)) return -4;   // buffer-resource byte offsets
  size_t lds = (size_t)(TK + 4) * g.SRS * 32 + (size_t)(TK + 2) * g.HRS * 32 +
               (size_t)((3 * R * ncf_ring_stride(TK * TL) + 64 + 3) & ~3) * 4 + 2 * 5 * 64 * 16;
  // > 80 KB: one 16-wave workgroup per CU (NW = 16) instead of two 8-wave ones
  const bool big = lds > 80 * 1024;
  const int nw = big ? 16 : 8;
  if ((TK + 2) * (TL + 2) > 512 || TK * TL > nw * (big ? 2 : 3) * 16 || (TK + 4) * (TL + 4) > nw * 64 || R < 1 ||
      IR < 1)
    return -2;
  if (lds > 160 * 1024) return -3;
  dim3 grid((unsigned)((size_t)V * g.nib * g.njb * g.nkt * g.nlt)), block(nw * 64);
#define NCF(H, A, B, C, W) hipLaunchKernelGGL((nc_fused_k3_kernel<H, A, B, C, W>), grid, block, lds, stream, (const bf16*)X, \
                                              (const u32x4*)W1p, b1, (const u32x4*)W2p, b2, Y, g)
  // the tiles ops/neigh_consensus.py fused_tiles picks at 3200 px (75x100 planes)
  // and 1600 px (37x50) get compile-time geometry; anything else the runtime one
  const bool t3200 = TK == 15 && TL == 20 && R == 10, t1600 = TK == 19 && TL == 17 && R == 8;
  const bool t3200b = big && TK == 15 && TL == 20 && R == 20;
  if (f16) {
    if (t3200b) NCF(true, 15, 20, 20, 16); else if (big) NCF(true, 0, 0, 0, 16);
    else if (t3200) NCF(true, 15, 20, 10, 8); else if (t1600) NCF(true, 19, 17, 8, 8); else NCF(true, 0, 0, 0, 8);
  } else {
    if (t3200b) NCF(false, 15, 20, 20, 16); else if (big) NCF(false, 0, 0, 0, 16);
    else if (t3200) NCF(false, 15, 20, 10, 8); else if (t1600) NCF(false, 19, 17, 8, 8); else NCF(false, 0, 0, 0, 8);
  }
#undef NCF
  return (int)hipGetLastError();
}

// fp8 fused stack: x0 bf16 [V,I,J,K,L]; W1a / W2a [64] x 32 B MX fragments of
// taps 0..7, W1b / W2b [64] x 8 B fragments of tap 8 (e4m3, weights * sw);
// b1 fp32 [16], b2 fp32 [1]; y fp32.  Scales: sx (x0), inv1 = 1 / (sw1 sx),
// sh (hidden), inv2 = 1 / (sw2 sh).
extern "C" int ncnet_nc_fused_k3_f8(const void* X, const void* W1a, const void* W1b, const float* b1, const void* W2a,
                                    const void* W2b, const float* b2, float* Y, int V, int I, int J, int K, int L, int R,
                                    int IR, int TK, int TL, float sx, float inv1, float sh, float inv2,
                                    hipStream_t stream) {
  NCFGeom g{};
  g.V = V; g.I = I; g.J = J; g.K = K; g.L = L;
  g.TK = TK; g.TL = TL; g.R = R; g.IR = IR;
  g.nkt = cdiv(K, TK); g.nlt = cdiv(L, TL); g.njb = cdiv(J, R); g.nib = cdiv(I, IR);
  g.SRS = TL + 18;
  g.HRS = TL + 16;
  if ((long long)I * J * K * L * 2 >= (1ll << 31)) return -4;
  const size_t lds = (size_t)(TK + 4) * g.SRS * 16 + (size_t)(TK + 2) * g.HRS * 16 +
                     (size_t)(3 * R * ncf_ring_stride(TK * TL) + 64) * 4;
  if ((TK + 2) * (TL + 2) > 512 || TK * TL > 8 * 3 * 16 || (TK + 4) * (TL + 4) > 512 || R < 1 || IR < 1) return -2;
  if (lds > 80 * 1024) return -3;
  NCF8Scales sc{sx, inv1, sh, inv2};
  dim3 grid((unsigned)((size_t)V * g.nib * g.njb * g.nkt * g.nlt)), block(512);
#define NCF8(A, B, C) hipLaunchKernelGGL((nc_fused_k3_f8_kernel<A, B, C>), grid, block, lds, stream, (const bf16*)X, \
                                         (const i32x8*)W1a, (const long*)W1b, b1, (const i32x8*)W2a, (const long*)W2b, b2, Y, g, sc)
  // ops/neigh_consensus.py runs the bf16 kernel's tiling (fused_tiles): the
  // 3200 px and 1600 px tiles get compile-time geometry
  if (TK == 15 && TL == 20 && R == 10) NCF8(15, 20, 10);
  else if (TK == 19 && TL == 17 && R == 8) NCF8(19, 17, 8);
  else NCF8(0, 0, 0);
#undef NCF8
  return (int)hipGetLastError();
}
