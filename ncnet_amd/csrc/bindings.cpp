// Python bindings for the gfx950 NC-Net kernels.
//
// Every entry point validates device, dtype, contiguity and the exact shapes
// the kernel's grid assumes BEFORE launching: a malformed call raises a Python
// exception instead of faulting the GPU.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

extern "C" {
int ncnet_conv16_fwd(const void*, const void*, const float*, const void*, void*, int, int, int, int, int, int, int, int, int,
                     long long, long long, hipStream_t);
int ncnet_set_tuning(const char*, int, int);
int ncnet_conv16_blk_fwd(const void*, const void*, const float*, float*, int, int, int, int, int, int, int, int, long long,
                         hipStream_t);
int ncnet_wgrad16(const void*, const void*, float*, float*, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_wgrad16p(const void*, const void*, float*, float*, int, int, int, int, int, int, int, int, int, long long,
                   long long, hipStream_t);
int ncnet_wgrad16v3(const void*, const void*, float*, float*, int, int, int, int, int, int, int, hipStream_t);
int ncnet_ijpack(const void*, int, void*, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_conv16f8_fwd(const void*, const void*, const float*, void*, int, int, int, int, int, int, int, int, int, float, hipStream_t);
int ncnet_ijsum(const float*, const float*, float*, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_bias_act(void*, const float*, long long, int, int, int, hipStream_t);
int ncnet_maxpool_bias_act(const void*, void*, const float*, int, int, int, int, int, int, int, int, int, int, int,
                           hipStream_t);
int ncnet_conv2d_nhwc_x3(const void*, const void*, const float*, const void*, void*, int, int, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_stem_im2col_x3(const float*, void*, int, int, int, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_maxpool_x3(const void*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_x3_to_f32(const void*, float*, long long, int, hipStream_t);
int ncnet_conv2d_nhwc(const void*, const void*, const float*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, hipStream_t);
int ncnet_cout1_taps_fwd(const void*, const void*, const float*, float*, int, int, int, int, int, int, int, hipStream_t);
int ncnet_gemm_lt(const void*, const void*, const float*, const void*, void*, int, int, int, int, int, int, hipStream_t);
int ncnet_l2norm_rows(const void*, int, void*, float*, int, int, float, void*, int, hipStream_t);
int ncnet_l2norm_rows_bwd(const float*, const float*, const float*, float*, int, int, hipStream_t);
int ncnet_corr_gemm(const void*, const void*, void*, const int*, const int*, int, int, int, int, long long, long long,
                    long long, int, float, int, hipStream_t);
int ncnet_corr_gemm_pool2(const void*, const void*, float*, uint8_t*, int, int, int, int, int, int, long long, long long,
                          float, int, hipStream_t);
int ncnet_stats_rows(const float*, float*, int*, float*, long long, int, int, hipStream_t);
int ncnet_stats_cols(const float*, float*, int*, float*, int, int, int, float*, int, int, hipStream_t);
int ncnet_gather_bf16(const float*, const int*, void*, long long, long long, hipStream_t);
int ncnet_reduce_cols(const float* const*, float* const*, const int* const*, const int*, const int*, const long long*,
                      int, hipStream_t);
int ncnet_stats2d(const float*, float*, int*, float*, float*, int*, float*, int, int, int, float*, int, hipStream_t);
int ncnet_match_candidates(const float*, const float*, const int*, const float*, const float*, const int*,
                           const uint8_t*, int, int, int, int, int, float*, float*, long long*, hipStream_t);
int ncnet_mm_apply(const float*, const float*, const float*, float*, void*, void*, int, int, int, float, int, int, int, int,
                   int, int, hipStream_t);
int ncnet_mm_bwd(const float*, const float*, const float*, const int*, const float*, const int*, float*, float*, float*,
                 int, int, int, float, float*, hipStream_t);
int ncnet_combine_fwd(const float*, float*, int, int, int, hipStream_t);
int ncnet_combine_bwd(const float*, const float*, void*, void*, int, int, int, hipStream_t);
int ncnet_softmax_max_bwd(const float*, const float*, const int*, const float*, const float*, const int*, const float*,
                          const float*, const float*, float*, int, int, int, int, float, const float*, hipStream_t);
int ncnet_score_sum(const float*, const float*, const float*, const float*, const float*, const float*, int, int, int, int,
                    float, float*, hipStream_t);
int ncnet_maxpool4d(const void*, int, float*, uint8_t*, int, int, int, int, int, int, hipStream_t);
int ncnet_transpose(const void*, void*, int, int, int, int, hipStream_t);
int ncnet_nonfinite_count(const float*, long long, int*, hipStream_t);
int ncnet_adam_masked(float*, float*, float*, float*, long long, const int*, const float*, float, float, float, float,
                      float, float, hipStream_t);
int ncnet_adam_finalize(float*, int*, int*, hipStream_t);
int ncnet_resize_norm_u8(const void*, const long long*, float*, int, int, int, const float*, const float*, hipStream_t);
int ncnet_debug_selftest(int*, hipStream_t);
int ncnet_pad_geom(int, int, int, int*, int*);
int ncnet_pad_planes(const void*, int, void*, int, int, int, int, int, int, int, hipStream_t);
int ncnet_conv1x16(const void*, const void*, const float*, const void*, void*, int, int, int, int, int, int, int, int, long long, long long, hipStream_t);
int ncnet_wgrad1x16(const void*, const void*, float*, float*, int, int, int, int, int, int, int, hipStream_t);
int ncnet_nc_fused_k3(const void*, const void*, const float*, const void*, const float*, float*, int, int, int, int,
                      int, int, int, int, int, int, hipStream_t);
int ncnet_nc_fused_k3_f8(const void*, const void*, const void*, const float*, const void*, const void*, const float*,
                         float*, int, int, int, int, int, int, int, int, int, float, float, float, float, hipStream_t);
}

namespace {

using torch::Tensor;

// PyTorch-ROCm exposes HIP devices as device type "cuda": use the masquerading guard/stream.
hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(const Tensor& t, const char* name, c10::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
void check_shape(const Tensor& t, const char* name, std::vector<int64_t> shape) {
  TORCH_CHECK(t.sizes().vec() == shape, name, " has shape ", t.sizes(), ", expected ", c10::IntArrayRef(shape));
}
void ok(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " launch failed (code ", rc, ")"); }
template <typename T>
const T* opt_ptr(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? (const T*)t->data_ptr() : nullptr; }

int conv_pairs16(int ks) { return (ks * ks + 1) / 2; }
// Conv4d kernel sizes with HIP kernels: 5 and 3 (NC-Net's), 1 and 7.
void check_ks(int64_t ks) { TORCH_CHECK(ks == 1 || ks == 3 || ks == 5 || ks == 7, "Conv4d kernel size must be 1, 3, 5 or 7 (got ", ks, ")"); }

// X [V,I,J,K,L,16] (all KS*KS planes (i+di-P, j+dj-P)) or X [G,V,I,J,K,L,16]
// (group planes: G input groups at the (i, j) plane, Wp [G, ...], in-plane taps only).
// epi: 0 none -> bf16, 1 bias+ReLU -> bf16, 2 ReLU-mask M -> bf16,
//      4 fp32 channel-planar [nco,V,I,J,K,L] (first nco <= 16 output channels).
// padded 1-channel planes (csrc/conv1x.hip): {LP, PPL} of a (K, L) plane
std::vector<int64_t> pad_geom(int64_t K, int64_t L, int64_t ks) {
  int lp, ppl;
  ncnet_pad_geom((int)K, (int)L, (int)ks, &lp, &ppl);
  return {lp, ppl};
}

// x [V, R, C] (fp32 / bf16) -> y [N, PPL] bf16 padded planes (trans 0: N = V*R
// planes [I2, J2] = rows of x; trans 1: N = V*C planes of the A<->B swap).  y's halo
// must already be zero.
void pad_planes(Tensor x, Tensor y, int64_t I2, int64_t J2, int64_t ks, int64_t trans) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 3, "x must be a contiguous [V, R, C] GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be fp32 or bf16");
  check(y, "y", at::kBFloat16);
  check_ks(ks);
  const int64_t V = x.size(0), R = x.size(1), C = x.size(2);
  const int64_t planes = trans ? V * C : V * R;
  TORCH_CHECK(I2 * J2 == (trans ? R : C), "plane dims do not match x");
  const auto g = pad_geom(I2, J2, ks);
  check_shape(y, "y", {planes, g[1]});
  ok(ncnet_pad_planes(x.data_ptr(), x.scalar_type() == at::kBFloat16, y.data_ptr(), (int)V, (int)R, (int)C, (int)I2,
                      (int)J2, (int)ks, (int)trans, cur_stream(x)),
     "pad_planes");
}

// 1 -> 16 Conv4d on padded 1-channel planes Xp [V*I*J, PPL] with A fragments Wa
// [ks^2, 64, 8]; Y bf16 [V,I,J,K,L,16]; epi 1 (bias + ReLU) or 2 (ReLU mask M).
// Raises for shapes without an instantiation (ops/neigh_consensus.py fast1x_ok
// must never route one here: the outputs are uninitialised buffers).
bool conv1x16(Tensor Xp, Tensor Wa, c10::optional<Tensor> bias, c10::optional<Tensor> M, Tensor Y, int64_t ks,
              int64_t epi) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(Xp.device());
  check(Xp, "Xp", at::kBFloat16); check(Wa, "Wa", at::kBFloat16); check(Y, "Y", at::kBFloat16);
  check_ks(ks);
  // epi 1 / 2; | 4: the bf16x3 layer -- Xp [2, N, PPL] (hi, lo planes), Wa [2, ks^2, 64, 8]
  // (hi, lo fragments), Y [2, V,I,J,K,L,16] (hi, lo)
  const bool x3 = (epi & 4) != 0;
  const int e = (int)(epi & 3);
  TORCH_CHECK(e == 1 || e == 2, "conv1x16: epi must be 1 or 2 (| 4 for bf16x3)");
  const Tensor Y1 = x3 ? Y[0] : Y;
  TORCH_CHECK(!x3 || (Y.dim() == 7 && Y.size(0) == 2), "conv1x16 x3: Y must be [2,V,I,J,K,L,16]");
  TORCH_CHECK(Y1.dim() == 6 && Y1.size(5) == 16, "Y must be [V,I,J,K,L,16]");
  const int64_t V = Y1.size(0), I = Y1.size(1), J = Y1.size(2), K = Y1.size(3), L = Y1.size(4);
  const auto g = pad_geom(K, L, ks);
  if (x3) { check_shape(Xp, "Xp", {2, V * I * J, g[1]}); check_shape(Wa, "Wa", {2, ks * ks, 64, 8}); }
  else { check_shape(Xp, "Xp", {V * I * J, g[1]}); check_shape(Wa, "Wa", {ks * ks, 64, 8}); }
  if (e == 1) { TORCH_CHECK(bias.has_value()); check(*bias, "bias", at::kFloat); check_shape(*bias, "bias", {16}); }
  if (e == 2) { TORCH_CHECK(M.has_value()); check(*M, "M", at::kBFloat16); check_shape(*M, "M", {V, I, J, K, L, 16}); }
  const int nt = ncnet_set_tuning("nt_store", 0, 0);
  const long long xlo = x3 ? (long long)V * I * J * g[1] : 0, ylo = x3 ? (long long)Y1.numel() : 0;
  const int r = ncnet_conv1x16(Xp.data_ptr(), Wa.data_ptr(), opt_ptr<float>(bias), opt_ptr<void>(M), Y.data_ptr(),
                               (int)V, (int)I, (int)J, (int)K, (int)L, (int)ks, (int)epi, nt, xlo, ylo, cur_stream(Xp));
  TORCH_CHECK(r != -1, "conv1x16: no kernel instantiation for ks=", ks, " K=", K, " L=", L, " epi=", epi);
  ok(r, "conv1x16");
  return true;
}

// Weight-gradient partials of a Conv4d with a 1-channel operand (csrc/conv1x.hip
// wgrad1x16): D bf16 [V,I,J,K,L,16], X1 padded planes [V*I*J, PPL];
// part fp32 [G, ks^2, 32, 16] (G workgroups, one partial each), partb fp32 [G, 16]
// (the sum of D) or None.  Raises for shapes without an instantiation.
bool wgrad1x16(Tensor D, Tensor X1, Tensor part, c10::optional<Tensor> partb, int64_t ks) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(D.device());
  check(D, "D", at::kBFloat16); check(X1, "X1", at::kBFloat16); check(part, "part", at::kFloat);
  check_ks(ks);
  TORCH_CHECK(D.dim() == 6 && D.size(5) == 16, "D must be [V,I,J,K,L,16]");
  const int64_t V = D.size(0), I = D.size(1), J = D.size(2), K = D.size(3), L = D.size(4);
  const auto g = pad_geom(K, L, ks);
  check_shape(X1, "X1", {V * I * J, g[1]});
  TORCH_CHECK(part.dim() == 4 && part.size(0) >= 1, "part must be [G, ks^2, 32, 16]");
  const int64_t G = part.size(0);
  check_shape(part, "part", {G, ks * ks, 32, 16});
  if (partb.has_value()) { check(*partb, "partb", at::kFloat); check_shape(*partb, "partb", {G, 16}); }
  TORCH_CHECK(V * I * J < (1ll << 31), "too many planes");
  const int r = ncnet_wgrad1x16(D.data_ptr(), X1.data_ptr(), (float*)part.data_ptr(),
                                partb.has_value() ? (float*)partb->data_ptr() : nullptr, (int)G, (int)V, (int)I,
                                (int)J, (int)K, (int)L, (int)ks, cur_stream(D));
  TORCH_CHECK(r != -1, "wgrad1x16: no kernel instantiation for ks=", ks, " K=", K, " L=", L);
  ok(r, "wgrad1x16");
  return true;
}

void conv16_fwd(Tensor X, Tensor Wp, c10::optional<Tensor> bias, c10::optional<Tensor> M, Tensor Y, int64_t ks, int64_t epi) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Wp, "Wp", at::kBFloat16);
  check_ks(ks);
  const bool grp = X.dim() == 7;
  TORCH_CHECK((X.dim() == 6 || grp) && X.size(-1) == 16, "X must be [V,I,J,K,L,16] or [G,V,I,J,K,L,16]");
  const int64_t npg = grp ? X.size(0) : 0;
  std::vector<int64_t> vs(X.sizes().begin() + (grp ? 1 : 0), X.sizes().end());   // [V,I,J,K,L,16]
  TORCH_CHECK(epi == 0 || epi == 1 || epi == 2 || epi == 4, "conv16_fwd: epi must be 0, 1, 2 or 4");
  int64_t nco = 16;
  if (epi == 4) {
    check(Y, "Y", at::kFloat);
    nco = Y.size(0);
    TORCH_CHECK(nco >= 1 && nco <= 16, "planar output channels out of range");
    check_shape(Y, "Y", {nco, vs[0], vs[1], vs[2], vs[3], vs[4]});
  } else {
    check(Y, "Y", at::kBFloat16);
    check_shape(Y, "Y", vs);
  }
  check_shape(Wp, "Wp", {grp ? npg : ks * ks, conv_pairs16(ks), 64, 8});
  if (epi == 1) { TORCH_CHECK(bias.has_value()); check(*bias, "bias", at::kFloat); check_shape(*bias, "bias", {16}); }
  if (epi == 2) { TORCH_CHECK(M.has_value()); check(*M, "M", at::kBFloat16); check_shape(*M, "M", vs); }
  ok(ncnet_conv16_fwd(X.data_ptr(), Wp.data_ptr(), opt_ptr<float>(bias), opt_ptr<void>(M), Y.data_ptr(), vs[0],
                      vs[1], vs[2], vs[3], vs[4], ks, epi, (int)npg, (int)nco, 0, 0, cur_stream(X)),
     "conv16_fwd");
}

// Launcher tuning switch ``name`` (common.h NcnetTuning): returns its value
// before the call and sets it when ``value`` is given.  A/B tests and kbench.
int64_t set_tuning(const std::string& name, c10::optional<int64_t> value) {
  const int old = ncnet_set_tuning(name.c_str(), value.has_value() ? (int)*value : 0, value.has_value() ? 1 : 0);
  TORCH_CHECK(old != INT32_MIN, "set_tuning: unknown switch ", name);
  return old;
}

// element offset of b from a (same dtype, same device): the kernels address the
// lo operand of a bf16x3 layer relative to the hi one
static long long elem_offset(const Tensor& a, const Tensor& b) {
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.device() == b.device(), "hi / lo operands must match");
  const long long d = (long long)((const char*)b.data_ptr() - (const char*)a.data_ptr());
  TORCH_CHECK(d % (long long)a.element_size() == 0, "misaligned lo operand");
  return d / (long long)a.element_size();
}

// fp32-accurate ("bf16x3") Conv4d layer, KS 3 / 5:
//   y = conv(Xh, Wh) + conv(Xh, Wl) + conv(Xl, Wh)   (one kernel, fp32 accumulators)
// X / Xl: [V,I,J,K,L,16] or group planes [G,V,I,J,K,L,16]; Wp2 [2, planes, nq, 64, 8]
// (hi set, lo set); epi 1: y = relu(y + bias), epi 2: y = y * (M > 0) (M: the hi part of
// the previous layer's ReLU output).  Output split: Y = bf16(y), Yl = bf16(y - Y).
void conv16_fwd_x3(Tensor X, Tensor Xl, Tensor Wp2, c10::optional<Tensor> bias, c10::optional<Tensor> M, Tensor Y,
                   Tensor Yl, int64_t ks, int64_t epi) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Xl, "Xl", at::kBFloat16); check(Wp2, "Wp2", at::kBFloat16);
  check(Y, "Y", at::kBFloat16); check(Yl, "Yl", at::kBFloat16);
  TORCH_CHECK(ks == 3 || ks == 5, "conv16_fwd_x3: kernel size 3 or 5");
  const bool grp = X.dim() == 7;
  TORCH_CHECK((X.dim() == 6 || grp) && X.size(-1) == 16, "X must be [V,I,J,K,L,16] or [G,V,I,J,K,L,16]");
  TORCH_CHECK(Xl.sizes() == X.sizes(), "Xl must match X");
  const int64_t npg = grp ? X.size(0) : 0;
  std::vector<int64_t> vs(X.sizes().begin() + (grp ? 1 : 0), X.sizes().end());
  check_shape(Y, "Y", vs); check_shape(Yl, "Yl", vs);
  check_shape(Wp2, "Wp2", {2, grp ? npg : ks * ks, conv_pairs16(ks), 64, 8});
  TORCH_CHECK(epi == 1 || epi == 2, "conv16_fwd_x3: epi must be 1 or 2");
  if (epi == 1) { TORCH_CHECK(bias.has_value()); check(*bias, "bias", at::kFloat); check_shape(*bias, "bias", {16}); }
  if (epi == 2) { TORCH_CHECK(M.has_value()); check(*M, "M", at::kBFloat16); check_shape(*M, "M", vs); }
  ok(ncnet_conv16_fwd(X.data_ptr(), Wp2.data_ptr(), opt_ptr<float>(bias), opt_ptr<void>(M), Y.data_ptr(), vs[0],
                      vs[1], vs[2], vs[3], vs[4], ks, (int)epi | 64, (int)npg, 16, elem_offset(X, Xl),
                      elem_offset(Y, Yl), cur_stream(X)),
     "conv16_fwd_x3");
}

// Cout = 1 layer (<= 16 input channels) in output-plane-block mode:
// Y [V,I,J,K,L] fp32 = act(bias + conv); Wp [(ks+3)^2, nq, 64, 8] (packing.blk_out_weights).
void conv16_blk_fwd(Tensor X, Tensor Wp, c10::optional<Tensor> bias, Tensor Y, int64_t ks, int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Wp, "Wp", at::kBFloat16); check(Y, "Y", at::kFloat);
  check_ks(ks);
  TORCH_CHECK(X.dim() == 6 && X.size(-1) == 16, "X must be [V,I,J,K,L,16]");
  std::vector<int64_t> vs(X.sizes().begin(), X.sizes().end() - 1);
  check_shape(Y, "Y", vs);
  check_shape(Wp, "Wp", {(ks + 3) * (ks + 3), conv_pairs16(ks), 64, 8});
  if (bias.has_value()) { check(*bias, "bias", at::kFloat); TORCH_CHECK(bias->numel() == 1, "bias must have 1 element"); }
  ok(ncnet_conv16_blk_fwd(X.data_ptr(), Wp.data_ptr(), opt_ptr<float>(bias), Y.data_ptr<float>(), vs[0], vs[1], vs[2],
                          vs[3], vs[4], ks, (int)relu, 0, 0, cur_stream(X)),
     "conv16_blk_fwd");
}

// Cout = 1 layer with the in-plane taps as the MFMA rows (csrc/cout1.hip):
// Wt [ks*ks, 64, 8] (ops/packing.py cout1_taps_weights).  Returns false for a
// shape without an instantiation (nothing launched).
bool cout1_taps_fwd(Tensor X, Tensor Wt, c10::optional<Tensor> bias, Tensor Y, int64_t ks, int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Wt, "Wt", at::kBFloat16); check(Y, "Y", at::kFloat);
  check_ks(ks);
  TORCH_CHECK(X.dim() == 6 && X.size(-1) == 16, "X must be [V,I,J,K,L,16]");
  std::vector<int64_t> vs(X.sizes().begin(), X.sizes().end() - 1);
  check_shape(Y, "Y", vs);
  check_shape(Wt, "Wt", {ks * ks, 64, 8});
  if (bias.has_value()) { check(*bias, "bias", at::kFloat); TORCH_CHECK(bias->numel() == 1, "bias must have 1 element"); }
  TORCH_CHECK(vs[0] * vs[1] * vs[2] * vs[3] * vs[4] < (1LL << 40), "cout1_taps_fwd: volume too large");
  const int rc = ncnet_cout1_taps_fwd(X.data_ptr(), Wt.data_ptr(), opt_ptr<float>(bias), Y.data_ptr<float>(), vs[0],
                                      vs[1], vs[2], vs[3], vs[4], ks, (int)relu, cur_stream(X));
  if (rc == -1) return false;
  ok(rc, "cout1_taps_fwd");
  return true;
}

// bf16x3 Cout = 1 layer in output-plane-block mode: X / Xl hi / lo input blocks,
// Wp2 [2, (ks+3)^2, nq, 64, 8]; Y fp32 = act(bias + conv) accumulated over the three phases.
void conv16_blk_fwd_x3(Tensor X, Tensor Xl, Tensor Wp2, c10::optional<Tensor> bias, Tensor Y, int64_t ks,
                       int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Xl, "Xl", at::kBFloat16); check(Wp2, "Wp2", at::kBFloat16);
  check(Y, "Y", at::kFloat);
  TORCH_CHECK(ks == 3 || ks == 5, "conv16_blk_fwd_x3: kernel size 3 or 5");
  TORCH_CHECK(X.dim() == 6 && X.size(-1) == 16, "X must be [V,I,J,K,L,16]");
  TORCH_CHECK(Xl.sizes() == X.sizes(), "Xl must match X");
  std::vector<int64_t> vs(X.sizes().begin(), X.sizes().end() - 1);
  check_shape(Y, "Y", vs);
  check_shape(Wp2, "Wp2", {2, (ks + 3) * (ks + 3), conv_pairs16(ks), 64, 8});
  if (bias.has_value()) { check(*bias, "bias", at::kFloat); TORCH_CHECK(bias->numel() == 1, "bias must have 1 element"); }
  ok(ncnet_conv16_blk_fwd(X.data_ptr(), Wp2.data_ptr(), opt_ptr<float>(bias), Y.data_ptr<float>(), vs[0], vs[1],
                          vs[2], vs[3], vs[4], ks, (int)relu, 1, elem_offset(X, Xl), cur_stream(X)),
     "conv16_blk_fwd_x3");
}

// Weight gradient partials.  mode 0: all KS*KS plane offsets (di, dj); mode 2:
// plane-only (ij-encoded 1-channel layers).  variant 3 (sliding G ring, mode 0,
// KS 3/5) or 2.  part [rows = 2 * ngroups, mode ? 1 : ks*ks, ks*ks, 16, 16], partb [rows, 16].
void wgrad16(Tensor X, Tensor G, Tensor part, Tensor partb, int64_t ks, int64_t mode, int64_t variant) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(G, "G", at::kBFloat16); check(part, "part", at::kFloat); check(partb, "partb", at::kFloat);
  check_ks(ks);
  TORCH_CHECK(X.dim() == 6 && X.size(5) == 16, "X must be [V,I,J,K,L,16]");
  TORCH_CHECK(variant == 2 || variant == 3, "wgrad16 variant must be 2 or 3");
  TORCH_CHECK(mode == 0 || mode == 2, "wgrad16 mode must be 0 (full) or 2 (plane-only)");
  TORCH_CHECK(variant == 2 || (mode == 0 && (ks == 3 || ks == 5)), "wgrad16v3: full mode, ks 3 or 5");
  check_shape(G, "G", X.sizes().vec());
  const int64_t rows = part.size(0);
  TORCH_CHECK(rows > 0 && rows % 2 == 0, "wgrad16 needs an even number of partial rows");
  check_shape(part, "part", {rows, mode == 2 ? 1 : ks * ks, ks * ks, 16, 16});
  check_shape(partb, "partb", {rows, 16});
  if (variant == 3) {
    ok(ncnet_wgrad16v3(X.data_ptr(), G.data_ptr(), (float*)part.data_ptr(), (float*)partb.data_ptr(), X.size(0),
                       X.size(1), X.size(2), X.size(3), X.size(4), ks, rows / 2, cur_stream(X)),
       "wgrad16v3");
    return;
  }
  ok(ncnet_wgrad16(X.data_ptr(), G.data_ptr(), (float*)part.data_ptr(), (float*)partb.data_ptr(), X.size(0), X.size(1),
                   X.size(2), X.size(3), X.size(4), ks, rows / 2, (int)mode, cur_stream(X)), "wgrad16");
}

// Plane-only weight gradient of the ij-encoded layers (whole-plane tiles, K, L <= 25):
// X [nsets,V,I,J,K,L,16], G [ngg,V,I,J,K,L,16]; part [rows, nsets*ngg, ks*ks, 16, 16],
// partb [rows, nsets*ngg, 16] (rows = 2 * workgroup groups); nsets * ngg <= 2.
void wgrad16p(Tensor X, Tensor G, Tensor part, Tensor partb, int64_t ks) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(G, "G", at::kBFloat16); check(part, "part", at::kFloat); check(partb, "partb", at::kFloat);
  check_ks(ks);
  TORCH_CHECK(X.dim() == 7 && G.dim() == 7 && X.size(6) == 16, "X, G must be [n,V,I,J,K,L,16]");
  const int64_t nsets = X.size(0), ngg = G.size(0);
  TORCH_CHECK(nsets * ngg <= 2 && nsets >= 1 && ngg >= 1, "wgrad16p: nsets * ngg must be 1 or 2");
  TORCH_CHECK(X.sizes().slice(1).vec() == G.sizes().slice(1).vec(), "wgrad16p: X and G volumes differ");
  const int64_t rows = part.size(0);
  TORCH_CHECK(rows > 0 && rows % 2 == 0, "wgrad16p needs an even number of partial rows");
  check_shape(part, "part", {rows, nsets * ngg, ks * ks, 16, 16});
  check_shape(partb, "partb", {rows, nsets * ngg, 16});
  const int64_t vol = X[0].numel();
  ok(ncnet_wgrad16p(X.data_ptr(), G.data_ptr(), (float*)part.data_ptr(), (float*)partb.data_ptr(), X.size(1), X.size(2),
                    X.size(3), X.size(4), X.size(5), ks, rows / 2, (int)nsets, (int)ngg, vol, vol, cur_stream(X)),
     "wgrad16p");
}

// X [V,I,J,K,L] (bf16/fp32) -> S [G,V,I,J,K,L,16] bf16 (ij encoding, G = ceil(ks*ks/16))
void ijpack(Tensor X, Tensor S, int64_t ks, int64_t sgn) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  TORCH_CHECK(X.is_cuda() && X.is_contiguous() && (X.scalar_type() == at::kBFloat16 || X.scalar_type() == at::kFloat));
  TORCH_CHECK(X.dim() == 5, "X must be [V,I,J,K,L]");
  check_ks(ks);
  TORCH_CHECK(sgn == 1 || sgn == -1);
  const bool f8 = S.scalar_type() == at::kFloat8_e4m3fn;   // fp8 inference path
  check(S, "S", f8 ? at::kFloat8_e4m3fn : at::kBFloat16);
  check_shape(S, "S", {(ks * ks + 15) / 16, X.size(0), X.size(1), X.size(2), X.size(3), X.size(4), 16});
  ok(ncnet_ijpack(X.data_ptr(), X.scalar_type() == at::kBFloat16, S.data_ptr(), X.size(0), X.size(1), X.size(2),
                  X.size(3), X.size(4), ks, sgn, f8 ? 1 : 0, cur_stream(X)), "ijpack");
}

// Z [ks*ks,V,I,J,K,L] fp32 (channel-planar by combo q = di*ks + dj) -> y [V,I,J,K,L] fp32 (ij encoding)
void ijsum(Tensor Z, c10::optional<Tensor> bias, Tensor y, int64_t ks, int64_t relu, int64_t sgn) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(Z.device());
  check(Z, "Z", at::kFloat); check(y, "y", at::kFloat);
  check_ks(ks);
  TORCH_CHECK(sgn == 1 || sgn == -1);
  TORCH_CHECK(Z.dim() == 6 && Z.size(0) == ks * ks, "Z must be [ks*ks,V,I,J,K,L]");
  check_shape(y, "y", {Z.size(1), Z.size(2), Z.size(3), Z.size(4), Z.size(5)});
  if (bias.has_value()) { check(*bias, "bias", at::kFloat); check_shape(*bias, "bias", {1}); }
  ok(ncnet_ijsum((float*)Z.data_ptr(), opt_ptr<float>(bias), (float*)y.data_ptr(), Z.size(1), Z.size(2), Z.size(3),
                 Z.size(4), Z.size(5), ks, relu ? 1 : 0, (int)sgn, cur_stream(Z)), "ijsum");
}

// y: bf16, IEEE half, or OCP fp8 e4m3 holding fp8_scale * x / ||x|| (fp8_scale > 0);
// y_lo (bf16 y only): the rounding residual bf16(x / ||x|| - y) (bf16x3 mode)
void l2norm_rows(Tensor x, Tensor y, c10::optional<Tensor> inv, double fp8_scale, c10::optional<Tensor> y_lo) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.is_cuda() && x.is_contiguous());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat);
  const bool f8 = y.scalar_type() == at::kFloat8_e4m3fn, h = y.scalar_type() == at::kHalf;
  check(y, "y", f8 ? at::kFloat8_e4m3fn : h ? at::kHalf : at::kBFloat16);
  TORCH_CHECK(!f8 || fp8_scale > 0, "fp8 output needs fp8_scale > 0");
  TORCH_CHECK(x.dim() == 2 && y.sizes() == x.sizes(), "x,y must be [rows, C]");
  if (inv.has_value()) { check(*inv, "inv", at::kFloat); check_shape(*inv, "inv", {x.size(0)}); }
  if (y_lo.has_value()) {
    TORCH_CHECK(!f8 && !h, "l2norm_rows: y_lo needs bf16 y");
    check(*y_lo, "y_lo", at::kBFloat16); check_shape(*y_lo, "y_lo", y.sizes().vec());
  }
  ok(ncnet_l2norm_rows(x.data_ptr(), x.scalar_type() == at::kBFloat16, y.data_ptr(),
                       inv.has_value() ? (float*)inv->data_ptr() : nullptr, x.size(0), x.size(1),
                       f8 ? (float)fp8_scale : 0.f, y_lo.has_value() ? y_lo->data_ptr() : nullptr, h ? 1 : 0,
                       cur_stream(x)),
     "l2norm");
}

void l2norm_rows_bwd(Tensor x, Tensor g, Tensor inv, Tensor gx) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check(x, "x", at::kFloat); check(g, "g", at::kFloat); check(inv, "inv", at::kFloat); check(gx, "gx", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && g.sizes() == x.sizes() && gx.sizes() == x.sizes());
  check_shape(inv, "inv", {x.size(0)});
  ok(ncnet_l2norm_rows_bwd((float*)x.data_ptr(), (float*)g.data_ptr(), (float*)inv.data_ptr(), (float*)gx.data_ptr(),
                           x.size(0), x.size(1), cur_stream(x)), "l2norm_bwd");
}

// A [Ba, M, K], B [Bb, N, K] bf16 or IEEE half (or both OCP fp8 e4m3: C = out_scale * A.B^T);
// C [batch, M, N] fp32, or 16-bit of the operands' type (bf16 for fp8 operands)
void corr_gemm(Tensor A, Tensor B, Tensor C, c10::optional<Tensor> amap, c10::optional<Tensor> bmap,
               double out_scale) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const bool f8 = A.scalar_type() == at::kFloat8_e4m3fn, h = A.scalar_type() == at::kHalf;
  const auto dt = f8 ? at::kFloat8_e4m3fn : h ? at::kHalf : at::kBFloat16;
  check(A, "A", dt); check(B, "B", dt);
  TORCH_CHECK(!f8 || A.size(2) % 16 == 0, "fp8 K must be a multiple of 16");
  const auto c16 = h ? at::kHalf : at::kBFloat16;
  TORCH_CHECK(C.is_cuda() && C.is_contiguous() && (C.scalar_type() == at::kFloat || C.scalar_type() == c16),
              "corr_gemm: C must be fp32 or the operands' 16-bit type");
  TORCH_CHECK(A.dim() == 3 && B.dim() == 3 && C.dim() == 3);
  TORCH_CHECK(A.size(2) == B.size(2), "K mismatch");
  TORCH_CHECK(A.size(2) % 8 == 0, "K must be a multiple of 8");
  const int64_t batch = C.size(0);
  TORCH_CHECK(C.size(1) == A.size(1) && C.size(2) == B.size(1), "C shape mismatch");
  if (amap.has_value()) {
    // maps are built by ncnet_amd.ops.correlation from arange/roll (in range by
    // construction); no device->host read here, the call stays async.
    check(*amap, "amap", at::kInt); check_shape(*amap, "amap", {batch});
  } else TORCH_CHECK(A.size(0) == batch);
  if (bmap.has_value()) {
    check(*bmap, "bmap", at::kInt); check_shape(*bmap, "bmap", {batch});
  } else TORCH_CHECK(B.size(0) == batch);
  ok(ncnet_corr_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), opt_ptr<int>(amap), opt_ptr<int>(bmap), batch, A.size(1),
                     B.size(1), A.size(2), A.size(1) * A.size(2), B.size(1) * B.size(2), C.size(1) * C.size(2),
                     C.scalar_type() != at::kFloat, f8 ? (float)out_scale : 0.f, h ? 1 : 0, cur_stream(A)),
     "corr_gemm");
}

void corr_gemm_pool2(Tensor A, Tensor B, Tensor val, Tensor idx, int64_t hA, int64_t wA, int64_t hB, int64_t wB,
                     double out_scale) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const bool f8 = A.scalar_type() == at::kFloat8_e4m3fn, h = A.scalar_type() == at::kHalf;
  const auto dt = f8 ? at::kFloat8_e4m3fn : h ? at::kHalf : at::kBFloat16;
  check(A, "A", dt); check(B, "B", dt);
  check(val, "val", at::kFloat); check(idx, "idx", at::kByte);
  TORCH_CHECK(!f8 || A.size(2) % 16 == 0, "fp8 K must be a multiple of 16");
  TORCH_CHECK(A.dim() == 3 && B.dim() == 3 && A.size(0) == B.size(0));
  TORCH_CHECK(A.size(1) == hA * wA && B.size(1) == hB * wB && A.size(2) == B.size(2));
  TORCH_CHECK(hA % 2 == 0 && wA % 2 == 0 && hB % 2 == 0 && wB % 2 == 0, "pooling needs even feature sizes");
  TORCH_CHECK(A.size(2) % 8 == 0);
  check_shape(val, "val", {A.size(0), hA / 2, wA / 2, hB / 2, wB / 2});
  check_shape(idx, "idx", {A.size(0), hA / 2, wA / 2, hB / 2, wB / 2});
  ok(ncnet_corr_gemm_pool2(A.data_ptr(), B.data_ptr(), (float*)val.data_ptr(), (uint8_t*)idx.data_ptr(), A.size(0), hA,
                           wA, hB, wB, A.size(2), A.size(1) * A.size(2), B.size(1) * B.size(2),
                           f8 ? (float)out_scale : 0.f, h ? 1 : 0, cur_stream(A)),
     "corr_gemm_pool2");
}

// x [V,R,C] fp32 -> per-row (dim 2) stats [V,R]: max, first argmax, and se =
// sum exp(x - max) (sum_kind 1) or the plain sum (sum_kind 2)
void stats_rows(Tensor x, Tensor mx, c10::optional<Tensor> arg, c10::optional<Tensor> se, int64_t sum_kind) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check(x, "x", at::kFloat); check(mx, "mx", at::kFloat);
  TORCH_CHECK(x.dim() == 3);
  check_shape(mx, "mx", {x.size(0), x.size(1)});
  if (arg.has_value()) { check(*arg, "arg", at::kInt); check_shape(*arg, "arg", {x.size(0), x.size(1)}); }
  if (se.has_value()) { check(*se, "se", at::kFloat); check_shape(*se, "se", {x.size(0), x.size(1)}); }
  ok(ncnet_stats_rows((float*)x.data_ptr(), (float*)mx.data_ptr(), arg.has_value() ? (int*)arg->data_ptr() : nullptr,
                      se.has_value() ? (float*)se->data_ptr() : nullptr, x.size(0) * x.size(1), x.size(2),
                      (int)sum_kind, cur_stream(x)),
     "stats_rows");
}

// x [V,R,C] fp32 -> per-column (dim 1) stats [V,C] (sum_kind as stats_rows)
void stats_cols(Tensor x, Tensor mx, c10::optional<Tensor> arg, c10::optional<Tensor> se, int64_t sum_kind) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check(x, "x", at::kFloat); check(mx, "mx", at::kFloat);
  TORCH_CHECK(x.dim() == 3);
  check_shape(mx, "mx", {x.size(0), x.size(2)});
  if (arg.has_value()) { check(*arg, "arg", at::kInt); check_shape(*arg, "arg", {x.size(0), x.size(2)}); }
  if (se.has_value()) { check(*se, "se", at::kFloat); check_shape(*se, "se", {x.size(0), x.size(2)}); }
  // few wide columns (InLoc volumes): split the rows over chunks so the grid fills the chip
  const int64_t V = x.size(0), R = x.size(1), C = x.size(2);
  const int64_t blocks = V * ((C + 63) / 64);
  int64_t nchunk = 1;
  if (blocks < 1024) nchunk = std::min<int64_t>((2048 + blocks - 1) / blocks, (R + 63) / 64);
  Tensor work;
  if (nchunk > 1) work = at::empty({3 * V * nchunk * C}, x.options());
  ok(ncnet_stats_cols((float*)x.data_ptr(), (float*)mx.data_ptr(), arg.has_value() ? (int*)arg->data_ptr() : nullptr,
                      se.has_value() ? (float*)se->data_ptr() : nullptr, V, R, C,
                      nchunk > 1 ? (float*)work.data_ptr() : nullptr, (int)nchunk, (int)sum_kind, cur_stream(x)),
     "stats_cols");
}

// x [V,R,C] fp32 -> row stats [V,R] and column stats [V,C] in one pass
// (stats_rows + stats_cols); always true (kept boolean for the callers' fallbacks).
bool stats2d(Tensor x, Tensor rmx, Tensor rarg, c10::optional<Tensor> rse, Tensor cmx, Tensor carg,
             c10::optional<Tensor> cse, int64_t sum_kind) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 3);
  const int64_t V = x.size(0), R = x.size(1), C = x.size(2);
  check(rmx, "rmx", at::kFloat); check_shape(rmx, "rmx", {V, R});
  check(rarg, "rarg", at::kInt); check_shape(rarg, "rarg", {V, R});
  check(cmx, "cmx", at::kFloat); check_shape(cmx, "cmx", {V, C});
  check(carg, "carg", at::kInt); check_shape(carg, "carg", {V, C});
  if (sum_kind) {
    TORCH_CHECK(rse.has_value() && cse.has_value(), "stats2d: sum_kind needs rse and cse");
    check(*rse, "rse", at::kFloat); check_shape(*rse, "rse", {V, R});
    check(*cse, "cse", at::kFloat); check_shape(*cse, "cse", {V, C});
  }
  const int64_t nrt = (R + 63) / 64, nct = (C + 255) / 256;
  Tensor work = at::empty({3 * V * (nct * R + nrt * C)}, x.options());
  ok(ncnet_stats2d((float*)x.data_ptr(), (float*)rmx.data_ptr(), (int*)rarg.data_ptr(),
                   sum_kind ? (float*)rse->data_ptr() : nullptr, (float*)cmx.data_ptr(), (int*)carg.data_ptr(),
                   sum_kind ? (float*)cse->data_ptr() : nullptr, (int)V, (int)R, (int)C, (float*)work.data_ptr(),
                   (int)sum_kind, cur_stream(x)),
     "stats2d");
  return true;
}

// one volume's bidirectional match candidates from its column (B cells) and
// row (A cells) stats: m [N,5] fp32, sc [N] fp32, key [N] int64, N = R + C;
// code: packed 2-bit offsets uint8 [R*C] (k = 2) or none
void match_candidates(Tensor cmx, c10::optional<Tensor> cse, Tensor carg, Tensor rmx, c10::optional<Tensor> rse,
                      Tensor rarg, c10::optional<Tensor> code, int64_t fs1, int64_t fs2, int64_t fs3, int64_t fs4,
                      int64_t k, Tensor m, Tensor sc, Tensor key) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(cmx.device());
  const int64_t R = fs1 * fs2, C = fs3 * fs4;
  check(cmx, "cmx", at::kFloat); check_shape(cmx, "cmx", {C});
  check(carg, "carg", at::kInt); check_shape(carg, "carg", {C});
  check(rmx, "rmx", at::kFloat); check_shape(rmx, "rmx", {R});
  check(rarg, "rarg", at::kInt); check_shape(rarg, "rarg", {R});
  TORCH_CHECK(cse.has_value() == rse.has_value(), "match_candidates: both or neither softmax sums");
  if (cse.has_value()) { check(*cse, "cse", at::kFloat); check_shape(*cse, "cse", {C}); check(*rse, "rse", at::kFloat); check_shape(*rse, "rse", {R}); }
  if (code.has_value()) { check(*code, "code", at::kByte); TORCH_CHECK(code->numel() == R * C, "match_candidates: code size"); }
  check(m, "m", at::kFloat); check_shape(m, "m", {R + C, 5});
  check(sc, "sc", at::kFloat); check_shape(sc, "sc", {R + C});
  check(key, "key", at::kLong); check_shape(key, "key", {R + C});
  ok(ncnet_match_candidates((float*)cmx.data_ptr(), cse.has_value() ? (float*)cse->data_ptr() : nullptr,
                            (int*)carg.data_ptr(), (float*)rmx.data_ptr(), rse.has_value() ? (float*)rse->data_ptr() : nullptr,
                            (int*)rarg.data_ptr(), code.has_value() ? (uint8_t*)code->data_ptr() : nullptr, (int)fs1,
                            (int)fs2, (int)fs3, (int)fs4, (int)k, (float*)m.data_ptr(), (float*)sc.data_ptr(),
                            (long long*)key.data_ptr(), cur_stream(cmx)),
     "match_candidates");
}

// out[i] = bf16(src[idx[i]]) (0 where idx < 0): src fp32 [N], idx int32 [M], out bf16 [M]
void gather_bf16(Tensor src, Tensor idx, Tensor out) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  check(src, "src", at::kFloat); check(idx, "idx", at::kInt); check(out, "out", at::kBFloat16);
  TORCH_CHECK(idx.numel() == out.numel(), "gather_bf16: idx / out size");
  ok(ncnet_gather_bf16((float*)src.data_ptr(), (int*)idx.data_ptr(), out.data_ptr(), out.numel(), src.numel(),
                      cur_stream(src)),
     "gather_bf16");
}

// segments (src fp32 [R, N] contiguous, dst fp32, idx int32 [N] or None): dst[idx[j]] =
// sum_r src[r, j] (idx None: dst[j]); <= 4 segments, one launch, deterministic order
void reduce_cols(std::vector<Tensor> src, std::vector<Tensor> dst, std::vector<c10::optional<Tensor>> idx) {
  const int n = (int)src.size();
  TORCH_CHECK(n >= 1 && n <= 4 && (int)dst.size() == n && (int)idx.size() == n, "reduce_cols: 1..4 segments");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src[0].device());
  const float* s[4]; float* d[4]; const int* ix[4]; int R[4], N[4]; long long nd[4];
  for (int k = 0; k < n; ++k) {
    check(src[k], "src", at::kFloat); check(dst[k], "dst", at::kFloat);
    TORCH_CHECK(src[k].dim() == 2, "reduce_cols: src [R, N]");
    TORCH_CHECK(src[k].device() == src[0].device() && dst[k].device() == src[0].device(), "reduce_cols: one device");
    R[k] = (int)src[k].size(0); N[k] = (int)src[k].size(1);
    s[k] = (const float*)src[k].data_ptr(); d[k] = (float*)dst[k].data_ptr(); nd[k] = dst[k].numel();
    if (idx[k].has_value()) {
      check(*idx[k], "idx", at::kInt);
      TORCH_CHECK(idx[k]->numel() == N[k], "reduce_cols: idx [N]");
      ix[k] = (const int*)idx[k]->data_ptr();
    } else {
      TORCH_CHECK(nd[k] >= N[k], "reduce_cols: dst smaller than N");
      ix[k] = nullptr;
    }
  }
  ok(ncnet_reduce_cols(s, d, ix, R, N, nd, n, cur_stream(src[0])), "reduce_cols");
}

// pad (ks, I2, J2): out_x / out_xt are the zero-padded bf16 planes of csrc/conv1x.hip ([V*R, PPL] /
// [V*C, PPL], halos written too) of a square volume R = C = I2 * J2; else [V,R,C] / [V,C,R] bf16 or f16.
void mm_apply(Tensor c, Tensor rmax, Tensor cmax, c10::optional<Tensor> out, c10::optional<Tensor> out_x,
              c10::optional<Tensor> out_xt, double eps, std::vector<int64_t> pad) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c.device());
  check(c, "c", at::kFloat); check(rmax, "rmax", at::kFloat); check(cmax, "cmax", at::kFloat);
  TORCH_CHECK(c.dim() == 3);
  const int64_t V = c.size(0), R = c.size(1), C = c.size(2);
  check_shape(rmax, "rmax", {V, R}); check_shape(cmax, "cmax", {V, C});
  if (out.has_value()) { check(*out, "out", at::kFloat); check_shape(*out, "out", {V, R, C}); }
  // out_x / out_xt: bf16 or IEEE half (both the same)
  const bool h = (out_x.has_value() && out_x->scalar_type() == at::kHalf) ||
                 (out_xt.has_value() && out_xt->scalar_type() == at::kHalf);
  const auto xt = h ? at::kHalf : at::kBFloat16;
  int64_t pks = 0, I2 = 0, J2 = 0;
  if (!pad.empty()) {
    TORCH_CHECK(pad.size() == 3, "mm_apply: pad = (ks, I2, J2)");
    pks = pad[0]; I2 = pad[1]; J2 = pad[2];
    check_ks(pks);
    TORCH_CHECK(!h && I2 * J2 == R && R == C, "mm_apply pad: bf16 planes of a square volume, I2 * J2 = R = C");
    const auto g = pad_geom(I2, J2, pks);
    if (out_x.has_value()) { check(*out_x, "out_x", xt); check_shape(*out_x, "out_x", {V * R, g[1]}); }
    if (out_xt.has_value()) { check(*out_xt, "out_xt", xt); check_shape(*out_xt, "out_xt", {V * C, g[1]}); }
  } else {
    if (out_x.has_value()) { check(*out_x, "out_x", xt); check_shape(*out_x, "out_x", {V, R, C}); }
    if (out_xt.has_value()) { check(*out_xt, "out_xt", xt); check_shape(*out_xt, "out_xt", {V, C, R}); }
  }
  ok(ncnet_mm_apply((float*)c.data_ptr(), (float*)rmax.data_ptr(), (float*)cmax.data_ptr(),
                    out.has_value() ? (float*)out->data_ptr() : nullptr, out_x.has_value() ? out_x->data_ptr() : nullptr,
                    out_xt.has_value() ? out_xt->data_ptr() : nullptr, V, R, C, (float)eps, h ? 1 : 0, (int)pks,
                    (int)I2, (int)J2, (int)I2, (int)J2, cur_stream(c)),
     "mm_apply");
}

// one_pass: both sums of the backward in one pass over (c, g) (default), else the separate row / column passes
void mm_bwd(Tensor c, Tensor g, Tensor rmax, Tensor rarg, Tensor cmax, Tensor carg, Tensor gc, double eps,
            bool one_pass) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c.device());
  check(c, "c", at::kFloat); check(g, "g", at::kFloat); check(gc, "gc", at::kFloat);
  check(rmax, "rmax", at::kFloat); check(cmax, "cmax", at::kFloat); check(rarg, "rarg", at::kInt); check(carg, "carg", at::kInt);
  TORCH_CHECK(c.dim() == 3 && g.sizes() == c.sizes() && gc.sizes() == c.sizes());
  const int64_t V = c.size(0), R = c.size(1), C = c.size(2);
  check_shape(rmax, "rmax", {V, R}); check_shape(rarg, "rarg", {V, R});
  check_shape(cmax, "cmax", {V, C}); check_shape(carg, "carg", {V, C});
  auto rsum = torch::empty({V, R}, c.options());
  auto csum = torch::empty({V, C}, c.options());
  Tensor work;
  if (one_pass) work = torch::empty({V * (((C + 255) / 256) * R + ((R + 63) / 64) * C)}, c.options());
  ok(ncnet_mm_bwd((float*)c.data_ptr(), (float*)g.data_ptr(), (float*)rmax.data_ptr(), (int*)rarg.data_ptr(),
                  (float*)cmax.data_ptr(), (int*)carg.data_ptr(), (float*)rsum.data_ptr(), (float*)csum.data_ptr(),
                  (float*)gc.data_ptr(), V, R, C, (float)eps, one_pass ? (float*)work.data_ptr() : nullptr,
                  cur_stream(c)), "mm_bwd");
}

// z [2*Vh, R, C] (second half stored as [C, R]) -> y [Vh, R, C]
void combine_fwd(Tensor z, Tensor y, int64_t R, int64_t C) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(z.device());
  check(z, "z", at::kFloat); check(y, "y", at::kFloat);
  TORCH_CHECK(z.numel() % (2 * R * C) == 0);
  const int64_t Vh = z.numel() / (2 * R * C);
  TORCH_CHECK(y.numel() == Vh * R * C);
  ok(ncnet_combine_fwd((float*)z.data_ptr(), (float*)y.data_ptr(), Vh, R, C, cur_stream(z)), "combine_fwd");
}

void combine_bwd(Tensor g, Tensor z, Tensor gz, int64_t R, int64_t C, c10::optional<Tensor> gzl) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(z.device());
  check(g, "g", at::kFloat); check(z, "z", at::kFloat); check(gz, "gz", at::kBFloat16);
  TORCH_CHECK(z.numel() % (2 * R * C) == 0);
  TORCH_CHECK(gz.numel() == z.numel() && g.numel() * 2 == z.numel(), "combine_bwd: size mismatch");
  if (gzl.has_value()) { check(*gzl, "gzl", at::kBFloat16); TORCH_CHECK(gzl->numel() == z.numel()); }
  const int Vh = (int)(z.numel() / (2 * R * C));
  ok(ncnet_combine_bwd((float*)g.data_ptr(), (float*)z.data_ptr(), gz.data_ptr(), const_cast<void*>(opt_ptr<void>(gzl)), Vh, R, C,
                       cur_stream(z)),
     "combine_bwd");
}

// norm: 1 'softmax', 2 'l1' (eps), 0 None -- rse / cse from stats with the matching sum_kind
void softmax_max_bwd(Tensor x, Tensor rmax, Tensor rarg, Tensor rse, Tensor cmax, Tensor carg, Tensor cse, Tensor wr,
                     Tensor wc, Tensor gx, int64_t norm, double eps, c10::optional<Tensor> gscale) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check(x, "x", at::kFloat); check(gx, "gx", at::kFloat);
  TORCH_CHECK(x.dim() == 3 && gx.sizes() == x.sizes());
  TORCH_CHECK(norm >= 0 && norm <= 2, "softmax_max_bwd: norm must be 0 (None), 1 (softmax) or 2 (l1)");
  const int64_t V = x.size(0), R = x.size(1), C = x.size(2);
  check(rmax, "rmax", at::kFloat); check(rse, "rse", at::kFloat); check(rarg, "rarg", at::kInt);
  check(cmax, "cmax", at::kFloat); check(cse, "cse", at::kFloat); check(carg, "carg", at::kInt);
  check(wr, "wr", at::kFloat); check(wc, "wc", at::kFloat);
  check_shape(rmax, "rmax", {V, R}); check_shape(rse, "rse", {V, R}); check_shape(rarg, "rarg", {V, R});
  check_shape(cmax, "cmax", {V, C}); check_shape(cse, "cse", {V, C}); check_shape(carg, "carg", {V, C});
  check_shape(wr, "wr", {V}); check_shape(wc, "wc", {V});
  if (gscale.has_value()) { check(*gscale, "gscale", at::kFloat); TORCH_CHECK(gscale->numel() == 1, "gscale: one element"); }
  ok(ncnet_softmax_max_bwd((float*)x.data_ptr(), (float*)rmax.data_ptr(), (int*)rarg.data_ptr(), (float*)rse.data_ptr(),
                           (float*)cmax.data_ptr(), (int*)carg.data_ptr(), (float*)cse.data_ptr(), (float*)wr.data_ptr(),
                           (float*)wc.data_ptr(), (float*)gx.data_ptr(), V, R, C, (int)norm, (float)eps,
                           opt_ptr<float>(gscale), cur_stream(x)), "softmax_max_bwd");
}

// weak-loss score value out [] fp32 from the row / column stats (rse / cse: the sums of `norm`)
void score_sum(Tensor rmax, Tensor rse, Tensor cmax, Tensor cse, Tensor wr, Tensor wc, Tensor out, int64_t norm,
               double eps) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(rmax.device());
  for (auto* t : {&rmax, &rse, &cmax, &cse, &wr, &wc, &out}) check(*t, "score_sum operand", at::kFloat);
  TORCH_CHECK(norm >= 0 && norm <= 2, "score_sum: norm must be 0, 1 or 2");
  TORCH_CHECK(rmax.dim() == 2 && cmax.dim() == 2 && rmax.size(0) == cmax.size(0), "score_sum: [V, R] / [V, C] stats");
  const int64_t V = rmax.size(0), R = rmax.size(1), C = cmax.size(1);
  check_shape(rse, "rse", {V, R}); check_shape(cse, "cse", {V, C});
  check_shape(wr, "wr", {V}); check_shape(wc, "wc", {V});
  TORCH_CHECK(out.numel() == 1, "score_sum: out must have one element");
  ok(ncnet_score_sum((float*)rmax.data_ptr(), (float*)rse.data_ptr(), (float*)cmax.data_ptr(), (float*)cse.data_ptr(),
                     (float*)wr.data_ptr(), (float*)wc.data_ptr(), (int)V, (int)R, (int)C, (int)norm, (float)eps,
                     (float*)out.data_ptr(), cur_stream(rmax)), "score_sum");
}

void maxpool4d(Tensor x, Tensor y, Tensor code, int64_t ks) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16));
  TORCH_CHECK(x.dim() == 5, "x must be [V,I,J,K,L]");
  TORCH_CHECK(ks >= 1 && ks <= 4);
  for (int d = 1; d < 5; ++d) TORCH_CHECK(x.size(d) % ks == 0, "volume dims must be divisible by k_size");
  std::vector<int64_t> os = {x.size(0), x.size(1) / ks, x.size(2) / ks, x.size(3) / ks, x.size(4) / ks};
  check(y, "y", at::kFloat); check(code, "code", at::kByte);
  check_shape(y, "y", os); check_shape(code, "code", os);
  ok(ncnet_maxpool4d(x.data_ptr(), x.scalar_type() == at::kBFloat16, (float*)y.data_ptr(), (uint8_t*)code.data_ptr(),
                     x.size(0), x.size(1), x.size(2), x.size(3), x.size(4), ks, cur_stream(x)), "maxpool4d");
}

void transpose(Tensor x, Tensor y) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && y.is_contiguous() && x.scalar_type() == y.scalar_type());
  TORCH_CHECK(x.dim() == 3 && y.dim() == 3 && y.size(0) == x.size(0) && y.size(1) == x.size(2) && y.size(2) == x.size(1));
  ok(ncnet_transpose(x.data_ptr(), y.data_ptr(), x.element_size(), x.size(0), x.size(1), x.size(2), cur_stream(x)),
     "transpose");
}

}  // namespace

// In place Y = act(Y + b) over the channel axis: Y bf16, either a contiguous
// [rows, C] matrix or a channels-last [N, C, H, W] tensor; b fp32 [C].
// Y = act(maxpool_{k,stride,pad}(X) + b): X, Y channels-last [N, C, H, W] /
// [N, C, Ho, Wo] bf16 or fp16 (same dtype), b fp32 [C], C % 8 == 0.
void maxpool_bias_act(Tensor X, Tensor b, Tensor Y, int64_t k, int64_t stride, int64_t pad, int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  TORCH_CHECK(X.is_cuda() && X.dim() == 4 && X.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  (X.scalar_type() == at::kBFloat16 || X.scalar_type() == at::kHalf),
              "maxpool_bias_act: X must be a channels-last bf16 / fp16 [N, C, H, W] GPU tensor");
  TORCH_CHECK(Y.is_cuda() && Y.dim() == 4 && Y.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  Y.scalar_type() == X.scalar_type(), "maxpool_bias_act: Y must be channels-last like X");
  check(b, "b", at::kFloat);
  const int64_t N = X.size(0), C = X.size(1), H = X.size(2), W = X.size(3);
  TORCH_CHECK(k >= 1 && stride >= 1 && pad >= 0 && 2 * pad <= k, "maxpool_bias_act: bad window");
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  check_shape(Y, "Y", {N, C, Ho, Wo});
  check_shape(b, "b", {C});
  TORCH_CHECK(C % 8 == 0, "maxpool_bias_act: C must be a multiple of 8");
  ok(ncnet_maxpool_bias_act(X.data_ptr(), Y.data_ptr(), (const float*)b.data_ptr(), (int)N, (int)H, (int)W, (int)C,
                            (int)Ho, (int)Wo, (int)k, (int)stride, (int)pad, relu ? 1 : 0,
                            X.scalar_type() == at::kHalf ? 1 : 0, cur_stream(X)),
     "maxpool_bias_act");
}

void bias_act_(Tensor Y, Tensor b, int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(Y.device());
  TORCH_CHECK(Y.is_cuda() && (Y.scalar_type() == at::kBFloat16 || Y.scalar_type() == at::kHalf),
              "bias_act_: Y must be a bf16 / fp16 GPU tensor");
  int64_t C;
  if (Y.dim() == 4) {
    TORCH_CHECK(Y.is_contiguous(at::MemoryFormat::ChannelsLast), "bias_act_: 4-D Y must be channels-last");
    C = Y.size(1);
  } else {
    TORCH_CHECK(Y.dim() == 2 && Y.is_contiguous(), "bias_act_: Y must be [rows, C] contiguous");
    C = Y.size(1);
  }
  check(b, "b", at::kFloat);
  check_shape(b, "b", {C});
  TORCH_CHECK(C % 8 == 0, "bias_act_: C must be a multiple of 8");
  ok(ncnet_bias_act(Y.data_ptr(), (const float*)b.data_ptr(), Y.numel() / C, (int)C, relu ? 1 : 0,
                    Y.scalar_type() == at::kHalf ? 1 : 0, cur_stream(Y)),
     "bias_act_");
}

// fp8 inference Conv4d 16->16: X fp8 [V,I,J,K,L,16] or [G,V,I,J,K,L,16] (group planes),
// Wp fp8 [planes, ceil(ks*ks/2), 64, 8] (weights * wscale), oscale = 1 / wscale.
// epi 1: Y fp8 [V,I,J,K,L,16] = relu(oscale * acc + bias); epi 4: Y fp32 planar [nco, V,I,J,K,L].
void conv16f8_fwd(Tensor X, Tensor Wp, c10::optional<Tensor> bias, Tensor Y, int64_t ks, int64_t epi, double oscale) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kFloat8_e4m3fn); check(Wp, "Wp", at::kFloat8_e4m3fn);
  check_ks(ks);
  const bool grp = X.dim() == 7;
  TORCH_CHECK((X.dim() == 6 || grp) && X.size(-1) == 16, "X must be [V,I,J,K,L,16] or [G,V,I,J,K,L,16]");
  const int64_t npg = grp ? X.size(0) : 0;
  std::vector<int64_t> vs(X.sizes().begin() + (grp ? 1 : 0), X.sizes().end());
  TORCH_CHECK(epi == 1 || epi == 4, "fp8 conv supports epi 1 (bias+ReLU -> fp8) and 4 (planar fp32)");
  int64_t nco = 16;
  if (epi == 4) {
    check(Y, "Y", at::kFloat);
    nco = Y.size(0);
    TORCH_CHECK(nco >= 1 && nco <= 16);
    check_shape(Y, "Y", {nco, vs[0], vs[1], vs[2], vs[3], vs[4]});
  } else {
    check(Y, "Y", at::kFloat8_e4m3fn);
    check_shape(Y, "Y", vs);
    TORCH_CHECK(bias.has_value()); check(*bias, "bias", at::kFloat); check_shape(*bias, "bias", {16});
  }
  check_shape(Wp, "Wp", {grp ? npg : ks * ks, conv_pairs16(ks), 64, 8});
  ok(ncnet_conv16f8_fwd(X.data_ptr(), Wp.data_ptr(), opt_ptr<float>(bias), Y.data_ptr(), vs[0], vs[1], vs[2], vs[3],
                        vs[4], ks, epi, (int)npg, (int)nco, (float)oscale, cur_stream(X)),
     "conv16f8_fwd");
}

// Fused NC (1 -> 16 -> 1, k = 3): X bf16 or IEEE half [V,I,J,K,L] -> Y fp32 [V,I,J,K,L];
// W1p / W2p [5, 64, 8] of X's type; b1 [16], b2 [1] fp32; tile (TK, TL), R planes and IR rows per workgroup.
void nc_fused_k3(Tensor X, Tensor W1p, Tensor b1, Tensor W2p, Tensor b2, Tensor Y, int64_t R, int64_t IR, int64_t TK,
                 int64_t TL) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  const bool h = X.scalar_type() == at::kHalf;
  const auto dt = h ? at::kHalf : at::kBFloat16;
  check(X, "X", dt); check(W1p, "W1p", dt); check(W2p, "W2p", dt);
  check(b1, "b1", at::kFloat); check(b2, "b2", at::kFloat); check(Y, "Y", at::kFloat);
  TORCH_CHECK(X.dim() == 5, "X must be [V,I,J,K,L]");
  check_shape(Y, "Y", X.sizes().vec());
  check_shape(W1p, "W1p", {5, 64, 8}); check_shape(W2p, "W2p", {5, 64, 8});
  check_shape(b1, "b1", {16}); check_shape(b2, "b2", {1});
  TORCH_CHECK(R >= 1 && IR >= 1 && TK >= 1 && TL >= 1, "nc_fused_k3: bad tiling");
  ok(ncnet_nc_fused_k3(X.data_ptr(), W1p.data_ptr(), (const float*)b1.data_ptr(), W2p.data_ptr(),
                       (const float*)b2.data_ptr(), (float*)Y.data_ptr(), X.size(0), X.size(1), X.size(2), X.size(3),
                       X.size(4), (int)R, (int)IR, (int)TK, (int)TL, h ? 1 : 0, cur_stream(X)),
     "nc_fused_k3");
}

// Fused NC on e4m3 operands: X bf16 [V,I,J,K,L] -> Y fp32; W1a / W2a [64, 32] and
// W1b / W2b [64, 8] float8_e4m3fn fragments (taps 0-7 MX, tap 8); b1 [16], b2 [1]
// fp32; scales (sx, inv1, sh, inv2) as csrc/nc_fused.hip nc_fused_k3_f8_kernel.
void nc_fused_k3_f8(Tensor X, Tensor W1a, Tensor W1b, Tensor b1, Tensor W2a, Tensor W2b, Tensor b2, Tensor Y,
                    int64_t R, int64_t IR, int64_t TK, int64_t TL, double sx, double inv1, double sh, double inv2) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16);
  for (auto* t : {&W1a, &W1b, &W2a, &W2b}) check(*t, "W", at::kFloat8_e4m3fn);
  check(b1, "b1", at::kFloat); check(b2, "b2", at::kFloat); check(Y, "Y", at::kFloat);
  TORCH_CHECK(X.dim() == 5, "X must be [V,I,J,K,L]");
  check_shape(Y, "Y", X.sizes().vec());
  check_shape(W1a, "W1a", {64, 32}); check_shape(W2a, "W2a", {64, 32});
  check_shape(W1b, "W1b", {64, 8}); check_shape(W2b, "W2b", {64, 8});
  check_shape(b1, "b1", {16}); check_shape(b2, "b2", {1});
  TORCH_CHECK(R >= 1 && IR >= 1 && TK >= 1 && TL >= 1, "nc_fused_k3_f8: bad tiling");
  ok(ncnet_nc_fused_k3_f8(X.data_ptr(), W1a.data_ptr(), W1b.data_ptr(), (const float*)b1.data_ptr(), W2a.data_ptr(),
                          W2b.data_ptr(), (const float*)b2.data_ptr(), (float*)Y.data_ptr(), X.size(0), X.size(1),
                          X.size(2), X.size(3), X.size(4), (int)R, (int)IR, (int)TK, (int)TL, (float)sx, (float)inv1,
                          (float)sh, (float)inv2, cur_stream(X)),
     "nc_fused_k3_f8");
}

// NHWC implicit-GEMM conv with fused bias (+ residual) (+ ReLU).  X [N,Cin,H,W],
// W [Cout,Cin,KH,KW], R / Y [N,Cout,Ho,Wo]: all bf16 channels-last; bias fp32 [Cout].
void conv2d_nhwc(Tensor X, Tensor W, Tensor bias, c10::optional<Tensor> R, Tensor Y, int64_t stride, int64_t pad,
                 int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  auto cl = at::MemoryFormat::ChannelsLast;
  const bool h = X.scalar_type() == at::kHalf;
  const auto dt = h ? at::kHalf : at::kBFloat16;   // all operands bf16, or all IEEE half
  TORCH_CHECK(X.is_cuda() && (X.scalar_type() == at::kBFloat16 || h) && X.dim() == 4 && X.is_contiguous(cl),
              "conv2d_nhwc: X must be bf16 / fp16 channels-last [N,C,H,W]");
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == dt && W.dim() == 4 && W.is_contiguous(cl),
              "conv2d_nhwc: W must be channels-last [Cout,Cin,KH,KW] of X's dtype");
  const int64_t N = X.size(0), Cin = X.size(1), H = X.size(2), Wd = X.size(3);
  const int64_t Cout = W.size(0), KH = W.size(2), KW = W.size(3);
  TORCH_CHECK(W.size(1) == Cin, "conv2d_nhwc: Cin mismatch");
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0, "conv2d_nhwc: channels must be multiples of 64");
  const int64_t Ho = (H + 2 * pad - KH) / stride + 1, Wo = (Wd + 2 * pad - KW) / stride + 1;
  check(bias, "bias", at::kFloat); check_shape(bias, "bias", {Cout});
  TORCH_CHECK(Y.is_cuda() && Y.scalar_type() == dt && Y.is_contiguous(cl), "conv2d_nhwc: Y must be channels-last of X's dtype");
  check_shape(Y, "Y", {N, Cout, Ho, Wo});
  if (R.has_value()) {
    TORCH_CHECK(R->is_cuda() && R->scalar_type() == dt && R->is_contiguous(cl), "conv2d_nhwc: R must be channels-last of X's dtype");
    check_shape(*R, "R", {N, Cout, Ho, Wo});
  }
  TORCH_CHECK(N * Ho * Wo < (1LL << 31) && Cout * KH * KW * Cin < (1LL << 31), "conv2d_nhwc: sizes exceed int32");
  ok(ncnet_conv2d_nhwc(X.data_ptr(), W.data_ptr(), (const float*)bias.data_ptr(), R.has_value() ? R->data_ptr() : nullptr,
                       Y.data_ptr(), N, H, Wd, Cin, Cout, KH, KW, stride, pad, relu ? 1 : 0, h ? 1 : 0, cur_stream(X)),
     "conv2d_nhwc");
}

// 1x1 conv as a hipBLASLt GEMM with the fused bias (+ residual) (+ ReLU)
// epilogue (csrc/gemm_lt.hip).  X [N,Cin,H,W], W [Cout,Cin,1,1], R / Y
// [N,Cout,H,W]: bf16 / fp16 channels-last (or 2-D row-major [M, C]); bias fp32.
void gemm_lt(Tensor X, Tensor W, Tensor bias, c10::optional<Tensor> R, Tensor Y, int64_t relu, int64_t tune) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  const bool h = X.scalar_type() == at::kHalf;
  const auto dt = h ? at::kHalf : at::kBFloat16;
  auto rows = [&](const Tensor& t, const char* name, int64_t c) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt, "gemm_lt: ", name, " must be a GPU tensor of X's dtype");
    if (t.dim() == 4) {
      TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast) && t.size(1) == c,
                  "gemm_lt: ", name, " must be channels-last with ", c, " channels");
      return t.size(0) * t.size(2) * t.size(3);
    }
    TORCH_CHECK(t.dim() == 2 && t.is_contiguous() && t.size(1) == c, "gemm_lt: ", name, " must be [M, ", c, "]");
    return t.size(0);
  };
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 || h, "gemm_lt: X must be bf16 or fp16");
  const int64_t Cout = W.size(0), Cin = W.size(1);
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == dt && W.numel() == Cout * Cin &&
              (W.dim() == 2 ? W.is_contiguous() : W.is_contiguous(at::MemoryFormat::ChannelsLast)),
              "gemm_lt: W must be [Cout, Cin(, 1, 1)] of X's dtype");
  const int64_t M = rows(X, "X", Cin);
  TORCH_CHECK(rows(Y, "Y", Cout) == M, "gemm_lt: Y rows mismatch");
  if (R.has_value()) TORCH_CHECK(rows(*R, "R", Cout) == M, "gemm_lt: R rows mismatch");
  check(bias, "bias", at::kFloat); check_shape(bias, "bias", {Cout});
  TORCH_CHECK(M < (1LL << 31), "gemm_lt: M exceeds int32");
  ok(ncnet_gemm_lt(X.data_ptr(), W.data_ptr(), (const float*)bias.data_ptr(), R.has_value() ? R->data_ptr() : nullptr,
                   Y.data_ptr(), (int)M, (int)Cin, (int)Cout, relu ? 1 : 0, h ? 1 : 0, tune ? 1 : 0, cur_stream(X)),
     "gemm_lt");
}

// bf16x3 (fp32-accurate) trunk, csrc/conv2d.hip conv2d_nhwc_v3 X3 + csrc/epilogue.hip:
// activations are contiguous [N, H, W, 2C] bf16 = [hi | lo] channel pairs.
// W3 [Cout, KH, KW, 3 Cin] = [W_hi | W_hi | W_lo]; bias fp32 [Cout].
void conv2d_nhwc_x3(Tensor X, Tensor W3, Tensor bias, c10::optional<Tensor> R, Tensor Y, int64_t stride, int64_t pad,
                    int64_t relu) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(W3, "W3", at::kBFloat16); check(Y, "Y", at::kBFloat16);
  check(bias, "bias", at::kFloat);
  TORCH_CHECK(X.dim() == 4 && X.size(3) % 128 == 0, "conv2d_nhwc_x3: X must be [N,H,W,2 Cin], Cin % 64 == 0");
  const int64_t N = X.size(0), H = X.size(1), Wd = X.size(2), Cin = X.size(3) / 2;
  TORCH_CHECK(W3.dim() == 4 && W3.size(3) == 3 * Cin, "conv2d_nhwc_x3: W3 must be [Cout,KH,KW,3 Cin]");
  const int64_t Cout = W3.size(0), KH = W3.size(1), KW = W3.size(2);
  TORCH_CHECK(Cout % 64 == 0, "conv2d_nhwc_x3: Cout % 64");
  check_shape(bias, "bias", {Cout});
  const int64_t Ho = (H + 2 * pad - KH) / stride + 1, Wo = (Wd + 2 * pad - KW) / stride + 1;
  check_shape(Y, "Y", {N, Ho, Wo, 2 * Cout});
  if (R.has_value()) { check(*R, "R", at::kBFloat16); check_shape(*R, "R", {N, Ho, Wo, 2 * Cout}); }
  TORCH_CHECK(N * Ho * Wo < (1LL << 31) && N * H * Wd * 2 * Cin < (1LL << 40), "conv2d_nhwc_x3: sizes exceed int32");
  ok(ncnet_conv2d_nhwc_x3(X.data_ptr(), W3.data_ptr(), (const float*)bias.data_ptr(),
                          R.has_value() ? R->data_ptr() : nullptr, Y.data_ptr(), N, H, Wd, Cin, Cout, KH, KW, stride,
                          pad, relu ? 1 : 0, cur_stream(X)),
     "conv2d_nhwc_x3");
}

// fp32 NHWC image (an [N,C,H,W] channels-last tensor) -> stem im2col pairs A [N*Ho*Wo, 2 KP].
void stem_im2col_x3(Tensor X, Tensor A, int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  TORCH_CHECK(X.is_cuda() && X.scalar_type() == at::kFloat && X.dim() == 4 &&
                  X.is_contiguous(at::MemoryFormat::ChannelsLast), "stem_im2col_x3: X must be fp32 channels-last");
  check(A, "A", at::kBFloat16);
  const int64_t N = X.size(0), C = X.size(1), H = X.size(2), W = X.size(3);
  const int64_t Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(A.dim() == 2 && A.size(0) == N * Ho * Wo && A.size(1) % 16 == 0 && A.size(1) / 2 >= KH * KW * C,
              "stem_im2col_x3: A must be [N*Ho*Wo, 2 KP], KP % 8 == 0, KP >= KH*KW*C");
  ok(ncnet_stem_im2col_x3((const float*)X.data_ptr(), A.data_ptr(), N, H, W, C, KH, KW, stride, pad, Ho, Wo,
                          A.size(1) / 2, cur_stream(X)),
     "stem_im2col_x3");
}

void maxpool_x3(Tensor X, Tensor Y, int64_t k, int64_t stride, int64_t pad) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Y, "Y", at::kBFloat16);
  TORCH_CHECK(X.dim() == 4 && X.size(3) % 16 == 0, "maxpool_x3: X must be [N,H,W,2C], C % 8 == 0");
  const int64_t N = X.size(0), H = X.size(1), W = X.size(2), C = X.size(3) / 2;
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  check_shape(Y, "Y", {N, Ho, Wo, 2 * C});
  ok(ncnet_maxpool_x3(X.data_ptr(), Y.data_ptr(), N, H, W, C, Ho, Wo, k, stride, pad, cur_stream(X)), "maxpool_x3");
}

void x3_to_f32(Tensor X, Tensor Y) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check(X, "X", at::kBFloat16); check(Y, "Y", at::kFloat);
  const int64_t C = Y.size(-1);
  TORCH_CHECK(X.size(-1) == 2 * C && X.numel() == 2 * Y.numel() && C % 8 == 0, "x3_to_f32: X [..., 2C] -> Y [..., C]");
  ok(ncnet_x3_to_f32(X.data_ptr(), (float*)Y.data_ptr(), Y.numel() / C, C, cur_stream(X)), "x3_to_f32");
}

// Guarded flat Adam (csrc/optim.hip).  g may be longer than p (trailing
// loss-indicator slot); count / skipped int32 [1], step fp32 [1].
void nonfinite_count(Tensor g, Tensor count) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  check(g, "g", at::kFloat); check(count, "count", at::kInt); check_shape(count, "count", {1});
  ok(ncnet_nonfinite_count((const float*)g.data_ptr(), g.numel(), (int*)count.data_ptr(), cur_stream(g)), "nonfinite_count");
}

void adam_masked(Tensor p, Tensor g, Tensor m, Tensor v, Tensor count, Tensor step, double lr, double b1, double b2,
                 double eps, double wd, double gscale) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  for (auto* t : {&p, &g, &m, &v, &step}) check(*t, "adam buffer", at::kFloat);
  check(count, "count", at::kInt);
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() >= n && m.numel() == n && v.numel() == n, "adam_masked: buffer sizes differ");
  TORCH_CHECK(step.numel() == 1 && count.numel() == 1, "adam_masked: step/count must have one element");
  ok(ncnet_adam_masked((float*)p.data_ptr(), (float*)g.data_ptr(), (float*)m.data_ptr(), (float*)v.data_ptr(), n,
                       (const int*)count.data_ptr(), (const float*)step.data_ptr(), (float)lr, (float)b1, (float)b2,
                       (float)eps, (float)wd, (float)gscale, cur_stream(p)),
     "adam_masked");
}

void adam_finalize(Tensor step, Tensor count, Tensor skipped) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(step.device());
  check(step, "step", at::kFloat); check(count, "count", at::kInt); check(skipped, "skipped", at::kInt);
  TORCH_CHECK(step.numel() == 1 && count.numel() == 1 && skipped.numel() == 1, "adam_finalize: scalars expected");
  ok(ncnet_adam_finalize((float*)step.data_ptr(), (int*)count.data_ptr(), (int*)skipped.data_ptr(), cur_stream(step)),
     "adam_finalize");
}

// Batched resize + normalise of packed HWC uint8 images (csrc/dataprep.hip).
// src uint8 [bytes] (device), meta int64 [B, 3] = (byte offset, H, W) (device;
// validated against src by the caller before its host->device copy),
// out fp32 [B, 3, oh, ow]; mean / std: 3 floats each.
// 1 from a release build; 0 (after printing an NCNET_CHECK line) from the debug build.
int64_t debug_selftest(Tensor out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 1, "debug_selftest: int32 cuda");
  ok(ncnet_debug_selftest((int*)out.data_ptr(), cur_stream(out)), "debug_selftest");
  return out.cpu().item<int>();
}

void resize_norm_u8(Tensor src, Tensor meta, Tensor out, std::vector<double> mean, std::vector<double> stdv) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  check(src, "src", at::kByte); check(meta, "meta", at::kLong); check(out, "out", at::kFloat);
  TORCH_CHECK(src.dim() == 1, "src must be a flat byte buffer");
  TORCH_CHECK(meta.dim() == 2 && meta.size(1) == 3, "meta must be [B, 3]");
  TORCH_CHECK(out.dim() == 4 && out.size(0) == meta.size(0) && out.size(1) == 3, "out must be [B, 3, oh, ow]");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "mean / std need 3 values");
  const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  const float sd[3] = {(float)stdv[0], (float)stdv[1], (float)stdv[2]};
  ok(ncnet_resize_norm_u8(src.data_ptr(), (const long long*)meta.data_ptr(), (float*)out.data_ptr(), (int)out.size(0),
                          (int)out.size(2), (int)out.size(3), m, sd, cur_stream(src)),
     "resize_norm_u8");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for ncnet_amd";
  m.def("conv16_fwd", &conv16_fwd);
  m.def("pad_geom", &pad_geom);
  m.def("pad_planes", &pad_planes);
  m.def("conv1x16", &conv1x16);
  m.def("conv2d_nhwc_x3", &conv2d_nhwc_x3);
  m.def("stem_im2col_x3", &stem_im2col_x3);
  m.def("maxpool_x3", &maxpool_x3);
  m.def("x3_to_f32", &x3_to_f32);
  m.def("wgrad1x16", &wgrad1x16);
  m.def("conv16_blk_fwd", &conv16_blk_fwd);
  m.def("cout1_taps_fwd", &cout1_taps_fwd);
  m.def("conv16_fwd_x3", &conv16_fwd_x3);
  m.def("set_tuning", &set_tuning, py::arg("name"), py::arg("value") = py::none());
  m.def("conv16_blk_fwd_x3", &conv16_blk_fwd_x3);
  m.def("wgrad16p", &wgrad16p);
  m.def("wgrad16", &wgrad16);
  m.def("ijpack", &ijpack);
  m.def("conv16f8_fwd", &conv16f8_fwd);
  m.def("ijsum", &ijsum);
  m.def("bias_act_", &bias_act_);
  m.def("maxpool_bias_act", &maxpool_bias_act);
  m.def("conv2d_nhwc", &conv2d_nhwc);
  m.def("gemm_lt", &gemm_lt, py::arg("X"), py::arg("W"), py::arg("bias"), py::arg("R"), py::arg("Y"),
        py::arg("relu"), py::arg("tune") = 0);
  m.def("l2norm_rows", &l2norm_rows);
  m.def("l2norm_rows_bwd", &l2norm_rows_bwd);
  m.def("corr_gemm", &corr_gemm);
  m.def("corr_gemm_pool2", &corr_gemm_pool2);
  m.def("stats_rows", &stats_rows);
  m.def("stats_cols", &stats_cols);
  m.def("stats2d", &stats2d);
  m.def("gather_bf16", &gather_bf16);
  m.def("reduce_cols", &reduce_cols);
  m.def("match_candidates", &match_candidates);
  m.def("mm_apply", &mm_apply, py::arg("c"), py::arg("rmax"), py::arg("cmax"), py::arg("out"), py::arg("out_x"),
        py::arg("out_xt"), py::arg("eps"), py::arg("pad") = std::vector<int64_t>{});
  m.def("mm_bwd", &mm_bwd);
  m.def("combine_fwd", &combine_fwd);
  m.def("combine_bwd", &combine_bwd, py::arg("g"), py::arg("z"), py::arg("gz"), py::arg("R"), py::arg("C"),
        py::arg("gzl") = py::none());
  m.def("softmax_max_bwd", &softmax_max_bwd, py::arg("x"), py::arg("rmax"), py::arg("rarg"), py::arg("rse"),
        py::arg("cmax"), py::arg("carg"), py::arg("cse"), py::arg("wr"), py::arg("wc"), py::arg("gx"), py::arg("norm"),
        py::arg("eps"), py::arg("gscale") = py::none());
  m.def("score_sum", &score_sum);
  m.def("maxpool4d", &maxpool4d);
  m.def("transpose", &transpose);
  m.def("nc_fused_k3", &nc_fused_k3);
  m.def("nc_fused_k3_f8", &nc_fused_k3_f8);
  m.def("resize_norm_u8", &resize_norm_u8);
  m.def("debug_selftest", &debug_selftest);
  m.def("nonfinite_count", &nonfinite_count);
  m.def("adam_masked", &adam_masked);
  m.def("adam_finalize", &adam_finalize);
}
