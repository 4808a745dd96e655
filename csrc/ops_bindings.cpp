// Bindings of the generic HIP ops (csrc/kernels/ops.hip).
#include <torch/extension.h>

#include <cstdlib>
#include <cstdio>
#include <limits>
#include <c10/hip/HIPStream.h>

#include "kernels/bn.h"
#include "kernels/conv.h"
#include "kernels/gemm.h"
#include "kernels/gemm_f32.h"
#include "kernels/ops.h"
#include "kernels/pool.h"
#include "kernels/stem.h"

namespace {
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// TDL_DEBUG_POISON=1: outputs and partial-sum buffers of the conv kernels start as NaN instead of
// uninitialised (a row or pixel a kernel fails to write then shows up in the results)
int poison() {  // 1: partial-sum buffers, 2: and the gradient outputs
  static const int on = [] {
    const char* e = std::getenv("TDL_DEBUG_POISON");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  return on;
}
at::Tensor fresh(at::IntArrayRef shape, const at::TensorOptions& o, int level = 1) {
  const bool fp = o.dtype() == at::kFloat || o.dtype() == at::kBFloat16 || o.dtype() == at::kHalf;
  return (fp && poison() >= level) ? at::full(shape, std::numeric_limits<float>::quiet_NaN(), o) : at::empty(shape, o);
}

// (x [n, ...] f32, y [n]) = (X[idx], Y[idx]) in one launch; Y int64 or int32
std::vector<at::Tensor> gather_xy(at::Tensor X, at::Tensor Y, at::Tensor idx) {
  TORCH_CHECK(X.is_cuda() && Y.is_cuda() && idx.is_cuda(), "gather_xy: GPU tensors expected");
  TORCH_CHECK(X.is_contiguous() && Y.is_contiguous() && idx.is_contiguous(), "gather_xy: contiguous tensors expected");
  TORCH_CHECK(X.scalar_type() == at::kFloat && X.dim() >= 1, "gather_xy: X must be f32 [N, ...]");
  TORCH_CHECK((Y.scalar_type() == at::kLong || Y.scalar_type() == at::kInt) && Y.dim() == 1 && Y.size(0) == X.size(0),
              "gather_xy: Y must be int64 / int32 [N]");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.dim() == 1, "gather_xy: idx must be int32 [n]");
  const int64_t rows = idx.numel();
  auto shape = X.sizes().vec();
  shape[0] = rows;
  auto x = at::empty(shape, X.options());
  auto y = at::empty({rows}, Y.options());
  const int64_t row_elems = X.size(0) > 0 ? X.numel() / X.size(0) : 0;
  TORCH_CHECK(reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0, "gather_xy: X must be 16-byte aligned");
  tdl::gather_xy(X.data_ptr<float>(), Y.data_ptr(), idx.data_ptr<int>(), x.data_ptr<float>(), y.data_ptr(), rows,
                 row_elems, (int)Y.element_size(), cur_stream());
  return {x, y};
}

at::Tensor gather_rows(at::Tensor src, at::Tensor idx, double scale) {
  TORCH_CHECK(src.is_cuda() && idx.is_cuda(), "gather_rows: GPU tensors expected");
  TORCH_CHECK(src.is_contiguous() && idx.is_contiguous(), "gather_rows: contiguous tensors expected");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.dim() == 1, "gather_rows: idx must be int32 [n]");
  const int64_t rows = idx.numel();
  const int64_t row_elems = src.numel() / std::max<int64_t>(src.size(0), 1);
  std::vector<int64_t> shape(src.sizes().begin(), src.sizes().end());
  shape[0] = rows;
  auto out = fresh(shape, src.options().dtype(at::kFloat));
  if (src.scalar_type() == at::kFloat) {
    tdl::gather_rows_f32(src.data_ptr<float>(), idx.data_ptr<int>(), out.data_ptr<float>(), rows, row_elems,
                         (float)scale, cur_stream());
  } else if (src.scalar_type() == at::kByte) {
    tdl::gather_rows_u8(src.data_ptr<uint8_t>(), idx.data_ptr<int>(), out.data_ptr<float>(), rows, row_elems,
                        (float)scale, cur_stream());
  } else {
    TORCH_CHECK(false, "gather_rows: float32 or uint8 source expected");
  }
  return out;
}

at::Tensor gather_labels(at::Tensor src, at::Tensor idx) {
  TORCH_CHECK(src.is_cuda() && idx.is_cuda() && src.scalar_type() == at::kInt && idx.scalar_type() == at::kInt,
              "gather_labels: int32 GPU tensors expected");
  auto out = fresh({idx.numel()}, src.options());
  tdl::gather_i32(src.data_ptr<int>(), idx.data_ptr<int>(), out.data_ptr<int>(), idx.numel(), cur_stream());
  return out;
}
tdl::BnDType bn_dtype(const at::Tensor& x) {
  if (x.scalar_type() == at::kFloat) return tdl::BnDType::kF32;
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "batch_norm: float32 or bfloat16 activations expected");
  return tdl::BnDType::kBF16;
}

void bn_check(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() >= 2, "batch_norm: contiguous [..., C] GPU tensor expected");
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "batch_norm: C must be a multiple of 8 and <= 2048");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "batch_norm: 16-byte aligned data expected");
}

const float* opt_f32(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), "batch_norm: f32 GPU params");
  return t->data_ptr<float>();
}

// partial rows P of a [P + ceil(P/64)][2][C] f32 workspace produced by a conv epilogue
int parts_rows(const at::Tensor& t, int64_t C) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat && t.dim() == 3 && t.size(1) == 2 &&
                  t.size(2) == C,
              "batch_norm: part must be f32 [rows][2][C]");
  const int64_t rows = t.size(0);
  int64_t p = 1;
  while (p + (p + 63) / 64 < rows) ++p;  // invert rows = P + ceil(P / 64)
  TORCH_CHECK(p + (p + 63) / 64 == rows, "batch_norm: part rows must be P + ceil(P/64)");
  return (int)p;
}

// training forward: y = act(bn(x) [+ residual]); returns (y, stats[4][C] = mean, invstd, scale, shift);
// moving statistics updated in place (mean_off: folded conv bias, moving mean only)
static std::vector<at::Tensor> bn_forward_impl(at::Tensor x, c10::optional<at::Tensor> gamma,
                                               c10::optional<at::Tensor> beta, c10::optional<at::Tensor> moving_mean,
                                               c10::optional<at::Tensor> moving_var, double momentum, double eps,
                                               bool relu, c10::optional<at::Tensor> residual,
                                               c10::optional<at::Tensor> mean_off, c10::optional<at::Tensor> part_in,
                                               bool apply) {
  bn_check(x);
  const int64_t C = x.size(-1), M = x.numel() / C;
  const void* res = nullptr;
  if (residual.has_value() && residual->defined()) {
    bn_check(*residual);
    TORCH_CHECK(residual->scalar_type() == x.scalar_type() && residual->numel() == x.numel(),
                "batch_norm: residual must match x");
    res = residual->data_ptr();
  }
  const tdl::BnPlan plan = tdl::bn_plan(M, (int)C);
  auto f = x.options().dtype(at::kFloat);
  int given = 0;
  at::Tensor part;
  if (part_in.has_value() && part_in->defined()) {
    // [rows + ceil(rows/64)][2][C] from conv_fwd_stats: the first `rows` rows are the partial sums
    TORCH_CHECK(part_in->is_cuda() && part_in->is_contiguous() && part_in->scalar_type() == at::kFloat &&
                    part_in->dim() == 3 && part_in->size(1) == 2 && part_in->size(2) == C,
                "batch_norm: part must be f32 [rows][2][C]");
    given = parts_rows(*part_in, C);
    part = *part_in;
  } else {
    part = fresh({(int64_t)plan.part_rows * 2 * C}, f);
  }
  auto st = fresh({4, C}, f);  // mean, invstd, scale, shift
  float* mm = const_cast<float*>(opt_f32(moving_mean));
  float* mv = const_cast<float*>(opt_f32(moving_var));
  TORCH_CHECK((mm == nullptr) == (mv == nullptr), "batch_norm: moving mean and variance go together");
  hipStream_t s = cur_stream();
  float* sp = st.data_ptr<float>();
  tdl::bn_forward_stats(x.data_ptr(), bn_dtype(x), M, (int)C, part.data_ptr<float>(), opt_f32(gamma), opt_f32(beta),
                        opt_f32(mean_off), sp, sp + C, sp + 2 * C, sp + 3 * C, mm, mv, (float)momentum, (float)eps, s,
                        given);
  if (!apply) return {st};
  auto y = fresh(x.sizes(), x.options());
  tdl::bn_apply(x.data_ptr(), res, y.data_ptr(), bn_dtype(x), M, (int)C, sp + 2 * C, sp + 3 * C, relu ? 1 : 0, s);
  return {y, st};
}

// backward (mode 0 plain, 1 relu, 2 add+relu using y); returns (dx, dgamma, dbeta[, dz])
// dgamma_out / dbeta_out: f32 [C] tensors the parameter gradients are ADDED into (a trainer's slab
// views); the returned dgamma / dbeta are then those tensors
std::vector<at::Tensor> bn_backward(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> y,
                                    c10::optional<at::Tensor> gamma, at::Tensor st, int64_t mode,
                                    c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                                    c10::optional<at::Tensor> part_in) {
  bn_check(x);
  bn_check(dy);
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dy.numel() == x.numel(), "batch_norm backward: dy/x mismatch");
  TORCH_CHECK(mode >= 0 && mode <= 2, "batch_norm backward: bad mode");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(st.is_contiguous() && st.numel() == 4 * C && st.scalar_type() == at::kFloat, "batch_norm: stats [4][C]");
  const void* yp = nullptr;
  at::Tensor dz;
  if (mode == 2 && !(part_in.has_value() && part_in->defined())) {
    TORCH_CHECK(y.has_value() && y->defined(), "batch_norm backward mode 2 needs y");
    bn_check(*y);
    yp = y->data_ptr();
    dz = fresh(x.sizes(), x.options());
  } else if (mode == 2) {
    dz = dy;
  }
  const tdl::BnPlan plan = tdl::bn_plan(M, (int)C);
  auto f = x.options().dtype(at::kFloat);
  int given = 0;
  at::Tensor part;
  if (part_in.has_value() && part_in->defined()) {
    // (dz, part) from conv_dgrad_bn: dy IS the group's masked gradient dz (for an add+relu group
    // also returned as the residual's); mode 0: a plain BN whose output gradient is such a group's
    // dz (part2 of conv_dgrad_bn: sums of dz and dz * x)
    given = parts_rows(*part_in, C);
    part = *part_in;
  } else {
    part = fresh({(int64_t)plan.part_rows * 2 * C}, f);
  }
  auto out = fresh({5, C}, f);  // dgamma, dbeta, coef[3]
  auto dx = fresh(x.sizes(), x.options());
  float* o = out.data_ptr<float>();
  const float* sp = st.data_ptr<float>();
  auto check_out = [&](const c10::optional<at::Tensor>& t) {
    if (!t.has_value() || !t->defined()) return (float*)nullptr;
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat && t->numel() == C,
                "batch_norm backward: gradient outputs must be contiguous f32 [C]");
    return t->data_ptr<float>();
  };
  float* pg = check_out(dgamma_out);
  float* pb = check_out(dbeta_out);
  const int acc = (pg ? 1 : 0) | (pb ? 2 : 0);
  tdl::bn_backward(dy.data_ptr(), x.data_ptr(), yp, mode == 2 ? dz.data_ptr() : nullptr, dx.data_ptr(), bn_dtype(x), M,
                   (int)C, part.data_ptr<float>(), opt_f32(gamma), sp, sp + C, sp + 2 * C, sp + 3 * C, pg ? pg : o,
                   pb ? pb : o + C, o + 2 * C, (int)mode, acc, cur_stream(), given);
  at::Tensor g = pg ? *dgamma_out : out[0], b = pb ? *dbeta_out : out[1];
  if (mode == 2) return {dx, g, b, dz};
  return {dx, g, b};
}
std::vector<at::Tensor> bn_forward_train(at::Tensor x, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                                         c10::optional<at::Tensor> moving_mean, c10::optional<at::Tensor> moving_var,
                                         double momentum, double eps, bool relu, c10::optional<at::Tensor> residual,
                                         c10::optional<at::Tensor> mean_off, c10::optional<at::Tensor> part_in) {
  return bn_forward_impl(x, gamma, beta, moving_mean, moving_var, momentum, eps, relu, residual, mean_off, part_in,
                         true);
}

// the batch statistics only ([4][C]: mean, invstd, scale, shift; moving statistics updated): the
// normalisation is applied by the consumer (maxpool_fwd(bn_stats=...))
at::Tensor bn_stats_train(at::Tensor x, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                          c10::optional<at::Tensor> moving_mean, c10::optional<at::Tensor> moving_var, double momentum,
                          double eps, c10::optional<at::Tensor> mean_off, c10::optional<at::Tensor> part_in) {
  return bn_forward_impl(x, gamma, beta, moving_mean, moving_var, momentum, eps, false, c10::nullopt, mean_off,
                         part_in, false)[0];
}

static const float* bn_ss_of(const c10::optional<at::Tensor>& st, int64_t C) {
  if (!st.has_value() || !st->defined()) return nullptr;
  TORCH_CHECK(st->is_cuda() && st->is_contiguous() && st->scalar_type() == at::kFloat && st->numel() == 4 * C,
              "bn_stats must be the f32 [4][C] statistics of the batch norm");
  return st->data_ptr<float>() + 2 * C;  // scale[C], shift[C]
}

// max pool NHWC: returns (y, argmax bytes); pads = (top, left), output size given; bn_stats: x is a
// batch norm's input and the pool runs over relu(bn(x)) (the BN -> ReLU pass skipped)
std::vector<at::Tensor> maxpool_fwd(at::Tensor x, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t pt,
                                    int64_t pl, int64_t OH, int64_t OW, bool pad_zero,
                                    c10::optional<at::Tensor> bn_stats) {
  bn_check(x);
  TORCH_CHECK(x.dim() == 4, "maxpool: NHWC input expected");
  TORCH_CHECK(kh * kw < 255 && kh > 0 && kw > 0 && sh > 0 && sw > 0 && OH > 0 && OW > 0, "maxpool: bad geometry");
  tdl::PoolGeom g{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)OH, (int)OW,
                  (int)kh, (int)kw, (int)sh, (int)sw, (int)pt, (int)pl, pad_zero ? 1 : 0};
  auto y = fresh({x.size(0), OH, OW, x.size(3)}, x.options());
  auto arg = fresh({x.size(0), OH, OW, x.size(3)}, x.options().dtype(at::kByte));
  tdl::maxpool_forward(x.data_ptr(), y.data_ptr(), arg.data_ptr<uint8_t>(), bn_dtype(x) == tdl::BnDType::kBF16, g,
                       cur_stream(), bn_ss_of(bn_stats, x.size(3)));
  return {y, arg};
}

at::Tensor maxpool_bwd(at::Tensor dy, at::Tensor arg, std::vector<int64_t> in_shape, int64_t kh, int64_t kw,
                       int64_t sh, int64_t sw, int64_t pt, int64_t pl) {
  bn_check(dy);
  TORCH_CHECK(dy.dim() == 4 && arg.sizes() == dy.sizes() && arg.scalar_type() == at::kByte && arg.is_contiguous(),
              "maxpool backward: dy / argmax mismatch");
  TORCH_CHECK(in_shape.size() == 4 && in_shape[3] == dy.size(3) && in_shape[0] == dy.size(0), "maxpool: bad shape");
  tdl::PoolGeom g{(int)in_shape[0], (int)in_shape[1], (int)in_shape[2], (int)in_shape[3], (int)dy.size(1),
                  (int)dy.size(2), (int)kh, (int)kw, (int)sh, (int)sw, (int)pt, (int)pl, 0};
  auto dx = fresh(in_shape, dy.options());
  tdl::maxpool_backward(dy.data_ptr(), arg.data_ptr<uint8_t>(), dx.data_ptr(), bn_dtype(dy) == tdl::BnDType::kBF16, g,
                        cur_stream());
  return dx;
}

// backward of maxpool_fwd(bn_stats=...): (dz, part) -- dz the BN -> ReLU group's masked input gradient,
// part [P + ceil(P/64)][2][C] its BN backward sums (bn_backward(part=...))
std::vector<at::Tensor> maxpool_bwd_bn(at::Tensor dy, at::Tensor arg, std::vector<int64_t> in_shape, int64_t kh,
                                       int64_t kw, int64_t sh, int64_t sw, int64_t pt, int64_t pl, at::Tensor bn_x,
                                       at::Tensor bn_stats) {
  bn_check(dy);
  bn_check(bn_x);
  TORCH_CHECK(dy.dim() == 4 && arg.sizes() == dy.sizes() && arg.scalar_type() == at::kByte && arg.is_contiguous(),
              "maxpool backward: dy / argmax mismatch");
  TORCH_CHECK(in_shape.size() == 4 && in_shape[3] == dy.size(3) && in_shape[0] == dy.size(0), "maxpool: bad shape");
  TORCH_CHECK(bn_x.sizes() == at::IntArrayRef(in_shape) && bn_x.scalar_type() == dy.scalar_type(),
              "maxpool backward: bn_x must be the pool input's batch-norm input");
  const int64_t C = in_shape[3];
  TORCH_CHECK(C <= 2048 && ((C / 8) & (C / 8 - 1)) == 0, "maxpool backward (BN-fused): C / 8 must be a power of two");
  tdl::PoolGeom g{(int)in_shape[0], (int)in_shape[1], (int)in_shape[2], (int)in_shape[3], (int)dy.size(1),
                  (int)dy.size(2), (int)kh, (int)kw, (int)sh, (int)sw, (int)pt, (int)pl, 0};
  auto dx = fresh(in_shape, dy.options());
  const int64_t P = tdl::maxpool_backward_blocks(g);
  auto part = fresh({P + (P + 63) / 64, 2, C}, dy.options().dtype(at::kFloat));
  tdl::maxpool_backward(dy.data_ptr(), arg.data_ptr<uint8_t>(), dx.data_ptr(), bn_dtype(dy) == tdl::BnDType::kBF16, g,
                        cur_stream(), bn_x.data_ptr(), bn_ss_of(bn_stats, C), part.data_ptr<float>());
  return {dx, part};
}

tdl::ConvGeom conv_geom(const at::Tensor& x, int64_t oh, int64_t ow, int64_t k, int64_t kh, int64_t kw, int64_t sh,
                        int64_t sw, int64_t pt, int64_t pl) {
  TORCH_CHECK(x.dim() == 4, "conv: NHWC activations expected");
  tdl::ConvGeom g{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)oh, (int)ow, (int)k,
                  (int)kh, (int)kw, (int)sh, (int)sw, (int)pt, (int)pl};
  TORCH_CHECK(tdl::conv_bf16_supported(g), "conv: unsupported geometry (C and K must be multiples of 64)");
  return g;
}

void conv_check(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kBFloat16, "conv: ", what,
              " must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "conv: ", what, " must be 16-byte aligned");
}

// y[N,OH,OW,K] = conv(x[N,H,W,C], w_ohwi[K,KH,KW,C]); top/left padding pt/pl, bottom/right implied by OH/OW
// in_bn: x is the input of a BN -> ReLU (its [4][C] batch statistics); the conv runs over relu(bn(x))
static const float* conv_in_bn(const c10::optional<at::Tensor>& in_bn, const tdl::ConvGeom& g) {
  const float* ss = bn_ss_of(in_bn, g.C);
  TORCH_CHECK(!ss || tdl::conv_in_bn_supported(g),
              "conv: the input-side batch norm takes 1x1 stride-1 unpadded convolutions of <= 512 channels");
  return ss;
}

at::Tensor conv_fwd(at::Tensor x, at::Tensor w_ohwi, int64_t oh, int64_t ow, int64_t sh, int64_t sw, int64_t pt,
                    int64_t pl, c10::optional<at::Tensor> in_bn) {
  conv_check(x, "x");
  conv_check(w_ohwi, "w");
  TORCH_CHECK(w_ohwi.dim() == 4 && w_ohwi.size(3) == x.size(3), "conv_fwd: weights must be OHWI [K,KH,KW,C]");
  auto g = conv_geom(x, oh, ow, w_ohwi.size(0), w_ohwi.size(1), w_ohwi.size(2), sh, sw, pt, pl);
  const float* ss = conv_in_bn(in_bn, g);
  auto y = fresh({x.size(0), oh, ow, w_ohwi.size(0)}, x.options());
  tdl::conv_fwd_bf16(x.data_ptr(), w_ohwi.data_ptr(), y.data_ptr(), g, cur_stream(), nullptr, ss);
  return y;
}

// forward + batch-norm partial sums of y: returns (y, part[P + ceil(P/64)][2][K]) with P row tiles
std::vector<at::Tensor> conv_fwd_stats(at::Tensor x, at::Tensor w_ohwi, int64_t oh, int64_t ow, int64_t sh,
                                       int64_t sw, int64_t pt, int64_t pl, c10::optional<at::Tensor> in_bn) {
  conv_check(x, "x");
  conv_check(w_ohwi, "w");
  TORCH_CHECK(w_ohwi.dim() == 4 && w_ohwi.size(3) == x.size(3), "conv_fwd: weights must be OHWI [K,KH,KW,C]");
  auto g = conv_geom(x, oh, ow, w_ohwi.size(0), w_ohwi.size(1), w_ohwi.size(2), sh, sw, pt, pl);
  const float* ss = conv_in_bn(in_bn, g);
  auto y = fresh({x.size(0), oh, ow, w_ohwi.size(0)}, x.options());
  const int64_t M = (int64_t)g.N * g.OH * g.OW, bm = tdl::conv_fwd_row_tile(g, ss != nullptr);
  const int64_t P = (M + bm - 1) / bm;
  auto part = fresh({P + (P + 63) / 64, 2, (int64_t)g.K}, x.options().dtype(at::kFloat));
  tdl::conv_fwd_bf16(x.data_ptr(), w_ohwi.data_ptr(), y.data_ptr(), g, cur_stream(), part.data_ptr<float>(), ss);
  return {y, part};
}

// stride-1 input gradient: dx[N,H,W,C] from dy[N,OH,OW,K] and w_hwio[KH,KW,C,K]
const void* opt_residual(const c10::optional<at::Tensor>& r, const at::Tensor& like_dy, int64_t n, int64_t h,
                         int64_t w, int64_t c) {
  if (!r.has_value() || !r->defined()) return nullptr;
  conv_check(*r, "residual");
  TORCH_CHECK(r->dim() == 4 && r->size(0) == n && r->size(1) == h && r->size(2) == w && r->size(3) == c,
              "conv dgrad: residual must be shaped like dx");
  (void)like_dy;
  return r->data_ptr();
}

std::vector<at::Tensor> conv_dgrad_impl(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w, int64_t pt,
                                        int64_t pl, c10::optional<at::Tensor> residual,
                                        c10::optional<at::Tensor> bn_y, c10::optional<at::Tensor> bn_x,
                                        c10::optional<at::Tensor> bn_x2, c10::optional<at::Tensor> bn_stats);

// BN-group fusion operands of an input gradient (see conv.h): (bn_y, bn_x[, bn_x2]) tensors shaped
// like dx, and the part buffers [P + ceil(P/64)][2][C] for P row tiles
// bn_stats: the [4][C] statistics (mean, invstd, scale, shift) of a plain BN -> ReLU group's forward:
// the mask is recomputed from bn_x (bn_y may then be absent)
struct DgradBn {
  const void *by = nullptr, *bx = nullptr, *bx2 = nullptr;
  const float* ss = nullptr;
  at::Tensor part, part2;
  DgradBn(const c10::optional<at::Tensor>& bn_y, const c10::optional<at::Tensor>& bn_x,
          const c10::optional<at::Tensor>& bn_x2, const c10::optional<at::Tensor>& bn_stats, const at::Tensor& dy,
          int64_t h, int64_t w, int64_t c, int64_t P) {
    by = opt_residual(bn_y, dy, dy.size(0), h, w, c);
    bx = opt_residual(bn_x, dy, dy.size(0), h, w, c);
    bx2 = opt_residual(bn_x2, dy, dy.size(0), h, w, c);
    if (bn_stats.has_value() && bn_stats->defined()) {
      TORCH_CHECK(bn_stats->is_cuda() && bn_stats->is_contiguous() && bn_stats->scalar_type() == at::kFloat &&
                      bn_stats->numel() == 4 * c,
                  "conv_dgrad: bn_stats must be the f32 [4][C] statistics of the group's BN");
      ss = bn_stats->data_ptr<float>() + 2 * c;  // scale[C], shift[C]
    }
    TORCH_CHECK((by != nullptr || ss != nullptr) == (bx != nullptr), "conv_dgrad: bn_y (or bn_stats) and bn_x go together");
    TORCH_CHECK(bx2 == nullptr || bx != nullptr, "conv_dgrad: bn_x2 needs bn_x");
    auto f = dy.options().dtype(at::kFloat);
    if (bx) part = fresh({P + (P + 63) / 64, 2, c}, f);
    if (bx2) part2 = fresh({P + (P + 63) / 64, 2, c}, f);
  }
  float* p() { return bx ? part.data_ptr<float>() : nullptr; }
  float* p2() { return bx2 ? part2.data_ptr<float>() : nullptr; }
  std::vector<at::Tensor> out(const at::Tensor& dx) {
    if (bx2) return {dx, part, part2};
    if (bx) return {dx, part};
    return {dx};
  }
};

at::Tensor conv_dgrad(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w, int64_t pt, int64_t pl,
                      c10::optional<at::Tensor> residual) {
  return conv_dgrad_impl(dy, w_hwio, h, w, pt, pl, residual, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt)[0];
}

// input gradient with the fused backward of the BN -> Add -> ReLU group that produced the conv's
// input bn_y from bn_x: returns (dz, part[P + ceil(P/64)][2][C][, part2]); bn_x2: the input of the
// plain BN whose output is the group's residual (part2: its backward sums); bn_stats instead of bn_y:
// a plain BN -> ReLU group, mask recomputed from bn_x
std::vector<at::Tensor> conv_dgrad_bn(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w, int64_t pt, int64_t pl,
                                      c10::optional<at::Tensor> residual, c10::optional<at::Tensor> bn_y,
                                      at::Tensor bn_x, c10::optional<at::Tensor> bn_x2,
                                      c10::optional<at::Tensor> bn_stats) {
  return conv_dgrad_impl(dy, w_hwio, h, w, pt, pl, residual, bn_y, bn_x, bn_x2, bn_stats);
}

std::vector<at::Tensor> conv_dgrad_impl(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w, int64_t pt,
                                        int64_t pl, c10::optional<at::Tensor> residual,
                                        c10::optional<at::Tensor> bn_y, c10::optional<at::Tensor> bn_x,
                                        c10::optional<at::Tensor> bn_x2, c10::optional<at::Tensor> bn_stats) {
  conv_check(dy, "dy");
  conv_check(w_hwio, "w");
  TORCH_CHECK(w_hwio.dim() == 4 && w_hwio.size(3) == dy.size(3), "conv_dgrad: weights must be HWIO [KH,KW,C,K]");
  tdl::ConvGeom g{(int)dy.size(0), (int)h, (int)w, (int)w_hwio.size(2), (int)dy.size(1), (int)dy.size(2),
                  (int)dy.size(3), (int)w_hwio.size(0), (int)w_hwio.size(1), 1, 1, (int)pt, (int)pl};
  TORCH_CHECK(tdl::conv_bf16_supported(g), "conv_dgrad: unsupported geometry (C and K must be multiples of 64)");
  auto dx = fresh({dy.size(0), h, w, w_hwio.size(2)}, dy.options(), 2);
  const int64_t M = (int64_t)g.N * g.H * g.W, bm = tdl::conv_dgrad_row_tile(g);
  DgradBn bn(bn_y, bn_x, bn_x2, bn_stats, dy, h, w, w_hwio.size(2), (M + bm - 1) / bm);
  tdl::conv_dgrad_bf16(dy.data_ptr(), w_hwio.data_ptr(), dx.data_ptr(), g, cur_stream(),
                       opt_residual(residual, dy, dy.size(0), h, w, w_hwio.size(2)), bn.by, bn.bx, bn.p(), bn.bx2,
                       bn.p2(), bn.ss);
  return bn.out(dx);
}
// input gradient of a 1x1 stride-2 unpadded conv: dx[N,H,W,C] from dy[N,OH,OW,K] and w_hwio[1,1,C,K];
// with bn_y / bn_x[ / bn_x2] the fused BN-group backward as in conv_dgrad_bn: (dz, part[, part2])
std::vector<at::Tensor> conv_dgrad_s2_impl(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w,
                                           c10::optional<at::Tensor> residual, c10::optional<at::Tensor> bn_y,
                                           c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_x2,
                                           c10::optional<at::Tensor> bn_stats) {
  conv_check(dy, "dy");
  conv_check(w_hwio, "w");
  TORCH_CHECK(w_hwio.dim() == 4 && w_hwio.size(0) == 1 && w_hwio.size(1) == 1 && w_hwio.size(3) == dy.size(3),
              "conv_dgrad_s2: weights must be HWIO [1,1,C,K]");
  TORCH_CHECK(h <= 2 * dy.size(1) && w <= 2 * dy.size(2) && h > 2 * (dy.size(1) - 1) && w > 2 * (dy.size(2) - 1),
              "conv_dgrad_s2: (h, w) inconsistent with a stride-2 1x1 conv");
  tdl::ConvGeom g{(int)dy.size(0), (int)h, (int)w, (int)w_hwio.size(2), (int)dy.size(1), (int)dy.size(2),
                  (int)dy.size(3), 1, 1, 2, 2, 0, 0};
  TORCH_CHECK(tdl::conv_bf16_supported(g), "conv_dgrad_s2: unsupported geometry (C and K must be multiples of 64)");
  auto dx = fresh({dy.size(0), h, w, w_hwio.size(2)}, dy.options(), 2);
  const int64_t M = (int64_t)g.N * g.OH * g.OW, bm = tdl::conv_dgrad_s2_row_tile(g);
  DgradBn bn(bn_y, bn_x, bn_x2, bn_stats, dy, h, w, w_hwio.size(2), (M + bm - 1) / bm);
  tdl::conv_dgrad_s2_1x1_bf16(dy.data_ptr(), w_hwio.data_ptr(), dx.data_ptr(), g, cur_stream(),
                              opt_residual(residual, dy, dy.size(0), h, w, w_hwio.size(2)), bn.by, bn.bx, bn.p(),
                              bn.bx2, bn.p2(), bn.ss);
  return bn.out(dx);
}

at::Tensor conv_dgrad_s2(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w, c10::optional<at::Tensor> residual) {
  return conv_dgrad_s2_impl(dy, w_hwio, h, w, residual, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt)[0];
}

std::vector<at::Tensor> conv_dgrad_s2_bn(at::Tensor dy, at::Tensor w_hwio, int64_t h, int64_t w,
                                         c10::optional<at::Tensor> residual, c10::optional<at::Tensor> bn_y,
                                         at::Tensor bn_x, c10::optional<at::Tensor> bn_x2,
                                         c10::optional<at::Tensor> bn_stats) {
  return conv_dgrad_s2_impl(dy, w_hwio, h, w, residual, bn_y, bn_x, bn_x2, bn_stats);
}

// weight gradient: dw[KH,KW,C,K] (bf16, or added into the f32 `out` when given) from x[N,H,W,C] and
// dy[N,OH,OW,K]; deterministic split-K.  plan = [wmw, wnw, nsplit] (empty: the model's first choice)
at::Tensor conv_wgrad(at::Tensor x, at::Tensor dy, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t pt,
                      int64_t pl, c10::optional<at::Tensor> out, bool accumulate, std::vector<int64_t> plan,
                      c10::optional<at::Tensor> in_bn) {
  conv_check(x, "x");
  conv_check(dy, "dy");
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == x.size(0), "conv_wgrad: dy must be NHWC [N,OH,OW,K]");
  auto g = conv_geom(x, dy.size(1), dy.size(2), dy.size(3), kh, kw, sh, sw, pt, pl);
  const float* ss = conv_in_bn(in_bn, g);
  TORCH_CHECK(!ss || plan.empty() || (plan[0] != 0 && plan[0] * plan[1] <= 4 && (plan.size() == 3 || plan[3] == 0)),
              "conv_wgrad: the input-side batch norm runs on the register-staged plans (<= 4 waves, kind 0)");
  TORCH_CHECK(tdl::conv_wgrad_supported(g), "conv_wgrad: N*OH*OW must be < 2^24");
  TORCH_CHECK(plan.empty() || plan.size() == 3 || plan.size() == 4, "conv_wgrad: plan = [wmw, wnw, nsplit(, kind)]");
  if (!plan.empty() && plan[0] == 0) {  // [0, 0, 0]: the row kernel of 3x3 / C = 64 convs (wgrad3x3.hip)
    TORCH_CHECK(tdl::conv_wgrad3x3_c64_supported(g), "conv_wgrad: the 3x3 row kernel does not take this shape");
    auto ws = fresh({tdl::conv_wgrad3x3_c64_ws_elems(g)}, x.options().dtype(at::kFloat));
    if (out.has_value()) {
      auto& o = *out;
      TORCH_CHECK(o.is_cuda() && o.is_contiguous() && o.scalar_type() == at::kFloat &&
                      o.numel() == kh * kw * x.size(3) * dy.size(3),
                  "conv_wgrad: out must be a contiguous f32 tensor of KH*KW*C*K elements");
      tdl::conv_wgrad3x3_c64(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), nullptr, o.data_ptr<float>(), accumulate,
                             g, cur_stream());
      return o;
    }
    auto dw = fresh({kh, kw, x.size(3), dy.size(3)}, x.options());
    tdl::conv_wgrad3x3_c64(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), dw.data_ptr(), nullptr, false, g,
                           cur_stream());
    return dw;
  }
  tdl::WgradPlan p;
  if (plan.empty()) {
    p = tdl::conv_wgrad_plans(g, 1, ss != nullptr).at(0);
  } else {
    const int wmw = (int)plan[0], wnw = (int)plan[1];
    TORCH_CHECK((wmw == 1 || wmw == 2 || wmw == 4) && (wnw == 1 || wnw == 2 || wnw == 4) &&
                    (wmw * wnw <= 4 || (wmw * wnw == 8 && wmw != wnw)) &&
                    g.K % (64 * wmw) == 0 && plan[2] >= 1 &&
                    (plan.size() == 3 || plan[3] == 0 || (plan[3] == 1 && wmw == 2 && wnw == 2)),
                "conv_wgrad: bad plan");
    p = tdl::conv_wgrad_make_plan(g, wmw, wnw, (int)plan[2], plan.size() == 4 ? (int)plan[3] : 0);
  }
  auto ws = fresh({p.ws_elems}, x.options().dtype(at::kFloat));
  if (out.has_value()) {
    auto& o = *out;
    TORCH_CHECK(o.is_cuda() && o.is_contiguous() && o.scalar_type() == at::kFloat &&
                    o.numel() == kh * kw * x.size(3) * dy.size(3),
                "conv_wgrad: out must be a contiguous f32 tensor of KH*KW*C*K elements");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(o.data_ptr()) % 16 == 0, "conv_wgrad: out must be 16-byte aligned");
    tdl::conv_wgrad_bf16(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), p, nullptr, o.data_ptr<float>(),
                         accumulate, g, cur_stream(), ss);
    return o;
  }
  auto dw = fresh({kh, kw, x.size(3), dy.size(3)}, x.options());
  tdl::conv_wgrad_bf16(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), p, dw.data_ptr(), nullptr, false, g,
                       cur_stream(), ss);
  return dw;
}

// small-channel stride-2 conv (ResNet stem, csrc/kernels/stem.hip).  x [N,H,W,C] (bf16 or f32,
// C <= 4), w_hwio [KH,KW,C,K] bf16, zero padding (pt, pb, pl, pr) folded into the packed copy.
// Returns (y [N,OH,OW,K] bf16, xp packed image for the backward[, part [P + ceil(P/64)][2][K]])
std::vector<at::Tensor> stem_fwd(at::Tensor x, at::Tensor w_hwio, int64_t pt, int64_t pb, int64_t pl, int64_t pr,
                                 int64_t sh, int64_t sw, bool stats) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4 &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "stem: x must be a contiguous NHWC bf16/f32 GPU tensor");
  conv_check(w_hwio, "w");
  TORCH_CHECK(w_hwio.dim() == 4 && w_hwio.size(2) == x.size(3), "stem: weights must be HWIO [KH,KW,C,K]");
  const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3);
  const int KH = (int)w_hwio.size(0), KW = (int)w_hwio.size(1), K = (int)w_hwio.size(3);
  TORCH_CHECK(tdl::stem_supported(C, KH, KW, (int)sw, K) && sh >= 1 && pt >= 0 && pb >= 0 && pl >= 0 && pr >= 0,
              "stem: unsupported geometry");
  const int HP = H + (int)(pt + pb), WPv = W + (int)(pl + pr);
  const int OH = (HP - KH) / (int)sh + 1, OW = (WPv - KW) / 2 + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "stem: empty output");
  // packed width: every receptive field reads 8 columns (taps past KW are zero-weighted): 2(OW-1)+8
  const int WP = std::max(WPv, 2 * (OW - 1) + 8);
  const int HPp = std::max(HP, (OH - 1) * (int)sh + KH);
  TORCH_CHECK((long long)N * HPp * WP * 4 < (1LL << 31), "stem: packed image too large");
  auto xp = fresh({N, HPp, WP, 4}, x.options().dtype(at::kBFloat16));
  tdl::stem_pack(x.data_ptr(), x.scalar_type() == at::kBFloat16, xp.data_ptr(), N, H, W, C, HPp, WP, (int)pt, (int)pl,
                 cur_stream());
  auto wp = fresh({K, KH, 32}, w_hwio.options());
  tdl::stem_wpack(w_hwio.data_ptr(), wp.data_ptr(), KH, KW, C, K, cur_stream());
  auto y = fresh({N, OH, OW, K}, x.options().dtype(at::kBFloat16));
  const int64_t M = (int64_t)N * OH * OW, bm = tdl::stem_fwd_row_tile(), P = (M + bm - 1) / bm;
  at::Tensor part;
  if (stats) part = fresh({P + (P + 63) / 64, 2, (int64_t)K}, x.options().dtype(at::kFloat));
  tdl::stem_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), stats ? part.data_ptr<float>() : nullptr, N, HPp, WP, OH,
                OW, K, KH, (int)sh, cur_stream());
  if (stats) return {y, xp, part};
  return {y, xp};
}

// weight gradient of stem_fwd from its packed image: dW HWIO [KH,KW,C,K] bf16, or added into the f32
// `out` (accumulate) / written to it
at::Tensor stem_wgrad(at::Tensor xp, at::Tensor dy, int64_t kh, int64_t kw, int64_t c, int64_t sh,
                      c10::optional<at::Tensor> out, bool accumulate) {
  conv_check(xp, "xp");
  conv_check(dy, "dy");
  TORCH_CHECK(xp.dim() == 4 && xp.size(3) == 4 && dy.dim() == 4 && dy.size(0) == xp.size(0), "stem_wgrad: shapes");
  const int N = (int)xp.size(0), HP = (int)xp.size(1), WP = (int)xp.size(2);
  const int OH = (int)dy.size(1), OW = (int)dy.size(2), K = (int)dy.size(3);
  TORCH_CHECK(tdl::stem_supported((int)c, (int)kh, (int)kw, 2, K) && (OH - 1) * sh + kh <= HP &&
                  2 * (OW - 1) + 8 <= WP,
              "stem_wgrad: geometry inconsistent with the packed image");
  const int M = N * OH * OW;
  auto ws = fresh({tdl::stem_wgrad_ws_elems(M, K, (int)kh)}, dy.options().dtype(at::kFloat));
  if (out.has_value()) {
    auto& o = *out;
    TORCH_CHECK(o.is_cuda() && o.is_contiguous() && o.scalar_type() == at::kFloat && o.numel() == kh * kw * c * K,
                "stem_wgrad: out must be a contiguous f32 tensor of KH*KW*C*K elements");
    tdl::stem_wgrad(xp.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), N, HP, WP, OH, OW, K, (int)kh, (int)kw, (int)c,
                    (int)sh, o.data_ptr<float>(), nullptr, accumulate, cur_stream());
    return o;
  }
  auto dw = fresh({kh, kw, c, (int64_t)K}, dy.options());
  tdl::stem_wgrad(xp.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), N, HP, WP, OH, OW, K, (int)kh, (int)kw, (int)c,
                  (int)sh, nullptr, dw.data_ptr(), false, cur_stream());
  return dw;
}

// the model's best candidate plans: [[wmw, wnw, chunk, nsplit, kind], ...]
std::vector<std::vector<int64_t>> conv_wgrad_plans(std::vector<int64_t> x_shape, std::vector<int64_t> dy_shape,
                                                   int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t pt,
                                                   int64_t pl, int64_t max_plans, bool in_bn) {
  tdl::ConvGeom g{(int)x_shape[0], (int)x_shape[1], (int)x_shape[2], (int)x_shape[3], (int)dy_shape[1],
                  (int)dy_shape[2], (int)dy_shape[3], (int)kh, (int)kw, (int)sh, (int)sw, (int)pt, (int)pl};
  std::vector<std::vector<int64_t>> out;
  // the 3x3 / C = 64 row kernel first where it applies (it beats the split-K tiles on these shapes)
  if (!in_bn && tdl::conv_wgrad3x3_c64_supported(g)) out.push_back({0, 0, 0, 0, 0});
  for (const auto& p : tdl::conv_wgrad_plans(g, (int)max_plans, in_bn))
    out.push_back({p.wmw, p.wnw, p.chunk, p.nsplit, p.kind});
  return out;
}
// dst (bf16 slab) <- transposed copies of the HWIO f32 conv kernels in src (f32 slab); entries
// [E][4] (src off, dst off, R, K) and tiles [T][4] (entry, row tile, col tile, 0) int32 on the GPU
void slab_transpose_bf16(at::Tensor src, at::Tensor dst, at::Tensor entries, at::Tensor tiles) {
  TORCH_CHECK(src.is_cuda() && src.is_contiguous() && src.scalar_type() == at::kFloat, "slab_transpose: f32 src");
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous() && dst.scalar_type() == at::kBFloat16, "slab_transpose: bf16 dst");
  TORCH_CHECK(entries.is_cuda() && entries.scalar_type() == at::kInt && entries.dim() == 2 && entries.size(1) == 4,
              "slab_transpose: entries [E][4] int32");
  TORCH_CHECK(tiles.is_cuda() && tiles.scalar_type() == at::kInt && tiles.dim() == 2 && tiles.size(1) == 4,
              "slab_transpose: tiles [T][4] int32");
  tdl::slab_transpose_bf16(src.data_ptr<float>(), reinterpret_cast<uint16_t*>(dst.data_ptr()),
                           entries.data_ptr<int>(), tiles.data_ptr<int>(), (int)tiles.size(0), cur_stream());
}
void slab_cast_bf16(at::Tensor src, at::Tensor dst) {
  TORCH_CHECK(src.is_cuda() && src.is_contiguous() && src.scalar_type() == at::kFloat, "slab_cast: f32 src");
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous() && dst.scalar_type() == at::kBFloat16, "slab_cast: bf16 dst");
  TORCH_CHECK(src.numel() == dst.numel() && src.numel() % 8 == 0, "slab_cast: sizes (multiple of 8)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "slab_cast: 16-byte aligned buffers");
  tdl::cast_bf16(src.data_ptr<float>(), reinterpret_cast<uint16_t*>(dst.data_ptr()), src.numel(), cur_stream());
}
void bf16_check(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.stride(1) == 1, what,
              " must be a 2-D row-major bf16 GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.stride(0) % 8 == 0, what,
              " must be 16-byte aligned (rows too)");
}

// C = alpha * op(A) op(B) (+ bias), see kernels/gemm.h; A/B given in their STORED [rows][cols] form:
// ta = 0: a is [M][K], ta = 1: a is [K][M]; tb = 0: b is [N][K], tb = 1: b is [K][N].
// out: f32 [M][N] (+= when accumulate) or None -> a new bf16 [M][N]
at::Tensor gemm_bf16(at::Tensor a, int64_t ta, at::Tensor b, int64_t tb, c10::optional<at::Tensor> bias,
                     c10::optional<at::Tensor> out, bool accumulate, double alpha) {
  bf16_check(a, "gemm: a");
  bf16_check(b, "gemm: b");
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t N = tb ? b.size(1) : b.size(0), Kb = tb ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm: inner dimensions differ");
  TORCH_CHECK(tdl::gemm_bf16_supported((int)M, (int)N, (int)K), "gemm: M, N, K must be multiples of 8");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == N &&
                    reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0,
                "gemm: bias must be a 16-byte aligned contiguous f32 [N]");
    bp = bias->data_ptr<float>();
  }
  if (out.has_value() && out->defined()) {
    auto& o = *out;
    TORCH_CHECK(o.is_cuda() && o.scalar_type() == at::kFloat && o.dim() == 2 && o.size(0) == M && o.size(1) == N &&
                    o.stride(1) == 1 && o.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(o.data_ptr()) % 16 == 0,
                "gemm: out must be a 16-byte aligned row-major f32 [M][N]");
    tdl::gemm_bf16((int)ta, (int)tb, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), (int)M, (int)N, (int)K,
                   o.data_ptr<float>(), nullptr, o.stride(0), bp, (float)alpha, accumulate, cur_stream());
    return o;
  }
  auto c = fresh({M, N}, a.options());
  tdl::gemm_bf16((int)ta, (int)tb, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), (int)M, (int)N, (int)K,
                 nullptr, c.data_ptr(), N, bp, (float)alpha, false, cur_stream());
  return c;
}

// ---- generic f32 GEMM / convolution (kernels/gemm_f32.hip) ----
void f32_check(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), what,
              " must be a contiguous f32 GPU tensor");
}
bool al16(const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

void f32_run(int mode, tdl::F32GemmArgs& a, const at::TensorOptions& o) {
  TORCH_CHECK(a.Kred > 0, "f32 gemm: empty reduction");
  // TDL_F32_SPLIT="kmin,cap" (A/B of the split plan; default 64,1024)
  static const std::pair<int, int> plan = [] {
    int kmin = 64, cap = 1024;
    if (const char* e = std::getenv("TDL_F32_SPLIT")) std::sscanf(e, "%d,%d", &kmin, &cap);
    return std::make_pair(kmin < 16 ? 16 : kmin, cap < 1 ? 1 : cap);
  }();
  tdl::f32_gemm_plan(a, plan.first, plan.second);
  at::Tensor ws;
  if (a.splits > 1) {
    ws = at::empty({(int64_t)a.splits * a.M * a.N}, o);
    a.ws = ws.data_ptr<float>();
  }
  tdl::f32_gemm_launch(mode, a, cur_stream());
}

const float* f32_bias(const c10::optional<at::Tensor>& bias, int64_t n) {
  if (!bias.has_value() || !bias->defined()) return nullptr;
  f32_check(*bias, "f32 gemm: bias");
  TORCH_CHECK(bias->numel() == n, "f32 gemm: bias must have N elements");
  return bias->data_ptr<float>();
}

// out: f32 [rows][cols] given (accumulate: +=) or a new tensor
at::Tensor f32_out(c10::optional<at::Tensor>& out, at::IntArrayRef shape, const at::TensorOptions& o) {
  if (out.has_value() && out->defined()) {
    f32_check(*out, "f32 gemm: out");
    TORCH_CHECK(out->sizes() == shape, "f32 gemm: out has the wrong shape");
    return *out;
  }
  return fresh(shape, o);
}

// ReLU mask of an operand (the layer's output, same layout as the operand): nullptr when absent
const float* f32_mask(const c10::optional<at::Tensor>& mask, const at::Tensor& like, const char* what) {
  if (!mask.has_value() || !mask->defined()) return nullptr;
  f32_check(*mask, what);
  TORCH_CHECK(mask->numel() == like.numel(), what, " must have the operand's shape");
  return mask->data_ptr<float>();
}
bool mask_al16(const c10::optional<at::Tensor>& mask) {
  return !mask.has_value() || !mask->defined() || al16(*mask);
}
// bias gradient target [n] (written, or += when accumulating)
float* f32_dbias(c10::optional<at::Tensor>& dbias, int64_t n) {
  if (!dbias.has_value() || !dbias->defined()) return nullptr;
  f32_check(*dbias, "f32 gemm: dbias");
  TORCH_CHECK(dbias->numel() == n, "f32 gemm: dbias must have ", n, " elements");
  return dbias->data_ptr<float>();
}

// C = op(A) op(B) (+ bias) in f32; ta = 0: a is [M][K], 1: [K][M]; tb = 0: b is [N][K], 1: [K][N].
// act = 1: ReLU epilogue.  amask / bmask: operand * (mask > 0) (ReLU backward).  dbias: a row of ones
// appended to A, its output row (the column sums of op(B): a bias gradient) written to dbias.
at::Tensor gemm_f32(at::Tensor a, int64_t ta, at::Tensor b, int64_t tb, c10::optional<at::Tensor> bias,
                    c10::optional<at::Tensor> out, bool accumulate, int64_t act, c10::optional<at::Tensor> amask,
                    c10::optional<at::Tensor> bmask, c10::optional<at::Tensor> dbias) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm_f32: 2-D operands");
  f32_check(a, "gemm_f32: a");
  f32_check(b, "gemm_f32: b");
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t N = tb ? b.size(1) : b.size(0), Kb = tb ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm_f32: inner dimensions differ");
  auto c = f32_out(out, {M, N}, a.options());
  tdl::F32GemmArgs g{};
  g.a = a.data_ptr<float>();
  g.b = b.data_ptr<float>();
  g.na = a.numel();
  g.nb = b.numel();
  g.out = c.data_ptr<float>();
  g.bias = f32_bias(bias, N);
  g.sam = ta ? 1 : a.stride(0);
  g.sak = ta ? a.stride(0) : 1;
  g.sbk = tb ? b.stride(0) : 1;
  g.sbn = tb ? 1 : b.stride(0);
  g.M = (int)M;
  g.N = (int)N;
  g.Kred = (int)K;
  g.ldo = N;
  g.accumulate = accumulate && out.has_value() && out->defined();
  g.act = (int)act;
  g.amask = f32_mask(amask, a, "gemm_f32: amask");
  g.bmask = f32_mask(bmask, b, "gemm_f32: bmask");
  g.vec_a = g.sak == 1 && g.sam % 4 == 0 && K % 4 == 0 && al16(a) && mask_al16(amask);
  g.vec_b = g.sbn == 1 && g.sbk % 4 == 0 && N % 4 == 0 && al16(b) && mask_al16(bmask);
  g.dbias = f32_dbias(dbias, N);
  if (g.dbias != nullptr) {
    TORCH_CHECK(act == 0, "gemm_f32: dbias with an activation epilogue");
    g.ones_m = g.M++;  // the appended row of ones
  }
  f32_run(tdl::kF32Gemm, g, a.options());
  return c;
}

tdl::F32ConvGeom f32_geom(const at::Tensor& x_like, int64_t k, int64_t r, int64_t s, int64_t oh, int64_t ow, int64_t sh,
                          int64_t sw, int64_t pt, int64_t pl, int64_t dh, int64_t dw) {
  tdl::F32ConvGeom g{};
  g.n = (int)x_like.size(0);
  g.h = (int)x_like.size(1);
  g.w = (int)x_like.size(2);
  g.c = (int)x_like.size(3);
  g.k = (int)k;
  g.r = (int)r;
  g.s = (int)s;
  g.oh = (int)oh;
  g.ow = (int)ow;
  g.sh = (int)sh;
  g.sw = (int)sw;
  g.pt = (int)pt;
  g.pl = (int)pl;
  g.dh = (int)dh;
  g.dw = (int)dw;
  TORCH_CHECK(sh > 0 && sw > 0 && dh > 0 && dw > 0, "f32 conv: strides and dilations must be positive");
  return g;
}

// y[N][OH][OW][K] = conv(x NHWC, w HWIO) (+ bias); padding (pt, pl) top / left, the rest implied by OH / OW
at::Tensor conv_f32_fwd(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, int64_t oh, int64_t ow, int64_t sh,
                        int64_t sw, int64_t pt, int64_t pl, int64_t dh, int64_t dw, int64_t act) {
  f32_check(x, "conv_f32_fwd: x");
  f32_check(w, "conv_f32_fwd: w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(2) == x.size(3), "conv_f32_fwd: x NHWC, w [R][S][C][K]");
  const int64_t K = w.size(3);
  auto y = fresh({x.size(0), oh, ow, K}, x.options());
  tdl::F32GemmArgs g{};
  g.g = f32_geom(x, K, w.size(0), w.size(1), oh, ow, sh, sw, pt, pl, dh, dw);
  g.a = x.data_ptr<float>();
  g.b = w.data_ptr<float>();
  g.na = x.numel();
  g.nb = w.numel();
  g.out = y.data_ptr<float>();
  g.bias = f32_bias(bias, K);
  g.M = (int)(x.size(0) * oh * ow);
  g.N = (int)K;
  g.Kred = (int)(w.size(0) * w.size(1) * x.size(3));
  g.ldo = K;
  g.vec_a = x.size(3) % 4 == 0 && al16(x);
  g.vec_b = K % 4 == 0 && al16(w);
  g.act = (int)act;
  f32_run(tdl::kF32ConvFwd, g, x.options());
  return y;
}

// conv_f32_fwd followed by a 2x2 / stride-2 'valid' max pool, in one launch (the pool in the GEMM's
// epilogue, rows ordered by pool window): returns [y [N][OH][OW][K], pooled [N][OH/2][OW/2][K], argmax
// (uint8 window positions, the maxpool_fwd format, for maxpool_bwd)].  With odd OH / OW the last output
// row / column belongs to no window and is not computed (its y entries are left unset: their gradient
// is zero, and the backward only selects on them).
std::vector<at::Tensor> conv_f32_fwd_pool(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, int64_t oh,
                                          int64_t ow, int64_t sh, int64_t sw, int64_t pt, int64_t pl, int64_t dh,
                                          int64_t dw, int64_t act) {
  f32_check(x, "conv_f32_fwd_pool: x");
  f32_check(w, "conv_f32_fwd_pool: w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(2) == x.size(3), "conv_f32_fwd_pool: x NHWC, w [R][S][C][K]");
  TORCH_CHECK(oh >= 2 && ow >= 2, "conv_f32_fwd_pool: the output must hold at least one 2x2 window");
  const int64_t K = w.size(3), PH = oh / 2, PW = ow / 2;
  auto y = at::empty({x.size(0), oh, ow, K}, x.options());
  auto p = at::empty({x.size(0), PH, PW, K}, x.options());
  auto arg = at::empty({x.size(0), PH, PW, K}, x.options().dtype(at::kByte));
  tdl::F32GemmArgs g{};
  g.g = f32_geom(x, K, w.size(0), w.size(1), oh, ow, sh, sw, pt, pl, dh, dw);
  g.a = x.data_ptr<float>();
  g.b = w.data_ptr<float>();
  g.na = x.numel();
  g.nb = w.numel();
  g.out = y.data_ptr<float>();
  g.bias = f32_bias(bias, K);
  g.M = (int)(x.size(0) * PH * PW * 4);
  g.N = (int)K;
  g.Kred = (int)(w.size(0) * w.size(1) * x.size(3));
  g.ldo = K;
  g.vec_a = x.size(3) % 4 == 0 && al16(x);
  g.vec_b = K % 4 == 0 && al16(w);
  g.act = (int)act;
  g.pool = 1;
  g.pool_h = (int)PH;
  g.pool_w = (int)PW;
  g.plan_m = (int)(x.size(0) * oh * ow);  // the unfused conv's split: the same partial sums
  g.pout = p.data_ptr<float>();
  g.parg = arg.data_ptr<uint8_t>();
  f32_run(tdl::kF32ConvFwd, g, x.options());
  return {y, p, arg};
}

// dx[N][H][W][C] of a conv with dy [N][OH][OW][K] and wt = w as [R][S][K][C]
// pooled output gradient (pin_arg given: the backward of conv_f32_fwd_pool): dy = the pool's output gradient
// [N][PH][PW][K], dy_mask = the pooled maximum, pin_arg = its argmax, (out_h, out_w) = the conv's output size
static void f32_pin(tdl::F32GemmArgs& g, const at::Tensor& dy, const c10::optional<at::Tensor>& pin_arg,
                    const c10::optional<at::Tensor>& dy_mask, int64_t out_h, int64_t out_w, const char* what) {
  if (!pin_arg.has_value() || !pin_arg->defined()) return;
  TORCH_CHECK(pin_arg->is_cuda() && pin_arg->scalar_type() == at::kByte && pin_arg->is_contiguous() &&
                  pin_arg->sizes() == dy.sizes(), what, ": pin_arg must be a contiguous uint8 tensor shaped like dy");
  TORCH_CHECK(dy_mask.has_value() && dy_mask->defined(), what, ": pin_arg needs dy_mask (the pooled maximum)");
  TORCH_CHECK(out_h >= 2 * dy.size(1) && out_w >= 2 * dy.size(2) && out_h <= 2 * dy.size(1) + 1 &&
                  out_w <= 2 * dy.size(2) + 1, what, ": (out_h, out_w) must be the pooled conv's output size");
  g.pin_arg = pin_arg->data_ptr<uint8_t>();
  g.pool_h = (int)dy.size(1);
  g.pool_w = (int)dy.size(2);
}

at::Tensor conv_f32_dgrad(at::Tensor dy, at::Tensor wt, int64_t h, int64_t wd, int64_t sh, int64_t sw, int64_t pt,
                          int64_t pl, int64_t dh, int64_t dw, c10::optional<at::Tensor> dy_mask, bool w_hwio,
                          c10::optional<at::Tensor> pin_arg, int64_t out_h, int64_t out_w) {
  f32_check(dy, "conv_f32_dgrad: dy");
  f32_check(wt, "conv_f32_dgrad: wt");
  // wt: [R][S][K][C], or (w_hwio) the forward kernel [R][S][C][K] read transposed in the kernel
  TORCH_CHECK(dy.dim() == 4 && wt.dim() == 4 && wt.size(w_hwio ? 3 : 2) == dy.size(3),
              "conv_f32_dgrad: dy NHWC, wt [R][S][K][C] (or w [R][S][C][K] with w_hwio)");
  const int64_t C = wt.size(w_hwio ? 2 : 3), K = dy.size(3);
  auto dx = fresh({dy.size(0), h, wd, C}, dy.options());
  tdl::F32GemmArgs g{};
  const bool pin = pin_arg.has_value() && pin_arg->defined();
  g.g = f32_geom(dx, K, wt.size(0), wt.size(1), pin ? out_h : dy.size(1), pin ? out_w : dy.size(2), sh, sw, pt, pl,
                 dh, dw);
  f32_pin(g, dy, pin_arg, dy_mask, out_h, out_w, "conv_f32_dgrad");
  g.a = dy.data_ptr<float>();
  g.b = wt.data_ptr<float>();
  g.na = dy.numel();
  g.nb = wt.numel();
  g.out = dx.data_ptr<float>();
  g.M = (int)(dy.size(0) * h * wd);
  g.N = (int)C;
  g.Kred = (int)(wt.size(0) * wt.size(1) * K);
  g.ldo = C;
  g.amask = f32_mask(dy_mask, dy, "conv_f32_dgrad: dy_mask");
  g.vec_a = K % 4 == 0 && al16(dy) && mask_al16(dy_mask);
  g.vec_b = !w_hwio && C % 4 == 0 && al16(wt);
  g.b_hwio = w_hwio ? 1 : 0;
  f32_run(tdl::kF32ConvDgrad, g, dy.options());
  return dx;
}

// dW HWIO [R][S][C][K] of a conv with x NHWC and dy [N][OH][OW][K] (into / += out when given)
at::Tensor conv_f32_wgrad(at::Tensor x, at::Tensor dy, int64_t r, int64_t s, int64_t sh, int64_t sw, int64_t pt,
                          int64_t pl, int64_t dh, int64_t dw, c10::optional<at::Tensor> out, bool accumulate,
                          c10::optional<at::Tensor> dy_mask, c10::optional<at::Tensor> dbias,
                          c10::optional<at::Tensor> pin_arg, int64_t out_h, int64_t out_w) {
  f32_check(x, "conv_f32_wgrad: x");
  f32_check(dy, "conv_f32_wgrad: dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && x.size(0) == dy.size(0), "conv_f32_wgrad: x, dy NHWC");
  const int64_t C = x.size(3), K = dy.size(3);
  auto dW = f32_out(out, {r, s, C, K}, x.options());
  tdl::F32GemmArgs g{};
  const bool pin = pin_arg.has_value() && pin_arg->defined();
  const int64_t oh = pin ? out_h : dy.size(1), ow = pin ? out_w : dy.size(2);
  g.g = f32_geom(x, K, r, s, oh, ow, sh, sw, pt, pl, dh, dw);
  f32_pin(g, dy, pin_arg, dy_mask, out_h, out_w, "conv_f32_wgrad");
  g.a = dy.data_ptr<float>();
  g.b = x.data_ptr<float>();
  g.na = dy.numel();
  g.nb = x.numel();
  g.out = dW.data_ptr<float>();
  g.M = (int)K;
  g.N = (int)(r * s * C);
  TORCH_CHECK(dy.size(0) * oh * ow < (int64_t)1 << 31, "conv_f32_wgrad: reduction too long");
  g.Kred = (int)(dy.size(0) * oh * ow);
  g.ldo = K;
  g.trans_out = 1;
  g.accumulate = accumulate && out.has_value() && out->defined();
  g.vec_b = C % 4 == 0 && al16(x);
  g.amask = f32_mask(dy_mask, dy, "conv_f32_wgrad: dy_mask");
  g.dbias = f32_dbias(dbias, K);
  if (g.dbias != nullptr) g.ones_n = g.N++;  // the appended column of ones: sum over pixels of dy
  f32_run(tdl::kF32ConvWgrad, g, x.options());
  return dW;
}

at::Tensor gap_fwd(at::Tensor x) {
  conv_check(x, "gap: x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "gap: NHWC with C % 8 == 0");
  auto y = fresh({x.size(0), x.size(3)}, x.options());
  tdl::gap_fwd_bf16(x.data_ptr(), y.data_ptr(), (int)x.size(0), (int)(x.size(1) * x.size(2)), (int)x.size(3),
                    cur_stream());
  return y;
}

at::Tensor gap_bwd(at::Tensor dy, int64_t h, int64_t w) {
  conv_check(dy, "gap: dy");
  TORCH_CHECK(dy.dim() == 2 && dy.size(1) % 8 == 0, "gap: dy [N][C], C % 8 == 0");
  auto dx = fresh({dy.size(0), h, w, dy.size(1)}, dy.options());
  tdl::gap_bwd_bf16(dy.data_ptr(), dx.data_ptr(), (int)dy.size(0), (int)(h * w), (int)dy.size(1), cur_stream());
  return dx;
}
std::vector<at::Tensor> xent_fwd(at::Tensor z, at::Tensor labels) {
  TORCH_CHECK(z.is_cuda() && z.is_contiguous() && z.scalar_type() == at::kFloat && z.dim() == 2, "xent: f32 [N][K] logits");
  TORCH_CHECK(labels.is_cuda() && labels.is_contiguous() && labels.scalar_type() == at::kLong &&
                  labels.numel() == z.size(0), "xent: int64 [N] labels");
  auto loss = fresh({z.size(0)}, z.options());
  auto lse = fresh({z.size(0)}, z.options());
  tdl::softmax_xent_fwd(z.data_ptr<float>(), reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()), (int)z.size(0), (int)z.size(1),
                        loss.data_ptr<float>(), lse.data_ptr<float>(), cur_stream());
  return {loss, lse};
}

double* f64_scalar(const c10::optional<at::Tensor>& t, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kDouble && t->numel() == 1, what, ": f64 GPU scalar expected");
  return t->data_ptr<double>();
}

// the generic engine's fused loss head: (loss [] = sum / gn, dz [N][K] = (softmax - onehot) / gn), metric
// accumulators advanced in place
std::vector<at::Tensor> xent_head(at::Tensor z, at::Tensor labels, double gn, c10::optional<at::Tensor> lt_total,
                                  c10::optional<at::Tensor> lt_count, c10::optional<at::Tensor> acc_total,
                                  c10::optional<at::Tensor> acc_count) {
  TORCH_CHECK(z.is_cuda() && z.is_contiguous() && z.scalar_type() == at::kFloat && z.dim() == 2, "xent_head: f32 [N][K] logits");
  TORCH_CHECK(labels.is_cuda() && labels.is_contiguous() && labels.scalar_type() == at::kLong &&
                  labels.numel() == z.size(0), "xent_head: int64 [N] labels");
  TORCH_CHECK(gn > 0, "xent_head: global batch must be positive");
  auto loss = at::empty({}, z.options());
  auto dz = fresh(z.sizes(), z.options());
  // one workgroup up to 64K logits (the reference CNN's 64 x 10), else per-row waves + a finishing sum
  at::Tensor ws;
  if (z.numel() > 65536) ws = at::empty({2 * z.size(0)}, z.options());
  tdl::xent_head(z.data_ptr<float>(), reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()), (int)z.size(0),
                 (int)z.size(1), gn, loss.data_ptr<float>(), dz.data_ptr<float>(), f64_scalar(lt_total, "lt_total"),
                 f64_scalar(lt_count, "lt_count"), f64_scalar(acc_total, "acc_total"), f64_scalar(acc_count, "acc_count"),
                 ws.defined() ? ws.data_ptr<float>() : nullptr, cur_stream());
  return {loss, dz};
}

at::Tensor xent_bwd(at::Tensor z, at::Tensor labels, at::Tensor g) {
  TORCH_CHECK(z.is_cuda() && z.is_contiguous() && z.scalar_type() == at::kFloat && z.dim() == 2, "xent: f32 [N][K] logits");
  TORCH_CHECK(labels.is_contiguous() && labels.scalar_type() == at::kLong && labels.numel() == z.size(0), "xent: labels");
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && g.scalar_type() == at::kFloat && g.numel() == z.size(0), "xent: g");
  auto dz = fresh(z.sizes(), z.options());
  tdl::softmax_xent_bwd(z.data_ptr<float>(), reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()), (int)z.size(0), (int)z.size(1),
                        g.data_ptr<float>(), dz.data_ptr<float>(), cur_stream());
  return dz;
}
}  // namespace

void register_ops(pybind11::module& m) {
  m.def("xent_fwd", &xent_fwd, "sparse softmax cross-entropy forward: (loss, logsumexp)");
  m.def("xent_bwd", &xent_bwd, "sparse softmax cross-entropy backward: (softmax - onehot) * g");
  m.def("xent_head", &xent_head, "fused loss head: mean-reduced sparse softmax cross-entropy, its dlogits and "
        "the loss / accuracy metric accumulators", pybind11::arg("z"), pybind11::arg("labels"), pybind11::arg("gn"),
        pybind11::arg("lt_total") = pybind11::none(), pybind11::arg("lt_count") = pybind11::none(),
        pybind11::arg("acc_total") = pybind11::none(), pybind11::arg("acc_count") = pybind11::none());
  m.def("gemm_bf16", &gemm_bf16, "bf16 MFMA GEMM with either storage per operand (Dense fwd / dgrad / wgrad)",
        pybind11::arg("a"), pybind11::arg("ta"), pybind11::arg("b"), pybind11::arg("tb"),
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("accumulate") = false, pybind11::arg("alpha") = 1.0);
  m.def("gemm_f32", &gemm_f32, "f32 MFMA GEMM (v_mfma_f32_16x16x4_f32) with either storage per operand; "
        "ReLU epilogue, ReLU-masked operands, bias gradient as an appended row of ones",
        pybind11::arg("a"), pybind11::arg("ta"), pybind11::arg("b"), pybind11::arg("tb"),
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("accumulate") = false, pybind11::arg("act") = 0, pybind11::arg("amask") = pybind11::none(),
        pybind11::arg("bmask") = pybind11::none(), pybind11::arg("dbias") = pybind11::none());
  m.def("conv_f32_fwd_pool", &conv_f32_fwd_pool,
        "conv_f32_fwd + 2x2/2 'valid' max pool in the epilogue: [y, pooled, argmax]", pybind11::arg("x"),
        pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("oh"), pybind11::arg("ow"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("dh") = 1,
        pybind11::arg("dw") = 1, pybind11::arg("act") = 0);
  m.def("conv_f32_fwd", &conv_f32_fwd, "NHWC f32 implicit-GEMM convolution forward, any geometry (act 1: + ReLU)",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("oh"), pybind11::arg("ow"),
        pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("dh") = 1,
        pybind11::arg("dw") = 1, pybind11::arg("act") = 0);
  m.def("conv_f32_dgrad", &conv_f32_dgrad, "NHWC f32 convolution input gradient, any geometry (wt: [R][S][K][C]); "
        "dy_mask: dy * (mask > 0)",
        pybind11::arg("dy"), pybind11::arg("wt"), pybind11::arg("h"), pybind11::arg("w"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("dh") = 1, pybind11::arg("dw") = 1,
        pybind11::arg("dy_mask") = pybind11::none(), pybind11::arg("w_hwio") = false,
        pybind11::arg("pin_arg") = pybind11::none(), pybind11::arg("out_h") = 0, pybind11::arg("out_w") = 0);
  m.def("conv_f32_wgrad", &conv_f32_wgrad, "NHWC f32 convolution weight gradient (HWIO), deterministic split-K; "
        "dy_mask: dy * (mask > 0); dbias: the bias gradient from an appended column of ones",
        pybind11::arg("x"), pybind11::arg("dy"), pybind11::arg("r"), pybind11::arg("s"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("dh") = 1, pybind11::arg("dw") = 1,
        pybind11::arg("out") = pybind11::none(), pybind11::arg("accumulate") = false,
        pybind11::arg("dy_mask") = pybind11::none(), pybind11::arg("dbias") = pybind11::none(),
        pybind11::arg("pin_arg") = pybind11::none(), pybind11::arg("out_h") = 0, pybind11::arg("out_w") = 0);
  m.def("gap_fwd", &gap_fwd, "NHWC bf16 global average pooling");
  m.def("gap_bwd", &gap_bwd, "NHWC bf16 global average pooling backward");
  m.def("slab_cast_bf16", &slab_cast_bf16, "f32 -> bf16 copy of a whole weight slab (one launch)");
  m.def("bn_set_tuning", &tdl::bn_set_tuning, "BN kernel sweep hooks (max_parts, elem_blocks, elem_unroll; 0 = keep)");
  m.def("bn_set_elementwise", &tdl::bn_set_elementwise,
        "BN elementwise kernel family A/B hook (kind 0 grid-stride / 1 blocked, vectors per thread 2/4/8)");
  m.def("slab_transpose_bf16", &slab_transpose_bf16, "HWIO f32 conv kernels -> OHWI bf16, all in one launch");
  m.def("conv_dgrad_bn", &conv_dgrad_bn, "stride-1 conv input gradient + fused BN->Add->ReLU backward (dz, part[, part2])",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("h"), pybind11::arg("wd"), pybind11::arg("pt"),
        pybind11::arg("pl"), pybind11::arg("residual"), pybind11::arg("bn_y"), pybind11::arg("bn_x"),
        pybind11::arg("bn_x2") = pybind11::none(), pybind11::arg("bn_stats") = pybind11::none());
  m.def("conv_dgrad_s2_bn", &conv_dgrad_s2_bn,
        "1x1 stride-2 conv input gradient + fused BN->Add->ReLU backward (dz, part[, part2])", pybind11::arg("dy"),
        pybind11::arg("w"), pybind11::arg("h"), pybind11::arg("wd"), pybind11::arg("residual"), pybind11::arg("bn_y"),
        pybind11::arg("bn_x"), pybind11::arg("bn_x2") = pybind11::none(), pybind11::arg("bn_stats") = pybind11::none());
  m.def("conv_dgrad_s2", &conv_dgrad_s2, "NHWC bf16 1x1 stride-2 convolution input gradient (MFMA)",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("h"), pybind11::arg("wd"),
        pybind11::arg("residual") = pybind11::none());
  m.def("conv_wgrad", &conv_wgrad, "NHWC bf16 convolution weight gradient (MFMA, transposed LDS reads, split-K)",
        pybind11::arg("x"), pybind11::arg("dy"), pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("accumulate") = false, pybind11::arg("plan") = std::vector<int64_t>{},
        pybind11::arg("in_bn") = pybind11::none());
  m.def("conv_wgrad_plans", &conv_wgrad_plans, "weight-gradient candidate plans, best first: [[wmw, wnw, chunk, nsplit, kind]]",
        pybind11::arg("x_shape"), pybind11::arg("dy_shape"), pybind11::arg("kh"), pybind11::arg("kw"),
        pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("max_plans"),
        pybind11::arg("in_bn") = false);
  m.def("conv_force_tile", &tdl::conv_force_tile, "conv tile sweep hook (0 = heuristic)");
  m.def("conv_force_impl", &tdl::conv_force_impl,
        "conv main loop A/B hook: 1 v1 register staged, 2 default selection, 3 LDS-DMA ring, 4/5 dma1 at 4/3 waves "
        "per SIMD on 16x16x32 MFMAs, 6 dma1 on 32x32x16 MFMAs everywhere");
  m.def("f32_reduce16", &tdl::f32_reduce16,
        "f32 split-K reduce A/B hook: 16 outputs per wave over many slices (True, default) or one output per wave");
  m.def("conv_force_halo", &tdl::conv_force_halo, "halo (input-reuse) main loop for stride-1 multi-tap convs: 1 on, 0 off");
  m.def("conv_force_mfma", &tdl::conv_force_mfma, "dma1 MFMA form: 32 (32x32x16, default) or 16 (16x16x32)");
  m.def("conv_wgrad3x3_set_rows", &tdl::conv_wgrad3x3_set_rows, "3x3 row-kernel wgrad: output rows per slice (0 = auto)");
  m.def("conv_wgrad_force_single", &tdl::conv_wgrad_force_single,
        "weight-gradient A/B hook: single LDS stage at 3 waves/SIMD (True) or double-buffered (False, default)");
  m.def("maxpool_force_generic", &tdl::maxpool_force_generic,
        "max-pool A/B hook: generic window loops (True, default) or the unrolled 3x3 stride-2 kernels (False)");
  m.def("maxpool_w2", &tdl::maxpool_w2,
        "max-pool backward A/B hook: 2x2 stride-2 unpadded windows in scatter form (True, default) or the gather form");
  m.def("conv_force_depth", &tdl::conv_force_depth, "conv main-loop A/B hook: 0 single stage, 1/2 prefetch depth, 3 depth 2 without the short-reduction single-stage variant");
  m.def("stem_fwd", &stem_fwd, "small-channel stride-2 conv (ResNet stem): (y, packed x[, BN part])",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("pt"), pybind11::arg("pb"), pybind11::arg("pl"),
        pybind11::arg("pr"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("stats") = false);
  m.def("stem_wgrad", &stem_wgrad, "stem conv weight gradient from the packed image", pybind11::arg("xp"),
        pybind11::arg("dy"), pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("c"), pybind11::arg("sh"),
        pybind11::arg("out") = pybind11::none(), pybind11::arg("accumulate") = false);
  m.def("conv_fwd", &conv_fwd, "NHWC bf16 implicit-GEMM convolution forward (MFMA); in_bn: over relu(bn(x))",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("oh"), pybind11::arg("ow"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("in_bn") = pybind11::none());
  m.def("conv_fwd_stats", &conv_fwd_stats, "conv forward + batch-norm partial channel sums of its output",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("oh"), pybind11::arg("ow"), pybind11::arg("sh"),
        pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("in_bn") = pybind11::none());
  m.def("conv_dgrad", &conv_dgrad, "NHWC bf16 implicit-GEMM stride-1 convolution input gradient (MFMA)",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("h"), pybind11::arg("wd"), pybind11::arg("pt"),
        pybind11::arg("pl"), pybind11::arg("residual") = pybind11::none());
  m.def("gather_xy", &gather_xy, "a batch of (feature row, label) pairs of a device-resident dataset, one launch");
  m.def("gather_rows", &gather_rows, "row gather (+u8->f32 scale) of a device-resident dataset");
  m.def("gather_labels", &gather_labels);
  m.def("bn_forward_train", &bn_forward_train, "NHWC batch-norm training forward (+relu)", pybind11::arg("x"),
        pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("moving_mean"), pybind11::arg("moving_var"),
        pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("relu") = false,
        pybind11::arg("residual") = pybind11::none(), pybind11::arg("mean_off") = pybind11::none(),
        pybind11::arg("part") = pybind11::none());
  m.def("maxpool_fwd", &maxpool_fwd, "NHWC max pool forward (+argmax)", pybind11::arg("x"), pybind11::arg("kh"),
        pybind11::arg("kw"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("pt"), pybind11::arg("pl"),
        pybind11::arg("OH"), pybind11::arg("OW"), pybind11::arg("pad_zero"), pybind11::arg("bn_stats") = pybind11::none());
  m.def("maxpool_bwd_bn", &maxpool_bwd_bn, "NHWC max pool backward fused with the BN -> ReLU group's mask and sums");
  m.def("bn_stats_train", &bn_stats_train, "NHWC batch-norm training statistics only ([4][C])", pybind11::arg("x"),
        pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("moving_mean"), pybind11::arg("moving_var"),
        pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("mean_off") = pybind11::none(),
        pybind11::arg("part") = pybind11::none());
  m.def("maxpool_bwd", &maxpool_bwd, "NHWC max pool backward (gather form)");
  m.def("bn_backward", &bn_backward, "NHWC batch-norm training backward", pybind11::arg("dy"), pybind11::arg("x"),
        pybind11::arg("y"), pybind11::arg("gamma"), pybind11::arg("stats"), pybind11::arg("mode"),
        pybind11::arg("dgamma_out") = pybind11::none(), pybind11::arg("dbeta_out") = pybind11::none(),
        pybind11::arg("part") = pybind11::none());
}
