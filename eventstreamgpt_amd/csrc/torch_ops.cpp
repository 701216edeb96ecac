// PyTorch-ROCm custom operators (TORCH_LIBRARY(esgpt)) over the C ABI of libesgpt_amd.so.
//
// The reference (Jwoo5/EventStreamGPT) swaps ATen ops inside its module methods; the drop-in modules of this package
// call these operators instead (torch.ops.esgpt.*): the input layer (data_embedding_layer.py:351-708,
// transformer.py:594-672, 903-936), attention (transformer.py:171-217), the block elementwise stages and projections
// (transformer.py:350-461), the generative heads + losses (model_output.py:1253-1721) and AdamW
// (generative_modeling.py:460-485). Each operator allocates its outputs and workspaces with torch's caching
// allocator on the inputs' device and launches on torch's current HIP stream; no host synchronisation.
//
// Data-dependent errors go to a caller-owned device error block and split-K / cross-workgroup tickets to a
// caller-owned counter array (eventstreamgpt_amd/kernels.py: err_word / tickets). Both are side channels: the
// tickets are left as found, the error block only accumulates flags that the Python layer turns into the
// reference's exceptions. The schemas therefore list them as plain inputs, keeping every differentiable operator
// functional (torch.library.register_autograd requires that). Fake (meta) kernels and autograd formulas are
// registered from Python (eventstreamgpt_amd/ops.py).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <vector>

#include "../../include/esgpt_amd.h"

namespace {

using at::Tensor;
using c10::optional;

void* stream_of(const Tensor& t) {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

void check(int status, const char* what) {
  TORCH_CHECK(status == ESGPT_OK, "eventstreamgpt_amd: ", what, " failed (status ", status,
              status == ESGPT_ERR_INVALID_ARG ? ": invalid argument" :
              status == ESGPT_ERR_LAUNCH ? ": launch failure" :
              status == ESGPT_ERR_UNSUPPORTED ? ": unsupported configuration" : "", ")");
}

template <typename T>
T* ptr(const Tensor& t) { return t.defined() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr; }
template <typename T>
T* optr(const optional<Tensor>& t) { return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr; }

int dtype_code(at::ScalarType s) {
  if (s == at::kFloat) return ESGPT_F32;
  if (s == at::kBFloat16) return ESGPT_BF16;
  TORCH_CHECK(false, "eventstreamgpt_amd: unsupported activation dtype ", s);
}

void require_hip(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), "eventstreamgpt_amd: ", what, " must be a HIP device tensor (there is no CPU path)");
}

// ---- batch descriptor: PytorchBatch fields in the ABI's dtypes (contiguous copies only when needed) ----------
struct Batch {
  Tensor em, td, tm, di, dm, dv, dvm, si, sm;
  esgpt_batch b;
};

Tensor as(const Tensor& t, at::ScalarType s) { return t.to(s).contiguous(); }
Tensor as_opt(const optional<Tensor>& t, at::ScalarType s) {
  return (t.has_value() && t->defined()) ? as(*t, s) : Tensor();
}

Batch make_batch(const Tensor& event_mask, const Tensor& time_delta, const optional<Tensor>& time,
                 const Tensor& dyn_idx, const Tensor& dyn_meas, const Tensor& dyn_vals, const Tensor& dyn_vmask,
                 const optional<Tensor>& st_idx, const optional<Tensor>& st_meas) {
  require_hip(event_mask, "the batch");
  Batch x;
  x.em = as(event_mask, at::kBool);
  x.td = as(time_delta, at::kFloat);
  x.tm = as_opt(time, at::kFloat);
  x.di = as(dyn_idx, at::kLong);
  x.dm = as(dyn_meas, at::kLong);
  x.dv = as(dyn_vals, at::kFloat);
  x.dvm = as(dyn_vmask, at::kBool);
  x.si = as_opt(st_idx, at::kLong);
  x.sm = as_opt(st_meas, at::kLong);
  TORCH_CHECK(x.di.dim() == 3, "dynamic_indices must be [B, L, M]");
  x.b.dyn_idx = ptr<const int64_t>(x.di);
  x.b.dyn_meas = ptr<const int64_t>(x.dm);
  x.b.dyn_vals = ptr<const float>(x.dv);
  x.b.dyn_vmask = ptr<const uint8_t>(x.dvm);
  x.b.event_mask = ptr<const uint8_t>(x.em);
  x.b.time_delta = ptr<const float>(x.td);
  x.b.time_abs = x.tm.defined() ? ptr<const float>(x.tm) : nullptr;
  x.b.st_idx = x.si.defined() ? ptr<const int64_t>(x.si) : nullptr;
  x.b.st_meas = x.sm.defined() ? ptr<const int64_t>(x.sm) : nullptr;
  x.b.B = x.di.size(0);
  x.b.L = x.di.size(1);
  x.b.M = x.di.size(2);
  x.b.S = x.si.defined() ? x.si.size(1) : 0;
  return x;
}

// buckets: [] (un-bucketed) or [G, cat_bits[8], num_bits[8]] (bit patterns as int64)
bool make_buckets(at::IntArrayRef v, esgpt_buckets& k) {
  if (v.empty()) return false;
  TORCH_CHECK(v.size() == 17, "buckets must be [G, cat_bits x8, num_bits x8]");
  k.G = v[0];
  for (int g = 0; g < 8; ++g) {
    k.cat_bits[g] = static_cast<uint64_t>(v[1 + g]);
    k.num_bits[g] = static_cast<uint64_t>(v[9 + g]);
  }
  return true;
}

#define BATCH_ARGS                                                                                         \
  const Tensor &event_mask, const Tensor &time_delta, const optional<Tensor> &time, const Tensor &dyn_idx,  \
      const Tensor &dyn_meas, const Tensor &dyn_vals, const Tensor &dyn_vmask, const optional<Tensor> &st_idx, \
      const optional<Tensor> &st_meas
#define BATCH_PASS event_mask, time_delta, time, dyn_idx, dyn_meas, dyn_vals, dyn_vmask, st_idx, st_meas
#define BATCH_SCHEMA                                                                                    \
  "Tensor event_mask, Tensor time_delta, Tensor? time, Tensor dyn_idx, Tensor dyn_meas, Tensor dyn_vals, " \
  "Tensor dyn_vmask, Tensor? st_idx, Tensor? st_meas"

// ---- input layer ---------------------------------------------------------------------------------------------
// The temporal encoding's event times (the exclusive masked cumsum of time_delta) computed once per subject by
// esgpt_event_times and handed to the kernel as absolute times (flags gains ESGPT_EMB_TIME_ABS); the kernels would
// otherwise sum each event's prefix themselves. No-op when the batch carries absolute times or no encoding is asked.
Tensor event_times_for(Batch& bt, int64_t& flags, const Tensor& like) {
  if (!(flags & ESGPT_EMB_TIME) || (flags & ESGPT_EMB_TIME_ABS)) return Tensor();
  Tensor t = at::empty({bt.b.B, bt.b.L}, like.options().dtype(at::kFloat));
  check(esgpt_event_times(&bt.b, ptr<float>(t), stream_of(like)), "event_times");
  bt.b.time_abs = ptr<const float>(t);
  flags |= ESGPT_EMB_TIME_ABS;
  return t;
}

Tensor embed_joint(const Tensor& table, BATCH_ARGS, at::IntArrayRef buckets, const optional<Tensor>& sin_div,
                   const optional<Tensor>& cos_div, int64_t flags, double static_w, double dynamic_w, int64_t G,
                   const Tensor& err) {
  const c10::DeviceGuard guard(table.device());
  Batch bt = make_batch(BATCH_PASS);
  esgpt_buckets bk;
  const bool has_bk = make_buckets(buckets, bk);
  Tensor tab = as(table, at::kFloat);
  const int64_t V = tab.size(0), D = tab.size(1);
  Tensor out = at::empty({bt.b.B, bt.b.L, G, D}, tab.options());
  Tensor times = event_times_for(bt, flags, tab);
  check(esgpt_embed_joint_fwd(&bt.b, has_bk ? &bk : nullptr, ptr<const float>(tab), V, D, optr<const float>(sin_div),
                              optr<const float>(cos_div), (int)flags, (float)static_w, (float)dynamic_w,
                              ptr<float>(out), ptr<int32_t>(err), stream_of(tab)),
        "embed_joint");
  return out;
}

Tensor embed_split_bags(const Tensor& cat_table, const Tensor& num_table, BATCH_ARGS, at::IntArrayRef buckets,
                        int64_t flags, double cat_scale, double num_scale, double static_scale, int64_t G,
                        const Tensor& err) {
  const c10::DeviceGuard guard(cat_table.device());
  Batch bt = make_batch(BATCH_PASS);
  esgpt_buckets bk;
  const bool has_bk = make_buckets(buckets, bk);
  Tensor ct = as(cat_table, at::kFloat), nt = as(num_table, at::kFloat);
  const int64_t V = ct.size(0), Dc = ct.size(1), Dn = nt.size(1);
  Tensor x = at::empty({bt.b.B * bt.b.L * G, Dc + Dn}, ct.options());
  check(esgpt_embed_split_bags_fwd(&bt.b, has_bk ? &bk : nullptr, ptr<const float>(ct), Dc, ptr<const float>(nt), Dn,
                                   V, (int)flags, (float)cat_scale, (float)num_scale, (float)static_scale,
                                   ptr<float>(x), ptr<int32_t>(err), stream_of(ct)),
        "embed_split_bags");
  return x;
}

Tensor embed_epilogue(const Tensor& y, BATCH_ARGS, int64_t G, int64_t flags, const optional<Tensor>& sin_div,
                      const optional<Tensor>& cos_div) {
  const c10::DeviceGuard guard(y.device());
  Batch bt = make_batch(BATCH_PASS);
  Tensor yc = as(y, at::kFloat);
  const int64_t D = yc.size(-1);
  Tensor out = at::empty({bt.b.B, bt.b.L, G, D}, yc.options());
  Tensor times = event_times_for(bt, flags, yc);
  check(esgpt_embed_epilogue_fwd(&bt.b, G, D, ptr<const float>(yc), optr<const float>(sin_div),
                                 optr<const float>(cos_div), (int)flags, ptr<float>(out), stream_of(yc)),
        "embed_epilogue");
  return out;
}

Tensor embed_epilogue_bwd(const Tensor& dout, BATCH_ARGS, int64_t G, int64_t flags,
                          optional<at::ScalarType> dtype) {
  const c10::DeviceGuard guard(dout.device());
  Batch bt = make_batch(BATCH_PASS);
  Tensor d = as(dout, at::kFloat);
  const int64_t D = d.size(-1);
  const at::ScalarType dt = dtype.value_or(at::kFloat);
  TORCH_CHECK(dt == at::kFloat || dt == at::kBFloat16, "embed_epilogue_bwd: f32 or bf16 output");
  Tensor dy = at::empty({bt.b.B * bt.b.L * G, D}, d.options().dtype(dt));
  check(esgpt_embed_epilogue_bwd_ex(&bt.b, G, D, ptr<const float>(d), (int)flags, dy.data_ptr(), dtype_code(dt),
                                    stream_of(d)),
        "embed_epilogue_bwd");
  return dy;
}

// SPLIT projection operands: (x_lp | empty for f32, w_lp [D, Dc+Dn], bias f32 [D])
std::tuple<Tensor, Tensor, Tensor> split_proj_prep(const Tensor& x, const Tensor& cat_w, const Tensor& num_w,
                                                   const Tensor& cat_b, const Tensor& num_b, double a_c, double a_n,
                                                   at::ScalarType dtype) {
  const c10::DeviceGuard guard(x.device());
  TORCH_CHECK(dtype == at::kFloat || dtype == at::kBFloat16, "split_proj_prep: f32 or bf16");
  Tensor xf = as(x, at::kFloat), wc = as(cat_w, at::kFloat), wn = as(num_w, at::kFloat);
  Tensor bc = as(cat_b, at::kFloat), bn = as(num_b, at::kFloat);
  const int64_t D = wc.size(0), Dc = wc.size(1), Dn = wn.size(1), Dx = Dc + Dn;
  TORCH_CHECK(wn.size(0) == D && bc.numel() == D && bn.numel() == D && xf.size(-1) == Dx,
              "split_proj_prep: shapes");
  const int64_t N = xf.numel() / Dx;
  const bool conv = dtype == at::kBFloat16;
  Tensor x_lp = conv ? at::empty({N, Dx}, xf.options().dtype(dtype)) : at::empty({0}, xf.options());
  Tensor w_lp = at::empty({D, Dx}, xf.options().dtype(dtype));
  Tensor bias = at::empty({D}, xf.options());
  check(esgpt_split_proj_prep(ptr<const float>(xf), N, conv ? x_lp.data_ptr() : nullptr, ptr<const float>(wc),
                              ptr<const float>(wn), D, Dc, Dn, ptr<const float>(bc), ptr<const float>(bn), (float)a_c,
                              (float)a_n, w_lp.data_ptr(), ptr<float>(bias), dtype_code(dtype), stream_of(xf)),
        "split_proj_prep");
  return {x_lp, w_lp, bias};
}

// SPLIT projection gradients: the four parameter gradients written into the given tensors; returns dx f32 (empty
// without dx_lp)
Tensor split_proj_post(const optional<Tensor>& dx_lp_, const Tensor& dw, const Tensor& db, int64_t Dc, double a_c,
                       double a_n, const Tensor& cat_dw, const Tensor& num_dw, const Tensor& cat_db,
                       const Tensor& num_db) {
  const c10::DeviceGuard guard(dw.device());
  const int64_t D = dw.size(0), Dx = dw.size(1), Dn = Dx - Dc;
  TORCH_CHECK(dw.scalar_type() == at::kFloat && db.scalar_type() == at::kFloat && dw.is_contiguous() &&
                  db.is_contiguous() && db.numel() == D && Dc > 0 && Dn > 0,
              "split_proj_post: dw f32 [D, Dc+Dn], db f32 [D]");
  for (const Tensor* t : {&cat_dw, &num_dw, &cat_db, &num_db})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->device() == dw.device(),
                "split_proj_post: contiguous f32 outputs");
  TORCH_CHECK(cat_dw.numel() == D * Dc && num_dw.numel() == D * Dn && cat_db.numel() == D && num_db.numel() == D,
              "split_proj_post: output sizes");
  const bool has_dx = dx_lp_.has_value() && dx_lp_->defined();
  Tensor dx_lp = has_dx ? dx_lp_->contiguous() : Tensor();
  TORCH_CHECK(!has_dx || (dx_lp.scalar_type() == at::kBFloat16 && dx_lp.size(-1) == Dx), "split_proj_post: dx_lp");
  const int64_t N = has_dx ? dx_lp.numel() / Dx : 0;
  Tensor dx = has_dx ? at::empty({N, Dx}, dw.options()) : at::empty({0}, dw.options());
  check(esgpt_split_proj_post(has_dx ? dx_lp.data_ptr() : nullptr, N, has_dx ? ptr<float>(dx) : nullptr,
                              ptr<const float>(dw), ptr<const float>(db), D, Dc, Dn, (float)a_c, (float)a_n,
                              ptr<float>(cat_dw), ptr<float>(num_dw), ptr<float>(cat_db), ptr<float>(num_db),
                              has_dx ? ESGPT_BF16 : ESGPT_F32, stream_of(dw)),
        "split_proj_post");
  return dx;
}

// dsrc: rows of leading dimension ld (elements), D columns used (may be a column slice of a wider matrix)
Tensor embed_bag_bwd(const Tensor& dsrc, BATCH_ARGS, at::IntArrayRef buckets, int64_t selector, int64_t flags,
                     double dyn_scale, double static_scale, int64_t ld, int64_t D, int64_t V, int64_t G,
                     const optional<Tensor>& out) {
  const c10::DeviceGuard guard(dsrc.device());
  TORCH_CHECK(dsrc.scalar_type() == at::kFloat && dsrc.stride(-1) == 1, "embed_bag_bwd: f32 rows expected");
  Batch bt = make_batch(BATCH_PASS);
  esgpt_buckets bk;
  const bool has_bk = make_buckets(buckets, bk);
  // out given (TrainStep's zero-copy exchange buffer region): the table gradient is written there, fully
  const bool has_out = out.has_value() && out->defined();
  if (has_out)
    TORCH_CHECK(out->scalar_type() == at::kFloat && out->is_contiguous() && out->numel() == V * D &&
                    out->device() == dsrc.device(), "embed_bag_bwd: out must be contiguous f32 [V * D]");
  Tensor dtable = has_out ? out->view({V, D}) : at::empty({V, D}, dsrc.options());
  const size_t nb = esgpt_embed_bag_bwd_workspace(&bt.b, G, V, D);
  Tensor ws = at::empty({(int64_t)std::max<size_t>(nb, 1)}, dsrc.options().dtype(at::kByte));
  check(esgpt_embed_bag_bwd(&bt.b, has_bk ? &bk : nullptr, (int)selector, (int)flags, (float)dyn_scale,
                            (float)static_scale, ptr<const float>(dsrc), ld, D, V, ptr<float>(dtable), ws.data_ptr(),
                            nb, stream_of(dsrc)),
        "embed_bag_bwd");
  return has_out ? at::empty({0}, dsrc.options()) : dtable;  // never an alias of `out`
}

// ---- nested-attention glue + residual (structured.hip) ---------------------------------------------------------
// x undefined: h = mask ? dropout(y) : 0 (a plain dropout: the NA input layer's embedding_dropout)
Tensor residual(const optional<Tensor>& x_, const Tensor& y_, const optional<Tensor>& row_mask, int64_t mask_div,
                int64_t skip_T, double dropout_p, const optional<Tensor>& seed) {
  const c10::DeviceGuard guard(y_.device());
  require_hip(y_, "y");
  const bool has_x = x_.has_value() && x_->defined();
  Tensor x = has_x ? x_->contiguous() : Tensor(), y = y_.contiguous();
  const int64_t D = y.size(-1), N = y.numel() / D;
  TORCH_CHECK(mask_div >= 1 && skip_T >= 0 && (has_x || skip_T == 0), "esgpt.residual: mask_div / skip_T");
  if (has_x) {
    TORCH_CHECK(x.scalar_type() == at::kFloat, "esgpt.residual: x must be f32");
    TORCH_CHECK(x.size(-1) == D, "esgpt.residual: x / y widths");
    TORCH_CHECK(skip_T <= 1 ? x.numel() / D == N : (N % (skip_T - 1) == 0 && x.numel() / D == N / (skip_T - 1) * skip_T),
                "esgpt.residual: x rows must be N (or N / (T-1) * T with skip_T = T)");
  }
  Tensor rm = as_opt(row_mask, at::kBool);
  TORCH_CHECK(!rm.defined() || rm.numel() * mask_div == N, "esgpt.residual: row_mask must hold N / mask_div rows");
  Tensor h = at::empty({N, D}, y.options().dtype(at::kFloat));
  check(esgpt_residual_fwd(has_x ? ptr<const float>(x) : nullptr, y.data_ptr(), dtype_code(y.scalar_type()),
                           rm.defined() ? ptr<const uint8_t>(rm) : nullptr, mask_div, skip_T, (float)dropout_p,
                           optr<const uint64_t>(seed), N, D, ptr<float>(h), stream_of(y)),
        "residual");
  return h;
}

std::tuple<Tensor, Tensor> residual_bwd(const Tensor& dh_, const optional<Tensor>& row_mask, int64_t mask_div,
                                        int64_t skip_T, int64_t x_rows, bool need_dx, double dropout_p,
                                        const optional<Tensor>& seed, at::ScalarType y_dtype) {
  const c10::DeviceGuard guard(dh_.device());
  Tensor dh = dh_.to(at::kFloat).contiguous();
  const int64_t D = dh.size(-1), N = dh.numel() / D;
  TORCH_CHECK(mask_div >= 1 && skip_T >= 0, "esgpt.residual_bwd: mask_div / skip_T");
  TORCH_CHECK(!need_dx || (skip_T <= 1 ? x_rows == N : (N % (skip_T - 1) == 0 && x_rows == N / (skip_T - 1) * skip_T)),
              "esgpt.residual_bwd: x_rows must be N (or N / (T-1) * T with skip_T = T)");
  Tensor rm = as_opt(row_mask, at::kBool);
  TORCH_CHECK(!rm.defined() || rm.numel() * mask_div == N, "esgpt.residual_bwd: row_mask must hold N / mask_div rows");
  Tensor dy = at::empty({N, D}, dh.options().dtype(y_dtype));
  Tensor dx = need_dx ? at::empty({x_rows, D}, dh.options()) : Tensor();
  check(esgpt_residual_bwd(ptr<const float>(dh), rm.defined() ? ptr<const uint8_t>(rm) : nullptr, mask_div, skip_T,
                           (float)dropout_p, optr<const uint64_t>(seed), N, D, need_dx ? ptr<float>(dx) : nullptr,
                           dy.data_ptr(), dtype_code(y_dtype), stream_of(dh)),
        "residual_bwd");
  return {dx, dy};
}

Tensor na_split(const Tensor& x_, const Tensor& event_mask) {
  const c10::DeviceGuard guard(x_.device());
  require_hip(x_, "x");
  Tensor x = x_.to(at::kFloat).contiguous();
  TORCH_CHECK(x.dim() == 4, "esgpt.na_split: x must be [B, L, G, D]");
  const int64_t B = x.size(0), L = x.size(1), G = x.size(2), D = x.size(3);
  Tensor m = as_opt(event_mask, at::kBool);
  TORCH_CHECK(m.defined() && m.numel() == B * L, "esgpt.na_split: event_mask must hold B * L events");
  Tensor per = at::empty({B, L, D}, x.options());
  check(esgpt_na_split_fwd(ptr<const float>(x), ptr<const uint8_t>(m), B * L, G, D, ptr<float>(per), stream_of(x)),
        "na_split");
  return per;
}

void na_split_bwd_(const Tensor& dper_, const Tensor& event_mask, Tensor dx) {
  const c10::DeviceGuard guard(dper_.device());
  Tensor dper = dper_.to(at::kFloat).contiguous();
  TORCH_CHECK(dx.is_contiguous() && dx.scalar_type() == at::kFloat && dx.dim() == 4, "esgpt.na_split_bwd_: dx");
  Tensor m = as_opt(event_mask, at::kBool);
  TORCH_CHECK(m.defined() && m.numel() == dx.size(0) * dx.size(1) && dper.numel() == m.numel() * dx.size(3),
              "esgpt.na_split_bwd_: event_mask must hold B * L events and dper B * L rows of D");
  check(esgpt_na_split_bwd(ptr<const float>(dper), ptr<const uint8_t>(m), dx.size(0) * dx.size(1), dx.size(2),
                           dx.size(3), ptr<float>(dx), stream_of(dper)),
        "na_split_bwd");
}

Tensor na_assemble(const Tensor& ctx_, const Tensor& x_) {
  const c10::DeviceGuard guard(x_.device());
  require_hip(x_, "x");
  Tensor ctx = ctx_.to(at::kFloat).contiguous(), x = x_.to(at::kFloat).contiguous();
  TORCH_CHECK(x.dim() == 4, "esgpt.na_assemble: x must be [B, L, G, D]");
  const int64_t B = x.size(0), L = x.size(1), G = x.size(2), D = x.size(3);
  TORCH_CHECK(ctx.numel() == B * L * D, "esgpt.na_assemble: ctx must hold B * L rows of D");
  Tensor seq = at::empty({B * L, G + 1, D}, x.options());
  check(esgpt_na_assemble_fwd(ptr<const float>(ctx), ptr<const float>(x), B, L, G, D, ptr<float>(seq), stream_of(x)),
        "na_assemble");
  return seq;
}

std::tuple<Tensor, Tensor> na_assemble_bwd(const Tensor& dseq_, int64_t B, int64_t L) {
  const c10::DeviceGuard guard(dseq_.device());
  Tensor dseq = dseq_.to(at::kFloat).contiguous();
  const int64_t G = dseq.size(-2) - 1, D = dseq.size(-1);
  TORCH_CHECK(G >= 1 && dseq.numel() == B * L * (G + 1) * D, "esgpt.na_assemble_bwd: dseq must be [B * L, G + 1, D]");
  Tensor dctx = at::empty({B, L, D}, dseq.options());
  Tensor dx = at::empty({B, L, G, D}, dseq.options());  // level G-1: esgpt.na_split_bwd_
  check(esgpt_na_assemble_bwd(ptr<const float>(dseq), B, L, G, D, ptr<float>(dctx), ptr<float>(dx), stream_of(dseq)),
        "na_assemble_bwd");
  return {dctx, dx};
}

// NA output layer operands: x f32 [B, L, G, D] -> (head [B·L·(G-1), D], last [B·L, D]) in dtype
std::tuple<Tensor, Tensor> na_head_split(const Tensor& x_, at::ScalarType dtype) {
  const c10::DeviceGuard guard(x_.device());
  require_hip(x_, "x");
  Tensor x = x_.to(at::kFloat).contiguous();
  TORCH_CHECK(x.dim() == 4 && x.size(2) >= 2, "esgpt.na_head_split: x must be [B, L, G >= 2, D]");
  const int64_t BL = x.size(0) * x.size(1), G = x.size(2), D = x.size(3);
  Tensor head = at::empty({BL * (G - 1), D}, x.options().dtype(dtype));
  Tensor last = at::empty({BL, D}, x.options().dtype(dtype));
  check(esgpt_na_head_split_fwd(ptr<const float>(x), BL, G, D, head.data_ptr(), last.data_ptr(), dtype_code(dtype),
                                stream_of(x)),
        "na_head_split");
  return {head, last};
}

Tensor na_head_split_bwd(const optional<Tensor>& dhead_, const optional<Tensor>& dlast_, int64_t B, int64_t L,
                         int64_t G) {
  const Tensor& any = (dhead_.has_value() && dhead_->defined()) ? *dhead_ : *dlast_;
  const c10::DeviceGuard guard(any.device());
  const at::ScalarType dt = any.scalar_type();
  Tensor dh = (dhead_.has_value() && dhead_->defined()) ? dhead_->to(dt).contiguous() : Tensor();
  Tensor dl = (dlast_.has_value() && dlast_->defined()) ? dlast_->to(dt).contiguous() : Tensor();
  const int64_t D = any.size(-1);
  TORCH_CHECK(G >= 2 && (!dh.defined() || dh.numel() == B * L * (G - 1) * D) && (!dl.defined() || dl.numel() == B * L * D),
              "esgpt.na_head_split_bwd: gradient shapes");
  Tensor dx = at::empty({B, L, G, D}, any.options().dtype(at::kFloat));
  check(esgpt_na_head_split_bwd(dh.defined() ? dh.data_ptr() : nullptr, dl.defined() ? dl.data_ptr() : nullptr,
                                dtype_code(dt), B * L, G, D, ptr<float>(dx), stream_of(any)),
        "na_head_split_bwd");
  return dx;
}

// ---- attention (packed qkv [Bs, T, 3D]) ------------------------------------------------------------------------
std::tuple<Tensor, Tensor, Tensor> attention(const Tensor& qkv_, const optional<Tensor>& key_mask,
                                             const optional<Tensor>& query_mask, int64_t H, int64_t window,
                                             bool static_kv_first, double dropout_p, const optional<Tensor>& seed) {
  const c10::DeviceGuard guard(qkv_.device());
  require_hip(qkv_, "qkv");
  Tensor qkv = qkv_.contiguous();
  const int64_t Bs = qkv.size(0), T = qkv.size(1), D3 = qkv.size(2), D = D3 / 3, hd = D / H;
  const int64_t skf = static_kv_first ? 1 : 0, Lk = T, Lq = T - skf;
  const int64_t es = qkv.element_size();
  char* base = reinterpret_cast<char*>(qkv.data_ptr());
  Tensor km = as_opt(key_mask, at::kBool), qm = as_opt(query_mask, at::kBool);
  Tensor o = at::empty({Bs, Lq, D}, qkv.options());
  Tensor lse = at::empty({Bs, H, Lq}, qkv.options().dtype(at::kFloat));
  // the dropout keep bits the MFMA forward draws, for the backward (empty when the path does not use them)
  const int64_t nkeep = esgpt_attn_keep_words(Bs, H, Lq, Lk, hd, T, D3, D, dtype_code(qkv.scalar_type()),
                                              (float)dropout_p);
  Tensor keep = at::empty({nkeep}, qkv.options().dtype(at::kInt));
  check(esgpt_attn_fwd_ex(base + skf * D3 * es, base + D * es, base + 2 * D * es, D3, T, o.data_ptr(), D,
                          ptr<float>(lse), km.defined() ? ptr<const uint8_t>(km) : nullptr,
                          qm.defined() ? ptr<const uint8_t>(qm) : nullptr, Bs, H, Lq, Lk, hd, window,
                          (float)dropout_p, optr<const uint64_t>(seed), dtype_code(qkv.scalar_type()),
                          nkeep ? reinterpret_cast<uint32_t*>(keep.data_ptr()) : nullptr, stream_of(qkv)),
        "attention");
  return {o, lse, keep};
}

Tensor attention_bwd(const Tensor& qkv_, const Tensor& o, const Tensor& dout_, const Tensor& lse,
                     const optional<Tensor>& key_mask, const optional<Tensor>& query_mask, int64_t H, int64_t window,
                     bool static_kv_first, double dropout_p, const optional<Tensor>& seed,
                     const optional<Tensor>& keep, const Tensor& tickets) {
  const c10::DeviceGuard guard(qkv_.device());
  Tensor qkv = qkv_.contiguous();
  Tensor dout = dout_.to(qkv.scalar_type()).contiguous();
  const int64_t Bs = qkv.size(0), T = qkv.size(1), D3 = qkv.size(2), D = D3 / 3, hd = D / H;
  const int64_t skf = static_kv_first ? 1 : 0, Lk = T, Lq = T - skf;
  const int64_t es = qkv.element_size();
  // static_kv_first: the kernels write every row of dk / dv and the dq rows after token 0, and zero token 0's dq
  Tensor dqkv = at::empty_like(qkv);
  const size_t nb = esgpt_attn_bwd_workspace(Bs, H, Lq, Lk, hd);
  Tensor ws = at::empty({(int64_t)std::max<size_t>(nb, 1)}, qkv.options().dtype(at::kByte));
  int32_t* counters = esgpt_attn_bwd_counters(Bs, H, Lk) <= tickets.numel() ? ptr<int32_t>(tickets) : nullptr;
  Tensor km = as_opt(key_mask, at::kBool), qm = as_opt(query_mask, at::kBool);
  char* base = reinterpret_cast<char*>(qkv.data_ptr());
  char* dbase = reinterpret_cast<char*>(dqkv.data_ptr());
  const int64_t nkeep = esgpt_attn_keep_words(Bs, H, Lq, Lk, hd, T, D3, D, dtype_code(qkv.scalar_type()),
                                              (float)dropout_p);
  const uint32_t* kp = nullptr;
  if (nkeep && keep.has_value() && keep->defined() && keep->numel() == nkeep) {
    TORCH_CHECK(keep->scalar_type() == at::kInt && keep->is_contiguous() && keep->device() == qkv.device(),
                "esgpt.attention_bwd: keep must be the int32 tensor attention returned");
    kp = reinterpret_cast<const uint32_t*>(keep->data_ptr());
  }
  check(esgpt_attn_bwd_lead(base + skf * D3 * es, base + D * es, base + 2 * D * es, D3, T, o.data_ptr(), D,
                          dout.data_ptr(), D, ptr<const float>(lse), km.defined() ? ptr<const uint8_t>(km) : nullptr,
                          qm.defined() ? ptr<const uint8_t>(qm) : nullptr, dbase + skf * D3 * es, dbase + D * es,
                          dbase + 2 * D * es, D3, Bs, H, Lq, Lk, hd, window, (float)dropout_p,
                          optr<const uint64_t>(seed), kp, dtype_code(qkv.scalar_type()), ws.data_ptr(), nb, counters,
                          skf, stream_of(qkv)),
        "attention_bwd");
  return dqkv;
}

// ---- generation: KV cache ----------------------------------------------------------------------------------------
void kv_append(const Tensor& qkv, const Tensor& k_cache, const Tensor& v_cache, int64_t past) {
  const c10::DeviceGuard guard(qkv.device());
  TORCH_CHECK(qkv.is_contiguous() && k_cache.is_contiguous() && v_cache.is_contiguous(), "kv_append: contiguous");
  const int64_t B = qkv.size(0), Lq = qkv.size(1), D3 = qkv.size(2), cap = k_cache.size(1), D = k_cache.size(2);
  check(esgpt_kv_append(qkv.data_ptr(), D3, k_cache.data_ptr(), v_cache.data_ptr(), B, Lq, past, cap, D,
                        dtype_code(qkv.scalar_type()), stream_of(qkv)),
        "kv_append");
}

Tensor attn_decode(const Tensor& qkv, const Tensor& k_cache, const Tensor& v_cache, const optional<Tensor>& key_mask,
                   const optional<Tensor>& query_mask, int64_t H, int64_t Lk, int64_t window) {
  const c10::DeviceGuard guard(qkv.device());
  const int64_t B = qkv.size(0), Lq = qkv.size(1), D3 = qkv.size(2), D = D3 / 3, cap = k_cache.size(1);
  Tensor km = as_opt(key_mask, at::kBool), qm = as_opt(query_mask, at::kBool);
  Tensor o = at::empty({B, Lq, D}, qkv.options());
  check(esgpt_attn_decode(qkv.data_ptr(), D3, k_cache.data_ptr(), v_cache.data_ptr(),
                          km.defined() ? ptr<const uint8_t>(km) : nullptr,
                          qm.defined() ? ptr<const uint8_t>(qm) : nullptr, o.data_ptr(), D, B, H, Lq, Lk, cap, D / H,
                          window, dtype_code(qkv.scalar_type()), stream_of(qkv)),
        "attn_decode");
  return o;
}

// ---- output-layer losses -------------------------------------------------------------------------------------------
std::vector<esgpt_loss_term> make_terms(at::IntArrayRef t) {
  TORCH_CHECK(t.size() % 8 == 0, "terms: 8 ints per term");
  std::vector<esgpt_loss_term> out(std::max<size_t>(1, t.size() / 8));
  for (size_t i = 0; i < t.size() / 8; ++i) {
    out[i] = esgpt_loss_term{(int32_t)t[8 * i], (int32_t)t[8 * i + 1], (int32_t)t[8 * i + 2], (int32_t)t[8 * i + 3],
                             (int32_t)t[8 * i + 4], (int32_t)t[8 * i + 5], (int32_t)t[8 * i + 6], 0};
  }
  return out;
}

// losses f32 [n_terms + 2] (per term, -TTE_LL, total) and d(total)/d(zc), d(total)/d(zt), the position-0 bias rows
std::tuple<Tensor, Tensor, Tensor, Tensor> output_loss(const Tensor& zc_, const optional<Tensor>& zt_,
                                                       const optional<Tensor>& zc_bias, BATCH_ARGS, int64_t n_levels,
                                                       int64_t shift, at::IntArrayRef terms, at::IntArrayRef tte_i,
                                                       at::ArrayRef<double> tte_f, const Tensor& err, int64_t path) {
  const c10::DeviceGuard guard(zc_.device());
  Batch bt = make_batch(BATCH_PASS);
  Tensor zc = zc_.contiguous();
  const bool same = !(zt_.has_value() && zt_->defined());
  Tensor zt = same ? zc : zt_->contiguous();
  Tensor bias = (zc_bias.has_value() && zc_bias->defined()) ? zc_bias->to(zc.scalar_type()).contiguous() : Tensor();
  auto tv = make_terms(terms);
  const int n_terms = (int)(terms.size() / 8);
  TORCH_CHECK(tte_i.size() == 3 && tte_f.size() == 2, "tte spec: [kind, K, col], [mean_log, std_log]");
  esgpt_tte_spec tte{(int32_t)tte_i[0], (int32_t)tte_i[1], (int32_t)tte_i[2], 0, (float)tte_f[0], (float)tte_f[1]};
  Tensor dzc = at::empty_like(zc);
  Tensor dzt = same ? at::empty({0}, zc.options()) : at::empty_like(zt);
  const int64_t ldc = zc.size(-1);
  Tensor dbias = shift ? at::empty({bt.b.B, ldc}, zc.options().dtype(at::kFloat)) : at::empty({0}, zc.options().dtype(at::kFloat));
  Tensor losses = at::empty({n_terms + 2}, zc.options().dtype(at::kFloat));
  const size_t nb = esgpt_output_loss_workspace(bt.b.B, bt.b.L, n_terms);
  Tensor ws = at::empty({(int64_t)std::max<size_t>(nb, 1)}, zc.options().dtype(at::kByte));
  check(esgpt_output_loss_ex(&bt.b, zc.data_ptr(), ldc, n_levels, (int)shift,
                             bias.defined() ? bias.data_ptr() : nullptr, zt.data_ptr(), zt.size(-1),
                             dtype_code(zc.scalar_type()), tv.data(), n_terms, &tte, dzc.data_ptr(),
                             same ? dzc.data_ptr() : dzt.data_ptr(), shift ? ptr<float>(dbias) : nullptr,
                             ptr<float>(losses), ws.data_ptr(), nb, ptr<int32_t>(err), (int)path, stream_of(zc)),
        "output_loss");
  return {losses, dzc, dzt, dbias};
}

// ---- block elementwise stages -----------------------------------------------------------------------------------
std::tuple<Tensor, Tensor, Tensor, Tensor> residual_ln(const optional<Tensor>& x, const optional<Tensor>& y,
                                                       const optional<Tensor>& bias, const Tensor& ln_w,
                                                       const Tensor& ln_b, const optional<Tensor>& row_mask,
                                                       double p, const optional<Tensor>& seed, double eps,
                                                       at::ScalarType out_dtype, int64_t skip_T) {
  const c10::DeviceGuard guard(ln_w.device());
  Tensor xc = (x.has_value() && x->defined()) ? x->to(at::kFloat).contiguous() : Tensor();
  Tensor yc = (y.has_value() && y->defined()) ? y->contiguous() : Tensor();
  Tensor bc = (bias.has_value() && bias->defined()) ? bias->to(at::kFloat).contiguous() : Tensor();
  TORCH_CHECK(xc.defined() || yc.defined(), "residual_ln: x or y required");
  TORCH_CHECK(skip_T == 0 || (xc.defined() && yc.defined()), "residual_ln: skip_T needs x and y");
  const Tensor& ref = yc.defined() ? yc : xc;  // output rows (x has more under skip_T)
  const int64_t N = ref.size(0), D = ref.size(1);
  TORCH_CHECK(skip_T == 0 || (N % (skip_T - 1) == 0 && xc.size(0) == N / (skip_T - 1) * skip_T),
              "residual_ln: x must hold T rows per T-1 output rows under skip_T");
  const at::ScalarType y_dtype = yc.defined() ? yc.scalar_type() : at::kFloat;
  auto f32 = ln_w.options().dtype(at::kFloat);
  Tensor h = at::empty({N, D}, f32), out = at::empty({N, D}, f32.dtype(out_dtype));
  Tensor mean = at::empty({N}, f32), rstd = at::empty({N}, f32);
  Tensor rm = as_opt(row_mask, at::kBool);
  check(esgpt_residual_ln_fwd_ex(xc.defined() ? ptr<const float>(xc) : nullptr,
                                 yc.defined() ? yc.data_ptr() : nullptr, dtype_code(y_dtype),
                                 bc.defined() ? ptr<const float>(bc) : nullptr,
                                 rm.defined() ? ptr<const uint8_t>(rm) : nullptr, (float)p, optr<const uint64_t>(seed),
                                 ptr<const float>(ln_w), ptr<const float>(ln_b), (float)eps, N, D, skip_T,
                                 ptr<float>(h), out.data_ptr(), dtype_code(out_dtype), ptr<float>(mean),
                                 ptr<float>(rstd), stream_of(ln_w)),
        "residual_ln");
  return {h, out, mean, rstd};
}

// (dx f32 [N, D] | empty, dy y_dtype [N, D] | empty, sums f32 [3, D] = (d ln_w, d ln_b, d bias))
std::tuple<Tensor, Tensor, Tensor> residual_ln_bwd_impl(const optional<Tensor>& dh, const Tensor& dout_,
                                                        const Tensor& h, const Tensor& mean, const Tensor& rstd,
                                                        const Tensor& ln_w, const optional<Tensor>& row_mask, double p,
                                                        const optional<Tensor>& seed, bool need_dx, bool need_dy,
                                                        at::ScalarType y_dtype, at::ScalarType out_dtype,
                                                        bool deferred, Tensor* part_out, int64_t skip_T);

std::tuple<Tensor, Tensor, Tensor> residual_ln_bwd(const optional<Tensor>& dh, const Tensor& dout_, const Tensor& h,
                                                   const Tensor& mean, const Tensor& rstd, const Tensor& ln_w,
                                                   const optional<Tensor>& row_mask, double p,
                                                   const optional<Tensor>& seed, bool need_dx, bool need_dy,
                                                   at::ScalarType y_dtype, at::ScalarType out_dtype,
                                                   const Tensor& tickets, int64_t skip_T) {
  return residual_ln_bwd_impl(dh, dout_, h, mean, rstd, ln_w, row_mask, p, seed, need_dx, need_dy, y_dtype,
                              out_dtype, false, nullptr, skip_T);
}

// The same backward with the column sums deferred: returns (dx, dy, part) — part f32 [n_parts, 3, D] holds the
// per-block partials; esgpt::colsum_flush later sums any number of them in one launch.
std::tuple<Tensor, Tensor, Tensor> residual_ln_bwd_partials(const optional<Tensor>& dh, const Tensor& dout_,
                                                            const Tensor& h, const Tensor& mean, const Tensor& rstd,
                                                            const Tensor& ln_w, const optional<Tensor>& row_mask,
                                                            double p, const optional<Tensor>& seed, bool need_dx,
                                                            bool need_dy, at::ScalarType y_dtype,
                                                            at::ScalarType out_dtype, int64_t skip_T) {
  Tensor part;
  auto r = residual_ln_bwd_impl(dh, dout_, h, mean, rstd, ln_w, row_mask, p, seed, need_dx, need_dy, y_dtype,
                                out_dtype, true, &part, skip_T);
  return {std::get<0>(r), std::get<1>(r), part};
}

// sums[i][c] = Σ_b parts[i][b][c] for every pair, one launch (esgpt_colsum_jobs); sums[i] written in place.
void colsum_flush(at::TensorList parts, at::TensorList sums) {
  TORCH_CHECK(parts.size() == sums.size(), "colsum_flush: one sums tensor per partial table");
  if (parts.empty()) return;
  const c10::DeviceGuard guard(parts[0].device());
  std::vector<esgpt_colsum_job> jobs(parts.size());
  for (size_t i = 0; i < parts.size(); ++i) {
    TORCH_CHECK(parts[i].is_contiguous() && sums[i].is_contiguous() && parts[i].scalar_type() == at::kFloat &&
                    sums[i].scalar_type() == at::kFloat && parts[i].numel() % sums[i].numel() == 0,
                "colsum_flush: contiguous f32 [n, width] partials and [width] sums");
    jobs[i] = esgpt_colsum_job{ptr<const float>(parts[i]), parts[i].numel() / sums[i].numel(), sums[i].numel(),
                               ptr<float>(sums[i])};
  }
  check(esgpt_colsum_jobs(jobs.data(), (int64_t)jobs.size(), stream_of(parts[0])), "colsum_flush");
}

std::tuple<Tensor, Tensor, Tensor> residual_ln_bwd_impl(const optional<Tensor>& dh, const Tensor& dout_,
                                                        const Tensor& h, const Tensor& mean, const Tensor& rstd,
                                                        const Tensor& ln_w, const optional<Tensor>& row_mask, double p,
                                                        const optional<Tensor>& seed, bool need_dx, bool need_dy,
                                                        at::ScalarType y_dtype, at::ScalarType out_dtype,
                                                        bool deferred, Tensor* part_out, int64_t skip_T) {
  const c10::DeviceGuard guard(h.device());
  const int64_t N = h.size(0), D = h.size(1);
  const int64_t xN = skip_T ? N / (skip_T - 1) * skip_T : N;  // rows of x (dx)
  Tensor dout = dout_.to(out_dtype).contiguous();
  Tensor dhc = (dh.has_value() && dh->defined()) ? dh->to(at::kFloat).contiguous() : Tensor();
  auto f32 = h.options().dtype(at::kFloat);
  Tensor dx = need_dx ? at::empty({xN, D}, f32) : at::empty({0}, f32);
  Tensor dy = need_dy ? at::empty({N, D}, f32.dtype(y_dtype)) : at::empty({0}, f32.dtype(y_dtype));
  Tensor part = at::empty({std::max<int64_t>(1, esgpt_residual_ln_partials(N)), 3 * D}, f32);
  Tensor sums = deferred ? Tensor() : at::empty({3, D}, f32);
  Tensor rm = as_opt(row_mask, at::kBool);
  check(esgpt_residual_ln_bwd_ex(dhc.defined() ? ptr<const float>(dhc) : nullptr, dout.data_ptr(),
                                 dtype_code(out_dtype), ptr<const float>(h), ptr<const float>(mean),
                                 ptr<const float>(rstd), ptr<const float>(ln_w),
                                 rm.defined() ? ptr<const uint8_t>(rm) : nullptr, (float)p, optr<const uint64_t>(seed),
                                 N, D, skip_T, need_dx ? ptr<float>(dx) : nullptr, need_dy ? dy.data_ptr() : nullptr,
                                 dtype_code(y_dtype), ptr<float>(part), deferred ? nullptr : ptr<float>(sums),
                                 stream_of(h)),
        "residual_ln_bwd");
  if (part_out) *part_out = part;
  return {dx, dy, sums};
}

Tensor bias_act(const Tensor& f_, const Tensor& bias, int64_t act) {
  const c10::DeviceGuard guard(f_.device());
  Tensor f = f_.contiguous();
  Tensor g = at::empty_like(f);
  check(esgpt_bias_act_fwd(f.data_ptr(), ptr<const float>(bias), (int)act, f.size(0), f.size(1), g.data_ptr(),
                           dtype_code(f.scalar_type()), stream_of(f)),
        "bias_act");
  return g;
}

std::tuple<Tensor, Tensor> bias_act_bwd(const Tensor& dg_, const Tensor& f, const Tensor& bias, int64_t act) {
  const c10::DeviceGuard guard(f.device());
  Tensor dg = dg_.to(f.scalar_type()).contiguous();
  const int64_t N = f.size(0), F = f.size(1);
  Tensor dz = at::empty_like(f);
  Tensor part = at::empty({esgpt_bias_act_partials(N) * F}, f.options().dtype(at::kFloat));
  Tensor dbias = at::empty({F}, f.options().dtype(at::kFloat));
  check(esgpt_bias_act_bwd(dg.data_ptr(), f.data_ptr(), ptr<const float>(bias), (int)act, N, F, dz.data_ptr(),
                           ptr<float>(part), ptr<float>(dbias), dtype_code(f.scalar_type()), stream_of(f)),
        "bias_act_bwd");
  return {dz, dbias};
}

Tensor column_sum(const Tensor& x_) {
  const c10::DeviceGuard guard(x_.device());
  Tensor x = x_.contiguous();
  const int64_t N = x.size(0), F = x.size(1);
  Tensor part = at::empty({esgpt_column_sum_partials(N) * F}, x.options().dtype(at::kFloat));
  Tensor out = at::empty({F}, x.options().dtype(at::kFloat));
  check(esgpt_column_sum(x.data_ptr(), dtype_code(x.scalar_type()), N, F, ptr<float>(part), ptr<float>(out),
                         stream_of(x)),
        "column_sum");
  return out;
}

// ---- projections ---------------------------------------------------------------------------------------------------
void gemm_into(int64_t a_layout, const Tensor& a, int64_t lda, int64_t b_layout, const Tensor& b, int64_t ldb,
               int64_t M, int64_t N, int64_t K, const optional<Tensor>& bias, const optional<Tensor>& alpha,
               const Tensor& c, bool accumulate, const Tensor& tickets) {
  const size_t nb = esgpt_gemm_workspace(M, N, K);
  Tensor ws = nb ? at::empty({(int64_t)nb}, a.options().dtype(at::kByte)) : Tensor();
  TORCH_CHECK(!nb || esgpt_gemm_counters(M, N) <= tickets.numel(), "GEMM tile grid exceeds the ticket array");
  if (a.scalar_type() == at::kFloat) {  // f32 operands (the reference precision): exact-f32 MFMA, f32 output
    TORCH_CHECK(b.scalar_type() == at::kFloat && c.scalar_type() == at::kFloat, "gemm: f32 operands need f32 B and C");
    check(esgpt_gemm_f32((int)a_layout, ptr<const float>(a), lda, (int)b_layout, ptr<const float>(b), ldb, M, N, K,
                         optr<const float>(bias), optr<const float>(alpha), ptr<float>(c), c.stride(0),
                         accumulate ? 1 : 0, ws.defined() ? ws.data_ptr() : nullptr, nb, ptr<int32_t>(tickets),
                         stream_of(a)),
          "gemm_f32");
    return;
  }
  check(esgpt_gemm_bf16((int)a_layout, a.data_ptr(), lda, (int)b_layout, b.data_ptr(), ldb, M, N, K,
                        optr<const float>(bias), optr<const float>(alpha), c.data_ptr(), c.stride(0),
                        dtype_code(c.scalar_type()), accumulate ? 1 : 0, ws.defined() ? ws.data_ptr() : nullptr, nb,
                        ptr<int32_t>(tickets), stream_of(a)),
        "gemm");
}

// C[M, N] = alpha·A·B (+ bias) in a fresh tensor of out_dtype (layouts: include/esgpt_amd.h)
Tensor gemm(int64_t a_layout, const Tensor& a, int64_t lda, int64_t b_layout, const Tensor& b, int64_t ldb, int64_t M,
            int64_t N, int64_t K, const optional<Tensor>& bias, const optional<Tensor>& alpha, at::ScalarType out_dtype,
            const Tensor& tickets) {
  const c10::DeviceGuard guard(a.device());
  Tensor c = at::empty({M, N}, a.options().dtype(out_dtype));
  gemm_into(a_layout, a, lda, b_layout, b, ldb, M, N, K, bias, alpha, c, false, tickets);
  return c;
}

// in-place form (accumulate into / overwrite an existing f32 or bf16 matrix)
void gemm_(const Tensor& c, int64_t a_layout, const Tensor& a, int64_t lda, int64_t b_layout, const Tensor& b,
           int64_t ldb, int64_t M, int64_t N, int64_t K, const optional<Tensor>& bias, const optional<Tensor>& alpha,
           bool accumulate, const Tensor& tickets) {
  const c10::DeviceGuard guard(a.device());
  gemm_into(a_layout, a, lda, b_layout, b, ldb, M, N, K, bias, alpha, c, accumulate, tickets);
}

// y = x·wᵀ (+ bias) (bf16); act >= 0: pre = x·wᵀ + bias and y = act(pre) (pre empty when act < 0)
std::tuple<Tensor, Tensor> linear_act(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, int64_t act) {
  const c10::DeviceGuard guard(x.device());
  TORCH_CHECK(x.stride(-1) == 1 && w.is_contiguous(), "linear: row-major x and w expected");
  const int64_t T = x.size(0), din = x.size(1), dout = w.size(0);
  Tensor y = at::empty({T, dout}, x.options());
  Tensor pre = act >= 0 ? at::empty({T, dout}, x.options()) : at::empty({0}, x.options());
  if (x.scalar_type() == at::kFloat) {
    TORCH_CHECK(w.scalar_type() == at::kFloat, "linear: f32 x needs an f32 w");
    check(esgpt_linear_fwd_f32(ptr<const float>(x), x.stride(0), ptr<const float>(w), T, din, dout,
                               optr<const float>(bias), (int)act, act >= 0 ? ptr<float>(pre) : nullptr, ptr<float>(y),
                               dout, stream_of(x)),
          "linear_fwd_f32");
    return {pre, y};
  }
  check(esgpt_linear_fwd(x.data_ptr(), x.stride(0), w.data_ptr(), T, din, dout, optr<const float>(bias), (int)act,
                         act >= 0 ? pre.data_ptr() : nullptr, y.data_ptr(), dout, stream_of(x)),
        "linear_fwd");
  return {pre, y};
}

// Row-tile mask (esgpt_gemm_row_tiles) of the GEMM launches issued while it lives; cleared on exit.
struct RowTilesScope {
  explicit RowTilesScope(const optional<Tensor>& t, int64_t rows) {
    const bool on = t.has_value() && t->defined();
    if (on)
      TORCH_CHECK(t->scalar_type() == at::kByte && t->is_contiguous() && t->numel() >= (rows + 63) / 64,
                  "row_tiles: uint8 [ceil(rows / 64)] expected");
    esgpt_gemm_row_tiles(on ? ptr<const uint8_t>(*t) : nullptr);
  }
  ~RowTilesScope() { esgpt_gemm_row_tiles(nullptr); }
};

// tiles[t] = 1 iff some event overlapping rows [64t, 64t + 64) is not padded (event e owns rows_per_event rows)
Tensor row_tiles(const Tensor& event_mask, int64_t rows_per_event) {
  const c10::DeviceGuard guard(event_mask.device());
  Tensor em = as(event_mask, at::kBool);
  const int64_t n = em.numel();
  Tensor t = at::empty({(n * rows_per_event + 63) / 64}, em.options().dtype(at::kByte));
  check(esgpt_row_tiles(ptr<const uint8_t>(em), n, rows_per_event, ptr<uint8_t>(t), stream_of(em)), "row_tiles");
  return t;
}

// (dx bf16 [T, in] | empty, dw f32 [out, in], db f32 [out] | empty) of y = x·wᵀ (one grouped launch)
// The weight-gradient stream of a device: one pool stream per device for the life of the process (every split
// backward's dW launch is ordered on it, so they may share one split-K workspace pool and ticket array).
c10::hip::HIPStream weight_grad_stream(c10::DeviceIndex dev) {
  static std::vector<optional<c10::hip::HIPStream>> streams(64);
  TORCH_CHECK(dev >= 0 && dev < 64, "eventstreamgpt_amd: device index out of range");
  if (!streams[dev].has_value()) streams[dev] = c10::hip::getStreamFromPool(false, dev);
  return *streams[dev];
}

// bank[i] = counter + i, counter += bank.numel() (one launch; both int64 device tensors, updated in place)
// With err: the step's error block is zeroed by the same launch (esgpt_step_begin).
void seed_bank(const Tensor& counter, const Tensor& bank, const optional<Tensor>& err) {
  const c10::DeviceGuard guard(counter.device());
  TORCH_CHECK(counter.scalar_type() == at::kLong && bank.scalar_type() == at::kLong && counter.numel() == 1 &&
                  bank.is_contiguous() && counter.is_cuda() && bank.is_cuda(),
              "seed_bank: int64 device counter [1] and contiguous int64 bank");
  const bool has_err = err.has_value() && err->defined();
  TORCH_CHECK(!has_err || (err->is_cuda() && err->nbytes() >= 16 && err->is_contiguous()), "seed_bank: error block");
  check(esgpt_step_begin(ptr<int64_t>(counter), ptr<int64_t>(bank), bank.numel(),
                         has_err ? reinterpret_cast<int32_t*>(err->data_ptr()) : nullptr, stream_of(counter)),
        "seed_bank");
}

// The current stream waits for every weight-gradient launch queued so far (before dW / db are read).
void weight_grad_join(const Tensor& like) {
  const c10::DeviceGuard guard(like.device());
  const auto side = weight_grad_stream(like.device().index());
  check(esgpt_stream_wait(stream_of(like), reinterpret_cast<void*>(side.stream())), "weight_grad_join");
}

// Keeps a tensor's memory from being reused by other streams' allocations until the work queued on `s` is done.
void used_on(const Tensor& t, const c10::hip::HIPStream& s) {
  if (t.defined() && t.numel()) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), s);
}

std::tuple<Tensor, Tensor, Tensor> linear_bwd(const Tensor& dy_, const Tensor& x, const Tensor& w,
                                              const optional<Tensor>& alpha, int64_t act, const optional<Tensor>& pre,
                                              bool need_dx, bool need_db, const Tensor& tickets,
                                              const optional<Tensor>& db_extra_, const optional<Tensor>& dw_tickets,
                                              const optional<Tensor>& dw_out, const optional<Tensor>& db_out,
                                              const optional<Tensor>& row_tiles_) {
  const c10::DeviceGuard guard(x.device());
  const RowTilesScope rts(row_tiles_, dy_.size(0));  // the dX rows (token rows)
  // dw_tickets given: split form — dX on the current stream, dW / db on the device's weight-gradient stream (with
  // their own ticket array, workspace and outputs allocated in that stream's order); weight_grad_join before use
  const bool f32op = x.scalar_type() == at::kFloat;
  // the f32 (reference-precision) form runs grouped on the current stream
  const bool split = !f32op && dw_tickets.has_value() && dw_tickets->defined();
  Tensor dy = f32op ? dy_.to(at::kFloat).contiguous() : dy_.contiguous();
  Tensor db_extra;
  if (db_extra_.has_value() && db_extra_->defined() && db_extra_->numel()) {
    db_extra = as(*db_extra_, at::kFloat);
    TORCH_CHECK(need_db && db_extra.dim() == 2 && db_extra.size(1) == dy.size(1), "linear_bwd: db_extra [n, out]");
  }
  const int64_t T = dy.size(0), dout = dy.size(1), din = x.size(1);
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dx = need_dx ? at::empty({T, din}, dy.options()) : at::empty({0}, dy.options());
  const size_t nb = f32op ? esgpt_linear_bwd_f32_workspace(T, din, dout, need_dx ? 1 : 0)
                          : esgpt_linear_bwd_workspace(T, din, dout, need_dx ? 1 : 0);
  const Tensor& tk = split ? *dw_tickets : tickets;
  TORCH_CHECK(!nb || esgpt_gemm_counters(dout, din) <= tk.numel(), "GEMM tile grid exceeds the ticket array");
  const bool has_pre = pre.has_value() && pre->defined();
  const auto cur = c10::hip::getCurrentHIPStream(x.device().index());
  const auto side = split ? weight_grad_stream(x.device().index()) : cur;
  Tensor dw, db, ws;
  void* s_cur = reinterpret_cast<void*>(cur.stream());
  // fork first: under HIP-graph capture the side stream must have joined the capture before it allocates, so that
  // its blocks come from the graph's private pool (and no allocation reaches the driver mid-capture)
  if (split) check(esgpt_stream_wait(reinterpret_cast<void*>(side.stream()), s_cur), "linear_bwd fork");
  // dw_out / db_out given: the gradients go there (a DDP exchange buffer region, TrainStep's zero-copy exchange)
  // and the returned dw / db are empty
  const bool has_dwo = dw_out.has_value() && dw_out->defined();
  const bool has_dbo = need_db && db_out.has_value() && db_out->defined();
  if (has_dwo)
    TORCH_CHECK(dw_out->scalar_type() == at::kFloat && dw_out->is_contiguous() && dw_out->numel() == dout * din &&
                    dw_out->device() == x.device(), "linear_bwd: dw_out must be contiguous f32 [out * in]");
  if (has_dbo)
    TORCH_CHECK(db_out->scalar_type() == at::kFloat && db_out->is_contiguous() && db_out->numel() == dout &&
                    db_out->device() == x.device(), "linear_bwd: db_out must be contiguous f32 [out]");
  {
    const c10::hip::HIPStreamGuard sg(side);  // the dW product's allocations in its stream's order
    dw = has_dwo ? at::empty({0}, f32) : at::empty({dout, din}, f32);
    db = (need_db && !has_dbo) ? at::empty({dout}, f32) : at::empty({0}, f32);
    ws = nb ? at::empty({(int64_t)nb}, x.options().dtype(at::kByte)) : Tensor();
  }
  float* dwp = has_dwo ? ptr<float>(*dw_out) : ptr<float>(dw);
  float* dbp = need_db ? (has_dbo ? ptr<float>(*db_out) : ptr<float>(db)) : nullptr;
  const void* dxp = need_dx ? dx.data_ptr() : nullptr;
  if (f32op) {
    TORCH_CHECK(w.scalar_type() == at::kFloat && (!has_pre || pre->scalar_type() == at::kFloat),
                "linear_bwd: f32 x needs f32 w and pre");
    check(esgpt_linear_bwd_f32(ptr<const float>(dy), dy.stride(0), ptr<const float>(x), x.stride(0),
                               ptr<const float>(w), T, din, dout, optr<const float>(alpha), (int)act,
                               has_pre ? ptr<const float>(*pre) : nullptr, has_pre ? pre->stride(0) : 0,
                               reinterpret_cast<float*>(const_cast<void*>(dxp)), need_dx ? din : 0, dwp, dbp,
                               ws.defined() ? ws.data_ptr() : nullptr, nb,
                               ptr<int32_t>(tickets), db_extra.defined() ? ptr<const float>(db_extra) : nullptr,
                               db_extra.defined() ? db_extra.size(0) : 0, s_cur),
          "linear_bwd_f32");
  } else if (split) {
    check(esgpt_linear_bwd_split(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), T, din, dout,
                                 optr<const float>(alpha), (int)act, has_pre ? pre->data_ptr() : nullptr,
                                 has_pre ? pre->stride(0) : 0, const_cast<void*>(dxp), need_dx ? din : 0, dwp, dbp,
                                 ws.defined() ? ws.data_ptr() : nullptr, nb, ptr<int32_t>(tk),
                                 db_extra.defined() ? ptr<const float>(db_extra) : nullptr,
                                 db_extra.defined() ? db_extra.size(0) : 0, s_cur,
                                 reinterpret_cast<void*>(side.stream())),
          "linear_bwd");
    // operands the weight-gradient stream reads: not reused by the current stream's later allocations until
    // that stream's reads are done (under graph capture: not reused within the capture)
    used_on(dy, side);
    used_on(x, side);
    used_on(dy_, side);
    if (alpha.has_value()) used_on(*alpha, side);
    used_on(db_extra, side);
  } else {
    check(esgpt_linear_bwd_ex(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), T, din, dout,
                              optr<const float>(alpha), (int)act, has_pre ? pre->data_ptr() : nullptr,
                              has_pre ? pre->stride(0) : 0, const_cast<void*>(dxp), need_dx ? din : 0, dwp, dbp,
                              ws.defined() ? ws.data_ptr() : nullptr, nb, ptr<int32_t>(tickets),
                              db_extra.defined() ? ptr<const float>(db_extra) : nullptr,
                              db_extra.defined() ? db_extra.size(0) : 0, s_cur),
          "linear_bwd");
  }
  return {dx, dw, db};
}

// y = x·wᵀ (+ bias) with the bf16 weight shadow w; `masters` are the f32 parameters (row blocks of w) that receive
// the weight gradient in the registered backward — unused here (ProjFn of the drop-in modules).
Tensor linear(const Tensor& x_, const Tensor& w, const optional<Tensor>& bias, at::TensorList masters,
              const Tensor& tickets, const optional<Tensor>& row_tiles_) {
  const c10::DeviceGuard guard(x_.device());
  const RowTilesScope rts(row_tiles_, x_.size(0));
  Tensor x = x_.contiguous();
  const int64_t T = x.size(0), din = x.size(1), dout = w.size(0);
  Tensor y = at::empty({T, dout}, x.options());
  gemm_into(ESGPT_GEMM_K_CONTIG, x, din, ESGPT_GEMM_K_CONTIG, w, din, T, dout, din, bias, c10::nullopt, y, false,
            tickets);
  return y;
}

// InnerMLP (transformer.py:378-391): pre = x·W_fcᵀ + b_fc, g = act(pre), y = g·W_projᵀ (+ b_proj when given).
// Returns (y, act'(pre), g), kept for the backward: c_fc's epilogue stores the activation's derivative at the
// pre-activation (ESGPT_ACT_DERIV) instead of the pre-activation, so c_proj's input-gradient epilogue multiplies
// instead of evaluating act' (the forward evaluates the same normal density for act anyway).
std::tuple<Tensor, Tensor, Tensor> mlp(const Tensor& x_, const Tensor& w_fc, const Tensor& w_pj, const Tensor& b_fc,
                                       const optional<Tensor>& b_pj, int64_t act, const Tensor& p_fc,
                                       const Tensor& p_pj, const Tensor& tickets,
                                       const optional<Tensor>& row_tiles_) {
  const c10::DeviceGuard guard(x_.device());
  const RowTilesScope rts(row_tiles_, x_.size(0));
  Tensor x = x_.contiguous();
  TORCH_CHECK(act >= 0 && act <= 2, "mlp: act must be 0 (GELU), 1 (tanh GELU) or 2 (ReLU)");
  auto pg = linear_act(x, w_fc, b_fc, act | ESGPT_ACT_DERIV);
  Tensor g = std::get<1>(pg);
  const int64_t T = g.size(0), F = g.size(1), D = w_pj.size(0);
  Tensor y = at::empty({T, D}, x.options());
  gemm_into(ESGPT_GEMM_K_CONTIG, g, F, ESGPT_GEMM_K_CONTIG, w_pj, F, T, D, F, b_pj, c10::nullopt, y, false, tickets);
  return {y, std::get<0>(pg), g};
}

// Generative heads + fused losses (model_output.py:1253-1721): zc = xc·wcᵀ + bc (bf16 GEMM; wc / bc padded to a
// multiple of 8 rows), zt likewise for a separate TTE head (NA), then output_loss. Returns (losses, dzc, dzt, dbias)
// — the unscaled loss gradients w.r.t. the logits, consumed by the registered backward (scaled there by the incoming
// d(total) read from device memory). cw/cb/tw/tb: the f32 parameters receiving the head gradients (unused here).
std::tuple<Tensor, Tensor, Tensor, Tensor> head_loss(const Tensor& xc, const optional<Tensor>& xt, BATCH_ARGS,
                                                     at::IntArrayRef terms, at::IntArrayRef tte_i,
                                                     at::ArrayRef<double> tte_f, int64_t shift, int64_t n_levels,
                                                     const Tensor& wc, const Tensor& bc, const optional<Tensor>& wt,
                                                     const optional<Tensor>& bt, at::TensorList cw, at::TensorList cb,
                                                     at::TensorList tw, at::TensorList tb, const Tensor& err,
                                                     const Tensor& tickets, const optional<Tensor>& zb_in) {
  const c10::DeviceGuard guard(xc.device());
  Tensor zc = linear(xc, wc, bc, {}, tickets, c10::nullopt);
  optional<Tensor> zt;
  if (wt.has_value() && wt->defined()) zt = linear(*xt, *wt, bt, {}, tickets, c10::nullopt);
  optional<Tensor> zb;  // the head bias in the logits' dtype: position 0 reads Linear(zeros) = bias
  if (shift) zb = (zb_in.has_value() && zb_in->defined()) ? *zb_in : bc.to(zc.scalar_type());
  return output_loss(zc, zt, zb, BATCH_PASS, n_levels, shift, terms, tte_i, tte_f, err, ESGPT_LOSS_PATH_AUTO);
}

// ---- parameter packing -----------------------------------------------------------------------------------------
// One launch: group g = srcs[o_g .. o_g + group_sizes[g]) flattened and concatenated into a new 1-D tensor of dtype
// code dtypes[g] (ESGPT_F32 / ESGPT_BF16) followed by tails[g] zeros. srcs: contiguous f32 device tensors.
std::vector<Tensor> pack(at::TensorList srcs, at::IntArrayRef group_sizes, at::IntArrayRef tails,
                         at::IntArrayRef dtypes) {
  TORCH_CHECK(!srcs.empty() && group_sizes.size() == tails.size() && tails.size() == dtypes.size(), "pack: arguments");
  const c10::DeviceGuard guard(srcs[0].device());
  std::vector<Tensor> outs;
  std::vector<esgpt_pack_seg> segs;
  size_t k = 0;
  for (size_t gi = 0; gi < group_sizes.size(); ++gi) {
    TORCH_CHECK(dtypes[gi] == ESGPT_F32 || dtypes[gi] == ESGPT_BF16, "pack: dtype code");
    TORCH_CHECK(group_sizes[gi] >= 0 && tails[gi] >= 0 && k + group_sizes[gi] <= srcs.size(), "pack: group sizes");
    int64_t n = 0;
    for (int64_t j = 0; j < group_sizes[gi]; ++j) {
      const Tensor& t = srcs[k + j];
      require_hip(t, "pack");
      TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous(), "pack: contiguous f32 sources expected");
      n += t.numel();
    }
    const bool bf = dtypes[gi] == ESGPT_BF16;
    Tensor out = at::empty({n + tails[gi]}, srcs[0].options().dtype(bf ? at::kBFloat16 : at::kFloat));
    const size_t esz = bf ? 2 : 4;
    int64_t off = 0;
    for (int64_t j = 0; j < group_sizes[gi]; ++j, ++k) {
      const Tensor& t = srcs[k];
      const bool last = j + 1 == group_sizes[gi];
      segs.push_back(esgpt_pack_seg{t.data_ptr<float>(), static_cast<char*>(out.data_ptr()) + off * esz, t.numel(),
                                    t.numel() + (last ? tails[gi] : 0), (int32_t)dtypes[gi], 0});
      off += t.numel();
    }
    if (group_sizes[gi] == 0 && tails[gi] > 0)
      segs.push_back(esgpt_pack_seg{nullptr, out.data_ptr(), 0, tails[gi], (int32_t)dtypes[gi], 0});
    outs.push_back(out);
  }
  TORCH_CHECK(k == srcs.size(), "pack: group sizes do not cover srcs");
  check(esgpt_pack(segs.data(), (int64_t)segs.size(), stream_of(srcs[0])), "pack");
  return outs;
}

// ---- optimizer -------------------------------------------------------------------------------------------------------
void adamw(const Tensor& table, const Tensor& blocks, double lr, double beta1, double beta2, double eps, double wd,
           int64_t step, const optional<Tensor>& per_tensor, const Tensor& err) {
  const c10::DeviceGuard guard(table.device());
  check(esgpt_adamw(reinterpret_cast<const esgpt_adam_tensor*>(table.data_ptr()), ptr<const int64_t>(blocks),
                    blocks.numel(), (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, step,
                    optr<const float>(per_tensor), ptr<const int32_t>(err), stream_of(table)),
        "adamw");
}

// The device-side optimizer step (HIP-graph replayable): prepare (counters, lr, per-tensor table) + update.
void adamw_dev(const Tensor& table, const Tensor& blocks, const Tensor& counters, const Tensor& active,
               int64_t n_params, int64_t kind, int64_t warmup, int64_t total, double power, double init_lr,
               double end_lr, double beta1, double beta2, double eps, double wd, const Tensor& per_tensor,
               const Tensor& lr_dev, const Tensor& err, const optional<Tensor>& copy_src,
               const optional<Tensor>& ring, const optional<Tensor>& ring_ctr, const optional<Tensor>& ring_tab,
               int64_t host_words) {
  const c10::DeviceGuard guard(table.device());
  TORCH_CHECK(counters.scalar_type() == at::kLong && counters.numel() == n_params + 1, "adamw_dev: counters");
  const bool tb = ring_tab.has_value() && ring_tab->defined();
  const bool rg = ring.has_value() && ring->defined();
  const bool cp = copy_src.has_value() && copy_src->defined();
  const bool rc = ring_ctr.has_value() && ring_ctr->defined();
  const int64_t n_copy = cp ? copy_src->numel() : 0;
  TORCH_CHECK(!cp || rg || tb, "adamw_dev: copy_src needs a ring");
  TORCH_CHECK(!(rg && tb), "adamw_dev: ring and ring_tab are exclusive");
  TORCH_CHECK(host_words == 0 || (tb && rc), "adamw_dev: host_words needs ring_tab and ring_ctr");
  if (tb)
    TORCH_CHECK(ring_tab->scalar_type() == at::kLong && ring_tab->dim() == 1 && ring_tab->is_contiguous() &&
                    ring_tab->numel() >= 1 && (!rc || (ring_ctr->scalar_type() == at::kLong && ring_ctr->numel() == 1)),
                "adamw_dev: ring_tab: contiguous int64 [entries] of entry addresses, ring_ctr int64 [1]");
  if (cp)
    TORCH_CHECK(copy_src->scalar_type() == at::kFloat && copy_src->is_contiguous() && n_copy <= 1024,
                "adamw_dev: copy_src: contiguous f32, at most 1024 elements");
  if (rg)
    TORCH_CHECK(ring->scalar_type() == at::kFloat && ring->dim() == 2 && ring->is_contiguous() &&
                    ring->size(1) == ((n_copy + 3) & ~int64_t(3)) + 4 && ring->size(0) >= 1 &&
                    (!rc || (ring_ctr->scalar_type() == at::kLong && ring_ctr->numel() == 1)),
                "adamw_dev: ring: contiguous f32 [entries, round_up(n_copy, 4) + 4], ring_ctr int64 [1]");
  TORCH_CHECK(active.scalar_type() == at::kInt && per_tensor.numel() >= 2 * active.numel(), "adamw_dev: active / per");
  esgpt_lr_schedule sc{kind, warmup, total, power, init_lr, end_lr};
  void* st = stream_of(table);
  if (tb)
    check(esgpt_adamw_prepare_tab(ptr<int64_t>(counters), active.numel() ? ptr<const int32_t>(active) : nullptr,
                                  (int)active.numel(), (int)n_params, &sc, beta1, beta2, ptr<float>(per_tensor),
                                  ptr<float>(lr_dev), ptr<const int32_t>(err),
                                  cp ? ptr<const float>(*copy_src) : nullptr, n_copy,
                                  reinterpret_cast<float* const*>(ring_tab->data_ptr()),
                                  rc ? ptr<int64_t>(*ring_ctr) : nullptr, ring_tab->numel(),
                                  reinterpret_cast<int32_t*>(static_cast<uintptr_t>(host_words)), st),
          "adamw_prepare_tab");
  else
    check(esgpt_adamw_prepare_ex(ptr<int64_t>(counters), active.numel() ? ptr<const int32_t>(active) : nullptr,
                                 (int)active.numel(), (int)n_params, &sc, beta1, beta2, ptr<float>(per_tensor),
                                 ptr<float>(lr_dev), ptr<const int32_t>(err),
                                 cp ? ptr<const float>(*copy_src) : nullptr, n_copy,
                                 rg ? ptr<float>(*ring) : nullptr, rc ? ptr<int64_t>(*ring_ctr) : nullptr,
                                 rg ? ring->size(0) : 1, st),
          "adamw_prepare");
  check(esgpt_adamw_dev(reinterpret_cast<const esgpt_adam_tensor*>(table.data_ptr()), ptr<const int64_t>(blocks),
                        blocks.numel(), ptr<const float>(lr_dev), (float)beta1, (float)beta2, (float)eps, (float)wd,
                        ptr<const float>(per_tensor), ptr<const int32_t>(err), st),
        "adamw_dev");
}

}  // namespace

TORCH_LIBRARY(esgpt, m) {
  m.def("embed_joint(Tensor table, " BATCH_SCHEMA ", int[] buckets, Tensor? sin_div, Tensor? cos_div, int flags, "
        "float static_w, float dynamic_w, int G, Tensor err) -> Tensor");
  m.def("embed_split_bags(Tensor cat_table, Tensor num_table, " BATCH_SCHEMA ", int[] buckets, int flags, "
        "float cat_scale, float num_scale, float static_scale, int G, Tensor err) -> Tensor");
  m.def("embed_epilogue(Tensor y, " BATCH_SCHEMA ", int G, int flags, Tensor? sin_div, Tensor? cos_div) -> Tensor");
  m.def("embed_epilogue_bwd(Tensor dout, " BATCH_SCHEMA ", int G, int flags, ScalarType? dtype=None) -> Tensor");
  m.def("split_proj_prep(Tensor x, Tensor cat_w, Tensor num_w, Tensor cat_b, Tensor num_b, float a_c, float a_n, "
        "ScalarType dtype) -> (Tensor, Tensor, Tensor)");
  m.def("split_proj_post(Tensor? dx_lp, Tensor dw, Tensor db, int Dc, float a_c, float a_n, Tensor(a!) cat_dw, "
        "Tensor(b!) num_dw, Tensor(c!) cat_db, Tensor(d!) num_db) -> Tensor");
  m.def("embed_bag_bwd(Tensor dsrc, " BATCH_SCHEMA ", int[] buckets, int selector, int flags, float dyn_scale, "
        "float static_scale, int ld, int D, int V, int G, Tensor(a!)? out=None) -> Tensor");
  m.def("attention(Tensor qkv, Tensor? key_mask, Tensor? query_mask, int H, int window, bool static_kv_first, "
        "float dropout_p, Tensor? seed) -> (Tensor, Tensor, Tensor)");
  m.def("attention_bwd(Tensor qkv, Tensor o, Tensor dout, Tensor lse, Tensor? key_mask, Tensor? query_mask, int H, "
        "int window, bool static_kv_first, float dropout_p, Tensor? seed, Tensor? keep, Tensor tickets) -> Tensor");
  m.def("residual(Tensor? x, Tensor y, Tensor? row_mask, int mask_div, int skip_T, float dropout_p, Tensor? seed) "
        "-> Tensor");
  m.def("residual_bwd(Tensor dh, Tensor? row_mask, int mask_div, int skip_T, int x_rows, bool need_dx, "
        "float dropout_p, Tensor? seed, ScalarType y_dtype) -> (Tensor, Tensor)");
  m.def("na_split(Tensor x, Tensor event_mask) -> Tensor");
  m.def("na_split_bwd_(Tensor dper, Tensor event_mask, Tensor(a!) dx) -> ()");
  m.def("na_assemble(Tensor ctx, Tensor x) -> Tensor");
  m.def("na_assemble_bwd(Tensor dseq, int B, int L) -> (Tensor, Tensor)");
  m.def("na_head_split(Tensor x, ScalarType dtype) -> (Tensor, Tensor)");
  m.def("na_head_split_bwd(Tensor? dhead, Tensor? dlast, int B, int L, int G) -> Tensor");
  m.def("kv_append(Tensor qkv, Tensor(a!) k_cache, Tensor(b!) v_cache, int past) -> ()");
  m.def("attn_decode(Tensor qkv, Tensor k_cache, Tensor v_cache, Tensor? key_mask, Tensor? query_mask, int H, "
        "int Lk, int window) -> Tensor");
  m.def("output_loss(Tensor zc, Tensor? zt, Tensor? zc_bias, " BATCH_SCHEMA ", int n_levels, int shift, int[] terms, "
        "int[] tte_i, float[] tte_f, Tensor err, int path=0) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("residual_ln(Tensor? x, Tensor? y, Tensor? bias, Tensor ln_w, Tensor ln_b, Tensor? row_mask, float p, "
        "Tensor? seed, float eps, ScalarType out_dtype, int skip_T=0) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("residual_ln_bwd(Tensor? dh, Tensor dout, Tensor h, Tensor mean, Tensor rstd, Tensor ln_w, Tensor? row_mask, "
        "float p, Tensor? seed, bool need_dx, bool need_dy, ScalarType y_dtype, ScalarType out_dtype, "
        "Tensor tickets, int skip_T=0) -> (Tensor, Tensor, Tensor)");
  m.def("bias_act(Tensor f, Tensor bias, int act) -> Tensor");
  m.def("bias_act_bwd(Tensor dg, Tensor f, Tensor bias, int act) -> (Tensor, Tensor)");
  m.def("column_sum(Tensor x) -> Tensor");
  m.def("gemm(int a_layout, Tensor a, int lda, int b_layout, Tensor b, int ldb, int M, int N, int K, Tensor? bias, "
        "Tensor? alpha, ScalarType out_dtype, Tensor tickets) -> Tensor");
  m.def("gemm_(Tensor(a!) c, int a_layout, Tensor a, int lda, int b_layout, Tensor b, int ldb, int M, int N, int K, "
        "Tensor? bias, Tensor? alpha, bool accumulate, Tensor tickets) -> ()");
  m.def("linear_act(Tensor x, Tensor w, Tensor? bias, int act) -> (Tensor, Tensor)");
  m.def("linear_bwd(Tensor dy, Tensor x, Tensor w, Tensor? alpha, int act, Tensor? pre, bool need_dx, bool need_db, "
        "Tensor tickets, Tensor? db_extra=None, Tensor? dw_tickets=None, Tensor(a!)? dw_out=None, "
        "Tensor(b!)? db_out=None, Tensor? row_tiles=None) -> (Tensor, Tensor, Tensor)");
  m.def("weight_grad_join(Tensor like) -> ()");
  m.def("seed_bank(Tensor(a!) counter, Tensor(b!) bank, Tensor(c!)? err=None) -> ()");
  m.def("residual_ln_bwd_partials(Tensor? dh, Tensor dout, Tensor h, Tensor mean, Tensor rstd, Tensor ln_w, "
        "Tensor? row_mask, float p, Tensor? seed, bool need_dx, bool need_dy, ScalarType y_dtype, "
        "ScalarType out_dtype, int skip_T=0) -> (Tensor, Tensor, Tensor)");
  m.def("colsum_flush(Tensor[] parts, Tensor(a!)[] sums) -> ()");
  m.def("linear(Tensor x, Tensor w, Tensor? bias, Tensor[] masters, Tensor tickets, Tensor? row_tiles=None) "
        "-> Tensor");
  m.def("row_tiles(Tensor event_mask, int rows_per_event) -> Tensor");
  m.def("mlp(Tensor x, Tensor w_fc, Tensor w_pj, Tensor b_fc, Tensor? b_pj, int act, Tensor p_fc, Tensor p_pj, "
        "Tensor tickets, Tensor? row_tiles=None) -> (Tensor, Tensor, Tensor)");
  m.def("head_loss(Tensor xc, Tensor? xt, " BATCH_SCHEMA ", int[] terms, int[] tte_i, float[] tte_f, int shift, "
        "int n_levels, Tensor wc, Tensor bc, Tensor? wt, Tensor? bt, Tensor[] cw, Tensor[] cb, Tensor[] tw, "
        "Tensor[] tb, Tensor err, Tensor tickets, Tensor? zb) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("pack(Tensor[] srcs, int[] group_sizes, int[] tails, int[] dtypes) -> Tensor[]");
  m.def("adamw_dev(Tensor table, Tensor blocks, Tensor(a!) counters, Tensor active, int n_params, int kind, "
        "int warmup, int total, float power, float init_lr, float end_lr, float beta1, float beta2, float eps, "
        "float weight_decay, Tensor(b!) per_tensor, Tensor(c!) lr_dev, Tensor err, Tensor? copy_src=None, "
        "Tensor(d!)? ring=None, Tensor(e!)? ring_ctr=None, Tensor? ring_tab=None, int host_words=0) -> ()");
  m.def("adamw(Tensor table, Tensor blocks, float lr, float beta1, float beta2, float eps, float weight_decay, "
        "int step, Tensor? per_tensor, Tensor err) -> ()");
}

TORCH_LIBRARY_IMPL(esgpt, CUDA, m) {
  m.impl("embed_joint", &embed_joint);
  m.impl("embed_split_bags", &embed_split_bags);
  m.impl("embed_epilogue", &embed_epilogue);
  m.impl("embed_epilogue_bwd", &embed_epilogue_bwd);
  m.impl("split_proj_prep", &split_proj_prep);
  m.impl("split_proj_post", &split_proj_post);
  m.impl("embed_bag_bwd", &embed_bag_bwd);
  m.impl("residual", &residual);
  m.impl("residual_bwd", &residual_bwd);
  m.impl("na_split", &na_split);
  m.impl("na_split_bwd_", &na_split_bwd_);
  m.impl("na_assemble", &na_assemble);
  m.impl("na_assemble_bwd", &na_assemble_bwd);
  m.impl("na_head_split", &na_head_split);
  m.impl("na_head_split_bwd", &na_head_split_bwd);
  m.impl("attention", &attention);
  m.impl("attention_bwd", &attention_bwd);
  m.impl("kv_append", &kv_append);
  m.impl("attn_decode", &attn_decode);
  m.impl("output_loss", &output_loss);
  m.impl("residual_ln", &residual_ln);
  m.impl("residual_ln_bwd", &residual_ln_bwd);
  m.impl("bias_act", &bias_act);
  m.impl("bias_act_bwd", &bias_act_bwd);
  m.impl("column_sum", &column_sum);
  m.impl("gemm", &gemm);
  m.impl("gemm_", &gemm_);
  m.impl("linear_act", &linear_act);
  m.impl("linear_bwd", &linear_bwd);
  m.impl("weight_grad_join", &weight_grad_join);
  m.impl("seed_bank", &seed_bank);
  m.impl("residual_ln_bwd_partials", &residual_ln_bwd_partials);
  m.impl("colsum_flush", &colsum_flush);
  m.impl("linear", &linear);
  m.impl("row_tiles", &row_tiles);
  m.impl("mlp", &mlp);
  m.impl("head_loss", &head_loss);
  m.impl("pack", &pack);
  m.impl("adamw", &adamw);
  m.impl("adamw_dev", &adamw_dev);
}
