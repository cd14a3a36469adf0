// Python bindings of the gfx950 kernels (torch tensors -> raw launchers).
// Every op launches on the *current* HIP stream of the tensor's device, so it
// composes with torch's stream semantics and with HIP-graph capture.
#include <cstdlib>
#include <cstring>
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <vector>

#include "launchers.h"

namespace dpa {
void register_comm(pybind11::module& m);     // comm/reducer.cpp
void register_runtime(pybind11::module& m);  // runtime/streams.cpp
}

#define CHECK_DEV(x) TORCH_CHECK((x).is_cuda(), #x " must be a HIP tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be float32")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bfloat16")
#define CHECK_ALIGNED(x) \
  TORCH_CHECK(reinterpret_cast<uintptr_t>((x).data_ptr()) % 16 == 0, #x " must be 16-byte aligned")

static inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

// ---- optimizer --------------------------------------------------------------
static void sqnorm(const at::Tensor& g, at::Tensor& partial, at::Tensor& out, double scale,
                   double max_norm) {
  CHECK_DEV(g); CHECK_CONTIG(g); CHECK_ALIGNED(g);
  CHECK_F32(partial); CHECK_F32(out);
  TORCH_CHECK(g.numel() % 4 == 0, "flat grad buffer must be padded to a multiple of 4");
  TORCH_CHECK(out.numel() >= 3, "out needs 3 floats");
  const bool bf = g.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || g.scalar_type() == at::kFloat, "grad must be fp32 or bf16");
  const c10::DeviceGuard guard(g.device());
  dpa::launch_sqnorm(g.data_ptr(), bf, g.numel(), partial.data_ptr<float>(), (int)partial.numel(),
                     (float)scale, (float)max_norm, out.data_ptr<float>(), cur_stream());
}

static void adamw_ema(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v,
                      c10::optional<at::Tensor> p16, std::vector<at::Tensor> emas,
                      std::vector<double> rates, double lr, double beta1, double beta2, double eps,
                      double wd, int64_t step, double grad_scale, c10::optional<at::Tensor> clip,
                      c10::optional<at::Tensor> skip) {
  for (auto* t : {&p, &m, &v}) { CHECK_DEV((*t)); CHECK_CONTIG((*t)); CHECK_F32((*t)); CHECK_ALIGNED((*t)); }
  CHECK_DEV(g); CHECK_CONTIG(g); CHECK_ALIGNED(g);
  const int64_t n = p.numel();
  TORCH_CHECK(n % 4 == 0, "flat buffers must be padded to a multiple of 4");
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "size mismatch");
  TORCH_CHECK(emas.size() == rates.size(), "ema/rates mismatch");
  const bool bf = g.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || g.scalar_type() == at::kFloat, "grad must be fp32 or bf16");
  std::vector<float*> bufs;
  std::vector<float> r;
  for (size_t i = 0; i < emas.size(); ++i) {
    CHECK_F32(emas[i]); CHECK_CONTIG(emas[i]); CHECK_ALIGNED(emas[i]);
    TORCH_CHECK(emas[i].numel() == n, "ema size mismatch");
    bufs.push_back(emas[i].data_ptr<float>());
    r.push_back((float)rates[i]);
  }
  uint16_t* p16p = nullptr;
  if (p16.has_value() && p16->defined()) {
    CHECK_BF16((*p16)); CHECK_CONTIG((*p16));
    TORCH_CHECK(p16->numel() == n, "bf16 shadow size mismatch");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(p16->data_ptr()) % 8 == 0, "bf16 shadow must be 8B aligned");
    p16p = reinterpret_cast<uint16_t*>(p16->data_ptr());
  }
  const float* clipp = nullptr;
  if (clip.has_value() && clip->defined()) { CHECK_F32((*clip)); clipp = clip->data_ptr<float>(); }
  const int* skipp = nullptr;
  if (skip.has_value() && skip->defined()) {
    CHECK_DEV((*skip));
    TORCH_CHECK(skip->scalar_type() == at::kInt && skip->numel() >= 1, "skip flag: int32 device tensor");
    skipp = skip->data_ptr<int>();
  }
  const c10::DeviceGuard guard(p.device());
  dpa::launch_adamw_ema(p.data_ptr<float>(), g.data_ptr(), bf, m.data_ptr<float>(),
                        v.data_ptr<float>(), p16p, bufs.data(), r.data(), (int)bufs.size(), n,
                        (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, step,
                        (float)grad_scale, clipp, cur_stream(), skipp);
}

static void ema_update(at::Tensor& e, const at::Tensor& p, double rate) {
  CHECK_F32(e); CHECK_F32(p); CHECK_ALIGNED(e); CHECK_ALIGNED(p);
  TORCH_CHECK(e.numel() == p.numel() && e.numel() % 4 == 0, "ema size");
  const c10::DeviceGuard guard(p.device());
  dpa::launch_ema(e.data_ptr<float>(), p.data_ptr<float>(), e.numel(), (float)rate, cur_stream());
}

static void cast_bf16(const at::Tensor& src, at::Tensor& dst) {
  CHECK_F32(src); CHECK_BF16(dst); CHECK_ALIGNED(src);
  TORCH_CHECK(src.numel() == dst.numel() && src.numel() % 4 == 0, "cast size");
  const c10::DeviceGuard guard(src.device());
  dpa::launch_cast_bf16(src.data_ptr<float>(), reinterpret_cast<uint16_t*>(dst.data_ptr()),
                        src.numel(), cur_stream());
}

// ---- fused linear + cross-entropy ---------------------------------------------
static inline const uint16_t* bf_ptr(const at::Tensor& t) {
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
static inline const uint16_t* opt_bf_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? bf_ptr(*t) : nullptr;
}

static void check_lxent(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b,
                        const at::Tensor& tgt) {
  CHECK_DEV(x); CHECK_DEV(W); CHECK_DEV(tgt);
  CHECK_BF16(x); CHECK_BF16(W); CHECK_CONTIG(x); CHECK_CONTIG(W); CHECK_CONTIG(tgt);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && x.size(1) == W.size(1), "x [N,E], W [V,E]");
  TORCH_CHECK(x.size(1) == 128 || x.size(1) == 256, "lxent: E must be 128 or 256");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.numel() == x.size(0), "target [N] int64");
  if (b.has_value() && b->defined()) {
    CHECK_BF16((*b)); CHECK_CONTIG((*b));
    TORCH_CHECK(b->numel() == W.size(0), "bias [V]");
  }
}

static std::vector<at::Tensor> lxent_fwd(const at::Tensor& x, const at::Tensor& W,
                                         c10::optional<at::Tensor> b, const at::Tensor& tgt) {
  check_lxent(x, W, b, tgt);
  const c10::DeviceGuard guard(x.device());
  const int N = (int)x.size(0), V = (int)W.size(0), E = (int)x.size(1);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({N}, f32), lse = at::empty({N}, f32);
  at::Tensor ws = at::empty({dpa::lxent_workspace_floats(N, V)}, f32);
  if (N > 0)
    dpa::launch_lxent_fwd(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), tgt.data_ptr<int64_t>(), N, V, E,
                          loss.data_ptr<float>(), lse.data_ptr<float>(), ws.data_ptr<float>(),
                          cur_stream());
  return {loss, lse};
}

static std::vector<at::Tensor> lxent_fwd_dx(const at::Tensor& x, const at::Tensor& W,
                                            c10::optional<at::Tensor> b, const at::Tensor& tgt) {
  check_lxent(x, W, b, tgt);
  const c10::DeviceGuard guard(x.device());
  const int N = (int)x.size(0), V = (int)W.size(0), E = (int)x.size(1);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({N}, f32), lse = at::empty({N}, f32), dxu = at::empty({N, E}, f32);
  const int64_t wsn = N > 0 ? dpa::lxent_fwd_dx_workspace_floats(N, V, E) : 0;
  at::Tensor ws = at::empty({wsn}, f32);
  if (N > 0)
    dpa::launch_lxent_fwd_dx(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), tgt.data_ptr<int64_t>(), N, V, E,
                             loss.data_ptr<float>(), lse.data_ptr<float>(), dxu.data_ptr<float>(), cur_stream(),
                             wsn ? ws.data_ptr<float>() : nullptr);
  return {loss, lse, dxu};
}

static void emb_grad(const at::Tensor& ids, const at::Tensor& dy, at::Tensor& dW);

// onehot_scatter: the dW kernel leaves out the target one-hot (softmax only) and it is added
// here as dW[t] -= g x_t, db[t] -= g over the valid targets, by the sorted segment-sum scatter
// of the embedding backward - a compare, subtract and select less per logit in the kernel
// dw_acc / db_acc: fp32 buffers of W's / b's shape (the parameters' flat .grad views) the kernel
// accumulates into directly (its token splits' partials go through a scratch summed in split
// order); the matching results are then undefined - no zero-filled [V, E] result and no
// autograd-side add per call
static std::vector<at::Tensor> lxent_bwd(const at::Tensor& dloss, const at::Tensor& x,
                                         const at::Tensor& W, c10::optional<at::Tensor> b,
                                         const at::Tensor& tgt, const at::Tensor& lse, bool need_dx,
                                         bool need_dw, bool need_db, bool onehot_scatter,
                                         c10::optional<at::Tensor> dw_acc, c10::optional<at::Tensor> db_acc) {
  check_lxent(x, W, b, tgt);
  CHECK_F32(dloss); CHECK_F32(lse); CHECK_CONTIG(dloss); CHECK_CONTIG(lse);
  const c10::DeviceGuard guard(x.device());
  const int N = (int)x.size(0), V = (int)W.size(0), E = (int)x.size(1);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor dx, dW, db;
  if (need_dx) {
    dx = at::empty_like(x);
    at::Tensor acc;
    if (dpa::lxent_dx_needs_acc(N)) acc = at::zeros({(int64_t)N * E}, f32);
    if (N > 0)
      dpa::launch_lxent_dx(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), tgt.data_ptr<int64_t>(),
                           lse.data_ptr<float>(), dloss.data_ptr<float>(), N, V, E,
                           reinterpret_cast<uint16_t*>(dx.data_ptr()),
                           acc.defined() ? acc.data_ptr<float>() : nullptr, cur_stream());
  }
  auto acc_ok = [&](const c10::optional<at::Tensor>& t, int64_t numel) {
    return t.has_value() && t->defined() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
           t->numel() == numel && t->device() == x.device();
  };
  const bool ext_w = need_dw && acc_ok(dw_acc, (int64_t)V * E), ext_b = need_db && acc_ok(db_acc, V);
  if (need_dw || need_db) {
    dW = ext_w ? *dw_acc : at::zeros({V, E}, f32);
    if (need_db) db = ext_b ? *db_acc : at::zeros({V}, f32);
    const bool scatter = onehot_scatter && need_dw && (E == 128 || E == 256);
    if (N > 0) {
      const int64_t wsn = dpa::lxent_dw_ws_floats(N, V, E);
      at::Tensor ws = wsn > 0 ? at::empty({wsn}, f32) : at::Tensor();
      dpa::launch_lxent_dw(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), tgt.data_ptr<int64_t>(),
                           lse.data_ptr<float>(), dloss.data_ptr<float>(), N, V, E,
                           dW.data_ptr<float>(), need_db ? db.data_ptr<float>() : nullptr,
                           cur_stream(), !scatter, wsn > 0 ? ws.data_ptr<float>() : nullptr);
    }
    if (scatter && N > 0) {
      const at::Tensor valid = tgt.ge(0).logical_and(tgt.lt(V));
      const at::Tensor ng = at::where(valid, dloss.neg(), at::zeros({}, dloss.options()));
      emb_grad(tgt, x.to(at::kFloat).mul_(ng.unsqueeze(1)), dW);  // ids outside [0, V) are skipped
      if (need_db) db.index_add_(0, tgt.clamp(0, V - 1), ng);
    }
    if (!need_dw || ext_w) dW = at::Tensor();
    if (ext_b) db = at::Tensor();
  }
  return {dx, dW, db};
}

// ---- fused dropout + residual + LayerNorm ------------------------------------------
static std::vector<at::Tensor> add_ln_fwd(const at::Tensor& y, c10::optional<at::Tensor> res,
                                          const at::Tensor& g, const at::Tensor& b, double p,
                                          double eps, int64_t seed, int64_t offset,
                                          c10::optional<at::Tensor> pos, c10::optional<at::Tensor> temb,
                                          int64_t L, bool post, bool save_h, bool h_guard) {
  CHECK_DEV(y); CHECK_BF16(y); CHECK_CONTIG(y); CHECK_BF16(g); CHECK_BF16(b);
  TORCH_CHECK(y.dim() == 2, "y must be [R, D]");
  const int64_t R = y.size(0);
  const int D = (int)y.size(1);
  TORCH_CHECK(g.numel() == D && b.numel() == D, "gamma/beta size");
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    CHECK_BF16((*res)); CHECK_CONTIG((*res));
    TORCH_CHECK(res->sizes() == y.sizes(), "residual shape");
    rp = bf_ptr(*res);
  }
  // row-broadcast terms: pos [L, D] (row % L), temb [R / L, D] (row / L)
  const uint16_t* pp = nullptr;
  const uint16_t* tp = nullptr;
  if (pos.has_value() && pos->defined()) {
    CHECK_BF16((*pos)); CHECK_CONTIG((*pos));
    TORCH_CHECK(L > 0 && R % L == 0 && pos->numel() == L * D, "pos must be [L, D] with R % L == 0");
    pp = bf_ptr(*pos);
  }
  if (temb.has_value() && temb->defined()) {
    CHECK_BF16((*temb)); CHECK_CONTIG((*temb));
    TORCH_CHECK(L > 0 && R % L == 0 && temb->numel() == (R / L) * D, "temb must be [R / L, D]");
    tp = bf_ptr(*temb);
  }
  const c10::DeviceGuard guard(y.device());
  // save_h = false: no bf16 copy of h.  h_guard: the copy is written only for a gamma with
  // some |gamma| < 0.125 (norm.hip LN_XO_GMIN) - add_ln_bwd(beta=, hcopy=) reads it then and
  // reconstructs xhat from the output otherwise
  at::Tensor out = at::empty_like(y), hs = save_h ? at::empty_like(y) : at::Tensor();
  auto f32 = y.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({R}, f32), rstd = at::empty({R}, f32);
  bool ok = dpa::launch_add_ln_fwd(bf_ptr(y), rp, bf_ptr(g), bf_ptr(b),
                                   reinterpret_cast<uint16_t*>(out.data_ptr()),
                                   save_h ? reinterpret_cast<uint16_t*>(hs.data_ptr()) : nullptr,
                                   mean.data_ptr<float>(),
                                   rstd.data_ptr<float>(), R, D, (float)p, (float)eps,
                                   (uint32_t)seed, (uint32_t)offset, cur_stream(), pp, tp, (int)L, post,
                                   save_h && h_guard);
  TORCH_CHECK(ok, "add_ln_fwd: unsupported hidden size ", D);
  return {out, hs, mean, rstd};
}

static std::vector<at::Tensor> add_ln_bwd(const at::Tensor& dout, const at::Tensor& hs,
                                          const at::Tensor& mean, const at::Tensor& rstd,
                                          const at::Tensor& g, double p, int64_t seed,
                                          int64_t offset, bool need_dres, bool need_dy,
                                          bool want_dyb, c10::optional<at::Tensor> dh_in, bool post,
                                          c10::optional<at::Tensor> dg_acc, c10::optional<at::Tensor> db_acc,
                                          c10::optional<at::Tensor> dyb_acc, c10::optional<at::Tensor> part_buf,
                                          bool part_acc, c10::optional<at::Tensor> beta,
                                          c10::optional<at::Tensor> hcopy, bool pair_hash) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONTIG(dout); CHECK_BF16(hs); CHECK_CONTIG(hs);
  TORCH_CHECK(hs.sizes() == dout.sizes(), "add_ln_bwd: hsave/out shape");
  // beta given: `hs` is the LN output (forward with save_h=false), xhat = (out - beta) / gamma
  const uint16_t* btp = nullptr;
  if (beta.has_value() && beta->defined()) {
    CHECK_BF16((*beta)); CHECK_CONTIG((*beta));
    TORCH_CHECK(beta->numel() == dout.size(1) && !post, "add_ln_bwd: beta [D], pre-dropout placement only");
    TORCH_CHECK(hcopy.has_value() && hcopy->defined() && hcopy->sizes() == dout.sizes(),
                "add_ln_bwd: beta needs hcopy (the forward's guarded h copy)");
    CHECK_BF16((*hcopy)); CHECK_CONTIG((*hcopy));
    btp = bf_ptr(*beta);
  }
  const uint16_t* hcp = btp ? bf_ptr(*hcopy) : nullptr;
  const uint16_t* dhp = nullptr;
  if (dh_in.has_value() && dh_in->defined()) {
    CHECK_BF16((*dh_in)); CHECK_CONTIG((*dh_in));
    TORCH_CHECK(dh_in->sizes() == dout.sizes(), "dh_in shape");
    dhp = bf_ptr(*dh_in);
  }
  const int64_t R = dout.size(0);
  const int D = (int)dout.size(1);
  const c10::DeviceGuard guard(dout.device());
  at::Tensor dres, dy;
  if (need_dres) dres = at::empty_like(dout);
  if (need_dy) dy = at::empty_like(dout);
  auto f32 = dout.options().dtype(at::kFloat);
  // dgamma, dbeta and colsum(dy) as consecutive rows of one scratch buffer (one memset),
  // or accumulated straight onto given fp32 .grad buffers (returned undefined then: no
  // autograd-side add and no memset)
  auto acc_ok = [&](const c10::optional<at::Tensor>& t) {
    return t.has_value() && t->defined() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
           t->numel() == D && t->device() == dout.device();
  };
  at::Tensor acc3 = at::empty({3, D}, f32);
  at::Tensor dg = acc3[0], db = acc3[1], dyb;
  if (need_dy && want_dyb) dyb = acc3[2];
  int zero_mask = 7;
  const bool ext_g = acc_ok(dg_acc), ext_b = acc_ok(db_acc), ext_y = dyb.defined() && acc_ok(dyb_acc);
  if (ext_g) { dg = *dg_acc; zero_mask &= ~1; }
  if (ext_b) { db = *db_acc; zero_mask &= ~2; }
  if (ext_y) { dyb = *dyb_acc; zero_mask &= ~4; }
  const int64_t wsn = dpa::ln_bwd_ws_floats(R, D);
  at::Tensor ws;
  int part_mode = 0;
  if (part_buf.has_value() && part_buf->defined()) {
    // deferred column sums (caller-owned partials, reduced later by ln_colreduce): only
    // when every accumulator is a caller buffer - nothing is returned for them
    TORCH_CHECK(wsn > 0 && part_buf->numel() == wsn && part_buf->scalar_type() == at::kFloat &&
                    part_buf->is_contiguous() && part_buf->device() == dout.device(),
                "add_ln_bwd: part_buf must be fp32 [ln_bwd_partials(R, D)] on the device");
    TORCH_CHECK(ext_g && ext_b && (!dyb.defined() || ext_y), "add_ln_bwd: part_buf needs dg/db/dyb_acc");
    ws = *part_buf;
    part_mode = part_acc ? 2 : 1;
  } else if (wsn > 0) {
    ws = at::empty({wsn}, f32);
  }
  bool ok = dpa::launch_add_ln_bwd(
      bf_ptr(dout), bf_ptr(hs), mean.data_ptr<float>(), rstd.data_ptr<float>(), bf_ptr(g),
      need_dres ? reinterpret_cast<uint16_t*>(dres.data_ptr()) : nullptr,
      need_dy ? reinterpret_cast<uint16_t*>(dy.data_ptr()) : nullptr,
      dyb.defined() ? dyb.data_ptr<float>() : nullptr,
      dg.data_ptr<float>(), db.data_ptr<float>(), R, D, (float)p, (uint32_t)seed, (uint32_t)offset,
      cur_stream(), dhp, post, zero_mask, wsn > 0 ? ws.data_ptr<float>() : nullptr, part_mode, btp, hcp,
      pair_hash);
  TORCH_CHECK(ok, "add_ln_bwd: unsupported hidden size ", D);
  return {dres, dy, ext_g ? at::Tensor() : dg, ext_b ? at::Tensor() : db, ext_y ? at::Tensor() : dyb};
}

// floats of the caller-owned partial buffer add_ln_bwd(part_buf=...) takes for R x D (0: the
// shape has no two-stage column sums, no deferral)
static int64_t ln_bwd_partials(int64_t R, int64_t D) { return dpa::ln_bwd_ws_floats(R, (int)D); }

// dg += colsum, db += colsum (, dyb += colsum) of partials accumulated by add_ln_bwd(part_buf=...)
// (dpos [L][H] fp32 or empty, dtemb [B][H] fp32 or empty) of d [B * L][H] bf16 in one read;
// empty list if the shape is not supported
static std::vector<at::Tensor> seq_pos_sums(const at::Tensor& d, int64_t L, bool need_pos, bool need_temb) {
  CHECK_DEV(d); CHECK_BF16(d); CHECK_CONTIG(d);
  TORCH_CHECK(d.dim() == 2 && L > 0 && d.size(0) % L == 0, "d [B * L, H]");
  const int64_t B = d.size(0) / L, H = d.size(1);
  const c10::DeviceGuard guard(d.device());
  auto f32 = d.options().dtype(at::kFloat);
  at::Tensor dpos = need_pos ? at::zeros({L, H}, f32) : at::Tensor();
  at::Tensor dtemb = need_temb ? at::empty({B, H}, f32) : at::Tensor();
  at::Tensor part = need_pos ? at::empty({(int64_t)dpa::seq_pos_groups((int)B) * L * H}, f32) : at::Tensor();
  if (!dpa::launch_seq_pos_sums(reinterpret_cast<const uint16_t*>(d.data_ptr()), (int)B, (int)L, (int)H,
                                need_pos ? dpos.data_ptr<float>() : nullptr,
                                need_temb ? dtemb.data_ptr<float>() : nullptr,
                                need_pos ? part.data_ptr<float>() : nullptr, cur_stream()))
    return {};
  return {dpos, dtemb};
}

static void ln_colreduce(const at::Tensor& part, int64_t R, int64_t D, at::Tensor& dg, at::Tensor& db,
                         c10::optional<at::Tensor> dyb) {
  CHECK_DEV(part); CHECK_F32(part); CHECK_CONTIG(part); CHECK_F32(dg); CHECK_F32(db);
  TORCH_CHECK(part.numel() == dpa::ln_bwd_ws_floats(R, (int)D) && dg.numel() == D && db.numel() == D,
              "ln_colreduce shapes");
  float* yp = nullptr;
  if (dyb.has_value() && dyb->defined()) {
    CHECK_F32((*dyb));
    TORCH_CHECK(dyb->numel() == D, "ln_colreduce dyb");
    yp = dyb->data_ptr<float>();
  }
  const c10::DeviceGuard guard(part.device());
  TORCH_CHECK(dpa::launch_ln_colreduce(part.data_ptr<float>(), R, (int)D, dg.data_ptr<float>(),
                                       db.data_ptr<float>(), yp, cur_stream()),
              "ln_colreduce: no two-stage shape");
}

// dst += column sums of fp32 partials [rows, cols] (the kept gemm_nn_dact partials)
static void colsum_acc(const at::Tensor& part, at::Tensor& dst) {
  CHECK_DEV(part); CHECK_F32(part); CHECK_CONTIG(part); CHECK_F32(dst); CHECK_CONTIG(dst);
  TORCH_CHECK(part.dim() == 2 && dst.numel() == part.size(1), "colsum_acc shapes");
  const c10::DeviceGuard guard(part.device());
  if (!dpa::launch_colsum_acc(part.data_ptr<float>(), (int)part.size(0), (int)part.size(1), dst.data_ptr<float>(),
                              cur_stream()))
    dst.add_(part.sum(0));
}

// ---- bias + activation epilogues ------------------------------------------------------
static std::vector<at::Tensor> bias_act_fwd(at::Tensor& z, c10::optional<at::Tensor> b, int64_t act) {
  CHECK_DEV(z); CHECK_BF16(z); CHECK_CONTIG(z);
  TORCH_CHECK(z.dim() == 2 && z.size(1) % 8 == 0, "z must be [R, N] with N % 8 == 0");
  const int64_t R = z.size(0);
  const int N = (int)z.size(1);
  const uint16_t* bp = opt_bf_ptr(b);
  if (bp) TORCH_CHECK(b->numel() == N, "bias size");
  const c10::DeviceGuard guard(z.device());
  at::Tensor y = act == 0 ? z : at::empty_like(z);
  if (bp || act != 0)
    dpa::launch_bias_act_fwd(reinterpret_cast<uint16_t*>(z.data_ptr()), bp,
                             act == 0 ? nullptr : reinterpret_cast<uint16_t*>(y.data_ptr()), R, N,
                             (int)act, cur_stream());
  return {z, y};
}

static std::vector<at::Tensor> bias_act_bwd(const at::Tensor& dy, const at::Tensor& zy, int64_t act,
                                            bool want_db) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy);
  const int64_t R = dy.size(0);
  const int N = (int)dy.size(1);
  TORCH_CHECK(N % 8 == 0, "N % 8");
  const c10::DeviceGuard guard(dy.device());
  at::Tensor dz = act == 0 ? dy : at::empty_like(dy);
  at::Tensor db;
  if (want_db) db = at::zeros({N}, dy.options().dtype(at::kFloat));
  if (act != 0 || want_db) {
    CHECK_CONTIG(zy);
    at::Tensor ws = want_db ? at::empty({dpa::bias_act_bwd_ws_floats(R, N)}, dy.options().dtype(at::kFloat))
                            : at::Tensor();
    dpa::launch_bias_act_bwd(bf_ptr(dy), bf_ptr(zy),
                             act == 0 ? nullptr : reinterpret_cast<uint16_t*>(dz.data_ptr()),
                             want_db ? db.data_ptr<float>() : nullptr, R, N, (int)act, cur_stream(),
                             want_db ? ws.data_ptr<float>() : nullptr);
  }
  return {dz, db};
}

// ---- attention ---------------------------------------------------------------------
static std::vector<at::Tensor> attn_fwd(const at::Tensor& qkv, int64_t heads, double p, bool causal,
                                        int64_t seed, int64_t offset, bool head_major) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_CONTIG(qkv);
  TORCH_CHECK(qkv.dim() == 3, "qkv must be [B, L, 3*H*D]");
  const int B = (int)qkv.size(0), L = (int)qkv.size(1), H = (int)heads;
  TORCH_CHECK(H > 0 && qkv.size(2) % (3LL * H) == 0, "attn: qkv width must be 3*H*D");
  const int D = (int)(qkv.size(2) / (3LL * H));
  TORCH_CHECK(D == 64 || D == 128, "attn: head_dim must be 64 or 128");
  TORCH_CHECK(L % 64 == 0, "attn: L must be a multiple of 64");
  const c10::DeviceGuard guard(qkv.device());
  at::Tensor out = at::empty({B, L, (int64_t)H * D}, qkv.options());
  at::Tensor lse = at::empty({B, H, L}, qkv.options().dtype(at::kFloat));
  TORCH_CHECK(!head_major || dpa::attn128_supports(L, D, causal),
              "attn_fwd: the head-major qkv layout needs L == 128, head_dim 64, bidirectional");
  const bool ok = dpa::launch_attn_fwd(bf_ptr(qkv), reinterpret_cast<uint16_t*>(out.data_ptr()),
                                       lse.data_ptr<float>(), B, L, H, D, (float)p, causal, (uint32_t)seed,
                                       (uint32_t)offset, cur_stream(), head_major);
  TORCH_CHECK(ok, "attn_fwd: no kernel for this shape");
  return {out, lse};
}

// dsts[i] = srcs[i]^T (bf16 2-D, rows / cols multiples of 64), batched into launches of <= MAXN
static bool transpose_bf16_batch(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "transpose_bf16_batch: src / dst lists differ");
  if (srcs.empty()) return true;
  // every shape is validated before the first chunk launches: a False return means nothing ran
  for (const at::Tensor& a : srcs)
    if (a.dim() != 2 || a.size(0) % 64 || a.size(1) % 64) return false;
  const c10::DeviceGuard guard(srcs[0].device());
  size_t i = 0;
  while (i < srcs.size()) {
    dpa::TransposeBatch d{};
    int n = 0, tiles = 0;
    for (; i < srcs.size() && n < dpa::TransposeBatch::MAXN; ++i, ++n) {
      const at::Tensor &a = srcs[i], &b = dsts[i];
      TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && a.dim() == 2 &&
                      b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && b.size(0) == a.size(1) &&
                      b.size(1) == a.size(0) && a.device() == b.device(),
                  "transpose_bf16_batch: bf16 contiguous [R, C] -> [C, R]");
      d.src[n] = reinterpret_cast<const uint16_t*>(a.data_ptr());
      d.dst[n] = reinterpret_cast<uint16_t*>(b.data_ptr());
      d.rows[n] = (int)a.size(0);
      d.cols[n] = (int)a.size(1);
      d.tile_start[n] = tiles;
      tiles += (int)(a.size(0) / 64) * (int)(a.size(1) / 64);
    }
    d.n = n;
    d.tile_start[n] = tiles;
    if (!dpa::launch_transpose_bf16_batch(d, cur_stream())) return false;
  }
  return true;
}

static void attn_colpart_reduce(const at::Tensor& part, int64_t R, int64_t H, int64_t D, at::Tensor db) {
  CHECK_DEV(part);
  TORCH_CHECK(part.scalar_type() == at::kFloat && db.scalar_type() == at::kFloat && part.is_contiguous() &&
                  db.is_contiguous() && part.numel() >= R * H * 3 * D && db.numel() == 3 * H * D &&
                  D % 64 == 0 && R > 0,
              "attn_colpart_reduce: fp32 part [R*H][3D], db [3HD]");
  const c10::DeviceGuard guard(part.device());
  dpa::launch_colpart_reduce(part.data_ptr<float>(), db.data_ptr<float>(), (int)R, (int)H, (int)D, cur_stream());
}

static std::vector<at::Tensor> attn_bwd(const at::Tensor& dout, const at::Tensor& qkv,
                                        const at::Tensor& out, const at::Tensor& lse, int64_t heads,
                                        double p, bool causal, int64_t seed, int64_t offset,
                                        bool want_db, bool head_major, c10::optional<at::Tensor> db_acc,
                                        c10::optional<at::Tensor> part_out) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONTIG(dout); CHECK_CONTIG(out); CHECK_CONTIG(qkv);
  const int B = (int)qkv.size(0), L = (int)qkv.size(1), H = (int)heads;
  TORCH_CHECK(dout.sizes() == out.sizes(), "dout shape");
  TORCH_CHECK(H > 0 && qkv.size(2) % (3LL * H) == 0, "attn: qkv width must be 3*H*D");
  const int D = (int)(qkv.size(2) / (3LL * H));
  TORCH_CHECK(D == 64 || D == 128, "attn: head_dim must be 64 or 128");
  TORCH_CHECK(L % 64 == 0 && out.size(2) == (int64_t)H * D, "attn_bwd: shapes");
  TORCH_CHECK(lse.numel() == (int64_t)B * H * L, "attn_bwd: lse shape");
  TORCH_CHECK(!head_major || dpa::attn128_supports(L, D, causal),
              "attn_bwd: the head-major qkv layout needs L == 128, head_dim 64, bidirectional");
  const c10::DeviceGuard guard(qkv.device());
  at::Tensor dqkv = at::empty_like(qkv);
  auto f32 = qkv.options().dtype(at::kFloat);
  at::Tensor delta = at::empty({B, H, L}, f32);
  at::Tensor dq, colpart, db;
  if (dpa::attn_bwd_needs_dq_acc(L)) dq = at::zeros({B, L, H, D}, f32);
  // db_acc: the qkv bias gradient accumulated straight onto this fp32 .grad (returned undefined)
  const bool acc = want_db && db_acc.has_value() && db_acc->defined() && db_acc->scalar_type() == at::kFloat &&
                   db_acc->is_contiguous() && db_acc->numel() == 3LL * H * D && db_acc->device() == qkv.device();
  // part_out: a caller-owned fp32 slot of attn_colpart_rows * 3 D floats; the bias-gradient
  // partials are left there for a later colpart_reduce (deferral window), db is not produced
  const int64_t cp_n = dpa::attn_colpart_rows(B, L, H, D, causal) * 3 * D;
  const bool defer = want_db && acc && part_out.has_value() && part_out->defined() &&
                     part_out->scalar_type() == at::kFloat && part_out->is_contiguous() &&
                     part_out->numel() >= cp_n && part_out->device() == qkv.device();
  if (want_db) {
    colpart = defer ? *part_out : at::empty({cp_n}, f32);
    db = acc ? *db_acc : at::empty({3 * H * D}, f32);
  }
  bool got = dpa::launch_attn_bwd(
      bf_ptr(qkv), bf_ptr(out), bf_ptr(dout), lse.data_ptr<float>(), delta.data_ptr<float>(),
      reinterpret_cast<uint16_t*>(dqkv.data_ptr()), dq.defined() ? dq.data_ptr<float>() : nullptr,
      want_db ? colpart.data_ptr<float>() : nullptr, want_db ? db.data_ptr<float>() : nullptr, B, L,
      H, D, (float)p, causal, (uint32_t)seed, (uint32_t)offset, cur_stream(), head_major, acc, defer);
  if (defer) {
    TORCH_CHECK(got, "attn_bwd: deferred column sums on a path without partials");
    return {dqkv, at::Tensor()};
  }
  if (want_db && !got) {
    // no fused column sums on this path (L != 128): one column-sum pass over the bf16 dqkv,
    // accumulated onto db (zeroed unless it is the parameter's .grad)
    if (!acc) db.zero_();
    const int Nq = (int)(3LL * H * D);
    at::Tensor ws = at::empty({dpa::bias_act_bwd_ws_floats((int64_t)B * L, Nq)}, db.options());
    dpa::launch_bias_act_bwd(bf_ptr(dqkv), nullptr, nullptr, db.data_ptr<float>(), (int64_t)B * L, Nq, 0,
                             cur_stream(), ws.data_ptr<float>());
    got = true;
  }
  // contract: with a usable db_acc the bias gradient is always accumulated (result undefined)
  return {dqkv, got && !acc ? db : at::Tensor()};
}

// ---- GEMMs ---------------------------------------------------------------------------
// want_deriv: 0 z = pre-activation; 1 z = act'(pre-activation) (bf16) when the persistent kernel
// runs; 2 z = act' as u8 codes in the persistent kernels' tile-native layout ([T * N] uint8, read
// back only by gemm_nn_dact(act=5)).  Returns (y, z, mode): the z that was written (0 / 1 / 2).
static std::tuple<at::Tensor, at::Tensor, int64_t> gemm_nt(const at::Tensor& x, const at::Tensor& W,
                                                           c10::optional<at::Tensor> b, int64_t act,
                                                           int64_t want_deriv, int64_t head_major_L) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(W); CHECK_CONTIG(x); CHECK_CONTIG(W);
  const int T = (int)x.size(0), K = (int)x.size(1), N = (int)W.size(0);
  TORCH_CHECK(W.size(1) == K, "gemm_nt: W [N, K]");
  const c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty({T, N}, x.options());
  at::Tensor z;
  if (want_deriv == 2 && (act == 1 || act == 3) && head_major_L <= 0) {
    at::Tensor z8 = at::empty({(int64_t)T * N}, x.options().dtype(at::kByte));
    if (dpa::launch_gemmp_nt(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), reinterpret_cast<uint16_t*>(y.data_ptr()),
                             reinterpret_cast<uint16_t*>(z8.data_ptr()), T, N, K, (int)act, dpa::device_cu_count(),
                             cur_stream(), true, 0, true))
      return {y, z8, 2};
  }
  if (act == 1 || act == 3) z = at::empty({T, N}, x.options());
  bool deriv = want_deriv != 0 && z.defined();
  // head_major_L > 0: y stored as [T / L, N / 64, L, 64] (heads of 64 columns; the L = 128
  // attention reads each head contiguously)
  int hm = 0;
  if (head_major_L > 0) {
    while ((1LL << hm) < head_major_L) ++hm;
    TORCH_CHECK((1LL << hm) == head_major_L && act == 0, "gemm_nt: head-major store needs a power-of-2 L, no act");
  }
  bool ok = dpa::launch_gemm_nt(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b),
                                reinterpret_cast<uint16_t*>(y.data_ptr()),
                                z.defined() ? reinterpret_cast<uint16_t*>(z.data_ptr()) : nullptr, T, N,
                                K, (int)act, cur_stream(), &deriv, hm);
  TORCH_CHECK(ok, "gemm_nt: unsupported shape T=", T, " N=", N, " K=", K);
  return {y, z, deriv ? 1 : 0};
}

// h = res + dropout_p(x W^T + b) (post-LN sublayer branch + residual in the GEMM epilogue;
// pair-hash dropout bits, regenerated by add_ln_bwd(pair_hash=True)); undefined when the shape
// does not tile for the persistent kernel (the caller composes the old way)
static at::Tensor gemm_nt_res(const at::Tensor& x, const at::Tensor& W, c10::optional<at::Tensor> b,
                              const at::Tensor& res, double p, int64_t seed, int64_t offset) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(W); CHECK_CONTIG(x); CHECK_CONTIG(W);
  CHECK_BF16(res); CHECK_CONTIG(res);
  const int T = (int)x.size(0), K = (int)x.size(1), N = (int)W.size(0);
  TORCH_CHECK(W.size(1) == K && res.dim() == 2 && res.size(0) == T && res.size(1) == N, "gemm_nt_res shapes");
  const c10::DeviceGuard guard(x.device());
  at::Tensor h = at::empty({T, N}, x.options());
  if (!dpa::launch_gemmp_nt_res(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), bf_ptr(res),
                                reinterpret_cast<uint16_t*>(h.data_ptr()), T, N, K, dpa::device_cu_count(),
                                cur_stream(), (float)p, (uint32_t)seed, (uint32_t)offset))
    return at::Tensor();
  return h;
}

// y = x . W^T (+ b) into a preallocated row-major [T, N] tensor (a row slice of a larger
// buffer, e.g. the LM head's [tokens, padded vocab] logits).
static void gemm_nt_into(const at::Tensor& x, const at::Tensor& W, c10::optional<at::Tensor> b,
                         at::Tensor& out) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(W); CHECK_BF16(out); CHECK_CONTIG(x); CHECK_CONTIG(W);
  CHECK_CONTIG(out);
  const int T = (int)x.size(0), K = (int)x.size(1), N = (int)W.size(0);
  TORCH_CHECK(W.size(1) == K && out.dim() == 2 && out.size(0) == T && out.size(1) == N, "gemm_nt_into shapes");
  const c10::DeviceGuard guard(x.device());
  bool ok = dpa::launch_gemm_nt(bf_ptr(x), bf_ptr(W), opt_bf_ptr(b), reinterpret_cast<uint16_t*>(out.data_ptr()),
                                nullptr, T, N, K, 0, cur_stream(), nullptr);
  TORCH_CHECK(ok, "gemm_nt_into: unsupported shape T=", T, " N=", N, " K=", K);
}

// dx = dy . W into a preallocated [T, K] tensor.
static void gemm_nn_into(const at::Tensor& dy, const at::Tensor& W, at::Tensor& dx) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_BF16(W); CHECK_BF16(dx); CHECK_CONTIG(dy); CHECK_CONTIG(W);
  CHECK_CONTIG(dx);
  const int T = (int)dy.size(0), N = (int)dy.size(1), K = (int)W.size(1);
  TORCH_CHECK(W.size(0) == N && dx.size(0) == T && dx.size(1) == K, "gemm_nn_into shapes");
  const c10::DeviceGuard guard(dy.device());
  bool ok = dpa::launch_gemm_nn(bf_ptr(dy), bf_ptr(W), reinterpret_cast<uint16_t*>(dx.data_ptr()), T, N, K,
                                cur_stream());
  TORCH_CHECK(ok, "gemm_nn_into: unsupported shape T=", T, " N=", N, " K=", K);
}

// (sorted ids, permutation) with equal ids adjacent in index order: the stable counting sort of
// csrc/sort.hip (block histograms, scans, ordered scatter) for vocabularies up to 81919, else a
// stable at::sort.
static std::tuple<at::Tensor, at::Tensor> bucket_sort_ids(const at::Tensor& ids, int64_t V) {
  const at::Tensor flat = ids.reshape({-1}).contiguous();
  const int64_t n = flat.numel();
  auto i64 = flat.options().dtype(at::kLong);
  at::Tensor sorted = at::empty({n}, i64), perm = at::empty({n}, i64);
  const int Vc = (int)std::min<int64_t>(V, 1 << 20);
  at::Tensor ws = at::empty({dpa::id_sort_workspace_ints(n, Vc)}, flat.options().dtype(at::kInt));
  if (V < (1 << 17) &&
      dpa::launch_id_bucket_sort(flat.data_ptr<int64_t>(), n, (int)V, ws.data_ptr<int>(),
                                 sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), cur_stream()))
    return {sorted, perm};
  return at::sort(flat, /*stable=*/true, 0, false);
}

static std::vector<at::Tensor> id_sort(const at::Tensor& ids, int64_t V) {
  CHECK_DEV(ids);
  TORCH_CHECK(ids.scalar_type() == at::kLong && V > 0, "id_sort: int64 ids, V > 0");
  const c10::DeviceGuard guard(ids.device());
  if (ids.numel() == 0) return {ids.reshape({-1}), ids.reshape({-1})};
  at::Tensor s, p;
  std::tie(s, p) = bucket_sort_ids(ids, V);
  return {s, p};
}

// order of a 0/1 (any nonzero = 1) int64 mask: nonzero entries first, both parts in index order
static at::Tensor partition01(const at::Tensor& mask) {
  CHECK_DEV(mask);
  TORCH_CHECK(mask.scalar_type() == at::kLong, "partition01: int64 mask");
  const c10::DeviceGuard guard(mask.device());
  const at::Tensor flat = mask.reshape({-1}).contiguous();
  const int64_t n = flat.numel();
  at::Tensor order = at::empty({n}, flat.options());
  if (n == 0) return order;
  at::Tensor ws = at::empty({dpa::partition01_workspace_ints(n)}, flat.options().dtype(at::kInt));
  TORCH_CHECK(dpa::launch_partition01(flat.data_ptr<int64_t>(), n, ws.data_ptr<int>(), order.data_ptr<int64_t>(),
                                      cur_stream()),
              "partition01: unsupported size ", n);
  return order;
}

// dW[ids[i]] += dy[i] (fp32 accumulate): counting sort of the ids, then one wave per run
// of equal ids sums its rows in registers and adds once (csrc/diffusion.hip) - the
// token-embedding backward without ATen's index_add.
static void emb_grad(const at::Tensor& ids, const at::Tensor& dy, at::Tensor& dW) {
  CHECK_DEV(ids); CHECK_DEV(dy); CHECK_DEV(dW); CHECK_CONTIG(dy); CHECK_CONTIG(dW); CHECK_F32(dW);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "emb_grad: int64 ids");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kFloat, "emb_grad: bf16/fp32 dy");
  const int64_t NT = ids.numel(), E = dW.size(1);
  TORCH_CHECK(dy.numel() == NT * E, "emb_grad: dy [ids..., E]");
  if (NT == 0) return;
  const c10::DeviceGuard guard(dW.device());
  at::Tensor sorted, perm;
  std::tie(sorted, perm) = bucket_sort_ids(ids, dW.size(0));
  const bool b16 = dy.scalar_type() == at::kBFloat16;
  at::Tensor part = at::empty({dpa::emb_grad_part_floats(NT, (int)E, false)}, dW.options());
  TORCH_CHECK(dpa::launch_emb_grad(sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(),
                                   b16 ? nullptr : dy.data_ptr<float>(), b16 ? bf_ptr(dy) : nullptr, NT, (int)E,
                                   (int)dW.size(0), dW.data_ptr<float>(), part.data_ptr<float>(), cur_stream()),
              "emb_grad: unsupported embedding width ", E);
}

// optional transposed weight W^T [K][N] (bf16, contiguous) of a data-gradient GEMM: nullptr when
// absent; a tensor of any other shape / dtype is a caller bug
static const uint16_t* wt_ptr(const c10::optional<at::Tensor>& wt, const at::Tensor& W) {
  if (!wt.has_value() || !wt->defined()) return nullptr;
  TORCH_CHECK(wt->scalar_type() == at::kBFloat16 && wt->is_contiguous() && wt->dim() == 2 &&
                  wt->size(0) == W.size(1) && wt->size(1) == W.size(0) && wt->device() == W.device(),
              "wt must be W^T: bf16 contiguous [K, N]");
  return reinterpret_cast<const uint16_t*>(wt->data_ptr());
}

static at::Tensor gemm_nn(const at::Tensor& dy, const at::Tensor& W, c10::optional<at::Tensor> wt) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_BF16(W); CHECK_CONTIG(dy); CHECK_CONTIG(W);
  const int T = (int)dy.size(0), N = (int)dy.size(1), K = (int)W.size(1);
  TORCH_CHECK(W.size(0) == N, "gemm_nn: W [N, K]");
  const c10::DeviceGuard guard(dy.device());
  at::Tensor dx = at::empty({T, K}, dy.options());
  bool ok = dpa::launch_gemm_nn(bf_ptr(dy), bf_ptr(W), reinterpret_cast<uint16_t*>(dx.data_ptr()), T,
                                N, K, cur_stream(), wt_ptr(wt, W));
  TORCH_CHECK(ok, "gemm_nn: unsupported shape");
  return dx;
}

// dx += dy . W in place (the residual-branch gradient accumulated by the dgrad GEMM);
// false when the shape does not tile (caller adds separately).
static bool gemm_nn_acc_(const at::Tensor& dy, const at::Tensor& W, at::Tensor& dx, c10::optional<at::Tensor> wt) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_BF16(W); CHECK_BF16(dx);
  CHECK_CONTIG(dy); CHECK_CONTIG(W); CHECK_CONTIG(dx);
  const int T = (int)dy.size(0), N = (int)dy.size(1), K = (int)W.size(1);
  TORCH_CHECK(W.size(0) == N && dx.size(0) == T && dx.size(1) == K, "gemm_nn_acc_ shapes");
  const c10::DeviceGuard guard(dy.device());
  return dpa::launch_gemmp_nn_acc(bf_ptr(dy), bf_ptr(W), reinterpret_cast<uint16_t*>(dx.data_ptr()), T, N, K,
                                  dpa::device_cu_count(), cur_stream(), wt_ptr(wt, W));
}

// dz = (dy . W) * act'(aux) [, db = colsum(dz) fp32 when want_db]; returns undefined
// tensors when the shape does not tile for a fused kernel (caller falls back to dgrad +
// separate act backward).  The persistent kernel writes per-tile column partials that
// one reduction turns into db (no second pass over dz).
static std::vector<at::Tensor> gemm_nn_dact(const at::Tensor& dy, const at::Tensor& W,
                                            const at::Tensor& aux, int64_t act, bool want_db,
                                            c10::optional<at::Tensor> db_acc,
                                            c10::optional<at::Tensor> part_out, c10::optional<at::Tensor> wt) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_BF16(W);
  CHECK_CONTIG(dy); CHECK_CONTIG(W); CHECK_CONTIG(aux);
  const int T = (int)dy.size(0), N = (int)dy.size(1), K = (int)W.size(1);
  // act 5: aux = u8 act' codes of gemm_nt(want_deriv=2) ([T * K] bytes, tile-native)
  if (act == 5) {
    TORCH_CHECK(aux.scalar_type() == at::kByte && aux.numel() == (int64_t)T * K, "gemm_nn_dact: act 5 aux u8 [T*K]");
  } else {
    TORCH_CHECK(aux.scalar_type() == at::kBFloat16 && aux.dim() == 2 && aux.size(0) == T && aux.size(1) == K,
                "gemm_nn_dact: bf16 aux [T, K]");
  }
  TORCH_CHECK(W.size(0) == N, "gemm_nn_dact shapes");
  const c10::DeviceGuard guard(dy.device());
  at::Tensor dz = at::empty({T, K}, dy.options());
  uint16_t* dzp = reinterpret_cast<uint16_t*>(dz.data_ptr());
  // part_out: the caller keeps the column-sum partials [(T/256)*2, K] and reduces them later
  // (several micro-batches' partials in one colsum_acc launch); nothing is returned for db
  const bool keep = want_db && part_out.has_value() && part_out->defined();
  // db_acc: the column sums accumulated straight onto this fp32 .grad (contract: always
  // accumulated when db_acc is usable; the result is then undefined)
  const bool acc = !keep && want_db && db_acc.has_value() && db_acc->defined() &&
                   db_acc->scalar_type() == at::kFloat && db_acc->is_contiguous() && db_acc->numel() == K &&
                   db_acc->device() == dy.device();
  at::Tensor part;
  if (keep) {
    TORCH_CHECK(T % 256 == 0 && part_out->scalar_type() == at::kFloat && part_out->is_contiguous() &&
                    part_out->numel() == (int64_t)(T / 256) * 2 * K && part_out->device() == dy.device(),
                "gemm_nn_dact: part_out must be fp32 [(T/256)*2, K]");
    part = *part_out;
  } else if (want_db && T % 256 == 0) {
    part = at::empty({(int64_t)(T / 256) * 2, K}, dy.options().dtype(at::kFloat));
  }
  if (dpa::launch_gemmp_nn(bf_ptr(dy), bf_ptr(W), dzp, reinterpret_cast<const uint16_t*>(aux.data_ptr()),
                           (int)act, T, N, K, dpa::device_cu_count(), cur_stream(),
                           part.defined() ? part.data_ptr<float>() : nullptr, wt_ptr(wt, W))) {
    if (keep) return {dz, at::Tensor()};
    if (acc) {
      if (!part.defined() || !dpa::launch_colsum_acc(part.data_ptr<float>(), (int)part.size(0), K,
                                                     db_acc->data_ptr<float>(), cur_stream()))
        db_acc->add_(dz.sum(0, false, at::kFloat));
      return {dz, at::Tensor()};
    }
    return {dz, part.defined() ? part.sum(0) : at::Tensor()};
  }
  // no persistent kernel for this shape: the column sums from dz itself (a kept partial slot
  // gets them in row 0, zeros elsewhere; all zeros when no fused kernel ran either - the
  // caller then computes db itself)
  if (keep) part_out->zero_();
  // u8 act' codes (act 5) are read only by the persistent kernel: decline, and the caller decodes
  // the codes and runs the plain dgrad + bias_act_bwd (a launcher gate flipped between the q8
  // forward and this backward, e.g. set_gemm256(False) in an A/B, must not crash the step)
  if (act == 5) return {at::Tensor(), at::Tensor()};
  if (dpa::launch_gemm256_nn_dact(bf_ptr(dy), bf_ptr(W), bf_ptr(aux), dzp, T, N, K, (int)act, cur_stream())) {
    if (!want_db) return {dz, at::Tensor()};
    at::Tensor cs = dz.sum(0, false, at::kFloat);
    if (keep) (*part_out)[0].copy_(cs);
    if (keep || acc) {
      if (acc) db_acc->add_(cs);
      return {dz, at::Tensor()};
    }
    return {dz, cs};
  }
  return {at::Tensor(), at::Tensor()};
}

static void gemm_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor& dW,
                       c10::optional<at::Tensor> db) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_BF16(x); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  CHECK_F32(dW); CHECK_CONTIG(dW);
  const int T = (int)dy.size(0), N = (int)dy.size(1), K = (int)x.size(1);
  TORCH_CHECK(x.size(0) == T && dW.size(0) == N && dW.size(1) == K, "gemm_wgrad shapes");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    CHECK_F32((*db)); TORCH_CHECK(db->numel() == N, "db size");
    dbp = db->data_ptr<float>();
  }
  const c10::DeviceGuard guard(dy.device());
  // A 128-wide side (DiffuSeq's 128 <-> 768 up / down projections) is not a 256 x 256 tile
  // shape: the 128-tile kernel then merges its ~170 token splits with device-scope fp32
  // atomics, which run at the memory side (0.39 ms for a 0.05 TFLOP gradient).  Zero-padding
  // that side to 256 (a [T, 256] copy) runs it on the 256 x 256 split-K kernel with its
  // workspace merge instead; the padded half of the result is discarded.
  constexpr bool pad_ok = true;
  const int Np = (N + 255) / 256 * 256, Kp = (K + 255) / 256 * 256;
  if (pad_ok && (Np != N || Kp != K) && N % 64 == 0 && K % 64 == 0 && T % 256 == 0 && T >= 256 &&
      (int64_t)Np * Kp <= 2 * (int64_t)N * K) {
    at::Tensor dyp = Np == N ? dy : at::constant_pad_nd(dy, {0, Np - N});
    at::Tensor xp = Kp == K ? x : at::constant_pad_nd(x, {0, Kp - K});
    at::Tensor dWp = at::zeros({Np, Kp}, dW.options());
    at::Tensor dbp2 = dbp ? at::zeros({Np}, dW.options()) : at::Tensor();
    const int64_t wsp = dpa::gemm256_wgrad_workspace_floats(T, Np, Kp);
    at::Tensor wsb = at::empty({wsp}, dW.options());
    if (dpa::launch_gemm256_wgrad(bf_ptr(dyp), bf_ptr(xp), dWp.data_ptr<float>(),
                                  dbp ? dbp2.data_ptr<float>() : nullptr, T, Np, Kp, cur_stream(),
                                  wsp ? wsb.data_ptr<float>() : nullptr)) {
      dW.add_(dWp.narrow(0, 0, N).narrow(1, 0, K));
      if (dbp) db->add_(dbp2.narrow(0, 0, N));
      return;
    }
  }
  // split-K merge workspace (stream-ordered caching-allocator block, freed after the launch)
  const int64_t wsn = dpa::gemm256_wgrad_workspace_floats(T, N, K);
  at::Tensor ws = at::empty({wsn}, dW.options());
  bool ok = dpa::launch_gemm_wgrad(bf_ptr(dy), bf_ptr(x), dW.data_ptr<float>(), dbp, T, N, K,
                                   cur_stream(), wsn ? ws.data_ptr<float>() : nullptr);
  TORCH_CHECK(ok, "gemm_wgrad: unsupported shape");
}

// dW += sum_s dy_s^T x_s (+ db += colsum) over equal-length token segments in one launch
// (the reference schedule's deferred micro-batch weight gradients); false if the shape is not
// supported by the multi-segment kernel (the caller then runs the segments one by one)
static bool gemm_wgrad_multi(const std::vector<at::Tensor>& dys, const std::vector<at::Tensor>& xs, at::Tensor& dW,
                             c10::optional<at::Tensor> db) {
  TORCH_CHECK(!dys.empty() && dys.size() == xs.size(), "gemm_wgrad_multi: segment lists");
  const int nseg = (int)dys.size();
  if (nseg > 8) return false;  // g256::WG_MAXSEG
  CHECK_F32(dW); CHECK_CONTIG(dW);
  const int T = (int)dys[0].size(0), N = (int)dys[0].size(1), K = (int)xs[0].size(1);
  std::vector<const uint16_t*> dp(nseg), xp(nseg);
  for (int i = 0; i < nseg; ++i) {
    CHECK_DEV(dys[i]); CHECK_BF16(dys[i]); CHECK_BF16(xs[i]); CHECK_CONTIG(dys[i]); CHECK_CONTIG(xs[i]);
    TORCH_CHECK(dys[i].dim() == 2 && xs[i].dim() == 2 && dys[i].size(0) == T && dys[i].size(1) == N &&
                xs[i].size(0) == T && xs[i].size(1) == K, "gemm_wgrad_multi: segment shapes");
    TORCH_CHECK(dys[i].device() == dW.device() && xs[i].device() == dW.device(), "gemm_wgrad_multi: devices");
    dp[i] = bf_ptr(dys[i]);
    xp[i] = bf_ptr(xs[i]);
  }
  TORCH_CHECK(dW.size(0) == N && dW.size(1) == K, "gemm_wgrad_multi: dW shape");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    CHECK_F32((*db)); TORCH_CHECK(db->numel() == N, "db size");
    dbp = db->data_ptr<float>();
  }
  const c10::DeviceGuard guard(dW.device());
  const int64_t wsn = dpa::gemm256_wgrad_workspace_floats(T, N, K, nseg);
  at::Tensor ws = at::empty({wsn}, dW.options());
  return dpa::launch_gemm256_wgrad_multi(dp.data(), xp.data(), nseg, dW.data_ptr<float>(), dbp, T, N, K,
                                         cur_stream(), wsn ? ws.data_ptr<float>() : nullptr);
}

// Grouped weight gradients (one launch per deferral flush): site i adds sum_s dys[i][s]^T xs[i][s]
// into dWs[i] (+ column sums of the dy segments into dbs[i] when defined).  False (nothing
// launched) when a site does not tile; the caller then runs the sites one by one.  The site table
// goes to the device through a pinned staging copy on the current stream.
static bool gemm_wgrad_grouped(const std::vector<std::vector<at::Tensor>>& dys,
                               const std::vector<std::vector<at::Tensor>>& xs, const std::vector<at::Tensor>& dWs,
                               const std::vector<c10::optional<at::Tensor>>& dbs) {
  const size_t ns = dys.size();
  TORCH_CHECK(ns > 0 && xs.size() == ns && dWs.size() == ns && dbs.size() == ns, "gemm_wgrad_grouped: site lists");
  std::vector<dpa::WgGroupSite> sites(ns);
  for (size_t i = 0; i < ns; ++i) {
    const auto& d = dys[i];
    const auto& x = xs[i];
    const at::Tensor& dW = dWs[i];
    TORCH_CHECK(!d.empty() && d.size() == x.size(), "gemm_wgrad_grouped: segment lists of site ", i);
    if (d.size() > 8) return false;
    CHECK_F32(dW); CHECK_CONTIG(dW);
    const int64_t T = d[0].size(0), M = d[0].size(1), N = x[0].size(1);
    TORCH_CHECK(dW.dim() == 2 && dW.size(0) == M && dW.size(1) == N, "gemm_wgrad_grouped: dW shape of site ", i);
    dpa::WgGroupSite& s = sites[i];
    s = dpa::WgGroupSite{};
    for (size_t k = 0; k < d.size(); ++k) {
      CHECK_DEV(d[k]); CHECK_BF16(d[k]); CHECK_BF16(x[k]); CHECK_CONTIG(d[k]); CHECK_CONTIG(x[k]);
      TORCH_CHECK(d[k].dim() == 2 && x[k].dim() == 2 && d[k].size(0) == T && d[k].size(1) == M &&
                  x[k].size(0) == T && x[k].size(1) == N, "gemm_wgrad_grouped: segment shapes of site ", i);
      TORCH_CHECK(d[k].device() == dWs[0].device() && x[k].device() == dWs[0].device() &&
                  dW.device() == dWs[0].device(), "gemm_wgrad_grouped: devices");
      s.a[k] = bf_ptr(d[k]);
      s.b[k] = bf_ptr(x[k]);
    }
    if (T % 128 || T > (int64_t)INT32_MAX) return false;
    s.dW = dW.data_ptr<float>();
    if (dbs[i].has_value() && dbs[i]->defined()) {
      CHECK_F32((*dbs[i])); CHECK_CONTIG((*dbs[i]));
      TORCH_CHECK(dbs[i]->numel() == M, "gemm_wgrad_grouped: db size of site ", i);
      s.colsum = dbs[i]->data_ptr<float>();
    }
    s.nseg = (int)d.size();
    s.M = (int)M;
    s.N = (int)N;
    s.ktiles = (int)(T / 64);
  }
  const int ntiles = dpa::wgrad_group_prepare(sites.data(), (int)ns);
  if (ntiles <= 0) return false;
  const c10::DeviceGuard guard(dWs[0].device());
  const int64_t bytes = (int64_t)(ns * sizeof(dpa::WgGroupSite));
  at::Tensor host = at::empty({bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  std::memcpy(host.data_ptr(), sites.data(), (size_t)bytes);
  at::Tensor dev = at::empty({bytes}, dWs[0].options().dtype(at::kByte));
  dev.copy_(host, /*non_blocking=*/true);
  return dpa::launch_wgrad_group(reinterpret_cast<const dpa::WgGroupSite*>(dev.data_ptr()), (int)ns, ntiles,
                                 cur_stream());
}

// ---- row softmax cross-entropy (chunked wide-E linear-CE) ------------------------------
static void check_i64(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kLong && t.is_contiguous(), name,
              " must be a contiguous int64 HIP tensor");
}

// (loss, lse) outputs: the caller's [R] fp32 slices when given (a chunk of the whole
// batch's vectors: no per-chunk copy), else fresh tensors
static std::pair<at::Tensor, at::Tensor> xent_rows_outs(const at::Tensor& lg, const c10::optional<at::Tensor>& loss_out,
                                                        const c10::optional<at::Tensor>& lse_out) {
  auto f32 = lg.options().dtype(at::kFloat);
  at::Tensor loss = loss_out.has_value() ? *loss_out : at::empty({lg.size(0)}, f32);
  at::Tensor lse = lse_out.has_value() ? *lse_out : at::empty({lg.size(0)}, f32);
  for (const at::Tensor* t : {&loss, &lse})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == lg.size(0),
                "loss / lse outputs must be contiguous fp32 [R] HIP tensors");
  return {loss, lse};
}

static std::vector<at::Tensor> xent_rows_fwd(const at::Tensor& lg, int64_t V, const at::Tensor& tgt,
                                             const c10::optional<at::Tensor>& loss_out,
                                             const c10::optional<at::Tensor>& lse_out) {
  CHECK_DEV(lg); CHECK_BF16(lg); CHECK_CONTIG(lg); CHECK_ALIGNED(lg);
  check_i64(tgt, "target");
  TORCH_CHECK(lg.dim() == 2 && lg.size(1) % 8 == 0 && V > 0 && V <= lg.size(1),
              "logits [R, ld] with ld % 8 == 0 and V <= ld");
  TORCH_CHECK(tgt.numel() == lg.size(0), "target [R]");
  const c10::DeviceGuard guard(lg.device());
  auto [loss, lse] = xent_rows_outs(lg, loss_out, lse_out);
  dpa::launch_xent_rows_fwd(bf_ptr(lg), lg.size(1), (int)V, tgt.data_ptr<int64_t>(), lg.size(0),
                            loss.data_ptr<float>(), lse.data_ptr<float>(), cur_stream());
  return {loss, lse};
}

// in place: logits -> softmax - onehot (unscaled); returns (loss, lse) (empty list if refused)
static std::vector<at::Tensor> xent_rows_fwd_grad_(at::Tensor& lg, int64_t V, const at::Tensor& tgt,
                                                   const c10::optional<at::Tensor>& loss_out,
                                                   const c10::optional<at::Tensor>& lse_out) {
  CHECK_DEV(lg); CHECK_BF16(lg); CHECK_CONTIG(lg); CHECK_ALIGNED(lg);
  check_i64(tgt, "target");
  TORCH_CHECK(lg.dim() == 2 && lg.size(1) % 8 == 0 && V > 0 && V <= lg.size(1),
              "logits [R, ld] with ld % 8 == 0 and V <= ld");
  TORCH_CHECK(tgt.numel() == lg.size(0), "target [R]");
  const c10::DeviceGuard guard(lg.device());
  auto [loss, lse] = xent_rows_outs(lg, loss_out, lse_out);
  if (!dpa::launch_xent_rows_fwd_grad(reinterpret_cast<uint16_t*>(lg.data_ptr()), lg.size(1), (int)V,
                                      tgt.data_ptr<int64_t>(), lg.size(0), loss.data_ptr<float>(),
                                      lse.data_ptr<float>(), cur_stream()))
    return {};
  return {loss, lse};
}

static void xent_rows_bwd_(at::Tensor& lg, int64_t V, const at::Tensor& tgt, const at::Tensor& lse,
                           const at::Tensor& dloss) {
  CHECK_DEV(lg); CHECK_BF16(lg); CHECK_CONTIG(lg); CHECK_ALIGNED(lg);
  check_i64(tgt, "target");
  CHECK_F32(lse); CHECK_F32(dloss); CHECK_CONTIG(lse); CHECK_CONTIG(dloss);
  TORCH_CHECK(lg.dim() == 2 && lg.size(1) % 8 == 0 && V > 0 && V <= lg.size(1), "logits [R, ld]");
  const int64_t R = lg.size(0);
  TORCH_CHECK(tgt.numel() == R && lse.numel() == R && dloss.numel() == R, "per-row tensors [R]");
  const c10::DeviceGuard guard(lg.device());
  dpa::launch_xent_rows_bwd(reinterpret_cast<uint16_t*>(lg.data_ptr()), lg.size(1), (int)V,
                            tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), dloss.data_ptr<float>(), R,
                            cur_stream());
}

// ---- DiffuSeq diffusion kernels ------------------------------------------------------------
static void check_diffusion_common(const at::Tensor& ids, const at::Tensor& t, const at::Tensor& W) {
  check_i64(ids, "ids");
  check_i64(t, "t");
  CHECK_DEV(W); CHECK_F32(W); CHECK_CONTIG(W); CHECK_ALIGNED(W);
  TORCH_CHECK(ids.dim() == 2 && t.dim() == 1 && t.size(0) == ids.size(0), "ids [B, L], t [B]");
  TORCH_CHECK(W.dim() == 2 && W.size(1) % 4 == 0, "W [V, E] with E % 4 == 0");
}

static std::vector<at::Tensor> emb_qsample_fwd(const at::Tensor& ids, const at::Tensor& mask,
                                               const at::Tensor& t, const at::Tensor& W,
                                               const at::Tensor& sa, const at::Tensor& s1a, double std0,
                                               int64_t seed, int64_t offset, bool want_x16) {
  check_diffusion_common(ids, t, W);
  check_i64(mask, "mask");
  TORCH_CHECK(mask.sizes() == ids.sizes(), "mask [B, L]");
  CHECK_DEV(sa); CHECK_F32(sa); CHECK_CONTIG(sa); CHECK_DEV(s1a); CHECK_F32(s1a); CHECK_CONTIG(s1a);
  TORCH_CHECK(sa.numel() == s1a.numel() && sa.numel() > 0, "schedule tables [T]");
  const int64_t B = ids.size(0), L = ids.size(1), E = W.size(1);
  const c10::DeviceGuard guard(W.device());
  auto bf = W.options().dtype(at::kBFloat16);
  at::Tensor xs = at::empty({B, L, E}, W.options()), xt = at::empty({B, L, E}, bf), x16;
  if (want_x16) x16 = at::empty({B, L, E}, bf);
  if (B * L > 0)
    dpa::launch_emb_qsample_fwd(ids.data_ptr<int64_t>(), mask.data_ptr<int64_t>(), t.data_ptr<int64_t>(),
                                W.data_ptr<float>(), sa.data_ptr<float>(), s1a.data_ptr<float>(), B * L,
                                (int)L, (int)E, (int)W.size(0), (float)std0, (uint32_t)seed,
                                (uint32_t)offset, xs.data_ptr<float>(),
                                want_x16 ? reinterpret_cast<uint16_t*>(x16.data_ptr()) : nullptr,
                                reinterpret_cast<uint16_t*>(xt.data_ptr()), cur_stream());
  return {xs, x16, xt};
}

static void emb_qsample_bwd(const at::Tensor& ids, const at::Tensor& mask, const at::Tensor& t,
                            const at::Tensor& sa, c10::optional<at::Tensor> d_xs,
                            c10::optional<at::Tensor> d_xs16, c10::optional<at::Tensor> d_xt,
                            at::Tensor& dW) {
  check_diffusion_common(ids, t, dW);
  check_i64(mask, "mask");
  CHECK_DEV(sa); CHECK_F32(sa); CHECK_CONTIG(sa);
  const int64_t B = ids.size(0), L = ids.size(1), E = dW.size(1), n = B * L * E;
  const float* p_xs = nullptr;
  const uint16_t* p_xs16 = nullptr;
  const uint16_t* p_xt16 = nullptr;
  const float* p_xt32 = nullptr;
  if (d_xs.has_value() && d_xs->defined()) {
    CHECK_F32((*d_xs)); CHECK_CONTIG((*d_xs));
    TORCH_CHECK(d_xs->numel() == n, "d_x_start size");
    p_xs = d_xs->data_ptr<float>();
  }
  if (d_xs16.has_value() && d_xs16->defined()) {
    CHECK_BF16((*d_xs16)); CHECK_CONTIG((*d_xs16));
    TORCH_CHECK(d_xs16->numel() == n, "d_x_start16 size");
    p_xs16 = bf_ptr(*d_xs16);
  }
  if (d_xt.has_value() && d_xt->defined()) {
    CHECK_CONTIG((*d_xt));
    TORCH_CHECK(d_xt->numel() == n, "d_x_t size");
    if (d_xt->scalar_type() == at::kBFloat16) p_xt16 = bf_ptr(*d_xt);
    else { CHECK_F32((*d_xt)); p_xt32 = d_xt->data_ptr<float>(); }
  }
  const c10::DeviceGuard guard(dW.device());
  if (n > 0) {
    // stable counting sort of the token ids -> runs of equal ids summed in registers, one
    // writer per gradient row (deterministic; csrc/sort.hip, csrc/diffusion.hip)
    at::Tensor sorted, perm, part;
    if (E == 128 || E == 256) {
      std::tie(sorted, perm) = bucket_sort_ids(ids, dW.size(0));
      part = at::empty({dpa::emb_grad_part_floats(B * L, (int)E, true)}, dW.options());
    }
    dpa::launch_emb_qsample_bwd(ids.data_ptr<int64_t>(), mask.data_ptr<int64_t>(), t.data_ptr<int64_t>(),
                                sa.data_ptr<float>(), p_xs, p_xs16, p_xt16, p_xt32, B * L, (int)L, (int)E,
                                (int)dW.size(0), dW.data_ptr<float>(), cur_stream(),
                                sorted.defined() ? sorted.data_ptr<int64_t>() : nullptr,
                                perm.defined() ? perm.data_ptr<int64_t>() : nullptr,
                                part.defined() ? part.data_ptr<float>() : nullptr);
  };
}

static void check_loss_inputs(const at::Tensor& xs, const at::Tensor& out, const at::Tensor& ids,
                              const at::Tensor& t, const at::Tensor& W) {
  check_diffusion_common(ids, t, W);
  CHECK_DEV(xs); CHECK_F32(xs); CHECK_CONTIG(xs); CHECK_ALIGNED(xs);
  CHECK_DEV(out); CHECK_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat,
              "model output must be bf16 or fp32");
  TORCH_CHECK(xs.dim() == 3 && xs.size(0) == ids.size(0) && xs.size(1) == ids.size(1) &&
                  xs.size(2) == W.size(1) && out.sizes() == xs.sizes(),
              "x_start / output [B, L, E] matching ids and W");
}

static std::vector<at::Tensor> diff_loss_fwd(const at::Tensor& xs, const at::Tensor& out,
                                             const at::Tensor& ids, const at::Tensor& t,
                                             const at::Tensor& W, double sa_last) {
  check_loss_inputs(xs, out, ids, t, W);
  const int64_t B = xs.size(0), L = xs.size(1), E = xs.size(2);
  const c10::DeviceGuard guard(xs.device());
  at::Tensor mse = at::empty({B}, xs.options()), tT = at::empty({B}, xs.options());
  if (B > 0)
    dpa::launch_diff_loss_fwd(xs.data_ptr<float>(), out.data_ptr(), out.scalar_type() == at::kBFloat16,
                              ids.data_ptr<int64_t>(), t.data_ptr<int64_t>(), W.data_ptr<float>(), (int)B,
                              (int)L, (int)E, (int)W.size(0), (float)sa_last, mse.data_ptr<float>(),
                              tT.data_ptr<float>(), cur_stream());
  return {mse, tT};
}

static std::vector<at::Tensor> diff_loss_bwd(const at::Tensor& xs, const at::Tensor& out,
                                             const at::Tensor& ids, const at::Tensor& t,
                                             const at::Tensor& W, c10::optional<at::Tensor> dmse,
                                             c10::optional<at::Tensor> dtT, double sa_last, bool need_dout,
                                             bool need_dxs, c10::optional<at::Tensor> dW, bool fold_t0) {
  check_loss_inputs(xs, out, ids, t, W);
  const int64_t B = xs.size(0), L = xs.size(1), E = xs.size(2);
  const float* pm = nullptr;
  const float* pt = nullptr;
  if (dmse.has_value() && dmse->defined()) {
    CHECK_F32((*dmse)); CHECK_CONTIG((*dmse)); TORCH_CHECK(dmse->numel() == B, "dmse [B]");
    pm = dmse->data_ptr<float>();
  }
  if (dtT.has_value() && dtT->defined()) {
    CHECK_F32((*dtT)); CHECK_CONTIG((*dtT)); TORCH_CHECK(dtT->numel() == B, "dtT [B]");
    pt = dtT->data_ptr<float>();
  }
  float* pw = nullptr;
  if (dW.has_value() && dW->defined()) {
    CHECK_F32((*dW)); CHECK_CONTIG((*dW)); TORCH_CHECK(dW->sizes() == W.sizes(), "dW like W");
    pw = dW->data_ptr<float>();
  }
  const c10::DeviceGuard guard(xs.device());
  at::Tensor d_out, d_xs;
  if (need_dout) d_out = at::empty_like(out);
  if (need_dxs) d_xs = at::empty_like(xs);
  if (B > 0 && (need_dout || need_dxs || pw))
    dpa::launch_diff_loss_bwd(xs.data_ptr<float>(), out.data_ptr(), out.scalar_type() == at::kBFloat16,
                              ids.data_ptr<int64_t>(), t.data_ptr<int64_t>(), W.data_ptr<float>(), pm, pt,
                              (int)B, (int)L, (int)E, (int)W.size(0), (float)sa_last,
                              need_dout ? d_out.data_ptr() : nullptr,
                              need_dxs ? d_xs.data_ptr<float>() : nullptr, pw, cur_stream(), fold_t0 && need_dxs);
  return {d_out, d_xs};
}

// Bump the device-side Philox offset base of every kernel translation unit that draws noise
// or dropout (common.h g_rng_base): a replayed HIP graph's baked offsets + the base = fresh
// numbers per replay.  Stream-ordered on the current stream.
static void rng_base_add(int64_t d) {
  const auto s = cur_stream();
  dpa::rng_base_add_attention((uint32_t)d, s);
  dpa::rng_base_add_attention128((uint32_t)d, s);
  dpa::rng_base_add_diffusion((uint32_t)d, s);
  dpa::rng_base_add_norm((uint32_t)d, s);
  dpa::rng_base_add_gemm256((uint32_t)d, s);
}

static at::Tensor timestep_emb(const at::Tensor& ts, int64_t dim, double max_period) {
  CHECK_DEV(ts); CHECK_F32(ts); CHECK_CONTIG(ts);
  TORCH_CHECK(ts.dim() == 1 && dim > 0, "timesteps [B]");
  const c10::DeviceGuard guard(ts.device());
  at::Tensor out = at::empty({ts.size(0), dim}, ts.options().dtype(at::kBFloat16));
  if (ts.numel() > 0)
    dpa::launch_timestep_emb(ts.data_ptr<float>(), (int)ts.size(0), (int)dim, (float)max_period,
                             reinterpret_cast<uint16_t*>(out.data_ptr()), cur_stream());
  return out;
}

static bool gemm_supported(int64_t M, int64_t N, int64_t K) {
  return M % 128 == 0 && N % 128 == 0 && K % 128 == 0;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "distributed_pipeline_amd native gfx950 kernels";
  dpa::register_comm(m);
  dpa::register_runtime(m);
  m.def("sqnorm", &sqnorm, "flat grad L2 norm + clip coefficient (device)");
  m.def("adamw_ema", &adamw_ema, "fused AdamW + EMA + bf16 shadow refresh");
  m.def("ema_update", &ema_update, "flat EMA update");
  m.def("cast_bf16", &cast_bf16, "flat fp32->bf16");
  m.def("transpose_bf16_batch", &transpose_bf16_batch,
        "dsts[i] = srcs[i]^T for bf16 matrices with 64-multiple sides, one launch per 96 (False: a shape does not tile)");
  m.def("add_ln_fwd", &add_ln_fwd,
        "LN(dropout(y [+pos] [+temb]) + res) (post: dropout(LN(...))) -> (out, hsave, mean, rstd)",
        py::arg("y"), py::arg("res"), py::arg("gamma"), py::arg("beta"), py::arg("p"), py::arg("eps"),
        py::arg("seed"), py::arg("offset"), py::arg("pos") = py::none(), py::arg("temb") = py::none(),
        py::arg("L") = 1, py::arg("post") = false, py::arg("save_h") = true, py::arg("h_guard") = false);
  m.def("add_ln_bwd", &add_ln_bwd, "backward of add_ln_fwd -> (dres, dy, dgamma, dbeta, colsum(dy))",
        py::arg("dout"), py::arg("hsave"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"),
        py::arg("p"), py::arg("seed"), py::arg("offset"), py::arg("need_dres"), py::arg("need_dy"),
        py::arg("want_dy_colsum") = false, py::arg("dh_in") = py::none(), py::arg("post") = false,
        py::arg("dg_acc") = py::none(), py::arg("db_acc") = py::none(), py::arg("dyb_acc") = py::none(),
        py::arg("part_buf") = py::none(), py::arg("part_acc") = false, py::arg("beta") = py::none(),
        py::arg("hcopy") = py::none(), py::arg("pair_hash") = false);
  m.def("colsum_acc", &colsum_acc, "dst += colsum(part) (fp32 partials [rows, cols])");
  m.def("ln_bwd_partials", &ln_bwd_partials, "floats of add_ln_bwd's deferred partial buffer (0: none)");
  m.def("ln_colreduce", &ln_colreduce, "dg/db(/dyb) += column sums of add_ln_bwd partials",
        py::arg("part"), py::arg("R"), py::arg("D"), py::arg("dg"), py::arg("db"), py::arg("dyb") = py::none());
  m.def("bias_act_fwd", &bias_act_fwd, "z += bias (in place); y = act(z) -> (z, y)");
  m.def("bias_act_bwd", &bias_act_bwd, "dz = dy*act'(zy); db = colsum(dz) -> (dz, db)");
  m.def("gemm_nt_into", &gemm_nt_into, "y = x W^T (+b) into a preallocated [T, N] tensor");
  m.def("gemm_nn_into", &gemm_nn_into, "dx = dy W into a preallocated [T, K] tensor");
  m.def("emb_grad", &emb_grad, "dW[ids] += dy (sorted segment sum, fp32)");
  m.def("id_sort", &id_sort, "counting sort of int64 ids into V + 1 buckets -> (sorted ids, permutation)");
  m.def("partition01", &partition01, "stable partition order of an int64 0/1 mask (nonzero first)");
  m.def("attn128_supports", &dpa::attn128_supports, "the persistent L = 128 attention covers (L, D, causal)");
  m.def("attn_fwd", &attn_fwd, "fused attention forward (head_dim 64/128) -> (out, lse)", py::arg("qkv"),
        py::arg("heads"), py::arg("p"), py::arg("causal"), py::arg("seed"), py::arg("offset"),
        py::arg("head_major") = false);
  m.def("attn_bwd", &attn_bwd, "fused attention backward -> (dqkv, colsum(dqkv) or None)",
        py::arg("dout"), py::arg("qkv"), py::arg("out"), py::arg("lse"), py::arg("heads"), py::arg("p"),
        py::arg("causal"), py::arg("seed"), py::arg("offset"), py::arg("want_db") = false,
        py::arg("head_major") = false, py::arg("db_acc") = py::none(), py::arg("part_out") = py::none());
  m.def("attn_colpart_rows", &dpa::attn_colpart_rows,
        "rows of attn_bwd's bias-gradient partials ([rows][3 D] fp32) for (B, L, H, D, causal)");
  m.def("attn_colpart_reduce", &attn_colpart_reduce,
        "db[3 H D] += column sums of R x H rows of attn_bwd partials (deferred bias gradient)");
  m.def("gemm_nt", &gemm_nt,
        "y = act(x W^T + b) (bf16 MFMA) -> (y, z, z_is_derivative): z is the pre-activation, or "
        "act'(pre-activation) when want_deriv and the persistent kernel ran (backward act code 4)",
        py::arg("x"), py::arg("W"), py::arg("b"), py::arg("act"), py::arg("want_deriv") = 0,
        py::arg("head_major_L") = 0);
  m.def("gemm_nt_res", &gemm_nt_res, "h = res + dropout_p(x W^T + b) in the GEMM epilogue (None: shape not tiled)",
        py::arg("x"), py::arg("W"), py::arg("b"), py::arg("res"), py::arg("p"), py::arg("seed"), py::arg("offset"));
  m.def("gemm_nn", &gemm_nn, "dx = dy W (bf16 MFMA; wt = W^T takes the row-form operand path)", py::arg("dy"),
        py::arg("W"), py::arg("wt") = py::none());
  m.def("gemm_nn_dact", &gemm_nn_dact,
        "dz = (dy W) * act'(aux) (bf16 MFMA, fused act backward) -> (dz, colsum(dz) fp32 or None)",
        py::arg("dy"), py::arg("W"), py::arg("aux"), py::arg("act"), py::arg("want_db") = false,
        py::arg("db_acc") = py::none(), py::arg("part_out") = py::none(), py::arg("wt") = py::none());
  m.def("gemm_nn_acc_", &gemm_nn_acc_, "dx += dy W in place (bf16 MFMA); False if the shape does not tile",
        py::arg("dy"), py::arg("W"), py::arg("dx"), py::arg("wt") = py::none());
  m.def("gemm_wgrad", &gemm_wgrad, "dW += dy^T x, db += colsum(dy) (fp32 atomics, split-K)");
  m.def("gemm_wgrad_multi", &gemm_wgrad_multi, "dW += sum_s dy_s^T x_s over equal token segments, one launch",
        py::arg("dys"), py::arg("xs"), py::arg("dW"), py::arg("db") = py::none());
  m.def("gemm_wgrad_grouped", &gemm_wgrad_grouped,
        "dW_i += sum_s dy_is^T x_is for several Linears in one launch (no token split); false if a site does not tile",
        py::arg("dys"), py::arg("xs"), py::arg("dWs"), py::arg("dbs"));
  m.def("gemm_supported", &gemm_supported, "shape check for the native GEMMs");
  m.def("set_gemm256", &dpa::set_gemm256, "enable/disable the 256x256 8-phase GEMM path");
  m.def("set_gemmp_grid_cap", &dpa::set_gemmp_grid_cap, "cap the persistent GEMM grid (0 = #CUs)");
  m.def("set_wgrad4w", &dpa::set_wgrad4w,
        "weight gradients without in-kernel bias sums on the one-wave-per-SIMD kernel (wgrad4w.hip; default on)");
  m.def("set_gemmp_half", &dpa::set_gemmp_half,
        "128-row tiles of the persistent GEMMs: 0 off, 1 auto (when they finish sooner), 2 always, -1 default");
  m.def("set_gemmp_dynamic", &dpa::set_gemmp_dynamic,
        "dynamic per-XCD tile queues for the persistent GEMMs (on for world > 1; env DPA_GEMMP_DYNAMIC wins)");
  m.def("lxent_fwd", &lxent_fwd, "fused linear + cross-entropy forward -> (loss, lse)");
  m.def("lxent_fwd_dx", &lxent_fwd_dx,
        "fused linear-CE forward + unscaled input gradient -> (loss, lse, dxu fp32 [N, E])");
  m.def("lxent_bwd", &lxent_bwd, "fused linear + cross-entropy backward -> (dx, dW fp32, db fp32)",
        pybind11::arg("dloss"), pybind11::arg("x"), pybind11::arg("W"), pybind11::arg("b"), pybind11::arg("tgt"),
        pybind11::arg("lse"), pybind11::arg("need_dx"), pybind11::arg("need_dw"), pybind11::arg("need_db"),
        pybind11::arg("onehot_scatter") = false, pybind11::arg("dw_acc") = pybind11::none(),
        pybind11::arg("db_acc") = pybind11::none());
  m.def("seq_pos_sums", &seq_pos_sums, "(sum over b, sum over l) of a [B*L, H] bf16 gradient in one read",
        pybind11::arg("d"), pybind11::arg("L"), pybind11::arg("need_pos"), pybind11::arg("need_temb"));
  m.def("xent_rows_fwd", &xent_rows_fwd, "row softmax-CE over bf16 logits [R, ld] -> (loss, lse)",
        pybind11::arg("lg"), pybind11::arg("V"), pybind11::arg("tgt"), pybind11::arg("loss_out") = pybind11::none(),
        pybind11::arg("lse_out") = pybind11::none());
  m.def("xent_rows_bwd_", &xent_rows_bwd_, "in place: logits -> dloss * (softmax - onehot)");
  m.def("xent_rows_fwd_grad_", &xent_rows_fwd_grad_,
        "in place: logits -> softmax - onehot (unscaled), returns (loss, lse) or [] if the row is too long",
        pybind11::arg("lg"), pybind11::arg("V"), pybind11::arg("tgt"), pybind11::arg("loss_out") = pybind11::none(),
        pybind11::arg("lse_out") = pybind11::none());
  m.def("emb_qsample_fwd", &emb_qsample_fwd,
        "DiffuSeq embedding gather + x_start noise + masked q_sample -> (x_start, x_start bf16, x_t bf16)");
  m.def("emb_qsample_bwd", &emb_qsample_bwd, "scatter-add of the q_sample gradients into dW (fp32)");
  m.def("diff_loss_fwd", &diff_loss_fwd, "DiffuSeq per-sample (mse, tT) losses");
  m.def("diff_loss_bwd", &diff_loss_bwd, "backward of diff_loss_fwd -> (d_out, d_x_start)", py::arg("xs"),
        py::arg("out"), py::arg("ids"), py::arg("t"), py::arg("W"), py::arg("dmse"), py::arg("dtT"),
        py::arg("sa_last"), py::arg("need_dout"), py::arg("need_dxs"), py::arg("dW"), py::arg("fold_t0") = false);
  m.def("rng_base_add", &rng_base_add, "advance the device-side Philox offset base (graph replays)");
  m.def("timestep_emb", &timestep_emb, "sinusoidal timestep embedding [cos | sin] -> bf16");
}
