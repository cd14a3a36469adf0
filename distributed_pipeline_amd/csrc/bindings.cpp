// Python bindings of the gfx950 kernels (torch tensors -> raw launchers).
// Every op launches on the *current* HIP stream of the tensor's device, so it
// composes with torch's stream semantics and with HIP-graph capture.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <vector>

#include "launchers.h"

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
                      double wd, int64_t step, double grad_scale, c10::optional<at::Tensor> clip) {
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
  const c10::DeviceGuard guard(p.device());
  dpa::launch_adamw_ema(p.data_ptr<float>(), g.data_ptr(), bf, m.data_ptr<float>(),
                        v.data_ptr<float>(), p16p, bufs.data(), r.data(), (int)bufs.size(), n,
                        (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, step,
                        (float)grad_scale, clipp, cur_stream());
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

PYBIND11_MODULE(_C, m) {
  m.doc() = "distributed_pipeline_amd native gfx950 kernels";
  m.def("sqnorm", &sqnorm, "flat grad L2 norm + clip coefficient (device)");
  m.def("adamw_ema", &adamw_ema, "fused AdamW + EMA + bf16 shadow refresh");
  m.def("ema_update", &ema_update, "flat EMA update");
  m.def("cast_bf16", &cast_bf16, "flat fp32->bf16");
}
