// Stream-plan primitives (SURVEY 5.8 / the step's stream -> hardware-queue placement).
//
// HIP multiplexes every stream of a process onto GPU_MAX_HW_QUEUES (4 on the MI355X boxes)
// pooled HSA queues: a new stream takes the least-used pooled queue of its priority, so which
// queue a torch pool stream lands on depends on how many streams were taken before it, and two
// streams that share a queue serialise (a kernel waits for the one ahead of it in the queue).
// A stream created with a CU mask gets an HSA queue of its own instead (the mask is a queue
// property, so such a queue is never shared); with every CU in the mask it runs anywhere.
// The trainer's stream plan (distributed_pipeline_amd/runtime/streams.py) creates each side
// stream of the step this way, once, in a fixed order.
#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <vector>

namespace dpa {

#define DPA_RT_CHECK(x)                                                            \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));          \
  } while (0)

// mode 0: plain non-blocking stream (pooled queue); 1: dedicated queue (full CU mask);
// 2: non-blocking stream at `priority` (pooled queue of that priority).  Returns the handle.
static int64_t stream_create(int64_t mode, int64_t priority) {
  hipStream_t s = nullptr;
  if (mode == 1) {
    int dev = 0, ncu = 0;
    DPA_RT_CHECK(hipGetDevice(&dev));
    DPA_RT_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint32_t> mask((ncu + 31) / 32, 0xffffffffu);
    if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
    DPA_RT_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  } else if (mode == 2) {
    DPA_RT_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, (int)priority));
  } else {
    DPA_RT_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  return (int64_t)reinterpret_cast<uintptr_t>(s);
}

static void stream_destroy(int64_t h) {
  if (h) DPA_RT_CHECK(hipStreamDestroy(reinterpret_cast<hipStream_t>((uintptr_t)h)));
}

static std::vector<int64_t> stream_cu_mask(int64_t h) {
  std::vector<uint32_t> m(16, 0u);
  DPA_RT_CHECK(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>((uintptr_t)h), (uint32_t)m.size(), m.data()));
  return std::vector<int64_t>(m.begin(), m.end());
}

void register_runtime(pybind11::module& m) {
  m.def("stream_create", &stream_create,
        "create a HIP stream: mode 0 pooled queue, 1 dedicated queue (full CU mask), 2 priority",
        pybind11::arg("mode"), pybind11::arg("priority") = 0);
  m.def("stream_destroy", &stream_destroy, "destroy a stream created by stream_create");
  m.def("stream_cu_mask", &stream_cu_mask, "CU mask words of a stream");
}

}  // namespace dpa
