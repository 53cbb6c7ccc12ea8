// Stream-ordered copies done by a kernel on the stream's own queue: the kernel reads (or writes)
// the pinned host buffer directly over the fabric with 16-B accesses. Outside a graph a
// hipMemcpyAsync between pinned host and device memory may be handed to a DMA engine, which
// adds an engine hand-off to every batch of a short pipeline stage; inside a graph it becomes a
// blit kernel anyway. Recordable by the direct-launch driver (oplist.h).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "oplist.h"

namespace py = pybind11;

namespace igp {
namespace {

__global__ void __launch_bounds__(256) pull_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                        size_t n16, uint8_t* __restrict__ dtail,
                                                        const uint8_t* __restrict__ stail, int ntail) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dtail[threadIdx.x] = stail[threadIdx.x];
}

void launch_pull_copy(void* dst, const void* src, size_t n, hipStream_t st) {
  const size_t n16 = n / 16;
  const int ntail = (int)(n - n16 * 16);
  const int blocks = (int)std::min<size_t>(std::max<size_t>((n16 + 255) / 256, 1), 1024);
  IGP_LAUNCH(pull_copy_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<uint4*>(dst),
                     reinterpret_cast<const uint4*>(src), n16, reinterpret_cast<uint8_t*>(dst) + n16 * 16,
                     reinterpret_cast<const uint8_t*>(src) + n16 * 16, ntail);
}

}  // namespace

void register_copy(py::module_& m) {
  // dst / src: device or pinned host pointers, both 16-B aligned
  m.def("pull_copy", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s) {
    if (!dst || !src || (dst | src) & 15) throw std::runtime_error("pull_copy: pointers must be non-null, 16-B aligned");
    if (n == 0) return;
    auto f = [dst, src, n](hipStream_t st) {
      launch_pull_copy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n, st);
    };
    if (OpList* r = recording()) {
      r->ops.emplace_back(f);
      return;
    }
    f(reinterpret_cast<hipStream_t>(s));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("pull_copy: ") + hipGetErrorString(e));
  });
}

}  // namespace igp
