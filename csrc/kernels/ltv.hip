// K9 ltv_segment: vectorised LTVPredictor (services/risk/internal/prediction/ltv.go:113-382),
// one thread per player (row logic in ltv.h). Golden: golden/ltv.py.
#include "common.h"
#include "launch.h"
#include "ltv.h"

namespace igp {

__global__ void ltv_kernel(LtvArgs a) {
  __shared__ float zero_row[P_NCOLS];
  if (threadIdx.x < P_NCOLS) zero_row[threadIdx.x] = 0.f;
  __syncthreads();  // before any early exit: every thread of the block reaches it
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.B) return;
  const float* p;
  if (a.slots) {
    const int s = a.slots[i];
    p = s >= 0 ? a.pf + (size_t)s * P_NCOLS : zero_row;
  } else {
    p = a.pf + (size_t)i * P_NCOLS;
  }
  ltv_row(p, a.ltv_model ? a.ltv_model + i : nullptr, a.out + (size_t)i * 6);
}

// element-parallel gather: consecutive threads write consecutive columns of a row
__global__ void __launch_bounds__(256) ltv_assemble_kernel(LtvAssembleArgs a) {
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(idx / a.x_w), c = (int)(idx % a.x_w);
  if (r >= a.n_rows) return;
  float v = 0.f;
  const int s = r < n_live ? a.slots[r] : -1;
  if (s >= 0) {
    if (c < P_NCOLS) {
      const float x = a.pf_tab[(size_t)s * P_NCOLS + c];
      v = copysignf(log1pf(fabsf(x)), x);
    } else if (a.ext_tab && c - P_NCOLS < a.ext_w) {
      v = a.ext_tab[(size_t)s * a.ext_w + (c - P_NCOLS)];
    }
  }
  a.X[(size_t)r * a.x_w + c] = v;
}

void launch_ltv_assemble(const LtvAssembleArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  const size_t total = (size_t)a.n_rows * a.x_w;
  IGP_LAUNCH(ltv_assemble_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
}

void launch_ltv(const LtvArgs& a, hipStream_t st) {
  if (a.B <= 0) return;
  IGP_LAUNCH(ltv_kernel, dim3((a.B + 255) / 256), dim3(256), 0, st, a);
}

}  // namespace igp
