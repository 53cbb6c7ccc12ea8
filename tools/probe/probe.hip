// Toolchain probe: hipcc 7.2 code objects under torch's bundled HIP 7.0 runtime.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void addk(float* x, int n){ int i=blockIdx.x*blockDim.x+threadIdx.x; if(i<n) x[i]+=1.f; }
// one wave: D = A(16x32 bf16, all 1.0) * B(32x16, all 1.0) -> every element 32
__global__ void mfmak(float* out){
  bf16x8 a, b; for(int j=0;j<8;++j){ a[j]=0x3f80; b[j]=0x3f80; }
  f32x4 c = {0,0,0,0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  int l = threadIdx.x; for(int r=0;r<4;++r) out[l*4+r]=c[r];
}
__global__ void xcck(unsigned* out){ unsigned v; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v)); if(threadIdx.x==0) out[blockIdx.x]=v; }
void launch(uintptr_t p, int n, uintptr_t s){ hipLaunchKernelGGL(addk, dim3((n+255)/256), dim3(256), 0, (hipStream_t)s, (float*)p, n); }
void mfma(uintptr_t p, uintptr_t s){ hipLaunchKernelGGL(mfmak, dim3(1), dim3(64), 0, (hipStream_t)s, (float*)p); }
void xcc(uintptr_t p, int nb, uintptr_t s){ hipLaunchKernelGGL(xcck, dim3(nb), dim3(64), 0, (hipStream_t)s, (unsigned*)p); }
PYBIND11_MODULE(_probe, m){ m.def("launch", &launch); m.def("mfma", &mfma); m.def("xcc", &xcc); }
