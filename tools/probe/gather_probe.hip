// Memory floor of the feature-assembly access pattern (K1, csrc/kernels/features.hip): 8192
// requests per batch, each reading one random account's rows of the HBM feature store
// (ts ring 1 KiB, amount ring 2 KiB, HLL 512 B, ext 392 B, AcctRT 64 B, AcctBatch 80 B), 16
// lanes per request as K1 does. Variants isolate which reads set the time.
//   hipcc --offload-arch=gfx950 -O3 -o gather_probe tools/probe/gather_probe.hip && ./gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                                       \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                         \
      return 1;                                                                                     \
    }                                                                                               \
  } while (0)

struct Tabs {
  const uint4* ts;    // [C][64] uint4 (256 x u32)
  const uint4* amt;   // [C][128] uint4 (256 x i64)
  const uint32_t* hll;  // [C][128]
  const float* ext;   // [C][98]
  const uint4* rt;    // [C][4]
  const uint4* bat;   // [C][5]
  const int* slots;   // [B]
  float* out;         // [B]
  int B;
  float* X;           // [B][128] model-input rows (K1 output shape)
  uint4* feat;        // [B][8] 128-B FeatRec rows
};

template <int V>
__global__ void __launch_bounds__(256) gather(Tabs t) {
  const int lane = threadIdx.x & 63, ql = lane & 15;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (row >= t.B) return;
  const int s = t.slots[row];
  uint32_t acc = 0;
  float facc = 0.f;
  if (V == 0 || V == 2 || V == 4 || V == 6) {  // ring
    uint4 a[4], b[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = t.ts[(size_t)s * 64 + ql + 16 * i];
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = t.amt[(size_t)s * 128 + 2 * (ql + 16 * (i >> 1)) + (i & 1)];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += a[i].x ^ a[i].w;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += b[i].y;
  }
  if (V == 0 || V == 3 || V == 6) {  // HLL 8 x 4 B, ext 7 x 4 B (K1's shapes)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += t.hll[(size_t)s * 128 + ql + 16 * i];
#pragma unroll
    for (int i = 0; i < 7; ++i) facc += t.ext[(size_t)s * 98 + min(ql + 16 * i, 97)];
  }
  if (V == 4) {  // HLL / ext as 16-B loads
    const uint4* h4 = reinterpret_cast<const uint4*>(t.hll + (size_t)s * 128);
    const uint4 h0 = h4[ql], h1 = h4[16 + ql];
    acc += h0.x + h1.w;
    const float4* e4 = reinterpret_cast<const float4*>(t.ext + (size_t)s * 100);
    const float4 e0 = e4[ql], e1 = e4[min(16 + ql, 24)];
    facc += e0.x + e1.y;
  }
  if (V == 0 || V == 1 || V == 4 || V == 6) {  // account rows (every lane of the quarter loads them)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += t.rt[(size_t)s * 4 + i].x;
#pragma unroll
    for (int i = 0; i < 5; ++i) acc += t.bat[(size_t)s * 5 + i].y;
  }
  facc += (float)acc;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) facc += __shfl_xor(facc, o, 64);
  if (V >= 5) {  // K1's output stores: X row (30 + 98 floats, 4 B lanes) + FeatRec by one lane
    float* xr = t.X + (size_t)row * 128;
    xr[ql] = facc;
    if (ql + 16 < 30) xr[ql + 16] = facc;
#pragma unroll
    for (int u = 0; u < 7; ++u)
      if (ql + 16 * u < 98) xr[30 + ql + 16 * u] = facc + u;
    if (ql == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) t.feat[(size_t)row * 8 + k] = make_uint4(acc, k, 0, 0);
    }
  }
  if (ql == 0) t.out[row] = facc;
}

// every launch reads a different random batch (slots [reps + 5][B]) so no batch is L2/MALL-warm
template <int V>
float time_variant(Tabs t, hipStream_t st, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int* base = t.slots;
  for (int i = 0; i < 5; ++i) {
    t.slots = base + (size_t)(reps + i) * t.B;
    hipLaunchKernelGGL(gather<V>, dim3((t.B + 15) / 16), dim3(256), 0, st, t);
  }
  hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) {
    t.slots = base + (size_t)i * t.B;
    hipLaunchKernelGGL(gather<V>, dim3((t.B + 15) / 16), dim3(256), 0, st, t);
  }
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const size_t C = argc > 1 ? std::atol(argv[1]) : (1 << 20);
  const int B = 8192, reps = 50;
  void *ts, *amt, *hll, *ext, *rt, *bat, *slots, *out, *X, *feat;
  CK(hipMalloc(&ts, C * 1024));
  CK(hipMalloc(&amt, C * 2048));
  CK(hipMalloc(&hll, C * 512));
  CK(hipMalloc(&ext, C * 400));
  CK(hipMalloc(&rt, C * 64));
  CK(hipMalloc(&bat, C * 80));
  CK(hipMalloc(&slots, (size_t)(reps + 5) * B * 4));
  CK(hipMalloc(&out, B * 4));
  CK(hipMalloc(&X, (size_t)B * 512));
  CK(hipMalloc(&feat, (size_t)B * 128));
  CK(hipMemset(ts, 1, C * 1024));
  CK(hipMemset(amt, 2, C * 2048));
  CK(hipMemset(hll, 3, C * 512));
  CK(hipMemset(ext, 0, C * 400));
  CK(hipMemset(rt, 4, C * 64));
  CK(hipMemset(bat, 5, C * 80));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  Tabs t{(const uint4*)ts, (const uint4*)amt, (const uint32_t*)hll, (const float*)ext, (const uint4*)rt,
         (const uint4*)bat, (const int*)slots, (float*)out, B, (float*)X, (uint4*)feat};
  std::mt19937_64 g(1);
  std::vector<int> hs((size_t)(reps + 5) * B);
  for (int round = 0; round < 2; ++round) {
    for (auto& x : hs) x = (int)(g() % C);
    CK(hipMemcpy(slots, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    std::printf("accounts %zu round %d (us per batch of %d requests)\n", C, round, B);
    std::printf("  full K1 loads (ring+hll+ext+rows) %7.2f\n", time_variant<0>(t, st, reps));
    std::printf("  account rows only (rt+batch)      %7.2f\n", time_variant<1>(t, st, reps));
    std::printf("  ring only (3 KiB)                 %7.2f\n", time_variant<2>(t, st, reps));
    std::printf("  hll+ext only (4-B lanes)          %7.2f\n", time_variant<3>(t, st, reps));
    std::printf("  full, hll/ext as 16-B loads       %7.2f\n", time_variant<4>(t, st, reps));
    std::printf("  stores only (X row + FeatRec)     %7.2f\n", time_variant<5>(t, st, reps));
    std::printf("  full loads + K1 stores            %7.2f\n", time_variant<6>(t, st, reps));
  }
  return 0;
}
