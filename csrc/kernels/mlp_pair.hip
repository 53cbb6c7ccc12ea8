// K3 MLP chain, pair-cluster form (cfg 4's LTV MLP 256 -> 4 x 512 -> 1 at serving batches).
//
// Why: the one-workgroup chain (mlp_fused.hip) walks ALL weights of the chain (1.84 MB bf16)
// through every CU for every 32 or 64 rows. An XCD's L2 hands a CU ~70 GB/s of shared lines
// (MI355X_MICROARCH.md, gather table: "rows shared by every workgroup"), so each 64-row block
// spends >= 26 us streaming weights for ~12 us of MFMA work, and the measured chain ran at
// ~15 % of the bf16 peak.
//
// Here two workgroups on two CUs (equal blockIdx % 8: one XCD under round-robin dispatch, a
// speed bonus only) own 128 rows together and SPLIT EVERY LAYER'S OUTPUT COLUMNS: member m
// computes columns [256 m, 256 m + 256) for all 128 rows, streaming only its half of each
// layer's weights (256 KB per 512 x 512 layer), then the members swap their 64-KB halves of
// the activation tile through L2 (16-B `sc1` stores, an agent-scope counter, `global_load_lds`
// of the partner's half straight into the LDS image). Per 128 rows and layer a CU moves
// 256 KB of weights + 64 KB of activations instead of 2 x 512 KB: 3.2x less L2 -> CU traffic
// per row, at the price of one cluster hand-off per hidden layer.
//
// LDS image of the activation tile: [member half][128 rows][256 columns] bf16, member-major so
// that a handed-off half is one contiguous 64-KB block (copied verbatim: both members use the
// same swizzle); the 16-B chunk (row, c) of a half sits at row * 32 + (c ^ (row & 15)), so a
// 16-row A-fragment read touches 16 distinct chunks of each 256-B bank row. The tile is updated
// in place: a layer's outputs stay in registers until every wave has finished reading its input.
//
// Waves: 8 per workgroup, wave w = all 8 row tiles x column tiles {2w, 2w + 1} of the member's
// 16: per k-step 16 MFMAs (v_mfma_f32_16x16x32_bf16), 2 B-fragment loads (fragment-packed,
// k-step-major weights, ops/kernels.py pack_fragments) prefetched PF k-steps ahead, 8 A reads.
// Numerics are those of mlp_fused.hip's bf16 path (bf16 weights and activations, f32
// accumulation in the same k order, bf16 rounding of each hidden activation); only the order of
// the final N -> 1 sum differs (member partials added in member order).
//
// Every cross-CU wait is bounded (a pair that is not co-resident sets *pair_err and both
// members exit; the host then falls back to the one-workgroup kernel).
#include "common.h"
#include "launch.h"
#include "ltv.h"

namespace igp {
namespace {

typedef __attribute__((ext_vector_type(8))) short mp_bf16x8;
typedef __attribute__((ext_vector_type(4))) float mp_f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int mp_u32x4;

constexpr int MP_ROWS = 128;
constexpr int MP_HALF = 256;                 // columns per member
constexpr int MP_BLK = MP_ROWS * MP_HALF;    // bf16 per half image (64 KB)
constexpr int MP_CH = MP_BLK / 8;            // 16-B chunks per half (4096)
constexpr int MP_PF = 4;                     // weight k-steps in flight (2 fragments each; 8 / 12 spill)
constexpr int MP_SC1 = 16;
constexpr uint64_t MP_WAIT_TICKS = 20000000;  // 200 ms of wall_clock64: never hang the GPU

__device__ __forceinline__ int mp_chunk(int row, int c) { return row * 32 + (c ^ (row & 15)); }

__device__ __forceinline__ float mp_act(float v, int act) {
  switch (act) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: return 1.f / (1.f + expf(-v));
    case 3: return tanhf(v);
    default: return v;
  }
}

__device__ __forceinline__ bool mp_wait(int32_t* cnt, int target) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    for (int n = 0; n < 64; ++n) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
      __builtin_amdgcn_s_sleep(1);
    }
    if (wall_clock64() - t0 > MP_WAIT_TICKS) return false;
  }
}

// acc[m][j] += T[rows 16m..][k] . W[col tile nt0 + j][k] over NKS k-steps
template <int NKS, int PFD>
__device__ __forceinline__ void mp_mma(const uint16_t* __restrict__ T, const uint16_t* __restrict__ W, int nt0,
                                       int lane, mp_f32x4 (&acc)[8][2]) {
  constexpr int PF = PFD < NKS ? PFD : NKS - 1;
  constexpr int RING = PF + 1;
  mp_bf16x8 fb[RING][2];
  const uint16_t* wt = W + (size_t)nt0 * 512 + lane * 8;  // k-step-major tiles: [ks][32 column tiles]
  auto load = [&](int ks, mp_bf16x8 (&d)[2]) {
    d[0] = *reinterpret_cast<const mp_bf16x8*>(wt + (size_t)ks * 32 * 512);
    d[1] = *reinterpret_cast<const mp_bf16x8*>(wt + ((size_t)ks * 32 + 1) * 512);
  };
#pragma unroll
  for (int p = 0; p < PF; ++p) load(p, fb[p]);
  const int r16 = lane & 15, q = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (ks + PF < NKS) load(ks + PF, fb[(ks + PF) % RING]);
    __builtin_amdgcn_sched_barrier(0);
    const uint16_t* half = T + (ks >> 3) * MP_BLK;
    const int c = (ks & 7) * 4 + q;
    mp_bf16x8 fa[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = 16 * m + r16;
      fa[m] = *reinterpret_cast<const mp_bf16x8*>(half + mp_chunk(row, c) * 8);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 8; ++m)
        acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[ks % RING][j], acc[m][j], 0, 0, 0);
  }
}

template <int PFD>
__global__ void __launch_bounds__(512, 1) mlp_pair_kernel(MlpChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* const T = reinterpret_cast<uint16_t*>(smem);                 // [2][MP_BLK]
  float* const pfl = reinterpret_cast<float*>(T + 2 * MP_BLK);            // [128][P_NCOLS]
  float* const part = pfl + MP_ROWS * P_NCOLS;                            // [8][128]
  float* const mlv = part + 8 * MP_ROWS;                                  // [128]
  int* const sflag = reinterpret_cast<int*>(mlv + MP_ROWS);

  const int b = blockIdx.x;
  const int mem = (b >> 3) & 1;
  const int cl = (b >> 4) * 8 + (b & 7);
  const int row0 = cl * MP_ROWS;
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  if (row0 >= n_live || cl >= a.pair_clusters) return;  // uniform over the pair
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int32_t* const cnt = a.pair_sync + cl * 16;
  // outputs start as NaN: a pair that gives up (bounded wait) leaves them so, and the host
  // detects it (LtvGpu.wait) instead of reading the previous batch's values
  if (mem == 0 && tid < MP_ROWS && row0 + tid < n_live) {
    if (a.ml) a.ml[row0 + tid] = __builtin_nanf("");
    if (a.ltv_out)
      for (int k = 0; k < 6; ++k) a.ltv_out[(size_t)(row0 + tid) * 6 + k] = __builtin_nanf("");
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      a.pair_x + (size_t)cl * 4 * MP_BLK, 0, 4 * MP_BLK * 2, 0x00020000);

  // ---- input tile: 4 threads per row, 16-B chunks of 8 columns (zeros past in_live / n_live)
  {
    const int r = tid >> 2, row = row0 + r;
    const bool live = row < n_live;
    const int s = (live && a.slots) ? a.slots[row] : -1;
    const int K0 = a.in_w;
    for (int c8 = (tid & 3); c8 * 8 < K0; c8 += 4) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = c8 * 8 + i;
        float x = 0.f;
        if (live && c < a.in_live) {
          if (a.slots) {
            if (s >= 0) {
              if (c < P_NCOLS) x = a.pf_tab[(size_t)s * P_NCOLS + c];
              else if (a.ext_tab && c - P_NCOLS < a.ext_w) x = a.ext_tab[(size_t)s * a.ext_w + (c - P_NCOLS)];
            }
          } else {
            x = a.X[(size_t)row * a.ldx + c];
          }
        }
        if (a.slots && c < P_NCOLS) {
          if (a.ltv_out) pfl[r * P_NCOLS + c] = x;
          x = copysignf(log1pf(fabsf(x)), x);  // [sign*log1p|profile| (25) | extended features]
        }
        v[i] = x;
      }
      uint4 u;
      u.x = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
      u.y = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
      u.z = (uint32_t)f32_to_bf16(v[4]) | ((uint32_t)f32_to_bf16(v[5]) << 16);
      u.w = (uint32_t)f32_to_bf16(v[6]) | ((uint32_t)f32_to_bf16(v[7]) << 16);
      *reinterpret_cast<uint4*>(T + (c8 >> 5) * MP_BLK + mp_chunk(r, c8 & 31) * 8) = u;
    }
  }
  __syncthreads();

  const int nt0 = mem * 16 + wave * 2;  // this wave's first output column tile (of N/16)
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  for (int l = 0; l < a.n_layers; ++l) {
    mp_f32x4 acc[8][2];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m][0] = acc[m][1] = mp_f32x4{0.f, 0.f, 0.f, 0.f};
    switch (a.K[l] >> 5) {
      case 2: mp_mma<2, PFD>(T, a.W[l], nt0, lane, acc); break;
      case 4: mp_mma<4, PFD>(T, a.W[l], nt0, lane, acc); break;
      case 6: mp_mma<6, PFD>(T, a.W[l], nt0, lane, acc); break;
      case 8: mp_mma<8, PFD>(T, a.W[l], nt0, lane, acc); break;
      case 10: mp_mma<10, PFD>(T, a.W[l], nt0, lane, acc); break;
      case 12: mp_mma<12, PFD>(T, a.W[l], nt0, lane, acc); break;
      case 14: mp_mma<14, PFD>(T, a.W[l], nt0, lane, acc); break;
      default: mp_mma<16, PFD>(T, a.W[l], nt0, lane, acc); break;
    }
    const float* bias = a.bias[l];
    const int act = a.act[l];
    if (l + 1 == a.n_layers) {
      // last hidden layer: this member's partial of y = sum_n act(h + b) * w2 over its columns
      float rs[8][4];
#pragma unroll
      for (int m = 0; m < 8; ++m) rs[m][0] = rs[m][1] = rs[m][2] = rs[m][3] = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = (nt0 + j) * 16 + ccol;
        const float bb = bias ? bias[col] : 0.f, w = a.w2[col];
#pragma unroll
        for (int m = 0; m < 8; ++m)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) rs[m][qq] += mp_act(acc[m][j][qq] + bb, act) * w;
      }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          float v = rs[m][qq];
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          if (ccol == 0) part[wave * MP_ROWS + m * 16 + crow + qq] = v;
        }
      break;
    }
    __syncthreads();  // every wave has read the layer's input tile
    uint16_t* const own = T + mem * MP_BLK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl16 = (wave * 2 + j) * 16 + ccol;  // column inside the member's half
      const float bb = bias ? bias[mem * MP_HALF + cl16] : 0.f;
      const int c = cl16 >> 3, e = cl16 & 7;
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int row = m * 16 + crow + qq;
          own[mp_chunk(row, c) * 8 + e] = f32_to_bf16(mp_act(acc[m][j][qq] + bb, act));
        }
    }
    __syncthreads();
    // hand-off: my half -> slab[parity][mem] (sc1), arrive, wait for the partner, its half -> LDS
    const int par = l & 1;
#pragma unroll
    for (int i = 0; i < MP_CH / 512; ++i) {
      const int c = i * 512 + tid;
      const mp_u32x4 v = __builtin_bit_cast(mp_u32x4, *reinterpret_cast<const uint4*>(own + c * 8));
      __builtin_amdgcn_raw_buffer_store_b128(v, xr, c * 16, ((par * 2 + mem) * MP_BLK) * 2, MP_SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool ok = mp_wait(cnt, 2 * (l + 1));
      if (!ok) atomicExch(a.pair_err, 1);
      *sflag = ok;
    }
    __syncthreads();
    if (!*sflag) return;
    {
      const uint16_t* src = a.pair_x + (size_t)cl * 4 * MP_BLK + (size_t)(par * 2 + (mem ^ 1)) * MP_BLK;
      uint16_t* dst = T + (mem ^ 1) * MP_BLK;
#pragma unroll
      for (int i = 0; i < MP_CH / 64 / 8; ++i) {  // 64 pieces of 1 KB, 8 per wave
        const int piece = wave * 8 + i;
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + piece * 512 + lane * 8),
                                         (__attribute__((address_space(3))) void*)(dst + piece * 512), 16, 0, MP_SC1);
      }
    }
    __syncthreads();
  }

  // ---- head: member partials (rows in fixed wave order), member 0 adds both in member order
  __syncthreads();
  float* const gpart = a.pair_part + (size_t)cl * 2 * MP_ROWS;
  if (tid < MP_ROWS) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += part[w * MP_ROWS + tid];
    __hip_atomic_store(gpart + mem * MP_ROWS + tid, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true;
    if (mem == 0) {
      ok = mp_wait(cnt, 2 * a.n_layers);
      if (!ok) atomicExch(a.pair_err, 1);
    }
    *sflag = ok;
  }
  __syncthreads();
  if (mem != 0 || !*sflag) return;
  if (tid < MP_ROWS) {
    const float s0 = __hip_atomic_load(gpart + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float s1 = __hip_atomic_load(gpart + MP_ROWS + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float y = mp_act(s0 + s1 + a.b2, a.act2);
    mlv[tid] = y;
    const int row = row0 + tid;
    if (row < n_live) {
      if (a.ml) a.ml[row] = y;
      if (a.ltv_out) ltv_row(pfl + tid * P_NCOLS, &mlv[tid], a.ltv_out + (size_t)row * 6);
    }
  }
  __syncthreads();
  if (tid == 0) __hip_atomic_exchange(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

int mlp_pair_clusters(int n_rows) { return (n_rows + MP_ROWS - 1) / MP_ROWS; }

bool mlp_pair_eligible(const MlpChainArgs& a) {
  if (a.split || !a.pair_x || !a.pair_sync || !a.pair_part || !a.pair_err) return false;
  if (mlp_pair_clusters(a.n_rows) > a.pair_clusters) return false;
  for (int l = 0; l < a.n_layers; ++l)
    if (a.N[l] != 2 * MP_HALF) return false;
  return a.K[0] % 64 == 0 && a.K[0] <= 2 * MP_HALF;
}

size_t mlp_pair_lds_bytes() {
  return (size_t)2 * MP_BLK * 2 + (size_t)MP_ROWS * P_NCOLS * 4 + (size_t)8 * MP_ROWS * 4 + MP_ROWS * 4 + 16;
}

// grid: 16 workgroups per 8 pairs (b = 16 q + 8 member + g, pair = 8 q + g)
void launch_mlp_pair(const MlpChainArgs& a, hipStream_t st) {
  const int ncl = mlp_pair_clusters(a.n_rows);
  const char* pfe = getenv("IGP_MP_PF");  // A/B of the weight prefetch depth
  const int pf = pfe ? atoi(pfe) : MP_PF;
  if (pf == 8)
    IGP_LAUNCH(mlp_pair_kernel<8>, dim3(((ncl + 7) / 8) * 16), dim3(512), mlp_pair_lds_bytes(), st, a);
  else
    IGP_LAUNCH(mlp_pair_kernel<MP_PF>, dim3(((ncl + 7) / 8) * 16), dim3(512), mlp_pair_lds_bytes(), st, a);
}

}  // namespace igp
