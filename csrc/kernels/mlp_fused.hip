// K3 MLP chain fused into one kernel (VERDICT r1 "fused 4-layer MLP ... activation tile in
// LDS, weights streamed from L2"): cfg 4's LTV model, input [rows, 256] -> 4 x (Gemm 512 + Relu)
// -> Gemm 512 -> 1, plus (optionally) the model input gather from the HBM player tables and the
// K9 churn / segment / next-best-action epilogue.
//
// One workgroup = 32 rows, 4 waves (8192 rows -> 256 workgroups, one per CU). The 32-row
// activation tile lives in LDS for the whole chain (bf16, two 32 x 512 buffers ping-ponged
// between layers: 66.5 KB), so hidden activations never touch HBM and the chain is one launch
// instead of five. Each wave owns a quarter of a layer's output columns (N/4 <= 128: eight
// 16-column MFMA tiles x two 16-row tiles, v_mfma_f32_16x16x32_bf16, f32 accumulators). A
// fragments come from LDS (ds_read_b128; 16-B chunks XOR-swizzled by row, mc_idx, spread a read over all
// 64 banks); B fragments are 16-byte loads straight from the weights [N][K] (L2-resident: the
// whole 4 x 512 chain is 1.8 MB bf16, every workgroup reads it), prefetched two K-steps ahead
// into a 3-deep register ring. Bias + activation + bf16 rounding of a hidden layer happen in
// the epilogue that writes the next layer's LDS tile; the last hidden layer's epilogue instead
// applies the N -> 1 head (per-lane partial dots, xor-shuffle row sums, a 4-wave LDS reduce).
//
// Numerics = the unfused bf16 path (gemm.hip / mlp_head): bf16 weights and activations, f32
// accumulation, bf16 rounding of each hidden activation.
//
// SPLIT (the ONNX model's f32 contract, default for fp32 plans): every weight and activation is
// carried as a pair of bf16 values hi + lo (hi = bf16(x), lo = bf16(x - hi), ~17 significant
// bits), and each product runs as three MFMAs, hi*hi + hi*lo + lo*hi (lo*lo, ~2^-18 relative,
// is dropped), accumulated in f32: f32-faithful to ~1e-5 relative at bf16 MFMA rates, where the
// f32 MFMA (v_mfma_f32_16x16x4_f32) would run the chain ~16x slower. The hi and lo activation
// tiles both live in LDS (4 x 32 x 512 bf16 = 128 KB).
#include "common.h"
#include "launch.h"
#include "ltv.h"

namespace igp {

typedef __attribute__((ext_vector_type(8))) short mc_bf16x8;
typedef __attribute__((ext_vector_type(4))) float mc_f32x4;

constexpr int MC_LDA = 512;  // bf16 elements per LDS row (1024 B, 64 chunks of 16 B, swizzled)
// element (row, col) of an LDS activation tile: 16-B chunk col / 8 of the row stored at chunk
// (col / 8) ^ (row & 15). ds_read_b128 serves a wave in 4 lane groups ({0-3, 12-15, 20-27}, ...,
// MI355X_MICROARCH.md LDS table); with the old 1040-B pitch rows r and r + 12 of one group hit
// the same bank (SQ_LDS_BANK_CONFLICT ~2 cycles per LDS instruction, profiles/r3/n); swizzled,
// every group of an A-fragment read touches 16 distinct 16-B bank slots.
__device__ __forceinline__ int mc_idx(int row, int col) {
  return row * MC_LDA + ((((col >> 3) ^ (row & 15))) << 3) + (col & 7);
}
constexpr int MC_PF = 5;  // k-steps of weight fragments prefetched ahead
// the split chain's (hi + lo fragments: twice the registers per k-step): one k-step ahead. Two
// ahead spilled 2 VGPRs at 2 waves per SIMD and ran slower (8192 rows: 120 -> 124-126 us alone,
// cfg4 engine_only 137.6 -> 133.9 M, profiles/r6/z); three spilled 47
constexpr int MC_PFS = 1;

__device__ __forceinline__ float mc_act(float v, int act) {
  switch (act) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: return 1.f / (1.f + expf(-v));
    case 3: return tanhf(v);
    default: return v;
  }
}

// one layer's MFMA loop: acc[m][j] += Hin[m-th 16 rows][:K] . W[col tile j][:K]^T.
// W arrives fragment-packed (MlpChainPack): tile (nt, ks) = 64 lanes x 8 bf16 contiguous, lane l
// holding W[16 nt + (l & 15)][32 ks + 8 (l >> 4) .. +8], so each B-fragment load is one fully
// coalesced 1 KB wave read (row-major W made it 16 half-used 128-B lines per instruction and
// the texture path, not the MFMA, set the pace: 92 -> see profiles/NOTES.md).
template <int NKS, int MT, int JT, bool SPLIT, int PFD = MC_PF>
__device__ __forceinline__ void mc_layer_mma(const uint16_t* __restrict__ Hin, const uint16_t* __restrict__ Hlo,
                                             const uint16_t* __restrict__ W, const uint16_t* __restrict__ Wlo, int N,
                                             int colw, int NT, int lane, mc_f32x4 (&acc)[MT][JT]) {
  const int NTT = N >> 4;  // column tiles of the layer: a k-step's tiles are NTT x 1 KB contiguous
  if constexpr (SPLIT) {
    // hi*hi + hi*lo + lo*hi per k-step; both weight halves prefetched PFD k-steps ahead (a ring
    // of PFD + 1 fragment sets: 8 x 16 B per lane per k-step at JT = 4)
    constexpr int PF = PFD < NKS ? PFD : NKS - 1;
    constexpr int RING = PF + 1;
    mc_bf16x8 fh[RING][JT], fl[RING][JT];
    const int kq = 8 * (lane >> 4);
    const size_t woff = (size_t)(colw >> 4) * 512 + lane * 8;
    int jt[JT];
#pragma unroll
    for (int j = 0; j < JT; ++j) jt[j] = j < NT ? j : NT - 1;
    auto load = [&](int ks, mc_bf16x8 (&dh)[JT], mc_bf16x8 (&dl)[JT]) {
#pragma unroll
      for (int j = 0; j < JT; ++j) {
        dh[j] = *reinterpret_cast<const mc_bf16x8*>(W + woff + ((size_t)ks * NTT + jt[j]) * 512);
        dl[j] = *reinterpret_cast<const mc_bf16x8*>(Wlo + woff + ((size_t)ks * NTT + jt[j]) * 512);
      }
    };
#pragma unroll
    for (int p = 0; p < PF; ++p) load(p, fh[p], fl[p]);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks + PF < NKS) load(ks + PF, fh[(ks + PF) % RING], fl[(ks + PF) % RING]);
      __builtin_amdgcn_sched_barrier(0);
      mc_bf16x8 ah[MT], al[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int o = mc_idx(16 * m + (lane & 15), ks * 32 + kq);
        ah[m] = *reinterpret_cast<const mc_bf16x8*>(&Hin[o]);
        al[m] = *reinterpret_cast<const mc_bf16x8*>(&Hlo[o]);
      }
#pragma unroll
      for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[m], fh[ks % RING][j], acc[m][j], 0, 0, 0);
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], fl[ks % RING][j], acc[m][j], 0, 0, 0);
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], fh[ks % RING][j], acc[m][j], 0, 0, 0);
        }
    }
    return;
  }
  // PF k-steps of B fragments in flight (5 by default: deeper rings spill, r3/q)
  constexpr int PF = PFD < NKS ? PFD : NKS - 1;
  constexpr int RING = PF + 1;
  mc_bf16x8 fb[RING][JT];
  const int kq = 8 * (lane >> 4);
  const uint16_t* wt = W + (size_t)(colw >> 4) * 512 + lane * 8;  // this wave's first n-tile
  // branch-free: tiles j >= NT (layers narrower than 512) re-load tile NT-1 and their
  // accumulators are never read; a guarded load made hipcc branch and wait vmcnt(0) per load
  int jt[JT];
#pragma unroll
  for (int j = 0; j < JT; ++j) jt[j] = j < NT ? j : NT - 1;
  auto load = [&](int ks, mc_bf16x8 (&dst)[JT]) {
#pragma unroll
    for (int j = 0; j < JT; ++j) dst[j] = *reinterpret_cast<const mc_bf16x8*>(wt + ((size_t)ks * NTT + jt[j]) * 512);
  };
#pragma unroll
  for (int p = 0; p < PF; ++p) load(p, fb[p]);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (ks + PF < NKS) load(ks + PF, fb[(ks + PF) % RING]);
    // keep the prefetch at the top of the step: without this fence the scheduler sank each
    // load next to its MFMAs and the loop ran at vmcnt(1) (one load in flight per wave)
    __builtin_amdgcn_sched_barrier(0);
    mc_bf16x8 fa[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
      fa[m] = *reinterpret_cast<const mc_bf16x8*>(&Hin[mc_idx(16 * m + (lane & 15), ks * 32 + kq)]);
#pragma unroll
    for (int j = 0; j < JT; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[ks % RING][j], acc[m][j], 0, 0, 0);
  }
}

// the bf16 pair of an f32 value: hi = bf16(x), lo = bf16(x - hi)
__device__ __forceinline__ void mc_split(float x, uint16_t& hi, uint16_t& lo) {
  hi = f32_to_bf16(x);
  lo = f32_to_bf16(x - __uint_as_float((uint32_t)hi << 16));
}

// NBUF = 2: the activation tile is ping-ponged between layers; NBUF = 1 (64-row split tiles,
// whose hi + lo tiles fill 128 KB of LDS once): a layer's outputs wait in the accumulators until
// every wave has read its input, then overwrite the tile in place (one more barrier per layer).
template <int MC_ROWS, int WAVES, bool SPLIT, int PFD = MC_PF, int NBUF = 2>
__global__ void __launch_bounds__(64 * WAVES) mlp_chain_kernel(MlpChainArgs a) {
  constexpr int MT = MC_ROWS / 16;            // 16-row MFMA tiles per wave
  constexpr int THREADS = 64 * WAVES;
  constexpr int PARTS = THREADS / MC_ROWS;    // staging threads per row
  constexpr int JT = 32 / WAVES;              // 16-column tiles per wave at N = 512
  // [0, NBUF): hi tiles (ping-pong when NBUF = 2); SPLIT: [NBUF, 2 NBUF) the matching lo tiles
  __shared__ __attribute__((aligned(16))) uint16_t H[(SPLIT ? 2 : 1) * NBUF][MC_ROWS * MC_LDA];
  __shared__ float part[WAVES][MC_ROWS];
  __shared__ float mlv[MC_ROWS];
  __shared__ float pfl[MC_ROWS][P_NCOLS];  // raw profile rows for the K9 epilogue
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * MC_ROWS;
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  if (row0 >= n_live) return;  // uniform per block, before any barrier

  // ---- stage the 32-row input tile (bf16) into H[0]: thread t stages row t/8, columns
  // [32 (t%8), +32), all 32 loads issued before the first use (one memory round trip, not 32);
  // LTV: the raw 25 profile values of each row are kept in LDS for the K9 epilogue
  const int K0 = a.in_w;  // padded to the first layer's K (a multiple of 64); columns >= in_live are 0
  {
    const int r = tid / PARTS, row = row0 + r;
    const bool live = row < n_live;
    const int s = (live && a.slots) ? a.slots[row] : -1;
    for (int c0 = (tid % PARTS) * 32; c0 < K0; c0 += PARTS * 32) {
      float v[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int c = c0 + i;
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
        v[i] = x;
      }
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int c = c0 + i;
        float x = v[i];
        if (a.slots && c < P_NCOLS) {
          if (a.ltv_out) pfl[r][c] = x;
          x = copysignf(log1pf(fabsf(x)), x);  // [sign*log1p|profile| (25) | extended features]
        }
        if constexpr (SPLIT) {
          mc_split(x, H[0][mc_idx(r, c)], H[NBUF][mc_idx(r, c)]);
        } else {
          H[0][mc_idx(r, c)] = f32_to_bf16(x);
        }
      }
    }
  }
  __syncthreads();

  int cur = 0;
  for (int l = 0; l < a.n_layers; ++l) {
    const int K = a.K[l], N = a.N[l], NT = N / (16 * WAVES);
    const int colw = wave * (N / WAVES);
    mc_f32x4 acc[MT][JT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < JT; ++j) acc[m][j] = mc_f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* Hin = H[cur];
    const uint16_t* Hlo = H[SPLIT ? NBUF + cur : cur];
    const uint16_t* Wl = SPLIT ? a.W_lo[l] : nullptr;
    switch (K >> 5) {  // K-steps of 32 (the host allows 2..16)
      case 2: mc_layer_mma<2, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      case 4: mc_layer_mma<4, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      case 6: mc_layer_mma<6, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      case 8: mc_layer_mma<8, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      case 10: mc_layer_mma<10, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      case 12: mc_layer_mma<12, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      case 14: mc_layer_mma<14, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
      default: mc_layer_mma<16, MT, JT, SPLIT, PFD>(Hin, Hlo, a.W[l], Wl, N, colw, NT, lane, acc); break;
    }
    const float* bias = a.bias[l];
    const int act = a.act[l];
    if (l + 1 < a.n_layers) {
      // hidden layer: bias + act -> bf16 -> the next layer's LDS tile
      const int nxt = NBUF == 2 ? cur ^ 1 : 0;
      uint16_t* Hout = H[nxt];
      uint16_t* Hout_lo = H[SPLIT ? NBUF + nxt : nxt];
      if constexpr (NBUF == 1) __syncthreads();  // every wave has read this layer's input tile
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < JT; ++j) {
          if (j >= NT) continue;
          const int col = colw + j * 16 + (lane & 15);
          const float b = bias ? bias[col] : 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int o = mc_idx(m * 16 + 4 * (lane >> 4) + q, col);
            const float v = mc_act(acc[m][j][q] + b, act);
            if constexpr (SPLIT) mc_split(v, Hout[o], Hout_lo[o]);
            else Hout[o] = f32_to_bf16(v);
          }
        }
      __syncthreads();
      cur = nxt;
      continue;
    }
    // last hidden layer: y[r] = act2(sum_n act(h[r][n] + b[n]) * w2[n] + b2)
    float rs[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m) rs[m][0] = rs[m][1] = rs[m][2] = rs[m][3] = 0.f;
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      if (j >= NT) continue;
      const int col = colw + j * 16 + (lane & 15);
      const float b = bias ? bias[col] : 0.f, w = a.w2[col];
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) rs[m][q] += mc_act(acc[m][j][q] + b, act) * w;
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = rs[m][q];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if ((lane & 15) == 0) part[wave][m * 16 + 4 * (lane >> 4) + q] = v;
      }
  }
  __syncthreads();
  if (tid < MC_ROWS) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) sum += part[w][tid];
    const float y = mc_act(sum + a.b2, a.act2);
    mlv[tid] = y;
    const int row = row0 + tid;
    if (row < n_live) {  // rows past the device live count stay untouched
      if (a.ml) a.ml[row] = y;
      if (a.ltv_out) ltv_row(pfl[tid], &mlv[tid], a.ltv_out + (size_t)row * 6);  // K9, learned LTV
    }
  }
}

void launch_mlp_chain(const MlpChainArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  const int r = a.rows_per_block;
  if (a.split) {  // f32-faithful: hi + lo tiles fill the LDS (64 rows: each tile once, NBUF = 1)
    if (a.waves == 8 && r == 64)
      IGP_LAUNCH((mlp_chain_kernel<64, 8, true, MC_PFS, 1>), dim3((a.n_rows + 63) / 64), dim3(512), 0, st, a);
    else if (a.waves == 8)
      IGP_LAUNCH((mlp_chain_kernel<32, 8, true, MC_PFS>), dim3((a.n_rows + 31) / 32), dim3(512), 0, st, a);
    else
      IGP_LAUNCH((mlp_chain_kernel<32, 4, true, MC_PFS>), dim3((a.n_rows + 31) / 32), dim3(256), 0, st, a);
    return;
  }
  if (a.waves == 8 && r == 64) {
    // 64 rows x 8 waves (4 x 4 MFMA tiles per wave): per k-step a CU issues as many MFMA cycles
    // as it needs L1 cycles for the 32 KB of weight fragments (32 rows: half); a batch then
    // occupies half the CUs and the per-slot streams keep two batches in flight. Weights
    // prefetched 5 k-steps ahead: deeper rings (8 / 10) spilled and ran slower (r3/q)
    IGP_LAUNCH((mlp_chain_kernel<64, 8, false, 5>), dim3((a.n_rows + 63) / 64), dim3(512), 0, st, a);
  } else if (a.waves == 8) {
    // 32 rows x 8 waves: a k-step is 8 MFMAs per wave (~0.11 us at two waves per SIMD) against
    // ~1 us of L2 latency for the weight fragments every CU of the XCD reads at the same time
    IGP_LAUNCH((mlp_chain_kernel<32, 8, false, 5>), dim3((a.n_rows + 31) / 32), dim3(512), 0, st, a);
  }
  else if (r == 64)
    IGP_LAUNCH((mlp_chain_kernel<64, 4, false>), dim3((a.n_rows + 63) / 64), dim3(256), 0, st, a);
  else if (r == 16)
    IGP_LAUNCH((mlp_chain_kernel<16, 4, false>), dim3((a.n_rows + 15) / 16), dim3(256), 0, st, a);
  else
    IGP_LAUNCH((mlp_chain_kernel<32, 4, false>), dim3((a.n_rows + 31) / 32), dim3(256), 0, st, a);
}

}  // namespace igp
