// K3 layer-wise MLP (cfg 4): one large-tile MFMA GEMM launch per layer, the
// alternative to the fused chain (mlp_fused.hip) for big batches.
//
// Why: the fused chain partitions a batch by rows only, so at 8192 rows each CU owns 32-64 rows
// and re-reads every layer's full weight matrix from L2 for them: per 32-wide k-step it needs
// 32 KB of weights for 64 x 512 x 32 MACs, i.e. it runs at the CU's L2 bandwidth, not its MFMA
// rate, and 8192 / 64 = 128 workgroups leave half the chip idle. Here a layer is a plain GEMM
// tiled 128 rows x 128 columns (8192 x 512 -> 256 tiles = one per CU), each CU reading 128 KB
// of activations and 128 KB of weights per layer; the 8 MB activation matrix between layers
// stays in L2 / the 256 MB Infinity Cache. Five launches (4 layers + finish) instead of one,
// ~1.2 us per kernel boundary (MI355X_MICROARCH.md 'boundary').
//
// Tile: 256 threads = 4 waves in 2 x 2, each wave 64 x 64 (4 x 4 v_mfma_f32_16x16x32_bf16
// tiles, f32 accumulators); K in 64-wide steps staged through LDS (two buffers, 144-B padded
// rows: the 16 lanes of an A/B fragment read land in 16 distinct 4-bank groups), the next
// step's global loads in flight under the current step's MFMAs.
// SPLIT: every operand is a bf16 pair (hi, lo = bf16(x - hi)), three MFMAs per product
// (hi*hi + hi*lo + lo*hi): f32-faithful to ~1e-5 relative (the chain's SPLIT numerics).
//
// Block -> tile mapping is XCD-aware: workgroup b runs on XCD b % 8 under round-robin dispatch;
// XCD x gets a contiguous run of tiles ordered (row tile, column tile), so the column tiles of a
// row tile share its activation rows in that XCD's L2.
//
// Sources (A): 0 bf16 activations [M][lda] (+ lo), 1 dense f32 X [M][ldx], 2 the LTV gather
// (slots into the [C][25] profile table, sign*log1p, then the [C][ext_w] extended table).
// Epilogues: 0 act(acc + b) -> bf16 Y [M][ldy] (+ lo) through an LDS transpose (16-B row-
// contiguous stores); 1 the N -> 1 head: per row sum over the tile's 128 columns of
// act(acc + b) * w2 -> part[column tile][row] (fixed order; the finish kernel adds the tiles,
// b2, act2 and runs K9).
#include "common.h"
#include "launch.h"
#include "ltv.h"

namespace igp {
namespace {

typedef __attribute__((ext_vector_type(8))) short ml_bf16x8;
typedef __attribute__((ext_vector_type(4))) float ml_f32x4;

constexpr int ML_BM = 128, ML_BN = 128, ML_BK = 64;
constexpr int ML_LDS = ML_BK + 8;      // bf16 per staged row (144 B)
constexpr int ML_CH = ML_BM * ML_BK / 8 / 256;  // 16-B chunks per thread per operand per k-step (4)

__device__ __forceinline__ float ml_act(float v, int act) {
  switch (act) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: return 1.f / (1.f + expf(-v));
    case 3: return tanhf(v);
    default: return v;
  }
}

__device__ __forceinline__ uint32_t ml_pack(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// 8 f32 -> one 16-B chunk of bf16 (hi) and, SPLIT, of the residuals (lo)
template <bool SPLIT>
__device__ __forceinline__ void ml_cvt8(const float (&f)[8], uint4& hi, uint4& lo) {
  hi = make_uint4(ml_pack(f[0], f[1]), ml_pack(f[2], f[3]), ml_pack(f[4], f[5]), ml_pack(f[6], f[7]));
  if constexpr (SPLIT) {
    float r[8];
    const uint32_t h[4] = {hi.x, hi.y, hi.z, hi.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f[j] - __uint_as_float((h[j >> 1] >> (16 * (j & 1))) << 16);
    lo = make_uint4(ml_pack(r[0], r[1]), ml_pack(r[2], r[3]), ml_pack(r[4], r[5]), ml_pack(r[6], r[7]));
  }
}

template <bool SPLIT, int SRC, int EPI>
__global__ void __launch_bounds__(256) mlp_layer_kernel(MlpLayerArgs a) {
  constexpr int NB = SPLIT ? 2 : 1;  // operand planes: hi (+ lo)
  __shared__ __attribute__((aligned(16))) uint16_t sA[NB][2][ML_BM * ML_LDS];
  __shared__ __attribute__((aligned(16))) uint16_t sB[NB][2][ML_BN * ML_LDS];
  __shared__ float hpart[2][ML_BM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order (see the header)
  const int per = (a.tiles + 7) >> 3;
  const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (tile >= a.tiles) return;
  const int rt = tile / a.col_tiles, ct = tile - rt * a.col_tiles;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = rt * ML_BM, col0 = ct * ML_BN;
  if (row0 >= M) return;  // uniform per block, before any barrier
  const int n_kt = a.K / ML_BK;

  uint4 ra[NB][ML_CH], rb[NB][ML_CH];
  int slot[ML_CH];
  if constexpr (SRC == 2) {
#pragma unroll
    for (int c = 0; c < ML_CH; ++c) {
      const int row = row0 + ((tid + c * 256) >> 3);
      slot[c] = row < M ? a.slots[row] : -1;
    }
  }
  auto load = [&](int kt) {
    const int k0 = kt * ML_BK;
#pragma unroll
    for (int c = 0; c < ML_CH; ++c) {
      const int ch = tid + c * 256;
      const int r = ch >> 3, kc = k0 + (ch & 7) * 8;
      const int row = row0 + r;
      if constexpr (SRC == 0) {
        const size_t o = (size_t)row * a.lda + kc;
        ra[0][c] = row < M ? *reinterpret_cast<const uint4*>(a.A + o) : make_uint4(0, 0, 0, 0);
        if constexpr (SPLIT) ra[1][c] = row < M ? *reinterpret_cast<const uint4*>(a.A_lo + o) : make_uint4(0, 0, 0, 0);
      } else {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = kc + j;
          float x = 0.f;
          if (row < M && k < a.in_live) {
            if constexpr (SRC == 1) {
              x = a.X[(size_t)row * a.ldx + k];
            } else {
              const int s = slot[c];
              if (s >= 0) {
                if (k < P_NCOLS) {
                  const float p = a.pf_tab[(size_t)s * P_NCOLS + k];
                  x = copysignf(log1pf(fabsf(p)), p);
                } else if (a.ext_tab && k - P_NCOLS < a.ext_w) {
                  x = a.ext_tab[(size_t)s * a.ext_w + (k - P_NCOLS)];
                }
              }
            }
          }
          f[j] = x;
        }
        uint4 lo;
        ml_cvt8<SPLIT>(f, ra[0][c], lo);
        if constexpr (SPLIT) ra[1][c] = lo;
      }
      // W [N_pad][K]: zero padded to the 128-column tile and the 64-wide k-step
      const size_t wo = (size_t)(col0 + r) * a.K + kc;
      rb[0][c] = *reinterpret_cast<const uint4*>(a.W + wo);
      if constexpr (SPLIT) rb[1][c] = *reinterpret_cast<const uint4*>(a.W_lo + wo);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int p = 0; p < NB; ++p)
#pragma unroll
      for (int c = 0; c < ML_CH; ++c) {
        const int ch = tid + c * 256;
        const int o = (ch >> 3) * ML_LDS + (ch & 7) * 8;
        *reinterpret_cast<uint4*>(&sA[p][buf][o]) = ra[p][c];
        *reinterpret_cast<uint4*>(&sB[p][buf][o]) = rb[p][c];
      }
  };

  ml_f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = ml_f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < n_kt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < n_kt) load(kt + 1);  // next step's global loads in flight under the MFMAs
#pragma unroll
    for (int kk = 0; kk < ML_BK / 32; ++kk) {
      const int kof = kk * 32 + 8 * (lane >> 4);
      ml_bf16x8 fa[NB][4], fb[NB][4];
#pragma unroll
      for (int p = 0; p < NB; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          fa[p][i] = *reinterpret_cast<const ml_bf16x8*>(&sA[p][cur][(wm * 64 + i * 16 + (lane & 15)) * ML_LDS + kof]);
          fb[p][i] = *reinterpret_cast<const ml_bf16x8*>(&sB[p][cur][(wn * 64 + i * 16 + (lane & 15)) * ML_LDS + kof]);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (SPLIT) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
        }
    }
    if (kt + 1 < n_kt) store(cur ^ 1);
    __syncthreads();
  }

  if constexpr (EPI == 0) {
    // act(acc + b) -> bf16 tile in LDS (the A staging buffers are free now), then 16-B stores of
    // whole row runs: 128 columns = 256 B per row
    uint16_t* T = &sA[0][0][0];                           // [128][136] hi over both buffers of plane 0
    uint16_t* Tl = SPLIT ? &sA[NB - 1][0][0] : nullptr;   // lo over plane 1
    constexpr int TS = ML_BN + 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = wn * 64 + j * 16 + (lane & 15);
      const float b = a.bias ? a.bias[col0 + cl] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = wm * 64 + i * 16 + 4 * (lane >> 4) + q;
          const float v = ml_act(acc[i][j][q] + b, a.act);
          const uint16_t h = f32_to_bf16(v);
          T[rl * TS + cl] = h;
          if constexpr (SPLIT) Tl[rl * TS + cl] = f32_to_bf16(v - __uint_as_float((uint32_t)h << 16));
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < (ML_BM * ML_BN / 8) / 256; ++c) {
      const int ch = tid + c * 256;
      const int rl = ch >> 4, cc = (ch & 15) * 8;
      const int row = row0 + rl;
      if (row >= M) continue;
      const size_t o = (size_t)row * a.ldy + col0 + cc;
      *reinterpret_cast<uint4*>(a.Y + o) = *reinterpret_cast<const uint4*>(&T[rl * TS + cc]);
      if constexpr (SPLIT) *reinterpret_cast<uint4*>(a.Y_lo + o) = *reinterpret_cast<const uint4*>(&Tl[rl * TS + cc]);
    }
  } else {
    // head partial: per row, sum over this tile's columns of act(acc + b) * w2
    float rs[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) rs[i][0] = rs[i][1] = rs[i][2] = rs[i][3] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = col0 + wn * 64 + j * 16 + (lane & 15);
      const float b = a.bias ? a.bias[col] : 0.f, w = a.w2[col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) rs[i][q] += ml_act(acc[i][j][q] + b, a.act) * w;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = rs[i][q];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if ((lane & 15) == 0) hpart[wn][wm * 64 + i * 16 + 4 * (lane >> 4) + q] = v;
      }
    __syncthreads();
    if (tid < ML_BM) {
      const int row = row0 + tid;
      if (row < M) a.part[(size_t)ct * a.M + row] = hpart[0][tid] + hpart[1][tid];
    }
  }
}

// finish: y = act2(sum of the column tiles' partials + b2) -> ml and / or K9 (ltv_row) rows
__global__ void __launch_bounds__(256) mlp_layer_finish_kernel(MlpLayerArgs a) {
  __shared__ float zero_row[P_NCOLS];
  if (threadIdx.x < P_NCOLS) zero_row[threadIdx.x] = 0.f;
  __syncthreads();
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= M) return;
  float s = 0.f;
  for (int t = 0; t < a.col_tiles; ++t) s += a.part[(size_t)t * a.M + row];
  float y = ml_act(s + a.b2, a.act2);
  if (a.ml) a.ml[row] = y;
  if (a.ltv_out) {
    const int sl = a.slots[row];
    ltv_row(sl >= 0 ? a.pf_tab + (size_t)sl * P_NCOLS : zero_row, &y, a.ltv_out + (size_t)row * 6);
  }
}

template <bool SPLIT>
void launch_layer(const MlpLayerArgs& a, hipStream_t st) {
  const dim3 grid(8 * ((a.tiles + 7) / 8)), block(256);
  if (a.epi == 0) {
    if (a.src == 0) IGP_LAUNCH((mlp_layer_kernel<SPLIT, 0, 0>), grid, block, 0, st, a);
    else if (a.src == 1) IGP_LAUNCH((mlp_layer_kernel<SPLIT, 1, 0>), grid, block, 0, st, a);
    else IGP_LAUNCH((mlp_layer_kernel<SPLIT, 2, 0>), grid, block, 0, st, a);
  } else {
    if (a.src == 0) IGP_LAUNCH((mlp_layer_kernel<SPLIT, 0, 1>), grid, block, 0, st, a);
    else if (a.src == 1) IGP_LAUNCH((mlp_layer_kernel<SPLIT, 1, 1>), grid, block, 0, st, a);
    else IGP_LAUNCH((mlp_layer_kernel<SPLIT, 2, 1>), grid, block, 0, st, a);
  }
}

}  // namespace

void launch_mlp_layer(const MlpLayerArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  if (a.split) launch_layer<true>(a, st);
  else launch_layer<false>(a, st);
}

void launch_mlp_layer_finish(const MlpLayerArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  IGP_LAUNCH(mlp_layer_finish_kernel, dim3((a.M + 255) / 256), dim3(256), 0, st, a);
}

}  // namespace igp
