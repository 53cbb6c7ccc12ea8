// K3 layer-wise MLP (cfg 4): one MFMA GEMM launch per layer over the whole
// chip, the alternative to the fused chain (mlp_fused.hip) for big batches.
//
// Why: the fused chain partitions a batch by rows only, so at 8192 rows each CU owns 64 rows and
// re-streams every layer's full weight matrix from L2 for them (a 32-wide k-step = 32 KB of
// weights per 64 x 512 x 32 MACs: L2-bandwidth bound), and 8192 / 64 = 128 workgroups leave
// half the chip idle. Here a layer is a GEMM cut into 256 tiles (one per CU at 8192 x 512), each
// CU reading only its tile's activation rows and weight columns; the 8 MB activation matrix
// between layers stays in L2 / the 256 MB Infinity Cache.
//
// The first version staged 64-wide k-steps through LDS with one step of prefetch: ~30 us per
// 8192 x 512 x 512 layer (profiles/r4/f): every k-step exposed a full memory round trip while
// its MFMAs take ~0.1 us. So now a tile's WHOLE activation block is requested at once: the
// kernel starts with every A load of the tile in flight as LDS-DMA (`global_load_lds`, 1 KB per
// wave instruction, no registers), landing as an MFMA-fragment image (1 KB block per (16-row
// tile, 32-wide k-step), lane l's 16 B at l * 16: every A-fragment read is one conflict-free
// ds_read_b128); the weights, L2-resident and shared by all row tiles, stream as fragment-packed
// 1-KB wave loads (pack_fragments, k-step major) into a register ring PF k-steps deep. One
// memory round trip per layer instead of one per k-step.
//
// Tiles: BM x BN with 4 waves, each wave 64 x 64 (4 x 4 v_mfma_f32_16x16x32_bf16, f32
// accumulators): bf16 128 x 128 (A image 128 KB at K = 512), SPLIT 64 x 256 (hi + lo images,
// 128 KB). SPLIT: every operand a bf16 pair (hi, lo = bf16(x - hi)), three MFMAs per product
// (hi*hi + hi*lo + lo*hi): f32-faithful to ~1e-5 relative, the chain's SPLIT numerics.
//
// Block -> tile order is XCD-aware: workgroup b runs on XCD b % 8 under round-robin dispatch;
// XCD x gets a contiguous run of tiles ordered (row tile, column tile), so the column tiles of a
// row tile share its activation rows in that XCD's L2.
//
// Sources (A): 0 bf16 activations [M][lda] (+ lo; LDS-DMA), 1 dense f32 X [M][ldx], 2 the LTV
// gather (slots into the [C][25] profile table, sign*log1p, then the [C][ext_w] extended table)
// - 1 / 2 are converted in registers and stored into the same image. Epilogues: 0 act(acc + b)
// -> bf16 Y [M][ldy] (+ lo) through an LDS transpose (16-B row-contiguous stores); 1 the N -> 1
// head: per row, sum over the tile's columns of act(acc + b) * w2 -> part[column tile][row]
// (fixed order; the finish kernel adds the tiles, b2, act2 and runs K9).
#include "common.h"
#include "launch.h"
#include "ltv.h"

namespace igp {
namespace {

typedef __attribute__((ext_vector_type(8))) short ml_bf16x8;
typedef __attribute__((ext_vector_type(4))) float ml_f32x4;

constexpr int ML_LDS_BYTES = 128 * 1024;  // the A image (and the epilogue's output tile)

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

template <bool SPLIT>
struct MlTile {
  static constexpr int BM = SPLIT ? 64 : 128;   // rows per tile
  static constexpr int BN = SPLIT ? 256 : 128;  // columns per tile
  static constexpr int WM = BM / 64;            // waves along rows (2 / 1)
  static constexpr int WN = 4 / WM;             // waves along columns (2 / 4)
  static constexpr int RT = BM / 16;            // 16-row tiles of the A image
  static constexpr int PF = SPLIT ? 5 : 8;      // weight k-steps in flight (register ring)
};

// A image: block (plane p, k-step ks, row tile rt) of 512 bf16 at ((p * NKS + ks) * RT + rt) * 512;
// lane l's fragment (row rt * 16 + (l & 15), k ks * 32 + 8 (l >> 4) .. +8) at + l * 8
template <bool SPLIT, int NKS>
__device__ __forceinline__ int ml_blk(int p, int ks, int rt) {
  return ((p * NKS + ks) * MlTile<SPLIT>::RT + rt) * 512;
}

template <bool SPLIT, int SRC, int EPI, int NKS>
__device__ __forceinline__ void ml_body(const MlpLayerArgs& a, uint16_t* img, float (&hpart)[4][128], int row0,
                                        int col0, int ct, int M) {
  using T = MlTile<SPLIT>;
  constexpr int NB = SPLIT ? 2 : 1;  // operand planes: hi (+ lo)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WN, wn = wave % T::WN;
  // phase trace (tools/mlp_layerwise_bench.py --trace): wall clock (100 MHz) of blocks < 64, wave 0
  int64_t* const tr = (a.trace && blockIdx.x < 64 && tid == 0) ? a.trace + (size_t)blockIdx.x * 8 : nullptr;
#define ML_MARK(k) \
  if (tr) tr[k] = (int64_t)wall_clock64()
  ML_MARK(0);

  // ---- 1. the tile's whole A block -> the LDS image
  if constexpr (SRC == 0) {
    // LDS-DMA: (planes x NKS x RT) blocks of 1 KB, wave w issues blocks w, w + 4, ...
    constexpr int NBLK = NB * NKS * T::RT;
    static_assert(NBLK % 4 == 0, "blocks per wave");
    const int rmax = a.M - 1;  // rows past the live count read (finite) stale rows, never stored
#pragma unroll
    for (int j = 0; j < NBLK / 4; ++j) {
      const int b = wave + 4 * j;
      const int p = b / (NKS * T::RT), r = b % (NKS * T::RT);
      const int ks = r / T::RT, rt = r % T::RT;
      const int row = min(row0 + rt * 16 + (lane & 15), rmax);
      const uint16_t* src = (p ? a.A_lo : a.A) + (size_t)row * a.lda + ks * 32 + 8 * (lane >> 4);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                       (__attribute__((address_space(3))) void*)(img + b * 512), 16, 0, 0);
    }
  } else {
    // converted sources: chunk c = (k-step, row tile, lane) -> 8 f32 gathered, bf16 (+ lo); two
    // chunks' loads in flight per thread per round (PER / 2 round trips, not PER)
    constexpr int PER = NKS * T::RT * 64 / 256;
    static_assert(PER % 2 == 0, "chunks per thread");
#pragma unroll
    for (int g0 = 0; g0 < PER; g0 += 2) {
      float f[2][8];
      int cks[2], crt[2], cl[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + (g0 + u) * 256;
        const int l = c & 63, r = c >> 6;
        const int ks = r / T::RT, rt = r % T::RT;
        cks[u] = ks, crt[u] = rt, cl[u] = l;
        const int row = row0 + rt * 16 + (l & 15);
        const int k0 = ks * 32 + 8 * (l >> 4);
        int s = -1;
        if constexpr (SRC == 2) s = row < M ? a.slots[row] : -1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = k0 + j;
          float x = 0.f;
          if (row < M && k < a.in_live) {
            if constexpr (SRC == 1) {
              x = a.X[(size_t)row * a.ldx + k];
            } else if (s >= 0) {
              if (k < P_NCOLS) {
                const float pv = a.pf_tab[(size_t)s * P_NCOLS + k];
                x = copysignf(log1pf(fabsf(pv)), pv);
              } else if (a.ext_tab && k - P_NCOLS < a.ext_w) {
                x = a.ext_tab[(size_t)s * a.ext_w + (k - P_NCOLS)];
              }
            }
          }
          f[u][j] = x;
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        uint4 hi, lo;
        ml_cvt8<SPLIT>(f[u], hi, lo);
        *reinterpret_cast<uint4*>(img + ml_blk<SPLIT, NKS>(0, cks[u], crt[u]) + cl[u] * 8) = hi;
        if constexpr (SPLIT) *reinterpret_cast<uint4*>(img + ml_blk<SPLIT, NKS>(1, cks[u], crt[u]) + cl[u] * 8) = lo;
      }
    }
  }

  // ---- 2. weight ring: fragment-packed W [NKS][N/16][64][8], this wave's 4 column tiles
  const int NT = a.n_tiles;
  const size_t woff = ((size_t)((col0 >> 4) + wn * 4) * 64 + lane) * 8;
  constexpr int PF = T::PF < NKS ? T::PF : NKS - 1;
  constexpr int RING = PF + 1;
  ml_bf16x8 fb[RING][NB][4];
  auto wload = [&](int ks, ml_bf16x8 (&dst)[NB][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t o = woff + ((size_t)ks * NT + j) * 512;
      dst[0][j] = *reinterpret_cast<const ml_bf16x8*>(a.W + o);
      if constexpr (SPLIT) dst[1][j] = *reinterpret_cast<const ml_bf16x8*>(a.W_lo + o);
    }
  };
  ML_MARK(1);
#pragma unroll
  for (int p = 0; p < PF; ++p) wload(p, fb[p]);
  // the image: every wave's LDS-DMA landed (vmcnt), then every wave's (barrier)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ML_MARK(2);
  __syncthreads();
  ML_MARK(3);

  // ---- 3. MFMAs
  ml_f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = ml_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (ks + PF < NKS) wload(ks + PF, fb[(ks + PF) % RING]);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top of the step
    ml_bf16x8 fa[NB][4];
#pragma unroll
    for (int p = 0; p < NB; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[p][i] = *reinterpret_cast<const ml_bf16x8*>(img + ml_blk<SPLIT, NKS>(p, ks, wm * 4 + i) + lane * 8);
    const auto& w = fb[ks % RING];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (SPLIT) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][i], w[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], w[1][j], acc[i][j], 0, 0, 0);
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], w[0][j], acc[i][j], 0, 0, 0);
      }
  }

  ML_MARK(4);
  if constexpr (EPI == 0) {
    // ---- 4a. act(acc + b) -> bf16 tile in LDS (over the consumed A image), then 16-B stores of
    // whole row runs
    __syncthreads();  // every wave done reading the image
    constexpr int TS = T::BN + 8;
    uint16_t* Th = img;
    uint16_t* Tl = img + T::BM * TS;
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
          Th[rl * TS + cl] = h;
          if constexpr (SPLIT) Tl[rl * TS + cl] = f32_to_bf16(v - __uint_as_float((uint32_t)h << 16));
        }
    }
    __syncthreads();
    constexpr int CPR = T::BN / 8;  // 16-B chunks per row
#pragma unroll
    for (int c = 0; c < T::BM * CPR / 256; ++c) {
      const int ch = tid + c * 256;
      const int rl = ch / CPR, cc = (ch % CPR) * 8;
      const int row = row0 + rl;
      if (row >= M) continue;
      const size_t o = (size_t)row * a.ldy + col0 + cc;
      *reinterpret_cast<uint4*>(a.Y + o) = *reinterpret_cast<const uint4*>(&Th[rl * TS + cc]);
      if constexpr (SPLIT) *reinterpret_cast<uint4*>(a.Y_lo + o) = *reinterpret_cast<const uint4*>(&Tl[rl * TS + cc]);
    }
  } else {
    // ---- 4b. head partial: per row, sum over this tile's columns of act(acc + b) * w2
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
    if (tid < T::BM) {
      const int row = row0 + tid;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < T::WN; ++w) sum += hpart[w][tid];  // fixed order
      if (row < M) a.part[(size_t)ct * a.M + row] = sum;
    }
  }
  if (tr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ML_MARK(5);
  }
#undef ML_MARK
}

template <bool SPLIT, int SRC, int EPI>
__global__ void __launch_bounds__(256) mlp_layer_kernel(MlpLayerArgs a) {
  using T = MlTile<SPLIT>;
  __shared__ __attribute__((aligned(16))) uint16_t img[ML_LDS_BYTES / 2];
  __shared__ float hpart[4][128];
  // XCD-aware tile order (see the header)
  const int per = (a.tiles + 7) >> 3;
  const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (tile >= a.tiles) return;
  const int rt = tile / a.col_tiles, ct = tile - rt * a.col_tiles;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = rt * T::BM, col0 = ct * T::BN;
  if (row0 >= M) return;  // uniform per block, before any barrier
  switch (a.K >> 5) {  // k-steps of 32 (the host allows 64..512 in steps of 64)
    case 2: ml_body<SPLIT, SRC, EPI, 2>(a, img, hpart, row0, col0, ct, M); break;
    case 4: ml_body<SPLIT, SRC, EPI, 4>(a, img, hpart, row0, col0, ct, M); break;
    case 6: ml_body<SPLIT, SRC, EPI, 6>(a, img, hpart, row0, col0, ct, M); break;
    case 8: ml_body<SPLIT, SRC, EPI, 8>(a, img, hpart, row0, col0, ct, M); break;
    case 10: ml_body<SPLIT, SRC, EPI, 10>(a, img, hpart, row0, col0, ct, M); break;
    case 12: ml_body<SPLIT, SRC, EPI, 12>(a, img, hpart, row0, col0, ct, M); break;
    case 14: ml_body<SPLIT, SRC, EPI, 14>(a, img, hpart, row0, col0, ct, M); break;
    default: ml_body<SPLIT, SRC, EPI, 16>(a, img, hpart, row0, col0, ct, M); break;
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

int mlp_layer_tile_rows(int split) { return split ? MlTile<true>::BM : MlTile<false>::BM; }
int mlp_layer_tile_cols(int split) { return split ? MlTile<true>::BN : MlTile<false>::BN; }

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
