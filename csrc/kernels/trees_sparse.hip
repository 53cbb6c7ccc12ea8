// K2b tree_sparse: ONNX-ML TreeEnsemble on the pointer layout (csrc/runtime/trees.h Sparse) for
// what the complete-tree kernel (trees.hip) cannot take: depth > 12, very unbalanced trees
// (where the complete layout would be mostly padding) and MIN / MAX aggregates. Semantics:
// the CPU executor (csrc/runtime/trees.cpp eval_raw + post_transform).
//
// Block = 256 threads = 4 waves over 64 samples (lane = sample); the waves split the tree group,
// each lane keeps ILP traversals in flight so the dependent 16-B node loads (L2 hits for
// ensembles of a few MB) overlap. The block's X tile ([64][W+1] f32, W = largest feature id + 1)
// is staged in LDS when it fits, so the per-visit feature read is an LDS access. The waves'
// accumulators meet in LDS; one tree group finishes in place (aggregate, base, post transform),
// several write partials [G][rows][K] for tree_sparse_finish_kernel. MIN / MAX use +-inf as
// "no tree wrote this target" (the executor's untouched accumulator stays 0).
#include "common.h"
#include "launch.h"
#include "tree_post.h"

namespace igp {

constexpr int TS_ROWS = 64;
constexpr int TS_ILP = 4;
constexpr int TS_LEAF = 7;
constexpr int TS_MAX_STAGED_W = 256;

__device__ __forceinline__ float ts_init(int agg) {
  return agg == 2 ? INFINITY : agg == 3 ? -INFINITY : 0.f;
}

__device__ __forceinline__ float ts_combine(int agg, float acc, float v) {
  return agg == 2 ? fminf(acc, v) : agg == 3 ? fmaxf(acc, v) : acc + v;
}

__device__ __forceinline__ bool ts_true(float x, float thr, uint32_t meta) {
  const uint32_t mode = (meta >> 16) & 7u;
  bool c = mode == 0 ? (x <= thr) : mode == 1 ? (x < thr) : mode == 2 ? (x >= thr)
         : mode == 3 ? (x > thr) : mode == 4 ? (x == thr) : (x != thr);
  return c || (((meta >> 19) & 1u) && isnan(x));
}

template <int KT>
__device__ __forceinline__ void ts_finish(const TreeSparseArgs& a, const float* acc, int row) {
  float z[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (k >= a.k) break;
    float v = acc[k];
    if (a.aggregate >= 2 && isinf(v)) v = 0.f;
    if (a.aggregate == 1) v /= (float)a.n_trees;
    if (a.base) v += a.base[k];
    z[k] = v;
  }
  float* o = a.out + (size_t)row * a.n_out;
  if (a.binary_class >= 0) {
    tree_post_binary(a.post, a.binary_class, a.all_positive, z[0], o);
    return;
  }
  tree_post_inplace(a.post, a.k, z);
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (k >= a.k) break;
    o[k] = z[k];
  }
}

template <int KT, bool STAGED>
__global__ void __launch_bounds__(256) tree_sparse_kernel(TreeSparseArgs a, int trees_per_group, int feat_w,
                                                          float* partial) {
  extern __shared__ float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * TS_ROWS, g = blockIdx.y;
  const int row = row0 + lane;
  const bool live = row < a.n_rows;
  float* sx = smem;                                           // [64][feat_w + 1]
  float* red = smem + (STAGED ? TS_ROWS * (feat_w + 1) : 0);  // [4][64][KT]
  if constexpr (STAGED) {
    for (int e = tid; e < TS_ROWS * feat_w; e += 256) {
      const int r = e / feat_w, c = e - r * feat_w;
      sx[r * (feat_w + 1) + c] = row0 + r < a.n_rows ? a.X[(size_t)(row0 + r) * a.x_stride + c] : 0.f;
    }
    __syncthreads();
  }
  const float* xr = a.X + (size_t)(live ? row : 0) * a.x_stride;
  auto feature = [&](int f) -> float {
    if constexpr (STAGED) return sx[lane * (feat_w + 1) + f];
    else return xr[f];
  };
  float acc[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) acc[k] = ts_init(a.aggregate);
  const int t_begin = g * trees_per_group;
  const int t_end = min(a.n_trees, t_begin + trees_per_group);
  const int K = a.k;
  const int4* nodes = reinterpret_cast<const int4*>(a.nodes);
  for (int tb = t_begin + wave * TS_ILP; tb < t_end; tb += 4 * TS_ILP) {
    int cur[TS_ILP];
#pragma unroll
    for (int j = 0; j < TS_ILP; ++j) cur[j] = tb + j < t_end ? a.roots[tb + j] : -1;
    int leaf[TS_ILP];
#pragma unroll
    for (int j = 0; j < TS_ILP; ++j) leaf[j] = -1;
    // at most depth + 1 visits per tree (the host checked the trees are acyclic and bounded)
    for (int d = 0; d <= a.depth; ++d) {
      int4 nd[TS_ILP];
#pragma unroll
      for (int j = 0; j < TS_ILP; ++j) nd[j] = cur[j] >= 0 ? nodes[cur[j]] : make_int4(0, 0, 0, 0);
      bool more = false;
#pragma unroll
      for (int j = 0; j < TS_ILP; ++j) {
        if (cur[j] < 0) continue;
        const uint32_t meta = (uint32_t)nd[j].x;
        if (((meta >> 16) & 7u) == TS_LEAF) {
          leaf[j] = nd[j].z;
          cur[j] = -1;
          continue;
        }
        const float x = feature((int)(meta & 0xffffu));
        cur[j] = ts_true(x, __int_as_float(nd[j].y), meta) ? nd[j].z : nd[j].w;
        more = true;
      }
      if (!__any(more)) break;
    }
#pragma unroll
    for (int j = 0; j < TS_ILP; ++j) {
      if (leaf[j] < 0) continue;
      const float* w = a.leaf_w + (size_t)leaf[j] * K;
      const uint8_t* h = a.leaf_has + (size_t)leaf[j] * K;
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        if (k >= K) break;
        if (a.aggregate < 2 || h[k]) acc[k] = ts_combine(a.aggregate, acc[k], w[k]);
      }
    }
  }
  // the four waves' accumulators -> LDS -> one value per (row, target), waves in order
#pragma unroll
  for (int k = 0; k < KT; ++k) red[(wave * TS_ROWS + lane) * KT + k] = acc[k];
  __syncthreads();
  if (wave != 0 || !live) return;
  float s[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    float v = red[lane * KT + k];
#pragma unroll
    for (int w = 1; w < 4; ++w) v = ts_combine(a.aggregate, v, red[(w * TS_ROWS + lane) * KT + k]);
    s[k] = v;
  }
  if (partial) {
#pragma unroll
    for (int k = 0; k < KT; ++k)
      if (k < K) partial[((size_t)g * a.n_rows + row) * K + k] = s[k];
    return;
  }
  ts_finish<KT>(a, s, row);
}

template <int KT>
__global__ void tree_sparse_finish_kernel(TreeSparseArgs a, const float* partial, int groups) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.n_rows) return;
  float s[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (k >= a.k) break;
    float v = ts_init(a.aggregate);
    for (int g = 0; g < groups; ++g) v = ts_combine(a.aggregate, v, partial[((size_t)g * a.n_rows + row) * a.k + k]);
    s[k] = v;
  }
  ts_finish<KT>(a, s, row);
}

template <int KT>
static void launch_sparse_k(const TreeSparseArgs& a, int groups, float* partial, hipStream_t st) {
  const int tpg = (a.n_trees + groups - 1) / groups;
  const int feat_w = a.feat_w;
  const bool staged = feat_w <= TS_MAX_STAGED_W;
  const size_t red_bytes = (size_t)4 * TS_ROWS * KT * 4;
  const size_t x_bytes = staged ? (size_t)TS_ROWS * (feat_w + 1) * 4 : 0;
  dim3 grid((a.n_rows + TS_ROWS - 1) / TS_ROWS, groups);
  float* p = groups > 1 ? partial : nullptr;
  if (staged)
    IGP_LAUNCH((tree_sparse_kernel<KT, true>), grid, dim3(256), x_bytes + red_bytes, st, a, tpg, feat_w, p);
  else
    IGP_LAUNCH((tree_sparse_kernel<KT, false>), grid, dim3(256), red_bytes, st, a, tpg, feat_w, p);
  if (groups > 1)
    IGP_LAUNCH(tree_sparse_finish_kernel<KT>, dim3((a.n_rows + 255) / 256), dim3(256), 0, st, a, partial,
                       groups);
}

// partial: [groups][n_rows][K] f32 scratch when groups > 1
void launch_tree_sparse(const TreeSparseArgs& a, int groups, float* partial, hipStream_t st) {
  const int k = a.k;
  if (k <= 1) launch_sparse_k<1>(a, groups, partial, st);
  else if (k <= 2) launch_sparse_k<2>(a, groups, partial, st);
  else if (k <= 4) launch_sparse_k<4>(a, groups, partial, st);
  else if (k <= 8) launch_sparse_k<8>(a, groups, partial, st);
  else if (k <= 16) launch_sparse_k<16>(a, groups, partial, st);
  else if (k <= 32) launch_sparse_k<32>(a, groups, partial, st);
  else launch_sparse_k<64>(a, groups, partial, st);
}

}  // namespace igp
