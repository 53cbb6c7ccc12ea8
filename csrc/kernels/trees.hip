// K2 tree_ensemble: ONNX-ML TreeEnsemble{Classifier,Regressor} on the complete-tree layout
// (csrc/runtime/trees.h). Semantics: CPU executor (csrc/runtime/trees.cpp).
//
// Block = 256 threads = 4 waves, 64 samples. The block's X tile and its tree group's node table
// (8 B/node) are staged in LDS. The tile is feature-major, [F][64]: lane r reads sample r's
// feature at [f][r], bank r whatever feature its traversal reached, so a wave's reads never
// conflict (the row-major [64][F+1] tile put lane r's read in bank (r + f) % 32). Traversal: lane = sample, the four waves split the group's
// trees, each lane keeps 4 traversals in flight (independent LDS chains hide ds_read latency).
//  * K < 16: each lane accumulates its leaf values directly (4-32 B per visit).
//  * K >= 16 (leaf vectors, e.g. stacked GBDT->MLP embeddings): traversal only records leaf
//    indices in LDS; a second phase puts lanes on the K targets so that each wave-load reads
//    whole contiguous leaf rows (coalesced) instead of 64 scattered 16-B pieces.
// Several tree groups per sample tile (small batches) write partial sums to a slab; a
// finisher (or the consuming mlp_head kernel) adds base values and the post transform.
#include "common.h"
#include "ensemble.h"
#include "head_f32.h"
#include "launch.h"
#include "tree_post.h"

namespace igp {

constexpr int TR_ROWS = 64;
constexpr int TR_ILP = 4;
typedef unsigned int tr_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int tree_step(int i, float x, float2 nd) {
  const uint32_t m = __float_as_uint(nd.y);
  const int mode = (m >> 16) & 7;
  const float t = nd.x;
  bool c = mode == 0 ? (x <= t) : mode == 1 ? (x < t) : mode == 2 ? (x >= t)
         : mode == 3 ? (x > t) : mode == 4 ? (x == t) : (x != t);
  c = c || (((m >> 19) & 1u) && isnan(x));
  return 2 * i + (c ? 1 : 2);
}

__device__ __forceinline__ void post_row(const TreeArgs& a, const float* s, float* o, int K) {
  if (a.binary_class >= 0) {
    float v = s[0];
    if (a.average) v /= (float)a.n_trees;
    if (a.base) v += a.base[0];
    tree_post_binary(a.post, a.binary_class, a.all_positive, v, o);
    return;
  }
  for (int k = 0; k < K; ++k) {
    float v = s[k];
    if (a.average) v /= (float)a.n_trees;
    if (a.base) v += a.base[k];
    o[k] = v;
  }
  tree_post_inplace(a.post, K, o);
}

// element-wise post transforms (NONE / LOGISTIC / PROBIT); the softmax family is row-wise
__device__ __forceinline__ float post_elem(int post, float v) {
  if (post == TP_LOGISTIC) return 1.f / (1.f + expf(-v));
  if (post == TP_PROBIT) return 1.41421356f * tp_erfinv(2 * v - 1);
  return v;
}
__host__ __device__ __forceinline__ bool post_rowwise(const TreeArgs& a) {
  return a.post == TP_SOFTMAX || a.post == TP_SOFTMAX_ZERO || a.binary_class >= 0;
}

template <bool LEQ>
__device__ __forceinline__ int tree_next(int i, float x, float2 nd) {
  if constexpr (LEQ) {
    const bool c = x <= nd.x || (((__float_as_uint(nd.y) >> 19) & 1u) && isnan(x));
    return 2 * i + (c ? 1 : 2);
  }
  else return tree_step(i, x, nd);
}

// One workgroup's share of the ensemble: its 64-row tile x its tree group (blockIdx.y).
// WT: the group partials are stored write-through (sc1) for an in-launch consumer
// (tree_head_kernel); otherwise plain stores for the next kernel.
template <int K, bool LEQ, bool WT>
__device__ __forceinline__ void tree_block(const TreeArgs& a, int trees_per_group, int feat_w, int nodes_in_lds,
                                           float* partial, char* smem) {
  constexpr bool TWO_PHASE = K >= 16;
  float* sx = reinterpret_cast<float*>(smem);                       // [feat_w][64]
  const size_t x_bytes = ((size_t)TR_ROWS * feat_w * 4 + 15) & ~size_t(15);
  const size_t red_b = TWO_PHASE ? (size_t)TR_ROWS * K * 4 : (size_t)5 * TR_ROWS * K * 4;
  const size_t base_b = x_bytes > red_b ? x_bytes : red_b;
  float2* sn = reinterpret_cast<float2*>(smem + base_b);             // group node table
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * TR_ROWS;
  const int g = blockIdx.y;
  const int t0 = g * trees_per_group;
  const int t1 = min(a.n_trees, t0 + trees_per_group);
  const int nt = t1 - t0;
  const int n_int = (1 << a.depth) - 1;
  const int n_leaf = 1 << a.depth;
  const size_t node_b = ((size_t)trees_per_group * n_int * 8 + 15) & ~size_t(15);
  uint16_t* sleaf = reinterpret_cast<uint16_t*>(smem + base_b + (nodes_in_lds ? node_b : 0));
  // phase trace: wave 0 of blocks x = 0, 64 of groups 0..3: [sample][phase] wall_clock64
  const int tsmp = g * 2 + (blockIdx.x >> 6);
  int64_t* const trow = (a.trace && tid == 0 && (blockIdx.x & 63) == 0 && tsmp < 8) ? a.trace + tsmp * 8 : nullptr;
#define TR_MARK(k) \
  if (trow) trow[k] = (int64_t)wall_clock64()
  TR_MARK(0);

  // stage the X tile and the group's node table: the node table's first chunk is loaded with
  // the whole X tile in flight (one memory round trip), then both are stored. X is read one row
  // per lane (lane r = sample r, its row's 16-B chunks cg, cg + 4, ...): the feature-major
  // stores of a wave then hit 64 different banks as well
  const float2* gn = a.nodes + (size_t)t0 * n_int;
  {
    constexpr int UN = 32, UC = 8;
    const int ntot = nodes_in_lds ? nt * n_int : 0;
    float2 w[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int e = u * 256 + tid;
      w[u] = e < ntot ? gn[e] : make_float2(0.f, 0.f);
    }
    const int r = lane, row = row0 + r;
    const bool live = row < a.n_rows;
    const float* xr = a.X + (size_t)(live ? row : 0) * a.x_stride;
    if ((feat_w & 3) == 0 && (a.x_stride & 3) == 0) {  // 16-byte loads (the usual case)
      const int f4 = feat_w >> 2;
      for (int c0 = wave; c0 < f4; c0 += 4 * UC) {
        float4 q[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u) {
          const int ch = c0 + 4 * u;
          q[u] = live && ch < f4 ? *reinterpret_cast<const float4*>(xr + 4 * ch) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UC; ++u) {
          const int ch = c0 + 4 * u;
          if (ch < f4) {
            float* d = sx + (4 * ch) * TR_ROWS + r;
            d[0] = q[u].x; d[TR_ROWS] = q[u].y; d[2 * TR_ROWS] = q[u].z; d[3 * TR_ROWS] = q[u].w;
          }
        }
      }
    } else {
      for (int c = wave; c < feat_w; c += 4) sx[c * TR_ROWS + r] = live ? xr[c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int e = u * 256 + tid;
      if (e < ntot) sn[e] = w[u];
    }
    for (int e = UN * 256 + tid; e < ntot; e += 256) sn[e] = gn[e];
  }
  __syncthreads();
  TR_MARK(1);

  float acc[TWO_PHASE ? 1 : K];
#pragma unroll
  for (int k = 0; k < (TWO_PHASE ? 1 : K); ++k) acc[k] = 0.f;

  // traversal: lane = sample, TR_ILP trees per wave in flight. The trees of a wave are uniform
  // (scalar tree index), so a missing tree past the group end is a scalar condition, not an
  // exec-masked branch; each level issues the TR_ILP node reads, then the TR_ILP feature reads
  // (the node table from LDS - ds_read, not a flat load through the vector memory path - and
  // the X tile, conflict-free), then the TR_ILP compares
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  auto traverse = [&](const float2* nodes) {
    for (int tb = t0 + wv; tb < t1; tb += 4 * TR_ILP) {
      int idx[TR_ILP], nb[TR_ILP];
#pragma unroll
      for (int q = 0; q < TR_ILP; ++q) {
        const int tq = tb + 4 * q;
        nb[q] = (tq < t1 ? tq - t0 : 0) * n_int;
        idx[q] = 0;
      }
      for (int d = 0; d < a.depth; ++d) {
        float2 nd[TR_ILP];
        float xv[TR_ILP];
#pragma unroll
        for (int q = 0; q < TR_ILP; ++q) nd[q] = nodes[nb[q] + idx[q]];
#pragma unroll
        for (int q = 0; q < TR_ILP; ++q) xv[q] = sx[(__float_as_uint(nd[q].y) & 0xffff) * TR_ROWS + lane];
#pragma unroll
        for (int q = 0; q < TR_ILP; ++q) idx[q] = tree_next<LEQ>(idx[q], xv[q], nd[q]);
      }
#pragma unroll
      for (int q = 0; q < TR_ILP; ++q) {
        const int tq = tb + 4 * q;
        if (tq >= t1) break;
        if constexpr (TWO_PHASE) {
          sleaf[lane * nt + (tq - t0)] = (uint16_t)(idx[q] - n_int);
        } else {
          const float* lf = a.leaves + ((size_t)tq * n_leaf + (idx[q] - n_int)) * K;
          if constexpr (K % 4 == 0) {
#pragma unroll
            for (int k = 0; k < K; k += 4) {
              const float4 v = *reinterpret_cast<const float4*>(lf + k);
              acc[k] += v.x; acc[k + 1] += v.y; acc[k + 2] += v.z; acc[k + 3] += v.w;
            }
          } else {
#pragma unroll
            for (int k = 0; k < K; ++k) acc[k] += lf[k];
          }
        }
      }
    }
  };
  if (nodes_in_lds) traverse(sn);
  else traverse(gn);
  TR_MARK(2);
  __syncthreads();
  TR_MARK(3);
  float* red = sx;  // reuse the X tile region: [5][64][K] (K < 16) or [64][K] (two-phase)
  if constexpr (TWO_PHASE) {
    // phase 2: lanes over 16-B column chunks of the targets, K/4 lanes read one whole leaf row
    // (coalesced). 16-B loads: a quarter of the load instructions of one-target-per-lane, so
    // the same bytes need a quarter of the dependent L2 round trips (the step count, not
    // bandwidth, sets the time: the leaves are L2 hits)
    constexpr int LPR = K / 4;          // lanes per row
    constexpr int SPP = 256 / LPR;      // samples per pass
    const int k4 = tid % LPR, sp = tid / LPR;
    const bool rowwise = !partial && post_rowwise(a);
    // each thread owns columns 4 k4 .. 4 k4 + 3 of rows sp, sp + SPP, ...: its rows advance
    // through the trees together, RPT x TU independent loads in flight per step. Per row the
    // trees are still summed in order t0, t0+1, ... (same sums as a scalar loop)
    constexpr int RPT = TR_ROWS / SPP;  // rows per thread
    float4 v[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    // leaf loads through a buffer resource: per-lane offset (leaf, k4) in a VGPR, the tree's
    // base (uniform) in an SGPR offset
    const float* lbase = a.leaves + (size_t)t0 * n_leaf * K;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lbase), 0, nt * n_leaf * K * 4, 0x00020000);
    const int tstride = n_leaf * K * 4;  // bytes per tree
    constexpr int TU = RPT >= 4 ? 4 : 8;  // trees per step
    auto ld = [&](int l, int t) {
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (l * K + 4 * k4) * 4, t * tstride, 0));
    };
    int t = 0;
    for (; t + TU <= nt; t += TU) {
      float4 p[RPT][TU];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const uint16_t* li = sleaf + (sp + j * SPP) * nt + t;
#pragma unroll
        for (int u = 0; u < TU; ++u) p[j][u] = ld((int)li[u], t + u);
      }
#pragma unroll
      for (int j = 0; j < RPT; ++j)
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          v[j].x += p[j][u].x; v[j].y += p[j][u].y; v[j].z += p[j][u].z; v[j].w += p[j][u].w;
        }
    }
    for (; t < nt; ++t) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const float4 q = ld((int)sleaf[(sp + j * SPP) * nt + t], t);
        v[j].x += q.x; v[j].y += q.y; v[j].z += q.z; v[j].w += q.w;
      }
    }
    TR_MARK(4);
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int r = sp + j * SPP;
      const int row = row0 + r;
      if (row >= a.n_rows) continue;
      if (partial) {
        if constexpr (WT) {
          // 16-B write-through store: the line leaves this XCD's L2, so the tile's last-arriving
          // group block (any XCD, behind its agent acquire) reads it fresh
          const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(partial, 0, 0x7fffffff, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(tr_u32x4, v[j]), prs,
                                                 (int)((((size_t)g * a.n_rows + row) * K + 4 * k4) * 4), 0, 16);
        } else {
          *reinterpret_cast<float4*>(partial + ((size_t)g * a.n_rows + row) * K + 4 * k4) = v[j];
        }
      } else if (rowwise) {
        *reinterpret_cast<float4*>(red + r * K + 4 * k4) = v[j];
      } else {
        float vv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int k = 4 * k4 + c;
          if (a.average) vv[c] /= (float)a.n_trees;
          if (a.base) vv[c] += a.base[k];
          a.out[(size_t)row * a.n_out + k] = post_elem(a.post, vv[c]);
        }
      }
    }
    TR_MARK(5);
    if (!rowwise) return;
    __syncthreads();
    for (int r = tid; r < TR_ROWS; r += 256) {
      const int row = row0 + r;
      if (row < a.n_rows) post_row(a, red + r * K, a.out + (size_t)row * a.n_out, K);
    }
    return;
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) red[(wave * TR_ROWS + lane) * K + k] = acc[k];
    __syncthreads();
    for (int e = tid; e < TR_ROWS * K; e += 256) {
      const int r = e / K, k = e - r * K;
      const int row = row0 + r;
      const float v = red[(0 * TR_ROWS + r) * K + k] + red[(1 * TR_ROWS + r) * K + k] +
                      red[(2 * TR_ROWS + r) * K + k] + red[(3 * TR_ROWS + r) * K + k];
      if (row >= a.n_rows) continue;
      if (partial) partial[((size_t)g * a.n_rows + row) * K + k] = v;
      else red[(4 * TR_ROWS + r) * K + k] = v;
    }
    if (partial) return;
    __syncthreads();
    for (int r = tid; r < TR_ROWS; r += 256) {
      const int row = row0 + r;
      if (row < a.n_rows) post_row(a, red + (4 * TR_ROWS + r) * K, a.out + (size_t)row * a.n_out, K);
    }
  }
}

#undef TR_MARK

template <int K, bool LEQ>
__global__ void __launch_bounds__(256) tree_kernel(TreeArgs a, int trees_per_group, int feat_w,
                                                   int nodes_in_lds, float* partial) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tree_block<K, LEQ, false>(a, trees_per_group, feat_w, nodes_in_lds, partial, smem);
}

// ---------------------------------------------------------------------------------------------
// cfg3 stacked model in one launch: TreeEnsemble (K = 32 leaf vectors, grouped) -> f32 MLP head
// -> K5 ensemble. Every group block stores its [64][32] partial write-through and takes a ticket
// on its tile's counter; the tile's last arriver (whichever XCD it runs on) runs one agent-scope
// acquire, reduces the group partials in group order (+ base, / T: the same sums as
// head_a_f32), and runs the head of the reference-precision kernel (mlp_head_f32_fast_kernel:
// the same MFMA sequence per 16-row fragment, the same hidden-chunk and wave order, so Y is
// bit-identical) and the fused K5 on its 64 rows. Removes the head launch and its hand-off;
// the partial slab is read once, by one block per tile.
constexpr int TH_LR = 32 + 4;  // LDS row stride of the A tile and W1 (floats)

template <bool LEQ, int ACT>
__global__ void __launch_bounds__(256) tree_head_kernel(TreeArgs a, HeadArgs h, int trees_per_group, int feat_w,
                                                        int nodes_in_lds, float* partial, int groups,
                                                        unsigned int* tile_cnt) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tree_block<32, LEQ, true>(a, trees_per_group, feat_w, nodes_in_lds, partial, smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n1p = (h.N1 + 63) & ~63;
  float* sA = reinterpret_cast<float*>(smem);  // [64][TH_LR]
  float* sW = sA + TR_ROWS * TH_LR;             // [n1p][TH_LR]
  float* sred = sW + n1p * TH_LR;               // [4][64]
  float* sb1 = sred + 4 * TR_ROWS;              // [n1p]
  float* sw2 = sb1 + n1p;                       // [n1p]
  unsigned int* ecnt = reinterpret_cast<unsigned int*>(sw2 + n1p);  // [MET_N]
  int* sflag = reinterpret_cast<int*>(ecnt + MET_N);
  // publish: every wave's partial stores complete, then one ticket per block
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned int old = __hip_atomic_fetch_add(&tile_cnt[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned int)(groups - 1);
    if (last) __hip_atomic_store(&tile_cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sflag[0] = last;
  }
  __syncthreads();
  if (!sflag[0]) return;
  const int M = h.m_ptr ? min(*h.m_ptr, h.M) : h.M;
  const int row0 = blockIdx.x * TR_ROWS;
  const bool fm = h.fuse_ens && h.ens.metrics;
  if (row0 >= M) {  // no live row in this tile: the fused ensemble still writes the inert rows
    if (h.fuse_ens)
      for (int r = row0 + tid; r < min(row0 + TR_ROWS, h.ens.n_rows); r += 256) ensemble_row(h.ens, r, true, 0.f, nullptr);
    return;
  }
  // weights first (read-only: no acquire needed), in flight across the acquire
  const float* const W1 = reinterpret_cast<const float*>(h.W1);
  constexpr int KQ = 8;  // float4 chunks per 32-float W1 row
  const int total = n1p * KQ;
  float4 wv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int ch = u * 256 + tid;
    wv[u] = ch < total ? *reinterpret_cast<const float4*>(W1 + (size_t)(ch / KQ) * 32 + (ch % KQ) * 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (fm)
    for (int i = tid; i < MET_N; i += 256) ecnt[i] = 0;
  __syncthreads();
  // A tile: sum_g partial[g][row][k] in group order (+ base, / T), 2 x 16-B chunks per thread;
  // up to 8 groups' loads in flight per round (the weights go to LDS under the first round)
  const int gl = groups - 1;
  float fa[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int g0 = 0; g0 < groups; g0 += 8) {
    float4 p[2][8];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = c * 256 + tid, r = ch >> 3, kc = (ch & 7) * 4;
#pragma unroll
      for (int g = 0; g < 8; ++g)
        p[c][g] = *reinterpret_cast<const float4*>(
            partial + ((size_t)min(g0 + g, gl) * a.n_rows + min(row0 + r, a.n_rows - 1)) * 32 + kc);
    }
    if (g0 == 0) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int ch = u * 256 + tid;
        if (ch < total) *reinterpret_cast<float4*>(&sW[(ch / KQ) * TH_LR + (ch % KQ) * 4]) = wv[u];
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int g = 0; g < 8; ++g)
        if (g0 + g <= gl) {
          fa[c][0] += p[c][g].x; fa[c][1] += p[c][g].y; fa[c][2] += p[c][g].z; fa[c][3] += p[c][g].w;
        }
  }
  for (int ch = 8 * 256 + tid; ch < total; ch += 256)
    *reinterpret_cast<float4*>(&sW[(ch / KQ) * TH_LR + (ch % KQ) * 4]) =
        *reinterpret_cast<const float4*>(W1 + (size_t)(ch / KQ) * 32 + (ch % KQ) * 4);
  for (int n = tid; n < n1p; n += 256) {
    sb1[n] = (n < h.N1 && h.b1) ? h.b1[n] : 0.f;
    sw2[n] = n < h.N1 ? h.w2[n] : 0.f;
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = c * 256 + tid, r = ch >> 3, kc = (ch & 7) * 4;
    float f[4] = {0.f, 0.f, 0.f, 0.f};
    if (row0 + r < M) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] = fa[c][j];
        if (h.p_average) f[j] /= (float)h.p_ntrees;
        f[j] += h.pbase ? h.pbase[kc + j] : 0.f;
      }
    }
    *reinterpret_cast<float4*>(&sA[r * TH_LR + kc]) = make_float4(f[0], f[1], f[2], f[3]);
  }
  __syncthreads();
  // 4 row fragments of 16 x (4 waves x 16 hidden columns per 64-column chunk)
  float4 av[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      av[i][s] = *reinterpret_cast<const float4*>(&sA[(i * 16 + (lane & 15)) * TH_LR + s * 16 + 4 * (lane >> 4)]);
  float part[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) part[i][q] = 0.f;
  for (int c0 = 0; c0 < h.N1; c0 += 64) {
    const int n = c0 + wave * 16 + (lane & 15);
    float4 bv[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) bv[s] = *reinterpret_cast<const float4*>(&sW[n * TH_LR + s * 16 + 4 * (lane >> 4)]);
    const float b1 = sb1[n];
    const float w2 = sw2[n];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) acc = mfma4_f32(av[i][s], bv[s], acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) part[i][q] += act_fn(acc[q] + b1, ACT) * w2;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = part[i][q];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      part[i][q] = v;
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) sred[wave * TR_ROWS + i * 16 + (lane >> 4) * 4 + q] = part[i][q];
  }
  __syncthreads();
  if (tid < TR_ROWS) {
    const int row = row0 + tid;
    float y = 0.f;
    if (row < M) {
      const float v = sred[tid] + sred[TR_ROWS + tid] + sred[2 * TR_ROWS + tid] + sred[3 * TR_ROWS + tid];
      y = act_fn(v + h.b2, h.act2);
      h.Y[(size_t)row * h.ldy] = y;
    }
    if (h.fuse_ens && row < h.ens.n_rows) ensemble_row(h.ens, row, true, y, fm ? ecnt : nullptr);
  }
  if (fm) {
    __syncthreads();
    ensemble_metrics_flush(h.ens, ecnt, tid, 256);
  }
}

__global__ void tree_finish_kernel(TreeArgs a, const float* partial, int groups) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.n_rows) return;
  const int K = a.k;
  float s[64];
  for (int k = 0; k < K; ++k) {
    float v = 0.f;
    for (int g = 0; g < groups; ++g) v += partial[((size_t)g * a.n_rows + row) * K + k];
    s[k] = v;
  }
  post_row(a, s, a.out + (size_t)row * a.n_out, K);
}

// the finish kernel with the scorer's K5 ensemble in its epilogue (cfg 2: a grouped tree
// classifier is the whole model): the row's ensemble reads the model column this thread just
// wrote, so the standalone ensemble launch (and its queue slot) goes away. Rows past n_rows up to
// ens.n_rows get their (zero) results as in ensemble_kernel.
__global__ void __launch_bounds__(256) tree_finish_ens_kernel(TreeArgs a, const float* partial, int groups) {
  __shared__ unsigned int cnt[MET_N];
  const int tid = threadIdx.x;
  const bool fm = a.ens.metrics != nullptr;
  if (fm) {
    for (int i = tid; i < MET_N; i += 256) cnt[i] = 0;
    __syncthreads();
  }
  const int row = blockIdx.x * 256 + tid;
  if (row < a.n_rows) {
    const int K = a.k;
    float s[64];
    for (int k = 0; k < K; ++k) {
      float v = 0.f;
      for (int g = 0; g < groups; ++g) v += partial[((size_t)g * a.n_rows + row) * K + k];
      s[k] = v;
    }
    post_row(a, s, a.out + (size_t)row * a.n_out, K);
  }
  if (row < a.ens.n_rows) ensemble_row(a.ens, row, false, 0.f, fm ? cnt : nullptr);
  if (fm) {
    __syncthreads();
    ensemble_metrics_flush(a.ens, cnt, tid, 256);
  }
}

// regressor / multi-output without a row-wise post transform: one thread per (row, target)
__global__ void tree_finish_elem_kernel(TreeArgs a, const float* partial, int groups) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = a.k;
  if (e >= a.n_rows * K) return;
  const int k = e % K;
  float v = 0.f;
  for (int g = 0; g < groups; ++g) v += partial[(size_t)g * a.n_rows * K + e];
  if (a.average) v /= (float)a.n_trees;
  if (a.base) v += a.base[k];
  a.out[e] = post_elem(a.post, v);  // n_out == K
}

template <int K, bool LEQ>
static void launch_kl(const TreeArgs& a, int groups, float* partial, int no_finish, hipStream_t st) {
  const int tpg = (a.n_trees + groups - 1) / groups;
  const int feat_w = a.x_stride;
  const int n_int = (1 << a.depth) - 1;
  const size_t x_bytes = ((size_t)TR_ROWS * feat_w * 4 + 15) & ~size_t(15);
  const size_t red_bytes = K >= 16 ? (size_t)TR_ROWS * K * 4 : (size_t)5 * TR_ROWS * K * 4;
  const size_t node_bytes = ((size_t)tpg * n_int * 8 + 15) & ~size_t(15);
  const size_t leaf_bytes = K >= 16 ? (size_t)TR_ROWS * tpg * 2 : 0;
  const size_t base = x_bytes > red_bytes ? x_bytes : red_bytes;
  int in_lds = (base + node_bytes + leaf_bytes) <= 96 * 1024;  // keep >= 1 block/CU with headroom
  const size_t lds = base + (in_lds ? node_bytes : 0) + leaf_bytes;
  dim3 grid((a.n_rows + TR_ROWS - 1) / TR_ROWS, groups);
  IGP_LAUNCH((tree_kernel<K, LEQ>), grid, dim3(256), lds, st, a, tpg, feat_w, in_lds,
                     groups > 1 ? partial : nullptr);
  if (groups > 1 && !no_finish) {
    if (a.fuse_ens) {
      const int rows = a.n_rows > a.ens.n_rows ? a.n_rows : a.ens.n_rows;
      IGP_LAUNCH(tree_finish_ens_kernel, dim3((rows + 255) / 256), dim3(256), 0, st, a, partial, groups);
    } else if (!post_rowwise(a) && a.n_out == K)
      IGP_LAUNCH(tree_finish_elem_kernel, dim3((a.n_rows * K + 255) / 256), dim3(256), 0, st, a,
                         partial, groups);
    else
      IGP_LAUNCH(tree_finish_kernel, dim3((a.n_rows + 255) / 256), dim3(256), 0, st, a, partial, groups);
  }
}

template <int K>
static void launch_k(const TreeArgs& a, int groups, float* partial, int no_finish, hipStream_t st) {
  if (a.all_leq) launch_kl<K, true>(a, groups, partial, no_finish, st);
  else launch_kl<K, false>(a, groups, partial, no_finish, st);
}
// partial scratch: [groups][n_rows][K] f32, provided by the caller when groups > 1.
// no_finish: leave the partial slab for a consumer that reduces it (mlp_head).
void launch_tree_ensemble_grouped(const TreeArgs& a, int groups, float* partial, hipStream_t st) {
  const int nf = a.no_finish;
  switch (a.k) {
    case 1: launch_k<1>(a, groups, partial, nf, st); break;
    case 2: launch_k<2>(a, groups, partial, nf, st); break;
    case 4: launch_k<4>(a, groups, partial, nf, st); break;
    case 8: launch_k<8>(a, groups, partial, nf, st); break;
    case 16: launch_k<16>(a, groups, partial, nf, st); break;
    case 32: launch_k<32>(a, groups, partial, nf, st); break;
    case 64: launch_k<64>(a, groups, partial, nf, st); break;
    default: break;  // host validates K before launch
  }
}

void launch_tree_ensemble(const TreeArgs& a, hipStream_t st) { launch_tree_ensemble_grouped(a, 1, nullptr, st); }

bool tree_head_supported(const TreeArgs& a, const HeadArgs& h, int groups) {
  return a.k == 32 && groups > 1 && groups <= 16 && a.post == 0 && a.binary_class < 0 && h.w1_f32 && h.k_pad == 32 &&
         h.K == 32 && h.N1 > 0 && h.N1 <= 512 && h.act1 >= 0 && h.act1 <= 3 && h.M == a.n_rows && !h.trace;
}

void launch_tree_head(const TreeArgs& a, const HeadArgs& h, int groups, float* partial, unsigned int* tile_cnt,
                      hipStream_t st) {
  const int tpg = (a.n_trees + groups - 1) / groups;
  const int feat_w = a.x_stride;
  const int n_int = (1 << a.depth) - 1;
  const size_t x_bytes = ((size_t)TR_ROWS * feat_w * 4 + 15) & ~size_t(15);
  const size_t red_bytes = (size_t)TR_ROWS * 32 * 4;
  const size_t node_bytes = ((size_t)tpg * n_int * 8 + 15) & ~size_t(15);
  const size_t leaf_bytes = (size_t)TR_ROWS * tpg * 2;
  const size_t base = x_bytes > red_bytes ? x_bytes : red_bytes;
  const int in_lds = (base + node_bytes + leaf_bytes) <= 96 * 1024;
  const size_t tree_lds = base + (in_lds ? node_bytes : 0) + leaf_bytes;
  const size_t n1p = (size_t)((h.N1 + 63) & ~63);
  const size_t head_lds = ((size_t)TR_ROWS + n1p) * TH_LR * 4 + 4 * TR_ROWS * 4 + 2 * n1p * 4 + MET_N * 4 + 16;
  const size_t lds = tree_lds > head_lds ? tree_lds : head_lds;
  dim3 grid((a.n_rows + TR_ROWS - 1) / TR_ROWS, groups);
#define TH_CASE(L, ACT) \
  if (a.all_leq == L && h.act1 == ACT) { \
    IGP_LAUNCH((tree_head_kernel<L, ACT>), grid, dim3(256), lds, st, a, h, tpg, feat_w, in_lds, partial, groups, tile_cnt); \
    return; \
  }
  TH_CASE(true, 0) TH_CASE(true, 1) TH_CASE(true, 2) TH_CASE(true, 3)
  TH_CASE(false, 0) TH_CASE(false, 1) TH_CASE(false, 2) TH_CASE(false, 3)
#undef TH_CASE
}

}  // namespace igp
