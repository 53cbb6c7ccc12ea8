// K3 dense layers on the CDNA4 matrix cores: Y[M,N] = act(X[M,K] . W^T + b).
//
// W is stored bf16 [N_pad][K_pad] (each output column's weights contiguous in K), so both
// MFMA operand fragments are 16-byte contiguous LDS reads (mfma_f32_16x16x32_bf16:
// lane l holds A[l&15][8(l>>4)..+8] and B[8(l>>4)..+8][l&15]). X may be f32 (cast to bf16
// while staging, fusing the producer's dtype conversion) or bf16; accumulation is f32;
// bias + activation are fused into the epilogue. 4 waves in a 2x2 arrangement, BK = 64,
// two LDS buffers: tile k+1 is loaded to registers while tile k's MFMAs run.
#include "common.h"
#include "ensemble.h"
#include "head_f32.h"
#include "launch.h"

namespace igp {

typedef __attribute__((ext_vector_type(8))) short bf16x8;

constexpr int G_BK = 64;
constexpr int G_PAD = 8;  // bf16 elements of row padding (144-byte rows)

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

template <int BM, int BN>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a) {
  constexpr int LDS_ROW = G_BK + G_PAD;
  constexpr int FM = BM / 32;  // fragments per wave along M (wave covers BM/2 rows)
  constexpr int FN = BN / 32;
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][BN * LDS_ROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = blockIdx.y * BM;
  const int col0 = blockIdx.x * BN;
  if (row0 >= M) return;
  const uint16_t* const W = reinterpret_cast<const uint16_t*>(a.W);
  const int K = a.K;
  const int k_pad = a.ldw;
  const int n_kt = (K + G_BK - 1) / G_BK;

  // staging: A tile BM x 64 -> BM*8 chunks of 8 elements; B tile BN x 64 -> BN*8 chunks
  constexpr int A_CHUNKS = BM * G_BK / 8 / 256;
  constexpr int B_CHUNKS = BN * G_BK / 8 / 256;
  uint4 ra[A_CHUNKS], rb[B_CHUNKS];

  auto load_tile = [&](int kt) {
    const int k0 = kt * G_BK;
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      const int r = ch >> 3, kc = (ch & 7) * 8;
      const int row = row0 + r, k = k0 + kc;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < M) {
        if (a.x_bf16) {
          const uint16_t* src = reinterpret_cast<const uint16_t*>(a.X) + (size_t)row * a.ldx + k;
          if (k + 8 <= K) {
            v = *reinterpret_cast<const uint4*>(src);
          } else {
            uint16_t t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] = (k + j < K) ? src[j] : 0;
            v = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
          }
        } else {
          const float* src = reinterpret_cast<const float*>(a.X) + (size_t)row * a.ldx + k;
          float f[8];
          if (k + 8 <= K && ((a.ldx & 3) == 0)) {
            const float4 p = *reinterpret_cast<const float4*>(src);
            const float4 q = *reinterpret_cast<const float4*>(src + 4);
            f[0] = p.x; f[1] = p.y; f[2] = p.z; f[3] = p.w; f[4] = q.x; f[5] = q.y; f[6] = q.z; f[7] = q.w;
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = (k + j < K) ? src[j] : 0.f;
          }
          v = make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                         pack_bf16x2(f[6], f[7]));
        }
      }
      ra[c] = v;
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      const int r = ch >> 3, kc = (ch & 7) * 8;
      const int n = col0 + r, k = k0 + kc;
      // W is zero padded to [N_pad][K_pad] with N_pad a multiple of 128, K_pad of 64
      rb[c] = (k < k_pad) ? *reinterpret_cast<const uint4*>(W + (size_t)n * k_pad + k) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      *reinterpret_cast<uint4*>(&sA[buf][(ch >> 3) * LDS_ROW + (ch & 7) * 8]) = ra[c];
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      *reinterpret_cast<uint4*>(&sB[buf][(ch >> 3) * LDS_ROW + (ch & 7) * 8]) = rb[c];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < n_kt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < n_kt) load_tile(kt + 1);  // global loads in flight under the MFMAs
#pragma unroll
    for (int kk = 0; kk < G_BK / 32; ++kk) {
      bf16x8 fa[FM], fb[FN];
      const int kof = kk * 32 + 8 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * (BM / 2) + i * 16 + (lane & 15);
        fa[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][r * LDS_ROW + kof]);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * (BN / 2) + j * 16 + (lane & 15);
        fb[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][r * LDS_ROW + kof]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < n_kt) {
      store_tile(cur ^ 1);
    }
    __syncthreads();
  }

  // epilogue: bias + activation, f32 or bf16 stores
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = col0 + wn * (BN / 2) + j * 16 + (lane & 15);
      if (col >= a.N) continue;
      const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = row0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + q;
        if (row >= M) continue;
        const float v = act_fn(acc[i][j][q] + b, a.act);
        if (a.y_bf16) reinterpret_cast<uint16_t*>(a.Y)[(size_t)row * a.ldy + col] = f32_to_bf16(v);
        else reinterpret_cast<float*>(a.Y)[(size_t)row * a.ldy + col] = v;
      }
    }
}

// N == 1 heads (logistic / final regression): one wave per row, lanes over K.
__global__ void __launch_bounds__(256) gemv_kernel(GemmArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  if (row >= M) return;
  float s = 0.f;
  for (int k = lane; k < a.K; k += 64) {
    const float x = a.x_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(a.X)[(size_t)row * a.ldx + k])
                             : reinterpret_cast<const float*>(a.X)[(size_t)row * a.ldx + k];
    s += x * (a.w_f32 ? reinterpret_cast<const float*>(a.W)[k] : bf16_to_f32(reinterpret_cast<const uint16_t*>(a.W)[k]));
  }
  s = wave_sum(s);
  if (lane == 0) {
    const float v = act_fn(s + (a.bias ? a.bias[0] : 0.f), a.act);
    if (a.y_bf16) reinterpret_cast<uint16_t*>(a.Y)[(size_t)row * a.ldy] = f32_to_bf16(v);
    else reinterpret_cast<float*>(a.Y)[(size_t)row * a.ldy] = v;
  }
}

// Fused dense + N==1 head: y[r] = act2( sum_n act1(x[r] . W1[n] + b1[n]) * w2[n] + b2 ).
// 32 rows per block (8192 rows -> 256 blocks, one per CU); the A tile (32 x K_pad bf16) and,
// when it fits, all of W1 (N1_pad x K_pad bf16) are staged in LDS once, so the MFMA loop reads
// only LDS. The four waves split each 64-column chunk of the hidden layer (16 columns each);
// the 32 x N1 hidden tile lives only in accumulators: bias + act1 + w2-weighting happen in
// registers, rows are reduced across lanes (xor shuffles) and across the waves through LDS.
constexpr int HD_ROWS = 32;
constexpr int HD_W_LDS_MAX = 64 * 1024;  // W1 staged in LDS up to this many bytes

// the 8 f32 inputs of row `row`, columns kc..kc+7 (zero past K / M); returns false when the
// chunk is already bf16 (x_bf16 input, packed into *raw)
__device__ __forceinline__ bool head_a_f32(const HeadArgs& a, int row, int kc, int M, float f[8], uint4* raw) {
  if (row >= M) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
    return true;
  }
  if (a.partial) {
    // reduce the tree ensemble's group partials: sum_g P[g][row][k] (+ base, / T)
    if (kc + 8 <= a.K && (a.K & 3) == 0 && a.groups <= 8) {
      // straight-line: every group's pair of 16-B loads (clamped group index) and the base
      // values in flight at once (a loop waited per group), summed in group order as before
      const int gl = a.groups - 1;
      float4 p[8], q[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const float4* src = reinterpret_cast<const float4*>(a.partial + ((size_t)min(g, gl) * a.M + row) * a.K + kc);
        p[g] = src[0];
        q[g] = src[1];
      }
      float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
      if (a.pbase) {
        b0 = reinterpret_cast<const float4*>(a.pbase + kc)[0];
        b1 = reinterpret_cast<const float4*>(a.pbase + kc)[1];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        if (g <= gl) {
          f[0] += p[g].x; f[1] += p[g].y; f[2] += p[g].z; f[3] += p[g].w;
          f[4] += q[g].x; f[5] += q[g].y; f[6] += q[g].z; f[7] += q[g].w;
        }
      }
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (a.p_average) f[j] /= (float)a.p_ntrees;
        f[j] += bb[j];  // 0 without a base: x + 0 == x
      }
      return true;
    } else if (kc + 8 <= a.K && (a.K & 3) == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = 0.f;
      for (int g = 0; g < a.groups; ++g) {
        const float4* src = reinterpret_cast<const float4*>(a.partial + ((size_t)g * a.M + row) * a.K + kc);
        const float4 p = src[0], q = src[1];
        f[0] += p.x; f[1] += p.y; f[2] += p.z; f[3] += p.w; f[4] += q.x; f[5] += q.y; f[6] += q.z; f[7] += q.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = 0.f;
        if (kc + j < a.K)
          for (int g = 0; g < a.groups; ++g) v += a.partial[((size_t)g * a.M + row) * a.K + kc + j];
        f[j] = v;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kc + j;
      if (k < a.K) {
        if (a.p_average) f[j] /= (float)a.p_ntrees;
        if (a.pbase) f[j] += a.pbase[k];
      } else {
        f[j] = 0.f;
      }
    }
  } else if (a.x_bf16) {
    const uint16_t* src = reinterpret_cast<const uint16_t*>(a.X) + (size_t)row * a.ldx + kc;
    uint16_t t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = (kc + j < a.K) ? src[j] : 0;
    *raw = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = bf16_to_f32(t[j]);
    return false;
  } else {
    const float* src = reinterpret_cast<const float*>(a.X) + (size_t)row * a.ldx + kc;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (kc + j < a.K) ? src[j] : 0.f;
  }
  return true;
}

__device__ __forceinline__ uint4 head_a_chunk(const HeadArgs& a, int row, int kc, int M) {
  float f[8];
  uint4 raw;
  if (!head_a_f32(a, row, kc, M, f, &raw)) return raw;
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                    pack_bf16x2(f[6], f[7]));
}

__global__ void __launch_bounds__(256) mlp_head_kernel(HeadArgs a, int w_lds) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint16_t* const W1 = reinterpret_cast<const uint16_t*>(a.W1);
  const int kp = a.k_pad;
  const int lds_row = kp + G_PAD;
  const int n1p = (a.N1 + 63) & ~63;
  uint16_t* sA = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sW = sA + HD_ROWS * lds_row;
  float* sred = reinterpret_cast<float*>(smem + (((size_t)(HD_ROWS + (w_lds ? n1p : 0)) * lds_row * 2 + 15) &
                                                 ~size_t(15)));
  float* sb1 = sred + 4 * HD_ROWS;  // [n1p] b1, then [n1p] w2 (zero past N1)
  float* sw2 = sb1 + n1p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = blockIdx.x * HD_ROWS;
  __shared__ unsigned int ecnt[MET_N];  // fused K5 metrics
  const bool fm = a.fuse_ens && a.ens.metrics;
  if (row0 >= M) {
    // past the live rows: the fused ensemble still writes the inert rows' (zero) results
    if (a.fuse_ens)
      for (int r = row0 + tid; r < min(row0 + HD_ROWS, a.ens.n_rows); r += 256) ensemble_row(a.ens, r, true, 0.f, nullptr);
    return;
  }
  if (fm)
    for (int i = tid; i < MET_N; i += 256) ecnt[i] = 0;
  int64_t* const trow = (a.trace && tid == 0 && (blockIdx.x & 31) == 0 && blockIdx.x < 256) ? a.trace + (blockIdx.x >> 5) * 8 : nullptr;
#define HD_MARK(k) \
  if (trow) trow[k] = (int64_t)wall_clock64()
  HD_MARK(0);
  const int kch = kp / 8;  // 16-byte chunks per row
  // stage W1, b1 / w2 and the A tile with one memory round trip in the common case: the first
  // W1 pass, the head vectors and the first A chunk are all issued before anything is stored
  // (b1 / w2 used to be global loads inside the column loop: one dependent round trip per
  // 64-column chunk)
  constexpr int UN = 4;
  const int wtotal = w_lds ? n1p * kch : 0;
  uint4 wv[UN];
#pragma unroll
  for (int u = 0; u < UN; ++u) {
    const int ch = u * 256 + tid;
    wv[u] = ch < wtotal ? *reinterpret_cast<const uint4*>(W1 + (size_t)(ch / kch) * kp + (ch % kch) * 8)
                        : make_uint4(0, 0, 0, 0);
  }
  const float b1v = (tid < a.N1 && a.b1) ? a.b1[tid] : 0.f;
  const float w2v = tid < a.N1 ? a.w2[tid] : 0.f;
  const int ach = HD_ROWS * kch;
  const uint4 av = tid < ach ? head_a_chunk(a, row0 + tid / kch, (tid % kch) * 8, M) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int u = 0; u < UN; ++u) {
    const int ch = u * 256 + tid;
    if (ch < wtotal) *reinterpret_cast<uint4*>(&sW[(ch / kch) * lds_row + (ch % kch) * 8]) = wv[u];
  }
  if (tid < n1p) {
    sb1[tid] = b1v;
    sw2[tid] = w2v;
  }
  for (int n = tid + 256; n < n1p; n += 256) {
    sb1[n] = (n < a.N1 && a.b1) ? a.b1[n] : 0.f;
    sw2[n] = n < a.N1 ? a.w2[n] : 0.f;
  }
  if (tid < ach) *reinterpret_cast<uint4*>(&sA[(tid / kch) * lds_row + (tid % kch) * 8]) = av;
  if (wtotal > 256 * UN) {
    const int total = wtotal;
    for (int base = 256 * UN; base < total; base += 256 * UN) {
      uint4 v[UN];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int ch = base + u * 256 + tid;
        v[u] = ch < total ? *reinterpret_cast<const uint4*>(W1 + (size_t)(ch / kch) * kp + (ch % kch) * 8)
                          : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int ch = base + u * 256 + tid;
        if (ch < total) *reinterpret_cast<uint4*>(&sW[(ch / kch) * lds_row + (ch % kch) * 8]) = v[u];
      }
    }
  }
  for (int ch = tid + 256; ch < ach; ch += 256) {
    const int r = ch / kch, kc = (ch % kch) * 8;
    *reinterpret_cast<uint4*>(&sA[r * lds_row + kc]) = head_a_chunk(a, row0 + r, kc, M);
  }
  __syncthreads();
  HD_MARK(1);
  float part[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) part[i][q] = 0.f;
  for (int c0 = 0; c0 < a.N1; c0 += 64) {
    const int n = c0 + wave * 16 + (lane & 15);  // this lane's B-fragment column
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int k0 = 0; k0 < kp; k0 += 32) {
      const int kof = k0 + 8 * (lane >> 4);
      const bf16x8 fb = w_lds ? *reinterpret_cast<const bf16x8*>(&sW[n * lds_row + kof])
                              : *reinterpret_cast<const bf16x8*>(W1 + (size_t)n * kp + kof);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(&sA[(i * 16 + (lane & 15)) * lds_row + kof]);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[i], 0, 0, 0);
      }
    }
    const float b1 = sb1[n];
    const float w2 = sw2[n];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) part[i][q] += act_fn(acc[i][q] + b1, a.act1) * w2;
  }
  // reduce over the 16 lanes that share rows (lane & 15 = column), then over the 4 waves
#pragma unroll
  for (int i = 0; i < 2; ++i)
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
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) sred[wave * HD_ROWS + i * 16 + (lane >> 4) * 4 + q] = part[i][q];
  }
  HD_MARK(2);
  __syncthreads();
  HD_MARK(3);
  if (tid < HD_ROWS) {
    const int row = row0 + tid;
    float y = 0.f;
    if (row < M) {
      const float v = sred[tid] + sred[HD_ROWS + tid] + sred[2 * HD_ROWS + tid] + sred[3 * HD_ROWS + tid];
      y = act_fn(v + a.b2, a.act2);
      a.Y[(size_t)row * a.ldy] = y;
    }
    if (a.fuse_ens && row < a.ens.n_rows) ensemble_row(a.ens, row, true, y, fm ? ecnt : nullptr);
  }
  if (fm) {
    __syncthreads();
    ensemble_metrics_flush(a.ens, ecnt, tid, 256);
  }
  if (trow) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HD_MARK(4);
  }
#undef HD_MARK
}


// ---------------------------------------------------------------------------------------------
// Reference-precision (fp32) variants: the ONNX fraud model contract is f32
// (onnx_model.go:221-238), and final = int(0.4 rule + 0.6 ml 100) truncates, so a bf16 head
// (~1e-2 ml error) moves decisions across thresholds. These keep every operand in f32 and run
// on v_mfma_f32_16x16x4_f32: lane l supplies A[l & 15][k] and B[k][l & 15] with
// k = 4 (l >> 4) + j for the j-th of four consecutive MFMAs, so one 16-B LDS read per operand
// feeds four MFMAs and four MFMAs cover 16 k (the sum over k is order-free up to rounding).

// mlp_head in f32: same blocking as the bf16 kernel (32 rows per block, 4 waves x 16 hidden
// columns per 64-column chunk), A tile and W1 (f32 [n1p][k_pad]) staged in LDS with rows
// padded by 4 floats.
__global__ void __launch_bounds__(256) mlp_head_f32_kernel(HeadArgs a, int w_lds) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const float* const W1 = reinterpret_cast<const float*>(a.W1);
  const int kp = a.k_pad;
  const int lds_row = kp + 4;
  const int n1p = (a.N1 + 63) & ~63;
  float* sA = smf;
  float* sW = sA + HD_ROWS * lds_row;
  float* sred = sW + (w_lds ? n1p * lds_row : 0);
  float* sb1 = sred + 4 * HD_ROWS;
  float* sw2 = sb1 + n1p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = blockIdx.x * HD_ROWS;
  __shared__ unsigned int ecnt[MET_N];
  const bool fm = a.fuse_ens && a.ens.metrics;
  if (row0 >= M) {
    if (a.fuse_ens)
      for (int r = row0 + tid; r < min(row0 + HD_ROWS, a.ens.n_rows); r += 256) ensemble_row(a.ens, r, true, 0.f, nullptr);
    return;
  }
  if (fm)
    for (int i = tid; i < MET_N; i += 256) ecnt[i] = 0;
  // phase trace of 8 sample blocks (tools/kbench.py): start / staged / mfma done / synced / stored
  int64_t* const trow = (a.trace && tid == 0 && (blockIdx.x & 31) == 0 && blockIdx.x < 256) ? a.trace + (blockIdx.x >> 5) * 8 : nullptr;
#define HF_MARK(k) \
  if (trow) trow[k] = (int64_t)wall_clock64()
  HF_MARK(0);
  const int kq = kp / 4;  // float4 chunks per row
  if (w_lds) {
    const int total = n1p * kq;
    for (int base = 0; base < total; base += 256 * 4) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ch = base + u * 256 + tid;
        v[u] = ch < total ? *reinterpret_cast<const float4*>(W1 + (size_t)(ch / kq) * kp + (ch % kq) * 4)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ch = base + u * 256 + tid;
        if (ch < total) *reinterpret_cast<float4*>(&sW[(ch / kq) * lds_row + (ch % kq) * 4]) = v[u];
      }
    }
  }
  for (int n = tid; n < n1p; n += 256) {
    sb1[n] = (n < a.N1 && a.b1) ? a.b1[n] : 0.f;
    sw2[n] = n < a.N1 ? a.w2[n] : 0.f;
  }
  const int k8 = kp / 8;
  for (int ch = tid; ch < HD_ROWS * k8; ch += 256) {
    const int r = ch / k8, kc = (ch % k8) * 8;
    float f[8];
    uint4 raw;
    head_a_f32(a, row0 + r, kc, M, f, &raw);
    *reinterpret_cast<float4*>(&sA[r * lds_row + kc]) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(&sA[r * lds_row + kc + 4]) = make_float4(f[4], f[5], f[6], f[7]);
  }
  __syncthreads();
  HF_MARK(1);
  float part[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) part[i][q] = 0.f;
  for (int c0 = 0; c0 < a.N1; c0 += 64) {
    const int n = c0 + wave * 16 + (lane & 15);
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int k0 = 0; k0 < kp; k0 += 16) {
      const int kk = k0 + 4 * (lane >> 4);
      const float4 bv = w_lds ? *reinterpret_cast<const float4*>(&sW[n * lds_row + kk])
                              : *reinterpret_cast<const float4*>(W1 + (size_t)n * kp + kk);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float4 av = *reinterpret_cast<const float4*>(&sA[(i * 16 + (lane & 15)) * lds_row + kk]);
        acc[i] = mfma4_f32(av, bv, acc[i]);
      }
    }
    const float b1 = sb1[n];
    const float w2 = sw2[n];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) part[i][q] += act_fn(acc[i][q] + b1, a.act1) * w2;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
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
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) sred[wave * HD_ROWS + i * 16 + (lane >> 4) * 4 + q] = part[i][q];
  }
  HF_MARK(2);
  __syncthreads();
  HF_MARK(3);
  if (tid < HD_ROWS) {
    const int row = row0 + tid;
    float y = 0.f;
    if (row < M) {
      const float v = sred[tid] + sred[HD_ROWS + tid] + sred[2 * HD_ROWS + tid] + sred[3 * HD_ROWS + tid];
      y = act_fn(v + a.b2, a.act2);
      a.Y[(size_t)row * a.ldy] = y;
    }
    if (a.fuse_ens && row < a.ens.n_rows) ensemble_row(a.ens, row, true, y, fm ? ecnt : nullptr);
  }
  if (fm) {
    __syncthreads();
    ensemble_metrics_flush(a.ens, ecnt, tid, 256);
  }
  if (trow) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HF_MARK(4);
  }
#undef HF_MARK
}

// mlp_head f32, specialised on k_pad (KP = 32 / 64) and the hidden activation (ACT), W1 staged
// in LDS: what the generic kernel above lost to its runtime shape (compiler output of the generic
// k loop: a flat load selecting LDS or global W1 per k-step behind a full vmcnt/lgkmcnt wait, the
// two accumulators shuffled through AGPR moves every iteration, and a four-way activation switch
// per element; phase trace 5 us staging + 5 us for 64 MFMAs per wave). Here every staging load
// (the first 8 W1 chunks per thread, b1 / w2, the A chunk with all tree-group partials) is in
// flight before anything is stored (one memory round trip), the A fragments of both row tiles
// stay in registers across the column chunks, and the k loop is unrolled. Same MFMA sequence
// and summation order as the generic kernel: bit-identical results.
template <int KP, int ACT>
__global__ void __launch_bounds__(256) mlp_head_f32_fast_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  constexpr int LR = KP + 4;  // LDS row stride (floats)
  constexpr int KQ = KP / 4;  // float4 chunks per W1 row
  constexpr int K8 = KP / 8;  // 8-float A chunks per row
  constexpr int KS = KP / 16;  // k-steps of four 16x16x4 MFMAs
  const float* const W1 = reinterpret_cast<const float*>(a.W1);
  const int n1p = (a.N1 + 63) & ~63;
  float* sA = smf;
  float* sW = sA + HD_ROWS * LR;
  float* sred = sW + n1p * LR;
  float* sb1 = sred + 4 * HD_ROWS;
  float* sw2 = sb1 + n1p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = blockIdx.x * HD_ROWS;
  __shared__ unsigned int ecnt[MET_N];
  const bool fm = a.fuse_ens && a.ens.metrics;
  if (row0 >= M) {
    if (a.fuse_ens)
      for (int r = row0 + tid; r < min(row0 + HD_ROWS, a.ens.n_rows); r += 256) ensemble_row(a.ens, r, true, 0.f, nullptr);
    return;
  }
  if (fm)
    for (int i = tid; i < MET_N; i += 256) ecnt[i] = 0;
  int64_t* const trow = (a.trace && tid == 0 && (blockIdx.x & 31) == 0 && blockIdx.x < 256) ? a.trace + (blockIdx.x >> 5) * 8 : nullptr;
#define HQ_MARK(k) \
  if (trow) trow[k] = (int64_t)wall_clock64()
  HQ_MARK(0);
  const int total = n1p * KQ;
  float4 wv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int ch = u * 256 + tid;
    wv[u] = ch < total ? *reinterpret_cast<const float4*>(W1 + (size_t)(ch / KQ) * KP + (ch % KQ) * 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float b1v = (tid < a.N1 && a.b1) ? a.b1[tid] : 0.f;
  const float w2v = tid < a.N1 ? a.w2[tid] : 0.f;
  const bool has_a = tid < HD_ROWS * K8;
  float f[8];
  uint4 raw;
  if (has_a) head_a_f32(a, row0 + tid / K8, (tid % K8) * 8, M, f, &raw);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int ch = u * 256 + tid;
    if (ch < total) *reinterpret_cast<float4*>(&sW[(ch / KQ) * LR + (ch % KQ) * 4]) = wv[u];
  }
  for (int ch = 8 * 256 + tid; ch < total; ch += 256)  // W1 wider than 8 chunks per thread
    *reinterpret_cast<float4*>(&sW[(ch / KQ) * LR + (ch % KQ) * 4]) =
        *reinterpret_cast<const float4*>(W1 + (size_t)(ch / KQ) * KP + (ch % KQ) * 4);
  if (tid < n1p) {
    sb1[tid] = b1v;
    sw2[tid] = w2v;
  }
  for (int n = tid + 256; n < n1p; n += 256) {
    sb1[n] = (n < a.N1 && a.b1) ? a.b1[n] : 0.f;
    sw2[n] = n < a.N1 ? a.w2[n] : 0.f;
  }
  if (has_a) {
    const int r = tid / K8, kc = (tid % K8) * 8;
    *reinterpret_cast<float4*>(&sA[r * LR + kc]) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(&sA[r * LR + kc + 4]) = make_float4(f[4], f[5], f[6], f[7]);
  }
  for (int ch = tid + 256; ch < HD_ROWS * K8; ch += 256) {
    const int r = ch / K8, kc = (ch % K8) * 8;
    head_a_f32(a, row0 + r, kc, M, f, &raw);
    *reinterpret_cast<float4*>(&sA[r * LR + kc]) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(&sA[r * LR + kc + 4]) = make_float4(f[4], f[5], f[6], f[7]);
  }
  __syncthreads();
  HQ_MARK(1);
  float4 av[2][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      av[i][s] = *reinterpret_cast<const float4*>(&sA[(i * 16 + (lane & 15)) * LR + s * 16 + 4 * (lane >> 4)]);
  float part[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) part[i][q] = 0.f;
  for (int c0 = 0; c0 < a.N1; c0 += 64) {
    const int n = c0 + wave * 16 + (lane & 15);
    float4 bv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) bv[s] = *reinterpret_cast<const float4*>(&sW[n * LR + s * 16 + 4 * (lane >> 4)]);
    const float b1 = sb1[n];
    const float w2 = sw2[n];
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      acc0 = mfma4_f32(av[0][s], bv[s], acc0);
      acc1 = mfma4_f32(av[1][s], bv[s], acc1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      part[0][q] += act_fn(acc0[q] + b1, ACT) * w2;
      part[1][q] += act_fn(acc1[q] + b1, ACT) * w2;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
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
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) sred[wave * HD_ROWS + i * 16 + (lane >> 4) * 4 + q] = part[i][q];
  }
  HQ_MARK(2);
  __syncthreads();
  HQ_MARK(3);
  if (tid < HD_ROWS) {
    const int row = row0 + tid;
    float y = 0.f;
    if (row < M) {
      const float v = sred[tid] + sred[HD_ROWS + tid] + sred[2 * HD_ROWS + tid] + sred[3 * HD_ROWS + tid];
      y = act_fn(v + a.b2, a.act2);
      a.Y[(size_t)row * a.ldy] = y;
    }
    if (a.fuse_ens && row < a.ens.n_rows) ensemble_row(a.ens, row, true, y, fm ? ecnt : nullptr);
  }
  if (fm) {
    __syncthreads();
    ensemble_metrics_flush(a.ens, ecnt, tid, 256);
  }
  if (trow) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HQ_MARK(4);
  }
#undef HQ_MARK
}

// f32 dense layer: 64 x 64 output tile per block, 4 waves in 2 x 2 (32 x 32 each = 2 x 2
// fragments), BK = 32 floats staged in two LDS buffers (next tile's global loads in flight
// under the current tile's MFMAs).
constexpr int GF_BK = 32;
constexpr int GF_ROW = GF_BK + 4;
__global__ void __launch_bounds__(256) gemm_f32_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) float sA[2][64 * GF_ROW];
  __shared__ __attribute__((aligned(16))) float sB[2][64 * GF_ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = a.m_ptr ? min(*a.m_ptr, a.M) : a.M;
  const int row0 = blockIdx.y * 64, col0 = blockIdx.x * 64;
  if (row0 >= M) return;
  const float* const W = reinterpret_cast<const float*>(a.W);
  const int K = a.K, k_pad = a.ldw;
  const int n_kt = (K + GF_BK - 1) / GF_BK;
  float4 ra[2], rb[2];
  auto load_tile = [&](int kt) {
    const int k0 = kt * GF_BK;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = tid + c * 256;          // 512 chunks = 64 rows x 8 float4
      const int r = ch >> 3, kc = (ch & 7) * 4;
      const int row = row0 + r, k = k0 + kc;
      float f[4] = {0.f, 0.f, 0.f, 0.f};
      if (row < M) {
        if (a.x_bf16) {
          const uint16_t* src = reinterpret_cast<const uint16_t*>(a.X) + (size_t)row * a.ldx + k;
#pragma unroll
          for (int j = 0; j < 4; ++j) f[j] = (k + j < K) ? bf16_to_f32(src[j]) : 0.f;
        } else {
          const float* src = reinterpret_cast<const float*>(a.X) + (size_t)row * a.ldx + k;
          if (k + 4 <= K && (a.ldx & 3) == 0) {
            const float4 p = *reinterpret_cast<const float4*>(src);
            f[0] = p.x; f[1] = p.y; f[2] = p.z; f[3] = p.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) f[j] = (k + j < K) ? src[j] : 0.f;
          }
        }
      }
      ra[c] = make_float4(f[0], f[1], f[2], f[3]);
      const int n = col0 + r;
      rb[c] = (k < k_pad) ? *reinterpret_cast<const float4*>(W + (size_t)n * k_pad + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = tid + c * 256;
      *reinterpret_cast<float4*>(&sA[buf][(ch >> 3) * GF_ROW + (ch & 7) * 4]) = ra[c];
      *reinterpret_cast<float4*>(&sB[buf][(ch >> 3) * GF_ROW + (ch & 7) * 4]) = rb[c];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < n_kt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < n_kt) load_tile(kt + 1);
#pragma unroll
    for (int kk = 0; kk < GF_BK; kk += 16) {
      const int kof = kk + 4 * (lane >> 4);
      float4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const float4*>(&sA[cur][(wm * 32 + i * 16 + (lane & 15)) * GF_ROW + kof]);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const float4*>(&sB[cur][(wn * 32 + j * 16 + (lane & 15)) * GF_ROW + kof]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma4_f32(fa[i], fb[j], acc[i][j]);
    }
    if (kt + 1 < n_kt) store_tile(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = col0 + wn * 32 + j * 16 + (lane & 15);
      if (col >= a.N) continue;
      const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = row0 + wm * 32 + i * 16 + (lane >> 4) * 4 + q;
        if (row >= M) continue;
        const float v = act_fn(acc[i][j][q] + b, a.act);
        if (a.y_bf16) reinterpret_cast<uint16_t*>(a.Y)[(size_t)row * a.ldy + col] = f32_to_bf16(v);
        else reinterpret_cast<float*>(a.Y)[(size_t)row * a.ldy + col] = v;
      }
    }
}

void launch_mlp_head(const HeadArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  if (a.w1_f32) {
    const size_t lds_row = (size_t)a.k_pad + 4;
    const size_t n1p = (size_t)((a.N1 + 63) & ~63);
    const int w_lds = n1p * lds_row * 4 <= (size_t)(96 * 1024);
    const size_t lds = ((size_t)HD_ROWS + (w_lds ? n1p : 0)) * lds_row * 4 + 4 * HD_ROWS * sizeof(float) +
                       2 * n1p * sizeof(float);
    const dim3 grid((a.M + HD_ROWS - 1) / HD_ROWS);
    if (w_lds && (a.k_pad == 32 || a.k_pad == 64) && a.act1 >= 0 && a.act1 <= 3) {
#define HQ_CASE(KP, ACT) \
  if (a.k_pad == KP && a.act1 == ACT) { IGP_LAUNCH((mlp_head_f32_fast_kernel<KP, ACT>), grid, dim3(256), lds, st, a); return; }
      HQ_CASE(32, 0) HQ_CASE(32, 1) HQ_CASE(32, 2) HQ_CASE(32, 3)
      HQ_CASE(64, 0) HQ_CASE(64, 1) HQ_CASE(64, 2) HQ_CASE(64, 3)
#undef HQ_CASE
    }
    IGP_LAUNCH(mlp_head_f32_kernel, grid, dim3(256), lds, st, a, w_lds);
    return;
  }
  const size_t lds_row = (size_t)a.k_pad + G_PAD;
  const size_t n1p = (size_t)((a.N1 + 63) & ~63);
  const int w_lds = n1p * lds_row * 2 <= (size_t)HD_W_LDS_MAX;
  const size_t lds = ((((size_t)HD_ROWS + (w_lds ? n1p : 0)) * lds_row * 2 + 15) & ~size_t(15)) +
                     4 * HD_ROWS * sizeof(float) + 2 * n1p * sizeof(float);
  IGP_LAUNCH(mlp_head_kernel, dim3((a.M + HD_ROWS - 1) / HD_ROWS), dim3(256), lds, st, a, w_lds);
}

void launch_gemm(const GemmArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  if (a.w_f32) {
    IGP_LAUNCH(gemm_f32_kernel, dim3((a.N + 63) / 64, (a.M + 63) / 64), dim3(256), 0, st, a);
    return;
  }
  const bool big = a.M >= 4096 && a.N >= 128;
  if (big) {
    dim3 grid((a.N + 127) / 128, (a.M + 127) / 128);
    IGP_LAUNCH((gemm_kernel<128, 128>), grid, dim3(256), 0, st, a);
  } else {
    dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
    IGP_LAUNCH((gemm_kernel<64, 64>), grid, dim3(256), 0, st, a);
  }
}

void launch_gemv(const GemmArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  IGP_LAUNCH(gemv_kernel, dim3((a.M + 3) / 4), dim3(256), 0, st, a);
}

}  // namespace igp
