// K4: stacked ONNX GRU (1-2 layers, forward, layout 0) over a per-account event history,
// with the N=1 head (Gemm + Sigmoid) fused — the CheckBonusAbuse model of config 5.
//
// Batch-parallel recurrence: a workgroup owns M = 16*RT sequences and runs ALL T steps of
// BOTH layers for them, so no grid-wide synchronisation is ever needed (every wave's exit is
// unconditional). Per step and layer:
//   gates[M, 3H] = x_t[M, K] . W^T  +  h_{t-1}[M, H] . R^T        (MFMA 16x16x32 bf16)
// Weights stream from L2 as fragment-packed 1 KiB wave loads (shared by the RT row tiles);
// x_t / h_{t-1} A-fragments come from LDS (bf16, ping-pong buffers per layer); the f32
// hidden state never leaves registers: lane (l&15, l>>4) of the wave that owns hidden tile
// ht computes the same (row, unit) every step, so z/r/h~ combine lane-locally.
// Layer 2 consumes layer 1's h_t straight from LDS (Y never touches HBM). The layer-1 input
// of step t+1 is prefetched into registers during step t (from the HBM event ring, mode 1,
// or a dense [T][B][I] tensor, mode 0).
#include "common.h"
#include "launch.h"

namespace igp {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace {

constexpr int GRU_PAD = 8;  // bf16 row padding in LDS (16 B)

__device__ __forceinline__ float sig_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_(float x) { return 1.f - 2.f / (__expf(2.f * x) + 1.f); }

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// Weight fragments come through a buffer resource: the per-lane part is ONE VGPR (lane*16)
// shared by every fragment load and the fragment index goes into the scalar offset, so no
// 64-bit per-load addresses are materialised (they were hoisted out of the time loop and spilled).
struct WFrag {
  __amdgpu_buffer_rsrc_t rsrc;
  int voff;
};

__device__ __forceinline__ WFrag wfrag(const uint16_t* base, size_t elems, int lane) {
  WFrag w;
  w.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, (int)(elems * 2), 0x00020000);
  w.voff = lane * 16;
  return w;
}

__device__ __forceinline__ bf16x8 ld_frag(const WFrag& w, int nt, int KS, int ks) {
  const int soff = __builtin_amdgcn_readfirstlane((nt * KS + ks) * 1024);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, w.voff, soff, 0);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 lds_frag(const uint16_t* base, int stride, int row, int k) {
  const uint4 v = *reinterpret_cast<const uint4*>(base + row * stride + k);
  return *reinterpret_cast<const bf16x8*>(&v);
}


// One GRU layer step for this wave's hidden tiles. KSX/KSH: K/32 of the input / hidden parts.
// The recurrence is latency-bound on the streamed weight fragments: tiles are processed in
// groups of G (G*RT <= 2, so accumulators stay at 32 floats) and every k-step issues the
// 3*G fragments of the group at once; with the k loop unrolled by 2 ~12 loads are in flight.
template <int RT, int KSX, int KSH, int LBR, int NW>
__device__ __forceinline__ void layer_step(const WFrag& gW, const WFrag& gR, const float* bias, const uint16_t* in,
                                           int in_stride, const uint16_t* hprev, uint16_t* hnext,
                                           uint16_t* rb, float (&hs)[KSH * 2 / NW][RT][4], int lane, int wave) {
  constexpr int HT = KSH * 2;      // hidden tiles of 16 units
  constexpr int HTW = HT / NW;     // per wave
  constexpr int G = (RT == 1 && HTW >= 2) ? 2 : 1;
  constexpr int H = KSH * 32;
  constexpr int HS = H + GRU_PAD;
  const int arow = lane & 15, akof = 8 * (lane >> 4);
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  float zk[LBR ? 1 : HTW][RT][4];  // linear_before_reset = 0: z and the x-part of h~ wait for r*h
  float xk[LBR ? 1 : HTW][RT][4];
#pragma unroll
  for (int g0 = 0; g0 < HTW; g0 += G) {
    f32x4 az[G][RT], ar[G][RT], ax[G][RT], ah[G][RT];
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) az[u][rt] = ar[u][rt] = ax[u][rt] = ah[u][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSX; ++ks) {  // input projection x_t . W^T
      bf16x8 bz[G], br[G], bh[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int ht = wave + NW * (g0 + u);
        bz[u] = ld_frag(gW, ht, KSX, ks);
        br[u] = ld_frag(gW, HT + ht, KSX, ks);
        bh[u] = ld_frag(gW, 2 * HT + ht, KSX, ks);
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 a = lds_frag(in, in_stride, rt * 16 + arow, ks * 32 + akof);
#pragma unroll
        for (int u = 0; u < G; ++u) {
          az[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bz[u], az[u][rt], 0, 0, 0);
          ar[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, br[u], ar[u][rt], 0, 0, 0);
          ax[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[u], ax[u][rt], 0, 0, 0);
        }
      }
    }
#pragma unroll 2
    for (int ks = 0; ks < KSH; ++ks) {  // recurrent projection h_{t-1} . R^T
      bf16x8 bz[G], br[G], bh[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int ht = wave + NW * (g0 + u);
        bz[u] = ld_frag(gR, ht, KSH, ks);
        br[u] = ld_frag(gR, HT + ht, KSH, ks);
        if constexpr (LBR != 0) bh[u] = ld_frag(gR, 2 * HT + ht, KSH, ks);
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 a = lds_frag(hprev, HS, rt * 16 + arow, ks * 32 + akof);
#pragma unroll
        for (int u = 0; u < G; ++u) {
          az[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bz[u], az[u][rt], 0, 0, 0);
          ar[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, br[u], ar[u][rt], 0, 0, 0);
          if constexpr (LBR != 0) ah[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[u], ah[u][rt], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int i = g0 + u;
      const int j = (wave + NW * i) * 16 + ccol;
      const float bz_ = bias[j] + bias[3 * H + j];
      const float br_ = bias[H + j] + bias[4 * H + j];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = sig_(az[u][rt][r] + bz_);
          const float rr = sig_(ar[u][rt][r] + br_);
          if constexpr (LBR != 0) {
            const float hh = tanh_(ax[u][rt][r] + bias[2 * H + j] + rr * (ah[u][rt][r] + bias[5 * H + j]));
            const float h = (1.f - z) * hh + z * hs[i][rt][r];
            hs[i][rt][r] = h;
            hnext[(rt * 16 + crow + r) * HS + j] = f32_to_bf16(h);
          } else {
            zk[i][rt][r] = z;
            xk[i][rt][r] = ax[u][rt][r];
            rb[(rt * 16 + crow + r) * HS + j] = f32_to_bf16(rr * hs[i][rt][r]);
          }
        }
    }
  }
  if constexpr (LBR == 0) {
    // h~ = tanh(x Wh + (r * h_{t-1}) Rh + b): needs r for every unit of the row -> barrier
    __syncthreads();
#pragma unroll
    for (int g0 = 0; g0 < HTW; g0 += G) {
      f32x4 ah[G][RT];
#pragma unroll
      for (int u = 0; u < G; ++u)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) ah[u][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int ks = 0; ks < KSH; ++ks) {
        bf16x8 bh[G];
#pragma unroll
        for (int u = 0; u < G; ++u) bh[u] = ld_frag(gR, 2 * HT + wave + NW * (g0 + u), KSH, ks);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const bf16x8 a = lds_frag(rb, HS, rt * 16 + arow, ks * 32 + akof);
#pragma unroll
          for (int u = 0; u < G; ++u)
            ah[u][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[u], ah[u][rt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int i = g0 + u;
        const int j = (wave + NW * i) * 16 + ccol;
        const float bxh = bias[2 * H + j], bhh = bias[5 * H + j];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float hh = tanh_(xk[i][rt][r] + bxh + ah[u][rt][r] + bhh);
            const float z = zk[i][rt][r];
            const float h = (1.f - z) * hh + z * hs[i][rt][r];
            hs[i][rt][r] = h;
            hnext[(rt * 16 + crow + r) * HS + j] = f32_to_bf16(h);
          }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// f32-faithful split mode (the ONNX model's f32 contract, default for fp32 plans): weights and
// activations are bf16 pairs hi + lo (hi = bf16(x), lo = bf16(x - hi)), each product runs as
// three MFMAs (lo*hi + hi*lo + hi*hi; lo*lo ~2^-18 relative is dropped) into f32 accumulators,
// and the hidden state stays f32 in registers. ~1e-5 relative to fp32 at 3x the bf16 MFMA
// count; the f32 MFMA (v_mfma_f32_16x16x4_f32) would be ~16x slower than bf16.
__device__ __forceinline__ void gru_split(float x, uint16_t& hi, uint16_t& lo) {
  hi = f32_to_bf16(x);
  lo = f32_to_bf16(x - __uint_as_float((uint32_t)hi << 16));
}

#define GRU_MMA3(acc, ah, al, bh, bl)                                      \
  do {                                                                     \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);   \
  } while (0)

template <int RT, int KSX, int KSH, int LBR, int NW>
__device__ __forceinline__ void layer_step_x3(const WFrag& gW, const WFrag& gWl, const WFrag& gR, const WFrag& gRl,
                                              const float* bias, const uint16_t* in, const uint16_t* inl, int in_stride,
                                              const uint16_t* hprev, const uint16_t* hprevl, uint16_t* hnext,
                                              uint16_t* hnextl, uint16_t* rb, uint16_t* rbl,
                                              float (&hs)[KSH * 2 / NW][RT][4], int lane, int wave) {
  constexpr int HT = KSH * 2;
  constexpr int HTW = HT / NW;
  constexpr int H = KSH * 32;
  constexpr int HS = H + GRU_PAD;
  const int arow = lane & 15, akof = 8 * (lane >> 4);
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  float zk[LBR ? 1 : HTW][RT][4];
  float xk[LBR ? 1 : HTW][RT][4];
#pragma unroll
  for (int i = 0; i < HTW; ++i) {
    const int ht = wave + NW * i;
    f32x4 az[RT], ar[RT], ax[RT], ah[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) az[rt] = ar[rt] = ax[rt] = ah[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSX; ++ks) {  // x_t . W^T
      const bf16x8 bz = ld_frag(gW, ht, KSX, ks), bzl = ld_frag(gWl, ht, KSX, ks);
      const bf16x8 br = ld_frag(gW, HT + ht, KSX, ks), brl = ld_frag(gWl, HT + ht, KSX, ks);
      const bf16x8 bh = ld_frag(gW, 2 * HT + ht, KSX, ks), bhl = ld_frag(gWl, 2 * HT + ht, KSX, ks);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 a = lds_frag(in, in_stride, rt * 16 + arow, ks * 32 + akof);
        const bf16x8 al = lds_frag(inl, in_stride, rt * 16 + arow, ks * 32 + akof);
        GRU_MMA3(az[rt], a, al, bz, bzl);
        GRU_MMA3(ar[rt], a, al, br, brl);
        GRU_MMA3(ax[rt], a, al, bh, bhl);
      }
    }
#pragma unroll 2
    for (int ks = 0; ks < KSH; ++ks) {  // h_{t-1} . R^T
      const bf16x8 bz = ld_frag(gR, ht, KSH, ks), bzl = ld_frag(gRl, ht, KSH, ks);
      const bf16x8 br = ld_frag(gR, HT + ht, KSH, ks), brl = ld_frag(gRl, HT + ht, KSH, ks);
      bf16x8 bh, bhl;
      if constexpr (LBR != 0) {
        bh = ld_frag(gR, 2 * HT + ht, KSH, ks);
        bhl = ld_frag(gRl, 2 * HT + ht, KSH, ks);
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const bf16x8 a = lds_frag(hprev, HS, rt * 16 + arow, ks * 32 + akof);
        const bf16x8 al = lds_frag(hprevl, HS, rt * 16 + arow, ks * 32 + akof);
        GRU_MMA3(az[rt], a, al, bz, bzl);
        GRU_MMA3(ar[rt], a, al, br, brl);
        if constexpr (LBR != 0) GRU_MMA3(ah[rt], a, al, bh, bhl);
      }
    }
    const int j = ht * 16 + ccol;
    const float bz_ = bias[j] + bias[3 * H + j];
    const float br_ = bias[H + j] + bias[4 * H + j];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = sig_(az[rt][r] + bz_);
        const float rr = sig_(ar[rt][r] + br_);
        const int o = (rt * 16 + crow + r) * HS + j;
        if constexpr (LBR != 0) {
          const float hh = tanh_(ax[rt][r] + bias[2 * H + j] + rr * (ah[rt][r] + bias[5 * H + j]));
          const float h = (1.f - z) * hh + z * hs[i][rt][r];
          hs[i][rt][r] = h;
          gru_split(h, hnext[o], hnextl[o]);
        } else {
          zk[i][rt][r] = z;
          xk[i][rt][r] = ax[rt][r];
          gru_split(rr * hs[i][rt][r], rb[o], rbl[o]);
        }
      }
  }
  if constexpr (LBR == 0) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < HTW; ++i) {
      const int ht = wave + NW * i;
      f32x4 ah[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) ah[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int ks = 0; ks < KSH; ++ks) {
        const bf16x8 bh = ld_frag(gR, 2 * HT + ht, KSH, ks), bhl = ld_frag(gRl, 2 * HT + ht, KSH, ks);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const bf16x8 a = lds_frag(rb, HS, rt * 16 + arow, ks * 32 + akof);
          const bf16x8 al = lds_frag(rbl, HS, rt * 16 + arow, ks * 32 + akof);
          GRU_MMA3(ah[rt], a, al, bh, bhl);
        }
      }
      const int j = ht * 16 + ccol;
      const float bxh = bias[2 * H + j], bhh = bias[5 * H + j];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float hh = tanh_(xk[i][rt][r] + bxh + ah[rt][r] + bhh);
          const float z = zk[i][rt][r];
          const float h = (1.f - z) * hh + z * hs[i][rt][r];
          hs[i][rt][r] = h;
          const int o = (rt * 16 + crow + r) * HS + j;
          gru_split(h, hnext[o], hnextl[o]);
        }
    }
  }
}

}  // namespace

template <int RT, int KSH, int NW>
__device__ __forceinline__ void emit_outputs(const GruArgs& a, float (&hs)[KSH * 2 / NW][RT][4], float* red, int row0,
                                             int n_live, int lane, int wave, int tid) {
  constexpr int M = RT * 16, H = KSH * 32, HTW = KSH * 2 / NW;
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  if (a.yh) {
#pragma unroll
    for (int i = 0; i < HTW; ++i)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = row0 + rt * 16 + crow + r;
          if (row < n_live) a.yh[(size_t)row * H + (wave + NW * i) * 16 + ccol] = hs[i][rt][r];
        }
  }
  if (a.head_w) {
    float part[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[rt][r] = 0.f;
#pragma unroll
    for (int i = 0; i < HTW; ++i) {
      const float w = a.head_w[(wave + NW * i) * 16 + ccol];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[rt][r] += hs[i][rt][r] * w;
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = part[rt][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
        if (ccol == 0) red[wave * M + rt * 16 + crow + r] = v;
      }
    __syncthreads();
    if (tid < M && row0 + tid < n_live) {
      float v = a.head_b;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[w * M + tid];
      if (a.head_act == 2) v = 1.f / (1.f + expf(-v));
      a.out[row0 + tid] = v;
    }
  }
}

template <int RT, int KSX, int KSH, int LBR, int NW>
__global__ void __launch_bounds__(NW * 64) gru_kernel(GruArgs a) {
  constexpr int M = RT * 16;
  constexpr int H = KSH * 32;
  constexpr int HS = H + GRU_PAD;
  constexpr int XS = KSX * 32 + GRU_PAD;
  constexpr int HTW = KSH * 2 / NW;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  const int row0 = blockIdx.x * M;
  if (row0 >= n_live) return;
  const WFrag w0 = wfrag(a.layer[0].W, (size_t)3 * H * KSX * 32, lane), r0 = wfrag(a.layer[0].R, (size_t)3 * H * H, lane);
  const WFrag w1 = wfrag(a.layer[1].W, (size_t)3 * H * H, lane), r1 = wfrag(a.layer[1].R, (size_t)3 * H * H, lane);

  // ---- LDS carve-up: hb[layer][pingpong][M][HS] | xb[pingpong][M][XS] | rb[M][HS] | bias[2][6H] | red[4][M]
  uint16_t* const hb = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const xb = hb + 4 * M * HS;
  uint16_t* const rb = xb + 2 * M * XS;
  float* const bias = reinterpret_cast<float*>(rb + M * HS);
  float* const red = bias + 12 * H;
#define HB(l, b) (hb + ((l) * 2 + (b)) * (M * HS))
#define XB(b) (xb + (b) * (M * XS))

  // zero h_0 (both layers, both buffers) and the x buffers (their K padding stays zero)
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(smem);
    const int words = (4 * M * HS + 2 * M * XS) / 2;
    for (int i = tid; i < words; i += NT) z[i] = 0u;
  }
  for (int i = tid; i < 6 * H; i += NT) bias[i] = a.layer[0].bias[i];
  if (a.n_layers == 2)
    for (int i = tid; i < 6 * H; i += NT) bias[6 * H + i] = a.layer[1].bias[i];

  // ---- layer-1 input staging: thread -> (row rr, 8-element chunk c), fixed for all t
  const int I = a.I;
  const int chunks = I >> 3;
  const int my_rr = tid / max(chunks, 1), my_c = tid - my_rr * max(chunks, 1);
  const bool stager = chunks > 0 && my_rr < M;
  const int grow = row0 + my_rr;
  int slot = -1, head = 0, valid_from = a.T;
  if (stager && grow < n_live) {
    if (a.mode == 1) {
      slot = a.slots[grow];
      if (slot >= 0) {
        const AcctRT r = a.rt[slot];
        const int cnt = min(r.ev_count, a.T);
        head = r.ev_head;
        valid_from = a.T - cnt;
      }
    } else {
      valid_from = 0;
    }
  }
  auto load_x = [&](int t) -> uint4 {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (a.reverse) t = a.T - 1 - t;  // direction=reverse: forward over the time-reversed sequence
    if (!stager || t < valid_from || t < 0) return v;
    if (a.mode == 1) {
      int idx = (head - a.T + t) % a.ev_ring;
      if (idx < 0) idx += a.ev_ring;
      v = *reinterpret_cast<const uint4*>(a.ev + (((size_t)slot * a.ev_ring + idx) * I + my_c * 8));
    } else {
      const float* src = a.X + (((size_t)t * a.x_rows + grow) * I + my_c * 8);
      const float4 f0 = *reinterpret_cast<const float4*>(src);
      const float4 f1 = *reinterpret_cast<const float4*>(src + 4);
      v.x = (uint32_t)f32_to_bf16(f0.x) | ((uint32_t)f32_to_bf16(f0.y) << 16);
      v.y = (uint32_t)f32_to_bf16(f0.z) | ((uint32_t)f32_to_bf16(f0.w) << 16);
      v.z = (uint32_t)f32_to_bf16(f1.x) | ((uint32_t)f32_to_bf16(f1.y) << 16);
      v.w = (uint32_t)f32_to_bf16(f1.z) | ((uint32_t)f32_to_bf16(f1.w) << 16);
    }
    return v;
  };
  __syncthreads();  // zeroing done before the first staged row lands
  if (stager) *reinterpret_cast<uint4*>(XB(0) + my_rr * XS + my_c * 8) = load_x(0);

  float hs0[HTW][RT][4], hs1[HTW][RT][4];
#pragma unroll
  for (int i = 0; i < HTW; ++i)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) hs0[i][rt][r] = hs1[i][rt][r] = 0.f;
  __syncthreads();

  for (int t = 0; t < a.T; ++t) {
    const int pb = t & 1, nb = pb ^ 1;
    const uint4 xn = (t + 1 < a.T) ? load_x(t + 1) : make_uint4(0, 0, 0, 0);
    layer_step<RT, KSX, KSH, LBR, NW>(w0, r0, bias, XB(pb), XS, HB(0, pb), HB(0, nb), rb, hs0, lane, wave);
    __syncthreads();
    if (a.n_layers == 2) {
      layer_step<RT, KSH, KSH, LBR, NW>(w1, r1, bias + 6 * H, HB(0, nb), HS, HB(1, pb), HB(1, nb), rb, hs1, lane,
                                        wave);
    }
    if (stager && t + 1 < a.T) *reinterpret_cast<uint4*>(XB(nb) + my_rr * XS + my_c * 8) = xn;
    __syncthreads();
  }

  // ---- outputs from the last layer's registers (static register indexing in both branches)
  if (a.n_layers == 2)
    emit_outputs<RT, KSH, NW>(a, hs1, red, row0, n_live, lane, wave, tid);
  else
    emit_outputs<RT, KSH, NW>(a, hs0, red, row0, n_live, lane, wave, tid);
#undef HB
#undef XB
}

// Batch-parallel recurrence in split mode (layer_step_x3): the same structure as gru_kernel,
// with every LDS activation tile doubled into hi / lo halves (16 rows per workgroup keeps it
// within the LDS: ~96 KB at H = 256).
template <int RT, int KSX, int KSH, int LBR, int NW>
__global__ void __launch_bounds__(NW * 64) gru_x3_kernel(GruArgs a) {
  constexpr int M = RT * 16;
  constexpr int H = KSH * 32;
  constexpr int HS = H + GRU_PAD;
  constexpr int XS = KSX * 32 + GRU_PAD;
  constexpr int HTW = KSH * 2 / NW;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  const int row0 = blockIdx.x * M;
  if (row0 >= n_live) return;
  const size_t wx = (size_t)3 * H * KSX * 32, wh = (size_t)3 * H * H;
  const WFrag w0 = wfrag(a.layer[0].W, wx, lane), w0l = wfrag(a.layer[0].W_lo, wx, lane);
  const WFrag r0 = wfrag(a.layer[0].R, wh, lane), r0l = wfrag(a.layer[0].R_lo, wh, lane);
  const WFrag w1 = wfrag(a.layer[1].W, wh, lane), w1l = wfrag(a.layer[1].W_lo, wh, lane);
  const WFrag r1 = wfrag(a.layer[1].R, wh, lane), r1l = wfrag(a.layer[1].R_lo, wh, lane);

  // LDS: hb[2 halves][layer][pingpong][M][HS] | xb[2 halves][pingpong][M][XS] | rb[2 halves][M][HS]
  //      (LBR = 0 only) | bias[2][6H] | red[NW][M]
  uint16_t* const hb = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const xb = hb + 8 * M * HS;
  uint16_t* const rb = xb + 4 * M * XS;
  float* const bias = reinterpret_cast<float*>(rb + (LBR ? 0 : 2 * M * HS));
  float* const red = bias + 12 * H;
#define HB(half, l, b) (hb + ((half) * 4 + (l) * 2 + (b)) * (M * HS))
#define XB(half, b) (xb + ((half) * 2 + (b)) * (M * XS))
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(smem);
    const int words = (8 * M * HS + 4 * M * XS) / 2;
    for (int i = tid; i < words; i += NT) z[i] = 0u;
  }
  for (int i = tid; i < 6 * H; i += NT) bias[i] = a.layer[0].bias[i];
  if (a.n_layers == 2)
    for (int i = tid; i < 6 * H; i += NT) bias[6 * H + i] = a.layer[1].bias[i];

  const int I = a.I;
  const int chunks = I >> 3;
  const int my_rr = tid / max(chunks, 1), my_c = tid - my_rr * max(chunks, 1);
  const bool stager = chunks > 0 && my_rr < M;
  const int grow = row0 + my_rr;
  int slot = -1, head = 0, valid_from = a.T;
  if (stager && grow < n_live) {
    if (a.mode == 1) {
      slot = a.slots[grow];
      if (slot >= 0) {
        const AcctRT r = a.rt[slot];
        head = r.ev_head;
        valid_from = a.T - min(r.ev_count, a.T);
      }
    } else {
      valid_from = 0;
    }
  }
  // x_t as (hi, lo) bf16 halves: the event ring holds bf16 values (lo = 0); dense f32 input splits
  auto load_x = [&](int t, uint4& hi, uint4& lo) {
    hi = lo = make_uint4(0, 0, 0, 0);
    if (t >= a.T) return;
    if (a.reverse) t = a.T - 1 - t;
    if (!stager || t < valid_from) return;
    if (a.mode == 1) {
      int idx = (head - a.T + t) % a.ev_ring;
      if (idx < 0) idx += a.ev_ring;
      hi = *reinterpret_cast<const uint4*>(a.ev + (((size_t)slot * a.ev_ring + idx) * I + my_c * 8));
    } else {
      const float* src = a.X + (((size_t)t * a.x_rows + grow) * I + my_c * 8);
      uint16_t h8[8], l8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) gru_split(src[e], h8[e], l8[e]);
      hi = make_uint4(h8[0] | (uint32_t)h8[1] << 16, h8[2] | (uint32_t)h8[3] << 16, h8[4] | (uint32_t)h8[5] << 16,
                      h8[6] | (uint32_t)h8[7] << 16);
      lo = make_uint4(l8[0] | (uint32_t)l8[1] << 16, l8[2] | (uint32_t)l8[3] << 16, l8[4] | (uint32_t)l8[5] << 16,
                      l8[6] | (uint32_t)l8[7] << 16);
    }
  };
  __syncthreads();
  if (stager) {
    uint4 h, l;
    load_x(0, h, l);
    *reinterpret_cast<uint4*>(XB(0, 0) + my_rr * XS + my_c * 8) = h;
    *reinterpret_cast<uint4*>(XB(1, 0) + my_rr * XS + my_c * 8) = l;
  }
  float hs0[HTW][RT][4], hs1[HTW][RT][4];
#pragma unroll
  for (int i = 0; i < HTW; ++i)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) hs0[i][rt][r] = hs1[i][rt][r] = 0.f;
  __syncthreads();

  for (int t = 0; t < a.T; ++t) {
    const int pb = t & 1, nb = pb ^ 1;
    uint4 xh, xl;
    load_x(t + 1, xh, xl);
    layer_step_x3<RT, KSX, KSH, LBR, NW>(w0, w0l, r0, r0l, bias, XB(0, pb), XB(1, pb), XS, HB(0, 0, pb), HB(1, 0, pb),
                                         HB(0, 0, nb), HB(1, 0, nb), rb, rb + M * HS, hs0, lane, wave);
    __syncthreads();
    if (a.n_layers == 2) {
      layer_step_x3<RT, KSH, KSH, LBR, NW>(w1, w1l, r1, r1l, bias + 6 * H, HB(0, 0, nb), HB(1, 0, nb), HS,
                                           HB(0, 1, pb), HB(1, 1, pb), HB(0, 1, nb), HB(1, 1, nb), rb, rb + M * HS,
                                           hs1, lane, wave);
    }
    if (stager && t + 1 < a.T) {
      *reinterpret_cast<uint4*>(XB(0, nb) + my_rr * XS + my_c * 8) = xh;
      *reinterpret_cast<uint4*>(XB(1, nb) + my_rr * XS + my_c * 8) = xl;
    }
    __syncthreads();
  }
  if (a.n_layers == 2)
    emit_outputs<RT, KSH, NW>(a, hs1, red, row0, n_live, lane, wave, tid);
  else
    emit_outputs<RT, KSH, NW>(a, hs0, red, row0, n_live, lane, wave, tid);
#undef HB
#undef XB
}

static size_t gru_x3_lds_bytes(int RT, int KSX, int KSH, int NW, int lbr) {
  const int M = RT * 16, H = KSH * 32, HS = H + GRU_PAD, XS = KSX * 32 + GRU_PAD;
  return (size_t)8 * M * HS * 2 + (size_t)4 * M * XS * 2 + (lbr ? 0 : (size_t)2 * M * HS * 2) +
         (size_t)2 * 6 * H * 4 + (size_t)NW * M * 4;
}

// rows per workgroup (GruArgs.tile_rows: 0 / 16 -> 16): 32 rows (RT = 2, linear_before_reset, tiles
// within the LDS: 155 KB at H = 256) feed every streamed hi / lo weight fragment to two row
// tiles; a 4096-row batch then fills 128 CUs, which pays only when another slot's batch runs
// beside it (the cfg5 bench's per-slot streams, engine/abuse.py overlap).
template <int KSX, int KSH>
static void launch_gru_x3(const GruArgs& a, hipStream_t st) {
  constexpr int NW = KSH >= 4 ? 8 : 4;
  const dim3 block(NW * 64);
  const int lbr = a.layer[0].lbr ? 1 : 0;
  if constexpr (KSH == 8) {
    // H = 256: 16 waves (one hidden tile each, four waves per SIMD) keep twice the weight loads
    // in flight per CU at the same LDS footprint: +16 % at 16 rows on one stream, +3-8 % at 32
    // rows with the slots' streams overlapped (tools/gru_x3_bench.py, profiles/r4/m); waves = 8
    // keeps the 8-wave kernel
    if (a.waves != 8 && lbr) {
      const int rt = a.tile_rows == 32 ? 2 : 1;
      const size_t lds = gru_x3_lds_bytes(rt, KSX, KSH, 16, 1);
      if (rt == 2 && lds <= 160 * 1024) {
        IGP_LAUNCH((gru_x3_kernel<2, KSX, KSH, 1, 16>), dim3((a.n_rows + 31) / 32), dim3(1024), lds, st, a);
        return;
      }
      if (rt == 1) {
        IGP_LAUNCH((gru_x3_kernel<1, KSX, KSH, 1, 16>), dim3((a.n_rows + 15) / 16), dim3(1024), lds, st, a);
        return;
      }
    }
  }
  if (lbr && a.tile_rows == 32 && gru_x3_lds_bytes(2, KSX, KSH, NW, 1) <= 160 * 1024) {
    IGP_LAUNCH((gru_x3_kernel<2, KSX, KSH, 1, NW>), dim3((a.n_rows + 31) / 32), block,
               gru_x3_lds_bytes(2, KSX, KSH, NW, 1), st, a);
    return;
  }
  const dim3 grid((a.n_rows + 15) / 16);
  const size_t lds = gru_x3_lds_bytes(1, KSX, KSH, NW, lbr);
  if (lbr)
    IGP_LAUNCH((gru_x3_kernel<1, KSX, KSH, 1, NW>), grid, block, lds, st, a);
  else
    IGP_LAUNCH((gru_x3_kernel<1, KSX, KSH, 0, NW>), grid, block, lds, st, a);
}

// Two stacked layers, layer-pipelined: waves [0, NW/2) run layer 1 at step t while waves
// [NW/2, NW) run layer 2 at step t-1 (it needs h1_{t-1} and h2_{t-2}, both complete after the
// previous barrier). The two layers' weight-fragment load chains overlap and each step costs
// one block barrier. Buffers: H1[s] lives in hb1[(s+1)&1], H2[s] in hb2[(s+1)&1], H[-1] = 0.
template <int RT, int KSX, int KSH, int LBR, int NW>
__global__ void __launch_bounds__(NW * 64) gru2_pipe_kernel(GruArgs a) {
  constexpr int M = RT * 16;
  constexpr int H = KSH * 32;
  constexpr int HS = H + GRU_PAD;
  constexpr int XS = KSX * 32 + GRU_PAD;
  constexpr int NWL = NW / 2;               // waves per layer
  constexpr int HTW = KSH * 2 / NWL;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int layer = wave / NWL, lw = wave - layer * NWL;   // wave-uniform
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  const int row0 = blockIdx.x * M;
  if (row0 >= n_live) return;
  const WFrag w0 = wfrag(a.layer[0].W, (size_t)3 * H * KSX * 32, lane), r0 = wfrag(a.layer[0].R, (size_t)3 * H * H, lane);
  const WFrag w1 = wfrag(a.layer[1].W, (size_t)3 * H * H, lane), r1 = wfrag(a.layer[1].R, (size_t)3 * H * H, lane);

  // LDS: hb[layer][pingpong][M][HS] | xb[2][M][XS] | rb[layer][M][HS] | bias[2][6H] | red[NWL][M]
  uint16_t* const hb = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const xb = hb + 4 * M * HS;
  uint16_t* const rb = xb + 2 * M * XS;
  float* const bias = reinterpret_cast<float*>(rb + 2 * M * HS);
  float* const red = bias + 12 * H;
#define HB(l, b) (hb + ((l) * 2 + (b)) * (M * HS))
#define XB(b) (xb + (b) * (M * XS))
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(smem);
    const int words = (4 * M * HS + 2 * M * XS) / 2;
    for (int i = tid; i < words; i += NT) z[i] = 0u;
  }
  for (int i = tid; i < 6 * H; i += NT) {
    bias[i] = a.layer[0].bias[i];
    bias[6 * H + i] = a.layer[1].bias[i];
  }
  const int I = a.I;
  const int chunks = I >> 3;
  const int my_rr = tid / max(chunks, 1), my_c = tid - my_rr * max(chunks, 1);
  const bool stager = chunks > 0 && my_rr < M;
  const int grow = row0 + my_rr;
  int slot = -1, head = 0, valid_from = a.T;
  if (stager && grow < n_live) {
    if (a.mode == 1) {
      slot = a.slots[grow];
      if (slot >= 0) {
        const AcctRT r = a.rt[slot];
        head = r.ev_head;
        valid_from = a.T - min(r.ev_count, a.T);
      }
    } else {
      valid_from = 0;
    }
  }
  auto load_x = [&](int t) -> uint4 {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t >= a.T) return v;
    if (a.reverse) t = a.T - 1 - t;
    if (!stager || t < valid_from) return v;
    if (a.mode == 1) {
      int idx = (head - a.T + t) % a.ev_ring;
      if (idx < 0) idx += a.ev_ring;
      v = *reinterpret_cast<const uint4*>(a.ev + (((size_t)slot * a.ev_ring + idx) * I + my_c * 8));
    } else {
      const float* src = a.X + (((size_t)t * a.x_rows + grow) * I + my_c * 8);
      const float4 f0 = *reinterpret_cast<const float4*>(src);
      const float4 f1 = *reinterpret_cast<const float4*>(src + 4);
      v.x = (uint32_t)f32_to_bf16(f0.x) | ((uint32_t)f32_to_bf16(f0.y) << 16);
      v.y = (uint32_t)f32_to_bf16(f0.z) | ((uint32_t)f32_to_bf16(f0.w) << 16);
      v.z = (uint32_t)f32_to_bf16(f1.x) | ((uint32_t)f32_to_bf16(f1.y) << 16);
      v.w = (uint32_t)f32_to_bf16(f1.z) | ((uint32_t)f32_to_bf16(f1.w) << 16);
    }
    return v;
  };
  __syncthreads();
  if (stager) *reinterpret_cast<uint4*>(XB(0) + my_rr * XS + my_c * 8) = load_x(0);
  float hs[HTW][RT][4];
#pragma unroll
  for (int i = 0; i < HTW; ++i)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) hs[i][rt][r] = 0.f;
  __syncthreads();

  for (int t = 0; t <= a.T; ++t) {
    const uint4 xn = load_x(t + 1);
    if (layer == 0) {
      if (t < a.T)  // H1[t] from x_t and H1[t-1]
        layer_step<RT, KSX, KSH, LBR, NWL>(w0, r0, bias, XB(t & 1), XS, HB(0, t & 1), HB(0, (t + 1) & 1),
                                           rb, hs, lane, lw);
      else if (LBR == 0)
        __syncthreads();  // match the other half's internal barrier
    } else {
      if (t >= 1)   // H2[t-1] from H1[t-1] and H2[t-2]
        layer_step<RT, KSH, KSH, LBR, NWL>(w1, r1, bias + 6 * H, HB(0, t & 1), HS, HB(1, (t - 1) & 1),
                                           HB(1, t & 1), rb + M * HS, hs, lane, lw);
      else if (LBR == 0)
        __syncthreads();
    }
    if (stager && t + 1 < a.T) *reinterpret_cast<uint4*>(XB((t + 1) & 1) + my_rr * XS + my_c * 8) = xn;
    __syncthreads();
  }

  // ---- outputs: H2[T-1] in the layer-2 waves' registers
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  if (layer == 1 && a.yh) {
#pragma unroll
    for (int i = 0; i < HTW; ++i)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = row0 + rt * 16 + crow + r;
          if (row < n_live) a.yh[(size_t)row * H + (lw + NWL * i) * 16 + ccol] = hs[i][rt][r];
        }
  }
  if (a.head_w) {
    if (layer == 1) {
      float part[RT][4];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[rt][r] = 0.f;
#pragma unroll
      for (int i = 0; i < HTW; ++i) {
        const float w = a.head_w[(lw + NWL * i) * 16 + ccol];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) part[rt][r] += hs[i][rt][r] * w;
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = part[rt][r];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
          if (ccol == 0) red[lw * M + rt * 16 + crow + r] = v;
        }
    }
    __syncthreads();
    if (tid < M && row0 + tid < n_live) {
      float v = a.head_b;
#pragma unroll
      for (int w = 0; w < NWL; ++w) v += red[w * M + tid];
      if (a.head_act == 2) v = 1.f / (1.f + expf(-v));
      a.out[row0 + tid] = v;
    }
  }
#undef HB
#undef XB
}

static size_t gru_pipe_lds_bytes(int RT, int KSX, int KSH, int NW) {
  const int M = RT * 16, H = KSH * 32, HS = H + GRU_PAD, XS = KSX * 32 + GRU_PAD;
  return (size_t)4 * M * HS * 2 + (size_t)2 * M * XS * 2 + (size_t)2 * M * HS * 2 + (size_t)2 * 6 * H * 4 +
         (size_t)NW * M * 4;
}

static size_t gru_lds_bytes(int RT, int KSX, int KSH, int NW) {
  const int M = RT * 16, H = KSH * 32, HS = H + GRU_PAD, XS = KSX * 32 + GRU_PAD;
  return (size_t)4 * M * HS * 2 + (size_t)2 * M * XS * 2 + (size_t)M * HS * 2 + (size_t)2 * 6 * H * 4 +
         (size_t)NW * M * 4;
}

template <int RT, int KSX, int KSH, int NW>
static void launch_gru_w(const GruArgs& a, hipStream_t st) {
  const int M = RT * 16;
  const dim3 grid((a.n_rows + M - 1) / M), block(NW * 64);
  const size_t lds = gru_lds_bytes(RT, KSX, KSH, NW);
  if (a.layer[0].lbr)
    IGP_LAUNCH((gru_kernel<RT, KSX, KSH, 1, NW>), grid, block, lds, st, a);
  else
    IGP_LAUNCH((gru_kernel<RT, KSX, KSH, 0, NW>), grid, block, lds, st, a);
}

template <int RT, int KSX, int KSH, int NW>
static void launch_gru_pipe(const GruArgs& a, hipStream_t st) {
  const int M = RT * 16;
  const dim3 grid((a.n_rows + M - 1) / M), block(NW * 64);
  const size_t lds = gru_pipe_lds_bytes(RT, KSX, KSH, NW);
  if (a.layer[0].lbr)
    IGP_LAUNCH((gru2_pipe_kernel<RT, KSX, KSH, 1, NW>), grid, block, lds, st, a);
  else
    IGP_LAUNCH((gru2_pipe_kernel<RT, KSX, KSH, 0, NW>), grid, block, lds, st, a);
}

template <int RT, int KSX, int KSH>
static void launch_gru_t(const GruArgs& a, hipStream_t st) {
  if (a.n_layers == 2 && a.pipeline) {
    // 2 hidden tiles per wave: H/32 waves per layer (H=256: 16 waves = 1024 threads)
    if constexpr (KSH == 8) {
      return launch_gru_pipe<RT, KSX, KSH, 16>(a, st);
    } else if constexpr (KSH == 4) {
      return launch_gru_pipe<RT, KSX, KSH, 8>(a, st);
    } else {
      return launch_gru_pipe<RT, KSX, KSH, 4>(a, st);
    }
  }
  if constexpr (KSH >= 4) {  // 8 waves: 2 hidden tiles per wave (measured faster than 4 for H >= 128)
    if (a.waves != 4) return launch_gru_w<RT, KSX, KSH, 8>(a, st);
  }
  launch_gru_w<RT, KSX, KSH, 4>(a, st);
}

template <int RT, int KSX>
static void launch_gru_h(const GruArgs& a, hipStream_t st) {
  switch (a.H) {
    case 64: launch_gru_t<RT, KSX, 2>(a, st); break;
    case 128: launch_gru_t<RT, KSX, 4>(a, st); break;
    case 256: launch_gru_t<RT, KSX, 8>(a, st); break;
    default: break;
  }
}

void launch_gru(const GruArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return;
  static int n_cu = [] {
    int dev = 0, v = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  if (a.split) {
    // small micro-batches: the weight-stationary split clusters (16 workgroups per 32 rows, a
    // whole CU each), while a launch takes at most half the chip (the serving abuse device runs
    // them on one stream, so the scorer's kernels keep the other half and every cluster becomes
    // resident; its bounded waits only guard against what cannot); larger ones: the
    // batch-parallel split kernel
    if (a.ws && gru_wsx_eligible(a) && gru_wsx_clusters(a.n_rows) * 16 <= n_cu / 2) {
      return launch_gru_wsx(a, st);
    }
    const int ksx = a.layer[0].kx_pad / 32;
    switch (a.H) {
      case 64: if (ksx == 1) launch_gru_x3<1, 2>(a, st); else launch_gru_x3<2, 2>(a, st); break;
      case 128: if (ksx == 1) launch_gru_x3<1, 4>(a, st); else launch_gru_x3<2, 4>(a, st); break;
      default: if (ksx == 1) launch_gru_x3<1, 8>(a, st); else launch_gru_x3<2, 8>(a, st); break;
    }
    return;
  }
  // weight-stationary clusters while all of them fit one wave of the chip (1 workgroup per CU);
  // beyond that the batch-parallel kernel at 32 rows per workgroup streams weights at a better
  // rate than two waves of clusters (tools/gru_bench.py: 8192 rows 5.6 M vs 4.5 M seq/s)
  if (a.ws && gru_ws_eligible(a)) {
    // ws = 3: two 64-row clusters per CU (all co-resident at <= 2 workgroups per CU)
    if (a.ws == 3 ? gru_ws2_clusters(a.n_rows) * 8 <= 2 * n_cu : gru_ws_clusters(a.n_rows) * 8 <= n_cu) {
      return launch_gru_ws(a, st);
    }
  }
  // rows per workgroup: every CU streams the full weight set each step (a per-CU L2 bandwidth
  // bound, tools/gru_bench.py), so 32 rows amortise each fragment over two MFMA row tiles once
  // the batch fills the 256 CUs at 32 rows; below that 16 keeps more CUs streaming.
  const int tr = a.tile_rows ? a.tile_rows : (a.n_rows >= 32 * 256 ? 32 : 16);
  const int ksx = a.layer[0].kx_pad / 32;
  if (tr == 32) {
    if (ksx == 1) launch_gru_h<2, 1>(a, st); else launch_gru_h<2, 2>(a, st);
  } else {
    if (ksx == 1) launch_gru_h<1, 1>(a, st); else launch_gru_h<1, 2>(a, st);
  }
}

}  // namespace igp
