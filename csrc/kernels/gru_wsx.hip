// K4-WSX: f32-faithful weight-stationary GRU for small micro-batches (CheckBonusAbuse latency,
// VERDICT r4 item 7). The cfg5 shape - 2 stacked layers, H = 256, linear_before_reset = 1,
// input width <= 32 - in split mode: weights and activations as bf16 pairs hi + lo, three MFMAs
// per product (lo*hi + hi*lo + hi*hi, the order of gru.hip layer_step_x3), f32 hidden state.
//
// Why: the batch-parallel split kernel (gru_x3_kernel) streams all 2.4 MB of hi + lo weights
// from L2 through every workgroup on every step - ~20 us per step whatever the batch, so a call
// of one row still waits 2+ ms for its 100 steps. Here the weights never move and a step costs
// one short MFMA chain plus one cluster hand-off:
//
//   cluster  = 16 workgroups with equal blockIdx % 8 (one XCD under round-robin placement: the
//              hand-off then stays in that XCD's L2) that own 32 sequences together;
//   member m = hidden units [16m, 16m + 16) of BOTH layers. Its four waves split K: wave
//              (layer l, half k) keeps the hi and lo B fragments of its k-steps in registers
//              (layer 1: x + h k-steps 0..3 | h k-steps 4..7; layer 2: the input part h1 | the
//              recurrent part h2, 8 k-steps each = 192 registers) and accumulates partial gate
//              sums (z, r, input part of h~, recurrent part of h~) for the 32 rows;
//   combine  = the k-half-0 wave hands its partials over LDS to the k-half-1 wave, which adds
//              them, applies the gates and keeps the f32 state of its 16 columns;
//   hand-off = each member publishes its 16 columns of h1_t and h2_{t-1} as hi / lo bf16 (4 KB,
//              one 16-B sc1 store per thread) and gathers the other 15 slices straight into its
//              LDS images (global_load_lds, 15 per wave).
// The layers are pipelined (layer 1 at step t, layer 2 at step t-1: both read h1_{t-1}), so a
// step is ONE hand-off. Counters, bounded waits (a cluster that is not co-resident sets
// *ws_err, every wave exits, outputs stay NaN and the host falls back to gru_x3) and the final
// counter reset follow gru_ws.hip.
#include "common.h"
#include "launch.h"

namespace igp {
namespace {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int X_CL = 16;                 // member workgroups per cluster
constexpr int X_M = 32;                  // sequences per cluster
constexpr int X_RT = X_M / 16;           // MFMA row tiles
constexpr int X_H = 256;
constexpr int X_HT = X_H / 16;           // hidden tiles (= members)
constexpr int X_XS = 32 + 8;             // LDS row stride of the input tile (bf16)
constexpr int X_BLK = X_M * 16;          // bf16 per (image, member) block: 32 rows x 16 columns
constexpr int X_IMG = X_CL * X_BLK;      // bf16 per image (h1 hi, h1 lo, h2 hi, h2 lo)
constexpr int X_SLICE = 4 * X_BLK;       // bf16 per member slice (its block of the 4 images)
constexpr uint64_t X_WAIT_TICKS = 20000000;  // 200 ms of wall_clock64 (100 MHz): never hang the GPU
constexpr int X_SC1 = 16;                // buffer aux bit: sc1 (L2-coherent, bypasses L1)

// v_exp_f32 + v_rcp_f32 (1 ulp, as gru_ws.hip): the IEEE divide sequence made the gate epilogue
// (24 divides per lane per step) as long as the step's MFMAs (tools/gru_wsx_trace.py)
__device__ __forceinline__ float xsig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float xtanh(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f); }

__device__ __forceinline__ void xsplit(float x, uint16_t& hi, uint16_t& lo) {
  hi = f32_to_bf16(x);
  lo = f32_to_bf16(x - __uint_as_float((uint32_t)hi << 16));
}

// 16-B chunk (row, q) of a 32 x 16 block: rows 8..15 of a row tile swap their two chunks, so a
// 16-row A-fragment read (one chunk per lane) covers all 64 banks once
__device__ __forceinline__ int xchunk(int row, int q) { return row * 2 + (q ^ ((row >> 3) & 1)); }

// packed fragment (nt, ks) of a [N/16][KS][64][8] bf16 weight (ops/kernels.py pack_fragments)
__device__ __forceinline__ bf16x8 xwfrag(const uint16_t* p, int nt, int KS, int ks, int lane) {
  const uint4 v = *reinterpret_cast<const uint4*>(p + (((size_t)nt * KS + ks) * 64 + lane) * 8);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 xlds(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}

#define XMMA3(acc, ah, al, bh, bl)                                         \
  do {                                                                     \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);   \
  } while (0)

// bounded poll of the cluster counter by one lane; false on timeout, after poisoning the
// counter (gru.hip kClusterPoison): the members still to arrive and every launch queued behind
// this one then fail their waits too instead of passing them early on a part-advanced count
__device__ __forceinline__ bool xwait(int32_t* cnt, int target) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    for (int n = 0; n < 64; ++n) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
      __builtin_amdgcn_s_sleep(1);
    }
    if (wall_clock64() - t0 > X_WAIT_TICKS) {
      __hip_atomic_exchange(cnt, kClusterPoison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

// a wave's role: layer L, K half KH; NK k-steps; KX of them (the first) read the input part
template <int L, int KH>
struct XRole {
  static constexpr int layer = L, half = KH;
  static constexpr int NK = L == 0 ? (KH == 0 ? 5 : 4) : 8;
  // k-steps of this role that multiply the input (x for layer 1, h1 for layer 2): they feed the
  // input half of h~ (linear_before_reset); the rest feed the recurrent half
  static constexpr int KX = L == 0 ? (KH == 0 ? 1 : 0) : (KH == 0 ? 8 : 0);
};

__global__ void __launch_bounds__(256, 1) gru_wsx_kernel(GruArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: IMG[4][X_IMG] bf16 (h1 hi, h1 lo, h2 hi, h2 lo) | X[2 buf][2 part][M][XS] bf16 |
  //      PZ[2 layers][RT][4 groups][64 lanes] f32x4 | red[M] f32 | xmeta[4M] int2 | flag
  uint16_t* const IMG = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const XB = IMG + 4 * X_IMG;
  f32x4* const PZ = reinterpret_cast<f32x4*>(XB + 2 * 2 * X_M * X_XS);
  float* const red = reinterpret_cast<float*>(PZ + 2 * X_RT * 4 * 64);
  int2* const xmeta = reinterpret_cast<int2*>(red + X_M);
  int* const sflag = reinterpret_cast<int*>(xmeta + 4 * X_M);

  const int b = blockIdx.x;
  const int mem = (b >> 3) & (X_CL - 1);           // member: hidden units [16 mem, 16 mem + 16)
  const int cl = (b >> 7) * 8 + (b & 7);           // cluster: members share blockIdx % 8
  const int row0 = cl * X_M;
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  if (row0 >= n_live || cl >= a.ws_clusters) return;  // uniform over the cluster's 16 members
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  const int j = mem * 16 + ccol;                   // this lane's hidden unit (epilogue)
  const int T = a.T;
  int32_t* const cnt = a.ws_sync + cl * 16;
  // outputs start as NaN: a cluster that gives up (bounded wait) leaves them so, and the host
  // detects it instead of reading the previous batch's values
  if (a.head_w && mem == 0 && tid < X_M && row0 + tid < n_live) a.out[row0 + tid] = __builtin_nanf("");
  if (a.yh)
    for (int e = tid; e < X_M * 16; e += 256) {
      const int row = row0 + e / 16;
      if (row < n_live) a.yh[(size_t)row * X_H + mem * 16 + e % 16] = __builtin_nanf("");
    }
  {  // h_{-1} = 0 in every image; input columns past I stay zero
    uint32_t* z = reinterpret_cast<uint32_t*>(smem);
    const int words = (4 * X_IMG + 2 * 2 * X_M * X_XS) / 2;
    for (int i = tid; i < words; i += 256) z[i] = 0u;
  }
  // ---- layer-1 input chunks (row, 8-element piece): event-ring slot / head / first valid step
  const int I = a.I;
  const int chunks = I >> 3;  // 1..4
  const int nchunk = X_M * chunks;  // <= 128: one per thread of the two layer-1 waves
  for (int c = tid; c < nchunk; c += 256) {
    const int grow = row0 + c / chunks;
    int slot = -1, head = 0, from = T;
    if (grow < n_live) {
      if (a.mode == 1) {
        slot = a.slots[grow];
        if (slot >= 0) {
          const AcctRT r = a.rt[slot];
          head = r.ev_head;
          from = T - min(r.ev_count, T);
        }
      } else {
        from = 0;
      }
    }
    xmeta[c] = make_int2(slot, head | (from << 16));
  }
  // x_t chunk c as (hi, lo) bf16 x 8: event rings hold bf16 (lo = 0); dense f32 input is split
  auto load_x = [&](int c, int t, uint4& hi, uint4& lo) {
    hi = lo = make_uint4(0, 0, 0, 0);
    const int2 m = xmeta[c];
    const int from = m.y >> 16;
    if (t >= T) return;
    if (a.reverse) t = T - 1 - t;  // direction=reverse: forward over the time-reversed sequence
    if (t < from) return;
    const int row = c / chunks, q = c - row * chunks;
    if (a.mode == 1) {
      if (m.x < 0) return;
      int idx = ((m.y & 0xffff) - T + t) % a.ev_ring;
      if (idx < 0) idx += a.ev_ring;
      hi = *reinterpret_cast<const uint4*>(a.ev + (((size_t)m.x * a.ev_ring + idx) * I + q * 8));
    } else {
      const float* src = a.X + (((size_t)t * a.x_rows + row0 + row) * I + q * 8);
      const float4 f0 = *reinterpret_cast<const float4*>(src);
      const float4 f1 = *reinterpret_cast<const float4*>(src + 4);
      const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      uint16_t h[8], l[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) xsplit(f[e], h[e], l[e]);
      hi = make_uint4(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16), h[4] | ((uint32_t)h[5] << 16),
                      h[6] | ((uint32_t)h[7] << 16));
      lo = make_uint4(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16), l[4] | ((uint32_t)l[5] << 16),
                      l[6] | ((uint32_t)l[7] << 16));
    }
  };
  auto x_slot = [&](int buf, int part, int c) -> uint4* {
    const int row = c / chunks, q = c - row * chunks;
    return reinterpret_cast<uint4*>(XB + (buf * 2 + part) * (X_M * X_XS) + row * X_XS + q * 8);
  };
  __syncthreads();
  const int layer = wave >> 1, kh = wave & 1;
  const int ltid = kh * 64 + lane;  // thread index among the two waves of this layer
  if (layer == 0 && ltid < nchunk) {
    uint4 hi, lo;
    load_x(ltid, 0, hi, lo);
    *x_slot(0, 0, ltid) = hi;
    *x_slot(0, 1, ltid) = lo;
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      a.ws_x + (size_t)cl * 2 * X_CL * X_SLICE, 0, 2 * X_CL * X_SLICE * 2, 0x00020000);
  const uint16_t* const slab = a.ws_x + (size_t)cl * 2 * X_CL * X_SLICE;

  // the recurrence, specialised per role: each wave runs exactly one instantiation (one set of
  // stationary weights in its registers); all of them execute the same barrier sequence
  auto run = [&](auto role) -> bool {
    using R = decltype(role);
    constexpr int L = R::layer, KH = R::half, NK = R::NK, KX = R::KX;
    bf16x8 wzh[NK], wzl[NK], wrh[NK], wrl[NK], whh[NK], whl[NK];
    {
      const GruLayerArgs& la = a.layer[L];
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        // the weight matrix and k-step behind local k-step i (see XRole)
        const bool isW = (L == 0) ? (KH == 0 && i == 0) : (KH == 0);
        const uint16_t* ph = isW ? la.W : la.R;
        const uint16_t* pl = isW ? la.W_lo : la.R_lo;
        const int KS = (L == 0 && isW) ? 1 : 8;
        const int ks = (L == 0) ? (KH == 0 ? (i == 0 ? 0 : i - 1) : 4 + i) : i;
        wzh[i] = xwfrag(ph, mem, KS, ks, lane);
        wzl[i] = xwfrag(pl, mem, KS, ks, lane);
        wrh[i] = xwfrag(ph, X_HT + mem, KS, ks, lane);
        wrl[i] = xwfrag(pl, X_HT + mem, KS, ks, lane);
        whh[i] = xwfrag(ph, 2 * X_HT + mem, KS, ks, lane);
        whl[i] = xwfrag(pl, 2 * X_HT + mem, KS, ks, lane);
      }
    }
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (KH == 1) {
      const float* bs = a.layer[L].bias;  // Wb z,r,h | Rb z,r,h
      bv[0] = bs[j] + bs[3 * X_H + j];
      bv[1] = bs[X_H + j] + bs[4 * X_H + j];
      bv[2] = bs[2 * X_H + j];
      bv[3] = bs[5 * X_H + j];
    }
    float hs[X_RT][4];
#pragma unroll
    for (int rt = 0; rt < X_RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) hs[rt][r] = 0.f;
    // A fragments of local k-step i, row tile rt: (hi, lo)
    const int arow = lane & 15, aq = (lane >> 4) & 1, amem_off = lane >> 5;
    auto afrag = [&](int i, int rt, bf16x8& ah, bf16x8& al, int xb) {
      const int row = rt * 16 + arow;
      if (L == 0 && KH == 0 && i == 0) {  // x_t: [M][XS] hi / lo
        const uint16_t* p = XB + (xb * 2) * (X_M * X_XS) + row * X_XS + 8 * (lane >> 4);
        ah = xlds(p);
        al = xlds(p + X_M * X_XS);
        return;
      }
      // h k-step kk of image pair `im` (0: h1, 1: h2): members 2 kk, 2 kk + 1
      int kk, im;
      if constexpr (L == 0) {
        kk = KH == 0 ? i - 1 : 4 + i;
        im = 0;
      } else {
        kk = i;
        im = KH;
      }
      const uint16_t* p = IMG + (2 * im) * X_IMG + (2 * kk + amem_off) * X_BLK + xchunk(row, aq) * 8;
      ah = xlds(p);
      al = xlds(p + X_IMG);
    };
    __syncthreads();  // x_0 staged by both layer-1 waves
    // phase marks of workgroup 0 (tools/gru_wsx_trace.py): [t][8] wall_clock64 at step start,
    // MFMAs done (the wave of layer 2, K half 1), barrier A, own columns, published, counter,
    // gathered
    int64_t* const trace = (a.ws_trace && b == 0 && L == 1 && KH == 1 && lane == 0) ? a.ws_trace : nullptr;
#define XMARK(t, k) \
  if (trace && (t) < 64) trace[(t) * 8 + (k)] = (int64_t)wall_clock64()
    uint16_t* const own_hi = IMG + (2 * L) * X_IMG + mem * X_BLK;
    uint16_t* const own_lo = own_hi + X_IMG;
    f32x4* const pz = PZ + L * (X_RT * 4 * 64);

    for (int t = 0; t <= T; ++t) {
      XMARK(t, 0);
      const bool act = L == 0 ? (t < T) : (t >= 1);
      uint4 xh = make_uint4(0, 0, 0, 0), xl = xh;
      if (L == 0 && ltid < nchunk) load_x(ltid, t + 1, xh, xl);
      f32x4 acc[X_RT][4];
#pragma unroll
      for (int rt = 0; rt < X_RT; ++rt)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[rt][g] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (act) {
        // per k-step the three products (lo*hi, hi*lo, hi*hi - the accumulation order of
        // XMMA3 / gru.hip) phase by phase over both row tiles and the three gates: six
        // independent MFMAs between two that share an accumulator
#pragma unroll
        for (int i = 0; i < NK; ++i) {
          bf16x8 ah[X_RT], al[X_RT];
#pragma unroll
          for (int rt = 0; rt < X_RT; ++rt) afrag(i, rt, ah[rt], al[rt], t & 1);
          const int gh = i < KX ? 2 : 3;
#pragma unroll
          for (int ph = 0; ph < 3; ++ph) {
#pragma unroll
            for (int rt = 0; rt < X_RT; ++rt) {
              const bf16x8 A = ph == 0 ? al[rt] : ah[rt];
              const bf16x8 Bz = ph == 1 ? wzl[i] : wzh[i];
              const bf16x8 Br = ph == 1 ? wrl[i] : wrh[i];
              const bf16x8 Bh = ph == 1 ? whl[i] : whh[i];
              acc[rt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bz, acc[rt][0], 0, 0, 0);
              acc[rt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Br, acc[rt][1], 0, 0, 0);
              if (gh == 2) acc[rt][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bh, acc[rt][2], 0, 0, 0);
              else acc[rt][3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bh, acc[rt][3], 0, 0, 0);
            }
          }
        }
        if constexpr (KH == 0) {
#pragma unroll
          for (int rt = 0; rt < X_RT; ++rt)
#pragma unroll
            for (int g = 0; g < 4; ++g) pz[(rt * 4 + g) * 64 + lane] = acc[rt][g];
        }
      }
      if (L == 0 && ltid < nchunk) {
        *x_slot((t + 1) & 1, 0, ltid) = xh;
        *x_slot((t + 1) & 1, 1, ltid) = xl;
      }
      XMARK(t, 1);
      __syncthreads();  // every wave is done reading the images / x_t; the partials are in LDS
      XMARK(t, 2);
      if (KH == 1 && act) {  // combine the two K halves, gates, f32 state, own columns hi / lo
#pragma unroll
        for (int rt = 0; rt < X_RT; ++rt) {
          f32x4 p[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) p[g] = pz[(rt * 4 + g) * 64 + lane];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float z = xsig(acc[rt][0][r] + p[0][r] + bv[0]);
            const float rr = xsig(acc[rt][1][r] + p[1][r] + bv[1]);
            const float hh = xtanh(acc[rt][2][r] + p[2][r] + bv[2] + rr * (acc[rt][3][r] + p[3][r] + bv[3]));
            const float h = (1.f - z) * hh + z * hs[rt][r];
            hs[rt][r] = h;
            const int row = rt * 16 + crow + r;
            const int o = xchunk(row, ccol >> 3) * 8 + (ccol & 7);
            uint16_t vh, vl;
            xsplit(h, vh, vl);
            own_hi[o] = vh;
            own_lo[o] = vl;
          }
        }
      }
      if (t == T) break;
      __syncthreads();  // own columns of both layers in the images
      XMARK(t, 3);
      // publish: this member's block of each image (4 x 1 KB: one 16-B chunk per thread)
      const int par = t & 1;
      {
        const int blk = tid >> 6, ch = tid & 63;
        const uint16_t* src = IMG + blk * X_IMG + mem * X_BLK + ch * 8;
        const u32x4 v = __builtin_bit_cast(u32x4, *reinterpret_cast<const uint4*>(src));
        __builtin_amdgcn_raw_buffer_store_b128(v, xr, ch * 16, (((par * X_CL + mem) * 4 + blk) * X_BLK) * 2, X_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      XMARK(t, 4);
      if (tid == 0) {
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = xwait(cnt, X_CL * (t + 1));
        if (!ok) atomicExch(a.ws_err, 1);
        *sflag = ok;
      }
      __syncthreads();
      XMARK(t, 5);
      if (!*sflag) return false;
      // the other 15 members' blocks straight into the images: 60 global_load_lds of 1 KB
      // (15 per wave), sc1 (L2-coherent)
#pragma unroll
      for (int i = 0; i < 15; ++i) {
        const int g = wave * 15 + i;
        const int m2i = g >> 2;
        const int m2 = m2i + (m2i >= mem);
        const int blk = g & 3;
        const uint16_t* src = slab + (size_t)((par * X_CL + m2) * 4 + blk) * X_BLK + lane * 8;
        uint16_t* dst = IMG + blk * X_IMG + m2 * X_BLK;
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                         (__attribute__((address_space(3))) void*)(dst), 16, 0, X_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      XMARK(t, 6);
    }
#undef XMARK
    if constexpr (L == 1 && KH == 1) {  // h2_{T-1} of this member's 16 columns
      if (a.yh) {
#pragma unroll
        for (int rt = 0; rt < X_RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = row0 + rt * 16 + crow + r;
            if (row < n_live) a.yh[(size_t)row * X_H + j] = hs[rt][r];
          }
      }
      if (a.head_w) {
        const float w = a.head_w[j];
#pragma unroll
        for (int rt = 0; rt < X_RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = hs[rt][r] * w;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
            if (ccol == 0) red[rt * 16 + crow + r] = v;
          }
      }
    }
    return true;
  };
  bool ok_run;
  if (layer == 0) ok_run = kh == 0 ? run(XRole<0, 0>{}) : run(XRole<0, 1>{});
  else ok_run = kh == 0 ? run(XRole<1, 0>{}) : run(XRole<1, 1>{});
  if (!ok_run) return;

  float* const part = a.ws_part + (size_t)cl * X_CL * X_M;
  __syncthreads();
  if (a.head_w && tid < X_M) __hip_atomic_store(part + mem * X_M + tid, red[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // final arrival: member 0 waits for all sixteen, combines the head partials in member order,
  // then returns the counter to 0 with an atomic (no member touches it again in this launch)
  if (tid == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true;
    if (mem == 0) {
      ok = xwait(cnt, X_CL * (T + 1));
      if (!ok) atomicExch(a.ws_err, 1);
    }
    *sflag = ok;
  }
  __syncthreads();
  if (mem != 0 || !*sflag) return;
  if (a.head_w && tid < X_M && row0 + tid < n_live) {
    float v = a.head_b;
#pragma unroll
    for (int m2 = 0; m2 < X_CL; ++m2)
      v += __hip_atomic_load(part + m2 * X_M + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.head_act == 2) v = 1.f / (1.f + expf(-v));
    a.out[row0 + tid] = v;
  }
  if (tid == 0) __hip_atomic_exchange(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#undef XMMA3

size_t gru_wsx_lds_bytes() {
  return (size_t)4 * X_IMG * 2 + (size_t)2 * 2 * X_M * X_XS * 2 + (size_t)2 * X_RT * 4 * 64 * 16 + (size_t)X_M * 4 +
         (size_t)4 * X_M * 8 + 16;
}

}  // namespace

int gru_wsx_clusters(int n_rows) { return (n_rows + X_M - 1) / X_M; }

bool gru_wsx_eligible(const GruArgs& a) {
  return a.split && a.ws_x && a.ws_sync && a.ws_err && a.n_layers == 2 && a.H == X_H && a.layer[0].lbr == 1 &&
         a.layer[1].lbr == 1 && a.layer[0].kx_pad == 32 && a.layer[0].W_lo && a.layer[0].R_lo && a.layer[1].W_lo &&
         a.layer[1].R_lo && a.I <= 32 && (a.I & 7) == 0 && a.T >= 1 && a.T < 32768 &&
         (a.mode != 1 || a.ev_ring <= 65535) && (a.head_w == nullptr || a.ws_part != nullptr) &&
         gru_wsx_clusters(a.n_rows) <= a.ws_clusters;
}

// grid: 128 workgroups per 8 clusters (b = 128 q + 8 member + g, cluster = 8 q + g)
void launch_gru_wsx(const GruArgs& a, hipStream_t st) {
  const int ncl = gru_wsx_clusters(a.n_rows);
  IGP_LAUNCH(gru_wsx_kernel, dim3(((ncl + 7) / 8) * 128), dim3(256), gru_wsx_lds_bytes(), st, a);
}

}  // namespace igp
