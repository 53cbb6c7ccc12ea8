// K4-WS: weight-stationary clustered GRU for the config-5 shape (2 stacked layers, H = 256,
// linear_before_reset = 1, input width <= 32) + the fused N=1 head.
//
// Why: the batch-parallel K4 (gru.hip) gives every workgroup 16-32 whole sequences, so every CU
// streams all 1.2 MB of bf16 weights from L2 on every step; at batch 4096 that is a per-CU L2
// bandwidth bound (~12 us per step). Here the weights never move:
//
//   cluster  = 8 workgroups (equal blockIdx % 8: one XCD under round-robin placement, which is
//              only a speed bonus) that own 128 sequences together;
//   member m = hidden units [32m, 32m+32) of BOTH layers; wave w of it = (layer w>>1, hidden tile
//              2m + (w&1)) keeps its 3 gates' B fragments in VGPRs for the whole launch
//              (layer 1: x part 1 + h part 8 k-steps, layer 2: 8 + 8 k-steps);
//   per step every member needs the full h of its 128 rows as the MFMA A operand, so after a
//              step each member publishes its 32 columns (16 KB, both layers) and gathers the
//              other seven slices into LDS.
//
// The two layers are pipelined (layer 1 at step t, layer 2 at step t-1: both read h1_{t-1}),
// so each step costs ONE cluster hand-off. Hand-off protocol (MI355X_MICROARCH.md,
// inter-workgroup visibility, first row of the sc1 table): every byte stored with 16-B `sc1`
// buffer stores, every storing wave `s_waitcnt vmcnt(0)`, a workgroup barrier, then ONE lane
// adds to the cluster's monotonic counter (agent-scope atomic); consumers poll it with `sc1`
// loads, barrier, and read every handed-off byte with 16-B `sc1` buffer loads. A counter starts
// at 0 (allocation) and member 0 returns it to 0 with an atomic after the cluster's final
// arrival. Every poll is bounded: a cluster that is not co-resident (another persistent kernel
// holding CUs) sets *ws_err and every wave exits; the host then resets and falls back.
//
// The f32 hidden state never leaves registers (lane-local z/r/h~ combine, as in gru.hip); the
// head is a fixed-order sum of per-member f32 partials (deterministic).
#include "common.h"
#include "launch.h"

namespace igp {
namespace {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int WS_CL = 8;              // workgroups per cluster
constexpr int WS_M = 128;             // sequences per cluster
constexpr int WS_RT = WS_M / 16;      // MFMA row tiles
constexpr int WS_H = 256;
constexpr int WS_HT = WS_H / 16;      // hidden tiles
constexpr int WS_HS = WS_H + 8;       // LDS row stride (bf16), conflict-free A-fragment reads
constexpr int WS_XS = 32 + 8;
constexpr int WS_UW = WS_H / WS_CL;   // hidden units per member (32)
constexpr int WS_SLICE = 2 * WS_M * WS_UW;  // bf16 per member slice (both layers)
constexpr int WS_CH = WS_SLICE / 8;   // 16-B chunks per slice (1024)
constexpr uint64_t WS_WAIT_TICKS = 20000000;  // 200 ms of wall_clock64 (100 MHz): never hang the GPU
constexpr int SC1 = 16;               // buffer aux bit: sc1 (L2-coherent, bypasses L1)

// v_exp_f32 + v_rcp_f32 (1 ulp): the IEEE divide sequence would cost ~10 VALU per gate
__device__ __forceinline__ float sig_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f); }

__device__ __forceinline__ bf16x8 lds_frag(const uint16_t* base, int stride, int row, int k) {
  const uint4 v = *reinterpret_cast<const uint4*>(base + row * stride + k);
  return __builtin_bit_cast(bf16x8, v);
}

// packed fragment (nt, ks) of a [N/16][KS][64][8] bf16 weight (ops/kernels.py pack_fragments)
__device__ __forceinline__ bf16x8 wfrag(const uint16_t* p, int nt, int KS, int ks, int lane) {
  const uint4 v = *reinterpret_cast<const uint4*>(p + (((size_t)nt * KS + ks) * 64 + lane) * 8);
  return __builtin_bit_cast(bf16x8, v);
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// one layer's step for this wave's hidden tile over all 8 row tiles, two at a time.
// L = 0: A = [x_t | h1_{t-1}] (1 + 8 k-steps); L = 1: A = [h1_{t-1} | h2_{t-2}] (8 + 8).
// x-part -> ax (the input half of h~), h-part -> ah (recurrent half, scaled by r): LBR = 1.
// The A fragments of k-step ks+1 are read from LDS before the MFMAs of ks are issued (the
// weights hold ~200 registers, so without an explicit prefetch one A buffer serialises LDS
// latency against every three MFMAs). Software-pipelined over row-tile pairs: the gate
// epilogue (exp / rcp / fma, ~20 VALU per element) of pair p-1 is placed beside the MFMAs of
// pair p, so it issues in the MFMA pipe's free VALU slots instead of after them (the
// accumulators are double-buffered in AGPRs).
template <int L>
__device__ __forceinline__ void ws_mfma_pair(const bf16x8 (&wz)[16], const bf16x8 (&wr)[16], const bf16x8 (&wh)[16],
                                             const uint16_t* X, const uint16_t* H1, const uint16_t* H2, int rt0,
                                             int lane, f32x4 (&acc)[4][2]) {
  constexpr int NK = L == 0 ? 9 : 16;  // k-steps
  constexpr int NX = L == 0 ? 1 : 8;   // k-steps of the input part
  const int arow = lane & 15, akof = 8 * (lane >> 4);
  auto afrag = [&](int ks, int rt) -> bf16x8 {
    if constexpr (L == 0) {
      return ks == 0 ? lds_frag(X, WS_XS, rt * 16 + arow, akof)
                     : lds_frag(H1, WS_HS, rt * 16 + arow, (ks - 1) * 32 + akof);
    } else {
      return ks < 8 ? lds_frag(H1, WS_HS, rt * 16 + arow, ks * 32 + akof)
                    : lds_frag(H2, WS_HS, rt * 16 + arow, (ks - 8) * 32 + akof);
    }
  };
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[g][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 cur[2] = {afrag(0, rt0), afrag(0, rt0 + 1)};
#pragma unroll
  for (int ks = 0; ks < NK; ++ks) {
    bf16x8 nxt[2] = {cur[0], cur[1]};
    if (ks + 1 < NK) {
      nxt[0] = afrag(ks + 1, rt0);
      nxt[1] = afrag(ks + 1, rt0 + 1);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      acc[0][u] = MFMA(cur[u], wz[ks], acc[0][u]);
      acc[1][u] = MFMA(cur[u], wr[ks], acc[1][u]);
      if (ks < NX) acc[2][u] = MFMA(cur[u], wh[ks], acc[2][u]);
      else acc[3][u] = MFMA(cur[u], wh[ks], acc[3][u]);
    }
    cur[0] = nxt[0];
    cur[1] = nxt[1];
  }
}

__device__ __forceinline__ void ws_epilogue(const f32x4 (&acc)[4][2], float (&hs)[WS_RT][4], const float (&bv)[4],
                                            int rt0) {
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = sig_(acc[0][u][r] + bv[0]);
      const float rr = sig_(acc[1][u][r] + bv[1]);
      const float hh = tanh_(acc[2][u][r] + bv[2] + rr * (acc[3][u][r] + bv[3]));
      hs[rt0 + u][r] = (1.f - z) * hh + z * hs[rt0 + u][r];
    }
}

// row tiles [RT0, RT0 + NRT) of one layer's step (NRT even)
template <int L, int RT0 = 0, int NRT = WS_RT>
__device__ __forceinline__ void ws_layer(const bf16x8 (&wz)[16], const bf16x8 (&wr)[16], const bf16x8 (&wh)[16],
                                         const uint16_t* X, const uint16_t* H1, const uint16_t* H2,
                                         float (&hs)[WS_RT][4], const float (&bv)[4], int lane) {
  f32x4 acc[2][4][2];
  ws_mfma_pair<L>(wz, wr, wh, X, H1, H2, RT0, lane, acc[0]);
#pragma unroll
  for (int p = 1; p < NRT / 2; ++p) {
    ws_mfma_pair<L>(wz, wr, wh, X, H1, H2, RT0 + 2 * p, lane, acc[p & 1]);
    ws_epilogue(acc[(p - 1) & 1], hs, bv, RT0 + 2 * (p - 1));
  }
  ws_epilogue(acc[(NRT / 2 - 1) & 1], hs, bv, RT0 + NRT - 2);
}
#undef MFMA

// bounded poll of a cluster counter by one lane; returns false on timeout, after poisoning both
// counters of the cluster (`base`: cnt[0] and cnt[8], gru.hip kClusterPoison) so that no member
// still to arrive and no launch queued behind this one passes a wait on a part-advanced count
__device__ __forceinline__ bool ws_wait(int32_t* cnt, int target, int32_t* base) {
  const uint64_t t0 = wall_clock64();
  for (;;) {
    for (int n = 0; n < 64; ++n) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
      __builtin_amdgcn_s_sleep(1);
    }
    if (wall_clock64() - t0 > WS_WAIT_TICKS) {
      __hip_atomic_exchange(base, kClusterPoison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(base + 8, kClusterPoison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

// SPLIT: the cluster's 128 sequences as two independent 64-row halves in a software pipeline
// (GruArgs.ws == 2): the hand-off of one half (sc1 stores draining, counter, gather) runs beside
// the other half's MFMAs; counters cnt[0] (half A) and cnt[8] (half B).
template <bool SPLIT>
__global__ void __launch_bounds__(256, 1) gru_ws_kernel(GruArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: H1[M][HS] | H2[M][HS] | X[2][M][XS] (bf16) | red[2][M] f32 | xmeta[4M] | flag
  uint16_t* const H1 = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const H2 = H1 + WS_M * WS_HS;
  uint16_t* const Xb = H2 + WS_M * WS_HS;
  float* const red = reinterpret_cast<float*>(Xb + 2 * WS_M * WS_XS);
  int2* const xmeta = reinterpret_cast<int2*>(red + 2 * WS_M);  // per input chunk {slot, head | from << 16}
  int* const sflag = reinterpret_cast<int*>(xmeta + 4 * WS_M);

  const int b = blockIdx.x;
  const int mem = (b >> 3) & 7;            // member: hidden units [32 mem, 32 mem + 32)
  const int cl = (b >> 6) * 8 + (b & 7);   // cluster: members share blockIdx % 8
  const int row0 = cl * WS_M;
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  if (row0 >= n_live || cl >= a.ws_clusters) return;  // uniform over the cluster's 8 members
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int layer = wave >> 1;
  const int ht = mem * 2 + (wave & 1);
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  const int j = ht * 16 + ccol;            // this lane's hidden unit
  const int T = a.T;
  int32_t* const cnt = a.ws_sync + cl * 16;
  // outputs start as NaN: a cluster that gives up (bounded wait) leaves them so, and the host
  // detects it (AbuseGpu.wait) instead of reading the previous batch's values
  if (a.head_w && mem == 0 && tid < WS_M && row0 + tid < n_live) a.out[row0 + tid] = __builtin_nanf("");
  if (a.yh)
    for (int e = tid; e < WS_M * WS_UW; e += 256) {
      const int row = row0 + e / WS_UW;
      if (row < n_live) a.yh[(size_t)row * WS_H + mem * WS_UW + e % WS_UW] = __builtin_nanf("");
    }

  // ---- weights -> registers (stationary for the whole launch)
  bf16x8 wz[16], wr[16], wh[16];
  if (layer == 0) {
    const uint16_t* W = a.layer[0].W;
    const uint16_t* R = a.layer[0].R;
    wz[0] = wfrag(W, ht, 1, 0, lane);
    wr[0] = wfrag(W, WS_HT + ht, 1, 0, lane);
    wh[0] = wfrag(W, 2 * WS_HT + ht, 1, 0, lane);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      wz[1 + ks] = wfrag(R, ht, 8, ks, lane);
      wr[1 + ks] = wfrag(R, WS_HT + ht, 8, ks, lane);
      wh[1 + ks] = wfrag(R, 2 * WS_HT + ht, 8, ks, lane);
    }
  } else {
    const uint16_t* W = a.layer[1].W;
    const uint16_t* R = a.layer[1].R;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      wz[ks] = wfrag(W, ht, 8, ks, lane);
      wr[ks] = wfrag(W, WS_HT + ht, 8, ks, lane);
      wh[ks] = wfrag(W, 2 * WS_HT + ht, 8, ks, lane);
      wz[8 + ks] = wfrag(R, ht, 8, ks, lane);
      wr[8 + ks] = wfrag(R, WS_HT + ht, 8, ks, lane);
      wh[8 + ks] = wfrag(R, 2 * WS_HT + ht, 8, ks, lane);
    }
  }
  float bv[4];
  {
    const float* bs = a.layer[layer].bias;  // Wb z,r,h | Rb z,r,h
    bv[0] = bs[j] + bs[3 * WS_H + j];
    bv[1] = bs[WS_H + j] + bs[4 * WS_H + j];
    bv[2] = bs[2 * WS_H + j];
    bv[3] = bs[5 * WS_H + j];
  }

  // ---- zero the LDS state (h_{-1} = 0; X columns past I stay zero)
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(smem);
    const int words = (2 * WS_M * WS_HS + 2 * WS_M * WS_XS) / 2;
    for (int i = tid; i < words; i += 256) z[i] = 0u;
  }
  // ---- layer-1 input: chunk c = (row c / chunks, 8-element piece c % chunks); its source
  // (event-ring slot / head / first valid step) goes to LDS once, and only the two layer-0
  // waves stage x_{t+1} (<= 4 chunks per lane), so the layer-1 waves carry no staging registers
  const int I = a.I;
  const int chunks = I >> 3;  // 1..4
  const int nchunk = WS_M * chunks;
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
  auto load_x = [&](int c, int t) -> uint4 {
    uint4 v = make_uint4(0, 0, 0, 0);
    const int2 m = xmeta[c];
    const int from = m.y >> 16;
    if (t >= T) return v;
    if (a.reverse) t = T - 1 - t;  // direction=reverse: forward over the time-reversed sequence
    if (t < from) return v;
    const int row = c / chunks, q = c - row * chunks;
    if (a.mode == 1) {
      if (m.x < 0) return v;
      int idx = ((m.y & 0xffff) - T + t) % a.ev_ring;
      if (idx < 0) idx += a.ev_ring;
      v = *reinterpret_cast<const uint4*>(a.ev + (((size_t)m.x * a.ev_ring + idx) * I + q * 8));
    } else {
      const float* src = a.X + (((size_t)t * a.x_rows + row0 + row) * I + q * 8);
      const float4 f0 = *reinterpret_cast<const float4*>(src);
      const float4 f1 = *reinterpret_cast<const float4*>(src + 4);
      v.x = (uint32_t)f32_to_bf16(f0.x) | ((uint32_t)f32_to_bf16(f0.y) << 16);
      v.y = (uint32_t)f32_to_bf16(f0.z) | ((uint32_t)f32_to_bf16(f0.w) << 16);
      v.z = (uint32_t)f32_to_bf16(f1.x) | ((uint32_t)f32_to_bf16(f1.y) << 16);
      v.w = (uint32_t)f32_to_bf16(f1.z) | ((uint32_t)f32_to_bf16(f1.w) << 16);
    }
    return v;
  };
  auto x_slot = [&](int buf, int c) -> uint4* {
    const int row = c / chunks, q = c - row * chunks;
    return reinterpret_cast<uint4*>(Xb + buf * (WS_M * WS_XS) + row * WS_XS + q * 8);
  };
  __syncthreads();
  if (layer == 0)
    for (int c = tid; c < nchunk; c += 128) *x_slot(0, c) = load_x(c, 0);

  float hs[WS_RT][4];
#pragma unroll
  for (int rt = 0; rt < WS_RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) hs[rt][r] = 0.f;

  // exchange slab of this cluster: [parity][member][layer][M][32] bf16 (16-B sc1 traffic)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      a.ws_x + (size_t)cl * 2 * WS_CL * WS_SLICE, 0, 2 * WS_CL * WS_SLICE * 2, 0x00020000);
  uint16_t* const Hl = layer == 0 ? H1 : H2;
  __syncthreads();

  int64_t* const trace = (a.ws_trace && b == 0 && tid == 0) ? a.ws_trace : nullptr;
#define WS_MARK(t, k) \
  if (trace && (t) < 64) trace[(t) * 6 + (k)] = (int64_t)wall_clock64()
  if constexpr (SPLIT) {
    int32_t* const cntB = cnt + 8;
    // own columns of half h (rows 64h .. 64h + 63) of this wave's layer -> LDS
    auto own_cols = [&](int h) {
#pragma unroll
      for (int rt = 0; rt < WS_RT / 2; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) Hl[((4 * h + rt) * 16 + crow + r) * WS_HS + j] = f32_to_bf16(hs[4 * h + rt][r]);
    };
    // this member's slice of half h (both layers, 512 16-B chunks, 2 per thread) -> slab, no wait
    auto publish = [&](int h, int par) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = i * 512 + 256 * h + tid;
        const int row = (c >> 2) & (WS_M - 1), q = c & 3;
        const uint16_t* src = (i ? H2 : H1) + row * WS_HS + mem * WS_UW + q * 8;
        const u32x4 v = __builtin_bit_cast(u32x4, *reinterpret_cast<const uint4*>(src));
        __builtin_amdgcn_raw_buffer_store_b128(v, xr, c * 16, ((par * WS_CL + mem) * WS_SLICE) * 2, SC1);
      }
    };
    // the other seven members' slices of half h (14 chunks per thread) -> LDS
    auto gather = [&](int h, int par) {
      u32x4 v[14];
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int k = i * 256 + tid;
        int m2 = k >> 9;
        m2 += m2 >= mem;
        const int w = k & 511;
        const int c = (w >> 8) * 512 + 256 * h + (w & 255);
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, c * 16, ((par * WS_CL + m2) * WS_SLICE) * 2, SC1);
      }
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int k = i * 256 + tid;
        int m2 = k >> 9;
        m2 += m2 >= mem;
        const int w = k & 511;
        const int c = (w >> 8) * 512 + 256 * h + (w & 255);
        const int row = (c >> 2) & (WS_M - 1), q = c & 3;
        *reinterpret_cast<uint4*>(((w >> 8) ? H2 : H1) + row * WS_HS + m2 * WS_UW + q * 8) = __builtin_bit_cast(uint4, v[i]);
      }
    };
    // arrival (one lane) + bounded wait for all members; false: give up (the cluster exits)
    auto arrive_wait = [&](int32_t* c, int target, bool arrive) -> bool {
      if (tid == 0) {
        if (arrive) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
        if (target > 0) {
          ok = ws_wait(c, target, cnt);
          if (!ok) atomicExch(a.ws_err, 1);
        }
        *sflag = ok;
      }
      __syncthreads();
      return *sflag != 0;
    };
    for (int t = 0; t <= T; ++t) {
      WS_MARK(t, 0);
      const bool act = layer == 0 ? (t < T) : (t >= 1);
      // ---- half A of step t (+ x_{t+1} staging for all rows)
      if (layer == 0) {
        uint4 xn[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = tid + 128 * u;
          xn[u] = c < nchunk ? load_x(c, t + 1) : make_uint4(0, 0, 0, 0);
        }
        if (act) ws_layer<0, 0, WS_RT / 2>(wz, wr, wh, Xb + (t & 1) * (WS_M * WS_XS), H1, H2, hs, bv, lane);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = tid + 128 * u;
          if (c < nchunk) *x_slot((t + 1) & 1, c) = xn[u];
        }
      } else if (act) {
        ws_layer<1, 0, WS_RT / 2>(wz, wr, wh, Xb + (t & 1) * (WS_M * WS_XS), H1, H2, hs, bv, lane);
      }
      __syncthreads();  // every wave is done reading rows A
      WS_MARK(t, 1);
      if (t < T && act) own_cols(0);
      // half B of step t-1: its stores drained under half A's MFMAs -> arrive
      if (t >= 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(cntB, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (t < T) publish(0, t & 1);  // drains under the gather and half B's MFMAs
      if (t >= 1) {
        if (!arrive_wait(cntB, WS_CL * t, false)) return;
        gather(1, (t - 1) & 1);
        __syncthreads();
      }
      WS_MARK(t, 2);
      // ---- half B of step t
      if (layer == 0) {
        if (act) ws_layer<0, WS_RT / 2, WS_RT / 2>(wz, wr, wh, Xb + (t & 1) * (WS_M * WS_XS), H1, H2, hs, bv, lane);
      } else if (act) {
        ws_layer<1, WS_RT / 2, WS_RT / 2>(wz, wr, wh, Xb + (t & 1) * (WS_M * WS_XS), H1, H2, hs, bv, lane);
      }
      __syncthreads();  // every wave is done reading rows B
      WS_MARK(t, 3);
      if (t == T) break;
      if (act) own_cols(1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // half A's stores of step t
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish(1, t & 1);
      if (!arrive_wait(cnt, WS_CL * (t + 1), false)) return;
      gather(0, t & 1);
      __syncthreads();
      WS_MARK(t, 4);
    }
  } else
  for (int t = 0; t <= T; ++t) {
    WS_MARK(t, 0);
    const bool act = layer == 0 ? (t < T) : (t >= 1);
    if (layer == 0) {
      uint4 xn[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = tid + 128 * u;
        xn[u] = c < nchunk ? load_x(c, t + 1) : make_uint4(0, 0, 0, 0);
      }
      if (act) ws_layer<0>(wz, wr, wh, Xb + (t & 1) * (WS_M * WS_XS), H1, H2, hs, bv, lane);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = tid + 128 * u;
        if (c < nchunk) *x_slot((t + 1) & 1, c) = xn[u];
      }
    } else if (act) {
      ws_layer<1>(wz, wr, wh, Xb, H1, H2, hs, bv, lane);
    }
    if (a.ws_trace && b == 0 && (tid & 127) == 0 && t < 64) {  // per-layer compute end (wave 0 / wave 2)
      if (tid == 0) a.ws_trace[64 * 6 + t * 2] = (int64_t)wall_clock64();
      else a.ws_trace[64 * 6 + t * 2 + 1] = (int64_t)wall_clock64();
    }
    if (a.ws_trace && b == 0 && tid == 0 && t == 0) {
      a.ws_trace[64 * 8] = (int64_t)wall_clock64();
      a.ws_trace[64 * 8 + 1] = (int64_t)clock64();
    }
    if (a.ws_trace && b == 0 && tid == 0 && t == T - 1) {
      a.ws_trace[64 * 8 + 2] = (int64_t)wall_clock64();
      a.ws_trace[64 * 8 + 3] = (int64_t)clock64();
    }
    __syncthreads();  // every wave is done reading H1 / H2 / X of this step
    WS_MARK(t, 1);
    if (t == T) break;
    // own new columns into LDS (h1_t from layer 0, h2_{t-1} from layer 1) + x_{t+1}
    if (act) {
#pragma unroll
      for (int rt = 0; rt < WS_RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) Hl[(rt * 16 + crow + r) * WS_HS + j] = f32_to_bf16(hs[rt][r]);
    }
    __syncthreads();
    // publish this member's slice (both layers) with sc1 stores
    const int par = t & 1;
#pragma unroll
    for (int i = 0; i < WS_CH / 256; ++i) {
      const int c = i * 256 + tid;
      const int L = c >> 9, row = (c >> 2) & (WS_M - 1), q = c & 3;
      const uint16_t* src = (L ? H2 : H1) + row * WS_HS + mem * WS_UW + q * 8;
      const u32x4 v = __builtin_bit_cast(u32x4, *reinterpret_cast<const uint4*>(src));
      __builtin_amdgcn_raw_buffer_store_b128(v, xr, c * 16, ((par * WS_CL + mem) * WS_SLICE) * 2, SC1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    WS_MARK(t, 2);
    if (tid == 0) {
      __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool ok = ws_wait(cnt, WS_CL * (t + 1), cnt);
      if (!ok) atomicExch(a.ws_err, 1);
      *sflag = ok;
    }
    __syncthreads();
    WS_MARK(t, 3);
    if (!*sflag) return;
    // gather the other 7 members' slices into H1 / H2 (sc1 loads, 14 in flight per lane)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u32x4 v[14];
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int c = (h * 14 + i) * 256 + tid;  // over 7 x 1024 chunks
        int m2 = c >> 10;
        m2 += m2 >= mem;
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, (c & 1023) * 16, ((par * WS_CL + m2) * WS_SLICE) * 2, SC1);
      }
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int c = (h * 14 + i) * 256 + tid;
        int m2 = c >> 10;
        m2 += m2 >= mem;
        const int cc = c & 1023;
        const int L = cc >> 9, row = (cc >> 2) & (WS_M - 1), q = cc & 3;
        *reinterpret_cast<uint4*>((L ? H2 : H1) + row * WS_HS + m2 * WS_UW + q * 8) = __builtin_bit_cast(uint4, v[i]);
      }
    }
    __syncthreads();
    WS_MARK(t, 4);
  }
#undef WS_MARK

  // ---- outputs: layer-2 waves hold h2_{T-1} (f32) for rows 0..127 of their tile
  if (layer == 1 && a.yh) {
#pragma unroll
    for (int rt = 0; rt < WS_RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + rt * 16 + crow + r;
        if (row < n_live) a.yh[(size_t)row * WS_H + j] = hs[rt][r];
      }
  }
  float* const part = a.ws_part + (size_t)cl * WS_CL * WS_M;
  if (a.head_w) {
    if (layer == 1) {
      const float w = a.head_w[j];
#pragma unroll
      for (int rt = 0; rt < WS_RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = hs[rt][r] * w;
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
          if (ccol == 0) red[(wave & 1) * WS_M + rt * 16 + crow + r] = v;
        }
    }
    __syncthreads();
    if (tid < WS_M) {
      const float v = red[tid] + red[WS_M + tid];
      __hip_atomic_store(part + mem * WS_M + tid, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // final arrival: member 0 waits for all eight, combines the head partials, then returns the
  // counter to 0 with an atomic (no member touches it again in this launch). The reset must
  // take the atomic path: a memset node between graph replays left a stale counter line
  // visible to the next replay's sc1 polls.
  if (tid == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true;
    if (mem == 0) {
      ok = ws_wait(cnt, WS_CL * (T + 1), cnt);
      if (!ok) atomicExch(a.ws_err, 1);
    }
    *sflag = ok;
  }
  __syncthreads();
  if (mem != 0 || !*sflag) return;
  if (a.head_w && tid < WS_M && row0 + tid < n_live) {
    float v = a.head_b;
#pragma unroll
    for (int m2 = 0; m2 < WS_CL; ++m2)
      v += __hip_atomic_load(part + m2 * WS_M + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.head_act == 2) v = 1.f / (1.f + expf(-v));
    a.out[row0 + tid] = v;
  }
  if (tid == 0) {
    __hip_atomic_exchange(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (SPLIT) __hip_atomic_exchange(cnt + 8, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ============================================================================================
// Two clusters per CU (ws = 3): 64-row clusters, 4 waves per workgroup, TWO co-resident
// workgroups per CU (80 KB LDS each, <= 256 VGPRs per wave). Same member split and hand-off
// protocol as above, but every SIMD now hosts two waves of two independent clusters, so one
// cluster's hand-off (sc1 stores draining, counter poll, gather) and gate epilogue issue while
// the other cluster's wave keeps the MFMA pipe busy - the hardware interleaves what the
// single-wave kernel had to serialise (NOTES: 9.4 us/step = 5.5 compute + 3.9 hand-off).
// Layer balance: a layer-2 wave issues 192 MFMAs per step, a layer-1 wave 108; roles follow the
// wave's SIMD so that every SIMD hosts one wave of each layer (see the kernel's prologue).
constexpr int W2_M = 64;
constexpr int W2_RT = W2_M / 16;
constexpr int W2_SLICE = 2 * W2_M * WS_UW;  // bf16 per member slice (both layers)
constexpr int W2_CH = W2_SLICE / 8;         // 16-B chunks per slice (512)
constexpr int W2_BLK = W2_M * WS_UW;        // bf16 per (layer, member) block of the LDS image (4 KB)
// LDS image of h (per layer): [member][64 rows][32 columns] bf16, member-major so that a k-step
// of 32 is one member's block and a handed-off slice is 2 contiguous 4-KB blocks - gathered
// with global_load_lds (1 KB per wave instruction, no registers: the stationary weights leave
// none). The 16-B chunk (row, q) sits at row * 4 + (q ^ ((row >> 2) & 3)): a 16-row A-fragment
// read then touches 16 distinct chunks of every 256-B bank row (conflict-free), and the swizzle
// is the same in every member's block, so slices are copied verbatim.
__device__ __forceinline__ int w2_chunk(int row, int q) { return row * 4 + (q ^ ((row >> 2) & 3)); }

// one row tile of one layer's step: acc = A(rt) . [Wz | Wr | Wh] over NK k-steps
template <int L>
__device__ __forceinline__ void w2_tile(const bf16x8 (&wz)[16], const bf16x8 (&wr)[16], const bf16x8 (&wh)[16],
                                        const uint16_t* X, const uint16_t* H1, const uint16_t* H2, int rt, int lane,
                                        f32x4 (&acc)[4]) {
  constexpr int NK = L == 0 ? 9 : 16;
  constexpr int NX = L == 0 ? 1 : 8;
  const int arow = rt * 16 + (lane & 15), akof = 8 * (lane >> 4);
  const int hoff = w2_chunk(arow, lane >> 4) * 8;  // k-step ks reads member block ks
  auto hfrag = [&](const uint16_t* Hb, int blk) -> bf16x8 {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Hb + blk * W2_BLK + hoff));
  };
  auto afrag = [&](int ks) -> bf16x8 {
    if constexpr (L == 0) {
      return ks == 0 ? lds_frag(X, WS_XS, arow, akof) : hfrag(H1, ks - 1);
    } else {
      return ks < 8 ? hfrag(H1, ks) : hfrag(H2, ks - 8);
    }
  };
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 cur = afrag(0);
#pragma unroll
  for (int ks = 0; ks < NK; ++ks) {
    const bf16x8 nxt = ks + 1 < NK ? afrag(ks + 1) : cur;
    // one k-step ahead only: left alone the scheduler hoists every A read of the tile (and
    // runs out of the ~60 registers the stationary weights leave)
    __builtin_amdgcn_sched_barrier(0);
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur, wz[ks], acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur, wr[ks], acc[1], 0, 0, 0);
    if (ks < NX) acc[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur, wh[ks], acc[2], 0, 0, 0);
    else acc[3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur, wh[ks], acc[3], 0, 0, 0);
    cur = nxt;
  }
}

template <int L>
__device__ __forceinline__ void w2_layer(const bf16x8 (&wz)[16], const bf16x8 (&wr)[16], const bf16x8 (&wh)[16],
                                         const uint16_t* X, const uint16_t* H1, const uint16_t* H2,
                                         float (&hs)[W2_RT][4], const float (&bv)[4], int lane) {
#pragma unroll
  for (int rt = 0; rt < W2_RT; ++rt) {
    f32x4 acc[4];
    w2_tile<L>(wz, wr, wh, X, H1, H2, rt, lane, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = sig_(acc[0][r] + bv[0]);
      const float rr = sig_(acc[1][r] + bv[1]);
      const float hh = tanh_(acc[2][r] + bv[2] + rr * (acc[3][r] + bv[3]));
      hs[rt][r] = (1.f - z) * hh + z * hs[rt][r];
    }
  }
}

template <int L>
struct W2Layer {
  static constexpr int value = L;
};

__global__ void __launch_bounds__(256, 2) gru_ws2_kernel(GruArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: H1[8 blocks] | H2[8 blocks] (swizzled images) | X[2][M][XS] (bf16) | red[2][M] f32 | xmeta[4M] | flag
  uint16_t* const H1 = reinterpret_cast<uint16_t*>(smem);
  uint16_t* const H2 = H1 + WS_CL * W2_BLK;
  uint16_t* const Xb = H2 + WS_CL * W2_BLK;
  float* const red = reinterpret_cast<float*>(Xb + 2 * W2_M * WS_XS);
  int2* const xmeta = reinterpret_cast<int2*>(red + 2 * W2_M);
  int* const sflag = reinterpret_cast<int*>(xmeta + 4 * W2_M);

  const int b = blockIdx.x;
  const int mem = (b >> 3) & 7;
  const int cl = (b >> 6) * 8 + (b & 7);
  const int row0 = cl * W2_M;
  const int n_live = a.m_ptr ? min(*a.m_ptr, a.n_rows) : a.n_rows;
  if (row0 >= n_live || cl >= 2 * a.ws_clusters) return;  // uniform over the cluster's 8 members
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Roles by SIMD: a layer-2 wave issues 192 MFMAs per step, a layer-1 wave 108, and the two
  // co-resident workgroups of a CU are blocks b and b + 256 (breadth-first dispatch, recorded by
  // tools/gru_ws_trace.py). A workgroup's four waves sit on four different SIMDs, in an order
  // whose start varies, so the roles follow the SIMD the wave got (HW_ID bits 5:4): SIMDs 0-1
  // run layer 1 and SIMDs 2-3 layer 2 in the first half of the grid, the other way round in the
  // second, and every SIMD hosts one wave of each layer (300 MFMAs per step, not up to 384).
  // When the four SIMD ids are not distinct, roles fall back to the wave index.
  int* const ssid = sflag + 4;
  const int sid = (int)((__builtin_amdgcn_s_getreg(0xF804) >> 4) & 3u);  // HW_ID.SIMD_ID
  if (lane == 0) ssid[wave] = sid;
  __syncthreads();
  const bool by_simd = ((1 << ssid[0]) | (1 << ssid[1]) | (1 << ssid[2]) | (1 << ssid[3])) == 15;
  const int role = __builtin_amdgcn_readfirstlane(by_simd ? sid : wave);
  const int layer = (role >> 1) ^ ((b >> 8) & 1);
  const int tile = role & 1;
  const int ht = mem * 2 + tile;
  const int crow = (lane >> 4) * 4, ccol = lane & 15;
  const int j = ht * 16 + ccol;
  const int T = a.T;
  int32_t* const cnt = a.ws_sync + cl * 16;
  if (a.head_w && mem == 0 && tid < W2_M && row0 + tid < n_live) a.out[row0 + tid] = __builtin_nanf("");
  if (a.yh)
    for (int e = tid; e < W2_M * WS_UW; e += 256) {
      const int row = row0 + e / WS_UW;
      if (row < n_live) a.yh[(size_t)row * WS_H + mem * WS_UW + e % WS_UW] = __builtin_nanf("");
    }
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(smem);
    const int words = (2 * WS_CL * W2_BLK + 2 * W2_M * WS_XS) / 2;
    for (int i = tid; i < words; i += 256) z[i] = 0u;
  }
  const int I = a.I;
  const int chunks = I >> 3;
  const int nchunk = W2_M * chunks;  // <= 256
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
  auto load_x = [&](int c, int t) -> uint4 {
    uint4 v = make_uint4(0, 0, 0, 0);
    const int2 m = xmeta[c];
    const int from = m.y >> 16;
    if (t >= T) return v;
    if (a.reverse) t = T - 1 - t;
    if (t < from) return v;
    const int row = c / chunks, q = c - row * chunks;
    if (a.mode == 1) {
      if (m.x < 0) return v;
      int idx = ((m.y & 0xffff) - T + t) % a.ev_ring;
      if (idx < 0) idx += a.ev_ring;
      v = *reinterpret_cast<const uint4*>(a.ev + (((size_t)m.x * a.ev_ring + idx) * I + q * 8));
    } else {
      const float* src = a.X + (((size_t)t * a.x_rows + row0 + row) * I + q * 8);
      const float4 f0 = *reinterpret_cast<const float4*>(src);
      const float4 f1 = *reinterpret_cast<const float4*>(src + 4);
      v.x = (uint32_t)f32_to_bf16(f0.x) | ((uint32_t)f32_to_bf16(f0.y) << 16);
      v.y = (uint32_t)f32_to_bf16(f0.z) | ((uint32_t)f32_to_bf16(f0.w) << 16);
      v.z = (uint32_t)f32_to_bf16(f1.x) | ((uint32_t)f32_to_bf16(f1.y) << 16);
      v.w = (uint32_t)f32_to_bf16(f1.z) | ((uint32_t)f32_to_bf16(f1.w) << 16);
    }
    return v;
  };
  auto x_slot = [&](int buf, int c) -> uint4* {
    const int row = c / chunks, q = c - row * chunks;
    return reinterpret_cast<uint4*>(Xb + buf * (W2_M * WS_XS) + row * WS_XS + q * 8);
  };
  const int ltid = tile * 64 + lane;  // thread index among the two layer-0 waves
  __syncthreads();
  if (layer == 0)
    for (int c = ltid; c < nchunk; c += 128) *x_slot(0, c) = load_x(c, 0);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      a.ws_x + (size_t)cl * 2 * WS_CL * W2_SLICE, 0, 2 * WS_CL * W2_SLICE * 2, 0x00020000);
  int64_t* const trace = (a.ws_trace && b == 0 && tid == 0) ? a.ws_trace : nullptr;
  // placement record (trace runs only): which XCD / SE / CU / SIMD each workgroup's wave 0 got
  if (a.ws_trace && tid == 0 && b < 1024)
    a.ws_trace[64 * 8 + 4 + b] = ((int64_t)__builtin_amdgcn_s_getreg(0xF814) << 32) |
                                 (uint32_t)__builtin_amdgcn_s_getreg(0xF804);  // XCC_ID | HW_ID

  // the whole recurrence, specialised per layer: each wave runs exactly one instantiation, so
  // the register allocator sees one set of stationary weights (192 registers for layer 2, 108
  // for layer 1) instead of both sets merged across a branch. Both instantiations execute the
  // same sequence of workgroup barriers.
  auto run = [&](auto Lc) -> bool {
    constexpr int L = decltype(Lc)::value;
    bf16x8 wz[16], wr[16], wh[16];
    if constexpr (L == 0) {
      const uint16_t* W = a.layer[0].W;
      const uint16_t* R = a.layer[0].R;
      wz[0] = wfrag(W, ht, 1, 0, lane);
      wr[0] = wfrag(W, WS_HT + ht, 1, 0, lane);
      wh[0] = wfrag(W, 2 * WS_HT + ht, 1, 0, lane);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        wz[1 + ks] = wfrag(R, ht, 8, ks, lane);
        wr[1 + ks] = wfrag(R, WS_HT + ht, 8, ks, lane);
        wh[1 + ks] = wfrag(R, 2 * WS_HT + ht, 8, ks, lane);
      }
    } else {
      const uint16_t* W = a.layer[1].W;
      const uint16_t* R = a.layer[1].R;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        wz[ks] = wfrag(W, ht, 8, ks, lane);
        wr[ks] = wfrag(W, WS_HT + ht, 8, ks, lane);
        wh[ks] = wfrag(W, 2 * WS_HT + ht, 8, ks, lane);
        wz[8 + ks] = wfrag(R, ht, 8, ks, lane);
        wr[8 + ks] = wfrag(R, WS_HT + ht, 8, ks, lane);
        wh[8 + ks] = wfrag(R, 2 * WS_HT + ht, 8, ks, lane);
      }
    }
    float bv[4];
    {
      const float* bs = a.layer[L].bias;
      bv[0] = bs[j] + bs[3 * WS_H + j];
      bv[1] = bs[WS_H + j] + bs[4 * WS_H + j];
      bv[2] = bs[2 * WS_H + j];
      bv[3] = bs[5 * WS_H + j];
    }
    float hs[W2_RT][4];
#pragma unroll
    for (int rt = 0; rt < W2_RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) hs[rt][r] = 0.f;
    uint16_t* const Hl = L == 0 ? H1 : H2;
    __syncthreads();
#define WS_MARK(t, k) \
  if (trace && (t) < 64) trace[(t) * 6 + (k)] = (int64_t)wall_clock64()
    for (int t = 0; t <= T; ++t) {
      WS_MARK(t, 0);
      const bool act = L == 0 ? (t < T) : (t >= 1);
      if constexpr (L == 0) {
        uint4 xn[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = ltid + 128 * u;
          xn[u] = c < nchunk ? load_x(c, t + 1) : make_uint4(0, 0, 0, 0);
        }
        if (act) w2_layer<0>(wz, wr, wh, Xb + (t & 1) * (W2_M * WS_XS), H1, H2, hs, bv, lane);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = ltid + 128 * u;
          if (c < nchunk) *x_slot((t + 1) & 1, c) = xn[u];
        }
      } else {
        if (act) w2_layer<1>(wz, wr, wh, Xb, H1, H2, hs, bv, lane);
      }
      __syncthreads();  // every wave is done reading H1 / H2 / X of this step
      WS_MARK(t, 1);
      if (t == T) break;
      if (act) {
        const int cq = (tile * 16 + ccol) >> 3, ce = ccol & 7;  // this lane's column in the member block
#pragma unroll
        for (int rt = 0; rt < W2_RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rt * 16 + crow + r;
            Hl[mem * W2_BLK + w2_chunk(row, cq) * 8 + ce] = f32_to_bf16(hs[rt][r]);
          }
      }
      const int par = t & 1;
      __syncthreads();
      // publish: this member's two blocks, verbatim (512 chunks, 2 per thread)
#pragma unroll
      for (int i = 0; i < W2_CH / 256; ++i) {
        const int c = i * 256 + tid;
        const uint16_t* src = ((c >> 8) ? H2 : H1) + mem * W2_BLK + (c & 255) * 8;
        const u32x4 v = __builtin_bit_cast(u32x4, *reinterpret_cast<const uint4*>(src));
        __builtin_amdgcn_raw_buffer_store_b128(v, xr, c * 16, ((par * WS_CL + mem) * W2_SLICE) * 2, SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      WS_MARK(t, 2);
      if (tid == 0) {
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = ws_wait(cnt, WS_CL * (t + 1), cnt);
        if (!ok) atomicExch(a.ws_err, 1);
        *sflag = ok;
      }
      __syncthreads();
      WS_MARK(t, 3);
      if (!*sflag) return false;
      // the other 7 members' slices straight into the LDS image: 7 x 8 KB = 56 global_load_lds
      // of 1 KB (14 per wave), sc1 (L2-coherent); the barrier below waits vmcnt(0) for them
      {
        const uint16_t* slab = a.ws_x + (size_t)cl * 2 * WS_CL * W2_SLICE + (size_t)par * WS_CL * W2_SLICE;
#pragma unroll
        for (int i = 0; i < 14; ++i) {
          const int g = wave * 14 + i;
          const int m2i = g >> 3;
          const int m2 = m2i + (m2i >= mem);
          const int Lg = (g >> 2) & 1, kb = g & 3;
          const uint16_t* src = slab + (size_t)m2 * W2_SLICE + Lg * W2_BLK + kb * 512 + lane * 8;
          uint16_t* dst = (Lg ? H2 : H1) + m2 * W2_BLK + kb * 512;
          __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                           (__attribute__((address_space(3))) void*)(dst), 16, 0, SC1);
        }
      }
      __syncthreads();
      WS_MARK(t, 4);
    }
#undef WS_MARK
    if constexpr (L == 1) {
      if (a.yh) {
#pragma unroll
        for (int rt = 0; rt < W2_RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = row0 + rt * 16 + crow + r;
            if (row < n_live) a.yh[(size_t)row * WS_H + j] = hs[rt][r];
          }
      }
      if (a.head_w) {
        const float w = a.head_w[j];
#pragma unroll
        for (int rt = 0; rt < W2_RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = hs[rt][r] * w;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
            if (ccol == 0) red[tile * W2_M + rt * 16 + crow + r] = v;
          }
      }
    }
    return true;
  };
  const bool ok_run = layer == 0 ? run(W2Layer<0>{}) : run(W2Layer<1>{});
  if (!ok_run) return;

  float* const part = a.ws_part + (size_t)cl * WS_CL * W2_M;
  if (a.head_w) {
    __syncthreads();
    if (tid < W2_M) {
      const float v = red[tid] + red[W2_M + tid];
      __hip_atomic_store(part + mem * W2_M + tid, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true;
    if (mem == 0) {
      ok = ws_wait(cnt, WS_CL * (T + 1), cnt);
      if (!ok) atomicExch(a.ws_err, 1);
    }
    *sflag = ok;
  }
  __syncthreads();
  if (mem != 0 || !*sflag) return;
  if (a.head_w && tid < W2_M && row0 + tid < n_live) {
    float v = a.head_b;
#pragma unroll
    for (int m2 = 0; m2 < WS_CL; ++m2)
      v += __hip_atomic_load(part + m2 * W2_M + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.head_act == 2) v = 1.f / (1.f + expf(-v));
    a.out[row0 + tid] = v;
  }
  if (tid == 0) __hip_atomic_exchange(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

size_t gru_ws_lds_bytes() {
  return (size_t)2 * WS_M * WS_HS * 2 + (size_t)2 * WS_M * WS_XS * 2 + (size_t)2 * WS_M * 4 + (size_t)4 * WS_M * 8 + 16;
}
static size_t gru_ws2_lds_bytes() {  // ... | flag word, 3 spare | 4 SIMD ids
  return (size_t)2 * WS_CL * W2_BLK * 2 + (size_t)2 * W2_M * WS_XS * 2 + (size_t)2 * W2_M * 4 + (size_t)4 * W2_M * 8 + 32;
}

int gru_ws_clusters(int n_rows) { return (n_rows + WS_M - 1) / WS_M; }
int gru_ws2_clusters(int n_rows) { return (n_rows + W2_M - 1) / W2_M; }

bool gru_ws_eligible(const GruArgs& a) {
  return a.ws_x && a.ws_sync && a.ws_err && a.n_layers == 2 && a.H == WS_H && a.layer[0].lbr == 1 &&
         a.layer[1].lbr == 1 && a.layer[0].kx_pad == 32 && a.I <= 32 && a.T >= 1 && a.T < 32768 &&
         (a.mode != 1 || a.ev_ring <= 65535) &&
         (a.head_w == nullptr || a.ws_part != nullptr) && gru_ws_clusters(a.n_rows) <= a.ws_clusters;
}

// grid: 64 workgroups per 8 clusters (b = 64 q + 8 member + g, cluster = 8 q + g)
void launch_gru_ws(const GruArgs& a, hipStream_t st) {
  if (a.ws == 3) {
    const int ncl2 = gru_ws2_clusters(a.n_rows);
    IGP_LAUNCH(gru_ws2_kernel, dim3(((ncl2 + 7) / 8) * 64), dim3(256), gru_ws2_lds_bytes(), st, a);
    return;
  }
  const int ncl = gru_ws_clusters(a.n_rows);
  const int grid = ((ncl + 7) / 8) * 64;
  if (a.ws == 2) IGP_LAUNCH(gru_ws_kernel<true>, dim3(grid), dim3(256), gru_ws_lds_bytes(), st, a);
  else IGP_LAUNCH(gru_ws_kernel<false>, dim3(grid), dim3(256), gru_ws_lds_bytes(), st, a);
}

}  // namespace igp
