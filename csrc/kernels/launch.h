// Kernel argument blocks and host launch entry points of the _hipk extension.
// Every launch takes an explicit hipStream_t (torch's current stream from Python) and
// performs no allocation or synchronisation, so all of them are hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../include/records.h"
#include "oplist.h"

namespace igp {

// events of one account per batch held in its dedup list (more: ordered scan of the batch)
constexpr int DEDUP_LIST = 64;

// scorer batches rotate over DEDUP_RING dedup regions by BatchHdr::seq: batch q's state stage
// clears the region of batch q + DEDUP_AHEAD (= q - 1's, consumed by then), so batch q+1's dedup
// insert (copy stream) can run while batch q is still in K1 / update_segments on the state stream.
// The copy of batch q waits for the state stage of batch q - DEDUP_AHEAD (the native driver keeps
// one post-state event per ring entry and only queues the wait when the host does not already see
// that batch complete). Eight regions let the pipeline run up to seven batches deep without that
// wait: with four, depth 4 collapsed (r4 NOTES). Region DEDUP_STANDALONE: event ingestion.
constexpr int DEDUP_RING = 8;
constexpr int DEDUP_AHEAD = DEDUP_RING - 1;
constexpr int DEDUP_STANDALONE = DEDUP_RING;
__host__ __device__ inline int dedup_ring_region(int seq) { return (int)((unsigned)seq % DEDUP_RING); }

// Dedup scratch: DEDUP_RING + 1 regions, each = keys/first/count/fill [cap] + list [cap][DEDUP_LIST] + mlist [dmax]
// + 2 counters (update.h dedup_region).
struct UpdateArgs {
  const ScoreCfg* cfg;
  const BatchHdr* hdr;      // scorer path: live count + seq parity (nullable -> n, region)
  int32_t n;
  int32_t n_max;            // grid coverage
  const ReqRec* req;        // events (ReqRec.ts = event time)
  uint32_t* ring_ts;
  int64_t* ring_amt;
  uint8_t* hll;
  AcctRT* rt;
  uint16_t* ev;             // event ring bf16 [C][ev_ring][16] (nullable)
  int32_t ring_size;
  int32_t ev_ring;
  int32_t ev_dim;
  int32_t* dbuf;
  int32_t dcap;             // power of two >= 2 * dmax
  int32_t dmax;
  int32_t region;           // -1: hdr->seq & 1; else fixed region (2 = standalone)
  // scorer dedup insert only (nullable): the pinned host slab [BatchHdr | ReqRec x n]; the kernel
  // reads the batch from it and writes the device copy (hdr, req) for the later stages
  const char* src;
  const int32_t* hll_lc;    // [257] linear-counting table (the cached HLL estimates, AcctRT)
  // scorer dedup insert of the rows-region exchange only (nullable): the rows come from this
  // owner's chunk of every sender's block of the node-shared rows region (sender p's chunk at
  // xrecv + p * xpstride: header record {slot = count, ts = sender clock} + up to xc rows); the
  // kernel compacts them into req (sender order, then row order), writes route[i] = p * xc + j,
  // route[n_max] = rows over capacity, and the header {n, seq (from xhdr), now}
  const ReqRec* xrecv;
  int32_t* route;
  const int4* xhdr;
  int32_t xn, xc;
  int32_t xpstride;
};

struct AssembleArgs {
  const BatchHdr* hdr;
  const ScoreCfg* cfg;
  const ReqRec* req;        // [n_rows]
  const uint32_t* ring_ts;
  const int64_t* ring_amt;
  const uint8_t* hll;       // [C][2][256]
  const AcctRT* rt;
  const AcctBatch* batch;
  const float* ext;         // [C][ext_width]
  const uint64_t* bl_keys;  // blacklist open-addressing table (nullable)
  const uint32_t* bl_exp;
  const uint64_t* ip_keys;  // ip-intel table (nullable)
  const uint32_t* ip_flags;
  const int32_t* hll_lc;    // [257]: floor(256 ln(256 / v) + 0.5), HLL linear counting by zero count v
  float* X;                 // [n_rows][x_stride]
  FeatRec* feat;            // [n_rows]
  // [n_rows][128 B] D2H image of each row (nullable): the raw FeatRec, or for a request with
  // ReqRec.tx_type bit FV_ENC_BIT the encoded risk.v1 FeatureVector body (features.hip write_fenc)
  uint8_t* fenc;
  // nullable: fenc is routed like EnsembleArgs::route - live row i's image goes to
  // fenc + p * fenc_stride + j * 128 bytes (route[i] = p * fenc_c + j); padding rows write none
  const int32_t* fenc_route;
  int32_t fenc_c;
  int32_t fenc_stride;
  int32_t* dbuf;            // dedup regions (nullable: no score-then-update)
  int32_t dcap;
  int32_t dmax;
  int32_t x_stride;
  int32_t ring_size;
  int32_t n_rows;           // rows covered by the launch (graph bucket)
  int64_t* trace;           // [8 waves][8] phase timestamps (nullable; tools/kbench.py --trace)
  // score-then-update (dbuf != null): the batch's dedup insert ran before K1 (dedup_insert);
  // each wave applies its request's event when it is the account's only one in the batch
  // and opens the segment of a multi-event account (applied by update_segments after K1)
  UpdateArgs upd;
};


void launch_feature_assemble(const AssembleArgs& a, hipStream_t st);
// standalone event ingestion (event bus / history replay): reset + insert + single + segments
void launch_feature_update(const UpdateArgs& a, hipStream_t st);
// scorer path: dedup insert of the batch (before K1; K1 applies single-event accounts) ...
void launch_dedup_insert(const UpdateArgs& a, hipStream_t st);
// ... and the tail after K1: segment fill + per-account wave apply of multi-event accounts
void launch_update_segments(const UpdateArgs& a, hipStream_t st);

// ---- K2 tree ensemble (complete layout)
struct EnsembleArgs {
  const BatchHdr* hdr;
  const ScoreCfg* cfg;
  const FeatRec* feat;
  const float* X;           // for the heuristic model
  int32_t x_stride;
  const float* ml;          // model output (nullable)
  ResultRec* out;
  ResultRec* host_out;      // nullable: pinned host rows written directly (no D2H copy node)
  unsigned long long* metrics;  // [128] score histogram(101) | actions(4) | ml_high | rows (nullable)
  int32_t n_rows;
  // nullable: host_out is routed - live row i goes to host_out + (p * route_stride bytes) + j rows,
  // route[i] = p * route_c + j (the exchange's compacted rows back into their senders' chunks of
  // the node-shared results region; padding rows are not written)
  const int32_t* route;
  int32_t route_c;
  int32_t route_stride;
};
struct TreeArgs {
  const BatchHdr* hdr;      // nullable: all n_rows live
  const float* X;           // [n][x_stride]
  const float2* nodes;      // [T][2^D-1] (threshold, meta bits)
  const float* leaves;      // [T][2^D][K]
  const float* base;        // [K] (nullable)
  float* out;               // [n][n_out]
  int32_t x_stride;
  int32_t n_rows;
  int32_t n_trees;
  int32_t depth;
  int32_t k;                // targets per leaf
  int32_t n_out;            // output columns (2 in the binary-classifier case)
  int32_t post;             // 0 none, 1 logistic, 2 softmax
  int32_t average;          // 1 = AVERAGE aggregate
  int32_t binary_class;     // -1 unless classifier binary case
  int32_t all_positive;
  int32_t no_finish;        // grouped launch: leave partials for the consumer (mlp_head)
  int32_t all_leq;          // every node BRANCH_LEQ (fast decision path; missing tracks allowed)
  int64_t* trace;           // nullable: phase trace of sample blocks (tools/tree_bench.py)
  int32_t fuse_ens;         // grouped launch: K5 in the finish kernel's epilogue (ml = out)
  EnsembleArgs ens;
};
void launch_tree_ensemble(const TreeArgs& a, hipStream_t st);
void launch_tree_ensemble_grouped(const TreeArgs& a, int groups, float* partial, hipStream_t st);

// ---- K2b general trees on the pointer layout (csrc/runtime/trees.h Sparse)
struct TreeSparseArgs {
  const float* X;           // [n][x_stride]
  const int32_t* nodes;     // [N][4] {meta, threshold bits, true child, false child | leaf row}
  const int32_t* roots;     // [T] root node of each tree
  const float* leaf_w;      // [L][K]
  const uint8_t* leaf_has;  // [L][K] target written by the leaf (MIN / MAX)
  const float* base;        // [K] (nullable)
  float* out;               // [n][n_out]
  int32_t x_stride;
  int32_t n_rows;
  int32_t n_trees;
  int32_t depth;            // longest root-to-leaf path (bounds the traversal loop)
  int32_t k;                // targets (<= 64)
  int32_t n_out;
  int32_t post;             // tree_post.h TreePostKind
  int32_t aggregate;        // 0 sum, 1 average, 2 min, 3 max
  int32_t binary_class;     // -1 unless classifier binary case
  int32_t all_positive;
  int32_t feat_w;           // largest feature id + 1 (the staged X tile width)
};
void launch_tree_sparse(const TreeSparseArgs& a, int groups, float* partial, hipStream_t st);

// ---- K3 dense layers: Y = act(X W^T + b)
struct GemmArgs {
  const void* X;            // [M][ldx] f32 or bf16
  const void* W;            // bf16 or f32 (w_f32) [N_pad][K_pad] (row n = output column n)
  const float* bias;        // [N] nullable
  void* Y;                  // [M][ldy] f32 or bf16
  const int32_t* m_ptr;     // live rows in device memory (nullable -> M)
  int32_t M, N, K;          // logical sizes; K_pad = round_up(K, 32)
  int32_t ldx, ldy, ldw;
  int32_t x_bf16, y_bf16;
  int32_t act;              // 0 none, 1 relu, 2 sigmoid, 3 tanh
  int32_t w_f32;            // 1: f32 weights, f32 MFMA (v_mfma_f32_16x16x4_f32), reference precision
};
void launch_gemm(const GemmArgs& a, hipStream_t st);
void launch_gemv(const GemmArgs& a, hipStream_t st);  // N == 1 heads

// DAG join of two branches (join.hip): op 0 Y = A + B (na columns), op 1 Y = [A | B]
struct JoinArgs {
  const void* A;
  const void* B;
  void* Y;
  const int32_t* m_ptr;     // live rows in device memory (nullable -> M)
  int32_t M, na, nb, op;
  int32_t lda, ldb, ldy;
  int32_t a_bf16, b_bf16, y_bf16;
};
void launch_join(const JoinArgs& a, hipStream_t st);

// dense(N1) + act1 + dense(N1 -> 1) + act2 fused; W1 bf16 [N1_pad(64)][k_pad(32)]
// ---- K5 ensemble + action + metrics
struct HeadArgs {
  const void* X;
  const void* W1;           // bf16, or f32 when w1_f32 (reference-precision head)
  const float* b1;          // [N1] nullable
  const float* w2;          // [N1] f32
  float b2;
  float* Y;                 // [M][ldy] f32 (column 0)
  const int32_t* m_ptr;
  int32_t M, K, N1, k_pad;
  int32_t ldx, ldy;
  int32_t x_bf16;
  int32_t act1, act2;
  // optional: X is a tree partial slab [groups][M][K] to be reduced (+base, /T) while staging
  const float* partial;
  const float* pbase;
  int32_t groups;
  int32_t p_average;
  int32_t p_ntrees;
  int64_t* trace;           // nullable: phase trace of 8 sample blocks (tools/kbench.py)
  // optional fused K5: each block runs the ensemble of its rows on the Y values it computed
  // (ml = Y[row], the plan's ml_col 0); the standalone ensemble launch is then skipped
  int32_t fuse_ens;
  EnsembleArgs ens;
  int32_t w1_f32;           // 1: f32 W1 / activations, v_mfma_f32_16x16x4_f32 (no bf16 rounding anywhere)
};
void launch_mlp_head(const HeadArgs& a, hipStream_t st);

// cfg3 stacked model in one launch (trees.hip tree_head_kernel): grouped K = 32 tree ensemble
// whose last-arriving group block per 64-row tile runs the f32 head (+ fused K5) on the tile.
// h.partial / h.groups describe the slab the tree blocks write; tile_cnt: zeroed uint32 per tile.
bool tree_head_supported(const TreeArgs& a, const HeadArgs& h, int groups);
void launch_tree_head(const TreeArgs& a, const HeadArgs& h, int groups, float* partial, unsigned int* tile_cnt,
                      hipStream_t st);

void launch_ensemble(const EnsembleArgs& a, hipStream_t st);

// Cluster counters of the weight-stationary GRU kernels (gru_ws.hip, gru_wsx.hip): a member
// whose bounded wait times out stores this value into its cluster's counters before it exits.
// Every later wait on them then fails as well (no launch can add its way back to a target from
// here), so counters that a failed launch left part-advanced are never passed early; the host
// zeroes them when it falls back (GruPack.disable_ws) - a successful launch leaves them at 0.
constexpr int32_t kClusterPoison = -(1 << 30);

// ---- K4 GRU sequence (recurrent weights resident in VGPRs)
// ---- K4 GRU (1-2 stacked ONNX GRU layers, forward, layout 0) + optional N=1 head
// Weights are fragment-packed on the host: P[nt][ks][lane][8] = W[nt*16 + (lane&15)]
// [ks*32 + 8*(lane>>4) + j], so one wave load of a B fragment is 1 KiB contiguous.
struct GruLayerArgs {
  const uint16_t* W;        // packed bf16, N = 3H rows, K = kx_pad (input dim padded to 32)
  const uint16_t* R;        // packed bf16, N = 3H rows, K = H
  const float* bias;        // [6H]: Wb z,r,h | Rb z,r,h
  int32_t kx_pad;
  int32_t lbr;              // linear_before_reset
  const uint16_t* W_lo;     // split mode: bf16 residuals (w - bf16(w)), same fragment order
  const uint16_t* R_lo;
};
struct GruArgs {
  GruLayerArgs layer[2];
  int32_t n_layers, H, T, I;
  // input: mode 0 dense X f32 [T][x_rows][I]; mode 1 per-account event ring (bf16 [C][ring][I])
  int32_t mode;
  const float* X;
  int32_t x_rows;
  const uint16_t* ev;
  const AcctRT* rt;
  const int32_t* slots;     // [rows] (-1 -> empty history)
  int32_t ev_ring;
  const int32_t* m_ptr;     // live row count on device (nullable)
  int32_t n_rows;
  float* yh;                // [rows][H] last layer's final hidden state (nullable)
  const float* head_w;      // [H] (nullable): out[r] = act(h . w + b)
  float head_b;
  int32_t head_act;         // 0 none, 2 sigmoid
  float* out;               // [rows]
  int32_t tile_rows;        // 0 auto | 16 | 32 rows per workgroup
  int32_t waves;            // 0 auto (4) | 8 waves per workgroup (H >= 128)
  int32_t pipeline;         // 2 layers: layer-pipelined kernel (layer 1 @ t || layer 2 @ t-1)
  // weight-stationary cluster path (gru_ws.hip), used when the workspace is given and the
  // model is the 2 x 256, linear_before_reset = 1, input <= 32 shape
  int32_t ws;               // 0 off | 1 use when eligible | 2 two-half pipeline | 3 two 64-row clusters per CU
  int32_t ws_clusters;      // workspace capacity in 128-row clusters
  int32_t* ws_sync;         // [2 ws_clusters][16] step counters (back to 0 after every launch)
  uint16_t* ws_x;           // [ws_clusters][2][8][2][128][32] bf16 hand-off slabs
  float* ws_part;           // [ws_clusters][8][128] head partials
  int32_t* ws_err;          // [1] set when a cluster was not co-resident (bounded wait expired)
  int64_t* ws_trace;        // [64][6] phase timestamps of workgroup 0 (nullable; tools/gru_bench.py)
  int32_t split;            // 1: f32-faithful bf16 hi/lo pairs, three MFMAs per product (gru.hip x3)
  int32_t reverse;          // 1: ONNX direction=reverse (every layer): time steps read last to first
};
void launch_gru(const GruArgs& a, hipStream_t st);
bool gru_ws_eligible(const GruArgs& a);
void launch_gru_ws(const GruArgs& a, hipStream_t st);
int gru_ws_clusters(int n_rows);
int gru_ws2_clusters(int n_rows);  // 64-row clusters (ws = 3)
// split (f32-faithful) weight-stationary clusters of 16 workgroups x 32 rows (gru_wsx.hip);
// the workspace is then sized in 32-row clusters: ws_sync [clusters][16], ws_x
// [clusters][2][16][4][32][16] bf16, ws_part [clusters][16][32]
bool gru_wsx_eligible(const GruArgs& a);
void launch_gru_wsx(const GruArgs& a, hipStream_t st);
int gru_wsx_clusters(int n_rows);

// ---- K9 LTV / churn / segment
struct LtvArgs {
  const float* pf;          // [B][25] player features (golden.ltv.PLAYER_COLUMNS), or the table when slots != null
  const int32_t* slots;     // [B] rows of the device-resident player table (nullable; -1 -> empty profile)
  const float* ltv_model;   // [B] learned LTV (nullable -> formula)
  float* out;               // [B][6]: ltv, churn, survival, confidence, segment, nba
  int32_t B;
};
void launch_ltv(const LtvArgs& a, hipStream_t st);

// LTV model input from the device-resident tables: X[r] = [sign*log1p|pf[slot]| (25) | ext[slot] (ext_w)]
struct LtvAssembleArgs {
  const int32_t* slots;
  const float* pf_tab;      // [C][25]
  const float* ext_tab;     // [C][ext_w] (nullable)
  int32_t ext_w;
  float* X;                 // [rows][x_w], x_w = 25 + ext_w
  int32_t x_w;
  const int32_t* m_ptr;     // live rows (nullable)
  int32_t n_rows;
};
void launch_ltv_assemble(const LtvAssembleArgs& a, hipStream_t st);

// ---- K3 fused MLP chain (mlp_fused.hip): up to 8 dense layers with the activation tile in LDS,
// the last one followed by an N -> 1 head; optional LTV input gather and K9 epilogue
constexpr int MC_MAX_LAYERS = 8;
struct MlpChainArgs {
  const float* X;           // dense input [rows][ldx] f32 (when slots == null)
  int32_t ldx;
  const int32_t* slots;     // LTV gather: player slots [rows] (-1: empty profile)
  const float* pf_tab;      // [C][25]
  const float* ext_tab;     // [C][ext_w] (nullable)
  int32_t ext_w;
  int32_t in_w;             // staged input width = K[0] (multiple of 64)
  int32_t in_live;          // real input columns (<= in_w; the rest are zero)
  const int32_t* m_ptr;     // live rows in device memory (nullable)
  int32_t n_rows;
  int32_t n_layers;
  const uint16_t* W[MC_MAX_LAYERS];  // bf16 [N][K] row-major
  const float* bias[MC_MAX_LAYERS];  // [N] (nullable)
  int32_t N[MC_MAX_LAYERS];          // multiple of 64, <= 512
  int32_t K[MC_MAX_LAYERS];          // multiple of 64, <= 512; K[l] == N[l-1]
  int32_t act[MC_MAX_LAYERS];
  const float* w2;          // head [N_last] f32
  float b2;
  int32_t act2;
  float* ml;                // [rows] head output (nullable)
  float* ltv_out;           // [rows][6] K9 output (nullable; needs slots + pf_tab)
  int32_t rows_per_block;   // 16, 32 (default) or 64 rows per workgroup
  int32_t waves;            // 4 (default) or 8 (32 rows; each wave owns N/8 columns)
  const uint16_t* W_lo[MC_MAX_LAYERS];  // split (f32-faithful) mode: bf16 residuals w - bf16(w)
  int32_t split;            // 1: three-MFMA bf16 pairs (hi*hi + hi*lo + lo*hi)
};
void launch_mlp_chain(const MlpChainArgs& a, hipStream_t st);

}  // namespace igp
