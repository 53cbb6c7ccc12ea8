// C ABI between the native serving core (host runtime, _native: csrc/runtime/serve_core.cpp)
// and the device pipelines that execute its micro-batches:
//   * the single-GPU three-stream pipeline      (_hipk PipeDriver,  csrc/kernels/driver.hip)
//   * the owner-routed RCCL exchange pipeline   (_hipk XchgDriver,  csrc/kernels/exchange.hip)
//   * CPU shards                                 (_native CpuDevice / ShmXchgDevice, cpu_device.cpp)
// A plain function table keeps the two extension modules independent (no shared C++ types
// across the module boundary): a device hands out a pointer to its table, the core calls it
// from its own threads without the GIL.
#pragma once
#include <stdint.h>

#define IGP_DEVICE_OPS_ABI 4

#ifdef __cplusplus
extern "C" {
#endif

typedef struct IgpDeviceOps {
  uint32_t abi;       // IGP_DEVICE_OPS_ABI
  int32_t depth;      // pipeline slots (batches in flight)
  int32_t world;      // ranks of the exchange (1: single-shard pipeline)
  int32_t exchange;   // 0: rows = [cap] ReqRec of one batch; 1: rows = [world][cap + 1] ReqRec owner chunks
  int32_t cap;        // rows per batch (exchange: per-owner chunk capacity C)
  int32_t features_always;  // 1: results always carry FeatRec rows (exchange: fixed-size collectives)
  void* ctx;
  // the slot's host request buffer (pinned for GPU devices); valid once the slot's previous
  // batch was waited for
  char* (*rows)(void* ctx, int32_t slot);
  // launch the slot's batch: n live rows (exchange: ignored, counts ride in the chunk
  // headers), batch sequence number, scoring clock. Returns 0, or -1 with a message in err.
  int32_t (*submit)(void* ctx, int32_t slot, int32_t n, int32_t seq, int64_t now, int32_t want_features, char* err,
                    int32_t errlen);
  // block until the slot's batch completed: 0 ok, 1 timeout (timeout_us >= 0), -1 error
  int32_t (*wait)(void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen);
  // results of the slot's last batch. exchange == 0: ResultRec[n] and FeatRec[n] (features may
  // be null when not requested). exchange == 1: the returned chunks, [world][cap * W] bytes (or
  // res_owner_stride apart)
  // with W = 8 (+128 with features): cap ResultRec, then cap FeatRec per owner; features()
  // is unused.
  const void* (*results)(void* ctx, int32_t slot);
  const void* (*features)(void* ctx, int32_t slot);
  // exchange == 1: bytes from one owner's chunk to the next in results() (0: cap * W, the
  // chunks back to back). The per-GPU D2H result path hands out a node-shared region laid out
  // [owner][sender][cap * W], so a sender's chunks are world * cap * W apart.
  int64_t res_owner_stride;
} IgpDeviceOps;

#ifdef __cplusplus
}
#endif
