// C ABI between the native account-RPC core (host runtime, _native: csrc/runtime/acct_core.cpp)
// and the devices that run its per-account models in micro-batches:
//   * GPU  (_hipk ModelDriver, csrc/kernels/model_driver.hip): the LTV chain (gather + MLP + K9
//          epilogue in one kernel) or the abuse step (K1 feature rows + the GRU over the HBM
//          event rings), recorded launches or captured graphs per (bucket, slot)
//   * CPU  (_native CpuLtvDevice / CpuAbuseDevice, csrc/runtime/acct_devices.cpp)
// A request row is just the account's feature-store slot on the owner shard (-1: unknown
// account). Same conventions as device_ops.h: the core calls the table from its own threads
// without the GIL; a slot's host buffers stay untouched by the device until its next submit.
#pragma once
#include <stdint.h>

#define IGP_MODEL_OPS_ABI 1

#ifdef __cplusplus
extern "C" {
#endif

enum { IGP_MODEL_LTV = 1, IGP_MODEL_ABUSE = 2 };

typedef struct IgpModelOps {
  uint32_t abi;        // IGP_MODEL_OPS_ABI
  int32_t kind;        // IGP_MODEL_LTV | IGP_MODEL_ABUSE
  int32_t depth;       // pipeline slots
  int32_t cap;         // rows per batch
  int32_t has_model;   // ABUSE: out0 carries the sequence model's score
  int32_t pad;
  void* ctx;
  // the slot's request rows: int32 slots [cap] (pinned host memory for GPU devices)
  int32_t* (*slots)(void* ctx, int32_t slot);
  // launch the slot's batch of n rows at clock `now` (unix s). 0, or -1 with a message in err
  int32_t (*submit)(void* ctx, int32_t slot, int32_t n, int64_t now, char* err, int32_t errlen);
  // block until the slot's batch completed: 0 ok, 1 timeout (timeout_us >= 0), -1 error
  int32_t (*wait)(void* ctx, int32_t slot, int64_t timeout_us, char* err, int32_t errlen);
  // results of the slot's last batch, row order:
  //   LTV    out0 = float [n][6]: ltv, churn, survival days, confidence, segment, next-best-action id
  //   ABUSE  out0 = float [n] model score (unused when has_model == 0), out1 = FeatRec [n] (records.h)
  const void* (*out0)(void* ctx, int32_t slot);
  const void* (*out1)(void* ctx, int32_t slot);
} IgpModelOps;

#ifdef __cplusplus
}
#endif
