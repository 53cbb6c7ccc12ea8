// CPU model devices of the native account-RPC core (model_ops.h): the GPU-less / degraded
// twins of the GPU LTV chain and abuse step (csrc/kernels/model_driver.hip), GIL-free.
//
// * CpuLtvDevice    K9 (csrc/include/ltv_logic.h, the same row logic as the kernels) over the
//                   host player table (engine/ltv.py PlayerTable rows of this owner), with the
//                   learned LTV model through exec::Executor when one is loaded
// * CpuAbuseDevice  the account's live feature row (CpuScorer::features, K1's host twin) and
//                   the sequence model over its event history (exec::Executor)
// Python twins (the per-call engine path): engine/ltv.py LtvService._cpu, engine/abuse.py
// AbuseService.check.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../include/model_ops.h"
#include "../include/records.h"
#include "cpu_scorer.h"
#include "executor.h"

namespace igp {

class CpuLtvDevice {
 public:
  // rows: [capacity][25] f32 profile rows; present: [capacity] (nonzero: profile loaded); ext:
  // [capacity][ext_w] (nullable). The arrays belong to the caller and outlive the device.
  CpuLtvDevice(const float* rows, const uint8_t* present, const float* ext, int ext_w, int64_t capacity,
               std::shared_ptr<exec::Executor> model, std::string in_name, std::string out_name, int model_width,
               int depth, int cap);
  const IgpModelOps* ops() const { return &ops_; }

 private:
  struct Slot {
    std::vector<int32_t> slots;
    std::vector<float> out;
  };
  void run(Slot& s, int n);
  const float* rows_;
  const uint8_t* present_;
  const float* ext_;
  int ext_w_;
  int64_t cap_rows_;
  std::shared_ptr<exec::Executor> model_;
  std::string in_, out_;
  int width_;
  std::vector<Slot> slots_;
  IgpModelOps ops_{};
};

class CpuAbuseDevice {
 public:
  CpuAbuseDevice(std::shared_ptr<CpuScorer> sc, std::shared_ptr<exec::Executor> model, std::string in_name,
                 std::string out_name, int depth, int cap);
  const IgpModelOps* ops() const { return &ops_; }

 private:
  struct Slot {
    std::vector<int32_t> slots;
    std::vector<float> score;
    std::vector<FeatRec> feat;
  };
  void run(Slot& s, int n, int64_t now);
  std::shared_ptr<CpuScorer> sc_;
  std::shared_ptr<exec::Executor> model_;
  std::string in_, out_;
  std::vector<Slot> slots_;
  IgpModelOps ops_{};
};

}  // namespace igp
