// K9 row logic for the kernels (ltv.hip, mlp_fused.hip): the shared definition in
// csrc/include/ltv_logic.h with device qualifiers.
#pragma once
#include <hip/hip_runtime.h>

#define IGP_LTV_FN __device__ __forceinline__
#include "../include/ltv_logic.h"
