// Device-side records of khb_check (k_check.hip) shared with the ABI layer (khbsgs.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device/confirm.hpp"

namespace khbk {

struct CheckIn {            // khb_check_in with the chunk base as little-endian limbs
  khb::U8 start;
  uint32_t a;
  uint32_t target;
};

struct CheckOut {
  khb::U8 key;
  uint32_t found, l2_hits, l3_hits, bp_hits;
};

void launch_check(hipStream_t stream, const khb::CheckTables& T, const CheckIn* in, const khb::CPt* targets,
                  uint32_t n_targets, CheckOut* out, uint32_t n);

}  // namespace khbk
