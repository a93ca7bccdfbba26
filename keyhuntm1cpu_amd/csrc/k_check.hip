// k_check: the second and third check of level-1 candidates on the device (khb_check),
// bsgs_secondcheck / bsgs_thirdcheck of keyhunt.cpp:4271-4368 as restated in device/confirm.hpp.
// One lane per candidate; 64-lane workgroups (a batch is a few to a few thousand candidates).
#include <hip/hip_runtime.h>

#include "check_kernel.hpp"

namespace khbk {

__global__ __launch_bounds__(64) void k_check(khb::CheckTables T, const CheckIn* __restrict__ in,
                                              const khb::CPt* __restrict__ targets, uint32_t n_targets,
                                              CheckOut* __restrict__ out, uint32_t n) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const CheckIn c = in[g];
  khb::CheckResult r{};
  CheckOut o{};
  if (c.target < n_targets) {
    const khb::CPt t = targets[c.target];
    o.found = khb::second_check(T, c.start, c.a, t, r) ? 1u : 0u;
  } else {
    o.found = 0xffffffffu;                     // rejected on the host before the launch; never reached
  }
  o.key = r.key;
  o.l2_hits = r.l2_hits;
  o.l3_hits = r.l3_hits;
  o.bp_hits = r.bp_hits;
  out[g] = o;
}

void launch_check(hipStream_t stream, const khb::CheckTables& T, const CheckIn* in, const khb::CPt* targets,
                  uint32_t n_targets, CheckOut* out, uint32_t n) {
  hipLaunchKernelGGL(k_check, dim3((n + 63) / 64), dim3(64), 0, stream, T, in, targets, n_targets, out, n);
}

}  // namespace khbk
