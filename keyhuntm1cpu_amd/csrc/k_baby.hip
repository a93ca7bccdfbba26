// k_giant_scan instance for the baby-step table build (kBaby, khb_build_baby; scan_kernels.hpp).
#include "scan_kernels.hpp"

namespace khbk {

void launch_baby(uint32_t blocks, hipStream_t stream, const ScanArgs& A) {
  hipLaunchKernelGGL(k_giant_scan<kBaby>, dim3(blocks), dim3(kBlock), 0, stream, A);
}

}  // namespace khbk
