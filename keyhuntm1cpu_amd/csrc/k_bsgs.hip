// k_giant_scan instances for -m bsgs: the scan (ungated, gated, gated with the stage-1 fold) and the
// x dump (kDump: the 8 x 32 walk; kDumpG: the 9 x 29-bit walk when KHB_F9WALK builds it).
#include "scan_kernels.hpp"

namespace khbk {

void launch_bsgs(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A) {
  switch (mode) {
    case kScan: hipLaunchKernelGGL(k_giant_scan<kScan>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kScanG: hipLaunchKernelGGL(k_giant_scan<kScanG>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kScanG1: hipLaunchKernelGGL(k_giant_scan<kScanG1>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
#if KHB_F9WALK
    case kDumpG: hipLaunchKernelGGL(k_giant_scan<kDumpG>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
#else
    case kDump: hipLaunchKernelGGL(k_giant_scan<kDump>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
#endif
    default: break;
  }
}

}  // namespace khbk
