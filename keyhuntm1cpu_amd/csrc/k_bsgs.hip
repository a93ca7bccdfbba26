// k_giant_scan instances for -m bsgs: the scan (ungated, gated, gated with the stage-1 fold, and with the stage-0 filter in front of it) and the
// x dump (kDump) of the same walk for parity tests.
#include "scan_kernels.hpp"

namespace khbk {

void launch_bsgs(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A) {
  switch (mode) {
    case kScan: hipLaunchKernelGGL(k_giant_scan<kScan>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kScanG: hipLaunchKernelGGL(k_giant_scan<kScanG>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kScanG1: hipLaunchKernelGGL(k_giant_scan<kScanG1>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kScanG2: hipLaunchKernelGGL(k_giant_scan<kScanG2>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kDump: hipLaunchKernelGGL(k_giant_scan<kDump>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    default: break;
  }
}

}  // namespace khbk
