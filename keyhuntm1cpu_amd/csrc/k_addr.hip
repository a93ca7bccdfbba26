// k_giant_scan instances for -m address / -m rmd160 (uncompress, compress, both) and the x||y dump (scan_kernels.hpp).
#include "scan_kernels.hpp"

namespace khbk {

void launch_addr(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A) {
  switch (mode) {
    case kAddrU: hipLaunchKernelGGL(k_giant_scan<kAddrU>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kAddrC: hipLaunchKernelGGL(k_giant_scan<kAddrC>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kAddrB: hipLaunchKernelGGL(k_giant_scan<kAddrB>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kAddrDump: hipLaunchKernelGGL(k_giant_scan<kAddrDump>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    default: break;
  }
}

}  // namespace khbk
