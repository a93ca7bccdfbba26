// k_giant_scan instances for -m address / -m rmd160 with -e (endomorphism: the hashes of beta*x and beta^2*x and,
// for uncompressed keys, of the negated points; keyhunt.cpp:2646-2763), in a translation unit of their own so that
// `make -j` compiles them beside the plain address kernels (k_addr.hip).
#include "scan_kernels.hpp"

namespace khbk {

void launch_addr_e(int mode, uint32_t blocks, hipStream_t stream, const ScanArgs& A) {
  switch (mode) {
    case kAddrUE: hipLaunchKernelGGL(k_giant_scan<kAddrUE>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kAddrCE: hipLaunchKernelGGL(k_giant_scan<kAddrCE>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    case kAddrBE: hipLaunchKernelGGL(k_giant_scan<kAddrBE>, dim3(blocks), dim3(kBlock), 0, stream, A); break;
    default: break;
  }
}

}  // namespace khbk
