// Timing-only experiment (round 5), spliced into keyhuntm1cpu_amd/csrc/scan_kernels.hpp by
// tools/experiments/half_patch.py (calib_build.sh half <name>): the half prefix stream.  Exact (the same x),
// measured +1.1 % whole-bench and -1.7 % kernel time, below the 2 % bar for the product (DESIGN.md §5,
// profiles/r05d, r05e).
// walk_group_g over the half prefix stream (KHB_HALF_STREAM): the forward pass stored only the odd prefixes.
// After the peeled step 511 the walk goes in pairs (even i, odd i - 1): the even step needs P_{i-1}, stored,
// and then loads P_{i-3}; the odd step rebuilds P_{i-2} = P_{i-3} * dx_{i-2} (one extra product per pair).
// Same points, same order and bit-identical x: P_{i-2} is the forward pass's own product of the same
// operands in the same order.
template <bool STAGE1>
__device__ __forceinline__ void half_points(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, const Fe& negCx,
                                            const Fe& negCy, const Fe& idx, int i, uint32_t base, uint32_t job) {
  const GsnTable gsn{A.gsn};
  Fe u, s, x1, x2;
  const AffPt g = gsn.pt(i);
  fm_add_lazy(u, gsn.nx(i), negCx);             // nu = -(C.x + GSn.x)
  fm_add_lazy(s, g.y, C.y);
  fm_mul(s, s, idx);
  fm_sqr_add(x1, s, u);
  x_out<kScanG>(A, x1);
  fm_add_lazy(s, g.y, negCy);
  fm_mul(s, s, idx);
  fm_sqr_add(x2, s, u);
  x_out<kScanG>(A, x2);
  gate_pair<STAGE1>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);
}

template <bool STAGE1>
__device__ __forceinline__ void walk_group_g_half(const ScanArgs& A, ProbeQueue& Q, const AffPt& C, Fe inv,
                                                  uint32_t job, uint32_t j, const Fe* scr) {
  const size_t S = A.stride;
  const GsnTable gsn{A.gsn};
  const uint32_t base = j * KHB_GROUP;
  Fe negCx, negCy;
  {
    Fe p;
#pragma unroll
    for (int k = 0; k < 8; ++k) p.v[k] = k == 0 ? KHB_P0 : (k == 1 ? KHB_P1 : 0xFFFFFFFFu);
    fm_sub(negCx, p, C.x);
    fm_sub(negCy, p, C.y);
  }
  Fe pre = scr_ld(scr + (size_t)(kHalf - 3) * S);          // P_509
  Fe idx, dx;
  // odd step 511: pts[0] = C - GSn[511] only
  {
    Fe u, s, x1;
    fm_add_lazy(dx, gsn.x(kHalf - 2), negCx);
    fm_mul(idx, pre, dx);                                  // P_510 = P_509 * dx_510
    fm_mul(idx, inv, idx);
    fm_add_lazy(dx, gsn.x(kHalf - 1), negCx);
    fm_mul(inv, inv, dx);
    const AffPt g = gsn.pt(kHalf - 1);
    fm_add_lazy(u, gsn.nx(kHalf - 1), negCx);
    fm_add_lazy(s, g.y, C.y);
    fm_mul(s, s, idx);
    fm_sqr_add(x1, s, u);
    x_out<kScanG>(A, x1);
    gate_pair<STAGE1>(A, Q, x1, base, false, x1, 0, job);
  }
  // pairs (even i, odd i - 1), i = 510 ... 2; pre = P_{i-1} on entry
  for (int i = (int)kHalf - 2; i >= 2; i -= 2) {
    fm_mul(idx, inv, pre);                                 // even step i: P_{i-1} (odd index, stored)
    if (i > 2) pre = scr_ld(scr + (size_t)(i - 3) * S);    // P_{i-3} for step i - 1 (and i - 2)
    fm_add_lazy(dx, gsn.x(i), negCx);
    fm_mul(inv, inv, dx);
    half_points<STAGE1>(A, Q, C, negCx, negCy, idx, i, base, job);
    // odd step i - 1: P_{i-2} = P_{i-3} * dx_{i-2} (i - 1 = 1: P_0 = dx_0)
    fm_add_lazy(dx, gsn.x(i - 2), negCx);
    if (i > 2) {
      fm_mul(idx, pre, dx);
      fm_mul(idx, inv, idx);
    } else {
      fm_mul(idx, inv, dx);
    }
    fm_add_lazy(dx, gsn.x(i - 1), negCx);
    fm_mul(inv, inv, dx);
    half_points<STAGE1>(A, Q, C, negCx, negCy, idx, i - 1, base, job);
  }
  half_points<STAGE1>(A, Q, C, negCx, negCy, inv, 0, base, job);     // step 0: idx = inv
  probe<false>(A, Q, C.x, job, j, kHalf);
}

