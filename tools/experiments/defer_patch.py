# Patch for tools/experiments/calib_build.sh: test each walk step's gate blocks one walk step after
# their loads (kScanG, no stage-1 fold), with the pending x pair carried in registers instead of LDS.
# Needs the VGPR room of 3 waves/SIMD (build with -DKHB_WAVES_PER_SIMD=3).  Exact (same candidates).
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = """// Gate bits of x (blocked gate), or without a gate L1 bit 0 (a = the first XXH64)."""
b = """// A walk step's gate test in flight: both blocks loaded, tested one walk step later.
struct GateDefer {
  GatePend q1, q2;
  Fe x1, x2;
  uint32_t s1, s2;
  bool has2;
};

__device__ __forceinline__ GateDefer gate_defer_issue(const ScanArgs& A, const Fe& x1, uint32_t s1, bool has2,
                                                      const Fe& x2, uint32_t s2) {
  return GateDefer{gate_issue(A, x1), gate_issue(A, x2), x1, x2, s1, s2, has2};
}

__device__ __forceinline__ void gate_defer_resolve(const ScanArgs& A, ProbeQueue& Q, const GateDefer& d,
                                                   uint32_t job) {
  const bool h1 = d.q1.pass(), h2 = d.has2 && d.q2.pass();
  if (__ballot(h1 || h2) == 0) return;
  q_push(Q, h1, d.x1, job, d.s1);
  q_drain(A, Q, kDrainAt);
  q_push(Q, h2, d.x2, job, d.s2);
  q_drain(A, Q, kDrainAt);
}

// Gate bits of x (blocked gate), or without a gate L1 bit 0 (a = the first XXH64)."""
assert a in s; s = s.replace(a, b)
a = """    x_out<kScanG>(A, x1);
    gate_pair<STAGE1>(A, Q, x1, base, false, x1, 0, job);
  }"""
b = """    x_out<kScanG>(A, x1);
    if constexpr (STAGE1) gate_pair<STAGE1>(A, Q, x1, base, false, x1, 0, job);
  }
  GateDefer D;
  if constexpr (!STAGE1) D = gate_defer_issue(A, x1, base, false, x1, 0);"""
assert a in s; s = s.replace(a, b)
a = """    gate_pair<STAGE1>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);
  }
  probe<false>(A, Q, C.x, job, j, kHalf);        // the centre, pts[512]"""
b = """    if constexpr (STAGE1) {
      gate_pair<STAGE1>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);
    } else {
      const GateDefer N = gate_defer_issue(A, x1, base + kHalf - 1 - (uint32_t)i, true, x2,
                                           base + kHalf + 1 + (uint32_t)i);
      gate_defer_resolve(A, Q, D, job);
      D = N;
    }
  }
  if constexpr (!STAGE1) gate_defer_resolve(A, Q, D, job);
  probe<false>(A, Q, C.x, job, j, kHalf);        // the centre, pts[512]"""
assert a in s; s = s.replace(a, b)
open(p, 'w').write(s)
