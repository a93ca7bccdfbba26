# Timing experiment (round 5) for tools/experiments/calib_build.sh: issue the stage-1 fold load of a walk step's first
# x before its second x is computed (a scheduling barrier keeps the load there), so ~half a step of VALU work covers
# its L2 latency; the second x's load is issued as before.  Exact (the same test on the same words): perf_variants
# compares its candidates with the product's.  Round 2 measured the same idea with the whole gate in the MALL
# (no gain); round 5's fold serves 83 % of the probes from L2 and the zero-gate PMC shows 4.3 points of VALU
# utilisation lost to the gate's misses (profiles/r05l).
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = '''// Gate bits of x (blocked gate), or without a gate L1 bit 0 (a = the first XXH64).'''
b = '''// gate_pair with the first x's stage-1 block already loaded (early_patch.py)
__device__ __forceinline__ void gate_pair_pre(const ScanArgs& A, ProbeQueue& Q, const Fe& x1, uint2 f1, uint32_t step1,
                                              const Fe& x2, uint32_t step2, uint32_t job) {
  const uint32_t s2 = gate_s2(A);
  const GateBits b1 = gate_bits(x1.v[1], s2), b2 = gate_bits(x2.v[1], s2);
  const uint2 f2 = gate_block(A.gate1, A.gate1_mask, x2);
  const bool s1 = gate_block_pass(f1, b1), s2p = gate_block_pass(f2, b2);
  if (__ballot(s1 || s2p) == 0) return;
  uint2 w1, w2;
  if (s1) w1 = gate_block(A.gate, A.gate_mask, x1);
  if (s2p) w2 = gate_block(A.gate, A.gate_mask, x2);
  const bool h1 = s1 && gate_block_pass(w1, b1);
  const bool h2 = s2p && gate_block_pass(w2, b2);
  if (__ballot(h1 || h2) == 0) return;
  q_push(Q, h1, x1, job, step1);
  q_drain(A, Q, kDrainAt);
  q_push(Q, h2, x2, job, step2);
  q_drain(A, Q, kDrainAt);
}

''' + a
assert a in s
s = s.replace(a, b, 1)
a = '''    fm_sqr_add(x1, s, u);
    x_out<kScanG>(A, x1);
    fm_add_lazy(s, g.y, negCy);               // GSn.y - C.y
    fm_mul(s, s, idx);
    fm_sqr_add(x2, s, u);
    x_out<kScanG>(A, x2);
    gate_pair<STAGE1>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);'''
b = '''    fm_sqr_add(x1, s, u);
    x_out<kScanG>(A, x1);
    uint2 f1{};
    if constexpr (STAGE1) {
      f1 = gate_block(A.gate1, A.gate1_mask, x1);
      __builtin_amdgcn_sched_barrier(0);
    }
    fm_add_lazy(s, g.y, negCy);               // GSn.y - C.y
    fm_mul(s, s, idx);
    fm_sqr_add(x2, s, u);
    x_out<kScanG>(A, x2);
    if constexpr (STAGE1)
      gate_pair_pre(A, Q, x1, f1, base + kHalf - 1 - (uint32_t)i, x2, base + kHalf + 1 + (uint32_t)i, job);
    else
      gate_pair<STAGE1>(A, Q, x1, base + kHalf - 1 - (uint32_t)i, true, x2, base + kHalf + 1 + (uint32_t)i, job);'''
assert a in s
s = s.replace(a, b, 1)
open(p, 'w').write(s)
