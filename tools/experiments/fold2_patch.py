# Timing patch for tools/experiments/calib_build.sh: the stage-1 fold tested with probes 0 and 1 only (the
# full gate still tests all three, so the candidates are unchanged): ~3 VALU less per x against more x
# reading the full gate.
p = 'keyhuntm1cpu_amd/csrc/scan_kernels.hpp'
s = open(p).read()
a = "const bool s1 = gate_block_pass(f1.x, f1.y, x1.v[1], gm), s2 = has2 && gate_block_pass(f2.x, f2.y, x2.v[1], gm);"
b = ("const GateMask fm{gm.m1, 1u};\n"
     "    const bool s1 = gate_block_pass(f1.x, f1.y, x1.v[1], fm), s2 = has2 && gate_block_pass(f2.x, f2.y, x2.v[1], fm);")
assert a in s
s = s.replace(a, b)
open(p, 'w').write(s)
