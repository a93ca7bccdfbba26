# Timing-only patch for tools/experiments/calib_build.sh (round 5): the prefix stream with plain loads and stores
# (plainscr_patch.py) folded to (i & KHB_SCR_MASK) entries per group (scr_patch.py), so that it stays in the caches:
# KHB_SCR_MASK=1 keeps 2 entries per group (134 MB per slot at 262,144 lanes), 0 keeps 1 (67 MB).  Results are wrong
# by design (the walk reads the wrong prefixes); perf_variants skips their parity check (TIMING_ONLY).
import runpy
import os
here = os.path.dirname(os.path.abspath(__file__))
runpy.run_path(os.path.join(here, "plainscr_patch.py"))
runpy.run_path(os.path.join(here, "scr_patch.py"))
