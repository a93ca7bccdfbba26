#!/bin/bash
# Where the idle VALU quad-cycles go (round 5): SQ_ACTIVE_INST_VALU / _VALU2 / GRBM_GUI_ACTIVE over one bench-sized
# launch of the product with the real gate, with the all-zero gate (no gate misses), and of the cache-resident prefix
# stream build (scr1plain, timing only).  tools/pmc_summary.py's formula.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-util_ab}; mkdir -p $O
L=keyhuntm1cpu_amd/lib/libkhbsgs.so
V=keyhuntm1cpu_amd/lib/variants
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
JOBS=4096 GATE=1 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc $C -d $O/real -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/real.log 2>&1 || exit 1
JOBS=4096 GATE=1 GATE_ZERO=13 ROUNDS=1 timeout -s KILL 200 rocprofv3 --pmc $C -d $O/zero -o pmc --output-format csv -- python3 tools/perf_variants.py $L > $O/zero.log 2>&1 || exit 1
JOBS=4096 GATE=1 ROUNDS=1 TIMING_ONLY=scr1plain timeout -s KILL 200 rocprofv3 --pmc $C -d $O/scr1 -o pmc --output-format csv -- python3 tools/perf_variants.py $V/libkhbsgs_scr1plain.so > $O/scr1.log 2>&1 || exit 1
python3 - "$O" <<'PY'
import csv, collections, glob, sys
o = sys.argv[1]
for tag in ("real", "zero", "scr1"):
    f = sorted(glob.glob(f"{o}/{tag}/**/*counter_collection.csv", recursive=True))[-1]
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "k_giant_scan" in r["Kernel_Name"]:
            d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for did in sorted(d)[-2:]:
        q = d[did]
        quads = 1024 * q["GRBM_GUI_ACTIVE"] / 8 / 4
        print(tag, did, "util %.2f %%" % (100 * (q["SQ_ACTIVE_INST_VALU"] - q["SQ_ACTIVE_INST_VALU2"]) / quads),
              "dual %.3f" % (2 * q["SQ_ACTIVE_INST_VALU2"] / q["SQ_INSTS_VALU"]),
              "wait_inst_any/wave_cycles %.3f" % (q["SQ_WAIT_INST_ANY"] / q["SQ_WAVE_CYCLES"]),
              "grbm %.3e" % q["GRBM_GUI_ACTIVE"])
PY
