#!/bin/bash
# Timing-only calibration builds of the product walk (round 3, profiles/r03_calibration/): apply a
# temporary patch to device/fe_asm.hpp, build lib/variants/libkhbsgs_<name>.so, restore the source.
#   pad_patch.py: after every field multiply, KHB_PAD_N instructions of kind KHB_PAD_OP
#                 (1 v_mov, 2 v_add_u32, 3 v_add_co, 4 v_addc, 5 mad->vcc, 6 mad->sgpr, 7 v_mul_lo,
#                 8 s_nop, 9 v_add3) in 4 independent chains; KHB_PAD_OP=0 is the barrier-only control.
#   rm_patch.py:  KHB_RM_FOLD / KHB_RM_T / KHB_RM_P replace existing carry chains or mads by
#                 full-rate ops (results wrong by design; perf_variants skips the parity check for _rm*).
#   pair_patch.py: the paired reduction (exact; slower at 4 waves because it spills).
#   defer_patch.py: the gate tested one walk step after its loads, pending x pair in registers.
#   nonop_patch.py: the carry-hazard s_nop pads removed (timing only).
#   block_patch.py: KHB_BLOCK threads per workgroup.
#   scr_patch.py: KHB_SCR_MASK=m keeps the prefix scratch in (i & m) entries per group (no HBM stream).
#   addrwalk_patch.py: the -m address kernels without the hashing (count-only: the x/y walk's VALU).
#   plainscr_patch.py: the prefix-scratch stream with plain loads and stores (the product's are non-temporal).
#   fold2_patch.py: the stage-1 gate fold tested with two of the three probes (candidates unchanged).
#   (round 5's half_patch.py is now the build define KHB_HALF_STREAM in scan_kernels.hpp: build_variant.sh half -DKHB_HALF_STREAM=1.)
#   scrplain_patch.py: scr_patch with plain accesses (the stream cache-resident; scr2plain / scr1plain, round 5).
#   early_patch.py: the first x's stage-1 fold load issued before the second x is computed (round 5).
# Usage: tools/experiments/calib_build.sh pad|rm|scr|pair|defer|nonop|block|addrwalk|plainscr|fold2|scrplain|early <name> [-DKEY=VAL ...]
set -e
KIND=$1; NAME=$2; shift 2
S1=keyhuntm1cpu_amd/csrc/device/fe_asm.hpp
S2=keyhuntm1cpu_amd/csrc/scan_kernels.hpp
cp $S1 /tmp/calib_fe_asm.hpp; cp $S2 /tmp/calib_scan_kernels.hpp
trap 'cp /tmp/calib_fe_asm.hpp $S1; cp /tmp/calib_scan_kernels.hpp $S2' EXIT
python3 tools/experiments/${KIND}_patch.py
tools/build_variant.sh $NAME "$@"
