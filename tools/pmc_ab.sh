#!/bin/bash
# PMC comparison of library builds on the kbench workload (GPU box).
# usage: tools/pmc_ab.sh lib1.so lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in "$@"; do
  tag=$(basename $lib .so)
  P64GPU_LIB=$R/$lib bash $R/tools/pmc.sh $tag "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
    "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
    "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
    -- python3 $R/tools/kbench.py --reps 3 || exit 1
done
