#!/bin/bash
# PMC passes of tools/kbench.py against one library build (development aid):
#   tools/pmc_lib.sh TAG LIB "COUNTERS1" "COUNTERS2" ...
# one rocprofv3 run per counter group; summary in gpurun_out/pmc_TAG/summary.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; LIB=$2; shift 2
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  P64GPU_LIB=$R/$LIB timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/g$i -o run --output-format csv -- python3 $R/tools/kbench.py --reps 3 > $OUT/g$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/g$i.log; exit 1; }
  i=$((i+1))
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.txt
grep -E "k_intra_mbg|k_recon_mbg|k_inter_mbg|k_motion|k_encode" $OUT/summary.txt
