#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing) over a command.
# usage: tools/pmc.sh TAG "GROUP1" "GROUP2" ... -- python3 script args
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
GROUPS_=()
while [ "$1" != "--" ]; do GROUPS_+=("$1"); shift; done
shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "${GROUPS_[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/g$i -o run --output-format csv -- "$@" > $OUT/g$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  i=$((i+1))
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
