#!/bin/bash
# rocprofv3 kernel-trace averages of k_motion<2> per content for several
# library builds (development aid): tools/me_prof.sh abtest/lib_a.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  for c in ${CONTENTS:-synth pan15 noise flat}; do
    OUT=$R/gpurun_out/meprof_${tag}_${c}_sl${SL:-31}
    rm -rf $OUT
    P64GPU_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/tools/me_time.py --reps ${REPS:-20} --contents $c --search-limit ${SL:-31} > $OUT.log 2>&1 || { echo "prof $tag $c failed"; tail -3 $OUT.log; exit 1; }
    find $OUT -name "*kernel_stats.csv" | xargs cat | python3 -c "
import csv,sys
for r in csv.DictReader(sys.stdin):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0]
    if 'k_motion' in n or 'tile' in n: print(f\"$tag $c {n:16s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:8.1f} us  min {float(r['MinNs'])/1e3:8.1f}\")"
  done
done
