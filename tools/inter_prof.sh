#!/bin/bash
# rocprofv3 kernel-trace averages of tools/inter_time.py for several library
# builds (development aid): CONTENTS="survey synth" tools/inter_prof.sh abtest/lib_a.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  for c in ${CONTENTS:-survey}; do
    OUT=$R/gpurun_out/interprof_${tag}_${c}
    rm -rf $OUT
    P64GPU_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/tools/inter_time.py --content $c > $OUT.log 2>&1 || { echo "prof $tag $c failed"; tail -3 $OUT.log; exit 1; }
    find $OUT -name "*kernel_stats.csv" | xargs cat | python3 -c "
import csv,sys
for r in csv.DictReader(sys.stdin):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0]
    if 'k_inter' in n or 'k_motion' in n: print(f\"$tag $c {n:40s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:8.1f} us\")"
  done
done
