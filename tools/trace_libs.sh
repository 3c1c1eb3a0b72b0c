#!/bin/bash
# rocprofv3 kernel-trace averages of tools/kbench.py for several library
# builds (development aid): tools/trace_libs.sh abtest/lib_a.so abtest/lib_b.so ...
# (SCRIPT=tools/stream_time.py: the bench stream instead of kbench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  OUT=$R/gpurun_out/trace_$tag
  rm -rf $OUT
  P64GPU_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/${SCRIPT:-tools/kbench.py} --reps ${REPS:-10} > $OUT.log 2>&1 || { echo "trace $tag failed"; tail -3 $OUT.log; exit 1; }
  echo "== $tag"
  find $OUT -name "*kernel_stats.csv" | xargs cat | python3 -c "
import csv,sys
for r in csv.DictReader(sys.stdin):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0]
    if n.startswith(('k_','void k_')): print(f\"{n:28s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:8.1f} us  min {float(r['MinNs'])/1e3:8.1f}\")"
done
