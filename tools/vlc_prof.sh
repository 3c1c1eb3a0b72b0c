#!/bin/bash
# rocprofv3 kernel-trace averages of the GPU entropy coder (tools/vlcbench.py)
# per content for several library builds (development aid):
#   CONTENTS="survey synth" tools/vlc_prof.sh abtest/lib_a.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  for c in ${CONTENTS:-survey synth}; do
    OUT=$R/gpurun_out/vlcprof_${tag}_${c}
    rm -rf $OUT
    P64GPU_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/tools/vlcbench.py $c > $OUT.log 2>&1 || { echo "prof $tag $c failed"; tail -3 $OUT.log; exit 1; }
    grep -h "inter\|intra" $OUT.log | sed "s/^/$tag $c /"
    find $OUT -name "*kernel_stats.csv" | xargs cat | python3 -c "
import csv,sys
for r in csv.DictReader(sys.stdin):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0]
    if 'vlc' in n or 'rocclr_fill' in n: print(f\"$tag $c {n:22s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:8.1f} us\")"
  done
done
