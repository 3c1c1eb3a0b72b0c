#!/bin/bash
# Round-4 clock experiment (GPU box): the inter line at 20 and 200 steps with
# and without the clock spin-up before the timed region, the rocprofv3 kernel
# trace of the 20-step line with it, and the driver's exact command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c
rm -rf $O && mkdir -p $O
cd $R
B="python3 bench.py --no-cpu --no-vlc --no-extra --warmup 5"
for k in 20 200; do for sp in 0 150 500; do
  timeout -k 10 300 $B --steps $k --spinup-ms $sp > $O/s${k}_${sp}.json 2> $O/s${k}_${sp}.err || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof20 -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/prof20.json 2> $O/prof20.err || exit 1
find $O/prof20 -name "*kernel_trace.csv" -exec cp {} $O/prof20_trace.csv \;
find $O/prof20 -name "*kernel_stats.csv" -exec cp {} $O/prof20_stats.csv \;
cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver2.json 2> $O/driver2.err || exit 1
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$(basename $f)', round(d['value']/1e8,3), d['roofline']['kernel_avg_us'], d.get('steady_state'), [(k, v['roofline']['kernel_avg_us'], v.get('steady_state')) for k, v in d.get('configs', {}).items()])"; done
cd $R
timeout -k 10 600 env P64GPU_LIB=abtest/lib_sadcount.so python3 tools/sad_count_run.py --steps 20 --warmup 5 > $O/sadcount20.json 2> $O/sadcount20.err || exit 1
cat $O/sadcount20.json | head -c 600; echo
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
