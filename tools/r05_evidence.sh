#!/bin/bash
# Round-5 evidence run (GPU box): the GPU test suite, smoke(), the driver's
# exact bench command (`bench.py --gpus 1 --steps 20 --warmup 5`), the
# rocprofv3 kernel trace + stats of the same command (--no-cpu: the CPU legs
# spawn the reference, which must not run under the profiler) reduced to the
# timed region (tools/timed_region.py).  Everything lands under
# gpurun_out/$TAG/; each GPU step has its own time limit and the script
# stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05}
KEY=${KEY:-352x288_full31_q8_S256_survey}
O=$R/gpurun_out/$TAG
rm -rf $O && mkdir -p $O
cd $R
echo "head $(cat $R/.head_sha 2>/dev/null || echo unknown)" > $O/summary.txt
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log >> $O/summary.txt
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
  cat $O/smoke.log >> $O/summary.txt
fi
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json >> $O/summary.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
cd $R
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
for k in "" k_intra_mbg k_recon_mbg; do
  python3 tools/timed_region.py $O/kernel_trace.csv 20 --json $O/timed_region.json --key $KEY $k >> $O/timed_region.txt
done
cat $O/timed_region.txt >> $O/summary.txt
if [ -n "$EXTRA" ]; then
  for c in $EXTRA; do
    timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu $(echo $c | tr ',' ' ') > $O/extra_$(echo $c | tr ',= -' '____').json 2>> $O/extra.err || exit 1
  done
fi
cat $O/summary.txt | cut -c1-400
