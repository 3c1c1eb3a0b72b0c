#!/bin/bash
# Round-3 evidence run (GPU box): the full GPU test suite, smoke(), the default
# bench line and the rocprofv3 kernel-trace summary of the same command.
# Everything lands under gpurun_out/; each GPU step has its own time limit and
# the script stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r03}
mkdir -p $R/gpurun_out
cd $R
git_head=$(cat $R/.head_sha 2>/dev/null || echo unknown)
echo "head $git_head" > gpurun_out/${TAG}_summary.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log >> gpurun_out/${TAG}_summary.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
cat gpurun_out/${TAG}_smoke.log >> gpurun_out/${TAG}_summary.txt
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json >> gpurun_out/${TAG}_summary.txt
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu > $R/gpurun_out/${TAG}_bench_prof.json 2> $R/gpurun_out/${TAG}_bench_prof.err || exit 1
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/${TAG}_kernel_stats.csv \;
