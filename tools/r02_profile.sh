#!/bin/bash
# Round-2 evidence run (GPU box): the default bench line, then the rocprofv3
# kernel-trace summary of the same command, copied into gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_r02
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r02 -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || exit 1
find $R/gpurun_out/prof_r02 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r02_kernel_stats.csv \;
