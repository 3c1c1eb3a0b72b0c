#!/bin/bash
# Round-3 closing measurements (GPU box): the default bench line again (it
# quotes the kernel split from profiles/r03_kernel_stats.csv, refreshed from
# the evidence run), the TSS / stress / 4CIF lines (tools/r03_lines.sh) and
# the PMC passes (tools/pmc_bench.sh).  Stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail -5 gpurun_out/r03_bench.err; exit 1; }
bash tools/r03_lines.sh || exit 1
[ -n "$NOPMC" ] && exit 0
bash tools/pmc_bench.sh > gpurun_out/pmc_bench.log 2>&1 || { tail -5 gpurun_out/pmc_bench.log; exit 1; }
