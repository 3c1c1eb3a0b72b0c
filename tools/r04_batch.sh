#!/bin/bash
# Round-4 batch (GPU box): the GPU suite + an A/B of two library builds
# (tools/r04_abl.sh), the bench lines of the stress contents, TSS and 4CIF
# (the driver's step counts, CPU baselines included), then the PMC passes
# (tools/pmc_bench.sh).  Stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/batch
mkdir -p $O
if [ -n "$LIBS" ]; then
  TESTS=1 bash tools/r04_abl.sh || exit 1
fi
if [ -n "$LIBS2" ]; then
  LIBS="$LIBS2" CONFIGS="$CONFIGS2" bash tools/r04_abl.sh || exit 1
fi
for c in "--content pan15" "--content noise" "--content flat" "--mode tss" "--config 4cif"; do
  t=$(echo $c | tr -d ' -' )
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 $c > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $c failed"; tail -5 $O/bench_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$t.json').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
done
[ -n "$NOPMC" ] && exit 0
bash tools/pmc_bench.sh > $O/pmc.log 2>&1 || { tail -10 $O/pmc.log; exit 1; }
tail -6 $O/pmc.log
