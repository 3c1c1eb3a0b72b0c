#!/bin/bash
# Round-3 bench lines besides the default (GPU box): TSS, stress contents and
# 4CIF, each a bench.py JSON line under gpurun_out/r03_bench_<name>.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 400 python3 bench.py --no-extra "$@" > gpurun_out/r03_bench_$name.json 2> gpurun_out/r03_bench_$name.err || { tail -5 gpurun_out/r03_bench_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03_bench_$name.json')); print('$name', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
}
for spec in ${LINES:-tss:--mode=tss pan15:--content=pan15 noise:--content=noise flat:--content=flat 4cif:--config=4cif}; do
  name=${spec%%:*}; args=${spec#*:}
  run $name ${args//,/ }
done
