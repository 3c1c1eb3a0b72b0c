#!/bin/bash
# Throughput sweeps of the default inter line (GPU box): sequences per GPU,
# quantiser and search limit, one bench.py JSON line each under
# gpurun_out/sweep_<name>.json (no CPU leg, no nested configs, no VLC).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu --no-vlc --steps 100 "$@" > gpurun_out/sweep_$name.json 2> gpurun_out/sweep_$name.err || { tail -5 gpurun_out/sweep_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sweep_$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
run base
for s in 16 32 64 128 512 1024; do run S$s --streams $s; done
for q in 1 4 16 31; do run q$q --quant $q; done
run base2
for sl in 15 7; do run sl$sl --search-limit $sl; done
