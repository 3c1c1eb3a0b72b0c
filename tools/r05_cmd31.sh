#!/bin/bash
# the other contents and configs at head (--no-cpu), one line each
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h
rm -rf $O && mkdir -p $O
cd $R
for c in "--content noise" "--content pan15" "--content flat" "--content synth --mode tss" "--config 4cif"; do
  tag=$(echo $c | tr ' -' '__' | sed 's/^_*//')
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu $c > $O/bench_$tag.json 2>> $O/err.log || { echo "fail $c"; tail -5 $O/err.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], (d['roofline'].get('kernels_us_live') or {}))"
done
