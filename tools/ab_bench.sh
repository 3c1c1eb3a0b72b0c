#!/bin/bash
# bench.py's own config (default decode) under several library builds
# (development aid): CONFIG=decode tools/ab_bench.sh abtest/lib_a.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for lib in "$@"; do
  tag=$(basename $lib .so)
  P64GPU_LIB=$R/$lib timeout -k 10 300 python3 bench.py --config ${CONFIG:-decode} --no-cpu --steps ${STEPS:-100} ${ARGS} \
    > gpurun_out/abb_$tag.json 2> gpurun_out/abb_$tag.err || { echo "bench $tag failed"; tail -3 gpurun_out/abb_$tag.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/abb_$tag.json').read().strip().splitlines()[-1])
print('$tag', d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('kernel_avg_us'))"
done
