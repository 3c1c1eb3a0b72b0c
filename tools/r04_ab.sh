#!/bin/bash
# A/B of environment-selected kernel variants in one box session (GPU box):
#   CONFIG=intra VAR=P64GPU_AB_INTRA VALUES="0 4 3" REPS=2 bash tools/r04_ab.sh
# runs bench.py --config $CONFIG --no-cpu --steps $STEPS for every value, REPS
# times alternating, and prints ms per step and the roofline fraction.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$TESTS" \
      > $O/tests_$v.log 2>&1 || { tail -20 $O/tests_$v.log; exit 1; }
    echo "tests $VAR=$v: $(tail -1 $O/tests_$v.log)"
  done
fi
for r in $(seq ${REPS:-2}); do for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python3 bench.py --config ${CONFIG:-intra} --no-cpu --steps ${STEPS:-100} $ARGS \
    > $O/${CONFIG}_${v}_$r.json 2> $O/${CONFIG}_${v}_$r.err || { echo "bench $v failed"; tail -5 $O/${CONFIG}_${v}_$r.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/${CONFIG}_${v}_$r.json').read().strip().splitlines()[-1])
rf=d['roofline']; print('$VAR=$v rep $r', d['ms_per_step'], rf.get('kernel_avg_us'), rf.get('frac'), d.get('steady_state',{}).get('kernels_us_live'), d.get('verified_vs_oracle', d.get('verified_vs_encoder')))"
done; done
