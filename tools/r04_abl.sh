#!/bin/bash
# A/B of library builds in one box session (GPU box):
#   LIBS="abtest/lib_old.so abtest/lib_new.so" CONFIGS="intra inter" REPS=2 bash tools/r04_abl.sh
# bench.py --no-cpu --no-vlc --no-extra --steps $STEPS per (config, library),
# alternating; TESTS=1 first runs the GPU suite on the tree's own library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abl
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  echo "tests: $(tail -1 $O/tests.log)"
fi
for c in ${CONFIGS:-intra}; do for r in $(seq ${REPS:-2}); do for lib in $LIBS; do
  t=$(basename $lib .so)
  P64GPU_LIB=$R/$lib timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-vlc --no-extra --steps ${STEPS:-100} $ARGS \
    > $O/${c}_${t}_$r.json 2> $O/${c}_${t}_$r.err || { echo "bench $c $t failed"; tail -5 $O/${c}_${t}_$r.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/${c}_${t}_$r.json').read().strip().splitlines()[-1])
rf=d['roofline']; print('$c $t rep $r', d['ms_per_step'], rf.get('kernel_avg_us'), rf.get('frac'), d.get('steady_state',{}).get('kernels_us_live'), d.get('verified_vs_oracle', d.get('verified_vs_encoder')))"
done; done; done
