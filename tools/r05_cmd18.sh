#!/bin/bash
# k_motion A/B: the map build without store guards, rows in pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
P64GPU_LIB=$R/abtest/lib_mapb.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "full or motion or me_ or bench_scale" > gpurun_out/t18.log 2>&1 || { tail -30 gpurun_out/t18.log; exit 1; }
tail -1 gpurun_out/t18.log
CONTENTS="survey synth noise" REPS=15 bash tools/me_prof.sh abtest/lib_base.so abtest/lib_mapb.so abtest/lib_base.so abtest/lib_mapb.so || exit 1
