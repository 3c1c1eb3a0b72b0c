#!/bin/bash
# k_motion A/B: the scalar range of the current sub-block averages; ME parity tests on the variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
P64GPU_LIB=$R/abtest/lib_srange.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t27.log 2>&1 || { tail -30 gpurun_out/t27.log; exit 1; }
tail -1 gpurun_out/t27.log
CONTENTS="survey synth" REPS=15 bash tools/me_prof.sh abtest/lib_base.so abtest/lib_srange.so abtest/lib_base.so abtest/lib_srange.so || exit 1
