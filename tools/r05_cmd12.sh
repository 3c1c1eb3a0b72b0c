#!/bin/bash
# VLC int8-staging A/B: stream tests on the tree's library, then per-kernel
# times of the coder for the base and variant builds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t12.log 2>&1 || { tail -30 gpurun_out/t12.log; exit 1; }
tail -3 gpurun_out/t12.log
CONTENTS="survey synth" bash tools/vlc_prof.sh abtest/lib_vlcw.so abtest/lib_vlc2.so abtest/lib_vlc3.so
