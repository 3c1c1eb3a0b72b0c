#!/bin/bash
# VLC A/B: header codes kept in registers
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
P64GPU_LIB=$R/abtest/lib_vlch.so timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t24.log 2>&1 || { tail -30 gpurun_out/t24.log; exit 1; }
tail -1 gpurun_out/t24.log
CONTENTS="survey synth" bash tools/vlc_prof.sh abtest/lib_vlc4.so abtest/lib_vlch.so abtest/lib_vlc4.so abtest/lib_vlch.so || exit 1
