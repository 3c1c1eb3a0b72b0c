#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t22.log 2>&1 || { tail -30 gpurun_out/t22.log; exit 1; }
tail -1 gpurun_out/t22.log
