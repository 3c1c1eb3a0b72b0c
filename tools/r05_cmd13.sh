#!/bin/bash
# stream tests, VLC A/B (kernel trace), the GPU suite, one default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t13.log 2>&1 || { tail -30 gpurun_out/t13.log; exit 1; }
tail -1 gpurun_out/t13.log
CONTENTS="survey synth" bash tools/vlc_prof.sh abtest/lib_vlcw.so abtest/lib_vlc2.so abtest/lib_vlc3.so || exit 1
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g13.log 2>&1 || { tail -30 gpurun_out/g13.log; exit 1; }
tail -1 gpurun_out/g13.log
cd $R && timeout -k 10 600 python -u bench.py > gpurun_out/bench13.json 2> gpurun_out/bench13.err || { tail -20 gpurun_out/bench13.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$R/gpurun_out/bench13.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d.get('with_vlc'))[:600])"
