#!/bin/bash
# stream tests, VLC A/B (wave vs workgroup look-back), one default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1 || { tail -30 gpurun_out/t16.log; exit 1; }
tail -1 gpurun_out/t16.log
CONTENTS="survey synth" bash tools/vlc_prof.sh abtest/lib_vlc3.so abtest/lib_vlc4.so || exit 1
cd $R && timeout -k 10 600 python -u bench.py > gpurun_out/bench16.json 2> gpurun_out/bench16.err || { tail -20 gpurun_out/bench16.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$R/gpurun_out/bench16.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d.get('with_vlc'))[:400], json.dumps(d.get('other_content')))"
