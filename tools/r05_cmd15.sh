#!/bin/bash
# one default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench15.json 2> gpurun_out/bench15.err || { tail -20 gpurun_out/bench15.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$R/gpurun_out/bench15.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d.get('with_vlc'))[:700])"
