mkdir -p gpurun_out/vlc && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vlc or encode or stream" > gpurun_out/vlc/tests.log 2>&1; tail -3 gpurun_out/vlc/tests.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/vlc/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 20 --no-extra > $GRAFT_REPO_ROOT/gpurun_out/vlc/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/vlc/bench.err
cd $GRAFT_REPO_ROOT; python3 -c "
import json; d=json.loads(open('gpurun_out/vlc/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['with_vlc'])"; grep vlc gpurun_out/vlc/prof/*kernel_stats.csv | cut -c1-200
