#!/bin/bash
# Round-4 diagnosis (GPU box): why the driver's 20-step line is slower than the
# 200-step one.  The driver's exact command twice, the same without the CPU
# legs, and rocprofv3 kernel traces (per dispatch: duration and the gaps
# between dispatches) of the 20- and 200-step commands.  Each GPU step has its
# own time limit; the script stops at the first failing one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04d
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_a.json 2> $O/b20_a.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/b20_nocpu.json 2> $O/b20_nocpu.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-extra --no-vlc > $O/b200.json 2> $O/b200.err || exit 1
cd /tmp && export TMPDIR=/tmp
for k in 20 200; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$k -o run --output-format csv -- \
    python3 $R/bench.py --steps $k --warmup 5 --no-cpu > $O/prof$k.json 2> $O/prof$k.err || exit 1
  find $O/prof$k -name "*kernel_trace.csv" -exec cp {} $O/prof${k}_trace.csv \;
  find $O/prof$k -name "*kernel_stats.csv" -exec cp {} $O/prof${k}_stats.csv \;
done
cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_b.json 2> $O/b20_b.err || exit 1
ls $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
