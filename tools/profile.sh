#!/bin/bash
# Profile the bench workload with rocprofv3 (run on the GPU box via gpurun).
# Pass 1: kernel trace + stats; passes 2-5: PMC counters, one group per pass
# (never combined with tracing, per the pool's rules).  Output: gpurun_out/prof/
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu --no-verify $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ARGS > $OUT/trace.log 2>&1
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc_$tag -o run --output-format csv -- python3 $ARGS > $OUT/pmc_$tag.log 2>&1
done
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
echo profile done
