#!/bin/bash
# Profile the bench workload with rocprofv3 on the GPU box (via gpurun).
# Pass 1: kernel trace + stats; then PMC passes, one counter group per run
# (never combined with tracing).  Writes gpurun_out/prof/ and a summary
# gpurun_out/prof/summary.json (bench.py reads the traffic from
# profiles/pmc_traffic.json once it is copied there).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu --no-verify $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ARGS > $OUT/trace.log 2>&1
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SPI_RA_SGPR_SIMD_FULL_CSN"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc_$tag -o run --output-format csv -- python3 $ARGS > $OUT/pmc_$tag.log 2>&1
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
python3 $R/tools/prof_json.py $OUT "$*" > $OUT/summary.json
cat $OUT/summary.json
