#!/bin/bash
# PMC passes over the entropy coder (tools/vlc_time.py; development aid, GPU
# box): one rocprofv3 --pmc pass per counter group, never with tracing; the
# per-kernel means land in gpurun_out/$TAG/vlc_pmc.json (tools/vlc_pmc.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-vlcpmc}
OUT=$R/gpurun_out/$TAG/vlcpmc
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
         "FETCH_SIZE" "WRITE_SIZE")
i=0
for grp in "${GROUPS_[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/g$i -o run --output-format csv -- python3 $R/tools/vlc_time.py --reps 3 "$@" \
    > $OUT/g$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/g$i.log; exit 1; }
  i=$((i+1))
done
python3 $R/tools/vlc_pmc.py $OUT > $R/gpurun_out/$TAG/vlc_pmc.json
cat $R/gpurun_out/$TAG/vlc_pmc.json
