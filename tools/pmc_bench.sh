#!/bin/bash
# PMC evidence for bench.py's roofline.traffic and valu_busy (GPU box):
# one rocprofv3 --pmc pass per counter group (never with tracing), over the
# default workload (k_motion<2>, k_inter_mbg, k_intra_mbg, k_recon_mbg on survey and synth content)
# and the stress contents, plus a calibration pass over tools/ubench_valu
# (kernels of known VALU issue rate).  tools/pmc_merge.py turns the output
# into profiles/pmc_traffic.json entries.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcb
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
run() {  # tag, program args...
  local tag=$1; shift
  local i=0
  for grp in "${GROUPS_[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/$tag/g$i -o run --output-format csv -- "$@" > $OUT/$tag/g$i.log 2>&1 \
      || { echo "pmc $tag pass $i failed"; tail -5 $OUT/$tag/g$i.log; exit 1; }
    i=$((i+1))
  done
  echo "pmc $tag done"
}
B="$R/bench.py --steps 10 --warmup 2 --no-cpu --no-verify --no-vlc --eager --spinup-ms 0"
for t in calib survey synth noise pan15 flat; do mkdir -p $OUT/$t; done
run calib $R/tools/ubench_valu new
run survey python3 $B --content survey
run synth python3 $B --content synth
for c in ${STRESS-noise pan15 flat}; do run $c python3 $B --content $c --no-extra; done
