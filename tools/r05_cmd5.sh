# k_motion A/B (survivor routing thresholds) + PMC of k_motion on survey + capture probes
R=${GRAFT_REPO_ROOT:-$(pwd)}
CONTENTS="survey synth pan15" REPS=15 bash tools/me_prof.sh abtest/lib_base.so abtest/lib_h16.so abtest/lib_h32.so || exit 1
mkdir -p gpurun_out/pmc5
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc5/h32 -o run --output-format csv -- python3 $R/tools/me_time.py --reps 3 --contents survey,synth > $R/gpurun_out/pmc5/h32.log 2>&1 || { echo pmc failed; tail -5 $R/gpurun_out/pmc5/h32.log; exit 1; }
cd $R
find gpurun_out/pmc5/h32 -name "*counter_collection.csv" | head -1 | xargs python3 -c "
import csv,sys,collections
d=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Kernel_Name']
    if 'k_motion' not in n: continue
    d[r['Dispatch_Id']][r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in list(d.items())[:8]:
    print(k, {c: sum(x) for c,x in v.items()})
"
for m in null_launch unforked; do
  timeout -k 10 60 python3 tools/capture_probe.py $m > gpurun_out/cap/$m.log 2>&1; rc=$?
  echo "probe $m rc=$rc: $(tail -3 gpurun_out/cap/$m.log | tr '\n' ' ' | cut -c1-400)"
  [ $rc -ne 0 ] && exit 0
done
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vlc or stream or cli or decode" > gpurun_out/t_vlc.log 2>&1; tail -2 gpurun_out/t_vlc.log
CONTENTS="survey synth" bash tools/vlc_prof.sh abtest/lib_base.so abtest/lib_vlcs.so
