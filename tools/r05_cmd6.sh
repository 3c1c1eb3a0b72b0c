R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/cap
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_h16m.log 2>&1; tail -2 gpurun_out/t_h16m.log
CONTENTS="survey synth pan15 noise flat" REPS=15 bash tools/me_prof.sh abtest/lib_base.so abtest/lib_h16.so abtest/lib_h16m.so || exit 1
CONTENTS="survey synth" bash tools/vlc_prof.sh abtest/lib_base.so abtest/lib_h16m.so
for m in null_launch unforked; do
  timeout -k 10 60 python3 tools/capture_probe.py $m > gpurun_out/cap/$m.log 2>&1; rc=$?
  echo "probe $m rc=$rc: $(tail -3 gpurun_out/cap/$m.log | tr '\n' ' ' | cut -c1-400)"
  [ $rc -ne 0 ] && exit 0
done
