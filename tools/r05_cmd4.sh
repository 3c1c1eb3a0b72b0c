timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_halves.log 2>&1; tail -3 gpurun_out/t_halves.log
CONTENTS="survey synth noise pan15 flat" REPS=15 bash tools/me_prof.sh abtest/lib_base.so abtest/lib_halves.so || exit 1
mkdir -p gpurun_out/cap
for m in joined lib_side external unjoined; do
  timeout -k 10 60 python3 tools/capture_probe.py $m > gpurun_out/cap/$m.log 2>&1; rc=$?
  echo "probe $m rc=$rc: $(tail -2 gpurun_out/cap/$m.log | tr '\n' ' ' | cut -c1-300)"
  [ $rc -ne 0 ] && exit 0
done
