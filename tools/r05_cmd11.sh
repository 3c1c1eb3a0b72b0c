R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t11.log 2>&1 || { tail -30 gpurun_out/t11.log; exit 1; }
tail -1 gpurun_out/t11.log
CONTENTS="survey synth" bash tools/inter_prof.sh abtest/lib_d61.so abtest/lib_d16.so abtest/lib_d32.so abtest/lib_d48.so abtest/lib_d61.so | grep inter
