# executed-SAD counts (survey, synth), PMC passes (calib, survey, synth), ME routing A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for c in survey synth; do
  P64GPU_LIB=$R/abtest/lib_sadcount.so timeout -k 10 300 python3 tools/sad_count_run.py --content $c > gpurun_out/sad_$c.json 2> gpurun_out/sad_$c.err || { tail -5 gpurun_out/sad_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sad_$c.json')); print('$c', d['byte_absdiff_per_mb'])"
done
STRESS="" bash tools/pmc_bench.sh || exit 1
cd $R
CONTENTS="survey synth pan15" REPS=15 bash tools/me_prof.sh abtest/lib_g16.so abtest/lib_g8.so
CONTENTS="survey synth" bash tools/inter_prof.sh abtest/lib_g16.so abtest/lib_noidct.so abtest/lib_nolvl.so abtest/lib_norec.so
