#!/bin/bash
# One GPU lease, parametrised (replaces round 5's one-off tools/r05_cmd*.sh):
#   tools/lease.sh TAG step [step ...]
# steps (run in order; the first failure ends the lease, each GPU step under
# its own time limit; everything lands under gpurun_out/TAG/):
#   tests[=a,b,...]          pytest -m gpu (all, or -k "a or b or ...")
#   smoke                    __graft_entry__.smoke()
#   bench[=args,comma,sep]   bench.py --gpus 1 --steps 20 --warmup 5 [args] -> bench[_args].json
#   prof[=args]              rocprofv3 --kernel-trace --stats of the bench (--no-cpu) + timed region
#   pmc                      tools/pmc_bench.sh: its PMC passes over every content (into gpurun_out/pmcb)
#   probe[=args]             tools/vlc_fault_probe.py with the bounds-checked coder
#   sadcount=content         executed v_sad_u8 work of k_motion (abtest/lib_sadcount.so, tools/sad_count.py)
#   py=script.py[,args]      any tracked python tool, e.g. py=tools/stream_time.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "head $(cat $R/.head_sha 2>/dev/null || echo unknown)" >> $O/summary.txt
KEY=${KEY:-352x288_full31_q8_S256_survey}
for st in "$@"; do
  name=${st%%=*}
  arg=""
  [ "$st" != "$name" ] && arg=${st#*=}
  sfx=$(echo "$arg" | tr ',= -' '____' | tr -s '_')
  echo "== $st $(date +%T)" | tee -a $O/summary.txt
  case $name in
    tests)
      sel=()
      [ -n "$arg" ] && sel=(-k "$(echo "$arg" | sed 's/,/ or /g')")  # a,b: -k "a or b"
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${sel[@]}" \
        > $O/gpu_tests$sfx.log 2>&1 || { tail -40 $O/gpu_tests$sfx.log; exit 1; }
      tail -1 $O/gpu_tests$sfx.log | tee -a $O/summary.txt ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
      cat $O/smoke.log >> $O/summary.txt ;;
    bench)
      timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 $(echo $arg | tr ',' ' ') \
        > $O/bench$sfx.json 2> $O/bench$sfx.err || { tail -20 $O/bench$sfx.err; exit 1; }
      cut -c1-600 $O/bench$sfx.json | tee -a $O/summary.txt ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$sfx -o run \
        --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu $(echo $arg | tr ',' ' ') \
        > $O/bench_prof$sfx.json 2> $O/bench_prof$sfx.err) || { tail -20 $O/bench_prof$sfx.err; exit 1; }
      find $O/prof$sfx -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats$sfx.csv \;
      find $O/prof$sfx -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace$sfx.csv \;
      for k in "" k_intra_mbg k_recon_mbg k_recon_pk; do
        python3 tools/timed_region.py $O/kernel_trace$sfx.csv 20 --json $O/timed_region$sfx.json --key $KEY $k \
          >> $O/timed_region$sfx.txt
      done
      cat $O/timed_region$sfx.txt >> $O/summary.txt ;;
    pmc)
      timeout -k 10 900 bash tools/pmc_bench.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; } ;;
    probe)
      P64GPU_LIB=$R/abtest/lib_vlccheck.so timeout -k 10 300 python3 -u tools/vlc_fault_probe.py $(echo $arg | tr ',' ' ') \
        > $O/probe$sfx.log 2>&1 || { cat $O/probe$sfx.log; exit 1; }
      cat $O/probe$sfx.log | tee -a $O/summary.txt ;;
    sadcount)
      P64GPU_LIB=$R/abtest/lib_sadcount.so timeout -k 10 300 python3 -u tools/sad_count_run.py --content $arg \
        > $O/sad_$arg.json 2> $O/sad_$arg.err || { tail -20 $O/sad_$arg.err; exit 1; }
      cut -c1-300 $O/sad_$arg.json | tee -a $O/summary.txt ;;
    py)
      scr=${arg%%,*}
      rest=""
      [ "$scr" != "$arg" ] && rest=${arg#*,}
      timeout -k 10 600 python3 -u $scr $(echo $rest | tr ',' ' ') > $O/py_$(basename $scr .py).log 2>&1 \
        || { tail -30 $O/py_$(basename $scr .py).log; exit 1; }
      tail -40 $O/py_$(basename $scr .py).log | tee -a $O/summary.txt ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "lease $TAG done"
