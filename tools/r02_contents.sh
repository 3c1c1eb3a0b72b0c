#!/bin/bash
# Round-2 stress-content bench lines (GPU box): FULL SL=31 on pan15 / noise /
# flat, plus TSS on synth, each its own bench.py run (no CPU leg, no nested
# configs), JSON lines into gpurun_out/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for c in noise pan15 flat; do
  timeout -k 10 300 python3 bench.py --content $c --no-extra --no-cpu > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail -3 gpurun_out/bench_$c.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --mode tss --no-extra --no-cpu > gpurun_out/bench_tss.json 2> gpurun_out/bench_tss.err || { echo "bench tss failed"; exit 1; }
echo contents done
