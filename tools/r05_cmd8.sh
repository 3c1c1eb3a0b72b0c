# kernel trace of the with_vlc measurement (bench --no-extra), survey and synth
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for c in survey synth; do
  OUT=$R/gpurun_out/p8_$c
  rm -rf $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-extra --content $c > $OUT.json 2> $OUT.err || { tail -5 $OUT.err; exit 1; }
  find $OUT -name "*kernel_stats.csv" | xargs cat | python3 -c "
import csv,sys
for r in csv.DictReader(sys.stdin):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0]
    print(f\"$c {n[:60]:60s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:8.1f} us\")"
done
