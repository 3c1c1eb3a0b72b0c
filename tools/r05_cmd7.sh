R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1 || { tail -30 gpurun_out/t7.log; exit 1; }
tail -1 gpurun_out/t7.log
for c in survey synth; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --content $c > gpurun_out/b7_$c.json 2> gpurun_out/b7_$c.err || { tail -5 gpurun_out/b7_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/b7_$c.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['roofline'].get('kernels_us_live'), d['with_vlc'], d['verified_vs_oracle']['ok'])"
done
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --feed root --no-extra > gpurun_out/b7_root.json 2> gpurun_out/b7_root.err || { tail -5 gpurun_out/b7_root.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/b7_root.json').read().strip().splitlines()[-1])
print('root', d['value'], d['ms_per_step'], d['config'].get('gather'), d['verified_vs_oracle']['ok'])"
