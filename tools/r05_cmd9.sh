R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t9.log 2>&1 || { tail -30 gpurun_out/t9.log; exit 1; }
tail -1 gpurun_out/t9.log
bash tools/r05_cmd8.sh | grep -E "k_inter|k_vlc|k_intra"
for c in survey synth; do python3 -c "
import json; d=json.loads(open('gpurun_out/p8_$c.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['with_vlc'].get('macroblocks_per_s'), d['with_vlc'].get('ms_per_step'), d['with_vlc'].get('vlc_ms_last_step'))"; done
