#!/bin/bash
# PMC for the entropy coder (tools/vlcbench.py survey): VALU instructions, waves, cycles
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcvlc
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/g0 -o run --output-format csv -- python3 $R/tools/vlcbench.py survey > $OUT/g0.log 2>&1 || { echo fail; tail -5 $OUT/g0.log; exit 1; }
f=$(find $OUT/g0 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
    if 'vlc' in n:
        agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, d in agg.items():
    m = {k: sum(v) / len(v) for k, v in d.items()}
    w = m.get('SQ_WAVES', 1)
    print(n, {k: round(v) for k, v in m.items()}, 'valu/wave', round(m['SQ_INSTS_VALU'] / w), 'lds/wave', round(m['SQ_INSTS_LDS'] / w),
          'valu/simd/cycle', round(m['SQ_INSTS_VALU'] / 1024 / (m['GRBM_GUI_ACTIVE'] / 8), 3))
PY
