"""Average each PMC counter per kernel over the dispatches in a rocprofv3 csv tree."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(list)
meta = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size"], r["Grid_Size"])
for (k, c), v in sorted(agg.items()):
    if "at::native" in k or "rocclr" in k:
        continue
    print(f"{k:24s} {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}   vgpr/sgpr/lds/wg/grid={meta[k]}")
