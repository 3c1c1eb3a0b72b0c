"""Kernel times inside bench.py's timed region, from a rocprofv3 kernel trace
(development aid): the region is the K steps launched right before the first
k_clock dispatch after the spin-up (timed_region's clock probe).  Prints per
kernel the mean, min and max duration over the region and the region's span
per step, and the spin-up's per-replay means of the dominant kernel.
usage: python tools/timed_region.py <kernel_trace.csv> <K> [kernel-prefix ...]
       [--json profiles/r05_timed_region.json --key <bench.py workload key>]
(the default prefixes are the inter step's two kernels; pass k_intra_mbg or
k_recon_mbg for the nested configs)."""
import csv
import json
import statistics
import sys

args = sys.argv[1:]
jpath = None
if "--json" in args:  # also write {key: {kernel: mean us}} of every region found to this file
    i = args.index("--json")
    jpath = args[i + 1]
    del args[i:i + 2]
jkey = None
if "--key" in args:  # the workload key (bench.py content_key), required with --json
    i = args.index("--key")
    jkey = args[i + 1]
    del args[i:i + 2]
assert not jpath or jkey, "--json needs --key <bench.py workload key>"
path, K = args[0], int(args[1])
prefixes = args[2:] or ["k_motion", "k_inter_mbg"]
found = {}
rows = list(csv.DictReader(open(path)))
km = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0])
            for r in rows)
names = [n for _, _, n in km]
clocks = [i for i, n in enumerate(names) if n == "k_clock"]
assert clocks, "no k_clock dispatch: not a bench.py trace with the steady-state probe"
for ci, end in enumerate(clocks):
    start = clocks[ci - 1] + 1 if ci else 0
    seq = [(s, e, n) for s, e, n in km[start:end] if any(n.startswith(p) for p in prefixes)]
    per = len(prefixes)
    if len(seq) < per * K:
        continue
    timed = seq[-per * K:]
    print(f"timed region {ci} (before k_clock dispatch {end}): {K} steps")
    for p in prefixes:
        d = [(e - s) / 1e3 for s, e, n in timed if n.startswith(p)]
        if d:
            print(f"  {p:14s} mean {statistics.mean(d):8.2f} us  min {min(d):8.2f}  max {max(d):8.2f}  n {len(d)}")
            # (the first region with the kernel: the headline's; bench.py's
            # secondary content line runs the same kernels afterwards)
            found.setdefault(next(n for _, _, n in timed if n.startswith(p)), round(statistics.mean(d), 2))
    print(f"  span per step {(timed[-1][1] - timed[0][0]) / 1e3 / K:8.2f} us "
          f"(first start to last end; includes the gaps between dispatches)")
    sumk = sum(statistics.mean([(e - s) / 1e3 for s, e, n in timed if n.startswith(p)]) for p in prefixes)
    print(f"  kernel sum per step {sumk:8.2f} us")
if jpath:
    old = {}
    try:
        old = json.load(open(jpath))
    except (OSError, ValueError):
        pass
    old.setdefault(jkey, {}).update(found)
    json.dump(old, open(jpath, "w"), indent=1, sort_keys=True)
