"""Per-kernel means of the counters tools/vlc_pmc.sh collected (development aid):
python3 tools/vlc_pmc.py <dir>  -> JSON {kernel: {counter: mean, derived...}}"""
import collections
import csv
import glob
import json
import sys


def main():
    agg = collections.defaultdict(list)
    for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            if "vlc" in k:
                agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = collections.defaultdict(dict)
    for (k, c), v in agg.items():
        out[k][c] = sum(v) / len(v)
    for k, d in out.items():
        if d.get("SQ_WAVES"):
            d["wave_cycles_per_wave"] = d.get("SQ_WAVE_CYCLES", 0) / d["SQ_WAVES"]
        if d.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VALU"):
                if c in d:
                    d[c + "_frac"] = round(d[c] / d["SQ_WAVE_CYCLES"], 3)
        if d.get("GRBM_GUI_ACTIVE"):
            d["kernel_cycles_per_xcd"] = d["GRBM_GUI_ACTIVE"] / 8
        if "FETCH_SIZE" in d:
            d["hbm_bytes"] = int((2 * d["FETCH_SIZE"] + d.get("WRITE_SIZE", 0)) * 1024)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
