"""Fold a tools/pmc_bench.sh run into profiles/pmc_traffic.json (development aid).

    python tools/pmc_merge.py gpurun_out/pmcb /tmp/k.s [profiles/pmc_traffic.json]

/tmp/k.s is the ISA listing of k_search.hip (make asm, or hipcc -S
--cuda-device-only) used for each kernel's mean VALU issue cost.

Per kernel and workload it records, averaged over the profiled dispatches:
  hbm_bytes_per_launch  (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 -- gfx950's
                        FETCH_SIZE counts half of wide streaming reads
                        (MI355X_MICROARCH.md, HBM section)
  valu_insts_per_launch SQ_INSTS_VALU (wave instructions, all SIMDs)
  kernel_cycles         GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs:
                        calibrated on tools/ubench_valu, whose v_add3 kernel
                        gives 4.23e6 cycles per XCD for 4.10e6 expected)
  valu_issue_per_simd_cycle  SQ_INSTS_VALU / (1024 SIMDs x kernel_cycles)
  valu_busy             the same x the kernel's mean VALU issue cost (cycles
                        per wave instruction on one SIMD, priced by
                        tools/isa_mix.py from the static instruction mix with
                        the costs tools/ubench_valu measured): the fraction of
                        SIMD cycles the VALU spent issuing.  The calibration
                        kernels (100% VALU by construction) read 0.97 (v_add3,
                        4 cycles) and 0.87 (v_add_u32, 2 cycles).
SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU on this part (it counts
instructions, not cycles), so it is not used.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
import isa_mix  # noqa: E402

SIMDS = 1024
XCDS = 8
WORKLOADS = {  # pmc_bench.sh tag -> {kernel: bench.py pmc key}
    "synth": {"k_motion<2>": "352x288_full31_q8_S256_me", "k_inter_mbg<false, false, true, false>": "352x288_full31_q8_S256_inter",
              "k_intra_mbg<false, false, true, false>": "352x288_intra_q8_S256", "k_recon_pk": "352x288_decode_q8_S256",
              "k_recon_mbg": "352x288_decode_q8_S256_dense"},
    "survey": {"k_motion<2>": "352x288_full31_q8_S256_survey_me",
               "k_inter_mbg<false, false, true, false>": "352x288_full31_q8_S256_survey_inter",
               "k_intra_mbg<false, false, true, false>": "352x288_intra_q8_S256_survey",
               "k_recon_pk": "352x288_decode_q8_S256_survey",
               "k_recon_mbg": "352x288_decode_q8_S256_survey_dense"},
    "noise": {"k_motion<2>": "352x288_full31_q8_S256_noise_me",
              "k_inter_mbg<false, false, true, false>": "352x288_full31_q8_S256_noise_inter"},
    "pan15": {"k_motion<2>": "352x288_full31_q8_S256_pan15_me",
              "k_inter_mbg<false, false, true, false>": "352x288_full31_q8_S256_pan15_inter"},
    "flat": {"k_motion<2>": "352x288_full31_q8_S256_flat_me",
             "k_inter_mbg<false, false, true, false>": "352x288_full31_q8_S256_flat_inter"},
}
ASM_LABEL = {"k_encode<2>": "k_encodeILi2E", "k_intra_mbg<false, false, true, false>": "k_intra_mbgILb0ELb0ELb1ELb0E",
             "k_recon_blk": "k_recon_blk", "k_recon_mbg": "k_recon_mbg", "k_recon_pk": "k_recon_pk",
             "k_motion<2>": "k_motionILi2E",
             "k_inter_mbg<false, false, true, false>": "k_inter_mbgILb0ELb0ELb1ELb0E"}


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def means(tree):
    agg = collections.defaultdict(list)
    for f in glob.glob(tree + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def mean_cost(asm, label):
    lines = open(asm).read().splitlines()
    ops = collections.Counter()
    on = False
    for ln in lines:
        head = ln.split(";")[0].strip()
        if not on and head.endswith(":") and label in head and not ln.startswith((".", "\t")):
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end"):
                break
            s = ln.strip()
            if s and not s.startswith((";", ".", "//")) and not s.endswith(":") and s.startswith("v_"):
                ops[s.split()[0]] += 1
    n = sum(ops.values())
    return sum(isa_mix.cost(o) * c for o, c in ops.items()) / n


def main():
    root, asm = sys.argv[1], sys.argv[2]
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "pmc_traffic.json")
    db = json.load(open(dst)) if os.path.exists(dst) else {}
    cal = means(os.path.join(root, "calib"))
    for k, cyc_cost in (("k<1, false>", 4), ("k<29, false>", 2)):
        cyc = cal[(k, "GRBM_GUI_ACTIVE")] / XCDS
        print(f"calibration {k}: busy {cal[(k, 'SQ_INSTS_VALU')] * cyc_cost / (SIMDS * cyc):.3f}")
    for tag, kernels in WORKLOADS.items():
        m = means(os.path.join(root, tag))
        for kern, key in kernels.items():
            if (kern, "FETCH_SIZE") not in m:
                print(f"{tag}: no counters for {kern}")
                continue
            cyc = m[(kern, "GRBM_GUI_ACTIVE")] / XCDS
            insts = m[(kern, "SQ_INSTS_VALU")]
            cost = mean_cost(asm, ASM_LABEL[kern])
            issue = insts / (SIMDS * cyc)
            rec = {
                "kernel": kern,
                "hbm_bytes_per_launch": int((2 * m[(kern, "FETCH_SIZE")] + m[(kern, "WRITE_SIZE")]) * 1024),
                "fetch_bytes_raw": int(m[(kern, "FETCH_SIZE")] * 1024),
                "write_bytes": int(m[(kern, "WRITE_SIZE")] * 1024),
                "valu_insts_per_launch": int(insts),
                "waves_per_launch": int(m[(kern, "SQ_WAVES")]),
                "kernel_cycles": int(cyc),
                "valu_issue_per_simd_cycle": round(issue, 4),
                "valu_mean_cycles_per_inst": round(cost, 3),
                "valu_busy": round(issue * cost, 3),
                "source": "tools/pmc_bench.sh + tools/pmc_merge.py (rocprofv3 --pmc, one pass per "
                          "counter group, bench.py --eager; see the script headers)",
            }
            db[key] = rec
            print(key, json.dumps(rec))
    with open(dst, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
