#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (one directory per pass, run_counter_collection.csv each) into one
JSON of per-launch counter values per kernel, with the HBM byte corrections of MI355X_MICROARCH.md
(§HBM): FETCH_SIZE (KiB) x 1024 x 2 on gfx950 (it reports half the bytes of wide reads), WRITE_SIZE (KiB)
x 1024. Derived: VALU-busy share of wave cycles, memory-wait share, SALU/VALU instruction ratio, L2 hit
rate.

    python tools/pmc_summary.py OUT.json PASS_DIR [PASS_DIR ...]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        with open(f"{d}/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                if k.startswith("__amd_rocclr"):
                    continue
                k = k.replace("void ", "").split("(")[0]
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                launches[k][row["Counter_Name"]].add(row["Dispatch_Id"])
    res = {}
    for k, cs in acc.items():
        r = {c: v / max(1, len(launches[k][c])) for c, v in cs.items()}  # per launch
        r["launches"] = max(len(s) for s in launches[k].values())
        if "FETCH_SIZE" in r:
            r["hbm_read_bytes_gfx950_corrected"] = r["FETCH_SIZE"] * 1024.0 * 2.0
        if "WRITE_SIZE" in r:
            r["hbm_write_bytes"] = r["WRITE_SIZE"] * 1024.0
        if r.get("SQ_WAVE_CYCLES"):
            if "SQ_ACTIVE_INST_VALU" in r:
                r["valu_busy_of_wave_cycles"] = r["SQ_ACTIVE_INST_VALU"] / r["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_ANY" in r:
                r["wait_any_of_wave_cycles"] = r["SQ_WAIT_ANY"] / r["SQ_WAVE_CYCLES"]
        if r.get("SQ_INSTS_VALU") and "SQ_INSTS_SALU" in r:
            r["salu_per_valu"] = r["SQ_INSTS_SALU"] / r["SQ_INSTS_VALU"]
        if "TCC_HIT_sum" in r and "TCC_MISS_sum" in r and r["TCC_HIT_sum"] + r["TCC_MISS_sum"] > 0:
            r["l2_hit_rate"] = r["TCC_HIT_sum"] / (r["TCC_HIT_sum"] + r["TCC_MISS_sum"])
        res[k] = dict(sorted(r.items()))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, r in res.items():
        print(k[:70], {x: round(r[x], 4) if isinstance(r[x], float) and r[x] < 100 else r[x]
                       for x in ("hbm_read_bytes_gfx950_corrected", "hbm_write_bytes", "valu_busy_of_wave_cycles",
                                 "wait_any_of_wave_cycles", "salu_per_valu", "l2_hit_rate") if x in r})


if __name__ == "__main__":
    main()
