#!/bin/bash
# Round profile of the default bench workload (C4): rocprofv3 kernel-trace summary + PMC passes
# (one counter group per run, kernel-trace only), then a per-kernel JSON summary.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-r01}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --flops 0 > $OUT/stats.log 2>&1; rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --flops 0 > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc $i ($set) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<PY
import csv, collections, json, glob
out = {}
for f in sorted(glob.glob("$OUT/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "vr::dev" not in k: continue
        k = k.split("(")[0].replace("void ", "")
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, c), v in agg.items(): out.setdefault(k, {})[c] = v
for k, d in out.items():
    if "FETCH_SIZE" in d: d["hbm_read_bytes_gfx950_corrected"] = d["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in d: d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
json.dump(out, open("$OUT/pmc_summary.json", "w"), indent=1, sort_keys=True)
print(json.dumps({k: {c: d.get(c) for c in ("hbm_read_bytes_gfx950_corrected", "hbm_write_bytes")} for k, d in out.items()}, indent=1))
PY
