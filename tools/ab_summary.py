"""Summary of tools/ab_run.sh bench lines: python3 tools/ab_summary.py tag ..."""
import json, sys
for t in sys.argv[1:]:
    try:
        d = json.loads(open(f"gpurun_out/ab/{t}.log").read().strip().splitlines()[-1])
    except Exception as e:  # noqa
        print(t, "missing", e)
        continue
    st = d["roofline"]["stage_ms"]
    print(f"{t:10s} {d['value']:8.2f} Mrays/s  frame {d['ms_per_step']:7.2f} ms  secondary {st['secondary']:7.2f}  march {st['march']:6.2f}")
