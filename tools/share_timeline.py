"""Timeline of the last frame in a rocprofv3 kernel trace (csv): every kernel of the frame with its start
offset, duration and the idle gap before it, so a share's fixed costs (tails, gaps, small kernels) show.
    python3 tools/share_timeline.py DIR/run_kernel_trace.csv [first-kernel-substring, default march_kernel]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "march_kernel"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
frame = rows[starts[-1]:]
t0 = int(frame[0]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in frame:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
    print(f"{(s - t0) / 1e3:9.1f} us  +{(s - prev_end) / 1e3:7.1f} gap  {(e - s) / 1e3:9.1f} us  {name}")
    busy += e - s
    prev_end = max(prev_end, e)
print(f"frame {(prev_end - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, idle {(prev_end - t0 - busy) / 1e3:.1f} us")
