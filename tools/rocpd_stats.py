#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 rocpd database (rocprofv3 without --output-format csv):
    python3 tools/rocpd_stats.py DB [--top N]"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=10)
a = ap.parse_args()
c = sqlite3.connect(a.db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels group by {name} "
                 f"order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
for n, k, s, m in rows[:a.top]:
    print(f"{n[:70]:70s} {k:7d} {s / 1e6:9.2f} ms {m / 1e3:9.1f} us {100 * s / tot:5.1f} %")
print(f"total {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} dispatches")
