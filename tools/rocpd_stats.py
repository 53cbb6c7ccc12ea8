#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 rocpd SQLite database (``-o run`` default output):
python tools/rocpd_stats.py gpurun_out/prof3/run_results.db [--csv out.csv]"""
import argparse
import csv
import sqlite3
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
    name_col = "display_name" if "display_name" in cols else ("kernel_name" if "kernel_name" in cols else "name")
    rows = c.execute(f"""select s.{name_col}, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start)
                         from {disp} d join {sym} s on d.kernel_id = s.id group by s.{name_col}
                         order by sum(d.end - d.start) desc""").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = [dict(kernel=r[0], calls=r[1], total_us=r[2] / 1e3, avg_us=r[2] / r[1] / 1e3, min_us=r[3] / 1e3,
                max_us=r[4] / 1e3, pct=100.0 * r[2] / total) for r in rows]
    for o in out[:a.top]:
        print(f"{o['kernel'][:72]:72s} calls={o['calls']:6d} avg={o['avg_us']:9.1f}us pct={o['pct']:5.1f}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
