#!/usr/bin/env python3
"""Per-kernel mean of each PMC counter from a rocprofv3 ``--pmc --output-format csv`` run.

Usage: python tools/pmc_summary.py <dir containing *counter_collection.csv> [--batch B]
With ``--batch`` the read/write request counters are also reported per request row
(TCC_EA0_RDREQ x 64 B, see MI355X_MICROARCH.md: gfx950 tallies 128-B requests at 64 B, so
the byte figure is a lower bound of up to 2x)."""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=0)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for fn in files:
        with open(fn, newline="") as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"].split("(")[0][:60]
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add((fn, row.get("Dispatch_Id", row.get("Correlation_Id"))))
    for k in sorted(acc, key=lambda s: -len(disp[s])):
        n = len(disp[k])
        print(f"{k}  dispatches={n}")
        for c, v in sorted(acc[k].items()):
            line = f"    {c:28s} per dispatch {v / n:14.1f}"
            if a.batch and ("EA0_RDREQ" in c or "EA0_WRREQ" in c):
                line += f"   x64B per row {v / n * 64 / a.batch:9.1f} B"
            print(line)


if __name__ == "__main__":
    main()
