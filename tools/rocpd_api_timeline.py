#!/usr/bin/env python3
"""Merged host-API / kernel timeline of the last N events of a rocprofv3 database recorded with
--hip-trace --kernel-trace (which host call launched what, and when it ran on which queue):
python tools/rocpd_api_timeline.py run_results.db [--last 120] [--out file.txt]"""
import argparse
import sqlite3
import sys

KEEP = ("hipGraphLaunch", "hipEventSynchronize", "hipStreamWaitEvent", "hipEventRecord", "hipMemcpyAsync",
        "hipLaunchKernel", "hipExtLaunchKernel", "hipModuleLaunchKernel", "hipStreamSynchronize", "igp.")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=120)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ev = [(s, e, "API", n) for s, e, n in c.execute("select start, end, name from regions")
          if any(n.startswith(k) for k in KEEP)]
    ev += [(s, e, f"q{q}", n) for s, e, q, n in c.execute("select start, end, queue_id, name from kernels")]
    ev.sort()
    ev = ev[-a.last:]
    t0 = ev[0][0]
    lines = [f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}us {k:4s} {n[:70]}" for s, e, k, n in ev]
    text = "\n".join(lines)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    else:
        print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
