#!/usr/bin/env python3
"""Hardware queue of every kernel in a rocprofv3 kernel trace (``--kernel-trace --output-format
csv``): which queues a run used and which kernels - RCCL's included - each queue carried.
Evidence for the stream -> hardware-queue plan of engine/dp.py (GPU_MAX_HW_QUEUES = 4 on the
boxes). Usage: python tools/queue_map.py run_kernel_trace.csv [...]"""
import collections
import csv
import sys


def queue_map(path: str) -> str:
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(collections.Counter)
    for r in rows:
        per[r["Kernel_Name"].split("(")[0][:70]][(r["Queue_Id"], r.get("Stream_Id", "?"))] += 1
    queues = sorted({r["Queue_Id"] for r in rows}, key=int)
    out = [f"{path}: {len(rows)} dispatches on {len(queues)} hardware queues {queues}",
           f"{'kernel':72s} (queue, stream): dispatches"]
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1].values())):
        out.append(f"  {k:70s} " + ", ".join(f"q{q}/s{s}: {n}" for (q, s), n in sorted(v.items())))
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(queue_map(p))
        print()
