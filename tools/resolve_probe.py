#!/usr/bin/env python3
"""Host resolve cost under a uniform account spread: ScoreBatch payloads (8192 UUID rows each,
ids uniform over --accounts) -> C++ parse -> AccountIndex lookup, on T threads (GIL released).
Prints ns per row for parse and lookup. Usage: python tools/resolve_probe.py [accounts] [threads]"""
import os
import sys
import threading
import time


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    import bench_e2e as B
    from igaming_platform_amd.native import native
    N = native()
    accounts = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ix = N.AccountIndex(accounts + 4096)
    step = 1 << 17
    for s0 in range(0, accounts, step):
        ix.lookup([B.account_id(i) for i in range(s0, min(accounts, s0 + step))], True)
    pl = B.spread_payloads(accounts, 32, 8192, 11)
    batches = []
    for p in pl:
        rb = N.RequestBatch()
        rb.parse_batch(p)
        batches.append(rb)
    res = {}
    for T in sorted({1, threads}):
        per = 64 // T

        def work(k, out):
            t0 = time.perf_counter()
            for i in range(per):
                ix.lookup_batch(batches[(k * per + i) % len(batches)], False)
            out[k] = time.perf_counter() - t0
        out = [0.0] * T
        th = [threading.Thread(target=work, args=(k, out)) for k in range(T)]
        t0 = time.perf_counter()
        [t.start() for t in th]
        [t.join() for t in th]
        el = time.perf_counter() - t0
        rows = per * T * 8192
        res[T] = dict(lookup_ns_per_row_per_thread=round(max(out) / (per * 8192) * 1e9, 1),
                      aggregate_rows_per_s=round(rows / el / 1e6, 1))
    t0 = time.perf_counter()
    for p in pl[:8]:
        rb = N.RequestBatch()
        rb.parse_batch(p)
    res["parse_ns_per_row_1thread"] = round((time.perf_counter() - t0) / (8 * 8192) * 1e9, 1)
    print(res)
    return 0


if __name__ == "__main__":
    sys.exit(main())
