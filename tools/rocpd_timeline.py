#!/usr/bin/env python3
"""Dispatch timeline (start/end/duration/queue) of the last N kernels in a rocprofv3 rocpd
database, plus the GPU busy fraction over that window (union of kernel intervals):
python tools/rocpd_timeline.py gpurun_out/prof/run_results.db [--last 40] [--api]

With --api (a run traced with --kernel-trace --hip-runtime-trace) every dispatch also shows the
host side: when its launch call returned (same clock) and the lead = kernel start - launch
return. A lead near zero means the queue was waiting for the host, not for the GPU."""
import argparse
import sqlite3
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--skip-tail", type=int, default=0, help="drop the last K dispatches (teardown)")
    ap.add_argument("--api", action="store_true", help="join each dispatch with its HIP launch call")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = c.execute(f"select d.start, d.end, d.queue_id, s.display_name, d.event_id from {disp} d join {sym} s "
                     f"on d.kernel_id = s.id order by d.start").fetchall()
    launch = {}
    if a.api:  # a dispatch's event shares its stack id (the internal correlation id) with its launch call
        ev_stack = dict(c.execute("select id, stack_id from rocpd_event"))
        for name, st, en, tid, sid in c.execute("select name, start, end, tid, stack_id from regions"):
            launch.setdefault(sid, (name, st, en, tid))
        launch = {eid: launch.get(sid) for eid, sid in ev_stack.items() if sid in launch}
    if a.skip_tail:
        rows = rows[:-a.skip_tail]
    rows = rows[-a.last:]
    t0 = rows[0][0]
    for st, en, q, name, eid in rows:
        host = ""
        if a.api and launch.get(eid):
            api, hs, he, tid = launch[eid]
            host = f"  host {(he - t0) / 1e3:9.1f} lead {(st - he) / 1e3:7.1f}us t{tid} {api}"
        print(f"{(st - t0) / 1e3:9.1f} {(en - t0) / 1e3:9.1f} {(en - st) / 1e3:7.1f}us q={q} {name[:50]}{host}")
    busy, cur_s, cur_e = 0, None, None
    for st, en, _, _, _ in sorted(rows):
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    busy += cur_e - cur_s
    span = max(r[1] for r in rows) - t0
    print(f"window {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / span:.0f}%), "
          f"sum of kernel time {sum(r[1] - r[0] for r in rows) / 1e3:.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
