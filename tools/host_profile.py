#!/usr/bin/env python3
"""Per-call host CPU cost of unary ScoreTransaction (and the account RPCs) by thread group.

Runs the engine + native HTTP/2 server and the native open-loop load generator in this process
at one offered rate, and reads every thread's CPU time (/proc/self/task/*/stat, threads named by
csrc/runtime/thread_name.h) before and after: CPU microseconds per answered call for the load
generator, the HTTP/2 workers, the serving core's stepper / completion / finishers / link
thread, the device driver and Python. VERDICT r4 item 5 ("report per-call CPU cost by stage").

With ``--sample`` the process is also sampled (csrc/runtime/sampler.h, SIGPROF at 4 kHz of CPU
time) and the hottest functions of each thread group are printed (symbols from the shared
objects' symbol tables, `nm`).

Usage: python tools/host_profile.py [--backend cpu|gpu] [--rate 100000] [--seconds 3]
       [--clients 4] [--workers 4] [--rpc tx|ltv|abuse] [--sample]
"""
import bisect
import subprocess
import argparse
import collections
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

CLK = os.sysconf("SC_CLK_TCK")


def thread_cpu():
    """{tid: (name, cpu seconds)} of this process."""
    out = {}
    base = f"/proc/{os.getpid()}/task"
    for tid in os.listdir(base):
        try:
            with open(f"{base}/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"{base}/{tid}/stat") as f:
                st = f.read()
            fields = st[st.rindex(")") + 2:].split()
            out[int(tid)] = (name, (int(fields[11]) + int(fields[12])) / CLK)  # utime + stime
        except (FileNotFoundError, ProcessLookupError, ValueError):
            continue
    return out


def _maps():
    """[(start, end, path)] of the file-backed executable mappings, and each path's load base."""
    rows, base = [], {}
    with open(f"/proc/{os.getpid()}/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) < 6:
                continue
            lo, hi = (int(x, 16) for x in parts[0].split("-"))
            off, path = int(parts[2], 16), parts[5]
            if off == 0 and path not in base:
                base[path] = lo
            if "x" in parts[1]:
                rows.append((lo, hi, path))
    return rows, base


_SYMS = {}


def _symtab(path):
    if path not in _SYMS:
        addrs, names = [], []
        for flags in (["-C", "--defined-only"], ["-D", "-C", "--defined-only"]):
            try:
                out = subprocess.run(["nm", *flags, path], capture_output=True, text=True, timeout=60).stdout
            except Exception:
                continue
            for line in out.splitlines():
                parts = line.split(" ", 2)
                if len(parts) == 3 and parts[1].lower() in ("t", "w"):
                    addrs.append(int(parts[0], 16))
                    names.append(parts[2])
            if addrs:
                break
        order = sorted(range(len(addrs)), key=lambda i: addrs[i])
        _SYMS[path] = ([addrs[i] for i in order], [names[i] for i in order])
    return _SYMS[path]


def symbolise(pcs, maps, base):
    out = []
    los = [m[0] for m in maps]
    for pc in pcs:
        k = bisect.bisect_right(los, int(pc)) - 1
        if k < 0 or pc >= maps[k][1]:
            out.append("?")
            continue
        path = maps[k][2]
        va = int(pc) - base.get(path, maps[k][0])
        addrs, names = _symtab(path)
        j = bisect.bisect_right(addrs, va) - 1
        lib = os.path.basename(path)
        out.append(f"{lib}:{names[j][:90]}" if j >= 0 else f"{lib}:?")
    return out


def group(name: str) -> str:
    for g in ("h2-loadgen", "h2-worker", "h2-cold", "h2-batch", "core-step", "core-done", "core-fin", "core-link",
              "acct-"):
        if name.startswith(g):
            return g if g != "acct-" else name
    return "python/other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="cpu", choices=["cpu", "gpu"])
    ap.add_argument("--model", default="cfg1")
    ap.add_argument("--rpc", default="tx", choices=["tx", "ltv", "abuse"])
    ap.add_argument("--accounts", type=int, default=100000)
    ap.add_argument("--rate", type=float, default=100000)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--sample", action="store_true", help="also sample the hottest functions per thread group")
    a = ap.parse_args()
    import bench_e2e as BE
    from igaming_platform_amd.api.native_grpc import NativeRiskServer
    from igaming_platform_amd.native import native
    from igaming_platform_amd.proto import risk_v1 as P
    if a.rpc == "tx":
        eng = BE.build_engine(a.accounts, 8192, a.backend, a.model)
        payloads = BE.tx_payloads(a.accounts, 8192, seed=300)
    else:
        eng = BE.build_cold_engine(a.accounts, a.backend)
        payloads = BE.acct_payloads(a.accounts, a.rpc, 1 << 16, 300, 0.0)
    srv = NativeRiskServer(eng, port=0, workers=a.workers, batching=True).start()
    path = P.method_path(BE.RPC_PATHS[a.rpc])
    native().grpc_load("127.0.0.1", srv.port, path, payloads, 2000.0, 1.0, a.clients, 4096)  # warm up
    names = {}
    stop_names = threading.Event()

    def name_poll():  # the load generator's threads exist only while grpc_load runs
        while not stop_names.wait(0.2):
            names.update({t: n for t, (n, _) in thread_cpu().items()})
    poller = threading.Thread(target=name_poll, daemon=True)
    poller.start()
    before = thread_cpu()
    proc0 = os.times()
    if a.sample:
        native().sampler_start(4000, 1 << 21)
    t0 = time.perf_counter()
    r = native().grpc_load("127.0.0.1", srv.port, path, payloads, float(a.rate), a.seconds, a.clients, 8192)
    wall = time.perf_counter() - t0
    samples = native().sampler_stop() if a.sample else None
    proc1 = os.times()
    after = thread_cpu()
    stop_names.set()
    names.update({t: n for t, (n, _) in after.items()})
    lat = np.asarray(r["latency_ms"])
    sched = np.asarray(r["sched_ms"]) if "sched_ms" in r else None
    calls = max(len(lat), 1)
    by = collections.defaultdict(float)
    nthreads = collections.Counter()
    for tid, (name, cpu) in after.items():
        c0 = before.get(tid, (name, 0.0))[1]
        by[group(name)] += cpu - c0
        nthreads[group(name)] += 1
    # threads that ended inside the window (the load generator's): the process total minus the rest
    total = (proc1.user + proc1.system) - (proc0.user + proc0.system)
    by["h2-loadgen (exited threads)"] = max(0.0, total - sum(by.values()))
    core = eng.core.stats(False) if getattr(eng, "core", None) is not None else {}
    acct_st = None
    if a.rpc != "tx" and getattr(eng, "acct", None) is not None:
        st = eng.acct.router.stats(3 if a.rpc == "abuse" else 1)
        steps = max(int(st["steps"]), 1)
        acct_st = dict(steps=int(st["steps"]), rows_per_step=round(st["rows"] / steps, 1),
                       max_step_rows=int(st["max_step_rows"]), device_us_per_step=round(st["device_ns"] / steps / 1e3, 1),
                       queue_us_per_item=round(st["queue_ns"] / max(int(st["items"]), 1) / 1e3, 1),
                       wait_errors=int(st["wait_errors"]))
        drv = getattr(getattr(eng.acct, "devices", [None])[-1], "driver", None)
        if drv is not None and hasattr(drv, "fallbacks"):
            acct_st["cluster_fallbacks"] = int(drv.fallbacks)
    res = dict(backend=a.backend, rpc=a.rpc, offered_per_s=a.rate, achieved_per_s=round(len(lat) / float(r["elapsed"]), 1),
               errors=int(r["errors"]), p50_ms=round(float(np.percentile(lat, 50)), 3) if len(lat) else None,
               p99_ms=round(float(np.percentile(lat, 99)), 3) if len(lat) else None, wall_s=round(wall, 2),
               latency_ms_pct={str(q): round(float(np.percentile(lat, q)), 3) for q in (10, 50, 90, 95, 99, 99.9)}
               if len(lat) else None, account_router=acct_st,
               # the slowest call of every 100-ms window of the schedule: a periodic stall shows as
               # a few windows far above the rest
               window_max_ms=[round(float(lat[(sched >= w) & (sched < w + 100)].max()), 2)
                              for w in range(0, int(sched.max()) + 1, 100) if np.any((sched >= w) & (sched < w + 100))]
               if sched is not None and len(lat) else None,
               clients=a.clients, workers=a.workers,
               cpu_us_per_call={k: round(v / calls * 1e6, 2) for k, v in sorted(by.items(), key=lambda x: -x[1])},
               cpu_cores_busy={k: round(v / wall, 2) for k, v in sorted(by.items(), key=lambda x: -x[1])},
               threads=dict(nthreads),
               mean_rows_per_device_step=round(core.get("rows", 0) / max(core.get("steps", 1), 1), 1) if core else None)
    if samples is not None:
        pcs, tids = samples
        maps, base = _maps()
        syms = symbolise(pcs, maps, base)
        hot = collections.defaultdict(collections.Counter)
        for sym, tid in zip(syms, tids):
            hot[group(names.get(int(tid), "?"))][sym] += 1
        res["samples"] = int(len(pcs))
        res["hot"] = {g: [(s_, c) for s_, c in cnt.most_common(25)] for g, cnt in hot.items()}
    print(json.dumps(res), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(res) + "\n")
    srv.stop()
    eng.close()


if __name__ == "__main__":
    main()
