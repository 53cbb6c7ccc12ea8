#!/usr/bin/env python3
"""Headline benchmark: fraud scores/sec (whole node) + p99 score latency, MI355X.

BASELINE.json metric "fraud scores/sec (whole node) + p99 score latency at 1/2/4/8 MI355X";
default config = cfg 3, the data-parallel headline: GBDT+MLP stacked ensemble
(ONNX TreeEnsembleRegressor(100 trees, depth 7, 128 features, 32 targets) -> Gemm(32x256)
-> Relu -> Gemm(256x1) -> Sigmoid), micro-batch 8192 per GPU, DP over all GPUs with RCCL.

Default scope (serving), per rank: 16 ingress threads each send risk.v1 ScoreBatch request bytes
(8192 transactions, UUID account ids) into the rank's native serving core and get response bytes
back: C++ parse, node-shared AccountIndex resolve, micro-batch step clock, the GPU pipeline below,
response writer (FeatureVector bodies encoded on the device). One timed step = one round of
requests, one per ingress thread (16 x 8192 transactions per rank), nothing skipped.
Device micro-batch (per GPU, 8192 rows), three streams driven by the native driver
(engine/scorer.py, csrc/kernels/driver.hip; stage kernels issued from recorded op lists):
      copy:  H2D slab -> dedup insert
      state: feature_assemble (ring windows, HLL, blacklist, ip-intel, rules, single-event
             score-then-update, FeatureVector encode) -> multi-event update segments
      model: tree ensemble -> f32-MFMA head -> ensemble/action (+metrics), one launch
             -> results into pinned host memory
      batches i, i+1, i+2 overlap across the three stages
  N > 1: every rank ingests; the owner-routed RCCL exchange (two all-to-alls per device step)
  moves every row to the rank owning its account and the results back (engine/dp.py)
Per-GPU work is fixed as N grows (weak scaling). --scope engine_only: pre-resolved rows into the
device pipeline, one step = one 8192-row micro-batch (the device-pipeline number).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|heuristic]
For N > 1 run under torchrun (the driver does), or this script launches torchrun itself.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

# kernel arguments in device memory (igaming_platform_amd/__init__.py): set before any GPU call
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

DATA_PG = None  # replicas mode: the RCCL group of the results all-gather (None: the default group)
BASELINE_P99_MS = 50.0  # README.md:58 "< 50ms latency" (the only published number)

CONFIGS = ("cfg3", "cfg2", "cfg1", "heuristic", "cfg4", "cfg5")  # igaming_platform_amd/utils/benchkit.py


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="per-GPU micro-batch (default: the config's)")
    ap.add_argument("--accounts", type=int, default=1 << 20, help="feature-store accounts per GPU")
    ap.add_argument("--depth", type=int, default=0,
                    help="pipeline depth (batches in flight; up to 7, launch.h DEDUP_AHEAD); default 6 for the "
                         "fraud configs, 3 for cfg4 / cfg5 (one stream per slot: a fourth slot stream plus the "
                         "default stream exceed the box's 4 hardware queues - same-box A/B cfg4 135.5 vs 105.7 M, "
                         "cfg5 2.62 vs 2.42 M, profiles/r6/a)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the per-step RCCL all_gather")
    ap.add_argument("--numerics", default="auto", choices=["auto", "fp32", "bf16"],
                    help="dense-layer numerics: fp32 = the ONNX model's f32 contract (default; f32 MFMA heads, "
                         "split bf16x3 MFMA for the cfg4 chain and the cfg5 GRU), bf16 = bf16 MFMA with f32 accumulate")
    ap.add_argument("--dp-mode", default="exchange", choices=["exchange", "replicas"],
                    help="N > 1: exchange = every rank ingests 8192 rows/step spread over all owners and "
                         "the owner-routed RCCL exchange (the serving path, engine/dp.py) moves each row to "
                         "its owner and the results back; replicas = N independent single-GPU pipelines")
    ap.add_argument("--scope", default="auto", choices=["auto", "serving", "engine_only", "e2e", "grpc"],
                    help="auto (default): serving; for cfg4 / cfg5 that is PredictLTV / CheckBonusAbuse bytes "
                         "through every rank's native account router, owner-routed (acct_dp_bench); serving for "
                         "the fraud configs: the serving objects of every rank - "
                         "risk.v1 ScoreBatch request bytes (UUID account ids) -> the rank's native serving core "
                         "(C++ parse, node-shared AccountIndex, "
                         "owner-routed RCCL exchange steps for N > 1, GPU pipeline) -> response bytes with the "
                         "FeatureVector, every rank ingesting; engine_only: pre-resolved ReqRec rows into the "
                         "device pipeline (device-pipeline number); e2e / grpc: tools/bench_e2e.py")
    ap.add_argument("--threads", type=int, default=16,
                    help="serving scope: ingress threads per rank (the box gives each GPU 16 CPUs)")
    ap.add_argument("--rounds", type=int, default=32,
                    help="serving scope: ScoreBatch requests per ingress thread in one timed step (a step of "
                         "threads x rounds requests per rank keeps the driver's --steps 20 window >= 0.5 s)")
    ap.add_argument("--requests", type=int, default=0, help="serving scope: transactions per ScoreBatch request "
                    "(default: the config's micro-batch)")
    ap.add_argument("--rpc", default="batch", choices=["batch", "tx"], help="--scope grpc: ScoreBatch or unary "
                    "ScoreTransaction through the micro-batcher")
    ap.add_argument("--rates", default="",
                    help="--scope serving with cfg4 / cfg5, 1 GPU: offered PredictLTV / CheckBonusAbuse calls/s per "
                         "level, open loop over the native gRPC server (e.g. 25000,50000,100000,200000); without it "
                         "the owner-routed DP bench (every rank's account router, closed loop)")
    ap.add_argument("--calls", type=int, default=65536, help="cfg4 / cfg5 serving: calls per rank per step")
    ap.add_argument("--inflight", type=int, default=0,
                    help="cfg4 / cfg5 serving: outstanding calls per rank (0: (depth + 3) x the device step, so a "
                         "freed slot finds a full step queued while the answers of the step before it are still "
                         "on their way back)")
    ap.add_argument("--drive-threads", type=int, default=4,
                    help="cfg4 / cfg5 serving: threads submitting calls per rank (one thread: the submit loop "
                         "itself bounds the rate, profiles/r6/s)")
    ap.add_argument("--finishers", type=int, default=0,
                    help="cfg4 / cfg5 serving: answer-writing threads per account device (0: the config's)")
    ap.add_argument("--check-out", default="", help="cfg4 / cfg5 serving: after the timed run every rank answers "
                    "the same fixed calls and writes them to <check-out>.<rank>.json (tests/test_bench_acct.py)")
    ap.add_argument("--seconds", type=float, default=5.0, help="cfg4 / cfg5 serving: seconds per offered-load level")
    ap.add_argument("--zipf", type=float, default=0.0, help="serving: Zipf exponent of the account ids (0: uniform)")
    ap.add_argument("--payloads", type=int, default=128, help="serving: distinct ScoreBatch requests per rank "
                    "(their account ids spread over the whole population)")
    ap.add_argument("--sum-mode", default="sliding", choices=["sliding", "compat"],
                    help="fraud configs: the 1h amount sum - sliding (exact, from the tx ring: default) or compat "
                         "(the reference's INCRBY-with-TTL running sum, redis_store.go:136-138; quirk Q8)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    if a.numerics == "auto":  # the ONNX models' f32 contract everywhere (cfg4 / cfg5: split MFMA)
        a.numerics = "fp32"
    if a.scope == "auto":  # cfg4 / cfg5: the account-RPC serving path, owner-routed over every rank
        a.scope = "serving"
    a.depth_given = a.depth > 0
    if a.depth <= 0:
        # fraud configs: 6 slots - a serving slot stays held while its caller copies the step's
        # results and feature images out (~72 us), so at 4 the stepper waited for a slot 1.2 times
        # per step; same box, interleaved, 2 runs each: depth 4 / 5 / 6 / 7 = 116.8-121.0 /
        # 118.8-120.3 / 122.7-127.4 / 123.1-128.4 M (profiles/r6/ad)
        a.depth = 3 if a.config in ("cfg4", "cfg5") else 6
    return a


def numerics_desc(a) -> str:
    split = ("f32-faithful: bf16 hi/lo pairs of every weight and activation, three bf16 MFMAs per product "
             "(hi*hi + hi*lo + lo*hi), fp32 accumulate")
    if a.config == "cfg5":
        return (split + " and fp32 hidden state" if a.numerics == "fp32"
                else "bf16 MFMA weights/activations, fp32 accumulate and state")
    if a.config == "cfg4":
        return split if a.numerics == "fp32" else "bf16 MFMA weights/activations, fp32 accumulate"
    dense = ("fp32 MFMA (v_mfma_f32_16x16x4_f32) MLP" if a.numerics == "fp32"
             else "bf16 MFMA MLP (fp32 accumulate)")
    return f"fp32 features+trees, {dense}, fp64 ensemble"


def maybe_launch_torchrun(a) -> None:
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        port = 29500 + (os.getpid() % 1000)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port)] + sys.argv
        sys.exit(subprocess.call(cmd))


def gpu_index(local: int) -> int:
    """One rank per GPU. More ranks than GPUs (the 1-GPU box's multi-rank rehearsal of the
    node-shared exchange path, which opens no RCCL communicator) share them round-robin; RCCL
    itself refuses two ranks on one device. device_count() does not initialise the HIP runtime."""
    import torch
    n = torch.cuda.device_count()
    return local % n if 0 < n <= local else local


def acct_serving_bench(a) -> None:
    """cfg4 / cfg5 offered-load curve, 1 GPU (--rates): unary PredictLTV / CheckBonusAbuse calls
    over the native HTTP/2 server (bytes in -> the native account router -> micro-batches on the
    LTV chain / abuse step -> response bytes) from the native open-loop load generator; the value
    is the highest offered rate answered in full with p99 < 50 ms (tools/bench_e2e.py
    _native_open_loop)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import bench_e2e
    argv = ["--scope", "grpc", "--rpc", "ltv" if a.config == "cfg4" else "abuse", "--open-loop", "--accounts",
            str(a.accounts), "--rates", a.rates, "--seconds", str(a.seconds), "--numerics", a.numerics,
            "--zipf", str(a.zipf)] + (["--json-out", a.json_out] if a.json_out else [])
    return bench_e2e.main(argv)


NOW_ACCT = 1_760_000_000  # the account benches' clock (fixed: answers comparable across runs)


def acct_models(numerics: str, small: bool = False):
    """The cfg4 LTV MLP 4x512 over 256 features and the cfg5 abuse GRU 2x256 over the last 100
    events (random-init, deterministic), as ONNX bytes; the config they run under. ``small``:
    narrow models of the same structure (CPU protocol rehearsals only, never a benchmark)."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.onnx import builders
    cfg = Config()
    cfg.gpu.buckets = [64, 512, 4096]
    cfg.gpu.max_batch = 4096
    cfg.gpu.spmd_heartbeat_s = 0.0
    cfg.ltv_model.precision = cfg.abuse_model.precision = numerics
    w, h = (32, 16) if small else (512, 256)
    lm = builders.build("ltv_mlp", n_features=256, width=w, layers=4).SerializeToString()
    am = builders.build("gru", seq=100, in_dim=16, hidden=h).SerializeToString()
    return cfg, lm, am


def acct_dp_bench(a) -> None:
    """cfg4 / cfg5 through the account-RPC serving path on every rank (BASELINE
    config 5 "DP=8 over xGMI"): each rank runs its shard (its accounts' profile rows and HBM
    event rings) and its native ``AcctRouter``; every rank ingests PredictLTV / CheckBonusAbuse
    request bytes for account ids spread over ALL owners, and the router sends each call to the
    owner's model device over the node-shared /dev/shm mailbox (the owner micro-batches the
    calls of every sender into its LTV chain / abuse GRU step and mails the answer bytes back).
    No replicas, no all-gather: each call is computed once, on the GPU that holds its account.

    A step = ``--calls`` calls per rank, driven in-process closed-loop (``AcctRouter.drive``:
    at most ``--inflight`` outstanding, bytes in -> answer bytes out, no Python per call); the
    value is the whole job's answered calls per second, the latency per call submit -> answer.
    IGP_BENCH_BACKEND=cpu: the same objects on CPU shards (tests/test_bench_acct.py)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import bench_e2e
    from igaming_platform_amd.layouts import ACCTBATCH
    from igaming_platform_amd.native import native
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.hashing import SEED_ACCOUNT

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    kind = os.environ.get("IGP_BENCH_BACKEND", "gpu")
    if kind == "gpu":
        local = gpu_index(local)
        torch.cuda.set_device(local)
    comm = None
    if world > 1:
        dist.init_process_group("gloo")
        from igaming_platform_amd.parallel.comm import TorchComm
        comm = TorchComm("gloo")
    rpc_name = "ltv" if a.config == "cfg4" else "abuse"
    rpc = native().RPC_LTV if rpc_name == "ltv" else native().RPC_ABUSE
    small = os.environ.get("IGP_BENCH_SMALL_MODELS") == "1"  # CPU rehearsal (tests/test_bench_acct.py)
    if small and kind == "gpu":
        raise SystemExit("IGP_BENCH_SMALL_MODELS is for the CPU rehearsal only")
    cfg, lm, am = acct_models(a.numerics, small)
    # the account devices' pipeline slots (--depth; default: cfg5 3, cfg4 2 - same-box sweep
    # cfg5 1.66 / 1.84 / 1.63 M at 2 / 3 / 4, cfg4 4.28 / 1.58 M at 2 / 3, profiles/r6/n)
    cfg.gpu.acct_depth = max(2, a.depth) if getattr(a, "depth_given", True) else (2 if a.config == "cfg4" else 3)
    if a.finishers > 0:
        cfg.gpu.serve_finishers = a.finishers
    if a.inflight <= 0:
        a.inflight = (cfg.gpu.acct_depth + 3) * cfg.gpu.max_batch
    n_acc = a.accounts
    if world == 1:
        from igaming_platform_amd.engine.risk_engine import RiskEngine
        eng = RiskEngine(cfg, backend=kind, capacity=n_acc + 1024, ltv_model=lm, abuse_model=am)
        acct, registry, ltv, backend = eng.acct, eng.registry, eng.ltv, eng.backends[0]
    else:
        from igaming_platform_amd.engine.risk_engine import worker_acct, worker_node
        node = worker_node(cfg, comm, kind, n_acc + 1024)
        ltv, acct = worker_acct(cfg, node, lm, am)
        registry, backend = node.registry, node.local
    if acct is None or not acct.serves(rpc):
        raise RuntimeError("no native account router for this RPC")
    router = acct.router
    # this rank's accounts: the global population is world x n_acc UUIDs, owner = XXH64(id) % world
    # (an account's profile depends on its index only, not on the world size or its owner)
    total = n_acc * world
    step = 1 << 16
    for s0 in range(0, total, step):
        ids = [bench_e2e.account_id(i) for i in range(s0, min(total, s0 + step))]
        h = native().id_hashes(ids, SEED_ACCOUNT)
        mine = np.nonzero((h % np.uint64(world)).astype(np.int64) == rank)[0]
        if not len(mine):
            continue
        rng = np.random.default_rng(1000 + s0)
        rows = np.floor(rng.uniform(0, 1, (len(ids), 25)) * bench_e2e.PROFILE_SCALE).astype(np.float32)
        ext = rng.normal(0, 1, (len(ids), 231)).astype(np.float32)
        slots, owners = registry.resolve_ids([ids[i] for i in mine], insert=True)
        ltv.set_rows(slots, owners, rows[mine], ext[mine])
        # warehouse rows (the abuse rules' bonus / wager / deposit inputs)
        g = (s0 + mine).astype(np.int64)
        wb = np.zeros(len(mine), ACCTBATCH)
        wb["present"] = 1
        wb["total_deposits"] = (g % 97) * 700
        wb["total_bets"] = (g % 89) * 1300
        wb["bonus_claim_count"] = g % 6
        wb["bonus_wager_complete"] = (g % 5) / 5.0
        wb["account_created_at"] = NOW_ACCT - (g % 40) * 86400
        backend.set_batch_rows(slots, wb)
    if kind == "gpu":  # full 100-event histories in the shard's HBM event rings
        bench_e2e.fill_event_rings(backend.store, seed=77 + rank)
    if comm is not None:
        comm.barrier()
    payloads = bench_e2e.acct_payloads(total, rpc_name, 1 << 16, 300 + rank, a.zipf)
    per_step = a.calls
    now = NOW_ACCT
    router.drive(rpc, payloads, max(a.warmup, 1) * per_step, a.inflight, now, a.drive_threads)  # warm
    router.stats(3 if rpc_name == "abuse" else 1, True)  # the timed run's device steps only
    if comm is not None:
        comm.barrier()
    # IGP_BENCH_THREADS_OUT=<path>: per-thread CPU over the timed run (rank 0), as in the cfg3
    # serving bench - which of the router's threads (stepper, completion, finishers, mailbox) or
    # the drive threads, if any, is saturated
    threads_out = os.environ.get("IGP_BENCH_THREADS_OUT") if rank == 0 else None
    if threads_out:
        import host_profile
        cpu0, proc0 = host_profile.thread_cpu(), os.times()
    t0 = time.perf_counter()
    r = router.drive(rpc, payloads, a.steps * per_step, a.inflight, now, a.drive_threads)
    if comm is not None:
        comm.barrier()
    elapsed = time.perf_counter() - t0
    if threads_out:
        cpu1, proc1 = host_profile.thread_cpu(), os.times()
        busy, alive = {}, 0.0
        for tid, (name, cpu) in cpu1.items():
            d = cpu - cpu0.get(tid, (name, 0.0))[1]
            alive += d
            if d > 0:
                busy.setdefault(name, []).append(round(d / elapsed, 3))
        total = (proc1.user + proc1.system) - (proc0.user + proc0.system)
        with open(threads_out, "w") as f:  # the drive threads exit with drive(): total minus the rest
            json.dump({"elapsed_s": elapsed, "cpu_fraction_by_thread_name": busy,
                       "drive_threads_cores": round(max(0.0, total - alive) / elapsed, 2),
                       "process_cores": round(total / elapsed, 2)}, f, indent=1)
    lat = np.asarray(r["latency_ns"], np.float64)
    ok = lat[lat >= 0] / 1e6
    p99 = float(np.percentile(ok, 99)) if len(ok) else float("nan")
    p50 = float(np.percentile(ok, 50)) if len(ok) else float("nan")
    errors, cold = int(r["errors"]), int(r["cold"])
    st = router.stats(3 if rpc_name == "abuse" else 1)
    if comm is not None:  # the slowest rank's clock and latencies, every rank's errors
        mx = torch.tensor([elapsed, p99, p50], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed, p99, p50 = (float(x) for x in mx)
        ec = torch.tensor([errors, cold, int(router.remote_out)], dtype=torch.int64)
        dist.all_reduce(ec)
        errors, cold, remote = (int(x) for x in ec)
    else:
        remote = int(router.remote_out)
    c = benchkit.MODEL_CONFIGS[a.config]
    out = {
        "metric": c["metric"], "value": world * a.steps * per_step / elapsed, "unit": c["unit"], "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.numerics,
        "data": "synthetic (UUID account ids, random-init weights, random 100-event histories)",
        "config": {"model": c["desc"], "global_batch": per_step * world, "seq_len": 100 if a.config == "cfg5" else 1,
                   "parallelism": f"dp{world} (owner-routed: each call computed once, on its account's GPU)",
                   "calls_per_step_per_rank": per_step, "inflight_per_rank": a.inflight,
                   "device_pipeline_depth": cfg.gpu.acct_depth,
                   "submit_threads_per_rank": a.drive_threads, "finishers_per_device": cfg.gpu.serve_finishers,
                   "device_micro_batch_max": max(cfg.gpu.buckets), "accounts_per_gpu": n_acc,
                   "account_spread": f"zipf({a.zipf})" if a.zipf > 1 else "uniform",
                   "numerics": numerics_desc(a), "backend": kind,
                   **({"models": "SMALL rehearsal models (not the cfg4 / cfg5 sizes)"} if small else {})},
        "scope": "serving (risk.v1 request bytes in -> answer bytes out through every rank's native account "
                 "router and the /dev/shm owner mailbox, in-process closed loop)",
        "p99_latency_ms": p99, "p50_latency_ms": p50, "latency_what": "per call, submit -> answer bytes",
        "errors": errors, "cold_path_calls": cold, "remote_calls_rank_sum": remote,
        "device_steps_rank0": int(st.get("steps", 0)), "rows_per_device_step_rank0":
            round(st.get("items", 0) / max(int(st.get("steps", 1)), 1), 1),
        # where a call's time goes on rank 0 (acct_core.h AcctStats): queueing before its step,
        # the step on the device, the answer writing
        "device_us_per_step_rank0": round(st.get("device_ns", 0) / max(int(st.get("steps", 1)), 1) / 1e3, 1),
        "queue_us_per_call_rank0": round(st.get("queue_ns", 0) / max(int(st.get("items", 1)), 1) / 1e3, 1),
        "max_step_rows_rank0": int(st.get("max_step_rows", 0)),
        # the slot cycle (acct_core.h AcctStats): dev->submit, device done -> slot released, slot
        # free -> next step on it; why each step was issued (full / idle device / queue head aged)
        "slot_cycle_us_per_step_rank0": {k: round(st.get(k + "_ns", 0) / max(int(st.get("steps", 1)), 1) / 1e3, 1)
                                         for k in ("submit", "turn", "free", "finish")},
        "steps_by_reason_rank0": {k: int(st.get(k + "_steps", 0)) for k in ("full", "idle", "aged")},
        "cluster_fallbacks_rank0": sum(int(getattr(getattr(d, "driver", None), "fallbacks", 0) or 0)
                                       for d in getattr(acct, "devices", [])),
    }
    if errors:
        raise RuntimeError(f"{errors} calls failed ({cold} cold-path replies)")
    if a.check_out:  # every rank asks the same calls (accounts 0..47 + an unknown id) and dumps the answers
        check = [bench_e2e.acct_request(rpc_name, bench_e2e.account_id(i)) for i in range(min(total, 48))]
        check.append(bench_e2e.acct_request(rpc_name, "nobody"))
        for i, b in enumerate(check):
            router.submit(rpc, b, i, 0, now)
        got, t_end = {}, time.time() + 60
        while len(got) < len(check) and time.time() < t_end:
            for tag, b, e in router.poll(4096, 50000):
                got[int(tag)] = b.hex() if e is None else "error: " + e
        with open(f"{a.check_out}.{rank}.json", "w") as f:
            json.dump({"rank": rank, "world": world, "answers": [got.get(i) for i in range(len(check))]}, f)
        if comm is not None:
            comm.barrier()
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        router.stop()
        dist.destroy_process_group()
    else:
        eng.close()


def main():
    a = parse()
    if a.scope == "serving" and a.config in ("cfg4", "cfg5"):
        if a.rates:  # the 1-GPU offered-load curve over HTTP/2
            return acct_serving_bench(a)
        maybe_launch_torchrun(a)
        return acct_dp_bench(a)
    if a.scope == "serving":
        maybe_launch_torchrun(a)
        return serving_bench(a)
    if a.scope != "engine_only":  # 1 GPU, the request path end to end (tools/bench_e2e.py)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
        import bench_e2e
        argv = ["--scope", a.scope, "--rpc", a.rpc, "--accounts", str(a.accounts), "--steps", str(a.steps),
                "--warmup", str(a.warmup)] + (["--json-out", a.json_out] if a.json_out else [])
        return bench_e2e.main(argv)
    maybe_launch_torchrun(a)
    # HIP multiplexes streams onto GPU_MAX_HW_QUEUES hardware queues (default 4): the scorer's
    # copy / state / model streams, the default stream and RCCL's communication stream (N > 1)
    # each get a queue of their own when 8 are allowed. Set before the HIP runtime initialises; an
    # exported value wins (the GPU boxes export 4: same-box A/B 4 vs 8 neutral, profiles/NOTES.md).
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    # dmabuf IPC for RCCL / cross-process tensors: read when the HIP runtime initialises
    # (torch.cuda.set_device below), so it must be in the environment before that
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; IGP_DIST_BACKEND=gloo lets several ranks share one GPU to rehearse the
    # multi-rank path on a 1-GPU box (RCCL refuses two ranks on one device)
    backend = os.environ.get("IGP_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if backend != "nccl" else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0

    exchange = ((world > 1 and a.dp_mode == "exchange" and a.config not in benchkit.MODEL_CONFIGS)
                or os.environ.get("IGP_FORCE_EXCHANGE") == "1")
    if world > 1:
        if exchange or backend != "nccl":
            # the exchange moves rows over its own two RCCL communicators; the process group is
            # only the control plane (barriers, the final max-reduce), on the CPU over gloo: no
            # third communicator or its stream competes for the 4 hardware queues
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    if a.config in benchkit.MODEL_CONFIGS:
        return model_bench(a, world, rank, dev)

    if exchange:
        if dp_bench(a, world, rank, dev) is not None:  # (forced at N = 1: RCCL's single-rank path, for tests)
            return
    global DATA_PG
    if world > 1 and backend == "nccl" and dist.get_backend() != "nccl":
        DATA_PG = dist.new_group(backend="nccl")  # replicas fallback: results all-gather over RCCL
    S = benchkit.build(a.config, a.batch, a.accounts, dev, rank=rank, depth=a.depth,
                       use_graphs=not a.no_graphs, precision=a.numerics, sum_mode=a.sum_mode)
    sc, pool, B = S.scorer, S.pool, S.batch
    c = dict(desc=S.desc)
    n_acc = a.accounts

    gathered = torch.zeros(world * B * 2, dtype=torch.int32, device=dev) if world > 1 else None
    met_sum = torch.zeros(128, dtype=torch.int64, device=dev)

    gather_work = {}  # slot -> async all_gather still reading that slot's result rows

    def step(i: int, now: int):
        slot = sc.next_slot()
        if slot in gather_work:
            # the slot's result rows are rewritten by this batch's model graph: the model stream
            # waits for the gather that read them (issued `depth` batches ago, long finished),
            # so the collective never sits on the model stream's critical path
            with torch.cuda.stream(sc.mstream):
                gather_work.pop(slot).wait()
        # the wire decoder's output (raw REQREC rows) -> pinned slab -> three graphs; with the
        # native driver (default) the row copy and every launch are issued from C++
        p = sc.submit_rows(slot, pool[i % len(pool)], now)
        if world > 1 and not a.no_gather:
            with torch.cuda.stream(sc.mstream):  # results / metrics live on the model stream
                gather_work[slot] = dist.all_gather_into_tensor(gathered, sc.slots[slot].res[:B].reshape(-1),
                                                                async_op=True, group=DATA_PG)
                if i % 16 == 15:
                    met_sum.copy_(sc.metrics)
                    dist.all_reduce(met_sum, group=DATA_PG)
                if p.event is not None:
                    p.event.record(sc.mstream)
        return p

    inflight = []
    lat = []
    now = NOW0
    for i in range(a.warmup):
        inflight.append(step(i, now + i // 50))
        if len(inflight) >= a.depth:
            sc.wait(inflight.pop(0), unpack=False)
    for p in inflight:
        sc.wait(p, unpack=False)
    inflight = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        p = step(a.warmup + i, now + (a.warmup + i) // 50)
        inflight.append(p)
        if len(inflight) >= a.depth:
            q = inflight.pop(0)
            sc.wait(q, unpack=False)
            lat.append((time.perf_counter() - q.t_submit) * 1e3)
    for q in inflight:
        sc.wait(q, unpack=False)
        lat.append((time.perf_counter() - q.t_submit) * 1e3)
    for w in gather_work.values():
        w.wait()
    gather_work.clear()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    host = sc.driver.stats() if sc.driver is not None else {}
    stats = torch.tensor([elapsed, float(np.percentile(lat, 99)), float(np.percentile(lat, 50))],
                         dtype=torch.float64, device=dev if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed, p99, p50 = (float(x) for x in stats.cpu())
    total = world * B * a.steps
    out = {
        "metric": "fraud scores/sec (whole node) + p99 score latency",
        "value": total / elapsed,
        "unit": "scores/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.numerics,
        "data": "synthetic",
        "config": {
            "model": c["desc"],
            "global_batch": B * world,
            "seq_len": 1,
            "parallelism": f"dp{world}",
            "per_gpu_batch": B,
            "accounts_per_gpu": n_acc,
            "pipeline_depth": a.depth,
            "graphs": not a.no_graphs,
            "launch": "direct (recorded op lists)" if getattr(sc, "direct", False) else "hipGraph replay",
            "driver": "native" if sc.driver is not None else "python",
            "dp_mode": a.dp_mode if world > 1 else "none",
            "numerics": numerics_desc(a),
            "sum_mode": a.sum_mode,
        },
        "scope": "engine_only",
        "p99_latency_ms": p99,
        "p50_latency_ms": p50,
        "latency_baseline_ms": BASELINE_P99_MS,
        "latency_vs_baseline": BASELINE_P99_MS / p99 if p99 > 0 else None,
        "host_us_per_batch": {k: round(float(v), 2) for k, v in host.items()},
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def dp_bench(a, world: int, rank: int, dev) -> None:
    """N > 1, the serving path: each rank ingests a micro-batch of 8192 pre-resolved requests
    per step whose accounts are spread uniformly over all N owners; per step the owner-routed
    exchange (csrc/kernels/exchange.hip, two RCCL all-to-alls over xGMI) delivers every row to
    its owner, each GPU scores only the rows it owns (~8192 per step: 1/N from every rank), and
    the 8-byte results return to the ingress rank and to its pinned host memory. Counted rows
    are the rows actually sent and answered."""
    import torch
    import torch.distributed as dist
    from igaming_platform_amd.parallel.exchange import rccl_comms
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0
    if a.depth < 2:
        raise SystemExit("the exchange pipeline needs --depth >= 2")
    err = ""
    # communicator set-up under a deadline (a daemon thread: ncclCommInitRank blocks), so a
    # node where it cannot complete falls back to replicas instead of hanging the sweep
    import threading
    box = {}

    def _init():
        try:
            box["comms"] = rccl_comms(rank, world)
        except Exception as e:  # RCCL refused (e.g. ranks sharing a GPU): every rank falls back together
            box["err"] = f"{type(e).__name__}: {e}"
    th = threading.Thread(target=_init, daemon=True, name="rccl-init")
    th.start()
    th.join(float(os.environ.get("IGP_XCHG_INIT_S", "120")))
    comms = box.get("comms")
    if comms is None:
        err = box.get("err", "communicator set-up timed out")
    if world > 1:
        bad = torch.tensor([0 if comms is not None else 1], dtype=torch.int32)  # control plane (gloo, CPU)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if int(bad.item()):
            print(json.dumps({"warning": "exchange communicators failed; replicas fallback", "rank": rank,
                              "error": err}), file=sys.stderr, flush=True)
            a.dp_mode = "replicas (exchange init failed)"
            return None
    elif comms is None:
        raise RuntimeError(err)
    S = benchkit.build(a.config, a.batch, a.accounts, dev, rank=rank, depth=a.depth, precision=a.numerics,
                       dp=dict(world=world, comms=comms))
    sc, pool, B, C = S.scorer, S.pool, S.batch, S.chunk

    def step(i: int, now: int):
        slot = sc.next_slot()
        chunks, n = pool[i % len(pool)]
        return sc.submit_chunks(slot, C, now, chunks, n=n)

    # probe: two steps under a deadline (event wait; past it the communicators are aborted), so a
    # broken or hung exchange on a new node falls back to replicas instead of hanging the bench
    ok, err = 1, ""
    try:
        for i in range(2):
            sc.wait_x(step(i, NOW0), gather=False, timeout_s=float(os.environ.get("IGP_XCHG_PROBE_S", "60")))
    except Exception as e:
        ok, err = 0, f"{type(e).__name__}: {e}"
        sc.abort_exchange()
    if world > 1:
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = int(flag.item())
    if not ok:
        print(json.dumps({"warning": "exchange probe failed; replicas fallback", "rank": rank, "error": err}),
              file=sys.stderr, flush=True)
        a.dp_mode = "replicas (exchange probe failed)"
        return None
    inflight, lat, rows = [], [], 0
    for i in range(a.warmup):
        inflight.append(step(i, NOW0 + i // 50))
        if len(inflight) >= a.depth:
            sc.wait_x(inflight.pop(0), gather=False)
    for p in inflight:
        sc.wait_x(p, gather=False)
    inflight = []
    sc.xdriver.stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        p = step(a.warmup + i, NOW0 + (a.warmup + i) // 50)
        rows += p.n
        inflight.append(p)
        if len(inflight) >= a.depth:
            q = inflight.pop(0)
            sc.wait_x(q, gather=False)
            lat.append((time.perf_counter() - q.t_submit) * 1e3)
    for q in inflight:
        sc.wait_x(q, gather=False)
        lat.append((time.perf_counter() - q.t_submit) * 1e3)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    host = sc.xdriver.stats()
    stats = torch.tensor([elapsed, float(np.percentile(lat, 99)), float(np.percentile(lat, 50))], dtype=torch.float64)
    total = torch.tensor([rows], dtype=torch.int64)
    over = torch.tensor([sc.route_overflow(s, C) for s in range(sc.depth)], dtype=torch.int64)
    # device metrics of every shard, summed once after the timed window over the control plane
    # (in serving they feed /metrics through the core's own counters)
    met = sc.metrics.cpu()
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(total)
        dist.all_reduce(over)
        dist.all_reduce(met)
    elapsed, p99, p50 = (float(x) for x in stats.cpu())
    total = int(total.item())
    out = {
        "metric": "fraud scores/sec (whole node) + p99 score latency",
        "value": total / elapsed, "unit": "scores/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.numerics, "data": "synthetic",
        "config": {"model": S.desc, "global_batch": B * world, "seq_len": 1, "parallelism": f"dp{world}",
                   "per_gpu_batch": B, "accounts_per_gpu": a.accounts, "pipeline_depth": a.depth, "graphs": True,
                   "launch": "direct (recorded op lists)" if getattr(sc, "direct", False) else "hipGraph replay",
                   "driver": "native exchange (XchgDriver; two RCCL all-to-alls per step"
                             + (", captured in the hipGraphs)" if sc.captured else ", issued by the driver)"),
                   "dp_mode": "exchange", "chunk_capacity": C, "rows_scored": total,
                   "rows_scored_device_metrics": int(met[106]),
                   "control_plane": "gloo (CPU)" if world > 1 else "none",
                   "rows_dropped_by_route": int(over.sum().item()),
                   "numerics": numerics_desc(a),
                   # collective / queue knobs in effect, so a scaling curve is self-describing
                   "comm_env": {k: v for k, v in sorted(os.environ.items())
                                if k.startswith(("NCCL_", "RCCL_")) or k == "GPU_MAX_HW_QUEUES"}},
        "scope": "engine_only",
        "p99_latency_ms": p99, "p50_latency_ms": p50, "latency_baseline_ms": BASELINE_P99_MS,
        "latency_vs_baseline": BASELINE_P99_MS / p99 if p99 > 0 else None,
        "host_us_per_batch": {k: round(float(v), 2) for k, v in host.items()},
    }
    _emit(a, world, rank, out)
    return out


def _hot_by_thread(samples, names) -> dict:
    """{thread name: [(function, samples)]} from the native SIGPROF sampler (tools/host_profile.py)."""
    import collections
    import host_profile
    pcs, tids = samples
    maps, base = host_profile._maps()
    syms = host_profile.symbolise(pcs, maps, base)
    hot = collections.defaultdict(collections.Counter)
    for sym, tid in zip(syms, tids):
        hot[names.get(int(tid), ("exited", 0))[0]][sym] += 1
    return {k: c.most_common(12) for k, c in hot.items()}


def serving_bench(a) -> None:
    """The serving objects end to end, every rank ingesting (bench.py --gpus N runs
    the serving path, not a hand-built scorer). Per rank:

      * N = 1: ``RiskEngine`` (GPU backend) and its native serving core over the three-stream
        pipeline; N > 1: ``SpmdNode`` - the rank's shard joined to the owner-routed RCCL
        exchange (two all-to-alls per step over xGMI, every rank a sender), the node-shared
        account registry (/dev/shm) and the step clock, driven by the rank's serving core
      * ``--threads`` ingress threads call ``core.score_batch(request bytes)``: each request is
        a serialized risk.v1 ScoreBatchRequest of ``--requests`` transactions on UUID account
        ids spread over every owner; the response is the serialized ScoreBatchResponse with a
        FeatureVector per transaction (nothing skipped: parse, resolve, routing, feature
        assembly + store update, trees, MLP, ensemble, results back, serialization)

    A step = ``--rounds`` ScoreBatch requests per ingress thread (threads x rounds requests per
    rank; K steps timed, W untimed first); the value is the whole job's transactions per second,
    the latency the per-request bytes-in -> bytes-out time (it includes the micro-batch queueing
    inside the core)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import threading
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import bench_e2e
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.layouts import ACCTBATCH
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0, make_population

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IGP_BENCH_BACKEND=cpu: the same serving objects on CPU shards (protocol rehearsal without a GPU)
    kind = os.environ.get("IGP_BENCH_BACKEND", "gpu")
    if kind == "gpu":
        local = gpu_index(local)
        torch.cuda.set_device(local)

    def sync():
        if kind == "gpu":
            torch.cuda.synchronize(local)
    comm = None
    # IGP_BENCH_SPMD=1: the multi-GPU serving objects (SpmdNode: owner-routed RCCL exchange,
    # node-shared registry, step clock) at world 1 too - the N = 1 point of the exchange path
    spmd = world > 1 or os.environ.get("IGP_BENCH_SPMD") == "1"
    if spmd:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 1000))
        # the control plane (shm names, barriers, RCCL unique ids, result reduce) runs over gloo;
        # the hot path moves rows over the exchange's own RCCL communicators
        dist.init_process_group("gloo", **({} if world > 1 else dict(rank=0, world_size=1)))
        from igaming_platform_amd.parallel.comm import TorchComm
        comm = TorchComm("gloo")
    if a.config not in benchkit.CONFIGS or benchkit.CONFIGS[a.config]["model"] == "heuristic":
        raise SystemExit("serving scope: a fraud model config (cfg1 / cfg2 / cfg3)")
    c = benchkit.CONFIGS[a.config]
    B = a.requests or a.batch or c["batch"]
    cfg = Config()
    cfg.features.width = c["width"]
    cfg.features.sum_mode = a.sum_mode
    cfg.fraud_model.precision = a.numerics
    cfg.gpu.buckets = sorted({64, 512, 2048, B})
    cfg.gpu.max_batch = B
    cfg.gpu.serve_depth = a.depth
    cfg.gpu.spmd_heartbeat_s = 0.0
    n_acc = a.accounts
    fm = builders.build(c["model"]).SerializeToString()
    if not spmd:
        from igaming_platform_amd.engine.risk_engine import RiskEngine
        eng = RiskEngine(cfg, backend=kind, capacity=n_acc + 4096, fraud_model=fm)
        core, registry, backend = eng.core, eng.registry, eng.backends[0]
        mode = "native serving core over the single-GPU three-stream pipeline"
    else:
        from igaming_platform_amd.engine.risk_engine import SpmdNode, _load_onnx
        from igaming_platform_amd.features.tables import Blacklist, IPIntel
        node = SpmdNode(cfg, comm, kind, n_acc + 4096, _load_onnx(fm), "onnx",
                        Blacklist(cfg.gpu.blacklist_capacity), IPIntel(cfg.gpu.blacklist_capacity))
        core, registry, backend = node.core, node.registry, node.local
        from igaming_platform_amd.engine.dp import rows_mode
        rows_shm = node.results_mode == "d2h" and rows_mode() == "shm"
        mode = ("native serving core per rank, owner-routed exchange (every rank ingests): rows "
                + ("through the node-shared pinned rows region" if rows_shm else "over an RCCL all-to-all")
                + ", results " + ("written by each owner into node-shared pinned memory" if node.results_mode == "d2h"
                                  else "over the result all-to-all"))
    if core is None:
        raise RuntimeError("no native serving core (IGP native driver disabled?)")
    # this rank's accounts: the global population is world x n_acc UUIDs; a rank loads the
    # warehouse rows of the accounts it owns (owner = XXH64(id) % world)
    pop = make_population(n_acc, c["width"] - 30, seed=3, fast_hash=True)
    total = n_acc * world
    from igaming_platform_amd.native import native
    from igaming_platform_amd.utils.hashing import SEED_ACCOUNT
    step = 1 << 17
    for s0 in range(0, total, step):
        ids = [bench_e2e.account_id(i) for i in range(s0, min(total, s0 + step))]
        h = native().id_hashes(ids, SEED_ACCOUNT)
        mine = np.nonzero((h % np.uint64(world)).astype(np.int64) == rank)[0]
        if not len(mine):
            continue
        sel = [ids[i] for i in mine]
        slots, _ = registry.resolve_ids(sel, insert=True)
        rows = np.asarray(pop.batch[(s0 + mine) % n_acc], ACCTBATCH)
        ok = slots >= 0
        backend.set_batch_rows(slots[ok], rows[ok])
        if c["width"] > 30:
            backend.set_ext(slots[ok], pop.ext[(s0 + mine)[ok] % n_acc])
    # the request stream covers the population (6 replayed payloads kept 4.7 % of the
    # accounts hot): --payloads distinct requests, account ids uniform (default) or Zipf(--zipf)
    spread = {}
    payloads = bench_e2e.spread_payloads(total, a.payloads, B, seed=11 + rank, zipf=a.zipf, stats=spread)
    lat = []
    stage_rows = []  # per request: parse, resolve, queue, device, serialize, total (ns)
    lock = threading.Lock()
    timings = type(core).last_timings

    def run(n_req: int, t_base: int, record: bool):
        counter = {"i": 0}

        def worker():
            while True:
                with lock:
                    i = counter["i"]
                    if i >= n_req:
                        return
                    counter["i"] = i + 1
                t0 = time.perf_counter_ns()
                out = core.score_batch(payloads[i % len(payloads)], t_base + i // 50, t0)
                dt = (time.perf_counter_ns() - t0) / 1e6
                tm = timings()
                if len(out) < B:
                    raise RuntimeError("short response")
                if record:
                    with lock:
                        lat.append(dt)
                        stage_rows.append(tm[:6])
        th = [threading.Thread(target=worker) for _ in range(a.threads)]
        [t.start() for t in th]
        [t.join() for t in th]

    def barrier():
        if comm is not None:
            comm.barrier()

    # a serving step = --rounds rounds of ScoreBatch requests, one per ingress thread per round
    # (16 concurrent 8192-transaction requests per rank per round): timing single requests (the
    # driver's --steps 20) would measure the threads' ramp up and down, and one round per step
    # made the driver's timed window ~32 ms
    per_step = a.threads * max(1, a.rounds)
    run(max(a.warmup, 1) * per_step, NOW0 - 3600, False)   # history + warm graphs / caches
    barrier()
    sync()
    core.stats(True)
    if spmd:  # the exchange driver's wait counters: the timed run only
        xd0 = getattr(getattr(getattr(node, "local", None), "scorer", None), "xdriver", None)
        if xd0 is not None:
            xd0.stats()
    # IGP_BENCH_THREADS_OUT=<path>: per-thread CPU time over the timed run (rank 0; thread names
    # from csrc/runtime/thread_name.h) - which host thread, if any, is saturated
    threads_out = os.environ.get("IGP_BENCH_THREADS_OUT") if rank == 0 else None
    if threads_out:
        import host_profile
        cpu0, proc0 = host_profile.thread_cpu(), os.times()
        if os.environ.get("IGP_BENCH_SAMPLE") == "1":  # + the hottest functions per thread name
            from igaming_platform_amd.native import native as _nat
            _nat().sampler_start(4000, 1 << 21)
    t0 = time.perf_counter()
    run(a.steps * per_step, NOW0, True)
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if threads_out:
        samples = None
        if os.environ.get("IGP_BENCH_SAMPLE") == "1":
            from igaming_platform_amd.native import native as _nat
            samples = _nat().sampler_stop()
        cpu1, proc1 = host_profile.thread_cpu(), os.times()
        busy, alive = {}, 0.0
        for tid, (name, cpu) in cpu1.items():
            d = cpu - cpu0.get(tid, (name, 0.0))[1]
            alive += d
            if d > 0:
                busy.setdefault(name, []).append(round(d / elapsed, 3))
        # the ingress threads exit with run(): their share is the process total minus the rest
        total = (proc1.user + proc1.system) - (proc0.user + proc0.system)
        with open(threads_out, "w") as f:
            json.dump({"elapsed_s": elapsed, "cpu_fraction_by_thread_name": busy,
                       "ingress_threads_cores": round(max(0.0, total - alive) / elapsed, 2),
                       "process_cores": round(total / elapsed, 2),
                       "hot": _hot_by_thread(samples, cpu1) if samples is not None else None}, f)
    st = core.stats(True)
    rows = max(int(st["rows"]), 1)
    stages = {k[:-3] + "_ns_per_row": round(st[k] / rows, 1)
              for k in ("parse_ns", "resolve_ns", "pack_ns", "submit_ns", "copy_ns", "serialize_ns")}
    stages.update(device_us_per_step=round(st["device_ns"] / max(int(st["steps"]), 1) / 1e3, 1),
                  device_steps=int(st["steps"]), empty_steps=int(st["empty_steps"]),
                  mean_rows_per_device_step=round(st["rows"] / max(int(st["steps"]), 1), 1))
    # a step slot's cycle and the stepper's waits with rows queued (serve_core.h ServeStats)
    stages.update({k[:-3] + "_us_per_step": round(st[k] / max(int(st["steps"]), 1) / 1e3, 1)
                   for k in ("release_ns", "slot_wait_ns", "rows_wait_ns", "pack_ns", "submit_ns") if k in st})
    if st.get("slot_waits"):
        stages.update(slot_waits_per_step=round(st["slot_waits"] / max(int(st["steps"]), 1), 2),
                      inflight_at_slot_wait=round(st["slot_wait_inflight"] / st["slot_waits"], 2))
    p99, p50 = float(np.percentile(lat, 99)), float(np.percentile(lat, 50))
    # where a request's time goes, per request (tails, not sums): queue = enqueue -> its first
    # device step formed, device = that step formed -> all its rows back
    sr = np.asarray(stage_rows, np.float64) / 1e6
    stage_tails = {name: {"p50": round(float(np.percentile(sr[:, k], 50)), 3),
                          "p99": round(float(np.percentile(sr[:, k], 99)), 3)}
                   for k, name in enumerate(("parse", "resolve", "queue", "device", "serialize", "total"))}
    if comm is not None:  # the slowest rank's clock and latencies
        mx = torch.tensor([elapsed, p99, p50], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed, p99, p50 = (float(x) for x in mx)
    out = {
        "metric": "fraud scores/sec (whole node) + p99 score latency",
        "value": world * a.steps * per_step * B / elapsed, "unit": "scores/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.numerics, "data": "synthetic (UUID account ids, random-init weights)",
        "config": {"model": c["desc"], "global_batch": B * per_step * world, "seq_len": 1, "parallelism": f"dp{world}",
                   "per_gpu_batch": B, "transactions_per_request": B, "requests_per_step_per_rank": per_step,
                   "step": f"{max(1, a.rounds)} rounds of one 8192-transaction ScoreBatch request per ingress thread "
                           "(concurrent); device micro-batches of per_gpu_batch rows",
                   "synthetic_clock": "request i of a run is scored at NOW0 + i // 50 (s)",
                   "accounts_per_gpu": n_acc,
                   "ingress_threads_per_rank": a.threads, "pipeline_depth": a.depth, "serving": mode,
                   "account_spread": {"distribution": f"zipf({a.zipf})" if a.zipf > 1 else "uniform",
                                      "population": total, "requests_in_stream_per_rank": a.payloads,
                                      "distinct_accounts_in_stream_rank0": spread.get("distinct_accounts"),
                                      "transactions_in_stream_per_rank": spread.get("transactions")},
                   "numerics": numerics_desc(a), "sum_mode": a.sum_mode,
                   "comm_env": {k: v for k, v in sorted(os.environ.items())
                                if k.startswith(("NCCL_", "RCCL_")) or k == "GPU_MAX_HW_QUEUES"}},
        "scope": "serving (risk.v1 ScoreBatch bytes in -> bytes out, in-process, every rank ingesting)",
        "p99_latency_ms": p99, "p50_latency_ms": p50, "latency_what": "per ScoreBatch request, bytes in -> bytes "
        "out, including the serving core's micro-batch queueing",
        "latency_baseline_ms": BASELINE_P99_MS, "latency_vs_baseline": BASELINE_P99_MS / p99 if p99 > 0 else None,
        "host_stages_rank0": stages,
        "request_stage_ms_rank0": stage_tails,
    }
    if spmd:  # the exchange driver's host waits per step (mean / worst): senders' rows, owners' results
        xd = getattr(getattr(getattr(node, "local", None), "scorer", None), "xdriver", None)
        if xd is not None:
            out["exchange_waits_us_rank0"] = {k: round(float(v), 1) for k, v in xd.stats().items()}
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if spmd:
        node.core.stop()
        if world == 1:
            node.close()  # (N > 1: the communicators go with the processes; no teardown to wait on)
        dist.destroy_process_group()
    else:
        eng.close()


def _emit(a, world: int, rank: int, out: dict) -> None:
    import torch.distributed as dist
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def model_bench(a, world: int, rank: int, dev) -> None:
    """cfg4 (LTV MLP) / cfg5 (bonus-abuse GRU): the same timing contract as the headline."""
    import torch
    import torch.distributed as dist
    from igaming_platform_amd.utils import benchkit
    if world > 1 and not a.no_gather:
        # the results are all-gathered from the device output buffers: keep the LTV rows there
        # (IGP_LTV_HOST_OUT=1, the 1-GPU default, writes them straight to pinned host memory)
        os.environ["IGP_LTV_HOST_OUT"] = "0"
    S = benchkit.build_model(a.config, a.batch, a.accounts, dev, rank=rank, depth=a.depth,
                             use_graphs=not a.no_graphs, precision=a.numerics)
    R, B = S.runner, S.batch
    out_w = R.out[:B].numel()
    gathered = torch.zeros(world * out_w, dtype=torch.float32, device=dev) if world > 1 else None

    def step(i: int):
        p = R.submit(S.pool[i % len(S.pool)])
        if world > 1 and not a.no_gather:
            st = R.slot_stream(p[0]) if hasattr(R, "slot_stream") else R.stream
            ob = R.slot_out(p[0]) if hasattr(R, "slot_out") else R.out
            with torch.cuda.stream(st):
                dist.all_gather_into_tensor(gathered, ob[:B].reshape(-1))
                p[2].record(st)
        return p

    inflight, lat = [], []
    for i in range(a.warmup):
        inflight.append((step(i), time.perf_counter()))
        if len(inflight) >= a.depth:
            R.wait(inflight.pop(0)[0])
    for p, _ in inflight:
        R.wait(p)
    inflight = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        inflight.append((step(a.warmup + i), time.perf_counter()))
        if len(inflight) >= a.depth:
            p, ts = inflight.pop(0)
            R.wait(p)
            lat.append((time.perf_counter() - ts) * 1e3)
    for p, ts in inflight:
        R.wait(p)
        lat.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = torch.tensor([elapsed, float(np.percentile(lat, 99)), float(np.percentile(lat, 50))],
                         dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed, p99, p50 = (float(x) for x in stats.cpu())
    out = {
        "metric": S.metric, "value": world * B * a.steps / elapsed, "unit": S.unit, "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.numerics, "data": "synthetic",
        "config": {"model": S.desc, "global_batch": B * world, "seq_len": 100 if a.config == "cfg5" else 1,
                   "parallelism": f"dp{world}", "per_gpu_batch": B, "accounts_per_gpu": a.accounts,
                   "pipeline_depth": a.depth, "graphs": not a.no_graphs,
                   "numerics": numerics_desc(a)},
        "p99_latency_ms": p99, "p50_latency_ms": p50,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
