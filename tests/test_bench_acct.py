"""The cfg4 / cfg5 serving bench's owner-routed DP mode rehearsed on CPU shards (VERDICT r4
item 6): ``bench.py --config cfg5|cfg4 --gpus N --scope serving`` with IGP_BENCH_BACKEND=cpu runs
every rank's native AcctRouter; each rank ingests CheckBonusAbuse / PredictLTV bytes for account
ids spread over all owners and the /dev/shm mailbox carries each call to its owner. After the
timed run every rank answers the same fixed calls; at world 2 and 3 every rank's answers equal the
world-1 run (the single-process engine) byte for byte (PredictLTV's wall-clock stamp aside).

Reference: /root/reference/services/bonus/internal/service/bonus_engine.go:268-275 (CheckBonusAbuse
at the bonus service), BASELINE.json config 5 (DP=8)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, config, world, population=3000, threads=1):
    out = str(tmp_path / f"{config}-w{world}")
    env = dict(os.environ, IGP_BENCH_BACKEND="cpu", IGP_BENCH_SMALL_MODELS="1", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", config,
           "--accounts", str(population // world), "--steps", "2", "--warmup", "1", "--calls", "300",
           "--inflight", "256", "--check-out", out, "--drive-threads", str(threads)]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    answers = [json.load(open(f"{out}.{k}.json"))["answers"] for k in range(world)]
    return res, answers


def _norm(config, hexes):
    from igaming_platform_amd.proto import risk_v1 as P
    out = []
    for h in hexes:
        assert h is not None and not h.startswith("error"), h
        if config == "cfg4" and h:
            m = P.PredictLTVResponse.FromString(bytes.fromhex(h))
            m.ClearField("predicted_at")
            h = m.SerializeToString().hex()
        out.append(h)
    return out


@pytest.mark.dist
@pytest.mark.parametrize("config,worlds", [("cfg5", (2, 3)), ("cfg4", (2,))])
def test_acct_dp_bench_answers_equal_single_process(tmp_path, config, worlds):
    base, (ans1,) = _run(tmp_path, config, 1)
    assert base["n_gpus"] == 1 and base["errors"] == 0 and base["value"] > 0
    want = _norm(config, ans1)
    assert len(set(want)) > 1  # the fixed calls do not all have the same answer
    for w in worlds:
        # world 2: three submitting threads per rank (answers through the router's sink)
        res, per_rank = _run(tmp_path, config, w, threads=3 if w == 2 else 1)
        assert res["n_gpus"] == w and res["errors"] == 0 and res["cold_path_calls"] == 0
        assert res["config"]["submit_threads_per_rank"] == (3 if w == 2 else 1)
        # calls of every rank crossed the mailbox to other owners
        assert res["remote_calls_rank_sum"] > 0
        assert res["config"]["parallelism"].startswith(f"dp{w}")
        for k, got in enumerate(per_rank):
            assert _norm(config, got) == want, f"world {w} rank {k} answers differ from the single process"
