"""bench.py's driver contract, rehearsed on CPU shards (IGP_BENCH_BACKEND=cpu): the serving bench
at world 1 and 2 (``--gpus 2`` relaunches itself under torch.distributed.run, one rank per shard,
every rank ingesting through its serving core and the owner-routed exchange) prints ONE JSON
line with the fields the driver reads, n_gpus = world, dp<world> parallelism and the whole-job
value (the driver runs exactly this path on GPUs at N = 1, 2, 4, 8)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
          "vs_baseline", "dtype", "data", "config")


@pytest.mark.dist
@pytest.mark.parametrize("world", [1, 2])
def test_serving_bench_contract_on_cpu_shards(tmp_path, world):
    env = dict(os.environ, IGP_BENCH_BACKEND="cpu", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = tmp_path / "bench.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--accounts", "20000", "--threads", "2", "--rounds", "2", "--requests", "512", "--payloads", "8",
           "--json-out", str(out)]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, lines  # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d == json.loads(out.read_text())
    assert all(k in d for k in FIELDS)
    assert d["n_gpus"] == world and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["parallelism"] == f"dp{world}"
    # value = the whole job's transactions per second: world x steps x requests x rows / elapsed
    per_step = d["config"]["requests_per_step_per_rank"] * d["config"]["transactions_per_request"]
    assert d["value"] == pytest.approx(world * per_step / (d["ms_per_step"] / 1e3), rel=1e-6)
