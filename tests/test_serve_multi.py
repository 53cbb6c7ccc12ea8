"""The service binary with two ranks (torchrun, CPU shards): every rank listens on the same
risk.v1 port (SO_REUSEPORT) and answers ScoreBatch / ScoreTransaction through its own serving
core; cold RPCs reaching rank 1 are forwarded to rank 0. Reference: the risk service binary
services/risk/cmd/main.go:72-258 (one process, handler never registered)."""
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.dist
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_every_rank_serves_risk_v1_on_one_port():
    import grpc
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_e2e
    from igaming_platform_amd.proto import risk_v1 as P
    port, http, master = _free_port(), _free_port(), _free_port()
    env = dict(os.environ, GRPC_PORT=str(port), HTTP_PORT=str(http), PYTHONPATH=ROOT, RISK_SPMD_OP_TIMEOUT_S="20")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(master), "-m", "igaming_platform_amd.serve",
           "--backend", "cpu", "--accounts", "4096", "--host", "127.0.0.1", "--internal-port-offset", "7"]
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            start_new_session=True)
    try:
        t_end = time.time() + 120
        while time.time() < t_end:
            try:
                ch = grpc.insecure_channel(f"127.0.0.1:{port}")
                grpc.channel_ready_future(ch).result(timeout=1)
                ch.close()
                break
            except Exception:
                time.sleep(0.5)
        else:
            pytest.fail("server never listened")
        time.sleep(2.0)  # both ranks bound
        seen = 0
        for i in range(10):  # a new connection each time: the kernel spreads them over the ranks
            ch = grpc.insecure_channel(f"127.0.0.1:{port}")
            body = bench_e2e.make_payloads(1000, 1, 64, seed=i)[0]
            r = P.ScoreBatchResponse.FromString(ch.unary_unary(P.method_path("ScoreBatch"))(body, timeout=30))
            assert len(r.results) == 64 and all(1 <= x.action <= 3 for x in r.results)
            t = P.GetThresholdsResponse.FromString(ch.unary_unary(P.method_path("GetThresholds"))(b"", timeout=30))
            assert (t.block_threshold, t.review_threshold) == (80, 50)
            tx = P.ScoreTransactionResponse.FromString(
                ch.unary_unary(P.method_path("ScoreTransaction"))(bench_e2e.tx_payloads(1000, 1, seed=i)[0], timeout=30))
            assert 1 <= tx.action <= 3
            seen += 1
            ch.close()
        assert seen == 10
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            out, _ = proc.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            out, _ = proc.communicate()
    log = out.decode(errors="replace")
    assert "ingress grpc server listening" in log, log[-3000:]
