"""Risk service binary: ``python -m igaming_platform_amd.serve [--config cfg.yaml] [--backend auto]``.

Mirrors services/risk/cmd/main.go:72-258: env config (same names), JSON logging, engine
construction, gRPC server (risk.v1 + health + reflection, interceptors), HTTP endpoints,
the hourly batch-feature refresh ticker (a stub in the reference; here it reloads a
warehouse snapshot file when one is configured), periodic feature-store snapshots, and a
graceful shutdown on SIGINT/SIGTERM (health -> NOT_SERVING, 30 s grace).

``--synthetic-model gbdt|stacked|logistic`` generates a random-init ONNX fraud model (no
network / no checkpoints in this environment).
"""
from __future__ import annotations

import argparse
import os
import signal
import threading
import time

from .config import Config
from .obs.logging import setup_logger


def _fraud_model(a, cfg: Config):
    if not a.synthetic_model:
        return None
    from .onnx import builders
    kw = {"n_features": cfg.features.width} if a.synthetic_model == "logistic" else {}
    return builders.build(a.synthetic_model, **kw).SerializeToString()


def build_engine(a, cfg: Config, comm=None):
    from .engine.risk_engine import RiskEngine
    return RiskEngine(cfg, backend=a.backend, fraud_model=_fraud_model(a, cfg), capacity=a.accounts or None,
                      shards=a.shards, spmd=comm)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="MI355X risk scoring service (risk.v1)")
    ap.add_argument("--config", default=os.environ.get("CONFIG_PATH", ""))
    ap.add_argument("--backend", default="auto", choices=["auto", "gpu", "cpu"])
    ap.add_argument("--gpus", type=int, default=0, help="GPU shards (default: config / RISK_GPUS)")
    ap.add_argument("--shards", type=int, default=1, help="CPU shards (backend=cpu)")
    ap.add_argument("--accounts", type=int, default=0, help="feature-store accounts per shard")
    ap.add_argument("--synthetic-model", default="", choices=["", "gbdt", "stacked", "logistic"])
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--snapshot-dir", default=os.environ.get("RISK_SNAPSHOT_DIR", ""))
    ap.add_argument("--snapshot-every-s", type=float, default=300.0)
    ap.add_argument("--no-batching", action="store_true")
    ap.add_argument("--internal-port-offset", type=int, default=1000,
                    help="multi-GPU: rank 0 also listens on grpc_port + this for the cold RPCs the other "
                         "ranks forward")
    ap.add_argument("--grpc-server", default=os.environ.get("RISK_GRPC_SERVER", "native"), choices=["native", "aio"],
                    help="native: the C++ HTTP/2 server owns the public port (unary RPCs, ScoreTransaction "
                         "straight into the serving core) and the grpc.aio server serves streaming / "
                         "reflection on grpc_port + --internal-port-offset; aio: grpc.aio on the public port")
    ap.add_argument("--grpc-workers", type=int, default=4, help="native server: epoll worker threads")
    ap.add_argument("--audit-flush-every-s", type=float, default=2.0,
                    help="drain the risk_scores / ltv_predictions rings into AUDIT_DB this often")
    a = ap.parse_args(argv)
    # HIP multiplexes streams onto GPU_MAX_HW_QUEUES hardware queues (default 4): the scorer's
    # copy / state / model streams, the exchange's two RCCL streams and the default stream each
    # get a queue of their own with 8 (must be set before the HIP runtime initialises)
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    cfg = Config.load(a.config or None)
    if a.snapshot_dir:
        cfg.gpu.snapshot_dir = a.snapshot_dir  # failed shards are re-homed from here
    if a.gpus:
        cfg.gpu.devices = a.gpus
    log = setup_logger(cfg.server.log_level)
    comm = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # one process per GPU (torchrun): every rank serves the hot RPCs through its own core;
        # rank 0 also runs the control plane and the cold RPCs
        import torch
        from .parallel.comm import init_from_env
        backend = a.backend if a.backend != "auto" else ("gpu" if torch.cuda.is_available() else "cpu")
        a.backend = backend
        if backend == "gpu":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        # control plane over gloo (deadlines / heartbeats that fail without taking rank 0
        # down); GPU shards move their rows over RCCL communicators of their own
        comm = init_from_env("gloo")
        if comm.rank != 0:
            # every rank ingests: this rank's own risk.v1 listener (same port, SO_REUSEPORT)
            # serves ScoreBatch / ScoreTransaction through its serving core and forwards the
            # cold RPCs to rank 0's internal port
            from .api.grpc_server import IngressServer
            from .engine.risk_engine import serve_shard

            nodes = []

            def listen(node):
                nodes.append(node)
                node.start_audit_flusher(a.audit_flush_every_s, log)  # AUDIT_DB: this rank's rows
                up = f"127.0.0.1:{cfg.server.grpc_port + a.internal_port_offset}"
                if a.grpc_server == "native":
                    from .api.native_grpc import NativeIngressServer
                    return NativeIngressServer(node, up, port=cfg.server.grpc_port, host=a.host,
                                               workers=a.grpc_workers).start()
                return IngressServer(node, up, port=cfg.server.grpc_port, host=a.host).start()
            n, rows = serve_shard(cfg, comm, backend=backend, capacity=a.accounts or None,
                                  fraud_model=_fraud_model(a, cfg), on_node=listen)
            for node in nodes:
                node.stop_audit_flusher()
            log.info("shard worker stopped", extra={"fields": dict(rank=comm.rank, ops=n, rows_scored=rows)})
            return 0
    from .api.grpc_server import RiskServer
    from .api.http_server import HttpServer
    eng = build_engine(a, cfg, comm)
    if a.snapshot_dir and os.path.exists(os.path.join(a.snapshot_dir, "registry.json")):
        n = eng.restore(a.snapshot_dir)
        log.info("feature store restored", extra={"fields": dict(accounts=n, dir=a.snapshot_dir)})
    multi = comm is not None and comm.world > 1
    internal = cfg.server.grpc_port + a.internal_port_offset
    ngs = None
    if a.grpc_server == "native":
        # public port: the native server (every rank, SO_REUSEPORT); the grpc.aio server keeps
        # the streaming RPCs (health Watch, reflection) and the worker ranks' forwarded cold RPCs
        from .api.native_grpc import NativeRiskServer
        ngs = NativeRiskServer(eng, port=cfg.server.grpc_port, host=a.host, workers=a.grpc_workers,
                               batching=not a.no_batching).start()
        gs = RiskServer(eng, port=internal, host=a.host, batching=not a.no_batching).start()
    else:
        gs = RiskServer(eng, port=cfg.server.grpc_port, host=a.host, batching=not a.no_batching, reuseport=multi,
                        extra_ports=[internal] if multi else ()).start()
    hs = HttpServer(eng, port=cfg.server.http_port, host=a.host, timeout_s=cfg.server.http_timeout_s).start()
    stop = threading.Event()

    def _sig(signum, frame):
        log.info("shutdown signal", extra={"fields": dict(signal=signum)})
        stop.set()

    signal.signal(signal.SIGINT, _sig)
    signal.signal(signal.SIGTERM, _sig)
    from .engine.audit import flush_if_configured
    last_snap = last_flush = time.time()
    while not stop.wait(1.0):
        if a.snapshot_dir and time.time() - last_snap >= a.snapshot_every_s:
            eng.snapshot(a.snapshot_dir)
            last_snap = time.time()
        if time.time() - last_flush >= a.audit_flush_every_s:  # AUDIT_DB set: drain the audit rings
            flush_if_configured(eng, log)
            last_flush = time.time()
    if ngs is not None:
        ngs.stop()
    gs.stop(cfg.server.shutdown_grace_s)
    hs.stop()
    flush_if_configured(eng, log)  # rows scored during the grace period
    if a.snapshot_dir:
        eng.snapshot(a.snapshot_dir)
    eng.close()
    log.info("server stopped")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
