"""risk.v1 on the native HTTP/2 gRPC server (csrc/runtime/h2grpc.cpp).

The Python ``grpc.aio`` server (api/grpc_server.py) pays its own per-call cost (~100 us of
Python per unary call) and saturated near 9 k unary ScoreTransaction calls/s
(``profiles/r3/grpc_unary_open_loop_curve.json``). Here the transport is C++ (libnghttp2 through
dlopen, one epoll loop per worker thread, SO_REUSEPORT listeners):

* ScoreTransaction goes from the HTTP/2 DATA frame straight into the engine's serving core
  (C++ parse, AccountIndex, micro-batch FIFO) and back - no Python, no GIL;
* ScoreBatch runs ``ServeCore.score_batch`` on native batch threads;
* PredictLTV, GetPlayerSegment and CheckBonusAbuse go to the engine's native account router
  (engine/acct.py, csrc/runtime/acct_core.cpp): C++ parse, owner routing, micro-batches on the
  LTV chain / abuse step of the owner's GPU, response bytes written in C++ - no Python;
* every other unary RPC (blacklist, features, thresholds, grpc.health.v1 Check) - and the three
  above while the router is absent - calls the same :class:`RiskServicer` handlers as the Python
  server, bytes in / bytes out, on native cold threads that take the GIL.

A hot call that fails inside a native core (device error, step deadline) comes back through
the cold table with its path suffixed ``#retry:<error>``: the engine marks the shard unhealthy
(or fails the SPMD group over), so this call and the later ones are answered by the Python
path and its fallback, and the watcher turns the hot flag off.

While the engine must not take the native path (degraded shard, fault injection, audit-less
fallback...) a watcher flips the server's hot flag and the scoring RPCs go through the
engine's Python path instead (same semantics as :class:`grpc_server.NativeUnary`).
Streaming RPCs (health Watch, reflection) stay on the Python server; ``serve.py`` runs that one
on an internal port when the native server owns the public port.
Reference: services/risk/cmd/main.go:72-258 (the risk.v1 server), proto/risk/v1/risk.proto.
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Dict, Optional

import grpc

from ..native import native
from ..obs.logging import get_logger
from ..proto import health_v1 as HV
from ..proto import risk_v1 as P
from .batcher import MicroBatcher
from .grpc_server import HealthServicer, InvalidArgument, RAW, RiskServicer

log = get_logger("igaming_platform_amd.native_grpc")

OK, INVALID_ARGUMENT, INTERNAL, UNIMPLEMENTED = 0, 3, 13, 12


class NativeRiskServer:
    def __init__(self, engine, port: int = 0, host: str = "127.0.0.1", workers: int = 4, cold_threads: int = 4,
                 batch_threads: int = 8, batching: bool = True):
        self.engine = engine
        cfg = engine.cfg
        self.ltv_batcher = self.abuse_batcher = None
        if batching:
            wait = cfg.gpu.wait_us
            self.ltv_batcher = MicroBatcher(lambda ids, _t: engine.predict_ltv_batch(ids), 4096, wait, workers=1)
            self.abuse_batcher = MicroBatcher(lambda ids, _t: engine.check_bonus_abuse_batch(ids), 4096, wait,
                                              workers=1)
        self.health = HealthServicer()
        self.health.set(P.SERVICE, "SERVING")
        self._servicer = RiskServicer(engine, None, self.ltv_batcher, self.abuse_batcher)
        self._table = self._handlers()
        self._host, self._port_req, self._workers = host, port, workers
        core = getattr(engine, "core", None)
        acct = getattr(engine, "acct", None)
        self.srv = native().GrpcServer(core, self._cold, int(cold_threads), int(batch_threads if core is not None else 0),
                                       acct=acct.router if acct is not None else None)
        self.port = 0
        self._stop = threading.Event()
        self._watch: Optional[threading.Thread] = None
        self._seen = dict(hot_tx=0, hot_batch=0, hot_acct=0)

    # ------------------------------------------------------------------ cold handler table
    def _handlers(self) -> Dict[str, Callable[[bytes], bytes]]:
        s, e = self._servicer, self.engine
        table: Dict[str, Callable[[bytes], bytes]] = {}
        for rpc, req_name, _resp in P.METHODS:
            path = f"/{P.SERVICE}/{rpc}"
            if rpc in RAW:
                # the engine's Python path (the native path is off or the core is absent)
                table[path] = (lambda body, _e=e: _e.score_tx_bytes(body)) if rpc == "ScoreTransaction" else \
                    (lambda body, _e=e: _e.score_batch_bytes(body))
            else:
                fn, req_cls = getattr(s, rpc), P.M[req_name]
                table[path] = (lambda body, _f=fn, _c=req_cls: _f(_c.FromString(body), None).SerializeToString())
        hs = self.health
        table[f"/{HV.SERVICE}/Check"] = lambda body: hs.Check(HV.HealthCheckRequest.FromString(body), _Ctx()) \
            .SerializeToString()
        return table

    def _cold(self, path: str, body: bytes):
        if "#cold:" in path:  # no native core serves this call (owner without one, or stopping): no failover
            path = path.split("#cold:", 1)[0]
        elif "#retry:" in path:  # a hot call the native path failed: fail the shard over, then serve it here
            path, msg = path.split("#retry:", 1)
            try:
                self.engine.on_core_failure(msg)
            except Exception:
                log.error("core failure handling", exc_info=True)
        f = self._table.get(path)
        short = path.rsplit("/", 1)[-1]
        m = self.engine.metrics
        t0 = time.perf_counter()
        code = "OK"
        try:
            if f is None:
                code = "UNIMPLEMENTED"
                return UNIMPLEMENTED, f"method {path} is not served on this port"
            return f(body)
        except InvalidArgument as e:
            code = "INVALID_ARGUMENT"
            return INVALID_ARGUMENT, str(e)
        except _Abort as e:
            code = e.code_name
            return e.code, e.details
        except Exception:
            code = "INTERNAL"
            log.error("panic recovered", exc_info=True, extra={"fields": dict(method=path)})
            return INTERNAL, "internal server error"
        finally:
            m.requests.labels(method=short, code=code).inc()
            m.latency.labels(method=short).observe(time.perf_counter() - t0)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "NativeRiskServer":
        self.port = int(self.srv.start(self._host, int(self._port_req), int(self._workers)))
        self._watch = threading.Thread(target=self._watch_loop, name="native-grpc-watch", daemon=True)
        self._watch.start()
        log.info("native grpc server listening", extra={"fields": dict(port=self.port, workers=self._workers)})
        return self

    def _watch_loop(self) -> None:
        """Hot flag from the engine's state + the native calls into /metrics, every 100 ms."""
        e, m = self.engine, self.engine.metrics
        while not self._stop.wait(0.1):
            try:
                self.srv.set_hot(bool(e._native_ok()))
                st = self.srv.stats()
                for k, method in (("hot_tx", "ScoreTransaction"), ("hot_batch", "ScoreBatch"),
                                  ("hot_acct", "AccountRPC")):
                    d = int(st[k]) - self._seen[k]
                    if d > 0:
                        m.requests.labels(method=method, code="OK").inc(d)
                        self._seen[k] = int(st[k])
            except Exception:  # never let the watcher die
                log.error("native grpc watcher", exc_info=True)

    def stats(self) -> dict:
        return dict(self.srv.stats())

    def stop(self, grace: float = 5.0) -> None:
        self.health.set("", "NOT_SERVING")
        self.health.set(P.SERVICE, "NOT_SERVING")
        self._stop.set()
        if self._watch is not None:
            self._watch.join(timeout=2)
        self.srv.stop()
        for b in (self.ltv_batcher, self.abuse_batcher):
            if b is not None:
                b.close()


class _Abort(Exception):
    def __init__(self, code: int, code_name: str, details: str):
        super().__init__(details)
        self.code, self.code_name, self.details = code, code_name, details


class _Ctx:
    """The slice of grpc.ServicerContext the unary handlers use (health Check aborts with
    NOT_FOUND for an unknown service)."""

    def abort(self, code, details):
        raise _Abort(int(code.value[0]), code.name, details)

    def set_code(self, code):
        pass

    def set_details(self, details):
        pass


class NativeIngressServer:
    """The native server on a worker rank (>= 1) of a multi-GPU group (cf.
    :class:`grpc_server.IngressServer`): ScoreTransaction / ScoreBatch through THIS rank's
    serving core, every other unary RPC forwarded byte-for-byte to rank 0's internal port."""

    def __init__(self, node, upstream: str, port: int, host: str = "0.0.0.0", workers: int = 4):
        # PredictLTV / GetPlayerSegment / CheckBonusAbuse: this rank's native account router
        # (owner-routed over /dev/shm); the rest of the cold RPCs go to rank 0
        opts = [("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)]
        self._up = grpc.insecure_channel(upstream, options=opts)
        self.upstream = upstream
        self.health = HealthServicer()
        self.health.set(P.SERVICE, "SERVING")
        self._calls: Dict[str, Callable] = {}
        self._host, self._port_req, self._workers = host, port, workers
        acct = getattr(node, "acct", None)
        self.srv = native().GrpcServer(node.core, self._cold, 4, 8, acct=acct.router if acct is not None else None)
        self.port = 0

    def _cold(self, path: str, body: bytes):
        path = path.split("#retry:", 1)[0]  # a failed hot call: rank 0 answers it on its Python path
        if path == f"/{HV.SERVICE}/Check":
            try:
                return self.health.Check(HV.HealthCheckRequest.FromString(body), _Ctx()).SerializeToString()
            except _Abort as e:
                return e.code, e.details
        f = self._calls.get(path)
        if f is None:
            f = self._calls[path] = self._up.unary_unary(path)
        try:
            return f(body, timeout=30)  # rank 0 answers the cold RPC
        except grpc.RpcError as e:
            return int(e.code().value[0]), e.details() or ""

    def start(self) -> "NativeIngressServer":
        self.port = int(self.srv.start(self._host, int(self._port_req), int(self._workers)))
        log.info("ingress grpc server listening", extra={"fields": dict(port=self.port, upstream=self.upstream,
                                                                          server="native")})
        return self

    def stop(self, grace: float = 5.0) -> None:
        self.health.set(P.SERVICE, "NOT_SERVING")
        self.srv.stop()
        self._up.close()
