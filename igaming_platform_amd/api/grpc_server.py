"""risk.v1 gRPC server: raw-bytes generic handlers, interceptors, health, reflection.

Same service/method names and wire contract as the reference
(proto/risk/v1/risk.proto:10-32). Unlike the reference binary — which registers the
service only in a commented block (services/risk/cmd/main.go:98-142) — every RPC is served.

The two scoring RPCs never materialise per-field Python objects: the handlers receive the
request bytes (no deserializer), the C++ wire codec parses them, and the response bytes
come back from the C++ serializer. Unary ScoreTransaction goes through the micro-batcher.
Interceptors mirror the reference chain (main.go:303-353): logging (OK at debug, errors at
info), recovery (exceptions -> INTERNAL "internal server error"), metrics (the counters the
reference's no-op interceptor lists).
"""
from __future__ import annotations

import asyncio
import threading
import time
from concurrent import futures
from typing import Dict, Optional

import grpc

from ..obs.logging import get_logger
from ..proto import health_v1 as HV
from ..proto import reflection_v1 as RV
from ..proto import risk_v1 as P
from ..proto.builder import file_containing_symbol, file_descriptor_proto_bytes
from .batcher import MicroBatcher

log = get_logger("grpc")


def _ts(seconds: float):
    t = P.Timestamp()
    t.seconds = int(seconds)
    t.nanos = int((seconds - int(seconds)) * 1e9)
    return t


class InvalidArgument(ValueError):
    pass


HOT = {"ScoreTransaction", "ScoreBatch"}  # the scoring RPCs (fast metrics path)


# ============================================================================ interceptors
def _wrap_unary(h, fn_wrap):
    if h is None or h.unary_unary is None:
        return h
    return grpc.unary_unary_rpc_method_handler(fn_wrap(h.unary_unary), request_deserializer=h.request_deserializer,
                                               response_serializer=h.response_serializer)


class LoggingInterceptor(grpc.ServerInterceptor):
    """main.go:305-323: duration per call; OK at debug, errors at info."""

    def intercept_service(self, continuation, details):
        method = details.method

        def wrap(fn):
            def call(req, ctx):
                t0 = time.perf_counter()
                try:
                    return fn(req, ctx)
                finally:
                    code = ctx.code() if hasattr(ctx, "code") else None
                    fields = dict(method=method, duration_ms=round((time.perf_counter() - t0) * 1e3, 3))
                    if code not in (None, grpc.StatusCode.OK):
                        fields["code"] = str(code)
                        log.info("grpc request failed", extra={"fields": fields})
                    else:
                        log.debug("grpc request", extra={"fields": fields})
            return call
        return _wrap_unary(continuation(details), wrap)


class RecoveryInterceptor(grpc.ServerInterceptor):
    """main.go:329-342: a panic becomes codes.Internal "internal server error"."""

    def intercept_service(self, continuation, details):
        method = details.method

        def wrap(fn):
            def call(req, ctx):
                try:
                    return fn(req, ctx)
                except InvalidArgument as e:
                    ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
                except grpc.RpcError:
                    raise
                except Exception:
                    c = ctx.code() if hasattr(ctx, "code") else None
                    if c not in (None, grpc.StatusCode.OK):  # the handler already aborted with a status
                        raise
                    log.error("panic recovered", exc_info=True, extra={"fields": dict(method=method)})
                    ctx.abort(grpc.StatusCode.INTERNAL, "internal server error")
            return call
        return _wrap_unary(continuation(details), wrap)


class MetricsInterceptor(grpc.ServerInterceptor):
    """main.go:344-353 lists request count / latency / errors; they are recorded here."""

    def __init__(self, metrics):
        self.m = metrics

    def intercept_service(self, continuation, details):
        method = details.method.rsplit("/", 1)[-1]

        def wrap(fn):
            def call(req, ctx):
                t0 = time.perf_counter()
                code = "OK"
                try:
                    return fn(req, ctx)
                except BaseException:
                    code = "ERROR"
                    raise
                finally:
                    c = ctx.code() if hasattr(ctx, "code") else None
                    if c not in (None, grpc.StatusCode.OK):
                        code = c.name
                    self.m.requests.labels(method=method, code=code).inc()
                    self.m.latency.labels(method=method).observe(time.perf_counter() - t0)
            return call
        return _wrap_unary(continuation(details), wrap)


# ============================================================================ risk.v1
class RiskServicer:
    def __init__(self, engine, batcher: Optional[MicroBatcher] = None, ltv_batcher: Optional[MicroBatcher] = None,
                 abuse_batcher: Optional[MicroBatcher] = None):
        self.e = engine
        self.batcher = batcher
        # cold RPCs: concurrent unary calls merge into one batched engine call (one LTV graph /
        # one K1 feature read + one GRU launch per shard) instead of a device batch of one each
        self.ltv_batcher = ltv_batcher
        self.abuse_batcher = abuse_batcher

    def _ltv(self, account_id: str):
        if self.ltv_batcher is not None:
            return self.ltv_batcher.submit(account_id).result()
        return self.e.predict_ltv(account_id)

    def _abuse(self, account_id: str, bonus_id: str):
        if self.abuse_batcher is not None:
            return self.abuse_batcher.submit(account_id).result()
        return self.e.check_bonus_abuse(account_id, bonus_id)

    @staticmethod
    def ltv_response(req, r):
        return P.PredictLTVResponse(account_id=req.account_id, predicted_ltv=r.predicted_ltv, segment=r.segment,
                                    churn_risk=r.churn_risk, predicted_active_days=r.survival_days,
                                    confidence=r.confidence, next_best_action=r.next_best_action,
                                    predicted_at=_ts(time.time()))

    @staticmethod
    def segment_response(req, r):
        return P.GetPlayerSegmentResponse(account_id=req.account_id, segment=r.segment, ltv=r.predicted_ltv,
                                          churn_risk=r.churn_risk, recommended_actions=r.recommended_actions())

    @staticmethod
    def abuse_response(r):
        return P.CheckBonusAbuseResponse(is_abuser=r.is_abuser, abuse_score=r.abuse_score, signals=r.signals,
                                         linked_accounts=r.linked_accounts)

    # ---- scoring (raw bytes in / out)
    def ScoreTransaction(self, data: bytes, ctx) -> bytes:
        t0 = time.perf_counter()
        if self.batcher is not None:
            return self.batcher.submit(data, t0).result()
        return self.e.score_tx_bytes(data, t0)

    def ScoreBatch(self, data: bytes, ctx) -> bytes:
        return self.e.score_batch_bytes(data, time.perf_counter())

    # ---- LTV / segment
    def PredictLTV(self, req, ctx):
        if not req.account_id:
            raise InvalidArgument("account_id is required")
        return self.ltv_response(req, self._ltv(req.account_id))

    def GetPlayerSegment(self, req, ctx):
        if not req.account_id:
            raise InvalidArgument("account_id is required")
        return self.segment_response(req, self._ltv(req.account_id))

    def CheckBonusAbuse(self, req, ctx):
        if not req.account_id:
            raise InvalidArgument("account_id is required")
        return self.abuse_response(self._abuse(req.account_id, req.bonus_id))

    # ---- blacklist
    def AddToBlacklist(self, req, ctx):
        exp = req.expires_at.seconds if req.HasField("expires_at") else 0
        try:
            e = self.e.add_to_blacklist(req.type, req.value, req.reason, req.created_by, expires_at=exp)
        except ValueError as err:
            raise InvalidArgument(str(err))
        return P.AddToBlacklistResponse(success=True, id=e.id)

    def CheckBlacklist(self, req, ctx):
        ms = self.e.check_blacklist(req.device_id, req.fingerprint, req.ip_address, req.email)
        return P.CheckBlacklistResponse(
            is_blacklisted=bool(ms),
            matches=[P.BlacklistMatch(type=m.type, value=m.value, reason=m.reason, created_at=_ts(m.created_at))
                     for m in ms])

    # ---- features
    def GetFeatures(self, req, ctx):
        if not req.account_id:
            raise InvalidArgument("account_id is required")
        fv = P.FeatureVector()
        fv.ParseFromString(self.e.get_features_bytes(req.account_id))
        return P.GetFeaturesResponse(account_id=req.account_id, features=fv, computed_at=_ts(time.time()))

    # ---- thresholds (engine.go:491-504)
    def UpdateThresholds(self, req, ctx):
        try:
            b, r = self.e.update_thresholds(req.block_threshold, req.review_threshold)
        except ValueError as err:
            raise InvalidArgument(str(err))
        return P.UpdateThresholdsResponse(success=True, block_threshold=b, review_threshold=r)

    def GetThresholds(self, req, ctx):
        b, r = self.e.get_thresholds()
        return P.GetThresholdsResponse(block_threshold=b, review_threshold=r)


RAW = {"ScoreTransaction", "ScoreBatch"}


def risk_handler(servicer: RiskServicer) -> grpc.GenericRpcHandler:
    handlers = {}
    for rpc, req_name, resp_name in P.METHODS:
        fn = getattr(servicer, rpc)
        if rpc in RAW:
            handlers[rpc] = grpc.unary_unary_rpc_method_handler(fn)  # bytes in, bytes out
        else:
            handlers[rpc] = grpc.unary_unary_rpc_method_handler(
                fn, request_deserializer=P.M[req_name].FromString,
                response_serializer=lambda m: m.SerializeToString())
    return grpc.method_handlers_generic_handler(P.SERVICE, handlers)


# ============================================================================ grpc.health.v1
class HealthServicer:
    """Check + Watch; NOT_SERVING on shutdown (main.go:145-147, 249)."""

    def __init__(self):
        self._status: Dict[str, int] = {"": HV.STATUS["SERVING"]}
        self._cv = threading.Condition()

    def set(self, service: str, status: str) -> None:
        with self._cv:
            self._status[service] = HV.STATUS[status]
            self._cv.notify_all()

    def Check(self, req, ctx):
        with self._cv:
            st = self._status.get(req.service)
        if st is None:
            ctx.abort(grpc.StatusCode.NOT_FOUND, "unknown service")
        return HV.HealthCheckResponse(status=st)

    def Watch(self, req, ctx):
        last = None
        while ctx.is_active():
            with self._cv:
                st = self._status.get(req.service, HV.STATUS["SERVICE_UNKNOWN"])
                if st == last:
                    self._cv.wait(timeout=1.0)
                    continue
            last = st
            yield HV.HealthCheckResponse(status=st)


def health_handler(h: HealthServicer) -> grpc.GenericRpcHandler:
    ser = lambda m: m.SerializeToString()  # noqa: E731
    return grpc.method_handlers_generic_handler(HV.SERVICE, {
        "Check": grpc.unary_unary_rpc_method_handler(h.Check, request_deserializer=HV.HealthCheckRequest.FromString,
                                                     response_serializer=ser),
        "Watch": grpc.unary_stream_rpc_method_handler(h.Watch, request_deserializer=HV.HealthCheckRequest.FromString,
                                                      response_serializer=ser),
    })


# ============================================================================ reflection
SERVICES = [P.SERVICE, HV.SERVICE, "grpc.reflection.v1alpha.ServerReflection", "grpc.reflection.v1.ServerReflection"]


def _request_kind(data: bytes):
    """Which oneof member the reflection request carries (proto3 oneof presence on the wire)."""
    i, out = 0, {}
    while i < len(data):
        key, shift = 0, 0
        while True:
            b = data[i]; i += 1
            key |= (b & 0x7F) << shift; shift += 7
            if b < 0x80:
                break
        fno, wt = key >> 3, key & 7
        if wt == 2:
            ln, shift = 0, 0
            while True:
                b = data[i]; i += 1
                ln |= (b & 0x7F) << shift; shift += 7
                if b < 0x80:
                    break
            out[fno] = data[i:i + ln]
            i += ln
        elif wt == 0:
            while data[i] & 0x80:
                i += 1
            i += 1
        else:
            break
    return out


def reflection_handler(pkg: str) -> grpc.GenericRpcHandler:
    M = RV.M[pkg]

    def info(req_iter, ctx):
        for raw in req_iter:
            f = _request_kind(raw)
            orig = M["ServerReflectionRequest"].FromString(raw)
            resp = M["ServerReflectionResponse"](valid_host=orig.host, original_request=orig)
            try:
                if 7 in f:
                    resp.list_services_response.service.extend([M["ServiceResponse"](name=s) for s in SERVICES])
                elif 4 in f:
                    fname = file_containing_symbol(f[4].decode())
                    resp.file_descriptor_response.file_descriptor_proto.extend(_with_deps(fname))
                elif 3 in f:
                    resp.file_descriptor_response.file_descriptor_proto.extend(_with_deps(f[3].decode()))
                else:
                    resp.error_response.error_code = grpc.StatusCode.UNIMPLEMENTED.value[0]
                    resp.error_response.error_message = "not supported"
            except KeyError as e:
                resp.error_response.error_code = grpc.StatusCode.NOT_FOUND.value[0]
                resp.error_response.error_message = f"not found: {e}"
            yield resp.SerializeToString()

    return grpc.method_handlers_generic_handler(f"{pkg}.ServerReflection", {
        "ServerReflectionInfo": grpc.stream_stream_rpc_method_handler(info)})


def _with_deps(fname: str):
    from google.protobuf import descriptor_pb2
    out, seen, todo = [], set(), [fname]
    while todo:
        n = todo.pop()
        if n in seen:
            continue
        seen.add(n)
        b = file_descriptor_proto_bytes(n)
        out.append(b)
        todo.extend(descriptor_pb2.FileDescriptorProto.FromString(b).dependency)
    return out


# ============================================================================ asyncio server
class AioInterceptor(grpc.aio.ServerInterceptor):
    """The reference's interceptor chain (main.go:303-353) as one async wrapper: recovery
    (exceptions -> INTERNAL "internal server error"), metrics, logging (OK at debug, errors
    at info). The scoring RPCs' successful calls only bump plain counters
    (``Metrics.fast_rpc``): no prometheus label lookup, lock or histogram search per call."""

    def __init__(self, metrics):
        self.m = metrics

    async def intercept_service(self, continuation, details):
        h = await continuation(details)
        if h is None or h.unary_unary is None:
            return h
        inner, method = h.unary_unary, details.method
        short = method.rsplit("/", 1)[-1]
        m = self.m
        fast = m.fast_rpc(short) if short in HOT else None

        def account(code: str, dt: float) -> None:
            if code == "OK" and fast is not None:
                fast.observe(dt)
                return
            m.requests.labels(method=short, code=code).inc()
            m.latency.labels(method=short).observe(dt)
            if code != "OK":
                log.info("grpc request failed", extra={"fields": dict(method=method, code=code,
                                                                      duration_ms=round(dt * 1e3, 3))})
            elif log.isEnabledFor(10):
                log.debug("grpc request", extra={"fields": dict(method=method, duration_ms=round(dt * 1e3, 3))})

        async def call(req, ctx):
            t0 = time.perf_counter()
            code = "OK"
            try:
                return await inner(req, ctx)
            except InvalidArgument as e:
                code = "INVALID_ARGUMENT"
                await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            except grpc.aio.AbortError:
                c = ctx.code() if hasattr(ctx, "code") else None
                code = c.name if c is not None else "ABORTED"
                raise
            except Exception:
                code = "INTERNAL"
                log.error("panic recovered", exc_info=True, extra={"fields": dict(method=method)})
                await ctx.abort(grpc.StatusCode.INTERNAL, "internal server error")
            finally:
                account(code, time.perf_counter() - t0)

        return grpc.unary_unary_rpc_method_handler(call, request_deserializer=h.request_deserializer,
                                                   response_serializer=h.response_serializer)


INLINE = {"CheckBlacklist", "GetThresholds"}   # pure host work: never leaves the event loop


class NativeUnary:
    """Unary ScoreTransaction through a native serving core (engine/serving.py): the handler
    enqueues the request bytes (``core.submit_tx``: C++ parse + resolve, one row into the
    core's FIFO, where concurrent calls share device micro-batches) and awaits a future; one
    poller thread drains the core's completion queue and resolves a whole batch of futures
    with one ``call_soon_threadsafe``. No Python per-request thread, queue or lock on the hot
    path (the Python MicroBatcher is gone from ScoreTransaction)."""

    def __init__(self, core, loop, now_fn=None, ok_fn=None, fallback=None, pool=None):
        """``ok_fn() -> bool``: whether the native path may serve now (else ``fallback(bytes)``
        runs in ``pool``: the engine's Python path with its audit ring / fault injection /
        degraded-shard fallback)."""
        import itertools
        self.core, self.loop = core, loop
        self.ok_fn, self.fallback, self.pool = ok_fn, fallback, pool
        self._tags = itertools.count(1)
        self._pending: Dict[int, "asyncio.Future"] = {}
        self._stop = threading.Event()
        self.calls = 0
        self.now_fn = now_fn or (lambda: int(time.time()))
        self._th = threading.Thread(target=self._poll, name="native-unary-poll", daemon=True)
        self._th.start()

    async def call(self, data: bytes) -> bytes:
        if self.ok_fn is not None and not self.ok_fn():
            return await self.loop.run_in_executor(self.pool, self.fallback, data)
        fut = self.loop.create_future()
        tag = next(self._tags)
        self._pending[tag] = fut
        self.core.submit_tx(data, tag, self.now_fn(), time.perf_counter_ns())
        self.calls += 1
        return await fut

    def _resolve(self, items) -> None:
        for tag, body, err in items:
            fut = self._pending.pop(tag, None)
            if fut is None or fut.done():
                continue
            if err is not None:
                fut.set_exception(InvalidArgument(err) if "pb:" in err else RuntimeError(err))
            else:
                fut.set_result(body)

    def _poll(self) -> None:
        while not self._stop.is_set():
            items = self.core.poll(8192, 20000)
            if items:
                self.loop.call_soon_threadsafe(self._resolve, items)

    def close(self) -> None:
        self._stop.set()
        self._th.join(timeout=2)


def aio_risk_handler(servicer: RiskServicer, pool, inline_all: bool, native_tx: "NativeUnary" = None
                     ) -> grpc.GenericRpcHandler:
    """Async adapters over RiskServicer. Work that may wait on a GPU runs in ``pool`` so the
    event loop keeps accepting calls; on the CPU backend everything runs inline (cheapest)."""
    handlers = {}
    for rpc, req_name, resp_name in P.METHODS:
        fn = getattr(servicer, rpc)
        if rpc == "ScoreTransaction" and native_tx is not None:
            async def h(data, ctx, _n=native_tx):
                return await _n.call(data)
        elif rpc == "ScoreTransaction" and servicer.batcher is not None:
            async def h(data, ctx, _b=servicer.batcher):
                return await asyncio.wrap_future(_b.submit(data, time.perf_counter()))
        elif rpc in ("PredictLTV", "GetPlayerSegment") and servicer.ltv_batcher is not None:
            build = servicer.ltv_response if rpc == "PredictLTV" else servicer.segment_response

            async def h(req, ctx, _b=servicer.ltv_batcher, _build=build):
                if not req.account_id:
                    raise InvalidArgument("account_id is required")
                return _build(req, await asyncio.wrap_future(_b.submit(req.account_id)))
        elif rpc == "CheckBonusAbuse" and servicer.abuse_batcher is not None:
            async def h(req, ctx, _b=servicer.abuse_batcher):
                if not req.account_id:
                    raise InvalidArgument("account_id is required")
                return servicer.abuse_response(await asyncio.wrap_future(_b.submit(req.account_id)))
        elif inline_all or rpc in INLINE:
            async def h(req, ctx, _f=fn):
                return _f(req, ctx)
        else:
            async def h(req, ctx, _f=fn):
                return await asyncio.get_running_loop().run_in_executor(pool, _f, req, ctx)
        if rpc in RAW:
            handlers[rpc] = grpc.unary_unary_rpc_method_handler(h)
        else:
            handlers[rpc] = grpc.unary_unary_rpc_method_handler(
                h, request_deserializer=P.M[req_name].FromString, response_serializer=lambda m: m.SerializeToString())
    return grpc.method_handlers_generic_handler(P.SERVICE, handlers)


def aio_health_handler(h: HealthServicer) -> grpc.GenericRpcHandler:
    ser = lambda m: m.SerializeToString()  # noqa: E731

    async def check(req, ctx):
        with h._cv:
            st = h._status.get(req.service)
        if st is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "unknown service")
        return HV.HealthCheckResponse(status=st)

    async def watch(req, ctx):
        last = None
        while True:
            with h._cv:
                st = h._status.get(req.service, HV.STATUS["SERVICE_UNKNOWN"])
            if st != last:
                last = st
                yield HV.HealthCheckResponse(status=st)
            await asyncio.sleep(0.2)

    return grpc.method_handlers_generic_handler(HV.SERVICE, {
        "Check": grpc.unary_unary_rpc_method_handler(check, request_deserializer=HV.HealthCheckRequest.FromString,
                                                     response_serializer=ser),
        "Watch": grpc.unary_stream_rpc_method_handler(watch, request_deserializer=HV.HealthCheckRequest.FromString,
                                                      response_serializer=ser),
    })


def aio_reflection_handler(pkg: str) -> grpc.GenericRpcHandler:
    sync = reflection_handler(pkg)
    info = sync.service(type("D", (), {"method": f"/{pkg}.ServerReflection/ServerReflectionInfo"})()).stream_stream

    async def ainfo(req_iter, ctx):
        async for raw in req_iter:
            for out in info(iter([raw]), ctx):
                yield out

    return grpc.method_handlers_generic_handler(f"{pkg}.ServerReflection", {
        "ServerReflectionInfo": grpc.stream_stream_rpc_method_handler(ainfo)})


class RiskServer:
    """risk.v1 on a ``grpc.aio`` server whose event loop runs on a dedicated thread."""

    def __init__(self, engine, port: int = 0, host: str = "127.0.0.1", workers: int = 16,
                 batching: bool = True, max_batch: Optional[int] = None, wait_us: Optional[int] = None,
                 reuseport: bool = False, extra_ports=()):
        """``reuseport``: bind with SO_REUSEPORT so every rank of a multi-GPU group listens on
        the same port (the kernel spreads connections over the ranks); ``extra_ports``: more
        listening ports (rank 0's internal port for cold RPCs forwarded by the other ranks)."""
        self.engine = engine
        cfg = engine.cfg
        self.batcher = None
        self.native_tx = None
        self._reuseport = bool(reuseport)
        self._extra_ports = list(extra_ports)
        # unary ScoreTransaction: the serving core's own FIFO when the engine has one (the
        # Python MicroBatcher stays for engines without a core: golden / multi-shard CPU)
        use_native = batching and getattr(engine, "core", None) is not None
        if batching and not use_native:
            self.batcher = MicroBatcher(engine.score_tx_many_bytes, max_batch or cfg.gpu.max_batch,
                                        cfg.gpu.wait_us if wait_us is None else wait_us, workers=2,
                                        on_batch=lambda n: engine.metrics.batch_size.observe(n))
        self.ltv_batcher = self.abuse_batcher = None
        if batching:
            wait = cfg.gpu.wait_us if wait_us is None else wait_us
            self.ltv_batcher = MicroBatcher(lambda ids, _t: engine.predict_ltv_batch(ids), 4096, wait, workers=1)
            self.abuse_batcher = MicroBatcher(lambda ids, _t: engine.check_bonus_abuse_batch(ids), 4096, wait,
                                              workers=1)
        self.health = HealthServicer()
        self.health.set(P.SERVICE, "SERVING")
        self.pool = futures.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="risk-rpc")
        self._servicer = RiskServicer(engine, self.batcher, self.ltv_batcher, self.abuse_batcher)
        self._host, self._port_req = host, port
        self.loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self.loop.run_forever, name="risk-grpc-loop", daemon=True)
        self._thread.start()
        if use_native:
            self.native_tx = NativeUnary(engine.core, self.loop, ok_fn=engine._native_ok, fallback=engine.score_tx_bytes,
                                         pool=self.pool)
        self.server = None
        self.port = asyncio.run_coroutine_threadsafe(self._build(), self.loop).result(30)

    async def _build(self) -> int:
        self.server = grpc.aio.server(interceptors=[AioInterceptor(self.engine.metrics)],
                                      options=[("grpc.max_receive_message_length", 64 << 20),
                                               ("grpc.max_send_message_length", 64 << 20),
                                               ("grpc.so_reuseport", 1 if self._reuseport else 0)])
        inline = self.engine.kind != "gpu" and self.engine.group is None
        self.server.add_generic_rpc_handlers([aio_risk_handler(self._servicer, self.pool, inline, self.native_tx),
                                              aio_health_handler(self.health)] +
                                             [aio_reflection_handler(p) for p in RV.PKGS])
        for p in self._extra_ports:
            self.server.add_insecure_port(f"{self._host}:{p}")
        return self.server.add_insecure_port(f"{self._host}:{self._port_req}")

    def start(self) -> "RiskServer":
        asyncio.run_coroutine_threadsafe(self.server.start(), self.loop).result(30)
        log.info("grpc server listening", extra={"fields": dict(port=self.port)})
        return self

    def stop(self, grace: float = 5.0) -> None:
        self.health.set("", "NOT_SERVING")
        self.health.set(P.SERVICE, "NOT_SERVING")
        asyncio.run_coroutine_threadsafe(self.server.stop(grace), self.loop).result(grace + 30)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self._thread.join(timeout=5)
        self.pool.shutdown(wait=False)
        for b in (self.batcher, self.ltv_batcher, self.abuse_batcher, self.native_tx):
            if b is not None:
                b.close()


class IngressServer:
    """risk.v1 on a worker rank (>= 1) of a multi-GPU group: ScoreBatch and ScoreTransaction go
    through THIS rank's serving core (its own parse / resolve / exchange steps: every rank
    ingests), every other RPC is forwarded byte-for-byte to rank 0's internal port (the cold
    ops are rank 0's control plane). Same port as rank 0 with SO_REUSEPORT by default, so one
    address spreads connections over every rank of the node."""

    def __init__(self, node, upstream: str, port: int, host: str = "0.0.0.0", reuseport: bool = True, metrics=None):
        from ..obs.metrics import Metrics
        self.node, self.upstream = node, upstream
        self.metrics = metrics or Metrics()
        self.health = HealthServicer()
        self.health.set(P.SERVICE, "SERVING")
        self._host, self._port_req, self._reuseport = host, port, reuseport
        self.loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self.loop.run_forever, name="ingress-grpc-loop", daemon=True)
        self._thread.start()
        self.native_tx = NativeUnary(node.core, self.loop)
        self.port = asyncio.run_coroutine_threadsafe(self._build(), self.loop).result(30)

    async def _build(self) -> int:
        opts = [("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)]
        self._up = grpc.aio.insecure_channel(self.upstream, options=opts)
        self.server = grpc.aio.server(interceptors=[AioInterceptor(self.metrics)],
                                      options=opts + [("grpc.so_reuseport", 1 if self._reuseport else 0)])
        core, ntx = self.node.core, self.native_tx
        pool = futures.ThreadPoolExecutor(max_workers=16, thread_name_prefix="ingress-rpc")
        self._pool = pool
        handlers = {}
        for rpc, _, _ in P.METHODS:
            if rpc == "ScoreBatch":
                async def h(data, ctx, _c=core):
                    loop = asyncio.get_running_loop()
                    return await loop.run_in_executor(pool, _c.score_batch, data, int(time.time()),
                                                      time.perf_counter_ns())
            elif rpc == "ScoreTransaction":
                async def h(data, ctx, _n=ntx):
                    return await _n.call(data)
            else:
                fwd = self._up.unary_unary(P.method_path(rpc))

                async def h(data, ctx, _f=fwd):  # cold RPC: rank 0 answers it
                    return await _f(data, timeout=30)
            handlers[rpc] = grpc.unary_unary_rpc_method_handler(h)
        self.server.add_generic_rpc_handlers([grpc.method_handlers_generic_handler(P.SERVICE, handlers),
                                              aio_health_handler(self.health)])
        return self.server.add_insecure_port(f"{self._host}:{self._port_req}")

    def start(self) -> "IngressServer":
        asyncio.run_coroutine_threadsafe(self.server.start(), self.loop).result(30)
        log.info("ingress grpc server listening", extra={"fields": dict(port=self.port, upstream=self.upstream)})
        return self

    def stop(self, grace: float = 5.0) -> None:
        self.health.set(P.SERVICE, "NOT_SERVING")
        asyncio.run_coroutine_threadsafe(self.server.stop(grace), self.loop).result(grace + 30)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self._thread.join(timeout=5)
        self.native_tx.close()
        self._pool.shutdown(wait=False)
