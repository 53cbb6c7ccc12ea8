"""HTTP side endpoints of the risk service (services/risk/cmd/main.go:165-214):
``/metrics`` (Prometheus), ``/health`` (always 200), ``/ready`` (engine health),
``/debug/thresholds`` (the LIVE thresholds — the reference reports the static env config,
quirk Q7), ``/debug/score`` (``ScoreWithExplanation``; a stub in the reference),
``POST /admin/reload_model`` (model hot-reload), ``POST /admin/flush_audit``
(drain the risk_scores audit ring into ``server.audit_db``), plus ``/debug/features``,
``/debug/velocity`` (GetVelocity + CheckRateLimit), ``/debug/feature_importance`` and
``/debug/engine``."""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from ..layouts import FEATREC
from ..obs.logging import get_logger

log = get_logger("http")


def _device_metrics(engine) -> bytes:
    """K10 device counters in Prometheus text format: whole-group totals, plus the rows each
    shard scored (SPMD: one all-reduce of every rank's counter block, OP_METRICS) so owner skew
    across GPUs is visible."""
    per = engine.shard_metrics() if hasattr(engine, "shard_metrics") else None
    if per is None:
        return b""
    tot = per.sum(0)
    lines = ["# HELP risk_device_rows_total rows scored on the GPUs (K10 counters)",
             "# TYPE risk_device_rows_total counter", f"risk_device_rows_total {int(tot[106])}",
             "# HELP risk_shard_rows_total rows scored by each shard (owner-routed DP)",
             "# TYPE risk_shard_rows_total counter"]
    lines += [f'risk_shard_rows_total{{shard="{o}"}} {int(per[o, 106])}' for o in range(per.shape[0])]
    lines += ["# HELP risk_device_action_total decisions counted on the GPUs", "# TYPE risk_device_action_total counter"]
    for a, name in ((1, "approve"), (2, "review"), (3, "block")):
        lines.append(f'risk_device_action_total{{action="{name}"}} {int(tot[101 + a])}')
    lines += ["# HELP risk_device_score_total final-score histogram counted on the GPUs",
              "# TYPE risk_device_score_total counter"]
    for d in range(0, 101, 10):
        lines.append(f'risk_device_score_total{{decile="{d}"}} {int(tot[d:min(d + 10, 101)].sum())}')
    lines += [f"risk_device_ml_high_risk_total {int(tot[105])}", f"risk_device_blacklist_hits_total {int(tot[107])}"]
    return ("\n".join(lines) + "\n").encode()


def make_handler(engine):
    class H(BaseHTTPRequestHandler):
        server_version = "igaming-risk"

        def log_message(self, fmt, *args):  # routed to the JSON logger at debug
            log.debug("http " + fmt % args)

        def _send(self, code: int, body, ctype: str = "text/plain; charset=utf-8"):
            if isinstance(body, str):
                body = body.encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):
            u = urlparse(self.path)
            q = {k: v[-1] for k, v in parse_qs(u.query).items()}
            try:
                if u.path == "/metrics":
                    self._send(200, engine.metrics.render() + _device_metrics(engine),
                               "text/plain; version=0.0.4; charset=utf-8")
                elif u.path == "/health":
                    self._send(200, "OK")
                elif u.path == "/ready":
                    self._send(200, "Ready") if engine.ready() else self._send(503, "Not ready")
                elif u.path == "/debug/thresholds":
                    b, r = engine.get_thresholds()
                    self._send(200, json.dumps({"block_threshold": b, "review_threshold": r}), "application/json")
                elif u.path == "/debug/score":
                    if not q.get("account_id"):
                        return self._send(400, "account_id is required")
                    tx = dict(account_id=q["account_id"], amount=int(q.get("amount", 0)),
                              transaction_type=q.get("type", q.get("transaction_type", "deposit")),
                              device_id=q.get("device_id", ""), ip_address=q.get("ip", ""))
                    self._send(200, engine.explain(tx))
                elif u.path == "/debug/features":
                    if not q.get("account_id"):
                        return self._send(400, "account_id is required")
                    f = engine.get_features(q["account_id"])
                    self._send(200, json.dumps({k: f[k].item() for k in FEATREC.names}), "application/json")
                elif u.path == "/debug/velocity":  # GetVelocity + CheckRateLimit (redis_store.go:171-203)
                    if not q.get("account_id"):
                        return self._send(400, "account_id is required")
                    c1, c5, ch = engine.get_velocity(q["account_id"])
                    lim = engine.check_rate_limit(q["account_id"], q.get("max_per_min"), q.get("max_per_hour"))
                    self._send(200, json.dumps({"count_1m": c1, "count_5m": c5, "count_1h": ch, "rate_limited": lim}),
                               "application/json")
                elif u.path == "/debug/feature_importance":
                    self._send(200, json.dumps(engine.get_feature_importance()), "application/json")
                elif u.path == "/debug/engine":
                    self._send(200, json.dumps(engine.health()), "application/json")
                else:
                    self._send(404, "not found")
            except Exception as e:  # never take the side server down
                log.error("http handler error", exc_info=True)
                self._send(500, f"error: {e}")

        def do_POST(self):
            u = urlparse(self.path)
            try:
                if u.path == "/admin/reload_model":  # body: ONNX model bytes (empty: heuristic)
                    n = int(self.headers.get("Content-Length", "0"))
                    if n > 1 << 30:
                        return self._send(413, "model too large")
                    body = self.rfile.read(n) if n else b""
                    v = engine.reload_model(body)
                    self._send(200, json.dumps({"model_version": v, "model_kind": engine.model_kind}),
                               "application/json")
                elif u.path == "/admin/flush_audit":
                    path = engine.cfg.server.audit_db
                    if not path:
                        return self._send(409, "server.audit_db (AUDIT_DB) is not set")
                    self._send(200, json.dumps({"rows": engine.flush_audit(path)}), "application/json")
                else:
                    self._send(404, "not found")
            except ValueError as e:
                self._send(400, f"error: {e}")
            except Exception as e:
                log.error("http handler error", exc_info=True)
                self._send(500, f"error: {e}")

    return H


class HttpServer:
    def __init__(self, engine, port: int = 0, host: str = "127.0.0.1", timeout_s: float = 10.0):
        H = make_handler(engine)
        H.timeout = timeout_s  # read/write timeout (main.go:207-208)
        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self._t = threading.Thread(target=self.httpd.serve_forever, name="http", daemon=True)

    def start(self) -> "HttpServer":
        self._t.start()
        log.info("http server listening", extra={"fields": dict(port=self.port)})
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
