"""Wallet service binary: ``python -m igaming_platform_amd.wallet.serve``.

Env (services/wallet/cmd/main.go:54-62): GRPC_PORT (9080), DATABASE_URL (here a SQLite path or
``sqlite:///path``; default ./wallet.db), RISK_SERVICE_URL (localhost:9082, the risk gRPC port —
the compose file's :8082 HTTP value is quirk Q18 and is mapped to 9082), RISK_BLOCK_THRESHOLD (80),
RISK_REVIEW_THRESHOLD (50), LOG_LEVEL. Optional BONUS_CONFIG_PATH enables the bonus engine.
"""
from __future__ import annotations

import os
import signal
import threading

from ..obs.logging import setup_logger


def main() -> int:
    env = os.environ
    log = setup_logger(env.get("LOG_LEVEL", "info"))
    from ..clients.risk_client import RiskClient
    from .grpc_api import WalletServer
    from .repository import Database
    from .service import GrpcRisk, WalletService
    db_url = env.get("DATABASE_URL", "wallet.db")
    path = db_url[len("sqlite:///"):] if db_url.startswith("sqlite:///") else db_url
    if path.startswith("postgres"):
        log.warning("postgres URLs are not supported offline; using ./wallet.db")
        path = "wallet.db"
    risk_url = env.get("RISK_SERVICE_URL", "localhost:9082").replace("http://", "")
    if risk_url.endswith(":8082"):
        risk_url = risk_url[:-5] + ":9082"
    svc = WalletService(Database(path), risk=GrpcRisk(RiskClient(risk_url)),
                        block_threshold=int(env.get("RISK_BLOCK_THRESHOLD", 80)),
                        review_threshold=int(env.get("RISK_REVIEW_THRESHOLD", 50)))
    if env.get("BONUS_CONFIG_PATH"):
        from ..bonus.engine import BonusEngine, GrpcAbuseChecker
        from .repository import BonusRepository
        svc.bonus = BonusEngine.from_file(env["BONUS_CONFIG_PATH"], BonusRepository(svc.db),
                                          risk=GrpcAbuseChecker(RiskClient(risk_url)), wallet=svc)
    srv = WalletServer(svc, port=int(env.get("GRPC_PORT", 9080)), host="0.0.0.0").start()
    log.info("wallet service listening", extra={"fields": dict(port=srv.port, db=path, risk=risk_url)})
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *a: stop.set())
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    stop.wait()
    srv.stop(30.0)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
