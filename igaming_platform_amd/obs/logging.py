"""Structured JSON logs with the reference's level semantics (services/risk/cmd/main.go:278-299:
slog JSON handler, level from LOG_LEVEL; OK requests at debug, errors at info)."""
from __future__ import annotations

import json
import logging
import sys
import time

LEVELS = {"debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING, "warning": logging.WARNING,
          "error": logging.ERROR}


class JsonFormatter(logging.Formatter):
    def format(self, rec: logging.LogRecord) -> str:
        d = {"time": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(rec.created)) + f".{int(rec.msecs):03d}Z",
             "level": rec.levelname, "msg": rec.getMessage(), "logger": rec.name}
        extra = getattr(rec, "fields", None)
        if extra:
            d.update(extra)
        if rec.exc_info:
            d["error"] = self.formatException(rec.exc_info)
        return json.dumps(d, default=str)


def setup_logger(level: str = "info", stream=None) -> logging.Logger:
    log = logging.getLogger("igaming")
    log.handlers.clear()
    h = logging.StreamHandler(stream or sys.stdout)
    h.setFormatter(JsonFormatter())
    log.addHandler(h)
    log.setLevel(LEVELS.get((level or "info").lower(), logging.INFO))
    log.propagate = False
    return log


def get_logger(name: str = "") -> logging.Logger:
    return logging.getLogger("igaming" + ("." + name if name else ""))


def kv(logger: logging.Logger, level: int, msg: str, **fields) -> None:
    if logger.isEnabledFor(level):
        logger.log(level, msg, extra={"fields": fields})
