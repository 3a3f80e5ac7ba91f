"""Structured logging (zap in the reference) -> stdlib logging with a JSON formatter."""
from __future__ import annotations

import json
import logging
import sys
import time
from typing import Any, Optional

_CONFIGURED = False


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d = {
            "ts": round(record.created, 6),
            "level": record.levelname.lower(),
            "logger": record.name,
            "msg": record.getMessage(),
        }
        extra = getattr(record, "fields", None)
        if extra:
            d.update(extra)
        if record.exc_info:
            d["error"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def configure(level: str = "info", fmt: str = "json", output: str = "stdout") -> None:
    global _CONFIGURED
    root = logging.getLogger("llmq")
    root.handlers.clear()
    stream = sys.stderr if output == "stderr" else sys.stdout
    if output not in ("stdout", "stderr"):
        handler: logging.Handler = logging.FileHandler(output)
    else:
        handler = logging.StreamHandler(stream)
    if fmt == "json":
        handler.setFormatter(JsonFormatter())
    else:
        handler.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    root.addHandler(handler)
    root.setLevel(getattr(logging, level.upper(), logging.INFO))
    root.propagate = False
    _CONFIGURED = True


def get_logger(name: str) -> "FieldLogger":
    return FieldLogger(logging.getLogger("llmq." + name))


class FieldLogger:
    """zap-like ``logger.With(...)`` / ``logger.Info(msg, fields...)``."""

    __slots__ = ("_log", "_fields")

    def __init__(self, log: logging.Logger, fields: Optional[dict] = None):
        self._log = log
        self._fields = fields or {}

    def with_fields(self, **fields: Any) -> "FieldLogger":
        f = dict(self._fields)
        f.update(fields)
        return FieldLogger(self._log, f)

    def _emit(self, level: int, msg: str, fields: dict) -> None:
        if not self._log.isEnabledFor(level):
            return
        f = dict(self._fields)
        f.update(fields)
        self._log.log(level, msg, extra={"fields": f})

    def debug(self, msg: str, **f: Any) -> None:
        self._emit(logging.DEBUG, msg, f)

    def info(self, msg: str, **f: Any) -> None:
        self._emit(logging.INFO, msg, f)

    def warning(self, msg: str, **f: Any) -> None:
        self._emit(logging.WARNING, msg, f)

    warn = warning

    def error(self, msg: str, **f: Any) -> None:
        self._emit(logging.ERROR, msg, f)


def monotonic_ns() -> int:
    return time.monotonic_ns()
