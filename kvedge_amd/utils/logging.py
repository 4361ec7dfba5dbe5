"""Structured logs: one JSON object per line on stderr.

    from kvedge_amd.utils.logging import get_logger, log_event
    log = get_logger("kvedge.module")
    log_event(log, "rebuild", model="resnet50", batch=64, ok=True)

-> {"ts": "...Z", "level": "INFO", "logger": "kvedge.module", "event": "rebuild",
    "rank": 0, "model": "resnet50", "batch": 64, "ok": true}

``KVEDGE_LOG_FORMAT=text`` switches to a human-readable line, ``KVEDGE_LOG_LEVEL`` sets
the level (default INFO).  IoT Edge collects module stderr (`iotedge logs kvedge`), so
these lines are what an operator greps or ships to Log Analytics.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Any

_CONFIGURED = set()


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        out = {"ts": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created))
               + f".{int(record.msecs):03d}Z",
               "level": record.levelname, "logger": record.name,
               "event": getattr(record, "event", None) or record.getMessage()}
        rank = os.environ.get("RANK")
        if rank is not None:
            out["rank"] = int(rank)
        out.update(getattr(record, "fields", {}) or {})
        if record.exc_info:
            out["exc"] = self.formatException(record.exc_info)
        return json.dumps(out, default=str, sort_keys=False)


class TextFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        f = getattr(record, "fields", {}) or {}
        kv = " ".join(f"{k}={v}" for k, v in f.items())
        ev = getattr(record, "event", None) or record.getMessage()
        return f"{record.levelname[0]} {record.name}: {ev} {kv}".rstrip()


def get_logger(name: str = "kvedge", stream=None) -> logging.Logger:
    log = logging.getLogger(name)
    if name not in _CONFIGURED:
        h = logging.StreamHandler(stream or sys.stderr)
        fmt = os.environ.get("KVEDGE_LOG_FORMAT", "json").lower()
        h.setFormatter(TextFormatter() if fmt == "text" else JsonFormatter())
        log.addHandler(h)
        log.setLevel(os.environ.get("KVEDGE_LOG_LEVEL", "INFO").upper())
        log.propagate = False
        _CONFIGURED.add(name)
    return log


def log_event(log: logging.Logger, event: str, level: int = logging.INFO, **fields: Any):
    log.log(level, event, extra={"event": event, "fields": fields})
