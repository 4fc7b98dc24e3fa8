"""Structured (JSON-lines) logging for every process, with the rank of the
process attached (SURVEY §5 "structured JSON logs"; the reference used glog
V-levels in barrelman and log.Printf in the service).

``FOREMAST_LOG_FORMAT=json`` (default for the CLI) or ``text``;
``FOREMAST_LOG_LEVEL`` (default INFO)."""
from __future__ import annotations

import json
import logging
import os
import time


class JsonFormatter(logging.Formatter):
    def __init__(self, component: str = ""):
        super().__init__()
        self.component = component
        self.rank = os.environ.get("RANK")

    def format(self, record: logging.LogRecord) -> str:
        out = {"ts": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created)) + f".{int(record.msecs):03d}Z",
               "level": record.levelname.lower(), "logger": record.name, "msg": record.getMessage()}
        if self.component:
            out["component"] = self.component
        if self.rank is not None:
            out["rank"] = int(self.rank)
        for k, v in getattr(record, "fields", {}).items():
            out[k] = v
        if record.exc_info:
            out["exc"] = self.formatException(record.exc_info)
        return json.dumps(out, default=str)


def setup(component: str = "", fmt: str | None = None, level: str | None = None) -> None:
    fmt = (fmt or os.environ.get("FOREMAST_LOG_FORMAT", "json")).lower()
    level = (level or os.environ.get("FOREMAST_LOG_LEVEL", "INFO")).upper()
    h = logging.StreamHandler()
    if fmt == "json":
        h.setFormatter(JsonFormatter(component))
    else:
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(level)


def log_fields(logger: logging.Logger, level: int, msg: str, **fields) -> None:
    """Log with structured key/values (rendered as JSON fields)."""
    logger.log(level, msg, extra={"fields": fields})
