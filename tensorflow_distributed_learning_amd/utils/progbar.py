"""Keras-style progress bar (the default ``fit`` output, tf_dist_example.py:59)."""
from __future__ import annotations

import sys
import time
from typing import Dict, Optional


def _fmt_time(sec: float) -> str:
    if sec >= 1:
        return f"{sec:.0f}s"
    if sec >= 1e-3:
        return f"{sec * 1e3:.0f}ms"
    return f"{sec * 1e6:.0f}us"


def format_logs(logs: Dict[str, float]) -> str:
    out = []
    for k, v in logs.items():
        try:
            fv = float(v)
        except (TypeError, ValueError):
            continue
        out.append(f"{k}: {fv:.4e}" if abs(fv) < 1e-3 and fv != 0 else f"{k}: {fv:.4f}")
    return " - ".join(out)


class Progbar:
    def __init__(self, target: Optional[int], width: int = 30, verbose: int = 1, stream=None, unit_name="step"):
        self.target = target
        self.width = width
        self.verbose = verbose
        self.stream = stream or sys.stdout
        self.unit_name = unit_name
        self._start = time.time()
        self._seen = 0
        self._dynamic = hasattr(self.stream, "isatty") and self.stream.isatty()
        self._last_len = 0

    def update(self, current: int, logs: Optional[Dict[str, float]] = None, finalize: Optional[bool] = None):
        if finalize is None:
            finalize = self.target is not None and current >= self.target
        self._seen = current
        if self.verbose == 0:
            return
        elapsed = time.time() - self._start
        per = elapsed / max(1, current)
        logs_s = format_logs(logs or {})
        if self.verbose == 1:
            if not self._dynamic and not finalize:
                return
            if self.target is not None:
                nd = len(str(self.target))
                bar = f"{current:{nd}d}/{self.target} ["
                prog = float(current) / self.target if self.target else 1.0
                done = int(self.width * prog)
                if done > 0:
                    bar += "=" * (done - 1) + (">" if current < self.target else "=")
                bar += "." * (self.width - done) + "]"
            else:
                bar = f"{current:7d}/Unknown"
            if finalize:
                info = f" - {_fmt_time(elapsed)} {_fmt_time(per)}/{self.unit_name}"
            else:
                eta = per * ((self.target or current) - current)
                info = f" - ETA: {_fmt_time(eta)}"
            line = bar + info + (" - " + logs_s if logs_s else "")
            if self._dynamic:
                pad = max(0, self._last_len - len(line))
                self.stream.write("\r" + line + " " * pad)
                self._last_len = len(line)
                if finalize:
                    self.stream.write("\n")
            else:
                self.stream.write(line + "\n")
            self.stream.flush()
        elif self.verbose == 2 and finalize:
            nd = len(str(self.target)) if self.target else 1
            line = f"{current:{nd}d}/{self.target} - {_fmt_time(elapsed)} - {_fmt_time(per)}/{self.unit_name}"
            if logs_s:
                line += " - " + logs_s
            self.stream.write(line + "\n")
            self.stream.flush()
