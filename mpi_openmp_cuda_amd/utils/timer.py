"""Host stopwatch + per-phase timer (Python side of csrc/include/moc/runtime/timer.hpp; the reference's
vendored StopWatchLinux, inc/helper_timer.h:215-343, is never used by it)."""
from __future__ import annotations

import json
import time
from contextlib import contextmanager


class Stopwatch:
    def __init__(self):
        self.reset()

    def reset(self):
        self._t0 = None
        self.total = 0.0
        self.sessions = 0

    def start(self):
        self._t0 = time.perf_counter()

    def stop(self):
        if self._t0 is not None:
            self.total += time.perf_counter() - self._t0
            self.sessions += 1
            self._t0 = None

    @property
    def total_ms(self):
        return self.total * 1e3

    @property
    def average_ms(self):
        return self.total_ms / self.sessions if self.sessions else 0.0


class PhaseTimer:
    def __init__(self):
        self.phases = {}

    @contextmanager
    def phase(self, name, sync=None):
        if sync:
            sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync:
                sync()
            self.phases[name] = self.phases.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def json(self, **extra):
        d = {f"{k}_ms": round(v, 4) for k, v in self.phases.items()}
        d.update(extra)
        return json.dumps(d)
