"""Wall-clock helpers used by the facade, the server metrics and the benchmarks."""
from __future__ import annotations

import math
import time
from typing import Dict, List, Sequence


class Timer:
    """Accumulating named timers: ``with t("prefill"): ...``; ``t.summary()``."""

    def __init__(self):
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}
        self._name = None
        self._t0 = 0.0

    def __call__(self, name: str) -> "Timer":
        self._name = name
        return self

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        dt = time.perf_counter() - self._t0
        self.totals[self._name] = self.totals.get(self._name, 0.0) + dt
        self.counts[self._name] = self.counts.get(self._name, 0) + 1
        return False

    def summary(self) -> Dict[str, Dict[str, float]]:
        return {k: {"total_s": v, "count": self.counts[k], "mean_ms": v / self.counts[k] * 1e3}
                for k, v in self.totals.items()}


def percentile(values: Sequence[float], q: float) -> float:
    """Linear-interpolated percentile (q in [0, 100]) without numpy."""
    xs: List[float] = sorted(values)
    if not xs:
        return float("nan")
    k = (len(xs) - 1) * q / 100.0
    lo, hi = math.floor(k), math.ceil(k)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)
