"""rocprofv3 helpers: the command line the tools use and a kernel-stats summariser.

rocprofv3 is run with ``--kernel-trace --stats`` only (never together with PMC
counters); the program follows ``--`` directly (no env/bash launchers)."""
from __future__ import annotations

import csv
from typing import Dict, List, Sequence


def rocprof_cmd(out_dir: str, name: str, program: Sequence[str]) -> List[str]:
    return ["rocprofv3", "--kernel-trace", "--stats", "-d", out_dir, "-o", name, "--output-format", "csv", "--",
            *program]


def kernel_stats(path: str) -> List[Dict]:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
    return [{"name": r["Name"], "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
             "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["TotalDurationNs"]) / tot * 100}
            for r in rows]
