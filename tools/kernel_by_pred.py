"""Split a rocprofv3 kernel trace's per-kernel times by the kernel that ran BEFORE each dispatch.

One kernel template often serves several weight shapes (the 70B's Q4_K `gemv_kernel<12, 1, ...>`
runs both Wo - after attention - and the Q4_K half of the down projections - after gate/up), so
its stats row mixes a 9 us and a 33 us launch. Keyed by (kernel, predecessor) the shapes separate.

    python tools/kernel_by_pred.py gpurun_out/dec70prof/k_kernel_trace.csv [--min-calls 16]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.replace("void ", "")).strip()
    return name[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-calls", type=int, default=16)
    ap.add_argument("--grid", action="store_true", help="also key by the dispatch's grid (prefill T differ)")
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if args.grid:
                k += " [%s,%s,%s]" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    groups = defaultdict(list)
    for i in range(1, len(rows)):
        s, e, k = rows[i]
        groups[(k, rows[i - 1][2])].append((e - s) / 1e3)
    out = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
    print(f"{len(rows)} dispatches, {sum(e - s for s, e, _ in rows) / 1e3:.1f} us of kernels")
    print()
    print("| calls | med us | min us | max us | kernel | after |")
    print("|---:|---:|---:|---:|---|---|")
    for (k, p), ts in out:
        if len(ts) < args.min_calls:
            continue
        print(f"| {len(ts)} | {statistics.median(ts):.2f} | {min(ts):.2f} | {max(ts):.2f} | `{k}` | `{p}` |")


if __name__ == "__main__":
    main()
