"""Per-step kernel timeline from a rocprofv3 ``*_kernel_trace.csv``.

A decode / batch step is the run of kernels between two consecutive sampler stage-2
kernels (the last kernel of every step). For the last N steps this prints, per kernel
name, the total device time per step, the launch count per step and the idle time
(gap) before its launches - so "where does a 2.5 ms step go" splits into kernel time
and inter-kernel gaps.

    python tools/step_timeline.py gpurun_out/x/..._kernel_trace.csv [--steps 16] [--json out.json]
"""
import argparse
import collections
import csv
import json
import re


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)           # drop the argument list
    name = name.replace("void ", "").replace("lfk::", "")
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--end", default="sample_stage2", help="kernel name substring that ends a step")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    ends = [i for i, k in enumerate(ks) if args.end in k[2]]
    if len(ends) < 2:
        raise SystemExit("fewer than two step ends in the trace")
    ends = ends[-(args.steps + 1):]
    per = collections.defaultdict(lambda: [0.0, 0, 0.0])  # name -> [kernel ns, launches, gap ns]
    step_ns = []
    for a, b in zip(ends[:-1], ends[1:]):
        seg = ks[a + 1:b + 1]
        step_ns.append(seg[-1][1] - ks[a][1])
        prev_end = ks[a][1]
        for s, e, n in seg:
            p = per[short(n)]
            p[0] += e - s
            p[1] += 1
            p[2] += max(0, s - prev_end)
            prev_end = max(prev_end, e)
    n = len(step_ns)
    step = sum(step_ns) / n
    tot_k = sum(v[0] for v in per.values()) / n
    tot_g = sum(v[2] for v in per.values()) / n
    print(f"steps {n}: {step / 1e3:.1f} us per step = kernels {tot_k / 1e3:.1f} us + gaps {tot_g / 1e3:.1f} us")
    print(f"{'kernel us/step':>14} {'gap us/step':>12} {'launches':>9}  kernel")
    out = []
    for name, (k, c, g) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print(f"{k / n / 1e3:14.1f} {g / n / 1e3:12.1f} {c / n:9.1f}  {name}")
        out.append({"kernel": name, "us_per_step": round(k / n / 1e3, 2), "gap_us_per_step": round(g / n / 1e3, 2),
                    "launches_per_step": c / n})
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"steps": n, "us_per_step": round(step / 1e3, 1), "kernel_us": round(tot_k / 1e3, 1),
                       "gap_us": round(tot_g / 1e3, 1), "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
