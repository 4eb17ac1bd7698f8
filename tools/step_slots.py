"""Per-layer-slot kernel durations of the batch step from a rocprofv3 kernel trace (medians over
the last 20 steps, averaged over the layers): which of Q|K|V, attention, Wo, gate/up, down moved.
    python tools/step_slots.py gpurun_out/abp_<label>/bstep_kernel_trace.csv [--per-layer 5]"""
import collections
import csv
import statistics
import sys


def main(path, per_layer=5, prologue=4, layers=32):
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if "sample_stage1" in r["Kernel_Name"]]
    acc = collections.defaultdict(list)
    names = {}
    for a, b in zip(idx[-21:-1], idx[-20:]):
        for j, r in enumerate(rows[a + 1:b + 1]):
            acc[j].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
            names[j] = r["Kernel_Name"].split("(")[0].split("::")[-1][:24]
    slots = collections.defaultdict(list)
    for j, v in acc.items():
        if prologue <= j < prologue + layers * per_layer:
            slots[(j - prologue) % per_layer].append(statistics.median(v))
    out = {f"{k}:{names[prologue + k]}": round(statistics.mean(v), 2) for k, v in sorted(slots.items())}
    print(out, "sum", round(sum(out.values()), 2))


if __name__ == "__main__":
    main(sys.argv[1])
