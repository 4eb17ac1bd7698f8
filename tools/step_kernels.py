"""Per-step kernel table of a batch_bench rocprofv3 trace: the kernels after the last prefill
launch, grouped by (name, grid), per-step count and median duration.
    python tools/step_kernels.py gpurun_out/bprof_<tag>/bstep_kernel_trace.csv"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    names = [r["Kernel_Name"] for r in rows]
    last = max(i for i, n in enumerate(names) if "gemm_dq" in n or "prefill" in n)
    st = rows[last + 1:]
    nsteps = sum(1 for r in st if "sample_stage1" in r["Kernel_Name"])
    agg = collections.defaultdict(list)
    for r in st:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        agg[(r["Kernel_Name"].split("(")[0][-48:], r["Grid_Size_X"], r["Workgroup_Size_X"])].append(d)
    tot = 0.0
    for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        v.sort()
        tot += sum(v)
        print(f"{k[0]:48s} grid {int(k[1]) // int(k[2]):5d}  {len(v) / nsteps:5.1f}/step  med {v[len(v) // 2]:7.2f} us  "
              f"{sum(v) / nsteps:7.1f} us/step")
    t0, t1 = int(st[0]["Start_Timestamp"]), int(st[-1]["End_Timestamp"])
    print(f"steps {nsteps}: kernels {tot / nsteps:.1f} us/step, wall {(t1 - t0) / 1e3 / nsteps:.1f} us/step")


if __name__ == "__main__":
    main(sys.argv[1])


def one_step(path, layer_from=2, layers=2):
    """The kernel sequence of one step (the second to last), durations in order."""
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if "sample_stage1" in r["Kernel_Name"]]
    a, b = idx[-3], idx[-2]
    for r in rows[a + 1:b + 1]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        print(f"{r['Kernel_Name'].split('(')[0][-40:]:40s} grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):5d} {d:7.2f}")
