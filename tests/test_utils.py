import time

from llama_fastapi_k8s_gpu_amd.utils import Timer, percentile
from llama_fastapi_k8s_gpu_amd.utils.rocprof import kernel_stats, rocprof_cmd


def test_timer_and_percentile():
    t = Timer()
    for _ in range(3):
        with t("a"):
            time.sleep(0.001)
    s = t.summary()["a"]
    assert s["count"] == 3 and s["total_s"] > 0.002
    assert percentile([1, 2, 3, 4], 50) == 2.5
    assert percentile([5], 90) == 5


def test_rocprof_helpers(tmp_path):
    cmd = rocprof_cmd("gpurun_out/p", "x", ["python3", "bench.py"])
    assert cmd[cmd.index("--") + 1] == "python3" and "--pmc" not in cmd
    p = tmp_path / "k.csv"
    p.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
                 '"k1",2,3000,1500,75,1000,2000,0\n"k2",1,1000,1000,25,1000,1000,0\n')
    ks = kernel_stats(str(p))
    assert ks[0]["name"] == "k1" and abs(ks[0]["pct"] - 75) < 1e-9 and ks[1]["avg_us"] == 1.0
