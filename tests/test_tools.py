"""CPU checks of the profiling tools whose outputs DESIGN.md and bench.py
quote (tools/summarize_prof.py, tools/summarize_pmc.py, tools/trace_by_grid.py)
on synthetic rocprofv3 CSV files of the same layout, and of bench.py's
`roofline.traffic` lookup in the committed profiles."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(REPO, "tools")
FOLD_D = "void shmx::(anonymous namespace)::fold_kernel<double, 0, 2, 4, 3>(shmx::(anonymous namespace)::FoldArgs)"
FOLD_F = "void shmx::(anonymous namespace)::fold_kernel<float, 0, 2, 4, 3>(shmx::(anonymous namespace)::FoldArgs)"


def write_csv(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def run(*args, env=None):
    p = subprocess.run([sys.executable, *args], capture_output=True, text=True, env=env, timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout


def counters(path, name, kernels):
    write_csv(path, ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"],
              [[i, k, g, name, v] for i, (k, g, v) in enumerate(kernels)])


def test_summarize_prof_takes_the_double_fold_only(tmp_path):
    write_csv(str(tmp_path / "trace/x/kernel_stats.csv"), ["Name", "Calls", "AverageNs"],
              [[FOLD_D, 61, 121270.0], [FOLD_F, 40, 9000.0]])
    # per launch: FETCH_SIZE counts half of the streamed reads (KiB), WRITE_SIZE all writes
    counters(str(tmp_path / "fetch/x/counter_collection.csv"), "FETCH_SIZE",
             [(FOLD_F, "1", 100.0), (FOLD_D, "2", 262163.5), (FOLD_D, "2", 262163.5)])
    counters(str(tmp_path / "write/x/counter_collection.csv"), "WRITE_SIZE",
             [(FOLD_F, "1", 50.0), (FOLD_D, "2", 262144.0), (FOLD_D, "2", 262144.0)])
    out = tmp_path / "out"
    run(os.path.join(TOOLS, "summarize_prof.py"), str(tmp_path / "trace"), str(tmp_path / "fetch"),
        str(tmp_path / "write"), "rXX", env=dict(os.environ, PROFILES_OUT=str(out)))
    d = json.load(open(out / "rXX_pmc.json"))
    assert d["fold_double_sum"]["hbm_bytes_per_launch"] == 2 * 262163.5 * 1024 + 262144.0 * 1024
    assert d["fold_double_sum"]["alg_bytes_per_launch"] == 805306368
    assert "double" in d["fold_double_sum"]["kernel"]
    assert (out / "rXX_kernel_stats.csv").exists()
    # without the double fold there is no headline entry (never another kernel's bytes)
    counters(str(tmp_path / "fetch/x/counter_collection.csv"), "FETCH_SIZE", [(FOLD_F, "1", 100.0)])
    run(os.path.join(TOOLS, "summarize_prof.py"), str(tmp_path / "trace"), str(tmp_path / "fetch"),
        str(tmp_path / "write"), "rYY", env=dict(os.environ, PROFILES_OUT=str(out)))
    assert "fold_double_sum" not in json.load(open(out / "rYY_pmc.json"))


def test_summarize_pmc_maps_runs_to_configs(tmp_path):
    cfgs = [{"config": "a", "alg_bytes": 3072, "launches": 2},
            {"config": "b", "alg_bytes": 1024, "launches": 2},
            {"config": "c", "alg_bytes": 1024, "launches": 2, "shares_run": True},
            {"config": "d", "alg_bytes": 2048, "launches": 2}]
    (tmp_path / "log").write_text("".join(json.dumps(c) + "\n" for c in cfgs))
    # b and c launch the same kernel at the same grid: one run of 4 dispatches
    ks = [("shmx::A", "1")] * 2 + [("shmx::B", "2")] * 4 + [("shmx::D", "3")] * 2
    write_csv(str(tmp_path / "t/x/kernel_trace.csv"),
              ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Start_Timestamp", "End_Timestamp"],
              [[i, k, g, 0, 1000 * (i + 1)] for i, (k, g) in enumerate(ks)])
    fetch = {"A": 1.0, "B": 0.25, "D": 0.5}     # KiB, half of the reads
    write = {"A": 1.0, "B": 0.5, "D": 1.0}
    counters(str(tmp_path / "f/x/counter_collection.csv"), "FETCH_SIZE",
             [(k, g, fetch[k[-1]]) for k, g in ks])
    counters(str(tmp_path / "w/x/counter_collection.csv"), "WRITE_SIZE",
             [(k, g, write[k[-1]]) for k, g in ks])
    run(os.path.join(TOOLS, "summarize_pmc.py"), str(tmp_path / "log"), str(tmp_path / "t"),
        str(tmp_path / "f"), str(tmp_path / "w"), str(tmp_path / "out.json"))
    got = {e["config"]: e for e in json.load(open(tmp_path / "out.json"))["configs"]}
    assert [got[c]["kernel"] for c in "abcd"] == ["shmx::A", "shmx::B", "shmx::B", "shmx::D"]
    assert got["a"]["traffic_over_alg"] == 1.0 and got["b"]["traffic_over_alg"] == 1.0
    assert got["d"]["hbm_bytes_per_launch"] == 2048
    # the first launch of a run is dropped from the average (it pays the cold start)
    assert got["b"]["rocprof_avg_us"] == (4 + 5 + 6) / 3


def test_trace_by_grid_splits_sizes(tmp_path):
    write_csv(str(tmp_path / "x/kernel_trace.csv"),
              ["Kernel_Name", "Grid_Size", "Start_Timestamp", "End_Timestamp"],
              [[FOLD_D, "4096", 0, 8000], [FOLD_D, "4096", 0, 10000], [FOLD_D, "256", 0, 1000],
               ["other", "256", 0, 5000]])
    lines = [json.loads(x) for x in run(os.path.join(TOOLS, "trace_by_grid.py"), str(tmp_path),
                                        "fold_kernel").splitlines()]
    assert [(x["grid"], x["launches"], x["mean_us"], x["min_us"]) for x in lines] == \
        [("256", 1, 1.0, 1.0), ("4096", 2, 9.0, 8.0)]


def test_bench_reads_traffic_from_the_committed_profile():
    sys.path.insert(0, REPO)
    import bench
    # the newest committed counter summary was measured on the device code
    # this tree builds: its traffic is reported, ~1.0x the 768 MiB per launch
    v, note = bench.pmc_traffic("fold_double_sum")
    assert v is not None, note
    assert abs(v / (3 * 8 * 32 * 1024 * 1024) - 1) < 0.01, v
    assert bench.pmc_traffic("no_such_kernel")[0] is None


def test_call_timer_calls_the_entry_point_it_is_given():
    """tools/libcalltimer.so (bench.py's per-call timer from C) calls the
    given entry point warm + reps times with the given arguments and times
    each timed call."""
    import ctypes
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tools"), "libcalltimer.so"], check=True)
    L = ctypes.CDLL(os.path.join(REPO, "tools", "libcalltimer.so"))
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.call_timer_to_all.argtypes = [vp, vp, vp, i, i, i, i, vp, vp, i, i, ctypes.POINTER(ctypes.c_double)]
    seen = []
    proto = ctypes.CFUNCTYPE(None, vp, vp, i, i, i, i, vp, vp)
    cb = proto(lambda t, s, n, a, b, c, w, p: seen.append((t, s, n, a, b, c)))
    out = (ctypes.c_double * 7)()
    rc = L.call_timer_to_all(ctypes.cast(cb, vp), 16, 32, 5, 0, 1, 2, None, None, 3, 7, out)
    assert rc == 0 and len(seen) == 10
    assert all(x == (16, 32, 5, 0, 1, 2) for x in seen)
    assert all(v >= 0 for v in out)
