"""CPU checks of bench.py's host-side logic that the driver's multi-GPU run
depends on: the auto_recommendation table built from the crossover and
partial-set extras, and the $SHMEMX_AUTO_* values it prints (the library's
parser accepts exactly this form; tests/test_gpu_ipc.py::
test_auto_table_from_environment runs it)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def table(us, ok=None):
    """crossover-style {algo: {str(n): value}} from {algo: [v per bucket]}."""
    sizes = [str(n) for n in (1, 1 << 9, 1 << 16, 1 << 19, 1 << 24)]
    t = {a: dict(zip(sizes, v)) for a, v in us.items()}
    c = {a: {n: True for n in sizes} for a in us}
    for (a, i) in ok or ():
        c[a][sizes[i]] = False
    return t, c


def test_auto_recommendation_full_and_partial(bench):
    us, ok = table({"allreduce": [10, 12, 40, 200, 5000],
                    "rccl": [30, 31, 45, 150, 3000],
                    "direct": [20, 11, 35, 160, 2500],
                    "signal": [9, 9, 30, 140, 2400],      # fastest, but never a table choice
                    "a2a": ["shmemx_reduce_on_stream(double,sum): ENOTSUP"] * 5},
                   ok=[("direct", 4)])                   # a wrong result at 128 MiB: excluded
    half_us, half_ok = table({"a2a": [15, 16, 50, 300, 9000], "direct": [14, 20, 40, 250, 8000],
                              "gather": [30, 30, 60, 400, 12000], "signal": [13, 13, 35, 240, 7000]})
    rec = bench.auto_recommendation({"us_per_call": us, "correct": ok},
                                    {"first_half_us_per_call": half_us, "first_half_correct": half_ok,
                                     "every_other_us_per_call": half_us, "every_other_correct": half_ok})
    full = rec["full"]
    assert full["8B"]["fastest"] == "signal" and full["8B"]["table"] == "allreduce"
    assert full["4KiB"]["table"] == "direct"
    assert full["512KiB"]["table"] == "direct"
    assert full["4MiB"]["table"] == "rccl"
    assert full["128MiB"]["table"] == "rccl"              # direct's 2500 us cell was wrong
    assert "a2a" not in full["8B"]["us"]                   # error strings are not timings
    # cut points between buckets at the geometric mean of their byte sizes
    assert rec["env"]["SHMEMX_AUTO_FULL"] == "0:allreduce,181:direct,1482910:rccl"
    assert rec["env"]["SHMEMX_AUTO_PARTIAL"] == "0:direct,181:a2a,46340:direct"
    for shape in ("half", "strided"):
        assert rec[shape]["8B"]["table"] == "direct" and rec[shape]["8B"]["fastest"] == "signal"


def test_auto_recommendation_env_is_parseable_form(bench):
    """bytes ascending, one algorithm per cut, names the library accepts."""
    us, ok = table({"allreduce": [1, 1, 1, 1, 1]})
    rec = bench.auto_recommendation({"us_per_call": us, "correct": ok}, "needs N >= 4")
    assert rec["env"] == {"SHMEMX_AUTO_FULL": "0:allreduce"}
    assert set(rec) == {"full", "env"}
    rec = bench.auto_recommendation("error: boom", None)
    assert rec == {"env": {}}


def test_auto_recommendation_from_a_table_cut_short(bench):
    """The watchdog may print the line while the crossover is being measured:
    the tables then hold rows for the algorithms done so far and a partial
    row for the current one (bench.py fills them in place); the
    recommendation uses the cells present and leaves empty buckets out."""
    us, ok = table({"rccl": [30, 31, 45, 150, 3000], "allreduce": [10, 12, 40, 200, 5000]})
    # the third algorithm was cut after two sizes; the fourth never started
    us["direct"], ok["direct"] = {"1": 5, "512": 50}, {"1": True, "512": True}
    us["signal"], ok["signal"] = {}, {}
    rec = bench.auto_recommendation({"us_per_call": us, "correct": ok}, {})
    assert rec["full"]["8B"]["table"] == "direct"
    assert rec["full"]["4KiB"]["table"] == "allreduce"
    assert rec["full"]["128MiB"]["table"] == "rccl"
    assert rec["env"]["SHMEMX_AUTO_FULL"].startswith("0:direct,")
    # a crossover cut before its first cell: nothing to recommend, no error
    rec = bench.auto_recommendation({}, {})
    assert rec["env"] == {}


def test_fused_twoshot_recommendation(bench):
    """$SHMEMX_FUSED_TWOSHOT_KB from the fused-vs-unfused cells (sizes in
    doubles per PE: 64 Ki = 512 KiB, 256 Ki = 2 MiB, 1 Mi = 8 MiB)."""
    def cells(d, s):
        return {"direct": {"65536": {"fused": d[0], "unfused": 50}, "262144": {"fused": d[1], "unfused": 60},
                           "1048576": {"fused": d[2], "unfused": 90}},
                "signal": {"65536": {"fused": s[0], "unfused": 50}, "262144": {"fused": s[1], "unfused": 60},
                           "1048576": {"fused": s[2], "unfused": 90}}}
    f = bench.fused_twoshot_kb
    assert f(cells((40, 50, 80), (40, 50, 80))) == 8192            # fused wins everywhere
    assert f(cells((40, 50, 100), (40, 50, 80))) == 4096           # loses at 8 MiB for one algo
    assert f(cells((40, 70, 100), (40, 50, 80))) == 1024           # loses from 2 MiB
    assert f(cells((60, 50, 80), (40, 50, 80))) == 256             # loses at once
    assert f(None) is None and f({}) is None
    assert f({"direct": {"65536": {"fused": "ENOTSUP", "unfused": 5}}}) is None
    # through auto_recommendation, beside the table variables
    us = {"rccl": {"1": 5.0}}
    ok = {"rccl": {"1": True}}
    rec = bench.auto_recommendation({"us_per_call": us, "correct": ok,
                                     "twoshot_fused_vs_unfused_us": cells((40, 50, 100), (40, 50, 80))}, {})
    assert rec["env"]["SHMEMX_FUSED_TWOSHOT_KB"] == "4096"


def test_pin_base_takes_the_last_consecutive_cpus(bench, monkeypatch):
    """The CPU baseline pins to the LAST P consecutive CPUs of the job's set
    (CPU 0 of a share also takes interrupts and runtime threads)."""
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda _pid: {0, 1, 2, 3, 8, 9, 10, 11})
    assert bench.pin_base(1) == 11
    assert bench.pin_base(4) == 8
    assert bench.pin_base(5) == -1          # no 5 consecutive CPUs: unpinned
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda _pid: set(range(16)))
    assert bench.pin_base(8) == 8


@pytest.mark.parametrize("world", [1, 3])
def test_cpu_baseline_fields(bench, world):
    """cpu_baseline at N = 1 (the local fold on one core) and N > 1 (the line's
    config on N PE processes): algbw GiB/s (one PE's array per call time, as
    the GPU value), the whole job's rate beside it, cores = N, the CPUs,
    min <= median <= max of the timed calls and the wall time."""
    n = 1 << 16
    c = bench.cpu_baseline(n, 3, world)
    assert c["unit"] == "GiB/s" and c["kind"] == "port" and c["cores"] == world
    assert c["value"] > 0 and c["wall_s"] >= 0
    sp = c["spread"]
    assert sp["calls"] == 3 and sp["min_ms"] <= sp["median_ms"] <= sp["max_ms"]
    assert abs(c["value"] - n * 8 / (sp["median_ms"] * 1e-3) / (1 << 30)) < 0.01 * c["value"] + 1e-3
    assert abs(c["aggregate_GiBps"] - world * c["value"]) < 0.01 * c["aggregate_GiBps"] + 1e-3
    assert ("on %d PEs" % world in c["sample"]) == (world > 1)


def test_pmc_traffic_tied_to_device_code(bench, tmp_path):
    """roofline.traffic comes from a committed PMC summary only while the
    loaded library carries the device code it measured."""
    import json
    d = {"fold_double_sum": {"hbm_bytes_per_launch": 805346304.0},
         "library": {"device_code_sha256": "ab" * 32}}
    (tmp_path / "r09_pmc.json").write_text(json.dumps(d))
    v, note = bench.pmc_traffic("fold_double_sum", str(tmp_path), "ab" * 32)
    assert v == 805346304.0 and "r09_pmc.json" in note
    v, note = bench.pmc_traffic("fold_double_sum", str(tmp_path), "cd" * 32)
    assert v is None and "other device code" in note
    # a summary without the build's hash (rounds before 5) is never trusted
    del d["library"]
    (tmp_path / "r09_pmc.json").write_text(json.dumps(d))
    assert bench.pmc_traffic("fold_double_sum", str(tmp_path), "ab" * 32)[0] is None
    assert bench.pmc_traffic("fold_double_sum", str(tmp_path / "none"), "ab" * 32)[0] is None


def test_device_code_hash_reads_the_fatbin(bench):
    """The hash is of the library's .hip_fatbin section: stable for the built
    library, None for a file that is not one."""
    import shmem_mi355x as shm
    h = shm.device_code_sha256()
    assert h and len(h) == 64 and h == shm.device_code_sha256()
    assert shm.device_code_sha256(__file__) is None


def test_auto_recommendation_partial_sets_may_name_rccl(bench):
    """Partial sets get RCCL on their own communicators (round 5), so the
    partial table may name allreduce / rccl when they are the fastest correct
    choice; SIGNAL is timed but never a table choice."""
    sizes = [str(n) for n in (1, 1 << 9, 1 << 16, 1 << 19, 1 << 24)]
    us = {"allreduce": [9, 10, 30, 150, 4000], "rccl": [20, 22, 40, 120, 2500],
          "a2a": [15, 16, 50, 300, 9000], "direct": [8, 20, 40, 250, 8000], "signal": [5, 5, 5, 5, 5]}
    t = {a: dict(zip(sizes, v)) for a, v in us.items()}
    ok = {a: {n: True for n in sizes} for a in us}
    rec = bench.auto_recommendation({"us_per_call": {}, "correct": {}},
                                    {"first_half_us_per_call": t, "first_half_correct": ok,
                                     "every_other_us_per_call": t, "every_other_correct": ok})
    row = rec["strided"]
    assert [row[b]["table"] for b in ("8B", "4KiB", "512KiB", "4MiB", "128MiB")] == \
        ["direct", "allreduce", "allreduce", "rccl", "rccl"]
    assert row["8B"]["fastest"] == "signal"
    assert rec["env"]["SHMEMX_AUTO_PARTIAL"] == "0:direct,181:allreduce,1482910:rccl"
