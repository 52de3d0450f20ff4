"""bench.py's JSON line (the driver's contract) from synthetic timings, no GPU: the keys the
driver reads, whole-job throughput, the roofline object (busy-union rate averaged over
GPUs, frac against the 8 TB/s spec and against the measured read peak, PMC traffic only at
N = 1), and the exchange summary."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(steps=100, warmup=10):
    return argparse.Namespace(steps=steps, warmup=warmup, seed=1234)


def _cfg(name="c2"):
    cfg = dict(bench.CONFIGS[name])
    cfg["config"] = name
    return cfg


def test_contract_keys_and_throughput():
    cfg = _cfg()
    alg = 4299227136.0
    # one GPU: 100 launches of 0.6 ms each, back to back (busy 60 ms), 0.1 s wall
    out = bench.report(_args(), cfg, 1, 0.1, [(100, 60.0, 100 * alg, 60.0)],
                       {"measured_read_peak": 7200.0, "exchange": None})
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in out, k
    assert out["value"] == 1000.0 and out["ms_per_step"] == 1.0 and out["n_gpus"] == 1
    assert out["vs_baseline"] is None and out["higher_is_better"] is True and out["dtype"] == "f32"
    assert "workload" in out["config"]
    r = out["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["achieved"] - alg / 0.6e-3 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-3
    assert r["measured_read_peak"] == 7200.0
    assert abs(r["frac_of_measured_read_peak"] - r["achieved"] / 7200.0) < 1e-3
    assert r["traffic"] is None or r["traffic"] > alg  # PMC file (profiles/) when present
    # c2 times one launch in 8, lowered so that >= 16 launches are timed (100 steps: 1 in 6;
    # the driver's 20-step line: every launch)
    assert r["timing_sample_period"] == 6 and "one in every 6 launches" in r["avg_launch_ms_source"]
    assert bench.timing_period(_args(steps=20), cfg) == 1 and bench.timing_period(_args(steps=300), cfg) == 8
    out5 = bench.report(_args(), _cfg("c5"), 1, 0.1, [(100, 60.0, 100 * alg, 60.0)], {})
    assert out5["roofline"]["timing_sample_period"] == 1 and "every launch" in out5["roofline"]["avg_launch_ms_source"]


def test_c1_samples_its_timing_events():
    """c1 (latency-bound) brackets one launch in 16 with the HIP events; --timing-period
    overrides it; the roofline says which."""
    cfg = _cfg("c1")
    out = bench.report(_args(steps=3000), cfg, 1, 0.1, [(7, 0.1, 7 * 6.4e6, 0.1)], {})
    r = out["roofline"]
    assert r["timing_sample_period"] == 16 and "one in every 16 launches" in r["avg_launch_ms_source"]
    a = _args()
    a.timing_period = 1
    assert bench.timing_period(a, cfg) == 1 and bench.timing_period(_args(steps=300), _cfg("c2")) == 8
    # a short c1 line still leaves every other launch pre-armable: never below 2
    assert bench.timing_period(_args(steps=20), cfg) == 2 and bench.timing_period(_args(steps=100), cfg) == 6


def test_multi_gpu_rate_is_per_gpu_average_and_no_traffic():
    cfg = _cfg()
    per = [(50, 10.0, 50 * 1e9, 10.0), (50, 20.0, 50 * 1e9, 20.0)]
    out = bench.report(_args(), cfg, 2, 0.05, per, {})
    r = out["roofline"]
    assert abs(r["achieved"] - (5000.0 + 2500.0) / 2) < 0.1
    assert r["traffic"] is None
    assert out["n_gpus"] == 2 and out["value"] == 2000.0


def test_exchange_summary():
    assert bench.exchange_report((0, 0.0, 0.0)) is None
    x = bench.exchange_report((200, 1.74, 200 * 32768.0))
    assert x["launches"] == 200 and x["avg_us"] == 8.7
    assert x["remote_bytes_per_launch"] == 32768.0
    assert abs(x["remote_GBps"] - 200 * 32768.0 / 1.74e-3 / 1e9) < 1e-3


def test_provenance_fields():
    """the traffic figure names its source file (it is not measured in the
    bench run), the launch time names its source, and the rocprof average of the committed
    summary sits beside it with the fraction it implies."""
    cfg = _cfg()
    alg = 4299227136.0
    out = bench.report(_args(), cfg, 1, 0.1, [(100, 60.0, 100 * alg, 60.0)], {})
    r = out["roofline"]
    assert "HIP events" in r["avg_launch_ms_source"]
    if r["traffic"] is not None:
        assert r["traffic_source"].startswith("profiles/lsq_pmc_c2.json") and "not this run" in r["traffic_source"]
    # figures of an earlier traced run sit in their own sub-object, never beside
    # this run's measurements, with the tree they were taken on
    assert "rocprof_avg_launch_ms" not in r and "rocprof_frac" not in r
    cp = r.get("committed_profiles")
    assert cp is not None  # profiles/r03_c2_rocprof_window.json is committed
    ms = cp["rocprof_avg_launch_ms"]
    assert cp["source"].startswith("profiles/") and cp["tree_commit"]
    assert abs(cp["rocprof_frac"] - alg / (ms / 1e3) / 1e9 / 8000.0) < 1e-3


def test_cpu_baseline_records_host(monkeypatch, tmp_path):
    """cpu_baseline: `cores` = the threads used, plus the host's logical CPU count and model."""
    import json
    import subprocess
    exe = tmp_path / "cpu_baseline"
    exe.write_text("#!/bin/sh\necho '%s'\n" % json.dumps({"it_per_s": 50.0, "threads": 9, "epochs": 600, "seconds": 12.0,
                                                       "workers": 8, "alg_GBps": 215.0}))
    exe.chmod(0o755)
    real_run = subprocess.run
    monkeypatch.setattr(bench.os.path, "exists", lambda p: True)
    monkeypatch.setattr(bench.subprocess, "run", lambda cmd, **kw: real_run([str(exe)] + cmd[1:2], **kw))
    cb = bench.cpu_baseline(_cfg(), 1.0)
    assert cb["cores"] == 9 and cb["threads"] == 9 and cb["kind"] == "port"
    assert cb["host_cores"] == os.cpu_count()
    assert cb["host_cpu_model"] is None or isinstance(cb["host_cpu_model"], str)


def test_gen_shards_empty_worker_list():
    """a rank that serves no worker (c1's 3 workers on 4 or 8 ranks) gets []."""
    assert bench.gen_shards(None, None, _cfg("c1"), 1, []) == []
    for world in (4, 8):
        placement = [(w * world) // 3 for w in range(3)]
        empty = [r for r in range(world) if r not in placement]
        assert empty  # such ranks exist and must not crash


def test_trace_window_skips_launches_after_the_timed_region(tmp_path):
    """tools/trace_window.py averages the `launches` dispatches of the timed region: the ones
    before the bench's `launches_after_timed` (c5: waitall releases a held 1-task re-dispatch
    after the timed region; taking the last `launches` dispatches included it)."""
    import json
    import subprocess
    durations = [9.0, 8.5, 8.4, 8.4, 8.6, 1.2]  # warm-up, 4 timed, then the released 1-task launch
    with open(tmp_path / "trace.csv", "w") as f:
        f.write("Kernel_Name,Start_Timestamp,End_Timestamp\n")
        t = 0
        for d in durations:
            f.write('"mpa::lsqp4_kernel(mpa::LsqpBatch)",%d,%d\n' % (t, t + int(d * 1e6)))
            t += int(d * 1e6) + 1000
    line = {"steps": 4, "roofline": {"launches": 4, "avg_launch_ms": 8.475}, "launches_after_timed": 1}
    (tmp_path / "bench.log").write_text("progress\n" + json.dumps(line) + "\n")
    out = tmp_path / "w.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "trace_window.py"), "--trace",
                           str(tmp_path / "trace.csv"), "--bench-log", str(tmp_path / "bench.log"), "--kernel",
                           "lsqp4_kernel", "--out", str(out)])
    w = json.loads(out.read_text())
    assert w["launches"] == 4 and w["launches_after_timed"] == 1
    assert abs(w["avg_ms"] - (8.5 + 8.4 + 8.4 + 8.6) / 4) < 1e-9


def test_c1_mpi_cpu_baseline_runs():
    """bench.py's c1 CPU baseline (kind "mpi"): the restated coordinator and 3 worker
    processes over MPICH run the configs[0] descent and report their rate and cores."""
    import importlib.util
    if not os.path.exists("/opt/conda/bin/mpiexec"):
        pytest.skip("MPICH not present")
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    cfg = dict(b.CONFIGS["c1"], config="c1")
    r = b.mpi_baseline(cfg, 1)
    assert r["kind"] == "mpi" and r["value"] > 100 and r["processes"] == 4 and r["cores"] == 4, r
    assert "3 worker processes over MPICH" in r["sample"]


def test_c5_reports_its_matrix_core_side():
    """The batched variant's line carries its MFMA figures beside the HBM roofline: two bf16
    products (4 * rows * cols * k flops per task) at the HBM-measured rate, lsqp4 issuing 1.5x
    that (phase 2 multiplies the hi and the lo halves of the residual), against the dense bf16
    peak; the other configs carry none."""
    cfg = _cfg("c5")
    task = 4429971456.0  # one c5 task's algorithmic bytes
    out = bench.report(_args(), cfg, 1, 1.0, [(100, 745.0, 100 * 8 * task, 745.0)], {})
    r = out["roofline"]
    m = r["mfma"]
    flops_task = 4.0 * (1 << 20) * 2048 * 64
    alg_tf = 8 * flops_task / 7.45e-3 / 1e12
    assert abs(m["alg_TFLOPs"] - alg_tf) < 0.5 and abs(m["issued_TFLOPs"] - 1.5 * alg_tf) < 0.5
    assert m["peak_TFLOPs"] == 2500.0 and abs(m["frac_issued"] - 1.5 * alg_tf / 2500.0) < 1e-3
    assert abs(r["frac"] - 8 * task / 7.45e-3 / 1e9 / 8000.0) < 1e-3
    assert "mfma" not in bench.report(_args(), _cfg("c2"), 1, 0.1, [(100, 60.0, 100 * 4299227136.0, 60.0)], {})["roofline"]
