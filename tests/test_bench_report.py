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
