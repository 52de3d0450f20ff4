"""Benchmark of the asyncmap! hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1..c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
(`bench.py --gpus N` alone starts the N ranks itself, under torch.distributed.run as a child
process, and relays rank 0's line.)

One step = one coordinator epoch of the least-squares example on BASELINE configs[1] ("c2"):
    repochs = asyncmap!(pool, x, recvbuf, isendbuf, irecvbuf, comm; nwait=8)
    x -= eta * (n / #fresh) * sum_{repochs[i]==epoch} g_i          (device kernel)
with 8 logical workers, A 2^20 x 1024 fp32 row-sharded (512 MiB per worker).  At N = 1 the
8 workers are stream-workers of one GPU; at N > 1 the same 8 workers (same global problem:
strong scaling) are placed 8/N per GPU, one process per GPU, rank 0 coordinating through
shared-memory mailboxes.  Inputs are generated on the device
(Philox) and resident in HBM before the timed region.  `value` is
iterations/sec of the whole job (K / max over ranks of the timed region).

Rank 0 prints one JSON line with the roofline of the dominant kernel (lsq_grad_kernel, HIP
events on the stream it runs on, all ranks) and, at N = 1, the CPU baseline
(oracle/cpu_baseline: the C restatement of the reference's coordinator + worker threads).
"""
import argparse
import json
import os
import subprocess
import sys
import time
import uuid

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))

import numpy as np  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; the sparse headline is 2x)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "iterations/sec + shard-kernel HBM GB/s (% peak), nwait=k of 1/2/4/8 GPUs"

CONFIGS = {
    # the reference's own CPU example restated on the device: coordinator + 3 workers,
    # nwait = 2 (examples/iterative_example.jl structure; latency-bound)
    # timing_period: one launch in 16 (c1) / 8 (c2) carries the HIP timing events (their host
    # cost sits on c1's critical path; c2 +1.3 %, profiles/r03_c1_timing_ab.txt); the few-epoch
    # configs c3-c5 time every launch
    "c1": dict(rows=3 << 12, cols=64, workers=3, nwait=2, dtype="f64", timing_period=16,
               desc="BASELINE configs[0] shape: 3 workers, fp64 least squares A 3*2^12 x 64, nwait=2 (latency-bound)"),
    "c2": dict(rows=1 << 20, cols=1024, workers=8, nwait=8, dtype="f32", timing_period=8,
               desc="BASELINE configs[1]: fp32 least squares A 2^20x1024 row-sharded over 8 logical workers, "
                    "nwait=8 (no stragglers); 1 GPU = 8 stream-workers, N GPUs = 8/N workers per GPU"),
    # the other BASELINE configs at their full global size, 8 workers on ONE GPU (secondary
    # measurements and parity cases; the default bench line is c2)
    "c3": dict(rows=1 << 23, cols=2048, workers=8, nwait=6, dtype="f32", delay_mean_ms=1.0,
               desc="BASELINE configs[2] shape: fp32 A 2^23x2048 (8 GiB per worker), nwait=6, "
                    "injected Exp(1 ms) straggler delays per (worker, task)"),
    "c4": dict(rows=1 << 23, cols=2048, workers=8, nwait="worker1+5", dtype="f64", delay_mean_ms=1.0,
               stale_weight=0.5,
               desc="BASELINE configs[3] shape: fp64 A 2^23x2048 (16 GiB per worker), nwait = "
                    "worker 1 fresh + 5 others (test/kmap2.jl:65 style predicate), stale results folded in "
                    "at weight 0.5, Exp(1 ms) delays"),
    # measurement shapes, not bench lines: c3's / c4's tasks with nwait = n and no delays, one
    # batched launch per epoch, so the kernel line is the shard kernel's own roofline
    "c3k": dict(rows=1 << 23, cols=2048, workers=8, nwait=8, dtype="f32", timing_period=1,
                desc="measurement: c3's fp32 2^23x2048 tasks, nwait=8, no delays (kernel roofline)"),
    "c4k": dict(rows=1 << 23, cols=2048, workers=8, nwait=8, dtype="f64", timing_period=1,
                desc="measurement: c4's fp64 2^23x2048 tasks, nwait=8, no delays (kernel roofline)"),
    "c5": dict(rows=1 << 23, cols=2048, workers=8, nwait=7, dtype="bf16", iterates=64,
               desc="BASELINE configs[4] shape: batched 64-iterate variant, bf16 A 2^23x2048 "
                    "(4 GiB per worker), X 2048x64, fp32 accumulate (MFMA), nwait=7"),
}
# measurement shapes, not bench lines: ONE GPU's share of the node's run,
# i.e. the launch each GPU runs per epoch at N = 2 / 4 / 8 (8/N of the 8 workers of the same
# global problem, one batched launch of their tasks), nwait = n and no delays, so the line is
# that launch's own roofline and the denominator of DESIGN.md §5's scaling budget
for _base, _ns in (("c2", (2, 4, 8)), ("c3", (8,)), ("c4", (8,)), ("c5", (8,))):
    for _n in _ns:
        _c = dict(CONFIGS[_base])
        _w = 8 // _n
        _c.update(rows=_c["rows"] // _n, workers=_w, nwait=_w, timing_period=1)
        for _k in ("delay_mean_ms", "stale_weight"):
            _c.pop(_k, None)
        _c["desc"] = ("measurement: one GPU's share of %s at N = %d (%d task(s) of %d rows x %d %s per launch, "
                      "nwait = n, no delays)" % (_base, _n, _w, _c["rows"] // _w, _c["cols"], _c["dtype"]))
        CONFIGS["%sn%d" % (_base, _n)] = _c


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--timing-period", type=int, default=None,
                   help="time one in every k launches with HIP events (default: the config's, 1 or 16 for c1)")
    p.add_argument("--dry-run", action="store_true",
                   help="exercise the launcher, rank placement and max-over-ranks report with no GPU work "
                        "(tests/test_bench_launch.py)")
    return p.parse_args()


def host_cpu():
    """(logical CPUs of the host, CPU model name) for the cpu_baseline record."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count(), model


def cpu_baseline(cfg, seconds):
    """oracle/cpu_baseline (kind "port"): same state machine, n worker threads, fp32."""
    exe = os.path.join(ROOT, "oracle", "_build", "cpu_baseline")
    if not os.path.exists(exe):
        try:
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
        except Exception as e:
            return {"value": None, "unit": "iterations/s", "error": f"build failed: {e}"[:200]}
    cmd = [exe, "--workers", str(cfg["workers"]), "--rows", str(cfg["rows"]), "--cols", str(cfg["cols"]),
           "--nwait", str(cfg["nwait"]), "--seconds", str(seconds)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 4 + 240, check=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # report, never fake
        return {"value": None, "unit": "iterations/s", "error": str(e)[:200]}
    host_cores, host_model = host_cpu()
    return {"value": round(r["it_per_s"], 4), "unit": "iterations/s", "cores": r["threads"], "kind": "port",
            "threads": r["threads"], "host_cores": host_cores, "host_cpu_model": host_model,
            "sample": f"{r['epochs']} epochs in {r['seconds']:.1f} s of the full {cfg['config']} problem "
                      f"({r['workers']} worker threads + 1 coordinator thread, fp32, AVX2 loops, same state "
                      f"machine); {r['alg_GBps']:.1f} GB/s algorithmic"}


def mpi_baseline(cfg, seconds):
    """oracle/_build/mpi_lsq_baseline (kind "mpi"): BASELINE configs[0] as the reference runs
    it, the restated coordinator (src/MPIAsyncPools.jl over MPI's own verbs) and one worker
    PROCESS per worker computing its fp64 shard gradient, under MPICH's mpiexec."""
    exe = os.path.join(ROOT, "oracle", "_build", "mpi_lsq_baseline")
    mpi_dir = os.environ.get("MPI_DIR", "/opt/conda")
    mpiexec = os.path.join(mpi_dir, "bin", "mpiexec")
    if not os.path.exists(exe) and os.path.exists(os.path.join(mpi_dir, "include", "mpi.h")):
        try:
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "mpi", f"MPI_DIR={mpi_dir}"])
        except Exception as e:
            return {"value": None, "unit": "iterations/s", "error": f"build failed: {e}"[:200]}
    if not (os.path.exists(exe) and os.path.exists(mpiexec)):
        return {"value": None, "unit": "iterations/s", "error": "MPICH (mpiexec, mpi.h) not present on this host"}
    cmd = [mpiexec, "-n", str(cfg["workers"] + 1), exe, "--rows", str(cfg["rows"]), "--cols", str(cfg["cols"]),
           "--nwait", str(cfg["nwait"]), "--seconds", str(int(seconds))]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 4 + 120, check=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # report, never fake
        return {"value": None, "unit": "iterations/s", "error": str(e)[:200]}
    host_cores, host_model = host_cpu()
    return {"value": round(r["it_per_s"], 4), "unit": "iterations/s", "cores": r["processes"], "kind": "mpi",
            "processes": r["processes"], "host_cores": host_cores, "host_cpu_model": host_model,
            "sample": f"{r['epochs']} epochs in {r['seconds']:.1f} s of the full {cfg['config']} problem: 1 coordinator "
                      f"+ {r['workers']} worker processes over MPICH (mpiexec), the restated asyncmap! with MPI's own "
                      f"verbs, fp64 shard gradients, nwait={r['nwait']}"}


def step_size(rows, cols):
    """0.9 / L with L ~ ||A||^2 for U(-1,1)/sqrt(cols) entries."""
    L = rows / (3.0 * cols) * (1.0 + np.sqrt(cols / rows)) ** 2
    return 0.9 / L


TORCH_DT = {"f32": "float32", "f64": "float64", "bf16": "bfloat16"}


_T0 = time.perf_counter()


def progress(msg):
    """A line on stderr per phase: long configs (c3-c5 generate 32-128 GiB) never go silent."""
    print("[bench %.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def gen_shards(M, torch, cfg, seed, workers):
    """Rows of the given workers (1-based, consecutive) of the global synthetic problem on
    the current GPU, as row-range VIEWS of one allocation per GPU (the row-sharded A of
    BASELINE configs[1]; b: rows, the batched variant's B: rows x 64).  Against one fresh
    allocation per shard the layouts measured within run-to-run noise, the joint one the
    steadier on c2 (profiles/r01_shard_alloc_ab.txt); MPA_BENCH_SEPARATE=1 restores one
    allocation per shard for that A/B."""
    workers = list(workers)
    if not workers:  # a rank that serves no worker (c1's 3 workers over N = 4 or 8 ranks)
        return []
    n, rows, cols = cfg["workers"], cfg["rows"], cfg["cols"]
    per = rows // n
    dt = getattr(torch, TORCH_DT[cfg["dtype"]])
    k = cfg.get("iterates", 1)
    scale = 1.0 / np.sqrt(cols) if cfg["dtype"] == "f64" else float(np.float32(1.0 / np.sqrt(cols)))
    assert workers == list(range(workers[0], workers[0] + len(workers))), workers
    if os.environ.get("MPA_BENCH_SEPARATE") == "1":
        views = [(torch.empty(per, cols, dtype=dt, device="cuda"),
                  torch.empty((per, k) if k > 1 else per, dtype=dt, device="cuda")) for _ in workers]
    else:
        A = torch.empty(per * len(workers), cols, dtype=dt, device="cuda")
        b = torch.empty((per * len(workers), k) if k > 1 else per * len(workers), dtype=dt, device="cuda")
        views = [(A[j * per:(j + 1) * per], b[j * per:(j + 1) * per]) for j in range(len(workers))]
    for w, (Aw, bw) in zip(workers, views):
        M.generate(Aw, seed, 0, (w - 1) * per * cols, scale)
        M.generate(bw, seed, 1, (w - 1) * per * k, 1.0)
    return views


def delay_schedule(cfg, seed, w, count=4096):
    """Exp(mean) straggler delay per (worker, task), seeded (stored with the results)."""
    mean = cfg.get("delay_mean_ms")
    if not mean:
        return None
    rng = np.random.default_rng([seed, w])
    return (rng.exponential(mean * 1e6, size=count)).astype(np.int64)


def kernel_name(cfg):
    if cfg.get("iterates", 1) > 1:
        v = os.environ.get("MPA_LSQP", "1")
        if v == "8" and cfg["cols"] <= 2048:
            return "lsqp_kernel (bf16 MFMA single pass by iterate halves, eight waves, one launch per batch)"
        if v != "0" and cfg["cols"] <= 2048:
            return "lsqp4_kernel (bf16 MFMA single pass by iterate halves, one wave per SIMD, one launch per batch)"
        return "lsqb_resid_kernel + lsqb_grad_kernel (bf16 MFMA, two launches per batch)"
    return "lsq_grad_kernel (one batched launch per epoch per GPU)"


def read_peak(M, torch, nbytes=1 << 32):
    """Measured HBM read ceiling of this GPU (mpa_read_bandwidth): a plain non-temporal
    streaming read of a 4 GiB buffer (or `nbytes`: one launch's bytes of a per-GPU measurement
    config) at four grid sizes, best of them, outside the timed region.  Reported beside the spec
    peak so the roofline fraction can be read against what a read-only kernel reaches on the same
    box."""
    buf = torch.empty(int(nbytes) // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    best = max(M.read_bandwidth(buf, grid=g, reps=10) for g in (192, 512, 1024, 2048, 4096))
    del buf
    torch.cuda.empty_cache()
    return round(best, 1)


def exchange_report(xt):
    """The coordinator's epoch kernels in the timed region (mpa_comm_exchange_timing): the
    broadcast of the iterate to the idle workers and the gather of their replies happen
    inside them; `remote_*` counts the bytes that crossed to other processes' GPUs (over
    xGMI at N > 1; 0 at N = 1).  Payloads are cols x 4 B per worker, so the rate is
    latency-bound, not link-bound (xGMI ~153 GB/s per link)."""
    launches, ms, remote = xt
    if not launches:
        return None
    return {"kernel": "epoch_kernel (harvest + iterate update + dispatch, coordinator GPU)",
            "launches": launches, "avg_us": round(ms / launches * 1e3, 2),
            "remote_bytes_per_launch": remote / launches,
            "remote_GBps": round(remote / (ms / 1e3) / 1e9, 3) if ms > 0 else None}


def timing_period(args, cfg):
    """HIP events on one launch in k: the config's k, lowered so that a short run still times
    at least 16 launches (a 20-step c2 line at 1 in 8 timed only 3), but
    never below 2 on a k-of-n config (c1): with every launch timed the transport pre-arms none
    (transport_hip.cpp maybe_prearm), so a short line would measure another path than the
    shipped one.  nwait = n configs (c2) never pre-arm: every launch may be timed."""
    if getattr(args, "timing_period", None):
        return args.timing_period
    k = cfg.get("timing_period", 1)
    steps = getattr(args, "steps", None)
    if steps:
        floor = 2 if k > 1 and cfg["nwait"] != cfg["workers"] else 1
        k = max(floor, min(k, steps // 16))
    return k


def report(args, cfg, world, el, per_rank, extra):
    """per_rank: (launches, summed kernel ms, algorithmic bytes, busy ms) of each GPU.
    roofline.achieved = algorithmic bytes / busy time (the union of the launch intervals, so
    concurrent single-task launches of delayed workers are not double counted), averaged
    over the GPUs; avg_launch_ms = summed kernel ms / launches."""
    its = args.steps / el
    tp = timing_period(args, cfg)
    n, rows, cols = cfg["workers"], cfg["rows"], cfg["cols"]
    kl = sum(p[0] for p in per_rank)
    kms = sum(p[1] for p in per_rank)
    kbytes = sum(p[2] for p in per_rank)
    rates = [p[2] / (p[3] / 1e3) / 1e9 for p in per_rank if p[0] and p[3] > 0]
    achieved = sum(rates) / len(rates) if rates else None
    per_launch_bytes = kbytes / max(kl, 1)
    per_launch_s = kms / 1e3 / max(kl, 1)
    # HBM traffic per launch: NOT measured in this run (PMC counters need their own
    # rocprofv3 --pmc passes: tools/gpu.sh pmc, tools/pmc_summarize.py); read from the committed summary of the
    # same command and labelled with its file and date
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", f"lsq_pmc_{cfg['config']}.json")
    if os.path.exists(pmc) and world == 1:
        try:
            d = json.load(open(pmc))
            # per launch of THIS run: the measured traffic / algorithmic-bytes ratio times this
            # run's mean algorithmic bytes per launch (launches of the c5 bench carry 1, 7 or 8
            # tasks, so the summary is per task there)
            traffic = round(d["traffic_over_alg"] * per_launch_bytes, 1) if d.get("traffic_over_alg") else None
            traffic_src = "%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py, %s; not this run)" % (
                os.path.relpath(pmc, ROOT), d.get("date", "round-1 box"))
        except Exception:
            traffic = None
    # the same kernel's average duration in the committed rocprofv3 --kernel-trace --stats
    # summary of this command (profiles/), beside the in-process HIP-event figure
    rocprof = rocprof_avg_ms(cfg) if world == 1 else None
    es = {"f32": 4, "f64": 8, "bf16": 2}[cfg["dtype"]]
    k = cfg.get("iterates", 1)
    epoch_bytes = es * (rows * cols + rows * k) + n * cols * k * (es + (4 if k > 1 else es))
    cfg_out = {"workload": cfg["desc"], "rows": rows, "cols": cols, "workers": n, "nwait": cfg["nwait"],
               "shard_bytes": rows // n * cols * es, "parallelism": f"{n} logical workers on {world} GPU(s)"}
    if k > 1:
        cfg_out["iterates"] = k
    if cfg.get("delay_mean_ms"):
        cfg_out["delays"] = f"Exp(mean {cfg['delay_mean_ms']} ms) per (worker, task), seed {args.seed}"
    out = {
        "metric": METRIC,
        "value": round(its, 3),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": cfg["dtype"],
        "data": "synthetic (Philox4x32-10 generated on device, DESIGN.md §Data)",
        "config": cfg_out,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": kernel_name(cfg),
                     "alg_bytes_per_launch": per_launch_bytes, "avg_launch_ms": round(per_launch_s * 1e3, 4),
                     "avg_launch_ms_source": "HIP events recorded around %s on the stream it runs on "
                                             "(this run, timed region only); achieved = alg bytes / busy ms" % (
                                                 "every launch" if tp == 1 else "one in every %d launches" % tp),
                     "timing_sample_period": tp,
                     "launches_total": extra.pop("launches_total", None),
                     "launches": kl, "busy_ms": round(sum(p[3] for p in per_rank), 3)},
        "epoch_alg_GBps": round(epoch_bytes * its / 1e9, 1),
    }
    if rocprof:
        # figures of an EARLIER traced run of this command, kept apart from this run's
        # measurements and labelled with the tree they were taken on (they go stale
        # silently when the kernel changes)
        avg_ms, src, tree = rocprof
        out["roofline"]["committed_profiles"] = {
            "rocprof_avg_launch_ms": avg_ms, "source": src, "tree_commit": tree,
            "rocprof_frac": round(per_launch_bytes / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)}
    if k > 1 and achieved:
        # the batched variant's matrix-core side of the same launches: G = A^T (A X - B) is two
        # bf16 products, 2 * 2 * rows * cols * k flops per task; lsqp4 issues 1.5x that (phase 2
        # multiplies the hi and the lo bf16 halves of the fp32 residual, lsqp4_kernel.hip)
        rt = rows // n
        task_bytes = 2 * rt * cols + 2 * rt * k + 2 * cols * k + 4 * cols * k
        flop_per_byte = 4.0 * rt * cols * k / task_bytes
        alg_tf = achieved * 1e9 * flop_per_byte / 1e12
        out["roofline"]["mfma"] = {
            "alg_TFLOPs": round(alg_tf, 1), "issued_TFLOPs": round(1.5 * alg_tf, 1), "peak_TFLOPs": MFMA_BF16_PEAK_TFLOPS,
            "frac_alg": round(alg_tf / MFMA_BF16_PEAK_TFLOPS, 4), "frac_issued": round(1.5 * alg_tf / MFMA_BF16_PEAK_TFLOPS, 4),
            "note": "dense bf16 peak at 2.4 GHz (MI355X_MICROARCH.md); the 8-task launch holds 1.66 GHz in-kernel "
                    "(power-limited, profiles/r05_c5_clock.txt), i.e. a clock-scaled peak of ~1730 TFLOP/s"}
    rp = extra.pop("measured_read_peak", None)
    if rp:
        out["roofline"]["measured_read_peak"] = rp
        out["roofline"]["frac_of_measured_read_peak"] = round(achieved / rp, 4) if achieved else None
    rpl = extra.pop("measured_read_peak_launch_bytes", None)
    if rpl:
        out["roofline"]["measured_read_peak_launch_bytes"] = rpl
        out["roofline"]["frac_of_measured_read_peak_launch_bytes"] = round(achieved / rpl, 4) if achieved else None
    out.update(extra)
    return out


ROCPROF_STATS = {"c2": ("%s_c2_kernel_stats.csv", "lsq_grad_kernel"),
                 "c5": ("%s_c5_kernel_stats.csv", "lsqp4_kernel")}
PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02")   # newest first


def rocprof_avg_ms(cfg):
    """(average ms, source, tree commit) of the dominant kernel under rocprofv3 in the committed
    profiles of this config's bench command: the timed-region window of its kernel trace
    (tools/trace_window.py) of the newest round that has one, else the --stats summary; None
    without either."""
    pattern, kernel = ROCPROF_STATS.get(cfg["config"], (None, None))
    name = None
    for rnd in PROFILE_ROUNDS:
        if pattern and os.path.exists(os.path.join(ROOT, "profiles", pattern % rnd)):
            name = pattern % rnd
            break
    for rnd in PROFILE_ROUNDS:
        win = os.path.join(ROOT, "profiles", "%s_%s_rocprof_window.json" % (rnd, cfg["config"]))
        if pattern and os.path.exists(win):
            d = json.load(open(win))
            if d.get("kernel") == kernel:
                return round(d["avg_ms"], 4), "profiles/%s (last %d launches of the traced run = its timed region; %s)" % (
                    os.path.basename(win), d["launches"], d.get("date", "")), d.get("tree_commit")
    path = os.path.join(ROOT, "profiles", name) if name else None
    if not path or not os.path.exists(path):
        return None
    import csv
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                return round(float(row["AverageNs"]) / 1e6, 4), "profiles/%s (%s calls)" % (name, row["Calls"]), None
    return None


def _nwait(M, cfg):
    nw = cfg["nwait"]
    if isinstance(nw, str) and nw.startswith("worker1+"):
        return M.first_plus(int(nw.split("+")[1]))
    return nw


def register(comm, cfg, seed, w, A, b):
    """Task (and injected delay schedule) of worker w on the process that serves it."""
    if cfg.get("iterates", 1) > 1:
        comm.set_task_lsq_batch(w, A, b)
    else:
        comm.set_task_lsq(w, A, b)
    d = delay_schedule(cfg, seed, w)
    if d is not None:
        comm.set_delays(w, d)


def max_msg_bytes(cfg):
    es = {"f32": 4, "f64": 8, "bf16": 2}[cfg["dtype"]]
    k = cfg.get("iterates", 1)
    return cfg["cols"] * k * (4 if k > 1 else es)  # the reply is the larger payload


def make_loop(M, torch, cfg, pool, comm):
    """(loop(steps), x): the native coordinator loop of this config on rank 0's buffers."""
    n, cols, k = cfg["workers"], cfg["cols"], cfg.get("iterates", 1)
    nwait = _nwait(M, cfg)
    eta = step_size(cfg["rows"], cols)
    stale = cfg.get("stale_weight", 0.0)
    if k > 1:
        x = torch.zeros(cols * k, device="cuda")          # fp32 master iterate X (cols x 64)
        xb = torch.zeros(cols * k, dtype=torch.bfloat16, device="cuda")  # its bf16 message
        isend = torch.zeros(n * cols * k, dtype=torch.bfloat16, device="cuda")
        recv = torch.zeros(n * cols * k, device="cuda")
        irecv = torch.zeros_like(recv)

        def loop(steps):
            M.lsqb_descent(pool, comm, x, xb, recv, isend, irecv, nwait, eta, steps, stale_weight=stale)
    else:
        dt = getattr(torch, TORCH_DT[cfg["dtype"]])
        x = torch.zeros(cols, dtype=dt, device="cuda")
        isend = torch.zeros(n * cols, dtype=dt, device="cuda")
        recv = torch.zeros(n * cols, dtype=dt, device="cuda")
        irecv = torch.zeros_like(recv)

        def loop(steps):
            M.lsq_descent(pool, comm, x, recv, isend, irecv, nwait, eta, steps, stale_weight=stale)
    loop.bufs = (x, recv, isend, irecv)
    return loop, x


def run_single(args, cfg):
    import torch
    import mpiasyncpools as M

    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    n, cols = cfg["workers"], cfg["cols"]
    nwait = _nwait(M, cfg)
    k = cfg.get("iterates", 1)
    batched = k > 1
    if os.environ.get("MPA_BENCH_LSQ_GRID"):
        # measurement knob (grid sweeps on the product library): workgroups per least-squares
        # launch, mpa_tune("lsq_grid"); the line says so in its workload
        G = int(os.environ["MPA_BENCH_LSQ_GRID"])
        if M.lib().mpa_tune(b"lsq_grid", G) != 0:
            raise SystemExit("mpa_tune lsq_grid %d refused" % G)
        cfg["desc"] = "lsq_grid %d (MPA_BENCH_LSQ_GRID, not the shipped grid): " % G + cfg["desc"]
    comm = M.DeviceComm(n)
    shards = gen_shards(M, torch, cfg, args.seed, range(1, n + 1))
    torch.cuda.synchronize()
    progress("generated %d shards (%s)" % (n, cfg["config"]))
    for w, (A, b) in enumerate(shards, start=1):
        register(comm, cfg, args.seed, w, A, b)
    pool = M.MPIAsyncPool(n)
    eta = step_size(cfg["rows"], cols)
    loop, x = make_loop(M, torch, cfg, pool, comm)
    _, recv, isend, irecv = loop.bufs
    extra = {}
    if cfg["config"] in ("c1", "c2"):
        # the same loop from Python (asyncmap_ + weights + lsq_update per step), reported beside:
        # what a caller driving asyncmap! itself per epoch (the reference's own loop) sees
        w = np.zeros(n)

        def step():
            rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=nwait)
            fresh = rep == pool.epoch
            nf = int(fresh.sum())
            w[:] = fresh * (n / nf if nf else 0.0)
            comm.lsq_update(x, recv, n, w, eta)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        extra["python_loop_it_per_s"] = round(args.steps / (time.perf_counter() - t0), 3)
    # timed region: the coordinator loop in native code (mpa_lsq_descent / mpa_lsqb_descent)
    loop(args.warmup)
    torch.cuda.synchronize()
    progress("warmup done (%d epochs)" % args.warmup)
    comm.timing()
    comm.set_timing(True, timing_period(args, cfg))
    steps0 = {k: comm.counter(k) for k in ("head_steps", "epoch_kernels", "prearmed", "prearm_cancelled", "prearm_same")}
    launches0 = comm.counter("task_launches")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    timing = comm.timing()
    # where the timed region's epoch steps ran: at the head of the task launch, as their own
    # epoch kernel (the rest ride in launch tails, launch-ahead at nwait = n)
    extra["epoch_steps"] = {k: comm.counter(k) - v for k, v in steps0.items()}
    extra["launches_total"] = comm.counter("task_launches") - launches0  # timed or not
    extra["exchange"] = exchange_report(comm.exchange_timing())
    fresh = int((pool.repochs == pool.epoch).sum())
    # launches after the timed region (waitall releases held stale re-dispatches): counted, so
    # that a kernel trace of this command can drop them from its timed-region window
    # (tools/trace_window.py)
    l_end = comm.counter("task_launches")
    M.waitall_(pool, recv, irecv)
    torch.cuda.synchronize()
    extra["launches_after_timed"] = comm.counter("task_launches") - l_end
    comm.timing()
    comm.set_timing(False)
    extra["measured_read_peak"] = read_peak(M, torch)
    if timing[0] and timing[2] / timing[0] < 3.5e9:
        # a launch smaller than the 4 GiB probe (the per-GPU shares c2n2 / c2n4 / c2n8): the
        # same read at that size, whose ramp and tail weigh as they do in the launch
        extra["measured_read_peak_launch_bytes"] = read_peak(M, torch, timing[2] / timing[0] // 4096 * 4096)
    extra.update({"x_norm": float(torch.linalg.norm(x.float()).item()), "build": M.lib().mpa_build_info().decode(),
                  "loop": "native coordinator loop (mpa_lsq%s_descent)" % ("b" if batched else ""),
                  "fresh_at_last_epoch": fresh})
    if cfg["config"] == "c2":
        extra["loop"] += "; python loop beside it"
    # the CPU beside the device: c2 threaded (the bench's headline config), c1 as the reference
    # runs configs[0] (coordinator + worker processes over MPI)
    extra["cpu_baseline"] = None
    if not args.no_cpu_baseline and cfg["config"] == "c2":
        extra["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    elif not args.no_cpu_baseline and cfg["config"] == "c1":
        extra["cpu_baseline"] = mpi_baseline(cfg, args.cpu_seconds)
    print(json.dumps(report(args, cfg, 1, el, [timing], extra)), flush=True)
    comm.shutdown()
    comm.close()
    torch.cuda.synchronize()


def run_multi(args, cfg, rank, world, local):
    """One process per GPU: rank 0 coordinates; every rank serves the workers placed on it."""
    import torch
    import torch.distributed as dist
    import mpiasyncpools as M

    # MPA_BENCH_ONE_GPU=1 rehearses the N-process path with every rank on GPU 0 (1-GPU box).
    # Round 3's device-armed tasks waited in every workgroup and could only time out there (their
    # grids held the CUs rank 0's step needed, profiles/r03_rehearsal_n248.txt); an armed task now
    # waits behind one wave (door_wait_kernel), so the rehearsal runs the node's default path too
    one_gpu = os.environ.get("MPA_BENCH_ONE_GPU") == "1"
    torch.cuda.set_device(0 if one_gpu else local)
    dist.init_process_group("gloo")
    n = cfg["workers"]
    placement = bench_placement(n, world)
    name = [f"/mpa_bench_{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
    if rank == 0:
        comm = M.DistComm(n, placement, 0, name[0], max_msg_bytes(cfg))
    dist.broadcast_object_list(name, src=0)
    if rank != 0:
        comm = M.DistComm(n, placement, rank, name[0], max_msg_bytes(cfg))
    mine = [w for w in range(1, n + 1) if placement[w - 1] == rank]
    keep = gen_shards(M, torch, cfg, args.seed, mine)
    for w, (A, b) in zip(mine, keep):
        register(comm, cfg, args.seed, w, A, b)
    torch.cuda.synchronize()
    if rank == 0:
        progress("generated rank 0's shards (%s, %d ranks)" % (cfg["config"], world))
    dist.barrier()
    if rank == 0:
        pool = M.MPIAsyncPool(n)
        loop, x = make_loop(M, torch, cfg, pool, comm)
        _, recv, isend, irecv = loop.bufs
        loop(args.warmup)
        M.waitall_(pool, recv, irecv)
        torch.cuda.synchronize()
        progress("warmup done (%d epochs)" % args.warmup)
        comm.pause_servers()
    else:
        comm.serve()  # warmup session, returns at pause_servers
    comm.timing()
    comm.set_timing(True, timing_period(args, cfg))
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    if rank == 0:
        loop(args.steps)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        fresh = int((pool.repochs == pool.epoch).sum())
        M.waitall_(pool, recv, irecv)
        comm.shutdown()
    else:
        comm.serve()  # timed session, returns at shutdown
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    timing = comm.timing()
    comm.set_timing(False)
    xch = exchange_report(comm.exchange_timing()) if rank == 0 else None
    dist.barrier()
    stats = [None] * world
    dist.all_gather_object(stats, (el, timing, os.getpid()))
    if rank == 0:
        el_max = max(s[0] for s in stats)
        paths = sorted({comm.payload_path(w) for w in range(1, n + 1) if placement[w - 1] != 0} - {None})
        extra = {"x_norm": float(torch.linalg.norm(x.float()).item()), "build": M.lib().mpa_build_info().decode(),
                 "fresh_at_last_epoch": fresh, "placement": placement, "payload_path": "/".join(paths) or None, "rank0_elapsed_s": round(stats[0][0], 6), "cpu_baseline": None,
                 "exchange": xch, "rank_pids": [s[2] for s in stats]}
        print(json.dumps(report(args, cfg, world, el_max, [s[1] for s in stats], extra)), flush=True)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()


def bench_placement(n, world):
    """8/N consecutive workers per rank; MPA_BENCH_PLACEMENT (rehearsals only, e.g. "0,0,0,0,0,0,0,1":
    rank 0 serves seven workers and rank 1 one, the per-remote-worker control path of the 8-GPU
    node's placement on a one-GPU box) overrides it."""
    env = os.environ.get("MPA_BENCH_PLACEMENT")
    if env:
        pl = [int(v) for v in env.split(",")]
        if len(pl) != n or sorted(set(pl)) != list(range(world)):
            raise SystemExit(f"MPA_BENCH_PLACEMENT {env!r}: {n} ranks in 0..{world - 1}, each used")
        return pl
    return [(w * world) // n for w in range(n)]


def run_dry(args, cfg, rank, world):
    """--dry-run: the launcher, the rank placement, the barrier-bracketed timed region and
    the max-over-ranks report, with the GPU work replaced by a rank-dependent sleep (CPU
    tests of the N-process path; nothing here imports torch.cuda or the HIP library)."""
    n = cfg["workers"]
    placement = [(w * world) // n for w in range(n)]
    mine = [w for w in range(1, n + 1) if placement[w - 1] == rank]
    if os.environ.get("MPA_BENCH_DRY_FAIL_RANK") == str(rank):  # tests: a failing rank's exit code is relayed
        raise SystemExit(3)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.002 * (1 + rank))  # the last rank is the slowest: max-over-ranks is visible
    el = time.perf_counter() - t0
    stats = [(el, mine)]
    if dist is not None:
        dist.barrier()
        stats = [None] * world
        dist.all_gather_object(stats, (el, mine))
    if rank == 0:
        el_max = max(s[0] for s in stats)
        extra = {"dry_run": True, "placement": placement, "rank_workers": [s[1] for s in stats],
                 "rank_elapsed_s": [round(s[0], 6) for s in stats], "cpu_baseline": None}
        print(json.dumps(report(args, cfg, world, el_max, [(0, 0.0, 0.0, 0.0)] * world, extra)), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started without a launcher: run the N ranks (one process
    per GPU) under torch.distributed.run as ONE child process, started before this process
    has touched the GPU (nothing above imports torch), relay rank 0's JSON line to stdout and
    return the child's exit code.  The ranks' stderr passes through."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    progress("launching %d ranks: %s" % (args.gpus, " ".join(cmd[1:6])))
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for out in p.stdout:
        if out.lstrip().startswith("{"):
            line = out.strip()
        else:
            sys.stderr.write(out)
    rc = p.wait()
    if line:
        print(line, flush=True)
    return rc


def main():
    args = parse()
    cfg = dict(CONFIGS[args.config])
    cfg["config"] = args.config
    if os.environ.get("MPA_BENCH_ROWS"):
        # rehearsals only (the control path with shards so small that the exchange runs alone):
        # the line says so in its workload and is never a BASELINE measurement
        cfg["rows"] = int(os.environ["MPA_BENCH_ROWS"])
        cfg["desc"] = "REHEARSAL (MPA_BENCH_ROWS=%d, not the BASELINE size): " % cfg["rows"] + cfg["desc"]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        run_dry(args, cfg, rank, world)
    elif world == 1:
        run_single(args, cfg)
    else:
        run_multi(args, cfg, rank, world, local)


if __name__ == "__main__":
    main()
