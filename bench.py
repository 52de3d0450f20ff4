"""Benchmark of the asyncmap! hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

One step = one coordinator epoch of the least-squares example (BASELINE configs[1], "c2"):
    repochs = asyncmap!(pool, x, recvbuf, isendbuf, irecvbuf, comm; nwait=k)
    x -= eta * (n / #fresh) * sum_{repochs[i]==epoch} g_i          (device kernel)
with 8 logical stream-workers, A 2^20 x 1024 fp32 row-sharded (512 MiB per worker),
nwait = 8.  Inputs are generated on the device (Philox) and resident in
HBM before the timed region.  `value` is iterations/sec of the whole job.

Rank 0 prints one JSON line with the roofline of the dominant kernel (lsq_grad_kernel,
HIP events on the stream it runs on) and the CPU baseline (oracle/cpu_baseline: the C
restatement of the reference's coordinator + worker threads, a bounded sample).
"""
import argparse
import json
import os
import subprocess
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")  # one HSA queue per stream

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

CONFIGS = {
    # name: rows (global), cols, workers, nwait, dtype
    "c2": dict(rows=1 << 20, cols=1024, workers=8, nwait=8, dtype="f32",
               desc="1xMI355X, 8 logical stream-workers, fp32 least squares A 2^20x1024 row-sharded, nwait=8"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def cpu_baseline(cfg, seconds):
    """oracle/cpu_baseline (kind "port"): same state machine, n worker threads, fp32."""
    exe = os.path.join(ROOT, "oracle", "_build", "cpu_baseline")
    if not os.path.exists(exe):
        try:
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
        except Exception:
            return None
    cmd = [exe, "--workers", str(cfg["workers"]), "--rows", str(cfg["rows"]), "--cols", str(cfg["cols"]),
           "--nwait", str(cfg["nwait"]), "--seconds", str(seconds)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 4 + 240, check=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # report, never fake
        return {"value": None, "unit": "iterations/s", "error": str(e)[:200]}
    return {"value": round(r["it_per_s"], 4), "unit": "iterations/s", "cores": r["threads"], "kind": "port",
            "sample": f"{r['epochs']} epochs in {r['seconds']:.1f} s of the full {cfg['config']} problem "
                      f"({r['workers']} worker threads + 1 coordinator thread, fp32, AVX2 loops); "
                      f"{r['alg_GBps']:.1f} GB/s algorithmic"}


def main():
    args = parse()
    cfg = dict(CONFIGS[args.config])
    cfg["config"] = args.config
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        import multigpu  # noqa: F401  (placed next to bench.py)
        return multigpu.run(args, cfg, rank, world, local)

    import torch
    import mpiasyncpools as M

    torch.cuda.set_device(local)
    n, rows, cols, nwait = cfg["workers"], cfg["rows"], cfg["cols"], cfg["nwait"]
    per = rows // n
    tdt = torch.float32
    es = 4
    A = torch.empty(rows, cols, dtype=tdt, device="cuda")
    b = torch.empty(rows, dtype=tdt, device="cuda")
    M.generate(A, args.seed, 0, 0, float(np.float32(1.0 / np.sqrt(cols))))
    M.generate(b, args.seed, 1, 0, 1.0)
    comm = M.DeviceComm(n)
    for r in range(1, n + 1):
        comm.set_task_lsq(r, A[(r - 1) * per:r * per], b[(r - 1) * per:r * per])
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=tdt, device="cuda")
    isend = torch.zeros(n * cols, dtype=tdt, device="cuda")
    recv = torch.zeros(n * cols, dtype=tdt, device="cuda")
    irecv = torch.zeros_like(recv)
    L = rows / (3.0 * cols) * (1.0 + np.sqrt(cols / rows)) ** 2
    eta = 0.9 / L
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
    comm.timing()  # discard warmup launches
    comm.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    launches, kms, kbytes = comm.timing()
    comm.set_timing(False)
    M.waitall_(pool, recv, irecv)
    el = t1 - t0
    its = args.steps / el
    alg_bytes_epoch = es * (rows * cols + rows + 2 * n * cols)
    per_launch_bytes = kbytes / max(launches, 1)
    per_launch_s = kms / 1e3 / max(launches, 1)
    achieved = per_launch_bytes / per_launch_s / 1e9 if launches else None
    xnorm = float(torch.linalg.norm(x).item())

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "lsq_pmc_c2.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "iterations/sec + shard-kernel HBM GB/s (% peak), nwait=k of 1/2/4/8 GPUs",
        "value": round(its, 3),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox4x32-10 on device, DESIGN.md §Data)",
        "config": {"workload": cfg["desc"], "rows": rows, "cols": cols, "workers": n, "nwait": nwait,
                   "shard_bytes": per * cols * es, "parallelism": f"{n} stream-workers on {world} GPU"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                     "traffic": traffic,
                     "kernel": "lsq_grad_kernel<float,4,4> (one batched launch per epoch)",
                     "alg_bytes_per_launch": per_launch_bytes, "avg_launch_ms": round(per_launch_s * 1e3, 4),
                     "launches": launches},
        "epoch_alg_GBps": round(alg_bytes_epoch * its / 1e9, 1),
        "x_norm": xnorm,
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
