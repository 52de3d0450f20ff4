"""Per-epoch control-path budget of a two-process run from its rocprofv3 kernel traces
(VERDICT r04 item 6).

    python tools/n2_budget.py <trace dir> <bench JSON line file> [--epochs K]

The run is `bench.py --gpus 2` with both ranks on one GPU (MPA_BENCH_ONE_GPU=1) and the
placement of the 8-GPU node for ONE remote worker (MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1: rank 0
serves seven workers, rank 1 one, device-armed).  Each process writes its own kernel trace
(rocprofv3 -d <dir>/%pid%); the bench line names the ranks' pids.  Per epoch e of the timed
region (the last K dispatches of each process):

  rank 0: lsq_grad_kernel L0(e) -- its local tasks; the last one to finish waits for the remote
          `done` word, harvests, runs the epoch step and rings the remote doorbell (fused tail)
  rank 1: door_wait_kernel W(e) then lsq_grad_kernel L1(e) (armed: queued behind the wait)

  ring -> start   start L1(e) - end L0(e-1)   (the tail rings at its end; the wait sees the
                                                word, the queued task starts)
  door wait seen  end W(e) - end L0(e-1)
  remote task     end L1(e) - start L1(e)
  done -> end     end L0(e) - end L1(e)       (rank 0's launch after the remote reply: on one GPU
                                                its own seven tasks, which share the HBM, are longer)
  epoch           end L0(e) - end L0(e-1)
"""
import argparse
import csv
import glob
import json
import os
import statistics as st


def load(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def pid_of(path):
    for part in reversed(path.split(os.sep)):
        digits = part.split("_")[0]
        if digits.isdigit():
            return int(digits)
    return None


def med(v):
    return round(st.median(v) / 1e3, 2) if v else None


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("bench_json")
    p.add_argument("--epochs", type=int, default=None)
    a = p.parse_args()
    line = json.load(open(a.bench_json))
    pids = line.get("rank_pids") or []
    K = a.epochs or line["steps"]
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    by_pid = {}
    for f in files:
        by_pid.setdefault(pid_of(f), []).extend(load(f))
    if len(pids) != 2 or any(q not in by_pid for q in pids):
        raise SystemExit(f"trace pids {sorted(k for k in by_pid if k)} do not contain the ranks {pids}")
    r0 = [r for r in sorted(by_pid[pids[0]]) if "lsq_grad_kernel" in r[2]][-(K + 1):]
    r1 = [r for r in sorted(by_pid[pids[1]]) if "lsq_grad_kernel" in r[2]]
    w1 = [r for r in sorted(by_pid[pids[1]]) if "door_wait_kernel" in r[2]]
    out = {"epochs": len(r0) - 1, "rank1_door_waits": len(w1)}
    ring, seen, remote, step, epoch, local = [], [], [], [], [], []
    for e in range(1, len(r0)):
        prev_end = r0[e - 1][1]
        # the remote task rung by launch e - 1's tail: the first rank-1 task to start after its end
        # (10 us of slack for the two processes' clocks)
        cand = [r for r in r1 if prev_end - 10_000 <= r[0] <= r0[e][1]]
        if not cand:
            continue
        s1, e1 = cand[0][0], cand[0][1]
        ring.append(s1 - prev_end)
        remote.append(e1 - s1)
        step.append(r0[e][1] - e1)
        epoch.append(r0[e][1] - prev_end)
        local.append(r0[e][1] - r0[e][0])
        ws = [w for w in w1 if prev_end - 10_000 <= w[1] <= s1]
        if ws:
            seen.append(ws[-1][1] - prev_end)
    out.update({"ring_to_start_us": med(ring), "door_wait_sees_ring_us": med(seen), "remote_task_us": med(remote),
                "done_to_step_end_us": med(step), "epoch_us": med(epoch), "rank0_launch_us": med(local),
                "bench_ms_per_step": line.get("ms_per_step"), "exchange": line.get("exchange")})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
