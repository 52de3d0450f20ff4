"""Dispatch drift of a gated replay over the HOST transport (CPU) against the oracle, per worker and task:
where the device latency of a harvest comes from (profiles/r05_gated_hops.txt).

    python tools/cpu_gate_drift.py <golden scenario name>
"""
import sys, threading, uuid, numpy as np
sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo/mpistragglers.jl_amd")
import gated, mpiasyncpools as M
name = sys.argv[1]
sc = next(s for s in gated.scenarios() if s["name"] == name)
_, sched = gated.oracle_gate(sc)
n = sc["n"]
dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
pl = [1]*n; nm = f"/mpa_x_{uuid.uuid4().hex[:8]}"
coord = M.DistComm(n, pl, 0, nm, 256, transport="host"); server = M.DistComm(n, pl, 1, nm, 256, transport="host")
for w in range(1, n+1):
    server.set_task(w, "kmap2"); server.set_delays(w, dur[w-1])
th = threading.Thread(target=server.serve, daemon=True); th.start()
coord.set_gate(*sched)
with gated.no_gc():
    got, pool = gated.replay(M, sc, coord, lambda k: np.zeros(k), lambda b: b, gated.make_golden().predicate, snap=np.copy)
coord.shutdown(); th.join(60); server.close(); coord.close()
out, sim = gated.make_golden().run_scenario(sc, return_sim=True)
ev = sim.events()  # (w, t, post, done, seen)
# device dispatch time of each (worker, task t): stimestamps when it changes
t00 = None
posts = {}
cnt = [0]*n
prev = [None]*n
for k, g in enumerate(got):
    for i, s in enumerate(g["stimestamps"]):
        if s != prev[i] and s > 0:
            cnt[i] += 1; posts[(i, cnt[i])] = (s, k); prev[i] = s
base_dev = min(v[0] for v in posts.values())
base_or = min(e[2] for e in ev)
for (w, t, post, done, seen) in ev:
    if (w, t) in posts:
        dp, k = posts[(w, t)]
        print("w%d t%2d op%2d  post oracle %8.3f dev %8.3f  drift %7.3f" % (w, t, k, (post-base_or)/1e6, (dp-base_dev)/1e6, ((dp-base_dev)-(post-base_or))/1e6))
