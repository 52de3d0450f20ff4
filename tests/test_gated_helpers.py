"""The timing harness's own helpers (tests/gated.py), on CPU: the host watchdog process and
the GC-off context the device latency checks run in."""
import gc
import time

import gated


def test_no_gc_disables_and_restores_the_collector():
    assert gc.isenabled()
    with gated.no_gc():
        assert not gc.isenabled()
    assert gc.isenabled()
    gc.disable()
    try:
        with gated.no_gc():
            assert not gc.isenabled()
        assert not gc.isenabled()  # left as it was found
    finally:
        gc.enable()


def test_host_watchdog_reports_its_oversleep():
    w = gated.HostWatchdog()
    try:
        w.take()
        time.sleep(0.2)
        worst, over = w.take()
        assert 0.0 <= worst < 1000.0 and over >= 0
    finally:
        w.close()


def _synthetic(sc):
    """The oracle's own timeline as a replay record and a task trace (every hop exact; op k's
    host times shifted by 10 ns x k so that calls meeting at one virtual instant stay ordered)."""
    import numpy as np
    from oracle import OBS_CALL, OBS_POST, OBS_WAITALL
    _, sim = gated.make_golden().run_scenario(sc, return_sim=True)
    base = 10 ** 12
    n = sc["n"]
    ranks = sc.get("ranks", list(range(1, n + 1)))
    # op k's first observation: its phase-1 Test! (asyncmap!) or its Waitall! (a waitall! with
    # nothing in flight observes nothing: it starts where the previous op did)
    obs = [o for o in sim.observations()]
    k, post_op, first, j = -1, {}, [], 0
    for op in sc["ops"]:
        k += 1
        want = OBS_CALL if op["op"] == "asyncmap" else OBS_WAITALL
        while j < len(obs) and obs[j][0] == OBS_POST:  # posts of the previous op
            post_op[(obs[j][1], obs[j][2])] = k - 1
            j += 1
        if j < len(obs) and obs[j][0] == want:
            first.append(obs[j][4])
        else:
            first.append(first[-1] if first else 0)
            continue
        j += 1
        while j < len(obs) and obs[j][0] not in (OBS_CALL, OBS_WAITALL):
            if obs[j][0] == OBS_POST:
                post_op[(obs[j][1], obs[j][2])] = k
            j += 1
    got = [{"latency_s": [x / 1e9 for x in r["latency_ns"]], "t_ns": (base + first[k] + 10 * k, base + first[k] + 10 * k),
            "ranks": ranks} for k, r in enumerate(sc["results"])]
    tr = []
    for w, t, post, done, seen in sim.events():
        kp = post_op[(w, t)]
        nk = len(sc["results"])
        kh = next((k for k in range(kp, nk) if sc["results"][k]["latency_ns"][w] == seen - post and
                   first[k] <= seen and (k + 1 == nk or first[k + 1] >= seen)), None)
        if kh is None:
            continue
        e = np.zeros(len(gated.F), dtype=np.int64)
        for key, v in (("rank", ranks[w]), ("seq", t), ("post", base + post + 10 * kp), ("due", base + done),
                       ("pub", base + done + 10 * kp), ("gate", base + post), ("seen", base + seen),
                       ("harvest", base + seen + 10 * kh)):
            e[gated.F[key]] = v
        tr.append(e)
    return got, np.asarray(tr)


def test_hop_check_on_the_oracles_own_timeline():
    """gated.hop_check (the device latency check, tests/test_gpu_gated.py) passes the oracle's own
    timeline on every golden scenario -- gpu_sep_nwait2 included, whose final Waitall! harvest is
    triggered by another worker's completion -- and names the hop that a perturbation moves."""
    for sc in gated.scenarios():
        got, tr = _synthetic(sc)
        bad, stats = gated.hop_check(sc, got, tr)
        assert bad == [], (sc["name"], bad[:3])
    sc = next(s for s in gated.scenarios() if s["name"] == "gpu_sep_nwait2")
    got, tr = _synthetic(sc)
    late = tr.copy()
    late[5, gated.F["pub"]] += 2_000_000  # one task 2 ms late on the device
    kinds = {b[0] for b in gated.hop_check(sc, got, late)[0]}
    assert "task" in kinds
    slow = tr.copy()
    slow[5, gated.F["harvest"]] += 2_000_000  # one harvest 2 ms after its trigger
    kinds = {b[0] for b in gated.hop_check(sc, got, slow)[0]}
    assert "harvest" in kinds and "latency" in kinds
