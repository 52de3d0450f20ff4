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


def test_hop_check_harvest_held_back_by_the_previous_harvest():
    """A harvest cannot precede the call's previous harvest (the state machine harvests one
    completion at a time, in the oracle's order): when the chain drift posts a task late -- on time
    against its own post, so its task hop holds -- the next harvest of the same call waits for it,
    and that is not the next harvest's lateness (kmap2_n9 op 356, r06g).  A harvest late past its
    trigger AND the previous harvest is still a miss."""
    import numpy as np
    sc = next(s for s in gated.scenarios() if s["name"] == "kmap2_n9")
    got, tr = _synthetic(sc)
    F = gated.F
    starts = np.asarray([g["t_ns"][0] for g in got], dtype=np.int64)
    calls = np.searchsorted(starts, tr[:, F["harvest"]], side="right") - 1
    # a call with two harvests at different instants (a, then b)
    pair = None
    for k in np.unique(calls):
        idx = sorted(np.nonzero(calls == k)[0], key=lambda j: tr[j, F["harvest"]])
        end = starts[k + 1] if k + 1 < len(starts) else np.iinfo(np.int64).max
        for a, b in zip(idx, idx[1:]):
            room = end - tr[b, F["harvest"]] - (tr[b, F["pub"]] - tr[a, F["harvest"]])
            if tr[a, F["harvest"]] < tr[b, F["harvest"]] and tr[a, F["rank"]] != tr[b, F["rank"]] and room > 3_000_000:
                pair = (int(k), a, b)
                break
        if pair:
            break
    assert pair, "no call with two consecutive harvests"
    k, a, b = pair
    ranks = got[k]["ranks"]
    ia, ib = ranks.index(int(tr[a, F["rank"]])), ranks.index(int(tr[b, F["rank"]]))
    # task a posted late by the chain (on time against that post), so late that b -- which completed
    # after a on the oracle's clock -- completes before a now
    drift = int(tr[b, F["pub"]] - tr[a, F["harvest"]]) + 1_500_000
    held = tr.copy()
    for key in ("post", "due", "pub", "seen", "harvest"):
        held[a, F[key]] += drift
    new_b = held[a, F["harvest"]] + 1_000  # b harvested right after a
    lat = [list(g["latency_s"]) for g in got]
    lat[k][ib] += (new_b - held[b, F["harvest"]]) / 1e9
    held[b, F["seen"]] = held[b, F["harvest"]] = new_b
    got2 = [dict(g, latency_s=lat[j]) for j, g in enumerate(got)]
    bad = gated.hop_check(sc, got2, held)[0]
    assert bad == [], bad[:3]
    # b 2 ms after a's harvest as well: late past both its trigger and the previous harvest
    later = held.copy()
    later[b, F["seen"]] = later[b, F["harvest"]] = new_b + 2_000_000
    lat[k][ib] += 2e-3
    got3 = [dict(g, latency_s=lat[j]) for j, g in enumerate(got)]
    kinds = {(x[0], x[1], x[2]) for x in gated.hop_check(sc, got3, later)[0]}
    assert ("harvest", k, ib) in kinds, kinds
    del ia
