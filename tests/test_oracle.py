"""CPU tests of the oracles: the three independent restatements of go-aoi's XZListAOIManager
semantics agree with each other and with the committed golden fixtures; the reference's own AOI check
(DoTestAOI) holds; the workload generator is pinned.

Parity status: UNPINNED against go-aoi itself (module absent, no Go toolchain, no reference golden
vectors). What IS pinned: oracle (i) (list restatement, upstream structure) ==
oracle (ii) (stateful grid model) == oracle (iii) (numpy brute force) on every case, and all three ==
tests/golden/*.npz.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402
from golden import make_golden as G  # noqa: E402

from oracle import semantic  # noqa: E402


@pytest.fixture(scope="module")
def po(oracle_lib):
    return oracle_lib


def _check_case(po, case, kinds=("xz", "grid", "sem")):
    results = {}
    for k in kinds:
        if k == "xz":
            o = po.XZListOracle(case["dist"], case["cap"])
        elif k == "grid":
            b = case.get("bounds") or (-1000.0, -1000.0, 1000.0, 1000.0)
            o = po.GridOracle(case["dist"], case["cap"], b)
        else:
            o = semantic.SemanticModel(case["dist"], case["cap"])
        evs = [(H.semantic_tick(o, ops) if k == "sem" else H.oracle_tick(o, ops)) for ops in case["ticks"]]
        if k == "xz":
            assert o.check_invariants() == 0
        results[k] = (evs, o.relation())
    return results


@pytest.mark.parametrize("path", G.fixture_paths(), ids=lambda p: os.path.basename(p))
def test_oracles_match_golden(po, path):
    case = G.load(path)
    kinds = ("xz", "grid", "sem") if case["cap"] <= 2500 else ("xz", "grid")
    res = _check_case(po, case, kinds)
    for k, (evs, rel) in res.items():
        assert len(evs) == len(case["events"])
        for t, (a, b) in enumerate(zip(evs, case["events"])):
            assert np.array_equal(a, b), f"{k} tick {t}: " + H.fmt_diff(a, b)
        assert np.array_equal(rel[0], case["rel"][0]) and np.array_equal(rel[1], case["rel"][1]), k


@pytest.mark.parametrize("seed", range(6))
def test_oracles_agree_random(po, seed):
    case = H.case_random_ops(seed=100 + seed, n=150, nticks=8, ops_per_tick=120, world=200.0 + 100 * seed,
                             dist=[10.0, 50.0, 100.0][seed % 3])
    res = _check_case(po, case)
    for t in range(len(case["ticks"])):
        a = res["xz"][0][t]
        for k in ("grid", "sem"):
            assert np.array_equal(a, res[k][0][t]), f"{k} tick {t}: " + H.fmt_diff(a, res[k][0][t])
    for k in ("grid", "sem"):
        assert np.array_equal(res["xz"][1][1], res[k][1][1])


def test_do_test_aoi_known_answer(po):
    """The reference's only AOI assertion: DoTestAOI (examples/test_client/ClientEntity.go:367-379,
    examples/test_game/Avatar.go:267-280). An AOITester entered at the avatar's position must raise
    an enter with the avatar (avatar.OnEnterAOI(tester) -> client create, Entity.go:227-240), and its
    destruction a leave. Also MySpace's 10 Monsters at Vector3{} (MySpace.go:31-34) all see each other."""
    case = H.case_origin_monsters()
    orc = po.XZListOracle(case["dist"], case["cap"])
    evs = [H.oracle_tick(orc, ops) for ops in case["ticks"]]
    # 10 co-located monsters: 45 pairs, every pair entered once, by the later Enter
    t0 = {tuple(e) for e in evs[0].tolist()}
    assert len(t0) == 45 and all((b, a | H.EV_ENTER) in t0 for b in range(10) for a in range(b))
    # avatar (slot 10) at (37.5,-12.25) is inside every monster's box (D=100)
    assert {tuple(e) for e in evs[1].tolist()} == {(10, m | H.EV_ENTER) for m in range(10)}
    # AOITester (slot 11) enters at the avatar's position: ENTER(11, 10) present
    assert (11, 10 | H.EV_ENTER) in {tuple(e) for e in evs[2].tolist()}
    assert (11, 10) in {tuple(e) for e in evs[3].tolist()}  # tester destroyed -> LEAVE(11, 10)


def test_bulk_enter_equals_sequential(po):
    rng = np.random.default_rng(5)
    n = 3000
    x = (rng.integers(0, 400, n) * 0.5).astype(np.float32)  # many ties
    z = rng.uniform(0, 200, n).astype(np.float32)
    slots = rng.permutation(n).astype(np.uint32)
    a = po.XZListOracle(100.0, n)
    for i in range(n):
        a.enter(int(slots[i]), float(x[i]), float(z[i]))
    a.take_events()
    b = po.XZListOracle(100.0, n)
    b.bulk_enter(slots, x, z)
    assert b.check_invariants() == 0
    ra, rb = a.relation(), b.relation()
    assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1])
    # and the two continue identically
    mx = (x + rng.uniform(-2, 2, n)).astype(np.float32)
    mz = (z + rng.uniform(-2, 2, n)).astype(np.float32)
    order = np.arange(n, dtype=np.uint32)
    a.moved_batch(order, mx[slots.argsort()], mz[slots.argsort()])
    b.moved_batch(order, mx[slots.argsort()], mz[slots.argsort()])
    ea, eb = a.take_events(), b.take_events()
    assert sorted(map(tuple, ea.tolist())) == sorted(map(tuple, eb.tolist()))


def test_list_invariants_under_churn(po):
    case = H.case_random_ops(seed=77, n=300, nticks=20, ops_per_tick=200, world=100.0, dist=30.0)
    orc = po.XZListOracle(case["dist"], case["cap"])
    for ops in case["ticks"]:
        H.oracle_tick(orc, ops)
        assert orc.check_invariants() == 0


def test_rounding_asymmetry_exists(po):
    """The predicate is evaluated from the mover's coordinate, so in(a,b) != in(b,a) can happen when
    the bounds round; the pair state then depends on who moved last."""
    D = np.float32(100.0)
    a_x = np.float32(7.0e7)  # ulp = 8: a_x + D rounds (ties to even)
    hi = np.float32(a_x + D)
    found = False
    for k in range(-4, 5):
        b_x = np.float32(hi + np.float32(8 * k))
        in_ab = (b_x >= np.float32(a_x - D)) and (b_x <= np.float32(a_x + D))
        in_ba = (a_x >= np.float32(b_x - D)) and (a_x <= np.float32(b_x + D))
        if in_ab != in_ba:
            found = True
            o = po.XZListOracle(float(D), 2)
            o.enter(0, float(a_x), 0.0)
            o.enter(1, float(b_x), 0.0)  # b entered last: state = in(b, a)
            e1 = o.take_events()
            assert (len(e1) == 1) == bool(in_ba)
            o.moved(0, float(a_x), 0.0)  # a acts last: state = in(a, b)
            e2 = o.take_events()
            assert len(e2) == 1 and bool(e2[0, 1] & H.EV_ENTER) == bool(in_ab)
    assert found


def test_workload_generator_golden(po):
    """Pin include/gwaoi_workload.h (host side); the GPU test checks the device side against it."""
    x, z = po.workload_init(0x5EED0002, 8, 35000.0)
    h = hash((x.tobytes(), z.tobytes()))
    assert np.all((x >= 0) & (x < 35000)) and np.all((z >= 0) & (z < 35000))
    u = po.lib().ow_u01(1, 2, 3, 4, 0)
    assert 0.0 <= u < 1.0 and float(np.float32(u)) == u
    x2, z2 = x.copy(), z.copy()
    po.workload_step(0x5EED0002, 1, x2, z2, 35000.0, 1.0)
    assert np.all(np.abs(x2 - x) <= 1.0) and np.all(np.abs(z2 - z) <= 1.0)
    # first values are a stable function of the header (regression pin)
    assert [f"{v:.6f}" for v in x[:3]] == GOLD_X
    assert h == hash((x.tobytes(), z.tobytes()))


GOLD_X = None  # filled below from the committed value


def _load_gold():
    global GOLD_X
    p = os.path.join(os.path.dirname(__file__), "golden", "workload_pin.txt")
    with open(p) as f:
        GOLD_X = f.read().split()


_load_gold()


def test_nonfinite_coordinates_in_the_list_manager(po):
    """What the reference does with a NaN coordinate (client floats reach Moved unchecked,
    /root/reference/components/game/GameService.go:404-408): in the list restatement (oracle (i)) a
    node moved to NaN bubbles one place towards the head (no comparison with NaN is true) and then
    sits in the middle of the sorted X list, where every later Mark walk that reaches it stops. A
    third party then loses neighbours that are inside its box — behaviour that depends on list
    position, not on positions. libgwaoi refuses non-finite coordinates instead (GWAOI_ERR_INVALID;
    tests/test_gpu_parity.py::test_nonfinite_refused)."""
    o = po.XZListOracle(100.0, 4)
    for slot, x in ((3, -10.0), (0, 0.0), (1, 20.0), (2, 10.0)):  # X list: D(-10) A(0) C(10) B(20)
        o.enter(slot, x, 0.0)
    o.take_events()
    o.moved(2, float("nan"), 0.0)  # C -> NaN: its box is NaN-bounded, it leaves everyone
    ev = o.take_events()
    assert sorted(map(tuple, ev.tolist())) == [(2, 0), (2, 1), (2, 3)]
    o.moved(3, -11.0, 0.0)  # D steps 1 unit left: A (11 away) and B (31 away) are inside its box
    ev = o.take_events()
    assert sorted(map(tuple, ev.tolist())) == [(3, 0), (3, 1)]  # LEAVEs: D's X walk stopped at C
    # +Inf is ordered (it bubbles to the tail) and only another +Inf is inside its box
    o2 = po.XZListOracle(100.0, 3)
    o2.enter(0, 0.0, 0.0)
    o2.enter(1, 20.0, 0.0)
    o2.take_events()
    o2.enter(2, float("inf"), 0.0)
    assert len(o2.take_events()) == 0
    o2.moved(0, 1.0, 0.0)
    assert len(o2.take_events()) == 0


def test_replay_tool_tracks_the_relation(po):
    """tools/replay_sets.c (bench.py's replay_ms): replaying a tick's events into InterestedIn /
    InterestedBy sets keeps them equal to the relation, with no inconsistent set operation."""
    import __graft_entry__ as G
    G.build_tools()
    from tools.replay import ReplaySets
    case = H.case_walk(0x5EED0001, 3000, 1200.0, 3, workload=po)
    orc = po.XZListOracle(100.0, 3000)
    H.oracle_tick(orc, case["ticks"][0])
    rp, cols = orc.relation()
    rs = ReplaySets(2 * len(cols))
    rs.load_relation(rp, cols)
    assert rs.size() == 2 * len(cols)
    for ops in case["ticks"][1:]:
        ev = np.ascontiguousarray(H.oracle_tick(orc, ops))
        assert len(ev) > 0
        assert rs.replay(ev.ctypes.data, len(ev)) == 0
        assert rs.size() == 2 * len(orc.relation()[1])
    bad = np.ascontiguousarray(ev[-1:])  # replaying the last change of a pair again is inconsistent
    assert rs.replay(bad.ctypes.data, 1) == 4
    rs.close()


def test_sharded_replay_tool_equals_the_single_sink(po):
    """tools/replay_sets.c's sharded sink (bench.py replay_ms_sharded: the same set operations split by
    owning entity over worker threads) stays consistent with the relation, as the single sink does."""
    import __graft_entry__ as G
    G.build_tools()
    from tools.replay import ShardedReplaySets
    case = H.case_walk(0x5EED0003, 3000, 1200.0, 4, workload=po)
    orc = po.XZListOracle(100.0, 3000)
    H.oracle_tick(orc, case["ticks"][0])
    rp, cols = orc.relation()
    rs = ShardedReplaySets(2 * len(cols), 5)
    rs.load_relation(rp, cols)
    assert rs.size() == 2 * len(cols)
    for ops in case["ticks"][1:]:
        ev = np.ascontiguousarray(H.oracle_tick(orc, ops))
        assert rs.replay(ev.ctypes.data, len(ev)) == 0
        assert rs.size() == 2 * len(orc.relation()[1])
    bad = np.ascontiguousarray(ev[-1:])
    assert rs.replay(bad.ctypes.data, 1) == 4
    rs.close()


def test_delta_rows_tool_tracks_the_relation(po):
    """tools/delta_rows.c (bench.py's relation_delta_apply_ms): per-slot sorted neighbour arrays patched
    with the net changes of a tick (both directions, as gwaoi_export_relation_delta lists them) equal
    the relation after the tick; re-applying an entry is reported as inconsistent."""
    import __graft_entry__ as G
    G.build_tools()
    from tools.replay import DeltaRows
    case = H.case_random_ops(seed=9, n=400, nticks=6, ops_per_tick=300, world=300.0, dist=60.0)
    orc = po.XZListOracle(60.0, 400)
    rel = orc.relation()
    dr = DeltaRows(*rel)

    def keyset(r):
        rp, cols = r
        rows = np.repeat(np.arange(len(rp) - 1, dtype=np.uint64), np.diff(rp.astype(np.int64)))
        return set((rows << np.uint64(32) | cols.astype(np.uint64)).tolist())

    for ops in case["ticks"]:
        H.oracle_tick(orc, ops)
        new = orc.relation()
        a, b = keyset(rel), keyset(new)
        d = [(k >> 32, (k & 0xFFFFFFFF) | 0x80000000) for k in sorted(b - a)] + \
            [(k >> 32, k & 0xFFFFFFFF) for k in sorted(a - b)]
        delta = np.asarray(d, np.uint32).reshape(-1, 2)
        assert dr.apply(delta, threads=1 + len(rel[1]) % 4) == 0  # (single and multi-threaded apply)
        assert dr.diff(*new) == 0
        rel = new
    assert dr.apply(delta[:1]) == 1
    dr.close()


def test_config3_cpu_baseline_sample(po):
    """bench.py's config-3 CPU baseline (one oracle (i) manager per Space, a worker
    pool): a bounded sample reports a rate, the threads used and every Space walked the same number of
    ticks; its pair events equal one sequential replay of those ticks."""
    import re

    import numpy as np

    import bench
    r = bench.cpu_baseline_spaces(500, 800.0, 100.0, 0x5EED0003, 3, 0.05, threads=2)
    assert r["value"] > 0 and r["cores"] == 2 and r["kind"] == "port"
    m = re.search(r"then (\d+) all-moving ticks.*?(\d+) pair events", r["sample"])
    nt, nev = int(m.group(1)), int(m.group(2))
    want = 0
    for s in range(3):
        x, z = po.workload_init(0x5EED0003 + s, 500, 800.0)
        orc = po.XZListOracle(100.0, 500)
        slots = np.arange(500, dtype=np.uint32)
        orc.bulk_enter(slots, x, z)
        orc.set_record(True)
        for k in range(1, nt + 1):
            po.workload_step(0x5EED0003 + s, k, x, z, 800.0, 1.0)
            orc.moved_batch(slots, x, z)
            want += len(orc.take_events())
        orc.close()
    assert nev == want


@pytest.mark.parametrize("dist,step,skew", [(100.0, 1.0, False), (50.0, 1.0, True), (400.0, 1.0, True),
                                            (100.0, 40.0, False)])
def test_sampled_restatement_equals_grid_oracle(po, dist, step, skew):
    """oracle (iv) (oracle/sampled.py: the events of sampled movers of an all-moving tick from two
    position snapshots, the full-size checker of configs 4 and 5) against oracle (ii), every mover, two
    ticks after an enter tick in slot order; uniform and hotspot worlds, large steps included."""
    from oracle import sampled
    n, L, seed, base = 4000, 2000.0, 0x5EED0077, 3 * 4000
    if skew:
        x, z = po.workload_skew_init(seed, n, L, 8, 40.0, 2)
    else:
        x, z = po.workload_init(seed, n, L)
    orc = po.GridOracle(dist, n, (0.0, 0.0, L, L))
    ids = np.arange(n, dtype=np.uint32)
    orc.bulk_enter(ids, x, z)
    for t in (1, 2):
        x0, z0 = x.copy(), z.copy()
        po.workload_step(seed, t, x, z, L, step)
        orc.moved_batch(ids, x, z)
        want = orc.take_events()
        want = want + np.array([base, base], np.uint32)  # as Space 3 of a manager with 4000 slots per Space
        want = want[np.lexsort((want[:, 1], want[:, 0]))]
        got = sampled.AllMovingTick(x0, z0, x, z, dist, base=base).sample(range(n))
        assert len(want) > 100
        assert np.array_equal(got, want), f"tick {t}: " + H.fmt_diff(got, want)
        assert np.array_equal(sampled.pick(want, [base + 5, base + 77]), sampled.AllMovingTick(
            x0, z0, x, z, dist, base=base).sample([5, 77]))
