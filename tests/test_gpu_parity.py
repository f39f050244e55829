"""GPU parity tests: libgwaoi (hand-written HIP, gfx950) against the CPU oracles, through the C ABI.

Bar: bit-exact. Every tick's event list must equal the oracle's canonical event list element for
element (same pairs, same kinds, same order), and the exported relation must equal the oracle's
neighbour sets. Oracle (i) is the go-aoi XZListAOIManager restatement; oracle (ii) (stateful grid
model, cross-checked against (i) in test_oracle.py) is used where (i) is too slow (1M entities).
Parity against go-aoi itself is UNPINNED (module absent here; DESIGN.md "Oracle").
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402
from golden import make_golden as G  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def po(oracle_lib):
    return oracle_lib


def engine(case, **kw):
    from goworld_amd.engine import Engine
    return Engine(case["dist"], capacity=case["cap"], bounds=case.get("bounds"), **kw)


def assert_same(a, b, what):
    assert np.array_equal(a, b), what + ": " + H.fmt_diff(a, b)


def run_against_oracle(po, case, check_relation_every=1, eng=None, oracle="xz", cells_per_dist=None,
                       sweep_lds=True):
    eng = eng or engine(case)
    if cells_per_dist:
        eng.debug_set_cells_per_dist(cells_per_dist)
    if not sweep_lds:
        eng.debug_set_sweep_lds(False)
    if oracle == "xz":
        orc = po.XZListOracle(case["dist"], case["cap"])
    else:
        orc = po.GridOracle(case["dist"], case["cap"], case.get("bounds") or (-1000, -1000, 1000, 1000))
    for t, ops in enumerate(case["ticks"]):
        want = H.oracle_tick(orc, ops)
        got = H.gpu_tick(eng, ops)
        assert_same(got, want, f"{case['name']} tick {t}")
        if check_relation_every and t % check_relation_every == 0:
            rg, ro = eng.relation(), orc.relation()
            assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1]), f"relation tick {t}"
    return eng, orc


@pytest.mark.parametrize("path", G.fixture_paths(), ids=lambda p: os.path.basename(p))
def test_golden_fixtures(gpu, path):
    case = G.load(path)
    eng = engine(case)
    for t, ops in enumerate(case["ticks"]):
        got = H.gpu_tick(eng, ops)
        assert_same(got, case["events"][t], f"{case['name']} tick {t}")
    rp, cols = eng.relation()
    assert np.array_equal(rp, case["rel"][0]) and np.array_equal(cols, case["rel"][1])


@pytest.mark.parametrize("seed", range(8))
def test_random_op_mixes(gpu, po, seed):
    case = H.case_random_ops(seed=1000 + seed, n=[64, 300, 1000, 2000][seed % 4], nticks=10,
                             ops_per_tick=[40, 400, 800, 3000][seed % 4], world=[100.0, 300.0, 1000.0][seed % 3],
                             dist=[10.0, 50.0, 100.0][seed % 3], snap=seed % 2 == 0)
    run_against_oracle(po, case, check_relation_every=3)


@pytest.mark.parametrize("seed", range(3))
def test_global_sweep_path(gpu, po, seed):
    """The global-memory sweep path (taken by teleports, oversized regions and Leave ops) on its own."""
    case = H.case_random_ops(seed=300 + seed, n=800, nticks=8, ops_per_tick=900, world=400.0, dist=60.0)
    run_against_oracle(po, case, check_relation_every=4, sweep_lds=False)


def test_lds_and_global_sweep_agree_walk(gpu, po):
    """Config-1 style walk: LDS-staged and global sweep paths give identical events."""
    from goworld_amd.engine import Engine
    case = H.case_walk(0x5EED0007, 20000, 5000.0, 12, workload=po)
    a = Engine(case["dist"], capacity=case["cap"], bounds=case["bounds"])
    b = Engine(case["dist"], capacity=case["cap"], bounds=case["bounds"])
    b.debug_set_sweep_lds(False)
    for t, ops in enumerate(case["ticks"]):
        assert_same(H.gpu_tick(a, ops), H.gpu_tick(b, ops), f"tick {t}")


@pytest.mark.parametrize("cpd", [0.5, 1.0, 3.0, 4.0])
def test_cell_size_does_not_change_events(gpu, po, cpd):
    case = H.case_random_ops(seed=7, n=500, nticks=6, ops_per_tick=600, world=300.0, dist=40.0)
    run_against_oracle(po, case, check_relation_every=2, cells_per_dist=cpd)


def test_auto_extent_regrid(gpu, po):
    """No extent hint: the manager starts from Space.GetSpaceRange's +-1000 and regrids as entities
    appear far outside it (clamped edge cells in between) — events must not change."""
    case = H.case_random_ops(seed=9, n=400, nticks=8, ops_per_tick=300, world=20000.0, dist=100.0, snap=False)
    case["bounds"] = None
    run_against_oracle(po, case, check_relation_every=2)


def test_config1_walk_100_ticks(gpu, po):
    """N=10,000, L=3,500, D=100, seed 0x5EED0001, 100 ticks, against the
    go-aoi list restatement tick by tick."""
    case = H.case_walk(0x5EED0001, 10000, 3500.0, 101, workload=po)
    eng, orc = run_against_oracle(po, case, check_relation_every=25)
    assert eng.count()[0] == 10000


def test_device_staged_moves_and_generator(gpu, po):
    """Inputs resident in HBM (the bench path): the device generator is bit-identical to the host
    one, and device-staged ticks give the same events as host-staged ones."""
    from goworld_amd.engine import DeviceBuffer, wl_init, wl_iota, wl_step
    n, L, seed = 20000, 5000.0, 0x5EED0042
    bx, bz, bs = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n)
    wl_init(0, bx.ptr, bz.ptr, n, seed, L)
    wl_iota(0, bs.ptr, n)
    hx, hz = po.workload_init(seed, n, L)
    assert np.array_equal(bx.download(np.float32, n), hx) and np.array_equal(bz.download(np.float32, n), hz)
    from goworld_amd.engine import Engine
    a = Engine(100.0, n, bounds=(0, 0, L, L))
    b = Engine(100.0, n, bounds=(0, 0, L, L))
    for i in range(n):
        a.enter(i, float(hx[i]), float(hz[i]))
    for i in range(n):
        b.enter(i, float(hx[i]), float(hz[i]))
    assert_same(a.tick(), b.tick(), "enter tick")
    for t in range(1, 6):
        wl_step(0, bx.ptr, bz.ptr, bx.ptr, bz.ptr, n, seed, t, L, 1.0)
        po.workload_step(seed, t, hx, hz, L, 1.0)
        assert np.array_equal(bx.download(np.float32, n), hx)
        a.stage_moves(np.arange(n, dtype=np.uint32), hx, hz)
        b.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, n)
        assert_same(b.tick(), a.tick(), f"tick {t}")


def test_multi_space_batching(gpu, po):
    """Several independent Spaces (different D) in one manager: events equal those of one oracle per
    Space, in global op order; no pair ever crosses Spaces."""
    from goworld_amd.engine import Engine
    rng = np.random.default_rng(3)
    dists = [25.0, 50.0, 100.0, 200.0]
    per = 400
    ns = len(dists)
    cap = ns * per
    eng = Engine(capacity=cap, spaces=[(d, (0.0, 0.0, 1000.0, 1000.0)) for d in dists])
    orcs = [po.XZListOracle(d, cap) for d in dists]
    space_of = np.repeat(np.arange(ns), per)
    pos = rng.uniform(0, 1000, (cap, 2)).astype(np.float32)
    order = rng.permutation(cap)
    for t in range(6):
        want = []
        if t == 0:
            for s in order:
                eng.enter(int(s), float(pos[s, 0]), float(pos[s, 1]), space=int(space_of[s]))
                o = orcs[space_of[s]]
                o.enter(int(s), float(pos[s, 0]), float(pos[s, 1]))
                ev = o.take_events()
                if len(ev):
                    want.append(ev[np.argsort(ev[:, 1], kind="stable")])
        else:
            pos = (pos + rng.uniform(-5, 5, pos.shape)).astype(np.float32)
            mv = rng.permutation(cap)[: cap // 2]
            eng.stage_moves(mv.astype(np.uint32), pos[mv, 0], pos[mv, 1])
            for s in mv:
                o = orcs[space_of[s]]
                o.moved(int(s), float(pos[s, 0]), float(pos[s, 1]))
                ev = o.take_events()
                if len(ev):
                    want.append(ev[np.argsort(ev[:, 1], kind="stable")])
        want = np.concatenate(want) if want else np.zeros((0, 2), np.uint32)
        got = eng.tick()
        assert_same(got, want, f"multispace tick {t}")
        sm = got[:, 0]
        so = got[:, 1] & 0x7FFFFFFF
        assert np.all(space_of[sm] == space_of[so])


def test_seq_renormalisation(gpu, po):
    """The per-entity op sequence numbers are rank-compressed before they would overflow; events must
    be unaffected across the renormalisation."""
    case = H.case_random_ops(seed=21, n=300, nticks=12, ops_per_tick=250, world=200.0, dist=30.0)
    from goworld_amd.engine import Engine
    eng = Engine(case["dist"], capacity=case["cap"])
    orc = po.XZListOracle(case["dist"], case["cap"])
    for t, ops in enumerate(case["ticks"]):
        if t == 4:
            eng.debug_set_next_seq(0x7ff00000 - 700)
        want = H.oracle_tick(orc, ops)
        assert_same(H.gpu_tick(eng, ops), want, f"tick {t}")
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[1], ro[1])


def test_misuse_is_reported(gpu):
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_iota
    eng = Engine(100.0, 64)
    eng.enter(1, 0.0, 0.0)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.enter(1, 5.0, 5.0)
    assert e.value.code == _lib.GWAOI_ERR_STATE
    with pytest.raises(_lib.GwaoiError) as e:
        eng.moved(2, 0.0, 0.0)
    assert e.value.code == _lib.GWAOI_ERR_STATE
    with pytest.raises(_lib.GwaoiError) as e:
        eng.leave(3)
    assert e.value.code == _lib.GWAOI_ERR_STATE
    with pytest.raises(_lib.GwaoiError) as e:
        eng.moved(64, 0.0, 0.0)
    assert e.value.code == _lib.GWAOI_ERR_INVALID
    eng.tick()
    # device-staged batch naming an absent slot is caught on the device
    bs = DeviceBuffer(4 * 4)
    bs.upload(np.asarray([1, 5, 1, 1], np.uint32))
    bx = DeviceBuffer(16)
    bx.upload(np.zeros(4, np.float32))
    eng.stage_moves_device(bs.ptr, bx.ptr, bx.ptr, 2)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK
    # duplicate slot in a device-staged batch
    eng2 = Engine(100.0, 64)
    eng2.enter(1, 0.0, 0.0)
    eng2.tick()
    eng2.stage_moves_device(bs.ptr + 8, bx.ptr, bx.ptr, 2)
    with pytest.raises(_lib.GwaoiError) as e:
        eng2.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


def test_empty_and_tiny(gpu, po):
    from goworld_amd.engine import Engine
    eng = Engine(100.0, 4)
    assert len(eng.tick()) == 0  # nothing staged
    eng.enter(0, 1.0, 1.0)
    assert len(eng.tick()) == 0  # alone
    eng.enter(1, 1.0, 1.0)
    ev = eng.tick()
    assert ev.tolist() == [[1, 0 | H.EV_ENTER]]
    eng.leave(0)
    eng.leave(1)
    ev = eng.tick()
    assert ev.tolist() == [[0, 1]]  # 1 was 0's neighbour; when 1 leaves it has none
    rp, cols = eng.relation()
    assert len(cols) == 0 and eng.count()[0] == 0
    # re-enter the same slots, same tick as a move of the other (forces a sub-pass)
    eng.enter(0, 0.0, 0.0)
    eng.enter(1, 100.0, 100.0)
    eng.moved(0, -0.5, -0.5)  # second op on slot 0: flushes [enter 0, enter 1] first
    ev = eng.tick()
    assert ev.tolist() == [[1, 0 | H.EV_ENTER], [0, 1]]
    assert eng.last.n_subticks == 2


@pytest.mark.parametrize("L", [5000.0, 3500.0, 2400.0])
def test_relation_view_paths(gpu, po, L):
    """gwaoi_relation_device at three densities (20,000 entities, D = 100): mean row ~32 (slab rows
    sorted by the 32/64 register networks), ~65 (rows over 64 listed and finished by k_row_fix) and
    ~140 (rows longer than the slab keeps: the fill pass and the in-place sort). Rows equal oracle
    (ii)'s, in ascending order, before and after a tick of moves."""
    from goworld_amd.engine import Engine
    n, seed = 20000, 0x5EED0AA1
    x, z = po.workload_init(seed, n, L)
    eng = Engine(100.0, n, bounds=(0, 0, L, L))
    orc = po.GridOracle(100.0, n, (0, 0, L, L))
    slots = np.arange(n, dtype=np.uint32)
    orc.bulk_enter(slots, x, z)
    H.gpu_tick(eng, [(H.ENTER, i, float(x[i]), float(z[i])) for i in range(n)])
    for t in range(3):
        if t == 2:
            po.workload_step(seed, 1, x, z, L, 1.0)
            orc.moved_batch(slots, x, z)
            orc.take_events()
            eng.stage_moves(slots, x, z)
            eng.tick()
        rg, ro = eng.relation(), orc.relation()
        assert np.array_equal(rg[0], ro[0]), f"call {t}: row lengths"
        assert np.array_equal(rg[1], ro[1]), f"call {t}: rows"
    lens = np.diff(ro[0])
    assert lens.max() > {5000.0: 40, 3500.0: 64, 2400.0: 128}[L]


@pytest.mark.parametrize("seed", range(4))
def test_relation_incremental_from_events(gpu, po, seed):
    """gwaoi_relation_device kept up to date from each tick's events (k_rd_*: rows changed by rank
    arithmetic over the tick's changes, no rebuild from the grid) equals the view rebuilt from the grid
    (mode 1, a second manager fed the same calls) and oracle (i)'s neighbour sets after EVERY tick, over
    Enter/Leave/Moved mixes with repeated slots (sub-passes: one tick's events span several passes),
    teleports and leaves. Snapped positions crowd lattice points: rows with more than 32 changes in a
    tick take the sorted path (k_rd_sort_long + binary searches)."""
    case = H.case_random_ops(seed=2000 + seed, n=[300, 1000, 2000, 800][seed], nticks=12,
                             ops_per_tick=[200, 300, 400, 900][seed], world=[300.0, 1000.0, 400.0, 60.0][seed],
                             dist=[50.0, 100.0, 25.0, 10.0][seed], snap=seed % 2 == 0)
    eng, ref = engine(case), engine(case)
    ref.debug_relation_mode(1)
    orc = po.XZListOracle(case["dist"], case["cap"])
    for t, ops in enumerate(case["ticks"]):
        want = H.oracle_tick(orc, ops)
        assert_same(H.gpu_tick(eng, ops), want, f"{case['name']} tick {t}")
        H.gpu_tick(ref, ops)
        ra, rb, ro = eng.relation(), ref.relation(), orc.relation()
        assert np.array_equal(ra[0], ro[0]) and np.array_equal(ra[1], ro[1]), f"tick {t}: incremental vs oracle"
        assert np.array_equal(rb[0], ro[0]) and np.array_equal(rb[1], ro[1]), f"tick {t}: rebuilt vs oracle"
    n_inc, n_full, why = eng.debug_relation_mode()
    assert n_inc + n_full == len(case["ticks"])
    assert n_inc >= len(case["ticks"]) // 2, (n_inc, n_full, why)
    assert ref.debug_relation_mode()[0] == 0


@pytest.mark.slow
def test_config2_full_size_enter_and_four_ticks(gpu, po):
    """SURVEY.md §8(d) config 2 at full size: N=1,000,000, L=35,000, D=100, seed 0x5EED0002; the
    bulk enter tick (relation and every ENTER event) and four all-moving ticks against oracle (ii)."""
    from goworld_amd.engine import Engine
    n, L, seed = 1_000_000, 35000.0, 0x5EED0002
    x, z = po.workload_init(seed, n, L)
    eng = Engine(100.0, n, bounds=(0, 0, L, L))
    orc = po.GridOracle(100.0, n, (0, 0, L, L))
    slots = np.arange(n, dtype=np.uint32)
    orc.bulk_enter(slots, x, z)  # events suppressed on the oracle side: compare relation instead
    eng_ops = [(H.ENTER, i, float(x[i]), float(z[i])) for i in range(n)]
    ev0 = H.gpu_tick(eng, eng_ops)
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
    assert len(ev0) == len(ro[1]) // 2  # one ENTER per pair, raised by the later Enter
    # the enter tick's events exactly: Enters run in slot order, so pair {a < b} raises ENTER(b, a)
    # (mover b, other a) once; every event of the tick is such an ENTER, rows and columns ascending
    rp, cols = ro
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp.astype(np.int64)))
    keep = cols.astype(np.int64) < rows
    want0 = np.stack([rows[keep].astype(np.uint32), cols[keep].astype(np.uint32) | np.uint32(H.EV_ENTER)], axis=1)
    assert ev0.dtype == want0.dtype and np.array_equal(ev0, want0), "1M enter tick: " + H.fmt_diff(ev0[:100000], want0[:100000])
    for t in (1, 2, 3, 4):
        po.workload_step(seed, t, x, z, L, 1.0)
        orc.moved_batch(slots, x, z)
        ev = orc.take_events()
        want = ev[np.lexsort((ev[:, 1], ev[:, 0]))]  # rank == slot
        eng.stage_moves(slots, x, z)
        got = eng.tick()
        assert_same(got, want, f"1M tick {t}")
        assert len(got) > 10000
        # the view updated from the tick's 325k events equals oracle (ii)'s relation
        rg, ro = eng.relation(), orc.relation()
        assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1]), f"1M tick {t}: relation"
    assert eng.debug_relation_mode()[0] == 4, eng.debug_relation_mode()  # every moving tick: updated


@pytest.mark.parametrize("path", ["band", "ring", "all_global"])
def test_skewed_crowd_dense_path(gpu, po, path):
    """Config 5 in miniature: a small-D Space with Gaussian hotspots (~100x the mean
    density) and a large-D Space in one manager. Hotspot tiles and every D=400 tile exceed the sweep's
    LDS region: their movers take the wave-per-mover path (k_sweep_dense) with its reserved event slots,
    by the band walk (the default: per-cell key windows of the boxes' symmetric difference; the enter tick's
    movers have no band plan and are handed to the ring walk), by their whole rings (band off), or with every
    mover of the world on that path (LDS sweep off); relation after the enter tick and the last tick, events
    every tick, against oracle (ii)."""
    from goworld_amd.engine import Engine
    n, L = 60000, 8500.0  # the mean density of config 5 (1M in 35,000^2)
    spaces = [(50.0, 0x5EED0050), (400.0, 0x5EED0400)]
    eng = Engine(capacity=n * len(spaces), spaces=[(d, (0.0, 0.0, L, L)) for d, _ in spaces])
    if path == "ring":
        eng.debug_set_band(0)
    elif path == "all_global":
        eng.debug_set_sweep_lds(False)
    eng.set_timing(True)
    pos, orcs = [], []
    for k, (d, seed) in enumerate(spaces):
        x, z = po.workload_skew_init(seed, n, L, 4, 55.0)
        slots = np.arange(k * n, (k + 1) * n, dtype=np.uint32)
        eng.stage_enters(slots, x, z, space=k)
        o = po.GridOracle(d, n * len(spaces), (0, 0, L, L))
        o.bulk_enter(slots, x, z)
        pos.append((slots, x, z))
        orcs.append(o)

    def check_relation(what):
        rg = eng.relation()
        rel = [o.relation() for o in orcs]
        rp = sum(r[0].astype(np.int64) for r in rel)
        assert np.array_equal(rg[0], rp) and np.array_equal(rg[1], np.concatenate([r[1] for r in rel])), what

    ev0 = eng.tick()
    check_relation("enter tick")
    assert len(ev0) > 1_000_000
    for t in (1, 2, 3):
        want = []
        for (slots, x, z), (_, seed), o in zip(pos, spaces, orcs):
            po.workload_step(seed, t, x, z, L, 1.0)
            eng.stage_moves(slots, x, z)
            o.moved_batch(slots, x, z)
            want.append(o.take_events())
        want = np.concatenate(want)
        want = want[np.lexsort((want[:, 1], want[:, 0]))]  # rank == slot
        assert_same(eng.tick(), want, f"skew tick {t}")
        assert len(want) > 1000
    check_relation("last tick")
    st = eng.stats()
    assert st["dense_movers"] > n  # the global-memory path was taken
    assert (st["band_movers"] > n) == (path != "ring")


@pytest.mark.parametrize("seed", range(3))
def test_device_mixed_ops_with_silent(gpu, po, seed):
    """gwaoi_stage_ops_device: Enter/Leave/Moved from device arrays in one batch, some ops SILENT
    (applied, their mover's events not reported). Expected: the oracle's events for the same call
    sequence minus those raised by silent ops; the relation is unaffected by silence."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    case = H.case_random_ops(seed=500 + seed, n=1500, nticks=8, ops_per_tick=1200, world=600.0, dist=60.0,
                             dup=False)
    rng = np.random.default_rng(seed)
    eng = Engine(case["dist"], capacity=case["cap"])
    orc = po.XZListOracle(case["dist"], case["cap"])
    cap = case["cap"]
    bs, bx, bz, bk = DeviceBuffer(4 * cap), DeviceBuffer(4 * cap), DeviceBuffer(4 * cap), DeviceBuffer(cap)
    for t, ops in enumerate(case["ticks"]):
        kinds = np.asarray([o[0] for o in ops], np.uint8)
        silent = rng.random(len(ops)) < 0.3
        bs.upload(np.asarray([o[1] for o in ops], np.uint32))
        bx.upload(np.asarray([o[2] for o in ops], np.float32))
        bz.upload(np.asarray([o[3] for o in ops], np.float32))
        bk.upload(kinds | np.where(silent, _lib.GWAOI_OP_SILENT, 0).astype(np.uint8))
        want = H.oracle_tick(orc, ops)
        loud = {o[1] for o, sl in zip(ops, silent) if not sl}
        want = want[np.isin(want[:, 0], list(loud))] if len(want) else want
        eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, len(ops))
        got = eng.tick()
        assert_same(got, want, f"mixed tick {t}")
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
    with pytest.raises(_lib.GwaoiError) as e:  # host staging is refused once presence lives on the device
        eng.moved(0, 0.0, 0.0)
    assert e.value.code == _lib.GWAOI_ERR_STATE


def test_device_mixed_ops_validation(gpu):
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    eng = Engine(100.0, 16)
    bs, bx, bk = DeviceBuffer(64), DeviceBuffer(64), DeviceBuffer(16)
    bs.upload(np.asarray([1, 2], np.uint32))
    bx.upload(np.zeros(2, np.float32))
    bk.upload(np.asarray([_lib.GWAOI_OP_ENTER, _lib.GWAOI_OP_ENTER], np.uint8))
    eng.stage_ops_device(bs.ptr, bx.ptr, bx.ptr, bk.ptr, 2)
    assert eng.tick().tolist() == [[2, 1 | H.EV_ENTER]]
    bk.upload(np.asarray([_lib.GWAOI_OP_ENTER], np.uint8))  # slot 1 is present: Enter is misuse
    eng.stage_ops_device(bs.ptr, bx.ptr, bx.ptr, bk.ptr, 1)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


@pytest.mark.parametrize("silent", [False, True])
def test_device_enters_into_spaces(gpu, po, silent):
    """gwaoi_stage_ops_device_spaces: a device-staged bulk Enter into several Spaces (the bench's
    restore pass). Loud: the events of one oracle per Space in op order; silent: none, and the same
    relation either way. A Space id out of range fails the batch."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    rng = np.random.default_rng(11)
    dists, per = [30.0, 60.0, 120.0], 700
    cap = per * len(dists)
    eng = Engine(capacity=cap, spaces=[(d, (0.0, 0.0, 800.0, 800.0)) for d in dists])
    orcs = [po.XZListOracle(d, cap) for d in dists]
    order = rng.permutation(cap).astype(np.uint32)
    space_of = (order % len(dists)).astype(np.uint32)
    pos = rng.uniform(0, 800, (cap, 2)).astype(np.float32)
    want = []
    for s, sp in zip(order, space_of):
        o = orcs[sp]
        o.enter(int(s), float(pos[s, 0]), float(pos[s, 1]))
        ev = o.take_events()
        if len(ev):
            want.append(ev[np.argsort(ev[:, 1], kind="stable")])
    want = np.concatenate(want)
    bs, bx, bz, bk, bp = (DeviceBuffer(4 * cap) for _ in range(5))
    bs.upload(order)
    bx.upload(np.ascontiguousarray(pos[order, 0]))
    bz.upload(np.ascontiguousarray(pos[order, 1]))
    bk.upload(np.full(cap, _lib.GWAOI_OP_ENTER | (_lib.GWAOI_OP_SILENT if silent else 0), np.uint8))
    bp.upload(space_of)
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, cap, bp.ptr)
    got = eng.tick()
    if silent:
        assert len(got) == 0
    else:
        assert_same(got, want, "device enters into Spaces")
    rg = eng.relation()
    rel = [o.relation() for o in orcs]
    assert np.array_equal(rg[0], sum(r[0].astype(np.int64) for r in rel))
    # rows interleave Spaces: compare row by row
    cols = [np.split(r[1], r[0][1:-1].astype(np.int64)) for r in rel]
    gcols = np.split(rg[1], rg[0][1:-1].astype(np.int64))
    for s in range(cap):
        assert np.array_equal(gcols[s], cols[space_of[np.nonzero(order == s)[0][0]]][s]), f"row {s}"
    assert eng.count()[0] == cap
    bad = Engine(capacity=8, spaces=[(10.0, None), (20.0, None)])
    bs.upload(np.asarray([0, 1], np.uint32))
    bk.upload(np.asarray([_lib.GWAOI_OP_ENTER] * 2, np.uint8))
    bp.upload(np.asarray([1, 2], np.uint32))  # Space 2 does not exist
    bad.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, 2, bp.ptr)
    with pytest.raises(_lib.GwaoiError) as e:
        bad.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


def test_device_counted_batch(gpu, po):
    """gwaoi_stage_ops_device_n: the op count lives in device memory (n_max only bounds it). The
    events equal those of the same batch staged with its exact count; a count above the bound fails
    the batch."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    case = H.case_random_ops(seed=77, n=900, nticks=6, ops_per_tick=700, world=500.0, dist=50.0, dup=False)
    cap = case["cap"]
    a, b = Engine(case["dist"], capacity=cap), Engine(case["dist"], capacity=cap)
    orc = po.XZListOracle(case["dist"], cap)
    bs, bx, bz, bk, bn = DeviceBuffer(4 * cap), DeviceBuffer(4 * cap), DeviceBuffer(4 * cap), DeviceBuffer(cap), \
        DeviceBuffer(4)
    for t, ops in enumerate(case["ticks"]):
        bs.upload(np.asarray([o[1] for o in ops], np.uint32))
        bx.upload(np.asarray([o[2] for o in ops], np.float32))
        bz.upload(np.asarray([o[3] for o in ops], np.float32))
        bk.upload(np.asarray([o[0] for o in ops], np.uint8))
        bn.upload(np.asarray([len(ops)], np.uint32))
        want = H.oracle_tick(orc, ops)
        a.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, len(ops))
        b.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, cap, d_count=bn.ptr)  # bound = capacity
        ga, gb = a.tick(), b.tick()
        assert_same(ga, want, f"exact count tick {t}")
        assert_same(gb, want, f"device count tick {t}")
        assert b.last.n_ops == len(ops)
    bn.upload(np.asarray([5], np.uint32))
    b.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, 4, d_count=bn.ptr)  # 5 > bound 4
    with pytest.raises(_lib.GwaoiError) as e:
        b.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


def test_long_event_slices(gpu, po):
    """A crowd of 5,000 inside one AOI box: the i-th Enter raises i events, so per-op event slices run
    from 0 to 4,999 and the canonical ordering takes every path (insertion sort for short slices, one
    LDS bitonic chunk, and several chunks merged by rank past 2,048); a Leave and a teleport out of the
    crowd then raise 4,999 each. Bit-exact against oracle (i), the relation (rows of 4,999 neighbours)
    too."""
    rng = np.random.default_rng(0x511CE)
    n = 5000
    x = rng.uniform(0.0, 90.0, n).astype(np.float32)
    z = rng.uniform(0.0, 90.0, n).astype(np.float32)
    case = {"name": "crowd", "dist": 100.0, "cap": n, "bounds": (-500.0, -500.0, 500.0, 500.0), "ticks": [
        [(H.ENTER, i, float(x[i]), float(z[i])) for i in range(n)],
        [(H.LEAVE, 17, 0.0, 0.0), (H.MOVE, 3, 400.0, 400.0), (H.MOVE, 9, float(x[9]) + 0.5, float(z[9]))],
        [(H.MOVE, 3, float(x[3]), float(z[3])), (H.ENTER, 17, 45.0, 45.0)],
    ]}
    eng, _ = run_against_oracle(po, case, check_relation_every=1)  # rows of 4,999: chunked row sort
    rp_dev, cols_dev, nnz = eng.relation_device()
    assert rp_dev and cols_dev and nnz == len(eng.relation()[1])
    eng.close()


def test_nonfinite_refused(gpu):
    """NaN / +-Inf coordinates are refused (deliberate divergence): go-aoi's list manager
    takes them and a NaN node then cuts other entities' Mark walks (tests/test_oracle.py::
    test_nonfinite_coordinates_in_the_list_manager). Host calls return GWAOI_ERR_INVALID and stage
    nothing (batches are validated whole); a device batch fails its device check."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    eng = Engine(100.0, 16)
    eng.enter(0, 0.0, 0.0)
    eng.enter(1, 10.0, 0.0)
    assert eng.tick().tolist() == [[1, 0 | H.EV_ENTER]]
    for bad in (float("nan"), float("inf"), float("-inf")):
        with pytest.raises(_lib.GwaoiError) as e:
            eng.enter(2, bad, 0.0)
        assert e.value.code == _lib.GWAOI_ERR_INVALID
        with pytest.raises(_lib.GwaoiError) as e:
            eng.moved(0, 0.0, bad)
        assert e.value.code == _lib.GWAOI_ERR_INVALID
    with pytest.raises(_lib.GwaoiError) as e:  # one bad entry: none of the batch is staged
        eng.stage_moves(np.array([0, 1], np.uint32), np.array([1.0, float("nan")], np.float32),
                        np.zeros(2, np.float32))
    assert e.value.code == _lib.GWAOI_ERR_INVALID and eng.count() == (2, 0)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.stage_enters(np.array([2, 3], np.uint32), np.array([1.0, 2.0], np.float32),
                         np.array([0.0, float("inf")], np.float32))
    assert e.value.code == _lib.GWAOI_ERR_INVALID and eng.count() == (2, 0)
    eng.moved(0, 150.0, 0.0)  # the manager is still usable
    assert eng.tick().tolist() == [[0, 1]]
    bs, bx, bz = DeviceBuffer(8), DeviceBuffer(8), DeviceBuffer(8)
    bs.upload(np.array([0, 1], np.uint32))
    bx.upload(np.array([1.0, float("nan")], np.float32))
    bz.upload(np.zeros(2, np.float32))
    eng.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, 2)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK
