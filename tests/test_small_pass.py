"""Small passes: a pass with few ops is judged against the last full build's grid plus an
overlay of the slots with ops since, without rebuilding the grid (k_apply keeps the overlay,
k_sweep_small walks it). Bit-exact against oracle (i) on the same call sequences as the full path:
random Enter/Leave/Moved mixes (sub-passes from repeated slots included), the Go wrapper's call order
(every Enter and Leave flushed as its own pass, Space.go:188-251), device-staged batches, and readers
of the grid after small passes (relation view, sync fan-out: the grid is refreshed first)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def po(oracle_lib):
    return oracle_lib


def _engine(case, mode):
    from goworld_amd.engine import Engine
    eng = Engine(case["dist"], capacity=case["cap"], bounds=case.get("bounds"))
    eng.debug_small_pass(mode)
    return eng


def _same(a, b, what):
    assert np.array_equal(a, b), what + ": " + H.fmt_diff(a, b)


@pytest.mark.parametrize("seed", range(4))
def test_small_passes_random_mixes(gpu, po, seed):
    """Forced small passes (mode 2: whenever the overlay has room) on random op mixes: the first tick
    is a full pass (no grid yet), then the overlay grows tick after tick; the relation is checked (a
    grid reader: refreshes the grid, restarting the overlay) every third tick."""
    case = H.case_random_ops(seed=4000 + seed, n=[64, 300, 900, 2000][seed], nticks=14,
                             ops_per_tick=[12, 40, 120, 300][seed], world=[100.0, 300.0, 600.0, 1000.0][seed],
                             dist=[10.0, 50.0, 60.0, 100.0][seed], snap=seed % 2 == 0)
    eng = _engine(case, 2)
    orc = po.XZListOracle(case["dist"], case["cap"])
    for t, ops in enumerate(case["ticks"]):
        _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), f"tick {t}")
        if t % 3 == 2:
            rg, ro = eng.relation(), orc.relation()
            assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1]), f"relation tick {t}"
    assert eng.debug_small_pass() > 0


def test_small_passes_wrapper_call_order(gpu, po):
    """The cgo wrapper's default (SyncEnterLeave): a world walks in full passes while entities spawn and
    despawn one call at a time, each flushed as its own pass (small at 4,000 present)."""
    from goworld_amd.engine import Engine
    rng = np.random.default_rng(11)
    n, L, D = 5000, 2500.0, 100.0
    eng = Engine(D, capacity=n, bounds=(0.0, 0.0, L, L))
    orc = po.XZListOracle(D, n)
    pos = rng.uniform(0, L, (n, 2)).astype(np.float32)
    present = np.zeros(n, bool)
    first = np.arange(4000)
    ops = [(H.ENTER, int(s), float(pos[s, 0]), float(pos[s, 1])) for s in first]
    _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), "bulk enter")
    present[first] = True
    n0 = eng.debug_small_pass()
    for t in range(6):
        # one walking tick over everyone present (a full pass)
        mv = np.flatnonzero(present)
        pos[mv] = (pos[mv] + rng.uniform(-3, 3, (len(mv), 2))).astype(np.float32)
        ops = [(H.MOVE, int(s), float(pos[s, 0]), float(pos[s, 1])) for s in mv]
        _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), f"walk {t}")
        # a few spawns and despawns, each its own tick
        for _ in range(8):
            if rng.random() < 0.5 and (~present).any():
                s = int(rng.choice(np.flatnonzero(~present)))
                pos[s] = rng.uniform(0, L, 2).astype(np.float32)
                ops = [(H.ENTER, s, float(pos[s, 0]), float(pos[s, 1]))]
                present[s] = True
            else:
                s = int(rng.choice(np.flatnonzero(present)))
                ops = [(H.LEAVE, s, 0.0, 0.0)]
                present[s] = False
            _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), f"spawn/despawn {t}")
    assert eng.debug_small_pass() - n0 >= 40  # the single-op passes were small
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])


def test_small_passes_device_batches(gpu, po):
    """Small device-staged mixed batches (the check of every op's slot runs per op there), and a
    duplicate slot in one still fails the batch."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer
    case = H.case_random_ops(seed=77, n=600, nticks=8, ops_per_tick=30, world=400.0, dist=50.0, dup=False)
    eng = _engine(case, 2)
    orc = po.XZListOracle(case["dist"], case["cap"])
    cap = case["cap"]
    bs, bx, bz, bk = DeviceBuffer(4 * cap), DeviceBuffer(4 * cap), DeviceBuffer(4 * cap), DeviceBuffer(cap)
    present = set()
    for t, ops in enumerate(case["ticks"]):
        for kind, slot, _, _ in ops:
            if kind == H.ENTER:
                present.add(slot)
            elif kind == H.LEAVE:
                present.discard(slot)
        bs.upload(np.asarray([o[1] for o in ops], np.uint32))
        bx.upload(np.asarray([o[2] for o in ops], np.float32))
        bz.upload(np.asarray([o[3] for o in ops], np.float32))
        bk.upload(np.asarray([o[0] for o in ops], np.uint8))
        want = H.oracle_tick(orc, ops)
        eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, len(ops))
        _same(eng.tick(), want, f"tick {t}")
    assert eng.debug_small_pass() > 0
    s = min(present)
    bs.upload(np.asarray([s, s], np.uint32))  # one slot twice
    bk.upload(np.asarray([H.MOVE, H.MOVE], np.uint8))
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, 2)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


def test_small_and_full_passes_agree(gpu, po):
    """The same calls with small passes off and on (auto): identical events every tick."""
    case = H.case_random_ops(seed=91, n=3000, nticks=12, ops_per_tick=25, world=1500.0, dist=100.0)
    a, b = _engine(case, 0), _engine(case, 1)
    for t, ops in enumerate(case["ticks"]):
        _same(H.gpu_tick(b, ops), H.gpu_tick(a, ops), f"tick {t}")
    assert a.debug_small_pass() == 0


def test_small_pass_crowd_overflows_order_lds(gpu, po):
    """An Enter into a crowd: the single pass has more events than k_order_small's LDS holds (4,096), so
    the order stage falls back to the general kernels on the scanned counts; then a Leave of the same
    slot, and a Moved of a crowd member across the crowd (its slice needs the sort)."""
    from goworld_amd.engine import Engine
    rng = np.random.default_rng(5)
    n, D = 6000, 100.0
    eng = Engine(D, capacity=n + 1, bounds=(0.0, 0.0, 1000.0, 1000.0))
    eng.debug_small_pass(2)
    orc = po.XZListOracle(D, n + 1)
    pos = rng.uniform(450, 550, (n, 2)).astype(np.float32)  # every pair within D
    ops = [(H.ENTER, int(s), float(pos[s, 0]), float(pos[s, 1])) for s in range(n)]
    _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), "crowd enter")
    n0 = eng.debug_small_pass()
    for t, ops in enumerate([[(H.ENTER, n, 500.0, 500.0)], [(H.LEAVE, n, 0.0, 0.0)],
                             [(H.MOVE, 7, 451.0, 549.0)], [(H.ENTER, n, 520.0, 480.0), (H.MOVE, 9, 549.5, 450.5)]]):
        got, want = H.gpu_tick(eng, ops), H.oracle_tick(orc, ops)
        assert len(want) > 4096 or t == 2
        _same(got, want, f"crowd pass {t}")
    assert eng.debug_small_pass() - n0 == 4


def test_small_pass_above_fused_order_ops(gpu, po):
    """A forced small pass of 1,500 ops (mode 2): more ops than k_order_small takes, so the scan and
    the general order kernels run after k_sweep_small."""
    case = H.case_random_ops(seed=303, n=4000, nticks=4, ops_per_tick=1500, world=800.0, dist=60.0, dup=False)
    eng = _engine(case, 2)
    orc = po.XZListOracle(case["dist"], case["cap"])
    for t, ops in enumerate(case["ticks"]):
        _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), f"tick {t}")
    assert eng.debug_small_pass() >= 3


def test_single_op_pass_over_the_event_buffers(gpu, po):
    """A single Enter into a crowd of 70,000 (restored silently from a device batch): its 70,000 events
    exceed the event buffers, so the one-kernel pass (apply, sweep, order) overflows and the pass is
    re-run as a plain k_sweep_small without applying the op again; then the Leave of the same slot."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    rng = np.random.default_rng(23)
    n, D = 70000, 100.0
    bounds = (0.0, 0.0, 1000.0, 1000.0)
    x = rng.uniform(450, 550, n).astype(np.float32)
    z = rng.uniform(450, 550, n).astype(np.float32)
    eng = Engine(D, capacity=n + 1, bounds=bounds)
    bs, bx, bz, bk = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(n)
    bs.upload(np.arange(n, dtype=np.uint32))
    bx.upload(x)
    bz.upload(z)
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n)
    assert len(eng.tick()) == 0
    eng.adopt_device_state()
    orc = po.GridOracle(D, n + 1, bounds)
    orc.bulk_enter(np.arange(n, dtype=np.uint32), x, z)
    n0 = eng.debug_small_pass()
    for op in [(H.ENTER, n, 500.0, 500.0), (H.LEAVE, n, 0.0, 0.0)]:
        got, want = H.gpu_tick(eng, [op]), H.oracle_tick(orc, [op])
        assert len(want) == n
        _same(got, want, f"op {op[0]}")
    assert eng.debug_small_pass() - n0 == 2


def test_seq_renormalise_with_live_overlay(gpu, po):
    """a small pass that crosses the seq limit renormalises the seqs while the overlay holds
    copies of records with the old seqs. The overlay must start over (the grid is rebuilt from the
    slots' state), so the exact near-boundary tests read the renumbered seqs. Boundary-heavy world
    (snapped coordinates, D = 10 on a 1-unit lattice), small passes forced, bit-exact against oracle (i)
    before, across and after the renormalisation, and the relation after it."""
    case = H.case_random_ops(seed=8123, n=400, nticks=12, ops_per_tick=20, world=60.0, dist=10.0, snap=True)
    eng = _engine(case, 2)
    orc = po.XZListOracle(case["dist"], case["cap"])
    n0 = None
    for t, ops in enumerate(case["ticks"]):
        if t == 6:  # the overlay is non-empty here (small passes since tick 1): the next pass crosses the limit
            n0 = eng.debug_small_pass()
            eng.debug_set_next_seq(0x7ff00000 - 5)
        _same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), f"tick {t}")
    assert eng.debug_small_pass() > n0  # small passes ran after the renormalisation too
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
