"""gwaoi_stage_buffers / gwaoi_stage_moves_pinned (the zero-copy Moved path of the cgo wrapper,
INTEGRATION.md §2): the batch is validated on the device and a repeated slot splits it into
sub-passes there. Bar: bit-exact against oracle (i) (the go-aoi XZListAOIManager restatement) op by
op, and identical to the host-validated gwaoi_stage_moves; a refused batch stages nothing."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402

pytestmark = pytest.mark.gpu


def assert_same(a, b, what):
    assert np.array_equal(a, b), what + ": " + H.fmt_diff(a, b)


@pytest.mark.parametrize("seed,bounded,mode,chunk", [(31, True, "sync", 0), (32, False, "sync", 0),
                                                    (33, False, "sync", 0), (34, False, "async", 0),
                                                    (35, True, "async", 7), (36, False, "sync", 5),
                                                    (37, False, "async", 64)])
def test_pinned_random_ops_vs_oracle(gpu, oracle_lib, seed, bounded, mode, chunk):
    """Random Enter/Leave/Moved mixes with slots moved up to three times per tick, teleports and
    lattice ties; unbounded managers (NewXZListAOIManager(d): auto extent) see coordinates far outside
    their grid, reported by the device check. mode "async": the verdict and the repeat cut stay on the
    device (gwaoi_stage_moves_pinned_async); chunk: incremental pushes every `chunk` Moved calls."""
    from goworld_amd.engine import Engine
    case = H.case_random_ops(seed=seed, n=300, nticks=10, ops_per_tick=400, world=300.0, dist=40.0)
    eng = Engine(case["dist"], capacity=case["cap"], bounds=(-400.0, -400.0, 400.0, 400.0) if bounded else None)
    orc = oracle_lib.XZListOracle(case["dist"], case["cap"])
    rng = np.random.default_rng(seed)
    present = set()
    for t, ops in enumerate(case["ticks"]):
        for kind, s, _, _ in ops:
            if kind == H.ENTER:
                present.add(s)
            elif kind == H.LEAVE:
                present.discard(s)
        # extra moves of present slots, some far away (auto extent), appended: repeats of earlier slots
        extra = []
        for s in rng.choice(sorted(present), size=min(60, len(present)), replace=False):
            far = rng.random() < 0.2
            x, z = rng.uniform(-5000, 5000, 2) if far else rng.uniform(-300, 300, 2)
            extra.append((H.MOVE, int(s), float(np.float32(x)), float(np.float32(z))))
        ops = ops + extra
        want = H.oracle_tick(orc, ops)
        got = H.gpu_tick_pinned(eng, ops, mode=mode, chunk=chunk)
        assert_same(got, want, f"seed {seed} tick {t}")
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
    eng.close()


def test_pinned_equals_host_staging_walk(gpu, oracle_lib):
    """A config-1-style walk staged through the pinned buffers equals gwaoi_stage_moves and oracle (i),
    including a tick that moves every slot twice (two sub-passes found on the device)."""
    from goworld_amd.engine import Engine
    n, L = 20_000, 4000.0
    po = oracle_lib
    x, z = po.workload_init(0x5EED00A1, n, L)
    a = Engine(100.0, capacity=n, bounds=(0.0, 0.0, L, L))
    b = Engine(100.0, capacity=n, bounds=(0.0, 0.0, L, L))
    slots = np.arange(n, dtype=np.uint32)
    a.stage_enters(slots, x, z)
    b.stage_enters(slots, x, z)
    assert np.array_equal(a.tick(), b.tick())
    orc = po.XZListOracle(100.0, n)
    orc.bulk_enter(slots, x, z)
    orc.take_events()
    ps, px, pz = b.stage_buffers()
    for t in range(1, 5):
        po.workload_step(0x5EED00A1, t, x, z, L, 1.0)
        if t == 3:  # every slot twice: the second half of the batch repeats the first
            x2 = (x + np.float32(0.5)).astype(np.float32)
            ss, xs, zs = np.concatenate([slots, slots]), np.concatenate([x, x2]), np.concatenate([z, z])
            a.stage_moves(ss, xs, zs)
            for k in range(2):
                ps[:n], px[:n], pz[:n] = slots, (x, x2)[k], z
                b.stage_moves_pinned(n)
            ops = [(H.MOVE, int(ss[i]), float(xs[i]), float(zs[i])) for i in range(2 * n)]
            x[:] = x2
        else:
            a.stage_moves(slots, x, z)
            ps[:n], px[:n], pz[:n] = slots, x, z
            b.stage_moves_pinned(n)
            ops = [(H.MOVE, i, float(x[i]), float(z[i])) for i in range(n)]
        ea, eb = a.tick(), b.tick()
        assert_same(eb, ea, f"tick {t} pinned vs stage_moves")
        assert_same(eb, H.oracle_tick(orc, ops), f"tick {t} vs oracle (i)")
        assert len(eb) > 100
    a.close()
    b.close()


def test_pinned_refuses_bad_batch_and_stages_nothing(gpu):
    """Validation on the device, all-or-nothing like gwaoi_stage_moves: a slot not in a Space
    (GWAOI_ERR_STATE), a slot out of range or a non-finite coordinate (GWAOI_ERR_INVALID). Nothing of
    a refused batch is applied and the manager stays usable; ops staged before it still run."""
    from goworld_amd import _lib
    from goworld_amd.engine import Engine
    eng = Engine(100.0, 64)
    eng.enter(0, 0.0, 0.0)
    eng.enter(1, 10.0, 0.0)
    assert eng.tick().tolist() == [[1, 0 | H.EV_ENTER]]
    ps, px, pz = eng.stage_buffers()
    assert len(ps) == 64
    cases = [((0, 5), (1.0, 2.0), _lib.GWAOI_ERR_STATE),      # slot 5 not in a Space
             ((0, 64), (1.0, 2.0), _lib.GWAOI_ERR_INVALID),   # slot >= capacity
             ((0, 1), (1.0, float("nan")), _lib.GWAOI_ERR_INVALID),
             ((0, 1), (float("inf"), 1.0), _lib.GWAOI_ERR_INVALID)]
    for sl, xs, code in cases:
        eng.moved(1, 20.0, 0.0)  # staged before the batch: runs first, kept for the tick
        ps[:2], px[:2], pz[:2] = sl, xs, (0.0, 0.0)
        with pytest.raises(_lib.GwaoiError) as e:
            eng.stage_moves_pinned(2)
        assert e.value.code == code, (sl, xs)
        assert "nothing staged" in str(e.value)
        assert eng.tick().tolist() == []  # slot 1's move to 20 raised nothing; the batch nothing
    ps[:2], px[:2], pz[:2] = (0, 1), (150.0, 20.0), (0.0, 0.0)
    eng.stage_moves_pinned(2)
    assert eng.tick().tolist() == [[0, 1]]  # slot 0 leaves slot 1's box: the manager still works
    eng.close()


@pytest.mark.parametrize("chunk", [0, 4096])
def test_pinned_async_walk_with_sub_passes(gpu, oracle_lib, chunk):
    """The async path on a config-1-style walk: equal to gwaoi_stage_moves and oracle (i) every tick,
    including a tick whose batch moves every slot twice (the repeat cut found on the device and the
    second half run as a sub-pass by the pass that reads the verdict), with and without incremental
    pushes of the arrays."""
    from goworld_amd.engine import Engine
    n, L = 20_000, 4000.0
    po = oracle_lib
    x, z = po.workload_init(0x5EED00A2, n, L)
    a = Engine(100.0, capacity=2 * n, bounds=(0.0, 0.0, L, L))
    b = Engine(100.0, capacity=2 * n, bounds=(0.0, 0.0, L, L))
    slots = np.arange(n, dtype=np.uint32)
    a.stage_enters(slots, x, z)
    b.stage_enters(slots, x, z)
    assert np.array_equal(a.tick(), b.tick())
    orc = po.XZListOracle(100.0, 2 * n)
    orc.bulk_enter(slots, x, z)
    orc.take_events()
    ps, px, pz = b.stage_buffers()
    for t in range(1, 5):
        po.workload_step(0x5EED00A2, t, x, z, L, 1.0)
        if t == 3:  # every slot twice in ONE batch of 2n
            x2 = (x + np.float32(0.5)).astype(np.float32)
            ss, xs, zs = np.concatenate([slots, slots]), np.concatenate([x, x2]), np.concatenate([z, z])
            m = 2 * n
            x[:] = x2
        else:
            ss, xs, zs = slots, x.copy(), z.copy()
            m = n
        a.stage_moves(ss, xs, zs)
        ps[:m], px[:m], pz[:m] = ss, xs, zs
        if chunk:
            for k in range(chunk, m, chunk):
                b.stage_moves_pinned_partial(k)
        b.stage_moves_pinned_async(m)
        ops = [(H.MOVE, int(ss[i]), float(xs[i]), float(zs[i])) for i in range(m)]
        ea, eb = a.tick(), b.tick()
        assert_same(eb, ea, f"tick {t} async vs stage_moves")
        assert_same(eb, H.oracle_tick(orc, ops), f"tick {t} vs oracle (i)")
        assert len(eb) > 100
    a.close()
    b.close()


def test_pinned_async_refusal_reported_by_tick(gpu):
    """gwaoi_stage_moves_pinned_async: the same refusals as the sync call (codes and message), reported by
    the pass that reads the device's verdict; nothing of the batch applied, ops staged before it still run,
    the manager stays usable."""
    from goworld_amd import _lib
    from goworld_amd.engine import Engine
    eng = Engine(100.0, 64)
    eng.enter(0, 0.0, 0.0)
    eng.enter(1, 10.0, 0.0)
    assert eng.tick().tolist() == [[1, 0 | H.EV_ENTER]]
    ps, px, pz = eng.stage_buffers()
    cases = [((0, 5), (1.0, 2.0), _lib.GWAOI_ERR_STATE),
             ((0, 64), (1.0, 2.0), _lib.GWAOI_ERR_INVALID),
             ((0, 1), (1.0, float("nan")), _lib.GWAOI_ERR_INVALID),
             ((1, 1), (150.0, float("inf")), _lib.GWAOI_ERR_INVALID)]  # refused although it repeats a slot
    for sl, xs, code in cases:
        eng.moved(1, 20.0, 0.0)  # staged before the batch: runs first
        ps[:2], px[:2], pz[:2] = sl, xs, (0.0, 0.0)
        eng.stage_moves_pinned_async(2)
        with pytest.raises(_lib.GwaoiError) as e:
            eng.tick()
        assert e.value.code == code, (sl, xs)
        assert "nothing staged" in str(e.value)
        assert eng.tick().tolist() == []  # nothing of the batch was applied
    ps[:2], px[:2], pz[:2] = (0, 1), (150.0, 20.0), (0.0, 0.0)
    eng.stage_moves_pinned_async(2)
    assert eng.tick().tolist() == [[0, 1]]
    eng.close()


def test_pinned_partial_push_discarded_by_host_pass(gpu, oracle_lib):
    """An incremental push followed by a pass of host-staged ops (which writes the device op arrays): the
    final call copies the pushed entries again, so the batch is still exact against oracle (i)."""
    from goworld_amd.engine import Engine
    eng = Engine(40.0, 256)
    orc = oracle_lib.XZListOracle(40.0, 256)
    rng = np.random.default_rng(7)
    pos = rng.uniform(-100, 100, (200, 2)).astype(np.float32)
    ops = [(H.ENTER, i, float(pos[i, 0]), float(pos[i, 1])) for i in range(200)]
    assert_same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), "enter")
    ps, px, pz = eng.stage_buffers()
    for mode in ("sync", "async"):
        mv = rng.uniform(-100, 100, (150, 2)).astype(np.float32)
        ps[:150], px[:150], pz[:150] = np.arange(150, dtype=np.uint32), mv[:, 0], mv[:, 1]
        eng.stage_moves_pinned_partial(100)
        e1 = [(H.ENTER, 210, 5.0, 5.0)]  # a host-staged Enter run on its own (gwaoi_enter + tick)
        assert_same(H.gpu_tick(eng, e1), H.oracle_tick(orc, e1), "enter between push and flush")
        orc_ops = [(H.LEAVE, 210, 0.0, 0.0)]
        assert_same(H.gpu_tick(eng, orc_ops), H.oracle_tick(orc, orc_ops), "leave")
        (eng.stage_moves_pinned_async if mode == "async" else eng.stage_moves_pinned)(150)
        ops = [(H.MOVE, i, float(mv[i, 0]), float(mv[i, 1])) for i in range(150)]
        assert_same(eng.tick(), H.oracle_tick(orc, ops), mode)
    with pytest.raises(Exception):
        eng.stage_moves_pinned_partial(10)
        eng.stage_moves_pinned_partial(5)  # below what was pushed
    eng.close()
