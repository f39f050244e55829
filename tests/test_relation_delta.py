"""gwaoi_export_relation_delta (the relation consumer by delta): the net relation changes
of the last tick, computed on the GPU from the tick's events in O(events). Bar: exactly the symmetric
difference between oracle (i)'s relation after and before the tick, one entry per changed pair and
direction, with the right sign, no duplicates; pairs that entered and left inside one tick omitted."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402

pytestmark = pytest.mark.gpu


def pairs(rel):
    rp, cols = rel
    rows = np.repeat(np.arange(len(rp) - 1, dtype=np.uint64), np.diff(rp.astype(np.int64)))
    return set((rows << np.uint64(32) | cols.astype(np.uint64)).tolist())


def check_delta(delta, before, after, what):
    keys = delta[:, 0].astype(np.uint64) << np.uint64(32) | (delta[:, 1] & 0x7FFFFFFF).astype(np.uint64)
    assert len(set(keys.tolist())) == len(delta), f"{what}: duplicate entries"
    added = set(keys[(delta[:, 1] >> 31) == 1].tolist())
    removed = set(keys[(delta[:, 1] >> 31) == 0].tolist())
    assert added == after - before, f"{what}: added {len(added)} vs {len(after - before)}"
    assert removed == before - after, f"{what}: removed {len(removed)} vs {len(before - after)}"
    # entries come in pairs: (a, b) then (b, a), same sign
    assert np.array_equal(delta[0::2, 0], delta[1::2, 1] & 0x7FFFFFFF)
    assert np.array_equal(delta[1::2, 0], delta[0::2, 1] & 0x7FFFFFFF)
    assert np.array_equal(delta[0::2, 1] >> 31, delta[1::2, 1] >> 31)


@pytest.mark.parametrize("seed", [41, 42])
def test_delta_random_ops_vs_oracle(gpu, oracle_lib, seed):
    """Random Enter/Leave/Moved mixes with repeated slots (sub-passes: transient enter/leave pairs
    inside one tick) and teleports."""
    from goworld_amd.engine import Engine
    case = H.case_random_ops(seed=seed, n=300, nticks=10, ops_per_tick=300, world=300.0, dist=50.0)
    eng = Engine(case["dist"], capacity=case["cap"])
    orc = oracle_lib.XZListOracle(case["dist"], case["cap"])
    before = set()
    transient = 0
    for t, ops in enumerate(case["ticks"]):
        H.oracle_tick(orc, ops)
        ev = H.gpu_tick(eng, ops)
        after = pairs(orc.relation())
        d = eng.relation_delta()
        check_delta(d, before, after, f"seed {seed} tick {t}")
        transient += len(ev) - len(d) // 2
        before = after
    assert transient > 0  # the cases do hold pairs that cancel inside a tick
    eng.close()


def test_delta_walk_and_states(gpu, oracle_lib):
    """A 100k walk (config-2 density) tick by tick against oracle (ii) run in lockstep: the delta is the
    difference of the ORACLE's relations before and after each tick, and the GPU relation equals the
    oracle's. The export is refused before any tick and once a later pass has overwritten the tick's
    events."""
    from goworld_amd import _lib
    from goworld_amd.engine import Engine
    po = oracle_lib
    n, L, seed = 100_000, 11068.0, 0x5EED00B1
    x, z = po.workload_init(seed, n, L)
    eng = Engine(100.0, capacity=n, bounds=(0.0, 0.0, L, L))
    with pytest.raises(_lib.GwaoiError) as e:
        eng.relation_delta()
    assert e.value.code == _lib.GWAOI_ERR_STATE
    slots = np.arange(n, dtype=np.uint32)
    orc = po.GridOracle(100.0, n, (0.0, 0.0, L, L))
    orc.bulk_enter(slots, x, z)
    eng.stage_enters(slots, x, z)
    eng.tick()
    before = pairs(orc.relation())
    assert pairs(eng.relation()) == before
    for t in range(1, 4):
        po.workload_step(seed, t, x, z, L, 1.0)
        orc.moved_batch(slots, x, z)
        orc.take_events()
        eng.stage_moves(slots, x, z)
        ev = eng.tick()
        d = eng.relation_delta()
        after = pairs(orc.relation())
        assert pairs(eng.relation()) == after, f"walk tick {t}: relation"  # (runs no pass)
        check_delta(d, before, after, f"walk tick {t}")
        assert 0 < len(d) <= 2 * len(ev)  # both members moving: a leave then an enter can cancel
        assert np.array_equal(eng.relation_delta(), d)  # repeatable until the next pass
        before = after
    eng.moved(0, float(x[0]) + 1.0, float(z[0]))
    eng.tick()
    eng.moved(1, float(x[1]) + 1.0, float(z[1]))
    eng.relation()  # flushes the staged move: a pass ran after the tick
    with pytest.raises(_lib.GwaoiError) as e:
        eng.relation_delta()
    assert e.value.code == _lib.GWAOI_ERR_STATE
    eng.close()
