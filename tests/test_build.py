"""The one-pass tile build (k_bin_tfused) against the counting build and the oracle, through the C ABI.

The one-pass build buckets a pass's records by the PREVIOUS tile build's starts (25% + 15 records of
room per tile); a pass whose tile grew past that re-runs with the counting build. Both must give
bit-identical events and relations, and the re-run must leave no trace in the results: a burst that
crowds half the world into one tile is checked against oracle (ii) tick by tick.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402

pytestmark = pytest.mark.gpu


def walk_with_burst(seed, n=4000, L=2000.0, dist=25.0, nticks=8, burst_at=4, frac=0.5):
    """Tick 0 Enters n entities uniformly; every later tick moves every slot by up to 2 units, except
    tick `burst_at`, where `frac` of the slots jump into one 60 x 60 square (a tile that grows far past
    its room) and tick `burst_at` + 2, where they jump back out."""
    rng = np.random.default_rng(seed)
    p = rng.uniform(0, L, (n, 2)).astype(np.float32)
    ticks = [[(H.ENTER, i, float(p[i, 0]), float(p[i, 1])) for i in range(n)]]
    crowd = rng.random(n) < frac
    for t in range(1, nticks):
        step = rng.uniform(-2, 2, (n, 2)).astype(np.float32)
        p = np.clip(p + step, 0, L).astype(np.float32)
        if t == burst_at:
            p[crowd] = rng.uniform(700, 760, (int(crowd.sum()), 2)).astype(np.float32)
        if t == burst_at + 2:
            p[crowd] = rng.uniform(0, L, (int(crowd.sum()), 2)).astype(np.float32)
        ticks.append([(H.MOVE, i, float(p[i, 0]), float(p[i, 1])) for i in range(n)])
    return dict(name=f"burst_{seed}", dist=dist, cap=n, ticks=ticks, bounds=(0.0, 0.0, L, L))


def _engine(case):
    from goworld_amd.engine import Engine
    return Engine(case["dist"], capacity=case["cap"], bounds=case.get("bounds"))


def test_burst_reruns_and_matches_oracle(gpu, oracle_lib):
    case = walk_with_burst(7)
    eng = _engine(case)
    orc = oracle_lib.GridOracle(case["dist"], case["cap"], case["bounds"])
    for t, ops in enumerate(case["ticks"]):
        want = H.oracle_tick(orc, ops)
        got = H.gpu_tick(eng, ops)
        assert np.array_equal(got, want), f"tick {t}: " + H.fmt_diff(got, want)
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
    fused, counting, reruns = eng.debug_build_mode()
    assert fused >= 4, (fused, counting, reruns)   # the steady ticks take the one-pass build
    assert reruns >= 1, (fused, counting, reruns)  # the burst overflowed its tile's room
    assert counting >= 1 + reruns


@pytest.mark.parametrize("seed", range(4))
def test_one_pass_equals_counting_build(gpu, seed):
    """Random op mixes (Enters, Leaves, teleports, repeated staging) on a multi-tile world: the default
    manager and one held to the counting build give the same events and relation every tick."""
    case = H.case_random_ops(seed=700 + seed, n=3000, nticks=10, ops_per_tick=[200, 1500, 3000, 600][seed],
                             world=1500.0, dist=20.0, snap=seed % 2 == 0)
    a, b = _engine(case), _engine(case)
    b.debug_build_mode(1)
    for t, ops in enumerate(case["ticks"]):
        ea, eb = H.gpu_tick(a, ops), H.gpu_tick(b, ops)
        assert np.array_equal(ea, eb), f"tick {t}: " + H.fmt_diff(ea, eb)
        if t % 3 == 2:
            ra, rb = a.relation(), b.relation()
            assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1]), f"relation tick {t}"
    fa, ca, _ = a.debug_build_mode()
    fb, cb, rb_ = b.debug_build_mode()
    assert fa >= 1 and fb == 0 and rb_ == 0, (fa, ca, fb, cb)


def test_build_mode_rejects_unknown(gpu):
    from goworld_amd.engine import Engine
    from goworld_amd._lib import GwaoiError
    eng = Engine(10.0, capacity=16)
    with pytest.raises(GwaoiError):
        eng.debug_build_mode(2)
