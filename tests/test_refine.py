"""Refined cells (crowds): a grid cell of 8..64 records is split into sub-cells in the build, and the
wave-per-mover walk reads only the sub-cells its ring crosses (gwaoi_internal.h "Refined cells",
k_sweep_dense<true>). An acceleration only: the events must not change. Bar: bit-exact against oracle
(i) on crowded random op mixes (Enter/Leave/Moved, repeated slots, teleports, lattice ties), and
identical to the same manager with refinement off on a config-5 crowd."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402

pytestmark = pytest.mark.gpu


def assert_same(a, b, what):
    assert np.array_equal(a, b), what + ": " + H.fmt_diff(a, b)


@pytest.mark.parametrize("seed,dist,world", [(61, 50.0, 50.0), (62, 120.0, 150.0)])
def test_refined_crowd_random_ops_vs_oracle(gpu, oracle_lib, seed, dist, world):
    from goworld_amd.engine import Engine
    case = H.case_random_ops(seed=seed, n=1200, nticks=6, ops_per_tick=300, world=world, dist=dist)
    eng = Engine(case["dist"], capacity=case["cap"])
    eng.debug_set_refine(True)
    eng.set_timing(True)
    orc = oracle_lib.XZListOracle(case["dist"], case["cap"])
    for t, ops in enumerate(case["ticks"]):
        assert_same(H.gpu_tick(eng, ops), H.oracle_tick(orc, ops), f"seed {seed} tick {t}")
    st = eng.stats()
    assert st["refined_cells"] > 0 and st["dense_movers"] > 0, st
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
    eng.close()


def test_refined_equals_coarse_on_config5_crowd(gpu):
    """4 skewed Spaces x 250k (D = 50/100/200/400) at config 5's mean density, 50% in 64 hotspots
    (peak ~100x the mean): refinement on and off give the same events tick by tick."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces
    N, L, seed0, S = 250_000, 35000.0 * 0.5, 0x5EED0007, 4
    n = S * N
    bx, bz, bs, bk, bp = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(n), \
        DeviceBuffer(4 * n)
    wl_init_spaces(0, bx.ptr, bz.ptr, N, S, seed0, L, 64, 62.0, 2)
    wl_iota(0, bs.ptr, n)
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    bp.upload(np.repeat(np.arange(S, dtype=np.uint32), N))
    engs = []
    for refine in (False, True):
        e = Engine(capacity=n, spaces=[(d, (0.0, 0.0, L, L)) for d in (50.0, 100.0, 200.0, 400.0)])
        e.debug_set_refine(refine)
        e.set_timing(True)
        e.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n, bp.ptr)
        assert int(e.tick_device().count) == 0
        engs.append(e)
    for t in (1, 2, 3):
        wl_step_spaces(0, bx.ptr, bz.ptr, bx.ptr, bz.ptr, N, S, seed0, t, L, 1.0)
        evs = []
        for e in engs:
            e.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, n)
            evs.append(e.tick())
        assert_same(evs[1], evs[0], f"tick {t} refined vs coarse")
        assert len(evs[0]) > 100_000
    st = [e.stats() for e in engs]
    assert st[0]["refined_cells"] == 0 and st[1]["refined_cells"] > 1000, st
    assert st[1]["dense_movers"] > 0
    for e in engs:
        e.close()
