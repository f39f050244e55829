"""k_apply_moves4 (Moved-only device batches, four ops per thread, 16-B accesses for slot-ordered groups)
and the duplicate-slot check of device batches, through the C ABI.

- a group of four consecutive slots in which one op fails its check (NaN coordinate, absent slot) takes
  the per-op path and fails the batch (GWAOI_ERR_DEVICE_CHECK);
- the same slots named by two aligned groups (a duplicate across groups) fail the batch: the slots that
  acted (k_bin_tsort's per-tile counts) are fewer than the ops (k_place);
- a device-counted batch whose count is not a multiple of four gives the events of a host-staged manager.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _world(n, seed, L=400.0):
    rng = np.random.default_rng(seed)
    return rng.uniform(0, L, n).astype(np.float32), rng.uniform(0, L, n).astype(np.float32)


def _entered(n, x, z, absent=()):
    from goworld_amd.engine import Engine
    eng = Engine(60.0, n, bounds=(0.0, 0.0, 400.0, 400.0))
    for i in range(n):
        if i not in absent:
            eng.enter(i, float(x[i]), float(z[i]))
    eng.tick()
    return eng


def _dev(arr):
    from goworld_amd.engine import DeviceBuffer
    b = DeviceBuffer(max(4, arr.nbytes))
    b.upload(arr)
    return b


@pytest.mark.parametrize("bad", ["nan", "absent"])
def test_moves4_group_with_a_failing_op(gpu, bad):
    from goworld_amd import _lib
    n = 16
    x, z = _world(n, 1)
    eng = _entered(n, x, z, absent=(6,) if bad == "absent" else ())
    slots = np.arange(12, dtype=np.uint32)  # three aligned groups of four
    nx, nz = (x[:12] + 1.0).astype(np.float32), (z[:12] - 1.0).astype(np.float32)
    if bad == "nan":
        nx[5] = np.float32(np.nan)  # the middle of group 1
    bs, bx, bz = _dev(slots), _dev(nx), _dev(nz)
    eng.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, 12)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


def test_moves4_duplicate_across_groups(gpu):
    from goworld_amd import _lib
    n = 16
    x, z = _world(n, 2)
    eng = _entered(n, x, z)
    slots = np.concatenate([np.arange(8), np.arange(4, 8)]).astype(np.uint32)  # group 2 repeats group 1
    nx, nz = (x[slots] + 0.5).astype(np.float32), (z[slots] + 0.5).astype(np.float32)
    bs, bx, bz = _dev(slots), _dev(nx), _dev(nz)
    eng.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, 12)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.tick()
    assert e.value.code == _lib.GWAOI_ERR_DEVICE_CHECK


@pytest.mark.parametrize("n_dev", [1, 7, 10, 13])
def test_device_count_not_a_multiple_of_four(gpu, n_dev):
    from goworld_amd import _lib
    from goworld_amd.engine import Engine
    n = 400
    x, z = _world(n, 3)
    host = Engine(60.0, n, bounds=(0.0, 0.0, 400.0, 400.0))
    for i in range(n):
        host.enter(i, float(x[i]), float(z[i]))
    host.tick()
    dev = Engine(60.0, n, bounds=(0.0, 0.0, 400.0, 400.0))
    kinds = np.full(n, _lib.GWAOI_OP_ENTER, np.uint8)
    bs, bx, bz, bk = _dev(np.arange(n, dtype=np.uint32)), _dev(x), _dev(z), _dev(kinds)
    dev.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n)
    dev.tick()
    rng = np.random.default_rng(4)
    for t in range(3):
        slots = np.sort(rng.choice(n, 16, replace=False)).astype(np.uint32)
        nx = (x[slots] + rng.uniform(-30, 30, 16)).astype(np.float32)
        nz = (z[slots] + rng.uniform(-30, 30, 16)).astype(np.float32)
        x[slots[:n_dev]], z[slots[:n_dev]] = nx[:n_dev], nz[:n_dev]  # only the counted ops apply
        host.stage_moves(slots[:n_dev], nx[:n_dev], nz[:n_dev])
        want = host.tick()
        ds, dx, dz = _dev(slots), _dev(nx), _dev(nz)
        dk, dn = _dev(np.zeros(16, np.uint8)), _dev(np.asarray([n_dev], np.uint32))
        dev.stage_ops_device(ds.ptr, dx.ptr, dz.ptr, dk.ptr, 16, d_count=dn.ptr)
        got = dev.tick()
        assert np.array_equal(got, want), f"tick {t}: {got} vs {want}"
        assert dev.last.n_ops == n_dev
