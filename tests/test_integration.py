"""The drop-in boundary as GoWorld would use it:

  * the C ABI from plain C in the Go wrapper's call order (tests/abi_smoke.c, gcc-built);
  * goworld_amd.aoi.GPUAOIManager (the Python mirror of the Go wrapper) replaying each tick's events
    into AOICallback objects that keep InterestedIn / InterestedBy sets the way Entity.interest /
    uninterest do (/root/reference/engine/entity/Entity.go:227-246); the sets are checked against
    oracle (i)'s relation after every tick, and a released slot must not be reused before its events
    were replayed;
  * the uint32 overflow guards of the relation view and the sync fan-out, driven through
    the index-limit test hook.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMOKE_BIN = os.path.join(ROOT, "tests", "_bin", "abi_smoke")


def test_abi_smoke_compiles_as_c(tmp_path, gwaoi_lib):
    """include/gwaoi.h + gwaoi_tools.h are plain C: the smoke driver compiles with gcc -std=c11 -Werror
    and links against libgwaoi.so (what a cgo binding does). No GPU needed to link."""
    out = tmp_path / "abi_smoke"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "abi_smoke.c"), "-L" + os.path.join(ROOT, "goworld_amd"),
                    "-lgwaoi", "-lm", "-o", str(out)], check=True)
    assert out.exists()


@pytest.mark.gpu
def test_abi_smoke_c_driver(gpu):
    """tests/abi_smoke.c on the GPU: Enter with flush, Moved batched into one gwaoi_stage_moves per
    tick (a slot moved twice included), Leave after the pending moves, misuse and NaN reported."""
    if not os.path.exists(SMOKE_BIN):
        pytest.fail("tests/_bin/abi_smoke missing: run __graft_entry__.build()")
    r = subprocess.run([SMOKE_BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_smoke ok" in r.stdout


class Entity:
    """The AOI part of engine/entity's Entity: InitAOI(&e.aoi, dist, e, e) (Entity.go:210) and the
    callbacks (Entity.go:227-246): OnEnterAOI -> interest(other), OnLeaveAOI -> uninterest(other)."""

    def __init__(self, eid):
        from goworld_amd.aoi import AOI, InitAOI
        self.eid = eid
        self.aoi = AOI()
        InitAOI(self.aoi, 100.0, self, self)
        self.interested_in = set()
        self.interested_by = set()
        self.enter_calls = 0
        self.leave_calls = 0

    def OnEnterAOI(self, other_aoi):
        other = other_aoi.Data
        self.enter_calls += 1
        assert other not in self.interested_in, "double enter"
        self.interested_in.add(other)        # e.InterestedIn.Add(other)
        other.interested_by.add(self)        # other.InterestedBy.Add(e)

    def OnLeaveAOI(self, other_aoi):
        other = other_aoi.Data
        self.leave_calls += 1
        assert other in self.interested_in, "leave without enter"
        self.interested_in.discard(other)    # e.InterestedIn.Del(other)
        other.interested_by.discard(self)    # other.InterestedBy.Del(e)


def check_sets(ents, orc, what):
    rp, cols = orc.relation()
    for e in ents:
        want = {int(c) for c in cols[rp[e.eid]:rp[e.eid + 1]]}
        got_in = {o.eid for o in e.interested_in}
        got_by = {o.eid for o in e.interested_by}
        assert got_in == want, f"{what}: InterestedIn({e.eid}) {sorted(got_in ^ want)[:8]}"
        assert got_by == want, f"{what}: InterestedBy({e.eid}) {sorted(got_by ^ want)[:8]}"


@pytest.mark.gpu
@pytest.mark.parametrize("sync_enter_leave", [True, False])
def test_gpu_aoi_manager_replays_into_entity_sets(gpu, oracle_lib, sync_enter_leave):
    from goworld_amd.aoi import NewXZListAOIManager
    case = H.case_random_ops(seed=77 if sync_enter_leave else 78, n=300, nticks=10, ops_per_tick=220, world=400.0,
                             dist=100.0)
    mgr = NewXZListAOIManager(100.0, capacity=400, sync_enter_leave=sync_enter_leave)
    orc = oracle_lib.XZListOracle(100.0, 300)
    ents = [Entity(i) for i in range(300)]
    for t, ops in enumerate(case["ticks"]):
        for kind, s, x, z in ops:
            e = ents[s]
            if kind == H.ENTER:
                mgr.Enter(e.aoi, x, z)
                orc.enter(s, x, z)
            elif kind == H.LEAVE:
                slot = e.aoi._slot
                mgr.Leave(e.aoi)
                orc.leave(s)
                if not sync_enter_leave:  # the slot is held until the tick's events are replayed
                    assert slot not in mgr._free and mgr._by_slot[slot] is e.aoi
            else:
                mgr.Moved(e.aoi, x, z)
                orc.moved(s, x, z)
        mgr.Flush()
        orc.take_events()
        check_sets(ents, orc, f"tick {t}")
        assert not mgr._released
    # every pair event fired both callbacks (mover's first, then the other's)
    assert sum(e.enter_calls for e in ents) % 2 == 0 and sum(e.leave_calls for e in ents) % 2 == 0
    mgr.close()


@pytest.mark.gpu
def test_moved_twice_in_one_tick_replays(gpu):
    """The mirror batches Moved like the Go wrapper (one gwaoi_stage_moves_pinned per flush). A slot
    moved twice in one tick splits the batch into two sub-passes on the device: b walks into a's box
    and out again, so the tick replays ENTER then LEAVE of the pair (both callbacks each) and the sets
    end empty, exactly as two sequential go-aoi Moved calls."""
    from goworld_amd.aoi import NewXZListAOIManager
    mgr = NewXZListAOIManager(100.0, capacity=8)
    a, b, c = Entity(0), Entity(1), Entity(2)
    mgr.Enter(a.aoi, 0.0, 0.0)
    mgr.Enter(b.aoi, 150.0, 0.0)
    mgr.Enter(c.aoi, 400.0, 0.0)
    mgr.Flush()
    assert not a.interested_in and not b.interested_in
    mgr.Moved(b.aoi, 50.0, 0.0)
    mgr.Moved(c.aoi, 390.0, 0.0)
    mgr.Moved(b.aoi, 150.0, 0.0)  # repeats b: the device cuts the batch here
    assert mgr.Flush() == 2
    ev = mgr.last_events.tolist()
    sa, sb = a.aoi._slot, b.aoi._slot
    assert ev == [[sb, sa | 0x80000000], [sb, sa]]
    assert a.enter_calls == b.enter_calls == 1 and a.leave_calls == b.leave_calls == 1
    assert not a.interested_in and not b.interested_in and not a.interested_by
    mgr.close()


@pytest.mark.gpu
def test_slot_reuse_waits_for_replay(gpu):
    """Leave then Enter of another entity in one batched tick: the new entity must not get the leaver's
    slot before the leaver's LEAVE events were replayed (they name that slot)."""
    from goworld_amd.aoi import NewXZListAOIManager
    mgr = NewXZListAOIManager(100.0, capacity=3, sync_enter_leave=False)
    a, b, c = Entity(0), Entity(1), Entity(2)
    mgr.Enter(a.aoi, 0.0, 0.0)
    mgr.Enter(b.aoi, 10.0, 0.0)
    mgr.Flush()
    assert b in a.interested_in and a in b.interested_in
    old = b.aoi._slot
    mgr.Leave(b.aoi)
    mgr.Enter(c.aoi, 5.0, 0.0)  # capacity 3: c gets the third slot, not b's
    assert c.aoi._slot != old
    mgr.Flush()
    assert a.interested_in == {c} and c.interested_in == {a} and not b.interested_in and not b.interested_by
    assert old in mgr._free
    mgr.close()


@pytest.mark.gpu
def test_index_limit_guards(gpu, oracle_lib):
    """The relation view's row_ptr and the fan-out's pair offsets are uint32: a total above the limit
    fails with GWAOI_ERR_NOMEM before anything is sized or written (2^32 wraparound). The
    test hook lowers the limit to below this world's totals."""
    from goworld_amd import _lib
    from goworld_amd.sync import EntitySync
    from test_sync import check_collect, fill_sync, world
    eng, orc, x, z = world(oracle_lib, 1500, 900.0, 100.0, 5)
    nnz = len(orc.relation()[1])
    eng.debug_set_index_limit(nnz - 1)
    with pytest.raises(_lib.GwaoiError) as e:
        eng.relation_device()
    assert e.value.code == _lib.GWAOI_ERR_NOMEM
    eng.debug_set_index_limit(nnz)
    assert eng.relation_device()[2] == nnz
    sy = EntitySync(eng, 3)
    st = fill_sync(sy, np.random.default_rng(5), 1500, 3)
    eng.debug_set_index_limit(10)
    with pytest.raises(_lib.GwaoiError) as e:
        sy.collect_entity_sync_infos(keep_flags=True)
    assert e.value.code == _lib.GWAOI_ERR_NOMEM
    eng.debug_set_index_limit(1 << 40)  # clamped to 2^32 - 1
    check_collect(sy, orc, st, x, z, 3)


@pytest.mark.gpu
def test_adopt_device_state_then_host_staging(gpu, oracle_lib):
    """A silent bulk restore from HBM (mixed device batch, EntityManager.go:591-652) followed by host-staged
    Moved calls: gwaoi_adopt_device_state pulls presence back to the host mirror; events then equal the
    list oracle's for the same calls."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    case = H.case_walk(0x5EED00AD, 4000, 1400.0, 4, workload=oracle_lib)
    n = 4000
    x0 = np.asarray([o[2] for o in case["ticks"][0]], np.float32)
    z0 = np.asarray([o[3] for o in case["ticks"][0]], np.float32)
    eng = Engine(100.0, n, bounds=case["bounds"])
    bs, bx, bz, bk = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(n)
    bs.upload(np.arange(n, dtype=np.uint32))
    bx.upload(x0)
    bz.upload(z0)
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n)
    assert len(eng.tick()) == 0
    with pytest.raises(_lib.GwaoiError):
        eng.moved(0, 1.0, 1.0)  # presence lives on the device
    eng.adopt_device_state()
    assert eng.count() == (n, 0)
    orc = oracle_lib.XZListOracle(100.0, n)
    orc.bulk_enter(np.arange(n, dtype=np.uint32), x0, z0)
    for t, ops in enumerate(case["ticks"][1:], 1):
        want = H.oracle_tick(orc, ops)
        got = H.gpu_tick(eng, ops)
        assert np.array_equal(got, want), f"tick {t}: " + H.fmt_diff(got, want)
    rg, ro = eng.relation(), orc.relation()
    assert np.array_equal(rg[0], ro[0]) and np.array_equal(rg[1], ro[1])
