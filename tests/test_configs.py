"""Parity at the workload shapes of BASELINE.json configs 3, 4 and 5, through the C ABI.

  config 3  512 dungeon Spaces x 2,000 entities (L = 1,600, D = 100, seeds 0x5EED0003 + space) in ONE
            manager, against one oracle (i) (go-aoi XZListAOIManager restatement) per Space: the enter
            tick and 3 all-moving ticks.
  config 4  one 16M-entity world (L = 140,000) in 8 X-strips on one GPU (loopback exchange) against one
            manager over the whole world for 3 ticks, plus 8 strips of a 2M world against oracle (ii).
  config 5  skewed crowds, 4 Spaces with D = 50/100/200/400, 50% in 64 Gaussian hotspots: at 4 x 100k
            (peak density ~100x the mean) against oracle (ii) per Space; at full size (4 x 1M, SURVEY
            proportions) the LDS-staged sweep / wave-per-mover path on two different grids (D/4 cells
            and D/2 cells, so tiles, halos and the LDS-or-dense routing all differ) agree event for
            event, and every event of ~1,000 sampled movers per Space equals oracle (iv) (the closed
            form of an all-moving tick from two position snapshots, oracle/sampled.py); an x-quantile
            strip split of a skewed world equals one manager.
  config 4  also: the 16M single manager's tick-1 events of 8,000 sampled movers against oracle (iv).

Parity against go-aoi itself is UNPINNED: the oracles are the restatements.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import aoi_harness as H  # noqa: E402
import strips_cpu as SC  # noqa: E402

pytestmark = pytest.mark.gpu


def _sorted(ev):
    return ev[np.lexsort((ev[:, 1], ev[:, 0]))] if len(ev) else ev.reshape(0, 2)


def test_config3_512_spaces_vs_oracle_per_space(gpu, oracle_lib):
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    po = oracle_lib
    S, N, L, D, seed0 = 512, 2000, 1600.0, 100.0, 0x5EED0003
    n = S * N
    xs, zs = [], []
    for s in range(S):
        x, z = po.workload_init(seed0 + s, N, L)
        xs.append(x)
        zs.append(z)
    eng = Engine(capacity=n, spaces=[(D, (0.0, 0.0, L, L))] * S)
    orcs = [po.XZListOracle(D, N) for _ in range(S)]
    # tick 0: every entity enters its Space, slot = space * N + i, in slot order (device-staged batch)
    bs, bx, bz, bk, bp = (DeviceBuffer(4 * n) for _ in range(5))
    bs.upload(np.arange(n, dtype=np.uint32))
    bx.upload(np.concatenate(xs))
    bz.upload(np.concatenate(zs))
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER, np.uint8))
    bp.upload(np.repeat(np.arange(S, dtype=np.uint32), N))
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n, bp.ptr)
    got = eng.tick()
    want = []
    for s in range(S):
        orcs[s].bulk_enter(np.arange(N, dtype=np.uint32), xs[s], zs[s])
        rp, cols = orcs[s].relation()
        # the i-th Enter raises ENTER(i, o) for every earlier o in its box: one event per pair, mover = later
        rows = np.repeat(np.arange(N, dtype=np.uint32), np.diff(rp.astype(np.int64)))
        keep = cols < rows
        ev = np.stack([rows[keep] + s * N, (cols[keep] + s * N) | np.uint32(H.EV_ENTER)], axis=1).astype(np.uint32)
        want.append(_sorted(ev))
    want = np.concatenate(want)
    assert np.array_equal(got, want), "enter tick: " + H.fmt_diff(got, want)
    eng.adopt_device_state()  # the moves below are staged from host arrays
    slots = np.arange(N, dtype=np.uint32)
    for t in (1, 2, 3):
        want = []
        for s in range(S):
            po.workload_step(seed0 + s, t, xs[s], zs[s], L, 1.0)
            orcs[s].moved_batch(slots, xs[s], zs[s])
            ev = orcs[s].take_events()
            if len(ev):
                ev = ev + np.array([s * N, s * N], np.uint32)  # slot offset (the kind bit is above)
                want.append(_sorted(ev))
        want = np.concatenate(want)
        eng.stage_moves(np.arange(n, dtype=np.uint32), np.concatenate(xs), np.concatenate(zs))
        got = eng.tick()
        assert np.array_equal(got, want), f"tick {t}: " + H.fmt_diff(got, want)
        assert len(got) > 1000
        # the relation view, updated from the tick's events (the enter tick's view was rebuilt: its
        # device batch could hold SILENT ops), equals the 512 per-Space oracles' neighbour sets
        rp, cols = eng.relation()
        wrp, wcols, base = [np.zeros(1, np.int64)], [], 0
        for s in range(S):
            orp, ocols = orcs[s].relation()
            wrp.append(orp[1:].astype(np.int64) + base)
            wcols.append(ocols.astype(np.int64) + s * N)
            base += len(ocols)
        assert np.array_equal(rp.astype(np.int64), np.concatenate(wrp)), f"tick {t}: relation rows"
        assert np.array_equal(cols.astype(np.int64), np.concatenate(wcols)), f"tick {t}: relation cols"
    n_inc, n_full, why = eng.debug_relation_mode()
    assert n_inc == 2 and n_full == 1, (n_inc, n_full, why)  # ticks 2, 3 updated; tick 1's view rebuilt
    eng.close()


def _strip_world(po, n, L, world, seed, ticks, layout=None, skew=None, host_first=True):
    """Merged per-tick events of `world` loopback strips (events of tick 0 only counted: at 16M they run
    to 2.6e8 pairs)."""
    from goworld_amd.strips import LoopbackExchange, StripLayout, StripNode
    lay = layout or StripLayout(world, L, 100.0, 1.0)
    nodes = [StripNode(lay, r, n, device=0, seed=seed, skew=skew) for r in range(world)]
    out = [sum(int(nd.start(host_events=False).count) for nd in nodes)]
    for t in range(1, ticks):
        outs = [nd.prepare(t) for nd in nodes]
        ins = LoopbackExchange.exchange(outs)
        out.append(SC.merge_sorted([nd.finish(*i, host_events=True) for nd, i in zip(nodes, ins)]))
    for nd in nodes:
        nd.close()
    return out


def _whole_world(n, L, seed, ticks, skew=None, snaps=None):
    """One manager over the whole world, positions from the device generator; per-tick events (tick 0:
    the count only). snaps (a list): receives each moving tick's (x0, z0, x1, z1) snapshots."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces
    bx, bz, bs, bk = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(n)
    nhot, sigma, every = skew or (0, 0.0, 10)
    wl_init_spaces(0, bx.ptr, bz.ptr, n, 1, seed, L, nhot, sigma, every)
    wl_iota(0, bs.ptr, n)
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER, np.uint8))
    eng = Engine(100.0, capacity=n, bounds=(0.0, 0.0, L, L))
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n)
    out = [int(eng.tick_device().count)]
    eng.adopt_device_state()
    for t in range(1, ticks):
        before = (bx.download(np.float32, n), bz.download(np.float32, n)) if snaps is not None else None
        wl_step_spaces(0, bx.ptr, bz.ptr, bx.ptr, bz.ptr, n, 1, seed, t, L, 1.0)
        if snaps is not None:
            snaps.append(before + (bx.download(np.float32, n), bz.download(np.float32, n)))
        eng.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, n)
        out.append(eng.tick())
    eng.close()
    return out


def _sampled_movers(n, k, seed, hot_every=0):
    """k movers spread over [0, n) (and, with hot_every, as many from the hotspot share: slots with
    slot % hot_every == 1 are the generator's hotspot entities, include/gwaoi_workload.h)."""
    rng = np.random.default_rng(seed)
    pick = rng.choice(n, size=k, replace=False)
    if hot_every:
        pick = np.concatenate([pick, rng.choice(n // hot_every, size=k, replace=False) * hot_every + 1])
    return np.unique(pick)


def test_config4_16M_world_in_8_strips(gpu):
    """config 4 at its size: 16,000,000 entities, L = 140,000, 8 X-strips (loopback on one GPU); the
    owned movers' events of the 8 strips, merged, equal one manager over the whole world."""
    from oracle import sampled
    n, L, seed = 16_000_000, 140_000.0, 0x5EED0004
    snaps = []
    want = _whole_world(n, L, seed, 4, snaps=snaps)
    got = _strip_world(None, n, L, 8, seed, 4)
    assert got[0] == want[0] and want[0] > 100_000_000  # enter tick: pair counts (2.6e8 pairs)
    for t in (1, 2, 3):
        assert np.array_equal(got[t], want[t]), f"tick {t}: " + H.fmt_diff(got[t], want[t])
        assert len(got[t]) > 1_000_000
    # the single manager itself against oracle (iv) at 16M: every event of 8,000 sampled movers, tick 1
    movers = _sampled_movers(n, 8000, 1)
    ref = sampled.AllMovingTick(*snaps[0], 100.0).sample(movers)
    mine = sampled.pick(want[1], movers)
    assert len(ref) > 1000 and np.array_equal(mine, ref), "tick 1 sampled: " + H.fmt_diff(mine, ref)


def test_config4_2M_strips_vs_grid_oracle(gpu, oracle_lib):
    """8 strips of a 2M world (config-2 density) against oracle (ii) over the whole world."""
    po = oracle_lib
    n, L, seed = 2_000_000, float(np.sqrt(2_000_000 / (1_000_000 / 35000.0 ** 2))), 0x5EED0044
    x, z = po.workload_init(seed, n, L)
    orc = po.GridOracle(100.0, n, (0.0, 0.0, L, L))
    orc.bulk_enter(np.arange(n, dtype=np.uint32), x, z)
    got = _strip_world(po, n, L, 8, seed, 4)
    ids = np.arange(n, dtype=np.uint32)
    assert got[0] == len(orc.relation()[1]) // 2
    for t in (1, 2, 3):
        po.workload_step(seed, t, x, z, L, 1.0)
        orc.moved_batch(ids, x, z)
        want = _sorted(orc.take_events())
        assert np.array_equal(got[t], want), f"tick {t}: " + H.fmt_diff(got[t], want)


SKEW_D = (50.0, 100.0, 200.0, 400.0)


@pytest.mark.parametrize("band", [1, 0])
def test_config5_4x100k_vs_grid_oracle(gpu, oracle_lib, band):
    """4 skewed Spaces x 100,000 (D = 50/100/200/400), L scaled to config 5's mean density, 50% of the
    entities in 64 hotspots with sigma 39 (peak ~100x the mean, as config 5 at 1M with sigma 123): the
    silent bulk restore of the bench's first pass, the enter tick's relation and 2 moving ticks against
    oracle (ii) per Space; the global-memory movers by the band walk (1) and by their whole rings (0).
    (Also the regression case of round 4's unexplained fault in skew50's first pass)"""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine
    po = oracle_lib
    N, L, seed0 = 100_000, 35000.0 * np.sqrt(0.1), 0x5EED0005
    S = len(SKEW_D)
    n = S * N
    pos, orcs = [], []
    for s, d in enumerate(SKEW_D):
        x, z = po.workload_skew_init(seed0 + s, N, L, 64, 39.0, 2)
        pos.append((x, z))
        o = po.GridOracle(d, N, (0.0, 0.0, L, L))
        o.bulk_enter(np.arange(N, dtype=np.uint32), x, z)
        orcs.append(o)
    eng = Engine(capacity=n, spaces=[(d, (0.0, 0.0, L, L)) for d in SKEW_D])
    eng.set_timing(True)
    eng.debug_set_band(band)
    bs, bx, bz, bk, bp = (DeviceBuffer(4 * n) for _ in range(5))
    bs.upload(np.arange(n, dtype=np.uint32))
    bx.upload(np.concatenate([p[0] for p in pos]))
    bz.upload(np.concatenate([p[1] for p in pos]))
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    bp.upload(np.repeat(np.arange(S, dtype=np.uint32), N))
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n, bp.ptr)
    assert len(eng.tick()) == 0
    eng.adopt_device_state()
    rp, cols = eng.relation()
    rp = rp.astype(np.int64)
    for s, o in enumerate(orcs):
        orp, ocols = o.relation()
        grp = rp[s * N:(s + 1) * N + 1]
        assert np.array_equal(grp - grp[0], orp.astype(np.int64)), f"space {s} row lengths"
        assert np.array_equal(cols[grp[0]:grp[-1]] - np.uint32(s * N), ocols), f"space {s} neighbours"
    slots = np.arange(N, dtype=np.uint32)
    eng.debug_sweep_sizes(1)  # count the tiles each LDS sweep size walks in the moving ticks
    for t in (1, 2):
        want = []
        for s, o in enumerate(orcs):
            x, z = pos[s]
            po.workload_step(seed0 + s, t, x, z, L, 1.0)
            o.moved_batch(slots, x, z)
            ev = o.take_events()
            if len(ev):
                want.append(_sorted(ev + np.array([s * N, s * N], np.uint32)))
        want = np.concatenate(want)
        eng.stage_moves(np.arange(n, dtype=np.uint32), np.concatenate([p[0] for p in pos]),
                        np.concatenate([p[1] for p in pos]))
        got = eng.tick()
        assert np.array_equal(got, want), f"tick {t}: " + H.fmt_diff(got, want)
    st = eng.stats()
    assert st["dense_movers"] > 0 and (st["band_movers"] > 0) == bool(band)  # the path under test
    small, mid, big = eng.debug_sweep_sizes(0)
    # every LDS sweep size took part (D 50 / 100: small, D 200: mid, D 400: big): a planner or
    # cap change that reroutes a Space would drop a size's parity coverage here
    assert small > 0 and mid > 0 and big > 0, (small, mid, big)


def test_config5_full_size_two_grids_agree(gpu):
    """Config 5 at full size in SURVEY proportions (4 x 1M, D = 50/100/200/400, 50% in 64 hotspots per
    Space, sigma 123): no oracle holds its relation (billions of pairs), so two managers with different
    grids (D/4 and D/2 cells: other tiles, halos, LDS-or-dense routing; the band walk in the first, whole
    rings in the second) must agree event for event."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces
    N, L, seed0 = 1_000_000, 35000.0, 0x5EED0005
    S = len(SKEW_D)
    n = S * N
    bx, bz, bs, bk, bp = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(n), \
        DeviceBuffer(4 * n)
    wl_init_spaces(0, bx.ptr, bz.ptr, N, S, seed0, L, 64, 123.0, 2)
    wl_iota(0, bs.ptr, n)
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    bp.upload(np.repeat(np.arange(S, dtype=np.uint32), N))
    engs = []
    for cpd in (None, 2.0):
        e = Engine(capacity=n, spaces=[(d, (0.0, 0.0, L, L)) for d in SKEW_D])
        if cpd:
            e.debug_set_cells_per_dist(cpd)
            e.debug_set_band(0)
        e.set_timing(True)
        e.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n, bp.ptr)
        assert int(e.tick_device().count) == 0
        engs.append(e)
    for t in (1, 2):
        wl_step_spaces(0, bx.ptr, bz.ptr, bx.ptr, bz.ptr, N, S, seed0, t, L, 1.0)
        evs = []
        for e in engs:
            e.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, n)
            evs.append(e.tick())
        assert np.array_equal(evs[0], evs[1]), f"tick {t}: " + H.fmt_diff(evs[0], evs[1])
        assert len(evs[0]) > 1_000_000
    st = [e.stats() for e in engs]
    assert st[0]["band_movers"] > 0 and st[1]["band_movers"] == 0 and st[0]["grid_cells"] != st[1]["grid_cells"]
    for e in engs:
        e.close()


def test_config5_full_size_sampled_vs_semantic(gpu):
    """Config 5 at full size in SURVEY proportions (4 x 1M, D = 50/100/200/400, 50% in 64 hotspots per
    Space, sigma 123) against oracle (iv): every event of ~1,000 sampled movers per Space (half of them
    hotspot entities) in two all-moving ticks, from the position snapshots alone (oracle/sampled.py)."""
    from goworld_amd import _lib
    from goworld_amd.engine import DeviceBuffer, Engine, wl_init_spaces, wl_iota, wl_step_spaces
    from oracle import sampled
    N, L, seed0 = 1_000_000, 35000.0, 0x5EED0005
    S = len(SKEW_D)
    n = S * N
    bx, bz, bs, bk, bp = DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(4 * n), DeviceBuffer(n), \
        DeviceBuffer(4 * n)
    wl_init_spaces(0, bx.ptr, bz.ptr, N, S, seed0, L, 64, 123.0, 2)
    wl_iota(0, bs.ptr, n)
    bk.upload(np.full(n, _lib.GWAOI_OP_ENTER | _lib.GWAOI_OP_SILENT, np.uint8))
    bp.upload(np.repeat(np.arange(S, dtype=np.uint32), N))
    eng = Engine(capacity=n, spaces=[(d, (0.0, 0.0, L, L)) for d in SKEW_D])
    eng.set_timing(True)
    eng.stage_ops_device(bs.ptr, bx.ptr, bz.ptr, bk.ptr, n, bp.ptr)
    assert int(eng.tick_device().count) == 0
    for t in (1, 2):
        x0, z0 = bx.download(np.float32, n), bz.download(np.float32, n)
        wl_step_spaces(0, bx.ptr, bz.ptr, bx.ptr, bz.ptr, N, S, seed0, t, L, 1.0)
        x1, z1 = bx.download(np.float32, n), bz.download(np.float32, n)
        eng.stage_moves_device(bs.ptr, bx.ptr, bz.ptr, n)
        got = eng.tick()
        assert len(got) > 1_000_000
        for s, d in enumerate(SKEW_D):
            sl = slice(s * N, (s + 1) * N)
            movers = _sampled_movers(N, 500, 100 * t + s, hot_every=2)
            ref = sampled.AllMovingTick(x0[sl], z0[sl], x1[sl], z1[sl], d, base=s * N).sample(movers)
            mine = sampled.pick(got, movers + s * N)
            assert len(ref) > 500 and np.array_equal(mine, ref), f"tick {t} Space {s}: " + H.fmt_diff(mine, ref)
    st = eng.stats()
    assert st["band_movers"] > 0
    eng.close()


def test_config5_skewed_world_in_quantile_strips(gpu):
    """A skewed world (one Space of 400,000 at config 5's mean density, 10% in 64 hotspots with sigma 55:
    peak ~100x the mean) cut into 4 X-strips at the x-quantiles of its entities (SURVEY.md §8(e)
    config 5): the merged strip events equal one manager over the world. (Smaller than config 5's
    Spaces so that the loud enter tick's pairs stay ~1.5e7.)"""
    from goworld_amd.engine import DeviceBuffer, wl_init_spaces
    from goworld_amd.strips import StripLayout
    n, L, seed, skew = 400_000, 35000.0 * float(np.sqrt(0.4)), 0x5EED0055, (64, 55.0, 10)
    bx, bz = DeviceBuffer(4 * n), DeviceBuffer(4 * n)
    wl_init_spaces(0, bx.ptr, bz.ptr, n, 1, seed, L, *skew)
    x = bx.download(np.float32, n)
    lay = StripLayout.from_quantiles(4, x, L, 100.0, 1.0)
    counts = np.bincount(lay.owner_of(x), minlength=4)
    assert counts.min() > 0.2 * n  # ~equal entity counts per strip, unequal widths
    assert len(set(np.round(np.diff([0.0] + lay.edges + [L]), 1))) > 1
    want = _whole_world(n, L, seed, 4, skew=skew)
    got = _strip_world(None, n, L, 4, seed, 4, layout=lay, skew=skew)
    assert got[0] == want[0]
    for t in (1, 2, 3):
        assert np.array_equal(got[t], want[t]), f"tick {t}: " + H.fmt_diff(got[t], want[t])


def test_rccl_exchange_loopback(gpu):
    """gwaoi_strip_exchange on a one-rank RCCL communicator with both peers = itself: the two lists
    and their counts come back through RCCL (sends and receives match in issue order), and a side
    without a peer receives a zero count. (Two ranks cannot share one GPU in RCCL; the multi-rank
    protocol is tested over gloo, tests/test_strips.py.)"""
    import torch
    from goworld_amd import _lib
    from goworld_amd.strips import StripComm
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    comm = StripComm(StripComm.make_id(), 1, 0, 0)
    cap = 5000
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    left = torch.from_numpy(rng.integers(0, 2**31, (cap, 4), dtype=np.int64).astype(np.int32)).to(dev)
    right = torch.from_numpy(rng.integers(0, 2**31, (cap, 4), dtype=np.int64).astype(np.int32)).to(dev)
    counts = torch.tensor([1234, 4321, 0, 0], dtype=torch.int32, device=dev)
    li, ri = torch.zeros_like(left), torch.zeros_like(right)
    cin = torch.full((2,), -1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    import ctypes
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(_lib.load().gwaoi_strip_exchange(comm.handle, ctypes.c_void_p(st.cuda_stream), 0, 0, p(left), p(right),
                                                p(counts), cap, p(li), p(ri), p(cin)))
    torch.cuda.synchronize(dev)
    assert cin.tolist() == [1234, 4321]
    assert torch.equal(li, left) and torch.equal(ri, right)
    cin.fill_(-1)
    _lib.check(_lib.load().gwaoi_strip_exchange(comm.handle, ctypes.c_void_p(st.cuda_stream), -1, 0, p(left), p(right),
                                                p(counts), cap, p(li), p(ri), p(cin)))
    torch.cuda.synchronize(dev)
    assert cin.tolist() == [0, 4321]
    comm.close()


def test_strip_tick_rccl_single_rank_matches(gpu):
    """StripNode.tick_rccl (select -> RCCL exchange -> absorb_n -> emit -> tick, all on the stream) on a
    one-strip world equals the host-driven path tick for tick. The strip exchanges with itself (peers (0, 0):
    a loopback RCCL group; with no peer at all the node makes no RCCL call)."""
    import torch
    from goworld_amd.strips import StripComm, StripLayout, StripNode
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    n, L, seed = 200_000, 15652.0, 0x5EED0077
    lay = StripLayout(1, L, 100.0, 1.0)
    a = StripNode(lay, 0, n, device=0, seed=seed)
    b = StripNode(lay, 0, n, device=0, seed=seed)
    comm = StripComm(StripComm.make_id(), 1, 0, 0)
    assert np.array_equal(a.start(host_events=True), b.start(host_events=True))
    for t in range(1, 5):
        ea = a.finish(*a.prepare(t), host_events=True)
        eb = b.tick_rccl(t, comm, host_events=True, peers=(0, 0))
        assert np.array_equal(ea, eb), f"tick {t}"
        assert len(ea) > 1000
    torch.cuda.synchronize()
    comm.close()
    a.close()
    b.close()


def test_strip_local_slots_exhausted_keeps_manager_usable(gpu):
    """a region with more entities than its local slots (cap_l) used to emit Enters of slot 0
    when the free ring ran dry, which failed the manager's device check and left it unusable with the
    real cause hidden. Now the tick emits nothing, the error names GWAOI_STRIP_ERR_SLOTS, and the
    manager still runs passes."""
    import torch
    from goworld_amd import _lib
    from goworld_amd.strips import StripLayout, StripNode
    n, L = 20_000, 4000.0
    lay = StripLayout(1, L, 100.0, 1.0)
    nd = StripNode(lay, 0, n, device=0, seed=0x5EED0078, cap_l=1024)
    assert nd.cap_l == 1024
    with pytest.raises(_lib.GwaoiError) as ei:
        nd.start(host_events=True)
    assert "cap_l = 1024" in str(ei.value) and "flags 8" in str(ei.value)
    assert nd.eng.count()[0] == 0  # nothing applied
    ev = nd.eng.tick()  # the manager is not poisoned: an empty pass runs
    assert len(ev) == 0
    torch.cuda.synchronize()
    nd.close()


def test_strip_region_new_ids_over_cap_raises(gpu):
    """Region state (ABI 2.1): a tick that brings more ids into a region than cap_new emits nothing and the strip
    raises, naming GWAOI_STRIP_ERR_NEWLIST; the manager still runs passes. (3 strips, 40-unit steps: tens of halo
    crossings per tick against a cap_new of 2.)"""
    import torch
    from goworld_amd import _lib
    from goworld_amd.strips import LoopbackExchange, StripLayout, StripNode
    n, L, step = 12000, 3800.0, 40.0
    lay = StripLayout(3, L, 100.0, step)
    nodes = [StripNode(lay, r, n, device=0, seed=0x5EED0079, cap_new=2, sort_chunk=16) for r in range(3)]
    assert all(nd.R is not None for nd in nodes)
    for nd in nodes:
        nd.start()
    raised = []
    for t in range(1, 4):
        ins = LoopbackExchange.exchange([nd.prepare(t, step) for nd in nodes])
        for nd, i in zip(nodes, ins):
            try:
                nd.finish(*i)
            except _lib.GwaoiError as e:
                raised.append(str(e))
        if raised:
            break
    assert raised and all("flags 16" in m and "cap_new = 2" in m for m in raised), raised
    for nd in nodes:
        assert len(nd.eng.tick()) == 0  # the manager is not poisoned: an empty pass runs
    torch.cuda.synchronize()
    for nd in nodes:
        nd.close()


def test_strip_absorb_n_flags_a_cut_list(gpu):
    """a received count above the message capacity (the sender's list was cut) sets
    GWAOI_STRIP_ERR_OVERFLOW on the receiving rank too; a count within capacity sets nothing."""
    import ctypes

    import torch
    from goworld_amd import _lib
    L_ = _lib.load()
    dev = torch.device("cuda", 0)
    n, cap = 64, 16
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    ex, ez = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    recs = torch.zeros((cap, 4), dtype=torch.int32, device=dev)
    recs[:, 0] = torch.arange(cap, dtype=torch.int32, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for got, want_err in ((cap, 0), (cap + 5, 4)):
        cnt = torch.tensor([got], dtype=torch.int32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        flags.zero_()
        _lib.check(L_.gwaoi_strip_absorb_n(st, p(flags), p(ex), p(ez), p(recs), p(cnt), cap, p(err)))
        torch.cuda.synchronize(dev)
        assert int(err.item()) == want_err
        assert int((flags != 0).sum().item()) == cap  # min(count, cap) records absorbed
