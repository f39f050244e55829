"""X-strip partition of one Space over several GPUs (include/gwaoi_strips.h,
goworld_amd/strips.py). The events the strips report for their owned movers, merged, must equal the
events of ONE manager running the whole world (oracle (i)), tick by tick, bit for bit.

CPU: the product's exchange_dist over gloo with world_size 2 and 3, each rank a CPU restatement of a
strip (tests/strips_cpu.py). GPU: the HIP strip kernels + libgwaoi managers, several strips in one
process (loopback exchange), and two processes sharing the GPU with exchange_dist over gloo.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import strips_cpu as SC  # noqa: E402

N, L, D, SEED, TICKS = 6000, 2700.0, 100.0, 0x5EED0004, 6


def _layout(world, L=L):
    from goworld_amd.strips import StripLayout
    return StripLayout(world, L, D, 1.0)


def test_layout_geometry():
    lay = _layout(3)
    g0, g1, g2 = (lay.geom(r, N) for r in range(3))
    assert g0.has_left == 0 and g2.has_right == 0 and g1.has_left == 1 and g1.has_right == 1
    assert g0.xb == g1.xa and g1.xb == g2.xa
    assert g1.left_hi == g0.rb and g1.right_lo == g2.ra  # sender and receiver agree on every bound
    assert lay.halo > D + 1.0
    x = np.asarray([-5.0, 0.0, 899.999, 900.0, 1799.9, 1800.0, 2699.0], np.float32)
    assert lay.owner_of(x).tolist() == [0, 0, 0, 1, 1, 2, 2]
    with pytest.raises(ValueError):
        _layout(20)


def test_cpu_loopback_matches_one_manager(oracle_lib):
    from goworld_amd.strips import LoopbackExchange
    po = oracle_lib
    want = SC.global_events(po, N, L, D, SEED, TICKS)
    lay = _layout(3)
    nodes = [SC.CPUStripNode(lay, r, N, po, SEED) for r in range(3)]
    got = [SC.merge_sorted([nd.start() for nd in nodes])]
    for t in range(1, TICKS):
        outs = [nd.prepare(t) for nd in nodes]
        ins = LoopbackExchange.exchange(outs)
        got.append(SC.merge_sorted([nd.finish(*i) for nd, i in zip(nodes, ins)]))
    for t in range(TICKS):
        assert np.array_equal(got[t], want[t]), f"tick {t}: {len(got[t])} vs {len(want[t])}"
    assert sum(len(w) for w in want[1:]) > 100  # the walk raises events every tick


def _dist_worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    from goworld_amd.strips import exchange_dist
    from oracle import pyoracle as po
    lay = _layout(world)
    nd = SC.CPUStripNode(lay, rank, N, po, SEED)
    evs = [nd.start()]
    for t in range(1, TICKS):
        lo, ro = nd.prepare(t)
        li, ri = exchange_dist(lo, ro, rank, world)
        evs.append(nd.finish(li, ri))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), *evs)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_cpu_gloo_world(oracle_lib, tmp_path, world):
    """The product's halo exchange (exchange_dist) between processes over gloo."""
    import torch.multiprocessing as mp
    po = oracle_lib
    port = 29500 + (os.getpid() % 1000) + world
    mp.spawn(_dist_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    want = SC.global_events(po, N, L, D, SEED, TICKS)
    per = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    for t in range(TICKS):
        got = SC.merge_sorted([p[f"arr_{t}"] for p in per])
        assert np.array_equal(got, want[t]), f"tick {t}"


# ------------------------------------------------------------------------------------------------ GPU

@pytest.mark.gpu
@pytest.mark.parametrize("world,local,reg", [(1, True, 1), (3, True, 1), (4, True, 1), (3, True, 0), (3, False, 0),
                                             (3, True, 2)])
def test_gpu_strips_loopback(gpu, oracle_lib, world, local, reg):
    """HIP strip kernels + one libgwaoi manager per strip, all on cuda:0; every step's op list equals
    the CPU restatement's and the merged events equal one manager over the whole world. local: the
    managers index their entities by local slot (gwaoi_strip_emit_local), events translated back.
    reg 1: the region state (ABI 2.1: state in local-slot order, the emit merging the region list with the
    tick's new ids); 0: state by global id, kernels over the id range; 2: the region state with 16-entry sort
    chunks and steps of up to 40 units, so the tick's new ids and Leaves span several chunks (the merge's
    multi-chunk counts)."""
    from goworld_amd.strips import LoopbackExchange, StripLayout, StripNode
    po = oracle_lib
    n, Lw = 12000, 3800.0
    step = 40.0 if reg == 2 else 1.0
    want = SC.global_events(po, n, Lw, D, SEED, TICKS, step=step)
    lay = StripLayout(world, Lw, D, step)
    nodes = [StripNode(lay, r, n, device=0, seed=SEED, local_slots=local, region_state=reg > 0,
                       sort_chunk=16 if reg == 2 else 0, cap_new=128 if reg == 2 else 65536) for r in range(world)]
    assert all((nd.R is not None) == (reg > 0) for nd in nodes)
    cpu = [SC.CPUStripNode(lay, r, n, po, SEED) for r in range(world)]
    got = [SC.merge_sorted([nd.start(host_events=True) for nd in nodes])]
    for c in cpu:
        c.start()
    assert np.array_equal(got[0], want[0])
    for t in range(1, TICKS):
        outs = [nd.prepare(t, step) for nd in nodes]
        couts = [c.prepare(t, step) for c in cpu]
        for (a, b), (ca, cb) in zip(outs, couts):  # same records to send (order free)
            for x, y in ((a, ca), (b, cb)):
                xs = x.cpu().numpy().view(np.uint32)
                ys = y.numpy().view(np.uint32)
                assert np.array_equal(xs[np.argsort(xs[:, 0])], ys[np.argsort(ys[:, 0])])
        ins = LoopbackExchange.exchange(outs)
        cins = LoopbackExchange.exchange(couts)
        evs = []
        for nd, c, i, ci in zip(nodes, cpu, ins, cins):
            c.absorb(*ci)
            ids, kinds = c.ops()
            e = nd.finish(*i, host_events=True)
            gids = nd.last_op_ids()
            extra, miss = np.setdiff1d(gids, ids), np.setdiff1d(ids, gids)
            assert len(extra) == 0 and len(miss) == 0, (
                f"tick {t} rank {nd.rank}: gpu-only ops {extra[:8]} (kinds "
                f"{nd.kinds[: nd.last_ops].cpu().numpy()[np.isin(gids, extra)][:8]}), cpu-only {miss[:8]}; "
                f"cpu flags of gpu-only {c.flags[extra[:8]]}, ex {c.ex[extra[:8]]}, sx {c.sx[extra[:8]]}")
            assert np.array_equal(nd.kinds[: len(ids)].cpu().numpy(), kinds)
            c.emit()
            evs.append(e)
        got.append(SC.merge_sorted(evs))
        assert np.array_equal(got[t], want[t]), f"world {world} tick {t}: {len(got[t])} vs {len(want[t])}"
    if reg == 2:  # the tick's new ids took several sort chunks somewhere
        assert max(nd.max_new for nd in nodes) > 16
    for nd in nodes:
        nd.close()


@pytest.mark.gpu
def test_gpu_strips_two_processes(gpu, oracle_lib, tmp_path):
    """Two ranks (processes) on one GPU, halo exchange through exchange_dist over gloo (host staged)."""
    po = oracle_lib
    n, Lw = 12000, 3800.0
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={29700 + os.getpid() % 200}",
           os.path.join(HERE, "strips_worker.py"), str(tmp_path), str(n), str(Lw), str(TICKS)]
    r = subprocess.run(cmd, env=env, timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    want = SC.global_events(po, n, Lw, D, SEED, TICKS)
    per = [np.load(os.path.join(tmp_path, f"r{k}.npz")) for k in range(2)]
    for t in range(TICKS):
        got = SC.merge_sorted([p[f"arr_{t}"] for p in per])
        assert np.array_equal(got, want[t]), f"tick {t}"


@pytest.mark.gpu
@pytest.mark.parametrize("reg", [1, 0])
def test_gpu_strips_ingest_external_moves(gpu, oracle_lib, reg):
    """Strips driven by external moves (gwaoi_strip_ingest / gwaoi_strip_region_ingest: the owned entities' end
    positions handed in as (ids, x, z) device arrays, in a shuffled order) instead of the seeded walk kernel; the
    merged events equal one manager over the whole world, tick by tick. The CPU restatement supplies each tick's
    owned ids and their end positions."""
    import torch
    from goworld_amd.strips import LoopbackExchange, StripNode
    po = oracle_lib
    n, Lw, world = 12000, 3800.0, 3
    want = SC.global_events(po, n, Lw, D, SEED, TICKS)
    lay = _layout(world, Lw)
    nodes = [StripNode(lay, r, n, device=0, seed=SEED, region_state=reg > 0) for r in range(world)]
    assert all((nd.R is not None) == (reg > 0) for nd in nodes)
    cpu = [SC.CPUStripNode(lay, r, n, po, SEED) for r in range(world)]
    got = [SC.merge_sorted([nd.start(host_events=True) for nd in nodes])]
    for c in cpu:
        c.start()
    assert np.array_equal(got[0], want[0])
    rng = np.random.default_rng(7)
    dev = torch.device("cuda", 0)
    for t in range(1, TICKS):
        outs, couts = [], []
        for nd, c in zip(nodes, cpu):
            own = np.nonzero(c.flags & SC.O)[0]  # owned at the start of the tick
            couts.append(c.prepare(t))           # the walk's end positions (c.wx, c.wz) and the CPU's records
            perm = rng.permutation(len(own))
            ids = torch.from_numpy(own[perm].astype(np.int32)).to(dev)
            x = torch.from_numpy(np.ascontiguousarray(c.wx[own][perm])).to(dev)
            z = torch.from_numpy(np.ascontiguousarray(c.wz[own][perm])).to(dev)
            outs.append(nd.prepare(t, moves=(ids, x, z)))
        ins = LoopbackExchange.exchange(outs)
        got.append(SC.merge_sorted([nd.finish(*i, host_events=True) for nd, i in zip(nodes, ins)]))
        assert np.array_equal(got[t], want[t]), f"tick {t}: {len(got[t])} vs {len(want[t])}"
        for c, ci in zip(cpu, LoopbackExchange.exchange(couts)):  # the restatement advances too
            c.finish(*ci)
    for nd in nodes:
        nd.close()
