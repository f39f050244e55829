"""Regenerate the golden AOI fixtures in tests/golden/*.npz from oracle (i), the go-aoi
XZListAOIManager restatement (oracle/xzlist_aoi.c).

The reference holds no AOI golden vectors and go-aoi / Go are absent from this
image, so these fixtures pin the oracle and the product against each other and against future
regressions; they are NOT outputs of the reference itself (parity unpinned, DESIGN.md "Oracle").
Each fixture: the op script (per tick), the canonical events of every tick, the final relation.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import pyoracle  # noqa: E402
import aoi_harness as H  # noqa: E402


def cases():
    yield H.case_origin_monsters()
    yield H.case_boundaries()
    yield H.case_denormal()
    yield H.case_random_ops(seed=11, n=120, nticks=10, ops_per_tick=90, world=300.0, dist=50.0)
    yield H.case_random_ops(seed=12, n=400, nticks=6, ops_per_tick=500, world=150.0, dist=20.0, snap=False)
    yield H.case_walk(0x5EED0001, 2000, 1600.0, 6, workload=pyoracle)  # config-1 density (rho = 8e-4)


def save(case, path):
    kinds, slots, xs, zs, tptr = [], [], [], [], [0]
    for ops in case["ticks"]:
        for k, s, x, z in ops:
            kinds.append(k)
            slots.append(s)
            xs.append(x)
            zs.append(z)
        tptr.append(len(kinds))
    orc = pyoracle.XZListOracle(case["dist"], case["cap"])
    evs, eptr = [], [0]
    for ops in case["ticks"]:
        ev = H.oracle_tick(orc, ops)
        evs.append(ev)
        eptr.append(eptr[-1] + len(ev))
    assert orc.check_invariants() == 0
    rp, cols = orc.relation()
    np.savez_compressed(
        path, dist=np.float32(case["dist"]), cap=np.uint32(case["cap"]),
        bounds=np.asarray(case.get("bounds", (0, 0, 0, 0)), np.float32),
        op_kind=np.asarray(kinds, np.uint8), op_slot=np.asarray(slots, np.uint32),
        op_x=np.asarray(xs, np.float32), op_z=np.asarray(zs, np.float32), tick_ptr=np.asarray(tptr, np.uint32),
        ev=np.concatenate(evs).astype(np.uint32).reshape(-1, 2), ev_ptr=np.asarray(eptr, np.uint64),
        rel_rp=rp, rel_cols=cols)
    return eptr[-1]


def load(path):
    f = np.load(path, allow_pickle=False)
    tp = f["tick_ptr"]
    ticks = []
    for t in range(len(tp) - 1):
        a, b = int(tp[t]), int(tp[t + 1])
        ticks.append([(int(f["op_kind"][i]), int(f["op_slot"][i]), float(f["op_x"][i]), float(f["op_z"][i]))
                      for i in range(a, b)])
    ep = f["ev_ptr"]
    evs = [f["ev"][int(ep[t]):int(ep[t + 1])] for t in range(len(ep) - 1)]
    b = tuple(float(v) for v in f["bounds"])
    return dict(name=os.path.basename(path)[:-4], dist=float(f["dist"]), cap=int(f["cap"]), ticks=ticks,
                events=evs, rel=(f["rel_rp"], f["rel_cols"]), bounds=b if b[2] > b[0] else None)


def fixture_paths():
    return sorted(os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(".npz"))


if __name__ == "__main__":
    pyoracle.build()
    for c in cases():
        p = os.path.join(HERE, c["name"] + ".npz")
        n = save(c, p)
        print(f"{p}: {sum(len(t) for t in c['ticks'])} ops, {n} events, {os.path.getsize(p)} bytes")
    # workload generator pin (first three x of seed 0x5EED0002, N=8, L=35000)
    x, z = pyoracle.workload_init(0x5EED0002, 8, 35000.0)
    with open(os.path.join(HERE, "workload_pin.txt"), "w") as f:
        f.write(" ".join(f"{v:.6f}" for v in x[:3]) + "\n")
