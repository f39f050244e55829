import os, sys, subprocess, numpy as np, tempfile
ROOT = "/root/repo"; sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + "/tests")
import strips_cpu as SC
from oracle import pyoracle as po
n, Lw, TICKS = 12000, 3800.0, 6
d = tempfile.mkdtemp(dir=os.environ.get("GRAFT_REPO_ROOT", "/tmp") + "/gpurun_out")
env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=ROOT)
for it in range(2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           f"--master-port={29750 + it}", ROOT + "/tests/strips_worker.py", d, str(n), str(Lw), str(TICKS)]
    r = subprocess.run(cmd, env=env, timeout=200, capture_output=True, text=True)
    print("rc", r.returncode, r.stderr[-500:] if r.returncode else "")
    want = SC.global_events(po, n, Lw, 100.0, 0x5EED0004, TICKS)
    per = [np.load(os.path.join(d, f"r{k}.npz")) for k in range(2)]
    for t in range(TICKS):
        got = SC.merge_sorted([p[f"arr_{t}"] for p in per])
        if not np.array_equal(got, want[t]):
            gs = set(map(tuple, got.tolist())); ws = set(map(tuple, want[t].tolist()))
            miss = sorted(ws - gs); extra = sorted(gs - ws)
            print("tick", t, "got", len(got), "want", len(want[t]), "missing", len(miss), miss[:10], "extra", len(extra), extra[:10])
            for k in range(2):
                a = per[k][f"arr_{t}"]
                print("  rank", k, "events", len(a), "movers of missing in this rank's output:", sum(1 for m in miss if m[0] in set(a[:,0].tolist())))
        else:
            print("tick", t, "ok", len(got))
