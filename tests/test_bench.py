"""bench.py's multi-rank plumbing on the CPU: the self-launch decision and command line
(`bench.py --gpus N` without a launcher starts its own N ranks as a child), and a real 2-rank launch
through torch.distributed.run over gloo (--dry-run: rendezvous, barrier, max-over-ranks, no GPU work)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_self_launch_decision():
    import bench
    assert bench.self_launch_command(["--gpus", "1"], {}, 1, 0) is None
    # already under a launcher: never launch again
    assert bench.self_launch_command(["--gpus", "8"], {"WORLD_SIZE": "8"}, 8, 1234) is None
    cmd = bench.self_launch_command(["--gpus", "4", "--steps", "7"], {}, 4, 29512)
    assert cmd[0] == sys.executable
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29512" in cmd
    assert cmd[-4:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "7"][-4:]
    assert os.path.abspath(cmd[cmd.index("--master-port=29512") + 1]) == os.path.join(ROOT, "bench.py")


def test_self_launch_two_ranks_gloo():
    env = dict(os.environ, GWAOI_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["dry_run"] and r["backend"] == "gloo"
    assert abs(r["elapsed"] - 0.002) < 1e-9  # the max over both ranks
    # the N > 1 line carries the config-4 strips sub-measurement (every rank takes part: collective)
    st = r["strips"]
    assert st["workload"] == "strips" and st["n_gpus"] == 2 and st["dry_run"]
    assert abs(st["elapsed"] - 0.002) < 1e-9


def test_watchdog_ends_a_hung_rank():
    # a rank that outlives its watchdog exits with status 3 (no exec, no hang)
    code = ("import sys, time; sys.path.insert(0, %r); import bench; bench.arm_watchdog(0.5, 0); time.sleep(30)"
            % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3 and "watchdog" in p.stderr


def test_self_launch_propagates_failure():
    env = dict(os.environ, GWAOI_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    # the ranks start, then fail (no HIP device in this container): the parent exits non-zero, no JSON line
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--n", "1000", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
