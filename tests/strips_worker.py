"""One rank of tests/test_strips.py::test_gpu_strips_two_processes (launched by torch.distributed.run):
a StripNode on cuda:0 (ranks share the GPU), halo exchange by exchange_dist over gloo through host
memory; writes this rank's per-tick events to <outdir>/r<rank>.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    outdir, n, L, ticks = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from goworld_amd.strips import StripLayout, StripNode, exchange_dist
    lay = StripLayout(world, L, 100.0, 1.0)
    nd = StripNode(lay, rank, n, device=0, seed=0x5EED0004)
    evs = [nd.start(host_events=True)]
    for t in range(1, ticks):
        lo, ro = nd.prepare(t)
        li, ri = exchange_dist(lo, ro, rank, world, via_cpu=True)
        evs.append(nd.finish(li, ri, host_events=True))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), *evs)
    nd.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
