#!/bin/bash
# One GPU call: smoke(), the config-3 bench line (with its per-Space CPU baseline), and a 2-rank
# rehearsal of the multi-rank bench path (both ranks on the box's one GPU, gloo for the barrier and
# the max-over-ranks reduction). Every GPU step has its own time limit; set -e stops at a failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-xc}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python -u bench.py --workload config3 --steps 300 > gpurun_out/${TAG}_config3.json 2> gpurun_out/${TAG}_config3.err
GWAOI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 200 --warmup 5 --latency-ticks 0 \
  --host-staged-ticks 0 > gpurun_out/${TAG}_n2_gloo.json 2> gpurun_out/${TAG}_n2_gloo.err
