#!/bin/bash
# Short runs of every bench workload on one GPU (config 2/3/5 and the X-strip config 4 with 1 strip,
# plus 2 strips as 2 processes sharing the GPU over gloo).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-modes}
S=${STEPS:-100}
for wl in ${WLS-config3 skew strips}; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps $S --latency-ticks 5 --no-cpu-baseline > gpurun_out/${TAG}_$wl.json 2> gpurun_out/${TAG}_$wl.err
done
if [ -z "$NO2P" ]; then
GWAOI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 bench.py --gpus 2 --workload strips --per-gpu 1000000 --steps $S > gpurun_out/${TAG}_strips2p.json 2> gpurun_out/${TAG}_strips2p.err
fi
