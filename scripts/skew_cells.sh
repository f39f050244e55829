#!/bin/bash
# A/B of the cell side on config 5 (skew50): default D/4 vs absolute sides.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-sc}
WL=${WL:-skew50}
for cs in ${SIDES:-0 25 12.5}; do
  A=""; [ "$cs" != "0" ] && A="--cell-side $cs"
  timeout -k 10 200 python -u bench.py --workload $WL --steps ${STEPS:-5} --warmup 2 --latency-ticks 2 --no-cpu-baseline $A > gpurun_out/${TAG}_${WL}_$cs.json 2> gpurun_out/${TAG}_${WL}_$cs.err
done
