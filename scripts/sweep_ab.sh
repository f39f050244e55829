#!/bin/bash
# Sweep-kernel A/B on the config-2 bench: 0 = flat global-memory sweep, 1 = LDS-staged, 2 = staging only.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${TAG:-ab}
for mode in ${MODES:-0 1 2}; do
  timeout -k 10 120 python -u $R/bench.py --no-cpu-baseline --steps 300 --latency-ticks 10 --sweep-lds $mode ${BENCH_ARGS} > $R/gpurun_out/${TAG}_mode$mode.json 2> $R/gpurun_out/${TAG}_mode$mode.err
done
