#!/bin/bash
# Timed ticks without per-stage hipEvents (stage timing in 200 ticks after the timed region): configs 2/3. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b19}
for i in 0 1; do
  timeout -k 10 200 python -u bench.py --steps 1000 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_config2_$i.json 2> gpurun_out/${TAG}_config2_$i.err
  timeout -k 10 200 python -u bench.py --workload config3 --steps 300 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_config3_$i.json 2> gpurun_out/${TAG}_config3_$i.err
done
