#!/bin/bash
# k_sweep tile blocks write their events into per-tile regions of ev_tmp (counts stored, no flush
# atomics): the whole GPU suite, then config 2/3 and the crowd workloads. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b25}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
run() {
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_" || true)
  timeout -k 10 200 python -u bench.py --workload $1 --steps $2 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$n.json 2> gpurun_out/${TAG}_$1_$n.err
}
run config2 1000; run config3 300; run config2 1000; run config3 300; run skew 20; run skew50 20; run strips 100
