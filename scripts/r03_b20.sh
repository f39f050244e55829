#!/bin/bash
# tsort start loads issued together; gametick timed without per-stage hipEvents. Build/config tests, then
# config 2 twice and the gametick line. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b20}
timeout -k 10 300 python -u -m pytest tests/test_build.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for i in 0 1; do
  timeout -k 10 200 python -u bench.py --steps 1000 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_config2_$i.json 2> gpurun_out/${TAG}_config2_$i.err
done
timeout -k 10 300 python -u bench.py --workload gametick --steps 100 > gpurun_out/${TAG}_gametick.json 2> gpurun_out/${TAG}_gametick.err
