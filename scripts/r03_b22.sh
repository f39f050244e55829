#!/bin/bash
# Fan-out count pass without the per-wave atomics on one word (per-tile totals + k_fan_total): sync
# tests, then the gametick line twice. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b22}
timeout -k 10 300 python -u -m pytest tests/test_sync.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for i in 0 1; do
  timeout -k 10 300 python -u bench.py --workload gametick --steps 100 > gpurun_out/${TAG}_gametick_$i.json 2> gpurun_out/${TAG}_gametick_$i.err
done
