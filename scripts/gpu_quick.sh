#!/bin/bash
# Quick GPU iteration: parity tests, then a short config-2 bench (no CPU baseline).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-quick}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --latency-ticks 10 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
