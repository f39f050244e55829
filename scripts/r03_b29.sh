#!/bin/bash
# Relation count pass with per-tile totals (k_rel_total) instead of two same-address atomics per wave:
# the GPU suite, then config 2 with the relation timings. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b29}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 1000 --no-cpu-baseline > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
