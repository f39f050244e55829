#!/bin/bash
# Multi-Space geometry: cells backed off to the finest side that keeps the share's tile count (cf) vs
# the 1.25x steps (c0). Config-3 parity on cf first, then config 3 (and config 2, unaffected) alternated.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b31}
GWAOI_LIB=$R/variants/libgwaoi_cf.so timeout -k 10 500 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py tests/test_build.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in c0 cf c0 cf; do run config3 $v 300; done
run config2 cf 1000
