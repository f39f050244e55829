#!/bin/bash
# pl = before the per-tile event regions; pt = regions + k_place's region pass unrolled (4 entries per
# thread, loads first). Parity subset on pt, then configs 2/3 alternated. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b27}
GWAOI_LIB=$R/variants/libgwaoi_pw.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_build.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in pt pw pt pw; do run config2 $v 1000; run config3 $v 300; done
