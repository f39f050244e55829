#!/bin/bash
# Dense walk with its candidate rounds pipelined one deep (variants pipe6: 6 waves/SIMD, pipe5: 5):
# the crowd parity tests on pipe5, then A/B against dpp (the in-tree build) on skew50 and skew.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b11}
GWAOI_LIB=$R/variants/libgwaoi_pipe5.so timeout -k 10 500 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -k "config5 or skew" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps 20 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for w in skew50 skew; do for v in dpp pipe6 pipe5 dpp pipe6 pipe5; do run $w $v; done; done
