#!/bin/bash
# Crowd workloads: hd = HEAD (dense-list appends one atomic per wave), da = one atomic per tile block,
# da5 = da + event chunks of 512 slots per wave reservation in the dense walk (was 128). Crowd parity
# tests on da5 first. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b28}
GWAOI_LIB=$R/variants/libgwaoi_da5.so timeout -k 10 500 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py tests/test_build.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --stage-ticks 10 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in hd da da5 hd da da5; do run skew50 $v 20; run skew $v 20; done
for v in hd da5; do run config2 $v 1000; done
