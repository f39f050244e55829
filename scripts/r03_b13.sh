#!/bin/bash
# Config 2 and 3 A/B of the build kernels: dpp2 = every wave scan by DPP, bk = dpp2 + Space geometry
# in LDS for the bucket count/scatter + start-of-pass state loaded unconditionally.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b13}
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in dpp2 bk dpp2 bk dpp2 bk; do run config2 $v 500; done
for v in dpp2 bk dpp2 bk; do run config3 $v 300; done
for v in dpp2 bk; do run skew50 $v 20; done
