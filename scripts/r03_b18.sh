#!/bin/bash
# One-pass build on the strips workload (2M-slot strip: chunks of 8192 slots, the reloading variant) and
# the crowd workloads, counting vs one-pass, alternated. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b18}
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  extra=""; [ "$2" = cb ] && extra="--counting-build"
  timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline $extra > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in cb fz cb fz; do run strips $v 100; done
for v in cb fz; do run skew $v 20; run skew50 $v 20; done
