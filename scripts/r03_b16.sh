#!/bin/bash
# One-pass tile build A/B on one library (cb = --counting-build, every pass counted first; fz = the
# one-pass build from the previous build's tile starts): configs 2/3 and the crowd workloads
# alternated, then the strips workload (2M slots: the reloading variant) once. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b16}
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  extra=""; [ "$2" = cb ] && extra="--counting-build"
  timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline $extra > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in cb fz cb fz; do run config2 $v 400; run config3 $v 100; done
for v in cb fz; do run skew $v 20; run skew50 $v 20; done
run strips fz 50
