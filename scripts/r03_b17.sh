#!/bin/bash
# One-pass build without fences: build tests, then config 2/3 counting vs one-pass. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b17}
timeout -k 10 300 python -u -m pytest tests/test_build.py tests/test_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  extra=""; [ "$2" = cb ] && extra="--counting-build"
  timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline $extra > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in cb fz cb fz; do run config2 $v 400; run config3 $v 100; done
run strips fz 50
