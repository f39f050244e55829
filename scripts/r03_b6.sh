#!/bin/bash
# Dense walk A/B on the crowd workloads and on single-D crowds (variants/: base = the round's first
# commit's kernels, bs = batched + XCD-aware with the binary-search candidate locate, new = in-tree,
# the LDS candidate list with a per-lane fill for sparse parts). set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b6}
timeout -k 10 400 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -k "config5 or skew or strip" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # tag workload variant extra...
  local t=$1 w=$2 v=$3; shift 3
  n=$(ls gpurun_out/ | grep -c "^${TAG}_${t}_${v}_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 200 python -u bench.py --workload $w --steps 20 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline "$@" > gpurun_out/${TAG}_${t}_${v}_$n.json 2> gpurun_out/${TAG}_${t}_${v}_$n.err
}
for v in base bs new bs new; do run skew50 skew50 $v; done
for v in base bs new bs new; do run skew skew $v; done
for v in bs new; do run s50d100 skew50 $v --dists 100,100,100,100; done
for v in bs new; do run s50d400 skew50 $v --dists 400,400,400,400; done
