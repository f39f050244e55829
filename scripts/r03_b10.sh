#!/bin/bash
# GPU suite at the in-tree build (DPP wave scans in the sweep's staging and the dense walk, record
# gathers issued before the column-major pass), then A/B: prev = HEAD, dpp = in-tree, se0 = in-tree
# without the early gathers. set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b10}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in prev dpp se0 prev dpp se0; do run config2 $v 500; done
for w in skew50 skew; do for v in prev dpp prev dpp; do run $w $v 20; done; done
