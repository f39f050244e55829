#!/bin/bash
# GPU suite at the in-tree build (bk: every wave scan by DPP lane moves, build kernels with Space geometry in
# LDS and unconditional start-state loads), then config 2 against the
# previous build (variants/libgwaoi_dpp.so: DPP scans in the sweep staging and the dense walk only).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b12}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in dpp dpp2 bk dpp dpp2 bk; do run config2 $v 500; done
for v in dpp2 bk dpp2 bk; do run config3 $v 300; done
