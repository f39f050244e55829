#!/bin/bash
# Dense walk with DPP scans, geometry in the batch and a window locate (no binary search): crowd parity
# tests at the in-tree build, then A/B (prev = before, new = in-tree, w8 = new at 8 waves/SIMD) and the
# phase accounting of w8 (GW_STAMPS). set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b9}
timeout -k 10 500 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -k "config5 or skew or strip" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps 20 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for w in skew50 skew; do for v in prev new w8 prev new w8; do run $w $v; done; done
for w in skew50 skew; do
  GWAOI_LIB=$R/variants/libgwaoi_stamps8.so timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline --stamps gpurun_out/${TAG}_${w}_stamps.npy > gpurun_out/${TAG}_${w}_st.json 2> gpurun_out/${TAG}_${w}_st.err
done
