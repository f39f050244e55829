#!/bin/bash
# Grid cell budget A/B (variants: head = HEAD, cps5/cps8 = 5 / 8 cells per slot of capacity with a
# 16,384-tile bucket histogram): the crowd workloads, whose D = 50 Space is coarsened by the budget,
# and configs 2/3 (unaffected geometry). Crowd parity tests on cps8 first. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b14}
GWAOI_LIB=$R/variants/libgwaoi_cps8.so timeout -k 10 500 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -k "config5 or skew" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for w in skew50 skew; do for v in head cps5 cps8 head cps5 cps8; do run $w $v 20; done; done
for v in head cps8 head cps8; do run config2 $v 400; done
# ring-walk phase accounting of k_sweep on config 2 (GW_STAMPS build)
GWAOI_LIB=$R/variants/libgwaoi_stamps.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline --stamps gpurun_out/${TAG}_config2_stamps.npy > gpurun_out/${TAG}_config2_st.json 2> gpurun_out/${TAG}_config2_st.err
