#!/bin/bash
# FLAT-free emission and build A/B (variants: head = HEAD 33dbfd9, nf = LDS and global event stores kept
# apart + geometry from LDS or global by two code paths): GPU suite on nf first, then configs 2/3 and the
# crowd workloads alternated, then the ring-walk phase accounting of both (GW_STAMPS builds). set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b15}
GWAOI_LIB=$R/variants/libgwaoi_nf.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in head nf head nf; do run config2 $v 400; run config3 $v 100; done
for v in head nf; do run skew $v 20; run skew50 $v 20; done
for v in ost nfst; do
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline --stamps gpurun_out/${TAG}_config2_$v.npy > gpurun_out/${TAG}_config2_st_$v.json 2> gpurun_out/${TAG}_config2_st_$v.err
done
