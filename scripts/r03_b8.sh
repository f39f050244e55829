#!/bin/bash
# Dense-walk phase accounting (variants/libgwaoi_stamps.so, GW_STAMPS=1): skew50 and skew with their
# per-wave phase cycles dumped (bench.py --stamps; words 16*16383.. of the dump). set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b8}
for w in skew50 skew; do
  GWAOI_LIB=$R/variants/libgwaoi_stamps.so timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline --stamps gpurun_out/${TAG}_${w}_stamps.npy > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
done
