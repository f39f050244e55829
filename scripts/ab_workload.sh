#!/bin/bash
# A/B of the variants in variants/LIST on one workload (bench line per variant, same box).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-ab}
W=${W:-skew50}
for v in $(cat variants/LIST); do
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 300 python -u bench.py --workload $W --steps ${STEPS:-50} --latency-ticks 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${W}_${v}.json 2> gpurun_out/${TAG}_${W}_${v}.err
done
