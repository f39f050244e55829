#!/bin/bash
# Bench every variant listed in variants/LIST (config 2, short run, no CPU baseline).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-var}
for v in $(cat variants/LIST); do
  GWAOI_LIB=$R/variants/libgwaoi_$v.so VARGS="$(cat variants/args_$v 2>/dev/null)" ; GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --latency-ticks 10 ${BENCH_ARGS} $VARGS > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
done
