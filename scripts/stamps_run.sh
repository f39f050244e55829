#!/bin/bash
# Per-block sweep phase stamps for each GW_STAMPS variant in variants/LIST.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-st}
for v in $(cat variants/LIST); do
  GWAOI_LIB=$R/variants/libgwaoi_$v.so VARGS="$(cat variants/args_$v 2>/dev/null)" ; GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 50 --latency-ticks 0 --stamps gpurun_out/${TAG}_$v.npy ${BENCH_ARGS} $VARGS > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
done
