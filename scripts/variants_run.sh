#!/bin/bash
# Bench every variant listed in variants/LIST (config 2, short run, no CPU baseline). A name may
# repeat (A B A B: interleaved runs on one box); the n-th run of a name writes ${TAG}_${name}_n.json.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-var}
declare -A seen
for v in $(cat variants/LIST); do
  seen[$v]=$(( ${seen[$v]:-0} + 1 ))
  VARGS=""
  if [ -f variants/args_$v ]; then VARGS="$(cat variants/args_$v)"; fi
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps ${VSTEPS:-300} --latency-ticks 10 ${BENCH_ARGS} $VARGS > gpurun_out/${TAG}_${v}_${seen[$v]}.json 2> gpurun_out/${TAG}_${v}_${seen[$v]}.err
done
