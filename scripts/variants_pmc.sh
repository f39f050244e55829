#!/bin/bash
# Every variant in variants/LIST: bench timing (config 2) and one PMC pass of issue counters.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-vp}
PMC=${PMC:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY"}
for v in $(cat variants/LIST); do
  VARGS="$(cat variants/args_$v 2>/dev/null)"
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --latency-ticks 10 ${BENCH_ARGS} $VARGS > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
  (cd /tmp && export TMPDIR=/tmp && GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $R/gpurun_out/${TAG}_${v}_pmc -o run -- python3 $R/bench.py --steps 20 --warmup 2 --latency-ticks 0 --no-cpu-baseline ${BENCH_ARGS} $VARGS > $R/gpurun_out/${TAG}_${v}_pmc.log 2>&1)
done
