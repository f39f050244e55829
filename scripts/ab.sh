#!/bin/bash
# A/B of library variants (scripts/variants.py builds variants/libgwaoi_<name>.so and variants/LIST).
# Every name in variants/LIST is benched on each workload in WORKLOADS, in list order (repeat names in
# LIST to interleave runs on one box); then, with KSTATS=1, rocprofv3 kernel stats once per distinct
# variant on the first workload. Every GPU step time-limited; set -e ends at the first failure.
#   TAG, WORKLOADS (default config2), VSTEPS (300), BENCH_ARGS, SUITE=1 (GPU suite on variant $SUITE_LIB first)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-ab}
WORKLOADS=${WORKLOADS:-config2}
if [ -n "$SUITE_LIB" ]; then
  GWAOI_LIB=$R/variants/libgwaoi_$SUITE_LIB.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
fi
declare -A seen
for v in $(cat variants/LIST); do
  seen[$v]=$(( ${seen[$v]:-0} + 1 ))
  VARGS=""
  if [ -f variants/args_$v ]; then VARGS="$(cat variants/args_$v)"; fi
  for w in $WORKLOADS; do
    GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --steps ${VSTEPS:-300} --latency-ticks 0 --host-staged-ticks 0 --no-replay --p99-ticks ${P99:-0} ${BENCH_ARGS} $VARGS > gpurun_out/${TAG}_${w}_${v}_${seen[$v]}.json 2> gpurun_out/${TAG}_${w}_${v}_${seen[$v]}.err
  done
done
if [ -n "$KSTATS" ]; then
  w=${WORKLOADS%% *}
  for v in $(tr ' ' '\n' < variants/LIST | awk '!seen[$0]++'); do
    (cd /tmp && export TMPDIR=/tmp && GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${v}_prof -o run -- python3 $R/bench.py --workload $w --steps 100 --latency-ticks 0 --host-staged-ticks 0 --no-replay --p99-ticks 0 --small-reps 0 --no-cpu-baseline > $R/gpurun_out/${TAG}_${v}_prof.json 2> $R/gpurun_out/${TAG}_${v}_prof.err)
    python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_${v}_prof > $R/gpurun_out/${TAG}_${v}_kstats.txt
    rm -rf $R/gpurun_out/${TAG}_${v}_prof
  done
fi
