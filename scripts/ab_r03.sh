#!/bin/bash
# Round-3 A/B: every variant in variants/LIST benched interleaved (config 2, short), then rocprofv3
# kernel stats once per distinct variant. Every GPU step time-limited; set -e ends at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-ab}
BENCH_ARGS="${BENCH_ARGS:---host-staged-ticks 0 --no-replay}" VSTEPS=${VSTEPS:-300} TAG=$TAG bash scripts/variants_run.sh
for v in $(tr ' ' '\n' < variants/LIST | awk '!seen[$0]++'); do
  (cd /tmp && export TMPDIR=/tmp && GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${v}_prof -o run -- python3 $R/bench.py --steps 100 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > $R/gpurun_out/${TAG}_${v}_prof.json 2> $R/gpurun_out/${TAG}_${v}_prof.err)
  python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_${v}_prof > $R/gpurun_out/${TAG}_${v}_kstats.txt
  rm -rf $R/gpurun_out/${TAG}_${v}_prof
done
