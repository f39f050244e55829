#!/bin/bash
# rocprofv3 kernel stats of a short config-2 bench for every variant in variants/LIST.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${TAG:-pv}
for v in $(cat $R/variants/LIST); do
  (cd /tmp && export TMPDIR=/tmp && GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${v}_prof -o run -- python3 $R/bench.py --steps ${STEPS:-100} --latency-ticks 0 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/${TAG}_${v}.json 2> $R/gpurun_out/${TAG}_${v}.err)
  python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_${v}_prof > $R/gpurun_out/${TAG}_${v}_kstats.txt
done
