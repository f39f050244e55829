#!/bin/bash
# config 5 (skew50) per-D runs and a rocprofv3 kernel trace of the full workload.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-sp}
WL=${WL:-skew50}
for d in ${DS:-50 100 200 400}; do
  timeout -k 10 200 python -u bench.py --workload $WL --dists $d --steps ${STEPS:-5} --warmup 2 --latency-ticks 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${WL}_d$d.json 2> gpurun_out/${TAG}_${WL}_d$d.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --workload $WL --steps 5 --warmup 2 --latency-ticks 2 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/${TAG}_prof.json 2> $R/gpurun_out/${TAG}_prof.err
python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_prof > $R/gpurun_out/${TAG}_kstats.txt
