#!/bin/bash
# Bench lines + rocprofv3 kernel stats for the non-default workloads (gametick, strips, strips_skew,
# config3, skew50). Every GPU step is time-limited; set -e ends the script at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-wl}
for w in ${WORKLOADS:-gametick strips strips_skew}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-200} ${BENCH_ARGS} > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${w}_prof -o run -- python3 $R/bench.py --workload $w --steps 50 --warmup 5 --small-reps 0 ${BENCH_ARGS} > $R/gpurun_out/${TAG}_${w}_prof.json 2> $R/gpurun_out/${TAG}_${w}_prof.err)
  python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_${w}_prof > $R/gpurun_out/${TAG}_${w}_kstats.txt
  rm -rf $R/gpurun_out/${TAG}_${w}_prof
done
