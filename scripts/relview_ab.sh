#!/bin/bash
# A/B of the relation view (variants/LIST): bench's relation_view_ms plus rocprofv3 kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-rv}
for v in $(cat variants/LIST); do
  (cd /tmp && export TMPDIR=/tmp && GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${v}_prof -o run -- python3 $R/bench.py --steps 100 --latency-ticks 0 --host-staged-ticks 0 --no-cpu-baseline > $R/gpurun_out/${TAG}_$v.json 2> $R/gpurun_out/${TAG}_$v.err)
  python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_${v}_prof > $R/gpurun_out/${TAG}_${v}_kstats.txt
done
if [ -n "$GT" ]; then
  for v in $(cat variants/LIST); do
    (cd /tmp && export TMPDIR=/tmp && GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${v}_gtprof -o run -- python3 $R/bench.py --workload gametick --steps 50 --warmup 5 > $R/gpurun_out/${TAG}_${v}_gt.json 2> $R/gpurun_out/${TAG}_${v}_gt.err)
    python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_${v}_gtprof > $R/gpurun_out/${TAG}_${v}_gt_kstats.txt
  done
fi
