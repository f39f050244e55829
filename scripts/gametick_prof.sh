#!/bin/bash
# gametick workload (ingest + AOI tick + sync fan-out): bench line and rocprofv3 kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-gt}
timeout -k 10 300 python -u bench.py --workload gametick --steps ${STEPS:-200} ${BENCH_ARGS} > gpurun_out/${TAG}_gametick.json 2> gpurun_out/${TAG}_gametick.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_gtprof -o run -- python3 $R/bench.py --workload gametick --steps 50 ${BENCH_ARGS} > $R/gpurun_out/${TAG}_gtprof.json 2> $R/gpurun_out/${TAG}_gtprof.err
python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_gtprof > $R/gpurun_out/${TAG}_gt_kstats.txt
