#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per counter group, each under its own time
# limit; chained with set -e). Outputs under gpurun_out/${TAG}_pmc*/; summarise with
# scripts/make_pmc_latest.py (per workload, stamped) or scripts/pmc_summary.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${TAG:-pmc}
ARGS="--steps 20 --warmup 2 --latency-ticks 0 --small-reps 0 --no-cpu-baseline ${BENCH_ARGS}"
cd /tmp && export TMPDIR=/tmp
i=0
PMC_GROUPS=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE"}
IFS='|' read -ra GRPS <<< "$PMC_GROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/${TAG}_pmc$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_pmc$i.json 2> $R/gpurun_out/${TAG}_pmc$i.err
done
