#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per counter group, each under its own time
# limit; chained with set -e). Outputs under gpurun_out/${TAG}_pmc*/. Parse with scripts/pmc_summary.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${TAG:-pmc}
ARGS="--steps 20 --warmup 2 --latency-ticks 0 --no-cpu-baseline ${BENCH_ARGS}"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/${TAG}_counters_list.txt 2>&1 || true
i=0
PMC_GROUPS=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE TCC_HIT_sum TCC_MISS_sum|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE"}
IFS='|' read -ra GRPS <<< "$PMC_GROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/${TAG}_pmc$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_pmc$i.json 2> $R/gpurun_out/${TAG}_pmc$i.err
done
