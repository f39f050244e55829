#!/bin/bash
# k_sweep diagnosis on config 2: phase stamps (GW_STAMPS build in variants/) and two PMC passes with
# the stall / issue counters (one rocprofv3 run each, own time limit). Outputs gpurun_out/${TAG}_*.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-diag}
ARGS="--steps 20 --warmup 2 --latency-ticks 0 --no-cpu-baseline ${BENCH_ARGS}"
if [ -f variants/libgwaoi_stamps.so ]; then
  GWAOI_LIB=$R/variants/libgwaoi_stamps.so timeout -k 10 120 python -u bench.py $ARGS --stamps gpurun_out/${TAG}_stamps.npy \
    > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err
  python3 scripts/stamps.py gpurun_out/${TAG}_stamps.npy > gpurun_out/${TAG}_stamps.txt
fi
cd /tmp && export TMPDIR=/tmp
i=0
GROUPS_=${PMC_GROUPS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU|SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"}
IFS='|' read -ra GRPS <<< "$GROUPS_"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/${TAG}_pmc$i -o run -- python3 $R/bench.py $ARGS \
    > $R/gpurun_out/${TAG}_pmc$i.json 2> $R/gpurun_out/${TAG}_pmc$i.err
done
