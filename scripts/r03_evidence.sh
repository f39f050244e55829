#!/bin/bash
# Round-3 evidence at HEAD: scripts/round_final.sh (config-2 PMC passes -> profiles/pmc_latest.json,
# the GPU suite, the default bench line, rocprofv3 kernel stats of every workload), then PMC passes of
# the dense walk on skew50 (cache hits/misses, traffic, waits, VALU). set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${TAG:-r03_e1}
TAG=$TAG bash scripts/round_final.sh
PMC_GROUPS="FETCH_SIZE|TCC_HIT_sum TCC_MISS_sum|TCP_TOTAL_CACHE_ACCESSES_sum|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" BENCH_ARGS="--workload skew50 --steps 6 --warmup 2 --host-staged-ticks 0 --no-replay" TAG=${TAG}_skew50 bash scripts/pmc.sh
