#!/bin/bash
# Sweep-kernel A/B (flat global / LDS-staged / staging-only) and PMC passes; run via gpurun.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for mode in 0 1 2; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --latency-ticks 10 --sweep-lds $mode > gpurun_out/bench_mode$mode.json 2> gpurun_out/bench_mode$mode.err
done
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
for mode in ${PMC_MODES:-1}; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc1_m$mode -o run -- python3 $R/bench.py --steps 20 --warmup 2 --latency-ticks 0 --no-cpu-baseline --sweep-lds $mode > $R/gpurun_out/pmc1_m$mode.json 2> $R/gpurun_out/pmc1_m$mode.err
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc2_m$mode -o run -- python3 $R/bench.py --steps 20 --warmup 2 --latency-ticks 0 --no-cpu-baseline --sweep-lds $mode > $R/gpurun_out/pmc2_m$mode.json 2> $R/gpurun_out/pmc2_m$mode.err
done
