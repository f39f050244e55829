#!/bin/bash
# The round's evidence recipe, one GPU call (every GPU step under its own time limit; set -e stops at the
# first failure). Steps selected by STEPS_SEL (default: all):
#   pmc       PMC passes (scripts/pmc.sh) of config 2 (traffic + stall + LDS counters) and of every workload in
#             PMC_WORKLOADS (traffic only) -> profiles/pmc_latest.json, stamped with the library's source hash
#   suite     the GPU test suite (pytest -m gpu)
#   bench     the default bench line (config 2, CPU baseline) and its rocprofv3 kernel stats
#   workloads every workload in WORKLOADS: bench line + rocprofv3 kernel stats
#   loopback  an 8-strip world of 2M per strip on one GPU (scripts/strips_loopback_bench.py): every strip's
#             pipeline and the halo records it sends per tick
# Outputs: gpurun_out/${TAG}_*; copy what is judged into profiles/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-ev}
SEL=${STEPS_SEL:-pmc suite bench workloads loopback}
has() { [[ " $SEL " == *" $1 "* ]]; }
if has pmc; then
  PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
    BENCH_ARGS="--host-staged-ticks 0 --no-replay --p99-ticks 0" TAG=${TAG}_config2 bash scripts/pmc.sh
  python3 scripts/make_pmc_latest.py gpurun_out/${TAG}_config2_pmc config2 profiles/pmc_latest.json > gpurun_out/${TAG}_config2_pmc_latest.txt
  for w in ${PMC_WORKLOADS:-skew50 skew strips strips_skew gametick config3}; do
    PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
      BENCH_ARGS="--workload $w --steps 8 --warmup 2 --stage-ticks 4 --host-staged-ticks 0 --no-replay --p99-ticks 0" \
      TAG=${TAG}_$w bash scripts/pmc.sh
    python3 scripts/make_pmc_latest.py gpurun_out/${TAG}_${w}_pmc $w profiles/pmc_latest.json > gpurun_out/${TAG}_${w}_pmc_latest.txt
  done
  cp profiles/pmc_latest.json gpurun_out/${TAG}_pmc_latest.json
fi
if has suite; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
fi
if has bench; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_config2_prof -o run -- python3 $R/bench.py --steps 300 --latency-ticks 10 --p99-ticks 0 --small-reps 0 --no-cpu-baseline > $R/gpurun_out/${TAG}_config2_prof.json 2> $R/gpurun_out/${TAG}_config2_prof.err)
  python3 scripts/kstats.py gpurun_out/${TAG}_config2_prof > gpurun_out/${TAG}_config2_kstats.txt
  cp gpurun_out/${TAG}_config2_prof/run_kernel_stats.csv gpurun_out/${TAG}_config2_kernel_stats.csv 2>/dev/null || true
  rm -rf gpurun_out/${TAG}_config2_prof
fi
if has workloads; then
  STEPS=${WSTEPS:-100} WORKLOADS="${WORKLOADS:-config3 skew skew50 strips strips_skew gametick}" TAG=$TAG bash scripts/workloads_prof.sh
fi
if has loopback; then
  timeout -k 10 600 python -u scripts/strips_loopback_bench.py 8 2000000 20 > gpurun_out/${TAG}_strips_loopback.json 2> gpurun_out/${TAG}_strips_loopback.err
fi
