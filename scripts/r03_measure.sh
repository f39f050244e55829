#!/bin/bash
# Round-3 measurement call: the default bench line (config 2 + CPU baseline), rocprofv3 kernel stats of
# config 2, skew50 and skew, and PMC passes of the dense walks on skew50. Every GPU
# step under its own time limit; set -e ends the script at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-m}
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_config2_prof -o run -- python3 $R/bench.py --steps 300 --latency-ticks 10 --host-staged-ticks 0 --no-replay --no-cpu-baseline > $R/gpurun_out/${TAG}_config2_prof.json 2> $R/gpurun_out/${TAG}_config2_prof.err)
python3 scripts/kstats.py gpurun_out/${TAG}_config2_prof > gpurun_out/${TAG}_config2_kstats.txt
rm -rf gpurun_out/${TAG}_config2_prof
for w in ${WORKLOADS:-skew50 skew}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-60} > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${w}_prof -o run -- python3 $R/bench.py --workload $w --steps 20 --warmup 3 > $R/gpurun_out/${TAG}_${w}_prof.json 2> $R/gpurun_out/${TAG}_${w}_prof.err)
  python3 scripts/kstats.py gpurun_out/${TAG}_${w}_prof > gpurun_out/${TAG}_${w}_kstats.txt
  rm -rf gpurun_out/${TAG}_${w}_prof
done
if [ -n "${PMC_SKEW}" ]; then
  PMC_GROUPS="FETCH_SIZE|TCC_HIT_sum TCC_MISS_sum|TCP_TOTAL_CACHE_ACCESSES_sum|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" BENCH_ARGS="--workload skew50 --steps 6 --warmup 2" TAG=${TAG}_skew50 bash scripts/pmc.sh
fi
