#!/bin/bash
# Ablation (timing only): k_sweep without its two per-block flush atomics on single counters (fb) vs cur.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b24}
for v in cur fb cur fb; do
  n=$(ls gpurun_out/ | grep -c "^${TAG}_c2_${v}_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 200 python -u bench.py --steps 300 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_c2_${v}_$n.json 2> gpurun_out/${TAG}_c2_${v}_$n.err || true
done
