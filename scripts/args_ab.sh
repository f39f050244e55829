#!/bin/bash
# Bench-argument A/B on the default build: each line of $ARGS_FILE is "name bench-args..."; the n-th
# run of a name writes gpurun_out/${TAG}_${name}_n.json. Summary in gpurun_out/${TAG}_summary.txt.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-args}
declare -A seen
while read -r name rest; do
  [ -z "$name" ] && continue
  seen[$name]=$(( ${seen[$name]:-0} + 1 ))
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps ${VSTEPS:-100} --latency-ticks 0 --host-staged-ticks 0 $rest > gpurun_out/${TAG}_${name}_${seen[$name]}.json 2> gpurun_out/${TAG}_${name}_${seen[$name]}.err
done < ${ARGS_FILE:-variants/ARGS}
python3 scripts/vsum.py gpurun_out/${TAG}_*.json > gpurun_out/${TAG}_summary.txt 2>&1 || true
