#!/bin/bash
# Round-3 session-2 first call at HEAD: refinement tests first, then the whole GPU suite, the default
# bench line, and skew50/skew with rocprofv3 kernel stats. set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-a1}
timeout -k 10 300 python -u -m pytest tests/test_refine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_refine.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
for w in ${WORKLOADS:-skew50 skew}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 40 --no-replay > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${w}_prof -o run -- python3 $R/bench.py --workload $w --steps 15 --warmup 3 --host-staged-ticks 0 --no-replay > $R/gpurun_out/${TAG}_${w}_prof.json 2> $R/gpurun_out/${TAG}_${w}_prof.err)
  python3 scripts/kstats.py gpurun_out/${TAG}_${w}_prof > gpurun_out/${TAG}_${w}_kstats.txt
  rm -rf gpurun_out/${TAG}_${w}_prof
done
