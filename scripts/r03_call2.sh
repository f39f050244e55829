#!/bin/bash
# Refinement v2 check (tests + skew lines) then the grid/unroll A/B. set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-c2}
timeout -k 10 400 python -u -m pytest tests/test_refine.py tests/test_configs.py -k "refine or config5" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
WORKLOADS="skew50 skew" STEPS=40 TAG=$TAG bash -c 'for w in $WORKLOADS; do
  timeout -k 10 300 python -u bench.py --workload $w --steps $STEPS --no-replay > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d '$R'/gpurun_out/${TAG}_${w}_prof -o run -- python3 '$R'/bench.py --workload $w --steps 15 --warmup 3 --host-staged-ticks 0 --no-replay > '$R'/gpurun_out/${TAG}_${w}_prof.json 2> '$R'/gpurun_out/${TAG}_${w}_prof.err)
  python3 scripts/kstats.py gpurun_out/${TAG}_${w}_prof > gpurun_out/${TAG}_${w}_kstats.txt
  rm -rf gpurun_out/${TAG}_${w}_prof
done'
TAG=${TAG}_ab bash scripts/ab_r03.sh
