#!/bin/bash
# In-tree library at HEAD (the multi-Space geometry back-off): the whole GPU suite, then config 3 with
# its CPU baseline and rocprofv3 kernel stats, and config 2 once more. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-r03_e5b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --workload config3 --steps 300 > gpurun_out/${TAG}_config3.json 2> gpurun_out/${TAG}_config3.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_config3_prof -o run -- python3 $R/bench.py --workload config3 --steps 300 --latency-ticks 10 --host-staged-ticks 0 --no-replay --no-cpu-baseline > $R/gpurun_out/${TAG}_config3_prof.json 2> $R/gpurun_out/${TAG}_config3_prof.err)
python3 scripts/kstats.py gpurun_out/${TAG}_config3_prof > gpurun_out/${TAG}_config3_kstats.txt
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
