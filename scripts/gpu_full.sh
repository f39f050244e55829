#!/bin/bash
# The round's measured artefacts in one GPU call: PMC passes (-> profiles/pmc_latest.json, read by
# bench.py for `roofline.traffic`), parity tests, the default bench line, rocprofv3 kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-full}
PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES" TAG=${TAG} bash scripts/pmc.sh
cd $R
python3 scripts/make_pmc_latest.py gpurun_out/${TAG}_pmc 1000000 profiles/pmc_latest.json > gpurun_out/${TAG}_pmc_summary.txt
cp profiles/pmc_latest.json gpurun_out/${TAG}_pmc_latest.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 300 --latency-ticks 10 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof_bench.err
