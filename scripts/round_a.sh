#!/bin/bash
# Round evidence, part A: PMC traffic passes (-> profiles/pmc_latest.json, read by bench.py's
# roofline), the GPU test suite, the default bench line (config 2 + CPU baseline) and its rocprofv3
# kernel stats. Part B (scripts/workloads_prof.sh) runs the other workloads.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-final}
PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" TAG=$TAG bash scripts/pmc.sh
python3 scripts/make_pmc_latest.py gpurun_out/${TAG}_pmc 1000000 profiles/pmc_latest.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_config2_prof -o run -- python3 $R/bench.py --steps 300 --latency-ticks 10 --no-cpu-baseline > $R/gpurun_out/${TAG}_config2_prof.json 2> $R/gpurun_out/${TAG}_config2_prof.err)
python3 scripts/kstats.py gpurun_out/${TAG}_config2_prof > gpurun_out/${TAG}_config2_kstats.txt
