#!/bin/bash
# One GPU call: the GPU test suite on the default build, the variants of variants/LIST (config 2,
# scripts/variants_run.sh), then the parity file against a candidate variant (CAND, if set).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TAG=${TAG:-abs}
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
fi
TAG=$TAG bash scripts/variants_run.sh
for c in $CAND; do
  GWAOI_LIB=$R/variants/libgwaoi_$c.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_cand_${c}_pytest.log 2>&1
done
python3 scripts/vsum.py gpurun_out/${TAG}_*.json > gpurun_out/${TAG}_summary.txt 2>&1 || true
