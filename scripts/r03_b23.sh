#!/bin/bash
# Fan-out write pass LDS budget A/B (cur: 4096 pairs / 896 records staged, 3 blocks per CU; fp: 3072 / 512,
# 4 blocks; fq: 2560 / 448, 5 blocks): sync tests on fq, then the gametick line alternated. set -e.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b23}
GWAOI_LIB=$R/variants/libgwaoi_fq.so timeout -k 10 300 python -u -m pytest tests/test_sync.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for v in cur fp fq cur fp fq; do
  n=$(ls gpurun_out/ | grep -c "^${TAG}_gt_${v}_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 300 python -u bench.py --workload gametick --steps 100 > gpurun_out/${TAG}_gt_${v}_$n.json 2> gpurun_out/${TAG}_gt_${v}_$n.err
done
