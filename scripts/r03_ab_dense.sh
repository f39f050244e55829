#!/bin/bash
# Dense-walk A/B (variants/libgwaoi_{base,new}.so, interleaved) on the crowd workloads after the
# crowd parity tests of the in-tree build; rocprofv3 kernel stats of the in-tree build on skew50.
# Every GPU step time-limited; set -e ends the script at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 400 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py tests/test_refine.py -k "config5 or skew or refine" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
for w in ${WORKLOADS:-skew50 skew}; do
  for v in ${VARIANTS:-base new base new}; do
    n=$(ls gpurun_out/ | grep -c "^${TAG}_${w}_${v}_" || true)
    GWAOI_LIB=$R/variants/libgwaoi_$v.so timeout -k 10 200 python -u bench.py --workload $w --steps ${STEPS:-30} --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_${w}_${v}_$n.json 2> gpurun_out/${TAG}_${w}_${v}_$n.err
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --workload skew50 --steps 15 --warmup 3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.json 2> $R/gpurun_out/${TAG}_prof.err)
python3 scripts/kstats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_skew50_kstats.txt
rm -rf gpurun_out/${TAG}_prof
