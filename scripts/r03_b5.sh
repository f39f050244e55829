#!/bin/bash
# Dense walk with an LDS candidate list: crowd parity tests at the in-tree build, then A/B on the crowd
# workloads (variants/: base = the round's first commit's kernels, new = in-tree, p4w5 = 4 candidates
# per lane per round at 5 waves/SIMD, w5 = 2 per lane at 5 waves/SIMD). set -e: stop at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b5}
timeout -k 10 400 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -k "config5 or skew or strip" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for w in skew50 skew; do for v in base new p4w5 w5 new p4w5; do run $w $v 25; done; done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --workload skew50 --steps 20 --warmup 3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.json 2> $R/gpurun_out/${TAG}_prof.err)
python3 scripts/kstats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_skew50_kstats.txt
rm -rf gpurun_out/${TAG}_prof
