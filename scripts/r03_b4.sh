#!/bin/bash
# GPU suite at the in-tree build, then A/B (variants/: base = the round's first commit's kernels, new =
# in-tree, nx = new without the XCD-aware dense wave numbering) on config 2 and the crowd workloads.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${TAG:-b4}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
run() {  # workload variant steps
  n=$(ls gpurun_out/ | grep -c "^${TAG}_$1_$2_" || true)
  GWAOI_LIB=$R/variants/libgwaoi_$2.so timeout -k 10 200 python -u bench.py --workload $1 --steps $3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > gpurun_out/${TAG}_$1_$2_$n.json 2> gpurun_out/${TAG}_$1_$2_$n.err
}
for v in base new base new; do run config2 $v 400; done
for w in skew50 skew; do for v in base new; do run $w $v 25; done; done
for w in config2 skew50; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${w}_prof -o run -- python3 $R/bench.py --workload $w --steps 100 --warmup 3 --latency-ticks 0 --host-staged-ticks 0 --no-replay --no-cpu-baseline > $R/gpurun_out/${TAG}_${w}_prof.json 2> $R/gpurun_out/${TAG}_${w}_prof.err)
  python3 scripts/kstats.py gpurun_out/${TAG}_${w}_prof > gpurun_out/${TAG}_${w}_kstats.txt
  rm -rf gpurun_out/${TAG}_${w}_prof
done
