#!/bin/bash
# Sweep-kernel sensitivity to the cell size (cells per AOI distance), LDS path.
set -e
for cpd in ${CPDS:-2 3 4 6}; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --latency-ticks 10 --cells-per-dist $cpd > gpurun_out/bench_cpd$cpd.json 2> gpurun_out/bench_cpd$cpd.err
done
