/*
 * TEST INFRASTRUCTURE ONLY. Host-side wrappers of include/gwaoi_workload.h for the oracle library,
 * so Python tests and bench.py's cpu_baseline leg generate the exact inputs the device generator does.
 */
#include <stdint.h>

#include "gwaoi_workload.h"

void ow_init(uint64_t seed, uint32_t n, float L, float* x, float* z) {
  for (uint32_t i = 0; i < n; ++i) {
    x[i] = gww_init_coord(seed, n, i, 0, L);
    z[i] = gww_init_coord(seed, n, i, 1, L);
  }
}

/* advance every slot from tick-1 to tick (tick >= 1), in place */
void ow_step(uint64_t seed, uint64_t tick, uint32_t n, float L, float s, float* x, float* z) {
  for (uint32_t i = 0; i < n; ++i) {
    x[i] = gww_step_coord(x[i], seed, tick, n, i, 0, L, s);
    z[i] = gww_step_coord(z[i], seed, tick, n, i, 1, L, s);
  }
}

float ow_u01(uint64_t seed, uint64_t tick, uint64_t n, uint64_t slot, uint32_t axis) {
  return gww_u01(seed, tick, n, slot, axis);
}

/* config 5 (skewed crowd) initial placement, host side */
void ow_skew_init(uint64_t seed, uint32_t n, float L, uint32_t nhot, float sigma, uint32_t hot_every, float* x,
                  float* z) {
  for (uint32_t i = 0; i < n; ++i) {
    x[i] = gww_skew_init_coord(seed, n, i, 0, L, nhot, sigma, hot_every);
    z[i] = gww_skew_init_coord(seed, n, i, 1, L, nhot, sigma, hot_every);
  }
}
