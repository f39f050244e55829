/*
 * gwaoi_workload.h — the deterministic seeded random-walk workload of SURVEY.md §8(d), shared
 * bit-for-bit by the host (C oracle, tests) and the device (bench generator kernel in libgwaoi).
 *
 * Inputs: N slots, world [0,L)^2, step s, seed. Tick 0 places slot i uniformly:
 *     x0 = clamp_below_L(u(seed,0,i,0) * L),  z0 = clamp_below_L(u(seed,0,i,1) * L)
 * Tick t >= 1 moves every slot by a uniform step per axis, reflected at the world edges:
 *     x_t = reflect(x_{t-1} + (2u - 1) * s)
 * u is a float in [0,1) built from the top 24 bits of a splitmix64 hash of (seed, t*N + i, axis).
 * Every float op below is a single IEEE binary32 op with round-to-nearest-even; build both sides with
 * -ffp-contract=off (there is no a*b+c pair whose contraction could change a result anyway:
 * 2u-1 is exact and s multiplies an exact value).
 *
 * This is input synthesis only; it is not part of the AOI semantics under test.
 */
#ifndef GWAOI_WORKLOAD_H
#define GWAOI_WORKLOAD_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define GWW_HD __host__ __device__ __forceinline__
#else
#define GWW_HD static inline
#endif

GWW_HD uint64_t gww_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* u in [0,1), a multiple of 2^-24 (exactly representable as float). */
GWW_HD float gww_u01(uint64_t seed, uint64_t tick, uint64_t n, uint64_t slot, uint32_t axis) {
  uint64_t h = gww_splitmix64(gww_splitmix64(seed ^ (tick * n + slot)) + (uint64_t)axis);
  return (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f);
}

/* Largest float strictly below L (L > 0, finite). */
GWW_HD float gww_below(float L) {
  union { float f; uint32_t u; } c;
  c.f = L;
  c.u -= 1u;
  return c.f;
}

GWW_HD float gww_reflect(float v, float L) {
  if (v < 0.0f) v = -v;
  if (v >= L) v = L - (v - L);
  if (v >= L) v = gww_below(L);
  if (v < 0.0f) v = 0.0f;
  return v;
}

GWW_HD float gww_init_coord(uint64_t seed, uint64_t n, uint64_t slot, uint32_t axis, float L) {
  float v = gww_u01(seed, 0, n, slot, axis) * L;
  if (v >= L) v = gww_below(L);
  return v;
}

GWW_HD float gww_step_coord(float prev, uint64_t seed, uint64_t tick, uint64_t n, uint64_t slot,
                            uint32_t axis, float L, float s) {
  float u = gww_u01(seed, tick, n, slot, axis);
  float d = (u * 2.0f - 1.0f) * s;
  return gww_reflect(prev + d, L);
}

/* Skewed crowd: one id in `hot_every` (id % hot_every == 1) sits around one
 * of nhot hotspot centres (uniform in [L/8, 7L/8)^2) with an approximately Gaussian offset — the sum
 * of four uniforms minus 2 (Irwin-Hall, std 1/sqrt(3)) times sigma*sqrt(3) — the others are uniform in
 * [0,L)^2. Only binary32 add/mul, so host and device agree bit for bit (no libm transcendental whose
 * last bit could differ). Reflected into [0, L) like the walk. Moves then use gww_step_coord. */
GWW_HD float gww_skew_init_coord(uint64_t seed, uint64_t n, uint64_t id, uint32_t axis, float L, uint32_t nhot,
                                 float sigma, uint32_t hot_every) {
  if (nhot == 0u || hot_every == 0u || id % hot_every != 1u % hot_every) return gww_init_coord(seed, n, id, axis, L);
  const uint32_t h = (uint32_t)(gww_splitmix64(seed ^ (0xC0FFEEull + id)) % nhot);
  const float c = L * 0.125f + gww_u01(seed ^ 0x5A5A5A5Aull, 0, nhot, h, axis) * (L * 0.75f);
  float s = 0.0f;
  for (uint32_t k = 0; k < 4; ++k) s += gww_u01(seed, 1000003ull + k, n, id, axis);
  const float v = c + (s - 2.0f) * (sigma * 1.7320508f);
  return gww_reflect(v, L);
}

#endif /* GWAOI_WORKLOAD_H */
