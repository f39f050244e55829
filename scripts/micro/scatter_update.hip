// Micro-benchmark for DESIGN §8 "persistent cell-ordered grid" (verdict r4, item 4): the floor of an
// incremental grid at config 2 (1M slots). A persistent cell-ordered record store would still have to
// write every mover's record each tick (its start and end state change), through a slot -> record map
// whose order is the cells', i.e. a random permutation of the slots. Times, with hipEvents over 200
// launches each:
//   scatter : per slot, the 7 state words read coalesced, its 32-B record written at map[slot]
//   stream  : the same reads, the record written at [slot] (coalesced: the bandwidth floor)
//   gather  : per record in cell order, its slot's 7 state words gathered through the inverse map, the
//             record written coalesced (the other way round)
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/scatter_update scripts/micro/scatter_update.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

struct Rec {
  uint4 a, b;
};

__global__ void k_scatter(const float* px, const float* pz, const float* ox, const float* oz, const uint32_t* sq,
                          const uint32_t* oq, const uint32_t* op, const uint32_t* map, Rec* rec, uint32_t n) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  rec[map[s]] = Rec{make_uint4(__float_as_uint(px[s]), __float_as_uint(pz[s]), s, op[s]),
                    make_uint4(__float_as_uint(ox[s]), __float_as_uint(oz[s]), oq[s], sq[s])};
}

__global__ void k_stream(const float* px, const float* pz, const float* ox, const float* oz, const uint32_t* sq,
                         const uint32_t* oq, const uint32_t* op, Rec* rec, uint32_t n) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  rec[s] = Rec{make_uint4(__float_as_uint(px[s]), __float_as_uint(pz[s]), s, op[s]),
               make_uint4(__float_as_uint(ox[s]), __float_as_uint(oz[s]), oq[s], sq[s])};
}

__global__ void k_gather(const float* px, const float* pz, const float* ox, const float* oz, const uint32_t* sq,
                         const uint32_t* oq, const uint32_t* op, const uint32_t* inv, Rec* rec, uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t s = inv[j];
  rec[j] = Rec{make_uint4(__float_as_uint(px[s]), __float_as_uint(pz[s]), s, op[s]),
               make_uint4(__float_as_uint(ox[s]), __float_as_uint(oz[s]), oq[s], sq[s])};
}

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main() {
  const uint32_t n = 1000000;
  std::vector<uint32_t> map(n), inv(n);
  std::iota(map.begin(), map.end(), 0u);
  std::shuffle(map.begin(), map.end(), std::mt19937(7));
  for (uint32_t s = 0; s < n; ++s) inv[map[s]] = s;
  float *px, *pz, *ox, *oz;
  uint32_t *sq, *oq, *op, *dm, *di;
  Rec* rec;
  CK(hipMalloc(&px, 4 * n)); CK(hipMalloc(&pz, 4 * n)); CK(hipMalloc(&ox, 4 * n)); CK(hipMalloc(&oz, 4 * n));
  CK(hipMalloc(&sq, 4 * n)); CK(hipMalloc(&oq, 4 * n)); CK(hipMalloc(&op, 4 * n));
  CK(hipMalloc(&dm, 4 * n)); CK(hipMalloc(&di, 4 * n)); CK(hipMalloc(&rec, sizeof(Rec) * n));
  for (void* p : {(void*)px, (void*)pz, (void*)ox, (void*)oz, (void*)sq, (void*)oq, (void*)op}) CK(hipMemset(p, 0, 4 * n));
  CK(hipMemcpy(dm, map.data(), 4 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(di, inv.data(), 4 * n, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256), b(256);
  const int reps = 200;
  float ms[3];
  for (int v = 0; v < 3; ++v) {
    for (int w = 0; w < 2; ++w) {  // warm-up, then timed
      CK(hipEventRecord(e0));
      for (int r = 0; r < (w ? reps : 10); ++r) {
        if (v == 0) hipLaunchKernelGGL(k_scatter, g, b, 0, 0, px, pz, ox, oz, sq, oq, op, dm, rec, n);
        if (v == 1) hipLaunchKernelGGL(k_stream, g, b, 0, 0, px, pz, ox, oz, sq, oq, op, rec, n);
        if (v == 2) hipLaunchKernelGGL(k_gather, g, b, 0, 0, px, pz, ox, oz, sq, oq, op, di, rec, n);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[v], e0, e1));
    }
    ms[v] = ms[v] / reps * 1e3f;
  }
  std::printf("{\"n\": %u, \"scatter_us\": %.2f, \"stream_us\": %.2f, \"gather_us\": %.2f}\n", n, ms[0], ms[1], ms[2]);
  return 0;
}
