// Microbenchmark: how many workgroups run concurrently per CU as a function of block size and
// dynamic LDS bytes (stamps of each block's start/end; max overlap). Diagnostic tool only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_busy(unsigned long long* st, int iters) {
  extern __shared__ unsigned int lds[];
  if (threadIdx.x == 0) st[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  unsigned int v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1664525u + 1013904223u;
  lds[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + (lds[1] == 12345u);
}

int main() {
  const int nb = 4096;
  unsigned long long* d;
  hipMalloc(&d, 2 * nb * sizeof(unsigned long long));
  std::vector<unsigned long long> h(2 * nb);
  hipFuncSetAttribute((const void*)&k_busy, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  int threads[] = {256, 512, 576, 1024};
  int ldsk[] = {4, 16, 32, 40, 48, 52, 54, 56, 64};
  for (int t : threads)
    for (int lk : ldsk) {
      size_t lds = (size_t)lk * 1024;
      int occ = 0;
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)&k_busy, t, lds);
      hipLaunchKernelGGL(k_busy, dim3(nb), dim3(t), lds, 0, d, 20000);
      hipDeviceSynchronize();
      hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
      std::vector<std::pair<unsigned long long, int>> ev;
      for (int b = 0; b < nb; ++b) ev.push_back({h[2 * b], 1}), ev.push_back({h[2 * b + 1], -1});
      std::sort(ev.begin(), ev.end());
      int cur = 0, mx = 0;
      for (auto& e : ev) cur += e.second, mx = std::max(mx, cur);
      printf("threads %4d lds %2dKB: occupancy API %d/CU, measured max concurrent %d (%.2f/CU)\n", t, lk, occ, mx, mx / 256.0);
    }
  return 0;
}
