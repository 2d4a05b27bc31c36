// Workgroup dispatch-rate probe (round 5): every workgroup stamps wall_clock64 (100 MHz,
// device-wide) when it starts and when it ends; the spread of start stamps over the grid
// is the dispatch time.  Varies the grid size, the workgroup size, the LDS per workgroup
// and the work per workgroup (spin ~ns) to separate the dispatcher rate from residency.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void probe(unsigned long long* st, unsigned long long* en, int spin_ticks) {
  extern __shared__ float lds[];
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) lds[0] = 1.f;
  if (spin_ticks > 0) {
    while (wall_clock64() - t0 < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
  if (threadIdx.x == 0) { st[blockIdx.x] = t0; en[blockIdx.x] = wall_clock64() + (lds[0] > 2.f ? 1 : 0); }
}

int main() {
  const int grids[] = {256, 1024, 2048, 4096};
  const int wgs[] = {64, 256, 1024};
  const int ldss[] = {0, 40 * 1024};
  const int spins[] = {0, 200};   // ticks of 10 ns: 0 or 2 us of residency per workgroup
  unsigned long long *st, *en;
  hipMalloc(&st, 8 * 8192); hipMalloc(&en, 8 * 8192);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
  std::vector<unsigned long long> hs(8192), he(8192);
  printf("{\"rows\": [\n");
  bool first = true;
  for (int spin : spins) for (int lds : ldss) for (int wg : wgs) for (int g : grids) {
    float best_ms = 1e9f; double best_spread = 0, best_span = 0;
    for (int rep = 0; rep < 5; ++rep) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(probe, dim3(g), dim3(wg), lds, 0, st, en, spin);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      hipMemcpy(hs.data(), st, 8 * g, hipMemcpyDeviceToHost);
      hipMemcpy(he.data(), en, 8 * g, hipMemcpyDeviceToHost);
      const unsigned long long s0 = *std::min_element(hs.begin(), hs.begin() + g);
      const unsigned long long s1 = *std::max_element(hs.begin(), hs.begin() + g);
      const unsigned long long e1 = *std::max_element(he.begin(), he.begin() + g);
      if (ms < best_ms) { best_ms = ms; best_spread = (s1 - s0) * 0.01; best_span = (e1 - s0) * 0.01; }
      hipEventDestroy(a); hipEventDestroy(b);
    }
    printf("%s{\"grid\": %d, \"wg\": %d, \"lds\": %d, \"spin_us\": %.1f, \"start_spread_us\": %.2f, \"span_us\": %.2f, \"event_ms\": %.4f, \"wg_per_us\": %.1f}",
           first ? "" : ",\n", g, wg, lds, spin * 0.01, best_spread, best_span, best_ms, best_spread > 0 ? g / best_spread : 0.0);
    first = false;
  }
  printf("\n]}\n");
  hipFree(st); hipFree(en);
  return 0;
}
