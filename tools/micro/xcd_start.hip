// Microbenchmark: when does each XCD start a kernel's workgroups?  1024 workgroups x 256
// threads (the small step kernel's grid), each records s_memrealtime (100 MHz) at entry, its
// XCC_ID hardware register and the blockIdx, then spins ~2 us so that all stay resident.
// Launched back to back in a stream; prints, per XCC, the mean start offset from the
// kernel's first workgroup, and the blockIdx % 8 -> XCC mapping.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256) void k_start(uint64_t* t, uint32_t* xcc, int spin) {
  if (threadIdx.x == 0) {
    t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    xcc[blockIdx.x] = id & 0xFu;
  }
  uint32_t v = threadIdx.x;
  for (int i = 0; i < spin; ++i) v = v * 1664525u + 1013904223u;
  if (v == 0xFFFFFFFFu) t[0] = v;  // (keeps the loop)
}

int main() {
  const int nb = 1024, reps = 50;
  uint64_t* t;
  uint32_t* x;
  (void)hipMalloc(&t, nb * 8 * reps);
  (void)hipMalloc(&x, nb * 4 * reps);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_start, dim3(nb), dim3(256), 14336, 0, t + r * nb, x + r * nb, 1500);
  (void)hipDeviceSynchronize();
  std::vector<uint64_t> ht(nb * reps);
  std::vector<uint32_t> hx(nb * reps);
  (void)hipMemcpy(ht.data(), t, nb * 8 * reps, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hx.data(), x, nb * 4 * reps, hipMemcpyDeviceToHost);
  double start_xcc[8] = {0}, last_xcc[8] = {0};
  int cnt[8] = {0}, map_ok = 0;
  for (int r = 10; r < reps; ++r) {
    const uint64_t* tr = ht.data() + r * nb;
    const uint32_t* xr = hx.data() + r * nb;
    uint64_t t0 = *std::min_element(tr, tr + nb);
    uint64_t first[8], last[8];
    for (int k = 0; k < 8; ++k) { first[k] = ~0ull; last[k] = 0; }
    for (int b = 0; b < nb; ++b) {
      const uint32_t k = xr[b] & 7u;
      first[k] = std::min(first[k], tr[b] - t0);
      last[k] = std::max(last[k], tr[b] - t0);
      map_ok += (k == (uint32_t)(b % 8)) ? 1 : 0;
    }
    for (int k = 0; k < 8; ++k) { start_xcc[k] += first[k]; last_xcc[k] += last[k]; cnt[k]++; }
  }
  printf("blockIdx %% 8 == XCC_ID for %.1f %% of workgroups\n", 100.0 * map_ok / (nb * (reps - 10)));
  printf("XCC  first start  last start (us from the kernel's first workgroup)\n");
  for (int k = 0; k < 8; ++k)
    printf("%3d  %8.2f  %8.2f\n", k, start_xcc[k] / cnt[k] * 0.01, last_xcc[k] / cnt[k] * 0.01);
  return 0;
}
