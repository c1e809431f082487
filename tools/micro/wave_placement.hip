// Probe: where the dispatcher places the waves of a grid (XCC, SE, CU, SIMD per wave), for
// several workgroup sizes, to choose the workgroup shape of the step kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void probe(uint32_t* out, int iters) {
  uint32_t hw = 0, xcc = 0;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // some work so that all waves are resident together
  uint32_t v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1664525u + 1013904223u;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    out[2 * w] = hw;
    out[2 * w + 1] = (xcc & 0xF) | ((v & 1u) << 31);
  }
}

int main() {
  const int total_waves = 1024 * 4;
  uint32_t* d;
  (void)hipMalloc(&d, total_waves * 8);
  for (int wpg : {4}) {
    const int blocks = total_waves / wpg;
    (void)hipMemset(d, 0, total_waves * 8);
    probe<<<blocks, 64 * wpg>>>(d, 20000);
    (void)hipDeviceSynchronize();
    std::vector<uint32_t> h(total_waves * 2);
    (void)hipMemcpy(h.data(), d, total_waves * 8, hipMemcpyDeviceToHost);
    std::map<uint32_t, int> per_simd, per_cu, w0_per_simd;
    int same_simd_pairs = 0, pairs = 0;
    for (int w = 0; w < total_waves; ++w) {
      const uint32_t hw = h[2 * w], xcc = h[2 * w + 1] & 0xF;
      const uint32_t simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const uint32_t cu_key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
      per_cu[cu_key]++;
      per_simd[(cu_key << 2) | simd]++;
      if (w % wpg == 0) w0_per_simd[(cu_key << 2) | simd]++;
      if (wpg > 1 && (w % wpg) == 1) {
        const uint32_t hw0 = h[2 * (w - 1)];
        pairs++;
        if (((hw0 >> 4) & 3) == simd && ((hw0 >> 8) & 0xFFF) == ((hw >> 8) & 0xFFF)) same_simd_pairs++;
      }
    }
    std::map<int, int> hist_simd, hist_cu;
    for (auto& kv : per_simd) hist_simd[kv.second]++;
    for (auto& kv : per_cu) hist_cu[kv.second]++;
    printf("waves/WG=%d blocks=%d: CUs used %zu, SIMDs used %zu\n", wpg, blocks, per_cu.size(), per_simd.size());
    printf("  waves per SIMD histogram:");
    for (auto& kv : hist_simd) printf(" %d:%d", kv.first, kv.second);
    printf("\n  waves per CU histogram:");
    for (auto& kv : hist_cu) printf(" %d:%d", kv.first, kv.second);
    if (pairs) printf("\n  waves 0,1 of a WG on the same SIMD: %d of %d", same_simd_pairs, pairs);
    std::map<int, int> hist_w0;
    for (auto& kv : per_simd) hist_w0[w0_per_simd.count(kv.first) ? w0_per_simd[kv.first] : 0]++;
    printf("\n  wave-0s per SIMD histogram:");
    for (auto& kv : hist_w0) printf(" %d:%d", kv.first, kv.second);
    printf("\n");
  }
  return 0;
}
