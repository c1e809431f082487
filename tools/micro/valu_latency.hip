// Microbenchmark: dependent-issue latency vs independent throughput of VALU ops on gfx950,
// one wave per SIMD (256-thread workgroups, one per CU) and CH independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH, bool MUL>
__global__ void chain(uint32_t* out, int n) {
  uint32_t v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * (c + 1);
  const uint32_t k = 0x85EBCA6Bu;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if (MUL) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "v"(k));
        else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[c]) : "v"(k));
      }
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int CH, bool MUL>
void run(uint32_t* out, int blocks, const char* name) {
  const int n = 4000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(e0);
    chain<CH, MUL><<<blocks, 256>>>(out, n);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  const double insts_per_wave = (double)n * 16 * CH;
  const double waves_per_simd = blocks / 256.0;
  printf("%-10s chains=%d waves/SIMD=%.0f: %.2f cycles per wave-instruction @2.4GHz\n", name, CH,
         waves_per_simd, ms * 1e-3 * 2.4e9 / (insts_per_wave * waves_per_simd));
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)256 * 8 * 256 * 4);
  run<1, false>(out, 256, "xor");
  run<2, false>(out, 256, "xor");
  run<4, false>(out, 256, "xor");
  run<8, false>(out, 256, "xor");
  run<1, false>(out, 512, "xor");
  run<1, false>(out, 1024, "xor");
  run<1, true>(out, 256, "mul_lo");
  run<4, true>(out, 256, "mul_lo");
  run<8, true>(out, 256, "mul_lo");
  return 0;
}
