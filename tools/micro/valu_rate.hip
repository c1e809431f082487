// Microbenchmark: VALU issue cost of the keyed-RNG building blocks on gfx950.
// Inline-asm chains (4 independent registers) so the compiler cannot fold them; the kernel
// time over a grid of 8 waves per SIMD gives cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP4(ins)                                                     \
  asm volatile(ins " %0, %0, %4\n\t" ins " %1, %1, %4\n\t" ins " %2, %2, %4\n\t" ins " %3, %3, %4" \
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k))

template <int OP>
__global__ void chain(uint32_t* out, int n, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = a * 3u + 1u, c = a + 7u, d = a ^ 0x55u, k = seed | 1u;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (OP == 0) OP4("v_xor_b32");
      else if (OP == 1) OP4("v_mul_lo_u32");
      else if (OP == 2) OP4("v_mul_u32_u24");
      else if (OP == 3) OP4("v_mul_hi_u32");
      else if (OP == 4) OP4("v_lshrrev_b32");
      else if (OP == 5) OP4("v_pk_mul_lo_u16");
      else if (OP == 6) OP4("v_add_u32");
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}

int main() {
  const int blocks = 256 * 4 * 8, threads = 64, n = 2000;
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)blocks * threads * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"v_xor_b32", "v_mul_lo_u32", "v_mul_u32_u24", "v_mul_hi_u32", "v_lshrrev_b32",
                         "v_pk_mul_lo_u16", "v_add_u32"};
  for (int op = 0; op < 7; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      switch (op) {
        case 0: chain<0><<<blocks, threads>>>(out, n, 1); break;
        case 1: chain<1><<<blocks, threads>>>(out, n, 1); break;
        case 2: chain<2><<<blocks, threads>>>(out, n, 1); break;
        case 3: chain<3><<<blocks, threads>>>(out, n, 1); break;
        case 4: chain<4><<<blocks, threads>>>(out, n, 1); break;
        case 5: chain<5><<<blocks, threads>>>(out, n, 1); break;
        case 6: chain<6><<<blocks, threads>>>(out, n, 1); break;
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double per_simd = (double)blocks * n * 8 * 4 / (256.0 * 4);
        printf("%-18s %8.3f ms  %.2f cycles/wave-inst per SIMD @2.4GHz\n", names[op], ms, ms * 1e-3 * 2.4e9 / per_simd);
      }
    }
  }
  return 0;
}
