// Micro-benchmark: achievable HBM write bandwidth for the obs-store pattern of the step
// kernels (each workgroup streams one contiguous region with 16-byte stores, every wave-
// instruction 1 KiB contiguous).  Build: hipcc --offload-arch=gfx950 -O3 -o write_bw write_bw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void wr(u32x4* out, unsigned per_block, unsigned threads) {
  if (threadIdx.x >= threads) return;
  u32x4* o = out + (size_t)blockIdx.x * per_block;
  const u32x4 v = {threadIdx.x, blockIdx.x, 1u, 2u};
  for (unsigned q = threadIdx.x; q < per_block; q += threads) {
    if (NT) __builtin_nontemporal_store(v, o + q);
    else o[q] = v;
  }
}

int main(int argc, char** argv) {
  // default ~ the 31x31 obs of 65536 envs; argv[1] = MiB (28 ~ the 11x11 obs)
  const size_t total = (size_t)(argc > 1 ? atoi(argv[1]) : 194) << 20;
  u32x4* buf;
  hipMalloc(&buf, total + (64 << 20));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct Cfg { unsigned blocks, threads; bool nt; };
  std::vector<Cfg> cfgs = {{1024, 256, true}, {1024, 256, false}, {1024, 192, true}, {2048, 256, true},
                           {4096, 256, true}, {8192, 256, true}, {512, 256, true}, {256, 256, true},
                           {16384, 256, true}, {4096, 256, false}, {8192, 256, false}, {16384, 256, false}};
  for (const Cfg& c : cfgs) {
    const unsigned per_block = (unsigned)(total / 16 / c.blocks);
    float best = 1e9f;
    for (int rep = 0; rep < 20; ++rep) {
      hipEventRecord(a, 0);
      if (c.nt) hipLaunchKernelGGL(wr<true>, dim3(c.blocks), dim3(256), 0, 0, buf, per_block, c.threads);
      else hipLaunchKernelGGL(wr<false>, dim3(c.blocks), dim3(256), 0, 0, buf, per_block, c.threads);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep >= 3 && ms < best) best = ms;
    }
    const double bytes = (double)per_block * 16.0 * c.blocks;
    printf("blocks %5u threads %3u %s: %7.2f us  %7.1f GB/s\n", c.blocks, c.threads, c.nt ? "nt " : "reg", best * 1e3,
           bytes / (best * 1e-3) / 1e9);
  }
  return 0;
}
