// Microbenchmark: back-to-back graph-replayed launches of an empty kernel (one store per
// workgroup) for several grid shapes with the same 262144 threads: the per-launch cost that
// no kernel body can hide (the small step kernel runs 1024 x 256).  Also the same with the
// small kernel's dynamic LDS (14 KB per 256 threads) and a full-kernel-size SGPR count.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_empty(unsigned* out) {
  extern __shared__ unsigned lds[];
  if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
  if (out[0] == 0xFFFFFFFFu) lds[threadIdx.x] = 1u;  // (never: keeps the LDS allocation)
}

static float run(dim3 grid, dim3 block, size_t lds, hipStream_t s, unsigned* out, int reps) {
  hipGraph_t g;
  hipGraphExec_t e;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_empty, grid, block, lds, s, out);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(e, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9f;
  for (int it = 0; it < 5; ++it) {
    (void)hipEventRecord(a, s);
    (void)hipGraphLaunch(e, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  (void)hipGraphExecDestroy(e);
  (void)hipGraphDestroy(g);
  return best * 1e3f / reps;
}

int main() {
  unsigned* out;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  const int reps = 200;
  struct { unsigned nb, nt; } shapes[] = {{4096, 64}, {2048, 128}, {1024, 256}, {512, 512}, {256, 1024}, {64, 256}, {256, 256}};
  for (auto sh : shapes) {
    const float t0 = run(dim3(sh.nb), dim3(sh.nt), 0, s, out, reps);
    const float t1 = run(dim3(sh.nb), dim3(sh.nt), 56 * sh.nt, s, out, reps);
    printf("grid %5u x %4u: %6.3f us per launch, with %6u B LDS: %6.3f us\n", sh.nb, sh.nt, t0, 56 * sh.nt, t1);
  }
  return 0;
}
