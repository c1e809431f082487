// Microbenchmark: kernel-argument preloading on gfx950.  The memory-only step shape of
// floor.hip (load a group's state, one LDS barrier, store its obs and state), with the
// pointers either in a by-value struct (read by s_load from the kernarg segment, one memory
// round trip before the first global load) or as leading scalar arguments preloaded into
// SGPRs at wave launch (hipcc -mllvm -amdgpu-kernarg-preload-count=14).  Graph-replayed
// like bench.py.  Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=14
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct Bufs {
  uint4* hdr;
  double* food;
  uint4* bm;
  int8_t* act;
  uint8_t* obs;
  uint4* hdr_out;
  double* food_out;
  float* reward;
};

__device__ __forceinline__ void body(const uint4* hdr, const double* food, const uint4* bm, const int8_t* act,
                                     uint8_t* obs, uint4* hdr_out, double* food_out, float* reward) {
  extern __shared__ uint32_t lds[];
  const int64_t g = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int wave = threadIdx.x >> 6;
  if (wave == 0) {
    const uint4 h = hdr[g];
    const double f = food[g];
    const uint4 m = bm[g];
    const int a = act[g];
    const uint32_t v = h.x ^ h.y ^ m.x ^ m.w ^ (uint32_t)a ^ (uint32_t)(int64_t)f;
    lds[threadIdx.x] = v;
    hdr_out[g] = make_uint4(h.x + 1, h.y, h.z, h.w);
    food_out[g] = f * 0.5;
    reward[g] = (float)(v & 1u);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const uint32_t w = lds[threadIdx.x & 63];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4* out = reinterpret_cast<u32x4*>(obs + (size_t)blockIdx.x * 64 * 363);
  for (uint32_t u = threadIdx.x; u < 64 * 363 / 16; u += 256) {
    u32x4 q;
    for (int k = 0; k < 4; ++k) q[k] = ((w >> (4 * k + (u & 7))) & 0x01010101u);
    __builtin_nontemporal_store(q, out + u);
  }
}

__global__ __launch_bounds__(256) void k_struct(Bufs b) {
  body(b.hdr, b.food, b.bm, b.act, b.obs, b.hdr_out, b.food_out, b.reward);
}
__global__ __launch_bounds__(256) void k_preload(const uint4* hdr, const double* food, const uint4* bm,
                                                 const int8_t* act, uint8_t* obs, uint4* hdr_out, double* food_out,
                                                 Bufs b) {
  body(hdr, food, bm, act, obs, hdr_out, food_out, b.reward);
}

template <typename F>
static float time_graph(F launch, int steps) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipGraph_t graph;
  hipGraphExec_t exec;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 20; ++i) launch(s);
  (void)hipStreamEndCapture(s, &graph);
  (void)hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  for (int i = 0; i < 5; ++i) (void)hipGraphLaunch(exec, s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < steps / 20; ++i) (void)hipGraphLaunch(exec, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f / (float)steps;
}

int main() {
  const size_t B = 65536;
  Bufs b;
  (void)hipMalloc(&b.hdr, B * 16);
  (void)hipMalloc(&b.food, B * 8);
  (void)hipMalloc(&b.bm, B * 16);
  (void)hipMalloc(&b.act, B);
  (void)hipMalloc(&b.obs, B * 363);
  (void)hipMalloc(&b.hdr_out, B * 16);
  (void)hipMalloc(&b.food_out, B * 8);
  (void)hipMalloc(&b.reward, B * 4);
  (void)hipMemset(b.hdr, 0, B * 16);
  (void)hipMemset(b.food, 0, B * 8);
  (void)hipMemset(b.bm, 0, B * 16);
  (void)hipMemset(b.act, 0, B);
  for (int rep = 0; rep < 3; ++rep) {
    printf("struct   %.3f us/launch\n", time_graph([&](hipStream_t s) {
      hipLaunchKernelGGL(k_struct, dim3(1024), dim3(256), 14336, s, b); }, 4000));
    printf("preload  %.3f us/launch\n", time_graph([&](hipStream_t s) {
      hipLaunchKernelGGL(k_preload, dim3(1024), dim3(256), 14336, s, b.hdr, b.food, b.bm, b.act, b.obs, b.hdr_out,
                         b.food_out, b); }, 4000));
  }
  return 0;
}
