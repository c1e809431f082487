// Microbenchmark: the launch and memory floor of the default step's shape on gfx950.
// 1024 workgroups x 256 threads (B = 65536 envs, 64 per workgroup), ~14 KB LDS each, replayed
// in a hipGraph like bench.py:
//   empty   nothing but the launch
//   mem     each group loads its envs' state (hdr 16 B, food 8 B, bitmap 16 B, action 1 B per
//           env), one LDS barrier, then stores the group's 64 x 363 obs bytes with 16-byte
//           non-temporal stores plus 25 B of state per env: the step's HBM traffic, no compute
//   chain   mem with a dependent VALU chain of N instructions per wave between load and store
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

__global__ __launch_bounds__(1024) void k_empty(Bufs) {}

template <int CHAIN>
__global__ __launch_bounds__(256) void k_mem(Bufs b) {
  extern __shared__ uint32_t lds[];
  const int64_t g = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int wave = threadIdx.x >> 6;
  uint32_t v = 0;
  if (wave == 0) {
    const uint4 h = b.hdr[g];
    const double f = b.food[g];
    const uint4 m = b.bm[g];
    const int a = b.act[g];
    v = h.x ^ h.y ^ m.x ^ m.w ^ (uint32_t)a ^ (uint32_t)(int64_t)f;
#pragma unroll 1
    for (int i = 0; i < CHAIN; ++i) v = v * 0x85EBCA6Bu ^ (v >> 13);
    lds[threadIdx.x] = v;
    b.hdr_out[g] = make_uint4(h.x + 1, h.y, h.z, h.w);
    b.food_out[g] = f * 0.5;
    b.reward[g] = (float)(v & 1u);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const uint32_t w = lds[threadIdx.x & 63];
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4* out = reinterpret_cast<u32x4*>(b.obs + (size_t)blockIdx.x * 64 * 363);
  for (uint32_t u = threadIdx.x; u < 64 * 363 / 16; u += 256) {
    u32x4 q;
    for (int k = 0; k < 4; ++k) q[k] = ((w >> (4 * k + (u & 7))) & 0x01010101u);
    __builtin_nontemporal_store(q, out + u);
  }
}

template <typename K>
static float time_graph(K kern, Bufs b, int steps, int blocks = 1024, int threads = 256, int lds = 14336) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipGraph_t graph;
  hipGraphExec_t exec;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, s, b);
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

template <typename K>
static float time_stream(K kern, Bufs b, int steps, int blocks = 1024, int threads = 256, int lds = 14336) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, s, b);
  (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, s, b);
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
  printf("empty 1024x256   %.3f us/launch\n", time_graph(k_empty, b, 4000));
  printf("empty 512x512    %.3f us/launch\n", time_graph(k_empty, b, 4000, 512, 512, 28672));
  printf("empty 256x1024   %.3f us/launch\n", time_graph(k_empty, b, 4000, 256, 1024, 57344));
  printf("empty 4096x64    %.3f us/launch\n", time_graph(k_empty, b, 4000, 4096, 64, 3584));
  printf("empty 256x256    %.3f us/launch\n", time_graph(k_empty, b, 4000, 256, 256, 14336));
  printf("empty 1x64       %.3f us/launch\n", time_graph(k_empty, b, 4000, 1, 64, 0));
  printf("mem        %.3f us/launch\n", time_graph(k_mem<0>, b, 4000));
  printf("empty 1024x256 stream launches  %.3f us/launch\n", time_stream(k_empty, b, 4000));
  printf("mem stream launches             %.3f us/launch\n", time_stream(k_mem<0>, b, 4000));
  printf("chain 100 stream launches       %.3f us/launch\n", time_stream(k_mem<100>, b, 4000));
  printf("chain 100  %.3f us/launch\n", time_graph(k_mem<100>, b, 4000));
  printf("chain 400  %.3f us/launch\n", time_graph(k_mem<400>, b, 4000));
  printf("chain 1000 %.3f us/launch\n", time_graph(k_mem<1000>, b, 4000));
  return 0;
}
