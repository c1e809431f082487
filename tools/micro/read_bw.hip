// Calibration micro for rocprofv3's FETCH_SIZE at the read widths the per-step kernel uses
// (MI355X_MICROARCH.md §HBM: "FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
// streaming read (16 B/lane) ... other access widths are uncalibrated").  Each kernel reads a
// known byte count, coalesced, one element per lane per pass, at 1, 4, 8 or 16 bytes per lane,
// and writes one dword per workgroup (counted separately: 4 B x blocks).  Two sizes each: the
// per-step kernel's per-array footprint (65536 lanes) and a 256 MiB stream.  Under
//   rocprofv3 --pmc FETCH_SIZE -- tools/micro/bin/read_bw
// each dispatch's FETCH_SIZE (KiB) is set against the bytes this program prints for it.
// Build: hipcc --offload-arch=gfx950 -O3 -o read_bw read_bw.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ unsigned fold(T v) { return (unsigned)v; }
template <>
__device__ __forceinline__ unsigned fold(u32x2 v) { return v.x ^ v.y; }
template <>
__device__ __forceinline__ unsigned fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// every thread of the grid reads elements i, i + stride, ...; the XOR of what a workgroup read
// goes out as one dword, so no load is dead
template <typename T>
__global__ __launch_bounds__(256) void rd(const T* __restrict__ in, unsigned n, unsigned* out) {
  __shared__ unsigned acc[256];
  unsigned x = 0;
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x ^= fold(in[i]);
  acc[threadIdx.x] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned s = 0;
    for (int k = 0; k < 256; ++k) s ^= acc[k];
    out[blockIdx.x] = s;
  }
}

template <typename T>
static void run(const char* name, const void* buf, size_t bytes, unsigned blocks, unsigned* out) {
  const unsigned n = (unsigned)(bytes / sizeof(T));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(rd<T>, dim3(blocks), dim3(256), 0, 0, (const T*)buf, n, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-4s width %2zu B/lane: read %10zu B (%8.1f KiB), out %6u B, %8.2f us\n", name, sizeof(T), bytes,
           bytes / 1024.0, 4 * blocks, ms * 1e3);
  }
}

int main() {
  const size_t big = (size_t)256 << 20;
  void* buf;
  unsigned* out;
  if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 0x5A, big);
  (void)hipDeviceSynchronize();
  // per-step footprint: 65536 lanes, one element each (1024 workgroups of 256, as the step)
  run<unsigned char>("u8", buf, 65536, 256, out);
  run<unsigned>("u32", buf, 65536 * 4, 256, out);
  run<u32x2>("u64", buf, 65536 * 8, 256, out);
  run<u32x4>("u128", buf, 65536 * 16, 256, out);
  // streaming: 256 MiB at each width
  run<unsigned>("u32", buf, big, 4096, out);
  run<u32x2>("u64", buf, big, 4096, out);
  run<u32x4>("u128", buf, big, 4096, out);
  return 0;
}
