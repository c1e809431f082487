// Microbenchmark: when does each XCD start a kernel's workgroups?  1024 workgroups x 256
// threads (the small step kernel's grid, 14 KB LDS each), each records s_memrealtime (100 MHz)
// as its first instruction, its XCC_ID hardware register and the blockIdx, then spins ~2 us
// so that all stay resident.  Launched back to back in a stream (or replayed from a graph);
// prints, per XCC, the mean start offset from the kernel's first workgroup.  Variants: the
// kernel argument size (16 B of pointers vs a 672-byte by-value block like wab::Params) and
// the VGPR allocation (few vs ~128, by inline-asm clobbers), to find what delays XCDs 4-7 in
// the step kernel (profiles/r02_xcd/).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

struct Big {
  uint64_t* t;
  uint32_t* xcc;
  int spin;
  uint32_t pad[160];  // 672 bytes in all
};

template <bool VG>
__global__ __launch_bounds__(256) void k_big(Big b) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 0) {
    b.t[blockIdx.x] = t0;
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    b.xcc[blockIdx.x] = id & 0xFu;
  }
  uint32_t v = threadIdx.x ^ b.pad[threadIdx.x & 7];
  for (int i = 0; i < b.spin; ++i) v = v * 1664525u + 1013904223u;
  if (VG)
    asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14",
                 "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29",
                 "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44",
                 "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58",
                 "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72",
                 "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86",
                 "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100",
                 "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",
                 "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124",
                 "v125", "v126");
  if (v == 0xFFFFFFFFu) lds[threadIdx.x] = v;
  if (v == 0xFFFFFFFEu) b.t[0] = lds[(threadIdx.x + 1) & 255];
}

__global__ __launch_bounds__(256) void k_small(uint64_t* t, uint32_t* xcc, int spin) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 0) {
    t[blockIdx.x] = t0;
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    xcc[blockIdx.x] = id & 0xFu;
  }
  uint32_t v = threadIdx.x;
  for (int i = 0; i < spin; ++i) v = v * 1664525u + 1013904223u;
  if (v == 0xFFFFFFFFu) lds[threadIdx.x] = v;
  if (v == 0xFFFFFFFEu) t[0] = lds[(threadIdx.x + 1) & 255];
}

// the step's stores after the spin: `words` 16-byte stores per thread (non-temporal or plain)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void k_store(uint64_t* t, uint32_t* xcc, int spin, u32x4* out, int words) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  if (threadIdx.x == 0) {
    t[blockIdx.x] = t0;
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    xcc[blockIdx.x] = id & 0xFu;
  }
  uint32_t v = threadIdx.x;
  for (int i = 0; i < spin; ++i) v = v * 1664525u + 1013904223u;
  u32x4* o = out + (size_t)blockIdx.x * 256 * words;
  for (int k = 0; k < words; ++k) {
    const u32x4 q = {v, v + 1, v + 2, v + (uint32_t)k};
    if (NT) __builtin_nontemporal_store(q, o + k * 256 + threadIdx.x);
    else o[k * 256 + threadIdx.x] = q;
  }
}

static const int nb = 1024, reps = 40;

static void report(const char* name, uint64_t* t, uint32_t* x) {
  (void)hipDeviceSynchronize();
  std::vector<uint64_t> ht(nb * reps);
  std::vector<uint32_t> hx(nb * reps);
  (void)hipMemcpy(ht.data(), t, nb * 8 * reps, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hx.data(), x, nb * 4 * reps, hipMemcpyDeviceToHost);
  double mean_xcc[8] = {0};
  int cnt[8] = {0};
  for (int r = 10; r < reps; ++r) {
    const uint64_t* tr = ht.data() + r * nb;
    const uint32_t* xr = hx.data() + r * nb;
    const uint64_t t0 = *std::min_element(tr, tr + nb);
    for (int b = 0; b < nb; ++b) {
      mean_xcc[xr[b] & 7u] += (double)(tr[b] - t0);
      cnt[xr[b] & 7u]++;
    }
  }
  printf("%-28s", name);
  for (int k = 0; k < 8; ++k) printf(" %5.2f", mean_xcc[k] / cnt[k] * 0.01);
  printf("  (mean start by XCC, us)\n");
}

int main(int argc, char** argv) {
  const int spin = 1500;
  uint64_t* t;
  uint32_t* x;
  (void)hipMalloc(&t, nb * 8 * reps);
  (void)hipMalloc(&x, nb * 4 * reps);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  u32x4* out;
  (void)hipMalloc(&out, (size_t)nb * 256 * 6 * 16);  // 24 MB: the step's obs bytes
  Big b{};
  b.spin = spin;
  for (int pass = 0; pass < 2; ++pass) {
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_small, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, spin);
    report("16 B args, stream", t, x);
    for (int r = 0; r < reps; ++r) {
      b.t = t + r * nb;
      b.xcc = x + r * nb;
      hipLaunchKernelGGL(k_big<false>, dim3(nb), dim3(256), 14336, s, b);
    }
    report("672 B args, stream", t, x);
    for (int r = 0; r < reps; ++r) {
      b.t = t + r * nb;
      b.xcc = x + r * nb;
      hipLaunchKernelGGL(k_big<true>, dim3(nb), dim3(256), 14336, s, b);
    }
    report("672 B args, 128 VGPR, stream", t, x);
    // the same as a graph (the bench's launch)
    hipGraph_t graph;
    hipGraphExec_t exec;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int r = 0; r < reps; ++r) {
      b.t = t + r * nb;
      b.xcc = x + r * nb;
      hipLaunchKernelGGL(k_big<false>, dim3(nb), dim3(256), 14336, s, b);
    }
    (void)hipStreamEndCapture(s, &graph);
    (void)hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphLaunch(exec, s);
    report("672 B args, graph", t, x);
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_small, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, spin);
    (void)hipStreamEndCapture(s, &graph);
    (void)hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphLaunch(exec, s);
    report("16 B args, graph", t, x);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_store<true>, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, spin, out, 6);
    report("24 MB nt stores, stream", t, x);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_store<false>, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, spin, out, 6);
    report("24 MB plain stores, stream", t, x);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_store<false>, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, spin, out, 1);
    report("4 MB plain stores, stream", t, x);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_store<false>, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, 40, out, 6);
    report("24 MB plain, short spin", t, x);
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_store<true>, dim3(nb), dim3(256), 14336, s, t + r * nb, x + r * nb, 40, out, 6);
    report("24 MB nt, short spin", t, x);
  }
  return 0;
}
