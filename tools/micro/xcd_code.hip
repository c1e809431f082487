// Microbenchmark: does code size or the SGPR allocation delay the workgroups of XCDs 4-7 at
// kernel entry, as seen in the small step kernel (profiles/r02_xcd/)?  1024 workgroups x 256
// threads, 14 KB LDS (the step kernel's grid).  Each records s_memrealtime as its first
// instruction (entry) and after its work (end), plus its XCC_ID.  Variants:
//   base        a few dozen instructions (the earlier xcd_start.hip shape)
//   dead<N>     + N never-executed instructions (code size only)
//   sgpr        + a 104-SGPR allocation (inline-asm clobbers; the step kernel uses 106)
//   dead+sgpr   both
//   path<N>     N straight-line VALU instructions executed after the entry stamp (the i-cache
//               streams the path: a wave of the step kernel executes ~2-3 k instructions)
// Back-to-back launches in a graph (the bench's shape); per XCC: mean entry and mean end
// relative to the launch's first entry (us, 100 MHz clock).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

struct Args {
  uint64_t* t;  // [nb][2] entry, end
  uint32_t* xcc;
  int spin;
};

#define SGPR_CLOBBER                                                                                          \
  asm volatile("" ::: "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "s8", "s9", "s10", "s11", "s12", "s13",  \
               "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", \
               "s28", "s29", "s30", "s31", "s32", "s33", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41", \
               "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", \
               "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", \
               "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", \
               "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", \
               "s98", "s99", "s100", "s101")

template <int DEAD, bool SGPR, int PATH>
__global__ __launch_bounds__(256) void k_var(Args a) {
  uint64_t t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  extern __shared__ uint32_t lds[];
  uint32_t v = threadIdx.x;
  if constexpr (PATH > 0) {
    asm volatile(".rept %1\n\tv_add_u32 %0, %0, %0\n\t.endr" : "+v"(v) : "n"(PATH));
  }
  for (int i = 0; i < a.spin; ++i) v = v * 1664525u + 1013904223u;
  if constexpr (DEAD > 0) {
    if (a.spin < 0) asm volatile(".rept %1\n\tv_xor_b32 %0, %0, %0\n\t.endr" : "+v"(v) : "n"(DEAD));
  }
  if constexpr (SGPR) SGPR_CLOBBER;
  uint64_t t1;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (threadIdx.x == 0) {
    a.t[2 * blockIdx.x] = t0;
    a.t[2 * blockIdx.x + 1] = t1;
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    a.xcc[blockIdx.x] = id & 0xFu;
  }
  if (v == 0xFFFFFFFFu) lds[threadIdx.x] = v;
  if (v == 0xFFFFFFFEu) a.t[0] = lds[(threadIdx.x + 1) & 255];
}

static const int nb = 1024, reps = 40;

template <int DEAD, bool SGPR, int PATH>
static void run(const char* name, hipStream_t s, uint64_t* t, uint32_t* x, int spin) {
  hipGraph_t graph;
  hipGraphExec_t exec;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_var<DEAD, SGPR, PATH>), dim3(nb), dim3(256), 14336, s,
                       Args{t + (size_t)r * nb * 2, x + (size_t)r * nb, spin});
  (void)hipStreamEndCapture(s, &graph);
  (void)hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  for (int it = 0; it < 3; ++it) (void)hipGraphLaunch(exec, s);
  (void)hipStreamSynchronize(s);
  std::vector<uint64_t> ht((size_t)nb * 2 * reps);
  std::vector<uint32_t> hx((size_t)nb * reps);
  (void)hipMemcpy(ht.data(), t, ht.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost);
  double ent[8] = {0}, end[8] = {0};
  int cnt[8] = {0};
  double span = 0;
  for (int r = 10; r < reps; ++r) {
    const uint64_t* tr = ht.data() + (size_t)r * nb * 2;
    const uint32_t* xr = hx.data() + (size_t)r * nb;
    uint64_t t0 = ~0ull, t1 = 0;
    for (int b = 0; b < nb; ++b) { t0 = std::min(t0, tr[2 * b]); t1 = std::max(t1, tr[2 * b + 1]); }
    span += (double)(t1 - t0);
    for (int b = 0; b < nb; ++b) {
      ent[xr[b] & 7u] += (double)(tr[2 * b] - t0);
      end[xr[b] & 7u] += (double)(tr[2 * b + 1] - t0);
      cnt[xr[b] & 7u]++;
    }
  }
  printf("%-14s entry", name);
  for (int k = 0; k < 8; ++k) printf(" %5.2f", ent[k] / cnt[k] * 0.01);
  printf(" | end");
  for (int k = 0; k < 8; ++k) printf(" %5.2f", end[k] / cnt[k] * 0.01);
  printf(" | span %5.2f us\n", span / (reps - 10) * 0.01);
  (void)hipGraphExecDestroy(exec);
  (void)hipGraphDestroy(graph);
}

int main() {
  uint64_t* t;
  uint32_t* x;
  (void)hipMalloc(&t, (size_t)nb * 16 * reps);
  (void)hipMalloc(&x, (size_t)nb * 4 * reps);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  const int spin = 400;
  for (int pass = 0; pass < 2; ++pass) {
    run<0, false, 0>("base", s, t, x, spin);
    run<8192, false, 0>("dead8k", s, t, x, spin);
    run<0, true, 0>("sgpr", s, t, x, spin);
    run<8192, true, 0>("dead8k+sgpr", s, t, x, spin);
    run<0, false, 2048>("path2k", s, t, x, spin);
    run<0, false, 8192>("path8k", s, t, x, spin);
    run<8192, true, 2048>("all", s, t, x, spin);
  }
  return 0;
}
