// wab_device.h — device helpers shared by the step kernels (wab_step.hip, wab_step_q4.hip):
// the keyed RNG (definition: oracle/keyed_rng.py), threshold search, packed tiles, LDS bit ops.
#pragma once

#include <hip/hip_runtime.h>

#include "wab_params.h"

namespace wab {

enum : uint32_t {
  SITE_BUSH = 1, SITE_SPAWN = 2, SITE_DESPAWN = 3, SITE_START_FOOD = 4, SITE_START_ROLE = 5, SITE_GAP = 6
};
enum { MODE_STEP = 0, MODE_RESET = 1 };
enum { DIR_STAY = 0, DIR_RIGHT = 1, DIR_LEFT = 2, DIR_UP = 3, DIR_DOWN = 4 };

// ------------------------------------------------------------------------ keyed RNG
// Definition: oracle/keyed_rng.py (the golden vectors were generated under it).
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// episode key = mix64(env_key ^ episode), env_key = mix64(mix64(seed + golden) ^ env)
__device__ __forceinline__ uint64_t env_key(uint64_t seed, uint64_t env) {
  return mix64(mix64(seed + 0x9E3779B97F4A7C15ull) ^ env);
}
__device__ __forceinline__ uint64_t episode_key(uint64_t seed, uint64_t env, uint64_t ep) {
  return mix64(env_key(seed, env) ^ ep);
}

__device__ __forceinline__ uint32_t make_ts(uint32_t site, uint32_t k, int32_t turn) {
  return (site & 0xFu) | ((k & 0xFFu) << 4) | (((uint32_t)turn & 0xFFFFFu) << 12);
}

__device__ __forceinline__ uint32_t draw_lo21(uint32_t h1, uint32_t ts, uint32_t b0) {
  const uint32_t rot = (ts << 16) | (ts >> 16);
  return fmix32(h1 ^ rot ^ b0 ^ 0x9E3779B9u) >> 11;
}

// U >= T for U = hi << 21 | lo21 and T = th << 21 | tl; the low half is only hashed when
// the high 32 bits tie (probability 2^-32)
__device__ __forceinline__ bool U_ge(uint32_t h1, uint32_t hi, uint32_t ts, uint32_t b0, uint32_t th,
                                     uint32_t tl) {
  if (hi != th) return hi > th;
  return draw_lo21(h1, ts, b0) >= tl;
}

__device__ __forceinline__ uint64_t draw_U(uint32_t xy, uint32_t ts, uint32_t b0, uint32_t b1) {
  const uint32_t h1 = fmix32(xy ^ b0);
  const uint32_t hi = fmix32(h1 ^ ts ^ b1);
  return ((uint64_t)hi << 21) | draw_lo21(h1, ts, b0);
}

// number of thresholds T_k <= U: the reference's round(u**power * max) (wab_env.py:631-635);
// `thr` is the LDS copy of the sorted table (n <= 255).  16-ary search in two levels of
// independent LDS reads (two round trips instead of log2(n) dependent ones).
__device__ __forceinline__ int bush_value(const uint64_t* thr, int n, uint64_t U) {
  const int step = (n + 15) >> 4;  // <= 16
  int c = 0;
#pragma unroll
  for (int i = 1; i < 16; ++i) {
    const int k = i * step - 1;
    c += (k < n && thr[k] <= U) ? 1 : 0;
  }
  const int base = c * step;
  int c2 = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = base + j;
    c2 += (j < step && k < n && thr[k] <= U) ? 1 : 0;
  }
  return base + c2;
}

// The same count from a float guess: c = round(n * u^power) is within 1 of the count for any
// draw (the guess is off by ~1e-4 at power 100), so four thresholds pin it.  With T_0 = 0 and
// T_k = +inf for k > n, "T_k <= U" holds exactly for k <= count, so T_{c-1} <= U < T_{c+2}
// proves count in [c-1, c+1], and then count = c - 2 + #{k in c-1..c+1 : T_k <= U}.  A lane
// whose guess misses that bracket falls back to the search above: the result is exact
// whatever the guess.  Layout (bush_thr_pads): thr[k - 1] = T_k, thr[-1] = 0, thr[n] =
// thr[n + 1] = ~0.
__device__ __forceinline__ int bush_value_fast(const uint64_t* thr, int n, uint64_t U, float power) {
  if (n <= 0) return 0;
  const float u = (float)(uint32_t)(U >> 21) * 0x1p-32f;
  const float guess = (float)n * __builtin_amdgcn_exp2f(power * __builtin_amdgcn_logf(u));
  const int c = min(max((int)__builtin_rintf(guess), 1), n);  // (log2(0) = -inf: guess 0)
  const uint64_t t0 = thr[c - 2], t1 = thr[c - 1], t2 = thr[c], t3 = thr[c + 1];
  int v = c - 2 + (t0 <= U ? 1 : 0) + (t1 <= U ? 1 : 0) + (t2 <= U ? 1 : 0);
  if (!(t0 <= U && t3 > U)) v = bush_value(thr, n, U);
  return v;
}

// ------------------------------------------------------------------------ keyed spawn sets
// The wolves spawning among n tiles in a canonical order (the ring table, or view cells
// c = i*H + j), iid Bernoulli(q) drawn by geometric gaps (oracle/keyed_rng.py spawn_hits):
// the k-th draw (site 6, "tile" (k, 0)) gives G = #{g in 1..m : U < gap[g]} misses before
// the next hit among the m tiles left.  The first draw ends the set at once iff U < gap[n]
// (th, tl: gap[n] split), which at the default q = 0.0005 is 97.6 % of the ring draws: one
// hash chain per env-step instead of one per ring tile.  `gap` (LDS or global) is only read
// on a hit; hit(index) is called for each hit tile, ascending.
__device__ __forceinline__ int gap_count(const uint64_t* gap, int m, uint64_t U) {
  int g = 0;  // gap[0] = 2^53 > U; gap is non-increasing
  for (int s = m > 0 ? 1 << (31 - __builtin_clz((uint32_t)m)) : 0; s; s >>= 1)
    if (g + s <= m && U < gap[g + s]) g += s;
  return g;
}

// The same count from a float guess: gap[g] ~ (1 - q)^g 2^53, so G = floor(log2(u) / log2(1 - q))
// but within one of it near a boundary; gap[g] > U >= gap[g + 1] (one LDS round trip) proves
// G = g, else the search decides.  inv_l2 = 1 / log2(1 - q) (< 0; q > 0 on this path).
__device__ __forceinline__ int gap_count_fast(const uint64_t* gap, int m, uint64_t U, float inv_l2) {
  const float u = (float)(uint32_t)(U >> 21) * 0x1p-32f;
  const float gf = __builtin_amdgcn_logf(u) * inv_l2;  // u = 0: +inf
  const int g = gf >= (float)m ? m : (int)gf;
  const uint64_t a = gap[g], b = gap[min(g + 1, m)];
  if (U < a && (g == m || U >= b)) return g;
  return gap_count(gap, m, U);
}

// The tiles are taken in chunks of kGapChunk, each its own sequence (draw k of chunk c: "tile"
// (k, c)), so that `gap` has kGapChunk + 1 entries; (thf, tlf) is gap[kGapChunk] split, (th, tl)
// gap[m] of the last chunk.
template <typename Hit>
__device__ __forceinline__ void spawn_hits(const uint64_t* gap, int n, uint32_t thf, uint32_t tlf, uint32_t th,
                                           uint32_t tl, float inv_l2, int32_t turn, uint32_t b0, uint32_t b1,
                                           Hit&& hit) {
  const uint32_t ts = make_ts(SITE_GAP, 0, turn);
  for (int c = 0, base = 0; base < n; ++c, base += kGapChunk) {  // (uniform)
    const int m = min(kGapChunk, n - base);
    const bool last = base + kGapChunk >= n;
    const uint32_t h1 = fmix32(xy_pack(0, c) ^ b0);
    const uint32_t hi = fmix32(h1 ^ ts ^ b1);
    if (!U_ge(h1, hi, ts, b0, last ? th : thf, last ? tl : tlf)) continue;
    uint64_t U = ((uint64_t)hi << 21) | draw_lo21(h1, ts, b0);
    int pos = 0;
    for (uint32_t k = 1;; ++k) {
      const int G = gap_count_fast(gap, m - pos, U, inv_l2);
      if (G >= m - pos) break;
      pos += G;
      hit(base + pos);
      if (++pos >= m) break;
      U = draw_U(xy_pack((int32_t)k, c), ts, b0, b1);
    }
  }
}

// the pads of bush_value_fast's table around thr[0 .. n) (one lane)
__device__ __forceinline__ void bush_thr_pads(uint64_t* thr, int n) {
  thr[-1] = 0ull;
  thr[n] = ~0ull;
  thr[n + 1] = ~0ull;
}

// packed-tile add: both int16 halves wrap independently (v_pk_add_u16)
typedef unsigned short wab_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t xy_add(uint32_t a, uint32_t b) {
  wab_u16x2 va = __builtin_bit_cast(wab_u16x2, a), vb = __builtin_bit_cast(wab_u16x2, b);
  return __builtin_bit_cast(uint32_t, va + vb);
}

__device__ __forceinline__ uint32_t udiv(uint32_t x, uint32_t d, uint32_t magic) {
  uint32_t q = __umulhi(x, magic);
  const int32_t r = (int32_t)(x - q * d);
  if (r < 0) q -= 1; else if ((uint32_t)r >= d) q += 1;
  return q;
}

__device__ __forceinline__ void lds_set(uint32_t* s, uint32_t bit) { atomicOr(&s[bit >> 5], 1u << (bit & 31)); }

// OR the low `nbits` (<= 32) bits of v into the stream at bit offset `at`
__device__ __forceinline__ void lds_or_bits(uint32_t* s, uint32_t at, uint32_t v, uint32_t nbits) {
  if (nbits < 32) v &= (1u << nbits) - 1u;
  if (!v) return;
  const uint64_t m = (uint64_t)v << (at & 31);
  atomicOr(&s[at >> 5], (uint32_t)m);
  if (m >> 32) atomicOr(&s[(at >> 5) + 1], (uint32_t)(m >> 32));
}

// restrict_view: zero blind-spot cells of the three planes (mask_grid, wab_env.py:344-357)
__device__ __forceinline__ void apply_view_mask(const Params& p, uint32_t* s, uint32_t env_bit, int role) {
  const uint32_t* rows = p.mask_rows[role == 1 ? 1 : 0];
  for (int pl = 0; pl < 3; ++pl)
    for (int i = 0; i < 11; ++i) {
      const uint32_t base = env_bit + (uint32_t)(pl * p.W * p.S + i * p.S);
      const uint64_t m = (uint64_t)rows[i] << (base & 31);
      atomicAnd(&s[base >> 5], ~(uint32_t)m);
      if (m >> 32) atomicAnd(&s[(base >> 5) + 1], ~(uint32_t)(m >> 32));
    }
}

// 128-bit shifts of a W*H <= 128 bitmap held as two 64-bit halves
__device__ __forceinline__ void shl128(uint64_t& lo, uint64_t& hi, int n) {
  if (n >= 64) { hi = lo << (n - 64); lo = 0; }
  else if (n > 0) { hi = (hi << n) | (lo >> (64 - n)); lo <<= n; }
}
__device__ __forceinline__ void shr128(uint64_t& lo, uint64_t& hi, int n) {
  if (n >= 64) { lo = hi >> (n - 64); hi = 0; }
  else if (n > 0) { lo = (lo >> n) | (hi << (64 - n)); hi >>= n; }
}

// Pin a wave-uniform value (a kernel-argument field) to scalar registers.  A per-lane
// select between two kernel-argument fields otherwise compiles to a select of their
// addresses and a vector load from the kernarg segment, whose s_waitcnt vmcnt then also
// waits for every store the wave has in flight.
__device__ __forceinline__ uint32_t sreg(uint32_t v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ int32_t sreg(int32_t v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ double sreg(double v) {
  asm volatile("" : "+s"(v));
  return v;
}

// An opaque copy: whatever uses the value comes after this point.  Placed after a wave's last
// load, it keeps the compiler from folding the first uses of each loaded value (a +1, a
// mask) into the load's own block, where the wait for that load would stall the loads after
// it (one s_waitcnt for all of them instead of one per group).  After a load made on one
// path only, it also settles the wait there: the compiler otherwise treats the value as
// possibly in flight at every later use and waits with vmcnt(0), which also waits for every
// store the wave has issued since.
template <typename T>
__device__ __forceinline__ void opaque(T& v) {
  asm volatile("" : "+v"(v));
}

// A fresh copy of the kernel's parameter block, loaded from the kernel-argument segment
// behind an opaque pointer: the scalar loads of the fields a block of code uses then stay in
// that block.  (The kernel argument itself has every field loaded at the kernel's entry and,
// past the SGPR budget, spilled to VGPR lanes; a copy per wave branch and per phase keeps
// only what that branch uses live.)
__device__ __forceinline__ Params kernel_params(const Params& p0) {
#if __HIP_DEVICE_COMPILE__  // (the host pass only type-checks the kernel bodies)
  typedef const Params __attribute__((address_space(4))) KernargParams;
  KernargParams* pk = (KernargParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  return *pk;
#else
  return p0;
#endif
}

// Per-lane choice between two wave-uniform 64-bit values by masks: the compiler turns a
// plain ?: of two kernel-argument doubles into a scratch array indexed per lane.
__device__ __forceinline__ uint64_t sel64(bool c, uint64_t a, uint64_t b) {
  const uint64_t m = 0ull - (uint64_t)c;
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ double sel_f64(bool c, double a, double b) {
  return __longlong_as_double((long long)sel64(c, (uint64_t)__double_as_longlong(a), (uint64_t)__double_as_longlong(b)));
}

// The action table (wab_env.py:149-182: 0 up, 1 right, 2 down, 3 left, 4/5 role actions),
// decoded arithmetically: indexing the kernel-argument block with a per-lane value compiles
// to a vector load from the kernarg segment, a dependent memory round trip per step.
__device__ __forceinline__ void decode_action(const Params& p, int a, int& dx, int& dy, int& new_role) {
  dx = (a == 1) - (a == 3);
  dy = (a == 0) - (a == 2);
  const int32_t r4 = sreg(p.act_role[4]), r5 = sreg(p.act_role[5]);
  new_role = a == 4 ? r4 : a == 5 ? r5 : -1;
}

__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

// wab_counters.steps: one lane of workgroup 0 adds the batch size once per step launch (a
// no-return atomic: nothing waits for it)
__device__ __forceinline__ void count_steps(const Params& p) {
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&p.counters[CTR_STEPS], (unsigned long long)p.B);
}

// Hand-off of LDS data between two waves of one workgroup through an LDS flag, without a
// barrier: the producer's release store orders its earlier LDS writes before the flag, the
// consumer's acquire load its later LDS reads after it.  The producer always makes progress
// (it is in the same workgroup and waits on nothing), so the bound on the wait is only a hang
// guard: a wait that gives up is counted (CTR_HANDOFF_TIMEOUTS; the parity tests assert 0).
__device__ __forceinline__ void lds_publish(uint32_t* flag) {
  __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_await(const Params& p, const uint32_t* flag) {
  for (int spin = 0; spin < (1 << 20); ++spin) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) return;
    __builtin_amdgcn_s_sleep(1);
  }
  atomicAdd(&p.counters[CTR_HANDOFF_TIMEOUTS], 1ull);
}

// Workgroup barrier for LDS hand-offs only.  Waves of a block exchange data exclusively
// through LDS; __syncthreads() would also drain every outstanding global store
// (s_waitcnt vmcnt(0)) and put HBM write latency on the critical path of each phase.
// s_setprio takes an immediate: a wave-uniform run-time level through a branch
__device__ __forceinline__ void set_prio_dyn(uint32_t pr) {
  if (pr == 0u) __builtin_amdgcn_s_setprio(0);
  else if (pr == 1u) __builtin_amdgcn_s_setprio(1);
  else if (pr == 2u) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(3);
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// tile-table entry: world offset from the ostrich (int8, int8) and a bit index
__device__ __forceinline__ int tile_dx(uint32_t t) { return (int)(int8_t)(t & 0xFFu); }
__device__ __forceinline__ int tile_dy(uint32_t t) { return (int)(int8_t)((t >> 8) & 0xFFu); }
__device__ __forceinline__ uint32_t tile_bit(uint32_t t) { return t >> 16; }

}  // namespace wab
