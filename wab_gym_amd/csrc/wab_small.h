// wab_small.h — device helpers of the step kernels for small views (W*H <= 128 bits): 128-bit
// cell masks in two 64-bit registers, the LDS obs bit-stream, interleaved hash chains.
#pragma once

#include "wab_device.h"

namespace wab {

// 128-bit masks are only touched through these helpers: a dynamically indexed uint32_t[4]
// would be placed in scratch memory.

struct M128 {
  uint64_t lo, hi;
};
__device__ __forceinline__ M128 m_make(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  return M128{(uint64_t)w0 | ((uint64_t)w1 << 32), (uint64_t)w2 | ((uint64_t)w3 << 32)};
}
__device__ __forceinline__ void m_set(M128& m, uint32_t c) {
  const uint64_t b = 1ull << (c & 63u);
  m.lo |= c < 64u ? b : 0ull;
  m.hi |= c < 64u ? 0ull : b;
}
__device__ __forceinline__ void m_clear(M128& m, uint32_t c) {
  const uint64_t b = 1ull << (c & 63u);
  m.lo &= c < 64u ? ~b : ~0ull;
  m.hi &= c < 64u ? ~0ull : ~b;
}
__device__ __forceinline__ bool m_test(const M128& m, uint32_t c) {
  return (((c < 64u ? m.lo : m.hi) >> (c & 63u)) & 1ull) != 0ull;
}
template <int K>
__device__ __forceinline__ uint32_t m_word(const M128& m) {
  return (uint32_t)((K >= 2 ? m.hi : m.lo) >> (32 * (K & 1)));
}
__device__ __forceinline__ M128 m_and(const M128& a, const M128& b) { return M128{a.lo & b.lo, a.hi & b.hi}; }
__device__ __forceinline__ M128 m_andn(const M128& a, const M128& b) { return M128{a.lo & ~b.lo, a.hi & ~b.hi}; }
__device__ __forceinline__ M128 m_or(const M128& a, const M128& b) { return M128{a.lo | b.lo, a.hi | b.hi}; }

// OR a plane (a mask with no bits at or above 128) into the stream at bit offset `at`: the
// plane shifted to its dword alignment is five dwords, ORed without branches (the stream has
// slack after its last plane)
__device__ __forceinline__ void stream_or128(uint32_t* s, uint32_t at, const M128& v) {
  const uint32_t sh = at & 31u, r = 32u - sh;
  const uint32_t w0 = m_word<0>(v), w1 = m_word<1>(v), w2 = m_word<2>(v), w3 = m_word<3>(v);
  uint32_t* d = s + (at >> 5);
  atomicOr(d, w0 << sh);
  atomicOr(d + 1, sh ? __builtin_amdgcn_alignbit(w1, w0, r) : w1);
  atomicOr(d + 2, sh ? __builtin_amdgcn_alignbit(w2, w1, r) : w2);
  atomicOr(d + 3, sh ? __builtin_amdgcn_alignbit(w3, w2, r) : w3);
  atomicOr(d + 4, sh ? w3 >> r : 0u);
}
// clear bits [at, at + n) of the stream
__device__ __forceinline__ void stream_clear(uint32_t* s, uint32_t at, uint32_t n) {
  for (uint32_t o = 0; o < n; o += 32u) {
    const uint32_t nb = min(32u, n - o), b = at + o;
    const uint64_t m = (uint64_t)(nb < 32u ? (1u << nb) - 1u : ~0u) << (b & 31u);
    atomicAnd(&s[b >> 5], ~(uint32_t)m);
    if (m >> 32) atomicAnd(&s[(b >> 5) + 1], ~(uint32_t)(m >> 32));
  }
}

// K independent fmix32 chains, written step-interleaved so that a single wave issues them
// back to back (ILP) instead of waiting on each dependent result
template <int K>
__device__ __forceinline__ void fmix32xk(uint32_t h[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) h[k] ^= h[k] >> 16;
#pragma unroll
  for (int k = 0; k < K; ++k) h[k] *= 0x85EBCA6Bu;
#pragma unroll
  for (int k = 0; k < K; ++k) h[k] ^= h[k] >> 13;
#pragma unroll
  for (int k = 0; k < K; ++k) h[k] *= 0xC2B2AE35u;
#pragma unroll
  for (int k = 0; k < K; ++k) h[k] ^= h[k] >> 16;
}
__device__ __forceinline__ void fmix32x4(uint32_t h[4]) { fmix32xk<4>(h); }

__device__ __forceinline__ M128 view_mask_of(const Params& p, int role) {
  const bool g = role == 1;
  const M128 lo = m_make(sreg(p.view121[0][0]), sreg(p.view121[0][1]), sreg(p.view121[0][2]), sreg(p.view121[0][3]));
  const M128 hi = m_make(sreg(p.view121[1][0]), sreg(p.view121[1][1]), sreg(p.view121[1][2]), sreg(p.view121[1][3]));
  return M128{sel64(g, hi.lo, lo.lo), sel64(g, hi.hi, lo.hi)};
}


}  // namespace wab
