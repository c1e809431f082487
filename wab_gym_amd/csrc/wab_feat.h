// wab_feat.h — the PragmaticObsWrapper features (wab_env.py:726-824, flattened as
// actor_critic.py:188 does) of views whose planes fit 128 bits, from an LDS obs bit-stream.
// Shared by the standalone featurizer (wab_featurize_small_kernel, wab_features.hip) and the
// fused step + features path of the small-view step kernel (wab_step_small.hip).
//
// The scan of _get_nearest_things (:763-810) keeps the top two of the set cells under
// (distance ascending, np.where index descending): a later cell at equal distance replaces
// the nearest (:782-791).  So the nearest is the highest set bit of the first non-empty ring
// of cells at one distance, the second the next bit of that ring or the highest of the next
// non-empty ring; the direction counts (:812-824) are popcounts of four fixed cell masks.
// Per-cell tables (built once per workgroup in LDS): the packed encodings of every cell, the
// cells at each distance, the four count masks.
#pragma once

#include "wab_small.h"

namespace wab {

__device__ __forceinline__ void fset(uint32_t* s, uint32_t bit) { atomicOr(&s[bit >> 5], 1u << (bit & 31)); }

// feature count of PragmaticObsWrapper + flatten (wab_feature_dim): 16 (md+1) + 88 + 2 +
// (turns_empty + 1) + 2 + 3 + 121
__host__ __device__ inline int pragmatic_dim(int md, int turns_empty) { return 16 * (md + 1) + 88 + 2 + (turns_empty + 1) + 2 + 3 + 121; }

struct FeatTables {
  uint32_t* enc;   // [128] per cell: up | right << 8 | down << 16 | left << 24 (encoded values)
  uint4* ring;     // [md] cells at distance d
  uint4* cmask;    // [4] cells counted up, right, down, left
};

// LDS dwords of the tables
__host__ __device__ inline uint32_t feat_tables_words(int md) { return 128u + 4u * ((uint32_t)md + 4u); }

__device__ __forceinline__ FeatTables feat_tables_at(uint32_t* lds, int md) {
  FeatTables t;
  t.enc = lds;
  t.ring = reinterpret_cast<uint4*>(lds + 128);
  t.cmask = t.ring + md;
  return t;
}

// Build the tables (their LDS must be zero) with threads [0, nthreads); rows of S = H cells.
// Rows are measured from H//2 and columns from W//2 (:779-780); the host only picks this
// path when every such distance is below md (always on square views).
__device__ __forceinline__ void feat_tables_build(const FeatTables& t, int W, int H, int md, int tid, int nthreads) {
  for (int c = tid; c < W * H; c += nthreads) {
    const int r = c / H, col = c - (c / H) * H;
    const int rr = r - H / 2, rc = col - W / 2;
    const int up = rr < 0 ? -rr : 0, right = rc > 0 ? rc : 0, down = rr > 0 ? rr : 0, left = rc < 0 ? -rc : 0;
    t.enc[c] = (uint32_t)(up ? md - up : 0) | ((uint32_t)(right ? md - right : 0) << 8) |
               ((uint32_t)(down ? md - down : 0) << 16) | ((uint32_t)(left ? md - left : 0) << 24);  // :792-808
    const uint32_t bit = 1u << (c & 31), w = (uint32_t)c >> 5;
    atomicOr(reinterpret_cast<uint32_t*>(t.ring + (abs(rr) + abs(rc))) + w, bit);
    uint32_t* cm = reinterpret_cast<uint32_t*>(t.cmask);
    if (r < H / 2) atomicOr(&cm[0 * 4 + w], bit);
    if (col > W / 2) atomicOr(&cm[1 * 4 + w], bit);
    if (r > H / 2) atomicOr(&cm[2 * 4 + w], bit);
    if (col < W / 2) atomicOr(&cm[3 * 4 + w], bit);
  }
}

// bits [at, at + n) of an LDS bit-stream (n <= 128, four dwords of slack after it)
__device__ __forceinline__ M128 stream_get128(const uint32_t* s, uint32_t at, uint32_t n) {
  const uint32_t* d = s + (at >> 5);
  const uint32_t sh = at & 31u;
  const uint32_t w0 = d[0], w1 = d[1], w2 = d[2], w3 = d[3], w4 = d[4];
  M128 m = m_make(__builtin_amdgcn_alignbit(w1, w0, sh), __builtin_amdgcn_alignbit(w2, w1, sh),
                  __builtin_amdgcn_alignbit(w3, w2, sh), __builtin_amdgcn_alignbit(w4, w3, sh));
  if (n < 128u) {
    if (n >= 64u) m.hi &= (1ull << (n - 64u)) - 1ull;
    else { m.hi = 0ull; m.lo &= (1ull << n) - 1ull; }
  }
  return m;
}

__device__ __forceinline__ int m_top(const M128& m) {
  return m.hi ? 127 - (int)__clzll((long long)m.hi) : (m.lo ? 63 - (int)__clzll((long long)m.lo) : -1);
}
__device__ __forceinline__ M128 m_of(const uint4& v) { return m_make(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ int m_popc(const M128& m) { return __popcll(m.lo) + __popcll(m.hi); }

// nearest / second nearest (packed encodings, 0 when absent) and the capped direction
// counts of plane P
__device__ __forceinline__ void plane_features(const FeatTables& t, int md, M128 P, uint32_t& near, uint32_t& second,
                                               int counts[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) counts[k] = min(m_popc(m_and(P, m_of(t.cmask[k]))), 10);
  int n1 = -1, n2 = -1;
  for (int d = 0; d < md; ++d) {
    if (__all(n2 >= 0 || (P.lo | P.hi) == 0ull)) break;  // (wave-uniform exit)
    const M128 r = m_of(t.ring[d]);
    M128 m = m_and(P, r);
    P = m_andn(P, r);
    const int top = m_top(m);
    if (n1 < 0) {
      if (top >= 0) {
        n1 = top;
        m_clear(m, (uint32_t)top);
        n2 = m_top(m);
      }
    } else if (n2 < 0) {
      n2 = top;
    }
  }
  near = n1 >= 0 ? t.enc[n1] : 0u;
  second = n2 >= 0 ? t.enc[n2] : 0u;
}

// the split of plane_features over waves (the fused rollout): the capped direction counts alone
__device__ __forceinline__ void plane_counts(const FeatTables& t, const M128& P, int counts[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) counts[k] = min(m_popc(m_and(P, m_of(t.cmask[k]))), 10);
}

// ... and nearest / second nearest alone
__device__ __forceinline__ void plane_nearest(const FeatTables& t, int md, M128 P, uint32_t& near, uint32_t& second) {
  int n1 = -1, n2 = -1;
  for (int d = 0; d < md; ++d) {
    if (__all(n2 >= 0 || (P.lo | P.hi) == 0ull)) break;  // (wave-uniform exit)
    const M128 r = m_of(t.ring[d]);
    M128 m = m_and(P, r);
    P = m_andn(P, r);
    const int top = m_top(m);
    if (n1 < 0) {
      if (top >= 0) {
        n1 = top;
        m_clear(m, (uint32_t)top);
        n2 = m_top(m);
      }
    } else if (n2 < 0) {
      n2 = top;
    }
  }
  near = n1 >= 0 ? t.enc[n1] : 0u;
  second = n2 >= 0 ? t.enc[n2] : 0u;
}

// emit_plane's parts: the 8 nearest / second-nearest features, the 4 count features
__device__ __forceinline__ void emit_nearest(uint32_t* ob, uint32_t at, int plane, int md, uint32_t near,
                                             uint32_t second) {
  const uint32_t M1 = (uint32_t)md + 1u;
  const uint32_t base = at + (uint32_t)plane * (8u * M1 + 44u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fset(ob, base + (uint32_t)k * M1 + ((near >> (8 * k)) & 0xFFu));
    fset(ob, base + (4u + (uint32_t)k) * M1 + ((second >> (8 * k)) & 0xFFu));
  }
}

__device__ __forceinline__ void emit_counts(uint32_t* ob, uint32_t at, int plane, int md, const int counts[4]) {
  const uint32_t M1 = (uint32_t)md + 1u;
  const uint32_t base = at + (uint32_t)plane * (8u * M1 + 44u);
#pragma unroll
  for (int k = 0; k < 4; ++k) fset(ob, base + 8u * M1 + 11u * (uint32_t)k + (uint32_t)counts[k]);
}

// one plane's 12 one-hot features (plane 0 wolves, 1 bushes) of the env whose row starts at
// feature bit `at`
__device__ __forceinline__ void emit_plane(uint32_t* ob, uint32_t at, int plane, int md, uint32_t near,
                                           uint32_t second, const int counts[4]) {
  const uint32_t M1 = (uint32_t)md + 1u;
  const uint32_t base = at + (uint32_t)plane * (8u * M1 + 44u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fset(ob, base + (uint32_t)k * M1 + ((near >> (8 * k)) & 0xFFu));
    fset(ob, base + (4u + (uint32_t)k) * M1 + ((second >> (8 * k)) & 0xFFu));
    fset(ob, base + 8u * M1 + 11u * (uint32_t)k + (uint32_t)counts[k]);
  }
}

// standing_on_bush (bushes[md//2, md//2], :742), food turns, role, status, view mask
__device__ __forceinline__ void emit_scalars(uint32_t* ob, uint32_t at, int md, int turns_empty, uint32_t standing,
                                             uint32_t ft, uint32_t role, uint32_t status, bool restrict_view,
                                             const M128& vm) {
  uint32_t o = at + 16u * ((uint32_t)md + 1u) + 88u;
  fset(ob, o + standing);
  o += 2u;
  fset(ob, o + ft);
  o += (uint32_t)turns_empty + 1u;
  fset(ob, o + role);
  o += 2u;
  fset(ob, o + status);
  o += 3u;
  if (restrict_view) stream_or128(ob, o, vm);  // view_mask of _get_obs (:360-368), 121 bits
}

// feature bits [0, nf) -> float32 at out (16-byte aligned), 16-byte stores: thread t writes
// float4s u = t + nthreads * i (consecutive lanes, consecutive 16 bytes), i.e. the nibbles at
// bit 4 (t & 7) of dwords (t >> 3) + (nthreads / 8) i: one LDS read and four bit-field
// extracts and conversions per float4 (nthreads a multiple of 8)
// four float4s in flight per thread (one or two measured no better: 24.2-24.5 us per C5 step)
constexpr int kFeatStoreUnroll = 4;

__device__ __forceinline__ void nt_store_f4(const float4& f, float4* dst) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const f32x4 v = {f.x, f.y, f.z, f.w};
#ifndef WAB_FEAT_NT  // (tuning A/B: 0 = plain feature stores)
#define WAB_FEAT_NT 1
#endif
  if (WAB_FEAT_NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
  else *reinterpret_cast<f32x4*>(dst) = v;
}

// (NT: non-temporal stores)
template <bool NT = false>
__device__ __forceinline__ void store_feature_bits(const uint32_t* ob, float* out, uint32_t nf, int tid, int nthreads) {
  const uint32_t nq = nf >> 2, sh = 4u * ((uint32_t)tid & 7u), step = (uint32_t)nthreads >> 3;
  const uint32_t* src = ob + ((uint32_t)tid >> 3);
  float4* dst = reinterpret_cast<float4*>(out) + tid;
  const uint32_t n_i = nq > (uint32_t)tid ? (nq - (uint32_t)tid + (uint32_t)nthreads - 1u) / (uint32_t)nthreads : 0u;
#pragma unroll kFeatStoreUnroll
  for (uint32_t i = 0; i < n_i; ++i) {
    const uint32_t w = src[step * i];
    float4 f;
    f.x = (float)__builtin_amdgcn_ubfe(w, sh, 1u);
    f.y = (float)__builtin_amdgcn_ubfe(w, sh + 1u, 1u);
    f.z = (float)__builtin_amdgcn_ubfe(w, sh + 2u, 1u);
    f.w = (float)__builtin_amdgcn_ubfe(w, sh + 3u, 1u);
    if (NT) nt_store_f4(f, dst + (size_t)nthreads * i);
    else dst[(size_t)nthreads * i] = f;
  }
  for (uint32_t q = 4u * nq + (uint32_t)tid; q < nf; q += (uint32_t)nthreads)
    out[q] = ((ob[q >> 5] >> (q & 31u)) & 1u) ? 1.0f : 0.0f;
}

// ---- the view-mask lines.  Without restrict_view the view-mask block (the last 121 floats of
// a row) is all zeros whatever the obs: the whole 128-byte lines inside those blocks (~20 % of
// the row bytes) can be stored before anything is computed, and the final store skips them.
// Only whole lines: a line written in two parts at different times costs far more than its
// bytes (measured).
struct ViewLines {
  uint32_t delta;  // the group's first float modulo 128 bytes (line-space origin)
  uint32_t F;      // floats per row
  uint32_t vb;     // first byte of the view block within a row
};

__device__ __forceinline__ ViewLines view_lines(const float* out, uint32_t F) {
  ViewLines v;
  v.delta = (uint32_t)reinterpret_cast<uintptr_t>(out) & 127u;
  v.F = F;
  v.vb = 4u * (F - 121u);
  return v;
}

// the whole lines [first, end) (line space) inside row e's view block
__device__ __forceinline__ void row_view_lines(const ViewLines& v, uint32_t e, uint32_t& first, uint32_t& end) {
  const uint32_t row = v.delta + 4u * v.F * e;
  first = (row + v.vb + 127u) >> 7;
  end = (row + 4u * v.F) >> 7;
}

// zeros to the whole view-block lines of rows [e0, e0 + n_rows) of the group at out
__device__ __forceinline__ void view_zero_lines(float* out, uint32_t F, uint32_t e0, uint32_t n_rows, int t, int nt) {
  const ViewLines v = view_lines(out, F);
  constexpr uint32_t kPer = 32;  // chunk slots per row: <= 3 whole lines of 8 chunks in 484 bytes
  for (uint32_t u = (uint32_t)t; u < n_rows * kPer; u += (uint32_t)nt) {
    const uint32_t e = e0 + u / kPer, c = u % kPer;
    uint32_t first, end;
    row_view_lines(v, e, first, end);
    if (first * 8u + c < end * 8u)
      *reinterpret_cast<float4*>(reinterpret_cast<char*>(out) + (first * 128u + 16u * c - v.delta)) =
          make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

// store_feature_bits without the chunks in the whole view-block lines (view_zero_lines)
template <bool NT = false>
__device__ __forceinline__ void store_rows_skip_views(const uint32_t* ob, float* out, uint32_t nf, uint32_t F, int tid,
                                                      int nthreads) {
  const ViewLines v = view_lines(out, F);
  const uint32_t nq = nf >> 2, sh = 4u * ((uint32_t)tid & 7u), step = (uint32_t)nthreads >> 3;
  const uint32_t* src = ob + ((uint32_t)tid >> 3);
  // chunk u = tid + nthreads i starts at float 4u = e F + r (row e, offset r)
  uint32_t e = (4u * (uint32_t)tid) / F, r = 4u * (uint32_t)tid - e * F;
  const uint32_t adv = 4u * (uint32_t)nthreads, dq = adv / F, dr = adv - dq * F;
#pragma unroll kFeatStoreUnroll
  for (uint32_t i = 0, u = (uint32_t)tid; u < nq; ++i, u += (uint32_t)nthreads) {
    uint32_t first, end;
    row_view_lines(v, e, first, end);
    const uint32_t line = (v.delta + 16u * u) >> 7;
    if (line < first || line >= end) {
      const uint32_t w = src[step * i];
      float4 f;
      f.x = (float)__builtin_amdgcn_ubfe(w, sh, 1u);
      f.y = (float)__builtin_amdgcn_ubfe(w, sh + 1u, 1u);
      f.z = (float)__builtin_amdgcn_ubfe(w, sh + 2u, 1u);
      f.w = (float)__builtin_amdgcn_ubfe(w, sh + 3u, 1u);
      if (NT) nt_store_f4(f, reinterpret_cast<float4*>(out) + u);
      else reinterpret_cast<float4*>(out)[u] = f;
    }
    e += dq;
    r += dr;
    if (r >= F) {
      r -= F;
      e += 1u;
    }
  }
  for (uint32_t q = 4u * nq + (uint32_t)tid; q < nf; q += (uint32_t)nthreads)
    out[q] = ((ob[q >> 5] >> (q & 31u)) & 1u) ? 1.0f : 0.0f;
}

}  // namespace wab
