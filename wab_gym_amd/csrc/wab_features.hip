// wab_features.hip — config-5 device kernels for gfx950: the PragmaticObsWrapper
// featurizer (+ gym 0.17 flatten) and the discounted-return scan of actor_critic.py.
//
// wab_featurize_kernel: one 256-thread workgroup per 64 envs; `kind` selects the wrapper
// (PragmaticObsWrapper, or SuperBasicObservationWrapper: nearest bush, food, role, status).
//   phase 1  all threads   16-byte coalesced loads of the block's obs chunk, 1 byte -> 1 bit
//                          into an LDS bit-stream (the inverse of the step kernel's phase F)
//   phase 2  wave 0        lane = env: walk the set bits of the wolf and bush planes in
//                          row-major order (np.where order, wab_env.py:770), nearest /
//                          second-nearest / per-direction counts, scalars, view mask ->
//                          feature bits (one-hot layout of gym's flatten)
//   phase 3  all threads   expand feature bits to float32 with 16-byte coalesced stores
#include <hip/hip_runtime.h>

#include "wab_small.h"

namespace wab {

__device__ __forceinline__ void fset(uint32_t* s, uint32_t bit) { atomicOr(&s[bit >> 5], 1u << (bit & 31)); }

// nearest / second nearest / direction counts of one plane (_get_nearest_things :763-810,
// _get_num_things_each_direction :812-824); plane bits [base, base + W*S) of stream s
__device__ void scan_plane(const FeatParams& p, const uint32_t* s, uint32_t base, int near[4],
                           int second[4], int counts[4]) {
  int shortest = p.md, second_d = p.md;
  int si0 = 0, si1 = 0, s20 = 0, s21 = 0;
  bool any = false;
  int cu = 0, cr = 0, cd = 0, cl = 0;
  const uint32_t n = (uint32_t)(p.W * p.S);
  for (uint32_t d = base >> 5; (d << 5) < base + n; ++d) {
    uint32_t bits = s[d];
    const uint32_t lo = d << 5;
    if (lo < base) bits &= ~0u << (base - lo);
    if (lo + 32 > base + n) bits &= (base + n - lo >= 32) ? ~0u : ((1u << (base + n - lo)) - 1u);
    while (bits) {
      const int b = __ffs(bits) - 1;
      bits &= bits - 1;
      const int idx = (int)(lo + b - base);
      const int r = idx / p.S, c = idx - (idx / p.S) * p.S;
      any = true;
      const int rr = r - p.H / 2, rc = c - p.W / 2;          // :779-780
      const int tx = abs(rr) + abs(rc);
      if (tx <= shortest) {                                  // :782-787
        second_d = shortest;
        s20 = si0; s21 = si1;
        shortest = tx;
        si0 = rr; si1 = rc;
      } else if (tx <= second_d) {                           // :788-791
        second_d = tx;
        s20 = rr; s21 = rc;
      }
      cu += r < p.H / 2;
      cr += c > p.W / 2;
      cd += r > p.H / 2;
      cl += c < p.W / 2;
    }
  }
  counts[0] = min(cu, 10); counts[1] = min(cr, 10); counts[2] = min(cd, 10); counts[3] = min(cl, 10);
  if (!any) {
    for (int k = 0; k < 4; ++k) near[k] = second[k] = 0;
    return;
  }
  const int md = p.md;
  auto enc = [md](int a, int b, int o[4]) {                  // :792-808
    const int up = a < 0 ? -a : 0, right = b > 0 ? b : 0, down = a > 0 ? a : 0, left = b < 0 ? -b : 0;
    o[0] = up ? md - up : 0;
    o[1] = right ? md - right : 0;
    o[2] = down ? md - down : 0;
    o[3] = left ? md - left : 0;
  };
  enc(si0, si1, near);
  enc(s20, s21, second);
}

__global__ __launch_bounds__(256) void wab_featurize_kernel(FeatParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr int NE = 64;
  const int tid = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * NE;
  const int n_active = (int)min((int64_t)NE, p.B - g0);
  const uint32_t inW = (uint32_t)(NE * p.OB + 31) >> 5;
  const uint32_t outW = (uint32_t)(NE * p.F + 31) >> 5;
  uint32_t* in = lds;
  uint32_t* ob = lds + ((inW + 3) & ~3u);
  for (uint32_t i = tid; i < ((inW + 3) & ~3u) + outW; i += 256) lds[i] = 0;
  __syncthreads();
  // phase 1: obs bytes -> bits
  {
    const uint32_t nbytes = (uint32_t)n_active * (uint32_t)p.OB;
    const uint8_t* src = p.planes + (size_t)g0 * p.OB;
    for (uint32_t o = (uint32_t)tid * 16u; o < nbytes; o += 256u * 16u) {
      uint32_t m = 0;
      if (o + 16u <= nbytes) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + o);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int q = 0; q < 4; ++q) m |= (((w[k] >> (8 * q)) & 0xFFu) ? 1u : 0u) << (4 * k + q);
      } else {
        for (uint32_t q = 0; o + q < nbytes && q < 16u; ++q) m |= (src[o + q] ? 1u : 0u) << q;
      }
      if (m) atomicOr(&in[o >> 5], m << (o & 31));
    }
  }
  __syncthreads();
  // phase 2: lane = env
  if (tid < n_active) {
    const int e = tid;
    const int64_t g = g0 + e;
    const uint32_t ebit = (uint32_t)e * (uint32_t)p.OB;
    const uint32_t plane = (uint32_t)(p.W * p.S);
    int nw[4], sw[4], cw[4], nb[4], sb[4], cb[4];
    uint32_t at = (uint32_t)e * (uint32_t)p.F;
    if (p.kind == 1) {  // (nearest bush, food, role, status); nearest bush in Discrete(md) (:906)
      scan_plane(p, in, ebit + plane, nb, sb, cb);
      for (int k = 0; k < 4; ++k) {
        fset(ob, at + (uint32_t)nb[k]);
        at += (uint32_t)p.md;
      }
      fset(ob, at + p.food_turns[g]);
      at += (uint32_t)(p.turns_empty + 1);
      fset(ob, at + p.role[g]);
      at += 2;
      fset(ob, at + p.status[g]);
    } else {
    scan_plane(p, in, ebit, nw, sw, cw);
    scan_plane(p, in, ebit + plane, nb, sb, cb);
    const int* groups[6] = {nw, sw, cw, nb, sb, cb};
    const int sizes[6] = {p.md + 1, p.md + 1, 11, p.md + 1, p.md + 1, 11};
    for (int q = 0; q < 6; ++q)
      for (int k = 0; k < 4; ++k) {
        fset(ob, at + (uint32_t)groups[q][k]);
        at += (uint32_t)sizes[q];
      }
    const uint32_t sb_bit = ebit + plane + (uint32_t)((p.md / 2) * p.S + p.md / 2);  // :742
    fset(ob, at + ((in[sb_bit >> 5] >> (sb_bit & 31)) & 1u));
    at += 2;
    fset(ob, at + p.food_turns[g]);
    at += (uint32_t)(p.turns_empty + 1);
    const int role = p.role[g];
    fset(ob, at + (uint32_t)role);
    at += 2;
    fset(ob, at + p.status[g]);
    at += 3;
    if (p.view_mask) {
      for (int k = 0; k < 121; ++k)
        if (p.view_mask[g * 121 + k]) fset(ob, at + (uint32_t)k);
    } else if (p.restrict_view) {                         // view_mask of _get_obs (:360-368)
      const uint32_t* rows = p.mask_rows[role == 1 ? 1 : 0];
      for (int i = 0; i < 11; ++i)
        for (int j = 0; j < 11; ++j)
          if ((rows[i] >> j) & 1u) fset(ob, at + (uint32_t)(i * 11 + j));
    }
    }
  }
  __syncthreads();
  // phase 3: bits -> float32, 16-byte stores
  {
    const uint32_t nf = (uint32_t)n_active * (uint32_t)p.F;
    float* dst = p.out + (size_t)g0 * p.F;
    for (uint32_t q = (uint32_t)tid * 4u; q < nf; q += 256u * 4u) {
      const uint32_t v = (ob[q >> 5] >> (q & 31)) & 0xFu;
      if (q + 4u <= nf) {
        float4 f;
        f.x = (v & 1u) ? 1.0f : 0.0f;
        f.y = (v & 2u) ? 1.0f : 0.0f;
        f.z = (v & 4u) ? 1.0f : 0.0f;
        f.w = (v & 8u) ? 1.0f : 0.0f;
        *reinterpret_cast<float4*>(dst + q) = f;
      } else {
        for (uint32_t k = 0; q + k < nf; ++k) dst[q + k] = ((v >> k) & 1u) ? 1.0f : 0.0f;
      }
    }
  }
}

// ------------------------------------------------------------------ small views (W*H <= 128)
// wab_featurize_small_kernel: the same features for views whose planes fit 128 bits in rows
// of H bytes (S == H; the default 11x11).  The kernel is store-bound (1796 B written per env
// against 363 read), so what matters is how soon the stores start: no per-bit loops.
//   prologue  per-cell tables in LDS: the packed encodings (up, right, down, left) of every
//             cell, the cells at each taxicab distance (ring masks), the direction-count masks
//   phase 1   16-byte loads, 16 bytes -> one 16-bit LDS store (no zeroing, no atomics)
//   phase 2   lane = env, one plane per wave: W0 wolves, W1 bushes (+ standing on a bush),
//             W2 scalars and view mask.  The scan of _get_nearest_things (:763-810) keeps the
//             top two of the set cells under (distance ascending, np.where index descending)
//             (a later cell at equal distance replaces the nearest, :782-791), so the nearest
//             is the highest set bit of the first non-empty ring and the second the next bit
//             of that ring or the highest of the next non-empty one; counts are popcounts
//   phase 3   feature bits -> float32, 16-byte stores
struct FeatLds {
  uint32_t* in;     // 64 envs x OB bits (+ 4 dwords of slack)
  uint32_t* ob;     // 64 envs x F bits (+ 4 dwords of slack)
  uint32_t* enc;    // [128] per cell: up | right << 8 | down << 16 | left << 24 (encoded values)
  uint4* ring;      // [md] cells at distance d
  uint4* cmask;     // [4] cells counted up, right, down, left (:812-824)
};

__device__ __forceinline__ uint32_t feat_in_words(const FeatParams& p) { return ((uint32_t)(64 * p.OB + 31) >> 5) + 4u; }
__device__ __forceinline__ uint32_t feat_ob_words(const FeatParams& p) { return ((uint32_t)(64 * p.F + 31) >> 5) + 4u; }

__device__ __forceinline__ FeatLds feat_lds(uint32_t* lds, const FeatParams& p) {
  FeatLds s;
  const uint32_t a = (feat_in_words(p) + 3u) & ~3u, b = (feat_ob_words(p) + 3u) & ~3u;
  s.in = lds;
  s.ob = lds + a;
  s.enc = lds + a + b;
  s.ring = reinterpret_cast<uint4*>(lds + a + b + 128);
  s.cmask = s.ring + p.md;
  return s;
}

// bits [at, at + n) of an LDS bit-stream (n <= 128) as a 128-bit mask
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

// nearest / second nearest (packed encodings) and the capped direction counts of plane P
__device__ __forceinline__ void plane_features(const FeatLds& s, int md, M128 P, uint32_t& near, uint32_t& second,
                                               int counts[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) counts[k] = min(m_popc(m_and(P, m_of(s.cmask[k]))), 10);
  int n1 = -1, n2 = -1;
  for (int d = 0; d < md; ++d) {
    if (__all(n2 >= 0 || (P.lo | P.hi) == 0ull)) break;  // (wave-uniform exit)
    const M128 r = m_of(s.ring[d]);
    M128 m = m_and(P, r);
    P = m_andn(P, r);
    const int t = m_top(m);
    if (n1 < 0) {
      if (t >= 0) {
        n1 = t;
        m_clear(m, (uint32_t)t);
        n2 = m_top(m);
      }
    } else if (n2 < 0) {
      n2 = t;
    }
  }
  near = n1 >= 0 ? s.enc[n1] : 0u;
  second = n2 >= 0 ? s.enc[n2] : 0u;
}

__global__ __launch_bounds__(256) void wab_featurize_small_kernel(FeatParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const FeatLds s = feat_lds(lds, p);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const int n_active = (int)min((int64_t)64, p.B - g0);
  const uint32_t WH = (uint32_t)(p.W * p.H), md = (uint32_t)p.md;
  const int64_t g = g0 + lane;
  const bool active = lane < n_active;

  // phase 1 loads first (every one in flight before anything waits), then the scalars
  const uint32_t nbytes = (uint32_t)n_active * (uint32_t)p.OB;
  const uint8_t* src = p.planes + (size_t)g0 * p.OB;
  constexpr int kLoads = 6;  // 64 * 363 B = 1452 chunks of 16 B <= 6 per thread
  uint4 v[kLoads];
  const uint32_t full = nbytes >> 4;
#pragma unroll
  for (int k = 0; k < kLoads; ++k) {
    const uint32_t u = (uint32_t)tid + 256u * k;
    v[k] = u < full ? reinterpret_cast<const uint4*>(src)[u] : make_uint4(0u, 0u, 0u, 0u);
  }
  uint32_t ft = 0, role = 0, status = 0;
  if (wave == 2 && active) {
    ft = p.food_turns[g];
    role = p.role[g];
    status = p.status[g];
  }
  // prologue: zero the feature bits and the masks, then the tables
  {
    const uint32_t a = (feat_in_words(p) + 3u) & ~3u, b = (feat_ob_words(p) + 3u) & ~3u;
    for (uint32_t i = tid; i < b + 128u + 4u * (md + 4u); i += 256) lds[a + i] = 0u;
  }
  __syncthreads();
  for (uint32_t c = tid; c < WH; c += 256) {
    const int r = (int)(c / (uint32_t)p.S), col = (int)(c % (uint32_t)p.S);
    const int rr = r - p.H / 2, rc = col - p.W / 2;  // :779-780
    const int up = rr < 0 ? -rr : 0, right = rc > 0 ? rc : 0, down = rr > 0 ? rr : 0, left = rc < 0 ? -rc : 0;
    const int m = p.md;  // encodings :792-808
    s.enc[c] = (uint32_t)(up ? m - up : 0) | ((uint32_t)(right ? m - right : 0) << 8) |
               ((uint32_t)(down ? m - down : 0) << 16) | ((uint32_t)(left ? m - left : 0) << 24);
    const uint32_t bit = 1u << (c & 31u), w = c >> 5;
    uint32_t* ring = reinterpret_cast<uint32_t*>(s.ring + (abs(rr) + abs(rc)));
    atomicOr(&ring[w], bit);
    uint32_t* cm = reinterpret_cast<uint32_t*>(s.cmask);
    if (r < p.H / 2) atomicOr(&cm[0 * 4 + w], bit);
    if (col > p.W / 2) atomicOr(&cm[1 * 4 + w], bit);
    if (r > p.H / 2) atomicOr(&cm[2 * 4 + w], bit);
    if (col < p.W / 2) atomicOr(&cm[3 * 4 + w], bit);
  }
  {  // phase 1: one 16-bit unit per 16 obs bytes
    uint16_t* in16 = reinterpret_cast<uint16_t*>(s.in);
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
      const uint32_t u = (uint32_t)tid + 256u * k;
      if (u < full) {
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // byte != 0 -> bit: OR-fold each byte into its low bit
          uint32_t x = w[q] | (w[q] >> 4);
          x |= x >> 2;
          x |= x >> 1;
          x &= 0x01010101u;
          m |= (((x * 0x01020408u) >> 24) & 0xFu) << (4 * q);  // byte k -> bit k
        }
        in16[u] = (uint16_t)m;
      }
    }
    for (uint32_t u = full + (uint32_t)tid; u < (nbytes + 15u) >> 4; u += 256) {  // a partial last unit
      uint32_t m = 0;
      for (uint32_t q = 0; q < 16u && 16u * u + q < nbytes; ++q) m |= (src[16u * u + q] ? 1u : 0u) << q;
      in16[u] = (uint16_t)m;
    }
  }
  __syncthreads();
  // phase 2
  if (active) {
    const uint32_t ebit = (uint32_t)lane * (uint32_t)p.OB;
    const uint32_t at = (uint32_t)lane * (uint32_t)p.F;
    const uint32_t M1 = md + 1u;
    if (p.kind == 0) {
      if (wave <= 1) {  // W0 wolves, W1 bushes: near, second, counts
        uint32_t near, second;
        int counts[4];
        plane_features(s, p.md, stream_get128(s.in, ebit + (uint32_t)wave * WH, WH), near, second, counts);
        const uint32_t base = at + (uint32_t)wave * (8u * M1 + 44u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          fset(s.ob, base + (uint32_t)k * M1 + ((near >> (8 * k)) & 0xFFu));
          fset(s.ob, base + (4u + (uint32_t)k) * M1 + ((second >> (8 * k)) & 0xFFu));
          fset(s.ob, base + 8u * M1 + 11u * (uint32_t)k + (uint32_t)counts[k]);
        }
        if (wave == 1) {  // standing_on_bush = bushes[md//2, md//2] (:742)
          const uint32_t sb_bit = ebit + WH + (md / 2u) * (uint32_t)p.S + md / 2u;
          fset(s.ob, at + 16u * M1 + 88u + ((s.in[sb_bit >> 5] >> (sb_bit & 31u)) & 1u));
        }
      } else if (wave == 2) {
        uint32_t o = at + 16u * M1 + 88u + 2u;
        fset(s.ob, o + ft);
        o += (uint32_t)p.turns_empty + 1u;
        fset(s.ob, o + role);
        o += 2u;
        fset(s.ob, o + status);
        o += 3u;
        if (p.restrict_view) {  // view_mask of _get_obs (:360-368), 121 bits
          const uint32_t* vm = p.view121[role == 1u ? 1 : 0];
          stream_or128(s.ob, o, m_make(vm[0], vm[1], vm[2], vm[3]));
        }
      }
    } else {  // SuperBasicObservationWrapper: nearest bush in Discrete(md), food, role, status
      if (wave == 1) {
        uint32_t near, second;
        int counts[4];
        plane_features(s, p.md, stream_get128(s.in, ebit + WH, WH), near, second, counts);
#pragma unroll
        for (int k = 0; k < 4; ++k) fset(s.ob, at + (uint32_t)k * md + ((near >> (8 * k)) & 0xFFu));
      } else if (wave == 2) {
        uint32_t o = at + 4u * md;
        fset(s.ob, o + ft);
        o += (uint32_t)p.turns_empty + 1u;
        fset(s.ob, o + role);
        o += 2u;
        fset(s.ob, o + status);
      }
    }
  }
  __syncthreads();
  // phase 3: bits -> float32, 16-byte stores (F * 64 floats per block, 16-byte aligned)
  {
    const uint32_t nf = (uint32_t)n_active * (uint32_t)p.F;
    float* dst = p.out + (size_t)g0 * p.F;
    const uint32_t nq = nf >> 2;
    for (uint32_t u = (uint32_t)tid; u < nq; u += 256u) {
      const uint32_t q = 4u * u;
      const uint32_t b = (s.ob[q >> 5] >> (q & 31u)) & 0xFu;
      float4 f;
      f.x = (b & 1u) ? 1.0f : 0.0f;
      f.y = (b & 2u) ? 1.0f : 0.0f;
      f.z = (b & 4u) ? 1.0f : 0.0f;
      f.w = (b & 8u) ? 1.0f : 0.0f;
      reinterpret_cast<float4*>(dst)[u] = f;
    }
    for (uint32_t q = 4u * nq + (uint32_t)tid; q < nf; q += 256u)
      dst[q] = ((s.ob[q >> 5] >> (q & 31u)) & 1u) ? 1.0f : 0.0f;
  }
}

// actor_critic.finish_episode returns (actor_critic.py:139-143), one thread per env
__global__ __launch_bounds__(256) void wab_returns_kernel(const float* reward, const uint8_t* done, int32_t T,
                                                          int64_t B, double gamma, const float* bootstrap,
                                                          float* out) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  double R = bootstrap ? (double)bootstrap[b] : 0.0;
  for (int32_t t = T - 1; t >= 0; --t) {
    const int64_t i = (int64_t)t * B + b;
    if (done[i]) R = 0.0;
    R = (double)reward[i] + gamma * R;
    out[i] = (float)R;
  }
}

}  // namespace wab
