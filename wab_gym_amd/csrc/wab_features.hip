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

#include "wab_feat.h"

namespace wab {

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
// of H bytes (S == H; the default 11x11), table-driven (wab_feat.h).  The kernel is
// store-bound (1796 B written per env against 363 read), so what matters is how soon the
// stores start: no per-bit loops.
//   prologue  per-cell tables in LDS (wab_feat.h)
//   phase 1   16-byte loads, 16 bytes -> one 16-bit LDS store (no zeroing, no atomics)
//   phase 2   lane = env, one plane per wave: W0 wolves, W1 bushes (+ standing on a bush),
//             W2 scalars and view mask
//   phase 3   feature bits -> float32, 16-byte stores (without restrict_view, the whole lines
//             of the all-zero view-mask blocks go out first, while the phase-1 loads are in
//             flight, and phase 3 skips them)
__device__ __forceinline__ uint32_t feat_in_words(const FeatParams& p) { return ((uint32_t)(64 * p.OB + 31) >> 5) + 4u; }
__device__ __forceinline__ uint32_t feat_ob_words(const FeatParams& p) { return ((uint32_t)(64 * p.F + 31) >> 5) + 4u; }

__global__ __launch_bounds__(256) void wab_featurize_small_kernel(FeatParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t a = (feat_in_words(p) + 3u) & ~3u, b = (feat_ob_words(p) + 3u) & ~3u;
  uint32_t* in = lds;
  uint32_t* ob = lds + a;
  const FeatTables t = feat_tables_at(lds + a + b, p.md);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const int n_active = (int)min((int64_t)64, p.B - g0);
  const uint32_t WH = (uint32_t)(p.W * p.H), md = (uint32_t)p.md;
  const int64_t g = g0 + lane;
  const bool active = lane < n_active;

  // phase 1 loads first (every one in flight before anything waits), then the scalars
  const uint32_t nbytes = (uint32_t)n_active * (uint32_t)p.OB;
  const uint8_t* src = p.planes + (size_t)g0 * p.OB;
  constexpr int kLoads = 6;  // 64 * 384 B = 1536 chunks of 16 B <= 6 per thread
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
  // while the loads are in flight (issued after them, so no wait on a load waits for these):
  // the all-zero view-mask lines of the rows (wab_feat.h)
  const bool zero_views = p.kind == 0 && !p.restrict_view;
  if (zero_views) view_zero_lines(p.out + (size_t)g0 * p.F, (uint32_t)p.F, 0u, (uint32_t)n_active, tid, 256);
  // prologue: zero the feature bits and the tables, then build the tables
  for (uint32_t i = tid; i < b + feat_tables_words(p.md); i += 256) lds[a + i] = 0u;
  __syncthreads();
  feat_tables_build(t, p.W, p.H, p.md, tid, 256);
  {  // phase 1: one 16-bit unit per 16 obs bytes
    uint16_t* in16 = reinterpret_cast<uint16_t*>(in);
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
      const uint32_t u = (uint32_t)tid + 256u * k;
      if (u < full) {
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // byte != 0 -> its bit 0 (OR-fold within the byte), then the four flags to bits 0..3
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
    if (p.kind == 0) {
      if (wave <= 1) {  // W0 wolves, W1 bushes
        uint32_t near, second;
        int counts[4];
        plane_features(t, p.md, stream_get128(in, ebit + (uint32_t)wave * WH, WH), near, second, counts);
        emit_plane(ob, at, wave, p.md, near, second, counts);
      } else if (wave == 2) {
        const uint32_t sb_bit = ebit + WH + (md / 2u) * (uint32_t)p.S + md / 2u;  // :742
        const uint32_t* vm = p.view121[role == 1u ? 1 : 0];
        emit_scalars(ob, at, p.md, p.turns_empty, (in[sb_bit >> 5] >> (sb_bit & 31u)) & 1u, ft, role, status,
                     p.restrict_view != 0, m_make(vm[0], vm[1], vm[2], vm[3]));
      }
    } else {  // SuperBasicObservationWrapper: nearest bush in Discrete(md), food, role, status
      if (wave == 1) {
        uint32_t near, second;
        int counts[4];
        plane_features(t, p.md, stream_get128(in, ebit + WH, WH), near, second, counts);
#pragma unroll
        for (int k = 0; k < 4; ++k) fset(ob, at + (uint32_t)k * md + ((near >> (8 * k)) & 0xFFu));
      } else if (wave == 2) {
        uint32_t o = at + 4u * md;
        fset(ob, o + ft);
        o += (uint32_t)p.turns_empty + 1u;
        fset(ob, o + role);
        o += 2u;
        fset(ob, o + status);
      }
    }
  }
  __syncthreads();
  // phase 3: bits -> float32 (F * 64 floats per block, 16-byte aligned)
  if (zero_views)
    store_rows_skip_views(ob, p.out + (size_t)g0 * p.F, (uint32_t)n_active * (uint32_t)p.F, (uint32_t)p.F, tid, 256);
  else
    store_feature_bits(ob, p.out + (size_t)g0 * p.F, (uint32_t)n_active * (uint32_t)p.F, tid, 256);
}

// actor_critic.finish_episode returns (actor_critic.py:139-143): R_t = r_t + gamma R_{t+1},
// restarted after every done_t.  The scan is a serial chain in t, so each thread first issues
// the loads of a whole chunk of kReturnsChunk steps (registers), then runs the chain; VEC
// consecutive envs per thread (VEC independent chains, VEC-wide reward and done loads), VEC
// chosen by the host so that the grid still gives every SIMD a wave (B = 65536: VEC 1, 1024
// 64-thread workgroups).  Double accumulation (the reference's Python floats), no contraction
// (-ffp-contract=off), float32 out.  `tab` holds only the rewards whose float32 is not their
// double (wab_discounted_returns_exact; 0.1, 1.1 and -0.9 at the defaults): every other
// float32 reward converts to its exact double as is.
constexpr int kReturnsChunk = 32;

template <int VEC, int NE>
__global__ __launch_bounds__(64) void wab_returns_kernel(const float* __restrict__ reward,
                                                         const uint8_t* __restrict__ done, int32_t T, int64_t B,
                                                         double gamma, const float* __restrict__ bootstrap,
                                                         float* __restrict__ out, RewardTable tab) {
  const int64_t b = ((int64_t)blockIdx.x * 64 + threadIdx.x) * VEC;
  if (b >= B) return;
  // the NE table entries (the host pads to NE with copies of entry 0) in registers: a select
  // on a scalar-register operand would first copy it to a vector register, per use
  uint32_t tkey[NE > 0 ? NE : 1];
  double tval[NE > 0 ? NE : 1];
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    tkey[k] = tab.f32[k];
    tval[k] = tab.f64[k];
    opaque(tkey[k]);
    opaque(tval[k]);
  }
  double R[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) R[v] = bootstrap ? (double)bootstrap[b + v] : 0.0;
  for (int32_t hi = T - 1; hi >= 0; hi -= kReturnsChunk) {
    const int n = hi + 1 < kReturnsChunk ? hi + 1 : kReturnsChunk;  // steps hi, hi-1, .., hi-n+1
    float rf[kReturnsChunk][VEC];
    uint32_t dn[kReturnsChunk];
    // every load unconditional (a step past the segment's start re-reads step 0, unused): a
    // load under `if (j < n)` becomes a branch with its own wait, one round trip per step
#pragma unroll
    for (int j = 0; j < kReturnsChunk; ++j) {
      const int64_t i = (int64_t)(hi - j > 0 ? hi - j : 0) * B + b;
      if constexpr (VEC == 4) {
        const float4 r4 = *reinterpret_cast<const float4*>(reward + i);
        rf[j][0] = r4.x; rf[j][1] = r4.y; rf[j][2] = r4.z; rf[j][3] = r4.w;
        dn[j] = *reinterpret_cast<const uint32_t*>(done + i);
      } else if constexpr (VEC == 2) {
        const float2 r2 = *reinterpret_cast<const float2*>(reward + i);
        rf[j][0] = r2.x; rf[j][1] = r2.y;
        dn[j] = *reinterpret_cast<const uint16_t*>(done + i);
      } else {
        rf[j][0] = reward[i];
        dn[j] = done[i];
      }
    }
#pragma unroll
    for (int j = 0; j < kReturnsChunk; ++j) {
      if (j < n) {
        float o[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          if ((dn[j] >> (8 * v)) & 0xFFu) R[v] = 0.0;
          // the step's exact double reward when the table has it (the env's own rewards),
          // else the float32 as given
          double r = (double)rf[j][v];
#pragma unroll
          for (int k = 0; k < NE; ++k)
            if (__float_as_uint(rf[j][v]) == tkey[k]) r = tval[k];
          R[v] = r + gamma * R[v];  // (no contraction: -ffp-contract=off, the reference's op order)
          o[v] = (float)R[v];
        }
        const int64_t i = (int64_t)(hi - j) * B + b;
        if constexpr (VEC == 4)
          *reinterpret_cast<float4*>(out + i) = make_float4(o[0], o[1], o[2], o[3]);
        else if constexpr (VEC == 2)
          *reinterpret_cast<float2*>(out + i) = make_float2(o[0], o[1]);
        else
          out[i] = o[0];
      }
    }
  }
}

template __global__ void wab_returns_kernel<1, 0>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<1, 1>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<1, 2>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<1, 3>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<1, 4>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<1, 8>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<2, 0>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<2, 1>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<2, 2>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<2, 3>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<2, 4>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<2, 8>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<4, 0>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<4, 1>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<4, 2>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<4, 3>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<4, 4>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);
template __global__ void wab_returns_kernel<4, 8>(const float* __restrict__, const uint8_t* __restrict__, int32_t,
    int64_t, double, const float* __restrict__, float* __restrict__, RewardTable);

}  // namespace wab
