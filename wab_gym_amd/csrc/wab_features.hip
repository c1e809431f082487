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

#include "wab_params.h"

namespace wab {

struct FeatParams {
  int32_t W, H, S, OB, md, F, turns_empty, restrict_view;
  int32_t kind;  // 0 PragmaticObsWrapper (:726-824), 1 SuperBasicObservationWrapper (:900-927)
  int64_t B;
  uint32_t mask_rows[2][11];
  const uint8_t* planes;
  const uint8_t* food_turns;
  const uint8_t* role;
  const uint8_t* status;
  const uint8_t* view_mask;  // [B][11][11] or null (derive from role)
  float* out;                // [B][F]
};

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
