// wab_egocentric.hip — WolvesAndBushesEnvEgoCentric / ...EgocentricJustBushes observation
// (wab_env.py:930-979): `_get_bush_proximities` (:652-667) for every env of the batch.
//
// For each of the 5 squares the next action can reach (up, right, down, left, stay;
// generate_potential_actions :71-84) the reference takes the taxicab distance d to the
// nearest food>0 bush of its whole bush table — every tile that was ever in view this
// episode, not just the current view — and reports clip(Q - d, 0, Q), Q = W//2 + H//2 + 1;
// with no food>0 bush anywhere it reports Q for all five (the Series([0]*5) branch :664).
//
// Only bushes with d < Q matter, i.e. tiles within taxicab Q of the ostrich, so one wave
// per env works on a (2Q+1)^2 window around it (Q <= 31: one 64-bit row mask per lane):
//   1. seen window: OR the W x H view box of every earlier path position into per-row
//      masks (lane = row), then the current box;
//   2. bush bits: the keyed bush draw (the step kernel's generate_bushes) for the seen tiles
//      of the Q-diamond, minus eaten-log tiles with no berries left;
//   3. per candidate square, nearest set bit of each row (ctz/clz) + row offset, wave min.
// "Is there any food>0 bush at all" needs the whole seen set: a running count of food>0
// tiles ever seen (new tiles of the current box each turn, stored with the path entry)
// minus the emptied eaten-log entries (misc_ndep) answers it exactly.
#include <hip/hip_runtime.h>

#include "wab_device.h"
#include "wab_params.h"

namespace wab {

__device__ __forceinline__ uint64_t span_bits(int lo, int hi) {  // bits lo..hi, 0 <= lo <= hi <= 62
  return ((2ull << (hi - lo)) - 1ull) << lo;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

__global__ __launch_bounds__(64) void wab_egocentric_kernel(EgoParams p) {
  __shared__ uint64_t prev_rows[64], seen_rows[64];
  __shared__ uint32_t bush_rows[128];
  const int64_t g = blockIdx.x;
  const int lane = threadIdx.x;
  if (p.mask && !p.mask[g]) return;
  const uint4 h = p.hdr[g];
  if (h.w == 0xFFFFFFFFu) return;  // never reset: no observation exists
  const int Q = p.Q, cw = p.cw, ch = p.ch;
  const int turn = (int)h.y;
  const int ox = xy_x(h.x), oy = xy_y(h.x);
  const int dy_l = lane - Q;  // this lane's window row

  // 1. tiles seen before this turn (path[0 .. turn-1]) and now
  uint64_t prev = 0;
  const int n_prev = min(turn, p.cap);
  bool stale = turn > p.cap;
  uint32_t cnt_prev = 0;
  for (int k0 = 0; k0 < n_prev; k0 += 64) {
    uint4 e = make_uint4(0u, 0u, 0u, 0u);
    const bool have = k0 + lane < n_prev;
    if (have) e = p.path[(size_t)(k0 + lane) * p.B + g];
    stale |= have && e.z != h.w;
    const int m = min(64, n_prev - k0);
    for (int j = 0; j < m; ++j) {
      const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)e.x, j);
      const int rx = xy_x(t) - ox, ry = xy_y(t) - oy;
      if (abs(ry - dy_l) <= ch && rx - cw <= Q && rx + cw >= -Q)
        prev |= span_bits(max(rx - cw, -Q) + Q, min(rx + cw, Q) + Q);
    }
    if (k0 + 64 >= n_prev) cnt_prev = (uint32_t)__builtin_amdgcn_readlane((int)e.y, n_prev - 1 - k0);
  }
  const bool row_ok = lane <= 2 * Q;
  if (!row_ok) prev = 0;
  const uint64_t seen = prev | ((row_ok && abs(dy_l) <= ch) ? span_bits(Q - cw, Q + cw) : 0ull);
  prev_rows[lane] = prev;
  seen_rows[lane] = seen;
  bush_rows[2 * lane] = 0u;
  bush_rows[2 * lane + 1] = 0u;
  __syncthreads();

  // 2. food>0 tiles of the seen diamond (generate_n_bush_values: value >= 1 <=> U >= T_1)
  const uint64_t ek = episode_key(p.seed, (uint64_t)(p.env_base + g), (uint64_t)h.w);
  const uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
  const uint32_t ts = make_ts(SITE_BUSH, 0, 0), hb = ts ^ b1;
  uint32_t fresh = 0;
  for (int t = lane; t < p.n_diamond; t += 64) {
    const uint32_t d = p.diamond[t];
    const int dx = tile_dx(d), dy = tile_dy(d);
    const int r = dy + Q, c = dx + Q;
    if ((seen_rows[r] >> c) & 1ull) {
      const uint32_t h1 = fmix32(xy_pack(ox + dx, oy + dy) ^ b0);
      const uint32_t hi = fmix32(h1 ^ hb);
      if (U_ge(h1, hi, ts, b0, p.bush_th, p.bush_tl)) {
        atomicOr(&bush_rows[2 * r + (c >> 5)], 1u << (c & 31));
        fresh += !((prev_rows[r] >> c) & 1ull) && abs(dx) <= cw && abs(dy) <= ch;
      }
    }
  }
  const uint32_t live_seen = cnt_prev + wave_sum(fresh);
  __syncthreads();
  // eaten-log tiles with no berries left are not bushes any more (food > 0 filter :654)
  const uint32_t ne = misc_ne(h.z);
  for (uint32_t e = (uint32_t)lane; e < ne && e < (uint32_t)p.eaten_cap; e += 64u) {
    if (p.eaten_rem[(size_t)e * p.B + g] == 0) {
      const uint32_t t = p.eaten_xy[(size_t)e * p.B + g];
      const int rx = xy_x(t) - ox, ry = xy_y(t) - oy;
      if (abs(rx) <= Q && abs(ry) <= Q)
        atomicAnd(&bush_rows[2 * (ry + Q) + ((rx + Q) >> 5)], ~(1u << ((rx + Q) & 31)));
    }
  }
  __syncthreads();

  // 3. nearest bush per candidate square
  const uint64_t m = row_ok ? ((uint64_t)bush_rows[2 * lane] | ((uint64_t)bush_rows[2 * lane + 1] << 32)) : 0ull;
  int dist[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int cx = (k == 1) - (k == 3), cy = (k == 0) - (k == 2);
    const int c = cx + Q;
    int hd = 1 << 20;
    const uint64_t right = m >> c, left = m << (63 - c);
    if (right) hd = __builtin_ctzll(right);
    if (left) hd = min(hd, __builtin_clzll(left));
    dist[k] = wave_min(m ? abs(dy_l - cy) + hd : 1 << 20);
  }
  const bool any_live = live_seen > misc_ndep(h.z);
  if (lane < 5) {
    int d = dist[0];
#pragma unroll
    for (int k = 1; k < 5; ++k) d = lane == k ? dist[k] : d;
    const int v = any_live ? (d < Q ? Q - d : 0) : Q;
    p.out[(size_t)g * 5 + lane] = (uint8_t)v;
  }
  const bool wave_stale = __any(stale);
  if (lane == 0) {
    if (turn < p.cap) p.path[(size_t)turn * p.B + g] = make_uint4(h.x, live_seen, h.w, 0u);
    if (wave_stale || turn >= p.cap) atomicAdd(&p.counters[CTR_EGO_MISSING], 1ull);
  }
}

}  // namespace wab
