// wab_step_wide.hip — the fused step (and reset) for wide views: W, H <= 32 with rows of
// S = 16 or 32 bytes, no restrict_view (the 31x31-in-32x32 configuration C3 of SURVEY.md).
//
// At 31x31 the step is dominated by its output: 2976 obs bytes per env against ~230 bytes
// of state, so the kernel is organised around getting the obs stores out early, from all
// four SIMDs, with the remaining hash work overlapping their drain.  One 256-thread
// workgroup serves 64 envs; each wave runs one lane per env:
//
//          W0 dynamics            W1 bushes               W2 ring         W3
//   P0     state + log loads,     bitmap rows (one dword  ring offsets,   ostrich grids
//          despawn, pursuit,      per row), scroll,       gap table ->    -> obs plane 2
//          kill, wolf grids of S  entering row/column     LDS, the spawn  (first half)
//          -> obs plane 0         draws, emptied tiles,   set; ostrich
//                                 ostrich-tile value      grids (second
//                                                         half)
//   -- B1 --  S (the obs snapshot) is complete
//   P1     eat, hunger, starve,   obs plane 1 (bushes)    obs plane 1
//          reward/done, scalars,
//          job list; obs plane 1
//   -- B2 --
//   P2     W0: spawns, state stores; all: post-eat bitmaps, terminal obs of done envs
//   (done envs: B3, reset draws by ballot, B4, new episodes, their obs and bitmaps)
//
// Every wave issues its share of the obs stores as soon as S is complete; nothing after
// that issues a vector load (vmcnt also counts stores: a load would wait for the drain).
// The obs of a done env is written twice (S, then the new episode's first obs) by the same
// thread, so the later store wins.  The view bitmaps live in LDS as one dword per row
// (bit j = column j): the move scrolls them by a row index (x moves) or a shift (y moves),
// the entering strip is one row word or one bit per row, and an obs chunk is 16 bits of
// one row expanded to 16 bytes; every store wave-instruction writes 1 KiB contiguous.
// Reset (MODE_RESET) is the done-env path alone, so the bitmap layout stays private to
// this kernel: env-major, 32 dwords per env (one 128-byte line; rows past W unused).
#include <hip/hip_runtime.h>

#include "wab_small.h"

namespace wab {

#ifdef WAB_STAMPS
#define WIDE_STAMP(slot)                                                                 \
  do {                                                                                   \
    if (lane == 0 && p.stamps)                                                           \
      p.stamps[(size_t)blockIdx.x * kStampStride + (slot)] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#else
#define WIDE_STAMP(slot) do {} while (0)
#endif

constexpr int kWideSpec = 8;  // wolf slots W0 loads with the state, before the count is known

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// header, action, the move (:252-258) and the episode key: read by every wave
struct WHead {
  bool active, valid_action;
  uint4 hdr;
  int32_t ox, oy, turn;
  int dir, role;
  uint32_t cpos, b0, b1;
  uint64_t kenv;
};

template <int MODE>
__device__ __forceinline__ WHead whead(const Params& p, int64_t g, bool active) {
  WHead h;
  h.active = active;
  h.hdr = make_uint4(0u, 0u, 0u, 0u);
  int a = 0;
  if (active) {
    h.hdr = p.hdr[g];
    if (MODE == MODE_STEP) a = (int)p.actions[g];
  }
  h.kenv = env_key(p.seed, (uint64_t)(p.env_base + g));  // overlaps the loads
  h.ox = xy_x(h.hdr.x);
  h.oy = xy_y(h.hdr.x);
  h.turn = (int32_t)h.hdr.y + 1;
  h.role = (int)misc_role(h.hdr.z);
  h.dir = DIR_STAY;
  h.valid_action = true;
  if (MODE == MODE_STEP) {
    h.valid_action = a >= 0 && a < p.n_actions;
    if (h.valid_action) {
      int dx, dy, nr;
      decode_action(p, a, dx, dy, nr);
      h.ox += dx;
      h.oy += dy;
      h.dir = dx > 0 ? DIR_RIGHT : dx < 0 ? DIR_LEFT : dy > 0 ? DIR_UP : dy < 0 ? DIR_DOWN : DIR_STAY;
      if (nr >= 0) h.role = nr;
    }
  }
  h.cpos = xy_pack(h.ox, h.oy);
  const uint64_t ek = mix64(h.kenv ^ (uint64_t)h.hdr.w);
  h.b0 = (uint32_t)ek;
  h.b1 = (uint32_t)(ek >> 32);
  return h;
}

// bush bits of the row (x moves: bit j) or column (y moves: bit i) that scrolled into view
// (generate_bushes :613-629); cell (i, j) is world (ox + cw - i, oy + ch - j)
__device__ __forceinline__ uint32_t strip_bits(const Params& p, const WHead& h) {
  if (h.dir == DIR_STAY) return 0u;
  const bool horiz = h.dir == DIR_RIGHT || h.dir == DIR_LEFT;
  const int n = horiz ? p.H : p.W;
  const int i0 = h.dir == DIR_LEFT ? p.W - 1 : 0, j0 = h.dir == DIR_DOWN ? p.H - 1 : 0;
  const uint32_t ts = make_ts(SITE_BUSH, 0, 0), hk = ts ^ h.b1;
  uint32_t bits = 0;
  for (int c = 0; c < n; c += 4) {
    uint32_t h1[4], hh[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = horiz ? i0 : c + k, j = horiz ? c + k : j0;
      h1[k] = xy_pack(h.ox + p.cw - i, h.oy + p.ch - j) ^ h.b0;
    }
    fmix32x4(h1);
#pragma unroll
    for (int k = 0; k < 4; ++k) hh[k] = h1[k] ^ hk;
    fmix32x4(hh);
    uint32_t hit = 0, tie = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hit |= (hh[k] > p.bush_th ? 1u : 0u) << k;
      tie |= (hh[k] == p.bush_th ? 1u : 0u) << k;
    }
    const uint32_t in = n - c >= 4 ? 0xFu : (1u << (n - c)) - 1u;
    if (tie & in) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (((tie >> k) & 1u) && draw_lo21(h1[k], ts, h.b0) >= p.bush_tl) hit |= 1u << k;
    }
    bits |= (hit & in) << c;
  }
  return bits;
}

// a wolf's tile after pursuit (:267-286): one axis step toward the ostrich, ties along x
__device__ __forceinline__ uint32_t pursue(const Params& p, const WHead& h, uint32_t w) {
  if (!p.wolves_can_move) return w;
  int wx = xy_x(w), wy = xy_y(w);
  const int ddx = h.ox - wx, ddy = h.oy - wy;
  const bool alongx = abs(ddx) >= abs(ddy);
  wx += alongx ? sgn(ddx) : 0;
  wy += alongx ? 0 : sgn(ddy);
  return xy_pack(wx, wy);
}

// The despawn draws (:262-264) of the wolves beyond the register slots, rows SLOTS..nw-1 (the
// rare path: a ring spawn found every register slot taken).  Each is keyed like the register
// ones: its tile, and its occurrence index among all wolves before it in row order, on their
// pre-despawn positions (`wr` = rows 0..SLOTS-1, `live0` their mask).  Returns the survivors,
// bit k - SLOTS.  Rows are re-read from HBM (one lane's loads, rarely more than a few).
template <int SLOTS>
__device__ __forceinline__ uint32_t spill_despawn(const Params& p, const WHead& h, int64_t g, int nw,
                                               const uint32_t (&wr)[SLOTS], uint32_t live0) {
  uint32_t keep = 0;
  for (int k = SLOTS; k < nw && k < 32 + SLOTS; ++k) {
    const uint32_t wk = p.wolves[(int64_t)k * p.B + g];
    uint32_t occ = 0;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) occ += (((live0 >> t) & 1u) && wr[t] == wk) ? 1u : 0u;
    for (int t = SLOTS; t < k; ++t) occ += p.wolves[(int64_t)t * p.B + g] == wk ? 1u : 0u;
    const uint32_t ts = make_ts(SITE_DESPAWN, occ, h.turn);
    const uint32_t h1 = fmix32(wk ^ h.b0);
    const uint32_t hi = fmix32(h1 ^ ts ^ h.b1);
    if (U_ge(h1, hi, ts, h.b0, p.keep_th, p.keep_tl)) keep |= 1u << (k - SLOTS);
  }
  return keep;
}

// dst[i] = src[i] for i < n by one wave, four independent loads per lane in flight at a time
// (a plain strided loop waits for each load before its LDS store)
template <typename T>
__device__ __forceinline__ void copy_to_lds(T* dst, const T* src, int n, int lane) {
  for (int i0 = 0; i0 < n; i0 += 256) {
    T v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = src[min(i0 + 64 * k + lane, n - 1)];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + 64 * k + lane < n) dst[i0 + 64 * k + lane] = v[k];
  }
}

// 16 cells of one row -> 16 bytes
#ifndef WAB_WIDE_OBS_NT  // (tuning A/B: 0 = plain obs stores)
#define WAB_WIDE_OBS_NT 1
#endif
__device__ __forceinline__ void wide_obs_store(u32x4 v, u32x4* dst) {
  if (WAB_WIDE_OBS_NT) __builtin_nontemporal_store(v, dst);
  else *dst = v;
}
__device__ __forceinline__ u32x4 expand16(uint32_t v) {
  u32x4 q;
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = __umul24((v >> (4 * k)) & 0xFu, 0x00204081u) & 0x01010101u;
  return q;
}

// obs chunk r (16 bytes) of env e: plane k (wolf, bush, ostrich), row i, half
__device__ __forceinline__ uint32_t chunk_bits(const Params& p, const uint32_t* bm, const uint32_t* wp, uint32_t e,
                                               uint32_t r) {
  const uint32_t CPR = (uint32_t)p.S >> 4, WC = (uint32_t)p.W * CPR;
  const uint32_t k = (r >= WC ? 1u : 0u) + (r >= 2u * WC ? 1u : 0u);
  const uint32_t r2 = r - k * WC;
  const uint32_t i = CPR == 2u ? r2 >> 1 : r2;
  const uint32_t half = CPR == 2u ? r2 & 1u : 0u;
  const uint32_t* rows = k == 0u ? wp : bm;
  uint32_t row = rows[e * kWidePitch + i];
  if (k == 2u) row = i == (uint32_t)p.cw ? 1u << p.ch : 0u;  // the ostrich grid: self only
  return (row >> (16u * half)) & 0xFFFFu;
}

// Obs chunks (16 bytes), one plane at a time, each from the wave(s) that can write it first.
// The ostrich grid (plane 2) is the same in every observation (the centre cell): W3 writes it
// from the start (obs_plane2).  The wolf grid of S (plane 0) is complete once W0 has moved
// the wolves, long before the bush bitmap: W0 writes it then, while W1 still builds S
// (obs_plane0).  The bush grid (plane 1) follows from the threads of waves 0-2 after B1
// (obs_plane1).  Plane-k chunk r < W*S/16 of env e is always written by the same thread —
// W0 lane (e*WC + r) % 64 for plane 0, thread (e*WC + r) % kObsThreads for plane 1 — also
// when a done env's new-episode obs later overwrites it (obs_env), so both stores come from
// one thread in program order.
constexpr uint32_t kObsThreads = 192;

// plain stores: measured faster than non-temporal ones for this pattern
__device__ __forceinline__ void store16(const Params&, uint8_t* out, uint32_t q, const u32x4& v) {
  reinterpret_cast<u32x4*>(out)[q] = v;
}

// 16 bits of row chunk r (< WC) of one plane's rows
__device__ __forceinline__ uint32_t row_chunk(const uint32_t* rows, uint32_t CPR, uint32_t r) {
  const uint32_t i = CPR == 2u ? r >> 1 : r, half = CPR == 2u ? r & 1u : 0u;
  return (rows[i] >> (16u * half)) & 0xFFFFu;
}

// chunks [n * part0 / 8, n * part1 / 8) of the group's ostrich grids (in 64-chunk steps)
__device__ __forceinline__ void obs_plane2(const Params& p, uint8_t* out, uint32_t n_active, int lane, uint32_t part0 = 0,
                                           uint32_t part1 = 8) {
  const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4, WC = (uint32_t)p.W * CPR;
  const uint32_t n = n_active * WC;
  const uint32_t c0 = ((n * part0 / 8u) & ~63u) + (uint32_t)lane, c1 = part1 >= 8u ? n : (n * part1 / 8u) & ~63u;
  uint32_t e = 0, r = c0;
  while (r >= WC) { r -= WC; ++e; }
  for (uint32_t c = c0; c < c1; c += 64u) {
    const uint32_t i = CPR == 2u ? r >> 1 : r, half = CPR == 2u ? r & 1u : 0u;
    const uint32_t row = i == (uint32_t)p.cw ? 1u << p.ch : 0u;
    store16(p, out, e * CPE + 2u * WC + r, expand16((row >> (16u * half)) & 0xFFFFu));
    r += 64u;
    while (r >= WC) { r -= WC; ++e; }
  }
}

// plane k (0: wolf rows `rows` = wp, by the 64 lanes of W0; 1: bush rows = bm, by threads
// [0, kObsThreads)) of every env of the group
template <int K>
__device__ __forceinline__ void obs_plane(const Params& p, const uint32_t* rows, uint8_t* out, uint32_t n_active,
                                          int tid) {
  constexpr uint32_t NT = K == 0 ? 64u : kObsThreads;
  const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4, WC = (uint32_t)p.W * CPR;
  const uint32_t n = n_active * WC;
  uint32_t e = 0, r = (uint32_t)tid;
  while (r >= WC) { r -= WC; ++e; }
  for (uint32_t c = (uint32_t)tid; c < n; c += NT) {
    store16(p, out, e * CPE + (uint32_t)K * WC + r, expand16(row_chunk(rows + e * kWidePitch, CPR, r)));
    r += NT;
    while (r >= WC) { r -= WC; ++e; }
  }
}

// planes 0, 1 of one env, same thread mapping as obs_plane<0> and obs_plane<1>
__device__ __forceinline__ void obs_env(const Params& p, const uint32_t* bm, const uint32_t* wp, uint8_t* out,
                                        uint32_t e, int tid) {
  const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4, WC = (uint32_t)p.W * CPR;
  const uint32_t base = e * WC;
  if (tid < 64)
    for (uint32_t r = ((uint32_t)tid + 64u - base % 64u) % 64u; r < WC; r += 64u)
      store16(p, out, e * CPE + r, expand16(row_chunk(wp + e * kWidePitch, CPR, r)));
  if ((uint32_t)tid < kObsThreads)
    for (uint32_t r = ((uint32_t)tid + kObsThreads - base % kObsThreads) % kObsThreads; r < WC; r += kObsThreads)
      store16(p, out, e * CPE + WC + r, expand16(row_chunk(bm + e * kWidePitch, CPR, r)));
}

// all three planes of one env (terminal observations)
__device__ __forceinline__ void obs_env_all(const Params& p, const uint32_t* bm, const uint32_t* wp, uint8_t* out,
                                            uint32_t e, int tid) {
  const uint32_t CPE = (uint32_t)p.OB >> 4;
  for (uint32_t r = (uint32_t)tid; r < CPE; r += 256u) store16(p, out, e * CPE + r, expand16(chunk_bits(p, bm, wp, e, r)));
}

}  // namespace

template <int MODE, int SLOTS>
__global__ __launch_bounds__(256) void wab_step_wide(Params p0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const Params p = kernel_params(p0);  // (re-read per wave branch and phase below)
  const WideLayout L = wide_layout(p);
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  if (g0 >= p.B) return;  // (uniform over the workgroup)
#ifdef WAB_STAMPS
  if (threadIdx.x == 0 && p.stamps) {  // kernel entry (slot 32) and the XCD (slot 33)
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    p.stamps[(size_t)blockIdx.x * kStampStride + 32] = __builtin_amdgcn_s_memrealtime();
    p.stamps[(size_t)blockIdx.x * kStampStride + 33] = xcc & 0xFu;
  }
#endif
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int n_active = (int)min((int64_t)64, p.B - g0);
  const int64_t g = g0 + lane;
  const bool active = lane < n_active;
  uint32_t* bm = lds + L.bm;
  uint32_t* wp = lds + L.wp;
  uint32_t* spawn = lds + L.spawn;
  uint32_t* ring = lds + L.ring;
  uint64_t* gap = reinterpret_cast<uint64_t*>(lds + L.gap);  // (MODE_STEP; resets read p.gap)
  uint64_t* thr = reinterpret_cast<uint64_t*>(lds + L.thr) + 1;  // padded (bush_thr_pads)
  uint32_t* cval = lds + L.cval;
  uint32_t* info = lds + L.info;
  uint32_t* blk = lds + L.blk;
  uint32_t* jobEnv = lds + L.jobEnv;
  uint32_t* jobKey = lds + L.jobKey;
  constexpr uint32_t P = kWidePitch;
  const uint32_t OB = (uint32_t)p.OB;
  const uint32_t me = (uint32_t)lane * P;
  uint8_t* out = p.planes + (size_t)g0 * OB;
  const int RW = (p.R + 31) >> 5;                 // spawn-ring words

  const WHead h = whead<MODE>(p, g, active);

  // W0's per-env state (lane = env)
  double food = 0.0;
  uint32_t wr[SLOTS];
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) wr[k] = 0u;
  uint32_t live = 0;
  uint32_t spill_live = 0;  // surviving wolves of rows SLOTS.. (bit k - SLOTS)
  int status = 0, ne = 0, ndep = 0;
  bool job = false, emptied = false;
  unsigned long long eaten_of = 0, wolf_of = 0;

  if constexpr (MODE == MODE_STEP) {
    WIDE_STAMP(8 * wave);

    if (wave == 0) {
      // ------------------------------------------------ W0 P0: loads, despawn, pursuit, kill, wolf grid
      const Params p = kernel_params(p0);
      __builtin_amdgcn_s_setprio(3);  // the longest chain
      uint32_t lxy[4] = {0u, 0u, 0u, 0u}, lrem[4] = {0u, 0u, 0u, 0u};
      if (active) {
        food = p.food[g];
#pragma unroll
        for (int k = 0; k < kWideSpec && k < SLOTS; ++k) wr[k] = p.wolves[(int64_t)k * p.B + g];  // speculatively
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < p.eaten_cap) {
            lxy[i] = p.eaten_xy[(int64_t)i * p.B + g];
            lrem[i] = p.eaten_rem[(int64_t)i * p.B + g];
          }
      }
      for (int i = 0; i < p.W; ++i) wp[me + (uint32_t)i] = 0u;  // (while the loads are in flight)
      const int nw = (int)misc_nw(h.hdr.z);
      ne = (int)misc_ne(h.hdr.z);
      ndep = (int)misc_ndep(h.hdr.z);
      const int status_old = (int)misc_status(h.hdr.z);
#pragma unroll
      for (int k = kWideSpec; k < SLOTS; ++k)
        if (k < nw) wr[k] = p.wolves[(int64_t)k * p.B + g];
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) opaque(wr[k]);  // (loaded on some paths only: settle it here)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        opaque(lxy[i]);
        opaque(lrem[i]);
      }
      opaque(food);
      live = nw >= 32 ? ~0u : ((1u << nw) - 1u);
      // despawn (:262-264): one draw per wolf, keyed by its tile and its occurrence index
      // among the co-located wolves before it; groups of 4 slots
      {
        uint32_t keep = 0;
#pragma unroll
        for (int g4 = 0; g4 < SLOTS; g4 += 4) {
          const uint32_t live4 = (live >> g4) & 0xFu;
          if (!live4) continue;
          uint32_t h1[4], hh[4], ts[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int k = g4 + q;
            uint32_t occ = 0;
#pragma unroll
            for (int t = 0; t < k; ++t) occ += (((live >> t) & 1u) && wr[t] == wr[k]) ? 1u : 0u;
            ts[q] = make_ts(SITE_DESPAWN, occ, h.turn);
            h1[q] = wr[k] ^ h.b0;
          }
          fmix32x4(h1);
#pragma unroll
          for (int q = 0; q < 4; ++q) hh[q] = h1[q] ^ ts[q] ^ h.b1;
          fmix32x4(hh);
          uint32_t kp = 0, tie = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            kp |= (hh[q] > p.keep_th ? 1u : 0u) << q;
            tie |= (hh[q] == p.keep_th ? 1u : 0u) << q;
          }
          if (tie & live4) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (((tie >> q) & 1u) && draw_lo21(h1[q], ts[q], h.b0) >= p.keep_tl) kp |= 1u << q;
          }
          keep |= (kp & live4) << g4;
        }
        // wolves beyond the SLOTS register slots (rows SLOTS..nw-1 of the same array, up to
        // wolf_cap; a lane gets there only when a ring spawn found every register slot taken):
        // their despawn draws, keyed like the others (occurrence among every wolf before it,
        // pre-despawn positions)
        if (nw > SLOTS) spill_live = spill_despawn<SLOTS>(p, h, g, nw, wr, live);
        live = keep;
      }
      // pursuit (:267-286): one axis step toward the ostrich, ties along x; the wolf grid of S
      // (:412-428); kill (:291-297)
      bool kill = false;
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {
        if (!((live >> k) & 1u)) continue;
        int wx = xy_x(wr[k]), wy = xy_y(wr[k]);
        if (p.wolves_can_move) {
          const int ddx = h.ox - wx, ddy = h.oy - wy;
          const bool alongx = abs(ddx) >= abs(ddy);
          wx += alongx ? sgn(ddx) : 0;
          wy += alongx ? 0 : sgn(ddy);
          wr[k] = xy_pack(wx, wy);
        }
        const int ddx = h.ox - wx, ddy = h.oy - wy;
        if (active && abs(ddx) <= p.cw && abs(ddy) <= p.ch) wp[me + (uint32_t)(ddx + p.cw)] |= 1u << (ddy + p.ch);
        kill |= ddx == 0 && ddy == 0;
      }
      if (spill_live) {  // the surviving spilled wolves: pursuit, grid, kill (positions stay in HBM)
        for (uint32_t bits = spill_live; bits; bits &= bits - 1u) {
          const int k = SLOTS + __ffs(bits) - 1;
          const uint32_t w = pursue(p, h, p.wolves[(int64_t)k * p.B + g]);
          const int ddx = h.ox - xy_x(w), ddy = h.oy - xy_y(w);
          if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) wp[me + (uint32_t)(ddx + p.cw)] |= 1u << (ddy + p.ch);
          kill |= ddx == 0 && ddy == 0;
        }
      }
      kill = kill && !p.god_mode;
      // the wolf grids of S are complete (this wave wrote every env's rows): plane 0 now,
      // while W1 still builds the bush bitmap
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      obs_plane<0>(p, wp, out, (uint32_t)n_active, lane);
      // eaten log, first entries: the ostrich's tile
      int found = -1, found_rem = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < ne && lxy[k] == h.cpos) { found = k; found_rem = (int)lrem[k]; }
      WIDE_STAMP(1);
      lds_barrier();  // B1: S complete (bitmap rows, wolf grids); the ostrich-tile value
      WIDE_STAMP(2);
      // ------------------------------------------------ W0 P1: eat, starve, done; then obs
      double reward = 0.0;
      if (active) {
        const bool center_bush = ((bm[me + (uint32_t)p.cw] >> p.ch) & 1u) != 0u;
        if (center_bush && found < 0 && ne > 4) {
          for (int i = 4; i < ne; ++i)
            if (p.eaten_xy[(int64_t)i * p.B + g] == h.cpos) { found = i; found_rem = (int)p.eaten_rem[(int64_t)i * p.B + g]; }
        }
        const int rem = found >= 0 ? found_rem : (center_bush ? (int)cval[lane] : 0);
        if (rem > 0 && status_old == 0 && (h.role == 1 || p.lookout_only)) {  // eat (:299-313)
          food = food + p.fill;
          food = food < 0.0 ? 0.0 : (food > 1.0 ? 1.0 : food);
          reward += p.r_eat;
          bool logged = true;
          if (found >= 0) {
            p.eaten_rem[(int64_t)found * p.B + g] = (uint8_t)(rem - 1);
          } else if (ne < p.eaten_cap) {
            p.eaten_xy[(int64_t)ne * p.B + g] = h.cpos;
            p.eaten_rem[(int64_t)ne * p.B + g] = (uint8_t)(rem - 1);
            ne += 1;
          } else {
            eaten_of += 1;
            logged = false;
          }
          if (rem == 1) {  // emptied: gone from the cached view from the next step on
            emptied = true;
            if (logged) ndep += 1;
          }
        }
        food = food - p.hunger;  // :316-322
        const bool starved = food <= 0.0;
        if (starved) food = 0.0;
        status = starved ? 1 : kill ? 2 : status_old;
        const bool done = starved || kill || status_old != 0 || h.turn >= p.max_turns;
        {
          const double r_finish = sreg(p.r_finish), r_turn = sreg(p.r_turn);
          const double r_starve = sreg(p.r_starve), r_killed = sreg(p.r_killed);
          reward += sel_f64(status == 0, sel_f64(done, r_finish, r_turn), sel_f64(status == 1, r_starve, r_killed));
        }
        job = done && p.autoreset;
        __builtin_nontemporal_store((float)reward, p.reward + g);
        __builtin_nontemporal_store((uint8_t)(done ? 1 : 0), p.done + g);
        uint8_t* fts = reinterpret_cast<uint8_t*>(sel64(job, (uint64_t)p.t_food_turns, (uint64_t)p.food_turns));
        uint8_t* rls = reinterpret_cast<uint8_t*>(sel64(job, (uint64_t)p.t_role, (uint64_t)p.role));
        uint8_t* sts = reinterpret_cast<uint8_t*>(sel64(job, (uint64_t)p.t_status, (uint64_t)p.status));
        if (!job || p.t_planes) {
          fts[g] = (uint8_t)(int)ceil(food * (double)p.turns_empty);  // :450-452
          rls[g] = (uint8_t)h.role;
          sts[g] = (uint8_t)status;
        }
        if (!h.valid_action) atomicAdd(&p.counters[CTR_BAD_ACTIONS], 1ull);
      }
      info[lane] = (job ? 1u : 0u) | (emptied ? 2u : 0u);
      const unsigned long long jm = __ballot(job);
      if (job) {
        const int j = __popcll(jm & ((1ull << lane) - 1ull));
        const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));  // the new episode's key
        jobEnv[j] = (uint32_t)lane;
        *reinterpret_cast<uint2*>(&jobKey[2 * j]) = make_uint2((uint32_t)ek2, (uint32_t)(ek2 >> 32));
      }
      if (lane == 0) {
        blk[0] = (uint32_t)__popcll(jm);
        blk[1] = (uint32_t)jm;
        blk[2] = (uint32_t)(jm >> 32);
      }
      __builtin_amdgcn_s_setprio(0);
      WIDE_STAMP(3);
      obs_plane<1>(p, bm, out, (uint32_t)n_active, tid);
      WIDE_STAMP(4);
      lds_barrier();  // B2: job list, spawn masks
      WIDE_STAMP(5);
      // ------------------------------------------------ W0 P2: spawns, state of continuing envs
      if (active && !job) {
        int n_unplaced = 0;
        if (p.wolves_on) {
          for (int w = 0; w < RW; ++w) {
            uint32_t bits = spawn[(uint32_t)lane * L.spw + (uint32_t)w];
            while (bits) {
              const int b = __ffs(bits) - 1;
              bits &= bits - 1;
              const uint32_t t = xy_add(h.cpos, ring[32 * w + b]);
              bool placed = false;
#pragma unroll
              for (int k = 0; k < SLOTS; ++k)
                if (!placed && !((live >> k) & 1u)) { wr[k] = t; live |= 1u << k; placed = true; }
              n_unplaced += placed ? 0 : 1;  // every register slot taken: appended below
            }
          }
        }
        int n = 0;
#pragma unroll
        for (int k = 0; k < SLOTS; ++k)
          if ((live >> k) & 1u) p.wolves[(int64_t)(n++) * p.B + g] = wr[k];
        if (spill_live | n_unplaced) {  // rare: compact the spilled survivors (row k is read
                                        // before any row >= its new index is written), then
                                        // the spawns that found no register slot
          for (uint32_t bits = spill_live; bits; bits &= bits - 1u) {
            const int k = SLOTS + __ffs(bits) - 1;
            p.wolves[(int64_t)(n++) * p.B + g] = pursue(p, h, p.wolves[(int64_t)k * p.B + g]);
          }
          // the spawn tiles again, in the same order: the last n_unplaced of them
          int skip = -n_unplaced;
          for (int w = 0; w < RW; ++w)
            for (uint32_t bits = spawn[(uint32_t)lane * L.spw + (uint32_t)w]; bits; bits &= bits - 1u) skip += 1;
          for (int w = 0; w < RW && n_unplaced; ++w) {
            for (uint32_t bits = spawn[(uint32_t)lane * L.spw + (uint32_t)w]; bits; bits &= bits - 1u) {
              if (skip > 0) { skip -= 1; continue; }
              const uint32_t t = xy_add(h.cpos, ring[32 * w + __ffs(bits) - 1]);
              if (n < p.wolf_cap) p.wolves[(int64_t)(n++) * p.B + g] = t;
              else wolf_of += 1;
            }
          }
        }
        p.hdr[g] = make_uint4(h.cpos, (uint32_t)h.turn,
                              misc_pack((uint32_t)h.role, (uint32_t)status, (uint32_t)n, (uint32_t)ne, (uint32_t)ndep),
                              h.hdr.w);
        p.food[g] = food;
      }
    } else {
      const Params p = kernel_params(p0);
      if (wave == 1) {
        // ---------------------------------------------- W1 P0: the view bitmap
        __builtin_amdgcn_s_setprio(2);
        // every load up front (vmcnt retires in order; a copy loop would wait for each load
        // before issuing the next): thresholds, the first eaten-log entries (speculatively),
        // the bitmap rows (env-major: 32 dwords per env, eight 16-byte loads)
        const int nthr = p.max_berries;
        uint64_t tv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) tv[k] = nthr > 0 ? p.thresholds[min(64 * k + lane, nthr - 1)] : 0ull;
        const int64_t ga = active ? g : 0;
        uint32_t ex[4], er[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t row = min(k, p.eaten_cap - 1);
          ex[k] = p.eaten_xy[row * p.B + ga];
          er[k] = p.eaten_rem[row * p.B + ga];
        }
        uint32_t w[32];
        {
          const uint4* src = reinterpret_cast<const uint4*>(p.bushmap + (size_t)ga * 32u);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint4 v = src[k];
            w[4 * k] = v.x;
            w[4 * k + 1] = v.y;
            w[4 * k + 2] = v.z;
            w[4 * k + 3] = v.w;
          }
        }
        const uint32_t strip = active ? strip_bits(p, h) : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (64 * k + lane < nthr) thr[64 * k + lane] = tv[k];
        if (lane == 0) bush_thr_pads(thr, nthr);
        WIDE_STAMP(15);
        const uint32_t hmask = p.H >= 32 ? ~0u : ((1u << p.H) - 1u);
        const uint32_t top = 1u << (p.H - 1);
        // scroll (generate_bushes keeps the tiles in view, :613-629) + the entering strip
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          if (i >= p.W) break;
          const uint32_t wi = active ? w[i] : 0u;
          const uint32_t prev = (active && i > 0) ? w[i - 1] : 0u;
          const uint32_t next = (active && i < 31 && i + 1 < p.W) ? w[i + 1] : 0u;
          const uint32_t sb = (strip >> i) & 1u;
          uint32_t v = wi;
          v = h.dir == DIR_RIGHT ? (i == 0 ? strip : prev) : v;
          v = h.dir == DIR_LEFT ? (i == p.W - 1 ? strip : next) : v;
          v = h.dir == DIR_UP ? (((wi << 1) & hmask) | sb) : v;
          v = h.dir == DIR_DOWN ? ((wi >> 1) | (sb ? top : 0u)) : v;
          bm[me + (uint32_t)i] = v;
        }
        WIDE_STAMP(31);
        // emptied tiles that scrolled back into view are absent from S (:506): clear every
        // emptied log tile in view (idempotent for the ones already absent)
        const int ne1 = (int)misc_ne(h.hdr.z), ndep1 = (int)misc_ndep(h.hdr.z);
        if (active && ndep1 > 0 && h.dir != DIR_STAY) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int ddx = h.ox - xy_x(ex[k]), ddy = h.oy - xy_y(ex[k]);
            if (k < ne1 && er[k] == 0u && abs(ddx) <= p.cw && abs(ddy) <= p.ch)
              bm[me + (uint32_t)(ddx + p.cw)] &= ~(1u << (ddy + p.ch));
          }
          for (int i = 4; i < ne1; ++i) {  // (rare: more than 4 eaten tiles this episode)
            if (p.eaten_rem[(int64_t)i * p.B + g] != 0) continue;
            const uint32_t t = p.eaten_xy[(int64_t)i * p.B + g];
            const int ddx = h.ox - xy_x(t), ddy = h.oy - xy_y(t);
            if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) bm[me + (uint32_t)(ddx + p.cw)] &= ~(1u << (ddy + p.ch));
          }
        }
        // the generated berries of the ostrich's tile (:631-635), for W0
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        uint32_t cv = 0;
        if (active && ((bm[me + (uint32_t)p.cw] >> p.ch) & 1u))
          cv = (uint32_t)bush_value_fast(thr, p.max_berries, draw_U(h.cpos, make_ts(SITE_BUSH, 0, 0), h.b0, h.b1),
                                         p.bush_power);
        cval[lane] = cv;
        __builtin_amdgcn_s_setprio(0);
      } else {
        // ---------------------------------------------- W3 P0: the ostrich grids; W2 P0: ring
        // offsets and gap table -> LDS, the spawn set (spawn_wolves :527-576)
        __builtin_amdgcn_s_setprio(0);
        // the ostrich grids in two halves: W3 from the start, W2 after its ring word (it would
        // otherwise wait ~10 us at B1 while W3 alone issues them: 46.9 -> 46.3 us)
        if (wave == 3) obs_plane2(p, out, (uint32_t)n_active, lane, 0u, 4u);
        if (wave == 2) {
          copy_to_lds(ring, p.tables + p.ring_at, (p.R + 3) & ~3, lane);
          if (p.wolves_on) copy_to_lds(gap, p.gap, p.n_gap + 1, lane);  // (initial wolves: gap[WH])
          for (int w = 0; w < RW; ++w) spawn[(uint32_t)lane * L.spw + (uint32_t)w] = 0u;
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
          if (p.wolves_on && active)  // one draw unless a wolf spawns
            spawn_hits(gap, p.R, p.gap_full_th, p.gap_full_tl, p.gap_ring_th, p.gap_ring_tl, p.gap_inv_l2, h.turn, h.b0, h.b1, [&](int r) {
              spawn[(uint32_t)lane * L.spw + ((uint32_t)r >> 5)] |= 1u << (r & 31);
            });
          obs_plane2(p, out, (uint32_t)n_active, lane, 4u, 8u);
        }
      }
      WIDE_STAMP(8 * wave + 1);
      lds_barrier();  // B1
      WIDE_STAMP(8 * wave + 2);
      // ------------------------------------------------ P1: W1, W2 obs of S
      if (wave < 3) obs_plane<1>(p, bm, out, (uint32_t)n_active, tid);
      WIDE_STAMP(8 * wave + 3);
      WIDE_STAMP(8 * wave + 4);
      lds_barrier();  // B2
      WIDE_STAMP(8 * wave + 5);
    }
  } else {
    // ------------------------------------------------ MODE_RESET: the flagged envs are jobs
    if (wave == 0) {
      const Params p = kernel_params(p0);
      job = active && (p.reset_mask == nullptr || p.reset_mask[g] != 0);
      info[lane] = job ? 1u : 0u;
      const unsigned long long jm = __ballot(job);
      if (job) {
        const int j = __popcll(jm & ((1ull << lane) - 1ull));
        const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));  // 0xFFFFFFFF -> episode 0
        jobEnv[j] = (uint32_t)lane;
        *reinterpret_cast<uint2*>(&jobKey[2 * j]) = make_uint2((uint32_t)ek2, (uint32_t)(ek2 >> 32));
      }
      if (lane == 0) {
        blk[0] = (uint32_t)__popcll(jm);
        blk[1] = (uint32_t)jm;
        blk[2] = (uint32_t)(jm >> 32);
      }
    }
    lds_barrier();
  }

  const int n_jobs = (int)blk[0];
  const unsigned long long jmask = (unsigned long long)blk[1] | ((unsigned long long)blk[2] << 32);
  {  // (the tail: its own parameter copy)
  const Params p = kernel_params(p0);
  if constexpr (MODE == MODE_STEP) {
    // ------------------------------------------------ P2: bitmaps of the continuing envs (post-eat)
    for (uint32_t u = tid; u < 64u * 32u; u += 256) {  // env-major rows: 128 contiguous bytes per env
      const uint32_t e = u >> 5, i = u & 31u;
      if ((int)e >= n_active || ((jmask >> e) & 1ull) || i >= (uint32_t)p.W) continue;
      uint32_t v = bm[e * P + i];
      if ((info[e] & 2u) && i == (uint32_t)p.cw) v &= ~(1u << p.ch);  // eaten empty
      p.bushmap[(size_t)(g0 + e) * 32u + i] = v;
    }
    if (p.t_planes) {  // terminal obs: the step's own obs of every done env
      uint8_t* tout = p.t_planes + (size_t)g0 * OB;
      for (unsigned long long jj = jmask; jj; jj &= jj - 1) obs_env_all(p, bm, wp, tout, (uint32_t)(__ffsll(jj) - 1), tid);
    }
    if (wave == 0) {
      if (eaten_of) atomicAdd(&p.counters[CTR_EATEN_OVERFLOW], eaten_of);
      if (lane == 0 && n_jobs) atomicAdd(&p.block_resets[blockIdx.x], (unsigned long long)n_jobs);  // (no-return: a load here would wait for the stores)
      count_steps(p);
    }
  } else {
    if (tid == 0 && n_jobs) atomicAdd(&p.block_resets[blockIdx.x], (unsigned long long)n_jobs);  // (no-return: a load here would wait for the stores)
  }

  if (n_jobs > 0) {
    // ------------------------------------------------ done envs: new episodes (:231-248)
    if (MODE == MODE_STEP) lds_barrier();  // B3: the snapshot rows of the jobs are read
    // reset draws (generate_bushes) over the new view, ostrich at (0, 0): 32 lanes per row,
    // rows written by ballot; initialize_wolves (:578-593): the view's spawn set at turn 0, by
    // the job's own lane of W0
    const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0);
    const uint32_t rows2 = ((uint32_t)p.W + 1u) >> 1;  // wave-units of two rows
    for (int jj = 0; jj < n_jobs; ++jj) {
      const uint32_t e = jobEnv[jj];
      const uint2 kq = *reinterpret_cast<const uint2*>(&jobKey[2 * jj]);
      for (uint32_t r2 = (uint32_t)wave; r2 < rows2; r2 += 4u) {
        const uint32_t i = 2u * r2 + ((uint32_t)lane >> 5), j = (uint32_t)lane & 31u;
        const bool cell = i < (uint32_t)p.W && j < (uint32_t)p.H;
        const uint32_t xy = xy_pack(p.cw - (int)i, p.ch - (int)j);
        const uint32_t h1 = fmix32(xy ^ kq.x);
        const uint32_t hb = fmix32(h1 ^ ts_bush ^ kq.y);
        const bool bush = cell && U_ge(h1, hb, ts_bush, kq.x, p.bush_th, p.bush_tl);
        const unsigned long long bb = __ballot(bush);
        if ((lane & 31) == 0 && i < (uint32_t)p.W) bm[e * P + i] = (uint32_t)(lane ? bb >> 32 : bb);
      }
    }
    if (wave == 0 && active && ((jmask >> lane) & 1ull)) {
      const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));
      for (int i = 0; i < p.W; ++i) wp[me + (uint32_t)i] = 0u;
      if (p.wolves_on)
        spawn_hits(MODE == MODE_STEP ? gap : p.gap, p.WH, p.gap_full_th, p.gap_full_tl, p.gap_view_th, p.gap_view_tl, p.gap_inv_l2, 0, (uint32_t)ek2,
                   (uint32_t)(ek2 >> 32), [&](int c) {
                     const uint32_t i = (uint32_t)c / (uint32_t)p.H;
                     wp[me + i] |= 1u << ((uint32_t)c - i * (uint32_t)p.H);
                   });
    }
    lds_barrier();  // B4
    if (wave == 0 && active && ((jmask >> lane) & 1ull)) {
      // spawn_ostriches (:595-611) and the initial wolves, one per wolf cell of the view
      const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));
      const uint32_t kb0 = (uint32_t)ek2, kb1 = (uint32_t)(ek2 >> 32);
      const double food2 = p.start_food_random
                               ? (double)draw_U(xy_pack(0, 0), make_ts(SITE_START_FOOD, 0, 0), kb0, kb1) * 0x1p-53
                               : p.start_food;
      const int role2 = p.start_role_random
                            ? (int)(draw_U(xy_pack(0, 0), make_ts(SITE_START_ROLE, 0, 0), kb0, kb1) >> 52)
                            : p.start_role;
      int n = 0;
      for (int i = 0; i < p.W; ++i) {
        uint32_t bits = wp[me + (uint32_t)i];
        while (bits) {
          const int j = __ffs(bits) - 1;
          bits &= bits - 1;
          if (n < p.wolf_cap) p.wolves[(int64_t)(n++) * p.B + g] = xy_pack(p.cw - i, p.ch - j);
          else {
            wolf_of += 1;
            atomicAdd(&p.counters[CTR_WOLF_OVERFLOW_RESET], 1ull);
          }
        }
      }
      p.hdr[g] = make_uint4(xy_pack(0, 0), 0u, misc_pack((uint32_t)role2, 0u, (uint32_t)n, 0u, 0u), h.hdr.w + 1u);
      p.food[g] = food2;
      p.food_turns[g] = (uint8_t)(int)ceil(food2 * (double)p.turns_empty);
      p.role[g] = (uint8_t)role2;
      p.status[g] = 0;
    }
    // the new episodes' obs (same threads as their S chunks: ordered after them) and bitmaps
    for (int jj = 0; jj < n_jobs; ++jj) {
      const uint32_t e = jobEnv[jj];
      if (MODE == MODE_STEP) obs_env(p, bm, wp, out, e, tid);  // (plane 2 is already right)
      else obs_env_all(p, bm, wp, out, e, tid);
      for (uint32_t i = tid; i < (uint32_t)p.W; i += 256) p.bushmap[(size_t)(g0 + e) * 32u + i] = bm[e * P + i];
    }
  }
  if (wave == 0 && wolf_of) atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], wolf_of);
  }
#ifdef WAB_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  WIDE_STAMP(8 * wave + 6);
#endif
}

// --------------------------------------------------------------------------- multi-step launches
// wab_rollout on the wide kernel: each workgroup takes its 64 envs through Params::n_steps steps
// in one launch (the envs of a workgroup depend on nothing outside it).  The phases of a step
// are those of wab_step_wide<MODE_STEP>; what changes is where the state lives between steps
// and when the obs go out:
//   - every wave: the env's header (W0 writes the next one to LDS, nhdr) and the next step's
//     actions (W3 prefetches them with one scalar load per group into LDS, act);
//   - W0: food, the 8 register wolf slots (uncompacted, with a live mask; the rarely used rows
//     8.. stay in HBM, compacted at rows 8..8+nsp-1, read and written by the env's own lane) and
//     the first eaten-log entries (0..3 in registers, 4..7 in LDS, later ones in HBM, own lane);
//   - the view bitmaps and wolf grids live in LDS twice: step t builds its obs (S for the
//     continuing envs, the new episode for the done ones) in buffer t & 1 -- W1 scrolls the
//     other buffer's bitmaps into it, W0 draws the wolf grids -- while W2 and W3 store step
//     t - 1's obs from the other buffer.
// Obs stores.  A step's obs are 64 x 3 W rows of S bytes; the store waves write them as whole
// 128-byte lines in address order (thread q of 128 the rows q + 128 k, both halves of a 32-byte
// row from two back-to-back instructions: each wave-instruction pair covers 16 whole lines).
// They store while the compute waves work: up to B1 until W0 signals that it reached B1, up to
// B2 likewise, and after B2 whatever is left, so the compute of step t overlaps the drain of
// step t - 1 and no barrier waits for more than two rows of issue.  (The round-3 build stored
// each step's rows after its own B2, all 256 threads, then the done envs' lines after their new
// episodes: 41.5-46.1 us per step, a workgroup blocked on store issue for most of its step and
// the four workgroups of a CU in phase.)  Only step 0 loads state and only the last step stores
// it; W1 and W0 issue no vector load after step 0 on their common path.  The last step's obs
// go out after it by all 256 threads.  W0 (which owns the eaten log) clears the emptied tiles
// that scrolled back into view after W1's scroll (LDS flag); the eaten-empty centre bit of a
// continuing env (post-eat) is applied by W1 when it scrolls that bitmap in the next step.
// Co-located wolves are interchangeable (their despawn keys are (tile, occurrence index)
// whatever their order), so the uncompacted slots step exactly as the per-step kernel's
// compacted rows do.
namespace {

// a step-tagged hand-off: the producer stores a value that grows every step (no clearing)
__device__ __forceinline__ void lds_publish_step(uint32_t* flag, uint32_t v) {
  __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_await_step(const Params& p, const uint32_t* flag, uint32_t v) {
  for (int spin = 0; spin < (1 << 20); ++spin) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) return;
    __builtin_amdgcn_s_sleep(1);
  }
  atomicAdd(&p.counters[CTR_HANDOFF_TIMEOUTS], 1ull);
}

// whead of a carried header and action
__device__ __forceinline__ WHead whead_of(const Params& p, int64_t g, bool active, uint4 hdr, int a) {
  WHead h;
  h.active = active;
  h.hdr = active ? hdr : make_uint4(0u, 0u, 0u, 0u);
  a = active ? a : 0;
  h.kenv = env_key(p.seed, (uint64_t)(p.env_base + g));
  h.ox = xy_x(h.hdr.x);
  h.oy = xy_y(h.hdr.x);
  h.turn = (int32_t)h.hdr.y + 1;
  h.role = (int)misc_role(h.hdr.z);
  h.dir = DIR_STAY;
  h.valid_action = a >= 0 && a < p.n_actions;
  if (h.valid_action) {
    int dx, dy, nr;
    decode_action(p, a, dx, dy, nr);
    h.ox += dx;
    h.oy += dy;
    h.dir = dx > 0 ? DIR_RIGHT : dx < 0 ? DIR_LEFT : dy > 0 ? DIR_UP : dy < 0 ? DIR_DOWN : DIR_STAY;
    if (nr >= 0) h.role = nr;
  }
  h.cpos = xy_pack(h.ox, h.oy);
  const uint64_t ek = mix64(h.kenv ^ (uint64_t)h.hdr.w);
  h.b0 = (uint32_t)ek;
  h.b1 = (uint32_t)(ek >> 32);
  return h;
}

// the next step's 64 actions of the group into act: one 64-byte scalar load (lgkmcnt: no wait
// on this wave's stores), spread over lanes 0..15; a partial or misaligned group reads per lane
__device__ __forceinline__ void wide_prefetch_actions(const Params& p, uint32_t* act, int lane) {
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const int8_t* a = p.actions + p.B + g0;  // step t + 1 (p.actions is step t's slice)
  if (g0 + 64 <= p.B && (reinterpret_cast<uintptr_t>(a) & 3u) == 0u) {
    typedef const uint32_t __attribute__((address_space(4))) CU32;
    CU32* c = (CU32*)reinterpret_cast<uintptr_t>(a);
    asm volatile("" : "+s"(c));
    uint32_t v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = c[k];
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) d = lane == k ? v[k] : d;
    if (lane < 16) act[lane] = d;
  } else {
    const int8_t v = g0 + lane < p.B ? a[lane] : (int8_t)0;
    reinterpret_cast<int8_t*>(act)[lane] = v;
  }
}

// register slot k := v (k dynamic)
template <int SLOTS>
__device__ __forceinline__ void slot_set(uint32_t (&wr)[SLOTS], int k, uint32_t v) {
#pragma unroll
  for (int j = 0; j < SLOTS; ++j) wr[j] = j == k ? v : wr[j];
}

// A thread's position in a finished step's obs rows: row q (of the group's 3 W rows per env,
// in address order) is row rr of env e
struct RowCursor {
  uint32_t q, e, rr;
};
__device__ __forceinline__ RowCursor row_cursor(const Params& p, uint32_t q) {
  const uint32_t RPE = 3u * (uint32_t)p.W;
  RowCursor c;
  c.q = q;
  c.e = q / RPE;
  c.rr = q - c.e * RPE;
  return c;
}

// store obs row c.q (wolf rows wp, bush rows bm at kRollPitch; the ostrich grid is the centre
// cell alone) and move the cursor NT rows on
template <uint32_t NT>
__device__ __forceinline__ void roll_store_row(const Params& p, const uint32_t* bm, const uint32_t* wp, uint8_t* out,
                                               RowCursor& c) {
  const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4, W = (uint32_t)p.W, RPE = 3u * W;
  const uint32_t k = (c.rr >= W ? 1u : 0u) + (c.rr >= 2u * W ? 1u : 0u);
  const uint32_t i = c.rr - k * W;
  const uint32_t v = k == 2u ? (i == (uint32_t)p.cw ? 1u << p.ch : 0u) : (k == 0u ? wp : bm)[c.e * kRollPitch + i];
  const uint32_t ch0 = c.e * CPE + c.rr * CPR;  // the row's first 16-byte chunk
  store16(p, out, ch0, expand16(v & 0xFFFFu));
  if (CPR == 2u) store16(p, out, ch0 + 1u, expand16(v >> 16));
  c.q += NT;
  c.rr += NT;
  while (c.rr >= RPE) { c.rr -= RPE; ++c.e; }
}

// Obs rows by blocks of 64 (one wave-instruction pair per block, 16 whole 128-byte lines),
// claimed from a per-step LDS counter by whichever wave has nothing else to do, so that the
// store stream is spread over every idle wave and no wave ends its share much later than the
// others.  A queue: the rows of one step, [0, n_rows), its counter, and the done envs' mask when
// only the lines that touch no done env are wanted (the last step's S after B2).
struct RowQueue {
  uint32_t* ctr;
  uint32_t n_rows, n_blocks, magic;  // magic: row -> env division (umulhi, exact below 2^16 rows)
  const uint32_t* bm;
  const uint32_t* wp;
  uint8_t* out;
  unsigned long long jm;
  bool untouched_only;
  bool skip_p2;  // the ostrich plane's whole lines are stored by drain_plane2
};
__device__ __forceinline__ RowQueue row_queue(const Params& p, uint32_t* ctr, uint32_t n_rows, const uint32_t* bm,
                                              const uint32_t* wp, uint8_t* out) {
  RowQueue q;
  q.ctr = ctr;
  q.n_rows = n_rows;
  q.n_blocks = (n_rows * ((uint32_t)p.S >> 4) + 63u) >> 6;  // blocks of 64 16-byte chunks
  const uint32_t RPE = 3u * (uint32_t)p.W;
  q.magic = (uint32_t)((0x100000000ull + RPE - 1u) / RPE);
  q.bm = bm;
  q.wp = wp;
  q.out = out;
  q.jm = 0ull;
  q.untouched_only = false;
  q.skip_p2 = false;
  return q;
}
template <bool IF>
__device__ __forceinline__ void store_block(const Params& p, const RowQueue& q, uint32_t b, int lane);

// claim and store blocks until the queue is empty (true) or flag >= v (v > 0; false)
__device__ __forceinline__ bool drain_rows(const Params& p, const RowQueue& q, int lane, const uint32_t* flag = nullptr,
                                           uint32_t v = 0u) {
  while (true) {
    if (v && __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >= v)
      return false;
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(q.ctr, 1u);
    b = (uint32_t)__shfl((int)b, 0);
    if (b >= q.n_blocks) return true;
    if (q.untouched_only) store_block<true>(p, q, b, lane);
    else store_block<false>(p, q, b, lane);
  }
}

// roll_store_row for the rows whose 128-byte line touches a done env (jm) iff `touching`
template <uint32_t NT>
__device__ __forceinline__ void roll_store_row_if(const Params& p, const uint32_t* bm, const uint32_t* wp, uint8_t* out,
                                                  RowCursor& c, unsigned long long jm, bool touching) {
  const unsigned long long jn = jm | (jm << 1) | (jm >> 1);  // done envs and their neighbours
  bool t = false;
  if ((jn >> c.e) & 1ull) {
    const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4;
    const uint32_t n = ((uint32_t)min((int64_t)64, p.B - (int64_t)blockIdx.x * 64)) * CPE;
    const uint32_t ch = c.e * CPE + c.rr * CPR, c0 = ch & ~7u, c1 = min(c0 + 7u, n - 1u);
    t = ((jm >> __umulhi(c0, p.magic_CPE)) | (jm >> __umulhi(c1, p.magic_CPE))) & 1ull;  // (chunks < 2^16)
  }
  if (t == touching) {
    roll_store_row<NT>(p, bm, wp, out, c);
  } else {  // (advance only)
    const uint32_t RPE = 3u * (uint32_t)p.W;
    c.q += NT;
    c.rr += NT;
    while (c.rr >= RPE) { c.rr -= RPE; ++c.e; }
  }
}

// the last step's queue after B2: its S lines that touch no done env (blk: the job mask)
__device__ __forceinline__ RowQueue untouched_rows(const Params& p, uint32_t* ctr, uint32_t n_rows, const uint32_t* bm,
                                                   const uint32_t* wp, uint8_t* out, const uint32_t* blk) {
  RowQueue q = row_queue(p, ctr, n_rows, bm, wp, out);
  q.jm = (unsigned long long)blk[1] | ((unsigned long long)blk[2] << 32);
  q.untouched_only = true;
  q.skip_p2 = true;
  return q;
}

// Block b of a queue: lane l stores 16-byte chunk 64 b + l of the group's obs (one row half when
// rows are 32 bytes), non-temporal, so each wave-instruction writes 1 KiB contiguous, eight
// whole lines.  (Measured at B = 65536, T = 64, one box: rows per lane, the two halves from
// two back-to-back instructions, 40.4-40.7 us per step, non-temporal 102 us (partial lines);
// chunks 39.7, non-temporal chunks 38.9; the pattern's stores alone 34.1-35.9.)
template <bool IF>
__device__ __forceinline__ void store_block(const Params& p, const RowQueue& q, uint32_t b, int lane) {
  const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4, W = (uint32_t)p.W;
  const uint32_t ch = 64u * b + (uint32_t)lane, row = CPR == 2u ? ch >> 1 : ch, half = CPR == 2u ? ch & 1u : 0u;
  if (row >= q.n_rows) return;
  const uint32_t e = __umulhi(row, q.magic), rr = row - e * 3u * W;
  if (q.skip_p2) {  // (a whole line inside the env's ostrich plane: stored already)
    const int o0 = (int)(((64u * b + (uint32_t)lane) & ~7u) - e * CPE), p2 = (int)(2u * W * CPR);
    if (o0 >= p2 && o0 + 8 <= (int)(3u * W * CPR)) return;
  }
  if (IF) {  // (only the lines that touch no done env)
    const unsigned long long jn = q.jm | (q.jm << 1) | (q.jm >> 1);
    if ((jn >> e) & 1ull) {
      const uint32_t n = ((uint32_t)min((int64_t)64, p.B - (int64_t)blockIdx.x * 64)) * CPE;
      const uint32_t c0 = (e * CPE + rr * CPR) & ~7u, c1 = min(c0 + 7u, n - 1u);
      if (((q.jm >> __umulhi(c0, p.magic_CPE)) | (q.jm >> __umulhi(c1, p.magic_CPE))) & 1ull) return;
    }
  }
  const uint32_t k = (rr >= W ? 1u : 0u) + (rr >= 2u * W ? 1u : 0u);
  const uint32_t i = rr - k * W;
  const uint32_t v = k == 2u ? (i == (uint32_t)p.cw ? 1u << p.ch : 0u) : (k == 0u ? q.wp : q.bm)[e * kRollPitch + i];
  wide_obs_store(expand16((v >> (16u * half)) & 0xFFFFu), reinterpret_cast<u32x4*>(q.out) + e * CPE + rr * CPR + half);
}

// The last step's ostrich-plane lines: the plane is the centre cell alone, the same in every
// observation (a done env's new episode included), so its whole lines (inside one env's plane
// 2) can go out from the step's start, under the step's compute; one env per claimed block,
// 6-7 lines per instruction.  Claimed from ctr until the envs run out (true) or flag >= v
// (false).  (Measured, B = 65536: one-step launches into a 32-slot ring 59.1 -> 52.3 us; the
// same gated until W0's and W1's step-0 loads were in: 53.0; 64-step launches: unchanged.)
__device__ __forceinline__ bool drain_plane2(const Params& p, uint32_t* ctr, int n_active, uint8_t* out, int lane,
                                             const uint32_t* flag = nullptr, uint32_t v = 0u) {
  const uint32_t CPE = (uint32_t)p.OB >> 4, CPR = (uint32_t)p.S >> 4, W = (uint32_t)p.W;
  while (true) {
    if (v && __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >= v)
      return false;
    uint32_t e = 0;
    if (lane == 0) e = atomicAdd(ctr, 1u);
    e = (uint32_t)__shfl((int)e, 0);
    if (e >= (uint32_t)n_active) return true;
    const uint32_t base = e * CPE, a = (base + 2u * W * CPR + 7u) & ~7u, z = (base + 3u * W * CPR) & ~7u;
    const uint32_t ch = a + (uint32_t)lane;  // (z - a <= W * CPR <= 64)
    if (ch < z) {
      const uint32_t o = ch - base, rr = CPR == 2u ? o >> 1 : o, half = CPR == 2u ? o & 1u : 0u;
      const uint32_t v2 = rr - 2u * W == (uint32_t)p.cw ? 1u << p.ch : 0u;
      wide_obs_store(expand16((v2 >> (16u * half)) & 0xFFFFu), reinterpret_cast<u32x4*>(out) + ch);
    }
  }
}

// Diagnostic build (-DWAB_STAMPS): the middle step's phase stamps of the rollout build
// (tools/phase_stamps.py --rollout T --config wide31): W0 0..7, W1 8..13, W2 16..20, W3 24..27,
// the done-env section 36..39
#ifdef WAB_STAMPS
#define ROLLW_STAMP(slot)                                                                \
  do {                                                                                   \
    if (lane == 0 && p.stamps && t == T / 2)                                             \
      p.stamps[(size_t)blockIdx.x * kStampStride + (slot)] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#else
#define ROLLW_STAMP(slot) do {} while (0)
#endif

#ifndef WAB_WIDE_ROLL_FLOOR  // diagnostic: every step's work skipped, its obs stores kept
#define WAB_WIDE_ROLL_FLOOR 0
#endif

// step t of a multi-step launch: the I/O arrays advanced to their [t] slices
__device__ __forceinline__ void wide_step_slice(Params& p, int t) {
  const int64_t o = (int64_t)t * p.B;
  p.actions += o;
  p.planes += o * p.OB;
  p.food_turns += o;
  p.role += o;
  p.status += o;
  p.reward += o;
  p.done += o;
}

}  // namespace


// FIXW > 0: an instance for a FIXW x FIXW view in 32-byte rows (C3: 31 x 31), the geometry fields
// constants after each step's parameter load, so that the layout and index arithmetic fold
// (the host takes it only for a handle of exactly that geometry); 0: the handle's geometry.
template <int SLOTS, int FIXW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void wab_rollout_wide(Params p0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  if (g0 >= p0.B) return;  // (uniform over the workgroup)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int T = p0.n_steps;
#ifdef WAB_STAMPS
  if (tid == 0 && p0.stamps) {  // kernel entry (slot 32), the XCD (33)
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    p0.stamps[(size_t)blockIdx.x * kStampStride + 32] = __builtin_amdgcn_s_memrealtime();
    p0.stamps[(size_t)blockIdx.x * kStampStride + 33] = xcc & 0xFu;
  }
  if (lane == 0 && p0.stamps) {  // each wave's HW_ID (SIMD, CU, SE) in slots 40..43
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    p0.stamps[(size_t)blockIdx.x * kStampStride + 40 + wave] = hw;
  }
#endif
  const int n_active = (int)min((int64_t)64, p0.B - g0);
  const int64_t g = g0 + lane;
  const bool active = lane < n_active;
  constexpr uint32_t P = kRollPitch;
  const uint32_t me = (uint32_t)lane * P;

  // carried state (per wave: the header; W0: food, wolves, eaten log)
  uint4 hdr = make_uint4(0u, 0u, 0u, 0u);
  double food = 0.0;
  uint32_t wr[SLOTS];
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) wr[k] = 0u;
  uint32_t live = 0;  // occupied register slots
  int nsp = 0;        // wolves in HBM rows SLOTS..SLOTS+nsp-1
  uint32_t lxy[4] = {0u, 0u, 0u, 0u}, lrem[4] = {0u, 0u, 0u, 0u};
  {  // the step flags start below every step's value
    const WideRollLayout L = wide_roll_layout(p0);
    if (tid < 8) lds[L.flag + tid] = 0u;
    lds_barrier();
  }

  for (int t = 0; t < T; ++t) {
#ifdef WAB_STAMPS
    if (tid == 0 && p0.stamps && t == T / 2)  // the middle step's loop top
      p0.stamps[(size_t)blockIdx.x * kStampStride + 35] = __builtin_amdgcn_s_memrealtime();
#endif
    const bool last = t == T - 1;
    const int cur = t & 1;
    Params p = kernel_params(p0);
    if constexpr (FIXW > 0) {
      p.W = FIXW;
      p.H = FIXW;
      p.S = 32;
      p.cw = FIXW / 2;
      p.ch = FIXW / 2;
      p.OB = 3 * FIXW * 32;
      p.WH = FIXW * FIXW;
      p.SL = FIXW;
    }
    wide_step_slice(p, t);
    const WideRollLayout L = wide_roll_layout(p);
    // (buffers chosen by selects: a runtime index into the layout would put it in scratch)
    uint32_t* bm = lds + (cur ? L.bm[1] : L.bm[0]);  // this step's obs: bitmaps and wolf grids
    uint32_t* wp = lds + (cur ? L.wp[1] : L.wp[0]);
    uint32_t* bm_prev = lds + (cur ? L.bm[0] : L.bm[1]);  // the last step's (stored during this one)
    const uint32_t* wp_prev = lds + (cur ? L.wp[0] : L.wp[1]);
    uint32_t* spawn = lds + L.spawn;
    uint32_t* ring = lds + L.ring;
    uint64_t* gap = reinterpret_cast<uint64_t*>(lds + L.gap);
    uint64_t* thr = reinterpret_cast<uint64_t*>(lds + L.thr) + 1;
    uint32_t* cval = lds + L.cval;
    uint32_t* info = lds + L.info;
    uint32_t* blk = lds + L.blk;
    uint32_t* jobEnv = lds + L.jobEnv;
    uint32_t* jobKey = lds + L.jobKey;
    uint4* nhdr = reinterpret_cast<uint4*>(lds + L.nhdr);
    uint32_t* act = lds + L.act;
    uint32_t* flag = lds + L.flag;
    uint32_t* elxy = lds + L.elxy;
    uint8_t* elrem = reinterpret_cast<uint8_t*>(lds + L.elrem);
    const uint32_t OB = (uint32_t)p.OB;
    uint8_t* out = p.planes + (size_t)g0 * OB;
    uint8_t* out_prev = out - (size_t)p.B * OB;  // step t - 1's slice (t > 0)
    const int RW = (p.R + 31) >> 5;
    // the W0 -> store-wave phase signals of this step (flag[2]): B1 reached, B2 reached
    const uint32_t at_b1 = 2u * (uint32_t)t + 1u, at_b2 = 2u * (uint32_t)t + 2u;
    const uint32_t n_rows = (uint32_t)n_active * 3u * (uint32_t)p.W;  // the group's obs rows per step
    // step t - 1's rows, stored during this step (row-block counter flag[4 + (t - 1) % 2]); this
    // step's counter is cleared now (last used two steps ago)
    const RowQueue qp = row_queue(p, flag + 4 + ((t + 1) & 1), n_rows, bm_prev, wp_prev, out_prev);
    if (tid == 0) flag[4 + cur] = 0u;

    WHead h = {};  // (the header and action: W0 and W1 only)
    if (wave < 2) {
      int a = 0;
      if (t == 0) {
        if (active) {
          hdr = p.hdr[g];
          a = (int)p.actions[g];
        }
        if (wave == 1) {  // W1: the thresholds and bitmap rows in the same round trip (one-step launches
                          // into a ring: B1 at 12.9 -> 10.6 us, 52.35 -> 52.1 us per launch)
          const int nthr = p.max_berries;
          uint64_t tv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) tv[k] = nthr > 0 ? p.thresholds[min(64 * k + lane, nthr - 1)] : 0ull;
          const uint4* sp = reinterpret_cast<const uint4*>(p.bushmap + (size_t)(active ? g : 0) * 32u);
          uint4 v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = sp[k];
          __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t r[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (4 * k + q < p.W) bm_prev[me + (uint32_t)(4 * k + q)] = r[q];
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (64 * k + lane < nthr) thr[64 * k + lane] = tv[k];
          if (lane == 0) bush_thr_pads(thr, nthr);
        }
        // (every step-0 load settled inside its branch: the waitcnt pass would otherwise put
        // vmcnt(0) waits at the join that every later step executes too, each one waiting for all
        // of the wave's obs stores in flight)
        __builtin_amdgcn_s_waitcnt(0);
      } else {
        hdr = nhdr[lane];
        a = (int)reinterpret_cast<const int8_t*>(act)[lane];
      }
      h = whead_of(p, g, active, hdr, a);
    }
    if (WAB_WIDE_ROLL_FLOOR) {  // (diagnostic floor: the stores alone, every wave (2: W2, W3); results wrong)
      if (t > 0 && (WAB_WIDE_ROLL_FLOOR == 1 || wave >= 2)) drain_rows(p, qp, lane);
      lds_barrier();
      continue;
    }
    int status = 0, ne = 0, ndep = 0;
    bool job = false, emptied = false;
    unsigned long long eaten_of = 0, wolf_of = 0;
    uint32_t spill_live = 0;

    ROLLW_STAMP(8 * wave);
    if (wave == 0) {
      // ------------------------------------------------ W0 P0: (loads,) despawn, pursuit, kill, wolf grid
      __builtin_amdgcn_s_setprio(3);
      const int nw0 = (int)misc_nw(h.hdr.z);
      if (t == 0) {
        if (active) {
          food = p.food[g];
#pragma unroll
          for (int k = 0; k < SLOTS; ++k) wr[k] = p.wolves[(int64_t)k * p.B + g];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < p.eaten_cap) {
              lxy[i] = p.eaten_xy[(int64_t)i * p.B + g];
              lrem[i] = p.eaten_rem[(int64_t)i * p.B + g];
            }
          const int ne0 = (int)misc_ne(h.hdr.z);  // entries 4.. on chip (step 0: nothing stored yet)
          for (int i = 4; i < ne0 && i < kWideRollLog; ++i) {
            elxy[(i - 4) * 64 + lane] = p.eaten_xy[(int64_t)i * p.B + g];
            elrem[(i - 4) * 64 + lane] = p.eaten_rem[(int64_t)i * p.B + g];
          }
        }
        __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) opaque(wr[k]);
        opaque(food);
        live = nw0 >= 32 ? ~0u : ((1u << nw0) - 1u);
        live &= (SLOTS >= 32 ? ~0u : ((1u << SLOTS) - 1u));
        nsp = nw0 > SLOTS ? nw0 - SLOTS : 0;
      }
      if (!active) {
        live = 0u;
        nsp = 0;
      }
      for (int i = 0; i < p.W; ++i) wp[me + (uint32_t)i] = 0u;
      ne = (int)misc_ne(h.hdr.z);
      ndep = (int)misc_ndep(h.hdr.z);
      const int status_old = (int)misc_status(h.hdr.z);
      {  // despawn (:262-264), groups of 4 register slots; then the HBM rows
        uint32_t keep = 0;
#pragma unroll
        for (int g4 = 0; g4 < SLOTS; g4 += 4) {
          const uint32_t live4 = (live >> g4) & 0xFu;
          if (!live4) continue;
          uint32_t h1[4], hh[4], ts[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int k = g4 + q;
            uint32_t occ = 0;
#pragma unroll
            for (int u = 0; u < k; ++u) occ += (((live >> u) & 1u) && wr[u] == wr[k]) ? 1u : 0u;
            ts[q] = make_ts(SITE_DESPAWN, occ, h.turn);
            h1[q] = wr[k] ^ h.b0;
          }
          fmix32x4(h1);
#pragma unroll
          for (int q = 0; q < 4; ++q) hh[q] = h1[q] ^ ts[q] ^ h.b1;
          fmix32x4(hh);
          uint32_t kp = 0, tie = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            kp |= (hh[q] > p.keep_th ? 1u : 0u) << q;
            tie |= (hh[q] == p.keep_th ? 1u : 0u) << q;
          }
          if (tie & live4) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (((tie >> q) & 1u) && draw_lo21(h1[q], ts[q], h.b0) >= p.keep_tl) kp |= 1u << q;
          }
          keep |= (kp & live4) << g4;
        }
        if (nsp > 0) spill_live = spill_despawn<SLOTS>(p, h, g, SLOTS + nsp, wr, live);
        live = keep;
      }
      bool kill = false;
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {  // pursuit (:267-286), grid of S (:412-428), kill (:291-297)
        if (!((live >> k) & 1u)) continue;
        int wx = xy_x(wr[k]), wy = xy_y(wr[k]);
        if (p.wolves_can_move) {
          const int ddx = h.ox - wx, ddy = h.oy - wy;
          const bool alongx = abs(ddx) >= abs(ddy);
          wx += alongx ? sgn(ddx) : 0;
          wy += alongx ? 0 : sgn(ddy);
          wr[k] = xy_pack(wx, wy);
        }
        const int ddx = h.ox - wx, ddy = h.oy - wy;
        if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) wp[me + (uint32_t)(ddx + p.cw)] |= 1u << (ddy + p.ch);
        kill |= ddx == 0 && ddy == 0;
      }
      if (spill_live) {  // the surviving HBM-row wolves: pursued in place
        for (uint32_t bits = spill_live; bits; bits &= bits - 1u) {
          const int k = SLOTS + __ffs(bits) - 1;
          const uint32_t w = pursue(p, h, p.wolves[(int64_t)k * p.B + g]);
          p.wolves[(int64_t)k * p.B + g] = w;
          const int ddx = h.ox - xy_x(w), ddy = h.oy - xy_y(w);
          if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) wp[me + (uint32_t)(ddx + p.cw)] |= 1u << (ddy + p.ch);
          kill |= ddx == 0 && ddy == 0;
        }
      }
      kill = kill && !p.god_mode;
      // spawn_wolves (:527-576): the ring's spawn set this turn (one draw unless a wolf spawns),
      // read by this lane only (P2); step 0: once W2 has the gap table in LDS
      for (int w = 0; w < RW; ++w) spawn[(uint32_t)lane * L.spw + (uint32_t)w] = 0u;
      if (p.wolves_on) {
        if (t == 0) lds_await_step(p, flag + 1, 1u);
        if (active)
          spawn_hits(gap, p.R, p.gap_full_th, p.gap_full_tl, p.gap_ring_th, p.gap_ring_tl, p.gap_inv_l2, h.turn, h.b0,
                     h.b1, [&](int r) { spawn[(uint32_t)lane * L.spw + ((uint32_t)r >> 5)] |= 1u << (r & 31); });
      }
      ROLLW_STAMP(1);
      // emptied tiles that scrolled back into view are absent from S (:506): cleared from the
      // bitmap once W1 has scrolled it (the per-step kernel's W1 does this from its own loads)
      const bool clear = active && ndep > 0 && h.dir != DIR_STAY;
      if (__ballot(clear)) {
        lds_await_step(p, flag, (uint32_t)t + 1u);
        if (clear) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int ddx = h.ox - xy_x(lxy[k]), ddy = h.oy - xy_y(lxy[k]);
            if (k < ne && lrem[k] == 0u && abs(ddx) <= p.cw && abs(ddy) <= p.ch)
              bm[me + (uint32_t)(ddx + p.cw)] &= ~(1u << (ddy + p.ch));
          }
          for (int i = 4; i < ne && i < kWideRollLog; ++i) {  // (more than 4 eaten tiles: LDS)
            if (elrem[(i - 4) * 64 + lane] != 0u) continue;
            const uint32_t tt = elxy[(i - 4) * 64 + lane];
            const int ddx = h.ox - xy_x(tt), ddy = h.oy - xy_y(tt);
            if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) bm[me + (uint32_t)(ddx + p.cw)] &= ~(1u << (ddy + p.ch));
          }
          if (ne > kWideRollLog) {  // (rare: the rest in HBM)
            for (int i = kWideRollLog; i < ne; ++i) {
              if (p.eaten_rem[(int64_t)i * p.B + g] != 0) continue;
              const uint32_t tt = p.eaten_xy[(int64_t)i * p.B + g];
              const int ddx = h.ox - xy_x(tt), ddy = h.oy - xy_y(tt);
              if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) bm[me + (uint32_t)(ddx + p.cw)] &= ~(1u << (ddy + p.ch));
            }
          }
        }
      }
      int found = -1, found_rem = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < ne && lxy[k] == h.cpos) { found = k; found_rem = (int)lrem[k]; }
      ROLLW_STAMP(2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_publish_step(flag + 2, at_b1);  // (the store waves stop before B1)
      lds_barrier();  // B1
      ROLLW_STAMP(3);
      // ------------------------------------------------ W0 P1: eat, starve, done
      double reward = 0.0;
      if (active) {
        const bool center_bush = ((bm[me + (uint32_t)p.cw] >> p.ch) & 1u) != 0u;
        if (center_bush && found < 0 && ne > 4) {
          for (int i = 4; i < ne && i < kWideRollLog; ++i)
            if (elxy[(i - 4) * 64 + lane] == h.cpos) { found = i; found_rem = (int)elrem[(i - 4) * 64 + lane]; }
          if (ne > kWideRollLog)  // (rare)
            for (int i = kWideRollLog; i < ne; ++i)
              if (p.eaten_xy[(int64_t)i * p.B + g] == h.cpos) { found = i; found_rem = (int)p.eaten_rem[(int64_t)i * p.B + g]; }
        }
        const int rem = found >= 0 ? found_rem : (center_bush ? (int)cval[lane] : 0);
        if (rem > 0 && status_old == 0 && (h.role == 1 || p.lookout_only)) {  // eat (:299-313)
          food = food + p.fill;
          food = food < 0.0 ? 0.0 : (food > 1.0 ? 1.0 : food);
          reward += p.r_eat;
          bool logged = true;
          if (found >= 0 && found < 4) {  // (entries 0..3 live in registers)
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (found == k) lrem[k] = (uint32_t)(rem - 1);
          } else if (found >= 4) {  // (HBM written through: the state at the launch's end)
            if (found < kWideRollLog) elrem[(found - 4) * 64 + lane] = (uint8_t)(rem - 1);
            p.eaten_rem[(int64_t)found * p.B + g] = (uint8_t)(rem - 1);
          } else if (ne < p.eaten_cap) {
            if (ne < 4) {
#pragma unroll
              for (int k = 0; k < 4; ++k)
                if (ne == k) {
                  lxy[k] = h.cpos;
                  lrem[k] = (uint32_t)(rem - 1);
                }
            } else {
              if (ne < kWideRollLog) {
                elxy[(ne - 4) * 64 + lane] = h.cpos;
                elrem[(ne - 4) * 64 + lane] = (uint8_t)(rem - 1);
              }
              p.eaten_xy[(int64_t)ne * p.B + g] = h.cpos;
              p.eaten_rem[(int64_t)ne * p.B + g] = (uint8_t)(rem - 1);
            }
            ne += 1;
          } else {
            eaten_of += 1;
            logged = false;
          }
          if (rem == 1) {
            emptied = true;
            if (logged) ndep += 1;
          }
        }
        food = food - p.hunger;  // :316-322
        const bool starved = food <= 0.0;
        if (starved) food = 0.0;
        status = starved ? 1 : kill ? 2 : status_old;
        const bool done = starved || kill || status_old != 0 || h.turn >= p.max_turns;
        {
          const double r_finish = sreg(p.r_finish), r_turn = sreg(p.r_turn);
          const double r_starve = sreg(p.r_starve), r_killed = sreg(p.r_killed);
          reward += sel_f64(status == 0, sel_f64(done, r_finish, r_turn), sel_f64(status == 1, r_starve, r_killed));
        }
        job = done && p.autoreset;
        __builtin_nontemporal_store((float)reward, p.reward + g);
        __builtin_nontemporal_store((uint8_t)(done ? 1 : 0), p.done + g);
        if (!job) {
          p.food_turns[g] = (uint8_t)(int)ceil(food * (double)p.turns_empty);  // :450-452
          p.role[g] = (uint8_t)h.role;
          p.status[g] = (uint8_t)status;
        }
        if (!h.valid_action) atomicAdd(&p.counters[CTR_BAD_ACTIONS], 1ull);
      }
      info[lane] = (job ? 1u : 0u) | (emptied ? 2u : 0u);
      const unsigned long long jm = __ballot(job);
      if (job) {
        const int j = __popcll(jm & ((1ull << lane) - 1ull));
        const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));
        jobEnv[j] = (uint32_t)lane;
        *reinterpret_cast<uint2*>(&jobKey[2 * j]) = make_uint2((uint32_t)ek2, (uint32_t)(ek2 >> 32));
      }
      if (lane == 0) {
        blk[0] = (uint32_t)__popcll(jm);
        blk[1] = (uint32_t)jm;
        blk[2] = (uint32_t)(jm >> 32);
      }
      ROLLW_STAMP(4);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_publish_step(flag + 2, at_b2);
      lds_barrier();  // B2
      ROLLW_STAMP(5);
      // ------------------------------------------------ W0 P2: spawns; the next state of continuing envs
      if (active && !job) {
        int n_unplaced = 0;
        if (p.wolves_on) {
          for (int w = 0; w < RW; ++w) {
            uint32_t bits = spawn[(uint32_t)lane * L.spw + (uint32_t)w];
            while (bits) {
              const int b = __ffs(bits) - 1;
              bits &= bits - 1;
              const uint32_t tt = xy_add(h.cpos, ring[32 * w + b]);
              bool placed = false;
#pragma unroll
              for (int k = 0; k < SLOTS; ++k)
                if (!placed && !((live >> k) & 1u)) { wr[k] = tt; live |= 1u << k; placed = true; }
              n_unplaced += placed ? 0 : 1;
            }
          }
        }
        // the HBM rows: survivors compacted (row k read before any row >= its new index is
        // written), then the spawns that found no register slot, up to the cap
        int n = __popc(live);
        int ns = 0;
        for (uint32_t bits = spill_live; bits; bits &= bits - 1u) {
          const int k = SLOTS + __ffs(bits) - 1;
          if (k != SLOTS + ns) p.wolves[(int64_t)(SLOTS + ns) * p.B + g] = p.wolves[(int64_t)k * p.B + g];
          ns += 1;
        }
        n += ns;
        if (n_unplaced) {
          int skip = -n_unplaced;
          for (int w = 0; w < RW; ++w)
            for (uint32_t bits = spawn[(uint32_t)lane * L.spw + (uint32_t)w]; bits; bits &= bits - 1u) skip += 1;
          for (int w = 0; w < RW && n_unplaced; ++w) {
            for (uint32_t bits = spawn[(uint32_t)lane * L.spw + (uint32_t)w]; bits; bits &= bits - 1u) {
              if (skip > 0) { skip -= 1; continue; }
              const uint32_t tt = xy_add(h.cpos, ring[32 * w + __ffs(bits) - 1]);
              if (n < p.wolf_cap) {
                p.wolves[(int64_t)(SLOTS + ns) * p.B + g] = tt;
                ns += 1;
                n += 1;
              } else {
                wolf_of += 1;
              }
            }
          }
        }
        nsp = ns;
        hdr = make_uint4(h.cpos, (uint32_t)h.turn,
                         misc_pack((uint32_t)h.role, (uint32_t)status, (uint32_t)n, (uint32_t)ne, (uint32_t)ndep),
                         h.hdr.w);
        nhdr[lane] = hdr;
        if (last) {  // the state, compacted as the per-step kernel leaves it
          int m = 0;
#pragma unroll
          for (int k = 0; k < SLOTS; ++k)
            if ((live >> k) & 1u) p.wolves[(int64_t)(m++) * p.B + g] = wr[k];
          for (int i = 0; i < nsp; ++i)  // (m <= SLOTS: row SLOTS + i read before row m + i is written)
            if (m < SLOTS) p.wolves[(int64_t)(m + i) * p.B + g] = p.wolves[(int64_t)(SLOTS + i) * p.B + g];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < ne && i < p.eaten_cap) {
              p.eaten_xy[(int64_t)i * p.B + g] = lxy[i];
              p.eaten_rem[(int64_t)i * p.B + g] = (uint8_t)lrem[i];
            }
          p.hdr[g] = hdr;
          p.food[g] = food;
        }
      }
      __builtin_amdgcn_s_setprio(0);
    } else if (wave == 1) {
      // ---------------------------------------------- W1 P0: the view bitmap
      __builtin_amdgcn_s_setprio(2);
      // source: the last step's bitmaps (step 0: the state's, loaded with the header)
      uint32_t* src = bm_prev;
      // the last step's eaten-empty centre tile of a continuing env (its obs were pre-eat S),
      // applied to the source's centre row as it is read
      bool eaten_empty = false;
      if (t > 0) {
        const unsigned long long jmp = (unsigned long long)blk[1] | ((unsigned long long)blk[2] << 32);
        eaten_empty = active && !((jmp >> lane) & 1ull) && (info[lane] & 2u);
      }
      const uint32_t ccw = eaten_empty ? ~(1u << p.ch) : ~0u;
      const uint32_t strip = active ? strip_bits(p, h) : 0u;  // generate_bushes (:613-629)
      const uint32_t hmask = p.H >= 32 ? ~0u : ((1u << p.H) - 1u);
      const uint32_t top = 1u << (p.H - 1);
      const int Wv = p.W, cwv = p.cw;
      uint32_t prev_old = 0u;                   // the old row i - 1
      uint32_t nxt = active ? src[me] & (cwv == 0 ? ccw : ~0u) : 0u;  // the old row i
#pragma unroll 1
      for (int i0 = 0; i0 < Wv; i0 += 4) {  // scroll (:613-629) + the entering strip
        uint32_t old[5];
        old[0] = nxt;
#pragma unroll
        for (int q = 1; q < 5; ++q)
          old[q] = (active && i0 + q < Wv) ? src[me + (uint32_t)(i0 + q)] & (i0 + q == cwv ? ccw : ~0u) : 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = i0 + q;
          if (i >= Wv) break;
          const uint32_t wi = old[q];
          const uint32_t prev = q == 0 ? prev_old : old[q - 1];
          const uint32_t next = old[q + 1];
          const uint32_t sb = (strip >> i) & 1u;
          uint32_t v = wi;
          v = h.dir == DIR_RIGHT ? (i == 0 ? strip : prev) : v;
          v = h.dir == DIR_LEFT ? (i == Wv - 1 ? strip : next) : v;
          v = h.dir == DIR_UP ? (((wi << 1) & hmask) | sb) : v;
          v = h.dir == DIR_DOWN ? ((wi >> 1) | (sb ? top : 0u)) : v;
          bm[me + (uint32_t)i] = active ? v : 0u;
        }
        prev_old = old[3];
        nxt = old[4];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) lds_publish_step(flag, (uint32_t)t + 1u);  // (W0 clears the emptied tiles)
      ROLLW_STAMP(9);
      uint32_t cv = 0;  // the generated berries of the ostrich's tile (:631-635), for W0 (unused
                        // when W0 clears that tile: it is then in the log with no berries)
      if (active && ((bm[me + (uint32_t)p.cw] >> p.ch) & 1u))
        cv = (uint32_t)bush_value_fast(thr, p.max_berries, draw_U(h.cpos, make_ts(SITE_BUSH, 0, 0), h.b0, h.b1),
                                       p.bush_power);
      cval[lane] = cv;
      __builtin_amdgcn_s_setprio(0);
      ROLLW_STAMP(10);
      lds_barrier();  // B1
      ROLLW_STAMP(11);
      {
        const bool rest = t > 0 ? drain_rows(p, qp, lane, flag + 2, at_b2) : true;  // (idle until B2: store)
        if (last && rest) drain_plane2(p, flag + 6, n_active, out, lane, flag + 2, at_b2);
      }
      lds_barrier();  // B2
      ROLLW_STAMP(12);
    } else {
      // ---------------------------------------------- W2, W3: the store waves (step 0: W2 loads
      // the spawn tables for W0 first)
      // Issue priority rotating over the four co-resident workgroups of a CU (blockIdx b,
      // b + 256, b + 512, b + 768, dispatched in that order): at equal priority the arbiter
      // favours the oldest wave, so the youngest group's stores fell behind and its CU ran the
      // launch's tail alone (group durations by dispatch quarter 1720, 1930, 2170, 2440 us;
      // rotating: 1965, 2070, 2174, 2304).  C3 T = 64: 2728-2737 -> 2618-2628 us per launch
      // (tools/ab_wide.sh; every wave rotating: 2609-2633; static inverse-age priority 2786).
      // (one-step launches: priority = age, the youngest first; 59.1 us per step into a ring,
      // against 63.2 at priority 0 and 63.5 oldest first).  The 256 is MI355X's CU count
      // (one group per CU per dispatch round); elsewhere only the hint changes, not results.
      set_prio_dyn(((blockIdx.x >> 8) + (uint32_t)t) & 3u);
      if (wave == 2 && t == 0) {
        copy_to_lds(ring, p.tables + p.ring_at, (p.R + 3) & ~3, lane);
        if (p.wolves_on) copy_to_lds(gap, p.gap, p.n_gap + 1, lane);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) lds_publish_step(flag + 1, 1u);  // (W0 waits for the tables once)
      }
      ROLLW_STAMP(8 * wave + 1);
      {
        const bool rest = t > 0 ? drain_rows(p, qp, lane, flag + 2, at_b1) : true;  // step t - 1's rows until W0 reaches B1
        if (last && rest) drain_plane2(p, flag + 6, n_active, out, lane, flag + 2, at_b1);
      }
      ROLLW_STAMP(8 * wave + 2);
      lds_barrier();  // B1
      if (wave == 3 && !last) wide_prefetch_actions(p, act, lane);  // (read after this step's end)
      {
        const bool rest = t > 0 ? drain_rows(p, qp, lane, flag + 2, at_b2) : true;  // ... until W0 reaches B2
        if (last && rest) drain_plane2(p, flag + 6, n_active, out, lane, flag + 2, at_b2);
      }
      ROLLW_STAMP(8 * wave + 3);
      lds_barrier();  // B2
      if (t > 0) drain_rows(p, qp, lane);  // ... the rest, while W0 and W1 build the new episodes
      if (last) drain_plane2(p, flag + 6, n_active, out, lane);
      if (last) drain_rows(p, untouched_rows(p, flag + 4 + cur, n_rows, bm, wp, out, blk), lane);
      ROLLW_STAMP(8 * wave + 4);
    }

    const int n_jobs = (int)blk[0];
    const unsigned long long jmask = (unsigned long long)blk[1] | ((unsigned long long)blk[2] << 32);
    if (wave == 0) {
      if (eaten_of) atomicAdd(&p.counters[CTR_EATEN_OVERFLOW], eaten_of);
      if (lane == 0 && n_jobs) atomicAdd(&p.block_resets[blockIdx.x], (unsigned long long)n_jobs);
      count_steps(p);
    }
    if (n_jobs > 0 && wave < 2) {
      // ------------------------------------------------ done envs: new episodes (:231-248), by W0
      // and W1 (the store waves keep storing): reset draws (generate_bushes) over the new view,
      // ostrich at (0, 0), 32 lanes per row, rows written by ballot into this step's bitmaps;
      // initialize_wolves (:578-593): the view's spawn set at turn 0, by the job's own lane of W0
      const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0);
      const uint32_t rows2 = ((uint32_t)p.W + 1u) >> 1;
      for (int jj = 0; jj < n_jobs; ++jj) {
        const uint32_t e = jobEnv[jj];
        const uint2 kq = *reinterpret_cast<const uint2*>(&jobKey[2 * jj]);
        for (uint32_t r2 = (uint32_t)wave; r2 < rows2; r2 += 2u) {
          const uint32_t i = 2u * r2 + ((uint32_t)lane >> 5), j = (uint32_t)lane & 31u;
          const bool cell = i < (uint32_t)p.W && j < (uint32_t)p.H;
          const uint32_t xy = xy_pack(p.cw - (int)i, p.ch - (int)j);
          const uint32_t h1 = fmix32(xy ^ kq.x);
          const uint32_t hb = fmix32(h1 ^ ts_bush ^ kq.y);
          const bool bush = cell && U_ge(h1, hb, ts_bush, kq.x, p.bush_th, p.bush_tl);
          const unsigned long long bb = __ballot(bush);
          if ((lane & 31) == 0 && i < (uint32_t)p.W) bm[e * P + i] = (uint32_t)(lane ? bb >> 32 : bb);
        }
      }
      if (wave == 0 && active && ((jmask >> lane) & 1ull)) {
        // spawn_ostriches (:595-611) and the initial wolves, one per wolf cell of the view
        const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));
        const uint32_t kb0 = (uint32_t)ek2, kb1 = (uint32_t)(ek2 >> 32);
        for (int i = 0; i < p.W; ++i) wp[me + (uint32_t)i] = 0u;
        if (p.wolves_on)
          spawn_hits(gap, p.WH, p.gap_full_th, p.gap_full_tl, p.gap_view_th, p.gap_view_tl, p.gap_inv_l2, 0, kb0, kb1,
                     [&](int c) {
                       const uint32_t i = (uint32_t)c / (uint32_t)p.H;
                       wp[me + i] |= 1u << ((uint32_t)c - i * (uint32_t)p.H);
                     });
        const double food2 = p.start_food_random
                                 ? (double)draw_U(xy_pack(0, 0), make_ts(SITE_START_FOOD, 0, 0), kb0, kb1) * 0x1p-53
                                 : p.start_food;
        const int role2 = p.start_role_random
                              ? (int)(draw_U(xy_pack(0, 0), make_ts(SITE_START_ROLE, 0, 0), kb0, kb1) >> 52)
                              : p.start_role;
        int n = 0;
        live = 0u;
        for (int i = 0; i < p.W; ++i) {
          uint32_t bits = wp[me + (uint32_t)i];
          while (bits) {
            const int j = __ffs(bits) - 1;
            bits &= bits - 1;
            const uint32_t tt = xy_pack(p.cw - i, p.ch - j);
            if (n < SLOTS) {
              slot_set<SLOTS>(wr, n, tt);
              live |= 1u << n;
              if (last) p.wolves[(int64_t)n * p.B + g] = tt;
              n += 1;
            } else if (n < p.wolf_cap) {
              p.wolves[(int64_t)n * p.B + g] = tt;
              n += 1;
            } else {
              wolf_of += 1;
              atomicAdd(&p.counters[CTR_WOLF_OVERFLOW_RESET], 1ull);
            }
          }
        }
        nsp = n > SLOTS ? n - SLOTS : 0;
        food = food2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          lxy[i] = 0u;
          lrem[i] = 0u;
        }
        hdr = make_uint4(xy_pack(0, 0), 0u, misc_pack((uint32_t)role2, 0u, (uint32_t)n, 0u, 0u), h.hdr.w + 1u);
        nhdr[lane] = hdr;
        p.food_turns[g] = (uint8_t)(int)ceil(food2 * (double)p.turns_empty);
        p.role[g] = (uint8_t)role2;
        p.status[g] = 0;
        if (last) {
          p.hdr[g] = hdr;
          p.food[g] = food2;
        }
      }
    }
    if (wave < 2) {  // W0 and W1 are done with the step: they store too
      if (t > 0) drain_rows(p, qp, lane);
      if (last) drain_plane2(p, flag + 6, n_active, out, lane);
      if (last) drain_rows(p, untouched_rows(p, flag + 4 + cur, n_rows, bm, wp, out, blk), lane);
    }
    if (wave == 0) ROLLW_STAMP(39);
    if (wave == 0 && wolf_of) atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], wolf_of);
    lds_barrier();  // the step's end: its obs buffers are complete; the next step's inputs are in
#ifdef WAB_STAMPS
    if (tid == 0 && p0.stamps && t == T / 2)  // past the middle step's end barrier
      p0.stamps[(size_t)blockIdx.x * kStampStride + 38] = __builtin_amdgcn_s_memrealtime();
#endif
    if (last) {
      // the last step's obs lines that touch a done env (its new episode, its neighbours' S), by
      // all 256 threads; every env's bitmap rows (continuing: post-eat; done: the new episode's)
      if (jmask) {
        RowCursor c = row_cursor(p, (uint32_t)tid);
        while (c.q < n_rows) roll_store_row_if<256>(p, bm, wp, out, c, jmask, true);
      }
      for (uint32_t u = tid; u < 64u * 32u; u += 256) {
        const uint32_t e = u >> 5, i = u & 31u;
        if ((int)e >= n_active || i >= (uint32_t)p.W) continue;
        uint32_t v = bm[e * P + i];
        if (!((jmask >> e) & 1ull) && (info[e] & 2u) && i == (uint32_t)p.cw) v &= ~(1u << p.ch);
        p.bushmap[(size_t)(g0 + e) * 32u + i] = v;
      }
    }
  }
#ifdef WAB_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && p0.stamps)  // every store of the workgroup retired (slot 34)
    p0.stamps[(size_t)blockIdx.x * kStampStride + 34] = __builtin_amdgcn_s_memrealtime();
#endif
}

template __global__ void wab_rollout_wide<8, 0>(Params);
template __global__ void wab_rollout_wide<8, 31>(Params);

#define WAB_WIDE_INST(M, S) template __global__ void wab_step_wide<M, S>(Params);
WAB_WIDE_INST(MODE_STEP, 8)
WAB_WIDE_INST(MODE_RESET, 8)

}  // namespace wab
