// wab_step_small.hip — the fused step for small views (W*H <= 128 bits, S == H, spawn ring
// <= 128 tiles; the default 11x11 options).
//
// The step is bound by its per-env dependency chain and by VALU issue: a lone wave issues at
// best one instruction every ~4-5 cycles (twice that along a dependent chain;
// tools/micro/valu_latency.hip), the kernel at batch 4096 takes nearly as long as at 65536,
// and at 65536 (four waves per SIMD) the VALU pipe is busy about half of a workgroup's life,
// the rest being load latency and barrier waits (profiles/r01_small).  Each
// 64-env group (one env per lane) is served by four waves of one 256-thread workgroup, each
// running an independent part of the step; they meet at LDS barriers:
//
//          W0 bushes             W1 draws              W2 wolves             W3 ring
//   init   state + first eaten-  thresholds -> LDS     wolf slots, header    tile + gap tables
//          log loads                                                         -> LDS
//   -- B_init --
//   P0     scroll, log, eat,     the ostrich tile's    despawn, pursuit,     the ring's spawn
//          hunger, starve        value (LDS flag)      wolf grid of S, kill  set, entering
//                                                                            row/column draws
//   -- B1 --
//   P1     status, reward,       reset draws (cells    spawns, wolf slots,   reset draws (the
//          done, scalars,        0..63, LDS flag),     header                rest), new episodes
//          bushes, food          render S
//   -- B2 --  (B3: terminal obs, W0 copies S out and builds the new episodes)
//   all: obs bit-stream -> bytes, 16-byte stores
//
// FEAT (wab_step_features): W1 and W3 also store the all-zero view-mask lines of the feature
// rows right after B_init; after B2 W0-W2 compute the features from the bit-stream, one more
// barrier, and all threads store the float32 rows (the planes only if asked for).
//
// Every wave that needs "done" recomputes it from the flags handed over at B1 (starved from
// W0, killed from W2), so no wave waits for another's bookkeeping.  Draws are batched four
// at a time (fmix32x4) so dependent hash chains interleave; the rare threshold ties (high
// 32 bits equal) are resolved in a separate branch.  Wolf spawns are keyed sets
// (wab_device.h spawn_hits): one draw per env-step and per new episode unless a wolf spawns.
#include <hip/hip_runtime.h>

#include "wab_feat.h"

#ifndef WAB_ROLL_THROTTLE  // (tuning A/B: 1 = W0 / W2 drain their obs stores at each step's start)
#define WAB_ROLL_THROTTLE 0
#endif
#ifndef WAB_ROLL_OBS_NT  // (tuning A/B: 0 = plain obs stores in multi-step launches)
#define WAB_ROLL_OBS_NT 1
#endif
namespace wab {

// Diagnostic build (-DWAB_STAMPS): lane 0 of each wave records s_memrealtime (100 MHz) at
// phase boundaries into p.stamps[workgroup * kStampStride + slot] (W0 0..9, W1 10..15, W2 16..21, W3 22..27):
// a wave's stamps k, k+1, k+2, k+3 close its phases P0..P3 (the barrier waits sit at the
// start of the next phase), the last one the retirement of its obs stores.
#ifdef WAB_STAMPS
#define SMALL_STAMP(slot)                                                                \
  do {                                                                                   \
    if (lane == 0 && p.stamps && (!ROLL || t == p.n_steps / 2))                          \
      p.stamps[(size_t)blockIdx.x * kStampStride + (slot)] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#else
#define SMALL_STAMP(slot) do {} while (0)
#endif

namespace {

__device__ __forceinline__ void set_bit_if(M128& m, uint32_t c, bool on) {
  const uint64_t b = on ? 1ull << (c & 63u) : 0ull;
  m.lo |= c < 64u ? b : 0ull;
  m.hi |= c < 64u ? 0ull : b;
}
__device__ __forceinline__ uint4 m_pack(const M128& m) {
  return make_uint4((uint32_t)m.lo, (uint32_t)(m.lo >> 32), (uint32_t)m.hi, (uint32_t)(m.hi >> 32));
}
__device__ __forceinline__ M128 m_unpack(const uint4& v) { return m_make(v.x, v.y, v.z, v.w); }

// The part of the state every wave reads: header and action, the move (:252-258), the key.
struct Head {
  bool active, valid_action;
  uint4 hdr;
  int32_t ox, oy, turn;
  int dir, role;
  uint32_t cpos;
  uint64_t kenv;
};

// The header and action loads (head_fetch) are issued together with the rest of a wave's
// loads, and decoded (head_decode) only after all of them are in flight: a use between two
// groups of loads makes the second group wait a full memory round trip for the first.
struct HeadRaw {
  uint4 hdr;
  int a;
};
// (loads are unconditional, from env 0 for an inactive lane, so that no branch splits a
// wave's loads; head_decode zeroes an inactive lane's header)
__device__ __forceinline__ HeadRaw head_fetch(const Params& p, int64_t g, bool active) {
  const int64_t gl = active ? g : 0;
  HeadRaw r;
  r.hdr = p.hdr[gl];
  r.a = (int)p.actions[gl];
  return r;
}

__device__ __forceinline__ void opaque_head(HeadRaw& r) {
  opaque(r.hdr.x);
  opaque(r.hdr.y);
  opaque(r.hdr.z);
  opaque(r.hdr.w);
  opaque(r.a);
}

__device__ __forceinline__ Head head_decode(const Params& p, int64_t g, bool active, const HeadRaw& r) {
  Head h;
  h.active = active;
  h.hdr = active ? r.hdr : make_uint4(0u, 0u, 0u, 0u);
  const int a = active ? r.a : 0;
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
  return h;
}

// done (:328-340) from the flags of B1: starve overrides kill, which overrides the old status
__device__ __forceinline__ bool env_done(const Params& p, const Head& h, bool starved, bool killed) {
  return starved || killed || misc_status(h.hdr.z) != 0 || h.turn >= p.max_turns;
}

// Geometry specialisation.  G = 11 is the default options' geometry (11x11 view in 11-byte
// rows, wolf_spawn_margin 1: a 48-tile ring); G = 0 reads everything from the parameter block.
// With G = 11 the geometry fields are compile-time constants (specialise_geometry) and the ring
// offsets are immediates instead of scalar loads from the tile table (each a wait on the scalar
// cache inside the ring loop); fewer live uniform values also cut the SGPR spills.
template <int G>
__device__ __forceinline__ void specialise_geometry(Params& p) {
  if constexpr (G == 11) {
    p.W = 11; p.H = 11; p.S = 11; p.cw = 5; p.ch = 5; p.margin = 1;
    p.OB = 363; p.WH = 121; p.R = 48; p.NT = 169; p.RW = 2; p.WHW = 4; p.SL = 11;
    p.ring_at = 124;
    p.n_gap = kGapChunk;
    p.small_masks[0][0] = 0x00400801u; p.small_masks[0][1] = 0x00801002u;  // column 0 (j = 0)
    p.small_masks[0][2] = 0x01002004u; p.small_masks[0][3] = 0x00004008u;
    p.small_masks[1][0] = 0x00200400u; p.small_masks[1][1] = 0x00400801u;  // column H-1
    p.small_masks[1][2] = 0x00801002u; p.small_masks[1][3] = 0x01002004u;
    p.small_masks[2][0] = ~0u; p.small_masks[2][1] = ~0u; p.small_masks[2][2] = ~0u;
    p.small_masks[2][3] = (1u << 25) - 1u;
  }
}

// spawn-ring tile r of the G = 11 geometry: the host's table order (wab_create), the 13-wide
// bands y = 0 and y = 12 first, then the x = 0 / x = 12 columns of rows 1..11
__host__ __device__ constexpr uint32_t ring11(int r) {
  const int xi = r < 26 ? r % 13 : ((r - 26) / 11 < 1 ? 0 : 12);
  const int yi = r < 26 ? (r / 13 < 1 ? 0 : 12) : 1 + (r - 26) % 11;
  return ((uint32_t)(xi - 6) & 0xFFFFu) | ((uint32_t)(yi - 6) << 16);
}

// reset draws (generate_bushes) of jobs [j0, j0 + K) for view cell c (xy its world offset)
template <int K>
__device__ __forceinline__ void reset_draws(const Params& p, const uint32_t* jkey, int j0, uint32_t xy, uint32_t c,
                                            uint32_t* jbm) {
  const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0);
  uint32_t kb0[K], h1[K], hb[K];
#pragma unroll
  for (int q = 0; q < K; ++q) {
    const uint2 kq = *reinterpret_cast<const uint2*>(&jkey[2 * (j0 + q)]);
    kb0[q] = kq.x;
    h1[q] = xy ^ kq.x;
    hb[q] = ts_bush ^ kq.y;
  }
  fmix32xk<K>(h1);
#pragma unroll
  for (int q = 0; q < K; ++q) hb[q] ^= h1[q];
  fmix32xk<K>(hb);
  if (c < (uint32_t)p.WH) {
#pragma unroll
    for (int q = 0; q < K; ++q)
      if (U_ge(h1[q], hb[q], ts_bush, kb0[q], p.bush_th, p.bush_tl))
        atomicOr(&jbm[(j0 + q) * 4 + (c >> 5)], 1u << (c & 31));
  }
}

// reset draws (generate_bushes) of every job for view cells c = c0 + lane, into the jobs'
// bush bitmaps (the initial wolves are a spawn set: new_episode); jobs four, then two, then
// one at a time (a group has 1.6 jobs on average: no draw is made for a job that is absent)
__device__ __forceinline__ void reset_chunk(const Params& p, const uint32_t* tiles, const uint32_t* jkey, int n_jobs,
                                            uint32_t c0, int lane, uint32_t* jbm) {
  const uint32_t c = c0 + (uint32_t)lane;
  const uint32_t xy = c < (uint32_t)p.WH ? tiles[c] : 0u;  // ostrich at (0, 0)
  int j = 0;
  for (; j + 4 <= n_jobs; j += 4) reset_draws<4>(p, jkey, j, xy, c, jbm);
  if (n_jobs - j >= 2) {
    reset_draws<2>(p, jkey, j, xy, c, jbm);
    j += 2;
  }
  if (n_jobs - j == 1) reset_draws<1>(p, jkey, j, xy, c, jbm);
}

// the row or column that scrolled into view (generate_bushes :613-629): bit k is the bush
// presence of its cell k (x moves: row i0, cell (i0, k); y moves: column j0, cell (k, j0)),
// for the cells [c0, c1) (multiples of 4).  Consecutive cells are one tile apart, so their
// packed tiles are one packed 16-bit add from the first.
__device__ __forceinline__ uint32_t strip_draws(const Params& p, const Head& h, uint32_t b0, uint32_t b1, int c0,
                                                int c1) {
  uint32_t hits = 0;
  if (h.dir != DIR_STAY) {
    const bool horiz = h.dir == DIR_RIGHT || h.dir == DIR_LEFT;
    const int n = horiz ? p.H : p.W;
    const int i0 = h.dir == DIR_LEFT ? p.W - 1 : 0, j0 = h.dir == DIR_DOWN ? p.H - 1 : 0;
    const uint32_t xy0 = horiz ? xy_pack(h.ox - (i0 - p.cw), h.oy + p.ch) : xy_pack(h.ox + p.cw, h.oy - (j0 - p.ch));
    const uint32_t ts = make_ts(SITE_BUSH, 0, 0), hk = ts ^ b1;
    for (int c = c0; c < min(c1, p.SL); c += 4) {
      uint32_t h1[4], hh[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // cell c + k: the first tile minus c + k in y (x moves) or x
        const uint32_t d = (uint32_t)(-(c + k)) & 0xFFFFu;
        h1[k] = xy_add(xy0, horiz ? d << 16 : d) ^ b0;
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
      if (tie) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (((tie >> k) & 1u) && draw_lo21(h1[k], ts, b0) >= p.bush_tl) hit |= 1u << k;
      }
      hits |= hit << c;
    }
    hits &= n >= 32 ? ~0u : (1u << n) - 1u;
  }
  return hits;
}

// the strip's bits (strip_draws) as view cells: row i0 is the bits [i0 H, i0 H + H), column
// j0 the bits k H + j0
__device__ __forceinline__ M128 strip_cells(const Params& p, int dir, uint32_t hits) {
  M128 m = {0ull, 0ull};
  if (!hits) return m;
  if (dir == DIR_RIGHT || dir == DIR_LEFT) {
    m.lo = hits;
    shl128(m.lo, m.hi, dir == DIR_LEFT ? (p.W - 1) * p.H : 0);
  } else {
    const uint32_t j0 = dir == DIR_DOWN ? (uint32_t)p.H - 1u : 0u;
    for (uint32_t b = hits; b; b &= b - 1u) m_set(m, (uint32_t)(__ffs(b) - 1) * (uint32_t)p.H + j0);
  }
  return m;
}

struct Lds {
  uint32_t* tiles;  // [WH] view-cell world offsets (reset draws, initial wolves)
  uint64_t* thr;    // [max_berries] bush thresholds (W1), padded (bush_thr_pads)
  uint64_t* gap;    // [n_gap + 1] spawn-set gap table (W3; read on a hit only)
  uint32_t* stream; // 64 envs x OB bits: bit k = byte k of the group's obs chunk
  uint32_t* cval;   // [64] generated berries of the ostrich's tile (W1), then flag[0] = 1
  uint32_t* flag;   // [0] tile values ready (W1), [1] W1's reset draws done; zeroed by W0
                    // before B_init
  uint4* wolfp;     // [64] wolf grid of S (W2, P0)
  uint32_t* kill;   // [64] (W2, P0)
  uint4* bushp;     // [64] bush grid of S without the entering strip (W0, P0)
  uint32_t* strip;  // [2][64] bush bits of the strip that scrolled into view (W1, W3; P0)
  uint4* gone;      // [64] emptied tiles in view (W0, P0): cleared from the strip too
  uint32_t* info;   // [64] starved | role << 8 | eaten << 16 | emptied << 24 (W0, P0)
  uint4* spawn;     // [64] ring spawn sets (W3)
  uint32_t* jbm;    // [job][4] reset bush bitmaps (W1, W3)
  uint32_t* jkey;   // [2][job][2] the new episodes' keys: W1's copy, W3's copy
  uint32_t* scal;   // [64] fused features: food_turns | role << 8 | status << 16 of the obs
  uint32_t* carry;  // [64][8] multi-step launches: a new episode's role | wolves << 8, food, wolf cells (W3)
  uint32_t* act;    // [16] multi-step launches: the next step's 64 actions (W1)
  uint8_t* rcode;   // [n_steps][64] wab_rollout_features with returns: each step's reward code (W0)
  uint32_t* wcar;   // [slots][64] multi-step launches of 32-slot handles: W2's wolf slots between steps
  uint32_t* elxy;   // [kSmallLog - 4][64] multi-step launches: eaten-log entries 4.. (W0)
  uint8_t* elrem;   // [kSmallLog - 4][64]
};

__device__ __forceinline__ Lds lds_of(uint32_t* lds, const SmallLayout& L) {
  Lds s;
  s.tiles = lds + L.tiles;
  s.thr = reinterpret_cast<uint64_t*>(lds + L.thr) + 1;
  s.gap = reinterpret_cast<uint64_t*>(lds + L.gap);
  s.stream = lds + L.stream;
  s.cval = lds + L.cval;
  s.flag = lds + L.flag;
  s.elxy = lds + L.elog;
  s.elrem = reinterpret_cast<uint8_t*>(lds + L.elog + (uint32_t)(kSmallLog - 4) * 64u);
  s.wolfp = reinterpret_cast<uint4*>(lds + L.wolfp);
  s.kill = lds + L.kill;
  s.bushp = reinterpret_cast<uint4*>(lds + L.bushp);
  s.strip = lds + L.strip;
  s.gone = reinterpret_cast<uint4*>(lds + L.gone);
  s.info = lds + L.info;
  s.spawn = reinterpret_cast<uint4*>(lds + L.spawn);
  s.jbm = lds + L.jbm;
  s.jkey = lds + L.jkey;
  s.scal = lds + L.scal;
  s.carry = lds + L.carry;
  s.act = lds + L.act;
  s.wcar = lds + L.wcar;
  s.rcode = reinterpret_cast<uint8_t*>(lds + L.rcode);
  return s;
}

__device__ __forceinline__ bool info_starved(uint32_t v) { return (v & 1u) != 0u; }

// (Measured and reverted: the key-only part of the new episodes on W0 after its own P1 work
// instead of on W3 before its wait for W1: 9.05 -> 9.57 us.)
// After B1 the new episodes (W3) are the longest chain: W3 is raised to the top issue
// priority there and W0 lowered (A/B at B = 65536: 10.05 -> 10.02 us); in multi-step launches
// W3 goes back to 0 when a step starts.  W1 runs its reset draws (which W3 waits for) at issue
// priority 2 in multi-step launches (6.41 -> 6.33 us per step; per-step launches: 9.16-9.19 vs
// 9.13 us without).  Measured and dropped: priority by workgroup age for the helper waves
// (+0.09 us), two or four groups per workgroup (one barrier for all: 11.2 / 12.1 us), the spawn
// sets' gap thresholds evaluated without a table (binary powering from 16 doubles in the kernel
// arguments: 11.1 us, more SGPR spills; from device memory: 14.0 us).
constexpr int kW1ResetPrio = 2;

// A wave's issue priority `level` (0..3, by its role).  In a wab_rollout_features launch
// (`rot`) the levels fold to two (0, 1) and a boost of 2 alternates step by step between the
// co-resident workgroups of a CU (blockIdx b, b + 256, ...: at equal priority the arbiter
// favours the oldest): C5 T = 64 23.84-23.87 -> 23.36-23.37 us per step; the plain rollout
// measured slower with it (5.70-5.75 -> 5.93-5.94), and with the four levels rotating, role
// ignored (C5 23.74-23.75, default 5.95-5.97).  blockIdx >> 8 is the dispatch round on
// MI355X's 256 CUs (one workgroup per CU per round); on a part with another CU count it is a
// different partition of the groups: a scheduling hint only, results do not depend on it.
template <bool ROLL>
__device__ __forceinline__ void role_prio(uint32_t level, int t, bool rot) {
  if (ROLL && rot)
    set_prio_dyn((level >= 2u ? 1u : 0u) + 2u * (((blockIdx.x >> 8) + (uint32_t)t) & 1u));
  else
    set_prio_dyn(level);
}
// the entering strip's cells are drawn in two parts, [0, kStripW1) on W1 after the tile value
// and the rest on W3 after the spawn set
constexpr int kStripW1 = 8;
__device__ __forceinline__ M128 strip_of(const Params& p, const Lds& s, int lane, int dir) {
  return strip_cells(p, dir, s.strip[lane] | s.strip[64 + lane]);
}

// scan eaten-log entries [i0, i0 + 4): the entry on the ostrich's tile, and the emptied
// tiles in view (absent from S, :506)
__device__ __forceinline__ void scan_log(const Params& p, const Head& h, const uint32_t* lxy, const uint32_t* lrem,
                                         int i0, int ne, int& found, int& found_rem, M128& gone) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool in = i0 + k < ne;
    const uint32_t v = lxy[k];
    const int r = (int)lrem[k];
    if (in && v == h.cpos) {
      found = i0 + k;
      found_rem = r;
    }
    const int ddx = h.ox - xy_x(v), ddy = h.oy - xy_y(v);
    set_bit_if(gone, (uint32_t)((ddx + p.cw) * p.H + ddy + p.ch), in && r == 0 && abs(ddx) <= p.cw && abs(ddy) <= p.ch);
  }
}

// the ostrich's own cell of an obs segment: one bit (mask_grid never blinds the centre, but
// the mask is applied all the same)
__device__ __forceinline__ void stream_set_ostrich(const Params& p, uint32_t* stream, uint32_t ebit, int role) {
  const uint32_t ccb = (uint32_t)(p.cw * p.H + p.ch);
  if (p.restrict_view && m_test(view_mask_of(p, role), ccb)) return;
  const uint32_t bit = ebit + 2u * (uint32_t)p.WH + ccb;
  atomicOr(&stream[bit >> 5], 1u << (bit & 31u));
}

// render S (:393-444) of one env into the bit-stream: the wolf grid (W2), the bush grid (W0,
// plus the entering strip, W1/W3, minus emptied tiles), the ostrich; mask_grid (:344-357) by
// the fresh role
__device__ __forceinline__ void render_s(const Params& p, const Lds& s, int lane, uint32_t info, int dir) {
  const uint32_t WH = (uint32_t)p.WH;
  const uint32_t ebit = (uint32_t)lane * (uint32_t)p.OB;
  const int role = (int)((info >> 8) & 0xFFu);
  M128 wp = m_unpack(s.wolfp[lane]);
  M128 bp = m_or(m_unpack(s.bushp[lane]), m_andn(strip_of(p, s, lane, dir), m_unpack(s.gone[lane])));
  if (p.restrict_view) {
    const M128 vm = view_mask_of(p, role);
    wp = m_andn(wp, vm);
    bp = m_andn(bp, vm);
  }
  if (wp.lo | wp.hi) stream_or128(s.stream, ebit, wp);  // (most envs see no wolf)
  stream_or128(s.stream, ebit + WH, bp);
  stream_set_ostrich(p, s.stream, ebit, role);
}

// (Measured and reverted: the obs units that touch no done env stored right after B1 by W0-W2
// while W3 builds the new episodes: 10.34 -> 12.02 us at B = 65536, the stores of all groups
// then share the HBM while W0-W2 still have to reach B2.)

// Multi-step launches (wab_rollout): NT threads (index idx) store NK units each (u = idx + NT
// * k) of a finished step's stream into `planes` (that step's slice), non-temporal, clearing
// each unit after its read so the stream can be rendered into again.  (Measured and not
// adopted: the store instructions aligned to absolute 128-byte lines, plain stores, the units
// in smaller read/clear/store batches; the obs stores split over W0, W2 and W3.)
template <int NT, int NK>
__device__ __forceinline__ void store_units_nt(const Params& p, uint8_t* planes, uint32_t* stream, int idx) {
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const uint32_t OB = (uint32_t)p.OB;
  const uint32_t full = ((uint32_t)min((int64_t)64, p.B - g0) * OB) >> 4;
  uint8_t* out = planes + (size_t)g0 * OB;
  uint16_t* s16 = reinterpret_cast<uint16_t*>(stream);
  uint32_t v[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const uint32_t u = (uint32_t)(idx + NT * k);
    v[k] = u < full ? (uint32_t)s16[u] : 0u;
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const uint32_t u = (uint32_t)(idx + NT * k);
    if (u < full) s16[u] = 0;
  }
  if (!planes) return;  // (wab_rollout_features without planes: the stream is only cleared)
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const uint32_t u = (uint32_t)(idx + NT * k);
    if (u >= full) continue;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 q;
#pragma unroll
    for (int b = 0; b < 4; ++b) q[b] = (((v[k] >> (4 * b)) & 0xFu) * 0x00204081u) & 0x01010101u;
    if (WAB_ROLL_OBS_NT) __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out) + u);
    else reinterpret_cast<u32x4*>(out)[u] = q;
  }
}

// Multi-step launches store step t's obs during step t + 1 (streams alternate), by W0 and W2 in
// their slack before B2 (W1 and W3 never store).  Diagnostic build -DWAB_ROLL_FLOOR=1: every
// step's work skipped, its obs stores kept (the store pattern's own floor; results wrong by design)
#ifndef WAB_ROLL_FLOOR
#define WAB_ROLL_FLOOR 0
#endif

// --------------------------------------------------------------------------- multi-step launches
// wab_rollout runs its T steps in one launch (ROLL): each wave keeps its part of an env's state
// in registers from one step to the next (its view of the header; W0 also the food, the view
// bitmap and the first four eaten-log entries; W2 the wolf slots, uncompacted, with a live
// mask), a done env's new episode comes from W3 through LDS (Lds::carry), the next step's
// actions from W1 through LDS (Lds::act, one scalar load per group).  Only the first step
// loads state from HBM and only the last stores it; in between, a step issues no vector load
// on its common path, so nothing waits for the previous step's obs stores to drain.
struct CarryHdr {
  uint4 hdr;  // the env's header at the start of the next step, as far as this wave uses it
};
struct CarryW0 {
  uint8_t* prev_planes;   // the previous step's obs slice and stream, or null
  uint32_t* prev_stream;
  uint4 hdr;
  double food;
  uint32_t bw[4];            // view bitmap (post-eat)
  uint32_t lxy[4], lrem[4];  // eaten-log entries 0..3 (4 .. kSmallLog - 1 in LDS, later ones in HBM)
};
template <int SLOTS>
struct CarryW2 {
  static constexpr int NR = carry_reg_slots(SLOTS);
  uint8_t* prev_planes;
  uint32_t* prev_stream;
  uint4 hdr;
  uint32_t wr[NR > 0 ? NR : 1];  // wolf tiles, uncompacted: slots 0 .. NR-1 (the rest in Lds::wcar)
  uint32_t live;       // occupied slots
};

template <typename C>
struct CarryPtr {  // (W1, W3: the loop's previous-step fields, unused by these waves)
  uint8_t* prev_planes;
  uint32_t* prev_stream;
  C c;
};

__device__ __forceinline__ int act_of(const Lds& s, int lane) {
  return (int)reinterpret_cast<const int8_t*>(s.act)[lane];
}

// the next step's actions of the group into Lds::act: one 64-byte scalar load (scalar loads
// count in lgkmcnt, so no wait on this wave's stores), spread over lanes 0..15; a partial or
// misaligned group reads per lane
__device__ __forceinline__ void prefetch_actions(const Params& p, const Lds& s, int lane) {
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
    if (lane < 16) s.act[lane] = d;
  } else {
    const int8_t v = g0 + lane < p.B ? a[lane] : (int8_t)0;
    reinterpret_cast<int8_t*>(s.act)[lane] = v;
  }
}

// a done env's new episode as W3 left it in Lds::carry (after B2)
struct NewEp {
  uint32_t role, nw;
  double food;
  M128 wolves;  // wolf cells of the view
};
__device__ __forceinline__ NewEp carry_of(const Lds& s, int lane) {
  const uint4 a = *reinterpret_cast<const uint4*>(&s.carry[8 * lane]);
  const uint4 b = *reinterpret_cast<const uint4*>(&s.carry[8 * lane + 4]);
  NewEp n;
  n.role = a.x & 0xFFu;
  n.nw = (a.x >> 8) & 0xFFu;
  n.food = __longlong_as_double((long long)((uint64_t)a.y | ((uint64_t)a.z << 32)));
  n.wolves = m_make(a.w, b.x, b.y, b.z);
  return n;
}
__device__ __forceinline__ uint4 new_header(const NewEp& n, const Head& h) {
  return make_uint4(xy_pack(0, 0), 0u, misc_pack(n.role, 0u, n.nw, 0u, 0u), h.hdr.w + 1u);
}

// The new episode of a done env (reset :231-248, spawn_ostriches :595-611) in two parts: A
// needs only the new key (state, scalars, initial wolves = the view's spawn set at turn 0,
// initialize_wolves :578-593, and the wolf and ostrich planes of its obs segment, which must
// be clear); B the job's reset bush draws (bushmap, bush plane).  Returns the new role.
template <int SLOTS, bool ROLL = false>
__device__ __forceinline__ int new_episode_a(const Params& p, const Lds& s, const Head& h, int64_t g, uint32_t kb0,
                                             uint32_t kb1, uint32_t ebit, unsigned long long& wolf_of,
                                             bool last = true) {
  const double food2 = p.start_food_random
                           ? (double)draw_U(xy_pack(0, 0), make_ts(SITE_START_FOOD, 0, 0), kb0, kb1) * 0x1p-53
                           : p.start_food;
  const int role2 = p.start_role_random
                        ? (int)(draw_U(xy_pack(0, 0), make_ts(SITE_START_ROLE, 0, 0), kb0, kb1) >> 52)
                        : p.start_role;
  M128 nwm = {0ull, 0ull};
  if (p.wolves_on)
    spawn_hits(s.gap, p.WH, p.gap_full_th, p.gap_full_tl, p.gap_view_th, p.gap_view_tl, p.gap_inv_l2, 0, kb0, kb1, [&](int c) { m_set(nwm, (uint32_t)c); });
  if (nwm.lo | nwm.hi) {
    const M128 wp = p.restrict_view ? m_andn(nwm, view_mask_of(p, role2)) : nwm;
    stream_or128(s.stream, ebit, wp);
  }
  stream_set_ostrich(p, s.stream, ebit, role2);
  const bool store = !ROLL || last;  // (ROLL: the state stays on chip until the last step)
  int n = 0;  // initial wolves, one per wolf cell of the view (slot order is irrelevant)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint64_t bits = half ? nwm.hi : nwm.lo;
    while (bits) {
      const int b = __ffsll((unsigned long long)bits) - 1;
      bits &= bits - 1;
      if (n < SLOTS) {
        if (store) p.wolves[(int64_t)n * p.B + g] = s.tiles[64 * half + b];
        n += 1;
      } else {
        wolf_of += 1;
        atomicAdd(&p.counters[CTR_WOLF_OVERFLOW_RESET], 1ull);
      }
    }
  }
  if (store) {
    p.hdr[g] = make_uint4(xy_pack(0, 0), 0u, misc_pack((uint32_t)role2, 0u, (uint32_t)n, 0u, 0u), h.hdr.w + 1u);
    p.food[g] = food2;
  }
  if constexpr (ROLL) {  // for the next step's waves (the wolves as cells: W2 takes the first SLOTS)
    const uint64_t fb = (uint64_t)__double_as_longlong(food2);
    uint32_t* c = &s.carry[8 * (int)(g & 63)];
    *reinterpret_cast<uint4*>(c) = make_uint4((uint32_t)role2 | ((uint32_t)n << 8), (uint32_t)fb, (uint32_t)(fb >> 32),
                                              m_word<0>(nwm));
    *reinterpret_cast<uint4*>(c + 4) = make_uint4(m_word<1>(nwm), m_word<2>(nwm), m_word<3>(nwm), 0u);
  }
  const uint32_t ft2 = (uint32_t)(int)ceil(food2 * (double)p.turns_empty);
  p.food_turns[g] = (uint8_t)ft2;
  p.role[g] = (uint8_t)role2;
  p.status[g] = 0;
  if (p.features) s.scal[(int)(g & 63)] = ft2 | ((uint32_t)role2 << 8);
  return role2;
}

__device__ __forceinline__ void new_episode_b(const Params& p, const Lds& s, int64_t g, int j, uint32_t ebit,
                                              int role2, bool store = true) {
  const M128 nbm = m_unpack(*reinterpret_cast<const uint4*>(&s.jbm[4 * j]));
  stream_or128(s.stream, ebit + (uint32_t)p.WH, p.restrict_view ? m_andn(nbm, view_mask_of(p, role2)) : nbm);
  if (!store) return;  // (ROLL: W0 takes the bitmap from jbm itself)
  p.bushmap[g] = m_word<0>(nbm);
  if (p.WHW > 1) p.bushmap[p.B + g] = m_word<1>(nbm);
  if (p.WHW > 2) p.bushmap[2 * p.B + g] = m_word<2>(nbm);
  if (p.WHW > 3) p.bushmap[3 * p.B + g] = m_word<3>(nbm);
}

// --------------------------------------------------------------------------- fused features: early lines
// The view-mask blocks of the feature rows are all zeros without restrict_view, known before
// the step has computed anything: the whole 128-byte lines inside them (wab_feat.h) are stored
// right after B_init by W1 (rows 0..31) and W3 (rows 32..63), while the HBM is otherwise idle,
// and the final store skips them.
__device__ __forceinline__ void early_view_zeros(const Params& p, uint32_t e0, uint32_t n_rows, int lane) {
  const uint32_t F = (uint32_t)pragmatic_dim(p.W / 2 + p.H / 2 + 1, p.turns_empty);
  view_zero_lines(p.features + (size_t)blockIdx.x * 64u * F, F, e0, n_rows, lane, 64);
}

// --------------------------------------------------------------------------- fused returns
// wab_rollout_features: each step W0 keeps its env's reward as a code in LDS (ate, the outcome,
// done), and after the last step runs finish_episode's scan over the launch's steps
// (actor_critic.py:139-143: R = r + gamma R from the last step back, restarted after every
// done, R_T = bootstrap or 0), in double from the reward's own terms, float32 out.  The same
// doubles as wab_discounted_returns_exact recovers from the float32 rewards, so the two agree
// bit for bit (and this one needs no unambiguous reward table).
__device__ __forceinline__ uint8_t reward_code(bool ate, int status, bool done) {
  const uint32_t outcome = status == 0 ? (done ? 1u : 0u) : status == 1 ? 2u : 3u;
  return (uint8_t)((ate ? 1u : 0u) | (outcome << 1) | (done ? 8u : 0u));
}

__device__ __forceinline__ void rollout_returns(const Params& p, const Lds& s, int64_t g, bool active, int lane) {
  if (!active) return;
  const double r_eat = p.r_eat, gamma = p.gamma;
  const double rx[4] = {p.r_turn, p.r_finish, p.r_starve, p.r_killed};
  double R = p.bootstrap ? (double)p.bootstrap[g] : 0.0;
  for (int t = p.n_steps - 1; t >= 0; --t) {
    const uint32_t c = s.rcode[64 * t + lane];
    const uint32_t o = (c >> 1) & 3u;
    const double x = o == 0u ? rx[0] : o == 1u ? rx[1] : o == 2u ? rx[2] : rx[3];
    // the step's reward as W0 summed it: 0 + r_eat (if it ate) + r_x (:299-340)
    const double r = (c & 1u) ? (0.0 + r_eat) + x : 0.0 + x;
    if (c & 8u) R = 0.0;
    R = r + gamma * R;  // (no contraction: -ffp-contract=off)
    p.returns[(int64_t)t * p.B + g] = (float)R;
  }
}

// --------------------------------------------------------------------------- W0: bushes
template <int SLOTS, int G, bool ROLL = false>
__device__ __forceinline__ unsigned long long bushes_wave(const Params& p, const SmallLayout& L, uint32_t* lds, int lane,
                                                          CarryW0* carry = nullptr, int t = 0, bool last = true) {
  const Lds s = lds_of(lds, L);
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const int64_t g = g0 + lane;
  const bool active = g < p.B;
  const uint32_t OB = (uint32_t)p.OB;
  const uint32_t ccb = (uint32_t)(p.cw * p.H + p.ch);  // the ostrich's cell

  SMALL_STAMP(0);
  // loads in one round trip (state and the first eaten-log entries, speculatively)
  double food = 0.0;
  uint32_t bw0 = 0u, bw1 = 0u, bw2 = 0u, bw3 = 0u;
  uint32_t lxy[4] = {0u, 0u, 0u, 0u}, lrem[4] = {0u, 0u, 0u, 0u};
  HeadRaw hr;
  if (ROLL && t > 0) {  // (multi-step launch: the state this wave carried from the last step)
    hr.hdr = carry->hdr;
    hr.a = act_of(s, lane);
    food = carry->food;
    bw0 = carry->bw[0];
    bw1 = carry->bw[1];
    bw2 = carry->bw[2];
    bw3 = carry->bw[3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lxy[i] = carry->lxy[i];
      lrem[i] = carry->lrem[i];
    }
  } else {
  hr = head_fetch(p, g, active);
  {  // (unconditional: an inactive lane reads env 0; entries at or past eaten_cap read the
     // last entry and are never used, entry i counts only below the log length <= cap)
    const int64_t gl = active ? g : 0;
    food = p.food[gl];
    bw0 = p.bushmap[gl];
    if (p.WHW > 1) bw1 = p.bushmap[p.B + gl];
    if (p.WHW > 2) bw2 = p.bushmap[2 * p.B + gl];
    if (p.WHW > 3) bw3 = p.bushmap[3 * p.B + gl];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t at = (int64_t)min(i, p.eaten_cap - 1) * p.B + gl;
      lxy[i] = p.eaten_xy[at];
      lrem[i] = p.eaten_rem[at];
    }
  }
  opaque_head(hr);
  opaque(food);
  opaque(bw0);
  opaque(bw1);
  opaque(bw2);
  opaque(bw3);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    opaque(lxy[i]);
    opaque(lrem[i]);
  }
  }
  if (!active) {  // (env 0's values: an inactive lane must not eat, log or store anything)
    food = 0.0;
    bw0 = bw1 = bw2 = bw3 = 0u;
  }
  // (multi-step launches after step 0: the stream was cleared by the threads that stored it,
  // the flags by W1 after B2, the LDS tables are still there: no B_init)
  const bool init = !ROLL || t == 0;
  if (init) {
    uint4* z = reinterpret_cast<uint4*>(s.stream);
    for (uint32_t i = lane; i < L.stream_words / 4u; i += 64) z[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  const Head h = head_decode(p, g, active, hr);
  if (lane == 0 && init) {
    s.flag[0] = 0u;
    s.flag[1] = 0u;
  }
  if (init) lds_barrier();  // B_init: the hand-off flags are clear
  int ne = (int)misc_ne(h.hdr.z), ndep = (int)misc_ndep(h.hdr.z);
  if (ROLL && t == 0) {  // entries 4 .. kSmallLog - 1 into LDS, for the whole launch
    for (int i = 4; i < kSmallLog; ++i)
      if (active && i < ne && i < p.eaten_cap) {
        s.elxy[(i - 4) * 64 + lane] = p.eaten_xy[(int64_t)i * p.B + g];
        s.elrem[(i - 4) * 64 + lane] = p.eaten_rem[(int64_t)i * p.B + g];
      }
    __builtin_amdgcn_s_waitcnt(0);  // (settled inside the branch: no vmcnt wait at the join)
  }
  const int status_old = (int)misc_status(h.hdr.z);
  const int role = h.role;
  M128 bm = m_make(bw0, bw1, bw2, bw3);  // scroll (generate_bushes keeps the tiles in view, :613-629)
  if (h.dir == DIR_RIGHT || h.dir == DIR_UP) shl128(bm.lo, bm.hi, h.dir == DIR_RIGHT ? p.H : 1);
  else if (h.dir == DIR_LEFT || h.dir == DIR_DOWN) shr128(bm.lo, bm.hi, h.dir == DIR_LEFT ? p.H : 1);
  {
    const M128 valid = m_make(sreg(p.small_masks[2][0]), sreg(p.small_masks[2][1]), sreg(p.small_masks[2][2]),
                              sreg(p.small_masks[2][3]));
    const M128 col0 = m_make(sreg(p.small_masks[0][0]), sreg(p.small_masks[0][1]), sreg(p.small_masks[0][2]),
                             sreg(p.small_masks[0][3]));
    const M128 coll = m_make(sreg(p.small_masks[1][0]), sreg(p.small_masks[1][1]), sreg(p.small_masks[1][2]),
                             sreg(p.small_masks[1][3]));
    const bool up = h.dir == DIR_UP, down = h.dir == DIR_DOWN;  // the entering column is dropped
    const M128 drop = {sel64(up, col0.lo, 0ull) | sel64(down, coll.lo, 0ull),
                       sel64(up, col0.hi, 0ull) | sel64(down, coll.hi, 0ull)};
    bm = m_andn(m_and(bm, valid), drop);
  }
  SMALL_STAMP(1);
  SMALL_STAMP(2);
  // eaten log: the berries left on the ostrich's tile, and emptied tiles that scrolled back
  // into view (absent from S, :506); the first entries whatever the tile holds (clearing an
  // emptied tile that is already absent changes nothing), the rest when it can matter.  The
  // entering strip (W3) never holds the ostrich's tile; `gone` clears it where it is read.
  int found = -1, found_rem = 0;
  M128 gone = {0ull, 0ull};
  scan_log(p, h, lxy, lrem, 0, ne, found, found_rem, gone);
  bm = m_andn(bm, gone);
  bool center_bush = m_test(bm, ccb);
  if (ne > 4 && (center_bush || (ndep > 0 && h.dir != DIR_STAY))) {
    // multi-step launches: entries 4 .. kSmallLog - 1 from LDS (a vector load here would wait
    // for every obs store the wave has in flight), later ones from HBM
    const int i_hbm = ROLL ? kSmallLog : 4;
    if (ROLL)
      for (int i0 = 4; i0 < ne && i0 < kSmallLog; i0 += 4) {
        uint32_t exy[4], erem[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          exy[k] = s.elxy[(i0 + k - 4) * 64 + lane];
          erem[k] = s.elrem[(i0 + k - 4) * 64 + lane];
        }
        scan_log(p, h, exy, erem, i0, ne, found, found_rem, gone);
      }
    for (int i0 = i_hbm; i0 < ne; i0 += 4) {
      uint32_t exy[4] = {0u, 0u, 0u, 0u}, erem[4] = {0u, 0u, 0u, 0u};  // (entries 0..3 stay in lxy, lrem)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i0 + k < ne) {
          exy[k] = p.eaten_xy[(int64_t)(i0 + k) * p.B + g];
          erem[k] = p.eaten_rem[(int64_t)(i0 + k) * p.B + g];
        }
      scan_log(p, h, exy, erem, i0, ne, found, found_rem, gone);
    }
    bm = m_andn(bm, gone);
    center_bush = m_test(bm, ccb);
  }
  SMALL_STAMP(7);
  s.bushp[lane] = m_pack(bm);  // bush grid of S (pre-eat) but the strip
  s.gone[lane] = m_pack(gone);
  int rem = found_rem;         // berries left: the log, else the generated value (W1)
  if (found < 0) {
    rem = 0;
    if (center_bush) {
      lds_await(p, s.flag);  // W1 publishes the values right after B_init
      rem = (int)s.cval[lane];
    }
  }
  SMALL_STAMP(8);
  double reward = 0.0;
  unsigned long long eaten_of = 0;
  const bool ate = rem > 0 && status_old == 0 && (role == 1 || p.lookout_only);
  if (ate) {  // eat (:299-313), stale status
    food = food + p.fill;
    food = food < 0.0 ? 0.0 : (food > 1.0 ? 1.0 : food);
    reward += p.r_eat;
    bool logged = true;
    if (ROLL && found >= 0 && found < 4) {  // (entries 0..3 live in registers)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (found == k) lrem[k] = (uint32_t)(rem - 1);
    } else if (ROLL && found < 0 && ne < 4 && ne < p.eaten_cap) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (ne == k) {
          lxy[k] = h.cpos;
          lrem[k] = (uint32_t)(rem - 1);
        }
      ne += 1;
    } else if (ROLL && found >= 4 && found < kSmallLog) {  // (entries 4.. in LDS)
      s.elrem[(found - 4) * 64 + lane] = (uint8_t)(rem - 1);
    } else if (ROLL && found < 0 && ne >= 4 && ne < kSmallLog && ne < p.eaten_cap) {
      s.elxy[(ne - 4) * 64 + lane] = h.cpos;
      s.elrem[(ne - 4) * 64 + lane] = (uint8_t)(rem - 1);
      ne += 1;
    } else if (found >= 0) {
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
      m_clear(bm, ccb);
      if (logged) ndep += 1;
    }
  }
  food = food - p.hunger;  // :316-322
  const bool starved = food <= 0.0;
  if (starved) food = 0.0;
  s.info[lane] = (starved ? 1u : 0u) | ((uint32_t)role << 8) | ((uint32_t)ne << 16) | ((uint32_t)ndep << 24);
  SMALL_STAMP(3);
  lds_barrier();  // B1: kill flags in; starve flags, bush grid and counts out
  role_prio<ROLL>(1, t, p.features != nullptr);

  // status (starve overrides kill), reward/done (:328-340), scalars, bushes and food
  const bool killed = s.kill[lane] != 0u;
  const int status = starved ? 1 : killed ? 2 : status_old;
  const bool done = env_done(p, h, starved, killed);
  {
    const double r_finish = sreg(p.r_finish), r_turn = sreg(p.r_turn);
    const double r_starve = sreg(p.r_starve), r_killed = sreg(p.r_killed);
    reward += sel_f64(status == 0, sel_f64(done, r_finish, r_turn), sel_f64(status == 1, r_starve, r_killed));
  }
  const bool job = active && done && p.autoreset;
  if (ROLL && p.returns)  // the step's reward as a code for the returns at the launch's end
    s.rcode[64 * t + lane] = reward_code(ate, status, done);
  if (active) {
    const int ft = (int)ceil(food * (double)p.turns_empty);  // :450-452
    __builtin_nontemporal_store((float)reward, p.reward + g);
    __builtin_nontemporal_store((uint8_t)(done ? 1 : 0), p.done + g);
    // a done env's own scalars go to the terminal side buffer (pointers chosen by masks: an
    // if/else of the two stores is merged into a scratch-indexed pointer pair)
    uint8_t* fts = reinterpret_cast<uint8_t*>(sel64(job, (uint64_t)p.t_food_turns, (uint64_t)p.food_turns));
    uint8_t* rls = reinterpret_cast<uint8_t*>(sel64(job, (uint64_t)p.t_role, (uint64_t)p.role));
    uint8_t* sts = reinterpret_cast<uint8_t*>(sel64(job, (uint64_t)p.t_status, (uint64_t)p.status));
    if (!job || (!ROLL && p.t_planes)) {
      fts[g] = (uint8_t)ft;
      rls[g] = (uint8_t)role;
      sts[g] = (uint8_t)status;
    }
    if (p.features && !job) s.scal[lane] = (uint32_t)ft | ((uint32_t)role << 8) | ((uint32_t)status << 16);
    if (!job) {
      bm = m_or(bm, m_andn(strip_of(p, s, lane, h.dir), gone));
      if (!ROLL || last) {
        p.bushmap[g] = m_word<0>(bm);
        if (p.WHW > 1) p.bushmap[p.B + g] = m_word<1>(bm);
        if (p.WHW > 2) p.bushmap[2 * p.B + g] = m_word<2>(bm);
        if (p.WHW > 3) p.bushmap[3 * p.B + g] = m_word<3>(bm);
        p.food[g] = food;
      }
    }
  }
  if (eaten_of) atomicAdd(&p.counters[CTR_EATEN_OVERFLOW], eaten_of);
  if (active && !h.valid_action) atomicAdd(&p.counters[CTR_BAD_ACTIONS], 1ull);
  count_steps(p);
  const unsigned long long jm = __ballot(job);
  if (lane == 0 && jm) atomicAdd(&p.block_resets[blockIdx.x], (unsigned long long)__popcll(jm));  // (no-return: a load here would wait for the stores)
  if (ROLL && carry->prev_stream) store_units_nt<128, 12>(p, carry->prev_planes, carry->prev_stream, lane);
  SMALL_STAMP(4);
  lds_barrier();  // B2: S rendered (done envs too when their terminal obs is asked for)
  if (!ROLL && p.t_planes) {  // (terminal obs: per-step launches only)
    // terminal obs: the step's own obs of every done env (bytes); then its new episode
    unsigned long long wolf_of = 0;
    if (jm) {
      uint8_t* tout = p.t_planes + (size_t)g0 * OB;
      for (unsigned long long jj = jm; jj; jj &= jj - 1) {
        const uint32_t ee = (uint32_t)(__ffsll(jj) - 1);
        for (uint32_t k = lane; k < OB; k += 64) {
          const uint32_t bit = ee * OB + k;
          tout[bit] = (uint8_t)((s.stream[bit >> 5] >> (bit & 31)) & 1u);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (job) {
        const uint32_t ebit = (uint32_t)lane * OB;
        stream_clear(s.stream, ebit, OB);
        const int j = __popcll(jm & ((1ull << lane) - 1ull));
        const uint2 kq = *reinterpret_cast<const uint2*>(&s.jkey[2 * j]);  // the new key (W1's copy)
        const int role2 = new_episode_a<SLOTS>(p, s, h, g, kq.x, kq.y, ebit, wolf_of);
        new_episode_b(p, s, g, j, ebit, role2);
      }
    }
    if (wolf_of) atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], wolf_of);
    lds_barrier();  // B3
  }
  if constexpr (ROLL) {
    if (!last) {  // this wave's state for the next step (a new episode's from W3 and jbm)
      if (job) {
        const NewEp n = carry_of(s, lane);
        const int j = __popcll(jm & ((1ull << lane) - 1ull));
        const uint4 nb = *reinterpret_cast<const uint4*>(&s.jbm[4 * j]);
        carry->hdr = new_header(n, h);
        carry->food = n.food;
        carry->bw[0] = nb.x;
        carry->bw[1] = nb.y;
        carry->bw[2] = nb.z;
        carry->bw[3] = nb.w;
      } else {
        carry->hdr = make_uint4(h.cpos, (uint32_t)h.turn, misc_pack((uint32_t)role, (uint32_t)status, 0u, (uint32_t)ne,
                                                                    (uint32_t)ndep), h.hdr.w);
        carry->food = food;
        carry->bw[0] = m_word<0>(bm);
        carry->bw[1] = m_word<1>(bm);
        carry->bw[2] = m_word<2>(bm);
        carry->bw[3] = m_word<3>(bm);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        carry->lxy[i] = lxy[i];
        carry->lrem[i] = lrem[i];
      }
    } else if (active && !job) {  // the eaten-log entries kept in registers and LDS
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < ne && i < p.eaten_cap) {
          p.eaten_xy[(int64_t)i * p.B + g] = lxy[i];
          p.eaten_rem[(int64_t)i * p.B + g] = (uint8_t)lrem[i];
        }
      for (int i = 4; i < kSmallLog; ++i)
        if (i < ne && i < p.eaten_cap) {
          p.eaten_xy[(int64_t)i * p.B + g] = s.elxy[(i - 4) * 64 + lane];
          p.eaten_rem[(int64_t)i * p.B + g] = s.elrem[(i - 4) * 64 + lane];
        }
    }
  }
  if (ROLL && last && p.returns) rollout_returns(p, s, g, active, lane);
  SMALL_STAMP(5);
  return jm;
}

// --------------------------------------------------------------------------- W1: draws
template <int G, bool ROLL = false>
__device__ __forceinline__ unsigned long long draws_wave(const Params& p, const SmallLayout& L, uint32_t* lds, int lane,
                                                         CarryHdr* carry = nullptr, int t = 0, bool last = true) {
  const Lds s = lds_of(lds, L);
  const int64_t g = (int64_t)blockIdx.x * 64 + lane;
  SMALL_STAMP(10);
  role_prio<ROLL>(2, t, p.features != nullptr);  // the tile value is on the bushes wave's path
  HeadRaw hr;
  if (ROLL && t > 0) {  // (multi-step launch: the thresholds are in LDS since step 0)
    hr.hdr = carry->hdr;
    hr.a = act_of(s, lane);
  } else {
  hr = head_fetch(p, g, g < p.B);
  {  // every threshold load in flight at once (a copy loop waits for each before the next)
    const int nthr = p.max_berries;  // <= 255
    uint64_t tv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tv[k] = p.thresholds[min(64 * k + lane, max(nthr, 1) - 1)];  // (>= 1 entry)
    opaque_head(hr);
#pragma unroll
    for (int k = 0; k < 4; ++k) opaque(tv[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (64 * k + lane < nthr) s.thr[64 * k + lane] = tv[k];
    if (lane == 0) bush_thr_pads(s.thr, nthr);
  }
  }
  const Head h = head_decode(p, g, g < p.B, hr);
  if (!ROLL || t == 0) lds_barrier();  // B_init
  SMALL_STAMP(30);
  const uint64_t ek = mix64(h.kenv ^ (uint64_t)h.hdr.w);
  const uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
  SMALL_STAMP(31);
  // the generated berries of the ostrich's tile (:631-635), for W0
  s.cval[lane] =
      (uint32_t)bush_value_fast(s.thr, p.max_berries, draw_U(h.cpos, make_ts(SITE_BUSH, 0, 0), b0, b1), p.bush_power);
  lds_publish(s.flag);  // every lane: each orders its own cval entry
  role_prio<ROLL>(0, t, p.features != nullptr);
  if (p.features && !p.restrict_view && !ROLL)  // rows 0..31 (step_features)
    early_view_zeros(p, 0u, (uint32_t)min((int64_t)32, p.B - (int64_t)blockIdx.x * 64), lane);
  SMALL_STAMP(11);
  s.strip[lane] = strip_draws(p, h, b0, b1, 0, kStripW1);  // generate_bushes (:613-629): the entering strip
  SMALL_STAMP(12);
  lds_barrier();  // B1
  const uint32_t info = s.info[lane];
  const bool killed = s.kill[lane] != 0u;
  const bool job = h.active && p.autoreset && env_done(p, h, info_starved(info), killed);
  // the reset draws of the done envs for view cells [0, 64); W3 draws the rest and waits for
  // flag[1] before it builds the new episodes
  const unsigned long long jm = __ballot(job);
  if (jm) {
    // (W3 waits for these draws before it builds the new episodes: W1 at issue priority 2
    // while it makes them, multi-step launches: 6.41 -> 6.33 us per step, profiles/r03_ab2/)
    if (ROLL) role_prio<ROLL>(kW1ResetPrio, t, p.features != nullptr);
    if (job) {
      const uint64_t ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));  // the new episode's key
      const int j = __popcll(jm & ((1ull << lane) - 1ull));
      *reinterpret_cast<uint2*>(&s.jkey[2 * j]) = make_uint2((uint32_t)ek2, (uint32_t)(ek2 >> 32));
    }
    reset_chunk(p, s.tiles, s.jkey, __popcll(jm), 0u, lane, s.jbm);
    lds_publish(&s.flag[1]);
    if (ROLL) role_prio<ROLL>(0, t, p.features != nullptr);
  }
  if (h.active && (!job || (!ROLL && p.t_planes))) {
    // S of the continuing envs (and of the done ones when their terminal obs is asked for);
    // needed only at B2, so after the reset draws W3 waits for
    render_s(p, s, lane, info, h.dir);
  }
  // the next step's actions (in LDS by the step's end), after the draws W3 waits for: the
  // scalar load's wait is then off that chain
  if (ROLL && !last) prefetch_actions(p, s, lane);
  SMALL_STAMP(13);
  lds_barrier();  // B2
  if (!ROLL && p.t_planes) lds_barrier();  // B3
  SMALL_STAMP(14);
  if (ROLL && lane == 0) {  // every hand-off of this step is done: clear the flags for the next
    s.flag[0] = 0u;
    s.flag[1] = 0u;
  }
  if (ROLL && !last) {
    const uint32_t status = info_starved(info) ? 1u : killed ? 2u : misc_status(h.hdr.z);
    carry->hdr = job ? new_header(carry_of(s, lane), h)
                     : make_uint4(h.cpos, (uint32_t)h.turn, misc_pack((uint32_t)h.role, status, 0u, 0u, 0u), h.hdr.w);
  }
  return jm;
}

// --------------------------------------------------------------------------- W2: wolves
template <int SLOTS, int G, bool ROLL = false>
__device__ __forceinline__ unsigned long long wolves_wave(const Params& p, const SmallLayout& L, uint32_t* lds, int lane,
                                                          CarryW2<SLOTS>* carry = nullptr, int t = 0, bool last = true) {
  const Lds s = lds_of(lds, L);
  const int64_t g = (int64_t)blockIdx.x * 64 + lane;
  const bool active = g < p.B;
  SMALL_STAMP(16);
  // the first 8 slots load with the header, whatever the wolf count: a group of 64 envs
  // nearly always has a lane with more than 4 wolves, and loading the rest after the count
  // arrives costs a second memory round trip on the path to B1
  // wolf slots read with the header, speculatively (the rest after B_init, for envs with more
  // wolves); -DWAB_SPEC_WOLVES=k: the tuning A/B of that count
#ifndef WAB_SPEC_WOLVES
#define WAB_SPEC_WOLVES 8
#endif
  constexpr int kSpecSlots = SLOTS < WAB_SPEC_WOLVES ? SLOTS : WAB_SPEC_WOLVES;
  uint32_t wr[SLOTS];
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) wr[k] = 0u;
  HeadRaw hr;
  const bool carried = ROLL && t > 0;  // (multi-step launch: slots and mask from the last step)
  if (carried) {
    hr.hdr = carry->hdr;
    hr.a = act_of(s, lane);
    constexpr int NR = CarryW2<SLOTS>::NR;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) wr[k] = k < NR ? carry->wr[k < NR ? k : 0] : s.wcar[(k - NR) * 64 + lane];
  } else {
  {
    const int64_t gl = active ? g : 0;  // (unconditional; an inactive lane has no live wolf)
#pragma unroll
    for (int k = 0; k < kSpecSlots; ++k) wr[k] = p.wolves[(int64_t)k * p.B + gl];  // speculatively
  }
  hr = head_fetch(p, g, active);
  opaque_head(hr);
#pragma unroll
  for (int k = 0; k < kSpecSlots; ++k) opaque(wr[k]);
  }
  const Head h = head_decode(p, g, active, hr);
  if (!ROLL || t == 0) lds_barrier();  // B_init
  SMALL_STAMP(28);
  const int nw = (int)misc_nw(h.hdr.z);
  if (!carried) {
#pragma unroll
    for (int k = kSpecSlots; k < SLOTS; ++k)
      if (k < nw) wr[k] = p.wolves[(int64_t)k * p.B + g];
  }
  const uint64_t ek = mix64(h.kenv ^ (uint64_t)h.hdr.w);
  const uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
  uint32_t live = carried ? (h.active ? carry->live : 0u) : nw >= 32 ? ~0u : ((1u << nw) - 1u);

  // despawn (:262-264): one draw per wolf, keyed by its tile and its occurrence index among
  // the co-located wolves before it; groups of 4 slots, skipped when no lane has a wolf there
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
        h1[q] = wr[k] ^ b0;
      }
      fmix32x4(h1);
#pragma unroll
      for (int q = 0; q < 4; ++q) hh[q] = h1[q] ^ ts[q] ^ b1;
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
          if (((tie >> q) & 1u) && draw_lo21(h1[q], ts[q], b0) >= p.keep_tl) kp |= 1u << q;
      }
      keep |= (kp & live4) << g4;
    }
    live = keep;
  }
  SMALL_STAMP(29);
  // pursuit (:267-286): one axis step toward the ostrich, ties along x; grid of S; kill
  M128 wolfp = {0ull, 0ull};
  bool kill = false;
#pragma unroll
  for (int g4 = 0; g4 < SLOTS; g4 += 4) {
    if (!((live >> g4) & 0xFu)) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = g4 + q;
      const bool on = (live >> k) & 1u;
      int wx = xy_x(wr[k]), wy = xy_y(wr[k]);
      if (p.wolves_can_move) {
        const int ddx = h.ox - wx, ddy = h.oy - wy;
        const bool alongx = abs(ddx) >= abs(ddy);
        wx += alongx ? sgn(ddx) : 0;
        wy += alongx ? 0 : sgn(ddy);
        wr[k] = xy_pack(wx, wy);
      }
      const int ddx = h.ox - wx, ddy = h.oy - wy;
      set_bit_if(wolfp, (uint32_t)((ddx + p.cw) * p.H + ddy + p.ch), on && abs(ddx) <= p.cw && abs(ddy) <= p.ch);
      kill |= on && ddx == 0 && ddy == 0;
    }
  }
  kill = kill && !p.god_mode;  // :291-297
  s.wolfp[lane] = m_pack(wolfp);
  s.kill[lane] = kill ? 1u : 0u;
  SMALL_STAMP(17);
  SMALL_STAMP(18);
  lds_barrier();  // B1: the spawn set, the starve flags and the bushes' counts are in
  const uint32_t info = s.info[lane];
  const bool starved = info_starved(info);
  const bool job = active && p.autoreset && env_done(p, h, starved, kill);

  // spawn_wolves (:325-326): new wolves into free slots (outside the view, not in S)
  unsigned long long wolf_of = 0;
  const M128 spawn = m_unpack(s.spawn[lane]);
  if (active && (spawn.lo | spawn.hi)) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      uint64_t bits = half ? spawn.hi : spawn.lo;
      while (bits) {
        const int b = __ffsll((unsigned long long)bits) - 1;
        bits &= bits - 1;
        const int r = 64 * half + b;
        const uint32_t w = xy_add(h.cpos, G == 11 ? ring11(r) : p.tables[p.ring_at + r]);
        bool placed = false;
#pragma unroll
        for (int k = 0; k < SLOTS; ++k)
          if (!placed && !((live >> k) & 1u)) { wr[k] = w; live |= 1u << k; placed = true; }
        if (!placed) wolf_of += 1;
      }
    }
  }
  // the next state of a continuing env: wolf slots and header (a done env's come from its
  // new episode)
  if (active && !job && (!ROLL || last)) {
    int n = 0;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k)
      if ((live >> k) & 1u) p.wolves[(int64_t)(n++) * p.B + g] = wr[k];
    const uint32_t status = starved ? 1u : kill ? 2u : misc_status(h.hdr.z);
    p.hdr[g] = make_uint4(h.cpos, (uint32_t)h.turn,
                          misc_pack((info >> 8) & 0xFFu, status, (uint32_t)n, (info >> 16) & 0xFFu, info >> 24),
                          h.hdr.w);
  }
  if (wolf_of) atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], wolf_of);
  const unsigned long long jm = __ballot(job);
  if (ROLL && carry->prev_stream) store_units_nt<128, 12>(p, carry->prev_planes, carry->prev_stream, 64 + lane);
  SMALL_STAMP(19);
  lds_barrier();  // B2
  if (!ROLL && p.t_planes) lds_barrier();  // B3
  SMALL_STAMP(20);
  if (ROLL && !last) {  // the slots for the next step: a new episode's wolves from W3's cells
    if (job) {
      const NewEp n = carry_of(s, lane);
      M128 m = n.wolves;
      constexpr int NR = CarryW2<SLOTS>::NR;
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {
        const bool any = (m.lo | m.hi) != 0ull;
        const uint32_t c = m.lo ? (uint32_t)(__ffsll((unsigned long long)m.lo) - 1)
                                : (uint32_t)(__ffsll((unsigned long long)m.hi) + 63);
        const uint32_t w = any ? s.tiles[any ? c : 0u] : 0u;
        if (k < NR) carry->wr[k < NR ? k : 0] = w;
        else s.wcar[(k - NR) * 64 + lane] = w;
        if (any) m_clear(m, c);
      }
      carry->live = n.nw >= 32u ? ~0u : ((1u << n.nw) - 1u);
      carry->hdr = new_header(n, h);
    } else {
      constexpr int NR = CarryW2<SLOTS>::NR;
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {
        if (k < NR) carry->wr[k < NR ? k : 0] = wr[k];
        else s.wcar[(k - NR) * 64 + lane] = wr[k];
      }
      carry->live = live;
      const uint32_t status = starved ? 1u : kill ? 2u : misc_status(h.hdr.z);
      carry->hdr = make_uint4(h.cpos, (uint32_t)h.turn,
                              misc_pack((info >> 8) & 0xFFu, status, (uint32_t)__popc(live), (info >> 16) & 0xFFu,
                                        info >> 24),
                              h.hdr.w);
    }
  }
  return jm;
}

// --------------------------------------------------------------------------- W3: ring
template <int SLOTS, int G, bool ROLL = false>
__device__ __forceinline__ unsigned long long ring_wave(const Params& p, const SmallLayout& L, uint32_t* lds, int lane,
                                                        CarryHdr* carry = nullptr, int t = 0, bool last = true) {
  const Lds s = lds_of(lds, L);
  const int64_t g = (int64_t)blockIdx.x * 64 + lane;
  SMALL_STAMP(22);
  if (ROLL) role_prio<ROLL>(0, t, p.features != nullptr);  // (raised after B1 of the last step)
  HeadRaw hr;
  if (ROLL && t > 0) {  // (multi-step launch: the tables are in LDS since step 0)
    hr.hdr = carry->hdr;
    hr.a = act_of(s, lane);
    reinterpret_cast<uint4*>(s.jbm)[lane] = make_uint4(0u, 0u, 0u, 0u);  // reset bitmaps [64][4]
  } else {
  hr = head_fetch(p, g, g < p.B);
  if constexpr (G == 11) {  // view-cell offsets (cw - i, ch - j) of cell c = 11 i + j, computed
    for (int c = lane; c < 121; c += 64) s.tiles[c] = xy_pack(5 - c / 11, 5 - c % 11);
  } else {
    uint32_t tv[2];  // WH <= 128: both loads in flight at once
#pragma unroll
    for (int k = 0; k < 2; ++k) tv[k] = p.tables[min(64 * k + lane, p.WH - 1)];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (64 * k + lane < p.WH) s.tiles[64 * k + lane] = tv[k];
  }
  reinterpret_cast<uint4*>(s.jbm)[lane] = make_uint4(0u, 0u, 0u, 0u);  // reset bitmaps [64][4]
  {  // the spawn sets' gap table, every load in flight at once
    const int n = p.n_gap + 1;  // <= 129
    uint64_t gv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) gv[k] = p.gap[min(64 * k + lane, n - 1)];
    opaque_head(hr);
#pragma unroll
    for (int k = 0; k < 3; ++k) opaque(gv[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (64 * k + lane < n) s.gap[64 * k + lane] = gv[k];
  }
  }
  if (p.features) {  // zero the fused features' bits and tables (contiguous, 16-byte aligned;
                     // multi-step launches: the tables once, the bits every step)
    uint4* z = reinterpret_cast<uint4*>(lds + L.fbits);
    const uint32_t nz = ROLL && t > 0 ? L.ftab - L.fbits : L.fzero;
    for (uint32_t i = lane; i < nz / 4u; i += 64) z[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  const Head h = head_decode(p, g, g < p.B, hr);
  if (!ROLL || t == 0) lds_barrier();  // B_init
  if (p.features) {
    if (!ROLL || t == 0)
      feat_tables_build(feat_tables_at(lds + L.ftab, p.W / 2 + p.H / 2 + 1), p.W, p.H, p.W / 2 + p.H / 2 + 1, lane, 64);
    if (!p.restrict_view && !ROLL)  // rows 32..63 (step_features)
      early_view_zeros(p, 32u, (uint32_t)max((int64_t)0, min((int64_t)32, p.B - (int64_t)blockIdx.x * 64 - 32)), lane);
  }
  const uint64_t ek = mix64(h.kenv ^ (uint64_t)h.hdr.w);
  const uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
  // spawn_wolves (:527-576): the ring's spawn set this turn (one draw unless a wolf spawns)
  M128 spawn = {0ull, 0ull};
  if (p.wolves_on && h.active)
    spawn_hits(s.gap, p.R, p.gap_full_th, p.gap_full_tl, p.gap_ring_th, p.gap_ring_tl, p.gap_inv_l2, h.turn, b0, b1, [&](int r) { m_set(spawn, (uint32_t)r); });
  s.spawn[lane] = m_pack(spawn);
  s.strip[64 + lane] = strip_draws(p, h, b0, b1, kStripW1, 1 << 30);  // the entering strip, part 2
  SMALL_STAMP(23);
  lds_barrier();  // B1
  role_prio<ROLL>(3, t, p.features != nullptr);
  // reset draws of every done env (generate_bushes, initialize_wolves), all view cells, then
  // (unless the terminal obs is asked for: W0 after B2) the new episodes themselves
  const bool job = h.active && p.autoreset && env_done(p, h, info_starved(s.info[lane]), s.kill[lane] != 0u);
  const unsigned long long jm = __ballot(job);
  int role2 = 0;
  if (jm) {
    const int j = __popcll(jm & ((1ull << lane) - 1ull));
    uint32_t* jkey = s.jkey + 2 * 64;  // this wave's copy of the keys
    uint64_t ek2 = 0;
    if (job) {
      ek2 = mix64(h.kenv ^ (uint64_t)(h.hdr.w + 1u));  // the new episode's key
      *reinterpret_cast<uint2*>(&jkey[2 * j]) = make_uint2((uint32_t)ek2, (uint32_t)(ek2 >> 32));
    }
    const int n_jobs = __popcll(jm);
    for (uint32_t c0 = 64; c0 < (uint32_t)p.WH; c0 += 64)  // cells [0, 64): W1
      reset_chunk(p, s.tiles, jkey, n_jobs, c0, lane, s.jbm);
    SMALL_STAMP(24);
    if (ROLL || !p.t_planes) {
      // the part of the new episode that needs only its key, while W1 may still be drawing
      unsigned long long wolf_of = 0;
      const uint32_t ebit = (uint32_t)lane * (uint32_t)p.OB;
      if (job) role2 = new_episode_a<SLOTS, ROLL>(p, s, h, g, (uint32_t)ek2, (uint32_t)(ek2 >> 32), ebit, wolf_of, last);
      lds_await(p, &s.flag[1]);  // W1's part of the draws
      SMALL_STAMP(9);
      if (job) new_episode_b(p, s, g, j, ebit, role2, !ROLL || last);
      if (wolf_of) atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], wolf_of);
    }
  }
  SMALL_STAMP(25);
  lds_barrier();  // B2
  if (!ROLL && p.t_planes) lds_barrier();  // B3
  SMALL_STAMP(26);
  if (ROLL && !last) {
    const uint32_t status = info_starved(s.info[lane]) ? 1u : s.kill[lane] != 0u ? 2u : misc_status(h.hdr.z);
    carry->hdr = job ? new_header(carry_of(s, lane), h)
                     : make_uint4(h.cpos, (uint32_t)h.turn, misc_pack((uint32_t)h.role, status, 0u, 0u, 0u), h.hdr.w);
  }
  return jm;
}

// --------------------------------------------------------------------------- obs stores
// expand the 64-env bit-stream and store it with 16-byte stores, all 256 threads
// Multi-step launches: units [K0, K1) of the six per thread of a finished step's stream (p its
// step's slice), each cleared after its read (the last step's obs, stored at its end).  No
// partial tail: a multi-step launch needs B * OB % 16 == 0 (wab_rollout).
template <int K0, int K1>
__device__ __forceinline__ void store_units_of(const Params& p, uint32_t* stream, int tid) {
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const uint32_t OB = (uint32_t)p.OB;
  const uint32_t full = ((uint32_t)min((int64_t)64, p.B - g0) * OB) >> 4;
  uint8_t* out = p.planes + (size_t)g0 * OB;
  uint16_t* s16 = reinterpret_cast<uint16_t*>(stream);
  uint32_t v[K1 - K0];
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const uint32_t u = (uint32_t)tid + 256u * (uint32_t)k;
    v[k - K0] = u < full ? (uint32_t)s16[u] : 0u;
  }
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const uint32_t u = (uint32_t)tid + 256u * (uint32_t)k;
    if (u < full) s16[u] = 0;
  }
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const uint32_t u = (uint32_t)tid + 256u * (uint32_t)k;
    if (u >= full) break;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 q;
#pragma unroll
    for (int b = 0; b < 4; ++b) q[b] = (((v[k - K0] >> (4 * b)) & 0xFu) * 0x00204081u) & 0x01010101u;
    if (WAB_ROLL_OBS_NT) __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out) + u);
    else reinterpret_cast<u32x4*>(out)[u] = q;
  }
}

template <bool CLEAR = false>
__device__ __forceinline__ void store_obs(const Params& p, uint32_t* stream, int tid) {
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const uint32_t OB = (uint32_t)p.OB;
  const uint32_t limit = (uint32_t)min((int64_t)64, p.B - g0) * OB;
  uint8_t* out = p.planes + (size_t)g0 * OB;
  // one 16-bit unit of the stream -> 16 bytes: each wave-instruction stores 1 KiB contiguous.
  // A group has at most 64 * 384 bits (OB <= 3 * 128) = 1536 units: six per thread, all read
  // from LDS before the first is expanded (a loop waits for each read in turn)
  const uint16_t* s16 = reinterpret_cast<const uint16_t*>(stream);
  const uint32_t full = limit >> 4;
  uint32_t v[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t u = (uint32_t)tid + 256u * (uint32_t)k;
    v[k] = u < full ? (uint32_t)s16[u] : 0u;
  }
  if constexpr (CLEAR) {  // (multi-step launches: each unit cleared by the thread that read it)
    uint16_t* w16 = reinterpret_cast<uint16_t*>(stream);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint32_t u = (uint32_t)tid + 256u * (uint32_t)k;
      if (u < full) w16[u] = 0;
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t u = (uint32_t)tid + 256u * (uint32_t)k;
    if (u >= full) break;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 q;
#pragma unroll
    for (int b = 0; b < 4; ++b) q[b] = (((v[k] >> (4 * b)) & 0xFu) * 0x00204081u) & 0x01010101u;
#ifndef WAB_STEP_OBS_NT  // (tuning A/B: 0 = plain stores)
#define WAB_STEP_OBS_NT 1
#endif
    if (WAB_STEP_OBS_NT) __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out) + u);  // streamed: no L2 allocation
    else reinterpret_cast<u32x4*>(out)[u] = q;
  }
  for (uint32_t b = (full << 4) + tid; b < limit; b += 256)  // a partial last group
    out[b] = (uint8_t)((stream[b >> 5] >> (b & 31)) & 1u);
#ifdef WAB_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((tid & 63) == 0 && p.stamps) {
    const int slot[4] = {6, 15, 21, 27};
    p.stamps[(size_t)blockIdx.x * kStampStride + slot[tid >> 6]] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// --------------------------------------------------------------------------- fused features
// wab_step_features: PragmaticObsWrapper features (wab_feat.h) of the obs this step returns,
// from the rendered bit-stream (after B2, or B3) and the scalars each env's writer handed over:
// W0 the wolf plane, W1 the bush plane, W2 the scalars and view mask, one more barrier, then
// all 256 threads expand the feature bits to float32 (the featurizer's phases 2 and 3).
template <bool ROLL = false>
__device__ __forceinline__ void step_features(const Params& p, const SmallLayout& L, uint32_t* lds, int wave,
                                              int lane, int t = 0) {
  const int md = p.W / 2 + p.H / 2 + 1;
  const uint32_t F = (uint32_t)pragmatic_dim(md, p.turns_empty), WH = (uint32_t)p.WH;
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const uint32_t n_active = (uint32_t)min((int64_t)64, p.B - g0);
  const uint32_t* stream = lds + L.stream;
  uint32_t* ob = lds + L.fbits;
  if (ROLL && (uint32_t)lane < n_active) {
    // multi-step launches: the emit over all four waves (W0, W1 the two planes' nearest cells,
    // W2 both planes' direction counts, W3 the scalars and view mask)
    const uint32_t ebit = (uint32_t)lane * (uint32_t)p.OB, at = (uint32_t)lane * F;
    const FeatTables ft = feat_tables_at(lds + L.ftab, md);
    if (wave <= 1) {
      uint32_t near, second;
      plane_nearest(ft, md, stream_get128(stream, ebit + (uint32_t)wave * WH, WH), near, second);
      emit_nearest(ob, at, wave, md, near, second);
    } else if (wave == 2) {
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
        int counts[4];
        plane_counts(ft, stream_get128(stream, ebit + (uint32_t)pl * WH, WH), counts);
        emit_counts(ob, at, pl, md, counts);
      }
    } else {
      const uint32_t sc = lds[L.scal + lane];
      const uint32_t role = (sc >> 8) & 0xFFu;
      const uint32_t sb_bit = ebit + WH + (uint32_t)(md / 2) * (uint32_t)p.S + (uint32_t)(md / 2);  // :742
      emit_scalars(ob, at, md, p.turns_empty, (stream[sb_bit >> 5] >> (sb_bit & 31u)) & 1u, sc & 0xFFu, role,
                   sc >> 16, p.restrict_view != 0, view_mask_of(p, (int)role));
    }
  } else if ((uint32_t)lane < n_active && wave < 3) {
    const uint32_t ebit = (uint32_t)lane * (uint32_t)p.OB, at = (uint32_t)lane * F;
    if (wave <= 1) {  // W0 wolves, W1 bushes
      uint32_t near, second;
      int counts[4];
      plane_features(feat_tables_at(lds + L.ftab, md), md, stream_get128(stream, ebit + (uint32_t)wave * WH, WH), near,
                     second, counts);
      emit_plane(ob, at, wave, md, near, second, counts);
    } else {
      const uint32_t sc = lds[L.scal + lane];
      const uint32_t role = (sc >> 8) & 0xFFu;
      const uint32_t sb_bit = ebit + WH + (uint32_t)(md / 2) * (uint32_t)p.S + (uint32_t)(md / 2);  // :742
      emit_scalars(ob, at, md, p.turns_empty, (stream[sb_bit >> 5] >> (sb_bit & 31u)) & 1u, sc & 0xFFu, role,
                   sc >> 16, p.restrict_view != 0, view_mask_of(p, (int)role));
    }
  }
#ifdef WAB_STAMPS
  const auto stamp = [&](int slot) {  // (multi-step launches: the middle step, wave 0)
    if (ROLL && threadIdx.x == 0 && p.stamps && t == p.n_steps / 2)
      p.stamps[(size_t)blockIdx.x * kStampStride + slot] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(36);  // the feature bits emitted
#endif
  // (Measured and not adopted in multi-step launches: the rows of step t stored during step t + 1
  // by W0 and W2 in their slack, from double-buffered feature bits; the view-mask zero lines
  // stored early in each step.)  Multi-step launches store the rows non-temporal.
  lds_barrier();
  constexpr bool NT = ROLL;
  if (p.restrict_view || ROLL) store_feature_bits<NT>(ob, p.features + (size_t)g0 * F, n_active * F, (int)threadIdx.x, 256);
  else store_rows_skip_views<NT>(ob, p.features + (size_t)g0 * F, n_active * F, F, (int)threadIdx.x, 256);
#ifdef WAB_STAMPS
  stamp(37);  // wave 0's row stores issued
#endif
}

}  // namespace

// FEAT: wab_step_features (the fused featurizer); without it the feature code folds away
// The parameter block as each wave reads it: a fresh copy from the kernel-argument segment
// behind an opaque pointer, so that the scalar loads of its fields stay in the branch of
// the wave that uses them.  (A plain copy of the kernel argument has every field loaded at
// the kernel's entry, before the wave branch, and spilled to VGPR lanes: ~190 v_writelane /
// v_readlane and a chain of scalar-load waits ahead of every wave's first global load.)
template <int G, bool FEAT>
__device__ __forceinline__ Params wave_params(const Params& p0) {
#if __HIP_DEVICE_COMPILE__  // (the host pass only type-checks the kernel body)
  typedef const Params __attribute__((address_space(4))) KernargParams;
  KernargParams* pk = (KernargParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  Params p = *pk;
#else
  Params p = p0;
#endif
  specialise_geometry<G>(p);
  if constexpr (!FEAT) p.features = nullptr;
  return p;
}

// step t of a multi-step launch (Params::n_steps): the I/O arrays advanced to their [t] slices
__device__ __forceinline__ void step_slice(Params& p, int t) {
  if (t == 0) return;
  const int64_t o = (int64_t)t * p.B;
  p.actions += o;
  if (p.planes) p.planes += o * p.OB;
  p.food_turns += o;
  p.role += o;
  p.status += o;
  p.reward += o;
  p.done += o;
  if (p.features) p.features += o * pragmatic_dim(p.W / 2 + p.H / 2 + 1, p.turns_empty);
}

template <int SLOTS, int G, bool FEAT, bool ROLL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ROLL ? 4 : 1))) void wab_step_small(Params p0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
#ifdef WAB_STAMPS
  uint64_t t_entry;  // before the first kernel-argument load
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry)::"memory");
#endif
  if ((int64_t)blockIdx.x * 64 >= p0.B) return;  // (uniform over the workgroup)
#ifdef WAB_STAMPS
  if (threadIdx.x == 0 && p0.stamps) {  // kernel entry (slot 32), the XCD (33), first kernarg field in (34)
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    p0.stamps[(size_t)blockIdx.x * kStampStride + 34] = __builtin_amdgcn_s_memrealtime();
    p0.stamps[(size_t)blockIdx.x * kStampStride + 32] = t_entry;
    p0.stamps[(size_t)blockIdx.x * kStampStride + 33] = xcc & 0xFu;
  }
#endif
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // (uniform branches)
#ifdef WAB_STAMPS
  if (lane == 0 && p0.stamps) {  // each wave's HW_ID (SIMD, CU, SE) in slots 40..43
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    p0.stamps[(size_t)blockIdx.x * kStampStride + 40 + wave] = hw;
  }
#endif
#ifdef WAB_ONLY_WAVE  // static per-wave instruction counts (tools/isa_count.py); not a runnable build
  if (wave != WAB_ONLY_WAVE) return;
#endif
  if constexpr (!ROLL) {
    unsigned long long jm;  // the group's done envs (every wave computes the same mask)
    if (wave == 0) {
      // the bushes wave carries the longest chain and shares its SIMD with three helper waves
      // of other groups: let the arbiter issue its instructions first
      __builtin_amdgcn_s_setprio(3);
      const Params p = wave_params<G, FEAT>(p0);
      jm = bushes_wave<SLOTS, G>(p, small_layout(p), lds, lane);
      __builtin_amdgcn_s_setprio(0);
    } else if (wave == 1) {
      const Params p = wave_params<G, FEAT>(p0);
      jm = draws_wave<G>(p, small_layout(p), lds, lane);
    } else if (wave == 2) {
      const Params p = wave_params<G, FEAT>(p0);
      jm = wolves_wave<SLOTS, G>(p, small_layout(p), lds, lane);
    } else {
      const Params p = wave_params<G, FEAT>(p0);
      jm = ring_wave<SLOTS, G>(p, small_layout(p), lds, lane);
    }
    const Params p = wave_params<G, FEAT>(p0);
    const SmallLayout L = small_layout(p);
    (void)jm;
    if (!FEAT || p.planes) store_obs(p, lds + L.stream, threadIdx.x);
    if constexpr (FEAT) step_features(p, L, lds, wave, lane);
  } else {
    // wab_rollout: n_steps steps of this group, one after the other (the envs of a workgroup
    // depend on nothing outside it), each wave's state carried in registers from step to step
    // (see CarryW0): one barrier closes a step (its LDS is reused by the next)
    const int T = p0.n_steps;
#ifdef WAB_STAMPS
#define ROLL_LOOP_STAMP(slot, cond)                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0 && p0.stamps && (cond))                                             \
      p0.stamps[(size_t)blockIdx.x * kStampStride + (slot)] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define ROLL_LOOP_STAMP(slot, cond) do {} while (0)
#endif
    {  // the second stream starts clear (the first is cleared by W0 in step 0)
      const SmallLayout L = small_layout(p0);
      uint4* z = reinterpret_cast<uint4*>(lds + L.stream2);
      for (uint32_t i = threadIdx.x; i < L.stream_words / 4u; i += 256) z[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    // one step of wave W's part; step t renders into stream t & 1 while W0 and W2 store step
    // t - 1's obs from the other one; the last step's obs go out at its end, by every thread
#define WAB_ROLL_STEP(...)                                                                   \
    for (int t = 0; t < T; ++t) {                                                            \
      ROLL_LOOP_STAMP(35, t == T / 2);  /* the middle step's loop top (before its parameters) */ \
      if (WAB_ROLL_THROTTLE && (wave == 0 || wave == 2)) __builtin_amdgcn_s_waitcnt(0x0F70);  \
      Params p = wave_params<G, FEAT>(p0);                                                   \
      step_slice(p, t);                                                                      \
      const SmallLayout L0 = small_layout(p);                                                \
      SmallLayout L = L0;                                                                    \
      if (t & 1) L.stream = L0.stream2;                                                      \
      c.prev_planes = p.planes ? p.planes - (int64_t)p.B * p.OB : nullptr;                   \
      c.prev_stream = t > 0 ? lds + ((t & 1) ? L0.stream : L0.stream2) : nullptr;           \
      if (WAB_ROLL_FLOOR) {  /* diagnostic floor: the stores alone (results wrong by design) */ \
        lds_barrier();                                                                       \
        lds_barrier();                                                                       \
      } else {                                                                               \
        __VA_ARGS__;                                                                         \
      }                                                                                      \
      if (FEAT) step_features<true>(p, L, lds, wave, lane, t);  /* this step's rows */     \
      if (t == T - 1 && p.planes) {                                                          \
        lds_barrier();                                                                       \
        store_units_of<0, 6>(p, lds + L.stream, threadIdx.x);                                \
      }                                                                                      \
      lds_barrier();                                                                         \
      ROLL_LOOP_STAMP(38, t == T / 2);  /* past the middle step's end barrier */             \
    }
    if (wave == 0) {
      CarryW0 c;
      WAB_ROLL_STEP({
        role_prio<true>(3, t, p.features != nullptr);
        bushes_wave<SLOTS, G, true>(p, L, lds, lane, &c, t, t == T - 1);
        role_prio<true>(0, t, p.features != nullptr);
      })
    } else if (wave == 1) {
      CarryPtr<CarryHdr> c;
      WAB_ROLL_STEP(draws_wave<G, true>(p, L, lds, lane, &c.c, t, t == T - 1))
    } else if (wave == 2) {
      CarryW2<SLOTS> c;
      WAB_ROLL_STEP((wolves_wave<SLOTS, G, true>(p, L, lds, lane, &c, t, t == T - 1)))
    } else {
      CarryPtr<CarryHdr> c;
      WAB_ROLL_STEP((ring_wave<SLOTS, G, true>(p, L, lds, lane, &c.c, t, t == T - 1)))
    }
#undef WAB_ROLL_STEP
#undef ROLL_LOOP_STAMP
#ifdef WAB_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && p0.stamps)  // every store of the workgroup retired (slot 39)
      p0.stamps[(size_t)blockIdx.x * kStampStride + 39] = __builtin_amdgcn_s_memrealtime();
#endif
  }
}

template __global__ void wab_step_small<8, 0, false, false>(Params);
template __global__ void wab_step_small<8, 0, true, false>(Params);
template __global__ void wab_step_small<8, 0, false, true>(Params);
template __global__ void wab_step_small<8, 0, true, true>(Params);
template __global__ void wab_step_small<8, 11, false, false>(Params);
template __global__ void wab_step_small<8, 11, true, false>(Params);
template __global__ void wab_step_small<8, 11, false, true>(Params);
template __global__ void wab_step_small<8, 11, true, true>(Params);
template __global__ void wab_step_small<16, 0, false, false>(Params);
template __global__ void wab_step_small<16, 0, true, false>(Params);
template __global__ void wab_step_small<16, 0, false, true>(Params);
template __global__ void wab_step_small<16, 0, true, true>(Params);
template __global__ void wab_step_small<16, 11, false, false>(Params);
template __global__ void wab_step_small<16, 11, true, false>(Params);
template __global__ void wab_step_small<16, 11, false, true>(Params);
template __global__ void wab_step_small<16, 11, true, true>(Params);
template __global__ void wab_step_small<32, 0, false, false>(Params);
template __global__ void wab_step_small<32, 0, true, false>(Params);
template __global__ void wab_step_small<32, 0, false, true>(Params);
template __global__ void wab_step_small<32, 0, true, true>(Params);
template __global__ void wab_step_small<32, 11, false, false>(Params);
template __global__ void wab_step_small<32, 11, true, false>(Params);
template __global__ void wab_step_small<32, 11, false, true>(Params);
template __global__ void wab_step_small<32, 11, true, true>(Params);

}  // namespace wab
