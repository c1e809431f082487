// wab_step.hip — the fused batched Wolves-and-Bushes step for gfx950 (MI355X).
//
// One launch advances every env by one step (wab_env.py:250-342) and renders its
// observation (wab_env.py:359-452); the MODE_RESET instantiation performs reset
// (wab_env.py:231-248).  One 256-thread workgroup owns 64 envs:
//
//   phase A  all threads   zero the LDS bit-streams/masks, build the tile table
//            wave 0        lane = env: issue every state load, apply the move, then scroll
//                          the cached bush bitmap of the view by the move
//   phase B  all threads   4 threads per env, keyed draws for the tiles that entered the
//                          view (one row or column) -> bitmap, and for the wolf-spawn ring
//                          around the new position -> spawn mask
//   phase C  wave 0        eaten-tile corrections, bitmap -> bush plane, despawn, pursuit,
//                          kill, eat, hunger, starve, spawn -> slots, reward/done, stores;
//                          done-mask ballot -> compacted reset jobs (autoreset)
//   phase D  all threads   reset jobs: bush + initial-wolf draws over the new view
//   phase E  wave 0        reset envs: bitmap -> plane, wolves -> slots, stores
//   phase F  all threads   expand the bit-streams 1 bit -> 1 byte and store the block's
//                          contiguous obs chunk with 16-byte coalesced stores
//
// The obs chunk of a block is 64 * 3*W*S contiguous bytes of `planes`; in LDS it is held
// as a bit-stream whose bit k is byte k of the chunk, so every store of phase F is a full
// 1 KiB wave-instruction regardless of W, H.  Bush presence of the view is kept as a
// W*H-bit bitmap per env in HBM (bushmap), so a step only hashes the <= max(W, H) tiles
// that scroll into view instead of all W*H.  No MFMA: integer hashing, compares, bytes.
#include <hip/hip_runtime.h>

#include "wab_device.h"

namespace wab {

// bitmap word k of env e: bm[k * NE + e] (slot-major: lanes of wave 0 hit consecutive banks)
template <int NE>
__device__ __forceinline__ uint32_t& BM(uint32_t* bm, int k, int e) { return bm[k * NE + e]; }

// copy an env's W*H bush bitmap (bit i*H + j) into plane 1 of its stream segment
template <int NE>
__device__ __forceinline__ void bitmap_to_plane(const Params& p, uint32_t* bm, int e, uint32_t* s,
                                                uint32_t at) {
  if (p.S == p.H) {  // contiguous: one funnel-shifted copy
    for (int k = 0; k < p.WHW; ++k) {
      const uint32_t nb = min(32u, (uint32_t)(p.WH - 32 * k));
      lds_or_bits(s, at + 32u * k, BM<NE>(bm, k, e), nb);
    }
  } else {           // padded rows: row i -> bits [i*S, i*S + H)
    for (int i = 0; i < p.W; ++i) {
      const uint32_t c = (uint32_t)(i * p.H);
      for (int j0 = 0; j0 < p.H; j0 += 32) {
        const uint32_t n = min(32u, (uint32_t)(p.H - j0));
        const uint32_t b = c + j0;
        uint64_t w = BM<NE>(bm, b >> 5, e) >> (b & 31);
        if ((b & 31) + n > 32) w |= (uint64_t)BM<NE>(bm, (b >> 5) + 1, e) << (32 - (b & 31));
        lds_or_bits(s, at + (uint32_t)(i * p.S + j0), (uint32_t)w, n);
      }
    }
  }
}

// Diagnostic build (-DWAB_STAMPS): thread 0 of each block records s_memrealtime (100 MHz)
// at phase boundaries into p.stamps; the product build compiles these to nothing.
#ifdef WAB_STAMPS
#define WAB_STAMP(slot)                                                                    \
  do {                                                                                     \
    if (threadIdx.x == 0 && p.stamps)                                                      \
      p.stamps[(size_t)blockIdx.x * kStampStride + (slot)] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define WAB_STAMP(slot) do {} while (0)
#endif

template <int MODE, int SLOTS, bool SMALL>
__global__ __launch_bounds__(kThreads) void wab_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr int NE = kEnvsPerBlock;
  constexpr int G = kThreads / NE;  // threads per env in phase B
  const int tid = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * NE;
  const int n_active = (int)min((int64_t)NE, p.B - g0);
  const uint32_t streamW = (uint32_t)(NE * p.OB) >> 5;
  const uint32_t plane = (uint32_t)(p.W * p.S);
  const int NWd = SMALL ? min(p.WHW, 4) : p.WHW;

  const LdsLayout L = lds_layout(p, SLOTS);
  uint32_t* sA = lds + L.sA;          // step obs bits
  uint32_t* sB = lds + L.sB;          // reset obs bits
  uint32_t* spawnM = lds + L.spawnM;  // [NE][RW]
  uint32_t* wolfM = lds + L.wolfM;    // [job][WHW]
  uint32_t* bm = lds + L.bm;          // [WHW][NE] bush bitmaps
  uint32_t* masks = lds + L.masks;    // [3][WHW]: column 0, column H-1, valid bits
  uint32_t* tiles = lds + L.tiles;    // [NT]
  uint32_t* snap = lds + L.snap;      // [NE][4]: pos, b0, b1, turn20 | dir << 24
  uint32_t* jobEnv = lds + L.jobEnv;  // [NE]
  uint32_t* jobKey = lds + L.jobKey;  // [NE][2]
  uint32_t* blk = lds + L.blk;        // [0] n_jobs, [1..2] job mask
  uint64_t* thr = reinterpret_cast<uint64_t*>(lds + L.thr);  // [max_berries] bush thresholds

  // per-env registers of wave 0 (lane = env)
  const int e = tid;
  const bool envlane = tid < NE;
  const int64_t g = g0 + e;
  const bool active = envlane && e < n_active;
  int32_t ox = 0, oy = 0, turn = 0, role = 0, status = 0, nw = 0, ne = 0, ndep = 0, dir = DIR_STAY;
  double food = 0.0, reward = 0.0;
  uint32_t ep = 0, b0 = 0, b1 = 0;
  uint64_t ek_next = 0;  // key of the episode an auto-reset would start
  bool done = false;
  // eaten-log prefetch (phase A -> C): the first kLogPrefetch entries, when needed
  constexpr int kLogPrefetch = 4;
  uint32_t lxy[kLogPrefetch], lrem[kLogPrefetch];
#pragma unroll
  for (int i = 0; i < kLogPrefetch; ++i) { lxy[i] = 0u; lrem[i] = 0u; }
  bool need_log = false;
  unsigned long long bad = 0, eaten_of = 0, wolf_of = 0;
  // wolves of this env: slot registers + a live mask (slot order is irrelevant: co-located
  // wolves are interchangeable, so only the multiset of positions is state)
  uint32_t wr[SLOTS];
  uint32_t live = 0;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) wr[s] = 0u;

  WAB_STAMP(0);
  // ---------------------------------------------------------------- phase A
  if (MODE == MODE_STEP && active) {
    // every load is independent and issued up front: one memory round trip
    const uint4 hdr = p.hdr[g];
    const int a = (int)p.actions[g];
    const uint64_t kenv = env_key(p.seed, (uint64_t)(p.env_base + g));  // overlaps the loads
    food = p.food[g];
    const uint32_t w0 = p.wolves[g], w1 = p.wolves[p.B + g];  // slots 0, 1 speculatively
    uint32_t bmr[4] = {0u, 0u, 0u, 0u};
    if (SMALL) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < NWd) bmr[k] = p.bushmap[(int64_t)k * p.B + g];
    } else {
      for (int k = 0; k < NWd; ++k) BM<NE>(bm, k, e) = p.bushmap[(int64_t)k * p.B + g];
    }
    ox = xy_x(hdr.x);
    oy = xy_y(hdr.x);
    turn = (int32_t)hdr.y;
    role = (int)misc_role(hdr.z);
    status = (int)misc_status(hdr.z);
    nw = (int)misc_nw(hdr.z);
    ne = (int)misc_ne(hdr.z);
    ndep = (int)misc_ndep(hdr.z);
    ep = hdr.w;
    wr[0] = w0;
    wr[1] = w1;
#pragma unroll
    for (int s = 2; s < SLOTS; ++s)
      if (s < nw) wr[s] = p.wolves[(int64_t)s * p.B + g];
    live = nw >= 32 ? ~0u : ((1u << nw) - 1u);
    turn += 1;                                                       // :252
    if (a >= 0 && a < p.n_actions) {                                 // :253-258
      int dx, dy, nr;
      decode_action(p, a, dx, dy, nr);
      ox += dx;
      oy += dy;
      dir = dx > 0 ? DIR_RIGHT : dx < 0 ? DIR_LEFT : dy > 0 ? DIR_UP : dy < 0 ? DIR_DOWN : DIR_STAY;
      if (nr >= 0) role = nr;
    } else {
      bad += 1;
    }
    if (SMALL) {  // scroll the cached view bitmap by the move (:613-629 keeps old tiles)
      uint64_t lo = (uint64_t)bmr[0] | ((uint64_t)bmr[1] << 32);
      uint64_t hi = (uint64_t)bmr[2] | ((uint64_t)bmr[3] << 32);
      if (dir == DIR_RIGHT || dir == DIR_UP) shl128(lo, hi, dir == DIR_RIGHT ? p.H : 1);
      else if (dir == DIR_LEFT || dir == DIR_DOWN) shr128(lo, hi, dir == DIR_LEFT ? p.H : 1);
      uint32_t v[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] &= p.small_masks[2][k];
        if (dir == DIR_UP) v[k] &= ~p.small_masks[0][k];    // column 0 enters the view
        if (dir == DIR_DOWN) v[k] &= ~p.small_masks[1][k];  // column H-1 enters the view
        if (k < NWd) BM<NE>(bm, k, e) = v[k];
      }
    }
    const uint64_t ek = mix64(kenv ^ (uint64_t)ep);
    ek_next = mix64(kenv ^ (uint64_t)(ep + 1u));
    b0 = (uint32_t)ek;
    b1 = (uint32_t)(ek >> 32);
    // eaten log: needed for the berries on the ostrich's tile, or for emptied tiles that may
    // scroll back into view; issued now, consumed in phase C (latency hidden by phase B)
    {
      const uint32_t ccb = (uint32_t)(p.cw * p.H + p.ch);
      const bool center = SMALL ? ((BM<NE>(bm, ccb >> 5, e) >> (ccb & 31)) & 1u) != 0u : true;
      const bool center_in_strip = (dir == DIR_RIGHT || dir == DIR_LEFT) ? p.W == 1
                                   : (dir == DIR_UP || dir == DIR_DOWN) ? p.H == 1 : false;
      need_log = ne > 0 && (center || center_in_strip || (ndep > 0 && dir != DIR_STAY));
#pragma unroll
      for (int i = 0; i < kLogPrefetch; ++i)
        if (need_log && i < ne) {
          lxy[i] = p.eaten_xy[(int64_t)i * p.B + g];
          lrem[i] = p.eaten_rem[(int64_t)i * p.B + g];
        }
    }
    uint4 sn;
    sn.x = xy_pack(ox, oy);
    sn.y = b0;
    sn.z = b1;
    sn.w = ((uint32_t)turn & 0xFFFFFu) | ((uint32_t)dir << 24);
    *reinterpret_cast<uint4*>(&snap[e * 4]) = sn;
  }
  {
    for (uint32_t i = tid; i < L.bm; i += kThreads) lds[i] = 0;  // streams + masks
    if (!SMALL) {
      for (int k = tid; k < NWd; k += kThreads) {                // column / validity masks
        uint32_t c0 = 0, cl = 0, v = 0;
        for (int b = 0; b < 32; ++b) {
          const int c = 32 * k + b;
          if (c >= p.WH) break;
          v |= 1u << b;
          const int j = c % p.H;
          if (j == 0) c0 |= 1u << b;
          if (j == p.H - 1) cl |= 1u << b;
        }
        masks[k] = c0;
        masks[NWd + k] = cl;
        masks[2 * NWd + k] = v;
      }
    }
    for (int c = tid; c < p.NT; c += kThreads) {
      int dx, dy;
      uint32_t bit;
      if (c < p.WH) {
        const int i = c / p.H, j = c - (c / p.H) * p.H;
        dx = p.cw - i;  // world x = ox - (i - cw)   (grid axis 0 is ostrich_x - x, wab_env.py:403-409)
        dy = p.ch - j;
        bit = (uint32_t)(i * p.S + j);
      } else {
        const int r = c - p.WH, m = p.margin, Wm = p.W + 2 * m;
        int xi, yi;
        if (r < 2 * m * Wm) {
          const int band = r / Wm;
          xi = r - band * Wm;
          yi = band < m ? band : band + p.H;
        } else {
          const int r2 = r - 2 * m * Wm, band = r2 / p.H;
          yi = m + (r2 - band * p.H);
          xi = band < m ? band : band + p.W;
        }
        tiles[c] = xy_pack(xi - p.cw - m, yi - p.ch - m);  // ring: packed world offset
        continue;
      }
      tiles[c] = ((uint32_t)dx & 0xFFu) | (((uint32_t)dy & 0xFFu) << 8) | (bit << 16);
    }
    for (int k = tid; k < p.max_berries; k += kThreads) thr[k] = p.thresholds[k];
  }
  lds_barrier();

  if constexpr (MODE == MODE_STEP) {
    WAB_STAMP(1);
    if (!SMALL) {
      // scroll the cached view bitmap by the move (generate_bushes keeps old tiles, :613-629)
      if (active) {
        if (dir == DIR_RIGHT || dir == DIR_UP) {        // shift toward higher bit indices
          const int n = dir == DIR_RIGHT ? p.H : 1, q = n >> 5, r = n & 31;
          for (int k = NWd - 1; k >= 0; --k) {
            const uint32_t lo = k - q >= 0 ? BM<NE>(bm, k - q, e) : 0u;
            const uint32_t lo2 = (r && k - q - 1 >= 0) ? BM<NE>(bm, k - q - 1, e) : 0u;
            uint32_t v = r ? (lo << r) | (lo2 >> (32 - r)) : lo;
            v &= masks[2 * NWd + k];
            if (dir == DIR_UP) v &= ~masks[k];           // column 0 enters the view
            BM<NE>(bm, k, e) = v;
          }
          // (RIGHT: row 0 = bits [0, H) arrive as zeros from the shift)
        } else if (dir == DIR_LEFT || dir == DIR_DOWN) {  // shift toward lower bit indices
          const int n = dir == DIR_LEFT ? p.H : 1, q = n >> 5, r = n & 31;
          for (int k = 0; k < NWd; ++k) {
            const uint32_t hi = k + q < NWd ? BM<NE>(bm, k + q, e) : 0u;
            const uint32_t hi2 = (r && k + q + 1 < NWd) ? BM<NE>(bm, k + q + 1, e) : 0u;
            uint32_t v = r ? (hi >> r) | (hi2 << (32 - r)) : hi;
            v &= masks[2 * NWd + k];
            if (dir == DIR_DOWN) v &= ~masks[NWd + k];   // column H-1 enters the view
            BM<NE>(bm, k, e) = v;                         // (LEFT: row W-1 arrives as zeros)
          }
        }
      }
      lds_barrier();
    }
    WAB_STAMP(2);

    // -------------------------------------------------------------- phase B (keyed draws)
    {
      const int be = tid / G, sub = tid - (tid / G) * G;
      if (be < n_active) {
        const uint4 sn = *reinterpret_cast<const uint4*>(&snap[be * 4]);
        const uint32_t kb0 = sn.y;
        // spawn ring around the new position (spawn_wolves :527-576): the ring's spawn set
        // this turn, one draw unless a wolf spawns (keyed spawn sets, wab_device.h)
        uint32_t* sm = spawnM + be * p.RW;
        if (sub == 0 && p.wolves_on)
          spawn_hits(p.gap, p.R, p.gap_full_th, p.gap_full_tl, p.gap_ring_th, p.gap_ring_tl, p.gap_inv_l2, (int32_t)(sn.w & 0xFFFFFu), kb0, sn.z,
                     [&](int r) { atomicOr(&sm[r >> 5], 1u << (r & 31)); });
        // the row or column that scrolled into view (generate_bushes :613-629)
        const int bdir = (int)(sn.w >> 24);
        if (bdir != DIR_STAY) {
          const bool horiz = bdir == DIR_RIGHT || bdir == DIR_LEFT;
          const int n = horiz ? p.H : p.W;
          const int i0 = bdir == DIR_LEFT ? p.W - 1 : 0, j0 = bdir == DIR_DOWN ? p.H - 1 : 0;
          const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0), hb = ts_bush ^ sn.z;
          const int bx = xy_x(sn.x), by = xy_y(sn.x);
          for (int c = sub; c < n; c += G) {
            const int i = horiz ? i0 : c, j = horiz ? c : j0;
            const uint32_t h1 = fmix32(xy_pack(bx - (i - p.cw), by - (j - p.ch)) ^ kb0);
            const uint32_t hi = fmix32(h1 ^ hb);
            if (hi >= p.bush_th && (hi > p.bush_th || draw_lo21(h1, ts_bush, kb0) >= p.bush_tl)) {
              const uint32_t cb = (uint32_t)(i * p.H + j);
              atomicOr(&BM<NE>(bm, (int)(cb >> 5), be), 1u << (cb & 31));
            }
          }
        }
      }
    }
    lds_barrier();
    WAB_STAMP(3);

    // -------------------------------------------------------------- phase C (wab_env.py:259-342)
    if (active) {
      const uint32_t ebit = (uint32_t)e * (uint32_t)p.OB;
      const uint32_t cpos = xy_pack(ox, oy);
      const uint32_t ccb = (uint32_t)(p.cw * p.H + p.ch);  // bitmap bit of the ostrich's tile
      const bool center_bush = (BM<NE>(bm, ccb >> 5, e) >> (ccb & 31)) & 1u;
      // eaten-tile log, read only when it can matter: for the berries left on the ostrich's
      // tile, and for emptied tiles that may have scrolled back into view (absent from S, :506)
      int found = -1, found_rem = 0;
      if (need_log && (center_bush || (ndep > 0 && dir != DIR_STAY))) {
        for (int i = 0; i < ne; ++i) {
          uint32_t v = 0;
          int r = 0;
          if (i < kLogPrefetch) {
#pragma unroll
            for (int q = 0; q < kLogPrefetch; ++q)
              if (q == i) { v = lxy[q]; r = (int)lrem[q]; }
          } else {
            v = p.eaten_xy[(int64_t)i * p.B + g];
            r = (int)p.eaten_rem[(int64_t)i * p.B + g];
          }
          if (v == cpos) { found = i; found_rem = r; }
          const int ddx = ox - xy_x(v), ddy = oy - xy_y(v);
          if (r == 0 && abs(ddx) <= p.cw && abs(ddy) <= p.ch) {
            const uint32_t cb = (uint32_t)((ddx + p.cw) * p.H + ddy + p.ch);
            BM<NE>(bm, cb >> 5, e) &= ~(1u << (cb & 31));
          }
        }
      }
      WAB_STAMP(7);
      bitmap_to_plane<NE>(p, bm, e, sA, ebit + plane);               // bush grid (:430-444)
      WAB_STAMP(8);
      // despawn (:262-264): one draw per wolf, keyed by its tile and its occurrence index
      // among the co-located wolves before it
      uint32_t keep = 0;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (!((live >> s) & 1u)) continue;
        uint32_t k = 0;
#pragma unroll
        for (int t = 0; t < s; ++t) k += (((live >> t) & 1u) && wr[t] == wr[s]) ? 1u : 0u;
        const uint32_t ts = make_ts(SITE_DESPAWN, k, turn);
        const uint32_t h1 = fmix32(wr[s] ^ b0);
        const uint32_t hi = fmix32(h1 ^ ts ^ b1);
        if (U_ge(h1, hi, ts, b0, p.keep_th, p.keep_tl)) keep |= 1u << s;
      }
      live = keep;
      // pursuit (:267-286): one axis step toward the ostrich, ties along x; then S (:289)
      const int status_snap = status;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (!((live >> s) & 1u)) continue;
        int wx = xy_x(wr[s]), wy = xy_y(wr[s]);
        if (p.wolves_can_move) {
          const int ddx = ox - wx, ddy = oy - wy;
          if (abs(ddx) >= abs(ddy)) wx += sgn(ddx); else wy += sgn(ddy);
          wr[s] = xy_pack(wx, wy);
        }
        const int ddx = ox - wx, ddy = oy - wy;
        if (abs(ddx) <= p.cw && abs(ddy) <= p.ch)                     // wolf grid (:412-428)
          lds_set(sA, ebit + (uint32_t)((ddx + p.cw) * p.S + ddy + p.ch));
        if (ddx == 0 && ddy == 0 && !p.god_mode) status = 2;          // kill (:291-297)
      }
      lds_set(sA, ebit + 2 * plane + (uint32_t)(p.cw * p.S + p.ch));  // ostrich grid (:393-410)
      WAB_STAMP(9);
      // berries left on the ostrich's tile: eaten log, else the tile's generated value
      int rem;
      if (found >= 0)
        rem = found_rem;
      else if (center_bush)
        rem = bush_value(thr, p.max_berries, draw_U(cpos, make_ts(SITE_BUSH, 0, 0), b0, b1));
      else
        rem = 0;
      // eat (:299-313): stale snapshot status; clip only in this branch
      if (rem > 0 && status_snap == 0 && (role == 1 || p.lookout_only)) {
        food = food + p.fill;
        food = food < 0.0 ? 0.0 : (food > 1.0 ? 1.0 : food);
        reward += p.r_eat;
        bool logged = true;
        if (found >= 0) {
          p.eaten_rem[(int64_t)found * p.B + g] = (uint8_t)(rem - 1);
        } else if (ne < p.eaten_cap) {
          p.eaten_xy[(int64_t)ne * p.B + g] = cpos;
          p.eaten_rem[(int64_t)ne * p.B + g] = (uint8_t)(rem - 1);
          ne += 1;
        } else {
          eaten_of += 1;
          logged = false;
        }
        if (rem == 1) {  // emptied: gone from the cached view from the next step on
          BM<NE>(bm, ccb >> 5, e) &= ~(1u << (ccb & 31));
          if (logged) ndep += 1;
        }
      }
      WAB_STAMP(10);
      food = food - p.hunger;                                        // :316
      if (food <= 0.0) { status = 1; food = 0.0; }                   // :319-322
      if (p.restrict_view) apply_view_mask(p, sA, ebit, role);
      // spawn_wolves (:325-326, :527-576) on the ring around the new position
      for (int wd = 0; wd < p.RW; ++wd) {
        uint32_t bits = spawnM[e * p.RW + wd];
        while (bits) {
          const int b = __ffs(bits) - 1;
          bits &= bits - 1;
          const uint32_t w = xy_add(cpos, tiles[p.WH + wd * 32 + b]);
          bool placed = false;
#pragma unroll
          for (int s = 0; s < SLOTS; ++s)
            if (!placed && !((live >> s) & 1u)) { wr[s] = w; live |= 1u << s; placed = true; }
          if (!placed) wolf_of += 1;
        }
      }
      WAB_STAMP(11);
      // reward / done (:328-340)
      if (status == 0) {
        if (turn >= p.max_turns) { reward += p.r_finish; done = true; }
        else reward += p.r_turn;
      } else if (status == 1) {
        reward += p.r_starve; done = true;
      } else {
        reward += p.r_killed; done = true;
      }
      p.reward[g] = (float)reward;
      p.done[g] = done ? 1 : 0;
    }
  } else {
    // reset mode: the flagged envs become reset jobs
    if (active) {
      done = (p.reset_mask == nullptr) || (p.reset_mask[g] != 0);
      if (done) ep = p.hdr[g].w;
    }
  }

  WAB_STAMP(12);
  // ---------------------------------------------------------------- done-mask ballot -> jobs
  const bool job = active && done && (MODE == MODE_RESET || p.autoreset);
  unsigned long long jm = 0;
  if (tid < 64) {
    jm = __ballot(job);
    if (tid == 0) {
      blk[0] = (uint32_t)__popcll(jm);
      blk[1] = (uint32_t)jm;
      blk[2] = (uint32_t)(jm >> 32);
    }
  }
  if (active) {
    if (job) {
      if (MODE == MODE_STEP && p.t_planes) {
        p.t_food_turns[g] = (uint8_t)(int)ceil(food * (double)p.turns_empty);
        p.t_role[g] = (uint8_t)role;
        p.t_status[g] = (uint8_t)status;
      }
      // reset (:231-248, spawn_ostriches :595-611)
      const int j = __popcll(jm & ((1ull << e) - 1ull));
      ep += 1u;  // 0xFFFFFFFF -> 0 on the first reset
      const uint64_t ek = MODE == MODE_STEP ? ek_next : episode_key(p.seed, (uint64_t)(p.env_base + g), ep);
      b0 = (uint32_t)ek;
      b1 = (uint32_t)(ek >> 32);
      jobEnv[j] = (uint32_t)e;
      jobKey[2 * j] = b0;
      jobKey[2 * j + 1] = b1;
      for (int k = 0; k < NWd; ++k) BM<NE>(bm, k, e) = 0u;
      turn = 0;
      ox = 0;
      oy = 0;
      status = 0;
      ne = 0;
      ndep = 0;
      nw = 0;
      food = p.start_food_random
                 ? (double)draw_U(xy_pack(0, 0), make_ts(SITE_START_FOOD, 0, 0), b0, b1) * 0x1p-53
                 : p.start_food;
      role = p.start_role_random
                 ? (int)(draw_U(xy_pack(0, 0), make_ts(SITE_START_ROLE, 0, 0), b0, b1) >> 52)
                 : p.start_role;
    }
    if (MODE == MODE_STEP || job) {
      p.food_turns[g] = (uint8_t)(int)ceil(food * (double)p.turns_empty);  // :450-452
      p.role[g] = (uint8_t)role;
      p.status[g] = (uint8_t)status;
      p.food[g] = food;
    }
    if (MODE == MODE_STEP && !job) {
      nw = 0;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s)
        if ((live >> s) & 1u) p.wolves[(int64_t)(nw++) * p.B + g] = wr[s];
      for (int k = 0; k < NWd; ++k) p.bushmap[(int64_t)k * p.B + g] = BM<NE>(bm, k, e);
      p.hdr[g] = make_uint4(xy_pack(ox, oy), (uint32_t)turn,
                            misc_pack((uint32_t)role, (uint32_t)status, (uint32_t)nw, (uint32_t)ne,
                                      (uint32_t)ndep),
                            ep);
    }
  }
  if (envlane && (bad | eaten_of | wolf_of)) {
    if (bad) atomicAdd(&p.counters[CTR_BAD_ACTIONS], bad);
    if (eaten_of) atomicAdd(&p.counters[CTR_EATEN_OVERFLOW], eaten_of);
    if (wolf_of) atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], wolf_of);
  }
  if constexpr (MODE == MODE_STEP) count_steps(p);
  lds_barrier();
  WAB_STAMP(4);

  const int n_jobs = (int)blk[0];
  const unsigned long long done_mask = (unsigned long long)blk[1] | ((unsigned long long)blk[2] << 32);
  if (n_jobs > 0) {
    // -------------------------------------------------------------- phase D (reset draws)
    {
      const int WH = p.WH;
      const int items = n_jobs * WH;
      int ij = tid / WH, ic = tid - (tid / WH) * WH;
      const int stepJ = kThreads / WH, stepC = kThreads - (kThreads / WH) * WH;
      const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0);
      // initialize_wolves (:578-593): each job's view spawn set at turn 0, one thread per job
      if (p.wolves_on && tid < n_jobs) {
        const uint32_t je = jobEnv[tid];
        spawn_hits(p.gap, WH, p.gap_full_th, p.gap_full_tl, p.gap_view_th, p.gap_view_tl, p.gap_inv_l2, 0, jobKey[2 * tid], jobKey[2 * tid + 1], [&](int c) {
          lds_set(sB, je * (uint32_t)p.OB + tile_bit(tiles[c]));
          lds_set(wolfM + tid * p.WHW, (uint32_t)c);
        });
      }
      for (int q = tid; q < items; q += kThreads) {
        const uint32_t je = jobEnv[ij], kb0 = jobKey[2 * ij], kb1 = jobKey[2 * ij + 1];
        const uint32_t t = tiles[ic];
        const uint32_t xy = xy_pack(tile_dx(t), tile_dy(t));  // ostrich at (0, 0)
        const uint32_t h1 = fmix32(xy ^ kb0);
        const uint32_t hb = fmix32(h1 ^ ts_bush ^ kb1);
        if (U_ge(h1, hb, ts_bush, kb0, p.bush_th, p.bush_tl))         // generate_bushes
          atomicOr(&BM<NE>(bm, ic >> 5, (int)je), 1u << (ic & 31));
        ic += stepC;
        ij += stepJ;
        if (ic >= WH) { ic -= WH; ij += 1; }
      }
    }
    lds_barrier();
    // -------------------------------------------------------------- phase E (reset envs)
    if (job) {
      const int j = __popcll(done_mask & ((1ull << e) - 1ull));
      const uint32_t ebit = (uint32_t)e * (uint32_t)p.OB;
      bitmap_to_plane<NE>(p, bm, e, sB, ebit + plane);
      for (int k = 0; k < NWd; ++k) p.bushmap[(int64_t)k * p.B + g] = BM<NE>(bm, k, e);
      lds_set(sB, ebit + 2 * plane + (uint32_t)(p.cw * p.S + p.ch));
      if (p.restrict_view) apply_view_mask(p, sB, ebit, role);
      int n = 0;
      for (int wd = 0; wd < p.WHW; ++wd) {
        uint32_t bits = wolfM[j * p.WHW + wd];
        while (bits) {
          const int b = __ffs(bits) - 1;
          bits &= bits - 1;
          const uint32_t t = tiles[wd * 32 + b];
          if (n < SLOTS) p.wolves[(int64_t)(n++) * p.B + g] = xy_pack(tile_dx(t), tile_dy(t));
          else {
            atomicAdd(&p.counters[CTR_WOLF_OVERFLOW], 1ull);
            atomicAdd(&p.counters[CTR_WOLF_OVERFLOW_RESET], 1ull);
          }
        }
      }
      p.hdr[g] = make_uint4(xy_pack(0, 0), 0u, misc_pack((uint32_t)role, 0u, (uint32_t)n, 0u, 0u), ep);
    }
    if (tid == 0) atomicAdd(&p.block_resets[blockIdx.x], (unsigned long long)n_jobs);  // (no-return: a load here would wait for the stores)
    lds_barrier();
  }
  WAB_STAMP(5);

  // ---------------------------------------------------------------- phase F (expand + store)
  {
    const uint32_t OB = (uint32_t)p.OB;
    const uint32_t limit = (uint32_t)n_active * OB;      // valid bytes of this block's chunk
    uint8_t* out = p.planes + (size_t)g0 * OB;
    uint8_t* tout = (MODE == MODE_STEP && p.t_planes) ? p.t_planes + (size_t)g0 * OB : nullptr;
    const bool full_jobs = (MODE == MODE_RESET) && n_jobs == n_active;
    for (uint32_t d = tid; d < streamW; d += kThreads) {
      const uint32_t bo = d << 5;
      if (bo >= limit) break;
      uint32_t dm = 0;   // bits of this dword that belong to job (done / flagged) envs
      if (n_jobs > 0) {
        if (full_jobs) {
          dm = ~0u;
        } else {
          const uint32_t e_lo = udiv(bo, OB, p.magic_OB);
          const uint32_t e_hi = min(udiv(bo + 31u, OB, p.magic_OB), (uint32_t)NE - 1u);
          for (uint32_t ee = e_lo; ee <= e_hi; ++ee) {
            if (!((done_mask >> ee) & 1ull)) continue;
            const uint32_t lo = max(ee * OB, bo) - bo;
            const uint32_t hi = min((ee + 1u) * OB, bo + 32u) - bo;  // exclusive, <= 32
            dm |= (hi >= 32u ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
          }
        }
      }
      uint32_t v;
      if (MODE == MODE_STEP) v = (sA[d] & ~dm) | (sB[d] & dm);
      else v = sB[d];
      const uint32_t write_mask = (MODE == MODE_STEP) ? ~0u : dm;
      if (write_mask == ~0u && bo + 32u <= limit) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 q0, q1;
#pragma unroll
        for (int k = 0; k < 4; ++k) q0[k] = (((v >> (4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
#pragma unroll
        for (int k = 0; k < 4; ++k) q1[k] = (((v >> (16 + 4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
        // streamed out, never re-read by the kernel: non-temporal (no L2 allocation)
        __builtin_nontemporal_store(q0, reinterpret_cast<u32x4*>(out + bo));
        __builtin_nontemporal_store(q1, reinterpret_cast<u32x4*>(out + bo + 16));
      } else if (write_mask) {
        for (uint32_t k = 0; k < 32u && bo + k < limit; ++k)
          if ((write_mask >> k) & 1u) out[bo + k] = (uint8_t)((v >> k) & 1u);
      }
      if (MODE == MODE_STEP && tout && dm) {
        const uint32_t va = sA[d];
        for (uint32_t k = 0; k < 32u && bo + k < limit; ++k)
          if ((dm >> k) & 1u) tout[bo + k] = (uint8_t)((va >> k) & 1u);
      }
    }
  }
  WAB_STAMP(6);
}

// explicit instantiations used by wab_capi.hip
#define WAB_INST(M, S)                                           \
  template __global__ void wab_kernel<M, S, true>(Params);       \
  template __global__ void wab_kernel<M, S, false>(Params);
WAB_INST(MODE_STEP, 8)
WAB_INST(MODE_STEP, 16)
WAB_INST(MODE_STEP, 32)
WAB_INST(MODE_RESET, 8)
WAB_INST(MODE_RESET, 16)
WAB_INST(MODE_RESET, 32)

}  // namespace wab
