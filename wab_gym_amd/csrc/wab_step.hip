// wab_step.hip — the fused batched Wolves-and-Bushes step for gfx950 (MI355X).
//
// One launch advances every env by one step (wab_env.py:250-342) and renders its
// observation (wab_env.py:359-452); a second instantiation performs reset
// (wab_env.py:231-248).  One 256-thread workgroup owns 64 envs:
//
//   phase 0  all threads   zero the LDS bit-streams and masks, build the tile table
//   phase 1  wave 0        lane = env: load SoA state, move, despawn, pursue, kill, eat,
//                          hunger, starve; wolf + ostrich bits into stream A
//   phase 2  all threads   tile-parallel keyed draws: bush presence for the W*H viewport
//                          tiles -> stream A, wolf spawns on the margin ring -> spawn mask
//   phase 3  wave 0        eaten-tile corrections, view mask, spawn -> slots, reward/done,
//                          done-mask ballot -> compacted reset jobs (autoreset)
//   phase 4  all threads   reset jobs: bush + initial-wolf draws for the new episode
//                          -> stream B (skipped when the block has no done env)
//   phase 5  wave 0        reset envs: wolves into slots, ostrich bit, view mask
//   phase 6  all threads   expand the bit-streams 1 bit -> 1 byte and store the block's
//                          contiguous obs chunk with 16-byte coalesced stores
//
// The obs chunk of a block is 64 * 3*W*S contiguous bytes of `planes`; in LDS it is held
// as a bit-stream whose bit k is byte k of the chunk, so every store of phase 6 is a full
// 1 KiB wave-instruction regardless of W, H.  No MFMA: the work is integer hashing,
// compares and byte stores.
#include <hip/hip_runtime.h>

#include "wab_params.h"

namespace wab {

enum : uint32_t { SITE_BUSH = 1, SITE_SPAWN = 2, SITE_DESPAWN = 3, SITE_START_FOOD = 4, SITE_START_ROLE = 5 };
enum { MODE_STEP = 0, MODE_RESET = 1 };

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

__device__ __forceinline__ uint64_t episode_key(uint64_t seed, uint64_t env, uint64_t ep) {
  return mix64(mix64(mix64(seed + 0x9E3779B97F4A7C15ull) ^ env) ^ ep);
}

__device__ __forceinline__ uint32_t make_ts(uint32_t site, uint32_t k, int32_t turn) {
  return (site & 0xFu) | ((k & 0xFFu) << 4) | (((uint32_t)turn & 0xFFFFFu) << 12);
}

__device__ __forceinline__ uint32_t draw_lo21(uint32_t h1, uint32_t ts, uint32_t b0) {
  const uint32_t rot = (ts << 16) | (ts >> 16);
  return fmix32(h1 ^ rot ^ b0 ^ 0x9E3779B9u) >> 11;
}

// U >= thr for U = hi << 21 | lo21; the low half is only hashed when the high 32 bits tie
// (probability 2^-32).  thr may be 2^53 ("never").
__device__ __forceinline__ bool U_ge(uint32_t h1, uint32_t hi, uint32_t ts, uint32_t b0, uint64_t thr) {
  const uint64_t th = thr >> 21;
  if ((uint64_t)hi != th) return (uint64_t)hi > th;
  return draw_lo21(h1, ts, b0) >= (uint32_t)(thr & 0x1FFFFFu);
}

__device__ __forceinline__ uint64_t draw_U(uint32_t xy, uint32_t ts, uint32_t b0, uint32_t b1) {
  const uint32_t h1 = fmix32(xy ^ b0);
  const uint32_t hi = fmix32(h1 ^ ts ^ b1);
  return ((uint64_t)hi << 21) | draw_lo21(h1, ts, b0);
}

// number of thresholds T_k <= U: the reference's round(u**power * max) (wab_env.py:631-635)
__device__ __forceinline__ int bush_value(const Params& p, uint64_t U) {
  int lo = 0, hi = p.max_berries;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (p.thresholds[mid] <= U) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t udiv(uint32_t x, uint32_t d, uint32_t magic) {
  uint32_t q = __umulhi(x, magic);
  const int32_t r = (int32_t)(x - q * d);
  if (r < 0) q -= 1; else if ((uint32_t)r >= d) q += 1;
  return q;
}

__device__ __forceinline__ void lds_set(uint32_t* s, uint32_t bit) { atomicOr(&s[bit >> 5], 1u << (bit & 31)); }
__device__ __forceinline__ void lds_clear(uint32_t* s, uint32_t bit) { atomicAnd(&s[bit >> 5], ~(1u << (bit & 31))); }

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

__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

// unpack a tile-table entry: world offset from the ostrich and bit index
__device__ __forceinline__ int tile_dx(uint32_t t) { return (int)(int8_t)(t & 0xFFu); }
__device__ __forceinline__ int tile_dy(uint32_t t) { return (int)(int8_t)((t >> 8) & 0xFFu); }
__device__ __forceinline__ uint32_t tile_bit(uint32_t t) { return t >> 16; }

template <int MODE, int SLOTS>
__global__ __launch_bounds__(kThreads) void wab_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr int NE = kEnvsPerBlock;
  const int tid = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * NE;
  const int n_active = (int)min((int64_t)NE, p.B - g0);
  const uint32_t streamW = (uint32_t)(NE * p.OB) >> 5;
  const uint32_t plane = (uint32_t)(p.W * p.S);

  const LdsLayout L = lds_layout(p, SLOTS);
  uint32_t* sA = lds + L.sA;          // step obs bits
  uint32_t* sB = lds + L.sB;          // reset obs bits
  uint32_t* spawnM = lds + L.spawnM;  // [NE][RW]
  uint32_t* wolfM = lds + L.wolfM;    // [job][WHW]
  uint32_t* tiles = lds + L.tiles;    // [NT]
  uint32_t* snap = lds + L.snap;      // [NE][4]: pos, b0, b1, turn
  uint32_t* wl = lds + L.wl;          // [SLOTS][NE] wolves (phase 1/3 scratch)
  uint32_t* jobEnv = lds + L.jobEnv;  // [NE]
  uint32_t* jobKey = lds + L.jobKey;  // [NE][2]
  uint32_t* blk = lds + L.blk;        // [0] n_jobs, [1..2] job mask

  // ---------------------------------------------------------------- phase 0
  {
    for (uint32_t i = tid; i < L.tiles; i += kThreads) lds[i] = 0;  // streams + masks
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
        dx = xi - p.cw - m;
        dy = yi - p.ch - m;
        bit = (uint32_t)r;
      }
      tiles[c] = ((uint32_t)dx & 0xFFu) | (((uint32_t)dy & 0xFFu) << 8) | (bit << 16);
    }
  }
  __syncthreads();

  // per-env registers of wave 0 (lane = env)
  const int e = tid;
  const bool envlane = tid < NE;
  const int64_t g = g0 + e;
  const bool active = envlane && e < n_active;
  int32_t ox = 0, oy = 0, turn = 0, role = 0, status = 0, nw = 0, ne = 0;
  double food = 0.0, reward = 0.0;
  uint32_t ep = 0;
  int eat_idx = -1;
  bool done = false;
  unsigned long long bad = 0, eaten_of = 0, wolf_of = 0;

  if constexpr (MODE == MODE_STEP) {
    // -------------------------------------------------------------- phase 1 (wab_env.py:251-322)
    if (active) {
      const uint32_t pos = p.pos[g];
      food = p.food[g];
      turn = p.turn[g];
      const uint32_t misc = p.misc[g];
      ep = p.episode[g];
      role = (int)(misc & 0xFFu);
      status = (int)((misc >> 8) & 3u);
      nw = (int)((misc >> 10) & 63u);
      ne = (int)(misc >> 16);
      ox = xy_x(pos);
      oy = xy_y(pos);
      const uint64_t ek = episode_key(p.seed, (uint64_t)(p.env_base + g), ep);
      const uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
      const int a = (int)p.actions[g];
      turn += 1;                                                   // :252
      if (a >= 0 && a < p.n_actions) {                             // :253-258
        ox += p.act_dx[a];
        oy += p.act_dy[a];
        if (p.act_role[a] >= 0) role = p.act_role[a];
      } else {
        bad += 1;
      }
      // despawn (:262-264): decide every wolf on the old list, then compact (stable)
      for (int s = 0; s < nw; ++s) wl[s * NE + e] = p.wolves[(int64_t)s * p.B + g];
      uint32_t keep = 0;
      for (int s = 0; s < nw; ++s) {
        const uint32_t w = wl[s * NE + e];
        uint32_t k = 0;
        for (int t = 0; t < s; ++t) k += (wl[t * NE + e] == w) ? 1u : 0u;
        const uint32_t ts = make_ts(SITE_DESPAWN, k, turn);
        const uint32_t h1 = fmix32(w ^ b0);
        const uint32_t hi = fmix32(h1 ^ ts ^ b1);
        if (U_ge(h1, hi, ts, b0, p.keep_gt + 1)) keep |= 1u << s;
      }
      int n = 0;
      for (int s = 0; s < nw; ++s)
        if (keep & (1u << s)) wl[(n++) * NE + e] = wl[s * NE + e];
      nw = n;
      // pursuit (:267-286): one axis step toward the ostrich, ties along x
      if (p.wolves_can_move) {
        for (int s = 0; s < nw; ++s) {
          const uint32_t w = wl[s * NE + e];
          int wx = xy_x(w), wy = xy_y(w);
          const int ddx = ox - wx, ddy = oy - wy;
          if (abs(ddx) >= abs(ddy)) wx += sgn(ddx); else wy += sgn(ddy);
          wl[s * NE + e] = xy_pack(wx, wy);
        }
      }
      // snapshot S (:289): wolves now, bushes with food > 0 now, status now
      const int status_snap = status;
      const uint32_t cpos = xy_pack(ox, oy);
      const uint32_t ebit = (uint32_t)e * (uint32_t)p.OB;
      for (int s = 0; s < nw; ++s) {  // wolf grid bits (:412-428)
        const uint32_t w = wl[s * NE + e];
        const int ddx = ox - xy_x(w), ddy = oy - xy_y(w);
        if (abs(ddx) <= p.cw && abs(ddy) <= p.ch) lds_set(sA, ebit + (uint32_t)((ddx + p.cw) * p.S + ddy + p.ch));
        if (w == cpos && !p.god_mode) status = 2;                  // kill (:291-297)
      }
      lds_set(sA, ebit + 2 * plane + (uint32_t)(p.cw * p.S + p.ch));  // ostrich grid (:393-410)
      // berries left on the ostrich's tile: eaten log, else the tile's generated value
      int found = -1;
      for (int i = 0; i < ne; ++i) found = (p.eaten_xy[(int64_t)i * p.B + g] == cpos) ? i : found;
      int rem;
      if (found >= 0) {
        rem = p.eaten_rem[(int64_t)found * p.B + g];
      } else {
        const uint64_t U = draw_U(cpos, make_ts(SITE_BUSH, 0, 0), b0, b1);
        rem = U >= p.bush_t1 ? bush_value(p, U) : 0;
      }
      // eat (:299-313): stale snapshot status; clip only in this branch
      if (rem > 0 && status_snap == 0 && (role == 1 || p.lookout_only)) {
        food = food + p.fill;
        food = food < 0.0 ? 0.0 : (food > 1.0 ? 1.0 : food);
        reward += p.r_eat;
        if (found >= 0) {
          p.eaten_rem[(int64_t)found * p.B + g] = (uint8_t)(rem - 1);
          eat_idx = found;
        } else if (ne < p.eaten_cap) {
          p.eaten_xy[(int64_t)ne * p.B + g] = cpos;
          p.eaten_rem[(int64_t)ne * p.B + g] = (uint8_t)(rem - 1);
          eat_idx = ne;
          ne += 1;
        } else {
          eaten_of += 1;
        }
      }
      food = food - p.hunger;                                      // :316
      if (food <= 0.0) { status = 1; food = 0.0; }                 // :319-322
      uint4 sn;
      sn.x = cpos; sn.y = b0; sn.z = b1; sn.w = (uint32_t)turn;
      *reinterpret_cast<uint4*>(&snap[e * 4]) = sn;
    }
    __syncthreads();

    // -------------------------------------------------------------- phase 2 (tile-parallel draws)
    {
      const int NT = p.NT;
      const int items = n_active * NT;
      int ie = tid / NT, ic = tid - (tid / NT) * NT;
      const int stepE = kThreads / NT, stepC = kThreads - (kThreads / NT) * NT;
      const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0);
      for (int q = tid; q < items; q += kThreads) {
        const uint4 sn = *reinterpret_cast<const uint4*>(&snap[ie * 4]);
        const uint32_t t = tiles[ic];
        const uint32_t xy = xy_pack(xy_x(sn.x) + tile_dx(t), xy_y(sn.x) + tile_dy(t));
        const bool is_bush = ic < p.WH;
        const uint32_t ts = is_bush ? ts_bush : make_ts(SITE_SPAWN, 0, (int32_t)sn.w);
        const uint64_t thr = is_bush ? p.bush_t1 : p.spawn_lt;
        const uint32_t h1 = fmix32(xy ^ sn.y);
        const uint32_t hi = fmix32(h1 ^ ts ^ sn.z);
        const bool ge = U_ge(h1, hi, ts, sn.y, thr);
        if (is_bush) {
          if (ge) lds_set(sA, (uint32_t)ie * (uint32_t)p.OB + plane + tile_bit(t));   // bush present
        } else if (!ge) {
          lds_set(spawnM + ie * p.RW, tile_bit(t));                                  // wolf spawns
        }
        ic += stepC;
        ie += stepE;
        if (ic >= NT) { ic -= NT; ie += 1; }
      }
    }
    __syncthreads();

    // -------------------------------------------------------------- phase 3
    if (active) {
      const uint32_t ebit = (uint32_t)e * (uint32_t)p.OB;
      // bushes emptied before this step's eat are absent from S (:506): clear them
      for (int i = 0; i < ne; ++i) {
        const uint32_t v = p.eaten_xy[(int64_t)i * p.B + g];
        const int r = (int)p.eaten_rem[(int64_t)i * p.B + g] + (i == eat_idx ? 1 : 0);
        const int ddx = ox - xy_x(v), ddy = oy - xy_y(v);
        if (r == 0 && abs(ddx) <= p.cw && abs(ddy) <= p.ch)
          lds_clear(sA, ebit + plane + (uint32_t)((ddx + p.cw) * p.S + ddy + p.ch));
      }
      if (p.restrict_view) apply_view_mask(p, sA, ebit, role);
      // spawn_wolves (:325-326, :527-576) on the ring around the new position
      for (int wd = 0; wd < p.RW; ++wd) {
        uint32_t bits = spawnM[e * p.RW + wd];
        while (bits) {
          const int b = __ffs(bits) - 1;
          bits &= bits - 1;
          const uint32_t t = tiles[p.WH + wd * 32 + b];
          if (nw < SLOTS) wl[(nw++) * NE + e] = xy_pack(ox + tile_dx(t), oy + tile_dy(t));
          else wolf_of += 1;
        }
      }
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
    if (active) done = (p.reset_mask == nullptr) || (p.reset_mask[g] != 0);
  }

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
    const int ft = (int)ceil(food * (double)p.turns_empty);       // :450-452
    if (job) {
      if (MODE == MODE_STEP && p.t_planes) {
        p.t_food_turns[g] = (uint8_t)ft;
        p.t_role[g] = (uint8_t)role;
        p.t_status[g] = (uint8_t)status;
      }
      // reset (:231-248, spawn_ostriches :595-611)
      const int j = __popcll(jm & ((1ull << e) - 1ull));
      ep = (MODE == MODE_RESET) ? p.episode[g] + 1u : ep + 1u;
      const uint64_t ek = episode_key(p.seed, (uint64_t)(p.env_base + g), ep);
      const uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
      jobEnv[j] = (uint32_t)e;
      jobKey[2 * j] = b0;
      jobKey[2 * j + 1] = b1;
      turn = 0;
      ox = 0;
      oy = 0;
      status = 0;
      ne = 0;
      nw = 0;
      food = p.start_food_random
                 ? (double)draw_U(xy_pack(0, 0), make_ts(SITE_START_FOOD, 0, 0), b0, b1) * 0x1p-53
                 : p.start_food;
      role = p.start_role_random
                 ? (int)(draw_U(xy_pack(0, 0), make_ts(SITE_START_ROLE, 0, 0), b0, b1) >> 52)
                 : p.start_role;
      p.episode[g] = ep;
    }
    if (MODE == MODE_STEP || job) {
      p.food_turns[g] = (uint8_t)(int)ceil(food * (double)p.turns_empty);
      p.role[g] = (uint8_t)role;
      p.status[g] = (uint8_t)status;
      p.pos[g] = xy_pack(ox, oy);
      p.food[g] = food;
      p.turn[g] = turn;
    }
    if (MODE == MODE_STEP && !job) {
      for (int s = 0; s < nw; ++s) p.wolves[(int64_t)s * p.B + g] = wl[s * NE + e];
      p.misc[g] = misc_pack((uint32_t)role, (uint32_t)status, (uint32_t)nw, (uint32_t)ne);
    }
  }
  if (envlane && (bad | eaten_of | wolf_of)) {
    if (bad) atomicAdd(&p.counters[2], bad);
    if (eaten_of) atomicAdd(&p.counters[1], eaten_of);
    if (wolf_of) atomicAdd(&p.counters[0], wolf_of);
  }
  __syncthreads();

  const int n_jobs = (int)blk[0];
  const unsigned long long done_mask = (unsigned long long)blk[1] | ((unsigned long long)blk[2] << 32);
  if (n_jobs > 0) {
    // -------------------------------------------------------------- phase 4 (reset draws)
    {
      const int WH = p.WH;
      const int items = n_jobs * WH;
      int ij = tid / WH, ic = tid - (tid / WH) * WH;
      const int stepJ = kThreads / WH, stepC = kThreads - (kThreads / WH) * WH;
      const uint32_t ts_bush = make_ts(SITE_BUSH, 0, 0), ts_wolf = make_ts(SITE_SPAWN, 0, 0);
      for (int q = tid; q < items; q += kThreads) {
        const uint32_t je = jobEnv[ij], b0 = jobKey[2 * ij], b1 = jobKey[2 * ij + 1];
        const uint32_t t = tiles[ic];
        const uint32_t xy = xy_pack(tile_dx(t), tile_dy(t));  // ostrich at (0, 0)
        const uint32_t h1 = fmix32(xy ^ b0);
        const uint32_t ebit = je * (uint32_t)p.OB;
        const uint32_t hb = fmix32(h1 ^ ts_bush ^ b1);
        if (U_ge(h1, hb, ts_bush, b0, p.bush_t1)) lds_set(sB, ebit + plane + tile_bit(t));   // generate_bushes
        if (p.wolves_on) {                                                                  // initialize_wolves
          const uint32_t hw = fmix32(h1 ^ ts_wolf ^ b1);
          if (!U_ge(h1, hw, ts_wolf, b0, p.spawn_lt)) {
            lds_set(sB, ebit + tile_bit(t));
            lds_set(wolfM + ij * p.WHW, (uint32_t)ic);
          }
        }
        ic += stepC;
        ij += stepJ;
        if (ic >= WH) { ic -= WH; ij += 1; }
      }
    }
    __syncthreads();
    // -------------------------------------------------------------- phase 5 (reset envs)
    if (job) {
      const int j = __popcll(done_mask & ((1ull << e) - 1ull));
      const uint32_t ebit = (uint32_t)e * (uint32_t)p.OB;
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
          else atomicAdd(&p.counters[0], 1ull);
        }
      }
      p.misc[g] = misc_pack((uint32_t)role, 0u, (uint32_t)n, 0u);
    }
    if (tid == 0) p.block_resets[blockIdx.x] += (unsigned long long)n_jobs;
    __syncthreads();
  }

  // ---------------------------------------------------------------- phase 6 (expand + store)
  {
    const uint32_t OB = (uint32_t)p.OB;
    const uint32_t limit = (uint32_t)n_active * OB;      // valid bytes of this block's chunk
    uint8_t* out = p.planes + (size_t)g0 * OB;
    uint8_t* tout = (MODE == MODE_STEP && p.t_planes) ? p.t_planes + (size_t)g0 * OB : nullptr;
    const bool full_jobs = (MODE == MODE_RESET) && n_jobs == n_active;
    for (uint32_t d = tid; d < streamW; d += kThreads) {
      const uint32_t b0 = d << 5;
      if (b0 >= limit) break;
      uint32_t dm = 0;   // bits of this dword that belong to job (done / flagged) envs
      if (n_jobs > 0) {
        if (full_jobs) {
          dm = ~0u;
        } else {
          const uint32_t e_lo = udiv(b0, OB, p.magic_OB);
          const uint32_t e_hi = min(udiv(b0 + 31u, OB, p.magic_OB), (uint32_t)NE - 1u);
          for (uint32_t ee = e_lo; ee <= e_hi; ++ee) {
            if (!((done_mask >> ee) & 1ull)) continue;
            const uint32_t lo = max(ee * OB, b0) - b0;
            const uint32_t hi = min((ee + 1u) * OB, b0 + 32u) - b0;  // exclusive, <= 32
            dm |= (hi >= 32u ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
          }
        }
      }
      uint32_t v;
      if (MODE == MODE_STEP) v = (sA[d] & ~dm) | (sB[d] & dm);
      else v = sB[d];
      const uint32_t write_mask = (MODE == MODE_STEP) ? ~0u : dm;
      if (write_mask == ~0u && b0 + 32u <= limit) {
        uint4 q0, q1;
#pragma unroll
        for (int k = 0; k < 4; ++k) (&q0.x)[k] = (((v >> (4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
#pragma unroll
        for (int k = 0; k < 4; ++k) (&q1.x)[k] = (((v >> (16 + 4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
        *reinterpret_cast<uint4*>(out + b0) = q0;
        *reinterpret_cast<uint4*>(out + b0 + 16) = q1;
      } else if (write_mask) {
        for (uint32_t k = 0; k < 32u && b0 + k < limit; ++k)
          if ((write_mask >> k) & 1u) out[b0 + k] = (uint8_t)((v >> k) & 1u);
      }
      if (MODE == MODE_STEP && tout && dm) {
        const uint32_t va = sA[d];
        for (uint32_t k = 0; k < 32u && b0 + k < limit; ++k)
          if ((dm >> k) & 1u) tout[b0 + k] = (uint8_t)((va >> k) & 1u);
      }
    }
  }
}

// explicit instantiations used by wab_capi.hip
#define WAB_INST(M, S) template __global__ void wab_kernel<M, S>(Params);
WAB_INST(MODE_STEP, 8)
WAB_INST(MODE_STEP, 16)
WAB_INST(MODE_STEP, 32)
WAB_INST(MODE_RESET, 8)
WAB_INST(MODE_RESET, 16)
WAB_INST(MODE_RESET, 32)

}  // namespace wab
