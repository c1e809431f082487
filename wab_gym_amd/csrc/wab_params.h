// wab_params.h — kernel parameter block shared by the C-ABI host code and the HIP kernels.
//
// Everything the fused step needs, resolved once at wab_create from wab_config
// (include/wab.h) and passed by value as the kernel argument (scalar-loaded).
#pragma once

#include "wab_build_guard.h"

#include <stdint.h>

namespace wab {

constexpr int kEnvsPerBlock = 64;   // env lanes = wave 0 of the block
constexpr int kThreads = 256;       // 4 waves: waves 0..3 share the tile-parallel phases
constexpr int kMaxWolfSlots = 32;
constexpr int kGapChunk = 128;      // tiles per keyed spawn-set chunk (oracle/keyed_rng.py GAP_CHUNK)

// device counters (Params::counters, read back by wab_get_counters; rare events: atomics)
enum : int {
  CTR_WOLF_OVERFLOW = 0,
  CTR_EATEN_OVERFLOW = 1,
  CTR_BAD_ACTIONS = 2,
  CTR_EGO_MISSING = 3,
  CTR_STEPS = 4,             // + B per step launch (one lane of workgroup 0)
  CTR_HANDOFF_TIMEOUTS = 5,  // bounded LDS hand-off waits that gave up (must stay 0)
  CTR_WOLF_OVERFLOW_RESET = 6,  // the part of CTR_WOLF_OVERFLOW dropped by a reset (initial wolves)
  kNumCounters = 8
};

// per-env packed misc word: role [0,8) status [8,10) n_wolves [10,16) n_eaten [16,24)
// n_emptied [24,32) (eaten-log entries with no berries left)
__host__ __device__ inline uint32_t misc_pack(uint32_t role, uint32_t status, uint32_t nw, uint32_t ne,
                                              uint32_t ndep) {
  return (role & 0xFFu) | ((status & 3u) << 8) | ((nw & 63u) << 10) | ((ne & 0xFFu) << 16) |
         ((ndep & 0xFFu) << 24);
}
__host__ __device__ inline uint32_t misc_role(uint32_t m) { return m & 0xFFu; }
__host__ __device__ inline uint32_t misc_status(uint32_t m) { return (m >> 8) & 3u; }
__host__ __device__ inline uint32_t misc_nw(uint32_t m) { return (m >> 10) & 63u; }
__host__ __device__ inline uint32_t misc_ne(uint32_t m) { return (m >> 16) & 0xFFu; }
__host__ __device__ inline uint32_t misc_ndep(uint32_t m) { return m >> 24; }

// tiles are packed (x & 0xFFFF) | (y << 16) with x, y int16 (absolute world coordinates)
__host__ __device__ inline uint32_t xy_pack(int32_t x, int32_t y) {
  return ((uint32_t)x & 0xFFFFu) | ((uint32_t)y << 16);
}
__host__ __device__ inline int32_t xy_x(uint32_t p) { return (int32_t)(int16_t)(p & 0xFFFFu); }
__host__ __device__ inline int32_t xy_y(uint32_t p) { return (int32_t)(int16_t)(p >> 16); }

// diagnostic builds (-DWAB_STAMPS): int64 stamps per workgroup (tools/phase_stamps.py)
constexpr int kStampStride = 48;

struct Params {
  // ---- geometry
  int32_t W, H, S;          // viewport width (axis 0), height (axis 1), row stride in bytes
  int32_t cw, ch, margin;   // W/2, H/2, wolf_spawn_margin
  int32_t OB;               // obs bytes per env = 3*W*S (also obs bits per env in the LDS stream)
  int32_t WH, R, NT;        // bush tiles, ring tiles, WH + R
  int32_t RW, WHW;          // dwords of a ring mask / of a WH mask (WHW = bush bitmap words)
  int32_t SL;               // strip slots per env = max(W, H) (tiles entering the view on a move)
  uint32_t magic_OB;        // floor(2^32 / OB) + 1 (division helper)
  uint32_t magic_CPE;       // the same for OB / 16 (16-byte obs chunks per env, wide kernel)
  // ---- rules
  int32_t n_actions;
  int32_t act_role[6];      // role set by each action, -1 = NaN (unchanged); moves: decode_action()
  // "U >= T" tests on 53-bit draws U = hi << 21 | lo21, split as (T >> 21, T & 0x1FFFFF);
  // T = 2^53 ("never") is encoded (0xFFFFFFFF, 0xFFFFFFFF) which no (hi, lo21) reaches
  uint32_t keep_th, keep_tl;    // despawn: wolf kept iff U >= keep_gt + 1  (u > p, wab_env.py:263)
  uint32_t bush_th, bush_tl;    // bush present iff U >= T_1                 (wab_env.py:632-635)
  // wolf spawns (u < p/2, wab_env.py:573, :590) are drawn as sets by geometric gaps in
  // chunks of kGapChunk tiles (oracle/keyed_rng.py spawn_hits): gap[g] = floor((1 - q)^g
  // 2^53), g = 0..kGapChunk; the first draw of a chunk of m tiles is a miss of all of them
  // iff U < gap[m], tested split like the above for a full chunk and for the last one
  const uint64_t* gap;          // device [kGapChunk + 1]
  int32_t n_gap;                // kGapChunk (the tables' size)
  float gap_inv_l2;             // 1 / log2(1 - q) (the guess of gap_count_fast; the table decides)
  uint32_t gap_full_th, gap_full_tl;  // gap[kGapChunk]
  uint32_t gap_ring_th, gap_ring_tl;  // gap[m] of the ring's last chunk
  uint32_t gap_view_th, gap_view_tl;  // gap[m] of the view's last chunk
  const uint64_t* thresholds;  // device [max_berries] T_k
  const uint32_t* tables;      // device: [WH] view-cell world offsets (cw - i, ch - j), then from
  int32_t ring_at;             //   ring_at (16-B aligned) the R ring offsets, padded to a multiple of 4
  int32_t max_berries;
  float bush_power;            // the guess of bush_value_fast (the thresholds decide)
  double fill, hunger;
  double r_turn, r_killed, r_starve, r_finish, r_eat;
  double start_food;
  int32_t start_role, start_food_random, start_role_random;
  int32_t max_turns, turns_empty;
  int32_t lookout_only, restrict_view, wolves_on, wolves_can_move, god_mode, autoreset;
  uint32_t mask_rows[2][11];  // restrict_view: 11-bit row masks per role (bit j <=> mask[i][j])
  uint32_t small_masks[3][4]; // W*H <= 128: column 0, column H-1, valid-bit masks of the bitmap
  uint32_t view121[2][4];     // restrict_view at 11x11: the row masks as one 121-bit plane mask
  // ---- identity
  uint64_t seed;
  int64_t env_base;
  int64_t B;
  int32_t eaten_cap;
  int32_t n_steps;     // steps per launch (wab_rollout on the small kernel: the I/O arrays are
                       // [n_steps][...], step t at offset t * B; 1 otherwise)
  int32_t wolf_cap;    // wolf rows per env (wab_config.wolf_slots); the wide kernel keeps the
                       // first 8 in registers and the rest (rare) in their HBM rows
  // ---- state (device, SoA, env innermost)
  uint4* hdr;          // [B] {ostrich tile, turn, misc, episode (0xFFFFFFFF before the first reset)}
  double* food;        // [B]
  uint32_t* wolves;    // [slots][B] packed tiles
  uint32_t* eaten_xy;  // [cap][B] packed tiles
  uint8_t* eaten_rem;  // [cap][B] berries left
  uint32_t* bushmap;   // [WHW][B] bush presence of the current view, bit i*H + j (post-eat)
  unsigned long long* counters;      // [kNumCounters] (CTR_*)
  unsigned long long* block_resets;  // [n_blocks]: resets done by each block (owned; no-return atomic adds)
  // ---- io (device, caller-owned)
  const int8_t* actions;
  const uint8_t* reset_mask;
  uint8_t* planes;
  uint8_t* food_turns;
  uint8_t* role;
  uint8_t* status;
  float* reward;
  uint8_t* done;
  uint8_t* t_planes;   // terminal obs (nullable)
  uint8_t* t_food_turns;
  uint8_t* t_role;
  uint8_t* t_status;
  float* features;     // wab_step_features: PragmaticObsWrapper features [B][F] (else null)
  float* returns;      // wab_rollout_features: discounted returns [n_steps][B] (else null)
  const float* bootstrap;  // ... R after the last step [B] (null: 0)
  double gamma;
  unsigned long long* stamps;  // diagnostic builds only (-DWAB_STAMPS): [n_blocks][40] s_memrealtime
};

// LDS carve of one workgroup (dword offsets, each region 16-byte aligned).
struct LdsLayout {
  uint32_t sA, sB, spawnM, wolfM, bm, masks, tiles, snap, jobEnv, jobKey, blk, thr, total;
};

__host__ __device__ inline uint32_t lds_align4(uint32_t n) { return (n + 3u) & ~3u; }

__host__ __device__ inline LdsLayout lds_layout(const Params& p, int /*slots*/) {
  const uint32_t NE = (uint32_t)kEnvsPerBlock;
  const uint32_t streamW = (NE * (uint32_t)p.OB) >> 5;
  LdsLayout L;
  uint32_t o = 0;
  L.sA = o; o += lds_align4(streamW);
  L.sB = o; o += lds_align4(streamW);
  L.spawnM = o; o += lds_align4(NE * (uint32_t)p.RW);
  L.wolfM = o; o += lds_align4(NE * (uint32_t)p.WHW);
  L.bm = o; o += lds_align4(NE * (uint32_t)p.WHW);
  L.masks = o; o += lds_align4(3u * (uint32_t)p.WHW);
  L.tiles = o; o += lds_align4((uint32_t)p.NT);
  L.snap = o; o += NE * 4u;
  L.jobEnv = o; o += NE;
  L.jobKey = o; o += 2u * NE;
  L.blk = o; o += 4u;
  L.thr = o; o += lds_align4(2u * (uint32_t)p.max_berries);
  L.total = o;
  return L;
}

// wab_rollout_features computes the returns in the kernel for segments of at most this many
// steps (their reward codes in LDS); longer ones run wab_discounted_returns_exact after it
constexpr int kMaxFusedReturnSteps = 128;

// LDS of the four-wave small-view step (wab_step_small.hip): one 64-env group per
// workgroup (dwords)
// the small kernel's multi-step launches keep eaten-log entries 0..3 of an env in W0's
// registers and 4 .. kSmallLog - 1 in LDS; later ones stay in HBM
constexpr int kSmallLog = 12;
struct SmallLayout {
  uint32_t tiles, thr, gap, stream, stream_words, cval, flag, wolfp, kill, bushp, strip, gone, info, spawn, jbm, jkey;
  uint32_t carry, act;  // multi-step launches: the new episodes' state for the next step, its actions
  uint32_t elog;        // multi-step launches: eaten-log entries 4 .. kSmallLog - 1 (xy dwords, then rem bytes)
  uint32_t stream2;     // multi-step launches: the second obs bit-stream (steps alternate)
  uint32_t fbits, fzero, ftab, scal, total;  // fused features (wab_step_features): bits, tables, scalars
  uint32_t rcode;       // wab_rollout_features with returns: [n_steps][64] reward codes (bytes)
  uint32_t wcar;        // multi-step launches of 32-slot handles: W2's wolf slots between steps ([k][64])
};

// wolf slots a multi-step launch carries in W2's registers from step to step: all of them up to
// 16 slots; a 32-slot handle carries its slots in LDS (Lds::wcar), so that the carry and the
// step's own 32 slots do not overflow the 128 VGPRs (132 bytes per lane of scratch otherwise)
__host__ __device__ constexpr int carry_reg_slots(int slots) { return slots <= 16 ? slots : 0; }

__host__ __device__ inline SmallLayout small_layout(const Params& p) {
  // (the regions whose size depends on a runtime option come last, so that with the G = 11
  // geometry every other offset is a compile-time immediate, not a live scalar register)
  SmallLayout L;
  uint32_t o = 0;
  L.tiles = o; o += lds_align4((uint32_t)p.WH);
  L.stream_words = lds_align4((64u * (uint32_t)p.OB + 31u) >> 5);
  L.stream = o; o += L.stream_words + 4u;  // + slack for stream_or128's fifth dword
  L.cval = o; o += 64u;
  L.flag = o; o += 4u;
  L.wolfp = o; o += 64u * 4u;
  L.kill = o; o += 64u;
  L.bushp = o; o += 64u * 4u;
  L.strip = o; o += 2u * 64u;
  L.gone = o; o += 64u * 4u;
  L.info = o; o += 64u;
  L.spawn = o; o += 64u * 4u;
  L.jbm = o; o += 64u * 4u;
  L.jkey = o; o += 2u * 2u * 64u;
  L.carry = o; o += 8u * 64u;  // per env: role | new wolves << 8, food (2), wolf cells (4), pad
  L.act = o; o += 16u;         // 64 int8 actions
  L.elog = o; o += (uint32_t)(kSmallLog - 4) * 64u * 5u / 4u;
  L.stream2 = o; o += L.stream_words + 4u;
  L.wcar = o;
  if (p.wolf_cap > 16) o += (uint32_t)(p.wolf_cap - carry_reg_slots(p.wolf_cap)) * 64u;
  L.gap = o; o += lds_align4(2u * ((uint32_t)p.n_gap + 1u));          // spawn-set gap table
  L.thr = o; o += lds_align4(2u * ((uint32_t)p.max_berries + 4u));  // pad, T_1..T_n, 2 pads
  L.fbits = L.ftab = L.fzero = L.scal = o;
  if (p.features) {  // fused features: 64 envs x F bits (+ slack), the per-cell tables (zeroed
                     // together), the envs' scalars
    const int md = p.W / 2 + p.H / 2 + 1;
    const uint32_t F = (uint32_t)(16 * (md + 1) + 88 + 2 + (p.turns_empty + 1) + 2 + 3 + 121);
    L.fbits = o; o += lds_align4(((64u * F + 31u) >> 5) + 4u);
    L.ftab = o; o += lds_align4(128u + 4u * ((uint32_t)md + 4u));
    L.fzero = o - L.fbits;
    L.scal = o; o += 64u;
  }
  L.rcode = o;
  if (p.returns) o += 16u * (uint32_t)p.n_steps;  // one byte per env and step
  L.total = o;
  return L;
}

// LDS of the wide-view step (wab_step_wide.hip; W, H <= 32, rows of S = 16 or 32 bytes):
// one 64-env group per workgroup, view bitmaps as one dword per row (bit j = column j),
// env-major with a 33-dword pitch so that lanes (= envs) touching the same row hit
// different banks (dwords)
constexpr uint32_t kWidePitch = 33;
struct WideLayout {
  uint32_t bm, wp, spawn, spw, ring, gap, thr, cval, info, blk, jobEnv, jobKey;
  uint32_t total;
};

__host__ __device__ inline WideLayout wide_layout(const Params& p) {
  WideLayout L;
  uint32_t o = 0;
  L.bm = o; o += 64u * kWidePitch + 4u;       // bush bitmaps (snapshot, pre-eat)
  o = lds_align4(o);
  L.wp = o; o += 64u * kWidePitch + 4u;       // wolf grids
  o = lds_align4(o);
  L.spw = (((uint32_t)p.R + 31u) >> 5) | 1u;  // spawn-mask dwords per env (odd pitch)
  L.spawn = o; o += lds_align4(64u * L.spw);
  L.ring = o; o += lds_align4((uint32_t)p.R);  // spawn-ring offsets
  L.gap = o; o += lds_align4(2u * ((uint32_t)p.n_gap + 1u));  // spawn-set gap table
  L.thr = o; o += lds_align4(2u * ((uint32_t)p.max_berries + 4u));  // pad, T_1..T_n, 2 pads
  L.cval = o; o += 64u;                       // generated berries of the ostrich's tile
  L.info = o; o += 64u;                       // W0 -> all: job | emptied << 1
  L.blk = o; o += 4u;                         // n_jobs, job mask lo, hi
  L.jobEnv = o; o += 64u;
  L.jobKey = o; o += 128u;
  L.total = o;
  return L;
}

// LDS of the wide view's multi-step build (wab_rollout_wide): the view bitmaps and wolf grids
// twice (step t builds its obs in buffer t & 1 while the store waves write step t - 1's from
// the other), at a 31-dword pitch (W <= 31: odd viewports; odd, so lanes = envs still hit
// distinct banks), plus the state the waves carry between steps.  At 31x31 it is ~39 KB, so
// that four workgroups (B = 65536: all 1024 at once) fit a CU's 160 KB.
constexpr uint32_t kRollPitch = 31;
constexpr int kWideRollLog = 8;  // eaten-log entries W0 keeps on chip (0..3 in registers, 4..7 in
                                 // LDS; later ones, rare, in HBM)
struct WideRollLayout {
  uint32_t bm[2], wp[2], spawn, spw, ring, gap, thr, cval, info, blk, jobEnv, jobKey;
  uint32_t nhdr, act, flag;  // next headers (W0), next actions (W3), hand-off flags
  uint32_t elxy, elrem;      // eaten-log entries 4..kWideRollLog-1 (W0)
  uint32_t total;
};

__host__ __device__ inline WideRollLayout wide_roll_layout(const Params& p) {
  WideRollLayout L;
  uint32_t o = 0;
  for (int b = 0; b < 2; ++b) {
    L.bm[b] = o; o += lds_align4(64u * kRollPitch);
    L.wp[b] = o; o += lds_align4(64u * kRollPitch);
  }
  L.spw = (((uint32_t)p.R + 31u) >> 5) | 1u;
  L.spawn = o; o += lds_align4(64u * L.spw);
  L.ring = o; o += lds_align4((uint32_t)p.R);
  L.gap = o; o += lds_align4(2u * ((uint32_t)p.n_gap + 1u));
  L.thr = o; o += lds_align4(2u * ((uint32_t)p.max_berries + 4u));
  L.cval = o; o += 64u;
  L.info = o; o += 64u;
  L.blk = o; o += 4u;
  L.jobEnv = o; o += 64u;
  L.jobKey = o; o += 128u;
  L.nhdr = o; o += 64u * 4u;                  // uint4 per env
  L.act = o; o += 16u;                        // 64 int8 actions
  L.flag = o; o += 8u;  // [0] W1's scroll, [1] W2's tables (step 0), [2] W0 at B1 / B2 (step-tagged),
                        // [4], [5] the obs-row queues' block counters (by step parity)
  L.elxy = o; o += 64u * (uint32_t)(kWideRollLog - 4);   // [entry - 4][env] tiles
  L.elrem = o; o += 16u * (uint32_t)(kWideRollLog - 4);  // [entry - 4][env] berries left (bytes)
  L.total = o;
  return L;
}

// Egocentric bush proximities (wab_egocentric.hip): reads the step's per-env state and keeps
// a per-env path of ostrich tiles, one entry per turn of the current episode.
struct EgoParams {
  int32_t cw, ch, Q;        // Q = max_distance = W//2 + H//2 + 1 (wab_env.py:933-935), <= 31
  int32_t cap;              // path entries per env
  int32_t n_diamond;        // tiles with |dx| + |dy| <= Q
  int32_t eaten_cap;
  uint32_t bush_th, bush_tl;
  uint64_t seed;
  int64_t env_base, B;
  const uint4* hdr;
  const uint32_t* eaten_xy;
  const uint8_t* eaten_rem;
  const uint32_t* diamond;  // [n_diamond] packed (dx, dy) int8 offsets
  uint4* path;              // [cap][B] {ostrich tile, food>0 tiles seen so far, episode, 0}
  const uint8_t* mask;      // nullable: only envs with mask[i] != 0
  uint8_t* out;             // [B][5]
  unsigned long long* counters;  // [kNumCounters]: CTR_EGO_MISSING, path entries missing (stale or beyond cap)
};

// wab_featurize / wab_featurize_superbasic (wab_features.hip)
struct FeatParams {
  int32_t W, H, S, OB, md, F, turns_empty, restrict_view;
  int32_t kind;  // 0 PragmaticObsWrapper (:726-824), 1 SuperBasicObservationWrapper (:900-927)
  int64_t B;
  uint32_t mask_rows[2][11];
  uint32_t view121[2][4];    // the same masks as 121-bit cell masks (bit i*11 + j)
  const uint8_t* planes;
  const uint8_t* food_turns;
  const uint8_t* role;
  const uint8_t* status;
  const uint8_t* view_mask;  // [B][11][11] or null (derive from role)
  float* out;                // [B][F]
};

// The rewards one step of an env can return (wab_env.py:299-340: 0 + r_x, or 0 + r_eat + r_x
// for r_x in per turn / finishing / starving / killed) as (float32 bits, exact double) pairs:
// the double a float32 device reward came from (wab_discounted_returns_exact).  n = 0: none.
struct RewardTable {
  int32_t n;
  uint32_t f32[8];
  double f64[8];
};

// wab_render (wab_render.hip)
struct RenderParams {
  int32_t W, H, S, OB, scale, restrict_view;
  int32_t draw_health;       // the turns-until-starve text overlay (wab_env.py:496-500)
  int64_t B;
  uint32_t mask_rows[2][11];
  const uint8_t* planes;
  const uint8_t* food_turns;
  const uint8_t* role;
  const uint8_t* status;
  uint8_t* rgb;
};

}  // namespace wab
