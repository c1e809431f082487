/*
 * wab_oracle.c — TEST INFRASTRUCTURE: scalar C restatement of the reference step.
 *
 * Restates wab_env.py (johnmatthewtennant/wab-gym) `reset` (:231-248) and `step`
 * (:250-342) for one env at a time, looping over a batch.  Random draws follow the keyed
 * RNG defined in oracle/keyed_rng.py (the same definition the golden vectors were
 * generated under).  Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 *
 * Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 */
#include "wab_oracle.h"

#include "../wab_gym_amd/csrc/wab_glyphs.h" /* data: PIL digit coverage (tools/make_glyphs.py) */

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ keyed RNG */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

uint64_t wabo_episode_key(uint64_t seed, uint64_t env, uint64_t episode) {
  uint64_t a = mix64(seed + 0x9E3779B97F4A7C15ULL);
  uint64_t b = mix64(a ^ env);
  return mix64(b ^ episode);
}

uint64_t wabo_draw_U(uint64_t ek, uint32_t site, int64_t turn, int64_t x, int64_t y, uint32_t k) {
  uint32_t b0 = (uint32_t)ek, b1 = (uint32_t)(ek >> 32);
  uint32_t xy = (uint32_t)(x & 0xFFFF) | ((uint32_t)(y & 0xFFFF) << 16);
  uint32_t ts = (site & 0xFu) | ((k & 0xFFu) << 4) | ((uint32_t)(turn & 0xFFFFF) << 12);
  uint32_t h1 = fmix32(xy ^ b0);
  uint32_t hi = fmix32(h1 ^ ts ^ b1);
  uint32_t rot = (ts << 16) | (ts >> 16);
  uint32_t lo = fmix32(h1 ^ rot ^ b0 ^ 0x9E3779B9u);
  return ((uint64_t)hi << 21) | (uint64_t)(lo >> 11);
}

enum { SITE_BUSH = 1, SITE_SPAWN = 2, SITE_DESPAWN = 3, SITE_START_FOOD = 4, SITE_START_ROLE = 5, SITE_GAP = 6 };

/* wolf spawns as a set (keyed_rng.py: gap_thresholds, gap_count, spawn_hits): P[g] =
 * floor((1 - q)^g 2^53), q = T 2^-53, the power a running product in double */
static uint64_t* gap_thresholds(uint64_t T, int n) {
  uint64_t* P = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n + 1));
  const double omq = ldexp((double)((1ULL << 53) - T), -53);
  double p = 1.0;
  P[0] = 1ULL << 53;
  for (int g = 1; g <= n; ++g) {
    p = p * omq;
    P[g] = (uint64_t)floor(ldexp(p, 53));
  }
  return P;
}

/* misses before the next hit among m tiles: #{g in 1..m : U < P[g]} (m: none) */
static int gap_count(uint64_t U, const uint64_t* P, int m) {
  int lo = 0, hi = m;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (U < P[mid]) lo = mid; else hi = mid - 1;
  }
  return lo;
}

/* calls hit(ctx, index) for each tile in [0, n) that spawns a wolf at `turn`, ascending;
 * chunks of 128 tiles, each its own gap sequence (draw k of chunk c: "tile" (k, c)) */
enum { GAP_CHUNK = 128 };
static void spawn_hits(uint64_t ek, int64_t turn, int n, const uint64_t* P, void (*hit)(void*, int), void* ctx) {
  for (int c = 0; c * GAP_CHUNK < n; ++c) {
    const int base = c * GAP_CHUNK, m = n - base < GAP_CHUNK ? n - base : GAP_CHUNK;
    int pos = 0;
    for (uint32_t k = 0; pos < m; ++k) {
      const uint64_t U = wabo_draw_U(ek, SITE_GAP, turn, (int64_t)k, (int64_t)c, 0);
      const int G = gap_count(U, P, m - pos);
      if (G >= m - pos) break;
      pos += G;
      hit(ctx, base + pos);
      pos += 1;
    }
  }
}

/* ------------------------------------------------------------------ state */
typedef struct { int32_t x, y; } xy_t;
typedef struct { int32_t x, y, rem; } eaten_t;

typedef struct {
  int64_t env_id;
  int64_t episode; /* -1 before the first reset */
  uint64_t ek;
  int32_t turn, x, y, role, status;
  double food;
  int nw, capw;
  xy_t* wolves;
  int ne, cape;
  eaten_t* eaten;
  /* tiles ever in view this episode (the rows of the reference's `bushes` table,
   * generate_bushes wab_env.py:613-629): open-addressing set + insertion list */
  int nseen, capseen;
  uint64_t* seen_keys; /* capacity 2*capseen, 0 = empty */
  xy_t* seen;
} oenv;

struct wabo_batch {
  wab_config cfg;
  uint64_t* thresholds;
  int64_t batch;
  uint64_t seed;
  int n_actions;
  int act_dx[6], act_dy[6], act_role[6]; /* act_role -1 = NaN (no role change) */
  uint64_t keep_gt, spawn_lt;
  uint64_t* gap; /* gap_thresholds(spawn_lt, GAP_CHUNK) */
  double fill, hunger;
  int stride, plane_bytes, obs_bytes;
  oenv* envs;
};

/* masks wab_env.py:109-139 */
static const uint8_t LOOKOUT_MASK[11][11] = {
    {1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1}, {1, 1, 0, 0, 0, 0, 0, 0, 0, 1, 1},
    {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1}, {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1}, {1, 1, 0, 0, 0, 0, 0, 0, 0, 1, 1},
    {1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1}};
static const uint8_t GATHERER_MASK[11][11] = {
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1}, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1},
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1}, {1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1},
    {1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1}, {1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1},
    {1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1}, {1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1},
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1}, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1},
    {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1}};

/* number of k with U >= T_k: the reference's round(u**power * max) (wab_env.py:631-635) */
static int bush_value(const wabo_batch* b, uint64_t U) {
  int lo = 0, hi = b->cfg.max_berries_per_bush; /* count of thresholds <= U */
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (b->thresholds[mid] <= U) lo = mid + 1; else hi = mid;
  }
  return lo;
}

/* remaining berries at a tile: eaten log, else the tile's generated value (wab_env.py:613-629) */
static int bush_remaining(const wabo_batch* b, const oenv* e, int32_t x, int32_t y) {
  for (int i = 0; i < e->ne; ++i)
    if (e->eaten[i].x == x && e->eaten[i].y == y) return e->eaten[i].rem;
  return bush_value(b, wabo_draw_U(e->ek, SITE_BUSH, 0, x, y, 0));
}

static void set_remaining(oenv* e, int32_t x, int32_t y, int rem) {
  for (int i = 0; i < e->ne; ++i)
    if (e->eaten[i].x == x && e->eaten[i].y == y) { e->eaten[i].rem = rem; return; }
  if (e->ne == e->cape) {
    e->cape = e->cape ? 2 * e->cape : 16;
    e->eaten = (eaten_t*)realloc(e->eaten, sizeof(eaten_t) * (size_t)e->cape);
  }
  e->eaten[e->ne].x = x; e->eaten[e->ne].y = y; e->eaten[e->ne].rem = rem;
  e->ne++;
}

static uint64_t seen_key(int32_t x, int32_t y) {
  return ((uint64_t)(uint32_t)(x + 0x40000000) << 32) | (uint32_t)(y + 0x40000000);
}

static void seen_insert_key(oenv* e, uint64_t k) {
  const uint64_t m = 2 * (uint64_t)e->capseen - 1;
  uint64_t i = (k * 0x9E3779B97F4A7C15ull) >> 17;
  for (;; ++i)
    if (e->seen_keys[i & m] == 0) { e->seen_keys[i & m] = k; return; }
}

/* a tile enters view: it joins the bush table once (wab_env.py:619 skips known tiles) */
static void seen_add(oenv* e, int32_t x, int32_t y) {
  const uint64_t k = seen_key(x, y);
  if (e->capseen) {
    const uint64_t m = 2 * (uint64_t)e->capseen - 1;
    for (uint64_t i = (k * 0x9E3779B97F4A7C15ull) >> 17;; ++i) {
      if (e->seen_keys[i & m] == k) return;
      if (e->seen_keys[i & m] == 0) break;
    }
  }
  if (e->nseen == e->capseen) { /* grow: list x2, table rebuilt at 2x the list */
    e->capseen = e->capseen ? 2 * e->capseen : 256;
    e->seen = (xy_t*)realloc(e->seen, sizeof(xy_t) * (size_t)e->capseen);
    free(e->seen_keys);
    e->seen_keys = (uint64_t*)calloc(2 * (size_t)e->capseen, sizeof(uint64_t));
    for (int i = 0; i < e->nseen; ++i) seen_insert_key(e, seen_key(e->seen[i].x, e->seen[i].y));
  }
  seen_insert_key(e, k);
  e->seen[e->nseen].x = x; e->seen[e->nseen].y = y;
  e->nseen++;
}

static void seen_view(const wabo_batch* b, oenv* e) { /* visible_coords wab_env.py:510-525 */
  const int cw = b->cfg.width / 2, ch = b->cfg.height / 2;
  for (int tx = e->x - cw; tx <= e->x + cw; ++tx)
    for (int ty = e->y - ch; ty <= e->y + ch; ++ty) seen_add(e, tx, ty);
}

static void seen_clear(oenv* e) {
  if (e->capseen) memset(e->seen_keys, 0, 2 * (size_t)e->capseen * sizeof(uint64_t));
  e->nseen = 0;
}

static void push_wolf(oenv* e, int32_t x, int32_t y) {
  if (e->nw == e->capw) {
    e->capw = e->capw ? 2 * e->capw : 8;
    e->wolves = (xy_t*)realloc(e->wolves, sizeof(xy_t) * (size_t)e->capw);
  }
  e->wolves[e->nw].x = x; e->wolves[e->nw].y = y;
  e->nw++;
}

/* spawn_hits callbacks: tile index -> wolf (view cell c = i*H + j at (cw - i, ch - j); ring
 * tile r in the order of keyed_rng.ring_index) */
typedef struct { oenv* e; int W, H, m; } hit_ctx;

static void push_view_cell(void* v, int c) {
  const hit_ctx* h = (const hit_ctx*)v;
  push_wolf(h->e, h->e->x + h->W / 2 - c / h->H, h->e->y + h->H / 2 - c % h->H);
}

static void push_ring_tile(void* v, int r) {
  const hit_ctx* h = (const hit_ctx*)v;
  const int m = h->m, Wm = h->W + 2 * m;
  int xi, yi;
  if (r < 2 * m * Wm) {
    const int band = r / Wm;
    xi = r % Wm;
    yi = band < m ? band : band + h->H;
  } else {
    const int r2 = r - 2 * m * Wm, band = r2 / h->H;
    yi = m + r2 % h->H;
    xi = band < m ? band : band + h->W;
  }
  push_wolf(h->e, h->e->x + xi - h->W / 2 - m, h->e->y + yi - h->H / 2 - m);
}

/* ------------------------------------------------------------------ construction */
wabo_batch* wabo_create(const wab_config* cfg, int64_t batch, uint64_t seed, int64_t env_id_base) {
  if (cfg->width % 2 == 0 || cfg->height % 2 == 0) return NULL; /* wab_env.py:147-148 */
  wabo_batch* b = (wabo_batch*)calloc(1, sizeof(wabo_batch));
  b->cfg = *cfg;
  b->batch = batch;
  b->seed = seed;
  int nb = cfg->max_berries_per_bush;
  b->thresholds = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(nb > 0 ? nb : 1));
  for (int k = 0; k < nb; ++k) b->thresholds[k] = cfg->bush_thresholds[k];
  b->cfg.bush_thresholds = NULL;
  /* action tables wab_env.py:149-182: up (y+1), right (x+1), down (y-1), left (x-1) */
  static const int dx[6] = {0, 1, 0, -1, 0, 0}, dy[6] = {1, 0, -1, 0, 0, 0};
  for (int a = 0; a < 6; ++a) { b->act_dx[a] = dx[a]; b->act_dy[a] = dy[a]; b->act_role[a] = -1; }
  if (cfg->gatherer_only) { b->n_actions = 5; b->act_role[4] = 1; }
  else if (cfg->lookout_only) { b->n_actions = 5; b->act_role[4] = 0; }
  else { b->n_actions = 6; b->act_role[4] = 1; b->act_role[5] = 0; }
  /* u > despawn keeps a wolf (:263); u < chance/2 spawns one (:573) */
  b->keep_gt = (uint64_t)floor(ldexp(cfg->wolf_chance_to_despawn, 53));
  b->spawn_lt = (uint64_t)ceil(ldexp(cfg->chance_wolf_on_square / 2.0, 53));
  b->gap = gap_thresholds(b->spawn_lt, GAP_CHUNK);
  b->fill = 1.0 / (double)cfg->turns_to_fill_food;    /* :307-309 */
  b->hunger = 1.0 / (double)cfg->turns_to_empty_food; /* :316 */
  b->stride = cfg->plane_stride > 0 ? cfg->plane_stride : cfg->height;
  b->plane_bytes = cfg->width * b->stride;
  b->obs_bytes = 3 * b->plane_bytes;
  b->envs = (oenv*)calloc((size_t)batch, sizeof(oenv));
  for (int64_t i = 0; i < batch; ++i) {
    b->envs[i].env_id = env_id_base + i;
    b->envs[i].episode = -1;
  }
  return b;
}

void wabo_destroy(wabo_batch* b) {
  if (!b) return;
  for (int64_t i = 0; i < b->batch; ++i) {
    free(b->envs[i].wolves);
    free(b->envs[i].eaten);
    free(b->envs[i].seen);
    free(b->envs[i].seen_keys);
  }
  free(b->envs);
  free(b->thresholds);
  free(b->gap);
  free(b);
}

int wabo_num_actions(const wabo_batch* b) { return b->n_actions; }

typedef struct { int32_t* out; int cap, n; } hits_out;
static void collect_hit(void* v, int i) {
  hits_out* h = (hits_out*)v;
  if (h->n < h->cap) h->out[h->n] = i;
  h->n++;
}

int wabo_spawn_hits(const wabo_batch* b, uint64_t ek, int64_t turn, int n, int32_t* out, int cap) {
  hits_out h = {out, cap, 0};
  spawn_hits(ek, turn, n, b->gap, collect_hit, &h);
  return h.n;
}

uint64_t wabo_gap_threshold(const wabo_batch* b, int g) { return b->gap[g]; }

/* ------------------------------------------------------------------ observation */
/* grids from the snapshot (wab_env.py:393-444): planes are [3][W][stride] */
static void render_planes(const wabo_batch* b, const oenv* e, int center_rem, uint8_t* out) {
  const int W = b->cfg.width, H = b->cfg.height, S = b->stride;
  const int cw = W / 2, ch = H / 2;
  memset(out, 0, (size_t)b->obs_bytes);
  uint8_t* wolf = out;
  uint8_t* bush = out + b->plane_bytes;
  uint8_t* ost = out + 2 * b->plane_bytes;
  for (int i = 0; i < e->nw; ++i) {
    int ddx = e->x - e->wolves[i].x, ddy = e->y - e->wolves[i].y;
    if (abs(ddx) <= cw && abs(ddy) <= ch) wolf[(ddx + cw) * S + (ddy + ch)] = 1;
  }
  for (int i = 0; i < W; ++i)
    for (int j = 0; j < H; ++j) {
      int32_t bx = e->x - (i - cw), by = e->y - (j - ch);
      int rem = (i == cw && j == ch) ? center_rem : bush_remaining(b, e, bx, by);
      bush[i * S + j] = rem > 0;
    }
  ost[cw * S + ch] = 1; /* the ostrich itself, delta 0 */
}

/* mask_grid (wab_env.py:344-357) with the fresh role; only when restrict_view */
static void mask_planes(const wabo_batch* b, int role, uint8_t* out) {
  if (!b->cfg.restrict_view) return;
  const uint8_t(*m)[11] = role == 1 ? GATHERER_MASK : LOOKOUT_MASK;
  for (int p = 0; p < 3; ++p)
    for (int i = 0; i < 11; ++i)
      for (int j = 0; j < 11; ++j)
        if (m[i][j]) out[p * b->plane_bytes + i * b->stride + j] = 0;
}

static void scalars(const wabo_batch* b, const oenv* e, uint8_t* food_turns, uint8_t* role,
                    uint8_t* status) {
  food_turns[0] = (uint8_t)(int)ceil(e->food * (double)b->cfg.turns_to_empty_food); /* :452 */
  role[0] = (uint8_t)e->role;
  status[0] = (uint8_t)e->status;
}

/* ------------------------------------------------------------------ reset (wab_env.py:231-248) */
static void reset_one(wabo_batch* b, oenv* e, uint8_t* planes, uint8_t* food_turns, uint8_t* role,
                      uint8_t* status) {
  const wab_config* c = &b->cfg;
  e->episode += 1;
  e->ek = wabo_episode_key(b->seed, (uint64_t)e->env_id, (uint64_t)e->episode);
  e->turn = 0;
  e->x = 0; e->y = 0;
  e->status = 0;
  /* spawn_ostriches :595-611 */
  e->food = c->starting_food_random
                ? (double)wabo_draw_U(e->ek, SITE_START_FOOD, 0, 0, 0, 0) * 0x1p-53
                : c->starting_food;
  e->role = c->starting_role_random
                ? (int)floor((double)wabo_draw_U(e->ek, SITE_START_ROLE, 0, 0, 0, 0) * 0x1p-53 * 2.0)
                : c->starting_role;
  e->nw = 0;
  e->ne = 0;
  /* generate_bushes :613-629: values are a tile function; only the seen set is kept */
  seen_clear(e);
  seen_view(b, e);
  if (c->wolves) { /* initialize_wolves :578-593: the visible tiles' spawn set, turn 0 */
    hit_ctx hc = {e, c->width, c->height, 0};
    spawn_hits(e->ek, 0, c->width * c->height, b->gap, push_view_cell, &hc);
  }
  int center = bush_remaining(b, e, 0, 0);
  render_planes(b, e, center, planes);
  mask_planes(b, e->role, planes);
  scalars(b, e, food_turns, role, status);
}

void wabo_reset(wabo_batch* b, const uint8_t* mask, uint8_t* planes, uint8_t* food_turns,
                uint8_t* role, uint8_t* status) {
  for (int64_t i = 0; i < b->batch; ++i) {
    if (mask && !mask[i]) continue;
    reset_one(b, &b->envs[i], planes + i * b->obs_bytes, food_turns + i, role + i, status + i);
  }
}

/* ------------------------------------------------------------------ step (wab_env.py:250-342) */
static void step_one(wabo_batch* b, oenv* e, int a, uint8_t* planes, uint8_t* food_turns,
                     uint8_t* role, uint8_t* status, float* reward_out, uint8_t* done_out) {
  const wab_config* c = &b->cfg;
  double reward = 0.0;                                    /* :251 */
  e->turn += 1;                                           /* :252 */
  if (a >= 0 && a < b->n_actions) {                       /* :253-258 */
    e->x += b->act_dx[a];
    e->y += b->act_dy[a];
    if (b->act_role[a] >= 0) e->role = b->act_role[a];
  }
  seen_view(b, e); /* :259 generate_bushes (values implicit; the seen set grows) */
  /* :262-264 despawn: one draw per wolf in list order, keyed by its tile and its
   * occurrence index k among co-located wolves; decide all, then compact (stable) */
  {
    int n = 0;
    uint8_t keep[1024];
    uint8_t* kp = e->nw <= 1024 ? keep : (uint8_t*)malloc((size_t)e->nw);
    for (int i = 0; i < e->nw; ++i) {
      uint32_t k = 0;
      for (int j = 0; j < i; ++j)
        if (e->wolves[j].x == e->wolves[i].x && e->wolves[j].y == e->wolves[i].y) ++k;
      kp[i] = wabo_draw_U(e->ek, SITE_DESPAWN, e->turn, e->wolves[i].x, e->wolves[i].y, k) >
              b->keep_gt;
    }
    for (int i = 0; i < e->nw; ++i)
      if (kp[i]) e->wolves[n++] = e->wolves[i];
    if (kp != keep) free(kp);
    e->nw = n;
  }
  /* :267-286 pursuit: each wolf one axis step toward the ostrich, ties along x */
  if (c->wolves_can_move) {
    for (int i = 0; i < e->nw; ++i) {
      int ddx = e->x - e->wolves[i].x, ddy = e->y - e->wolves[i].y;
      if (abs(ddx) >= abs(ddy)) e->wolves[i].x += (ddx > 0) - (ddx < 0);
      else e->wolves[i].y += (ddy > 0) - (ddy < 0);
    }
  }
  /* :289 snapshot S: wolves now, bushes with food > 0 now, status/role now */
  const int status_snap = e->status;
  const int role_snap = e->role;
  const int center_rem = bush_remaining(b, e, e->x, e->y);
  render_planes(b, e, center_rem, planes);
  /* :291-297 kill */
  if (!c->god_mode) {
    for (int i = 0; i < e->nw; ++i)
      if (e->wolves[i].x == e->x && e->wolves[i].y == e->y) { e->status = 2; break; }
  }
  /* :299-313 eat (stale snapshot status; clip only in this branch) */
  if (center_rem > 0 && (role_snap == 1 || c->lookout_only) && status_snap == 0) {
    e->food += b->fill;
    e->food = e->food < 0.0 ? 0.0 : (e->food > 1.0 ? 1.0 : e->food);
    set_remaining(e, e->x, e->y, center_rem - 1);
    reward += c->reward_for_eating;
  }
  e->food -= b->hunger;                                   /* :316 */
  if (e->food <= 0.0) { e->status = 1; e->food = 0.0; }   /* :319-322 */
  /* :325-326 spawn_wolves (:527-576): ring around the new position */
  if (c->wolves) {
    const int m = c->wolf_spawn_margin;
    const int R = (c->width + 2 * m) * (c->height + 2 * m) - c->width * c->height;
    hit_ctx hc = {e, c->width, c->height, m};
    spawn_hits(e->ek, e->turn, R, b->gap, push_ring_tile, &hc);
  }
  /* :328-340 reward / done */
  int done;
  if (e->status == 0) {
    if (e->turn >= c->max_turns) { reward += c->reward_for_finishing; done = 1; }
    else { reward += c->reward_per_turn; done = 0; }
  } else if (e->status == 1) { reward += c->reward_for_starving; done = 1; }
  else { reward += c->reward_for_being_killed; done = 1; }
  /* :342 obs: grids from S (rendered above), scalars fresh */
  mask_planes(b, e->role, planes);
  scalars(b, e, food_turns, role, status);
  *reward_out = (float)reward;
  *done_out = (uint8_t)done;
}

void wabo_step(wabo_batch* b, const int8_t* actions, uint8_t* planes, uint8_t* food_turns,
               uint8_t* role, uint8_t* status, float* reward, uint8_t* done,
               uint8_t* terminal_planes, uint8_t* terminal_food_turns, uint8_t* terminal_role,
               uint8_t* terminal_status, int nthreads) {
  const int64_t B = b->batch;
  const int ob = b->obs_bytes;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1) if (nthreads > 1)
  for (int64_t i = 0; i < B; ++i) {
    oenv* e = &b->envs[i];
    step_one(b, e, actions[i], planes + i * ob, food_turns + i, role + i, status + i, reward + i,
             done + i);
    if (b->cfg.autoreset && done[i]) {
      if (terminal_planes) {
        memcpy(terminal_planes + i * ob, planes + i * ob, (size_t)ob);
        terminal_food_turns[i] = food_turns[i];
        terminal_role[i] = role[i];
        terminal_status[i] = status[i];
      }
      reset_one(b, e, planes + i * ob, food_turns + i, role + i, status + i);
    }
  }
}

void wabo_get_state(const wabo_batch* b, double* food, int32_t* x, int32_t* y, int32_t* turn,
                    int32_t* n_wolves, uint32_t* episode) {
  for (int64_t i = 0; i < b->batch; ++i) {
    const oenv* e = &b->envs[i];
    if (food) food[i] = e->food;
    if (x) x[i] = e->x;
    if (y) y[i] = e->y;
    if (turn) turn[i] = e->turn;
    if (n_wolves) n_wolves[i] = e->nw;
    if (episode) episode[i] = (uint32_t)e->episode;
  }
}

/* Eaten-log lengths and the entries with no berries left (diagnostics: tools/). */
void wabo_get_eaten_counts(const wabo_batch* b, int32_t* n_eaten, int32_t* n_emptied) {
  for (int64_t i = 0; i < b->batch; ++i) {
    const oenv* e = &b->envs[i];
    int z = 0;
    for (int k = 0; k < e->ne; ++k) z += e->eaten[k].rem == 0 ? 1 : 0;
    n_eaten[i] = e->ne;
    n_emptied[i] = z;
  }
}

/* ------------------------------------------------------------------ config-5 featurizer */
/* PragmaticObsWrapper.observation (wab_env.py:726-824) followed by gym 0.17 spaces.flatten
 * (actor_critic.py:188): Discrete(n) -> one-hot(n) float32, Tuple -> concatenation,
 * Box -> ravel.  planes [B][3][W][S] u8; view_mask [B][11][11] u8; out [B][F] f32. */
int wabo_feature_dim(int W, int H, int turns_empty) {
  const int md = W / 2 + H / 2 + 1;
  return 16 * (md + 1) + 88 + 2 + (turns_empty + 1) + 2 + 3 + 121;
}

static void nearest_things(const uint8_t* g, int W, int H, int S, int md, int near[4], int second[4],
                           int counts[4]) {
  int shortest = md, second_d = md;
  int si[2] = {0, 0}, s2[2] = {0, 0};
  int any = 0;
  counts[0] = counts[1] = counts[2] = counts[3] = 0;
  for (int r = 0; r < W; ++r)          /* np.where: row-major over (axis 0, axis 1) :770 */
    for (int c = 0; c < H; ++c) {
      if (g[r * S + c] != 1) continue;
      any = 1;
      const int rr = r - H / 2, rc = c - W / 2;   /* :779-780 (axis 0 measured with H) */
      const int tx = abs(rr) + abs(rc);
      if (tx <= shortest) {                        /* :782-787 */
        second_d = shortest;
        s2[0] = si[0]; s2[1] = si[1];
        shortest = tx;
        si[0] = rr; si[1] = rc;
      } else if (tx <= second_d) {                 /* :788-791 */
        second_d = tx;
        s2[0] = rr; s2[1] = rc;
      }
      if (r < H / 2) counts[0]++;                  /* up    binary_map[0:half_row, :]   :819 */
      if (c > W / 2) counts[1]++;                  /* right binary_map[:, half_col+1:]  :820 */
      if (r > H / 2) counts[2]++;                  /* down  binary_map[half_row+1:, :]  :821 */
      if (c < W / 2) counts[3]++;                  /* left  binary_map[:, 0:half_col]   :822 */
    }
  for (int k = 0; k < 4; ++k) counts[k] = counts[k] < 10 ? counts[k] : 10;  /* :734, :737 */
  if (!any) {
    for (int k = 0; k < 4; ++k) near[k] = second[k] = 0;
    return;
  }
  const int* idx[2] = {si, s2};
  int* outp[2] = {near, second};
  for (int q = 0; q < 2; ++q) {                    /* :792-808 */
    const int a = idx[q][0], b = idx[q][1];
    const int up = a < 0 ? -a : 0, right = b > 0 ? b : 0, down = a > 0 ? a : 0, left = b < 0 ? -b : 0;
    outp[q][0] = up ? md - up : 0;
    outp[q][1] = right ? md - right : 0;
    outp[q][2] = down ? md - down : 0;
    outp[q][3] = left ? md - left : 0;
  }
}

void wabo_featurize(int64_t B, int W, int H, int S, int turns_empty, const uint8_t* planes,
                    const uint8_t* food_turns, const uint8_t* role, const uint8_t* status,
                    const uint8_t* view_mask, float* out) {
  const int md = W / 2 + H / 2 + 1;
  const int F = wabo_feature_dim(W, H, turns_empty);
  for (int64_t i = 0; i < B; ++i) {
    const uint8_t* pl = planes + (size_t)i * 3 * W * S;
    float* o = out + (size_t)i * F;
    memset(o, 0, sizeof(float) * (size_t)F);
    int nw[4], sw[4], cw[4], nb[4], sb[4], cb[4];
    nearest_things(pl, W, H, S, md, nw, sw, cw);
    nearest_things(pl + W * S, W, H, S, md, nb, sb, cb);
    int off = 0;
    const int* groups[6] = {nw, sw, cw, nb, sb, cb};
    const int sizes[6] = {md + 1, md + 1, 11, md + 1, md + 1, 11};
    for (int gq = 0; gq < 6; ++gq)
      for (int k = 0; k < 4; ++k) { o[off + groups[gq][k]] = 1.0f; off += sizes[gq]; }
    const int standing = pl[W * S + (md / 2) * S + md / 2];  /* bushes[md//2, md//2] :742 */
    o[off + standing] = 1.0f; off += 2;
    o[off + food_turns[i]] = 1.0f; off += turns_empty + 1;
    o[off + role[i]] = 1.0f; off += 2;
    o[off + status[i]] = 1.0f; off += 3;
    for (int k = 0; k < 121; ++k) o[off + k] = (float)view_mask[(size_t)i * 121 + k];
  }
}

static const uint8_t GLYPHS_FLAT[10 * WAB_GLYPH_ROWS * WAB_GLYPH_ADVANCE] = {WAB_GLYPH_DATA};

/* draw_health (:496-500): ImageDraw.text((0, 0), str(food), fill="blue") on the scaled image,
 * PIL's default font: each digit's coverage a (wab_glyphs.h, baked from PIL by
 * tools/make_glyphs.py) blends the ink in by Pillow's rule DIV255(x * (255 - a) + ink * a) */
static void draw_count(uint8_t* img, int RW, int RH, int count) {
  char txt[8];
  int nd = 0;
  for (int v = count;; v /= 10) { txt[nd++] = (char)('0' + v % 10); if (v < 10) break; }
  for (int k = 0; k < nd; ++k) {
    const int digit = txt[nd - 1 - k] - '0';
    for (int r = 0; r < WAB_GLYPH_ROWS; ++r)
      for (int c = 0; c < WAB_GLYPH_ADVANCE; ++c) {
        const int y = WAB_GLYPH_ROW0 + r, x = k * WAB_GLYPH_ADVANCE + c;  /* PIL (x, y) = (axis 1, axis 0) */
        if (y >= RW || x >= RH) continue;
        const unsigned a = GLYPHS_FLAT[(digit * WAB_GLYPH_ROWS + r) * WAB_GLYPH_ADVANCE + c];
        uint8_t* px = img + ((size_t)y * RH + (size_t)x) * 3;
        for (int ch = 0; ch < 3; ++ch) {
          const unsigned ink = ch == 2 ? WAB_GLYPH_INK_B : 0u;
          const unsigned t = (unsigned)px[ch] * (255u - a) + ink * a + 128u;
          px[ch] = (uint8_t)(((t >> 8) + t) >> 8);
        }
      }
  }
}

/* render (wab_env.py:468-502): channel c of cell (i, j) is 255 * grid_c; an empty cell is 127
 * when killed, else 255 and then every channel goes through mask_grid with the ostrich's role
 * (:490-493: blind spots 0, only under restrict_view); each cell becomes a scale x scale block
 * (:494); draw_health draws the turns-until-starve count (:496-500).  The grids are the
 * observation's (already masked, which mask_grid leaves unchanged). */
void wabo_render(int64_t B, int W, int H, int S, int restrict_view, int scale, int draw_health,
                 const uint8_t* planes, const uint8_t* food_turns, const uint8_t* role, const uint8_t* status,
                 uint8_t* rgb) {
  const int RW = W * scale, RH = H * scale;
  for (int64_t e = 0; e < B; ++e) {
    const uint8_t* pl = planes + (size_t)e * 3 * W * S;
    const uint8_t(*m)[11] = role[e] == 1 ? GATHERER_MASK : LOOKOUT_MASK;
    uint8_t* img = rgb + (size_t)e * RW * RH * 3;
    for (int i = 0; i < W; ++i)
      for (int j = 0; j < H; ++j) {
        uint8_t c[3];
        for (int k = 0; k < 3; ++k) c[k] = pl[k * W * S + i * S + j] ? 255 : 0;
        if (!c[0] && !c[1] && !c[2]) c[0] = c[1] = c[2] = status[e] == 2 ? 127 : 255;
        if (status[e] != 2 && restrict_view && i < 11 && j < 11 && m[i][j]) c[0] = c[1] = c[2] = 0;
        for (int a = 0; a < scale; ++a)
          for (int b2 = 0; b2 < scale; ++b2) {
            uint8_t* px = img + ((size_t)(i * scale + a) * RH + (size_t)(j * scale + b2)) * 3;
            px[0] = c[0];
            px[1] = c[1];
            px[2] = c[2];
          }
      }
    if (draw_health) draw_count(img, RW, RH, food_turns[e]);
  }
}

/* WolvesAndBushesEnvEgoCentric._get_bush_proximities (wab_env.py:652-667), for the current
 * state of every env: the 5 squares reachable by up/right/down/left/stay
 * (generate_potential_actions :71-84), the taxicab distance d_k from each to the nearest
 * food>0 bush of the whole seen world, clip(md - d_k, 0, md) with md = W//2 + H//2 + 1
 * (:933-935); md for all five when no such bush exists (the Series([0]*5) branch :664). */
void wabo_egocentric(const wabo_batch* b, uint8_t* out) {
  static const int cx[5] = {0, 1, 0, -1, 0}, cy[5] = {1, 0, -1, 0, 0};
  const int md = b->cfg.width / 2 + b->cfg.height / 2 + 1;
  for (int64_t i = 0; i < b->batch; ++i) {
    const oenv* e = &b->envs[i];
    int best[5] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MAX, INT32_MAX};
    int any = 0;
    for (int s = 0; s < e->nseen; ++s) {
      const int32_t tx = e->seen[s].x, ty = e->seen[s].y;
      if (bush_remaining(b, e, tx, ty) <= 0) continue;
      any = 1;
      for (int k = 0; k < 5; ++k) {
        const int d = abs(e->x + cx[k] - tx) + abs(e->y + cy[k] - ty);
        if (d < best[k]) best[k] = d;
      }
    }
    for (int k = 0; k < 5; ++k) {
      const int v = any ? md - best[k] : md;
      out[i * 5 + k] = (uint8_t)(v < 0 ? 0 : v > md ? md : v);
    }
  }
}

int wabo_superbasic_dim(int W, int H, int turns_empty) {
  const int md = W / 2 + H / 2 + 1;
  return 4 * md + (turns_empty + 1) + 2 + 3;
}

/* SuperBasicObservationWrapper.observation (wab_env.py:914-927): the nearest bush of the bush
 * grid (_get_nearest_things :763-810), food, role, status; flattened by gym 0.17 (each
 * Discrete -> one-hot; the nearest-bush space is Discrete(max_distance), :906) */
void wabo_featurize_superbasic(int64_t B, int W, int H, int S, int turns_empty, const uint8_t* planes,
                               const uint8_t* food_turns, const uint8_t* role, const uint8_t* status,
                               float* out) {
  const int md = W / 2 + H / 2 + 1;
  const int F = wabo_superbasic_dim(W, H, turns_empty);
  for (int64_t i = 0; i < B; ++i) {
    const uint8_t* pl = planes + (size_t)i * 3 * W * S;
    float* o = out + (size_t)i * F;
    memset(o, 0, sizeof(float) * (size_t)F);
    int nb[4], sb[4], cb[4];
    nearest_things(pl + W * S, W, H, S, md, nb, sb, cb);
    int off = 0;
    for (int k = 0; k < 4; ++k) { o[off + nb[k]] = 1.0f; off += md; }
    o[off + food_turns[i]] = 1.0f; off += turns_empty + 1;
    o[off + role[i]] = 1.0f; off += 2;
    o[off + status[i]] = 1.0f;
  }
}

/* actor_critic.finish_episode returns (actor_critic.py:139-143): per env, reverse
 * R = r + gamma * R in double (Python floats), restarting after each done; f32 out.  The
 * rewards are the float32 device rewards; a reward whose float32 equals that of one of the
 * exact_values (the doubles a step can return) stands for that double. */
void wabo_discounted_returns(int64_t T, int64_t B, const float* reward, const uint8_t* done,
                             double gamma, const float* bootstrap, float* out, const double* exact_values,
                             int n_exact) {
  for (int64_t b = 0; b < B; ++b) {
    double R = bootstrap ? (double)bootstrap[b] : 0.0;
    for (int64_t t = T - 1; t >= 0; --t) {
      if (done[t * B + b]) R = 0.0;
      const float rf = reward[t * B + b];
      double r = (double)rf;
      for (int k = 0; k < n_exact; ++k)
        if ((float)exact_values[k] == rf) r = exact_values[k];
      R = r + gamma * R;
      out[t * B + b] = (float)R;
    }
  }
}
