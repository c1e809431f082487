/*
 * wab_torus_oracle.c — TEST INFRASTRUCTURE: scalar C restatement of the Environment 2.0
 * torus world (johnmatthewtennant/wab-gym `Environment 2.0/`), the checker of the HIP
 * kernel in wab_gym_amd/csrc/wab_torus.hip.  Loaded only by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg.
 *
 * It follows the reference's own sequence, one world at a time, one entity at a time:
 *   turn:    for i in id order: get_obs(i) (World.get_observations, World.py:360-377),
 *            then take_action(i, a) (WAB_Environment2.py:125-134 -> perform_entity_action
 *            World.py:325-334: act, X = x % W, default_game_update :93-132, compute_reward,
 *            is_done)
 *   reset:   reset_environment (WAB_Environment2.py:113-118)
 *   create:  create_ostriches / create_wolves / create_bushes with random positions
 * with Python's random.randint replaced by the keyed draws of oracle/keyed_rng.py (sites
 * 7-10), exactly as tests/golden/torus_harness.py injects them into the real modules.
 * Pinned by the golden vectors tests/golden/torus_*.npz (tests/test_torus_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/wab_torus.h"

uint64_t wabo_episode_key(uint64_t seed, uint64_t env, uint64_t episode);
uint64_t wabo_draw_U(uint64_t ek, uint32_t site, int64_t turn, int64_t x, int64_t y, uint32_t k);

enum { SITE_T_CREATE = 7, SITE_T_RESET = 8, SITE_T_EAT = 9, SITE_T_KILL = 10 };
enum { T_OSTRICH = 0, T_WOLF = 1, T_BUSH = 2 };

typedef struct {
  int64_t x, y;       /* the entity object's own coordinates (Entity.x / .y) */
  int64_t X, Y;       /* the frame's X / Y columns (World._entities) */
  int visible;        /* the frame's Visible column */
  double food;        /* Ostrich.food, Wolf.food, Bush.food */
  int role, status;   /* Ostrich.role / .status, Wolf.status */
} wabt_entity;

typedef struct {
  wab2_config cfg;
  int64_t B, N, NO, NW, NB, R;
  uint64_t seed;
  int64_t base;
  wabt_entity* e;     /* [B][N] */
  int64_t* turn;      /* World._current_turn */
  int64_t* episode;   /* reset_environment() calls */
} wabt;

static int64_t pymod(int64_t a, int64_t m) { return ((a % m) + m) % m; }

/* random.randint(a, b) under the keyed RNG (keyed_rng.randint_keyed) */
static int64_t randint_keyed(uint64_t ek, int site, int64_t turn, int64_t x, int64_t y, int64_t a, int64_t b) {
  const unsigned __int128 U = wabo_draw_U(ek, (uint32_t)site, turn, x, y, 0);
  return a + (int64_t)((U * (unsigned __int128)(b - a + 1)) >> 53);
}

static int type_of(const wabt* w, int64_t i) { return i < w->NO ? T_OSTRICH : i < w->NO + w->NW ? T_WOLF : T_BUSH; }

int wabt_record_size(const wab2_config* c) {
  const int N = c->num_ostriches + c->num_wolves + c->num_bushes;
  return (24 + 2 * N + c->num_bushes + 15) / 16 * 16;
}

/* the entity object's reset(new_x, new_y) (Ostrich.py:66-71, Wolf.py:70-75, Bush.py:52-56) */
static void reset_object(const wabt* w, wabt_entity* en, int type, int64_t x, int64_t y) {
  en->x = x;
  en->y = y;
  en->status = 0;
  if (type == T_OSTRICH) {
    en->food = w->cfg.ostrich_starting_food;
    en->role = w->cfg.starting_role;
  } else if (type == T_WOLF) {
    en->food = w->cfg.wolf_starting_food;
    en->role = 0;
  } else {
    en->food = (double)w->cfg.food_per_bush;
    en->role = 0;
  }
}

/* an explicit position of entity i in world b (pos [B][N][2] or NULL), or 0: the keyed draw
 * (a negative coordinate: WAB_Environment2_Single.reset's `new_x < 0 or new_y < 0`, :38) */
static int explicit_pos(const wabt* w, const int32_t* pos, int64_t b, int64_t i, int64_t* x, int64_t* y) {
  if (!pos) return 0;
  const int32_t* q = pos + (b * w->N + i) * 2;
  if (q[0] < 0 || q[1] < 0) return 0;
  *x = q[0];
  *y = q[1];
  return 1;
}

void* wabt_create_at(const wab2_config* cfg, int64_t B, uint64_t seed, int64_t base, const int32_t* pos);

void* wabt_create(const wab2_config* cfg, int64_t B, uint64_t seed, int64_t base) {
  return wabt_create_at(cfg, B, seed, base, NULL);
}

/* create_*(n, spawn_positions) (WAB_Environment2.py:61-110): the given positions, the random
 * ones where a pair is negative */
void* wabt_create_at(const wab2_config* cfg, int64_t B, uint64_t seed, int64_t base, const int32_t* pos) {
  wabt* w = (wabt*)calloc(1, sizeof(wabt));
  w->cfg = *cfg;
  w->B = B;
  w->NO = cfg->num_ostriches;
  w->NW = cfg->num_wolves;
  w->NB = cfg->num_bushes;
  w->N = w->NO + w->NW + w->NB;
  w->R = wabt_record_size(cfg);
  w->seed = seed;
  w->base = base;
  w->e = (wabt_entity*)calloc((size_t)(B * w->N), sizeof(wabt_entity));
  w->turn = (int64_t*)calloc((size_t)B, sizeof(int64_t));
  w->episode = (int64_t*)calloc((size_t)B, sizeof(int64_t));
  for (int64_t b = 0; b < B; ++b) {
    /* create_*: spawn_positions = [(randint(0, W-1), randint(0, H-1)) ...] (WAB_Environment2.py:64-106)
     * -> World.create_* puts the entity in the frame at that position, Visible (World.py:157-231) */
    const uint64_t ek = wabo_episode_key(seed, (uint64_t)(base + b), 0);
    for (int64_t i = 0; i < w->N; ++i) {
      wabt_entity* en = &w->e[b * w->N + i];
      int64_t x, y;
      if (!explicit_pos(w, pos, b, i, &x, &y)) {
        x = randint_keyed(ek, SITE_T_CREATE, 0, i, 0, 0, cfg->width - 1);
        y = randint_keyed(ek, SITE_T_CREATE, 0, i, 1, 0, cfg->height - 1);
      }
      reset_object(w, en, type_of(w, i), x, y);
      en->X = x;
      en->Y = y;
      en->visible = 1;
    }
  }
  return w;
}

void wabt_destroy(void* h) {
  wabt* w = (wabt*)h;
  free(w->e);
  free(w->turn);
  free(w->episode);
  free(w);
}

/* reset_environment (WAB_Environment2.py:113-118): every entity's reset() with
 * _get_random_spawn_indices (randint(0, W), randint(0, H): both ends included), then
 * reset_world (World.py:350-358): Visible = True; its X/Y assignments write a copy (no-op) */
static void reset_world(wabt* w, int64_t b, const int32_t* pos) {
  const int64_t ep = ++w->episode[b];
  const uint64_t ek = wabo_episode_key(w->seed, (uint64_t)(w->base + b), (uint64_t)ep);
  for (int64_t i = 0; i < w->N; ++i) {
    wabt_entity* en = &w->e[b * w->N + i];
    int64_t x, y;
    if (!explicit_pos(w, pos, b, i, &x, &y)) {  /* reset(new_x, new_y), WAB_Environment2_Single.py:36-41 */
      x = randint_keyed(ek, SITE_T_RESET, 0, i, 0, 0, w->cfg.width);
      y = randint_keyed(ek, SITE_T_RESET, 0, i, 1, 0, w->cfg.height);
    }
    reset_object(w, en, type_of(w, i), x, y);
    en->visible = 1;
  }
  w->turn[b] = 0;
}

void wabt_reset_at(void* h, const uint8_t* mask, const int32_t* pos) {
  wabt* w = (wabt*)h;
  for (int64_t b = 0; b < w->B; ++b)
    if (!mask || mask[b]) reset_world(w, b, pos);
}

void wabt_reset(void* h, const uint8_t* mask) { wabt_reset_at(h, mask, NULL); }

/* min(a, c, key=abs): the first argument on a tie */
static int64_t min_abs(int64_t a, int64_t c) { return llabs(c) < llabs(a) ? c : a; }

/* World._get_visible_objects (World.py:243-316) + _get_additional_obs (:318-323) of entity i,
 * encoded as a wab_torus.h record */
static void get_obs(const wabt* w, int64_t b, int64_t i, uint8_t* rec) {
  const wabt_entity* E = &w->e[b * w->N];
  const wabt_entity* me = &E[i];
  const int type = type_of(w, i);
  const int64_t W = w->cfg.width, H = w->cfg.height;
  int64_t r;  /* World.get_observations (:365-374) */
  if (type == T_OSTRICH) r = me->role == 1 ? w->cfg.gatherer_view_radius : w->cfg.lookout_view_radius;
  else if (type == T_WOLF) r = w->cfg.wolf_view_radius;
  else r = 0;
  const int64_t ex = me->X, ey = me->Y;
  memset(rec, 0, (size_t)w->R);
  uint32_t vis = 0;
  for (int64_t j = 0; j < w->N; ++j) {
    const wabt_entity* o = &E[j];
    int64_t dx = o->X - ex, dy = o->Y - ey;
    /* wrap-around, one side per axis (:255-291): Wrap_around_X is NaN (never chosen) off the
     * mask, min(..., key=abs) keeps Delta_X on ties */
    if (ex < r) {
      if (W - (r - ex) <= o->X) dx = min_abs(dx, -ex - (W - o->X));
    } else if (W < ex + r) {
      if (o->X <= r - W + ex) dx = min_abs(dx, o->X + W - ex);
    }
    if (ey < r) {
      if (H - (r - ey) <= o->Y) dy = min_abs(dy, -ey - (H - o->Y));
    } else if (H < ey + r) {
      if (o->Y <= r - H + ey) dy = min_abs(dy, o->Y + H - ey);
    }
    if (!(pow((double)(dx * dx + dy * dy), 0.5) <= (double)r)) continue;  /* :295-297 */
    if (!o->visible) continue;                                             /* :300 */
    vis |= 1u << j;
    rec[24 + 2 * j] = (uint8_t)(int8_t)dx;
    rec[24 + 2 * j + 1] = (uint8_t)(int8_t)dy;
    if (type_of(w, j) == T_BUSH) rec[24 + 2 * w->N + (j - w->NO - w->NW)] = (uint8_t)o->food;  /* [food] */
  }
  const double food = me->food;
  const int32_t x = (int32_t)me->x, y = (int32_t)me->y;
  memcpy(rec, &food, 8);
  memcpy(rec + 8, &x, 4);
  memcpy(rec + 12, &y, 4);
  memcpy(rec + 16, &vis, 4);
  if (type == T_OSTRICH) {  /* [x, y, food, role, status] (World.py:50-51) */
    rec[20] = (uint8_t)me->role;
    rec[21] = (uint8_t)me->status;
  } else if (type == T_WOLF) {  /* [x, y, food, is_running (False), status] (World.py:80-81) */
    rec[20] = 0;
    rec[21] = (uint8_t)me->status;
  }
  rec[22] = (uint8_t)type;
}

/* Bush.take_food (Bush.py:31-39) */
static double take_food(const wabt* w, wabt_entity* bush) {
  const double fg = (double)w->cfg.food_given_per_turn;
  if (bush->food >= fg) {
    bush->food -= fg;
    return fg;
  }
  const double before = bush->food;
  bush->food = 0;
  return before;
}

/* take_action(i, a): perform_entity_action (World.py:325-334) -> (reward, done) */
static void take_action(wabt* w, int64_t b, int64_t i, int a, float* reward, uint8_t* done) {
  wabt_entity* E = &w->e[b * w->N];
  wabt_entity* me = &E[i];
  const int type = type_of(w, i);
  if (type == T_OSTRICH) {  /* default_ostrich_act (:25-43) */
    if (a == 0) me->y += 1;
    else if (a == 1) me->x += 1;
    else if (a == 2) me->y -= 1;
    else if (a == 3) me->x -= 1;
    else if (a == 4) me->role = 0;
    else if (a == 5) me->role = 1;
  } else if (type == T_WOLF) {  /* default_wolf_act (:61-73) */
    if (a == 0) me->y += 1;
    else if (a == 1) me->x += 1;
    else if (a == 2) me->y -= 1;
    else if (a == 3) me->x -= 1;
  }
  me->X = pymod(me->x, w->cfg.width);
  me->Y = pymod(me->y, w->cfg.height);
  /* default_game_update (:93-132): the visible entities of the wanted type on the actor's
   * tile, in frame (id) order; one of them at random */
  if (type != T_BUSH) {
    const int want = type == T_WOLF ? T_OSTRICH : T_BUSH;
    int64_t cand[WAB2_MAX_ENTITIES];
    int n = 0;
    for (int64_t j = 0; j < w->N; ++j)
      if (E[j].visible && E[j].X == me->X && E[j].Y == me->Y && type_of(w, j) == want) cand[n++] = j;
    if (n > 0) {
      const uint64_t ek = wabo_episode_key(w->seed, (uint64_t)(w->base + b), (uint64_t)w->episode[b]);
      const int64_t j = randint_keyed(ek, type == T_WOLF ? SITE_T_KILL : SITE_T_EAT, w->turn[b], i, 0, 0, n - 1);
      if (type == T_WOLF) {
        me->food += w->cfg.wolf_food_for_eating_ostrich;  /* :113 */
        E[cand[j]].status = 2;                             /* :114 */
        E[j].visible = 0;                                  /* :115 loc[j]: label j */
      } else {
        me->food += take_food(w, &E[cand[j]]);  /* :126-127; the Visible update :131 is a no-op */
      }
    }
  }
  /* compute_reward (:21-22, :54-58, :84-85) and is_entity_done (:339-343) */
  if (type == T_OSTRICH) {
    *reward = me->status == 0 ? 1.0f : 0.0f;
    *done = me->status != 0;
  } else if (type == T_WOLF) {
    *reward = me->food > 10 ? 1.0f : 0.0f;
    *done = me->status == 1;
  } else {
    *reward = 0.0f;
    *done = 1;
  }
}

static void turn_world(wabt* w, int64_t b, const int8_t* act, uint8_t* rec, float* reward, uint8_t* done,
                       uint8_t* world_reset) {
  for (int64_t i = 0; i < w->N; ++i) {
    get_obs(w, b, i, rec + i * w->R);
    take_action(w, b, i, act[i], &reward[i], &done[i]);
  }
  w->turn[b] += 1;  /* WAB_Environment2.take_action :131-133 */
  int reset = 0;
  if (w->cfg.autoreset) {
    int all_done = w->NO > 0;
    for (int64_t k = 0; k < w->NO; ++k) all_done &= w->e[b * w->N + k].status != 0;
    reset = all_done || (w->cfg.max_turns > 0 && w->turn[b] >= w->cfg.max_turns);
  }
  if (reset) reset_world(w, b, NULL);
  if (world_reset) *world_reset = (uint8_t)reset;
}

/* one turn of every world: actions [B][N], records [B][N][R], reward/done [B][N], world_reset [B] */
void wabt_step(void* h, const int8_t* actions, uint8_t* records, float* reward, uint8_t* done,
               uint8_t* world_reset, int nthreads) {
  wabt* w = (wabt*)h;
  const int64_t N = w->N;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (int64_t b = 0; b < w->B; ++b)
    turn_world(w, b, actions + b * N, records + b * N * w->R, reward + b * N, done + b * N,
               world_reset ? world_reset + b : NULL);
}

void wabt_get_state(void* h, int32_t* df_xy, int32_t* obj_xy, double* food, uint8_t* visible, uint8_t* status,
                    int32_t* turn, uint32_t* episode) {
  wabt* w = (wabt*)h;
  for (int64_t b = 0; b < w->B; ++b) {
    for (int64_t i = 0; i < w->N; ++i) {
      const wabt_entity* en = &w->e[b * w->N + i];
      const int64_t q = b * w->N + i;
      if (df_xy) { df_xy[2 * q] = (int32_t)en->X; df_xy[2 * q + 1] = (int32_t)en->Y; }
      if (obj_xy) { obj_xy[2 * q] = (int32_t)en->x; obj_xy[2 * q + 1] = (int32_t)en->y; }
      if (food) food[q] = en->food;
      if (visible) visible[q] = (uint8_t)en->visible;
      if (status && i < w->NO) status[b * w->NO + i] = (uint8_t)en->status;
    }
    if (turn) turn[b] = (int32_t)w->turn[b];
    if (episode) episode[b] = (uint32_t)w->episode[b];
  }
}

/* test hooks: place world 0's entities (frame X/Y and object x/y = pos[i]) and run get_obs(i) */
void wabt_debug_place(void* h, const int32_t* pos) {
  wabt* w = (wabt*)h;
  for (int64_t i = 0; i < w->N; ++i) {
    w->e[i].X = w->e[i].x = pos[2 * i];
    w->e[i].Y = w->e[i].y = pos[2 * i + 1];
  }
}

void wabt_debug_obs(void* h, int64_t i, uint8_t* rec) { get_obs((const wabt*)h, 0, i, rec); }
