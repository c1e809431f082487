/*
 * wab_torus.h — C-ABI of the MI355X-native batched Environment 2.0 torus world.
 *
 * Drop-in boundary for `Environment 2.0/WAB_Environment2.py` (johnmatthewtennant/wab-gym,
 * SURVEY.md §8 f4): a W x H wrap-around world holding a fixed set of entities (ostriches,
 * wolves, bushes) that act one after another in entity-id order (World.py:325-334), each
 * seeing the objects within a Euclidean view radius across the wrap (World.py:243-316).
 * Here with a leading batch dimension: B independent worlds, one HIP launch per turn of
 * every world (or per T turns).  Conventions as in wab.h: plain pointers and sizes, device
 * pointers are HIP device addresses, `stream` a hipStream_t (NULL = legacy default), the
 * caller owns every I/O buffer, the handle owns per-world state, calls are stream-ordered and
 * asynchronous unless stated; 0 = success, negative WAB2_E_* on failure with the message
 * from wab2_last_error() (thread-local).
 *
 * Reference interface replaced (file:line in /root/reference/Environment 2.0):
 *   wab2_config       <- default_game_options (the keys World reads)   WAB_Environment2.py:9-50
 *   wab2_create       <- WAB_Environment2(W, H, options)               WAB_Environment2.py:55-59
 *                        + create_ostriches / create_wolves / create_bushes with random
 *                        positions, in that order                       WAB_Environment2.py:61-110
 *   wab2_create_at    <- the same with spawn_positions                  WAB_Environment2.py:61-110
 *   wab2_reset        <- reset_environment                              WAB_Environment2.py:113-118
 *                        (WAB_Environment2_Single.reset :36-41, World.reset_world :350-358)
 *   wab2_reset_at     <- the same with each entity's reset(new_x, new_y) WAB_Environment2_Single.py:36-41
 *   wab2_step         <- one turn: for every entity i in id order,      Env2Tests.py:40-88
 *                        get_obs(i) then take_action(i, a[i])            WAB_Environment2.py:120-134
 *                        (World.get_observations :360-377, perform_entity_action :325-334,
 *                        default_game_update :93-132)
 *   wab2_rollout      <- T turns of the same
 *   wab2_get_obs      <- get_obs(entity_id)                             WAB_Environment2.py:120-123
 *   wab2_take_action  <- take_action(entity_id, action) -> (reward, done) WAB_Environment2.py:125-134
 *   wab2_obs record   <- get_obs(i): [visible-objects frame, internal obs] World.py:243-323
 *
 * Randomness: every draw is Python's random.randint in the reference; here it is keyed
 * (oracle/keyed_rng.py sites 7-10): u(seed, world id, episode, site, turn, entity id, axis),
 * randint(a, b) = a + floor(U (b - a + 1) / 2^53).  Episode 0 = the create_* positions, the
 * e-th reset draws episode e.  Results depend only on (seed, world id, actions), not on the
 * batch size, shard or device.
 *
 * Semantics kept from the reference as it runs (pandas 2.3.3 in the build container; the
 * golden vectors of tests/golden/torus_*.npz come from the unmodified modules):
 *  - the frame's X/Y (World._entities) are what observation and eat/kill use; an entity's
 *    own x/y (reported in its internal obs) is unbounded; X = x mod W after each of its
 *    actions (World.py:331-332);
 *  - reset_world's `self._entities.iloc[i]["X"] = ...` (World.py:355-356) is a chained
 *    assignment that writes a copy: after a reset the frame keeps each entity's pre-reset
 *    X/Y until the entity next acts;
 *  - reset positions are randint(0, W) and randint(0, H), both ends included
 *    (WAB_Environment2_Single.py:45-46): x = W happens and reads as X = 0 once it acts;
 *  - `self._entities.iloc[j]["Visible"] = False` (World.py:131) is likewise a no-op, so an
 *    emptied bush stays visible and is eaten from for 0 (Bush.take_food);
 *  - a kill hides the ostrich whose frame LABEL is the tie-break index j among the tile's
 *    visible ostriches (`loc[j, "Visible"]`, World.py:115), not necessarily the one killed;
 *  - view wrap: only one side per axis (`if x < r ... elif W < x + r`, World.py:255-291), a
 *    wrapped delta replaces the plain one only if strictly shorter (min(key=abs));
 *  - radius by role at observation time: gatherer (role 1) gatherer_view_radius, lookout
 *    (role 0) lookout_view_radius; wolves wolf_view_radius; bushes 0 (World.py:365-374);
 *  - ostriches never starve (no hunger in Ostrich.py); killed ostriches keep acting.
 *
 * Batched-surface conventions (the reference never resets by itself): with autoreset, a world
 * in which every ostrich is done (status != 0) after a turn, or whose turn count reached
 * max_turns (> 0), is reset (reset_environment) at the end of that turn; world_reset[b] says
 * so.  Entities must be created ostriches first, then wolves, then bushes (as Env2Tests.py
 * does), which the id layout below assumes.
 */
#ifndef WAB_TORUS_H_
#define WAB_TORUS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WAB2_ABI_VERSION 1
#define WAB2_MAX_ENTITIES 32  /* num_ostriches + num_wolves + num_bushes */
#define WAB2_MAX_OSTRICHES 8
#define WAB2_MAX_SIDE 127     /* width, height (deltas are int8) */
#define WAB2_MAX_RADIUS (1 << 20) /* view radii (a radius past the world's diagonal already sees all of it) */

#define WAB2_OK 0
#define WAB2_E_INVALID (-1)
#define WAB2_E_HIP (-2)
#define WAB2_E_NOMEM (-3)

/* The options World reads (WAB_Environment2.py:9-50; the rest are unused by the code), the
 * world size and the entity counts.  Integers where the reference's values are integers. */
typedef struct wab2_config {
  int32_t width;                       /* 32: WAB_Environment2(world_width, ...), 1..127 */
  int32_t height;                      /* 32 */
  int32_t num_ostriches;               /* 1:  create_ostriches(n), 0..8 */
  int32_t num_wolves;                  /* 8:  create_wolves(n) */
  int32_t num_bushes;                  /* 16: create_bushes(n); total entities <= 32 */
  int32_t starting_role;               /* 1 (0 lookout, 1 gatherer; World.py:365-370) */
  double ostrich_starting_food;        /* 40.0 */
  int32_t food_per_bush;               /* 20 (Bush.initial_food), 0..255 */
  int32_t food_given_per_turn;         /* 5  (Bush.food_given_when_eaten), 0..255 */
  double wolf_starting_food;           /* 20 */
  double wolf_food_for_eating_ostrich; /* 10 */
  int32_t lookout_view_radius;         /* 9, integer in [0, WAB2_MAX_RADIUS] */
  int32_t gatherer_view_radius;        /* 5 */
  int32_t wolf_view_radius;            /* 6 */
  /* ---- batched-surface extensions ---- */
  int32_t max_turns;                   /* 80: autoreset cap (0 = none) */
  int32_t autoreset;                   /* 1 */
} wab2_config;

/* One observation record: entity i's get_obs() at its turn (World.py:360-377), fixed size
 * R = wab2_record_size() = round_up(24 + 2N + NB, 16) bytes (N entities, NB bushes):
 *   [0, 8)    f64  food            internal obs [2]   (Ostrich/Wolf/Bush .food)
 *   [8, 12)   i32  x               internal obs [0]   (the entity's own, unwrapped x)
 *   [12, 16)  i32  y               internal obs [1]
 *   [16, 20)  u32  visible         bit j: entity j is a row of the visible-objects frame
 *                                  (World.py:243-316; rows are in entity-id order)
 *   [20]      u8   flag            ostrich role / wolf is_running (internal obs [3]); bush 0
 *   [21]      u8   status          ostrich / wolf status (internal obs [4]); bush 0
 *   [22]      u8   type            0 ostrich, 1 wolf, 2 bush (the frame's Type of row i)
 *   [23]      u8   0
 *   [24, 24+2N)          i8 x 2   (Delta_X, Delta_Y) of entity j for a visible j, else 0
 *   [24+2N, 24+2N+NB)    u8       Additional_Data [food] of bush k (entity N-NB+k) if
 *                                  visible, else 0
 *   the rest                      0
 * Records are [B][N][R] (world-major, entity-id order): records of world b start at b*N*R. */
int wab2_abi_version(void);
const char* wab2_last_error(void);
int wab2_record_size(const wab2_config* cfg);

typedef struct wab2_handle wab2_handle;

/* Validate options, allocate state for `batch` worlds on HIP device `device` and create
 * their entities at keyed random positions (create_*; episode 0).  World b has id
 * world_id_base + b.  Synchronous.  A world can be stepped at once (the reference allows
 * take_action before any reset_environment) or reset first as Env2Tests.py does. */
int wab2_create(const wab2_config* cfg, int64_t batch, uint64_t seed, int64_t world_id_base,
                int device, wab2_handle** out);

/* wab2_create with caller-chosen positions: create_ostriches / create_wolves / create_bushes(n,
 * spawn_positions) (WAB_Environment2.py:61-110).  positions: HOST int32 [B][N][2] (x, y) in
 * entity-id order, or NULL (= wab2_create).  A pair with a negative coordinate takes the keyed
 * random position of that entity (the reference fills a short spawn_positions list with random
 * ones); otherwise it must be a tile of the world, [0, W) x [0, H) (World.create_* puts it in the
 * frame as given, where the random path only ever draws tiles).  Synchronous. */
int wab2_create_at(const wab2_config* cfg, int64_t batch, uint64_t seed, int64_t world_id_base,
                   int device, const int32_t* positions, wab2_handle** out);
int wab2_destroy(wab2_handle* h);
int64_t wab2_batch(const wab2_handle* h);

/* reset_environment() of all worlds, or of those with mask[b] != 0 (device u8 [B] or NULL). */
int wab2_reset(wab2_handle* h, const uint8_t* mask, void* stream);

/* reset_environment with caller-chosen positions: every entity's
 * WAB_Environment2_Single.reset(new_x, new_y) (WAB_Environment2_Single.py:36-41), then
 * World.reset_world.  positions: HOST int32 [B][N][2] or NULL (= wab2_reset); a pair with a
 * negative coordinate draws the random position (randint(0, W), randint(0, H), as the reference
 * does for new_x < 0 or new_y < 0), others lie in [0, W] x [0, H], the range of those random
 * draws (the reference takes any integers; its frame X/Y stay stale until the entity acts, as
 * after any reset).  Entries of unmasked worlds are ignored.  Synchronises `stream` when
 * positions != NULL. */
int wab2_reset_at(wab2_handle* h, const uint8_t* mask, const int32_t* positions, void* stream);

/* One turn of every world.  actions [B][N] int8 (any value: those outside an entity's act
 * branches are no-ops, as in World.py:25-81); obs [B][N][R] records; reward [B][N] f32 (the
 * reference's int / bool reward: ostrich 1 while alive, wolf food > 10, bush 0); done [B][N]
 * u8 (is_entity_done); world_reset [B] u8 or NULL (autoreset happened after this turn). */
int wab2_step(wab2_handle* h, const int8_t* actions, uint8_t* obs, float* reward, uint8_t* done,
              uint8_t* world_reset, void* stream);

/* T turns: actions [T][B][N], obs [T][B][N][R], reward/done [T][B][N], world_reset [T][B]
 * (or NULL): bit for bit T wab2_step calls, in ONE launch (state on chip between turns). */
int wab2_rollout(wab2_handle* h, const int8_t* actions, int32_t T, uint8_t* obs, float* reward,
                 uint8_t* done, uint8_t* world_reset, void* stream);

/* The reference's per-entity calls, batched over the worlds (WAB_Environment2.py:120-134; the
 * loop of Env2Tests.py:40-88): each world's entity `entity` observes, then acts, in id order.
 *   wab2_get_obs      obs [B][R]: entity's record in every world as it is now
 *                     (World.get_observations); any entity that has not acted this turn;
 *   wab2_take_action  actions [B] int8 -> reward [B] f32, done [B] u8 of that entity
 *                     (perform_entity_action + is_entity_done); entities act in id order,
 *                     each once per turn (the reference allows any order; this surface
 *                     requires ascending ids, so a turn is entities 0..N-1).  The call of
 *                     entity N-1 ends the turn: World.increment_turn and, with autoreset, the
 *                     resets (world_reset [B] u8 or NULL, written by every call).
 * wab2_step / wab2_rollout run whole turns and are refused while a turn is half done;
 * wab2_reset(mask = NULL) restarts the turn at entity 0, a masked reset only between turns. */
int wab2_get_obs(wab2_handle* h, int32_t entity, uint8_t* obs, void* stream);
int wab2_take_action(wab2_handle* h, int32_t entity, const int8_t* actions, float* reward, uint8_t* done,
                     uint8_t* world_reset, void* stream);

/* Hidden state to HOST arrays (any may be NULL; synchronises `stream`): the frame's X/Y
 * df_xy [B][N][2] i32, the entities' own x/y obj_xy [B][N][2] i32, food [B][N] f64, the
 * Visible column visible [B][N] u8, ostrich status [B][num_ostriches] u8, turn [B] i32,
 * episode [B] u32. */
int wab2_get_state(wab2_handle* h, int32_t* df_xy, int32_t* obj_xy, double* food, uint8_t* visible,
                   uint8_t* status, int32_t* turn, uint32_t* episode, void* stream);

typedef struct wab2_counters {
  uint64_t turns;   /* world-turns executed (B per turn) */
  uint64_t resets;  /* world resets (explicit and automatic) */
} wab2_counters;
int wab2_get_counters(wab2_handle* h, wab2_counters* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WAB_TORUS_H_ */
