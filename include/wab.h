/*
 * wab.h — C-ABI of the MI355X-native batched Wolves-and-Bushes step.
 *
 * This is the drop-in boundary for the hot path of johnmatthewtennant/wab-gym:
 * `WolvesAndBushesEnv.reset()/step()` (wab_env.py:103-342) with a leading batch
 * dimension.  Plain pointers and sizes only; every device pointer is a HIP device
 * address (e.g. a torch tensor's data_ptr()), every `stream` a hipStream_t (NULL =
 * the legacy default stream).  The caller owns all I/O buffers; the handle owns
 * per-env state in HBM and the constant tables.  Calls are stream-ordered and
 * asynchronous unless stated otherwise.  A handle is not thread-safe.  All calls
 * return 0 on success and a negative WAB_E_* code on failure; the message is
 * available from wab_last_error() (thread-local).
 *
 * Reference interface replaced (file:line in /root/reference):
 *   wab_config            <- default_game_options                   wab_env.py:11-39
 *   wab_create            <- WolvesAndBushesEnv.__init__            wab_env.py:106-186
 *                            (odd width/height check                wab_env.py:147-148)
 *   wab_reset             <- WolvesAndBushesEnv.reset               wab_env.py:231-248
 *   wab_step              <- WolvesAndBushesEnv.step                wab_env.py:250-342
 *   wab_obs               <- _get_obs 7-tuple                        wab_env.py:359-385
 *   wab_rollout           <- the per-step loop of actor_critic.main  actor_critic.py:185-200
 *                            with pre-chosen actions (T steps)
 *   wab_destroy           <- (gym.Env.close; nothing to free in the reference)
 *   wab_featurize         <- PragmaticObsWrapper.observation         wab_env.py:726-824
 *   wab_featurize_superbasic <- SuperBasicObservationWrapper.observation wab_env.py:900-927
 *   wab_step_features        <- PragmaticObsWrapper(env).step, actor_critic.py:180-192
 *   wab_rollout_features     <- T steps of actor_critic.main's loop     actor_critic.py:185-200
 *                               + finish_episode's returns              actor_critic.py:139-143
 *   wab_render            <- WolvesAndBushesEnv.render (rgb_array,   wab_env.py:468-502
 *                            draw_health text included)
 *   wab_render_envs       <- the same for a range of envs (Monitor video frames)
 *   wab_egocentric        <- WolvesAndBushesEnvEgoCentric._get_obs /  wab_env.py:930-979
 *                            _get_bush_proximities                   wab_env.py:652-667
 *                            + gym.spaces.flatten                    actor_critic.py:188
 *   wab_discounted_returns<- finish_episode's return loop             actor_critic.py:139-143
 *   wab_discounted_returns_exact <- the same on the env's own rewards   actor_critic.py:139-145
 */
#ifndef WAB_H_
#define WAB_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WAB_ABI_VERSION 5
#define WAB_MAX_WOLF_SLOTS 32 /* largest per-env live-wolf slot count (wab_config.wolf_slots) */
#define WAB_MAX_VIEW 63       /* largest odd width/height accepted */

/* error codes */
#define WAB_OK 0
#define WAB_E_INVALID (-1)    /* bad argument (ValueError in the reference) */
#define WAB_E_HIP (-2)        /* HIP runtime error */
#define WAB_E_NOMEM (-3)
#define WAB_E_STATE (-4)      /* call not allowed in the handle's current state */

/* Game options, field-for-field `default_game_options` (wab_env.py:11-39).
 * Booleans are int32 0/1.  `None` options of the reference are spelled with the
 * *_random flags.  The last block are batched-surface extensions. */
typedef struct wab_config {
  double reward_per_turn;          /* 0 */
  double reward_for_being_killed;  /* -1 */
  double reward_for_starving;      /* -1 */
  double reward_for_finishing;     /* 1 */
  double reward_for_eating;        /* 0.1 */
  int32_t gatherer_only;           /* 0  (action table wab_env.py:149-159) */
  int32_t lookout_only;            /* 1  (action table wab_env.py:160-170; eat gate :302) */
  int32_t restrict_view;           /* 0  (masks wab_env.py:109-139, applied :344-357) */
  int32_t starting_role;           /* 1 */
  int32_t starting_role_random;    /* 1 <=> starting_role None (wab_env.py:598-599) */
  int32_t starting_food_random;    /* 1 <=> starting_food None (wab_env.py:596-597) */
  double starting_food;            /* 1.0 */
  int32_t max_turns;               /* 80 */
  int32_t height;                  /* 11, odd */
  int32_t width;                   /* 11, odd */
  int32_t max_berries_per_bush;    /* 200, <= 255 */
  double bush_power;               /* 100 (informational: the threshold table carries it) */
  int32_t turns_to_fill_food;      /* 8 */
  int32_t turns_to_empty_food;     /* 40 */
  int32_t wolf_spawn_margin;       /* 1 */
  double chance_wolf_on_square;    /* 0.001 (spawn test is u < chance/2, wab_env.py:573) */
  double wolf_chance_to_despawn;   /* 0.05 (keep test is u > chance, wab_env.py:263) */
  int32_t wolves;                  /* 1 */
  int32_t wolves_can_move;         /* 1 */
  int32_t god_mode;                /* 0 (hidden key, wab_env.py:292) */
  /* ---- batched-surface extensions ---- */
  int32_t autoreset;               /* 1: a done env is reset inside the same step call */
  int32_t plane_stride;            /* bytes per grid row in `planes` (>= height; 0 = height) */
  int32_t eaten_capacity;          /* eaten-tile log slots per env, <= 255
                                    * (0 = max_turns clamped to [1, 255]) */
  int32_t wolf_slots;              /* live-wolf slots per env: 8 (0 = 8), 16 or 32; a spawn
                                    * beyond them is dropped and counted (wolf_overflow) */
  /* T_k (k = 1..max_berries_per_bush): the smallest 53-bit U with
   * round((U * 2^-53) ** bush_power * max_berries_per_bush) >= k (wab_env.py:632-635).
   * Copied at wab_create.  NULL: wab_create computes it with wab_bush_thresholds (libm);
   * the Python host passes the table of the reference's own numpy arithmetic
   * (wab_gym_amd.options.bush_thresholds; the two agree on every option set tested). */
  const uint64_t* bush_thresholds;
} wab_config;

/* One observation batch — the reference's 7-tuple (wab_env.py:374-385) with a
 * leading batch dimension.  All device pointers, caller-owned.
 *   planes     [B][3][width][plane_stride] u8 0/1: wolf, bush, ostrich grids.
 *              Axis 1 is x, cell [width/2 + (ox - x)][height/2 + (oy - y)]
 *              (wab_env.py:403-409); padding bytes are written as 0.
 *   food_turns [B] u8  ceil(food * turns_to_empty_food)   (wab_env.py:450-452)
 *   role       [B] u8                                      (wab_env.py:390-391)
 *   status     [B] u8  0 alive, 1 starved, 2 killed        (wab_env.py:387-388)
 * view_mask (7th element) is a pure function of role and options; the host side
 * derives it (wab_env.py:360-368). */
typedef struct wab_obs {
  uint8_t* planes;
  uint8_t* food_turns;
  uint8_t* role;
  uint8_t* status;
} wab_obs;

/* Device-side counters, read back by wab_get_counters (synchronising). */
typedef struct wab_counters {
  uint64_t wolf_overflow;    /* wolves dropped because all wolf_slots slots were live */
  uint64_t eaten_overflow;   /* eats not logged because the eaten-tile log was full */
  uint64_t bad_actions;      /* actions outside [0, n_actions): treated as no-op */
  uint64_t steps;            /* env-steps executed: B per step-kernel launch (graph replays
                              * of captured wab_step calls included) */
  uint64_t resets;           /* env resets executed */
  uint64_t ego_missing;      /* wab_egocentric calls that found a turn of the path unrecorded */
  uint64_t handoff_timeouts; /* waits on an in-workgroup LDS hand-off that gave up (a hang
                              * guard; nonzero means results are invalid; must stay 0) */
  uint64_t wolf_overflow_reset; /* the part of wolf_overflow dropped by resets (a new episode's
                                 * initial wolves beyond the slots); the rest are ring spawns */
  uint64_t rollout_launches;   /* wab_rollout / wab_rollout_features calls that ran as ONE launch
                                * (host-side tally) */
  uint64_t rollout_step_calls; /* ... that ran as T per-step calls instead (misaligned plane
                                * slices, other kernels; host-side tally) */
} wab_counters;

typedef struct wab_handle wab_handle;

/* ABI version compiled into the library (== WAB_ABI_VERSION). */
int wab_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char* wab_last_error(void);

/* Number of actions of the table selected by the options (5 or 6, wab_env.py:149-182). */
int wab_num_actions(const wab_config* cfg);

/* The bush-value threshold table of wab_config.bush_thresholds, in C: out[k-1] = the
 * smallest U in [1, 2^53] with nearbyint(pow(U * 2^-53, bush_power) * max_berries) >= k
 * (generate_n_bush_values, wab_env.py:631-635; 2^53 = no draw reaches k), by bisection
 * over the 2^53 grid.  Host only, synchronous, no device needed. */
int wab_bush_thresholds(double bush_power, int32_t max_berries, uint64_t* out);

/* Validate options and allocate state for `batch` envs on HIP device `device`.
 * Env i has global id env_id_base + i; every random draw is keyed by
 * (seed, global id, episode, ...), so results do not depend on batch size, shard
 * count or device.  Synchronous.  No env is reset yet: call wab_reset first. */
int wab_create(const wab_config* cfg, int64_t batch, uint64_t seed, int64_t env_id_base,
               int device, wab_handle** out);

/* Free the handle and its device state (synchronises the device). */
int wab_destroy(wab_handle* h);

/* Reset envs (all, or those with mask[i] != 0; mask is a device pointer or NULL) and
 * write their observations into `obs` (other envs' obs entries are left untouched).
 * The first reset of an env is episode 0; each later reset increments its episode. */
int wab_reset(wab_handle* h, const uint8_t* mask, const wab_obs* obs, void* stream);

/* One step of every env.  actions: [B] int8 device.  Writes obs, reward [B] f32
 * (the reference's double reward rounded to f32), done [B] u8.
 * With cfg.autoreset, an env that is done is reset in the same call: `obs` then holds
 * the new episode's first observation and, if `terminal` is non-NULL, the step's own
 * observation is written to `terminal` (only the done envs' entries are written).
 * Without autoreset the env keeps stepping after done exactly as the reference does
 * (stepping after done is not guarded, wab_env.py:250). */
int wab_step(wab_handle* h, const int8_t* actions, const wab_obs* obs, float* reward,
             uint8_t* done, const wab_obs* terminal, void* stream);

/* T steps, stream-ordered, no host synchronisation.  actions [T][B] int8; obs planes
 * [T][B][3][width][plane_stride] and the scalar arrays [T][B] (an obs "sequence");
 * reward/done [T][B].  Bit for bit T calls of wab_step with terminal = NULL.  Where the small
 * or the wide kernel steps the handle (wab_step_kernel "small" / "wide") and B * width *
 * plane_stride * 3 is a multiple of 16, this is ONE launch: each workgroup takes its 64 envs
 * through the T steps with their state on chip (loaded by the first step, stored by the
 * last); otherwise T wab_step launches (a step slice that is not 16-byte aligned goes through
 * a handle-owned [B] buffer, allocated synchronously by the first such call, and a
 * device-to-device copy on `stream`). */
int wab_rollout(wab_handle* h, const int8_t* actions, int32_t T, const wab_obs* obs_seq,
                float* reward, uint8_t* done, void* stream);

/* Read the device counters (synchronises `stream`). */
int wab_get_counters(wab_handle* h, wab_counters* out, void* stream);

/* Copy hidden per-env state to HOST arrays (any may be NULL; synchronises `stream`):
 * food [B] f64, x/y [B] i32, turn [B] i32, n_wolves [B] i32, episode [B] u32. */
int wab_get_state(wab_handle* h, double* food, int32_t* x, int32_t* y, int32_t* turn,
                  int32_t* n_wolves, uint32_t* episode, void* stream);

/* Batch size of a handle. */
int64_t wab_batch(const wab_handle* h);

/* Where the caller's wab_step observations go, a performance hint with no effect on results
 * (default WAB_OBS_SAME_BUFFER):
 *   WAB_OBS_SAME_BUFFER   every step into the same obs buffer (the env's own, as
 *                         BatchedWolvesAndBushesEnv.step does): the per-step kernel, which stores
 *                         each plane as soon as it is final (a 128-byte line at a plane or env
 *                         boundary written in two parts, which the Infinity Cache merges when the
 *                         buffer stays resident);
 *   WAB_OBS_FRESH_BUFFER  each step into a buffer the last steps did not write (a closed loop's
 *                         ring of obs slots): on the wide kernel (wab_step_kernel "wide"), without
 *                         terminal obs, a one-step launch of its rollout build, which stores whole
 *                         lines in address order after the step (C3 at B = 65536: 52 us per step
 *                         into a 32-slot ring, against 73 us for the per-step kernel).
 * Other kernels ignore it.  Host only, no synchronisation. */
#define WAB_OBS_SAME_BUFFER 0
#define WAB_OBS_FRESH_BUFFER 1
int wab_set_obs_placement(wab_handle* h, int32_t placement);

/* Name of the kernel wab_step launches for this handle: "small" (the four-wave kernel for
 * views of at most 128 cells in unpadded rows), "wide" (width <= 31 and height <= 32, in rows
 * of 16 or 32 bytes, without restrict_view: the 31x31 configuration; width 32 steps on "block")
 * or "block" (the general one).  Diagnostics only. */
const char* wab_step_kernel(const wab_handle* h);

/* ---- config 5 (actor_critic.py rollout) ------------------------------------------ */

/* Length of the flattened PragmaticObsWrapper observation for the handle's options
 * (449 for the defaults), or WAB_E_INVALID if the wrapper cannot index the grids. */
int wab_feature_dim(const wab_handle* h);

/* PragmaticObsWrapper.observation (wab_env.py:726-824) + gym 0.17 spaces.flatten
 * (actor_critic.py:188) on device: obs -> features [B][F] float32 one-hot values.
 * view_mask: [B][11][11] u8 device pointer, or NULL to derive it from role and the
 * options as _get_obs does (wab_env.py:360-368). */
int wab_featurize(wab_handle* h, const wab_obs* obs, const uint8_t* view_mask, float* features,
                  void* stream);

/* wab_step fused with wab_featurize: PragmaticObsWrapper(WolvesAndBushesEnv).step
 * (actor_critic.py:180-192 wraps the env, so the policy only ever sees the features;
 * wab_env.py:670-824 applied to the obs of wab_env.py:250-342).  features [B][F] float32
 * (F = wab_feature_dim) are those of the obs this step returns (after auto-reset), bit for
 * bit what wab_step followed by wab_featurize(view_mask = NULL) would produce; reward, done
 * and the obs scalars are written as by wab_step.  No terminal obs.
 * obs->planes may be NULL: the planes are then not returned.  When the small-view kernel
 * steps the handle (wab_step_kernel == "small") and its views fit the table-driven
 * featurizer, one kernel does both (planes rendered on chip, stored only if asked for);
 * otherwise the call is wab_step then wab_featurize on `stream` (without caller planes
 * through a handle-owned buffer the first such call allocates, synchronously).
 * features (and planes, if set) must be 16-byte aligned. */
int wab_step_features(wab_handle* h, const int8_t* actions, const wab_obs* obs, float* reward,
                      uint8_t* done, float* features, void* stream);

/* T steps of PragmaticObsWrapper(WolvesAndBushesEnv).step with pre-chosen actions (the loop of
 * actor_critic.main, actor_critic.py:185-200) and, if `returns` is non-NULL, the discounted
 * returns of the segment (finish_episode, actor_critic.py:139-143): bit for bit T calls of
 * wab_step_features (actions [T][B]; obs_seq scalars [T][B], planes [T][B][3][width][stride]
 * or NULL; reward, done [T][B]; features [T][B][F]) followed by wab_discounted_returns_exact
 * over the [T][B] reward/done (R_T = bootstrap[b], NULL = 0; returns [T][B] f32).  Where the
 * fused small-view kernel steps the handle this is ONE launch: every workgroup takes its 64 envs
 * through the T steps with the state in registers, step t's feature rows stored while step
 * t + 1 runs, and (T <= 128) the returns computed from each step's exact double reward at the
 * end; elsewhere T wab_step_features calls and wab_discounted_returns_exact (misaligned plane
 * slices as in wab_rollout).  Every step's features must be 16-byte aligned: B * F a multiple
 * of 4.  With returns, T > 128 (or a non-fused handle) needs the exact-reward scan: when two of
 * the options' rewards round to the same float32 the call fails before any step runs. */
int wab_rollout_features(wab_handle* h, const int8_t* actions, int32_t T, const wab_obs* obs_seq,
                         float* reward, uint8_t* done, float* features, double gamma,
                         const float* bootstrap, float* returns, void* stream);

/* SuperBasicObservationWrapper.observation (wab_env.py:900-927) + gym flatten: the nearest
 * bush of the bush grid (4 x Discrete(max_distance)), food, role, status -> one-hot float32
 * [B][wab_superbasic_dim(h)] (90 for the defaults).  features must be 16-byte aligned. */
int wab_superbasic_dim(const wab_handle* h);
int wab_featurize_superbasic(wab_handle* h, const wab_obs* obs, float* features, void* stream);

/* WolvesAndBushesEnv.render(mode="rgb_array", scale, draw_health) (wab_env.py:468-502) of an
 * observation this handle produced: rgb [B][W*scale][H*scale][3] u8 device pointer.  With
 * draw_health != 0 (the reference's default) the turns-until-starve count (obs->food_turns)
 * is drawn at (0, 0) in blue with the digit glyphs of PIL's default font (wab_glyphs.h). */
int wab_render(wab_handle* h, const wab_obs* obs, int32_t scale, int32_t draw_health, uint8_t* rgb,
               void* stream);
/* The same for envs [first, first + count) of the observation only: rgb [count][W*scale]
 * [H*scale][3] (one env's frames for the Monitor's video recorder, gym.wrappers.Monitor
 * via wab_env.py:1013, actor_critic.py:46). */
int wab_render_envs(wab_handle* h, const wab_obs* obs, int64_t first, int64_t count, int32_t scale,
                    int32_t draw_health, uint8_t* rgb, void* stream);

/* Bush proximities of the egocentric env variants (WolvesAndBushesEnvEgoCentric and
 * WolvesAndBushesEnvEgocentricJustBushes, wab_env.py:930-979) for the handle's current state:
 * proximity u8 [B][5] (device), for the squares reached by up, right, down, left, stay:
 * clip(md - d, 0, md), d = taxicab distance to the nearest food>0 bush among every tile seen
 * this episode, md = width//2 + height//2 + 1 (<= 31 required); md for all five when no such
 * bush exists (wab_env.py:664).  mask (device u8 [B], nullable) limits the envs written.
 * The handle keeps a path of ostrich tiles for this: call it after EVERY wab_reset and
 * wab_step of the envs it observes (turn t's entry is written at turn t); a missing entry
 * counts in wab_counters.ego_missing.  Not valid after wab_rollout. */
int wab_egocentric(wab_handle* h, const uint8_t* mask, uint8_t* proximity, void* stream);

/* Discounted returns of actor_critic.finish_episode (actor_critic.py:139-143) over a
 * [T][B] rollout: R_t = r_t + gamma * R_{t+1}, restarted after every done_t, R_T =
 * bootstrap[b] (NULL = 0).  Accumulated in double as the reference's Python floats are;
 * written as f32.  All pointers device. */
int wab_discounted_returns(const float* reward, const uint8_t* done, int32_t T, int64_t B,
                           double gamma, const float* bootstrap, float* returns, void* stream);

/* wab_discounted_returns over rewards that this handle's steps returned: each float32 reward
 * is first mapped back to the exact double the reference's step() returns (0 + r_x or
 * 0 + r_eat + r_x, wab_env.py:251-340; e.g. -0.8999999999999999 for 0.1 + -1, whose float32
 * is -0.9f), so the returns equal float32 of finish_episode's own double returns
 * (actor_critic.py:139-145) bit for bit.  Rewards outside that set are used as given.
 * WAB_E_INVALID if two of the options' rewards round to the same float32. */
int wab_discounted_returns_exact(const wab_handle* h, const float* reward, const uint8_t* done, int32_t T,
                                 int64_t B, double gamma, const float* bootstrap, float* returns,
                                 void* stream);

/* Test hook: the bush value (berries, generate_n_bush_values wab_env.py:631-635) the step
 * kernels give the 53-bit draws U[n] under h's threshold table, computed by the kernels' own
 * bracketed search (bush_value_fast).  U, out device pointers. */
int wab_debug_bush_values(wab_handle* h, const uint64_t* U, int32_t* out, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WAB_H_ */
