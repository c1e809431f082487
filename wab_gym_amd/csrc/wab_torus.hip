// wab_torus.hip — the batched Environment 2.0 torus world (include/wab_torus.h): kernels + C-ABI.
//
// Reference: `Environment 2.0/World.py` (get_observations :360-377, _get_visible_objects
// :243-316, perform_entity_action :325-334, default_game_update :93-132, reset_world
// :350-358), `WAB_Environment2.py` (create_* :61-110, reset_environment :113-118, take_action
// :125-134), the entity classes (`Ostrich.py`, `Wolf.py`, `Bush.py`).  Checked bit for bit
// against oracle/wab_torus_oracle.c and the golden vectors of the unmodified reference
// (tests/test_gpu_torus.py).
//
// One workgroup (256 threads, 4 waves) owns 64 worlds for all T turns of a launch; their
// state lives in LDS tables [entity][world] between turns (loaded by the first turn, stored
// by the last).  A turn of the reference is N sequential take_action calls, but the only
// cross-entity effects inside a turn are (a) positions: entity j's frame X/Y changes at its
// own act only, so observer i sees entity j at its NEW position iff j < i; (b) kills: a
// wolf's update hides an ostrich label for the observers after it; (c) eats: an ostrich's
// update lowers one bush's food for the observers after it.  So a turn is:
//   phase A  the sequential part, one lane per world: W0 moves the ostriches and resolves
//            their eats, W1 moves the wolves and resolves their kills (and the autoreset
//            decision), W2 moves the bushes (X = x mod W), W3 fetches the next turn's actions
//            with scalar loads (no wait on its stores);
//   phase B  every observation record, one lane per (world, observer) item, all four waves,
//            from the LDS tables; records go through a per-wave LDS stage so each store
//            instruction writes 1 KiB contiguous;
//   phase C  the turn's end, one lane per (entity, world): positions, roles, status,
//            Visible, food, autoreset draws.
// The waves exchange data only through LDS, so the phase barriers are LDS-only
// (wab::lds_barrier): __syncthreads() would also wait for every record store in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wab_torus.h"
#include "wab_device.h"

// Diagnostic builds only (tools/ab_torus.sh; results wrong by design): WAB2_ABLATE bit 1 skips
// the view computation of the records, bit 2 their global stores, bit 4 the bush-food bytes,
// bit 8 phase C, bit 16 the bush observers' rounds, bit 32 the movers' rounds, bit 64 phase A.
#ifndef WAB2_ABLATE
#define WAB2_ABLATE 0
#endif
// Diagnostic build only (tools/torus_stamps.py): WAB2_STAMPS=1 records s_memtime at the phase
// boundaries of the middle turn, per wave, into the buffer whose address the host reads from
// the WAB2_STAMPS_PTR environment variable ([n_blocks][4 waves][16] u64; the product library
// reads no environment variable).
#ifndef WAB2_STAMPS
#define WAB2_STAMPS 0
#endif
#if WAB2_STAMPS
#define WAB2_STAMP(k)                                                                                 \
  do {                                                                                                \
    if (t == p0.T / 2) {                                                                              \
      const uint64_t ts_ = __builtin_amdgcn_s_memtime();                                              \
      if (lane == 0) p0.stamps[((int64_t)blockIdx.x * 4 + wave) * 16 + (k)] = ts_;                    \
    }                                                                                                 \
  } while (0)
#else
#define WAB2_STAMP(k) \
  do {                \
  } while (0)
#endif

namespace wab2 {

using wab::draw_U;
using wab::episode_key;
using wab::lds_barrier;
using wab::make_ts;
using wab::xy_pack;

enum : uint32_t { SITE_T_CREATE = 7, SITE_T_RESET = 8, SITE_T_EAT = 9, SITE_T_KILL = 10 };
enum { T_OSTRICH = 0, T_WOLF = 1, T_BUSH = 2 };
constexpr int kWorlds = 64;   // worlds per workgroup
constexpr int kThreads = 256;
constexpr int kOMax = WAB2_MAX_OSTRICHES;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ostrich state byte: status (bits 0-1), role (bit 2), Visible (bit 3)
__device__ __forceinline__ int ost_status(uint32_t b) { return (int)(b & 3u); }
__device__ __forceinline__ int ost_role(uint32_t b) { return (int)((b >> 2) & 1u); }
__device__ __forceinline__ bool ost_visible(uint32_t b) { return (b >> 3) & 1u; }

struct TParams {
  // per-world state, SoA, world innermost ([entity][Bp])
  int32_t* ox;          // [N][Bp] the entity object's own x (unbounded for movers)
  int32_t* oy;          // [N][Bp]
  uint16_t* df;         // [N][Bp] the frame's X | Y << 8
  double* food;         // [NM][Bp] ostrich and wolf food
  uint8_t* bfood;       // [NB][Bp] bush food
  uint8_t* ost;         // [NO][Bp] ostrich state byte
  int32_t* turn;        // [Bp] World._current_turn
  uint32_t* episode;    // [Bp] reset_environment() calls
  unsigned long long* counters;  // [2]: turns, resets
  // I/O of a step / rollout launch
  const int8_t* actions;  // [T][B][N]
  uint8_t* obs;           // [T][B][N][R]
  float* reward;          // [T][B][N]
  uint8_t* done;          // [T][B][N]
  uint8_t* world_reset;   // [T][B] or null
  const uint8_t* mask;    // reset kernel: [B] or null
  const int32_t* pos;     // create / reset kernels: explicit positions [B][N][2] or null
  int64_t B, Bp, world_base;
  uint64_t seed;
  int32_t T, N, NO, NW, NB, NM, R, W, H;
  int32_t rl, rg, rw;     // lookout, gatherer, wolf view radius
  int32_t fpb, fg;        // food_per_bush, food_given_per_turn
  double ofood0, wfood0, wff;
  int32_t role0, max_turns, autoreset;
  int32_t act_scalar;     // actions may be read with scalar loads (4-byte aligned slices)
  // the launch's entity windows (a whole turn: both [0, N)): entities [a0, a1) act, in id
  // order, and the records of observers [o0, o1) are written, each as it observes before its
  // own act (wab2_get_obs: o = [i, i + 1), nothing acts; wab2_take_action: a = [i, i + 1))
  int32_t a0, a1, o0, o1;
  // (set by launch_torus) ceil(2^20 / n) for the window's n mover and n bush observers, so
  // that q / n = (q * magic) >> 20 for q < 2048; ceil(2^16 / (R / 16)); ceil(2^20 / N)
  uint32_t magic_m, magic_b, magic_cr, magic_n;
#if WAB2_STAMPS
  unsigned long long* stamps;
#endif
};

__device__ __forceinline__ int pymod(int a, int m) {
  const int r = a % m;
  return r < 0 ? r + m : r;
}

// random.randint(0, n - 1) under the keyed RNG: floor(U n / 2^53)
__device__ __forceinline__ int keyed_below(uint64_t ek, uint32_t site, int32_t turn, int32_t x, int32_t y, uint32_t n) {
  const uint64_t U = draw_U(xy_pack(x, y), make_ts(site, 0, turn), (uint32_t)ek, (uint32_t)(ek >> 32));
  return (int)((U * (uint64_t)n) >> 53);
}

// the ostrich and wolf act tables (World.py:25-43, 61-73): 0 up (y+1), 1 right, 2 down, 3 left
__device__ __forceinline__ int move_dx(int a) { return (a == 1) - (a == 3); }
__device__ __forceinline__ int move_dy(int a) { return (a == 0) - (a == 2); }

// LDS tables of the workgroup's 64 worlds.  Tables a lane-per-world phase walks by entity are
// entity-major ([e][64]: a wave's 64 lanes read 64 consecutive words); the two that phase B reads
// per observer are world-major, so an item reads two entities' positions with one ds_read_b64
// and a pair of bush foods with one ds_read_u16.
struct Lds {
  double* food;      // [NM][64] ostrich / wolf food before the launch
  int2* oxy;         // [NM][64] movers' own x, y (unbounded) before the launch
  uint8_t* stage;    // [4][32][R] record stage, per wave
  uint8_t* act0;     // [64][na] raw actions (world-major, as in HBM) of even turns
  uint8_t* act1;     // ... of odd turns
  uint32_t* pos;     // [64][Np] lo16: frame X|Y<<8 before the launch's acts; hi16: after the act
  int32_t* turn;     // [64]
  uint32_t* ep;      // [64]
  uint32_t* ep_reset;  // [64] episode of this turn's reset draws, 0: no reset
  uint16_t* omod;    // [NM][64] movers' x mod W | y mod H << 8 (the frame X/Y their next act gives)
  uint16_t* bxy;     // [NB][64] bushes' own x | y << 8 (in [0, W] x [0, H])
  uint16_t* ev;      // [NO][64] eat of ostrich k in this launch: bush index | food after << 8 (0xFF: none)
  uint8_t* bf0;      // [64][NBp] bush food before the launch's eats
  uint8_t* bf1;      // [64][NBp] after them
  uint8_t* gain;     // [NM][64] ostrich: berries eaten; wolf: 1 if it ate an ostrich
  uint8_t* ost;      // [NO][64] ostrich state byte before the launch
  uint8_t* hid;      // [NO][64] the wolf whose kill hid label k in this launch (0xFF: none)
  uint8_t* killed;   // [NO][64] status set to 2 in this launch
  uint8_t* alv;      // [NM + 1][64] the ostriches still Visible for observer i (i = NM: every bush):
                     // bit k, bits >= NO set (W1, phase A)
};

__host__ __device__ inline size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

// position-table row: 4 entities per dword-pair group (ceil(N / 4) groups) + 2 (an even row
// that spreads consecutive worlds over the LDS banks)
__host__ __device__ inline int pos_row(int N) { return 4 * ((N + 3) / 4) + 2; }
__host__ __device__ inline int bush_row(int NB) { return (NB + 3) & ~3; }

struct LdsLayout {
  size_t food, oxy, stage, act0, act1, pos, turn, ep, ep_reset, omod, bxy, ev, bf0, bf1, gain, ost, hid, killed,
      alv, total;
};

__host__ __device__ inline LdsLayout lds_layout(int N, int NO, int NM, int NB, int R) {
  LdsLayout L;
  size_t o = 0;
  L.food = o; o += align16((size_t)NM * kWorlds * 8);
  L.oxy = o; o += align16((size_t)NM * kWorlds * 8);
  L.stage = o; o += (size_t)4 * 32 * R;
  L.act0 = o; o += align16((size_t)kWorlds * N);
  L.act1 = o; o += align16((size_t)kWorlds * N);
  L.pos = o; o += align16((size_t)kWorlds * pos_row(N) * 4);
  L.turn = o; o += kWorlds * 4;
  L.ep = o; o += kWorlds * 4;
  L.ep_reset = o; o += kWorlds * 4;
  L.omod = o; o += align16((size_t)NM * kWorlds * 2);
  L.bxy = o; o += align16((size_t)NB * kWorlds * 2);
  L.ev = o; o += align16((size_t)NO * kWorlds * 2);
  L.bf0 = o; o += align16((size_t)kWorlds * bush_row(NB));
  L.bf1 = o; o += align16((size_t)kWorlds * bush_row(NB));
  L.gain = o; o += align16((size_t)NM * kWorlds);
  L.ost = o; o += align16((size_t)NO * kWorlds);
  L.hid = o; o += align16((size_t)NO * kWorlds);
  L.killed = o; o += align16((size_t)NO * kWorlds);
  L.alv = o; o += align16((size_t)(NM + 1) * kWorlds);
  L.total = o;
  return L;
}

__device__ __forceinline__ Lds lds_tables(uint8_t* base, int N, int NO, int NM, int NB, int R) {
  const LdsLayout L = lds_layout(N, NO, NM, NB, R);
  Lds s;
  s.food = reinterpret_cast<double*>(base + L.food);
  s.oxy = reinterpret_cast<int2*>(base + L.oxy);
  s.stage = base + L.stage;
  s.act0 = base + L.act0;
  s.act1 = base + L.act1;
  s.pos = reinterpret_cast<uint32_t*>(base + L.pos);
  s.turn = reinterpret_cast<int32_t*>(base + L.turn);
  s.ep = reinterpret_cast<uint32_t*>(base + L.ep);
  s.ep_reset = reinterpret_cast<uint32_t*>(base + L.ep_reset);
  s.omod = reinterpret_cast<uint16_t*>(base + L.omod);
  s.bxy = reinterpret_cast<uint16_t*>(base + L.bxy);
  s.ev = reinterpret_cast<uint16_t*>(base + L.ev);
  s.bf0 = base + L.bf0;
  s.bf1 = base + L.bf1;
  s.gain = base + L.gain;
  s.ost = base + L.ost;
  s.hid = base + L.hid;
  s.killed = base + L.killed;
  s.alv = base + L.alv;
  return s;
}

__device__ __forceinline__ uint64_t world_key(const TParams& p, int64_t g, uint32_t ep) {
  return episode_key(p.seed, (uint64_t)(p.world_base + g), ep);
}

// v + d wrapped into [0, m), for v in [0, m) and |d| <= 1 (or v in [0, m] and d = 0)
__device__ __forceinline__ int wrap1(int v, int m) { return v < 0 ? v + m : v >= m ? v - m : v; }

// the frame X|Y<<8 an act gives a mover whose x mod W | y mod H << 8 is `om`
__device__ __forceinline__ uint32_t moved(uint32_t om, int a, int W, int H) {
  return (uint32_t)wrap1((int)(om & 0xFFu) + move_dx(a), W) | ((uint32_t)wrap1((int)(om >> 8) + move_dy(a), H) << 8);
}

// A fresh copy of the kernel parameters, loaded from the kernel-argument segment behind an
// opaque pointer (wab_device.h kernel_params): each phase loads the fields it uses, instead of
// the whole block being held in (and spilled from) scalar registers across the turn loop.
__device__ __forceinline__ TParams kparams(const TParams& p0) {
#if __HIP_DEVICE_COMPILE__
  typedef const TParams __attribute__((address_space(4))) KP;
  KP* pk = (KP*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  return *pk;
#else
  return p0;
#endif
}

#ifndef WAB2_ACT_LATE  // (tuning A/B: 1 = the next turn's actions fetched by W3 at the end of phase B; measured slower)
#define WAB2_ACT_LATE 0
#endif
#ifndef WAB2_ACT_DRAIN  // (tuning A/B: 1 = drain the action loads; measured slower, below)
#define WAB2_ACT_DRAIN 0
#endif
// actions of turn t for the workgroup's worlds into act (raw [64][N] bytes), by one wave:
// dword loads, all issued before the first is used, when the slice is 4-byte aligned and the
// workgroup is full (the wave's stores of the previous turn, which the same vmcnt counts, are
// long retired by then); per-byte loads otherwise.
__device__ __forceinline__ void fetch_actions_wave(const TParams& p, int t, int64_t wg0, int nvalid, uint8_t* act,
                                                   int lane) {
  const int nbytes = kWorlds * p.N;
  const int8_t* src = p.actions + (int64_t)t * p.B * p.N + wg0 * p.N;
  if (p.act_scalar && nvalid == kWorlds) {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d32 = reinterpret_cast<uint32_t*>(act);
    constexpr int kMax = (WAB2_MAX_ENTITIES * kWorlds / 4 + 63) / 64;  // dwords per lane, at most 8
    uint32_t v[kMax];
    const int nd = nbytes / 4;
#pragma unroll
    for (int k = 0; k < kMax; ++k) v[k] = lane + 64 * k < nd ? s32[lane + 64 * k] : 0u;
#pragma unroll
    for (int k = 0; k < kMax; ++k)
      if (lane + 64 * k < nd) d32[lane + 64 * k] = v[k];
    // (the compiler's wait tracking carries these loads as pending into phase B, as it cannot
    // tell that the lanes whose stores were skipped loaded nothing, and puts a vmcnt(0) - a
    // wait for all of the wave's record stores - at the head of every bush round of every
    // wave.  Retiring them here removes those waits, and measured slower: 47.57 -> 47.63 us
    // per turn; the waits bound each wave's stores in flight to about one round)
    if (WAB2_ACT_DRAIN) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  } else {
    for (int q = lane; q < nbytes; q += 64)
      act[q] = q < nvalid * p.N ? (uint8_t)src[q] : (uint8_t)0;
  }
}

// reward / done of an entity after its own update (compute_reward World.py:21-22, 54-58,
// 84-85; is_entity_done :339-343): ostrich 1 while alive (int), wolf food > 10 (bool), bush 0;
// done: ostrich status != 0, wolf status == 1 (never set), bush always
__device__ __forceinline__ void reward_done(int type, int status, double food_after, float& rew, uint8_t& dn) {
  if (type == T_OSTRICH) {
    rew = status == 0 ? 1.0f : 0.0f;
    dn = status != 0;
  } else if (type == T_WOLF) {
    rew = food_after > 10.0 ? 1.0f : 0.0f;
    dn = 0;
  } else {
    rew = 0.0f;
    dn = 1;
  }
}

// One observer's view of one entity j (World._get_visible_objects, World.py:243-316): the
// (Delta_X, Delta_Y) byte pair if j is a row of the frame, else 0.  `xy` is j's frame X|Y<<8 as
// the observer sees it.  The wrap (:255-291) is folded into thresholds on X: the `if` side
// (x < r) replaces dx by dx - W exactly when X >= xl = max(W - r + x, x + W/2 + 1) (the
// mask and min(key=abs) choosing the wrapped, strictly shorter delta), the `elif` side by
// dx + W when X <= xr = min(r - W + x, x - W/2 - 1); the other side's threshold never holds.
struct View {
  int ex, ey, xl, xr, yl, yr, W, H, r2;
  uint32_t alive;
};

// branch-free (bit operations, not && / ?:, so that the compiler keeps one straight line and
// the item's position loads go out back to back): `valid` 1 for an entity that exists
__device__ __forceinline__ uint32_t view_pair(const View& v, uint32_t xy, int j, uint32_t valid, uint32_t& vis) {
  const int X = (int)(xy & 0xFFu), Y = (int)(xy >> 8);
  const int dx = X - v.ex - (v.W & -(int)(X >= v.xl)) + (v.W & -(int)(X <= v.xr));
  const int dy = Y - v.ey - (v.H & -(int)(Y >= v.yl)) + (v.H & -(int)(Y <= v.yr));
  const uint32_t ok = valid & (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy) <= v.r2) & (v.alive >> j);
  vis |= (ok & 1u) << j;
  return (((uint32_t)dx & 0xFFu) | (((uint32_t)dy & 0xFFu) << 8)) & (0u - (ok & 1u));
}

// The same on packed 16-bit halves (X, Y): one v_pk op per step for both axes, the squared
// distance one v_dot2 (the wrap thresholds as above, "never" = +/-0x4000 so that no
// difference leaves int16)
#ifndef WAB2_PACKED
#define WAB2_PACKED 1
#endif
typedef short s16x2 __attribute__((ext_vector_type(2)));

struct View2 {
  s16x2 e, lo, hi, wh;
  int r2;
};

// the byte pair X | Y << 8 as 16-bit halves (X, Y)
__device__ __forceinline__ s16x2 unpack_xy(uint32_t xy) {
  return __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(0u, xy, 0x0c010c00u));
}

// per-half sign mask of a packed difference (-1 where negative), kept as one v_pk_ashrrev_i16
// (the compiler otherwise splits `x >> 15` of a short2 into per-half compares and selects)
__device__ __forceinline__ s16x2 sign_mask2(s16x2 x) {
  uint32_t r, v = __builtin_bit_cast(uint32_t, x);
  // op_sel_hi:[0,1]: the high half also shifts by the constant's low 16 bits (15)
  asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(r) : "v"(v));
  return __builtin_bit_cast(s16x2, r);
}

// raw (before the alive / exists mask) visibility bit and delta byte pair of one entity
__device__ __forceinline__ uint32_t view_pair2(const View2& v, uint32_t xy, uint32_t& ok) {
  const s16x2 P = unpack_xy(xy);
  const s16x2 nl = sign_mask2(P - v.lo);  // -1: P < lo (no wrap down)
  const s16x2 nr = sign_mask2(v.hi - P);  // -1: P > hi (no wrap up)
  const s16x2 d = P - v.e - (v.wh & ~nl) + (v.wh & ~nr);
  // dx^2 + dy^2 as one v_dot2_i32_i16 with an inline-zero accumulator (the builtin becomes a
  // v_mov of the zero and a v_dot2c)
  int dd;
  asm("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(dd) : "v"(__builtin_bit_cast(uint32_t, d)));
  ok = (uint32_t)(dd <= v.r2);
  const uint32_t pair = __builtin_amdgcn_perm(0u, __builtin_bit_cast(uint32_t, d), 0x0c0c0200u);
  return pair & (0u - ok);
}

// A round's staged records out to HBM: chunk c (16 bytes) of stage slot r = c / CR is byte
// 16 (c - r CR) of record qq = q0 + r of the round, world ww = qq / nc, at its place in the
// [B][no][R] records; consecutive lanes on consecutive chunks.  Every LDS read of the lane is
// issued before its first store (a loop waited for each read in turn); KMAX >= chunks / 64 (0:
// the loop, for the generic instances, whose registers are at the ceiling).
#ifndef WAB2_COPY_HOIST  // (tuning A/B: 0 = one chunk at a time, each read waited for before its store)
#define WAB2_COPY_HOIST 1
#endif
#ifndef WAB2_COPY_UNCOND  // (tuning A/B: 0 = each hoisted read under its chunk's bound)
#define WAB2_COPY_UNCOND 1
#endif
#ifndef WAB2_DELTA_B64  // (tuning A/B: 0 = a mover's delta dwords one by one, vis by an LDS permute)
#define WAB2_DELTA_B64 1
#endif
#ifndef WAB2_BUSH_WIDE  // (tuning A/B: 0 = a bush record's food dwords one by one)
#define WAB2_BUSH_WIDE 1
#endif
#ifndef WAB2_STORE_THROTTLE  // (vmcnt(N) at each mover round's start; -1: none)
#define WAB2_STORE_THROTTLE 0
#endif
#ifndef WAB2_BUSH_THROTTLE  // (tuning A/B: 1 = vmcnt(0) also before a bush round's second half)
#define WAB2_BUSH_THROTTLE 0
#endif
#ifndef WAB2_POST_THROTTLE  // (tuning A/B: 1 = vmcnt(0) right after every copy-out)
#define WAB2_POST_THROTTLE 0
#endif
#ifndef WAB2_MOVER_CHUNKS  // (tuning A/B: 0 = a mover record's fields written one by one)
#define WAB2_MOVER_CHUNKS 1
#endif
#ifndef WAB2_MOVER_ROW128  // (tuning A/B: 0 = a mover round's bush-food pairs read one by one)
#define WAB2_MOVER_ROW128 1
#endif
// Record stores plain, not non-temporal: 46.77-46.89 -> 44.76-44.86 us per turn on one box
// (the per-step gym kernel measured the opposite for its obs stores)
#ifndef WAB2_REC_NT  // (tuning A/B: 1 = non-temporal record stores)
#define WAB2_REC_NT 0
#endif
__device__ __forceinline__ void rec_store(u32x4 v, u32x4* dst) {
  if (WAB2_REC_NT)
    __builtin_nontemporal_store(v, dst);
  else
    *dst = v;
}
template <int KMAX>
__device__ __forceinline__ void copy_out(const uint8_t* stage, uint8_t* rbase, int chunks, int lane, int q0, int w0r,
                                         int no, int nc, int R, int CR, uint32_t magic_cr, uint32_t magic) {
  if (!WAB2_COPY_HOIST || KMAX == 0) {  // (KMAX 0: the generic instances, at their VGPR ceiling)
    for (int c = lane; c < chunks; c += 64) {
      const int r = (int)(((uint32_t)c * magic_cr) >> 16);
      const int qq = q0 + r;
      const int ww = (int)(((uint32_t)qq * magic) >> 20);
      const uint32_t off = (uint32_t)(((ww - w0r) * no + (qq - ww * nc)) * R + 16 * (c - r * CR));
      rec_store(*reinterpret_cast<const u32x4*>(stage + 16 * c), reinterpret_cast<u32x4*>(rbase + off));
    }
    return;
  }
  constexpr int K = KMAX > 0 ? KMAX : 1;
  u32x4 val[K];
  uint32_t off[K];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    // (unconditional, inside the wave's stage: a read under `c < chunks` became a branch with
    // its own wait, the three reads one after another)
    const int c = WAB2_COPY_UNCOND ? min(lane + 64 * k, 32 * CR - 1) : lane + 64 * k;
    if (WAB2_COPY_UNCOND || c < chunks) {
      const int r = (int)(((uint32_t)c * magic_cr) >> 16);  // stage slot: c / CR
      const int qq = q0 + r;
      const int ww = (int)(((uint32_t)qq * magic) >> 20);
      off[k] = (uint32_t)(((ww - w0r) * no + (qq - ww * nc)) * R + 16 * (c - r * CR));
      val[k] = *reinterpret_cast<const u32x4*>(stage + 16 * c);
    }
  }
  // (all reads issued, then one wait: the compiler otherwise sank the last read into its store's
  // branch)
  if (WAB2_COPY_UNCOND)
#pragma unroll
    for (int k = 0; k < KMAX; ++k) asm volatile("" : "+v"(val[k]));
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (lane + 64 * k < chunks) rec_store(val[k], reinterpret_cast<u32x4*>(rbase + off[k]));
}

// NW dwords xs[] into the record stage at dword D0 of a record of RDW dwords, in the widest
// aligned writes (8 / 16 bytes; zeros past NW where the record's pad allows): a bush round's
// records are written by 32 lanes at stride R, so every write instruction is bank-conflicted
// alike and fewer, wider ones take fewer LDS cycles
template <int D0, int NW, int RDW>
__device__ __forceinline__ void put_dwords(uint8_t* rec, const uint32_t* xs) {
  if constexpr (NW > 0) {
    if constexpr (D0 % 4 == 0 && (NW >= 4 || D0 + 4 <= RDW)) {
      *reinterpret_cast<u32x4*>(rec + 4 * D0) = (u32x4){xs[0], NW > 1 ? xs[NW > 1 ? 1 : 0] : 0u, NW > 2 ? xs[NW > 2 ? 2 : 0] : 0u,
                                                        NW > 3 ? xs[NW > 3 ? 3 : 0] : 0u};
      put_dwords<D0 + 4, (NW > 4 ? NW - 4 : 0), RDW>(rec, xs + (NW > 4 ? 4 : 0));
    } else if constexpr (D0 % 2 == 0 && (NW >= 2 || D0 + 2 <= RDW)) {
      *reinterpret_cast<uint2*>(rec + 4 * D0) = make_uint2(xs[0], NW > 1 ? xs[NW > 1 ? 1 : 0] : 0u);
      put_dwords<D0 + 2, (NW > 2 ? NW - 2 : 0), RDW>(rec, xs + (NW > 2 ? 2 : 0));
    } else {
      *reinterpret_cast<uint32_t*>(rec + 4 * D0) = xs[0];
      put_dwords<D0 + 1, NW - 1, RDW>(rec, xs + (NW > 1 ? 1 : 0));
    }
  }
}

// NKK = ceil(N / 4): dword-pair groups of the delta array.  CNO, CNW, CNB > 0: an instance for
// whole turns (windows [0, N)) of those entity counts, whose table layout, record size, loop
// bounds and divisions are compile-time constants (the benched 1 / 8 / 16 world); 0: the counts
// and windows from the parameters.
template <int NKK, int CNO = 0, int CNW = 0, int CNB = 0>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) wab_torus_kernel(TParams p0) {
  constexpr bool kFixed = CNO + CNW + CNB > 0;
  constexpr int kN = CNO + CNW + CNB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int64_t wg0 = (int64_t)blockIdx.x * kWorlds;
  const int nvalid = (int)min((int64_t)kWorlds, p0.B - wg0);
  const int T = p0.T;
// every phase works from its own copy of the parameters and LDS table pointers (kparams)
#define WAB2_PHASE_PARAMS                                                                   \
  const TParams p = kparams(p0);                                                          \
  const int N = kFixed ? kN : p.N, NO = kFixed ? CNO : p.NO, NM = kFixed ? CNO + CNW : p.NM; \
  const int NB = kFixed ? CNB : p.NB, R = kFixed ? (24 + 2 * kN + CNB + 15) / 16 * 16 : p.R;  \
  const int W = p.W, H = p.H;                                                             \
  const Lds s = lds_tables(smem, N, NO, NM, NB, R);                                       \
  const int nent = N * kWorlds, a0 = kFixed ? 0 : p.a0, a1 = kFixed ? N : p.a1, na = a1 - a0; \
  const int wo0 = kFixed ? 0 : p.o0, wo1 = kFixed ? N : p.o1;                             \
  const uint32_t magic_m = kFixed ? ((1u << 20) + CNO + CNW - 1) / (CNO + CNW) : p.magic_m; \
  const uint32_t magic_b = kFixed ? ((1u << 20) + CNB - 1) / CNB : p.magic_b;              \
  const uint32_t magic_n = kFixed ? ((1u << 20) + kN - 1) / kN : p.magic_n;               \
  const uint32_t magic_cr = kFixed ? (65536u + R / 16 - 1) / (R / 16) : p.magic_cr;       \
  (void)wo0; (void)wo1; (void)magic_m; (void)magic_b; (void)magic_n; (void)magic_cr;      \
  const int Np = pos_row(N), NBp = bush_row(NB);                                          \
  (void)NO; (void)NM; (void)NB; (void)R; (void)W; (void)H; (void)nent; (void)na; (void)Np; (void)NBp

  // ---- prologue: state -> LDS tables, one lane per (entity, world); turn 0's actions
  {
    WAB2_PHASE_PARAMS;
    for (int q = tid; q < nent; q += kThreads) {
      const int e = q >> 6, w = q & 63;
      const int64_t a = (int64_t)e * p.Bp + wg0 + w;
      s.pos[w * Np + e] = p.df[a];
      const int ox = p.ox[a], oy = p.oy[a];
      if (e < NM) {
        s.oxy[e * kWorlds + w] = make_int2(ox, oy);
        s.omod[e * kWorlds + w] = (uint16_t)(pymod(ox, W) | (pymod(oy, H) << 8));
        s.food[e * kWorlds + w] = p.food[(int64_t)e * p.Bp + wg0 + w];
      } else {
        const int b = e - NM;
        s.bxy[b * kWorlds + w] = (uint16_t)((ox & 0xFF) | ((oy & 0xFF) << 8));
        s.bf0[w * NBp + b] = p.bfood[(int64_t)b * p.Bp + wg0 + w];
      }
      if (e < NO) s.ost[e * kWorlds + w] = p.ost[(int64_t)e * p.Bp + wg0 + w];
      if (e == 0) {
        s.turn[w] = p.turn[wg0 + w];
        s.ep[w] = p.episode[wg0 + w];
      }
    }
    // the acting entities' actions, [world][a1 - a0] as in HBM
    const int8_t* src = p.actions + wg0 * na;
    for (int q = tid; q < kWorlds * na; q += kThreads) s.act0[q] = q < nvalid * na ? (uint8_t)src[q] : (uint8_t)0;
  }
  lds_barrier();

  // (tuning A/B, tools/build_variants.sh -DWAB2_STAGGER=k: the odd dispatch rounds' workgroups
  // start k x ~3.5 us late, so that a CU's groups are not all in phase A / C at once)
#ifndef WAB2_STAGGER
#define WAB2_STAGGER 0
#endif
  if (WAB2_STAGGER && ((blockIdx.x >> 8) & 1u))
    for (int k = 0; k < WAB2_STAGGER; ++k) __builtin_amdgcn_s_sleep(127);
  int64_t resets = 0;
  for (int t = 0; t < T; ++t) {
    WAB2_STAMP(0);
    // ================= phase A: the sequential part of the turn, one lane per world
    if (WAB2_ABLATE & 64) {
    } else if (wave == 0) {
      WAB2_PHASE_PARAMS;
      const uint8_t* A = (t & 1) ? s.act1 : s.act0;
      // ostriches in id order: act (World.py:25-43), X = x mod W (:331-332), eat (:118-132)
      const int w = lane;
      uint32_t* posw = s.pos + w * Np;
      for (int k = 0; k < NBp; k += 4)
        *reinterpret_cast<uint32_t*>(s.bf1 + w * NBp + k) = *reinterpret_cast<const uint32_t*>(s.bf0 + w * NBp + k);
      const uint64_t ek = world_key(p, wg0 + w, s.ep[w]);
      const int32_t turn = s.turn[w];
      for (int k = a0; k < min(a1, NO); ++k) {
        const uint32_t np = moved(s.omod[k * kWorlds + w], (int)(int8_t)A[w * na + k - a0], W, H);
        reinterpret_cast<uint16_t*>(posw + k)[1] = (uint16_t)np;
        // the visible bushes on the tile, in frame (id) order: every bush is visible (the
        // Visible update of World.py:131 writes a copy), at its frame position (bushes act last)
        int n = 0;
        for (int b = 0; b < NB; ++b) n += (posw[NM + b] & 0xFFFFu) == np;
        uint32_t ev = 0xFFu, gain = 0;
        if (n > 0) {
          int j = keyed_below(ek, SITE_T_EAT, turn, k, 0, (uint32_t)n);
          int pick = 0;
          for (int b = 0; b < NB; ++b)
            if ((posw[NM + b] & 0xFFFFu) == np) {
              if (j == 0) pick = b;
              --j;
            }
          // Bush.take_food (Bush.py:31-39)
          int f = s.bf1[w * NBp + pick];
          const int amt = f >= p.fg ? p.fg : f;
          f = f >= p.fg ? f - p.fg : 0;
          s.bf1[w * NBp + pick] = (uint8_t)f;
          ev = (uint32_t)pick | ((uint32_t)f << 8);
          gain = (uint32_t)amt;
        }
        s.ev[k * kWorlds + w] = (uint16_t)ev;
        s.gain[k * kWorlds + w] = (uint8_t)gain;
      }
    } else if (wave == 1) {
      WAB2_PHASE_PARAMS;
      const uint8_t* A = (t & 1) ? s.act1 : s.act0;
      // wolves in id order: act (World.py:61-73), X = x mod W, kill (:107-116)
      const int w = lane;
      uint32_t* posw = s.pos + w * Np;
      const uint64_t ek = world_key(p, wg0 + w, s.ep[w]);
      const int32_t turn = s.turn[w];
      uint32_t opos[kOMax];  // the ostriches' frame X|Y (after their acts: they act first)
      uint32_t vis = 0, dead = 0, kills = 0, hid_by[kOMax];
#pragma unroll
      for (int k = 0; k < kOMax; ++k) {
        opos[k] = 0xFFFFFFFFu;
        hid_by[k] = 0xFFu;
        if (k < NO) {
          opos[k] = (k >= a0 && k < a1) ? moved(s.omod[k * kWorlds + w], (int)(int8_t)A[w * na + k - a0], W, H)
                                        : posw[k] & 0xFFFFu;
          const uint32_t ob = s.ost[k * kWorlds + w];
          vis |= (uint32_t)ost_visible(ob) << k;
          dead |= (uint32_t)(ost_status(ob) != 0) << k;
        }
      }
      const uint32_t vis0 = vis;  // (before this launch's kills)
      // eight wolves at a time: their moves' LDS reads issued together, then the kills in id order
      const int m0 = max(a0, NO), m1 = min(a1, NM);
      for (int mb = m0; mb < m1; mb += 8) {
        uint32_t np8[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int m = min(mb + jj, m1 - 1);
          np8[jj] = moved(s.omod[m * kWorlds + w], (int)(int8_t)A[w * na + m - a0], W, H);
        }
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int m = mb + jj;
          if (m >= m1) break;
          const uint32_t np = np8[jj];
          reinterpret_cast<uint16_t*>(posw + m)[1] = (uint16_t)np;
          uint32_t cand = 0;
#pragma unroll
          for (int k = 0; k < kOMax; ++k) cand |= (uint32_t)((vis >> k & 1u) && opos[k] == np) << k;
          uint32_t gain = 0;
          if (cand) {
            const int n = __builtin_popcount(cand);
            const int j = keyed_below(ek, SITE_T_KILL, turn, m, 0, (uint32_t)n);
            uint32_t c = cand;
            for (int r = 0; r < j; ++r) c &= c - 1;
            kills |= c & (0u - c);  // the j-th visible ostrich of the tile: status 2 (:114)
            gain = 1;
            // `loc[j, "Visible"] = False` (:115): the frame LABEL j, an ostrich id since the
            // ostriches were created first
#pragma unroll
            for (int k = 0; k < kOMax; ++k)
              if (k == j && (vis >> k & 1u)) {
                vis &= ~(1u << k);
                hid_by[k] = (uint32_t)m;
              }
          }
          s.gain[m * kWorlds + w] = (uint8_t)gain;
        }
      }
#pragma unroll
      for (int k = 0; k < kOMax; ++k)
        if (k < NO) {
          s.hid[k * kWorlds + w] = (uint8_t)hid_by[k];
          s.killed[k * kWorlds + w] = (uint8_t)(kills >> k & 1u);
        }
      // the Visible ostriches each observer sees: visible before the launch, not hidden by a
      // wolf of this launch that acted before it (hid_by < i); bits >= NO set (not ostriches)
      {
        uint32_t seen = vis0 | (0xFFu << NO);
        for (int i = 0; i <= NM; ++i) {
          s.alv[i * kWorlds + w] = (uint8_t)seen;
#pragma unroll
          for (int k = 0; k < kOMax; ++k)
            if (k < NO && hid_by[k] == (uint32_t)i) seen &= ~(1u << k);
        }
      }
      dead |= kills;
      // the turn ends with this launch when its last entity acts; then the batched surface's
      // autoreset: every ostrich done, or max_turns reached
      const bool all_dead = NO > 0 && dead == (1u << NO) - 1u;
      const bool rs = a1 == N && na > 0 && p.autoreset && (all_dead || (p.max_turns > 0 && turn + 1 >= p.max_turns));
      s.ep_reset[w] = rs ? s.ep[w] + 1u : 0u;
      const bool valid = w < nvalid;
      if (p.world_reset && valid) p.world_reset[(int64_t)t * p.B + wg0 + w] = (uint8_t)rs;
      resets += (rs && valid) ? 1 : 0;
    } else if (wave == 2) {
      WAB2_PHASE_PARAMS;
      // bushes act on nothing (World.py:9-10); their frame X/Y become x mod W, y mod H (own
      // x in [0, W], y in [0, H])
      const int w = lane;
      for (int b = max(a0, NM) - NM; b < a1 - NM; ++b) {
        const uint32_t bxy = s.bxy[b * kWorlds + w];
        const uint32_t np = (uint32_t)wrap1((int)(bxy & 0xFFu), W) | ((uint32_t)wrap1((int)(bxy >> 8), H) << 8);
        reinterpret_cast<uint16_t*>(s.pos + w * Np + NM + b)[1] = (uint16_t)np;
      }
    } else if (t + 1 < T && !(WAB2_ACT_LATE && kFixed)) {
      WAB2_PHASE_PARAMS;
      fetch_actions_wave(p, t + 1, wg0, nvalid, (t & 1) ? s.act0 : s.act1, lane);
    }
    WAB2_STAMP(1);
    lds_barrier();
    WAB2_STAMP(2);

    // ================= phase B: observation records (and, for a whole turn, reward and done).
    // Two classes of observers, each in rounds of 32 (world, observer) items per wave: the
    // movers (ostriches, wolves), whose view has a radius, and the bushes, whose radius is 0
    // (World.py:365-374): a bush sees the rows on its own tile, at delta (0, 0), so its items take
    // an equality test per entity and no view arithmetic, and never share a round (and its
    // divergent paths) with a mover.  Lanes l and l + 32 share item l: each computes half of the
    // observer's view (delta dwords k = 2kk + half, i.e. entities 4kk + 2 half + {0, 1}), so a
    // round's 32 records fit the wave's LDS stage and every lane is busy.
    {
      WAB2_PHASE_PARAMS;
      const int o0 = wo0, no = wo1 - wo0;
      uint8_t* stage = s.stage + wave * 32 * R;
      const int64_t item0 = wg0 * no;  // first record of the workgroup in [B][no]
      uint8_t* obs_t = p.obs + (int64_t)t * p.B * no * R;
      const bool whole_turn = a0 == 0 && a1 == N && o0 == 0 && no == N;
      const int hf = lane >> 5;
      const int nd = (N + 1) >> 1;        // delta dwords
      const int bb = 24 + 2 * N;          // first bush-food byte
      const int nbp = (NB + 1) >> 1;      // bush-food byte pairs
      const int CR = R >> 4;              // 16-byte chunks per record
      // chunks per lane of a 32-record copy-out: 32 CR / 64 (R <= 128 bytes: at most 4)
      constexpr int kCopyMax = kFixed ? (32 * ((24 + 2 * kN + CNB + 15) / 16) + 63) / 64 : 0;
      const uint32_t exist = N >= 32 ? 0xFFFFFFFFu : (1u << N) - 1u;
      // the stage starts zero: the bush rounds (first) then write only their headers and bush
      // bytes (their deltas are zero); the mover rounds write every byte
      for (int c = lane; c < 2 * R; c += 64) reinterpret_cast<u32x4*>(stage)[c] = (u32x4){0u, 0u, 0u, 0u};
      // Waves 0-1 take the bush rounds first and waves 2-3 the mover rounds first, so that bush
      // stores (little arithmetic per byte) run beside mover arithmetic on the same CU (50.98 →
      // 50.61 µs per turn; by workgroup instead of by wave 50.88).  A bush round writes only its
      // headers and bush bytes into a stage that is zero elsewhere: after mover rounds the
      // wave's stage is zeroed again.
#ifndef WAB2_ORDER  // (tuning A/B: 0 = waves 2-3 movers first; 1 = every wave movers first; 2 = bushes first)
#define WAB2_ORDER 0
#endif
      const bool movers_first = WAB2_ORDER == 0 ? wave >= 2 : WAB2_ORDER == 3 ? wave >= 1 : WAB2_ORDER == 4 ? wave >= 3 : WAB2_ORDER == 1;
      if (!movers_first) {
        // ---- the bush observers: one lane per (world, bush) item, 64 items per round, their
        // records staged and stored in two halves of 32
        {
          const int c0 = max(o0, NM), nc = max(0, wo1 - c0);
          const int nitems = (WAB2_ABLATE & 16) ? 0 : nvalid * nc;
          const int sh = bb & 3, d0 = bb >> 2, ndw = (sh + NB + 3) >> 2;
          for (int rnd = wave; rnd * 64 < nitems; rnd += 4) {
#if WAB2_STORE_THROTTLE >= 0
            // (as at a mover round's start; the compiler's own wait tracking had put this one
            // here already, from the action loads it carries as pending)
            __builtin_amdgcn_s_waitcnt((WAB2_STORE_THROTTLE & 15) | ((WAB2_STORE_THROTTLE >> 4) << 14) | 0x0F70);
#endif
            const int q = rnd * 64 + lane;
            const bool on = q < nitems;
            const int qc = on ? q : nitems - 1;
            const int w = (int)(((uint32_t)qc * magic_b) >> 20);
            const int i = c0 + qc - w * nc;
            // (the fixed instance: a bush observer; every mover has acted before it)
            if (kFixed) __builtin_assume(i >= NM && i < N);
            const uint32_t* posw = s.pos + w * Np;
            const uint32_t tgt = posw[i] & 0xFFFFu;  // (its frame X/Y before its act)
            // every wolf acts before a bush: the Visible ostriches of Lds::alv[NM]
            const uint32_t vmask = (0xFFFFFF00u | s.alv[NM * kWorlds + w]) & exist;
            const int jn = min(i, a1);
            uint2 pp[2 * NKK];
#pragma unroll
            for (int kk = 0; kk < 2 * NKK; ++kk) pp[kk] = *reinterpret_cast<const uint2*>(posw + 2 * kk);
            uint32_t vis = 0;
#pragma unroll
            for (int kk = 0; kk < 2 * NKK; ++kk) {
              const int j = 2 * kk;
              const uint32_t s0 = (uint32_t)((j >= a0) & (j < jn)) << 4, s1 = (uint32_t)((j + 1 >= a0) & (j + 1 < jn)) << 4;
              const uint32_t e0 = (uint32_t)(((pp[kk].x >> s0) & 0xFFFFu) == tgt);
              const uint32_t e1 = (uint32_t)(((pp[kk].y >> s1) & 0xFFFFu) == tgt);
              vis |= (e0 | (e1 << 1)) << j;
            }
            vis &= vmask;
            const uint8_t* row = s.bf1 + w * NBp;  // (bushes observe after every ostrich's eat)
            const uint32_t bxy = s.bxy[(i - NM) * kWorlds + w];
            const uint64_t fb = (uint64_t)__double_as_longlong((double)row[i - NM]);
            const uint64_t v64 = (uint64_t)vis << 8;  // (bit NM + b + 8: bush b, b >= -8)
            // the fixed instance: the row's dwords read once, before the halves' stage writes
            // (which the compiler would otherwise order each row read behind)
            constexpr int kRowW = kFixed ? (((24 + 2 * kN) & 3) + CNB + 3) / 4 : 1;
            uint32_t rdw[kRowW];
#pragma unroll
            for (int k = 0; k < kRowW; ++k) rdw[k] = kFixed ? *reinterpret_cast<const uint32_t*>(row + 4 * k) : 0u;
            for (int half = 0; half < 2; ++half) {
              const int q0 = rnd * 64 + 32 * half;
              if (q0 >= nitems) break;  // (uniform)
#if WAB2_BUSH_THROTTLE
              if (half) __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
              if (hf == half) {
                uint8_t* rec = stage + (lane & 31) * R;
                *reinterpret_cast<u32x4*>(rec) = (u32x4){(uint32_t)fb, (uint32_t)(fb >> 32), bxy & 0xFFu, bxy >> 8};
                *reinterpret_cast<uint2*>(rec + 16) = make_uint2(vis, (uint32_t)T_BUSH << 16);
                // the bush-food bytes as whole dwords from bb & ~3 (the record's bytes around them
                // are zero: deltas, tail): dword k holds bushes 4k - sh .. 4k - sh + 3
                if (kFixed) {
                  uint32_t xs[kRowW];
#pragma unroll
                  for (int k = 0; k < kRowW; ++k) {
                    uint32_t x = rdw[k];
                    if (sh) x = (x << (8 * sh)) | (k > 0 ? rdw[k > 0 ? k - 1 : 0] >> (32 - 8 * sh) : 0u);
                    const uint32_t b4 = (uint32_t)(v64 >> (NM + 4 * k - sh + 8)) & 0xFu;
                    xs[k] = x & (((b4 * 0x00204081u) & 0x01010101u) * 0xFFu);
                  }
                  if (!(WAB2_ABLATE & 4)) {
                    if (WAB2_BUSH_WIDE) {
                      put_dwords<kFixed ? (24 + 2 * kN) / 4 : 0, kRowW, kFixed ? (24 + 2 * kN + CNB + 15) / 16 * 4 : 0>(rec, xs);
                    } else {
#pragma unroll
                      for (int k = 0; k < kRowW; ++k) *reinterpret_cast<uint32_t*>(rec + 4 * (d0 + k)) = xs[k];
                    }
                  }
                } else
                for (int k = 0; k < ((WAB2_ABLATE & 4) ? 0 : ndw); ++k) {
                  uint32_t x = *reinterpret_cast<const uint32_t*>(row + 4 * k);
                  if (sh) x = (x << 16) | (k > 0 ? *reinterpret_cast<const uint32_t*>(row + 4 * k - 4) >> 16 : 0u);
                  const uint32_t b4 = (uint32_t)(v64 >> (NM + 4 * k - sh + 8)) & 0xFu;
                  *reinterpret_cast<uint32_t*>(rec + 4 * (d0 + k)) = x & (((b4 * 0x00204081u) & 0x01010101u) * 0xFFu);
                }
              }
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              const int chunks = min(32, nitems - q0) * CR;
              const int w0r = (int)(((uint32_t)q0 * magic_b) >> 20);
              uint8_t* rbase = obs_t + (item0 + (int64_t)w0r * no + (c0 - o0)) * R;
              copy_out<kCopyMax>(stage, rbase, (WAB2_ABLATE & 2) ? 0 : chunks, lane, q0, w0r, no, nc, R, CR, magic_cr, magic_b);
#if WAB2_POST_THROTTLE
              __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
              __builtin_amdgcn_wave_barrier();
            }
          }
        }
      }
      WAB2_STAMP(3);
      // ---- the movers
#pragma unroll
      for (int cls = 1; cls < 2; ++cls) {
        const bool bush = cls == 0;
        // the class's observers [c0, c1) of the window
        const int c0 = bush ? max(o0, NM) : o0, c1 = bush ? wo1 : min(wo1, NM);
        const int nc = max(0, c1 - c0);
        const uint32_t magic = bush ? magic_b : magic_m;  // q / nc = (q * magic) >> 20
        const int nitems = (WAB2_ABLATE & (bush ? 16 : 32)) ? 0 : nvalid * nc;
        for (int rnd = wave; rnd * 32 < nitems; rnd += 4) {
          // (tuning A/B: cap the wave's record stores in flight at a mover round's start)
#if WAB2_STORE_THROTTLE >= 0
          __builtin_amdgcn_s_waitcnt((WAB2_STORE_THROTTLE & 15) | ((WAB2_STORE_THROTTLE >> 4) << 14) | 0x0F70);
#endif
          const int q = rnd * 32 + (lane & 31);
          const bool on = q < nitems;
          const int qc = on ? q : nitems - 1;  // (lanes past the last item compute a copy of it)
          const int w = (int)(((uint32_t)qc * magic) >> 20);
          const int i = c0 + qc - w * nc;
          // (the fixed instance: a mover observer; every entity from NM on is then seen at its
          // position before the launch, with no per-entity select)
          if (kFixed) __builtin_assume(i >= 0 && i < NM);
          const int type = bush ? T_BUSH : i < NO ? T_OSTRICH : T_WOLF;
          const uint32_t* posw = s.pos + w * Np;
          const uint32_t pi = posw[i];
          const uint32_t ob = (!bush && type == T_OSTRICH) ? s.ost[i * kWorlds + w] : 0u;
          const int role = ost_role(ob), status = ost_status(ob);
          // ostriches still Visible when i observes (Lds::alv)
          const uint32_t alive = 0xFFFFFF00u | s.alv[min(i, NM) * kWorlds + w];
          // rows of the frame: alive (the ostriches) and existing (j < N)
          const uint32_t vmask = alive & exist & (!bush && (WAB2_ABLATE & 1) ? 0u : ~0u);
          // entity j is where observer i sees it: after its act if it acted in this launch
          // before i (a0 <= j < i), else at its frame position from before the launch
          const int jn = min(i, a1);
          uint32_t vis = 0, d[NKK];
          uint2 pp[NKK];  // this lane's entities of the world, all loads issued before any use
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) pp[kk] = *reinterpret_cast<const uint2*>(posw + 4 * kk + 2 * hf);
          if (bush) {
            // radius 0: the entities on the observer's tile (its frame X/Y before its act)
            const uint32_t tgt = pi & 0xFFFFu;
#pragma unroll
            for (int kk = 0; kk < NKK; ++kk) {
              const int j = 4 * kk + 2 * hf;
              const uint32_t s0 = (uint32_t)((j >= a0) & (j < jn)) << 4, s1 = (uint32_t)((j + 1 >= a0) & (j + 1 < jn)) << 4;
              const uint32_t e0 = (uint32_t)(((pp[kk].x >> s0) & 0xFFFFu) == tgt);
              const uint32_t e1 = (uint32_t)(((pp[kk].y >> s1) & 0xFFFFu) == tgt);
              vis |= ((vmask >> j) & (e0 | (e1 << 1))) << j;
              d[kk] = 0u;
            }
          } else {
            View v;
            v.ex = (int)(pi & 0xFFu);
            v.ey = (int)((pi >> 8) & 0xFFu);
            v.W = W;
            v.H = H;
            // World.get_observations (:365-374)
            const int r = type == T_OSTRICH ? (role == 1 ? p.rg : p.rl) : p.rw;
            const int rc = min(r, 255);
            v.r2 = rc * rc;  // (dx^2 + dy^2) ** 0.5 <= r  <=>  dx^2 + dy^2 <= r^2 (integers)
            v.xl = v.ex < r ? max(W - r + v.ex, v.ex + W / 2 + 1) : 0x7FFF;
            v.xr = (v.ex >= r && W < v.ex + r) ? min(r - W + v.ex, v.ex - W / 2 - 1) : -0x7FFF;
            v.yl = v.ey < r ? max(H - r + v.ey, v.ey + H / 2 + 1) : 0x7FFF;
            v.yr = (v.ey >= r && H < v.ey + r) ? min(r - H + v.ey, v.ey - H / 2 - 1) : -0x7FFF;
            v.alive = alive;
#if WAB2_PACKED
            View2 v2;
            v2.e = (s16x2){(short)v.ex, (short)v.ey};
            v2.lo = (s16x2){(short)min(v.xl, 0x4000), (short)min(v.yl, 0x4000)};
            v2.hi = (s16x2){(short)max(v.xr, -0x4000), (short)max(v.yr, -0x4000)};
            v2.wh = (s16x2){(short)W, (short)H};
            v2.r2 = v.r2;
#pragma unroll
            for (int kk = 0; kk < NKK; ++kk) {
              const int j = 4 * kk + 2 * hf;
              const uint32_t s0 = (uint32_t)((j >= a0) & (j < jn)) << 4, s1 = (uint32_t)((j + 1 >= a0) & (j + 1 < jn)) << 4;
              uint32_t ok0, ok1;
              const uint32_t p0 = view_pair2(v2, (pp[kk].x >> s0) & 0xFFFFu, ok0);
              const uint32_t p1 = view_pair2(v2, (pp[kk].y >> s1) & 0xFFFFu, ok1);
              const uint32_t m = (vmask >> j) & (ok0 | (ok1 << 1));
              vis |= m << j;
              d[kk] = (p0 & (0u - (m & 1u))) | ((p1 << 16) & (0u - (m >> 1)));
            }
#else
#pragma unroll
            for (int kk = 0; kk < NKK; ++kk) {
              const int j = 4 * kk + 2 * hf;
              // 16-bit shift by 16 where the entity acted before i in this launch (a0 <= j < i)
              const uint32_t s0 = (uint32_t)((j >= a0) & (j < jn)) << 4, s1 = (uint32_t)((j + 1 >= a0) & (j + 1 < jn)) << 4;
              const uint32_t x0 = (pp[kk].x >> s0) & 0xFFFFu, x1 = (pp[kk].y >> s1) & 0xFFFFu;
              d[kk] = view_pair(v, x0, j, (vmask >> j) & 1u, vis) | (view_pair(v, x1, j + 1, (vmask >> (j + 1)) & 1u, vis) << 16);
            }
#endif
          }
          if (kFixed && WAB2_DELTA_B64) {  // (the other half's bits by a half swap, not an LDS permute)
            const auto r = __builtin_amdgcn_permlane32_swap(vis, vis, false, false);
            vis |= hf ? r[0] : r[1];
          } else {
            vis |= __shfl_xor(vis, 32);
          }
          // internal obs (World.py:17-18, 50-51, 80-81)
          double food;
          int x, y;
          if (bush) {
            const uint32_t bxy = s.bxy[(i - NM) * kWorlds + w];
            x = (int)(bxy & 0xFFu);
            y = (int)(bxy >> 8);
            food = (double)s.bf1[w * NBp + i - NM];  // the bushes act after every ostrich
          } else {
            const int2 xy = s.oxy[i * kWorlds + w];
            x = xy.x;
            y = xy.y;
            food = s.food[i * kWorlds + w];
          }
          const uint32_t flags = type == T_OSTRICH ? (uint32_t)role | ((uint32_t)status << 8) : 0u;
          uint8_t* rec = stage + (lane & 31) * R;
          // (the benched geometry, 25 entities and 16 bushes in 96-byte records: each lane writes
          // three whole 16-byte chunks of its item's record, the lower half chunks 0, 2, 4 and the
          // upper half 1, 3, 5, the delta dwords exchanged between the halves by three
          // v_permlane32_swap: three stage writes per lane instead of about ten narrow ones, each
          // a write of 32 records at stride 96 B, as bank-conflicted whatever its width)
          constexpr bool kChunks = kFixed && WAB2_MOVER_CHUNKS && kN == 25 && CNB == 16 && NKK == 7;
          if (kChunks && !bush) {
            const u32x4 rv = *reinterpret_cast<const u32x4*>((type == T_OSTRICH ? s.bf0 : s.bf1) + w * NBp);
            uint32_t F[4] = {rv[0], rv[1], rv[2], rv[3]};  // bush food bytes 4q .. 4q + 3
            if (type == T_OSTRICH) {  // (the eats of the ostriches that acted before i)
              for (int k = a0; k < min(a1, NO); ++k)
                if (k < i) {
                  const uint32_t e = s.ev[k * kWorlds + w], b = e & 0xFFu, sb = 8u * (b & 3u);
#pragma unroll
                  for (int q = 0; q < 4; ++q)
                    if ((b >> 2) == (uint32_t)q) F[q] = (F[q] & ~(0xFFu << sb)) | (((e >> 8) & 0xFFu) << sb);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint32_t b4 = (vis >> (NM + 4 * q)) & 0xFu;
              F[q] &= ((WAB2_ABLATE & 4) ? 0u : ~0u) & (((b4 * 0x00204081u) & 0x01010101u) * 0xFFu);
            }
            // a' = {lo: a lo, hi: b lo}, b' = {lo: a hi, hi: b hi}: delta dword k = 2kk + half
            const auto S1 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);  // k 2, 3 | 6, 7
            const auto S2 = __builtin_amdgcn_permlane32_swap(d[2], d[4], false, false);  // k 4, 5 | 8, 9
            const auto S3 = __builtin_amdgcn_permlane32_swap(d[5], d[0], false, false);  // k 10, 11 | 0, 1
            const uint64_t fb = (uint64_t)__double_as_longlong(food);
            // bytes 72-75: entity 24's delta (the lower half's d[6]; entity 25 is absent) and
            // bush-food bytes 0-1 from byte 74; the rest of the bush food to byte 89, then pad
            const uint32_t dw18 = d[6] | (F[0] << 16), dw19 = (F[0] >> 16) | (F[1] << 16);
            const uint32_t dw20 = (F[1] >> 16) | (F[2] << 16), dw21 = (F[2] >> 16) | (F[3] << 16), dw22 = F[3] >> 16;
            const uint32_t ft = flags | ((uint32_t)type << 16);
            const u32x4 c1 = hf ? (u32x4){vis, ft, S3[0], S3[1]} : (u32x4){(uint32_t)fb, (uint32_t)(fb >> 32), (uint32_t)x, (uint32_t)y};
            const u32x4 c2 = (u32x4){S1[0], S1[1], S2[0], S2[1]};
            const u32x4 c3 = hf ? (u32x4){dw20, dw21, dw22, 0u} : (u32x4){S3[0], S3[1], dw18, dw19};
            *reinterpret_cast<u32x4*>(rec + 16 * hf) = c1;
            *reinterpret_cast<u32x4*>(rec + 32 + 16 * hf) = c2;
            *reinterpret_cast<u32x4*>(rec + 64 + 16 * hf) = c3;
          } else {
            if (hf == 0) {
              const uint64_t fb = (uint64_t)__double_as_longlong(food);
              *reinterpret_cast<uint4*>(rec) = make_uint4((uint32_t)fb, (uint32_t)(fb >> 32), (uint32_t)x, (uint32_t)y);
              *reinterpret_cast<uint2*>(rec + 16) = make_uint2(vis, flags | ((uint32_t)type << 16));
            } else if (!bush) {
              // (only the pad past the bush-food bytes: the deltas and those bytes are written below
              // in full, and nothing writes the pad non-zero; the stage is zeroed each turn)
              for (int z = (bb + 2 * nbp + 3) & ~3; z < R; z += 4) *reinterpret_cast<uint32_t*>(rec + z) = 0u;
            }
            if (!bush && kFixed && WAB2_DELTA_B64) {
              // delta dwords in pairs: one v_permlane32_swap of d[kk], d[kk + 1] gives the lower
              // half dwords 2kk, 2kk + 1 and the upper half 2kk + 2, 2kk + 3, each one 8-byte
              // stage write (half the writes of 32 records at stride R, each as bank-conflicted)
  #pragma unroll
              for (int kk = 0; kk < NKK; kk += 2) {
                if (kk + 1 < NKK) {
                  const auto r = __builtin_amdgcn_permlane32_swap(d[kk], d[kk + 1], false, false);
                  const int k0 = 2 * kk + 2 * hf;
                  if (k0 + 1 < nd) *reinterpret_cast<uint2*>(rec + 24 + 4 * k0) = make_uint2(r[0], r[1]);
                  else if (k0 < nd) *reinterpret_cast<uint32_t*>(rec + 24 + 4 * k0) = r[0];
                } else if (2 * kk + hf < nd) {
                  *reinterpret_cast<uint32_t*>(rec + 24 + 4 * (2 * kk + hf)) = d[kk];
                }
              }
            } else if (!bush) {  // (a bush's deltas are zero: the stage's, since the turn's first round)
  #pragma unroll
              for (int kk = 0; kk < NKK; ++kk)
                if (2 * kk + hf < nd) *reinterpret_cast<uint32_t*>(rec + 24 + 4 * (2 * kk + hf)) = d[kk];
            }
            // Additional_Data [food] of the visible bushes as the observer sees them: after the
            // eats of the ostriches that acted before it in this launch (bf1 for every observer
            // after the ostriches); byte pairs m = 2mm + half
            if (bush && !(WAB2_ABLATE & 4)) {
              // a bush sees bf1; its record's bytes around the bush-food ones are zero (deltas,
              // tail), so the region goes out as whole dwords from bb & ~3: dword k holds bushes
              // 4k - sh .. 4k - sh + 3, masked by their visibility bits
              const uint8_t* row = s.bf1 + w * NBp;
              const int sh = bb & 3, d0 = bb >> 2, ndw = (sh + NB + 3) >> 2;
              const uint64_t v64 = (uint64_t)vis << 8;  // (bit NM + b + 8: bush b, b >= -8)
              for (int k = hf; k < ndw; k += 2) {
                const int b = 4 * k - sh;
                uint32_t x = *reinterpret_cast<const uint32_t*>(row + 4 * k);
                if (sh) x = (x << 16) | (k > 0 ? *reinterpret_cast<const uint32_t*>(row + 4 * k - 4) >> 16 : 0u);
                const uint32_t b4 = (uint32_t)(v64 >> (NM + b + 8)) & 0xFu;
                *reinterpret_cast<uint32_t*>(rec + 4 * (d0 + k)) = x & (((b4 * 0x00204081u) & 0x01010101u) * 0xFFu);
              }
            }
            // (the fixed instance with a 16-byte row: the row in one ds_read_b128, its byte pairs
            // m = 2mm + half by shifts; the loop below waited for each pair's read in turn)
            constexpr bool kRow128 = kFixed && WAB2_MOVER_ROW128 && CNB % 4 == 0 && CNB <= 16 && ((CNB + 3) & ~3) == 16;
            if (kRow128 && !bush && !(WAB2_ABLATE & 4)) {
              const u32x4 rv = *reinterpret_cast<const u32x4*>((type == T_OSTRICH ? s.bf0 : s.bf1) + w * NBp);
  #pragma unroll
              for (int mm = 0; mm < (kRow128 ? CNB / 4 : 0); ++mm) {
                const int b = 4 * mm + 2 * hf;
                uint32_t f = (rv[mm] >> (16 * hf)) & 0xFFFFu;
                if (type == T_OSTRICH) {
                  for (int k = a0; k < min(a1, NO); ++k)
                    if (k < i) {
                      const uint32_t e = s.ev[k * kWorlds + w];
                      if ((e & 0xFFu) == (uint32_t)b) f = (f & 0xFF00u) | (e >> 8);
                      if ((e & 0xFFu) == (uint32_t)b + 1u) f = (f & 0x00FFu) | (e & 0xFF00u);
                    }
                }
                const uint32_t vb = vis >> (NM + b);
                f &= ((vb & 1u) ? 0x00FFu : 0u) | ((b + 1 < NB && (vb & 2u)) ? 0xFF00u : 0u);
                *reinterpret_cast<uint16_t*>(rec + bb + b) = (uint16_t)f;
              }
            }
            for (int m = hf; m < ((kRow128 || bush || (WAB2_ABLATE & 4)) ? 0 : nbp); m += 2) {
              const int b = 2 * m;
              const uint8_t* row = (type == T_OSTRICH ? s.bf0 : s.bf1) + w * NBp;
              uint32_t f = *reinterpret_cast<const uint16_t*>(row + b);
              if (!bush && type == T_OSTRICH) {
                for (int k = a0; k < min(a1, NO); ++k)
                  if (k < i) {
                    const uint32_t e = s.ev[k * kWorlds + w];
                    if ((e & 0xFFu) == (uint32_t)b) f = (f & 0xFF00u) | (e >> 8);
                    if ((e & 0xFFu) == (uint32_t)b + 1u) f = (f & 0x00FFu) | (e & 0xFF00u);
                  }
              }
              const uint32_t vb = vis >> (NM + b);
              f &= ((vb & 1u) ? 0x00FFu : 0u) | ((b + 1 < NB && (vb & 2u)) ? 0xFF00u : 0u);
              *reinterpret_cast<uint16_t*>(rec + bb + b) = (uint16_t)f;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          // the round's records: runs of consecutive records in HBM (a world's observers of this
          // class), 16 bytes per lane, consecutive lanes at consecutive addresses within a run
          const int q0 = rnd * 32;
          const int chunks = min(32, nitems - q0) * CR;
          const int w0r = (int)(((uint32_t)q0 * magic) >> 20);  // the round's first world
          uint8_t* rbase = obs_t + (item0 + (int64_t)w0r * no + (c0 - o0)) * R;  // its first record
          copy_out<kCopyMax>(stage, rbase, (WAB2_ABLATE & 2) ? 0 : chunks, lane, q0, w0r, no, nc, R, CR, magic_cr, magic);
#if WAB2_POST_THROTTLE
          __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
          __builtin_amdgcn_wave_barrier();
        }
      }
      if (movers_first) {
        for (int c = lane; c < 2 * R; c += 64) reinterpret_cast<u32x4*>(stage)[c] = (u32x4){0u, 0u, 0u, 0u};
        // ---- the bush observers: one lane per (world, bush) item, 64 items per round, their
        // records staged and stored in two halves of 32
        {
          const int c0 = max(o0, NM), nc = max(0, wo1 - c0);
          const int nitems = (WAB2_ABLATE & 16) ? 0 : nvalid * nc;
          const int sh = bb & 3, d0 = bb >> 2, ndw = (sh + NB + 3) >> 2;
          for (int rnd = wave; rnd * 64 < nitems; rnd += 4) {
#if WAB2_STORE_THROTTLE >= 0
            // (as at a mover round's start; the compiler's own wait tracking had put this one
            // here already, from the action loads it carries as pending)
            __builtin_amdgcn_s_waitcnt((WAB2_STORE_THROTTLE & 15) | ((WAB2_STORE_THROTTLE >> 4) << 14) | 0x0F70);
#endif
            const int q = rnd * 64 + lane;
            const bool on = q < nitems;
            const int qc = on ? q : nitems - 1;
            const int w = (int)(((uint32_t)qc * magic_b) >> 20);
            const int i = c0 + qc - w * nc;
            // (the fixed instance: a bush observer; every mover has acted before it)
            if (kFixed) __builtin_assume(i >= NM && i < N);
            const uint32_t* posw = s.pos + w * Np;
            const uint32_t tgt = posw[i] & 0xFFFFu;  // (its frame X/Y before its act)
            // every wolf acts before a bush: the Visible ostriches of Lds::alv[NM]
            const uint32_t vmask = (0xFFFFFF00u | s.alv[NM * kWorlds + w]) & exist;
            const int jn = min(i, a1);
            uint2 pp[2 * NKK];
#pragma unroll
            for (int kk = 0; kk < 2 * NKK; ++kk) pp[kk] = *reinterpret_cast<const uint2*>(posw + 2 * kk);
            uint32_t vis = 0;
#pragma unroll
            for (int kk = 0; kk < 2 * NKK; ++kk) {
              const int j = 2 * kk;
              const uint32_t s0 = (uint32_t)((j >= a0) & (j < jn)) << 4, s1 = (uint32_t)((j + 1 >= a0) & (j + 1 < jn)) << 4;
              const uint32_t e0 = (uint32_t)(((pp[kk].x >> s0) & 0xFFFFu) == tgt);
              const uint32_t e1 = (uint32_t)(((pp[kk].y >> s1) & 0xFFFFu) == tgt);
              vis |= (e0 | (e1 << 1)) << j;
            }
            vis &= vmask;
            const uint8_t* row = s.bf1 + w * NBp;  // (bushes observe after every ostrich's eat)
            const uint32_t bxy = s.bxy[(i - NM) * kWorlds + w];
            const uint64_t fb = (uint64_t)__double_as_longlong((double)row[i - NM]);
            const uint64_t v64 = (uint64_t)vis << 8;  // (bit NM + b + 8: bush b, b >= -8)
            // the fixed instance: the row's dwords read once, before the halves' stage writes
            // (which the compiler would otherwise order each row read behind)
            constexpr int kRowW = kFixed ? (((24 + 2 * kN) & 3) + CNB + 3) / 4 : 1;
            uint32_t rdw[kRowW];
#pragma unroll
            for (int k = 0; k < kRowW; ++k) rdw[k] = kFixed ? *reinterpret_cast<const uint32_t*>(row + 4 * k) : 0u;
            for (int half = 0; half < 2; ++half) {
              const int q0 = rnd * 64 + 32 * half;
              if (q0 >= nitems) break;  // (uniform)
#if WAB2_BUSH_THROTTLE
              if (half) __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
              if (hf == half) {
                uint8_t* rec = stage + (lane & 31) * R;
                *reinterpret_cast<u32x4*>(rec) = (u32x4){(uint32_t)fb, (uint32_t)(fb >> 32), bxy & 0xFFu, bxy >> 8};
                *reinterpret_cast<uint2*>(rec + 16) = make_uint2(vis, (uint32_t)T_BUSH << 16);
                // the bush-food bytes as whole dwords from bb & ~3 (the record's bytes around them
                // are zero: deltas, tail): dword k holds bushes 4k - sh .. 4k - sh + 3
                if (kFixed) {
                  uint32_t xs[kRowW];
#pragma unroll
                  for (int k = 0; k < kRowW; ++k) {
                    uint32_t x = rdw[k];
                    if (sh) x = (x << (8 * sh)) | (k > 0 ? rdw[k > 0 ? k - 1 : 0] >> (32 - 8 * sh) : 0u);
                    const uint32_t b4 = (uint32_t)(v64 >> (NM + 4 * k - sh + 8)) & 0xFu;
                    xs[k] = x & (((b4 * 0x00204081u) & 0x01010101u) * 0xFFu);
                  }
                  if (!(WAB2_ABLATE & 4)) {
                    if (WAB2_BUSH_WIDE) {
                      put_dwords<kFixed ? (24 + 2 * kN) / 4 : 0, kRowW, kFixed ? (24 + 2 * kN + CNB + 15) / 16 * 4 : 0>(rec, xs);
                    } else {
#pragma unroll
                      for (int k = 0; k < kRowW; ++k) *reinterpret_cast<uint32_t*>(rec + 4 * (d0 + k)) = xs[k];
                    }
                  }
                } else
                for (int k = 0; k < ((WAB2_ABLATE & 4) ? 0 : ndw); ++k) {
                  uint32_t x = *reinterpret_cast<const uint32_t*>(row + 4 * k);
                  if (sh) x = (x << 16) | (k > 0 ? *reinterpret_cast<const uint32_t*>(row + 4 * k - 4) >> 16 : 0u);
                  const uint32_t b4 = (uint32_t)(v64 >> (NM + 4 * k - sh + 8)) & 0xFu;
                  *reinterpret_cast<uint32_t*>(rec + 4 * (d0 + k)) = x & (((b4 * 0x00204081u) & 0x01010101u) * 0xFFu);
                }
              }
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              const int chunks = min(32, nitems - q0) * CR;
              const int w0r = (int)(((uint32_t)q0 * magic_b) >> 20);
              uint8_t* rbase = obs_t + (item0 + (int64_t)w0r * no + (c0 - o0)) * R;
              copy_out<kCopyMax>(stage, rbase, (WAB2_ABLATE & 2) ? 0 : chunks, lane, q0, w0r, no, nc, R, CR, magic_cr, magic_b);
#if WAB2_POST_THROTTLE
              __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
              __builtin_amdgcn_wave_barrier();
            }
          }
        }
      }
      WAB2_STAMP(4);
      // the next turn's actions, by W3 at the end of its rounds (it reaches the phase-B barrier
      // with the most slack, and the fetch's HBM round trip was the longest part of phase A);
      // the buffer is the one turn t - 1 used, read last in its phase C
      if (WAB2_ACT_LATE && kFixed && wave == 3 && t + 1 < T) fetch_actions_wave(p, t + 1, wg0, nvalid, (t & 1) ? s.act0 : s.act1, lane);
      // reward and done of a whole turn's (world, entity) items (compute_reward World.py:21-22,
      // 54-58, 84-85; is_entity_done :339-343), from the tables as the observers saw them (phase
      // C updates them after the barrier): the workgroup's [64][N] slice of [B][N] is contiguous,
      // so consecutive lanes store consecutive floats and bytes
      if (whole_turn) {
        const int64_t o = (int64_t)t * p.B * N + wg0 * N;
        // (branch-free: the lanes of one store hold every entity type; reward_done's cases as
        // selects, the table reads clamped into their tables)
        for (int q = tid; q < nvalid * N; q += kThreads) {
          const int w = (int)(((uint32_t)q * magic_n) >> 20), e = q - w * N;
          const int em = min(e, NM - 1), eo = min(e, NO - 1);
          const double food = NM > 0 ? s.food[em * kWorlds + w] : 0.0;
          const bool wolf_fed = (NM > 0 ? s.gain[em * kWorlds + w] : 0u) != 0u;
          const bool alive = NO > 0 && ost_status(s.ost[eo * kWorlds + w]) == 0;
          const bool ost = e < NO, wolf = e >= NO && e < NM;
          const bool wolf_rew = (wolf_fed ? food + p.wff : food) > 10.0;
          p.reward[o + q] = (ost ? alive : wolf && wolf_rew) ? 1.0f : 0.0f;
          p.done[o + q] = (uint8_t)(ost ? !alive : !wolf);
        }
      }
    }
    WAB2_STAMP(5);
    lds_barrier();
    WAB2_STAMP(6);

    // ================= phase C: the launch's end, one lane per (entity, world): the acting
    // entities' moves, roles and food, every ostrich's kills, the bushes' food, the autoreset
    {
      WAB2_PHASE_PARAMS;
      const uint8_t* A = (t & 1) ? s.act1 : s.act0;
      const bool whole_turn = a0 == 0 && a1 == N && wo0 == 0 && wo1 == N;
      for (int q = tid; q < ((WAB2_ABLATE & 8) ? 0 : nent); q += kThreads) {
        const int e = q >> 6, w = q & 63;
        const uint32_t epr = s.ep_reset[w];
        const bool acts = e >= a0 && e < a1;
        if (acts) s.pos[w * Np + e] >>= 16;  // the frame X/Y after the act (a reset leaves it)
        const int a = acts ? (int)(int8_t)A[w * na + e - a0] : -1;
        if (e < NM) {
          int2 xy = s.oxy[e * kWorlds + w];
          xy.x += move_dx(a);
          xy.y += move_dy(a);
          uint32_t om = acts ? moved(s.omod[e * kWorlds + w], a, W, H) : s.omod[e * kWorlds + w];
          double f = s.food[e * kWorlds + w];
          const uint32_t g = acts ? s.gain[e * kWorlds + w] : 0u;
          const uint32_t ob0 = e < NO ? s.ost[e * kWorlds + w] : 0u;  // before this launch's kills
          if (e < NO) {
            f += (double)g;
            uint32_t ob = ob0;
            if (a == 4) ob &= ~4u;
            if (a == 5) ob |= 4u;
            if (s.killed[e * kWorlds + w]) ob = (ob & ~3u) | 2u;
            if (s.hid[e * kWorlds + w] != 0xFFu) ob &= ~8u;
            if (epr) ob = ((uint32_t)p.role0 << 2) | 8u;
            s.ost[e * kWorlds + w] = (uint8_t)ob;
          } else {
            if (g) f += p.wff;
          }
          const double f_act = f;  // after the act, before a reset at the turn's end
          if (epr) f = e < NO ? p.ofood0 : p.wfood0;
          if (!whole_turn && acts && w < nvalid) {
            // take_action's (reward, done): an ostrich's status as its own update left it (the
            // wolves that may kill it act after it), a wolf's food after its update
            float rew;
            uint8_t dn;
            reward_done(e < NO ? T_OSTRICH : T_WOLF, ost_status(ob0), f_act, rew, dn);
            p.reward[(int64_t)(wg0 + w) * na + e - a0] = rew;
            p.done[(int64_t)(wg0 + w) * na + e - a0] = dn;
          }
          if (!epr) {  // (a reset world's new positions: the loop below)
            s.oxy[e * kWorlds + w] = xy;
            s.omod[e * kWorlds + w] = (uint16_t)om;
          }
          s.food[e * kWorlds + w] = f;
        } else {
          const int b = e - NM;
          s.bf0[w * NBp + b] = epr ? (uint8_t)p.fpb : s.bf1[w * NBp + b];
          if (!whole_turn && acts && w < nvalid) {
            p.reward[(int64_t)(wg0 + w) * na + e - a0] = 0.0f;
            p.done[(int64_t)(wg0 + w) * na + e - a0] = 1;
          }
        }
        if (e == 0 && a1 == N && na > 0) {  // the turn ends: World.increment_turn (WAB_Environment2.py:131-133)
          s.turn[w] = epr ? 0 : s.turn[w] + 1;
          if (epr) s.ep[w] = epr;
        }
      }
      // reset_environment's new positions, randint(0, W), randint(0, H) per entity
      // (WAB_Environment2_Single.py:45-46), for the worlds that reset (about one in 70 per
      // turn): a loop over those worlds, lane e drawing entity e's, instead of every lane of a
      // wave taking the draws' path whenever one of its 64 worlds resets
      if (!(WAB2_ABLATE & 8)) {
        for (uint64_t m = __ballot(s.ep_reset[lane] != 0u); m; m &= m - 1) {
          const int w = __builtin_ctzll(m);
          const uint64_t ek = world_key(p, wg0 + w, s.ep_reset[w]);
          for (int e = tid; e < N; e += kThreads) {
            const int nx = keyed_below(ek, SITE_T_RESET, 0, e, 0, (uint32_t)W + 1u);
            const int ny = keyed_below(ek, SITE_T_RESET, 0, e, 1, (uint32_t)H + 1u);
            if (e < NM) {
              s.oxy[e * kWorlds + w] = make_int2(nx, ny);
              s.omod[e * kWorlds + w] = (uint16_t)((uint32_t)wrap1(nx, W) | ((uint32_t)wrap1(ny, H) << 8));
            } else {
              s.bxy[(e - NM) * kWorlds + w] = (uint16_t)(nx | (ny << 8));
            }
          }
        }
      }
    }
    WAB2_STAMP(7);
    lds_barrier();
    WAB2_STAMP(8);
  }

  // ---- epilogue: LDS tables -> state
  {
    WAB2_PHASE_PARAMS;
    for (int q = tid; q < nent; q += kThreads) {
      const int e = q >> 6, w = q & 63;
      const int64_t a = (int64_t)e * p.Bp + wg0 + w;
      p.df[a] = (uint16_t)s.pos[w * Np + e];
      if (e < NM) {
        const int2 xy = s.oxy[e * kWorlds + w];
        p.ox[a] = xy.x;
        p.oy[a] = xy.y;
        p.food[(int64_t)e * p.Bp + wg0 + w] = s.food[e * kWorlds + w];
      } else {
        const int b = e - NM;
        const uint32_t bxy = s.bxy[b * kWorlds + w];
        p.ox[a] = (int32_t)(bxy & 0xFFu);
        p.oy[a] = (int32_t)(bxy >> 8);
        p.bfood[(int64_t)b * p.Bp + wg0 + w] = s.bf0[w * NBp + b];
      }
      if (e < NO) p.ost[(int64_t)e * p.Bp + wg0 + w] = s.ost[e * kWorlds + w];
      if (e == 0) {
        p.turn[wg0 + w] = s.turn[w];
        p.episode[wg0 + w] = s.ep[w];
      }
    }
  }
  if (wave == 1) {  // resets of this workgroup (W1 decided them), one atomic per wave
    unsigned long long tot = (unsigned long long)resets;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    if (lane == 0 && tot) atomicAdd(&p0.counters[1], tot);
  }
  if (blockIdx.x == 0 && tid == 0 && p0.a1 == p0.N && p0.a1 > p0.a0)
    atomicAdd(&p0.counters[0], (unsigned long long)p0.B * (unsigned long long)T);
#undef WAB2_PHASE_PARAMS
}

// an explicit position of entity e in world g (wab2_create_at / wab2_reset_at), or false: the
// keyed random draw (a negative coordinate asks for it, as WAB_Environment2_Single.reset's
// `new_x < 0 or new_y < 0` does, WAB_Environment2_Single.py:36-41)
__device__ __forceinline__ bool explicit_pos(const TParams& p, int64_t g, int e, int& x, int& y) {
  if (!p.pos || g >= p.B) return false;
  const int32_t* q = p.pos + (g * p.N + e) * 2;
  if (q[0] < 0 || q[1] < 0) return false;
  x = q[0];
  y = q[1];
  return true;
}

// create_ostriches / create_wolves / create_bushes: spawn_positions given, or random positions
// randint(0, W - 1), randint(0, H - 1) per entity (WAB_Environment2.py:61-110), episode 0; one
// lane per world
__global__ void wab_torus_create_kernel(TParams p) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= p.Bp) return;
  const uint64_t ek = world_key(p, g, 0);
  for (int e = 0; e < p.N; ++e) {
    int x, y;
    if (!explicit_pos(p, g, e, x, y)) {
      x = keyed_below(ek, SITE_T_CREATE, 0, e, 0, (uint32_t)p.W);
      y = keyed_below(ek, SITE_T_CREATE, 0, e, 1, (uint32_t)p.H);
    }
    const int64_t a = (int64_t)e * p.Bp + g;
    p.ox[a] = x;
    p.oy[a] = y;
    p.df[a] = (uint16_t)(x | (y << 8));
    if (e < p.NM) p.food[a] = e < p.NO ? p.ofood0 : p.wfood0;
    else p.bfood[(int64_t)(e - p.NM) * p.Bp + g] = (uint8_t)p.fpb;
    if (e < p.NO) p.ost[(int64_t)e * p.Bp + g] = (uint8_t)((p.role0 << 2) | 8);
  }
  p.turn[g] = 0;
  p.episode[g] = 0;
}

// reset_environment (WAB_Environment2.py:113-118) of the masked worlds, each entity's
// reset(new_x, new_y) with the given position or the random one (WAB_Environment2_Single.py:36-48);
// one lane per world
__global__ void wab_torus_reset_kernel(TParams p) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= p.B || (p.mask && !p.mask[g])) return;
  const uint32_t ep = p.episode[g] + 1u;
  const uint64_t ek = world_key(p, g, ep);
  for (int e = 0; e < p.N; ++e) {
    int x, y;
    if (!explicit_pos(p, g, e, x, y)) {
      x = keyed_below(ek, SITE_T_RESET, 0, e, 0, (uint32_t)p.W + 1u);
      y = keyed_below(ek, SITE_T_RESET, 0, e, 1, (uint32_t)p.H + 1u);
    }
    const int64_t a = (int64_t)e * p.Bp + g;
    p.ox[a] = x;
    p.oy[a] = y;
    if (e < p.NM) p.food[a] = e < p.NO ? p.ofood0 : p.wfood0;
    else p.bfood[(int64_t)(e - p.NM) * p.Bp + g] = (uint8_t)p.fpb;
    if (e < p.NO) p.ost[(int64_t)e * p.Bp + g] = (uint8_t)((p.role0 << 2) | 8);
  }
  p.turn[g] = 0;
  p.episode[g] = ep;
  atomicAdd(&p.counters[1], 1ull);
}

}  // namespace wab2

using wab2::TParams;

struct wab2_handle {
  TParams p;
  int next_entity = 0;  // the entity whose take_action comes next this turn (the same in every world)
  int device = 0;
  int n_blocks = 0;
  size_t lds = 0;
  int32_t* pos = nullptr;  // device copy of the last explicit positions (wab2_create_at / wab2_reset_at)
  std::vector<void*> allocs;
};

namespace {

thread_local std::string g_err2;

int fail(int code, const std::string& msg) {
  g_err2 = msg;
  return code;
}

#define HIP_TRY2(expr)                                                                \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(WAB2_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard2 {
  int prev = -1;
  explicit DeviceGuard2(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard2() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int record_size(const wab2_config* c) {
  const int N = c->num_ostriches + c->num_wolves + c->num_bushes;
  return (24 + 2 * N + c->num_bushes + 15) / 16 * 16;
}

std::string validate(const wab2_config* c) {
  if (!c) return "config is NULL";
  if (c->width < 1 || c->width > WAB2_MAX_SIDE || c->height < 1 || c->height > WAB2_MAX_SIDE)
    return "width and height must be in [1, 127]";
  if (c->num_ostriches < 0 || c->num_wolves < 0 || c->num_bushes < 0) return "negative entity count";
  if (c->num_ostriches > WAB2_MAX_OSTRICHES) return "at most 8 ostriches";
  const int N = c->num_ostriches + c->num_wolves + c->num_bushes;
  if (N < 1 || N > WAB2_MAX_ENTITIES) return "1 to 32 entities in all";
  if (c->starting_role != 0 && c->starting_role != 1) return "starting_role must be 0 or 1";
  if (c->food_per_bush < 0 || c->food_per_bush > 255 || c->food_given_per_turn < 0 || c->food_given_per_turn > 255)
    return "food_per_bush and food_given_per_turn must be in [0, 255]";
  // (a radius past the world's diagonal sees everything; the cap keeps r - W + ex and W < ex + r
  // of the view thresholds inside int32)
  if (c->lookout_view_radius < 0 || c->gatherer_view_radius < 0 || c->wolf_view_radius < 0 ||
      c->lookout_view_radius > WAB2_MAX_RADIUS || c->gatherer_view_radius > WAB2_MAX_RADIUS ||
      c->wolf_view_radius > WAB2_MAX_RADIUS)
    return "view radii must be in [0, 2^20]";
  if (c->max_turns < 0) return "max_turns must be >= 0";
  return "";
}

// explicit positions [B][N][2] (host, or NULL): each pair either has a negative coordinate (the
// keyed random draw) or lies in [0, xmax] x [0, ymax]
std::string check_positions(const int32_t* pos, int64_t B, int N, int xmax, int ymax, const char* who) {
  if (!pos) return "";
  for (int64_t k = 0; k < B * N; ++k) {
    const int32_t x = pos[2 * k], y = pos[2 * k + 1];
    if (x < 0 || y < 0) continue;
    if (x > xmax || y > ymax)
      return std::string(who) + ": position (" + std::to_string(x) + ", " + std::to_string(y) + ") of world " +
             std::to_string(k / N) + " entity " + std::to_string(k % N) + " outside [0, " + std::to_string(xmax) +
             "] x [0, " + std::to_string(ymax) + "] (a negative coordinate draws the random position)";
  }
  return "";
}

// whole turns of the benched world's counts (BASELINE config 3: 1 ostrich, 8 wolves, 16 bushes)
// have an instance of their own with the counts and the (whole) windows as constants
bool fixed_counts(const TParams& p) {
  return p.NO == 1 && p.NW == 8 && p.NB == 16 && p.a0 == 0 && p.a1 == p.N && p.o0 == 0 && p.o1 == p.N;
}

// the kernel instantiation for N entities: ceil(N / 4) dword-pair groups of the delta array
const void* torus_kernel(const TParams& p) {
  if (fixed_counts(p)) return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<7, 1, 8, 16>);
  switch ((p.N + 3) / 4) {
    case 1: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<1>);
    case 2: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<2>);
    case 3: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<3>);
    case 4: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<4>);
    case 5: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<5>);
    case 6: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<6>);
    case 7: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<7>);
    default: return reinterpret_cast<const void*>(&wab2::wab_torus_kernel<8>);
  }
}

uint32_t magic20(int n) { return n > 0 ? (uint32_t)(((1u << 20) + (uint32_t)n - 1u) / (uint32_t)n) : 0u; }

void launch_torus(const wab2_handle* h, const TParams& p0, hipStream_t stream) {
  const dim3 grid((unsigned)h->n_blocks), block(wab2::kThreads);
  TParams p = p0;
  p.magic_m = magic20(std::min(p.o1, p.NM) - p.o0);
  p.magic_b = magic20(p.o1 - std::max(p.o0, p.NM));
  p.magic_cr = (uint32_t)((65536 + p.R / 16 - 1) / (p.R / 16));
  p.magic_n = magic20(p.N);
#if WAB2_STAMPS
  p.stamps = (unsigned long long*)(uintptr_t)strtoull(getenv("WAB2_STAMPS_PTR") ? getenv("WAB2_STAMPS_PTR") : "0", nullptr, 0);
#endif
  if (fixed_counts(p)) {
    hipLaunchKernelGGL((wab2::wab_torus_kernel<7, 1, 8, 16>), grid, block, h->lds, stream, p);
    return;
  }
  switch ((p.N + 3) / 4) {
    case 1: hipLaunchKernelGGL(wab2::wab_torus_kernel<1>, grid, block, h->lds, stream, p); break;
    case 2: hipLaunchKernelGGL(wab2::wab_torus_kernel<2>, grid, block, h->lds, stream, p); break;
    case 3: hipLaunchKernelGGL(wab2::wab_torus_kernel<3>, grid, block, h->lds, stream, p); break;
    case 4: hipLaunchKernelGGL(wab2::wab_torus_kernel<4>, grid, block, h->lds, stream, p); break;
    case 5: hipLaunchKernelGGL(wab2::wab_torus_kernel<5>, grid, block, h->lds, stream, p); break;
    case 6: hipLaunchKernelGGL(wab2::wab_torus_kernel<6>, grid, block, h->lds, stream, p); break;
    case 7: hipLaunchKernelGGL(wab2::wab_torus_kernel<7>, grid, block, h->lds, stream, p); break;
    default: hipLaunchKernelGGL(wab2::wab_torus_kernel<8>, grid, block, h->lds, stream, p); break;
  }
}

}  // namespace

extern "C" {

int wab2_abi_version(void) { return WAB2_ABI_VERSION; }
const char* wab2_last_error(void) { return g_err2.c_str(); }
int wab2_record_size(const wab2_config* cfg) {
  const std::string v = validate(cfg);
  if (!v.empty()) return fail(WAB2_E_INVALID, v);
  return record_size(cfg);
}

int wab2_create(const wab2_config* cfg, int64_t batch, uint64_t seed, int64_t world_id_base, int device,
                wab2_handle** out) {
  return wab2_create_at(cfg, batch, seed, world_id_base, device, nullptr, out);
}

int wab2_create_at(const wab2_config* cfg, int64_t batch, uint64_t seed, int64_t world_id_base, int device,
                   const int32_t* positions, wab2_handle** out) {
  if (!out) return fail(WAB2_E_INVALID, "out is NULL");
  *out = nullptr;
  const std::string v = validate(cfg);
  if (!v.empty()) return fail(WAB2_E_INVALID, v);
  if (batch < 1) return fail(WAB2_E_INVALID, "batch must be >= 1");
  const int N = cfg->num_ostriches + cfg->num_wolves + cfg->num_bushes;
  // the frame holds create positions as they are (World.create_*, no modulo): on this surface
  // they are tiles of the world, [0, W) x [0, H)
  const std::string pv = check_positions(positions, batch, N, cfg->width - 1, cfg->height - 1, "wab2_create_at");
  if (!pv.empty()) return fail(WAB2_E_INVALID, pv);
  DeviceGuard2 dg(device);
  wab2_handle* h = new wab2_handle();
  h->device = device;
  TParams& p = h->p;
  p.N = cfg->num_ostriches + cfg->num_wolves + cfg->num_bushes;
  p.NO = cfg->num_ostriches;
  p.NW = cfg->num_wolves;
  p.NB = cfg->num_bushes;
  p.NM = p.NO + p.NW;
  p.R = record_size(cfg);
  p.W = cfg->width;
  p.H = cfg->height;
  p.rl = cfg->lookout_view_radius;
  p.rg = cfg->gatherer_view_radius;
  p.rw = cfg->wolf_view_radius;
  p.fpb = cfg->food_per_bush;
  p.fg = cfg->food_given_per_turn;
  p.ofood0 = cfg->ostrich_starting_food;
  p.wfood0 = cfg->wolf_starting_food;
  p.wff = cfg->wolf_food_for_eating_ostrich;
  p.role0 = cfg->starting_role;
  p.max_turns = cfg->max_turns;
  p.autoreset = cfg->autoreset ? 1 : 0;
  p.a0 = p.o0 = 0;
  p.a1 = p.o1 = p.N;
  p.B = batch;
  h->n_blocks = (int)((batch + wab2::kWorlds - 1) / wab2::kWorlds);
  p.Bp = (int64_t)h->n_blocks * wab2::kWorlds;
  p.seed = seed;
  p.world_base = world_id_base;
  const wab2::LdsLayout L = wab2::lds_layout(p.N, p.NO, p.NM, p.NB, p.R);
  h->lds = L.total;
  auto alloc = [&](void** ptr, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(ptr, bytes < 16 ? 16 : bytes);
    if (e == hipSuccess) {
      h->allocs.push_back(*ptr);
      e = hipMemset(*ptr, 0, bytes < 16 ? 16 : bytes);
    }
    return e;
  };
  const size_t NBp = (size_t)p.Bp;
  hipError_t e = hipSuccess;
  void* q = nullptr;
  if (e == hipSuccess) { e = alloc(&q, NBp * p.N * 4); p.ox = (int32_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * p.N * 4); p.oy = (int32_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * p.N * 2); p.df = (uint16_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * (p.NM ? p.NM : 1) * 8); p.food = (double*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * (p.NB ? p.NB : 1)); p.bfood = (uint8_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * (p.NO ? p.NO : 1)); p.ost = (uint8_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * 4); p.turn = (int32_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, NBp * 4); p.episode = (uint32_t*)q; }
  if (e == hipSuccess) { e = alloc(&q, 2 * sizeof(unsigned long long)); p.counters = (unsigned long long*)q; }
  if (e == hipSuccess && h->lds > 64 * 1024) {
    // the attribute is per kernel instance, which handles of other bush counts share: only ever
    // raise it (a later, smaller handle must not lower the limit an earlier one launches with)
    static std::mutex mu;
    static std::map<const void*, size_t> lds_set;
    std::lock_guard<std::mutex> lock(mu);
    size_t& cur = lds_set[torus_kernel(p)];
    if (h->lds > cur) {
      e = hipFuncSetAttribute(torus_kernel(p), hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds);
      if (e == hipSuccess) cur = h->lds;
    }
  }
  if (e == hipSuccess && positions) {
    const size_t bytes = (size_t)batch * p.N * 2 * sizeof(int32_t);
    e = alloc(&q, bytes);
    h->pos = (int32_t*)q;
    if (e == hipSuccess) e = hipMemcpy(h->pos, positions, bytes, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    TParams pc = p;
    pc.pos = h->pos;
    hipLaunchKernelGGL(wab2::wab_torus_create_kernel, dim3((unsigned)((p.Bp + 255) / 256)), dim3(256), 0, 0, pc);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    for (void* a : h->allocs) (void)hipFree(a);
    delete h;
    return fail(e == hipErrorOutOfMemory ? WAB2_E_NOMEM : WAB2_E_HIP, std::string("wab2_create: ") + hipGetErrorString(e));
  }
  *out = h;
  return WAB2_OK;
}

int wab2_destroy(wab2_handle* h) {
  if (!h) return WAB2_OK;
  DeviceGuard2 dg(h->device);
  (void)hipDeviceSynchronize();
  for (void* a : h->allocs) (void)hipFree(a);
  delete h;
  return WAB2_OK;
}

int64_t wab2_batch(const wab2_handle* h) { return h ? h->p.B : 0; }

int wab2_reset(wab2_handle* h, const uint8_t* mask, void* stream) {
  return wab2_reset_at(h, mask, nullptr, stream);
}

int wab2_reset_at(wab2_handle* h, const uint8_t* mask, const int32_t* positions, void* stream) {
  if (!h) return fail(WAB2_E_INVALID, "handle is NULL");
  if (mask && h->next_entity != 0)
    return fail(WAB2_E_INVALID, "wab2_reset: a masked reset only between turns (entity " +
                                    std::to_string(h->next_entity) + " acts next)");
  const TParams& hp = h->p;
  // the range of the random reset draws, randint(0, W) x randint(0, H) (a bush keeps its own x, y
  // in a byte each and its frame X = x mod W is one subtraction)
  const std::string pv = check_positions(positions, hp.B, hp.N, hp.W, hp.H, "wab2_reset_at");
  if (!pv.empty()) return fail(WAB2_E_INVALID, pv);
  h->next_entity = 0;  // reset_environment: num_entities_acted_this_turn = 0 (WAB_Environment2.py:117)
  DeviceGuard2 dg(h->device);
  TParams p = h->p;
  p.mask = mask;
  if (positions) {
    // the handle's position buffer (the last reset_at's launch has finished: synchronised below)
    const size_t bytes = (size_t)p.B * p.N * 2 * sizeof(int32_t);
    if (!h->pos) {
      void* q = nullptr;
      HIP_TRY2(hipMalloc(&q, bytes));
      h->allocs.push_back(q);
      h->pos = (int32_t*)q;
    }
    HIP_TRY2(hipMemcpyAsync(h->pos, positions, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    p.pos = h->pos;
  }
  hipLaunchKernelGGL(wab2::wab_torus_reset_kernel, dim3((unsigned)((p.B + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, p);
  HIP_TRY2(hipGetLastError());
  if (positions) HIP_TRY2(hipStreamSynchronize((hipStream_t)stream));  // the host array may go now
  return WAB2_OK;
}

int wab2_rollout(wab2_handle* h, const int8_t* actions, int32_t T, uint8_t* obs, float* reward, uint8_t* done,
                 uint8_t* world_reset, void* stream) {
  if (!h) return fail(WAB2_E_INVALID, "handle is NULL");
  if (T < 1) return fail(WAB2_E_INVALID, "T must be >= 1");
  if (!actions || !obs || !reward || !done) return fail(WAB2_E_INVALID, "actions, obs, reward and done are required");
  if (reinterpret_cast<uintptr_t>(obs) & 15u) return fail(WAB2_E_INVALID, "obs must be 16-byte aligned");
  if (h->next_entity != 0)
    return fail(WAB2_E_INVALID, "wab2_step/wab2_rollout: a turn is half done (entity " +
                                    std::to_string(h->next_entity) + " acts next: wab2_take_action)");
  DeviceGuard2 dg(h->device);
  TParams p = h->p;
  p.T = T;
  p.actions = actions;
  p.obs = obs;
  p.reward = reward;
  p.done = done;
  p.world_reset = world_reset;
  p.act_scalar = ((reinterpret_cast<uintptr_t>(actions) & 3u) == 0u && (p.B * p.N) % 4 == 0) ? 1 : 0;
  launch_torus(h, p, (hipStream_t)stream);
  HIP_TRY2(hipGetLastError());
  return WAB2_OK;
}

int wab2_step(wab2_handle* h, const int8_t* actions, uint8_t* obs, float* reward, uint8_t* done,
              uint8_t* world_reset, void* stream) {
  return wab2_rollout(h, actions, 1, obs, reward, done, world_reset, stream);
}

int wab2_get_obs(wab2_handle* h, int32_t entity, uint8_t* obs, void* stream) {
  if (!h) return fail(WAB2_E_INVALID, "handle is NULL");
  if (!obs || (reinterpret_cast<uintptr_t>(obs) & 15u)) return fail(WAB2_E_INVALID, "obs must be 16-byte aligned");
  if (entity < h->next_entity || entity >= h->p.N)
    return fail(WAB2_E_INVALID, "wab2_get_obs: entity " + std::to_string(entity) +
                                    " has acted this turn or does not exist (World.get_observations asserts "
                                    "the entity has not acted, World.py:362)");
  DeviceGuard2 dg(h->device);
  TParams p = h->p;
  p.T = 1;
  p.a0 = p.a1 = entity;  // nothing acts
  p.o0 = entity;
  p.o1 = entity + 1;
  p.obs = obs;
  p.actions = nullptr;
  p.reward = nullptr;
  p.done = nullptr;
  p.world_reset = nullptr;
  launch_torus(h, p, (hipStream_t)stream);
  HIP_TRY2(hipGetLastError());
  return WAB2_OK;
}

int wab2_take_action(wab2_handle* h, int32_t entity, const int8_t* actions, float* reward, uint8_t* done,
                     uint8_t* world_reset, void* stream) {
  if (!h) return fail(WAB2_E_INVALID, "handle is NULL");
  if (!actions || !reward || !done) return fail(WAB2_E_INVALID, "actions, reward and done are required");
  if (entity != h->next_entity)
    return fail(WAB2_E_INVALID, "wab2_take_action: entity " + std::to_string(h->next_entity) +
                                    " acts next (entities act in id order, once per turn)");
  DeviceGuard2 dg(h->device);
  TParams p = h->p;
  p.T = 1;
  p.a0 = entity;
  p.a1 = entity + 1;
  p.o0 = p.o1 = 0;  // no records
  p.obs = nullptr;
  p.actions = actions;
  p.reward = reward;
  p.done = done;
  p.world_reset = world_reset;
  launch_torus(h, p, (hipStream_t)stream);
  HIP_TRY2(hipGetLastError());
  h->next_entity = (entity + 1) % h->p.N;
  return WAB2_OK;
}

int wab2_get_state(wab2_handle* h, int32_t* df_xy, int32_t* obj_xy, double* food, uint8_t* visible, uint8_t* status,
                   int32_t* turn, uint32_t* episode, void* stream) {
  if (!h) return fail(WAB2_E_INVALID, "handle is NULL");
  DeviceGuard2 dg(h->device);
  const TParams& p = h->p;
  HIP_TRY2(hipStreamSynchronize((hipStream_t)stream));
  const size_t Bp = (size_t)p.Bp, B = (size_t)p.B, N = (size_t)p.N;
  std::vector<int32_t> ox(Bp * N), oy(Bp * N), tn(Bp);
  std::vector<uint16_t> df(Bp * N);
  std::vector<double> fd(Bp * (p.NM ? p.NM : 1));
  std::vector<uint8_t> bf(Bp * (p.NB ? p.NB : 1)), os(Bp * (p.NO ? p.NO : 1));
  std::vector<uint32_t> ep(Bp);
  HIP_TRY2(hipMemcpy(ox.data(), p.ox, ox.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(oy.data(), p.oy, oy.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(df.data(), p.df, df.size() * 2, hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(fd.data(), p.food, fd.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(bf.data(), p.bfood, bf.size(), hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(os.data(), p.ost, os.size(), hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(tn.data(), p.turn, tn.size() * 4, hipMemcpyDeviceToHost));
  HIP_TRY2(hipMemcpy(ep.data(), p.episode, ep.size() * 4, hipMemcpyDeviceToHost));
  for (size_t b = 0; b < B; ++b) {
    for (size_t e = 0; e < N; ++e) {
      const size_t a = e * Bp + b, q = b * N + e;
      if (df_xy) {
        df_xy[2 * q] = df[a] & 0xFF;
        df_xy[2 * q + 1] = df[a] >> 8;
      }
      if (obj_xy) {
        obj_xy[2 * q] = ox[a];
        obj_xy[2 * q + 1] = oy[a];
      }
      if (food) food[q] = (int)e < p.NM ? fd[a] : (double)bf[(e - p.NM) * Bp + b];
      if (visible) visible[q] = (int)e < p.NO ? (uint8_t)((os[a] >> 3) & 1) : (uint8_t)1;
      if (status && (int)e < p.NO) status[b * p.NO + e] = (uint8_t)(os[a] & 3);
    }
    if (turn) turn[b] = tn[b];
    if (episode) episode[b] = ep[b];
  }
  return WAB2_OK;
}

int wab2_get_counters(wab2_handle* h, wab2_counters* out, void* stream) {
  if (!h || !out) return fail(WAB2_E_INVALID, "handle or out is NULL");
  DeviceGuard2 dg(h->device);
  HIP_TRY2(hipStreamSynchronize((hipStream_t)stream));
  unsigned long long c[2];
  HIP_TRY2(hipMemcpy(c, h->p.counters, sizeof(c), hipMemcpyDeviceToHost));
  out->turns = c[0];
  out->resets = c[1];
  return WAB2_OK;
}

}  // extern "C"
