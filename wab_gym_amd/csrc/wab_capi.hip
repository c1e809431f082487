// wab_capi.hip — the C-ABI of include/wab.h on top of the fused HIP kernels.
//
// Owns per-env state in HBM (SoA, env innermost) and launches the step/reset kernels
// on the caller's stream.  No allocation, copy or synchronisation happens inside
// wab_step / wab_reset / wab_rollout, so they are safe to capture in a hipGraph.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/wab.h"
#include "wab_params.h"
#include "wab_device.h"
#include "wab_feat.h"

namespace wab {
template <int MODE, int SLOTS, bool SMALL>
__global__ void wab_kernel(Params p);
template <int SLOTS, int G, bool FEAT, bool ROLL>
__global__ void wab_step_small(Params p);
template <int MODE, int SLOTS>
__global__ void wab_step_wide(Params p);
template <int SLOTS, int FIXW>
__global__ void wab_rollout_wide(Params p);

__global__ void wab_featurize_kernel(FeatParams p);
__global__ void wab_featurize_small_kernel(FeatParams p);
__global__ void wab_render_kernel(RenderParams p);
__global__ void wab_egocentric_kernel(EgoParams p);
template <int VEC, int NE>
__global__ void wab_returns_kernel(const float* __restrict__ reward, const uint8_t* __restrict__ done, int32_t T,
                                   int64_t B, double gamma, const float* __restrict__ bootstrap,
                                   float* __restrict__ out, RewardTable tab);
}

using wab::Params;

struct wab_handle {
  Params p;
  int device = 0;
  int slots = 8;
  int n_blocks = 0;
  size_t lds_bytes = 0;
  int step_kernel = 0;         // KERNEL_BLOCK / KERNEL_SMALL
  size_t small_lds_bytes = 0;  // LDS of the small-view kernel
  size_t small_feat_lds_bytes = 0;  // ... with the fused featurizer (wab_step_features), 0: not fusable
  bool reset_done = false;
  std::vector<void*> allocs;
  uint8_t* scratch_planes = nullptr;  // wab_step_features without planes, not fusable (lazy)
  // egocentric observation (allocated by the first wab_egocentric call)
  uint4* ego_path = nullptr;
  uint32_t* ego_diamond = nullptr;
  int ego_cap = 0, ego_n_diamond = 0;
  bool small_g11 = false;    // the small kernel's 11x11 specialisation (geometry_11)
  wab::RewardTable rewards;  // exact doubles of the rewards a step returns (n = 0: ambiguous)
  size_t wide_lds_bytes = 0;  // LDS per workgroup of the wide kernel (see wab_create)
  size_t wide_roll_lds_bytes = 0;  // ... of its multi-step build (wab_rollout_wide)
  int32_t obs_placement = WAB_OBS_SAME_BUFFER;  // wab_set_obs_placement: which wide per-step build
  uint64_t rollout_launches = 0, rollout_step_calls = 0;  // wab_counters' host tallies
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return fail(WAB_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)

int n_actions_of(const wab_config* c) { return (c->gatherer_only || c->lookout_only) ? 5 : 6; }

// masks wab_env.py:109-139 as 11-bit row masks (bit j <=> mask[i][j] == 1)
const char* kLookout[11] = {"11100000111", "11000000011", "10000000001", "00000000000",
                            "00000000000", "00000000000", "00000000000", "00000000000",
                            "10000000001", "11000000011", "11100000111"};
const char* kGatherer[11] = {"11111111111", "11111111111", "11111111111", "11110001111",
                             "11100000111", "11100000111", "11100000111", "11110001111",
                             "11111111111", "11111111111", "11111111111"};

uint32_t row_mask(const char* s) {
  uint32_t m = 0;
  for (int j = 0; j < 11; ++j)
    if (s[j] == '1') m |= 1u << j;
  return m;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

template <int MODE, bool SMALL>
void* kernel_ptr(int slots) {
  switch (slots) {
    case 8: return reinterpret_cast<void*>(&wab::wab_kernel<MODE, 8, SMALL>);
    case 16: return reinterpret_cast<void*>(&wab::wab_kernel<MODE, 16, SMALL>);
    default: return reinterpret_cast<void*>(&wab::wab_kernel<MODE, 32, SMALL>);
  }
}

template <int MODE, bool SMALL>
void launch_as(wab_handle* h, const Params& p, hipStream_t stream) {
  const dim3 grid(h->n_blocks), block(wab::kThreads);
  switch (h->slots) {
    case 8: hipLaunchKernelGGL((wab::wab_kernel<MODE, 8, SMALL>), grid, block, h->lds_bytes, stream, p); break;
    case 16: hipLaunchKernelGGL((wab::wab_kernel<MODE, 16, SMALL>), grid, block, h->lds_bytes, stream, p); break;
    default: hipLaunchKernelGGL((wab::wab_kernel<MODE, 32, SMALL>), grid, block, h->lds_bytes, stream, p); break;
  }
}

// SMALL: the W*H-bit view bitmap fits 4 registers (default 11x11 = 121 bits)
bool small_map(const Params& p) { return p.WHW <= 4; }

// Step kernels.  The block kernel (wab_step.hip) handles every configuration; views whose
// planes fit 128 bits (W*H <= 128, unpadded rows, spawn ring <= 128 tiles, restrict_view only
// at exactly 11x11) step with the four-wave small-view kernel (wab_step_small.hip); other
// views of width <= 31 and height <= 32 in rows of 16 or 32 bytes without restrict_view step
// and reset with the wide-view kernel (wab_step_wide.hip, its own bitmap layout: one dword per
// row).
enum { KERNEL_BLOCK = 0, KERNEL_SMALL = 1, KERNEL_WIDE = 2 };

// (W, H >= 3: the strip that scrolls into view, drawn on another wave, never holds the
// ostrich's tile; W, H <= 32: its bits are one dword)
bool small_view(const Params& p) {
  return p.WH <= 128 && p.W >= 3 && p.H >= 3 && p.W <= 32 && p.H <= 32 && p.S == p.H && p.R <= 128 &&
         (!p.restrict_view || (p.W == 11 && p.H == 11));
}

// the default options' geometry (11x11 in 11-byte rows, a 48-tile spawn ring): the small
// kernel's compile-time specialisation G = 11
bool geometry_11(const Params& p) { return p.W == 11 && p.H == 11 && p.S == 11 && p.margin == 1; }

bool wide_view(const Params& p) {
  return !small_view(p) && p.W <= 31 && p.H <= 32 && (p.S == 16 || p.S == 32) && p.S >= p.H &&
         !p.restrict_view && wab::wide_layout(p).total * 4u <= 64u * 1024u &&
         wab::wide_roll_layout(p).total * 4u <= 64u * 1024u;
}

// the wide kernel holds kWideRegSlots wolves per env in registers whatever wolf_slots is; a lane
// with more works on the rest (rows kWideRegSlots..wolf_slots-1) from HBM (a rare path)
constexpr int kWideRegSlots = 8;
template <int MODE>
void* wide_kernel_ptr(int) {
  return reinterpret_cast<void*>(&wab::wab_step_wide<MODE, kWideRegSlots>);
}

// the wide rollout build: C3's geometry (31 x 31 in 32-byte rows) has an instance with it as
// constants (wab_rollout_wide<.., 31>), any other the generic one
bool wide_fixed31(const Params& p) {
  return p.W == 31 && p.H == 31 && p.S == 32 && p.cw == 15 && p.ch == 15 && p.OB == 3 * 31 * 32 && p.WH == 961 &&
         p.SL == 31;
}
void* wide_roll_kernel(const Params& p) {
  return wide_fixed31(p) ? reinterpret_cast<void*>(&wab::wab_rollout_wide<kWideRegSlots, 31>)
                         : reinterpret_cast<void*>(&wab::wab_rollout_wide<kWideRegSlots, 0>);
}
void launch_rollout_wide(int n_blocks, size_t lds, const Params& p, hipStream_t stream) {
  if (wide_fixed31(p))
    hipLaunchKernelGGL((wab::wab_rollout_wide<kWideRegSlots, 31>), dim3(n_blocks), dim3(256), lds, stream, p);
  else
    hipLaunchKernelGGL((wab::wab_rollout_wide<kWideRegSlots, 0>), dim3(n_blocks), dim3(256), lds, stream, p);
}

template <int G, bool ROLL = false>
void* small_kernel_ptr(int slots) {
  switch (slots) {
    case 8: return reinterpret_cast<void*>(&wab::wab_step_small<8, G, false, ROLL>);
    case 16: return reinterpret_cast<void*>(&wab::wab_step_small<16, G, false, ROLL>);
    default: return reinterpret_cast<void*>(&wab::wab_step_small<32, G, false, ROLL>);
  }
}

// ROLL: the multi-step build (Params::n_steps steps per launch, wab_rollout)
template <int G, bool FEAT = false, bool ROLL = false>
void launch_small(wab_handle* h, const Params& p, hipStream_t stream, size_t lds_bytes = 0) {
  const dim3 grid(h->n_blocks), block(256);  // one 64-env group per workgroup, four waves
  const size_t lds = lds_bytes ? lds_bytes : FEAT ? h->small_feat_lds_bytes : h->small_lds_bytes;
  switch (h->slots) {
    case 8: hipLaunchKernelGGL((wab::wab_step_small<8, G, FEAT, ROLL>), grid, block, lds, stream, p); break;
    case 16: hipLaunchKernelGGL((wab::wab_step_small<16, G, FEAT, ROLL>), grid, block, lds, stream, p); break;
    default: hipLaunchKernelGGL((wab::wab_step_small<32, G, FEAT, ROLL>), grid, block, lds, stream, p); break;
  }
}

template <int MODE>
int launch(wab_handle* h, const Params& p, hipStream_t stream) {
  if (h->n_blocks == 0) return WAB_OK;
  if (h->step_kernel == KERNEL_WIDE) {
    const dim3 grid(h->n_blocks), block(256);  // one 64-env group per workgroup, four waves
    const size_t lds = h->wide_lds_bytes;
    hipLaunchKernelGGL((wab::wab_step_wide<MODE, kWideRegSlots>), grid, block, lds, stream, p);
  } else if (MODE == 0 && h->step_kernel == KERNEL_SMALL) {
    if (p.n_steps > 1) {
      if (h->small_g11) launch_small<11, false, true>(h, p, stream);
      else launch_small<0, false, true>(h, p, stream);
    } else if (h->small_g11) {
      launch_small<11>(h, p, stream);
    } else {
      launch_small<0>(h, p, stream);
    }
  } else if (small_map(p)) launch_as<MODE, true>(h, p, stream);
  else launch_as<MODE, false>(h, p, stream);
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}

// wab_debug_bush_values: the step kernels' bush value (bush_value_fast over the padded LDS
// table) of arbitrary draws
__global__ __launch_bounds__(256) void bush_values_kernel(const uint64_t* thresholds, int n_thr, float power,
                                                          const uint64_t* U, int32_t* out, int64_t n) {
  __shared__ uint64_t tab[256 + 4];
  uint64_t* thr = tab + 1;
  for (int k = threadIdx.x; k < n_thr; k += 256) thr[k] = thresholds[k];
  if (threadIdx.x == 0) wab::bush_thr_pads(thr, n_thr);
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = wab::bush_value_fast(thr, n_thr, U[i], power);
}

// "U >= T" with U = hi << 21 | lo21 becomes (hi, lo21) >= (th, tl); T >= 2^53 never holds
void split_threshold(uint64_t T, uint32_t* th, uint32_t* tl) {
  if (T >= (1ull << 53)) {
    *th = 0xFFFFFFFFu;
    *tl = 0xFFFFFFFFu;
  } else {
    *th = (uint32_t)(T >> 21);
    *tl = (uint32_t)(T & 0x1FFFFFu);
  }
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

// flattened PragmaticObsWrapper length, or WAB_E_INVALID when bushes[md//2, md//2] (wab_env.py:742)
// is outside the grid
int feature_dim_of(const Params& p) {
  const int md = p.W / 2 + p.H / 2 + 1;
  if (md / 2 >= p.W || md / 2 >= p.H) return WAB_E_INVALID;
  return wab::pragmatic_dim(md, p.turns_empty);
}

// the table-driven featurizer (wab_feat.h) applies: planes of <= 128 cells in unpadded rows, and
// every cell's distance from the centre row H//2 / column W//2 (wab_env.py:779-780) below md
// (always on square views; non-square ones can reach md, beyond the tables' rings)
bool feat_small_ok(const Params& p) {
  const int md = p.W / 2 + p.H / 2 + 1;
  int max_dist = 0;
  for (int r = 0; r < p.W; ++r)
    for (int c = 0; c < p.H; ++c) max_dist = std::max(max_dist, std::abs(r - p.H / 2) + std::abs(c - p.W / 2));
  return p.W * p.H <= 128 && p.S == p.H && max_dist < md;
}

// the discounted-return scan: VEC envs per thread, the widest whose grid still gives each of
// the 1024 SIMDs a 64-thread wave and whose rows stay aligned; the reward table reduced to the
// entries whose float32 is not the double itself (the others convert exactly)
int launch_returns(const float* reward, const uint8_t* done, int32_t T, int64_t B, double gamma,
                   const float* bootstrap, float* returns, const wab::RewardTable& tab, void* stream) {
  wab::RewardTable inexact;
  std::memset(&inexact, 0, sizeof(inexact));
  for (int k = 0; k < tab.n; ++k) {
    float f;
    std::memcpy(&f, &tab.f32[k], 4);
    if ((double)f != tab.f64[k]) {
      inexact.f32[inexact.n] = tab.f32[k];
      inexact.f64[inexact.n] = tab.f64[k];
      inexact.n++;
    }
  }
  const auto fits = [&](int v) {
    const uintptr_t a = 4u * (uintptr_t)v - 1u;
    return B % v == 0 && B / v >= 64 * 1024 && ((uintptr_t)reward & a) == 0 && ((uintptr_t)returns & a) == 0 &&
           ((uintptr_t)done & (uintptr_t)(v - 1)) == 0;
  };
  const int vec = fits(4) ? 4 : fits(2) ? 2 : 1;
  const int ne = inexact.n <= 4 ? inexact.n : 8;
  for (int k = inexact.n; k < ne; ++k) {  // pads: copies of entry 0 (same key, same value)
    inexact.f32[k] = inexact.f32[0];
    inexact.f64[k] = inexact.f64[0];
  }
  const dim3 grid((unsigned)((B / vec + 63) / 64));
  hipStream_t s = (hipStream_t)stream;
#define WAB_RET(V, N) \
  hipLaunchKernelGGL((wab::wab_returns_kernel<V, N>), grid, dim3(64), 0, s, reward, done, T, B, gamma, bootstrap, returns, inexact)
#define WAB_RET_NE(V) \
  switch (ne) {                                                                                                   \
    case 0: WAB_RET(V, 0); break;                                                                                 \
    case 1: WAB_RET(V, 1); break;                                                                                 \
    case 2: WAB_RET(V, 2); break;                                                                                 \
    case 3: WAB_RET(V, 3); break;                                                                                 \
    case 4: WAB_RET(V, 4); break;                                                                                 \
    default: WAB_RET(V, 8);                                                                                       \
  }
  if (vec == 4) { WAB_RET_NE(4) }
  else if (vec == 2) { WAB_RET_NE(2) }
  else { WAB_RET_NE(1) }
#undef WAB_RET_NE
#undef WAB_RET
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}

// a handle-owned [B] obs planes buffer (16-byte aligned), allocated by the first call that needs it
uint8_t* scratch_planes(wab_handle* h) {
  if (!h->scratch_planes) {
    DeviceGuard guard(h->device);
    void* ptr = nullptr;
    const size_t bytes = std::max<size_t>(16, (size_t)h->p.B * (size_t)h->p.OB);
    if (hipMalloc(&ptr, bytes) != hipSuccess) return nullptr;
    h->allocs.push_back(ptr);
    h->scratch_planes = static_cast<uint8_t*>(ptr);
  }
  return h->scratch_planes;
}

int check_obs(const wab_obs* o, const char* what) {
  if (!o || !o->planes || !o->food_turns || !o->role || !o->status)
    return fail(WAB_E_INVALID, std::string(what) + ": every wab_obs pointer must be set");
  if (!aligned16(o->planes)) return fail(WAB_E_INVALID, std::string(what) + ": planes must be 16-byte aligned");
  return WAB_OK;
}

}  // namespace

extern "C" {

int wab_abi_version(void) { return WAB_ABI_VERSION; }

const char* wab_last_error(void) { return g_err.c_str(); }

int wab_num_actions(const wab_config* cfg) { return cfg ? n_actions_of(cfg) : WAB_E_INVALID; }

// generate_n_bush_values (wab_env.py:631-635): value(U) = round_half_even((U 2^-53) ** power * max).
// For each k the smallest U on the 2^53 grid with value >= k, by bisection (the value is
// monotone in U), evaluated with libm pow and rint in the reference's operation order.
int wab_bush_thresholds(double bush_power, int32_t max_berries, uint64_t* out) {
  g_err.clear();
  if (max_berries < 0 || max_berries > 255) return fail(WAB_E_INVALID, "max_berries_per_bush must be in [0, 255]");
  if (!(bush_power >= 0.0) || !std::isfinite(bush_power))
    return fail(WAB_E_INVALID, "bush_power must be a finite number >= 0");
  if (max_berries > 0 && !out) return fail(WAB_E_INVALID, "wab_bush_thresholds: NULL out");
  const double mx = (double)max_berries;
  auto value = [&](int64_t U) {
    volatile double u = (double)U * 0x1p-53;  // exact: U < 2^53
    volatile double pw = std::pow((double)u, bush_power);
    volatile double scaled = pw * mx;
    return std::nearbyint((double)scaled);  // default rounding: half to even, as np.round
  };
  for (int k = 1; k <= max_berries; ++k) {
    int64_t lo = 0, hi = (int64_t)1 << 53;  // value(lo) < k (taken, as by options.py), value(hi) >= k; 2^53 = "never"
    while (hi - lo > 1) {
      const int64_t mid = lo + (hi - lo) / 2;
      if (value(mid) >= (double)k) hi = mid; else lo = mid;
    }
    out[k - 1] = (uint64_t)hi;
  }
  return WAB_OK;
}

int64_t wab_batch(const wab_handle* h) { return h ? h->p.B : 0; }

const char* wab_step_kernel(const wab_handle* h) {
  if (!h) return "";
  return h->step_kernel == KERNEL_SMALL ? "small" : h->step_kernel == KERNEL_WIDE ? "wide" : "block";
}

int wab_set_obs_placement(wab_handle* h, int32_t placement) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_set_obs_placement: NULL handle");
  if (placement != WAB_OBS_SAME_BUFFER && placement != WAB_OBS_FRESH_BUFFER)
    return fail(WAB_E_INVALID, "wab_set_obs_placement: WAB_OBS_SAME_BUFFER or WAB_OBS_FRESH_BUFFER");
  h->obs_placement = placement;
  return WAB_OK;
}

int wab_create(const wab_config* c, int64_t batch, uint64_t seed, int64_t env_id_base, int device,
               wab_handle** out) {
  g_err.clear();
  if (!c || !out) return fail(WAB_E_INVALID, "wab_create: NULL argument");
  *out = nullptr;
  // --- validation (wab_env.py:147-148 and the limits of this implementation)
  if (c->width % 2 == 0 || c->height % 2 == 0)
    return fail(WAB_E_INVALID, "width and height must be odd numbers");
  if (c->width < 1 || c->height < 1 || c->width > WAB_MAX_VIEW || c->height > WAB_MAX_VIEW)
    return fail(WAB_E_INVALID, "width/height out of range [1, 63]");
  if (c->restrict_view && (c->width < 11 || c->height < 11))
    return fail(WAB_E_INVALID, "restrict_view needs width, height >= 11 (11x11 masks, wab_env.py:354)");
  if (c->max_berries_per_bush < 0 || c->max_berries_per_bush > 255)
    return fail(WAB_E_INVALID, "max_berries_per_bush must be in [0, 255]");
  if (!(c->bush_power >= 0.0) || !std::isfinite(c->bush_power))
    return fail(WAB_E_INVALID, "bush_power must be a finite number >= 0");
  if (c->turns_to_fill_food <= 0 || c->turns_to_empty_food <= 0)
    return fail(WAB_E_INVALID, "turns_to_fill_food / turns_to_empty_food must be > 0");
  if (c->turns_to_empty_food > 255) return fail(WAB_E_INVALID, "turns_to_empty_food must be <= 255 (u8 obs)");
  if (c->wolf_spawn_margin < 0 || c->width / 2 + c->wolf_spawn_margin > 120 ||
      c->height / 2 + c->wolf_spawn_margin > 120)
    return fail(WAB_E_INVALID, "wolf_spawn_margin out of range");
  const int slots = c->wolf_slots == 0 ? 8 : c->wolf_slots;
  if (slots != 8 && slots != 16 && slots != 32) return fail(WAB_E_INVALID, "wolf_slots must be 8, 16 or 32");
  const int S = c->plane_stride > 0 ? c->plane_stride : c->height;
  if (S < c->height || S > 64) return fail(WAB_E_INVALID, "plane_stride must be in [height, 64]");
  const int cap = c->eaten_capacity > 0 ? c->eaten_capacity
                                        : (c->max_turns < 1 ? 1 : (c->max_turns > 255 ? 255 : c->max_turns));
  if (cap > 255) return fail(WAB_E_INVALID, "eaten_capacity must be <= 255");
  if (batch < 0) return fail(WAB_E_INVALID, "batch must be >= 0");

  wab_handle* h = new wab_handle();
  Params& p = h->p;
  std::memset(&p, 0, sizeof(p));
  p.W = c->width;
  p.H = c->height;
  p.S = S;
  p.cw = c->width / 2;
  p.ch = c->height / 2;
  p.margin = c->wolves ? c->wolf_spawn_margin : 0;
  p.OB = 3 * p.W * p.S;
  p.WH = p.W * p.H;
  p.R = (p.W + 2 * p.margin) * (p.H + 2 * p.margin) - p.WH;
  p.NT = p.WH + p.R;
  p.RW = (p.R + 31) / 32;
  p.WHW = (p.WH + 31) / 32;
  p.SL = p.W > p.H ? p.W : p.H;
  p.magic_OB = (uint32_t)((1ull << 32) / (uint64_t)p.OB) + 1u;
  p.magic_CPE = p.OB >= 16 ? (uint32_t)((1ull << 32) / (uint64_t)(p.OB / 16)) + 1u : 1u;
  p.n_actions = n_actions_of(c);
  for (int a = 0; a < 6; ++a) p.act_role[a] = -1;  // moves: wab::decode_action (up right down left)
  if (c->gatherer_only) p.act_role[4] = 1;       // wab_env.py:149-159
  else if (c->lookout_only) p.act_role[4] = 0;   // :160-170
  else { p.act_role[4] = 1; p.act_role[5] = 0; } // :171-182
  // thresholds on the 53-bit draw U (u = U * 2^-53), each as a ">= T" test
  const uint64_t keep_ge = (uint64_t)std::floor(std::ldexp(c->wolf_chance_to_despawn, 53)) + 1;  // u > p (:263)
  const uint64_t spawn_ge = (uint64_t)std::ceil(std::ldexp(c->chance_wolf_on_square / 2.0, 53));  // u < p/2 (:573)
  p.max_berries = c->max_berries_per_bush;
  p.bush_power = (float)c->bush_power;
  // the caller's table (the Python host computes it with numpy), or the same table from libm
  std::vector<uint64_t> thr_own;
  const uint64_t* thr_host = c->bush_thresholds;
  if (p.max_berries > 0 && !thr_host) {
    thr_own.resize((size_t)p.max_berries);
    wab_bush_thresholds(c->bush_power, p.max_berries, thr_own.data());
    thr_host = thr_own.data();
  }
  const uint64_t bush_ge = p.max_berries > 0 ? thr_host[0] : (1ull << 53);          // food > 0
  split_threshold(keep_ge, &p.keep_th, &p.keep_tl);
  split_threshold(bush_ge, &p.bush_th, &p.bush_tl);
  // keyed spawn sets (oracle/keyed_rng.py gap_thresholds): gap[g] = floor((1 - q)^g 2^53),
  // the power a running product in double (1 - q exact), so the oracle gets the same table
  p.n_gap = wab::kGapChunk;
  std::vector<uint64_t> gap_host((size_t)p.n_gap + 1);
  {
    const double omq = std::ldexp((double)((1ull << 53) - spawn_ge), -53);
    double q = 1.0;
    gap_host[0] = 1ull << 53;
    for (int g = 1; g <= p.n_gap; ++g) {
      q = q * omq;
      gap_host[(size_t)g] = (uint64_t)std::floor(std::ldexp(q, 53));
    }
    p.gap_inv_l2 = spawn_ge > 0 ? (float)(1.0 / std::log2(omq)) : 0.0f;
    auto last_chunk = [](int n) { return n > 0 ? (n - 1) % wab::kGapChunk + 1 : 0; };
    split_threshold(gap_host[(size_t)wab::kGapChunk], &p.gap_full_th, &p.gap_full_tl);
    split_threshold(gap_host[(size_t)last_chunk(p.R)], &p.gap_ring_th, &p.gap_ring_tl);
    split_threshold(gap_host[(size_t)last_chunk(p.WH)], &p.gap_view_th, &p.gap_view_tl);
  }
  p.fill = 1.0 / (double)c->turns_to_fill_food;
  p.hunger = 1.0 / (double)c->turns_to_empty_food;
  p.r_turn = c->reward_per_turn;
  p.r_killed = c->reward_for_being_killed;
  p.r_starve = c->reward_for_starving;
  p.r_finish = c->reward_for_finishing;
  p.r_eat = c->reward_for_eating;
  {  // the step's possible rewards, accumulated from 0 as wab_env.py:251-340 does
    wab::RewardTable& t = h->rewards;
    t.n = 0;
    const double rx[4] = {p.r_turn, p.r_finish, p.r_starve, p.r_killed};
    bool ok = true;
    for (int k = 0; k < 4 && ok; ++k)
      for (int eat = 0; eat < 2 && ok; ++eat) {
        const double d = eat ? (0.0 + p.r_eat) + rx[k] : 0.0 + rx[k];
        const float f = (float)d;
        uint32_t fb;
        std::memcpy(&fb, &f, 4);
        bool dup = false;
        for (int i = 0; i < t.n; ++i)
          if (t.f32[i] == fb) {
            dup = true;
            if (t.f64[i] != d) ok = false;  // two doubles, one float32: not recoverable
          }
        if (!dup) { t.f32[t.n] = fb; t.f64[t.n] = d; t.n++; }
      }
    if (!ok) t.n = -1;
  }
  p.start_food = c->starting_food;
  p.start_role = c->starting_role;
  p.start_food_random = c->starting_food_random;
  p.start_role_random = c->starting_role_random;
  p.max_turns = c->max_turns;
  p.turns_empty = c->turns_to_empty_food;
  p.lookout_only = c->lookout_only;
  p.restrict_view = c->restrict_view;
  p.wolves_on = c->wolves;
  p.wolves_can_move = c->wolves_can_move;
  p.god_mode = c->god_mode;
  p.autoreset = c->autoreset;
  for (int i = 0; i < 11; ++i) {
    p.mask_rows[0][i] = row_mask(kLookout[i]);
    p.mask_rows[1][i] = row_mask(kGatherer[i]);
  }
  for (int c = 0; c < p.WH && c < 128; ++c) {  // bitmap masks for W*H <= 128 (bit c = i*H + j)
    const int j = c % p.H;
    p.small_masks[2][c >> 5] |= 1u << (c & 31);
    if (j == 0) p.small_masks[0][c >> 5] |= 1u << (c & 31);
    if (j == p.H - 1) p.small_masks[1][c >> 5] |= 1u << (c & 31);
  }
  if (p.W == 11 && p.H == 11)
    for (int r = 0; r < 2; ++r)
      for (int i = 0; i < 11; ++i)
        for (int j = 0; j < 11; ++j)
          if ((p.mask_rows[r][i] >> j) & 1u) p.view121[r][(i * 11 + j) >> 5] |= 1u << ((i * 11 + j) & 31);
  p.seed = seed;
  p.env_base = env_id_base;
  p.B = batch;
  p.eaten_cap = cap;
  h->device = device;
  h->slots = slots;
  p.wolf_cap = slots;
  p.n_steps = 1;
  h->n_blocks = (int)((batch + wab::kEnvsPerBlock - 1) / wab::kEnvsPerBlock);
  h->lds_bytes = (size_t)wab::lds_layout(p, slots).total * 4u;
  {
    h->step_kernel = small_view(p) ? KERNEL_SMALL : wide_view(p) ? KERNEL_WIDE : KERNEL_BLOCK;
    h->small_lds_bytes = (size_t)wab::small_layout(p).total * 4u;
    // wab_step_features fuses the featurizer into the small kernel when the table-driven
    // featurizer applies (see featurize): every cell within md of the centre row/column
    if (h->step_kernel == KERNEL_SMALL && feature_dim_of(p) >= 0 && feat_small_ok(p)) {
      Params q = p;
      q.features = reinterpret_cast<float*>(16);  // (layout only)
      h->small_feat_lds_bytes = (size_t)wab::small_layout(q).total * 4u;
    }
    h->small_g11 = geometry_11(p);
  }
  if (h->lds_bytes > 160u * 1024u) {
    delete h;
    return fail(WAB_E_INVALID, "viewport too large for the fused kernel's LDS budget");
  }

  DeviceGuard guard(device);
  auto alloc = [&](void** ptr, size_t bytes) -> int {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(ptr, bytes);
    if (e != hipSuccess) return fail(WAB_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    h->allocs.push_back(*ptr);
    return WAB_OK;
  };
  const size_t B = (size_t)batch;
  int rc = WAB_OK;
  rc |= alloc((void**)&p.hdr, B * 16);
  rc |= alloc((void**)&p.food, B * 8);
  rc |= alloc((void**)&p.wolves, B * 4 * (size_t)slots);
  rc |= alloc((void**)&p.eaten_xy, B * 4 * (size_t)cap);
  rc |= alloc((void**)&p.eaten_rem, B * (size_t)cap);
  rc |= alloc((void**)&p.bushmap, B * 4 * (size_t)(p.W <= 32 && p.WHW < 32 ? 32 : p.WHW));  // (wide: 32 per env)
  rc |= alloc((void**)&p.counters, wab::kNumCounters * 8);
  rc |= alloc((void**)&p.block_resets, (size_t)(h->n_blocks > 0 ? h->n_blocks : 1) * 8);
  uint64_t* thr = nullptr;
  rc |= alloc((void**)&thr, (size_t)(p.max_berries > 0 ? p.max_berries : 1) * 8);
  uint64_t* gap = nullptr;
  rc |= alloc((void**)&gap, gap_host.size() * 8);
  uint32_t* tab = nullptr;
  p.ring_at = (p.WH + 3) & ~3;
  const int n_tab = p.ring_at + ((p.R + 3) & ~3) + 4;  // + the kernel's one-ahead prefetch
  rc |= alloc((void**)&tab, (size_t)n_tab * 4);
  if (rc != WAB_OK) {
    std::string msg = g_err;
    wab_destroy(h);
    return fail(WAB_E_NOMEM, msg);
  }
  p.thresholds = thr;
  p.gap = gap;
  p.tables = tab;
  hipError_t e = hipSuccess;
  {  // view-cell offsets (cw - i, ch - j) for cell i*H + j, then the spawn-ring offsets
    std::vector<uint32_t> t((size_t)n_tab, 0u);
    for (int c = 0; c < p.WH; ++c) t[c] = wab::xy_pack(p.cw - c / p.H, p.ch - c % p.H);
    const int m = p.margin, Wm = p.W + 2 * m;
    for (int r = 0; r < p.R; ++r) {
      int xi, yi;
      if (r < 2 * m * Wm) {
        const int band = r / Wm;
        xi = r % Wm;
        yi = band < m ? band : band + p.H;
      } else {
        const int r2 = r - 2 * m * Wm, band = r2 / p.H;
        yi = m + r2 % p.H;
        xi = band < m ? band : band + p.W;
      }
      t[p.ring_at + r] = wab::xy_pack(xi - p.cw - m, yi - p.ch - m);
    }
    e = hipMemcpy(tab, t.data(), t.size() * 4, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemcpy(gap, gap_host.data(), gap_host.size() * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess && p.max_berries > 0)
    e = hipMemcpy(thr, thr_host, (size_t)p.max_berries * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess && B > 0) {  // every env: episode 0xFFFFFFFF (the first reset makes it 0)
    std::vector<uint4> init(B, make_uint4(0u, 0u, 0u, 0xFFFFFFFFu));
    e = hipMemcpy(p.hdr, init.data(), B * 16, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemset(p.counters, 0, wab::kNumCounters * 8);
  if (e == hipSuccess) e = hipMemset(p.block_resets, 0, (size_t)(h->n_blocks > 0 ? h->n_blocks : 1) * 8);
  for (void* k : {kernel_ptr<0, true>(slots), kernel_ptr<1, true>(slots), kernel_ptr<0, false>(slots),
                  kernel_ptr<1, false>(slots)})
    if (e == hipSuccess)
      e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_bytes);
  if (h->step_kernel == KERNEL_WIDE) {
    h->wide_lds_bytes = (size_t)wab::wide_layout(p).total * 4u;
    h->wide_roll_lds_bytes = (size_t)wab::wide_roll_layout(p).total * 4u;
    for (void* k : {wide_kernel_ptr<0>(slots), wide_kernel_ptr<1>(slots)})
      if (e == hipSuccess)
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->wide_lds_bytes);
    if (e == hipSuccess)
      e = hipFuncSetAttribute(wide_roll_kernel(p), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)h->wide_roll_lds_bytes);
  }
  if (e == hipSuccess && h->step_kernel == KERNEL_SMALL)
    for (void* k : {h->small_g11 ? small_kernel_ptr<11>(slots) : small_kernel_ptr<0>(slots),
                    h->small_g11 ? small_kernel_ptr<11, true>(slots) : small_kernel_ptr<0, true>(slots)})
      if (e == hipSuccess)
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->small_lds_bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    std::string msg = std::string("wab_create: ") + hipGetErrorString(e);
    wab_destroy(h);
    return fail(WAB_E_HIP, msg);
  }
  *out = h;
  return WAB_OK;
}

int wab_destroy(wab_handle* h) {
  if (!h) return WAB_OK;
  {
    DeviceGuard guard(h->device);
    (void)hipDeviceSynchronize();
    for (void* ptr : h->allocs) (void)hipFree(ptr);
  }
  delete h;
  return WAB_OK;
}

int wab_reset(wab_handle* h, const uint8_t* mask, const wab_obs* obs, void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_reset: NULL handle");
  if (int rc = check_obs(obs, "wab_reset")) return rc;
  if (mask && !h->reset_done)
    return fail(WAB_E_STATE, "wab_reset: the first reset must cover every env (mask = NULL)");
  Params p = h->p;
  p.reset_mask = mask;
  p.planes = obs->planes;
  p.food_turns = obs->food_turns;
  p.role = obs->role;
  p.status = obs->status;
  DeviceGuard guard(h->device);
  int rc = launch<1>(h, p, (hipStream_t)stream);
  if (rc == WAB_OK && !mask) h->reset_done = true;
  return rc;
}


int wab_step(wab_handle* h, const int8_t* actions, const wab_obs* obs, float* reward, uint8_t* done,
             const wab_obs* terminal, void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_step: NULL handle");
  if (!h->reset_done) return fail(WAB_E_STATE, "wab_step: call wab_reset before the first step");
  if (!actions || !reward || !done) return fail(WAB_E_INVALID, "wab_step: NULL actions/reward/done");
  if (int rc = check_obs(obs, "wab_step")) return rc;
  Params p = h->p;
  p.actions = actions;
  p.planes = obs->planes;
  p.food_turns = obs->food_turns;
  p.role = obs->role;
  p.status = obs->status;
  p.reward = reward;
  p.done = done;
  if (terminal && terminal->planes) {
    if (int rc = check_obs(terminal, "wab_step(terminal)")) return rc;
    p.t_planes = terminal->planes;
    p.t_food_turns = terminal->food_turns;
    p.t_role = terminal->role;
    p.t_status = terminal->status;
  }
  DeviceGuard guard(h->device);
  if (h->step_kernel == KERNEL_WIDE && !p.t_planes && h->obs_placement == WAB_OBS_FRESH_BUFFER &&
      ((size_t)p.B * (size_t)p.OB) % 16u == 0) {
    // The wide view, without terminal obs, each step into a buffer the last steps did not write
    // (wab_set_obs_placement(WAB_OBS_FRESH_BUFFER), a closed loop's ring of obs slots): the
    // rollout build with one step (its obs as whole 128-byte lines in address order after the
    // step).  Into one buffer rewritten every step (WAB_OBS_SAME_BUFFER, the env's own, which
    // the 256 MB Infinity Cache holds) the per-step kernel, which stores each plane as soon as it
    // is final (a line at a plane or env boundary in two parts, merged on die).  Measured at
    // B = 65536 (C3): into a 32-slot ring 52.0 against 73.1 us (round 3's per-step kernel), into
    // one buffer 62.5 against 45.9 us.  The results are the same either way.
    if (h->n_blocks == 0) return WAB_OK;
    p.n_steps = 1;
    launch_rollout_wide(h->n_blocks, h->wide_roll_lds_bytes, p, (hipStream_t)stream);
    HIP_TRY(hipGetLastError());
    return WAB_OK;
  }
  return launch<0>(h, p, (hipStream_t)stream);
}

int wab_rollout(wab_handle* h, const int8_t* actions, int32_t T, const wab_obs* obs_seq, float* reward,
                uint8_t* done, void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_rollout: NULL handle");
  if (T < 0) return fail(WAB_E_INVALID, "wab_rollout: T must be >= 0");
  if (int rc = check_obs(obs_seq, "wab_rollout")) return rc;
  const int64_t B = h->p.B;
  const size_t OB = (size_t)h->p.OB;
  const bool wide_roll = h->step_kernel == KERNEL_WIDE;
  if (T > 0 && (h->step_kernel == KERNEL_SMALL || wide_roll) && h->reset_done && actions && reward && done &&
      ((size_t)B * OB) % 16u == 0) {  // (every step's planes 16-byte aligned)
    // one launch: each workgroup runs its 64 envs through the T steps (Params::n_steps)
    Params p = h->p;
    p.actions = actions;
    p.planes = obs_seq->planes;
    p.food_turns = obs_seq->food_turns;
    p.role = obs_seq->role;
    p.status = obs_seq->status;
    p.reward = reward;
    p.done = done;
    p.n_steps = T;
    DeviceGuard guard(h->device);
    ++h->rollout_launches;
    if (h->step_kernel == KERNEL_WIDE) {
      if (h->n_blocks == 0) return WAB_OK;
      launch_rollout_wide(h->n_blocks, h->wide_roll_lds_bytes, p, (hipStream_t)stream);
      HIP_TRY(hipGetLastError());
      return WAB_OK;
    }
    return launch<0>(h, p, (hipStream_t)stream);
  }
  if (T > 0) ++h->rollout_step_calls;
  for (int32_t t = 0; t < T; ++t) {
    wab_obs o;
    uint8_t* dst = obs_seq->planes + (size_t)t * (size_t)B * OB;
    // (a step slice that is not 16-byte aligned, B * OB % 16 != 0: the step writes a handle-owned
    // buffer, copied to the slice on the stream; the first such call allocates it)
    o.planes = aligned16(dst) ? dst : scratch_planes(h);
    if (!o.planes) return fail(WAB_E_NOMEM, "wab_rollout: hipMalloc");
    o.food_turns = obs_seq->food_turns + (size_t)t * (size_t)B;
    o.role = obs_seq->role + (size_t)t * (size_t)B;
    o.status = obs_seq->status + (size_t)t * (size_t)B;
    int rc = wab_step(h, actions + (size_t)t * (size_t)B, &o, reward + (size_t)t * (size_t)B,
                      done + (size_t)t * (size_t)B, nullptr, stream);
    if (rc != WAB_OK) return rc;
    if (o.planes != dst) {
      DeviceGuard guard(h->device);
      HIP_TRY(hipMemcpyAsync(dst, o.planes, (size_t)B * OB, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    }
  }
  return WAB_OK;
}

int wab_get_counters(wab_handle* h, wab_counters* out, void* stream) {
  g_err.clear();
  if (!h || !out) return fail(WAB_E_INVALID, "wab_get_counters: NULL argument");
  DeviceGuard guard(h->device);
  unsigned long long c[wab::kNumCounters] = {};
  std::vector<unsigned long long> br((size_t)(h->n_blocks > 0 ? h->n_blocks : 1));
  HIP_TRY(hipMemcpyAsync(c, h->p.counters, sizeof(c), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipMemcpyAsync(br.data(), h->p.block_resets, br.size() * 8, hipMemcpyDeviceToHost,
                         (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  out->wolf_overflow = c[wab::CTR_WOLF_OVERFLOW];
  out->eaten_overflow = c[wab::CTR_EATEN_OVERFLOW];
  out->bad_actions = c[wab::CTR_BAD_ACTIONS];
  out->ego_missing = c[wab::CTR_EGO_MISSING];
  out->steps = c[wab::CTR_STEPS];
  out->handoff_timeouts = c[wab::CTR_HANDOFF_TIMEOUTS];
  out->wolf_overflow_reset = c[wab::CTR_WOLF_OVERFLOW_RESET];
  out->resets = 0;
  for (size_t i = 0; i < br.size(); ++i) out->resets += br[i];
  out->rollout_launches = h->rollout_launches;
  out->rollout_step_calls = h->rollout_step_calls;
  return WAB_OK;
}

int wab_get_state(wab_handle* h, double* food, int32_t* x, int32_t* y, int32_t* turn, int32_t* n_wolves,
                  uint32_t* episode, void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_get_state: NULL handle");
  DeviceGuard guard(h->device);
  const size_t B = (size_t)h->p.B;
  std::vector<uint4> hdr(B);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(hdr.data(), h->p.hdr, B * 16, hipMemcpyDeviceToHost, s));
  if (food) HIP_TRY(hipMemcpyAsync(food, h->p.food, B * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (size_t i = 0; i < B; ++i) {
    if (x) x[i] = wab::xy_x(hdr[i].x);
    if (y) y[i] = wab::xy_y(hdr[i].x);
    if (turn) turn[i] = (int32_t)hdr[i].y;
    if (n_wolves) n_wolves[i] = (int32_t)wab::misc_nw(hdr[i].z);
    if (episode) episode[i] = hdr[i].w;
  }
  return WAB_OK;
}

int wab_feature_dim(const wab_handle* h) {
  if (!h) return WAB_E_INVALID;
  return feature_dim_of(h->p);
}

namespace {
int featurize(wab_handle* h, int kind, const wab_obs* obs, const uint8_t* view_mask, float* features, void* stream,
              const char* what) {
  g_err.clear();
  if (!h || !features) return fail(WAB_E_INVALID, std::string(what) + ": NULL argument");
  if (int rc = check_obs(obs, what)) return rc;
  const int F = kind == 1 ? wab_superbasic_dim(h) : wab_feature_dim(h);
  if (F < 0) return fail(WAB_E_INVALID, std::string(what) + ": the wrapper cannot index this viewport");
  if ((reinterpret_cast<uintptr_t>(features) & 15u) != 0)
    return fail(WAB_E_INVALID, std::string(what) + ": features must be 16-byte aligned");
  const Params& p = h->p;
  wab::FeatParams fp;
  std::memset(&fp, 0, sizeof(fp));
  fp.W = p.W; fp.H = p.H; fp.S = p.S; fp.OB = p.OB;
  fp.md = p.W / 2 + p.H / 2 + 1;
  fp.F = F;
  fp.turns_empty = p.turns_empty;
  fp.restrict_view = p.restrict_view;
  fp.kind = kind;
  fp.B = p.B;
  std::memcpy(fp.mask_rows, p.mask_rows, sizeof(fp.mask_rows));
  fp.planes = obs->planes;
  fp.food_turns = obs->food_turns;
  fp.role = obs->role;
  fp.status = obs->status;
  fp.view_mask = view_mask;
  fp.out = features;
  for (int r = 0; r < 2; ++r)  // the view mask as 121 cell bits, bit i*11 + j
    for (int i = 0; i < 11; ++i)
      for (int j = 0; j < 11; ++j)
        if ((p.mask_rows[r][i] >> j) & 1u) fp.view121[r][(i * 11 + j) >> 5] |= 1u << ((i * 11 + j) & 31);
  if (h->n_blocks == 0) return WAB_OK;
  DeviceGuard guard(h->device);
  // views whose planes fit 128 bits in unpadded rows: the table-driven kernel
  // (wab_featurize_small_kernel, feat_small_ok); a caller-given view mask or larger views: the
  // general one
  const bool small = feat_small_ok(p) && !view_mask;
  const uint32_t inW = (uint32_t)(64 * p.OB + 31) / 32, outW = (uint32_t)(64 * F + 31) / 32;
  if (small) {
    const uint32_t a = (inW + 4 + 3) & ~3u, b = (outW + 4 + 3) & ~3u;
    const size_t lds = (size_t)(a + b + wab::feat_tables_words(fp.md)) * 4;
    hipLaunchKernelGGL(wab::wab_featurize_small_kernel, dim3(h->n_blocks), dim3(256), lds, (hipStream_t)stream, fp);
    HIP_TRY(hipGetLastError());
    return WAB_OK;
  }
  const size_t lds = (size_t)(((inW + 3) & ~3u) + outW) * 4;
  if (lds > 64 * 1024)
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<void*>(&wab::wab_featurize_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(wab::wab_featurize_kernel, dim3(h->n_blocks), dim3(256), lds, (hipStream_t)stream, fp);
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}
}  // namespace

int wab_featurize(wab_handle* h, const wab_obs* obs, const uint8_t* view_mask, float* features,
                  void* stream) {
  return featurize(h, 0, obs, view_mask, features, stream, "wab_featurize");
}

int wab_step_features(wab_handle* h, const int8_t* actions, const wab_obs* obs, float* reward, uint8_t* done,
                      float* features, void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_step_features: NULL handle");
  if (!h->reset_done) return fail(WAB_E_STATE, "wab_step_features: call wab_reset before the first step");
  if (!actions || !reward || !done || !features || !obs || !obs->food_turns || !obs->role || !obs->status)
    return fail(WAB_E_INVALID, "wab_step_features: NULL argument");
  if (!aligned16(features)) return fail(WAB_E_INVALID, "wab_step_features: features must be 16-byte aligned");
  if (obs->planes && !aligned16(obs->planes))
    return fail(WAB_E_INVALID, "wab_step_features: planes must be 16-byte aligned");
  if (wab_feature_dim(h) < 0) return fail(WAB_E_INVALID, "wab_step_features: the wrapper cannot index this viewport");
  if (!h->small_feat_lds_bytes) {
    // no fused kernel for these options: the step, then the featurizer, on the same stream
    // (without caller planes through a handle-owned buffer, allocated by the first such call)
    wab_obs o = *obs;
    if (!o.planes) {
      o.planes = scratch_planes(h);
      if (!o.planes) return fail(WAB_E_NOMEM, "wab_step_features: hipMalloc");
    }
    if (int rc = wab_step(h, actions, &o, reward, done, nullptr, stream)) return rc;
    return wab_featurize(h, &o, nullptr, features, stream);
  }
  Params p = h->p;
  p.actions = actions;
  p.planes = obs->planes;
  p.food_turns = obs->food_turns;
  p.role = obs->role;
  p.status = obs->status;
  p.reward = reward;
  p.done = done;
  p.features = features;
  if (h->n_blocks == 0) return WAB_OK;
  DeviceGuard guard(h->device);
  if (h->small_g11) launch_small<11, true>(h, p, (hipStream_t)stream);
  else launch_small<0, true>(h, p, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}

int wab_rollout_features(wab_handle* h, const int8_t* actions, int32_t T, const wab_obs* obs_seq, float* reward,
                         uint8_t* done, float* features, double gamma, const float* bootstrap, float* returns,
                         void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_rollout_features: NULL handle");
  if (T < 0) return fail(WAB_E_INVALID, "wab_rollout_features: T must be >= 0");
  if (!h->reset_done) return fail(WAB_E_STATE, "wab_rollout_features: call wab_reset before the first step");
  if (!actions || !reward || !done || !features || !obs_seq || !obs_seq->food_turns || !obs_seq->role ||
      !obs_seq->status)
    return fail(WAB_E_INVALID, "wab_rollout_features: NULL argument");
  const int F = wab_feature_dim(h);
  if (F < 0) return fail(WAB_E_INVALID, "wab_rollout_features: the wrapper cannot index this viewport");
  const int64_t B = h->p.B;
  const size_t OB = (size_t)h->p.OB;
  if (!aligned16(features) || (T > 1 && ((size_t)B * (size_t)F * 4u) % 16u != 0))
    return fail(WAB_E_INVALID, "wab_rollout_features: every step's features must be 16-byte aligned "
                               "(features aligned, batch * feature_dim a multiple of 4)");
  if (obs_seq->planes && !aligned16(obs_seq->planes))
    return fail(WAB_E_INVALID, "wab_rollout_features: planes must be 16-byte aligned");
  if (T == 0 || B == 0) return WAB_OK;
  bool fused_returns = returns && T <= wab::kMaxFusedReturnSteps;
  size_t roll_lds = 0;  // the fused launch's LDS (its reward codes grow with T)
  if (h->small_feat_lds_bytes && h->step_kernel == KERNEL_SMALL) {
    Params q = h->p;
    q.features = features;
    q.n_steps = T;
    q.returns = fused_returns ? returns : nullptr;
    roll_lds = (size_t)wab::small_layout(q).total * 4u;
    if (roll_lds > 64u * 1024u) roll_lds = 0;  // (T steps of the per-step fused launch instead)
    if (obs_seq->planes && ((size_t)B * OB) % 16u != 0) roll_lds = 0;  // (its 16-byte obs stores)
  }
  if (returns && !(roll_lds && fused_returns) && h->rewards.n < 0)  // (checked before anything runs)
    return fail(WAB_E_INVALID, "wab_rollout_features: returns of this segment need the exact-reward scan, and "
                               "two of the options' rewards round to the same float32 (pass returns = NULL)");
  if (roll_lds) {
    // one launch: each workgroup runs its 64 envs through the T steps with the featurizer fused
    // (wab_step_small<.., FEAT, ROLL>), the returns of the segment at its end
    Params p = h->p;
    p.actions = actions;
    p.planes = obs_seq->planes;
    p.food_turns = obs_seq->food_turns;
    p.role = obs_seq->role;
    p.status = obs_seq->status;
    p.reward = reward;
    p.done = done;
    p.features = features;
    p.n_steps = T;
    if (fused_returns) {
      p.returns = returns;
      p.bootstrap = bootstrap;
      p.gamma = gamma;
    }
    DeviceGuard guard(h->device);
    ++h->rollout_launches;
    if (h->small_g11) launch_small<11, true, true>(h, p, (hipStream_t)stream, roll_lds);
    else launch_small<0, true, true>(h, p, (hipStream_t)stream, roll_lds);
    HIP_TRY(hipGetLastError());
    if (fused_returns) return WAB_OK;
  } else {
    ++h->rollout_step_calls;
    for (int32_t t = 0; t < T; ++t) {  // (no fused kernel for these options: T fused-or-not steps)
      wab_obs o;
      o.planes = obs_seq->planes ? obs_seq->planes + (size_t)t * (size_t)B * OB : nullptr;
      uint8_t* dst = o.planes;
      if (dst && !aligned16(dst)) {  // (as in wab_rollout: through the handle's buffer)
        o.planes = scratch_planes(h);
        if (!o.planes) return fail(WAB_E_NOMEM, "wab_rollout_features: hipMalloc");
      }
      o.food_turns = obs_seq->food_turns + (size_t)t * (size_t)B;
      o.role = obs_seq->role + (size_t)t * (size_t)B;
      o.status = obs_seq->status + (size_t)t * (size_t)B;
      int rc = wab_step_features(h, actions + (size_t)t * (size_t)B, &o, reward + (size_t)t * (size_t)B,
                                 done + (size_t)t * (size_t)B, features + (size_t)t * (size_t)B * (size_t)F,
                                 stream);
      if (rc != WAB_OK) return rc;
      if (dst && o.planes != dst) {
        DeviceGuard guard(h->device);
        HIP_TRY(hipMemcpyAsync(dst, o.planes, (size_t)B * OB, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      }
    }
  }
  if (!returns) return WAB_OK;
  return wab_discounted_returns_exact(h, reward, done, T, B, gamma, bootstrap, returns, stream);
}

int wab_superbasic_dim(const wab_handle* h) {
  if (!h) return WAB_E_INVALID;
  const Params& p = h->p;
  return 4 * (p.W / 2 + p.H / 2 + 1) + (p.turns_empty + 1) + 2 + 3;
}

int wab_featurize_superbasic(wab_handle* h, const wab_obs* obs, float* features, void* stream) {
  return featurize(h, 1, obs, nullptr, features, stream, "wab_featurize_superbasic");
}

int wab_render(wab_handle* h, const wab_obs* obs, int32_t scale, int32_t draw_health, uint8_t* rgb, void* stream) {
  g_err.clear();
  if (!h) return fail(WAB_E_INVALID, "wab_render: NULL argument");
  return wab_render_envs(h, obs, 0, h->p.B, scale, draw_health, rgb, stream);
}

int wab_render_envs(wab_handle* h, const wab_obs* obs, int64_t first, int64_t count, int32_t scale,
                    int32_t draw_health, uint8_t* rgb, void* stream) {
  g_err.clear();
  if (!h || !rgb) return fail(WAB_E_INVALID, "wab_render: NULL argument");
  if (int rc = check_obs(obs, "wab_render")) return rc;
  if (scale < 1 || scale > 256) return fail(WAB_E_INVALID, "wab_render: scale must be in [1, 256]");
  if (first < 0 || count < 0 || first > h->p.B || count > h->p.B - first)
    return fail(WAB_E_INVALID, "wab_render_envs: [first, first + count) must lie in [0, B)");
  const Params& p = h->p;
  if ((uint64_t)p.W * scale * p.H * scale * 3 >= (1ull << 32))
    return fail(WAB_E_INVALID, "wab_render: image too large");
  wab::RenderParams rp;
  std::memset(&rp, 0, sizeof(rp));
  rp.W = p.W; rp.H = p.H; rp.S = p.S; rp.OB = p.OB;
  rp.scale = scale;
  rp.restrict_view = p.restrict_view;
  rp.draw_health = draw_health != 0;
  rp.B = count;
  std::memcpy(rp.mask_rows, p.mask_rows, sizeof(rp.mask_rows));
  rp.planes = obs->planes + (size_t)first * p.OB;
  rp.food_turns = obs->food_turns + first;
  rp.role = obs->role + first;
  rp.status = obs->status + first;
  rp.rgb = rgb;
  if (count == 0) return WAB_OK;
  const uint64_t per_env = (uint64_t)p.W * scale * p.H * scale * 3;
  const uint64_t words = (per_env + 3) / 4;
  const unsigned gx = (unsigned)std::min<uint64_t>((words + 255) / 256, 1024);
  DeviceGuard guard(h->device);
  for (int64_t e0 = 0; e0 < count; e0 += 65535) {  // grid.y is at most 65535 envs per launch
    wab::RenderParams r2 = rp;
    r2.planes = rp.planes + (size_t)e0 * p.OB;
    r2.food_turns = rp.food_turns + e0;
    r2.role = rp.role + e0;
    r2.status = rp.status + e0;
    r2.rgb = rp.rgb + (size_t)e0 * per_env;
    r2.B = std::min<int64_t>(65535, count - e0);
    hipLaunchKernelGGL(wab::wab_render_kernel, dim3(gx, (unsigned)r2.B), dim3(256), 0, (hipStream_t)stream, r2);
  }
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}

int wab_egocentric(wab_handle* h, const uint8_t* mask, uint8_t* proximity, void* stream) {
  g_err.clear();
  if (!h || !proximity) return fail(WAB_E_INVALID, "wab_egocentric: NULL argument");
  if (!h->reset_done) return fail(WAB_E_STATE, "wab_egocentric: reset the handle first");
  const Params& p = h->p;
  const int Q = p.cw + p.ch + 1;
  if (Q > 31) return fail(WAB_E_INVALID, "wab_egocentric: width//2 + height//2 must be <= 30");
  DeviceGuard guard(h->device);
  if (!h->ego_path) {
    const int cap = p.max_turns + 129;  // + stepping on after done without a reset
    std::vector<uint32_t> dia;
    for (int dy = -Q; dy <= Q; ++dy)
      for (int dx = -Q; dx <= Q; ++dx)
        if (std::abs(dx) + std::abs(dy) <= Q) dia.push_back(((uint32_t)dx & 0xFFu) | (((uint32_t)dy & 0xFFu) << 8));
    void* path = nullptr;
    void* d = nullptr;
    const size_t path_bytes = (size_t)cap * (size_t)(p.B > 0 ? p.B : 1) * 16;
    if (hipMalloc(&path, path_bytes) != hipSuccess) return fail(WAB_E_NOMEM, "wab_egocentric: hipMalloc");
    h->allocs.push_back(path);
    if (hipMalloc(&d, dia.size() * 4) != hipSuccess) return fail(WAB_E_NOMEM, "wab_egocentric: hipMalloc");
    h->allocs.push_back(d);
    HIP_TRY(hipMemcpy(d, dia.data(), dia.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(path, 0xFF, path_bytes, (hipStream_t)stream));  // episode 0xFFFFFFFF: unset
    h->ego_path = (uint4*)path;
    h->ego_diamond = (uint32_t*)d;
    h->ego_cap = cap;
    h->ego_n_diamond = (int)dia.size();
  }
  if (p.B == 0) return WAB_OK;
  wab::EgoParams ep;
  std::memset(&ep, 0, sizeof(ep));
  ep.cw = p.cw; ep.ch = p.ch; ep.Q = Q;
  ep.cap = h->ego_cap;
  ep.n_diamond = h->ego_n_diamond;
  ep.eaten_cap = p.eaten_cap;
  ep.bush_th = p.bush_th; ep.bush_tl = p.bush_tl;
  ep.seed = p.seed; ep.env_base = p.env_base; ep.B = p.B;
  ep.hdr = p.hdr; ep.eaten_xy = p.eaten_xy; ep.eaten_rem = p.eaten_rem;
  ep.diamond = h->ego_diamond;
  ep.path = h->ego_path;
  ep.mask = mask;
  ep.out = proximity;
  ep.counters = p.counters;
  hipLaunchKernelGGL(wab::wab_egocentric_kernel, dim3((unsigned)p.B), dim3(64), 0, (hipStream_t)stream, ep);
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}

int wab_discounted_returns(const float* reward, const uint8_t* done, int32_t T, int64_t B, double gamma,
                           const float* bootstrap, float* returns, void* stream) {
  g_err.clear();
  if (!reward || !done || !returns || T < 0 || B < 0)
    return fail(WAB_E_INVALID, "wab_discounted_returns: bad argument");
  if (T == 0 || B == 0) return WAB_OK;
  wab::RewardTable none;
  std::memset(&none, 0, sizeof(none));
  return launch_returns(reward, done, T, B, gamma, bootstrap, returns, none, stream);
}

int wab_discounted_returns_exact(const wab_handle* h, const float* reward, const uint8_t* done, int32_t T,
                                 int64_t B, double gamma, const float* bootstrap, float* returns, void* stream) {
  g_err.clear();
  if (!h || !reward || !done || !returns || T < 0 || B < 0)
    return fail(WAB_E_INVALID, "wab_discounted_returns_exact: bad argument");
  if (h->rewards.n < 0)
    return fail(WAB_E_INVALID, "wab_discounted_returns_exact: two of the options' rewards round to the same "
                               "float32; the double rewards are not recoverable");
  if (T == 0 || B == 0) return WAB_OK;
  DeviceGuard guard(h->device);
  return launch_returns(reward, done, T, B, gamma, bootstrap, returns, h->rewards, stream);
}

int wab_debug_bush_values(wab_handle* h, const uint64_t* U, int32_t* out, int64_t n, void* stream) {
  g_err.clear();
  if (!h || !U || !out || n < 0) return fail(WAB_E_INVALID, "wab_debug_bush_values: bad argument");
  if (n == 0) return WAB_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(bush_values_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, h->p.thresholds,
                     h->p.max_berries, h->p.bush_power, U, out, n);
  HIP_TRY(hipGetLastError());
  return WAB_OK;
}

#ifdef WAB_STAMPS
// diagnostic build only: per-block phase timestamps (see wab_step.hip, WAB_STAMP)
int wab_debug_set_stamps(wab_handle* h, unsigned long long* dev) {
  if (!h) return WAB_E_INVALID;
  h->p.stamps = dev;
  return WAB_OK;
}
#endif

}  // extern "C"
