// A C-ABI caller with no Python in the process: builds wab_config from the reference's
// default_game_options (wab_env.py:11-39) with bush_thresholds = NULL (wab_create then computes
// the table itself, wab_bush_thresholds), resets B envs, steps them T times with host-chosen
// actions and writes what it saw to a file:
//   actions [T][B] i8, reward [T][B] f32, done [T][B] u8, final planes [B][3][11][11] u8,
//   final food_turns / role / status [B] u8 each.
// tests/test_gpu_capi_demo.py replays the same actions through the Python host and compares.
//   usage: c_api_demo B T seed out.bin
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/wab.h"

#define CHECK_WAB(x)                                                          \
  do {                                                                        \
    if ((x) != WAB_OK) {                                                      \
      std::fprintf(stderr, "%s failed: %s\n", #x, wab_last_error());          \
      return 1;                                                               \
    }                                                                         \
  } while (0)
#define CHECK_HIP(x)                                                          \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  if (argc != 5) {
    std::fprintf(stderr, "usage: %s B T seed out.bin\n", argv[0]);
    return 2;
  }
  const int64_t B = std::atoll(argv[1]);
  const int T = std::atoi(argv[2]);
  const uint64_t seed = std::strtoull(argv[3], nullptr, 0);
  if (B <= 0 || T <= 0) return 2;

  wab_config c = {};  // default_game_options (wab_env.py:11-39)
  c.reward_per_turn = 0;
  c.reward_for_being_killed = -1;
  c.reward_for_starving = -1;
  c.reward_for_finishing = 1;
  c.reward_for_eating = 0.1;
  c.gatherer_only = 0;
  c.lookout_only = 1;
  c.restrict_view = 0;
  c.starting_role = 1;
  c.starting_food = 1.0;
  c.max_turns = 80;
  c.height = 11;
  c.width = 11;
  c.max_berries_per_bush = 200;
  c.bush_power = 100;
  c.turns_to_fill_food = 8;
  c.turns_to_empty_food = 40;
  c.wolf_spawn_margin = 1;
  c.chance_wolf_on_square = 0.001;
  c.wolf_chance_to_despawn = 0.05;
  c.wolves = 1;
  c.wolves_can_move = 1;
  c.autoreset = 1;
  c.bush_thresholds = nullptr;  // computed by wab_create (wab_bush_thresholds)

  wab_handle* h = nullptr;
  CHECK_WAB(wab_create(&c, B, seed, 0, 0, &h));
  const size_t OB = (size_t)3 * 11 * 11;
  uint8_t *planes, *scal, *done;
  int8_t* act;
  float* rew;
  CHECK_HIP(hipMalloc(&planes, B * OB));
  CHECK_HIP(hipMalloc(&scal, 3 * B));
  CHECK_HIP(hipMalloc(&done, B));
  CHECK_HIP(hipMalloc(&act, B));
  CHECK_HIP(hipMalloc(&rew, 4 * B));
  wab_obs o = {planes, scal, scal + B, scal + 2 * B};
  CHECK_WAB(wab_reset(h, nullptr, &o, nullptr));

  std::vector<int8_t> a_h((size_t)T * B);
  std::vector<float> r_h((size_t)T * B);
  std::vector<uint8_t> d_h((size_t)T * B);
  uint64_t s = seed;
  for (int t = 0; t < T; ++t) {
    for (int64_t i = 0; i < B; ++i) {  // splitmix64 stream, action = top bits mod 5
      uint64_t z = (s += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      a_h[(size_t)t * B + i] = (int8_t)((z ^ (z >> 31)) % 5);
    }
    CHECK_HIP(hipMemcpy(act, a_h.data() + (size_t)t * B, B, hipMemcpyHostToDevice));
    CHECK_WAB(wab_step(h, act, &o, rew, done, nullptr, nullptr));
    CHECK_HIP(hipMemcpy(r_h.data() + (size_t)t * B, rew, 4 * B, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(d_h.data() + (size_t)t * B, done, B, hipMemcpyDeviceToHost));
  }
  std::vector<uint8_t> p_h(B * OB), s_h(3 * B);
  CHECK_HIP(hipMemcpy(p_h.data(), planes, B * OB, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(s_h.data(), scal, 3 * B, hipMemcpyDeviceToHost));
  wab_counters ctr;
  CHECK_WAB(wab_get_counters(h, &ctr, nullptr));
  if (ctr.handoff_timeouts || ctr.wolf_overflow || ctr.eaten_overflow || ctr.bad_actions) {
    std::fprintf(stderr, "counters: handoff %llu wolf %llu eaten %llu bad %llu\n",
                 (unsigned long long)ctr.handoff_timeouts, (unsigned long long)ctr.wolf_overflow,
                 (unsigned long long)ctr.eaten_overflow, (unsigned long long)ctr.bad_actions);
    return 1;
  }
  FILE* f = std::fopen(argv[4], "wb");
  if (!f) return 1;
  std::fwrite(a_h.data(), 1, a_h.size(), f);
  std::fwrite(r_h.data(), 4, r_h.size(), f);
  std::fwrite(d_h.data(), 1, d_h.size(), f);
  std::fwrite(p_h.data(), 1, p_h.size(), f);
  std::fwrite(s_h.data(), 1, s_h.size(), f);
  std::fclose(f);
  CHECK_WAB(wab_destroy(h));
  for (void* p : {(void*)planes, (void*)scal, (void*)done, (void*)act, (void*)rew}) CHECK_HIP(hipFree(p));
  std::printf("c_api_demo: %lld envs x %d steps, %llu resets\n", (long long)B, T,
              (unsigned long long)ctr.resets);
  return 0;
}
