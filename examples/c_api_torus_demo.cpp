// A C-ABI caller of the Environment 2.0 torus world (include/wab_torus.h only, no Python in the
// process).
//   1. The reference's own known-answer tests, World_tests.py:5-45 and :49-88, through the HIP
//      kernel: worlds created at the tests' positions (wab2_create_at), the observer's record
//      (wab2_get_obs, after the other ostrich's wab2_take_action in the wrap test) decoded here
//      and checked row by row.
//   2. B worlds of the benched 32x32 1/8/16 world at caller-chosen create and reset positions
//      (wab2_create_at, wab2_reset_at; a negative pair asks for the random position), T turns of
//      wab2_step with host-chosen actions, then T turns in one wab2_rollout launch, everything
//      written to a file that tests/test_gpu_capi_demo.py replays through the Python host:
//        create_pos [B][N][2] i32, reset_pos [B][N][2] i32, actions [2T][B][N] i8,
//        records [2T][B][N][R] u8, reward [2T][B][N] f32, done [2T][B][N] u8,
//        world_reset [2T][B] u8.
//   usage: c_api_torus_demo B T seed out.bin
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/wab_torus.h"

#define CHECK_WAB2(x)                                                         \
  do {                                                                        \
    if ((x) != WAB2_OK) {                                                     \
      std::fprintf(stderr, "%s failed: %s\n", #x, wab2_last_error());         \
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

// default_game_options (WAB_Environment2.py:9-50), the keys World reads
static wab2_config default_config(int W, int H, int no, int nw, int nb) {
  wab2_config c;
  std::memset(&c, 0, sizeof(c));
  c.width = W;
  c.height = H;
  c.num_ostriches = no;
  c.num_wolves = nw;
  c.num_bushes = nb;
  c.starting_role = 1;
  c.ostrich_starting_food = 40.0;
  c.food_per_bush = 20;
  c.food_given_per_turn = 5;
  c.wolf_starting_food = 20;
  c.wolf_food_for_eating_ostrich = 10;
  c.lookout_view_radius = 9;
  c.gatherer_view_radius = 5;
  c.wolf_view_radius = 6;
  c.max_turns = 80;
  c.autoreset = 1;
  return c;
}

struct Row {
  int type, dx, dy, food;  // type 0 ostrich, 1 wolf, 2 bush; food: the bush's Additional_Data, else -1
  bool operator<(const Row& o) const {
    return type != o.type ? type < o.type : dx != o.dx ? dx < o.dx : dy != o.dy ? dy < o.dy : food < o.food;
  }
  bool operator==(const Row& o) const { return type == o.type && dx == o.dx && dy == o.dy && food == o.food; }
};

// the visible-objects rows of one record (wab_torus.h's layout), sorted: this surface numbers the
// entities ostriches, wolves, bushes where World_tests.py creates them in another order, so the
// rows are compared as a set
static std::vector<Row> rows_of(const uint8_t* rec, int no, int nw, int nb) {
  const int N = no + nw + nb;
  uint32_t vis;
  std::memcpy(&vis, rec + 16, 4);
  std::vector<Row> rows;
  for (int j = 0; j < N; ++j) {
    if (!((vis >> j) & 1u)) continue;
    const int type = j < no ? 0 : j < no + nw ? 1 : 2;
    const int food = type == 2 ? (int)rec[24 + 2 * N + (j - no - nw)] : -1;
    rows.push_back({type, (int)(int8_t)rec[24 + 2 * j], (int)(int8_t)rec[24 + 2 * j + 1], food});
  }
  std::sort(rows.begin(), rows.end());
  return rows;
}

// World_tests.py: a 20x20 world, `pos` in this surface's id order, the observer's record after
// `mover` (or -1) took action 0, against the expected rows
static int kat(const char* name, int no, int nw, int nb, int radius, const std::vector<int32_t>& pos, int mover,
               int observer, std::vector<Row> want) {
  wab2_config c = default_config(20, 20, no, nw, nb);
  c.lookout_view_radius = c.gatherer_view_radius = radius;
  const int N = no + nw + nb, B = 2;
  std::vector<int32_t> all((size_t)B * N * 2);
  for (int b = 0; b < B; ++b) std::copy(pos.begin(), pos.end(), all.begin() + (size_t)b * N * 2);
  wab2_handle* h = nullptr;
  CHECK_WAB2(wab2_create_at(&c, B, 0x5EED, 0, 0, all.data(), &h));
  const int R = wab2_record_size(&c);
  uint8_t* rec;
  int8_t* act;
  float* rew;
  uint8_t* done;
  CHECK_HIP(hipMalloc(&rec, (size_t)B * R));
  CHECK_HIP(hipMalloc(&act, B));
  CHECK_HIP(hipMalloc(&rew, 4 * B));
  CHECK_HIP(hipMalloc(&done, B));
  CHECK_HIP(hipMemset(act, 0, B));  // action 0: y + 1 (World.py:25-43)
  for (int i = 0; i < observer; ++i)  // the entities before the observer act first (ids ascending)
    if (i == mover) CHECK_WAB2(wab2_take_action(h, i, act, rew, done, nullptr, nullptr));
  CHECK_WAB2(wab2_get_obs(h, observer, rec, nullptr));
  std::vector<uint8_t> host((size_t)B * R);
  CHECK_HIP(hipMemcpy(host.data(), rec, host.size(), hipMemcpyDeviceToHost));
  std::sort(want.begin(), want.end());
  for (int b = 0; b < B; ++b) {
    const std::vector<Row> got = rows_of(host.data() + (size_t)b * R, no, nw, nb);
    if (got != want) {
      std::fprintf(stderr, "%s: world %d: %zu rows differ from the test's\n", name, b, got.size());
      for (const Row& r : got) std::fprintf(stderr, "  type %d (%d, %d) food %d\n", r.type, r.dx, r.dy, r.food);
      return 1;
    }
  }
  CHECK_WAB2(wab2_destroy(h));
  for (void* p : {(void*)rec, (void*)act, (void*)rew, (void*)done}) CHECK_HIP(hipFree(p));
  std::printf("c_api_torus_demo: %s: %zu rows as World_tests.py expects\n", name, want.size());
  return 0;
}

static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  if (argc != 5) {
    std::fprintf(stderr, "usage: %s B T seed out.bin\n", argv[0]);
    return 2;
  }
  const int64_t B = std::atoll(argv[1]);
  const int T = std::atoi(argv[2]);
  uint64_t s = std::strtoull(argv[3], nullptr, 0);
  if (B <= 0 || T <= 0) return 2;

  // 1. World_tests.py:5-45 (no wrap): ostrich (10, 10), wolves (5, 5), (15, 15), bushes
  //    (10, 5), (10, 10), (15, 10); radius 8
  if (kat("World_tests no-wrap", 1, 2, 3, 8, {10, 10, 5, 5, 15, 15, 10, 5, 10, 10, 15, 10}, -1, 0,
          {{1, -5, -5, -1}, {2, 0, -5, 20}, {0, 0, 0, -1}, {2, 0, 0, 20}, {2, 5, 0, 20}, {1, 5, 5, -1}}))
    return 1;
  //    World_tests.py:49-88 (wrap): the other ostrich (id 0 here) moves (15, 15) -> (15, 16), the
  //    observer at (19, 10) (id 1) looks with radius 10; the code returns a sixth row (the moved
  //    ostrich at (-4, 6)) where the test asserts five (tests/test_torus_oracle.py)
  if (kat("World_tests wrap", 2, 2, 2, 10, {15, 15, 19, 10, 5, 5, 15, 15, 10, 10, 15, 10}, 0, 1,
          {{1, 6, -5, -1}, {0, 0, 0, -1}, {2, -9, 0, 20}, {2, -4, 0, 20}, {1, -4, 5, -1}, {0, -4, 6, -1}}))
    return 1;

  // 2. the benched world at caller-chosen positions
  const wab2_config c = default_config(32, 32, 1, 8, 16);
  const int N = 25, R = wab2_record_size(&c);
  std::vector<int32_t> cpos((size_t)B * N * 2), rpos((size_t)B * N * 2);
  for (size_t k = 0; k < (size_t)B * N; ++k) {
    const uint64_t z = splitmix(s);
    const bool rnd = z % 5 == 0;  // a fifth of them: the random position
    cpos[2 * k] = rnd ? -1 : (int32_t)((z >> 8) % 32);
    cpos[2 * k + 1] = rnd ? -1 : (int32_t)((z >> 20) % 32);
    const uint64_t y = splitmix(s);
    rpos[2 * k] = y % 4 == 0 ? -1 : (int32_t)((y >> 8) % 33);  // x = W too, as randint(0, W) draws
    rpos[2 * k + 1] = (int32_t)((y >> 24) % 33);
  }
  wab2_handle* h = nullptr;
  CHECK_WAB2(wab2_create_at(&c, B, 0x5EED, 0, 0, cpos.data(), &h));
  CHECK_WAB2(wab2_reset_at(h, nullptr, rpos.data(), nullptr));
  const size_t BN = (size_t)B * N;
  int8_t* act;
  uint8_t *rec, *done, *wr;
  float* rew;
  CHECK_HIP(hipMalloc(&act, (size_t)T * BN));
  CHECK_HIP(hipMalloc(&rec, (size_t)T * BN * R));
  CHECK_HIP(hipMalloc(&rew, (size_t)T * BN * 4));
  CHECK_HIP(hipMalloc(&done, (size_t)T * BN));
  CHECK_HIP(hipMalloc(&wr, (size_t)T * B));
  std::vector<int8_t> a_h((size_t)2 * T * BN);
  for (size_t k = 0; k < a_h.size(); ++k) {
    const int i = (int)(k % N);
    a_h[k] = (int8_t)(splitmix(s) % (i == 0 ? 6 : i < 9 ? 5 : 1));  // ostrich 0..5, wolves 0..4, bushes 0
  }
  std::vector<uint8_t> rec_h((size_t)2 * T * BN * R), done_h((size_t)2 * T * BN), wr_h((size_t)2 * T * B);
  std::vector<float> rew_h((size_t)2 * T * BN);
  for (int t = 0; t < T; ++t) {  // T single turns
    CHECK_HIP(hipMemcpy(act, a_h.data() + (size_t)t * BN, BN, hipMemcpyHostToDevice));
    CHECK_WAB2(wab2_step(h, act, rec, rew, done, wr, nullptr));
    CHECK_HIP(hipMemcpy(rec_h.data() + (size_t)t * BN * R, rec, BN * R, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(rew_h.data() + (size_t)t * BN, rew, BN * 4, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(done_h.data() + (size_t)t * BN, done, BN, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(wr_h.data() + (size_t)t * B, wr, B, hipMemcpyDeviceToHost));
  }
  // T more turns in one launch
  CHECK_HIP(hipMemcpy(act, a_h.data() + (size_t)T * BN, (size_t)T * BN, hipMemcpyHostToDevice));
  CHECK_WAB2(wab2_rollout(h, act, T, rec, rew, done, wr, nullptr));
  CHECK_HIP(hipMemcpy(rec_h.data() + (size_t)T * BN * R, rec, (size_t)T * BN * R, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(rew_h.data() + (size_t)T * BN, rew, (size_t)T * BN * 4, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(done_h.data() + (size_t)T * BN, done, (size_t)T * BN, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(wr_h.data() + (size_t)T * B, wr, (size_t)T * B, hipMemcpyDeviceToHost));
  wab2_counters ctr;
  CHECK_WAB2(wab2_get_counters(h, &ctr, nullptr));
  FILE* f = std::fopen(argv[4], "wb");
  if (!f) return 1;
  std::fwrite(cpos.data(), 4, cpos.size(), f);
  std::fwrite(rpos.data(), 4, rpos.size(), f);
  std::fwrite(a_h.data(), 1, a_h.size(), f);
  std::fwrite(rec_h.data(), 1, rec_h.size(), f);
  std::fwrite(rew_h.data(), 4, rew_h.size(), f);
  std::fwrite(done_h.data(), 1, done_h.size(), f);
  std::fwrite(wr_h.data(), 1, wr_h.size(), f);
  std::fclose(f);
  CHECK_WAB2(wab2_destroy(h));
  for (void* p : {(void*)act, (void*)rec, (void*)rew, (void*)done, (void*)wr}) CHECK_HIP(hipFree(p));
  std::printf("c_api_torus_demo: %lld worlds x %d + %d turns, %llu world-turns, %llu resets\n", (long long)B, T, T,
              (unsigned long long)ctr.turns, (unsigned long long)ctr.resets);
  return 0;
}
