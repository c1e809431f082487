// wab_render.hip — WolvesAndBushesEnv.render(mode="rgb_array", scale, draw_health)
// (wab_env.py:468-502) for a batch, from the observation the step kernel wrote.
//
// rgb [B][W*scale][H*scale][3] u8: channel c of cell (i, j) is 255 * grid_c; an empty cell is
// 127 when the ostrich was killed, else 255, and then mask_grid (restrict_view blind spots,
// by role) zeroes it; each cell becomes a scale x scale block.  With draw_health the
// turns-until-starve count is drawn over it at (0, 0) in blue with PIL's default font
// (:496-500): the digit glyphs of wab_glyphs.h (tools/make_glyphs.py) blended by Pillow's
// rule out = DIV255(x * (255 - a) + ink * a).  One thread per output dword (4 bytes of
// consecutive pixels' channels), so stores coalesce.
#include <hip/hip_runtime.h>

#include "wab_glyphs.h"
#include "wab_params.h"

namespace wab {

__constant__ uint8_t kGlyphs[10 * WAB_GLYPH_ROWS * WAB_GLYPH_ADVANCE] = {WAB_GLYPH_DATA};

// the text overlay of one channel byte v at image row `row` (PIL y), column `col` (PIL x)
__device__ __forceinline__ uint8_t health_text(uint8_t v, uint32_t row, uint32_t col, uint32_t c, uint32_t ft) {
  const uint32_t r = row - (uint32_t)WAB_GLYPH_ROW0;  // (wraps above the glyphs' rows)
  const uint32_t nd = ft >= 100u ? 3u : ft >= 10u ? 2u : 1u;
  const uint32_t k = col / (uint32_t)WAB_GLYPH_ADVANCE;
  if (r >= (uint32_t)WAB_GLYPH_ROWS || k >= nd) return v;
  const uint32_t pow10 = nd - 1u - k == 2u ? 100u : nd - 1u - k == 1u ? 10u : 1u;
  const uint32_t digit = (ft / pow10) % 10u;
  const uint32_t a = kGlyphs[(digit * WAB_GLYPH_ROWS + r) * WAB_GLYPH_ADVANCE + (col - k * WAB_GLYPH_ADVANCE)];
  const uint32_t ink = c == 2u ? (uint32_t)WAB_GLYPH_INK_B : 0u;
  const uint32_t t = (uint32_t)v * (255u - a) + ink * a + 128u;  // Pillow's DIV255
  return (uint8_t)(((t >> 8) + t) >> 8);
}

__device__ __forceinline__ uint8_t cell_byte(const RenderParams& p, int64_t e, uint32_t row, uint32_t col, uint32_t c) {
  const int i = (int)(row / (uint32_t)p.scale), j = (int)(col / (uint32_t)p.scale);
  const uint8_t* pl = p.planes + (size_t)e * p.OB + (size_t)(i * p.S + j);
  const size_t plane = (size_t)p.W * p.S;
  const bool w = pl[0] != 0, b = pl[plane] != 0, s = pl[2 * plane] != 0;
  const bool killed = p.status[e] == 2;
  if (!(w | b | s)) {
    if (killed) return 127;
    const int role = p.role[e] == 1 ? 1 : 0;
    const bool blind = p.restrict_view && i < 11 && j < 11 && ((p.mask_rows[role][i] >> j) & 1u);
    return blind ? 0 : 255;
  }
  const bool on = c == 0 ? w : c == 1 ? b : s;
  return on ? 255 : 0;  // (objects never sit in blind spots: the observation is already masked)
}

__device__ __forceinline__ uint8_t render_byte(const RenderParams& p, int64_t e, uint32_t o) {
  const uint32_t RH = (uint32_t)(p.H * p.scale);
  const uint32_t px = o / 3u, c = o - px * 3u;
  const uint32_t row = px / RH, col = px - row * RH;
  const uint8_t v = cell_byte(p, e, row, col, c);
  return p.draw_health ? health_text(v, row, col, c, p.food_turns[e]) : v;
}

__global__ __launch_bounds__(256) void wab_render_kernel(RenderParams p) {
  const uint32_t per_env = (uint32_t)(p.W * p.scale) * (uint32_t)(p.H * p.scale) * 3u;
  const uint32_t words = (per_env + 3u) / 4u;
  const int64_t e = blockIdx.y;
  if (e >= p.B) return;
  uint8_t* out = p.rgb + (size_t)e * per_env;
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < words; q += gridDim.x * 256u) {
    const uint32_t o = q * 4u;
    if (o + 4u <= per_env && ((reinterpret_cast<uintptr_t>(out) & 3u) == 0)) {
      uint32_t v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) v |= (uint32_t)render_byte(p, e, o + k) << (8 * k);
      *reinterpret_cast<uint32_t*>(out + o) = v;
    } else {
      for (uint32_t k = 0; k < 4u && o + k < per_env; ++k) out[o + k] = render_byte(p, e, o + k);
    }
  }
}

}  // namespace wab
