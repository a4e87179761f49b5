/* Design study (not product, not a checker): per-wave fetches of the shadow (any-hit) packets under
 * other choices of the first child to descend into at a node (the rest keep slot order).
 *   order 0  lowest entered slot = smallest half area (the kernel)
 *   order 1  nearest entry distance of the lead ray
 *   order 2  farthest entry distance of the lead ray
 *   order 3  largest half area (highest entered slot)
 *   order 4  entered by the most live rays (lowest slot on ties)
 *   order 5  nearest entry distance of the lead ray among boxes it does not start inside (n > tmin)
 * Built and run by tools/anyhit_study.py. */
#include <stdint.h>
static int g_any_order = 0;
struct o4node_s;
#define OANY_CHOOSE(ent, vkey, lead, hm, live, nd, tmin) any_choose(ent, vkey, lead, hm, live, tmin)
static int any_choose(uint32_t ent, uint32_t (*vkey)[4], int lead, const uint64_t* hm, const int* live, float tmin);
#include "shadow_study.c"

static int any_choose(uint32_t ent, uint32_t (*vkey)[4], int lead, const uint64_t* hm, const int* live, float tmin) {
  int ib = __builtin_ctz(ent);
  if (g_any_order == 0) return ib;
  if (g_any_order == 3) return 31 - __builtin_clz(ent);
  uint64_t lm = 0;
  for (int l = 0; l < OPK; ++l) if (live[l]) lm |= 1ull << l;
  uint32_t tb = f2bits(tmin) & 0x7fffffffu;
  int best = -1;
  uint64_t bv = 0;
  for (int k = 0; k < 4; ++k) {
    if (!((ent >> k) & 1u)) continue;
    uint32_t key = vkey[lead][k];
    uint64_t v;
    switch (g_any_order) {
      case 1: v = 0xffffffffull - key; break;          /* smaller key better */
      case 2: v = key == 0x7f800000u ? 0 : key; break;  /* larger key better */
      case 4: v = (uint64_t)__builtin_popcountll(hm[k] & lm); break;
      default: v = key > tb ? (0x1ffffffffull - key) : (0xffffffffull - key) / 4; break;
    }
    if (best < 0 || v > bv) { best = k; bv = v; }
  }
  return best < 0 ? ib : best;
}

void set_any_order(int o) { g_any_order = o; }
