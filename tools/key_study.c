/* Design study (not product, not a checker): packet-walk fetches of a config's frame under other
 * nearest-first keys for closest-hit walks (entry distance n, exit distance f of the lead ray).
 *   key 0  |n| (the kernel)            key 1  |f|
 *   key 2  |n + f| / 2 (mid-point)     key 3  |n|, ties (n at tmin: the ray starts inside) by |f|
 * Built and run by tools/key_study.py (study_render = oracle_render with the key selected). */
#include <stdint.h>
static int g_key = 0;
static uint32_t key_of(float n, float f);
#define OCLOSEST_KEY(n, f) key_of(n, f)
#include "../oracle/rt_oracle.c"

static uint32_t key_of(float n, float f) {
  switch (g_key) {
    case 1: return f2bits(f) & 0x7fffffffu;
    case 2: return f2bits((n + f) * 0.5f) & 0x7fffffffu;
    case 3: {
      /* n == tmin (0 or 0.01 here) means the origin is inside: order those by exit distance, after
       * nothing else (they compare below every box entered later) */
      uint32_t nb = f2bits(n) & 0x7fffffffu;
      if (n <= 0.01f) return (f2bits(f) & 0x7fffffffu) >> 8; /* inside boxes: by exit, below any entry */
      return nb > 0x00800000u ? nb : 0x00800000u;
    }
    default: return f2bits(n) & 0x7fffffffu;
  }
}
void set_key(int k) { g_key = k; }
