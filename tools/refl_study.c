/* Design study (not product, not a checker): occupancy of the packets a RT_SHADE_REF frame traces
 * (primary, the plane's shadow rays, reflection rays), per kind: packets with a live ray and their
 * live rays. Built and run by tools/refl_study.py. */
#include <stdint.h>
static uint64_t g_pk[3][2]; /* kind: 0 primary, 1 shadow (any hit), 2 reflection (cull); [packets, live rays] */
static void pk_hook(int any, int cull, const int* alive);
#define OSTUDY_PACKET_HOOK(any, cull, alive) pk_hook(any, cull, alive)
#include "../oracle/rt_oracle.c"

static void pk_hook(int any, int cull, const int* alive) {
  int n = 0;
  for (int l = 0; l < OPK; ++l) n += alive[l] != 0;
  if (!n) return;
  const int kind = any ? 1 : (cull ? 2 : 0);
  __atomic_fetch_add(&g_pk[kind][0], 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&g_pk[kind][1], (uint64_t)n, __ATOMIC_RELAXED);
}
void pk_get(uint64_t out[6]) {
  for (int k = 0; k < 3; ++k) { out[2 * k] = g_pk[k][0]; out[2 * k + 1] = g_pk[k][1]; g_pk[k][0] = g_pk[k][1] = 0; }
}
