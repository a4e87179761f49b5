/* Design study (not product, not a checker): what the longest walks of a LAMBERT_SHADOW config are
 * made of. The oracle's packet emulation (the kernel's rules) gives every 8 x 8 tile's per-wave fetches; for the
 * costliest tiles, each 2 x 2 part (the tile balance's 16-way split) and each single lane (the floor: one ray's own
 * walk) is re-traced and its fetches split into TLAS nodes, BLAS nodes, triangles and instance records, by ray kind
 * (primary = closest hit, shadow = any hit). A wave's time follows its fetches (0.92 correlation on C4,
 * tools/tile_study.py): these are the dependent record loads of the wave's serial walk. Run by tools/path_study.py. */
#include <pthread.h>
static __thread unsigned long long g_nodes[2][2]; /* [blas][any] */
#define OSTUDY_NODE_HOOK(blas, any) (g_nodes[(blas) ? 1 : 0][(any) ? 1 : 0]++)
#include "../oracle/rt_oracle.c"

/* out (per call): [0] TLAS nodes primary [1] TLAS nodes shadow [2] BLAS nodes primary [3] BLAS nodes shadow
 *                 [4] triangle fetches [5] instance fetches [6] total fetches */
static void part_cost(const octx* c, uint32_t tx, uint32_t ty, const int* mask, unsigned long long out[7]) {
  uint32_t px[OPK], py[OPK];
  int inimg[OPK];
  float ox[OPK], oy[OPK];
  vec3 col[OPK];
  for (int l = 0; l < OPK; ++l) {
    px[l] = tx * 8 + (uint32_t)(l & 7);
    py[l] = ty * 8 + (uint32_t)(l >> 3);
    inimg[l] = mask[l] && px[l] < c->W && py[l] < c->H;
    ox[l] = oy[l] = 0.5f;
  }
  ostats st;
  memset(&st, 0, sizeof(st));
  memset(g_nodes, 0, sizeof(g_nodes));
  osample_packet(c, px, py, inimg, ox, oy, col, &st);
  out[0] = g_nodes[0][0]; out[1] = g_nodes[0][1]; out[2] = g_nodes[1][0]; out[3] = g_nodes[1][1];
  out[4] = st.v[10]; out[5] = st.v[11]; out[6] = st.v[9] + st.v[10] + st.v[11];
}

typedef struct { const octx* c; uint32_t tw, th, t0, nthr; unsigned long long* cost; } pjob;
static void* whole_worker(void* arg) {
  const pjob* j = (const pjob*)arg;
  int all[OPK];
  for (int l = 0; l < OPK; ++l) all[l] = 1;
  for (uint32_t t = j->t0; t < j->tw * j->th; t += j->nthr) {
    unsigned long long o[7];
    part_cost(j->c, t % j->tw, t / j->tw, all, o);
    j->cost[t] = o[6];
  }
  return NULL;
}

/* whole-tile costs of every tile (cost[tw * th]) */
int path_study_tiles(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t nl, uint32_t W,
                     uint32_t H, uint32_t nthreads, unsigned long long* cost) {
  octx c = {s, cb, L, nl, NULL, 1, 1, 0, W, H};
  const uint32_t tw = (W + 7) / 8, th = (H + 7) / 8;
  pthread_t thr[256];
  pjob jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (uint32_t t = 0; t < nthreads; ++t) {
    jobs[t] = (pjob){&c, tw, th, t, nthreads, cost};
    pthread_create(&thr[t], NULL, whole_worker, &jobs[t]);
  }
  for (uint32_t t = 0; t < nthreads; ++t) pthread_join(thr[t], NULL);
  return 0;
}

/* one tile: out[0..6] whole, then 16 parts (2 x 2 cells) x 7, then 64 single lanes x 7 */
int path_study_tile(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t nl, uint32_t W,
                    uint32_t H, uint32_t tx, uint32_t ty, unsigned long long* out) {
  octx c = {s, cb, L, nl, NULL, 1, 1, 0, W, H};
  int m[OPK];
  for (int l = 0; l < OPK; ++l) m[l] = 1;
  part_cost(&c, tx, ty, m, out);
  for (int q = 0; q < 16; ++q) {
    const int x0 = 2 * (q & 3), y0 = 2 * (q >> 2);
    for (int l = 0; l < OPK; ++l) m[l] = (l & 7) >= x0 && (l & 7) < x0 + 2 && (l >> 3) >= y0 && (l >> 3) < y0 + 2;
    part_cost(&c, tx, ty, m, out + 7 * (1 + q));
  }
  for (int k = 0; k < OPK; ++k) {
    for (int l = 0; l < OPK; ++l) m[l] = l == k;
    part_cost(&c, tx, ty, m, out + 7 * (17 + k));
  }
  return 0;
}
