/* Design study (not product, not a checker): per 8x8 tile of a LAMBERT_SHADOW config, the packet walk's cost
 * (per-wave node + triangle + instance fetches, the kernel's rules via the oracle's emulation) of the whole
 * 64-lane packet and of its sub-packets: the tile traced as 2 packets of 8x4 pixels, 4 of 4x4 or 16 of 2x2 (lanes
 * outside the sub-tile join dead). Built and run by tools/split_study.py, which simulates the launch's schedule
 * with the costly tiles split. Tile rows are spread over threads. */
#include <pthread.h>

#include "../oracle/rt_oracle.c"

#define SPLIT_COLS 23 /* per tile: full, 2 halves, 4 quadrants, 16 2x2 cells */

typedef struct {
  const octx* c;
  uint32_t tw, th, row0, nthr;
  uint64_t* out;
} sjob;

static uint64_t sub_cost(const octx* c, uint32_t tx, uint32_t ty, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h) {
  uint32_t px[OPK], py[OPK];
  int inimg[OPK];
  float ox[OPK], oy[OPK];
  vec3 col[OPK];
  for (int l = 0; l < OPK; ++l) {
    const uint32_t lx = (uint32_t)(l & 7), ly = (uint32_t)(l >> 3);
    px[l] = tx * 8 + lx;
    py[l] = ty * 8 + ly;
    inimg[l] = lx >= x0 && lx < x0 + w && ly >= y0 && ly < y0 + h;
    ox[l] = oy[l] = 0.5f;
  }
  ostats st;
  memset(&st, 0, sizeof(st));
  osample_packet(c, px, py, inimg, ox, oy, col, &st);
  return st.v[9] + st.v[10] + st.v[11];
}

static void* split_worker(void* arg) {
  const sjob* j = (const sjob*)arg;
  for (uint32_t ty = j->row0; ty < j->th; ty += j->nthr)
    for (uint32_t tx = 0; tx < j->tw; ++tx) {
      uint64_t* o = j->out + ((uint64_t)ty * j->tw + tx) * SPLIT_COLS;
      o[0] = sub_cost(j->c, tx, ty, 0, 0, 8, 8);
      for (uint32_t q = 0; q < 2; ++q) o[1 + q] = sub_cost(j->c, tx, ty, 0, 4 * q, 8, 4);
      for (uint32_t q = 0; q < 4; ++q) o[3 + q] = sub_cost(j->c, tx, ty, 4 * (q & 1), 4 * (q >> 1), 4, 4);
      for (uint32_t q = 0; q < 16; ++q) o[7 + q] = sub_cost(j->c, tx, ty, 2 * (q & 3), 2 * (q >> 2), 2, 2);
    }
  return NULL;
}

int split_study(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t nl, uint32_t W, uint32_t H,
                uint32_t nthreads, uint64_t* out) {
  octx c = {s, cb, L, nl, NULL, 1, 1, 0, W, H};
  const uint32_t tw = W / 8, th = H / 8;
  pthread_t th_[256];
  sjob jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (uint32_t t = 0; t < nthreads; ++t) {
    jobs[t] = (sjob){&c, tw, th, t, nthreads, out};
    pthread_create(&th_[t], NULL, split_worker, &jobs[t]);
  }
  for (uint32_t t = 0; t < nthreads; ++t) pthread_join(th_[t], NULL);
  return 0;
}
