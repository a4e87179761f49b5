/* Design study (not product, not a checker): packet-walk work of 4-wide vs 8-wide collapses of the
 * SAME binary LBVH (the SAH-optimal collapse DP generalised to W slots), for a config's primary and
 * shadow packets (8x8-pixel waves) on its first BLAS (an identity instance: world = object rays).
 * Counts per-wave node visits, per-live-lane box tests and per-wave triangle fetches with the
 * kernel's rules: closest hit nearest-first by the lead lane's entry distance, any hit lowest slot
 * first, slots in ascending half area, triangle children tested in place in slot order.
 * Built and run by tools/wide_study.py. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
typedef struct onode_s onode_fwd;
static void* g_bin = 0;
static uint32_t g_nbin = 0;
#define OSTUDY_BIN_HOOK(bin, nbin) study_keep_bin((const void*)(bin), (nbin), sizeof(*(bin)))
static void study_keep_bin(const void* bin, uint32_t nbin, size_t sz) {
  if (nbin <= g_nbin) return; /* keep the largest BLAS */
  free(g_bin);
  g_bin = malloc(nbin * sz);
  memcpy(g_bin, bin, nbin * sz);
  g_nbin = nbin;
}
#include "../oracle/rt_oracle.c"

#define WMAX 8
typedef struct { int child[WMAX]; float box[WMAX][6]; int count; } wnode;
static float* wC;   /* [nbin][WMAX+1] */
static int8_t* wS;
static int gW = 4;

static void wdp(const onode* bin, uint32_t nbin) {
  wC = (float*)malloc((size_t)nbin * (WMAX + 1) * 4);
  wS = (int8_t*)malloc((size_t)nbin * (WMAX + 1));
  int* st = (int*)malloc((size_t)nbin * 2 * 4 + 8);
  int* order = (int*)malloc((size_t)nbin * 4 + 4);
  int top = 0, no = 0;
  st[top++] = 0;
  while (top) {
    int v = st[--top];
    order[no++] = v;
    if (bin[v].c0 >= 0) st[top++] = bin[v].c0;
    if (bin[v].c1 >= 0) st[top++] = bin[v].c1;
  }
  for (int q = no - 1; q >= 0; --q) {
    int v = order[q];
    const onode* b = &bin[v];
    float bb[6];
    for (int a = 0; a < 3; ++a) { bb[a] = fminf(b->lo0[a], b->lo1[a]); bb[3 + a] = fmaxf(b->hi0[a], b->hi1[a]); }
    float cl[WMAX + 1], cr[WMAX + 1], D[WMAX + 1];
    int8_t J[WMAX + 1];
    for (int i = 1; i <= gW; ++i) {
      cl[i] = b->c0 >= 0 ? wC[b->c0 * (WMAX + 1) + i] : 0.0f;
      cr[i] = b->c1 >= 0 ? wC[b->c1 * (WMAX + 1) + i] : 0.0f;
    }
    for (int i = 2; i <= gW; ++i) {
      D[i] = INFINITY; J[i] = 1;
      for (int j = 1; j < i; ++j) { float c = cl[j] + cr[i - j]; if (c < D[i]) { D[i] = c; J[i] = (int8_t)j; } }
    }
    float self = half_area(bb) + D[gW];
    wC[v * (WMAX + 1) + 1] = self; wS[v * (WMAX + 1) + 1] = 0;
    for (int i = 2; i <= gW; ++i) {
      if (D[i] < self) { wC[v * (WMAX + 1) + i] = D[i]; wS[v * (WMAX + 1) + i] = J[i]; }
      else { wC[v * (WMAX + 1) + i] = self; wS[v * (WMAX + 1) + i] = 0; }
    }
  }
  free(st); free(order);
}

static void wexp(const onode* bin, int c, const float* cbox, int k, int* ref, float (*box)[6], int* cnt) {
  if (c < 0 || k == 1 || wS[c * (WMAX + 1) + k] == 0) { ref[*cnt] = c; memcpy(box[*cnt], cbox, 24); ++*cnt; return; }
  const onode* b = &bin[c];
  int j = wS[c * (WMAX + 1) + k];
  float l[6] = {b->lo0[0], b->lo0[1], b->lo0[2], b->hi0[0], b->hi0[1], b->hi0[2]};
  float r[6] = {b->lo1[0], b->lo1[1], b->lo1[2], b->hi1[0], b->hi1[1], b->hi1[2]};
  wexp(bin, b->c0, l, j, ref, box, cnt);
  wexp(bin, b->c1, r, k - j, ref, box, cnt);
}

static wnode* g_w = 0;
static int g_wn = 0;

static void wcollapse(const onode* bin, uint32_t nbin) {
  wdp(bin, nbin);
  int* q = (int*)malloc((size_t)nbin * 4 + 4);
  g_w = (wnode*)calloc((size_t)nbin + 1, sizeof(wnode));
  int head = 0, tail = 1;
  q[0] = 0;
  while (head < tail) {
    const onode* b = &bin[q[head]];
    float cl[WMAX + 1], cr[WMAX + 1];
    for (int i = 1; i <= gW; ++i) {
      cl[i] = b->c0 >= 0 ? wC[b->c0 * (WMAX + 1) + i] : 0.0f;
      cr[i] = b->c1 >= 0 ? wC[b->c1 * (WMAX + 1) + i] : 0.0f;
    }
    int bj = 1; float bc = INFINITY;
    for (int j = 1; j < gW; ++j) { float c = cl[j] + cr[gW - j]; if (c < bc) { bc = c; bj = j; } }
    int ref[WMAX]; float box[WMAX][6]; int cnt = 0;
    float l[6] = {b->lo0[0], b->lo0[1], b->lo0[2], b->hi0[0], b->hi0[1], b->hi0[2]};
    float r[6] = {b->lo1[0], b->lo1[1], b->lo1[2], b->hi1[0], b->hi1[1], b->hi1[2]};
    wexp(bin, b->c0, l, bj, ref, box, &cnt);
    wexp(bin, b->c1, r, gW - bj, ref, box, &cnt);
    for (int a = 1; a < cnt; ++a)
      for (int z = a; z > 0 && half_area(box[z]) < half_area(box[z - 1]); --z) {
        int tr = ref[z]; ref[z] = ref[z - 1]; ref[z - 1] = tr;
        float tb[6]; memcpy(tb, box[z], 24); memcpy(box[z], box[z - 1], 24); memcpy(box[z - 1], tb, 24);
      }
    wnode* nd = &g_w[head];
    nd->count = 0;
    for (int j = 0; j < WMAX; ++j) { nd->child[j] = O_EMPTY; for (int a = 0; a < 6; ++a) nd->box[j][a] = INFINITY; }
    for (int j = 0; j < cnt; ++j) {
      if (ref[j] == O_EMPTY) continue;
      nd->count++;
      memcpy(nd->box[j], box[j], 24);
      if (ref[j] >= 0) { q[tail] = ref[j]; nd->child[j] = tail++; }
      else nd->child[j] = ref[j];
    }
    ++head;
  }
  g_wn = tail;
  free(q); free(wC); free(wS);
}

typedef struct { uint64_t nodes, aabb, tris, packets, slots; } wst;

/* BLAS packet walk over g_w; tri leaves ~slot index into tris (leaf order) */
static void wwalk(const otri* tris, const vec3* o, const vec3* d, const int* alive, float tmin, float tmax, int any,
                  float* tbest, wst* st) {
  vec3 iv[OPK], no[OPK];
  int live[OPK];
  for (int l = 0; l < OPK; ++l) {
    live[l] = alive[l];
    tbest[l] = tmax;
    iv[l] = mk(sinv(d[l].x), sinv(d[l].y), sinv(d[l].z));
    no[l] = vneg(vmul(o[l], iv[l]));
  }
  st->packets++;
  if (olead(live) < 0) return;
  int stack[4096], sp = 0, ref = 0;
  for (;;) {
    const wnode* nd = &g_w[ref];
    st->nodes++;
    uint64_t hm[WMAX];
    uint32_t key[OPK][WMAX];
    for (int k = 0; k < WMAX; ++k) hm[k] = 0;
    for (int l = 0; l < OPK; ++l) {
      if (!live[l]) continue;
      st->aabb += (uint64_t)gW;
      for (int k = 0; k < gW; ++k) {
        const float* b = nd->box[k];
        float tlx = fmaf(b[0], iv[l].x, no[l].x), thx = fmaf(b[3], iv[l].x, no[l].x);
        float tly = fmaf(b[1], iv[l].y, no[l].y), thy = fmaf(b[4], iv[l].y, no[l].y);
        float tlz = fmaf(b[2], iv[l].z, no[l].z), thz = fmaf(b[5], iv[l].z, no[l].z);
        float n = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), tmin));
        float f = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tbest[l]));
        int h = n <= f * 1.0000004f;
        if (h) hm[k] |= 1ull << l;
        key[l][k] = h ? (f2bits(n) & 0x7fffffffu) : 0x7f800000u;
      }
    }
    uint32_t ent = 0;
    for (int k = 0; k < gW; ++k) if (hm[k]) ent |= 1u << k;
    /* triangles in place */
    for (int k = 0; k < gW; ++k) {
      if (!((ent >> k) & 1u) || nd->child[k] >= 0) continue;
      ent &= ~(1u << k);
      const otri* tr = tris + (~nd->child[k]);
      st->tris++;
      for (int l = 0; l < OPK; ++l) {
        if (!live[l]) continue;
        float t, u, v;
        if (omt(o[l], d[l], tr, 0.0f, &t, &u, &v) && t >= tmin && t < tbest[l]) {
          tbest[l] = t;
          if (any) live[l] = 0;
        }
      }
    }
    int lead = olead(live);
    if (lead < 0) return;
    if (any) {
      uint64_t lm = 0;
      for (int l = 0; l < OPK; ++l) if (live[l]) lm |= 1ull << l;
      for (int k = 0; k < gW; ++k) if (!(hm[k] & lm)) ent &= ~(1u << k);
    }
    if (ent) {
      int ib = __builtin_ctz(ent);
      if (!any) {
        uint32_t kb = 0xffffffffu;
        for (int k = 0; k < gW; ++k) if (((ent >> k) & 1u) && key[lead][k] < kb) { kb = key[lead][k]; ib = k; }
      }
      for (int k = gW - 1; k >= 0; --k) if (k != ib && ((ent >> k) & 1u)) stack[sp++] = nd->child[k];
      ref = nd->child[ib];
      continue;
    }
    if (sp == 0) return;
    ref = stack[--sp];
  }
}

/* out: [0] primary nodes [1] primary aabb [2] primary tris [3] shadow nodes [4] shadow aabb [5] shadow tris
 *      [6] primary packets [7] shadow packets [8] wide nodes */
int wide_study(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t W, uint32_t H, int width,
               uint64_t out[9]) {
  if (!g_bin) return 1;
  gW = width;
  wcollapse((const onode*)g_bin, g_nbin);
  const oblas* bl = &s->blas[s->inst[0].blas];
  octx c = {s, cb, L, 1, NULL, 1, 1, 0, W, H};
  wst ps, ss;
  memset(&ps, 0, sizeof(ps));
  memset(&ss, 0, sizeof(ss));
  for (uint32_t ty = 0; ty < (H + 7) / 8; ++ty)
    for (uint32_t tx = 0; tx < (W + 7) / 8; ++tx) {
      vec3 O[OPK], D[OPK], P[OPK], S[OPK];
      int in[OPK], need[OPK];
      float tb[OPK];
      for (int l = 0; l < OPK; ++l) {
        uint32_t px = tx * 8 + (uint32_t)(l & 7), py = ty * 8 + (uint32_t)(l >> 3);
        in[l] = px < W && py < H;
        oraygen(&c, px, in[l] ? py : 0, 0.5f, 0.5f, &O[l], &D[l]);
      }
      wwalk(bl->tris, O, D, in, 0.0f, 100000.0f, 0, tb, &ps);
      for (int l = 0; l < OPK; ++l) {
        need[l] = 0;
        S[l] = mk(0, 0, 1);
        P[l] = O[l];
        if (!in[l] || !(tb[l] < 100000.0f)) continue;
        P[l] = vadd(O[l], vscale(D[l], tb[l]));
        vec3 Ld = vnorm(vsub(ld3(L[0].position), P[l]));
        need[l] = 1; /* shadow ray toward light 0 for every hit (n.L test skipped: same for both widths) */
        S[l] = Ld;
      }
      wwalk(bl->tris, P, S, need, 0.01f, 100000.0f, 1, tb, &ss);
    }
  out[0] = ps.nodes; out[1] = ps.aabb; out[2] = ps.tris;
  out[3] = ss.nodes; out[4] = ss.aabb; out[5] = ss.tris;
  out[6] = ps.packets; out[7] = ss.packets; out[8] = (uint64_t)g_wn;
  free(g_w); g_w = 0;
  return 0;
}
