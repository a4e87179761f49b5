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

/* --- sweep-SAH binary tree over the LBVH's leaves (design study: the quality gap of the Morton build) --- */
typedef struct { int ref; float b[6]; float c[3]; } sleaf;
static sleaf* s_lv;
static onode* s_out;
static int s_n;
static int s_axis;
static int s_cmp(const void* a, const void* b) {
  float x = ((const sleaf*)a)->c[s_axis], y = ((const sleaf*)b)->c[s_axis];
  return x < y ? -1 : x > y ? 1 : (((const sleaf*)a)->ref < ((const sleaf*)b)->ref ? -1 : 1);
}
static void s_box(const sleaf* v, int n, float* bb) {
  for (int a = 0; a < 3; ++a) { bb[a] = INFINITY; bb[3 + a] = -INFINITY; }
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) { bb[a] = fminf(bb[a], v[i].b[a]); bb[3 + a] = fmaxf(bb[3 + a], v[i].b[3 + a]); }
}
/* returns the child ref (node index >= 0, or the leaf's ~tri ref) of the subtree over v[0, n) */
static int s_build(sleaf* v, int n) {
  if (n == 1) return v[0].ref;
  float* rarea = (float*)malloc((size_t)n * 4);
  int best_axis = 0, best_i = n / 2;
  float best = INFINITY;
  for (int a = 0; a < 3; ++a) {
    s_axis = a;
    qsort(v, (size_t)n, sizeof(sleaf), s_cmp);
    float bb[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int i = n - 1; i > 0; --i) {
      for (int k = 0; k < 3; ++k) { bb[k] = fminf(bb[k], v[i].b[k]); bb[3 + k] = fmaxf(bb[3 + k], v[i].b[3 + k]); }
      rarea[i] = half_area(bb);
    }
    float lb[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int i = 1; i < n; ++i) {
      for (int k = 0; k < 3; ++k) { lb[k] = fminf(lb[k], v[i - 1].b[k]); lb[3 + k] = fmaxf(lb[3 + k], v[i - 1].b[3 + k]); }
      float c = half_area(lb) * (float)i + rarea[i] * (float)(n - i);
      if (c < best) { best = c; best_axis = a; best_i = i; }
    }
  }
  free(rarea);
  s_axis = best_axis;
  qsort(v, (size_t)n, sizeof(sleaf), s_cmp);
  const int me = s_n++;
  float l[6], r[6];
  s_box(v, best_i, l);
  s_box(v + best_i, n - best_i, r);
  const int c0 = s_build(v, best_i);
  const int c1 = s_build(v + best_i, n - best_i);
  onode* o = &s_out[me];
  memset(o, 0, sizeof(*o));
  for (int a = 0; a < 3; ++a) { o->lo0[a] = l[a]; o->hi0[a] = l[3 + a]; o->lo1[a] = r[a]; o->hi1[a] = r[3 + a]; }
  o->c0 = c0;
  o->c1 = c1;
  return me;
}
/* replaces the kept binary LBVH with a sweep-SAH tree over the same leaves (same triangle refs) */
int wide_study_sah(void) {
  if (!g_bin) return 1;
  const onode* bin = (const onode*)g_bin;
  s_lv = (sleaf*)malloc(((size_t)g_nbin + 2) * sizeof(sleaf));
  int nl = 0;
  for (uint32_t i = 0; i < g_nbin; ++i)
    for (int side = 0; side < 2; ++side) {
      const int c = side ? bin[i].c1 : bin[i].c0;
      if (c >= 0 || c == O_EMPTY) continue;
      sleaf* L = &s_lv[nl++];
      L->ref = c;
      const float* lo = side ? bin[i].lo1 : bin[i].lo0;
      const float* hi = side ? bin[i].hi1 : bin[i].hi0;
      for (int a = 0; a < 3; ++a) { L->b[a] = lo[a]; L->b[3 + a] = hi[a]; L->c[a] = 0.5f * (lo[a] + hi[a]); }
    }
  s_out = (onode*)calloc((size_t)nl + 2, sizeof(onode));
  s_n = 0;
  s_build(s_lv, nl);
  free(s_lv);
  free(g_bin);
  g_bin = s_out;
  g_nbin = (uint32_t)s_n;
  return 0;
}

/* --- treelet restructuring of the binary LBVH (Karras & Aila 2013), design study ------------------------
 * cost of a subtree = sum of its internal nodes' half areas (every leaf is one triangle, so the leaves' terms are
 * the same in any topology); each node, children before parents, regroups the up to 7 subtrees under its treelet
 * (grown by opening the largest-area internal leaf, lowest position on ties) into the cost-optimal binary
 * topology (DP over the subsets), reusing the treelet's node slots. */
#define TL 7
static float t_box_area(const float* b) { return half_area(b); }
static void t_union(const float* a, const float* b, float* o) {
  for (int k = 0; k < 3; ++k) { o[k] = fminf(a[k], b[k]); o[3 + k] = fmaxf(a[3 + k], b[3 + k]); }
}
static float* t_cost; /* per binary node: its subtree cost */
static void t_node_box(const onode* b, float* bb) {
  for (int a = 0; a < 3; ++a) { bb[a] = fminf(b->lo0[a], b->lo1[a]); bb[3 + a] = fmaxf(b->hi0[a], b->hi1[a]); }
}
static void t_restructure(onode* bin, int n) {
  int lref[TL];
  float lbox[TL][6];
  int internal[TL];
  int nl = 2, ni = 1;
  internal[0] = n;
  lref[0] = bin[n].c0;
  lref[1] = bin[n].c1;
  for (int a = 0; a < 3; ++a) {
    lbox[0][a] = bin[n].lo0[a]; lbox[0][3 + a] = bin[n].hi0[a];
    lbox[1][a] = bin[n].lo1[a]; lbox[1][3 + a] = bin[n].hi1[a];
  }
  while (nl < TL) {
    int best = -1;
    float ba = -1.0f;
    for (int j = 0; j < nl; ++j)
      if (lref[j] >= 0 && t_box_area(lbox[j]) > ba) { ba = t_box_area(lbox[j]); best = j; }
    if (best < 0) break;
    const onode* g = &bin[lref[best]];
    internal[ni++] = lref[best];
    lref[best] = g->c0;
    lref[nl] = g->c1;
    for (int a = 0; a < 3; ++a) {
      lbox[best][a] = g->lo0[a]; lbox[best][3 + a] = g->hi0[a];
      lbox[nl][a] = g->lo1[a]; lbox[nl][3 + a] = g->hi1[a];
    }
    ++nl;
  }
  if (nl < 3) return;
  const int full = (1 << nl) - 1;
  float area[1 << TL], copt[1 << TL];
  int8_t split[1 << TL];
  float ubox[1 << TL][6];
  for (int m = 1; m <= full; ++m) {
    int first = __builtin_ctz(m);
    if ((m & (m - 1)) == 0) {
      memcpy(ubox[m], lbox[first], 24);
      copt[m] = lref[first] >= 0 ? t_cost[lref[first]] : 0.0f;
      area[m] = t_box_area(lbox[first]);
      split[m] = 0;
      continue;
    }
    t_union(ubox[m & (m - 1)], lbox[first], ubox[m]);
    area[m] = t_box_area(ubox[m]);
  }
  for (int m = 1; m <= full; ++m) {
    if ((m & (m - 1)) == 0) continue;
    /* partitions P | R with P holding m's lowest bit; the first strict minimum in ascending P */
    const int low = m & -m, rest = m ^ low;
    float best = INFINITY;
    int bp = low;
    for (int sub = rest;; sub = (sub - 1) & rest) {
      const int P = low | sub;
      if (P != m) {
        const float c = copt[P] + copt[m ^ P];
        if (c < best) { best = c; bp = P; }
      }
      if (sub == 0) break;
    }
    copt[m] = area[m] + best;
    split[m] = (int8_t)0;
    /* keep P in a side table: masks fit 7 bits */
    ((int8_t*)split)[m] = (int8_t)bp;
  }
  /* current cost of the treelet */
  float cur = 0.0f;
  for (int j = 0; j < ni; ++j) { float bb[6]; t_node_box(&bin[internal[j]], bb); cur += t_box_area(bb); }
  for (int j = 0; j < nl; ++j) cur += lref[j] >= 0 ? t_cost[lref[j]] : 0.0f;
  if (!(copt[full] < cur)) return;
  /* rebuild: node slots in order internal[0] (= n, the root), internal[1] ... */
  int slot = 0;
  int stack_m[TL * 2], stack_node[TL * 2], sp = 0;
  stack_m[sp] = full; stack_node[sp] = internal[slot++]; ++sp;
  while (sp) {
    --sp;
    const int m = stack_m[sp], nd = stack_node[sp];
    const int P = (uint8_t)split[m], R = m ^ P;
    int kids[2] = {P, R};
    int refs[2];
    for (int k = 0; k < 2; ++k) {
      const int km = kids[k];
      if ((km & (km - 1)) == 0) refs[k] = lref[__builtin_ctz(km)];
      else { refs[k] = internal[slot++]; stack_m[sp] = km; stack_node[sp] = refs[k]; ++sp; }
    }
    onode* o = &bin[nd];
    o->c0 = refs[0];
    o->c1 = refs[1];
    for (int a = 0; a < 3; ++a) {
      o->lo0[a] = ubox[P][a]; o->hi0[a] = ubox[P][3 + a];
      o->lo1[a] = ubox[R][a]; o->hi1[a] = ubox[R][3 + a];
    }
    t_cost[nd] = copt[m];
  }
}
/* binary cost of the kept tree: sum of internal half areas */
double wide_study_cost(void) {
  const onode* bin = (const onode*)g_bin;
  double c = 0.0;
  for (uint32_t i = 0; i < g_nbin; ++i) { float bb[6]; t_node_box(&bin[i], bb); c += t_box_area(bb); }
  return c;
}
int wide_study_treelet(int passes) {
  if (!g_bin) return 1;
  onode* bin = (onode*)g_bin;
  t_cost = (float*)calloc(g_nbin, sizeof(float));
  int* order = (int*)malloc((size_t)g_nbin * 4 + 4);
  int* st = (int*)malloc((size_t)g_nbin * 8 + 8);
  for (int pass = 0; pass < passes; ++pass) {
    int top = 0, no = 0;
    st[top++] = 0;
    while (top) {
      const int v = st[--top];
      order[no++] = v;
      if (bin[v].c0 >= 0) st[top++] = bin[v].c0;
      if (bin[v].c1 >= 0) st[top++] = bin[v].c1;
    }
    for (int q = no - 1; q >= 0; --q) { /* children before parents */
      const int v = order[q];
      float bb[6];
      t_node_box(&bin[v], bb);
      t_cost[v] = t_box_area(bb) + (bin[v].c0 >= 0 ? t_cost[bin[v].c0] : 0.0f) + (bin[v].c1 >= 0 ? t_cost[bin[v].c1] : 0.0f);
      t_restructure(bin, v);
    }
  }
  free(order); free(st); free(t_cost);
  return 0;
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
