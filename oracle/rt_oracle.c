/*
 * rt_oracle.c — CPU ORACLE (test infrastructure; see rt_oracle.h for the parity status).
 *
 * Scalar C restatement of the reference's DXR path. Every function cites the reference
 * (paths relative to UtkuGokalp/RealTimeRayTracing_GradProject) it follows. Floating-point
 * expressions are written operand by operand in the reference's evaluation order and compiled
 * with -ffp-contract=off; the only fused multiply-adds are the explicit fmaf() of the slab test.
 * The BVH is an LBVH built by the same deterministic algorithm as the device builder, so the
 * device tree can be compared node for node; the rendered image does not depend on the tree
 * (conservative culling + (t, instance, primitive) tie-break), which brute_force=1 verifies.
 */
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------------- */
/* small vector helpers                                                                      */
/* ---------------------------------------------------------------------------------------- */
typedef struct { float x, y, z; } vec3;
static inline vec3 mk(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static inline vec3 vadd(vec3 a, vec3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 vsub(vec3 a, vec3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 vmul(vec3 a, vec3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline vec3 vscale(vec3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline vec3 vneg(vec3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float vdot(vec3 a, vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline vec3 vcross(vec3 a, vec3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* HLSL normalize, pinned as v * (1/sqrt(dot)) */
static inline vec3 vnorm(vec3 a) { float inv = 1.0f / sqrtf(vdot(a, a)); return vscale(a, inv); }
static inline float fmax2(float a, float b) { return a > b ? a : b; }
static inline float fmin2(float a, float b) { return a < b ? a : b; }
static inline vec3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

/* ---------------------------------------------------------------------------------------- */
/* ingest: OBJFileManager::LoadObjFile (src/OBJ_FileManager.cpp:10-71)                       */
/* ---------------------------------------------------------------------------------------- */
static int is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

/* `ss >> float` (OBJ_FileManager.cpp:30) as libstdc++ extracts it in the "C" locale (num_get::_M_extract_float, then
 * __convert_to_v): the longest prefix [sign] digits [. digits] [e|E [sign] digits] is accepted (a second '.', an 'e'
 * before any digit or a second 'e' ends it), strtof must consume all of it (else 0, failbit), an overflow to +-inf
 * gives +-FLT_MAX and failbit; the stream stops right after the accepted characters. */
static int o_parse_float(const char** pp, const char* end, float* out) {
  const char* p = *pp;
  while (p < end && is_ws(*p)) ++p;
  char* buf = (char*)malloc((size_t)(end - p) + 2);
  size_t n = 0;
  if (!buf) { *pp = p; *out = 0.0f; return 0; }
  if (p < end && (*p == '+' || *p == '-')) buf[n++] = *p++;
  int mant = 0, dec = 0, sci = 0;
  while (p < end) {
    const char ch = *p;
    if (ch >= '0' && ch <= '9') { buf[n++] = ch; mant = 1; }
    else if (ch == '.' && !dec && !sci) { buf[n++] = '.'; dec = 1; }
    else if ((ch == 'e' || ch == 'E') && !sci && mant) {
      buf[n++] = 'e';
      sci = 1;
      if (++p == end) break;
      if (*p != '+' && *p != '-') continue; /* the character after the 'e' is examined again */
      buf[n++] = *p;
    } else break;
    ++p;
  }
  buf[n] = 0;
  *pp = p;
  char* ep = NULL;
  float v = strtof(buf, &ep);
  int ok = !(ep == buf || *ep != 0);
  free(buf);
  if (!ok) { *out = 0.0f; return 0; }
  if (v == HUGE_VALF || v == -HUGE_VALF) { *out = v > 0.0f ? FLT_MAX : -FLT_MAX; return 0; }
  *out = v;
  return 1;
}

static int o_parse_uint(const char** pp, const char* end, uint32_t* out) {
  const char* p = *pp;
  while (p < end && is_ws(*p)) ++p;
  int neg = 0;
  if (p < end && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
  if (p >= end || *p < '0' || *p > '9') { *pp = p; *out = 0; return 0; }
  uint64_t v = 0;
  int ovf = 0;
  while (p < end && *p >= '0' && *p <= '9') { v = v * 10 + (uint64_t)(*p - '0'); if (v > 0xffffffffull) ovf = 1; ++p; }
  *pp = p;
  if (ovf) { *out = 0xffffffffu; return 0; }
  *out = neg ? (uint32_t)(0u - (uint32_t)v) : (uint32_t)v;
  return 1;
}

int oracle_obj_parse(const char* text, size_t len, float** vtx6, uint32_t* nv, uint32_t** idx, uint32_t* ni) {
  size_t cv = 1024, ci = 1024, v = 0, i = 0;
  float* V = (float*)malloc(cv * 6 * sizeof(float));
  uint32_t* I = (uint32_t*)malloc(ci * sizeof(uint32_t));
  if (!V || !I) { free(V); free(I); return -1; }
  const char* p = text;
  const char* end = text + len;
  while (p < end) {
    const char* ls = p;
    while (p < end && *p != '\n') ++p;
    const char* le = p;
    if (p < end) ++p;
    if (le - ls < 2) continue;
    const char* q = ls + 1;
    if (ls[0] == 'v' && ls[1] == ' ') {
      float xyz[3] = {0, 0, 0};
      int ok = 1;
      for (int k = 0; k < 3 && ok; ++k) ok = o_parse_float(&q, le, &xyz[k]);
      if (v == cv) { cv *= 2; V = (float*)realloc(V, cv * 6 * sizeof(float)); }
      float* d = V + v * 6;
      d[0] = xyz[0]; d[1] = xyz[1]; d[2] = xyz[2]; d[3] = 0.0f; d[4] = 1.0f; d[5] = 0.0f;
      ++v;
    } else if (ls[0] == 'f' && ls[1] == ' ') {
      uint32_t f[3] = {0, 0, 0};
      int ok = 1;
      for (int k = 0; k < 3 && ok; ++k) ok = o_parse_uint(&q, le, &f[k]);
      if (i + 3 > ci) { ci *= 2; I = (uint32_t*)realloc(I, ci * sizeof(uint32_t)); }
      for (int k = 0; k < 3; ++k) I[i++] = f[k] - 1u;
    }
  }
  *vtx6 = V; *nv = (uint32_t)v; *idx = I; *ni = (uint32_t)i;
  return 0;
}

void oracle_free(void* p) { free(p); }

/* ComputeVertexNormals (src/D3D12HelloTriangle.cpp:1430-1462); XMVector3Normalize as v/len. */
static void xm_norm(const float* v, float* o) {
  float len = sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
  if (len > 0.0f) { o[0] = v[0] / len; o[1] = v[1] / len; o[2] = v[2] / len; }
  else { o[0] = o[1] = o[2] = 0.0f; }
}

int oracle_vertex_normals(float* V, uint32_t nv, const uint32_t* I, uint32_t ni) {
  if (ni % 3) return -1;
  for (uint32_t k = 0; k < ni; ++k) if (I[k] >= nv) return -1;
  float* acc = (float*)calloc((size_t)nv * 3 + 1, sizeof(float));
  for (uint32_t t = 0; t + 2 < ni; t += 3) {
    uint32_t a = I[t], b = I[t + 1], c = I[t + 2];
    const float *p0 = V + a * 6, *p1 = V + b * 6, *p2 = V + c * 6;
    float e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    float e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
    float cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    float n[3];
    xm_norm(cr, n);
    uint32_t ids[3] = {a, b, c};
    for (int k = 0; k < 3; ++k) {
      acc[ids[k] * 3 + 0] = acc[ids[k] * 3 + 0] + n[0];
      acc[ids[k] * 3 + 1] = acc[ids[k] * 3 + 1] + n[1];
      acc[ids[k] * 3 + 2] = acc[ids[k] * 3 + 2] + n[2];
    }
  }
  for (uint32_t v = 0; v < nv; ++v) {
    float n[3];
    xm_norm(acc + v * 3, n);
    V[v * 6 + 3] = -n[0]; V[v * 6 + 4] = -n[1]; V[v * 6 + 5] = -n[2];
  }
  free(acc);
  return 0;
}

/* glm::lookAtRH (glm/gtc/matrix_transform.inl:519-545), glm column-major memory. */
void oracle_camera_lookat(const float eye[3], const float center[3], const float up[3], float view[16]) {
  vec3 e = ld3(eye), c = ld3(center), u0 = ld3(up);
  vec3 f = vnorm(vsub(c, e));
  vec3 s = vnorm(vcross(f, u0));
  vec3 u = vcross(s, f);
  float r[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  r[0] = s.x; r[4] = s.y; r[8] = s.z;
  r[1] = u.x; r[5] = u.y; r[9] = u.z;
  r[2] = -f.x; r[6] = -f.y; r[10] = -f.z;
  r[12] = -vdot(s, e); r[13] = -vdot(u, e); r[14] = vdot(f, e);
  memcpy(view, r, sizeof(r));
}

/* general 4x4 inverse in double (XMMatrixInverse semantics; rounding pinned, parity unpinned) */
static void inv4(const float* mf, float* out) {
  double m[16], a[16];
  for (int i = 0; i < 16; ++i) m[i] = mf[i];
  /* Gauss-Jordan with partial pivoting on an augmented copy (independent of the product's cofactor form) */
  double A[4][8];
  for (int r = 0; r < 4; ++r) for (int c = 0; c < 8; ++c) A[r][c] = c < 4 ? m[r * 4 + c] : (c - 4 == r ? 1.0 : 0.0);
  for (int col = 0; col < 4; ++col) {
    int piv = col;
    for (int r = col + 1; r < 4; ++r) if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
    if (A[piv][col] == 0.0) { for (int i = 0; i < 16; ++i) out[i] = 0.0f; return; }
    if (piv != col) for (int c = 0; c < 8; ++c) { double t = A[col][c]; A[col][c] = A[piv][c]; A[piv][c] = t; }
    double d = A[col][col];
    for (int c = 0; c < 8; ++c) A[col][c] /= d;
    for (int r = 0; r < 4; ++r) if (r != col) { double f = A[r][col]; for (int c = 0; c < 8; ++c) A[r][c] -= f * A[col][c]; }
  }
  for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) a[r * 4 + c] = A[r][c + 4];
  for (int i = 0; i < 16; ++i) out[i] = (float)a[i];
}

/* UpdateCameraBuffer (src/D3D12HelloTriangle.cpp:1144-1170) */
void oracle_camera_buffer(const float view[16], uint32_t W, uint32_t H, float fov_deg, float zn, float zf, float cb[64]) {
  const float pi = 3.141592654f;
  float aspect = (float)W / (float)H;
  float fov = fov_deg * pi / 180.0f;
  float half = 0.5f * fov;
  float sn = (float)sin((double)half), cs = (float)cos((double)half);
  float h = cs / sn, w = h / aspect, fr = zf / (zn - zf);
  float proj[16] = {w, 0, 0, 0, 0, h, 0, 0, 0, 0, fr, -1.0f, 0, 0, fr * zn, 0};
  memcpy(cb, view, 64);
  memcpy(cb + 16, proj, 64);
  inv4(cb, cb + 32);
  inv4(cb + 16, cb + 48);
}

/* ---------------------------------------------------------------------------------------- */
/* LBVH (same algorithm as realtimeraytracing_gradproject_amd/csrc/rt_lbvh.hip)               */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
  float lo0[3], hi0[3], lo1[3], hi1[3];
  int32_t c0, c1;
  uint32_t pad0, pad1;
} onode; /* binary LBVH node: build intermediate */
/* traversal node: 4-wide, BFS order, SoA child boxes (== Bvh4Node of the device) */
#define O_EMPTY ((int32_t)(INT32_MIN + 1))
typedef struct {
  float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4];
  int32_t child[4];
  uint32_t count;
  int32_t first_inner; /* ref of the first internal child (consecutive refs in slot order), 0 if none */
  uint32_t inner_mask; /* bit k: child[k] >= 0 */
  uint32_t entry_base; /* first_inner << 8 | inner_mask << 4 (the device's packet-stack entry) */
} o4node;
typedef struct {
  float v0[3]; uint32_t prim;
  float e1[3]; uint32_t pad1;
  float e2[3]; uint32_t pad2;
} otri;

typedef struct {
  o4node* nodes;
  otri* tris; /* leaf order */
  float* vtx; /* {pos, normal} */
  uint32_t* idx; /* NULL for non-indexed */
  uint32_t ntri, nnodes, depth, nv, max_stack;
  float bounds[6];
} oblas;

typedef struct {
  float w2o[12], o2w[12], nrm[9];
  uint32_t instance_id, hit_group, blas;
  float face; /* +1, or -1 when the transform mirrors (front-face sense flipped for culling) */
  int translate; /* upper 3x3 exactly the identity: the object ray is (o + t, d) (InstanceRec::translate) */
} oinst;

struct oracle_scene {
  oblas* blas;
  int nblas, cblas;
  oinst* inst;
  uint32_t ninst;
  o4node* tlas;
  uint32_t tlas_nodes, tlas_depth, tlas_max_stack;
};

static uint32_t expand10(uint32_t x) {
  x = (x * 0x00010001u) & 0xFF0000FFu;
  x = (x * 0x00000101u) & 0x0F00F00Fu;
  x = (x * 0x00000011u) & 0xC30C30C3u;
  x = (x * 0x00000005u) & 0x49249249u;
  return x;
}

static int clz64(uint64_t v) { return v ? __builtin_clzll(v) : 64; }
static int odelta(const uint32_t* keys, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  uint64_t a = ((uint64_t)keys[i] << 32) | (uint32_t)i;
  uint64_t b = ((uint64_t)keys[j] << 32) | (uint32_t)j;
  return clz64(a ^ b);
}

static void box_of(int c, const float* nbox, const float* primbox, const uint32_t* sorted, float* b) {
  const float* p = c >= 0 ? nbox + (size_t)c * 6 : primbox + (size_t)sorted[~c] * 6;
  memcpy(b, p, 24);
}

/* builds nodes over n prim boxes; sorted receives leaf order; returns depth */
static float half_area(const float* b) {
  const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
  return (dx * dy + dy * dz) + dz * dx;
}

/* children of the 4-wide node rooted at binary node `root`: its two children, then the internal
 * candidate with the largest surface area (lowest slot on ties) is opened until there are four
 * (gather4 in rt_lbvh.hip) */
static int gather4(const onode* bin, int root, int ref[4], float box[4][6]) {
  const onode* b = &bin[root];
  ref[0] = b->c0;
  ref[1] = b->c1;
  for (int a = 0; a < 3; ++a) {
    box[0][a] = b->lo0[a]; box[0][3 + a] = b->hi0[a];
    box[1][a] = b->lo1[a]; box[1][3 + a] = b->hi1[a];
  }
  int cnt = 2;
  while (cnt < 4) {
    int best = -1;
    float bsa = 0.0f;
    for (int j = 0; j < cnt; ++j) {
      if (ref[j] < 0) continue;
      const float sa = half_area(box[j]);
      if (best < 0 || sa > bsa) { best = j; bsa = sa; }
    }
    if (best < 0) break;
    const onode* g = &bin[ref[best]];
    ref[best] = g->c0;
    ref[cnt] = g->c1;
    for (int a = 0; a < 3; ++a) {
      box[best][a] = g->lo0[a]; box[best][3 + a] = g->hi0[a];
      box[cnt][a] = g->lo1[a]; box[cnt][3 + a] = g->hi1[a];
    }
    ++cnt;
  }
  return cnt;
}

/* ---- SAH-optimal collapse (k_refit sah_dp + k_collapse gather4_dp in rt_lbvh.hip) -------------
 * cost(collapse) = sum of the half areas of its wide nodes: a wide node's visit tests all four
 * slots, and every triangle is tested under the same conditions in any collapse. C(n, i): least
 * cost of the subtree of binary node n as at most i slot roots; D(n, i) = min_j C(c0, j) +
 * C(c1, i - j); C(n, 1) = A(n) + D(n, 4); C(n, i) = min(C(n, 1), D(n, i)); ties keep the lowest j.
 * ORACLE_GREEDY_COLLAPSE=1 selects the earlier greedy largest-area opening (gather4) instead. */
static float* g_dpC;    /* [nbin][5] */
static int8_t* g_dpS;   /* [nbin][5]: 0 = n is a wide node, j > 0 = left gets j slots */
static int dp_on = -1;

static void dp_prepare(const onode* bin, uint32_t nbin) {
  g_dpC = (float*)malloc((size_t)nbin * 5 * sizeof(float));
  g_dpS = (int8_t*)malloc((size_t)nbin * 5);
  int* st = (int*)malloc((size_t)nbin * 2 * sizeof(int) + 8);
  int top = 0;
  st[top++] = 0;
  int* order = (int*)malloc((size_t)nbin * sizeof(int) + 4);
  int no = 0;
  while (top) {  /* pre-order, reversed below = children before parents */
    const int v = st[--top];
    order[no++] = v;
    if (bin[v].c0 >= 0) st[top++] = bin[v].c0;
    if (bin[v].c1 >= 0) st[top++] = bin[v].c1;
  }
  for (int q = no - 1; q >= 0; --q) {
    const int v = order[q];
    const onode* b = &bin[v];
    float bb[6];
    for (int a = 0; a < 3; ++a) {
      bb[a] = fminf(b->lo0[a], b->lo1[a]);
      bb[3 + a] = fmaxf(b->hi0[a], b->hi1[a]);
    }
    float cl[5], cr[5];
    for (int i = 1; i <= 4; ++i) {
      cl[i] = b->c0 >= 0 ? g_dpC[b->c0 * 5 + i] : 0.0f;
      cr[i] = b->c1 >= 0 ? g_dpC[b->c1 * 5 + i] : 0.0f;
    }
    float D[5];
    int8_t J[5];
    for (int i = 2; i <= 4; ++i) {
      D[i] = INFINITY; J[i] = 1;
      for (int j = 1; j < i; ++j) {
        const float c = cl[j] + cr[i - j];
        if (c < D[i]) { D[i] = c; J[i] = (int8_t)j; }
      }
    }
    const float self = half_area(bb) + D[4];
    g_dpC[v * 5 + 1] = self; g_dpS[v * 5 + 1] = 0;
    for (int i = 2; i <= 4; ++i) {
      if (D[i] < self) { g_dpC[v * 5 + i] = D[i]; g_dpS[v * 5 + i] = J[i]; }
      else { g_dpC[v * 5 + i] = self; g_dpS[v * 5 + i] = 0; }
    }
  }
  free(order); free(st);
}

/* slot roots of the subtree of binary ref c (leaf or internal) with k slots, left first */
static void dp_expand(const onode* bin, int c, const float* cbox, int k, int* ref, float (*box)[6], int* cnt) {
  if (c < 0 || g_dpS[c * 5 + k] == 0) {
    ref[*cnt] = c;
    memcpy(box[*cnt], cbox, 24);
    ++*cnt;
    return;
  }
  const onode* b = &bin[c];
  const int j = g_dpS[c * 5 + k];
  float l[6] = {b->lo0[0], b->lo0[1], b->lo0[2], b->hi0[0], b->hi0[1], b->hi0[2]};
  float r[6] = {b->lo1[0], b->lo1[1], b->lo1[2], b->hi1[0], b->hi1[1], b->hi1[2]};
  dp_expand(bin, b->c0, l, j, ref, box, cnt);
  dp_expand(bin, b->c1, r, k - j, ref, box, cnt);
}

/* BLAS: internal children first, stable (inner_first in rt_lbvh.hip); no visit order changes */
static void oinner_first(int cnt, int* ref, float (*box)[6]) {
  for (int x = 1; x < cnt; ++x)
    for (int y = x; y > 0 && ref[y] >= 0 && ref[y - 1] < 0; --y) {
      int tr = ref[y]; ref[y] = ref[y - 1]; ref[y - 1] = tr;
      float tb[6];
      memcpy(tb, box[y], 24); memcpy(box[y], box[y - 1], 24); memcpy(box[y - 1], tb, 24);
    }
}

static int gather4_dp(const onode* bin, int root, int ref[4], float box[4][6]) {
  const onode* b = &bin[root];
  /* root is a wide node: distribute its 4 slots as D(root, 4) chose */
  float cl[5], cr[5];
  for (int i = 1; i <= 4; ++i) {
    cl[i] = b->c0 >= 0 ? g_dpC[b->c0 * 5 + i] : 0.0f;
    cr[i] = b->c1 >= 0 ? g_dpC[b->c1 * 5 + i] : 0.0f;
  }
  int bj = 1;
  float bc = INFINITY;
  for (int jj = 1; jj < 4; ++jj) {
    const float c = cl[jj] + cr[4 - jj];
    if (c < bc) { bc = c; bj = jj; }
  }
  float l[6] = {b->lo0[0], b->lo0[1], b->lo0[2], b->hi0[0], b->hi0[1], b->hi0[2]};
  float r[6] = {b->lo1[0], b->lo1[1], b->lo1[2], b->hi1[0], b->hi1[1], b->hi1[2]};
  int cnt = 0;
  dp_expand(bin, b->c0, l, bj, ref, box, &cnt);
  dp_expand(bin, b->c1, r, 4 - bj, ref, box, &cnt);
  /* slots by ascending half area, stable (k_dp_expand) */
  for (int a = 1; a < cnt; ++a)
    for (int q = a; q > 0 && half_area(box[q]) < half_area(box[q - 1]); --q) {
      int tr = ref[q]; ref[q] = ref[q - 1]; ref[q - 1] = tr;
      float tb[6];
      memcpy(tb, box[q], 24); memcpy(box[q], box[q - 1], 24); memcpy(box[q - 1], tb, 24);
    }
  return cnt;
}

/* collapse the binary tree into 4-wide nodes (SAH DP, or greedy largest-area opening), BFS order
 * (k_collapse) */
static uint32_t collapse(const onode* bin, uint32_t nbin, o4node* out, uint32_t* count, uint32_t* max_stack,
                         int blas) {
#ifdef OSTUDY_BIN_HOOK /* design studies only (tools/wide_study.c): a copy of the binary tree */
  OSTUDY_BIN_HOOK(bin, nbin);
#endif
  if (dp_on < 0) dp_on = getenv("ORACLE_GREEDY_COLLAPSE") == NULL;
  if (dp_on) dp_prepare(bin, nbin);
  int* q = (int*)malloc((size_t)nbin * sizeof(int) + sizeof(int));
  int* ps = (int*)calloc((size_t)nbin + 1, sizeof(int)); /* siblings left on the stack above a node */
  int best = 0;
  int head = 0, tail = 1, level_end = 1;
  uint32_t depth = 0;
  q[0] = 0;
  while (head < level_end) {
    ++depth;
    for (; head < level_end; ++head) {
      int ref[4];
      float box[4][6];
      const int cnt = dp_on ? gather4_dp(bin, q[head], ref, box) : gather4(bin, q[head], ref, box);
      if (blas) oinner_first(cnt, ref, box);
      o4node nd;
      memset(&nd, 0, sizeof(nd));
      uint32_t valid = 0;
      for (int j = 0; j < 4; ++j) {
        int32_t r = O_EMPTY;
        /* unused slots: lo = hi = +inf, rejected by every slab test */
        nd.lox[j] = nd.loy[j] = nd.loz[j] = nd.hix[j] = nd.hiy[j] = nd.hiz[j] = INFINITY;
        if (j < cnt && ref[j] != O_EMPTY) {
          ++valid;
          nd.lox[j] = box[j][0]; nd.loy[j] = box[j][1]; nd.loz[j] = box[j][2];
          nd.hix[j] = box[j][3]; nd.hiy[j] = box[j][4]; nd.hiz[j] = box[j][5];
          if (ref[j] >= 0) {
            if (!nd.inner_mask) nd.first_inner = tail;
            nd.inner_mask |= 1u << j;
            q[tail] = ref[j]; r = tail; ps[tail] = ps[head] + cnt - 1; ++tail;
          }
          else r = ref[j];
        }
        nd.child[j] = r;
      }
      nd.count = valid;
      nd.entry_base = ((uint32_t)nd.first_inner << 8) | (nd.inner_mask << 4);
      if (ps[head] + cnt - 1 > best) best = ps[head] + cnt - 1;
      out[head] = nd;
    }
    level_end = tail;
  }
  *count = (uint32_t)tail;
  *max_stack = (uint32_t)best;
  free(ps);
  free(q);
  if (dp_on) { free(g_dpC); free(g_dpS); }
  return depth;
}

/* LBVH over n prim boxes -> 4-wide nodes (caller frees *out); returns levels */
static uint32_t lbvh(const float* primbox, uint32_t n, o4node** out4, uint32_t* count4, uint32_t* max_stack,
                     uint32_t* sorted, int leaf_ref_is_prim) {
  const uint32_t nbin = n > 1 ? n - 1 : 1;
  onode* nodes = (onode*)malloc((size_t)nbin * sizeof(onode));
  float cb[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) {
      float c = (primbox[i * 6 + k] + primbox[i * 6 + 3 + k]) * 0.5f;
      cb[k] = fmin2(cb[k], c);
      cb[3 + k] = fmax2(cb[3 + k], c);
    }
  uint32_t* keys = (uint32_t*)malloc((size_t)n * 4);
  uint32_t* k2 = (uint32_t*)malloc((size_t)n * 4);
  uint32_t* v2 = (uint32_t*)malloc((size_t)n * 4);
#ifdef ORACLE_STUDY_MORTON_CUBIC /* design study only (tools/morton_study.py): one scale for all axes */
  const float cext = fmaxf(fmaxf(cb[3] - cb[0], cb[4] - cb[1]), cb[5] - cb[2]);
#endif
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
#ifdef ORACLE_STUDY_MORTON_CUBIC
      float ext = cext;
#else
      float ext = cb[3 + k] - cb[k];
#endif
      float inv = ext > 0.0f ? 1.0f / ext : 0.0f;
      float c = (primbox[i * 6 + k] + primbox[i * 6 + 3 + k]) * 0.5f;
      float s = ((c - cb[k]) * inv) * 1024.0f;
      s = fminf(fmaxf(s, 0.0f), 1023.0f);
      q[k] = (uint32_t)s;
    }
    keys[i] = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    sorted[i] = i;
  }
  /* stable LSD counting sort, 4 x 8 bits */
  for (int pass = 0; pass < 4; ++pass) {
    int sh = pass * 8;
    uint32_t cnt[257];
    memset(cnt, 0, sizeof(cnt));
    for (uint32_t i = 0; i < n; ++i) cnt[((keys[i] >> sh) & 255u) + 1]++;
    for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t d = (keys[i] >> sh) & 255u;
      k2[cnt[d]] = keys[i];
      v2[cnt[d]] = sorted[i];
      cnt[d]++;
    }
    memcpy(keys, k2, (size_t)n * 4);
    memcpy(sorted, v2, (size_t)n * 4);
  }
  uint32_t depth = 1;
  if (n == 1) {
    onode nd;
    memset(&nd, 0, sizeof(nd));
    for (int k = 0; k < 3; ++k) {
      nd.lo0[k] = nd.lo1[k] = primbox[k];
      nd.hi0[k] = nd.hi1[k] = primbox[3 + k];
    }
    nd.c0 = ~0;
    nd.c1 = O_EMPTY;
    nodes[0] = nd;
  } else {
    int ni = (int)n - 1;
    int* child = (int*)malloc((size_t)ni * 8);
    int* pint = (int*)malloc((size_t)ni * 4);
    int* pleaf = (int*)malloc((size_t)n * 4);
    float* nbox = (float*)malloc((size_t)ni * 24);
    /* Karras 2012 (identical integer procedure to k_karras) */
    for (int i = 0; i < ni; ++i) {
      int d = (odelta(keys, (int)n, i, i + 1) - odelta(keys, (int)n, i, i - 1)) >= 0 ? 1 : -1;
      int dmin = odelta(keys, (int)n, i, i - d);
      int lmax = 2;
      while (odelta(keys, (int)n, i, i + lmax * d) > dmin) lmax <<= 1;
      int l = 0;
      for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (odelta(keys, (int)n, i, i + (l + t) * d) > dmin) l += t;
      int j = i + l * d;
      int dn = odelta(keys, (int)n, i, j);
      int s = 0, t = l;
      for (;;) {
        t = (t + 1) >> 1;
        if (odelta(keys, (int)n, i, i + (s + t) * d) > dn) s += t;
        if (t <= 1) break;
      }
      int g = i + s * d + (d < 0 ? d : 0);
      int lo = i < j ? i : j, hi = i < j ? j : i;
      int left = lo == g ? ~g : g, right = hi == g + 1 ? ~(g + 1) : g + 1;
      child[2 * i] = left;
      child[2 * i + 1] = right;
      if (left >= 0) pint[left] = i; else pleaf[~left] = i;
      if (right >= 0) pint[right] = i; else pleaf[~right] = i;
    }
    pint[0] = -1;
    /* refit: post-order over internal nodes (children before parents) */
    int* order = (int*)malloc((size_t)ni * 4);
    int* stack = (int*)malloc((size_t)ni * 4 + 4);
    int no = 0, sp = 0;
    stack[sp++] = 0;
    while (sp) {  /* pre-order, reversed later gives children-first for every parent */
      int v = stack[--sp];
      order[no++] = v;
      for (int k = 0; k < 2; ++k) if (child[2 * v + k] >= 0) stack[sp++] = child[2 * v + k];
    }
    for (int q = no - 1; q >= 0; --q) {
      int v = order[q];
      float a[6], b[6];
      box_of(child[2 * v], nbox, primbox, sorted, a);
      box_of(child[2 * v + 1], nbox, primbox, sorted, b);
      for (int k = 0; k < 3; ++k) {
        nbox[v * 6 + k] = fminf(a[k], b[k]);
        nbox[v * 6 + 3 + k] = fmaxf(a[3 + k], b[3 + k]);
      }
    }
    for (int i = 0; i < ni; ++i) {
      onode nd;
      int c[2] = {child[2 * i], child[2 * i + 1]};
      float b[2][6];
      for (int k = 0; k < 2; ++k) box_of(c[k], nbox, primbox, sorted, b[k]);
      for (int k = 0; k < 3; ++k) {
        nd.lo0[k] = b[0][k]; nd.hi0[k] = b[0][3 + k];
        nd.lo1[k] = b[1][k]; nd.hi1[k] = b[1][3 + k];
      }
      for (int k = 0; k < 2; ++k) if (c[k] < 0 && leaf_ref_is_prim) c[k] = ~(int)sorted[~c[k]];
      nd.c0 = c[0]; nd.c1 = c[1]; nd.pad0 = nd.pad1 = 0;
      nodes[i] = nd;
    }
    depth = 0;
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t d = 1;
      int node = pleaf[i];
      while (pint[node] >= 0) { node = pint[node]; ++d; }
      if (d > depth) depth = d;
    }
    free(order); free(stack); free(child); free(pint); free(pleaf); free(nbox);
  }
  free(keys); free(k2); free(v2);
  (void)depth;
  *out4 = (o4node*)malloc((size_t)nbin * sizeof(o4node));
  uint32_t levels = collapse(nodes, nbin, *out4, count4, max_stack, !leaf_ref_is_prim);
  free(nodes);
  return levels;
}

oracle_scene* oracle_scene_create(void) { return (oracle_scene*)calloc(1, sizeof(oracle_scene)); }

void oracle_scene_destroy(oracle_scene* s) {
  if (!s) return;
  for (int i = 0; i < s->nblas; ++i) {
    free(s->blas[i].nodes); free(s->blas[i].tris); free(s->blas[i].vtx); free(s->blas[i].idx);
  }
  free(s->blas); free(s->inst); free(s->tlas); free(s);
}

/* BottomLevelASGenerator semantics (nv_helpers_dx12/BottomLevelASGenerator.cpp:74-245) */
int oracle_add_blas(oracle_scene* s, const float* vtx6, uint32_t nv, const uint32_t* idx, uint32_t icount) {
  uint32_t ntri;
  if (!vtx6 || nv == 0) return -1;
  if (idx) {
    if (icount == 0 || icount % 3) return -1;
    for (uint32_t i = 0; i < icount; ++i) if (idx[i] >= nv) return -1;
    ntri = icount / 3;
  } else {
    if (nv % 3) return -1;
    ntri = nv / 3;
  }
  if (s->nblas == s->cblas) {
    s->cblas = s->cblas ? s->cblas * 2 : 4;
    s->blas = (oblas*)realloc(s->blas, (size_t)s->cblas * sizeof(oblas));
  }
  oblas* b = &s->blas[s->nblas];
  memset(b, 0, sizeof(*b));
  b->vtx = (float*)malloc((size_t)nv * 24);
  memcpy(b->vtx, vtx6, (size_t)nv * 24);
  if (idx) { b->idx = (uint32_t*)malloc((size_t)icount * 4); memcpy(b->idx, idx, (size_t)icount * 4); }
  b->nv = nv;
  b->ntri = ntri;
  float* box = (float*)malloc((size_t)ntri * 24);
  otri* un = (otri*)malloc((size_t)ntri * sizeof(otri));
  for (uint32_t p = 0; p < ntri; ++p) {
    uint32_t i0 = idx ? idx[3 * p] : 3 * p, i1 = idx ? idx[3 * p + 1] : 3 * p + 1, i2 = idx ? idx[3 * p + 2] : 3 * p + 2;
    const float *a = vtx6 + (size_t)i0 * 6, *bb = vtx6 + (size_t)i1 * 6, *c = vtx6 + (size_t)i2 * 6;
    otri t;
    for (int k = 0; k < 3; ++k) {
      t.v0[k] = a[k]; t.e1[k] = bb[k] - a[k]; t.e2[k] = c[k] - a[k];
      box[p * 6 + k] = fminf(fminf(a[k], bb[k]), c[k]) + 0.0f; /* canonical +0 */
      box[p * 6 + 3 + k] = fmaxf(fmaxf(a[k], bb[k]), c[k]) + 0.0f;
    }
    t.prim = p; t.pad1 = t.pad2 = 0;
    un[p] = t;
  }
  uint32_t* sorted = (uint32_t*)malloc((size_t)ntri * 4);
  b->depth = lbvh(box, ntri, &b->nodes, &b->nnodes, &b->max_stack, sorted, 0);
  b->tris = (otri*)malloc((size_t)ntri * sizeof(otri));
  for (uint32_t i = 0; i < ntri; ++i) b->tris[i] = un[sorted[i]];
  for (int k = 0; k < 3; ++k) { b->bounds[k] = INFINITY; b->bounds[3 + k] = -INFINITY; }
  for (uint32_t p = 0; p < ntri; ++p)
    for (int k = 0; k < 3; ++k) {
      b->bounds[k] = fminf(b->bounds[k], box[p * 6 + k]);
      b->bounds[3 + k] = fmaxf(b->bounds[3 + k], box[p * 6 + 3 + k]);
    }
  free(box); free(un); free(sorted);
  return s->nblas++;
}

static int inv3d(const double m[9], double inv[9]) {
  double c00 = m[4] * m[8] - m[5] * m[7];
  double c01 = m[5] * m[6] - m[3] * m[8];
  double c02 = m[3] * m[7] - m[4] * m[6];
  double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  if (det == 0.0) return 0;
  double r = 1.0 / det;
  inv[0] = c00 * r; inv[1] = (m[2] * m[7] - m[1] * m[8]) * r; inv[2] = (m[1] * m[5] - m[2] * m[4]) * r;
  inv[3] = c01 * r; inv[4] = (m[0] * m[8] - m[2] * m[6]) * r; inv[5] = (m[2] * m[3] - m[0] * m[5]) * r;
  inv[6] = c02 * r; inv[7] = (m[1] * m[6] - m[0] * m[7]) * r; inv[8] = (m[0] * m[4] - m[1] * m[3]) * r;
  return 1;
}

static vec3 xpoint(const float* m, vec3 p) {
  return mk(((m[0] * p.x + m[1] * p.y) + m[2] * p.z) + m[3], ((m[4] * p.x + m[5] * p.y) + m[6] * p.z) + m[7],
            ((m[8] * p.x + m[9] * p.y) + m[10] * p.z) + m[11]);
}
static vec3 xdir(const float* m, vec3 d) {
  return mk((m[0] * d.x + m[1] * d.y) + m[2] * d.z, (m[4] * d.x + m[5] * d.y) + m[6] * d.z,
            (m[8] * d.x + m[9] * d.y) + m[10] * d.z);
}
/* world -> object ray of an instance (inst_point / inst_dir in rt_device.hpp) */
static vec3 ipoint(const oinst* ir, vec3 p) {
  return ir->translate ? mk(p.x + ir->w2o[3], p.y + ir->w2o[7], p.z + ir->w2o[11]) : xpoint(ir->w2o, p);
}
static vec3 idir(const oinst* ir, vec3 d) { return ir->translate ? d : xdir(ir->w2o, d); }
static vec3 m3mul(const float* m, vec3 d) {
  return mk((m[0] * d.x + m[1] * d.y) + m[2] * d.z, (m[3] * d.x + m[4] * d.y) + m[5] * d.z,
            (m[6] * d.x + m[7] * d.y) + m[8] * d.z);
}

/* TopLevelASGenerator (nv_helpers_dx12/TopLevelASGenerator.cpp:64-249) +
 * UpdateInstancePropertiesBuffer (src/D3D12HelloTriangle.cpp:1181-1204) */
int oracle_set_instances(oracle_scene* s, const oracle_instance* in, uint32_t n) {
  if (!n) return -1;
  free(s->inst); free(s->tlas);
  s->inst = (oinst*)calloc(n, sizeof(oinst));
  s->ninst = n;
  float* box = (float*)malloc((size_t)n * 24);
  for (uint32_t i = 0; i < n; ++i) {
    if ((int)in[i].blas >= s->nblas) return -1;
    oinst* r = &s->inst[i];
    const float* M = in[i].xform;
    double L[9] = {M[0], M[1], M[2], M[4], M[5], M[6], M[8], M[9], M[10]}, Li[9];
    if (!inv3d(L, Li)) return -1;
    const double det = L[0] * (L[4] * L[8] - L[5] * L[7]) + L[1] * (L[5] * L[6] - L[3] * L[8]) +
                       L[2] * (L[3] * L[7] - L[4] * L[6]);
    r->face = det < 0.0 ? -1.0f : 1.0f;
    r->translate = M[0] == 1.0f && M[1] == 0.0f && M[2] == 0.0f && M[4] == 0.0f && M[5] == 1.0f && M[6] == 0.0f &&
                   M[8] == 0.0f && M[9] == 0.0f && M[10] == 1.0f;
    double t[3] = {M[3], M[7], M[11]};
    for (int a = 0; a < 3; ++a) {
      r->w2o[a * 4 + 0] = (float)Li[a * 3 + 0];
      r->w2o[a * 4 + 1] = (float)Li[a * 3 + 1];
      r->w2o[a * 4 + 2] = (float)Li[a * 3 + 2];
      r->w2o[a * 4 + 3] = (float)(-(Li[a * 3 + 0] * t[0] + Li[a * 3 + 1] * t[1] + Li[a * 3 + 2] * t[2]));
    }
    memcpy(r->o2w, M, 48);
    for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) r->nrm[a * 3 + b] = (float)Li[b * 3 + a];
    r->instance_id = in[i].instance_id;
    r->hit_group = in[i].hit_group;
    r->blas = in[i].blas;
    const float* bb = s->blas[in[i].blas].bounds;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int c = 0; c < 8; ++c) {
      vec3 p = mk((c & 1) ? bb[3] : bb[0], (c & 2) ? bb[4] : bb[1], (c & 4) ? bb[5] : bb[2]);
      vec3 w = xpoint(M, p);
      lo[0] = fminf(lo[0], w.x); lo[1] = fminf(lo[1], w.y); lo[2] = fminf(lo[2], w.z);
      hi[0] = fmaxf(hi[0], w.x); hi[1] = fmaxf(hi[1], w.y); hi[2] = fmaxf(hi[2], w.z);
    }
    for (int k = 0; k < 3; ++k) { box[i * 6 + k] = lo[k] + 0.0f; box[i * 6 + 3 + k] = hi[k] + 0.0f; }
  }
  uint32_t* sorted = (uint32_t*)malloc((size_t)n * 4);
  s->tlas_depth = lbvh(box, n, &s->tlas, &s->tlas_nodes, &s->tlas_max_stack, sorted, 1);
  free(sorted); free(box);
  return 0;
}

int oracle_blas_info(const oracle_scene* s, int b, uint32_t out[4]) {
  if (b < 0 || b >= s->nblas) return -1;
  out[0] = s->blas[b].ntri; out[1] = s->blas[b].nnodes; out[2] = s->blas[b].depth; out[3] = s->blas[b].max_stack;
  return 0;
}
int oracle_tlas_info(const oracle_scene* s, uint32_t out[4]) {
  if (!s->tlas) return -1;
  out[0] = s->ninst; out[1] = s->tlas_nodes; out[2] = s->tlas_depth; out[3] = s->tlas_max_stack;
  return 0;
}
int oracle_export_blas(const oracle_scene* s, int b, void* nodes, void* tris) {
  if (b < 0 || b >= s->nblas) return -1;
  if (nodes) memcpy(nodes, s->blas[b].nodes, (size_t)s->blas[b].nnodes * sizeof(o4node));
  if (tris) memcpy(tris, s->blas[b].tris, (size_t)s->blas[b].ntri * sizeof(otri));
  return 0;
}
int oracle_export_tlas(const oracle_scene* s, void* nodes) {
  if (!s->tlas) return -1;
  memcpy(nodes, s->tlas, (size_t)s->tlas_nodes * sizeof(o4node));
  return 0;
}

/* ---------------------------------------------------------------------------------------- */
/* traversal: DXR TraceRay semantics (closest hit / any hit), Common.hlsl:44-82               */
/* ---------------------------------------------------------------------------------------- */
/* v[0..8] = RT_STAT_* 0..8; v[9..11] record fetches (RT_STAT_NODE/TRI/INSTANCE_FETCHES): per ray in
 * otrace, once per emulated wave in opacket */
typedef struct { uint64_t v[12]; } ostats;
/* Counters: the checker build counts every test and fetch (compared with the device's). The CPU
 * baseline build (-DORACLE_NO_COUNTERS -O3, oracle/libbaseline.so: BASELINE.md section 3's scalar
 * traversal without counters) compiles them out; its frames are identical. */
#ifdef ORACLE_NO_COUNTERS
#define OST(i, n) ((void)0)
#else
#define OST(i, n) (st->v[i] += (n))
#endif
typedef struct { float t, u, v; uint32_t inst, prim; } ohit;

static inline float sinv(float d) { return fabsf(d) > 1e-20f ? 1.0f / d : (d < 0.0f ? -1e20f : 1e20f); }

/* slab tests of the 4 children of a node against [tmin, tbest]; +inf = missed or empty */
/* The slab operands are never NaN (finite origins, safe_inv never 0 or inf, +-inf planes of empty slots
 * times a finite inverse), and the sign of a zero min/max never changes a comparison or a key (keys drop the
 * sign bit), so the CPU baseline build may use plain compares (minss / maxss) instead of the libm calls
 * gcc emits for fminf / fmaxf without -ffast-math. Same frames (tests/test_oracle.py). */
#ifdef ORACLE_NO_COUNTERS
#define OMINF(a, b) ((a) < (b) ? (a) : (b))
#define OMAXF(a, b) ((a) > (b) ? (a) : (b))
#else
#define OMINF(a, b) fminf(a, b)
#define OMAXF(a, b) fmaxf(a, b)
#endif
static inline void oslab4(const o4node* nd, vec3 invd, vec3 noinv, float tmin, float tbest, float tn[4]) {
  for (int k = 0; k < 4; ++k) {
    float tlx = fmaf(nd->lox[k], invd.x, noinv.x), thx = fmaf(nd->hix[k], invd.x, noinv.x);
    float tly = fmaf(nd->loy[k], invd.y, noinv.y), thy = fmaf(nd->hiy[k], invd.y, noinv.y);
    float tlz = fmaf(nd->loz[k], invd.z, noinv.z), thz = fmaf(nd->hiz[k], invd.z, noinv.z);
    float n = OMAXF(OMAXF(OMINF(tlx, thx), OMINF(tly, thy)), OMAXF(OMINF(tlz, thz), tmin));
    float f = OMINF(OMINF(OMAXF(tlx, thx), OMAXF(tly, thy)), OMINF(OMAXF(tlz, thz), tbest));
    tn[k] = (nd->child[k] != O_EMPTY && n <= f * 1.0000004f) ? n : INFINITY;
  }
}

/* nearest-first order: comparator network (0,1)(2,3)(0,2)(1,3)(1,2), swap only when strictly nearer */
static inline void ocswap(float* t, int32_t* r, int a, int b) {
  if (t[b] < t[a]) { float tt = t[a]; t[a] = t[b]; t[b] = tt; int32_t rr = r[a]; r[a] = r[b]; r[b] = rr; }
}
static inline void osort4(float* t, int32_t* r) {
  ocswap(t, r, 0, 1); ocswap(t, r, 2, 3); ocswap(t, r, 0, 2); ocswap(t, r, 1, 3); ocswap(t, r, 1, 2);
}

/* Moller-Trumbore (the ray/triangle test DXR performs in hardware; formula pinned here).
 * face 0: both sides; +1/-1: RAY_FLAG_CULL_BACK_FACING_TRIANGLES, front = det * face > 0
 * (clockwise seen from the ray origin, DXR's default; face = -1 under a mirroring transform). */
/* The test's cross products are pinned as fused multiply-adds (C99 fmaf rounds once, exactly as the GPU's
 * v_fma_f32): cross_x = fma(a.y, b.z, -(a.z * b.y)) ...; its dot products stay unfused, (x + y) + z
 * (rt_device.hpp RT_MT_FMA: fused dots would raise the seam-probe leak count by ~40%). */
static inline float omt_dot(vec3 a, vec3 b) { return vdot(a, b); }
static inline vec3 omt_cross(vec3 a, vec3 b) {
  return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline int omt(vec3 o, vec3 d, const otri* tr, float face, float* t, float* u, float* v) {
  vec3 v0 = ld3(tr->v0), e1 = ld3(tr->e1), e2 = ld3(tr->e2);
  vec3 p = omt_cross(d, e2);
  float det = omt_dot(e1, p);
  if (det == 0.0f || det * face < 0.0f) return 0;
  float inv = 1.0f / det;
  vec3 s = vsub(o, v0);
  *u = omt_dot(s, p) * inv;
  if (!(*u >= 0.0f && *u <= 1.0f)) return 0;
  vec3 q = omt_cross(s, e1);
  *v = omt_dot(d, q) * inv;
  if (!(*v >= 0.0f && *u + *v <= 1.0f)) return 0;
  *t = omt_dot(e2, q) * inv;
  return 1;
}

static inline int better(float t, uint32_t inst, uint32_t prim, const ohit* h) {
  return t < h->t || (t == h->t && (inst < h->inst || (inst == h->inst && prim < h->prim)));
}

#define SENT INT32_MIN

/* deepest per-ray stack reached by otrace since the last reset (diagnostics for tests: a scene meant to
 * exercise the device's HBM overflow stack must really reach past its 32 LDS entries; racy across
 * render threads, read it after single-threaded renders) */
static int g_max_sp = 0;
#ifndef ORACLE_FLAGS
#define ORACLE_FLAGS "unknown"
#endif
/* compiler and flags of this build (bench.py's cpu_baseline reports them) */
const char* oracle_build_info(void) { return "gcc " __VERSION__ " " ORACLE_FLAGS; }
int oracle_max_stack_reached(int reset) { int m = g_max_sp; if (reset) g_max_sp = 0; return m; }
#ifdef ORACLE_NO_COUNTERS
#define OSP_TRACK() ((void)0)
#else
#define OSP_TRACK() do { if (sp > g_max_sp) g_max_sp = sp; } while (0)
#endif
#define OPUSH(X) do { if (sp < cap) { stack[sp++] = (X); OSP_TRACK(); } else OST(5, 1); } while (0)

static int otrace(const oracle_scene* s, vec3 o, vec3 d, float tmin, float tmax, int any, int cull, ohit* h,
                  ostats* st) {
  int stack[256];
  uint32_t maxb = 0;
  for (int b = 0; b < s->nblas; ++b) if (s->blas[b].max_stack > maxb) maxb = s->blas[b].max_stack;
  int cap = (int)(s->tlas_max_stack + 1 + maxb); /* same exact bound as the device (rt_api.cpp) */
  if (cap > 256) cap = 256;
  vec3 winvd = mk(sinv(d.x), sinv(d.y), sinv(d.z));
  vec3 wno = vneg(vmul(o, winvd));
  vec3 ro = o, rd = d, rinvd = winvd, rno = wno;
  const o4node* nodes = s->tlas;
  const otri* tris = NULL;
  uint32_t cur = 0;
  int in_blas = 0, found = 0, sp = 0, ref = 0;
  h->t = tmax; h->inst = 0xffffffffu; h->prim = 0xffffffffu; h->u = h->v = 0.0f;
  for (;;) {
    if (ref >= 0) {
      const o4node* nd = nodes + ref;
      float tn[4];
      int32_t r[4] = {nd->child[0], nd->child[1], nd->child[2], nd->child[3]};
      oslab4(nd, rinvd, rno, tmin, h->t, tn);
      OST(9, 1);
      for (int k = 0; k < 4; ++k) OST(2, r[k] != O_EMPTY);
      osort4(tn, r);
      if (tn[0] != INFINITY) {
        if (tn[3] != INFINITY) OPUSH(r[3]);
        if (tn[2] != INFINITY) OPUSH(r[2]);
        if (tn[1] != INFINITY) OPUSH(r[1]);
        ref = r[0];
        continue;
      }
    } else if (!in_blas) {
      cur = (uint32_t)(~ref);
      const oinst* ir = &s->inst[cur];
      OST(4, 1);
      OST(11, 1);
      if (sp < cap) {
        stack[sp++] = SENT;
        OSP_TRACK();
        ro = ipoint(ir, o);
        rd = idir(ir, d);
        rinvd = mk(sinv(rd.x), sinv(rd.y), sinv(rd.z));
        rno = vneg(vmul(ro, rinvd));
        nodes = s->blas[ir->blas].nodes;
        tris = s->blas[ir->blas].tris;
        in_blas = 1;
        ref = 0;
        continue;
      }
      OST(5, 1);
    } else {
      const otri* tr = tris + (~ref);
      float t, u, v;
      OST(3, 1);
      OST(10, 1);
      if (omt(ro, rd, tr, cull ? (float)cull * s->inst[cur].face : 0.0f, &t, &u, &v) && t >= tmin && better(t, cur, tr->prim, h)) {
        h->t = t; h->u = u; h->v = v; h->inst = cur; h->prim = tr->prim;
        found = 1;
        if (any) return 1;
      }
    }
    for (;;) {
      if (sp == 0) return found;
      ref = stack[--sp];
      if (ref != SENT) break;
      in_blas = 0; nodes = s->tlas; ro = o; rd = d; rinvd = winvd; rno = wno;
    }
  }
}

/* ---------------------------------------------------------------------------------------- */
/* Wave-packet traversal (trace_packet in rt_trace.hip): the 64 lanes of a wave walk one path */
/* together; a child is entered when any live lane's slab test accepts it. Emulated lane by   */
/* lane so the traversal order and the per-lane counters are those of the device.            */
/* ---------------------------------------------------------------------------------------- */
#ifndef OPK
#define OPK 64 /* lanes of an emulated packet (design studies may build 128: two rays per lane) */
#endif
#define OSTACK 4096 /* emulated per-child stack: its bound is at most 3 entries per tree level */

typedef struct {
  vec3 o[OPK], d[OPK], invd[OPK], no[OPK];
} opkray;

static uint32_t f2bits(float x) { uint32_t b; memcpy(&b, &x, 4); return b; }

static int olead(const int* live) {
  for (int l = 0; l < OPK; ++l) if (live[l]) return l;
  return -1;
}

/* one node (packet_node in rt_trace.hip): returns 1 with *next set, 0 when nothing is left to
 * descend into, 2 when an any-hit packet has no live lane left. leaves != NULL (BLAS level):
 * entered triangle children are tested here, in slot order, and never pushed. */
static int opk_node(const o4node* nd, const opkray* ry, float tmin, ohit* h, int* live, int* lead,
                    const otri* leaves, uint32_t cur, float face, int any, int* found, int* stack, int* sp,
                    int cap, int* next, ostats* st) {
  uint64_t hm[4] = {0, 0, 0, 0}; /* ballots (OPK <= 64; wider study builds use acc below) */
  uint8_t acc[OPK][4];           /* lane l's own slab test accepts child k (live lanes only) */
  uint32_t vkey[OPK][4];
  OST(9, 1); /* one node fetch per wave */
#ifdef OSTUDY_NODE_HOOK /* design studies only (tools/path_study.c): node fetches by tree level and ray kind */
  OSTUDY_NODE_HOOK(leaves != NULL, any);
#endif
  for (int l = 0; l < OPK; ++l) {
    for (int k = 0; k < 4; ++k) {
      float tlx = fmaf(nd->lox[k], ry->invd[l].x, ry->no[l].x), thx = fmaf(nd->hix[k], ry->invd[l].x, ry->no[l].x);
      float tly = fmaf(nd->loy[k], ry->invd[l].y, ry->no[l].y), thy = fmaf(nd->hiy[k], ry->invd[l].y, ry->no[l].y);
      float tlz = fmaf(nd->loz[k], ry->invd[l].z, ry->no[l].z), thz = fmaf(nd->hiz[k], ry->invd[l].z, ry->no[l].z);
      float n = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), tmin));
      float f = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), h[l].t));
      int hit = n <= f * 1.0000004f; /* empty slots hold +inf boxes: never accepted */
      acc[l][k] = (uint8_t)(hit && live[l]);
      if (hit && live[l] && l < 64) hm[k] |= 1ull << l;
#ifdef OCLOSEST_KEY /* design studies only (tools/key_study.c): another nearest-first key */
      vkey[l][k] = hit ? OCLOSEST_KEY(n, f) : 0x7f800000u;
#else
      vkey[l][k] = hit ? (f2bits(n) & 0x7fffffffu) : 0x7f800000u;
#endif
    }
    if (live[l]) OST(2, nd->count);
  }
  uint32_t ent = 0;
  for (int l = 0; l < OPK; ++l)
    for (int k = 0; k < 4; ++k) if (acc[l][k]) ent |= 1u << k;
  if (!ent) return 0;
  if (leaves) {
    uint32_t leafbits = 0;
    for (int k = 0; k < 4; ++k) if (nd->child[k] < 0) leafbits |= 1u << k;
    const uint32_t tl = ent & leafbits;
    ent &= ~leafbits;
    for (int k = 0; k < 4; ++k) {
      if (!((tl >> k) & 1u)) continue;
      const otri* tr = leaves + (~nd->child[k]);
      OST(10, 1); /* one triangle fetch per wave */
      for (int l = 0; l < OPK; ++l) {
        if (!live[l]) continue;
        float t, u, v;
        OST(3, 1);
        /* only a lane whose own slab test accepted the triangle's slot may take the hit (packet_tri's own mask) */
        if (acc[l][k] && omt(ry->o[l], ry->d[l], tr, face, &t, &u, &v) && t >= tmin &&
            better(t, cur, tr->prim, &h[l])) {
          h[l].t = t; h[l].u = u; h[l].v = v; h[l].inst = cur; h[l].prim = tr->prim;
          found[l] = 1;
          if (any) live[l] = 0;
        }
      }
    }
    if (any) {
      *lead = olead(live);
      if (*lead < 0) return 2;
      for (int k = 0; k < 4; ++k) {
        int keep = 0;
        for (int l = 0; l < OPK; ++l) keep |= acc[l][k] && live[l];
        if (!keep) ent &= ~(1u << k);
      }
    }
    if (!ent) return 0;
  }
  uint32_t key[4];
  for (int k = 0; k < 4; ++k) key[k] = ((ent >> k) & 1u) ? vkey[*lead][k] : 0xffffffffu;
  /* nearest first (lowest slot on ties), the other entered children pushed in descending slot order;
   * any-hit nodes skip the distance order: the lowest entered slot goes first */
  uint32_t kb = key[0];
  int rb = nd->child[0], ib = 0;
  if (any) {
#ifdef OANY_CHOOSE /* design studies only (tools/anyhit_study.c): another any-hit child order */
    ib = OANY_CHOOSE(ent, vkey, *lead, hm, live, nd, tmin);
#else
    ib = __builtin_ctz(ent);
#endif
    rb = nd->child[ib];
  } else {
    for (int k = 1; k < 4; ++k)
      if (key[k] < kb) { kb = key[k]; rb = nd->child[k]; ib = k; }
  }
  const uint32_t P = ent & ~(1u << ib);
  if (*sp + __builtin_popcount(P) > cap) /* never: cap is the exact worst case; counted per live lane */
    for (int l = 0; l < OPK; ++l) OST(5, live[l] ? 1u : 0u);
  for (int k = 3; k >= 0; --k) {
    if (!((P >> k) & 1u)) continue;
    if (*sp < OSTACK) stack[*sp] = nd->child[k];
    ++*sp;
  }
  *next = rb;
  return 1;
}

static void opacket(const oracle_scene* s, const vec3* o, const vec3* d, float tmin, float tmax, int any,
                    int cull, const int* alive, ohit* h, int* found, ostats* st) {
  int live[OPK];
  opkray w, b;
#ifdef OSTUDY_PACKET_HOOK /* design studies only (tools/refl_study.c): packet occupancy */
  OSTUDY_PACKET_HOOK(any, cull, alive);
#endif
  for (int l = 0; l < OPK; ++l) {
    live[l] = alive[l];
    found[l] = 0;
    h[l].t = tmax; h[l].inst = 0xffffffffu; h[l].prim = 0xffffffffu; h[l].u = h[l].v = 0.0f;
    w.o[l] = o[l]; w.d[l] = d[l];
    w.invd[l] = mk(sinv(d[l].x), sinv(d[l].y), sinv(d[l].z));
    w.no[l] = vneg(vmul(o[l], w.invd[l]));
  }
  int lead = olead(live);
  if (lead < 0) return;
  uint32_t maxb = 0;
  for (int q = 0; q < s->nblas; ++q) if (s->blas[q].max_stack > maxb) maxb = s->blas[q].max_stack;
  /* per-child entries: the exact bound of this (emulated) stack; the device keeps one entry per
   * BLAS node with pending children, an order-preserving compression of the same stack */
  const int cap = (int)(s->tlas_max_stack + 1 + maxb);
  int stack[OSTACK];
  int sp = 0, ref = 0, next;
  for (;;) {
    if (ref >= 0) {
      if (opk_node(s->tlas + ref, &w, tmin, h, live, &lead, NULL, 0u, 0.0f, any, found, stack, &sp, cap, &next,
                   st) == 1) {
        ref = next;
        continue;
      }
    } else {
      const uint32_t cur = (uint32_t)(~ref);
      const oinst* ir = &s->inst[cur];
      const oblas* bl = &s->blas[ir->blas];
      OST(11, 1); /* one instance-record fetch per wave */
      for (int l = 0; l < OPK; ++l) {
        if (live[l]) OST(4, 1);
        b.o[l] = ipoint(ir, o[l]);
        b.d[l] = idir(ir, d[l]);
        b.invd[l] = mk(sinv(b.d[l].x), sinv(b.d[l].y), sinv(b.d[l].z));
        b.no[l] = vneg(vmul(b.o[l], b.invd[l]));
      }
      const int base = sp;
      int bref = 0;
      for (;;) {
        /* only internal nodes reach here: triangle children are tested inside opk_node */
        const int r = opk_node(bl->nodes + bref, &b, tmin, h, live, &lead, bl->tris, cur, cull ? (float)cull * ir->face : 0.0f,
                               any, found, stack, &sp, cap, &next, st);
        if (r == 1) { bref = next; continue; }
        if (r == 2) return;
        if (sp == base) break;
        bref = stack[--sp];
      }
    }
    if (sp == 0) return;
    ref = stack[--sp];
  }
}

/* every triangle of every instance, original primitive order */
static int obrute(const oracle_scene* s, vec3 o, vec3 d, float tmin, float tmax, int any, int cull, ohit* h,
                  ostats* st) {
  int found = 0;
  h->t = tmax; h->inst = 0xffffffffu; h->prim = 0xffffffffu; h->u = h->v = 0.0f;
  for (uint32_t i = 0; i < s->ninst; ++i) {
    const oinst* ir = &s->inst[i];
    const oblas* b = &s->blas[ir->blas];
    vec3 ro = ipoint(ir, o), rd = idir(ir, d);
    for (uint32_t k = 0; k < b->ntri; ++k) {
      const otri* tr = &b->tris[k];
      float t, u, v;
      OST(3, 1);
      if (omt(ro, rd, tr, cull ? (float)cull * ir->face : 0.0f, &t, &u, &v) && t >= tmin && better(t, i, tr->prim, h)) {
        h->t = t; h->u = u; h->v = v; h->inst = i; h->prim = tr->prim;
        found = 1;
        if (any) return 1;
      }
    }
  }
  return found;
}

/* ---------------------------------------------------------------------------------------- */
/* shading (shaders/Hit.hlsl, Miss.hlsl, ShadowRay.hlsl)                                     */
/* ---------------------------------------------------------------------------------------- */
static float olog2(float x) {
  uint32_t b; memcpy(&b, &x, 4);
  int e = (int)((b >> 23) & 0xffu) - 127;
  uint32_t mb = (b & 0x7fffffu) | 0x3f800000u;
  float m; memcpy(&m, &mb, 4);
  if (m > 1.41421356f) { m = m * 0.5f; e = e + 1; }
  float f = m - 1.0f;
  float s = f * (1.0f / (2.0f + f)); /* the device's rcp_exact(2 + f) */
  float s2 = s * s;
  float p = 1.0f / 11.0f;
  p = p * s2 + 1.0f / 9.0f;
  p = p * s2 + 1.0f / 7.0f;
  p = p * s2 + 1.0f / 5.0f;
  p = p * s2 + 1.0f / 3.0f;
  p = p * s2 + 1.0f;
  float ln = (2.0f * s) * p;
  return (float)e + ln * 1.44269504f;
}
static float oexp2(float y) {
  if (y < -126.0f) return 0.0f;
  if (y > 127.0f) y = 127.0f;
  float fi = floorf(y + 0.5f);
  float f = y - fi;
  float a = f * 0.693147181f;
  float p = 1.0f / 40320.0f;
  p = p * a + 1.0f / 5040.0f;
  p = p * a + 1.0f / 720.0f;
  p = p * a + 1.0f / 120.0f;
  p = p * a + 1.0f / 24.0f;
  p = p * a + 1.0f / 6.0f;
  p = p * a + 0.5f;
  p = p * a + 1.0f;
  p = p * a + 1.0f;
  int i = (int)fi;
  uint32_t sb = (uint32_t)(i + 127) << 23;
  float sc; memcpy(&sc, &sb, 4);
  return p * sc;
}
/* HLSL pow(x, y) for x >= 0, pinned to a deterministic exp2(y log2 x) */
float oracle_pow(float x, float y) { if (!(x > 1e-30f)) return 0.0f; return oexp2(y * olog2(x)); }

static const float OPI = 3.14159265359f; /* Common.hlsl:1 */

/* ClosestHit's finalSurfaceColor = CalculateDirectLighting (Hit.hlsl:83-95) + CalculatePBRShading
 * (:97-174, FresnelSchlick :97-100, GGX :102-113, SchlickGGX :115-122, Smith :124-130), in the pinned
 * float32 form of the device's surface_ref (csrc/rt_trace.hip, round 6): one loop over the lights
 * (the direct term's -normalize(lp - P) and the PBR term's L and distance share one sqrt and one
 * reciprocal), pixel and material invariants out of the loop, each quotient a product with the
 * IEEE reciprocal 1.0f / x (the device's rcp_exact gives the same bits), the diffuse term
 * (1 - F) * ((1 - metallic) albedo / PI). The two sums keep their own accumulators and light order. */
static void osurface(vec3 P, vec3 n, vec3 cam, const oracle_light* Ls, uint32_t nl, const float* mat,
                     vec3* direct, vec3* pbr) {
  vec3 albedo = ld3(mat);
  float rough = mat[3], metal = mat[4];
  float a = rough * rough, a2 = a * a;
  float rp1 = rough + 1.0f;
  float k = (rp1 * rp1) / 8.0f;
  float omk = 1.0f - k;
  vec3 F0 = mk(0.04f + metal * (albedo.x - 0.04f), 0.04f + metal * (albedo.y - 0.04f), 0.04f + metal * (albedo.z - 0.04f));
  float km = 1.0f - metal;
  vec3 kdA = mk((km * albedo.x) / OPI, (km * albedo.y) / OPI, (km * albedo.z) / OPI);
  vec3 N = vneg(vscale(n, 1.0f / sqrtf(vdot(n, n))));
  vec3 Vd = vsub(cam, P);
  vec3 V = vscale(Vd, 1.0f / sqrtf(vdot(Vd, Vd)));
  float NdotV = fmax2(vdot(N, V), 0.0f);
  float ggx2 = NdotV * (1.0f / (NdotV * omk + k));
  float v4 = 4.0f * NdotV;
  vec3 cd = mk(0, 0, 0), L0 = mk(0, 0, 0);
  for (uint32_t l = 0; l < nl; ++l) {
    vec3 lp = ld3(Ls[l].position), lc = ld3(Ls[l].color);
    vec3 dv = vsub(lp, P);
    float dist = sqrtf(vdot(dv, dv));
    vec3 L = vscale(dv, 1.0f / dist);
    float ti = fmax2(0.0f, vdot(n, vneg(L)) * Ls[l].intensity);
    cd = vadd(cd, vscale(vmul(albedo, lc), ti));
    vec3 Hd = vadd(V, L);
    vec3 H = vscale(Hd, 1.0f / sqrtf(vdot(Hd, Hd)));
    float att = 1.0f / fmax2(dist * dist, 1.0f);
    vec3 radiance = vscale(lc, att);
    float x = 1.0f - fmax2(vdot(H, V), 0.0f);
    x = fmin2(fmax2(x, 0.0f), 1.0f);
    float x5 = ((x * x) * (x * x)) * x;
    vec3 F = mk(F0.x + (1.0f - F0.x) * x5, F0.y + (1.0f - F0.y) * x5, F0.z + (1.0f - F0.z) * x5);
    float NdotH = fmax2(vdot(N, H), 0.0f);
    float NdotH2 = NdotH * NdotH;
    float denom = NdotH2 * (a2 - 1.0f) + 1.0f;
    denom = (OPI * denom) * denom;
    float NDF = a2 * (1.0f / denom);
    float NdotL = fmax2(vdot(N, L), 0.0f);
    float ggx1 = NdotL * (1.0f / (NdotL * omk + k));
    float G = ggx1 * ggx2;
    float sp = (NDF * G) * (1.0f / (v4 * NdotL + 0.0001f));
    vec3 spec = vscale(F, sp);
    vec3 diff = mk((1.0f - F.x) * kdA.x, (1.0f - F.y) * kdA.y, (1.0f - F.z) * kdA.z);
    L0 = vadd(L0, vscale(vmul(vadd(diff, spec), radiance), NdotL));
  }
  vec3 c = vscale(L0, 0.2f);
  c = mk(c.x * (1.0f / (c.x + 1.0f)), c.y * (1.0f / (c.y + 1.0f)), c.z * (1.0f / (c.z + 1.0f)));
  float g = 1.0f / 2.2f;
  *direct = cd;
  *pbr = mk(oracle_pow(c.x, g), oracle_pow(c.y, g), oracle_pow(c.z, g));
}
static vec3 osurface_sum(vec3 P, vec3 n, vec3 cam, const oracle_light* Ls, uint32_t nl, const float* mat) {
  vec3 d, p;
  osurface(P, n, cam, Ls, nl, mat, &d, &p);
  return vadd(d, p);
}

/* the two terms of osurface alone (tests/test_oracle.py checks each against the float64 restatement) */
static vec3 opbr(vec3 n, vec3 cam, vec3 P, const oracle_light* Ls, uint32_t nl, const float* mat) {
  vec3 d, p;
  osurface(P, n, cam, Ls, nl, mat, &d, &p);
  return p;
}
static vec3 odirect(vec3 P, vec3 n, vec3 albedo, const oracle_light* L, uint32_t nl) {
  float mat[6] = {albedo.x, albedo.y, albedo.z, 0.5f, 0.0f, 0.0f};
  vec3 d, p;
  osurface(P, n, P, L, nl, mat, &d, &p);
  return d;
}

void oracle_pbr(const float n[3], const float cam[3], const float P[3], const oracle_light* lights, uint32_t nl,
                const float material[6], float out[3]) {
  vec3 r = opbr(ld3(n), ld3(cam), ld3(P), lights, nl, material);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void oracle_direct(const float n[3], const float P[3], const oracle_light* lights, uint32_t nl, const float albedo[3], float out[3]) {
  vec3 r = odirect(ld3(P), ld3(n), ld3(albedo), lights, nl);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

static void tri_ids(const oblas* b, uint32_t prim, uint32_t* i0, uint32_t* i1, uint32_t* i2) {
  if (b->idx) { *i0 = b->idx[3 * prim]; *i1 = b->idx[3 * prim + 1]; *i2 = b->idx[3 * prim + 2]; }
  else { *i0 = 3 * prim; *i1 = 3 * prim + 1; *i2 = 3 * prim + 2; }
}

/* CalculateInterpolatedWorldNormal (Hit.hlsl:67-81) */
static vec3 o_interp_normal(const oracle_scene* s, uint32_t inst, uint32_t prim, float u, float v) {
  const oinst* ir = &s->inst[inst];
  const oblas* b = &s->blas[ir->blas];
  uint32_t i0, i1, i2;
  tri_ids(b, prim, &i0, &i1, &i2);
  vec3 n0 = ld3(b->vtx + (size_t)i1 * 6 + 3), n1 = ld3(b->vtx + (size_t)i2 * 6 + 3), n2 = ld3(b->vtx + (size_t)i0 * 6 + 3);
  float bz = (1.0f - u) - v;
  vec3 n = vnorm(vadd(vadd(vscale(n0, u), vscale(n1, v)), vscale(n2, bz)));
  n = m3mul(ir->nrm, n);
  return vnorm(n);
}

/* PlaneClosestHit face normal (Hit.hlsl:218-222) */
static vec3 o_face_normal(const oracle_scene* s, uint32_t inst, uint32_t prim) {
  const oinst* ir = &s->inst[inst];
  const oblas* b = &s->blas[ir->blas];
  uint32_t i0, i1, i2;
  tri_ids(b, prim, &i0, &i1, &i2);
  vec3 p0 = ld3(b->vtx + (size_t)i0 * 6), p1 = ld3(b->vtx + (size_t)i1 * 6), p2 = ld3(b->vtx + (size_t)i2 * 6);
  vec3 n = vnorm(vcross(vsub(p1, p0), vsub(p2, p0)));
  return m3mul(ir->nrm, n);
}

typedef struct {
  const oracle_scene* s;
  const float* cb;
  const oracle_light* L;
  uint32_t nl;
  const float* mat;
  int mode, k, brute;
  uint32_t W, H;
  int split; /* the device's forced tile-balance layouts (rt_set_tile_balance 2..5): 1 every tile in 2 x 2 parts,
                2 in 4 x 4, 3 by tile position (tx + 2 ty) % 3 -> whole / 2 x 2 / 4 x 4, 4 in 8 x 8 (one pixel each);
                capped by the tile shape */
} octx;

static int trace_any(const octx* c, vec3 P, vec3 dir, ostats* st) {
  ohit h;
  OST(1, 1);
  vec3 d = vnorm(dir); /* CastShadowRay normalises (Common.hlsl:73) */
  return c->brute ? obrute(c->s, P, d, 0.01f, 100000.0f, 1, 0, &h, st)
                  : otrace(c->s, P, d, 0.01f, 100000.0f, 1, 0, &h, st);
}

#define O_MAX_REFLECT 18 /* kMaxReflectDepth (rt_device.hpp): 20 TraceRay levels (D3D12HelloTriangle.cpp:954) */

static vec3 vreflect(vec3 i, vec3 n) { /* HLSL reflect: i - 2 n dot(i, n) */
  float t = vdot(i, n);
  return mk(i.x - (2.0f * n.x) * t, i.y - (2.0f * n.y) * t, i.z - (2.0f * n.z) * t);
}

static vec3 omiss(const octx* c, uint32_t py) {
  float ramp = (float)py / (float)c->H; /* Miss.hlsl:8-9 (DispatchRaysIndex: the pixel row at every depth) */
  return mk(0.0f, 0.2f, 0.7f - 0.3f * ramp);
}

/* PlaneClosestHit (Hit.hlsl:207-241) for a hit at P (one shadow ray) */
static vec3 oplane(const octx* c, vec3 P, const ohit* h, ostats* st) {
  vec3 ld = vnorm(vsub(ld3(c->L[0].position), P));
  vec3 n = o_face_normal(c->s, h->inst, h->prim);
  int shadowed = vdot(n, ld) < 0.0f;
  int occ = trace_any(c, P, ld, st);
  if (!shadowed) shadowed = occ;
  float factor = shadowed ? 0.3f : 1.0f;
  float li = fmax2(0.0f, vdot(n, ld));
  float v = (1.0f * li) * factor;
  return mk(v, v, v);
}

/* HLSL lerp(x, y, s) = x + s (y - x), per channel */
static vec3 olerp(vec3 x, vec3 y, float s) {
  return mk(x.x + s * (y.x - x.x), x.y + s * (y.y - x.y), x.z + s * (y.z - x.z));
}

/* payload colour of a reflection chain as the recursion returns it (Hit.hlsl:194-203): level k
 * sets lerp(s_k, <colour of level k+1>, r) after its nested TraceRay returned, innermost first */
static vec3 ounwind(const vec3* sk, int n, vec3 col, float r) {
  for (int k = n - 1; k >= 0; --k) col = olerp(sk[k], col, r);
  return col;
}

/* RT_SHADE_REF for one camera ray: ClosestHit (Hit.hlsl:183-204) / PlaneClosestHit / Miss, with
 * the reflection rays of InstanceID 0 and 1 (ReflectRay :176-181, CastReflectionRay
 * Common.hlsl:58-69: origin offset 0.001, TMin 0.001, TMax 1000, back faces culled) when the
 * material's reflectivity r != 0; the nested lerps unwound innermost first (ounwind).
 * r == 0 traces no reflection. */
static vec3 oshade_ref(const octx* c, uint32_t py, vec3 O, vec3 D, int f, ohit h, ostats* st) {
  const float refl = c->mat[5];
  vec3 sk[O_MAX_REFLECT], ro = O, rd = D;
  for (int depth = 0;; ++depth) {
    vec3 term;
    if (!f) {
      term = omiss(c, py);
    } else {
      const oinst* ir = &c->s->inst[h.inst];
      vec3 P = vadd(ro, vscale(rd, h.t));
      if (ir->hit_group == 2u) {
        term = oplane(c, P, &h, st);
      } else {
        vec3 n = o_interp_normal(c->s, h.inst, h.prim, h.u, h.v);
        vec3 s = osurface_sum(P, n, ro, c->L, c->nl, c->mat);
        if (refl != 0.0f && (ir->instance_id == 0u || ir->instance_id == 1u) && depth < O_MAX_REFLECT) {
          sk[depth] = s;
          vec3 dir = vnorm(vnorm(vreflect(vnorm(rd), n)));
          ro = vadd(P, vscale(dir, 0.001f));
          rd = dir;
          OST(8, 1);
          f = c->brute ? obrute(c->s, ro, rd, 0.001f, 1000.0f, 0, 1, &h, st)
                       : otrace(c->s, ro, rd, 0.001f, 1000.0f, 0, 1, &h, st);
          continue;
        }
        term = s;
      }
    }
    return ounwind(sk, depth, term, refl);
  }
}

static void hlsl_mul4(const float* m, const float v[4], float r[4]) {
  for (int i = 0; i < 4; ++i) r[i] = ((m[i] * v[0] + m[4 + i] * v[1]) + m[8 + i] * v[2]) + m[12 + i] * v[3];
}

/* RayGen (RayGen.hlsl:28-43): camera ray of one sample */
static void oraygen(const octx* c, uint32_t px, uint32_t py, float ox, float oy, vec3* O, vec3* D) {
  float dx = (((float)px + ox) / (float)c->W) * 2.0f - 1.0f;
  float dy = (((float)py + oy) / (float)c->H) * 2.0f - 1.0f;
  float org[4], dcam[4], dw[4];
  const float z1[4] = {0, 0, 0, 1};
  hlsl_mul4(c->cb + 32, z1, org);
  const float ndc[4] = {dx, -dy, 1.0f, 1.0f};
  hlsl_mul4(c->cb + 48, ndc, dcam);
  const float dc4[4] = {dcam[0], dcam[1], dcam[2], 0.0f};
  hlsl_mul4(c->cb + 32, dc4, dw);
  *O = mk(org[0], org[1], org[2]);
  *D = vnorm(mk(dw[0], dw[1], dw[2]));
}

/* RayGen + hit/miss programs for one camera sample, one independent ray per pixel */
static vec3 osample(const octx* c, uint32_t px, uint32_t py, float ox, float oy, ostats* st) {
  vec3 O, D;
  oraygen(c, px, py, ox, oy, &O, &D);
  ohit h;
  OST(0, 1);
  int f = c->brute ? obrute(c->s, O, D, 0.0f, 100000.0f, 0, 0, &h, st)
                   : otrace(c->s, O, D, 0.0f, 100000.0f, 0, 0, &h, st);
  if (c->mode == 0) return oshade_ref(c, py, O, D, f, h, st);
  if (!f) return omiss(c, py);
  const oinst* ir = &c->s->inst[h.inst];
  vec3 P = vadd(O, vscale(D, h.t));
  int plane = ir->hit_group == 2u;
  vec3 n = plane ? o_face_normal(c->s, h.inst, h.prim) : vneg(o_interp_normal(c->s, h.inst, h.prim, h.u, h.v));
  float sum = 0.0f;
  for (uint32_t l = 0; l < c->nl; ++l) {
    vec3 L = vnorm(vsub(ld3(c->L[l].position), P));
    float nl = vdot(n, L);
    if (nl > 0.0f) {
      float factor = 1.0f;
      if (c->mode == 1 && trace_any(c, P, L, st)) factor = 0.3f;
      sum = sum + nl * factor;
    }
  }
  sum = sum / (float)c->nl;
  return mk(sum, sum, sum);
}

static uint32_t unorm8(float x) {
  if (!(x > 0.0f)) return 0u;
  if (x >= 1.0f) return 255u;
  return (uint32_t)(x * 255.0f + 0.5f);
}

/* One camera sample for the 64 lanes of a wave tile, traces as wave packets
 * (shade_sample_packet in rt_trace.hip): lanes without a ray of a kind join that packet dead. */
static void osample_packet(const octx* c, const uint32_t* px, const uint32_t* py, const int* inimg, const float* ox,
                           const float* oy, vec3* color, ostats* st) {
  vec3 O[OPK], D[OPK], P[OPK], sd[OPK];
  ohit h[OPK], hs[OPK];
  int found[OPK], occl[OPK], need[OPK];
  for (int l = 0; l < OPK; ++l) {
    oraygen(c, px[l], py[l], ox[l], oy[l], &O[l], &D[l]);
    if (inimg[l]) OST(0, 1);
  }
  opacket(c->s, O, D, 0.0f, 100000.0f, 0, 0, inimg, h, found, st);
  for (int l = 0; l < OPK; ++l) {
    color[l] = omiss(c, py[l]);
    P[l] = vadd(O[l], vscale(D[l], h[l].t));
  }
  if (c->mode == 0) {
    /* oshade_ref, level by level for the whole tile: each level's shadow rays and next
     * reflection rays are one packet each */
    const float refl = c->mat[5];
    vec3 ro[OPK], rd[OPK], ldir[OPK], nf[OPK];
    static _Thread_local vec3 sk[OPK][O_MAX_REFLECT];
    int act[OPK], nxt[OPK];
    for (int l = 0; l < OPK; ++l) {
      ro[l] = O[l]; rd[l] = D[l]; act[l] = inimg[l];
    }
    for (int depth = 0;; ++depth) {
      int any_next = 0;
      for (int l = 0; l < OPK; ++l) {
        need[l] = 0;
        nxt[l] = 0;
        sd[l] = mk(0, 0, 1);
        if (!act[l]) continue;
        vec3 term;
        if (!found[l]) {
          term = omiss(c, py[l]);
        } else {
          const oinst* ir = &c->s->inst[h[l].inst];
          P[l] = vadd(ro[l], vscale(rd[l], h[l].t));
          if (ir->hit_group == 2u) {
            ldir[l] = vnorm(vsub(ld3(c->L[0].position), P[l]));
            nf[l] = o_face_normal(c->s, h[l].inst, h[l].prim);
            need[l] = 1;
            sd[l] = vnorm(ldir[l]);
            OST(1, 1);
            continue;
          }
          vec3 n = o_interp_normal(c->s, h[l].inst, h[l].prim, h[l].u, h[l].v);
          vec3 s = osurface_sum(P[l], n, ro[l], c->L, c->nl, c->mat);
          if (refl != 0.0f && (ir->instance_id == 0u || ir->instance_id == 1u) && depth < O_MAX_REFLECT) {
            sk[l][depth] = s;
            vec3 dir = vnorm(vnorm(vreflect(vnorm(rd[l]), n)));
            ro[l] = vadd(P[l], vscale(dir, 0.001f));
            rd[l] = dir;
            nxt[l] = 1;
            any_next = 1;
            OST(8, 1);
            continue;
          }
          term = s;
        }
        color[l] = ounwind(sk[l], depth, term, refl);
        act[l] = 0;
      }
      opacket(c->s, P, sd, 0.01f, 100000.0f, 1, 0, need, hs, occl, st);
      for (int l = 0; l < OPK; ++l) {
        if (!need[l]) continue;
        int shadowed = vdot(nf[l], ldir[l]) < 0.0f;
        if (!shadowed) shadowed = occl[l];
        float factor = shadowed ? 0.3f : 1.0f;
        float li = fmax2(0.0f, vdot(nf[l], ldir[l]));
        float v = (1.0f * li) * factor;
        vec3 term = mk(v, v, v);
        color[l] = ounwind(sk[l], depth, term, refl);
        act[l] = 0;
      }
      if (!any_next) return;
      for (int l = 0; l < OPK; ++l) act[l] = nxt[l];
      opacket(c->s, ro, rd, 0.001f, 1000.0f, 0, 1, act, h, found, st);
    }
  }
  vec3 n[OPK], Ld[OPK];
  float sum[OPK], nl[OPK];
  for (int l = 0; l < OPK; ++l) {
    sum[l] = 0.0f;
    n[l] = mk(0, 0, 0);
    if (!found[l]) continue;
    n[l] = c->s->inst[h[l].inst].hit_group == 2u ? o_face_normal(c->s, h[l].inst, h[l].prim)
                                                 : vneg(o_interp_normal(c->s, h[l].inst, h[l].prim, h[l].u, h[l].v));
  }
  for (uint32_t li = 0; li < c->nl; ++li) {
    for (int l = 0; l < OPK; ++l) {
      Ld[l] = vnorm(vsub(ld3(c->L[li].position), P[l]));
      nl[l] = vdot(n[l], Ld[l]);
      need[l] = found[l] && nl[l] > 0.0f;
      occl[l] = 0;
      sd[l] = need[l] ? vnorm(Ld[l]) : mk(0, 0, 1);
      if (c->mode == 1 && need[l]) OST(1, 1);
    }
    if (c->mode == 1) opacket(c->s, P, sd, 0.01f, 100000.0f, 1, 0, need, hs, occl, st);
    for (int l = 0; l < OPK; ++l)
      if (need[l]) sum[l] = sum[l] + nl[l] * (occl[l] ? 0.3f : 1.0f);
  }
  for (int l = 0; l < OPK; ++l)
    if (found[l]) {
      float v = sum[l] / (float)c->nl;
      color[l] = mk(v, v, v);
    }
}

typedef struct {
  const octx* c;
  const uint32_t* rows;
  uint32_t nrows, tid, nthreads;
  uint8_t* rgba8;
  float* rgba32f;
  ostats st;
} ojob;

static void store_px(const ojob* j, size_t o, vec3 acc) {
  if (j->rgba8) {
    j->rgba8[o * 4 + 0] = (uint8_t)unorm8(acc.x);
    j->rgba8[o * 4 + 1] = (uint8_t)unorm8(acc.y);
    j->rgba8[o * 4 + 2] = (uint8_t)unorm8(acc.z);
    j->rgba8[o * 4 + 3] = 255;
  }
  if (j->rgba32f) {
    j->rgba32f[o * 4 + 0] = acc.x; j->rgba32f[o * 4 + 1] = acc.y;
    j->rgba32f[o * 4 + 2] = acc.z; j->rgba32f[o * 4 + 3] = 1.0f;
  }
}

/* Wave tiles as the device deals them (rt_trace.hip k_trace_frame_packet): spp 1 (and the sample
 * loop for spp 9): 8 x 8 pixels (pixel column, row-list entry), lane = 8 * (row % 8) + column % 8;
 * spp 4 / 16: the k x k samples of a pixel in consecutive lanes, (8 / k) x (8 / k) pixels per wave,
 * lane = k^2 * (8/k * (row % (8/k)) + column % (8/k)) + sample, sample = k * sy + sx; the pixel's
 * samples are summed in sample order as the loop adds them. */
static uint32_t olog2u(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

static void* render_tiles(void* arg) {
  ojob* j = (ojob*)arg;
  const octx* c = j->c;
  const int lanes_k = (c->k == 2 || c->k == 4) ? c->k : 1; /* samples held by lanes */
  const uint32_t ns = (uint32_t)(lanes_k * lanes_k), tp = 8u / (uint32_t)lanes_k;
  const uint32_t tw = (c->W + tp - 1) / tp, th = (j->nrows + tp - 1) / tp;
  /* tile balance (rt_trace.hip packet_geometry / k_tile_plan): the parts a tile is traced as, each its own
   * packet with the lanes outside its sub-rectangle dead; 4 x 4 parts need 4-pixel tile sides */
  const uint32_t kmax = tp >= 8u ? 3u : tp >= 4u ? 2u : tp >= 2u ? 1u : 0u;
  for (uint32_t t = j->tid; t < tw * th; t += j->nthreads) {
    const uint32_t tx = t % tw, ty = t / tw;
    uint32_t px[OPK], py[OPK], orow[OPK];
    int inimg[OPK], inpart[OPK];
    float ox[OPK], oy[OPK];
    vec3 acc[OPK], col[OPK];
    for (int l = 0; l < OPK; ++l) {
      const uint32_t s = (uint32_t)l % ns, p = (uint32_t)l / ns;
      px[l] = tx * tp + p % tp;
      orow[l] = ty * tp + p / tp;
      inimg[l] = px[l] < c->W && orow[l] < j->nrows;
      py[l] = inimg[l] ? (j->rows ? j->rows[orow[l]] : orow[l]) : 0;
      ox[l] = ((float)(s % (uint32_t)lanes_k) + 0.5f) / (float)lanes_k;
      oy[l] = ((float)(s / (uint32_t)lanes_k) + 0.5f) / (float)lanes_k;
      acc[l] = mk(0, 0, 0);
    }
    uint32_t code = c->split == 1 ? 1u : c->split == 2 ? 2u : c->split == 3 ? (tx + 2u * ty) % 3u : c->split == 4 ? 3u : 0u;
    if (code > kmax) code = kmax;
    const uint32_t nparts = code == 0u ? 1u : code == 1u ? 4u : code == 2u ? 16u : 64u, pq = 1u << code;
    for (uint32_t part = 0; part < nparts; ++part) {
      for (int l = 0; l < OPK; ++l) {
        const uint32_t p = (uint32_t)l / ns;
        inpart[l] = inimg[l] && ((p % tp) >> (olog2u(tp) - code)) == (part & (pq - 1u)) &&
                    ((p / tp) >> (olog2u(tp) - code)) == (part >> code);
      }
      if (lanes_k > 1) {
        osample_packet(c, px, py, inpart, ox, oy, col, &j->st);
        for (int l = 0; l < OPK; l += (int)ns)
          if (inpart[l])
            for (uint32_t q = 0; q < ns; ++q) acc[l] = vadd(acc[l], col[l + (int)q]);
      } else {
        for (int sy = 0; sy < c->k; ++sy)
          for (int sx = 0; sx < c->k; ++sx) {
            for (int l = 0; l < OPK; ++l) {
              ox[l] = ((float)sx + 0.5f) / (float)c->k;
              oy[l] = ((float)sy + 0.5f) / (float)c->k;
            }
            osample_packet(c, px, py, inpart, ox, oy, col, &j->st);
            for (int l = 0; l < OPK; ++l)
              if (inpart[l]) acc[l] = vadd(acc[l], col[l]);
          }
      }
    }
    for (int l = 0; l < OPK; l += (int)ns) {
      if (!inimg[l]) continue;
      vec3 a = acc[l];
      if (c->k > 1) {
        float n = (float)(c->k * c->k);
        a = mk(a.x / n, a.y / n, a.z / n);
      }
      store_px(j, (size_t)orow[l] * c->W + px[l], a);
    }
  }
  return NULL;
}

static void* render_rows(void* arg) {
  ojob* j = (ojob*)arg;
  const octx* c = j->c;
  for (uint32_t r = j->tid; r < j->nrows; r += j->nthreads) {
    uint32_t py = j->rows ? j->rows[r] : r;
    for (uint32_t px = 0; px < c->W; ++px) {
      vec3 acc = mk(0, 0, 0);
      for (int sy = 0; sy < c->k; ++sy)
        for (int sx = 0; sx < c->k; ++sx) {
          float ox = ((float)sx + 0.5f) / (float)c->k, oy = ((float)sy + 0.5f) / (float)c->k;
          acc = vadd(acc, osample(c, px, py, ox, oy, &j->st));
        }
      if (c->k > 1) {
        float ns = (float)(c->k * c->k);
        acc = mk(acc.x / ns, acc.y / ns, acc.z / ns);
      }
      store_px(j, (size_t)r * c->W + px, acc);
    }
  }
  return NULL;
}

int oracle_render_split(const oracle_scene* s, const float cb[64], const oracle_light* lights, uint32_t nlights,
                        const float material[6], int mode, int spp, uint32_t W, uint32_t H, const uint32_t* rows,
                        uint32_t nrows, uint8_t* rgba8, float* rgba32f, int nthreads, uint64_t* stats, int brute,
                        int schedule, int split) {
  if (!s || !s->tlas || !cb || !lights || nlights < 1 || nlights > 16 || W == 0 || H == 0) return -1;
  int k = 0;
  for (int q = 1; q <= 4; ++q) if (q * q == spp) k = q;
  if (!k || mode < 0 || mode > 2) return -1;
  if (!rows) nrows = H;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  octx c = {s, cb, lights, nlights, material, mode, k, brute, W, H, split};
  ojob jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; ++t) {
    memset(&jobs[t], 0, sizeof(ojob));
    jobs[t].c = &c; jobs[t].rows = rows; jobs[t].nrows = nrows;
    jobs[t].tid = (uint32_t)t; jobs[t].nthreads = (uint32_t)nthreads;
    jobs[t].rgba8 = rgba8; jobs[t].rgba32f = rgba32f;
  }
  /* the device runs wave packets unless asked for per-lane rays or the trees are too deep for
   * its one-VGPR stack (rt_trace.hip launch_mode) */
  uint32_t maxd = 0;
  for (int q = 0; q < s->nblas; ++q) if (s->blas[q].depth > maxd) maxd = s->blas[q].depth;
  const int packet = !brute && schedule == 0 && (s->tlas_max_stack + maxd) < OPK;
  void* (*fn)(void*) = packet ? render_tiles : render_rows;
  if (nthreads == 1) fn(&jobs[0]);
  else {
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
  if (stats)
    for (int t = 0; t < nthreads; ++t)
      for (int q = 0; q < 6; ++q) stats[q] += jobs[t].st.v[q];
  if (stats)
    for (int t = 0; t < nthreads; ++t)
      for (int q = 8; q < 12; ++q) stats[q] += jobs[t].st.v[q];
  if (stats) { stats[6] += (uint64_t)W * nrows; stats[7] += 1; }
  return 0;
}

int oracle_render(const oracle_scene* s, const float cb[64], const oracle_light* lights, uint32_t nlights,
                  const float material[6], int mode, int spp, uint32_t W, uint32_t H, const uint32_t* rows,
                  uint32_t nrows, uint8_t* rgba8, float* rgba32f, int nthreads, uint64_t* stats, int brute,
                  int schedule) {
  return oracle_render_split(s, cb, lights, nlights, material, mode, spp, W, H, rows, nrows, rgba8, rgba32f, nthreads,
                             stats, brute, schedule, 0);
}

/* RayGen's camera rays (oraygen: the exact float32 bits the frame traces) for n pixels (px[i], py[i]) at the
 * sample offset (ox, oy), in oracle_trace_rays' layout: 8 floats per ray (o.xyz, tmin 0, d.xyz, tmax 1e5,
 * CastDefaultRay, Common.hlsl:44-56). Test infrastructure: the full-size float64 cross-check compares the
 * float32 primary hits of these rays with its own. */
void oracle_camera_rays(const float cb[64], uint32_t W, uint32_t H, const uint32_t* px, const uint32_t* py, uint32_t n,
                        float ox, float oy, float* rays) {
  octx c;
  memset(&c, 0, sizeof(c));
  c.cb = cb;
  c.W = W;
  c.H = H;
  for (uint32_t i = 0; i < n; ++i) {
    vec3 O, D;
    oraygen(&c, px[i], py[i], ox, oy, &O, &D);
    float* r = rays + (size_t)i * 8;
    r[0] = O.x; r[1] = O.y; r[2] = O.z; r[3] = 0.0f;
    r[4] = D.x; r[5] = D.y; r[6] = D.z; r[7] = 100000.0f;
  }
}

int oracle_trace_rays(const oracle_scene* s, const float* rays, uint32_t n, uint32_t flags, uint32_t* hits,
                      float* uv, int brute, uint64_t* stats) {
  if (!s || !s->tlas) return -1;
  /* D3D12_RAY_FLAG values: 0x04 accept first hit, 0x10 cull back faces, 0x20 cull front faces */
  if ((flags & 0x30u) == 0x30u) return -1;
  const int any = (flags & 0x04u) != 0, cull = (flags & 0x10u) ? 1 : ((flags & 0x20u) ? -1 : 0);
  ostats st;
  memset(&st, 0, sizeof(st));
  for (uint32_t i = 0; i < n; ++i) {
    const float* r = rays + (size_t)i * 8;
    ohit h;
    int f = brute ? obrute(s, ld3(r), ld3(r + 4), r[3], r[7], any, cull, &h, &st)
                  : otrace(s, ld3(r), ld3(r + 4), r[3], r[7], any, cull, &h, &st);
    st.v[0]++;
    float t = f ? h.t : r[7];
    uint32_t tb; memcpy(&tb, &t, 4);
    hits[i * 4 + 0] = tb;
    hits[i * 4 + 1] = f ? h.inst : 0xffffffffu;
    hits[i * 4 + 2] = f ? h.prim : 0xffffffffu;
    hits[i * 4 + 3] = f ? 1u : 0u;
    if (uv) { uv[i * 2] = f ? h.u : 0.0f; uv[i * 2 + 1] = f ? h.v : 0.0f; }
  }
  if (stats) {
    for (int q = 0; q < 6; ++q) stats[q] += st.v[q];
    for (int q = 9; q < 12; ++q) stats[q] += st.v[q];
  }
  return 0;
}
