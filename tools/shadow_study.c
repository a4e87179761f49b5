/* Design study (not product, not a checker): how shadow-ray regrouping changes the packet
 * traversal's work. Compiled together with the oracle's restatement (one translation unit):
 *   gcc -O2 -shared -fPIC -ffp-contract=off -mfma -o /tmp/libstudy.so tools/shadow_study.c -lm -lpthread
 * For LAMBERT_SHADOW frames it traces the primary packets (8x8-pixel waves), collects every
 * shadow ray (Hit.hlsl:207-241 / Common.hlsl:71-82: one per light with n.L > 0) and traces them as
 * 64-ray any-hit packets under several groupings, counting per-wave node and triangle fetches
 * (the packet walk's cost unit: one scalar fetch + 64 lanes of slab/triangle VALU each).
 *   mode 0  per wave, per light (the kernel today)
 *   mode 1  per wave, all lights compacted (light-major)
 *   mode 2  per group of G consecutive waves (G x 8 x 8 px along x), per light compacted
 *   mode 3  per group of G waves, all lights compacted
 *   mode 4  per wave, per light, rays sorted by hit instance before packing (live ones only)
 *   mode 5  per group of G waves, per light, sorted by hit instance (then pixel)
 *   mode 6  per group of G waves, per light, sorted by the 30-bit Morton code of the origin
 *   mode 7  whole frame, per light, sorted by hit instance then origin Morton (a global wavefront sort)
 *   mode 8  whole frame, per light, sorted by origin Morton only
 */
#include "../oracle/rt_oracle.c"

typedef struct {
  vec3 P, d;
  uint32_t inst, light, pix;
} sray;

static int cmp_key(const void* a, const void* b) {
  const sray* x = (const sray*)a;
  const sray* y = (const sray*)b;
  if (x->inst != y->inst) return x->inst < y->inst ? -1 : 1;  /* inst holds the sort key (mode 6) */
  return x->pix < y->pix ? -1 : (x->pix > y->pix);
}

static uint32_t morton_of(vec3 p) {
  /* scene box of the grid configs: [-30, 30]^3 */
  float q[3] = {(p.x + 30.0f) / 60.0f, (p.y + 30.0f) / 60.0f, (p.z + 30.0f) / 60.0f};
  uint32_t m[3];
  for (int k = 0; k < 3; ++k) {
    float s = q[k] * 1024.0f;
    s = s < 0 ? 0 : (s > 1023 ? 1023 : s);
    m[k] = expand10((uint32_t)s);
  }
  return (m[0] << 2) | (m[1] << 1) | m[2];
}

static int cmp_inst(const void* a, const void* b) {
  const sray* x = (const sray*)a;
  const sray* y = (const sray*)b;
  if (x->inst != y->inst) return x->inst < y->inst ? -1 : 1;
  return x->pix < y->pix ? -1 : (x->pix > y->pix);
}

/* traces rays[0..n) as ceil(n/64) packets in the given order; returns packets */
static uint64_t trace_groups(const oracle_scene* s, const sray* rays, int n, ostats* st) {
  uint64_t packets = 0;
  for (int b = 0; b < n; b += OPK) {
    vec3 o[OPK], d[OPK];
    int alive[OPK], found[OPK];
    ohit h[OPK];
    for (int l = 0; l < OPK; ++l) {
      alive[l] = b + l < n;
      o[l] = alive[l] ? rays[b + l].P : mk(0, 0, 0);
      d[l] = alive[l] ? rays[b + l].d : mk(0, 0, 1);
    }
    opacket(s, o, d, 0.01f, 100000.0f, 1, 0, alive, h, found, st);
    ++packets;
  }
  return packets;
}

/* out[0] packets, out[1] node fetches, out[2] tri fetches, out[3] shadow rays, out[4] lane tests (aabb) */
int study_shadow(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t nl, uint32_t W, uint32_t H,
                 int mode, int G, uint64_t out[5]) {
  octx c = {s, cb, L, nl, NULL, 1, 1, 0, W, H};
  const uint32_t tw = (W + 7) / 8, th = (H + 7) / 8;
  ostats st;
  memset(&st, 0, sizeof(st));
  ostats pst;
  memset(&pst, 0, sizeof(pst));
  sray* buf = (sray*)malloc(sizeof(sray) * (size_t)OPK * 16 * (G > 0 ? G : 1));
  uint64_t packets = 0, nrays = 0;
  const int gsz = (mode == 2 || mode == 3 || mode == 5 || mode == 6) ? G : 1;
  const int global = mode == 7 || mode == 8;
  sray* gl[16] = {0};
  size_t gn[16] = {0};
  if (global)
    for (uint32_t li = 0; li < nl; ++li) gl[li] = (sray*)malloc(sizeof(sray) * (size_t)W * H);
  for (uint32_t ty = 0; ty < th; ++ty)
    for (uint32_t tx0 = 0; tx0 < tw; tx0 += (uint32_t)gsz) {
      int n_all = 0;
      sray* per_light[16];
      int n_light[16];
      (void)per_light;
      /* collect the shadow rays of the group's waves, wave-major, lane order, per light */
      static _Thread_local sray tmp[16][OPK * 16];
      for (uint32_t li = 0; li < nl; ++li) n_light[li] = 0;
      for (int g = 0; g < gsz && tx0 + (uint32_t)g < tw; ++g) {
        const uint32_t tx = tx0 + (uint32_t)g;
        vec3 O[OPK], D[OPK];
        int inimg[OPK], found[OPK];
        ohit h[OPK];
        uint32_t px[OPK], py[OPK];
        for (int l = 0; l < OPK; ++l) {
          px[l] = tx * 8 + (uint32_t)(l & 7);
          py[l] = ty * 8 + (uint32_t)(l >> 3);
          inimg[l] = px[l] < W && py[l] < H;
          oraygen(&c, px[l], inimg[l] ? py[l] : 0, 0.5f, 0.5f, &O[l], &D[l]);
        }
        opacket(s, O, D, 0.0f, 100000.0f, 0, 0, inimg, h, found, &pst);
        for (int l = 0; l < OPK; ++l) {
          if (!found[l]) continue;
          const vec3 P = vadd(O[l], vscale(D[l], h[l].t));
          const int plane = s->inst[h[l].inst].hit_group == 2u;
          const vec3 n = plane ? o_face_normal(s, h[l].inst, h[l].prim) : vneg(o_interp_normal(s, h[l].inst, h[l].prim, h[l].u, h[l].v));
          for (uint32_t li = 0; li < nl; ++li) {
            const vec3 Ld = vnorm(vsub(ld3(L[li].position), P));
            if (!(vdot(n, Ld) > 0.0f)) continue;
            sray r = {P, vnorm(Ld), h[l].inst, li, (uint32_t)(g * OPK + l)};
            tmp[li][n_light[li]++] = r;
          }
        }
      }
      if (global) {
        for (uint32_t li = 0; li < nl; ++li)
          for (int q = 0; q < n_light[li]; ++q) {
            sray r = tmp[li][q];
            r.pix = (ty * tw + tx0) * OPK + (uint32_t)q;
            const uint32_t m = morton_of(r.P);
            r.inst = mode == 7 ? (r.inst << 20) | (m >> 10) : m;
            gl[li][gn[li]++] = r;
          }
      } else if (mode == 0 || mode == 2 || mode == 4 || mode == 5 || mode == 6) {
        for (uint32_t li = 0; li < nl; ++li) {
          if (mode == 4 || mode == 5) qsort(tmp[li], (size_t)n_light[li], sizeof(sray), cmp_inst);
          if (mode == 6) {
            for (int q = 0; q < n_light[li]; ++q) tmp[li][q].inst = morton_of(tmp[li][q].P);
            qsort(tmp[li], (size_t)n_light[li], sizeof(sray), cmp_key);
          }
          packets += trace_groups(s, tmp[li], n_light[li], &st);
          nrays += (uint64_t)n_light[li];
        }
      } else {
        for (uint32_t li = 0; li < nl; ++li)
          for (int q = 0; q < n_light[li]; ++q) buf[n_all++] = tmp[li][q];
        packets += trace_groups(s, buf, n_all, &st);
        nrays += (uint64_t)n_all;
      }
    }
  if (global)
    for (uint32_t li = 0; li < nl; ++li) {
      qsort(gl[li], gn[li], sizeof(sray), cmp_key);
      packets += trace_groups(s, gl[li], (int)gn[li], &st);
      nrays += gn[li];
      free(gl[li]);
    }
  free(buf);
  out[0] = packets;
  out[1] = st.v[9];
  out[2] = st.v[10];
  out[3] = nrays;
  out[4] = st.v[2];
  return 0;
}
