/* Design study (not product, not a checker): would tracing two lights' shadow rays as ONE packet of two rays per lane
 * (trace_packet<ANY_HIT, STATS, R = 2>: 128 rays, the lead the first live ray in slot order r * 64 + lane) walk less
 * than the kernel's one 64-ray packet per light? Compiled with the oracle's packet emulation widened to 128 lanes:
 *   gcc -O2 -shared -fPIC -ffp-contract=off -mfma -DOPK=128 -o /tmp/libmerge.so tools/merge_study.c -lm -lpthread
 * A 64-ray packet is emulated as a 128-lane one whose upper 64 lanes are dead (they never enter a node), so the
 * per-light counts are the kernel's. Per 8 x 8 tile: the primary packet, then for each light the rays with n.L > 0
 * (Hit.hlsl:207-241, Common.hlsl:71-82) in their pixel's lane; lights paired (0,1), (2,3), ... into one packet. */
#include "../oracle/rt_oracle.c"

/* out[0] separate node fetches, [1] separate tri fetches, [2] merged node fetches, [3] merged tri fetches,
 * [4] separate lane box tests, [5] merged lane box tests, [6] separate packets, [7] merged packets */
int study_merge(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t nl, uint32_t W, uint32_t H,
                uint64_t out[8]) {
  octx c = {s, cb, L, nl, NULL, 1, 1, 0, W, H};
  const uint32_t tw = (W + 7) / 8, th = (H + 7) / 8;
  ostats pst, sep, mer;
  memset(&pst, 0, sizeof(pst));
  memset(&sep, 0, sizeof(sep));
  memset(&mer, 0, sizeof(mer));
  uint64_t npk_sep = 0, npk_mer = 0;
  for (uint32_t ty = 0; ty < th; ++ty)
    for (uint32_t tx = 0; tx < tw; ++tx) {
      vec3 O[OPK], D[OPK];
      int inimg[OPK], found[OPK];
      ohit h[OPK];
      for (int l = 0; l < OPK; ++l) {
        const uint32_t px = tx * 8 + (uint32_t)(l & 7), py = ty * 8 + (uint32_t)((l >> 3) & 7);
        inimg[l] = l < 64 && px < W && py < H;
        oraygen(&c, px < W ? px : 0, py < H ? py : 0, 0.5f, 0.5f, &O[l], &D[l]);
      }
      opacket(s, O, D, 0.0f, 100000.0f, 0, 0, inimg, h, found, &pst);
      vec3 P[64], Ld[16][64];
      int need[16][64];
      for (int l = 0; l < 64; ++l) {
        for (uint32_t li = 0; li < nl; ++li) need[li][l] = 0;
        if (!found[l]) continue;
        P[l] = vadd(O[l], vscale(D[l], h[l].t));
        const int plane = s->inst[h[l].inst].hit_group == 2u;
        const vec3 n = plane ? o_face_normal(s, h[l].inst, h[l].prim) : vneg(o_interp_normal(s, h[l].inst, h[l].prim, h[l].u, h[l].v));
        for (uint32_t li = 0; li < nl; ++li) {
          const vec3 d = vnorm(vsub(ld3(L[li].position), P[l]));
          Ld[li][l] = d;
          need[li][l] = vdot(n, d) > 0.0f;
        }
      }
      vec3 so[OPK], sd[OPK];
      int al[OPK], fd[OPK];
      ohit hs[OPK];
      for (uint32_t li = 0; li < nl; ++li) {  /* the kernel: one packet per light */
        int any = 0;
        for (int l = 0; l < OPK; ++l) {
          al[l] = l < 64 && need[li][l];
          any |= al[l];
          so[l] = al[l] ? P[l] : mk(0, 0, 0);
          sd[l] = al[l] ? Ld[li][l] : mk(0, 0, 1);
        }
        if (!any) continue;
        opacket(s, so, sd, 0.01f, 100000.0f, 1, 0, al, hs, fd, &sep);
        ++npk_sep;
      }
      for (uint32_t li = 0; li < nl; li += 2) {  /* two lights per packet: slot r = light li + r */
        int any = 0;
        for (int l = 0; l < OPK; ++l) {
          const uint32_t q = li + (uint32_t)(l >> 6);
          al[l] = q < nl && need[q][l & 63];
          any |= al[l];
          so[l] = al[l] ? P[l & 63] : mk(0, 0, 0);
          sd[l] = al[l] ? Ld[q][l & 63] : mk(0, 0, 1);
        }
        if (!any) continue;
        opacket(s, so, sd, 0.01f, 100000.0f, 1, 0, al, hs, fd, &mer);
        ++npk_mer;
      }
    }
  out[0] = sep.v[9]; out[1] = sep.v[10]; out[2] = mer.v[9]; out[3] = mer.v[10];
  out[4] = sep.v[2]; out[5] = mer.v[2]; out[6] = npk_sep; out[7] = npk_mer;
  return 0;
}
