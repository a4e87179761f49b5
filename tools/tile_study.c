/* Design study (not product, not a checker): per 8x8 tile of a LAMBERT_SHADOW config, the packet
 * walk's cost (per-wave node + triangle + instance fetches, primary and shadow packets, the kernel's
 * rules via the oracle's emulation) against the per-lane walk's (each lane's own node visits +
 * triangle tests; a SIMT wave pays about the maximum over its lanes). Built and run by
 * tools/tile_study.py. */
#include "../oracle/rt_oracle.c"

/* out[t*4 + 0] packet fetches, [1] max over lanes of own visits, [2] sum over lanes, [3] live lanes */
int tile_study(const oracle_scene* s, const float cb[64], const oracle_light* L, uint32_t nl, uint32_t W, uint32_t H,
               uint64_t* out) {
  octx c = {s, cb, L, nl, NULL, 1, 1, 0, W, H};
  const uint32_t tw = W / 8, th = H / 8;
  for (uint32_t ty = 0; ty < th; ++ty)
    for (uint32_t tx = 0; tx < tw; ++tx) {
      uint32_t px[OPK], py[OPK];
      int inimg[OPK];
      float ox[OPK], oy[OPK];
      vec3 col[OPK];
      for (int l = 0; l < OPK; ++l) {
        px[l] = tx * 8 + (uint32_t)(l & 7);
        py[l] = ty * 8 + (uint32_t)(l >> 3);
        inimg[l] = 1;
        ox[l] = oy[l] = 0.5f;
      }
      ostats st;
      memset(&st, 0, sizeof(st));
      osample_packet(&c, px, py, inimg, ox, oy, col, &st);
      uint64_t* o = out + ((uint64_t)ty * tw + tx) * 4;
      o[0] = st.v[9] + st.v[10] + st.v[11];
      uint64_t mx = 0, sum = 0;
      for (int l = 0; l < OPK; ++l) {
        ostats ls;
        memset(&ls, 0, sizeof(ls));
        vec3 O, D;
        oraygen(&c, px[l], py[l], 0.5f, 0.5f, &O, &D);
        ohit h;
        int f = otrace(s, O, D, 0.0f, 100000.0f, 0, 0, &h, &ls);
        if (f) {
          vec3 P = vadd(O, vscale(D, h.t));
          vec3 n = s->inst[h.inst].hit_group == 2u ? o_face_normal(s, h.inst, h.prim)
                                                   : vneg(o_interp_normal(s, h.inst, h.prim, h.u, h.v));
          for (uint32_t li = 0; li < nl; ++li) {
            vec3 Ld = vnorm(vsub(ld3(L[li].position), P));
            if (!(vdot(n, Ld) > 0.0f)) continue;
            ohit hs;
            otrace(s, P, vnorm(Ld), 0.01f, 100000.0f, 1, 0, &hs, &ls);
          }
        }
        const uint64_t v = ls.v[9] + ls.v[10] + ls.v[11];
        mx = v > mx ? v : mx;
        sum += v;
      }
      o[1] = mx;
      o[2] = sum;
      o[3] = OPK;
    }
  return 0;
}
