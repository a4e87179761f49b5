// Sanitizer driver of the host services (make asan -> build/asan/obj_ingest_fuzz; tools/asan_check.sh runs it):
// rt_mesh_parse_obj over seeded random text built from the characters the parser branches on (and any byte),
// truncated lines, overlong tokens and huge index values; every mesh then goes through
// rt_mesh_compute_vertex_normals (which must refuse out-of-range indices, not read past the vertices: the
// reference indexes out of bounds there, OBJ_FileManager.cpp:35-41 + D3D12HelloTriangle.cpp:1430-1462) and the
// camera manipulator gets random mouse / wheel input. Built with -fsanitize=address,undefined: any overflow, use
// after free or undefined behaviour aborts the run.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../include/rt_api.h"

namespace {
uint64_t g_state = 0x9e3779b97f4a7c15ull;
uint64_t next() {  // xorshift64*
  g_state ^= g_state >> 12;
  g_state ^= g_state << 25;
  g_state ^= g_state >> 27;
  return g_state * 2685821657736338717ull;
}
uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }

std::string random_text() {
  static const char kAlpha[] = "vf 0123456789+-.eE/\t\r\n#xX";
  std::string s;
  const uint32_t lines = 1 + below(40);
  for (uint32_t l = 0; l < lines; ++l) {
    switch (below(6)) {
      case 0: s += "v "; break;
      case 1: s += "f "; break;
      case 2: s += "v"; break;
      default: break;
    }
    const uint32_t n = below(4) == 0 ? below(600) : below(24);
    for (uint32_t k = 0; k < n; ++k)
      s += below(16) == 0 ? (char)below(256) : kAlpha[below(sizeof(kAlpha) - 1)];
    if (below(8)) s += '\n';
  }
  return s;
}
}  // namespace

int main(int argc, char** argv) {
  const uint32_t iters = argc > 1 ? (uint32_t)std::strtoul(argv[1], nullptr, 10) : 20000u;
  uint64_t verts = 0, faces = 0, refused = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    std::string s = random_text();
    if (it % 97 == 0) s = "v 1 2 3\nv 4 5 6\nv 7 8 9\nf 1 2 " + std::to_string(next()) + "\n";
    rt_mesh_t m = nullptr;
    if (rt_mesh_parse_obj(s.data(), s.size(), &m) != RT_OK || !m) {
      std::fprintf(stderr, "parse failed at iteration %u\n", it);
      return 1;
    }
    verts += rt_mesh_vertex_count(m);
    faces += rt_mesh_index_count(m) / 3;
    const rt_status st = rt_mesh_compute_vertex_normals(m);
    if (st != RT_OK) ++refused;
    rt_mesh_free(m);
  }
  rt_manipulator man;
  rt_manip_init(&man);
  rt_manip_set_window_size(&man, 1 + (int32_t)below(4000), 1 + (int32_t)below(4000));
  const float eye[3] = {1.5f, 1.5f, 1.5f}, at[3] = {0.0f, 0.0f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
  rt_manip_set_lookat(&man, eye, at, up);
  for (uint32_t it = 0; it < 20000u; ++it) {
    const int32_t x = (int32_t)below(8000) - 2000, y = (int32_t)below(8000) - 2000;
    switch (below(4)) {
      case 0: rt_manip_set_mouse_position(&man, x, y); break;
      case 1: rt_manip_motion(&man, x, y, (int32_t)below(6)); break;
      case 2: (void)rt_manip_mouse_move(&man, x, y, below(16)); break;
      default: rt_manip_wheel(&man, (int32_t)below(400) - 200); break;
    }
  }
  std::printf("obj_ingest_fuzz: %u texts, %llu vertices, %llu faces, %llu meshes refused by the normals "
              "(indices out of range); 20000 manipulator events\n", iters, (unsigned long long)verts,
              (unsigned long long)faces, (unsigned long long)refused);
  return 0;
}
