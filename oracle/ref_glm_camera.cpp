// Harness compiled ONLY in the dev container against the reference's vendored glm 0.9.8.5
// (/root/reference/glm, header-only) to produce golden camera matrices for the oracle and the
// product: glm::lookAt is what Manipulator::update computes (src/manipulator.cpp:305-314).
// Output: JSON on stdout, floats as IEEE-754 bit patterns. Never shipped, never run on the GPU box.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#include <glm/gtc/type_ptr.hpp>

static uint32_t bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

static void emit_mat(const char* key, const glm::mat4& m, bool last) {
  const float* p = glm::value_ptr(m);
  std::printf("   \"%s\": [", key);
  for (int i = 0; i < 16; ++i) std::printf("%u%s", bits(p[i]), i < 15 ? ", " : "");
  std::printf("]%s\n", last ? "" : ",");
}

int main() {
  const float cases[][9] = {
      {1.5f, 1.5f, 1.5f, 0, 0, 0, 0, 1, 0},          // reference (D3D12HelloTriangle.cpp:45)
      {10, 10, 10, 0, 0, 0, 0, 1, 0},                // Manipulator default m_pos (manipulator.h:126)
      {18, 14, 18, 0, 1, 0, 0, 1, 0},                // C4 camera
      {30, 22, 30, 0, 1, 0, 0, 1, 0},                // C5 camera
      {7, 5, 9, 0.2f, 1.3f, 0, 0, 1, 0},             // C2F camera
      {-3.25f, 0.5f, 7.125f, 1.0f, -2.0f, 0.5f, 0.1f, 0.9f, -0.2f},  // asymmetric, skewed up
  };
  const int n = sizeof(cases) / sizeof(cases[0]);
  std::printf("{\n \"source\": \"glm 0.9.8.5 lookAt (reference vendored glm), oracle/ref_glm_camera.cpp\",\n");
  std::printf(" \"lookat\": [\n");
  for (int c = 0; c < n; ++c) {
    const float* k = cases[c];
    glm::mat4 m = glm::lookAt(glm::vec3(k[0], k[1], k[2]), glm::vec3(k[3], k[4], k[5]), glm::vec3(k[6], k[7], k[8]));
    std::printf("  {\"eye\": [%.9g, %.9g, %.9g], \"center\": [%.9g, %.9g, %.9g], \"up\": [%.9g, %.9g, %.9g],\n", k[0],
                k[1], k[2], k[3], k[4], k[5], k[6], k[7], k[8]);
    emit_mat("view_bits", m, true);
    std::printf("  }%s\n", c < n - 1 ? "," : "");
  }
  std::printf(" ],\n \"rotate\": [\n");
  const float rots[][4] = {{0.3f, 0, 1, 0}, {-1.1f, 0.6f, 0.0f, -0.8f}, {2.5f, 0.267261f, 0.534522f, 0.801784f}};
  const int nr = sizeof(rots) / sizeof(rots[0]);
  for (int r = 0; r < nr; ++r) {
    glm::mat4 m = glm::rotate(glm::mat4(1.0f), rots[r][0], glm::vec3(rots[r][1], rots[r][2], rots[r][3]));
    std::printf("  {\"angle\": %.9g, \"axis\": [%.9g, %.9g, %.9g],\n", rots[r][0], rots[r][1], rots[r][2], rots[r][3]);
    emit_mat("m_bits", m, true);
    std::printf("  }%s\n", r < nr - 1 ? "," : "");
  }
  std::printf(" ]\n}\n");
  return 0;
}
