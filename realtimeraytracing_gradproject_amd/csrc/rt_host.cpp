// rt_host.cpp — host services of the C-ABI: OBJ mesh ingest, vertex normals, ground plane and
// camera matrices. Pure host C++ (no HIP calls), so these run without a GPU.
//
// Behaviour follows the reference host code (paths relative to the reference tree):
//   OBJFileManager::LoadObjFile               src/OBJ_FileManager.cpp:10-71
//   D3D12HelloTriangle::ComputeVertexNormals  src/D3D12HelloTriangle.cpp:1430-1462
//   D3D12HelloTriangle::CreatePlaneVB         src/D3D12HelloTriangle.cpp:1237-1271
//   Manipulator::setLookat/update             src/manipulator.cpp:26-32, 305-314 (glm::lookAtRH)
//   D3D12HelloTriangle::UpdateCameraBuffer    src/D3D12HelloTriangle.cpp:1144-1170
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rt_api.h"

struct rt_mesh {
  std::vector<float> vtx;  // 6 floats per vertex: position, normal (reference Vertex, stride 24 B)
  std::vector<uint32_t> idx;
};

namespace {

// Parses one float the way `std::stringstream >> float` does on the reference (libstdc++ num_get
// accumulates [+-0-9.eE] characters, then converts with strtof). Returns false on failure.
bool parse_float(const char*& p, const char* end, float& out) {
  while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
  const char* b = p;
  while (p < end && ((*p >= '0' && *p <= '9') || *p == '+' || *p == '-' || *p == '.' || *p == 'e' ||
                     *p == 'E'))
    ++p;
  if (p == b) {
    out = 0.0f;
    return false;
  }
  std::string tok(b, p);
  char* ep = nullptr;
  float v = std::strtof(tok.c_str(), &ep);
  if (ep == tok.c_str()) {
    out = 0.0f;
    return false;
  }
  out = v;
  return true;
}

// `std::stringstream >> unsigned int`: optional sign (a '-' negates modulo 2^32), digits.
bool parse_uint(const char*& p, const char* end, uint32_t& out) {
  while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
  bool negative = false;
  if (p < end && (*p == '+' || *p == '-')) {
    negative = *p == '-';
    ++p;
  }
  if (p >= end || *p < '0' || *p > '9') {
    out = 0;
    return false;
  }
  uint64_t v = 0;
  bool overflow = false;
  while (p < end && *p >= '0' && *p <= '9') {
    v = v * 10 + (uint64_t)(*p - '0');
    if (v > 0xffffffffull) overflow = true;
    ++p;
  }
  if (overflow) {
    out = 0xffffffffu;
    return false;
  }
  uint32_t r = (uint32_t)v;
  out = negative ? (uint32_t)(0u - r) : r;
  return true;
}

void parse_obj_text(const char* text, size_t len, rt_mesh* m) {
  const char* p = text;
  const char* end = text + len;
  while (p < end) {
    const char* ls = p;
    while (p < end && *p != '\n') ++p;
    const char* le = p;
    if (p < end) ++p;  // consume '\n' (std::getline)
    if (le - ls < 2) continue;
    const char* q = ls + 1;
    if (ls[0] == 'v' && ls[1] == ' ') {
      // After the first failed extraction the stream is in a fail state: later values stay 0
      // (the reference leaves them uninitialised; pinned to 0 here).
      float xyz[3] = {0.0f, 0.0f, 0.0f};
      bool ok = true;
      for (int k = 0; k < 3 && ok; ++k) ok = parse_float(q, le, xyz[k]);
      m->vtx.insert(m->vtx.end(), {xyz[0], xyz[1], xyz[2], 0.0f, 1.0f, 0.0f});
    } else if (ls[0] == 'f' && ls[1] == ' ') {
      uint32_t ijk[3] = {0, 0, 0};
      bool ok = true;
      for (int k = 0; k < 3 && ok; ++k) ok = parse_uint(q, le, ijk[k]);
      for (int k = 0; k < 3; ++k) m->idx.push_back(ijk[k] - 1u);  // i0--, unsigned wrap
    }
  }
}

// XMVector3Normalize (SSE path): v / sqrt(dot(v, v)); zero length -> 0.
inline void xm_normalize3(const float v[3], float out[3]) {
  float len = std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
  if (len > 0.0f) {
    out[0] = v[0] / len;
    out[1] = v[1] / len;
    out[2] = v[2] / len;
  } else {
    out[0] = out[1] = out[2] = 0.0f;
  }
}

// glm 0.9.8 float helpers: dot = (x*y).x + (x*y).y + (x*y).z; normalize = v * (1 / sqrt(dot)).
inline float g_dot(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
inline void g_cross(const float x[3], const float y[3], float r[3]) {
  r[0] = x[1] * y[2] - y[1] * x[2];
  r[1] = x[2] * y[0] - y[2] * x[0];
  r[2] = x[0] * y[1] - y[0] * x[1];
}
inline void g_normalize(const float v[3], float r[3]) {
  float inv = 1.0f / std::sqrt(g_dot(v, v));
  r[0] = v[0] * inv;
  r[1] = v[1] * inv;
  r[2] = v[2] * inv;
}

// General 4x4 inverse of XMMATRIX memory (row-major rows r[i]) computed in double and rounded
// once to float (XMMatrixInverse; its exact operation order is not available: parity unpinned).
void inverse4(const float* mf, float* out) {
  double m[16], inv[16];
  for (int i = 0; i < 16; ++i) m[i] = mf[i];
  inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] +
           m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
  inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] -
           m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
  inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] +
           m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
  inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] -
            m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
  inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] -
           m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
  inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] +
           m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
  inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] -
           m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
  inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] +
            m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
  inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] +
           m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
  inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] -
           m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
  inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] +
            m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
  inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] -
            m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
  inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] -
           m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
  inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] +
           m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
  inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] -
            m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
  inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] +
            m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
  double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
  double r = det != 0.0 ? 1.0 / det : 0.0;  // singular: XMMatrixInverse yields inf/NaN; pinned to 0
  for (int i = 0; i < 16; ++i) out[i] = (float)(inv[i] * r);
}

}  // namespace

extern "C" {

rt_status rt_mesh_parse_obj(const char* text, size_t len, rt_mesh_t* out) {
  if (!out || (!text && len)) return RT_E_INVALID;
  rt_mesh* m = new (std::nothrow) rt_mesh();
  if (!m) return RT_E_OOM;
  try {
    if (len) parse_obj_text(text, len, m);
  } catch (...) {
    delete m;
    return RT_E_OOM;
  }
  *out = m;
  return RT_OK;
}

rt_status rt_mesh_load_obj(const char* path, rt_mesh_t* out) {
  if (!path || !out) return RT_E_INVALID;
  std::ifstream file(path, std::ios::binary);
  if (!file.good()) return RT_E_IO;  // LoadObjFile returns false (OBJ_FileManager.cpp:12-16)
  std::stringstream ss;
  ss << file.rdbuf();
  std::string s = ss.str();
  return rt_mesh_parse_obj(s.data(), s.size(), out);
}

void rt_mesh_free(rt_mesh_t mesh) { delete mesh; }
uint32_t rt_mesh_vertex_count(rt_mesh_t m) { return m ? (uint32_t)(m->vtx.size() / 6) : 0; }
uint32_t rt_mesh_index_count(rt_mesh_t m) { return m ? (uint32_t)m->idx.size() : 0; }
const float* rt_mesh_vertices(rt_mesh_t m) { return m && !m->vtx.empty() ? m->vtx.data() : nullptr; }
const uint32_t* rt_mesh_indices(rt_mesh_t m) { return m && !m->idx.empty() ? m->idx.data() : nullptr; }

rt_status rt_mesh_compute_vertex_normals(rt_mesh_t m) {
  if (!m) return RT_E_INVALID;
  const size_t nv = m->vtx.size() / 6;
  if (m->idx.size() % 3) return RT_E_INVALID;
  for (uint32_t i : m->idx)
    if (i >= nv) return RT_E_INVALID;  // the reference indexes out of bounds (UB): refused here
  std::vector<float> acc(nv * 3, 0.0f);
  for (size_t t = 0; t + 2 < m->idx.size(); t += 3) {
    const uint32_t i0 = m->idx[t], i1 = m->idx[t + 1], i2 = m->idx[t + 2];
    const float* p0 = &m->vtx[i0 * 6];
    const float* p1 = &m->vtx[i1 * 6];
    const float* p2 = &m->vtx[i2 * 6];
    float e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    float e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
    float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    float n[3];
    xm_normalize3(c, n);
    for (uint32_t vi : {i0, i1, i2}) {
      acc[vi * 3 + 0] = acc[vi * 3 + 0] + n[0];
      acc[vi * 3 + 1] = acc[vi * 3 + 1] + n[1];
      acc[vi * 3 + 2] = acc[vi * 3 + 2] + n[2];
    }
  }
  for (size_t v = 0; v < nv; ++v) {
    float n[3];
    xm_normalize3(&acc[v * 3], n);
    m->vtx[v * 6 + 3] = -n[0];
    m->vtx[v * 6 + 4] = -n[1];
    m->vtx[v * 6 + 5] = -n[2];
  }
  return RT_OK;
}

void rt_plane_vertices(float out[36]) {
  const float s = 40.0f;  // planeScale, D3D12HelloTriangle.cpp:1239
  const float pos[6][3] = {{-s, -1.0f, +s}, {+s, -1.0f, +s}, {-s, -1.0f, -s},
                           {-s, -1.0f, -s}, {+s, -1.0f, +s}, {+s, -1.0f, -s}};
  for (int i = 0; i < 6; ++i) {
    out[i * 6 + 0] = pos[i][0];
    out[i * 6 + 1] = pos[i][1];
    out[i * 6 + 2] = pos[i][2];
    out[i * 6 + 3] = 0.0f;  // Vertex default normal (0,1,0), D3D12HelloTriangle.h:55
    out[i * 6 + 4] = 1.0f;
    out[i * 6 + 5] = 0.0f;
  }
}

void rt_camera_lookat(const float eye[3], const float center[3], const float up[3], float view[16]) {
  float cme[3] = {center[0] - eye[0], center[1] - eye[1], center[2] - eye[2]};
  float f[3], s[3], u[3], fu[3];
  g_normalize(cme, f);
  g_cross(f, up, fu);
  g_normalize(fu, s);
  g_cross(s, f, u);
  // glm column-major memory: Result[c][r] at view[c*4 + r].
  float r[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  r[0 * 4 + 0] = s[0];
  r[1 * 4 + 0] = s[1];
  r[2 * 4 + 0] = s[2];
  r[0 * 4 + 1] = u[0];
  r[1 * 4 + 1] = u[1];
  r[2 * 4 + 1] = u[2];
  r[0 * 4 + 2] = -f[0];
  r[1 * 4 + 2] = -f[1];
  r[2 * 4 + 2] = -f[2];
  r[3 * 4 + 0] = -g_dot(s, eye);
  r[3 * 4 + 1] = -g_dot(u, eye);
  r[3 * 4 + 2] = g_dot(f, eye);
  std::memcpy(view, r, sizeof(r));
}

void rt_camera_buffer(const float view[16], uint32_t W, uint32_t H, float fov_deg, float znear,
                      float zfar, float cb[64]) {
  const float xm_pi = 3.141592654f;  // XM_PI
  float aspect = (float)W / (float)H;  // DXSample.cpp:27
  float fov = fov_deg * xm_pi / 180.0f;
  float half = 0.5f * fov;
  // XMScalarSinCos is a minimax polynomial; pinned to correctly rounded double sin/cos.
  float sinf_ = (float)std::sin((double)half), cosf_ = (float)std::cos((double)half);
  float height = cosf_ / sinf_;
  float width = height / aspect;
  float frange = zfar / (znear - zfar);
  float proj[16] = {width, 0, 0, 0, 0, height, 0, 0, 0, 0, frange, -1.0f, 0, 0, frange * znear, 0};
  std::memcpy(cb, view, 16 * sizeof(float));
  std::memcpy(cb + 16, proj, 16 * sizeof(float));
  inverse4(cb, cb + 32);
  inverse4(cb + 16, cb + 48);
}

}  // extern "C"
