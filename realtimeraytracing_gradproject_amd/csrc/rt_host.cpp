// rt_host.cpp — host services of the C-ABI: OBJ mesh ingest, vertex normals, ground plane and
// camera matrices. Pure host C++ (no HIP calls), so these run without a GPU.
//
// Behaviour follows the reference host code (paths relative to the reference tree):
//   OBJFileManager::LoadObjFile               src/OBJ_FileManager.cpp:10-71
//   D3D12HelloTriangle::ComputeVertexNormals  src/D3D12HelloTriangle.cpp:1430-1462
//   D3D12HelloTriangle::CreatePlaneVB         src/D3D12HelloTriangle.cpp:1237-1271
//   Manipulator::setLookat/update             src/manipulator.cpp:26-32, 305-314 (glm::lookAtRH)
//   D3D12HelloTriangle::UpdateCameraBuffer    src/D3D12HelloTriangle.cpp:1144-1170
//   Manipulator motion/mouseMove/wheel/orbit/pan/dolly/trackball
//                                             src/manipulator.cpp:135-445
#include <cfloat>
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
// `std::stringstream >> float` as the C++ library extracts it (libstdc++ num_get::_M_extract_float in the "C" locale,
// then __convert_to_v): the longest prefix of [sign] digits [. digits] [e|E [sign] digits] — a second '.', an 'e'
// before any digit or a second 'e' ends it — goes to strtof, which must consume all of it, else the value is 0 and the
// stream fails ("1e", "1e+", "+", "."); an overflow to +-inf gives +-FLT_MAX and fails the stream too. The stream
// stops right after the accepted characters ("1.5.5" reads 1.5, and the next value starts at ".5"). Pinned against
// the reference's code path compiled here (tests/golden/obj_malformed.json).
bool parse_float(const char*& p, const char* end, float& out) {
  while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
  std::string tok;
  if (p < end && (*p == '+' || *p == '-')) tok += *p++;
  bool mant = false, dec = false, sci = false;
  while (p < end) {
    const char ch = *p;
    if (ch >= '0' && ch <= '9') {
      tok += ch;
      mant = true;
    } else if (ch == '.' && !dec && !sci) {
      tok += '.';
      dec = true;
    } else if ((ch == 'e' || ch == 'E') && !sci && mant) {
      tok += 'e';
      sci = true;
      if (++p == end) break;
      if (*p != '+' && *p != '-') continue;  // the character after the 'e' is examined again
      tok += *p;
    } else {
      break;
    }
    ++p;
  }
  char* ep = nullptr;
  const float v = std::strtof(tok.c_str(), &ep);
  if (ep == tok.c_str() || *ep != '\0') {
    out = 0.0f;
    return false;
  }
  if (v == HUGE_VALF || v == -HUGE_VALF) {
    out = v > 0.0f ? FLT_MAX : -FLT_MAX;
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

// ---- glm 0.9.8.5 primitives the manipulator composes, in glm's evaluation order so the results
// are bit-identical (g++ -ffp-contract=off on both sides). Matrices are glm column-major:
// element (column c, row r) at [c * 4 + r].
inline float g_length(const float v[3]) { return std::sqrt(g_dot(v, v)); }

// glm::rotate(mat4 m, angle, v) (gtc/matrix_transform.inl:19-47); gtx rotate(angle, v) passes m = I.
void g_rotate(const float m[16], float angle, const float v[3], float out[16]) {
  const float c = std::cos(angle), s = std::sin(angle);
  float a[3];
  g_normalize(v, a);
  const float k = 1.0f - c;
  const float t[3] = {k * a[0], k * a[1], k * a[2]};
  float R[3][3];
  R[0][0] = c + t[0] * a[0];
  R[0][1] = t[0] * a[1] + s * a[2];
  R[0][2] = t[0] * a[2] - s * a[1];
  R[1][0] = t[1] * a[0] - s * a[2];
  R[1][1] = c + t[1] * a[1];
  R[1][2] = t[1] * a[2] + s * a[0];
  R[2][0] = t[2] * a[0] + s * a[1];
  R[2][1] = t[2] * a[1] - s * a[0];
  R[2][2] = c + t[2] * a[2];
  float r[16];
  for (int col = 0; col < 3; ++col)
    for (int row = 0; row < 4; ++row)
      r[col * 4 + row] = (m[0 * 4 + row] * R[col][0] + m[1 * 4 + row] * R[col][1]) + m[2 * 4 + row] * R[col][2];
  for (int row = 0; row < 4; ++row) r[12 + row] = m[12 + row];
  std::memcpy(out, r, sizeof(r));
}

void g_rotate_identity(float angle, const float v[3], float out[16]) {
  const float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  g_rotate(I, angle, v, out);
}

// mat4 * vec4 (detail/type_mat4x4.inl:501-546): (c0*v0 + c1*v1) + (c2*v2 + c3*v3).
void g_mul_vec(const float m[16], const float v[4], float out[4]) {
  float r[4];
  for (int row = 0; row < 4; ++row)
    r[row] = (m[row] * v[0] + m[4 + row] * v[1]) + (m[8 + row] * v[2] + m[12 + row] * v[3]);
  std::memcpy(out, r, sizeof(r));
}

// mat4 * mat4 (detail/type_mat4x4.inl:595-613): column c = ((A0*B[c].x + A1*B[c].y) + A2*B[c].z) + A3*B[c].w.
void g_mul_mat(const float A[16], const float B[16], float out[16]) {
  float r[16];
  for (int col = 0; col < 4; ++col)
    for (int row = 0; row < 4; ++row)
      r[col * 4 + row] = ((A[row] * B[col * 4 + 0] + A[4 + row] * B[col * 4 + 1]) + A[8 + row] * B[col * 4 + 2]) +
                         A[12 + row] * B[col * 4 + 3];
  std::memcpy(out, r, sizeof(r));
}

// isZero / sign, manipulator.h:174-177, 183-186
inline bool m_is_zero(float a) { return std::fabs(a) < 1.1920928955078125e-07f; }
inline float m_sign(float s) { return s < 0.f ? -1.f : 1.f; }

// Manipulator::pan (manipulator.cpp:319-339): move eye and interest in the view plane.
void manip_pan(rt_manipulator* m, float dx, float dy) {
  if (m->mode == RT_MANIP_FLY) {
    dx *= -1;
    dy *= -1;
  }
  float z[3] = {m->pos[0] - m->interest[0], m->pos[1] - m->interest[1], m->pos[2] - m->interest[2]};
  const float reach = g_length(z) / 0.785f;  // a 45-degree field spans the eye distance
  float zn[3], xc[3], x[3], yc[3], y[3];
  g_normalize(z, zn);
  g_cross(m->up, zn, xc);
  g_normalize(xc, x);
  g_cross(zn, x, yc);
  g_normalize(yc, y);
  const float sx = -dx * reach, sy = dy * reach;
  for (int i = 0; i < 3; ++i) {
    const float d = x[i] * sx + y[i] * sy;
    m->pos[i] += d;
    m->interest[i] += d;
  }
}

// Manipulator::orbit (:345-398): rotate the eye about the interest point (or, inverted, the
// interest point about the eye) by dx turns about `up`, then dy turns about the view x axis; the
// tilt is dropped when it would flip the arm's x sign.
void manip_orbit(rt_manipulator* m, float dx, float dy, bool about_eye) {
  if (m_is_zero(dx) && m_is_zero(dy)) return;
  const float two_pi = 6.28318530717958647692f;
  dx *= two_pi;
  dy *= two_pi;
  const float* pivot = about_eye ? m->pos : m->interest;
  float* moving = about_eye ? m->interest : m->pos;
  float arm[3] = {moving[0] - pivot[0], moving[1] - pivot[1], moving[2] - pivot[2]};
  const float radius = g_length(arm);
  g_normalize(arm, arm);
  float zaxis[3];
  g_normalize(arm, zaxis);
  float rot[16], v4[4];
  g_rotate_identity(dx, m->up, rot);
  const float a4[4] = {arm[0], arm[1], arm[2], 0.0f};
  g_mul_vec(rot, a4, v4);
  arm[0] = v4[0];
  arm[1] = v4[1];
  arm[2] = v4[2];
  float xc[3], xaxis[3];
  g_cross(m->up, zaxis, xc);
  g_normalize(xc, xaxis);
  g_rotate_identity(dy, xaxis, rot);
  const float b4[4] = {arm[0], arm[1], arm[2], 0.0f};
  g_mul_vec(rot, b4, v4);
  if (m_sign(v4[0]) == m_sign(arm[0])) {
    arm[0] = v4[0];
    arm[1] = v4[1];
    arm[2] = v4[2];
  }
  const float p[3] = {pivot[0], pivot[1], pivot[2]};
  for (int i = 0; i < 3; ++i) moving[i] = arm[i] * radius + p[i];
}

// Manipulator::dolly (:403-445): move toward the interest point, never onto or through it.
void manip_dolly(rt_manipulator* m, float dx, float dy) {
  float z[3] = {m->interest[0] - m->pos[0], m->interest[1] - m->pos[1], m->interest[2] - m->pos[2]};
  float len = g_length(z);
  if (m_is_zero(len)) return;
  const float dd = m->mode != RT_MANIP_EXAMINE ? -dy : (std::fabs(dx) > std::fabs(dy) ? dx : -dy);
  float factor = m->speed * dd / len;
  len /= 10;
  len = len < 0.001f ? 0.001f : len;
  factor *= len;
  if (factor >= 1.0f) return;
  for (int i = 0; i < 3; ++i) z[i] *= factor;
  if (m->mode == RT_MANIP_WALK) {  // keep the height
    if (m->up[1] > m->up[2])
      z[1] = 0;
    else
      z[2] = 0;
  }
  for (int i = 0; i < 3; ++i) m->pos[i] += z[i];
  if (m->mode != RT_MANIP_EXAMINE)
    for (int i = 0; i < 3; ++i) m->interest[i] += z[i];
}

// projectOntoTBSphere (:283-300): sphere of radius tbsize near the centre, hyperbolic sheet beyond.
double manip_sphere_z(const rt_manipulator* m, const float p[2]) {
  const double d = std::sqrt(p[0] * p[0] + p[1] * p[1]);  // glm::length(vec2), float
  if (d < m->tbsize * 0.70710678118654752440) return std::sqrt(m->tbsize * m->tbsize - d * d);
  const double t = m->tbsize / 1.41421356237309504880;
  return t * t / d;
}

// Manipulator::trackball (:242-277): rotate eye and up about the axis through the two projected
// mouse points, expressed in world space by the current matrix.
void manip_trackball(rt_manipulator* m, int32_t x, int32_t y) {
  const int hw = m->width / 2, hh = m->height / 2;
  const float p0[2] = {(float)(2 * (m->mouse[0] - hw) / double(m->width)),
                       (float)(2 * (hh - m->mouse[1]) / double(m->height))};
  const float p1[2] = {(float)(2 * (x - hw) / double(m->width)), (float)(2 * (hh - y) / double(m->height))};
  const float a[3] = {p0[0], p0[1], (float)manip_sphere_z(m, p0)};
  const float b[3] = {p1[0], p1[1], (float)manip_sphere_z(m, p1)};
  float ac[3], axis[3];
  g_cross(a, b, ac);
  g_normalize(ac, axis);
  const float dab[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  double t = g_length(dab) / (2.f * m->tbsize);
  if (t > 1.0)
    t = 1.0;
  else if (t < -1.0)
    t = -1.0;
  const float rad = (float)(2.0 * std::asin(t));
  const float ax4[4] = {axis[0], axis[1], axis[2], 0.0f};
  float wa[4], rot[16];
  g_mul_vec(m->matrix, ax4, wa);
  g_rotate_identity(rad, wa, rot);
  const float off[4] = {m->pos[0] - m->interest[0], m->pos[1] - m->interest[1], m->pos[2] - m->interest[2], 1.0f};
  float o2[4];
  g_mul_vec(rot, off, o2);
  for (int i = 0; i < 3; ++i) m->pos[i] = m->interest[i] + o2[i];
  const float u4[4] = {m->up[0], m->up[1], m->up[2], 0.0f};
  float u2[4];
  g_mul_vec(rot, u4, u2);
  std::memcpy(m->up, u2, 12);
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

void rt_manip_init(rt_manipulator* m) {
  const float pos[3] = {10, 10, 10}, itr[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  std::memcpy(m->pos, pos, 12);
  std::memcpy(m->interest, itr, 12);
  std::memcpy(m->up, up, 12);
  m->roll = 0;
  m->width = m->height = 1;
  m->speed = 30;
  m->mouse[0] = m->mouse[1] = 0;
  m->tbsize = 0.8f;
  m->mode = RT_MANIP_EXAMINE;
  rt_manip_update(m);
}

void rt_manip_update(rt_manipulator* m) {
  rt_camera_lookat(m->pos, m->interest, m->up, m->matrix);
  if (!m_is_zero(m->roll)) {
    const float zaxis[3] = {0, 0, 1};
    float rot[16];
    g_rotate_identity(m->roll, zaxis, rot);
    g_mul_mat(m->matrix, rot, m->matrix);
  }
}

void rt_manip_set_lookat(rt_manipulator* m, const float eye[3], const float center[3], const float up[3]) {
  std::memmove(m->pos, eye, 12);
  std::memmove(m->interest, center, 12);
  std::memmove(m->up, up, 12);
  rt_manip_update(m);
}

void rt_manip_set_roll(rt_manipulator* m, float roll) {
  m->roll = roll;
  rt_manip_update(m);
}

void rt_manip_set_window_size(rt_manipulator* m, int32_t w, int32_t h) {
  m->width = w;
  m->height = h;
}

void rt_manip_set_mouse_position(rt_manipulator* m, int32_t x, int32_t y) {
  m->mouse[0] = static_cast<float>(x);
  m->mouse[1] = static_cast<float>(y);
}

void rt_manip_motion(rt_manipulator* m, int32_t x, int32_t y, int32_t action) {
  const float dx = float(x - m->mouse[0]) / float(m->width);
  const float dy = float(y - m->mouse[1]) / float(m->height);
  switch (action) {
    case RT_MANIP_ORBIT:
      manip_orbit(m, dx, dy, m->mode == RT_MANIP_TRACKBALL);
      break;
    case RT_MANIP_DOLLY:
      manip_dolly(m, dx, dy);
      break;
    case RT_MANIP_PAN:
      manip_pan(m, dx, dy);
      break;
    case RT_MANIP_LOOK_AROUND:
      if (m->mode == RT_MANIP_TRACKBALL)
        manip_trackball(m, x, y);
      else
        manip_orbit(m, dx, -dy, true);
      break;
    default:
      break;
  }
  rt_manip_update(m);
  m->mouse[0] = static_cast<float>(x);
  m->mouse[1] = static_cast<float>(y);
}

int32_t rt_manip_mouse_move(rt_manipulator* m, int32_t x, int32_t y, uint32_t in) {
  int32_t act = RT_MANIP_NONE;
  const bool examine = m->mode == RT_MANIP_EXAMINE;
  if (in & RT_INPUT_LMB) {
    if (((in & RT_INPUT_CTRL) && (in & RT_INPUT_SHIFT)) || (in & RT_INPUT_ALT))
      act = examine ? RT_MANIP_LOOK_AROUND : RT_MANIP_ORBIT;
    else if (in & RT_INPUT_SHIFT)
      act = RT_MANIP_DOLLY;
    else if (in & RT_INPUT_CTRL)
      act = RT_MANIP_PAN;
    else
      act = examine ? RT_MANIP_ORBIT : RT_MANIP_LOOK_AROUND;
  } else if (in & RT_INPUT_MMB) {
    act = RT_MANIP_PAN;
  } else if (in & RT_INPUT_RMB) {
    act = RT_MANIP_DOLLY;
  }
  if (act != RT_MANIP_NONE) rt_manip_motion(m, x, y, act);
  return act;
}

void rt_manip_wheel(rt_manipulator* m, int32_t value) {
  const float v = static_cast<float>(value);
  const float dx = (v * std::fabs(v)) / static_cast<float>(m->width);
  manip_dolly(m, dx * m->speed, dx * m->speed);
  rt_manip_update(m);
}

}  // extern "C"
