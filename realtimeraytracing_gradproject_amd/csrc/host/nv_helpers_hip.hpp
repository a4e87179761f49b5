// nv_helpers_hip.hpp — C++ host mirror of the reference's acceleration-structure helpers, ingest
// and camera manipulator, implemented over the C-ABI (include/rt_api.h). Same class and method
// names, argument meaning and error behaviour (std::logic_error for misuse, std::runtime_error
// for a failed call — the reference's ThrowIfFailed, DXSampleHelper.h:16-22), so application code
// written against nv_helpers_dx12 ports by swapping the namespace:
//
//   nv_helpers_dx12::BottomLevelASGenerator  nv_helpers_dx12/BottomLevelASGenerator.h:61-170
//   nv_helpers_dx12::TopLevelASGenerator     nv_helpers_dx12/TopLevelASGenerator.h:68-170
//   OBJFileManager                           include/OBJ_FileManager.h:6-17
//   nv_helpers_dx12::Manipulator / CameraManip  include/manipulator.h:33-148
//
// GPU buffers: the D3D12 versions take ID3D12Resource* for vertex/index data; here the geometry is
// passed as host pointers and the device copy is owned by the rt_ctx (the build copies it).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/rt_api.h"

namespace objl {
struct Vector3 {
  float X = 0, Y = 0, Z = 0;
  Vector3() = default;
  Vector3(float x, float y, float z) : X(x), Y(y), Z(z) {}
};
struct Vertex {  // include/OBJ_Loader.h:86-96 (only Position is filled by LoadObjFile)
  Vector3 Position;
};
}  // namespace objl

namespace nv_helpers_hip {

inline void ThrowIfFailed(rt_status st, rt_ctx_t ctx, const char* what) {
  if (st != RT_OK) {
    std::string msg = std::string(what) + " failed: " + rt_status_string(st);
    if (ctx) msg += std::string(" (") + rt_last_error(ctx) + ")";
    throw std::runtime_error(msg);
  }
}

// OBJFileManager::LoadObjFile (src/OBJ_FileManager.cpp:10-71): returns false when the file cannot
// be opened; appends to the output vectors like the reference.
class OBJFileManager {
 public:
  bool LoadObjFile(std::string path, std::vector<objl::Vertex>& vertices, std::vector<unsigned int>& indices) {
    rt_mesh_t m = nullptr;
    rt_status st = rt_mesh_load_obj(path.c_str(), &m);
    if (st == RT_E_IO) return false;
    ThrowIfFailed(st, nullptr, "rt_mesh_load_obj");
    const uint32_t nv = rt_mesh_vertex_count(m), ni = rt_mesh_index_count(m);
    const float* v = rt_mesh_vertices(m);
    const uint32_t* i = rt_mesh_indices(m);
    for (uint32_t k = 0; k < nv; ++k) {
      objl::Vertex vx;
      vx.Position = objl::Vector3(v[k * 6], v[k * 6 + 1], v[k * 6 + 2]);
      vertices.push_back(vx);
    }
    indices.insert(indices.end(), i, i + ni);
    rt_mesh_free(m);
    return true;
  }
};

// BottomLevelASGenerator: AddVertexBuffer* -> ComputeASBufferSizes -> Generate.
class BottomLevelASGenerator {
 public:
  // AddVertexBuffer overloads (BottomLevelASGenerator.h:84-128). vertexBuffer: host array of
  // vertexCount vertices of vertexSizeInBytes bytes, float3 position first (normal at +12 when
  // the stride is >= 24). indexBuffer == nullptr: non-indexed. transformBuffer must be null
  // (the reference never passes one, D3D12HelloTriangle.cpp:697-706).
  void AddVertexBuffer(const void* vertexBuffer, uint64_t vertexOffsetInBytes, uint32_t vertexCount,
                       uint32_t vertexSizeInBytes, const void* transformBuffer, uint64_t transformOffsetInBytes,
                       bool isOpaque = true) {
    AddVertexBuffer(vertexBuffer, vertexOffsetInBytes, vertexCount, vertexSizeInBytes, nullptr, 0, 0,
                    transformBuffer, transformOffsetInBytes, isOpaque);
  }
  void AddVertexBuffer(const void* vertexBuffer, uint64_t vertexOffsetInBytes, uint32_t vertexCount,
                       uint32_t vertexSizeInBytes, const uint32_t* indexBuffer, uint64_t indexOffsetInBytes,
                       uint32_t indexCount, const void* transformBuffer, uint64_t transformOffsetInBytes,
                       bool isOpaque = true) {
    (void)transformOffsetInBytes;
    (void)isOpaque;  // every triangle is opaque: no any-hit programs exist in the reference
    if (transformBuffer) throw std::logic_error("BottomLevelASGenerator: per-geometry transforms are not supported");
    if (vertexSizeInBytes < 12 || vertexSizeInBytes % 4) throw std::logic_error("BottomLevelASGenerator: bad vertex stride");
    if (m_sizesComputed) throw std::logic_error("BottomLevelASGenerator: AddVertexBuffer after ComputeASBufferSizes");
    const unsigned char* vb = static_cast<const unsigned char*>(vertexBuffer) + vertexOffsetInBytes;
    const uint32_t base = (uint32_t)(m_vtx.size() / 6);
    for (uint32_t k = 0; k < vertexCount; ++k) {
      const float* p = reinterpret_cast<const float*>(vb + (size_t)k * vertexSizeInBytes);
      m_vtx.insert(m_vtx.end(), {p[0], p[1], p[2]});
      if (vertexSizeInBytes >= 24) m_vtx.insert(m_vtx.end(), {p[3], p[4], p[5]});
      else m_vtx.insert(m_vtx.end(), {0.0f, 1.0f, 0.0f});
    }
    // geometries are concatenated into one primitive range (the reference uses one per BLAS)
    if (indexBuffer) {
      const uint32_t* ib = reinterpret_cast<const uint32_t*>(reinterpret_cast<const unsigned char*>(indexBuffer) +
                                                             indexOffsetInBytes);
      for (uint32_t k = 0; k < indexCount; ++k) m_idx.push_back(ib[k] + base);
    } else {
      for (uint32_t k = 0; k < vertexCount; ++k) m_idx.push_back(base + k);
    }
  }

  // BottomLevelASGenerator.cpp:123-170. Sizes are the device bytes the build will hold.
  void ComputeASBufferSizes(rt_ctx_t ctx, bool allowUpdate, uint64_t* scratchSizeInBytes, uint64_t* resultSizeInBytes) {
    (void)ctx;
    (void)allowUpdate;
    if (m_idx.empty()) throw std::logic_error("BottomLevelASGenerator: no geometry added");
    const uint64_t ntri = m_idx.size() / 3;
    *scratchSizeInBytes = ntri * (48 + 24 + 4 * 6);
    *resultSizeInBytes = (ntri > 1 ? ntri - 1 : 1) * 64 + ntri * 48 + m_vtx.size() * 4 + m_idx.size() * 4;
    m_sizesComputed = true;
  }

  // BottomLevelASGenerator.cpp:177-245: builds on the device; returns the BLAS handle.
  // updateOnly/previousResult: a rebuild of `previousResult` in place (model hot-reload).
  rt_blas_t Generate(rt_ctx_t ctx, bool updateOnly = false, rt_blas_t previousResult = 0) {
    if (!m_sizesComputed) throw std::logic_error("BottomLevelASGenerator: call ComputeASBufferSizes before Generate");
    const uint32_t nv = (uint32_t)(m_vtx.size() / 6);
    rt_blas_t out = previousResult;
    if (updateOnly)
      ThrowIfFailed(rt_blas_rebuild(ctx, previousResult, m_vtx.data(), nv, 24, m_idx.data(), (uint32_t)m_idx.size()),
                    ctx, "rt_blas_rebuild");
    else
      ThrowIfFailed(rt_blas_build(ctx, m_vtx.data(), nv, 24, m_idx.data(), (uint32_t)m_idx.size(), &out), ctx,
                    "rt_blas_build");
    return out;
  }

 private:
  std::vector<float> m_vtx;
  std::vector<uint32_t> m_idx;
  bool m_sizesComputed = false;
};

// 4x4 row-major matrix in XMMATRIX convention (row vectors, translation in row 3), as the
// reference passes to AddInstance.
struct Matrix4 {
  float m[16];
  static Matrix4 Identity() { return Matrix4{{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}}; }
  static Matrix4 Translation(float x, float y, float z) {  // XMMatrixTranslation
    Matrix4 r = Identity();
    r.m[12] = x;
    r.m[13] = y;
    r.m[14] = z;
    return r;
  }
};

class TopLevelASGenerator {
 public:
  // TopLevelASGenerator.h:88-99; the desc transform is XMMatrixTranspose(transform) as 3x4
  // (TopLevelASGenerator.cpp:190-192).
  void AddInstance(rt_blas_t bottomLevelAS, const Matrix4& transform, uint32_t instanceID, uint32_t hitGroupIndex) {
    rt_instance d{};
    d.blas = bottomLevelAS;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 4; ++c) d.xform3x4_rowmajor[r * 4 + c] = transform.m[c * 4 + r];
    d.instance_id = instanceID;
    d.hit_group = hitGroupIndex;
    m_instances.push_back(d);
  }
  void ComputeASBufferSizes(rt_ctx_t, bool allowUpdate, uint64_t* scratchSizeInBytes, uint64_t* resultSizeInBytes,
                            uint64_t* descriptorsSizeInBytes) {
    if (m_instances.empty()) throw std::logic_error("TopLevelASGenerator: no instances added");
    const uint64_t n = m_instances.size();
    *scratchSizeInBytes = n * 64;
    *resultSizeInBytes = (n > 1 ? n - 1 : 1) * 64;
    *descriptorsSizeInBytes = n * sizeof(rt_instance);
    m_allowUpdate = allowUpdate;
    m_sizesComputed = true;
  }
  // TopLevelASGenerator.cpp:148-249 (update path :202-222 requires allowUpdate).
  void Generate(rt_ctx_t ctx, bool updateOnly = false) {
    if (!m_sizesComputed) throw std::logic_error("TopLevelASGenerator: call ComputeASBufferSizes before Generate");
    if (updateOnly && !m_allowUpdate) throw std::logic_error("Cannot update a top-level AS not originally built for updates");
    ThrowIfFailed(rt_tlas_build(ctx, m_instances.data(), (uint32_t)m_instances.size(), updateOnly ? 1 : 0), ctx,
                  "rt_tlas_build");
  }
  void SetTransform(size_t i, const Matrix4& transform) {  // for refits
    TopLevelASGenerator tmp;
    tmp.AddInstance(m_instances.at(i).blas, transform, 0, 0);
    std::memcpy(m_instances[i].xform3x4_rowmajor, tmp.m_instances[0].xform3x4_rowmajor, sizeof(float) * 12);
  }

 private:
  std::vector<rt_instance> m_instances;
  bool m_allowUpdate = false;
  bool m_sizesComputed = false;
};

// Camera manipulator (manipulator.h:33-148) over the C-ABI rt_manip_* state: same class, enums and
// methods as nv_helpers_dx12::Manipulator; getMatrix() is the glm column-major view matrix.
class Manipulator {
 public:
  enum Modes { Examine = RT_MANIP_EXAMINE, Fly = RT_MANIP_FLY, Walk = RT_MANIP_WALK, Trackball = RT_MANIP_TRACKBALL };
  enum Actions { None = RT_MANIP_NONE, Orbit = RT_MANIP_ORBIT, Dolly = RT_MANIP_DOLLY, Pan = RT_MANIP_PAN,
                 LookAround = RT_MANIP_LOOK_AROUND };
  struct Inputs {
    bool lmb = false, mmb = false, rmb = false, shift = false, ctrl = false, alt = false;
    uint32_t bits() const {
      return (lmb ? RT_INPUT_LMB : 0u) | (mmb ? RT_INPUT_MMB : 0u) | (rmb ? RT_INPUT_RMB : 0u) |
             (shift ? RT_INPUT_SHIFT : 0u) | (ctrl ? RT_INPUT_CTRL : 0u) | (alt ? RT_INPUT_ALT : 0u);
    }
  };

  Manipulator() { rt_manip_init(&m_state); }
  Actions mouseMove(int x, int y, const Inputs& inputs) {
    return static_cast<Actions>(rt_manip_mouse_move(&m_state, x, y, inputs.bits()));
  }
  void setLookat(const float eye[3], const float center[3], const float up[3]) {
    rt_manip_set_lookat(&m_state, eye, center, up);
  }
  void getLookat(float eye[3], float center[3], float up[3]) const {
    std::memcpy(eye, m_state.pos, 12);
    std::memcpy(center, m_state.interest, 12);
    std::memcpy(up, m_state.up, 12);
  }
  void setWindowSize(int w, int h) { rt_manip_set_window_size(&m_state, w, h); }
  void setMousePosition(int x, int y) { rt_manip_set_mouse_position(&m_state, x, y); }
  void getMousePosition(int& x, int& y) const {
    x = static_cast<int>(m_state.mouse[0]);
    y = static_cast<int>(m_state.mouse[1]);
  }
  void setMode(Modes mode) { m_state.mode = mode; }
  Modes getMode() const { return static_cast<Modes>(m_state.mode); }
  void setRoll(float roll) { rt_manip_set_roll(&m_state, roll); }
  float getRoll() const { return m_state.roll; }
  const float* getMatrix() const { return m_state.matrix; }
  void setSpeed(float speed) { m_state.speed = speed; }
  float getSpeed() const { return m_state.speed; }
  void motion(int x, int y, int action = 0) { rt_manip_motion(&m_state, x, y, action); }
  void wheel(int value) { rt_manip_wheel(&m_state, value); }
  int getWidth() const { return m_state.width; }
  int getHeight() const { return m_state.height; }

 private:
  rt_manipulator m_state;
};

inline Manipulator& CameraManip() {  // manipulator.h:148 singleton
  static Manipulator m;
  return m;
}

}  // namespace nv_helpers_hip
