// rt_app.cpp — headless equivalent of the reference application class D3D12HelloTriangle
// (src/D3D12HelloTriangle.cpp), written against the C++ host mirror (nv_helpers_hip.hpp) over
// the C-ABI. OnInit / OnUpdate / OnRender / OnDestroy follow the reference's structure; the
// swap chain is replaced by a PPM dump of the RGBA8 frame and frame times are measured with HIP
// events instead of the vsync-bound chrono timer (:423, :466-470).
//
//   rt_app --model teapot.obj [--scene ref|single|grid8|grid16] [--width W --height H]
//          [--lights N] [--mode ref|lambert_shadow|primary] [--spp S] [--frames F]
//          [--eye x y z --center x y z] [--out frame.ppm] [--raw frame.rgba]
//          [--drag BUTTONS DX DY] [--out-pattern frame_%03d.ppm]
//          [--ranks N --rank R --comm-id FILE]
//
// --ranks tiles every frame over N processes (one per GPU, device = R % visible GPUs) through the C-ABI's
// frame loop: rt_render_strips renders rank R's interleaved strips, ncclGathers them into rank 0 and assembles
// the frame there. Rank 0 writes the communicator id (ncclGetUniqueId) to FILE, the other ranks
// read it; --ranks 1 runs the same loop over a world-1 communicator. Only rank 0 writes frames.
//
// --drag replays a mouse drag through the manipulator, as the reference's window messages do
// (OnButtonDown / OnMouseMove, D3D12HelloTriangle.cpp:1206-1234): button down at the window
// centre, then every frame the pointer moves by (DX, DY) pixels with BUTTONS held — a '+'-joined
// subset of lmb, mmb, rmb, shift, ctrl, alt (e.g. lmb = orbit, rmb = dolly, mmb = pan,
// lmb+alt = look around). --out-pattern writes every frame (printf pattern with the frame index).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nv_helpers_hip.hpp"

using namespace nv_helpers_hip;

namespace {

const rt_light kLights[6] = {  // Hit.hlsl:51-56
    {{1, 1, 1}, {0, 10, 0}, 0.2f},  {{1, 1, 1}, {10, 10, 0}, 0.2f},  {{1, 1, 1}, {-10, 10, 0}, 0.2f},
    {{1, 1, 1}, {0, 10, 10}, 0.2f}, {{1, 1, 1}, {0, 10, -10}, 0.2f}, {{1, 1, 1}, {0, -10, 0}, 0.2f}};

struct Options {
  std::string model = "teapot.obj", scene = "ref", mode = "ref", out, raw, drag, out_pattern;
  int drag_dx = 0, drag_dy = 0;
  int width = 1280, height = 720, lights = 6, spp = 1, frames = 1;
  int ranks = 0, rank = 0;  // --ranks N: frames tiled over N processes (0: one GPU, no communicator)
  std::string comm_id;
  float eye[3] = {1.5f, 1.5f, 1.5f}, center[3] = {0, 0, 0}, up[3] = {0, 1, 0};
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

class RayTracingApp {
 public:
  explicit RayTracingApp(const Options& o) : m_opt(o) {}

  // D3D12HelloTriangle::OnInit (:40-82)
  void OnInit() {
    CameraManip().setWindowSize(m_opt.width, m_opt.height);
    CameraManip().setLookat(m_opt.eye, m_opt.center, m_opt.up);
    int ndev = 1;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    ThrowIfFailed(rt_create(m_opt.ranks > 0 ? m_opt.rank % ndev : 0, &m_ctx), nullptr, "rt_create");
    LoadAssets();
    CreateAccelerationStructures();
    hip_check(hipMalloc(&m_output, (size_t)m_opt.width * m_opt.height * 4), "hipMalloc(output)");
    hip_check(hipStreamCreate(&m_stream), "hipStreamCreate");
    if (m_opt.ranks > 0) CreateCommunicator();
  }

  // The multi-GPU frame loop: rank 0's ncclUniqueId travels through a file (no MPI in this app).
  void CreateCommunicator() {
    unsigned char id[RT_COMM_ID_BYTES];
    if (m_opt.rank == 0) {
      ThrowIfFailed(rt_comm_get_unique_id(id), nullptr, "rt_comm_get_unique_id");
      if (m_opt.ranks > 1) {
        const std::string tmp = m_opt.comm_id + ".tmp";
        std::ofstream(tmp, std::ios::binary).write((const char*)id, sizeof(id));
        if (std::rename(tmp.c_str(), m_opt.comm_id.c_str()) != 0) throw std::runtime_error("cannot write " + m_opt.comm_id);
      }
    } else {
      for (int tries = 0;; ++tries) {
        std::ifstream f(m_opt.comm_id, std::ios::binary);
        if (f && f.read((char*)id, sizeof(id)) && f.gcount() == (std::streamsize)sizeof(id)) break;
        if (tries > 3000) throw std::runtime_error("no communicator id in " + m_opt.comm_id);
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    }
    ThrowIfFailed(rt_comm_init(m_ctx, (uint32_t)m_opt.ranks, (uint32_t)m_opt.rank, id, &m_comm), m_ctx, "rt_comm_init");
  }

  // D3D12HelloTriangle::OnButtonDown (:1206-1212): the reference negates the window coordinates
  void OnButtonDown(int x, int y) { CameraManip().setMousePosition(-x, -y); }

  // D3D12HelloTriangle::OnMouseMove (:1214-1234): no button held -> ignored
  void OnMouseMove(const Manipulator::Inputs& in, int x, int y) {
    if (!in.lmb && !in.rmb && !in.mmb) return;
    CameraManip().mouseMove(-x, -y, in);
  }

  // D3D12HelloTriangle::OnUpdate (:421-433): material from the UI defaults, camera buffer
  void OnUpdate() {
    rt_material mat = {{1, 1, 1}, 0.5f, 0.5f, 0.0f};  // UIConstructor.cpp:13-17, reflectivity pinned 0
    int mode = m_opt.mode == "ref" ? RT_SHADE_REF : m_opt.mode == "primary" ? RT_SHADE_PRIMARY : RT_SHADE_LAMBERT_SHADOW;
    ThrowIfFailed(rt_set_shading(m_ctx, kLights, (uint32_t)m_opt.lights, &mat, mode, m_opt.spp), m_ctx, "rt_set_shading");
    float cb[64];
    rt_camera_buffer(CameraManip().getMatrix(), (uint32_t)m_opt.width, (uint32_t)m_opt.height, 45.0f, 0.1f, 1000.0f, cb);
    ThrowIfFailed(rt_set_camera(m_ctx, cb), m_ctx, "rt_set_camera");
  }

  // D3D12HelloTriangle::OnRender (:436-471): dispatch, then wait (the fence)
  float OnRender() {
    hipEvent_t a, b;
    hip_check(hipEventCreate(&a), "event");
    hip_check(hipEventCreate(&b), "event");
    hip_check(hipEventRecord(a, m_stream), "event");
    if (m_comm) {
      // the frame tiled over the ranks: strips rendered here, gathered and assembled on rank 0
      const rt_status st = rt_render_strips(m_comm, (uint32_t)m_opt.width, (uint32_t)m_opt.height, 8, m_output, m_stream);
      if (st != RT_OK) throw std::runtime_error(std::string("rt_render_strips: ") + rt_comm_last_error(m_comm));
      // the frame is complete when the communicator's stream is: the timing stream waits for it
      hipEvent_t done;
      hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), "event");
      hip_check(hipEventRecord(done, (hipStream_t)rt_comm_stream(m_comm)), "event");
      hip_check(hipStreamWaitEvent(m_stream, done, 0), "event");
      (void)hipEventDestroy(done);
    } else {
      ThrowIfFailed(rt_dispatch_rays(m_ctx, (uint32_t)m_opt.width, (uint32_t)m_opt.height, nullptr, 0, m_output,
                                     nullptr, m_stream),
                    m_ctx, "rt_dispatch_rays");
    }
    hip_check(hipEventRecord(b, m_stream), "event");
    hip_check(hipStreamSynchronize(m_stream), "WaitForPreviousFrame");
    float ms = 0;
    hip_check(hipEventElapsedTime(&ms, a, b), "elapsed");
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms;
  }

  // The swap-chain copy (:599-607) becomes a file dump: PPM (RGB) and/or raw RGBA8.
  void Save(const std::string& ppm, const std::string& raw) {
    std::vector<unsigned char> px((size_t)m_opt.width * m_opt.height * 4);
    hip_check(hipMemcpy(px.data(), m_output, px.size(), hipMemcpyDeviceToHost), "download");
    if (!raw.empty()) {
      FILE* f = std::fopen(raw.c_str(), "wb");
      if (!f) throw std::runtime_error("cannot write " + raw);
      std::fwrite(px.data(), 1, px.size(), f);
      std::fclose(f);
    }
    if (!ppm.empty()) {
      FILE* f = std::fopen(ppm.c_str(), "wb");
      if (!f) throw std::runtime_error("cannot write " + ppm);
      std::fprintf(f, "P6\n%d %d\n255\n", m_opt.width, m_opt.height);
      for (size_t i = 0; i < px.size(); i += 4) std::fwrite(&px[i], 1, 3, f);
      std::fclose(f);
    }
  }

  bool IsRoot() const { return m_opt.ranks == 0 || m_opt.rank == 0; }

  void OnDestroy() {
    if (m_comm) rt_comm_destroy(m_comm);
    m_comm = nullptr;
    if (m_output) (void)hipFree(m_output);
    if (m_stream) (void)hipStreamDestroy(m_stream);
    if (m_ctx) rt_destroy(m_ctx);
  }

 private:
  // LoadAssets (:201-400): OBJ ingest + ComputeVertexNormals, plane VB
  void LoadAssets() {
    rt_mesh_t mesh = nullptr;
    rt_status st = rt_mesh_load_obj(m_opt.model.c_str(), &mesh);
    if (st == RT_E_IO) throw std::runtime_error("cannot open " + m_opt.model);  // assert at :337
    ThrowIfFailed(st, nullptr, "rt_mesh_load_obj");
    ThrowIfFailed(rt_mesh_compute_vertex_normals(mesh), nullptr, "ComputeVertexNormals");
    m_vertices.assign(rt_mesh_vertices(mesh), rt_mesh_vertices(mesh) + rt_mesh_vertex_count(mesh) * 6);
    m_indices.assign(rt_mesh_indices(mesh), rt_mesh_indices(mesh) + rt_mesh_index_count(mesh));
    rt_mesh_free(mesh);
    m_plane.resize(36);
    rt_plane_vertices(m_plane.data());
  }

  // CreateAccelerationStructures (:778-810)
  void CreateAccelerationStructures() {
    uint64_t scratch, result, descs;
    BottomLevelASGenerator modelAS;
    modelAS.AddVertexBuffer(m_vertices.data(), 0, (uint32_t)(m_vertices.size() / 6), 24, m_indices.data(), 0,
                            (uint32_t)m_indices.size(), nullptr, 0, true);
    modelAS.ComputeASBufferSizes(m_ctx, false, &scratch, &result);
    rt_blas_t model = modelAS.Generate(m_ctx);
    BottomLevelASGenerator planeAS;
    planeAS.AddVertexBuffer(m_plane.data(), 0, 6, 24, nullptr, 0);
    planeAS.ComputeASBufferSizes(m_ctx, false, &scratch, &result);
    rt_blas_t plane = planeAS.Generate(m_ctx);

    TopLevelASGenerator tlas;
    uint32_t id = 0;
    if (m_opt.scene == "ref") {  // :784-791
      const float t[6][3] = {{0, 0, 0}, {-5, 0, 5}, {-5, 0, 5}, {-5, 0, -5}, {5, 0, -5}, {5, 0, 5}};
      for (auto& p : t) tlas.AddInstance(model, Matrix4::Translation(p[0], p[1], p[2]), id++, RT_HITGROUP_MODEL);
    } else if (m_opt.scene == "single") {
      tlas.AddInstance(model, Matrix4::Identity(), id++, RT_HITGROUP_MODEL);
    } else {
      const int side = m_opt.scene == "grid16" ? 16 : 8;
      const float half = (side - 1) / 2.0f;
      for (int i = 0; i < side; ++i)
        for (int j = 0; j < side; ++j)
          tlas.AddInstance(model, Matrix4::Translation(((float)i - half) * 3.0f, 0.0f, ((float)j - half) * 3.0f), id++,
                           RT_HITGROUP_MODEL);
    }
    tlas.AddInstance(plane, Matrix4::Identity(), id++, RT_HITGROUP_PLANE);
    tlas.ComputeASBufferSizes(m_ctx, true, &scratch, &result, &descs);
    tlas.Generate(m_ctx);
  }

  Options m_opt;
  rt_ctx_t m_ctx = nullptr;
  rt_comm_t m_comm = nullptr;
  void* m_output = nullptr;
  hipStream_t m_stream = nullptr;
  std::vector<float> m_vertices, m_plane;
  std::vector<uint32_t> m_indices;
};

Manipulator::Inputs parse_buttons(const std::string& spec) {
  Manipulator::Inputs in;
  size_t b = 0;
  while (b <= spec.size()) {
    size_t e = spec.find('+', b);
    if (e == std::string::npos) e = spec.size();
    const std::string k = spec.substr(b, e - b);
    if (k == "lmb") in.lmb = true;
    else if (k == "mmb") in.mmb = true;
    else if (k == "rmb") in.rmb = true;
    else if (k == "shift") in.shift = true;
    else if (k == "ctrl") in.ctrl = true;
    else if (k == "alt") in.alt = true;
    else {
      std::fprintf(stderr, "unknown button %s in --drag\n", k.c_str());
      std::exit(2);
    }
    b = e + 1;
  }
  return in;
}

Options parse(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--model") o.model = next();
    else if (a == "--scene") o.scene = next();
    else if (a == "--mode") o.mode = next();
    else if (a == "--width") o.width = std::atoi(next());
    else if (a == "--height") o.height = std::atoi(next());
    else if (a == "--lights") o.lights = std::atoi(next());
    else if (a == "--spp") o.spp = std::atoi(next());
    else if (a == "--frames") o.frames = std::atoi(next());
    else if (a == "--out") o.out = next();
    else if (a == "--raw") o.raw = next();
    else if (a == "--eye") for (int k = 0; k < 3; ++k) o.eye[k] = (float)std::atof(next());
    else if (a == "--center") for (int k = 0; k < 3; ++k) o.center[k] = (float)std::atof(next());
    else if (a == "--drag") {
      o.drag = next();
      o.drag_dx = std::atoi(next());
      o.drag_dy = std::atoi(next());
    } else if (a == "--out-pattern") o.out_pattern = next();
    else if (a == "--ranks") o.ranks = std::atoi(next());
    else if (a == "--rank") o.rank = std::atoi(next());
    else if (a == "--comm-id") o.comm_id = next();
    else {
      std::fprintf(stderr, "unknown option %s\n", a.c_str());
      std::exit(2);
    }
  }
  return o;
}

}  // namespace

int main(int argc, char** argv) {
  Options o = parse(argc, argv);
  if (o.ranks < 0 || (o.ranks > 0 && (o.rank < 0 || o.rank >= o.ranks)) || (o.ranks > 1 && o.comm_id.empty())) {
    std::fprintf(stderr, "--ranks N needs 0 <= --rank < N and, for N > 1, --comm-id FILE\n");
    return 2;
  }
  RayTracingApp app(o);
  try {
    app.OnInit();
    const bool drag = !o.drag.empty();
    const Manipulator::Inputs buttons = drag ? parse_buttons(o.drag) : Manipulator::Inputs();
    int mx = o.width / 2, my = o.height / 2;
    if (drag) app.OnButtonDown(mx, my);
    float best = 1e30f, sum = 0.0f;
    for (int f = 0; f < o.frames; ++f) {
      if (drag && f > 0) {
        mx += o.drag_dx;
        my += o.drag_dy;
        app.OnMouseMove(buttons, mx, my);
      }
      app.OnUpdate();
      float ms = app.OnRender();
      sum += ms;
      best = ms < best ? ms : best;
      if (!o.out_pattern.empty() && app.IsRoot()) {
        char name[1024];
        std::snprintf(name, sizeof(name), o.out_pattern.c_str(), f);
        app.Save(name, "");
      }
    }
    if (app.IsRoot()) app.Save(o.out, o.raw);
    std::printf("{\"frames\": %d, \"ms_mean\": %.4f, \"ms_best\": %.4f, \"width\": %d, \"height\": %d}\n", o.frames,
                sum / o.frames, best, o.width, o.height);
    app.OnDestroy();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rt_app: %s\n", e.what());
    app.OnDestroy();
    return 1;
  }
  return 0;
}
