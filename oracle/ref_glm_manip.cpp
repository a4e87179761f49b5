// Golden-trajectory generator for the camera manipulator, compiled ONLY in the dev
// container against the reference's vendored glm 0.9.8.5 (/root/reference/glm, header-only).
// The reference's src/manipulator.cpp cannot be compiled here (it includes stdafx.h -> windows.h,
// d3d12.h), so the manipulator's state machine is restated below on top of the REAL glm
// primitives it calls (lookAt, rotate, normalize, cross, length, mat4*vec4, mat4*mat4): the glm
// arithmetic — where bit-level differences would come from — is the reference's own, the control
// flow follows the cited lines. Output: JSON on stdout (floats as IEEE-754 bit patterns), written
// to tests/golden/manipulator.json by tests/golden/make_golden.py. Never shipped, never run on
// the GPU box. Test infrastructure only.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#include <glm/gtc/type_ptr.hpp>
#include <glm/gtx/transform.hpp>

namespace {

enum { kExamine = 0, kFly = 1, kWalk = 2, kTrackball = 3 };           // manipulator.h:37
enum { kNone = 0, kOrbit = 1, kDolly = 2, kPan = 3, kLookAround = 4 };  // manipulator.h:38
enum { kLmb = 1, kMmb = 2, kRmb = 4, kShift = 8, kCtrl = 16, kAlt = 32 };  // Inputs, manipulator.h:39-40

struct Cam {  // defaults: manipulator.h:124-144
  glm::vec3 eye{10, 10, 10}, poi{0, 0, 0}, up{0, 1, 0};
  float roll = 0;
  glm::mat4 view{1};
  int w = 1, h = 1;
  float speed = 30;
  glm::vec2 mouse{0, 0};
  float tb = 0.8f;
  int mode = kExamine;
};

bool near_zero(float a) { return std::fabs(a) < std::numeric_limits<float>::epsilon(); }  // .h:174-177
float sgn(float s) { return s < 0.f ? -1.f : 1.f; }                                        // .h:183-186

void refresh(Cam& c) {  // update, manipulator.cpp:305-314
  c.view = glm::lookAt(c.eye, c.poi, c.up);
  if (!near_zero(c.roll)) c.view = c.view * glm::rotate(c.roll, glm::vec3(0, 0, 1));
}

void do_pan(Cam& c, float dx, float dy) {  // :319-339
  if (c.mode == kFly) {
    dx *= -1;
    dy *= -1;
  }
  glm::vec3 back = c.eye - c.poi;
  const float reach = static_cast<float>(glm::length(back)) / 0.785f;
  back = glm::normalize(back);
  glm::vec3 side = glm::normalize(glm::cross(c.up, back));
  glm::vec3 vert = glm::normalize(glm::cross(back, side));
  side *= -dx * reach;
  vert *= dy * reach;
  c.eye += side + vert;
  c.poi += side + vert;
}

void do_orbit(Cam& c, float dx, float dy, bool about_eye) {  // :345-398
  if (near_zero(dx) && near_zero(dy)) return;
  dx *= float(glm::two_pi<float>());
  dy *= float(glm::two_pi<float>());
  const glm::vec3 pivot = about_eye ? c.eye : c.poi;
  const glm::vec3 moving = about_eye ? c.poi : c.eye;
  glm::vec3 arm = moving - pivot;
  const float radius = glm::length(arm);
  arm = glm::normalize(arm);
  const glm::vec3 zaxis = glm::normalize(arm);
  glm::vec4 t = glm::rotate(dx, c.up) * glm::vec4(arm.x, arm.y, arm.z, 0);
  arm = glm::vec3(t.x, t.y, t.z);
  const glm::vec3 xaxis = glm::normalize(glm::cross(c.up, zaxis));
  t = glm::rotate(dy, xaxis) * glm::vec4(arm.x, arm.y, arm.z, 0);
  const glm::vec3 tilted(t.x, t.y, t.z);
  if (sgn(tilted.x) == sgn(arm.x)) arm = tilted;
  arm *= radius;
  (about_eye ? c.poi : c.eye) = arm + pivot;
}

void do_dolly(Cam& c, float dx, float dy) {  // :403-445
  glm::vec3 step = c.poi - c.eye;
  float dist = static_cast<float>(glm::length(step));
  if (near_zero(dist)) return;
  const float dd = c.mode != kExamine ? -dy : (std::fabs(dx) > std::fabs(dy) ? dx : -dy);
  float k = c.speed * dd / dist;
  dist /= 10;
  dist = dist < 0.001f ? 0.001f : dist;
  k *= dist;
  if (k >= 1.0f) return;
  step *= k;
  if (c.mode == kWalk) {
    if (c.up.y > c.up.z)
      step.y = 0;
    else
      step.z = 0;
  }
  c.eye += step;
  if (c.mode != kExamine) c.poi += step;
}

double sphere_z(const Cam& c, const glm::vec2& p) {  // projectOntoTBSphere, :283-300
  const double d = glm::length(p);
  if (d < c.tb * 0.70710678118654752440) return std::sqrt(c.tb * c.tb - d * d);
  const double t = c.tb / 1.41421356237309504880;
  return t * t / d;
}

void do_trackball(Cam& c, int x, int y) {  // :242-277
  const glm::vec2 a(2 * (c.mouse[0] - c.w / 2) / double(c.w), 2 * (c.h / 2 - c.mouse[1]) / double(c.h));
  const glm::vec2 b(2 * (x - c.w / 2) / double(c.w), 2 * (c.h / 2 - y) / double(c.h));
  const glm::vec3 pa(a[0], a[1], sphere_z(c, a));
  const glm::vec3 pb(b[0], b[1], sphere_z(c, b));
  const glm::vec3 axis = glm::normalize(glm::cross(pa, pb));
  double s = glm::length(pa - pb) / (2.f * c.tb);
  s = s > 1.0 ? 1.0 : (s < -1.0 ? -1.0 : s);
  const float angle = (float)(2.0 * std::asin(s));
  const glm::vec4 wa = c.view * glm::vec4(axis, 0);
  const glm::mat4 R = glm::rotate(angle, glm::vec3(wa.x, wa.y, wa.z));
  const glm::vec3 off = c.eye - c.poi;
  const glm::vec4 off2 = R * glm::vec4(off.x, off.y, off.z, 1);
  c.eye = c.poi + glm::vec3(off2.x, off2.y, off2.z);
  const glm::vec4 up2 = R * glm::vec4(c.up.x, c.up.y, c.up.z, 0);
  c.up = glm::vec3(up2.x, up2.y, up2.z);
}

void do_motion(Cam& c, int x, int y, int action) {  // :135-166
  const float dx = float(x - c.mouse[0]) / float(c.w);
  const float dy = float(y - c.mouse[1]) / float(c.h);
  if (action == kOrbit) do_orbit(c, dx, dy, c.mode == kTrackball);
  else if (action == kDolly) do_dolly(c, dx, dy);
  else if (action == kPan) do_pan(c, dx, dy);
  else if (action == kLookAround) {
    if (c.mode == kTrackball) do_trackball(c, x, y);
    else do_orbit(c, dx, -dy, true);
  }
  refresh(c);
  c.mouse[0] = static_cast<float>(x);
  c.mouse[1] = static_cast<float>(y);
}

int do_mouse_move(Cam& c, int x, int y, unsigned in) {  // :175-198
  int act = kNone;
  if (in & kLmb) {
    if (((in & kCtrl) && (in & kShift)) || (in & kAlt)) act = c.mode == kExamine ? kLookAround : kOrbit;
    else if (in & kShift) act = kDolly;
    else if (in & kCtrl) act = kPan;
    else act = c.mode == kExamine ? kOrbit : kLookAround;
  } else if (in & kMmb) {
    act = kPan;
  } else if (in & kRmb) {
    act = kDolly;
  }
  if (act != kNone) do_motion(c, x, y, act);
  return act;
}

void do_wheel(Cam& c, int value) {  // :203-214
  const float v = static_cast<float>(value);
  const float dx = (v * std::fabs(v)) / static_cast<float>(c.w);
  do_dolly(c, dx * c.speed, dx * c.speed);
  refresh(c);
}

uint32_t bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

void emit_vec(const char* key, const float* p, int n) {
  std::printf("\"%s\": [", key);
  for (int i = 0; i < n; ++i) std::printf("%u%s", bits(p[i]), i < n - 1 ? ", " : "");
  std::printf("]");
}

// Event: op + up to 9 numeric arguments (floats for lookat/roll/speed, ints otherwise).
struct Ev {
  const char* op;
  float a[9];
};

void run(const char* name, const std::vector<Ev>& evs) {
  Cam c;
  refresh(c);  // Manipulator::Manipulator, :17-20
  std::printf("  {\"name\": \"%s\", \"events\": [\n", name);
  for (size_t i = 0; i < evs.size(); ++i) {
    const Ev& e = evs[i];
    const std::string op = e.op;
    int ret = -1;
    if (op == "lookat") {  // :26-32
      c.eye = glm::vec3(e.a[0], e.a[1], e.a[2]);
      c.poi = glm::vec3(e.a[3], e.a[4], e.a[5]);
      c.up = glm::vec3(e.a[6], e.a[7], e.a[8]);
      refresh(c);
    } else if (op == "window") {
      c.w = (int)e.a[0];
      c.h = (int)e.a[1];
    } else if (op == "mouse") {
      c.mouse = glm::vec2((float)(int)e.a[0], (float)(int)e.a[1]);
    } else if (op == "mode") {
      c.mode = (int)e.a[0];
    } else if (op == "roll") {
      c.roll = e.a[0];
      refresh(c);
    } else if (op == "speed") {
      c.speed = e.a[0];
    } else if (op == "move") {
      ret = do_mouse_move(c, (int)e.a[0], (int)e.a[1], (unsigned)e.a[2]);
    } else if (op == "motion") {
      do_motion(c, (int)e.a[0], (int)e.a[1], (int)e.a[2]);
    } else if (op == "wheel") {
      do_wheel(c, (int)e.a[0]);
    }
    std::printf("   {\"op\": \"%s\", \"args\": [", e.op);
    const int nargs = op == "lookat" ? 9 : (op == "window" ? 2 : (op == "mouse" ? 2 : (op == "move" || op == "motion") ? 3 : 1));
    for (int k = 0; k < nargs; ++k) std::printf("%.9g%s", e.a[k], k < nargs - 1 ? ", " : "");
    std::printf("], \"ret\": %d, ", ret);
    emit_vec("eye", &c.eye[0], 3);
    std::printf(", ");
    emit_vec("center", &c.poi[0], 3);
    std::printf(", ");
    emit_vec("up", &c.up[0], 3);
    std::printf(", ");
    emit_vec("matrix", glm::value_ptr(c.view), 16);
    std::printf("}%s\n", i + 1 < evs.size() ? "," : "");
  }
  std::printf("  ]}");
}

}  // namespace

int main() {
  const float L = 1.5f;
  std::vector<std::pair<const char*, std::vector<Ev>>> seqs;
  // Examine mode (default): every mouse binding of mouseMove, plus wheel and roll.
  seqs.push_back({"examine", {
      {"window", {1280, 720}}, {"lookat", {L, L, L, 0, 0, 0, 0, 1, 0}}, {"mouse", {640, 360}},
      {"move", {700, 380, kLmb}}, {"move", {760, 350, kLmb}}, {"move", {760, 350, kLmb}},
      {"move", {770, 420, kLmb | kShift}}, {"move", {700, 400, kLmb | kCtrl}},
      {"move", {650, 380, kMmb}}, {"move", {640, 300, kRmb}}, {"move", {600, 320, kLmb | kAlt}},
      {"move", {610, 330, kLmb | kCtrl | kShift}}, {"move", {620, 340, 0}},
      {"wheel", {1}}, {"wheel", {-2}}, {"wheel", {120}}, {"wheel", {-120}}, {"roll", {0.3f}},
      {"move", {680, 300, kLmb}}, {"roll", {0}}, {"move", {500, 500, kLmb}},
      {"motion", {520, 480, kPan}}, {"motion", {530, 470, kDolly}}, {"motion", {560, 490, kLookAround}}}});
  // Trackball mode: LookAround -> trackball (inside the sphere and on the hyperbolic sheet),
  // Orbit -> orbit about the eye.
  seqs.push_back({"trackball", {
      {"window", {1920, 1080}}, {"lookat", {7, 5, 9, 0.2f, 1.3f, 0, 0, 1, 0}}, {"mode", {kTrackball}},
      {"mouse", {960, 540}}, {"move", {1000, 560, kLmb}}, {"move", {1100, 500, kLmb}},
      {"move", {1800, 100, kLmb}}, {"move", {1900, 60, kLmb}}, {"move", {200, 1000, kLmb | kAlt}},
      {"roll", {-0.7f}}, {"move", {400, 900, kLmb}}, {"move", {410, 880, kLmb | kShift}},
      {"move", {420, 870, kMmb}}}});
  // Fly and walk: pan is inverted, dolly moves the interest point, walk keeps the height.
  seqs.push_back({"fly_walk", {
      {"window", {800, 600}}, {"lookat", {-3.25f, 0.5f, 7.125f, 1.0f, -2.0f, 0.5f, 0.1f, 0.9f, -0.2f}},
      {"mode", {kFly}}, {"mouse", {400, 300}}, {"move", {430, 310, kLmb | kCtrl}},
      {"move", {430, 250, kLmb | kShift}}, {"move", {460, 240, kLmb}}, {"wheel", {-1}},
      {"mode", {kWalk}}, {"move", {460, 200, kRmb}}, {"move", {470, 230, kLmb | kShift}},
      {"lookat", {0, 0, 5, 0, 0, 0, 0, 0, 1}}, {"move", {480, 180, kRmb}},
      {"speed", {5}}, {"wheel", {2}}}});
  // Guards: dolly that would cross the interest point, dolly at the interest point, no-op orbit.
  seqs.push_back({"guards", {
      {"window", {100, 100}}, {"lookat", {0, 0, 1, 0, 0, 0, 0, 1, 0}}, {"mouse", {50, 50}},
      {"move", {50, 0, kRmb}}, {"move", {50, 50, kLmb}}, {"wheel", {1000}},
      {"lookat", {2, 2, 2, 2, 2, 2, 0, 1, 0}}, {"move", {60, 60, kRmb}},
      {"lookat", {10, 10, 10, 0, 0, 0, 0, 1, 0}}, {"move", {90, 60, kLmb}}, {"move", {95, 95, kLmb}}}});
  std::printf("{\n \"source\": \"manipulator state machine over glm 0.9.8.5 (reference vendored glm), "
              "oracle/ref_glm_manip.cpp\",\n \"sequences\": [\n");
  for (size_t s = 0; s < seqs.size(); ++s) {
    run(seqs[s].first, seqs[s].second);
    std::printf("%s\n", s + 1 < seqs.size() ? "," : "");
  }
  std::printf(" ]\n}\n");
  return 0;
}
