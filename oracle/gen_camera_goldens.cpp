// gen_camera_goldens.cpp — TEST INFRASTRUCTURE: golden camera bases from the
// reference's vendored GLM 0.9.8.5 (/root/reference/includes/glm, third-party).
//
// source/camera.cpp itself cannot be compiled here: camera.hpp includes
// <GLFW/glfw3.h>, which this image lacks (and stand-in headers are not
// allowed).  This generator therefore restates Camera's constructor
// (camera.cpp:8-14) and Camera::lookAt (camera.cpp:22-51) as calls into the
// REAL GLM: glm::normalize, glm::cross, glm::rotate, glm::radians, mat4*mat4,
// mat4*vec4 — so the goldens pin librm's glm-free camera (rm_host.cpp) to the
// GLM arithmetic the reference uploads as uniforms (main.cpp:103-106).
//
// Build + run (container only; the output is committed as
// tests/golden/camera_goldens.json):   make goldens
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "glm/glm.hpp"
#include "glm/gtc/matrix_transform.hpp"

namespace {

uint32_t bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

void emit3(const char* name, const glm::vec3& v, bool comma) {
  std::printf("\"%s\": [%u, %u, %u]%s", name, bits(v.x), bits(v.y), bits(v.z), comma ? ", " : "");
}

struct Cam {  // the members lookAt touches (camera.hpp:14-27)
  float mouseSensitivity, keyboardSpeed, xpos, ypos, angleX, angleY;
  glm::vec3 cameraPos, forward, up, right;
};

// camera.cpp:22-51, expressed with GLM calls
void look_at(Cam& c, bool zN, bool zP, bool xN, bool xP, bool halfSpeed, float deltaTime) {
  c.angleX = c.xpos * c.mouseSensitivity;
  c.angleY = c.ypos * c.mouseSensitivity;
  glm::mat4 rx = glm::rotate(glm::mat4(1.0), glm::radians(c.angleY), glm::vec3(1.0, 0.0, 0.0));
  glm::mat4 ry = glm::rotate(glm::mat4(1.0), glm::radians(c.angleX), glm::vec3(0.0, 1.0, 0.0));
  glm::mat4 r = ry * rx;
  c.forward = glm::normalize(glm::vec3(r * glm::vec4(0.0, 0.0, -1.0, 0.0)));
  c.up = glm::normalize(glm::vec3(r * glm::vec4(0.0, 1.0, 0.0, 0.0)));
  c.right = glm::normalize(glm::cross(c.forward, c.up));
  c.keyboardSpeed = halfSpeed ? 5.0f : 10.0f;
  if (zN) c.cameraPos += (c.keyboardSpeed * c.forward) * deltaTime;
  if (zP) c.cameraPos += (c.keyboardSpeed * (-c.forward)) * deltaTime;
  if (xN) c.cameraPos += (c.keyboardSpeed * (-c.right)) * deltaTime;
  if (xP) c.cameraPos += (c.keyboardSpeed * c.right) * deltaTime;
}

}  // namespace

int main() {
  struct Case {
    float xpos, ypos, px, py, pz;
    int zN, zP, xN, xP, half;
    float dt;
  };
  std::vector<Case> cases;
  // the synthetic sweep S(120) of SURVEY 8(d): yaw -20..20 deg, pitch -5 deg
  for (int f = 0; f < 120; ++f) {
    double yaw = -20.0 + 40.0 * f / 119.0;
    cases.push_back({(float)(yaw / 0.025), (float)(-5.0 / 0.025), 0.f, 0.f, 15.f, 0, 0, 0, 0, 0, 0.f});
  }
  // start-up frame D and a spread of mouse positions / motions
  cases.push_back({0.f, 0.f, 0.f, 0.f, 0.f, 0, 0, 0, 0, 0, 0.f});
  const float xs[] = {-7200.f, -3601.5f, -1080.f, -540.25f, -1.f, 0.5f, 333.f, 1080.f, 2400.f, 9999.f};
  const float ys[] = {-3000.f, -1234.5f, -540.f, -3.f, 0.f, 7.25f, 540.f, 1799.f, 3500.f};
  int k = 0;
  for (float x : xs)
    for (float y : ys) {
      int m = k++ % 7;
      cases.push_back({x, y, 1.5f * (k % 5) - 3.f, 0.25f * (k % 3), 20.f - k * 0.1f, m == 1, m == 2,
                       m == 3, m == 4, (m == 5 || m == 6), 0.016f + 0.001f * (k % 9)});
      if (m == 6) {  // two keys at once
        cases.back().zN = 1;
        cases.back().xP = 1;
      }
    }
  std::printf("{\"generator\": \"oracle/gen_camera_goldens.cpp against GLM 0.9.8.5 (reference includes/glm)\",\n");
  // constructor basis, camera.cpp:8-14 (main.cpp:40 arguments)
  {
    glm::vec3 pos(0, 0, 0), look(0, 0, -1), upp(0, 1, 0);
    glm::vec3 fwd = glm::normalize(look - pos);
    glm::vec3 right = glm::normalize(glm::cross(upp, fwd));
    std::printf(" \"ctor\": {");
    emit3("forward", fwd, true);
    emit3("right", right, false);
    std::printf("},\n");
  }
  std::printf(" \"mouseSensitivity\": %u,\n \"cases\": [\n", bits(0.025f));
  for (size_t i = 0; i < cases.size(); ++i) {
    const Case& cs = cases[i];
    Cam c;
    c.mouseSensitivity = 0.025f;
    c.keyboardSpeed = 10.0f;
    c.xpos = cs.xpos;
    c.ypos = cs.ypos;
    c.cameraPos = glm::vec3(cs.px, cs.py, cs.pz);
    look_at(c, cs.zN, cs.zP, cs.xN, cs.xP, cs.half, cs.dt);
    std::printf("  {\"xpos\": %u, \"ypos\": %u, \"pos\": [%u, %u, %u], \"keys\": [%d, %d, %d, %d, %d], "
                "\"dt\": %u, ",
                bits(cs.xpos), bits(cs.ypos), bits(cs.px), bits(cs.py), bits(cs.pz), cs.zN, cs.zP,
                cs.xN, cs.xP, cs.half, bits(cs.dt));
    emit3("forward", c.forward, true);
    emit3("up", c.up, true);
    emit3("right", c.right, true);
    emit3("cameraPos", c.cameraPos, false);
    std::printf("}%s\n", i + 1 < cases.size() ? "," : "");
  }
  std::printf(" ]\n}\n");
  return 0;
}
