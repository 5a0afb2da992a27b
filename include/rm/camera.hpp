// rm/camera.hpp — C++ mirror of the reference's Camera (source/camera.hpp:12-35,
// source/camera.cpp:8-51) without GLM/GLFW.  Same members, same methods, same
// arithmetic (implemented once in librm, rm_host.cpp, pinned bit-for-bit to
// GLM 0.9.8.5 by tests/golden/camera_goldens.json).
#pragma once

#include <rm_api.h>

namespace rm {

struct vec3 {
  float x = 0.0f, y = 0.0f, z = 0.0f;
  vec3() = default;
  vec3(float a, float b, float c) : x(a), y(b), z(c) {}
};

class Camera {
 public:
  int width;
  int height;
  float angleY;
  float angleX;
  float mouseSensitivity;
  float keyboardSpeed;
  float xpos;
  float ypos;

  vec3 cameraPos;
  vec3 forward;
  vec3 up;
  vec3 right;

  // camera.cpp:8-10
  Camera() noexcept
      : width(1024), height(1024), angleY(0.0f), angleX(0.0f), mouseSensitivity(1.0f),
        keyboardSpeed(10.0f), xpos(0.0f), ypos(0.0f), cameraPos(0, 0, 0), forward(0, 0, -1),
        up(0, 1, 0), right(1, 0, 0) {}

  // camera.cpp:11-14 (the `up` parameter shadows the member, which stays 0)
  Camera(int w, int h, float sens, float speed, vec3 pos, vec3 lookAt, vec3 upv) noexcept {
    rm_camera_state s;
    const float p[3] = {pos.x, pos.y, pos.z}, l[3] = {lookAt.x, lookAt.y, lookAt.z},
                u[3] = {upv.x, upv.y, upv.z};
    rm_camera_init(&s, w, h, sens, speed, p, l, u);
    assign(s);
  }

  // camera.cpp:16-20
  void setMouse(float x, float y) {
    xpos = x;
    ypos = y;
  }

  // camera.cpp:22-51
  void lookAt(bool zN, bool zP, bool xN, bool xP, bool halfSpeed, float deltaTime) {
    rm_camera_state s = state();
    rm_camera_look_at(&s, zN, zP, xN, xP, halfSpeed, deltaTime);
    assign(s);
  }

  // main.cpp:103-106 — the four setVec4("camera.*") uploads (w = 0)
  rm_camera toUniform() const {
    rm_camera c;
    rm_camera_state s = state();
    rm_camera_to_uniform(&s, &c);
    return c;
  }

  // The C-ABI view of this camera (rm_camera_state) and back, for rm_input_*.
  rm_camera_state state() const {
    rm_camera_state s;
    s.width = width;
    s.height = height;
    s.angleY = angleY;
    s.angleX = angleX;
    s.mouseSensitivity = mouseSensitivity;
    s.keyboardSpeed = keyboardSpeed;
    s.xpos = xpos;
    s.ypos = ypos;
    put(s.cameraPos, cameraPos);
    put(s.forward, forward);
    put(s.up, up);
    put(s.right, right);
    return s;
  }
  void assign(const rm_camera_state& s) {
    width = s.width;
    height = s.height;
    angleY = s.angleY;
    angleX = s.angleX;
    mouseSensitivity = s.mouseSensitivity;
    keyboardSpeed = s.keyboardSpeed;
    xpos = s.xpos;
    ypos = s.ypos;
    cameraPos = get(s.cameraPos);
    forward = get(s.forward);
    up = get(s.up);
    right = get(s.right);
  }
 private:
  static void put(float* d, const vec3& v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
  }
  static vec3 get(const float* d) { return vec3(d[0], d[1], d[2]); }
};

}  // namespace rm
