// rm/input.hpp — C++ mirror of the reference's GLFW input handling (main.cpp:20-39,
// 93-95, 155-234) and MouseInput (source/MousePosition.{hpp,cpp}) for any
// windowing front-end: the globals become one object, the callbacks become
// methods with the reference's names and GLFW's key/action codes.  The rules
// live once in librm (rm_input_*, rm_host.cpp), pinned bit-for-bit by
// tests/golden/input_goldens.json.
//
// A GLFW front-end wires it exactly where the reference does:
//   glfwSetKeyCallback(w, [](GLFWwindow*, int k, int sc, int a, int m) { in.key_callback(k, sc, a, m); });
//   glfwSetCursorPosCallback(w, [](GLFWwindow*, double x, double y) { in.mouse_callback(x, y); });
//   per frame: in.beginFrame(glfwGetTime()); in.processInput(held);  then in.upload(marching)
#pragma once

#include <rm_api.h>
#include <rm/camera.hpp>

namespace rm {

class Input {
 public:
  Camera& camera;  // the camera the callbacks move (the reference's global, main.cpp:40)

  explicit Input(Camera& cam, int screenWidth = 1080, int screenHeight = 1080) : camera(cam) {
    rm_input_init(&s_, screenWidth, screenHeight);
  }

  // main.cpp:93-95
  void beginFrame(double now) { rm_input_begin_frame(&s_, now); }

  // main.cpp:155-195; held = OR of RM_HELD_* (glfwGetKey(...) == GLFW_PRESS)
  void processInput(unsigned held) { withCamera([&](rm_camera_state* c) { rm_input_process(&s_, held, c); }); }

  // main.cpp:197-217 (scancode and mods are unused, as in the reference)
  void key_callback(int key, int /*scancode*/, int action, int /*mods*/) { rm_input_key(&s_, key, action); }

  // main.cpp:219-234
  void mouse_callback(double xpos, double ypos) {
    withCamera([&](rm_camera_state* c) { rm_input_mouse(&s_, xpos, ypos, c); });
  }

  // The uploads of main.cpp:101-120 that input drives (camera, AA, bounceVar,
  // mouse, iMouse, iTime) onto a uniform block.
  void toUniforms(rm_uniforms* u) const {
    rm_camera_state c = camera.state();
    rm_input_to_uniforms(&s_, &c, u);
  }

  bool shouldClose() const { return s_.shouldClose != 0; }
  bool AA() const { return s_.AA != 0; }
  int bounce() const { return s_.bounce; }
  bool showQuad() const { return s_.showQuad != 0; }
  const rm_input_state& state() const { return s_; }

 private:
  template <class F>
  void withCamera(F f) {
    rm_camera_state c = camera.state();
    f(&c);
    camera.assign(c);
  }
  rm_input_state s_;
};

}  // namespace rm
