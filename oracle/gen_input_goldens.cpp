// gen_input_goldens.cpp — TEST INFRASTRUCTURE: golden traces of the reference's
// interactive input path computed with the reference's
// vendored GLM 0.9.8.5 (/root/reference/includes/glm, third-party).
//
// main.cpp and source/MousePosition.cpp cannot be compiled here (they include
// <GLFW/glfw3.h>, absent from this image; stand-in headers are not allowed).
// This generator restates, with the reference's declared types (float globals,
// double callback arguments, a float halfSpeed, the unqualified C-library
// cos/sin of MousePosition.cpp), and with the REAL GLM for every vector op:
//   * the input globals                   main.cpp:23-39
//   * the frame clock                     main.cpp:93-95
//   * processInput (glfwGetKey -> a held-key mask)   main.cpp:155-195
//   * key_callback                        main.cpp:197-217
//   * mouse_callback                      main.cpp:219-234
//   * MouseInput::ProcessMouseOffset / EulerAngles   MousePosition.cpp:10-33
//   * Camera::setMouse / lookAt           camera.cpp:16-51
// and replays a deterministic pseudo-random event script, printing the script
// and the full state after every event as float bit patterns.  librm's
// rm_input_* (rm_host.cpp) must reproduce the trace bit for bit
// (tests/test_input.py).
//
//   make goldens   (container only; output committed as tests/golden/input_goldens.json)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "glm/glm.hpp"
#include "glm/gtc/matrix_transform.hpp"

// ---- the reference's globals (main.cpp:16-39, MousePosition.hpp:8) ----------
const unsigned int SCREEN_WIDTH = 1080;
const unsigned int SCREEN_HEIGHT = 1080;
bool zaxisPos = false;
bool zaxisNeg = false;
bool xaxisPos = false;
bool xaxisNeg = false;
bool AA = true;
bool showQuad = false;
float halfSpeed = false;
int bounce = 0;
float deltaTime = 0.0f;
float lastFrame = 0.0f;
float lastX = SCREEN_WIDTH / 2.0;
float lastY = SCREEN_HEIGHT / 2.0;
bool firstMouse = true;
bool shouldClose = false;
float MouseSensitivity = 0.001;

struct MouseInput {  // MousePosition.cpp:4-33
  float pitch = 0.0, yaw = 0.0;
  void ProcessMouseOffset(float xoffset, float yoffset) {
    xoffset *= MouseSensitivity;
    yoffset *= MouseSensitivity;
    yaw += xoffset;
    pitch += yoffset;
  }
  glm::vec3 EulerAngles() {
    glm::vec3 front;
    front.x = cos(glm::radians(yaw) * cos(glm::radians(pitch)));
    front.y = sin(glm::radians(pitch));
    front.z = sin(glm::radians(yaw) * cos(glm::radians(pitch)));
    return glm::vec3(glm::normalize(front));
  }
} mouse;

struct Camera {  // camera.cpp:11-51, main.cpp:40 arguments
  float mouseSensitivity = 0.025f, keyboardSpeed = 10.0f, xpos = 0, ypos = 0, angleX = 0, angleY = 0;
  glm::vec3 cameraPos{0, 0, 0}, forward, up{0, 0, 0}, right;
  Camera() {
    glm::vec3 pos(0, 0, 0), look(0, 0, -1), upp(0, 1, 0);
    forward = glm::normalize(look - pos);
    right = glm::normalize(glm::cross(upp, forward));
  }
  void setMouse(float x, float y) {
    xpos = x;
    ypos = y;
  }
  void lookAt(bool zN, bool zP, bool xN, bool xP, bool half, float dt) {
    angleX = xpos * mouseSensitivity;
    angleY = ypos * mouseSensitivity;
    glm::mat4 rx = glm::rotate(glm::mat4(1.0), glm::radians(angleY), glm::vec3(1.0, 0.0, 0.0));
    glm::mat4 ry = glm::rotate(glm::mat4(1.0), glm::radians(angleX), glm::vec3(0.0, 1.0, 0.0));
    glm::mat4 r = ry * rx;
    forward = glm::normalize(glm::vec3(r * glm::vec4(0.0, 0.0, -1.0, 0.0)));
    up = glm::normalize(glm::vec3(r * glm::vec4(0.0, 1.0, 0.0, 0.0)));
    right = glm::normalize(glm::cross(forward, up));
    keyboardSpeed = half ? 5.0f : 10.0f;
    if (zN) cameraPos += (keyboardSpeed * forward) * dt;
    if (zP) cameraPos += (keyboardSpeed * (-forward)) * dt;
    if (xN) cameraPos += (keyboardSpeed * (-right)) * dt;
    if (xP) cameraPos += (keyboardSpeed * right) * dt;
  }
} camera;

// glfw3.h codes
enum { KEY_A = 65, KEY_D = 68, KEY_L = 76, KEY_S = 83, KEY_W = 87, KEY_ESCAPE = 256,
       KEY_DOWN = 264, KEY_UP = 265, KEY_F1 = 290, RELEASE = 0, PRESS = 1, REPEAT = 2 };
enum { HELD_W = 1, HELD_A = 2, HELD_S = 4, HELD_D = 8, HELD_ESC = 16 };
unsigned held_now = 0;
bool getKey(int k) {  // glfwGetKey(window, k) == GLFW_PRESS
  unsigned m = k == KEY_W ? HELD_W : k == KEY_A ? HELD_A : k == KEY_S ? HELD_S
             : k == KEY_D ? HELD_D : k == KEY_ESCAPE ? HELD_ESC : 0;
  return (held_now & m) != 0;
}

void processInput() {  // main.cpp:155-195
  if (getKey(KEY_ESCAPE)) shouldClose = true;
  zaxisNeg = getKey(KEY_W);
  zaxisPos = getKey(KEY_S);
  xaxisPos = getKey(KEY_D);
  xaxisNeg = getKey(KEY_A);
  if ((getKey(KEY_W) && getKey(KEY_A)) || (getKey(KEY_W) && getKey(KEY_D)) ||
      (getKey(KEY_A) && getKey(KEY_S)) || (getKey(KEY_S) && getKey(KEY_D)))
    halfSpeed = true;
  else
    halfSpeed = false;
  camera.lookAt(zaxisNeg, zaxisPos, xaxisNeg, xaxisPos, halfSpeed, deltaTime);
}

void key_callback(int key, int action) {  // main.cpp:197-217
  if (key == KEY_UP && action == PRESS)
    if (bounce < 5) bounce += 1;
  if (key == KEY_DOWN && action == PRESS)
    if (bounce > 0) bounce -= 1;
  if (key == KEY_F1 && action == PRESS) AA = !AA;
  if (key == KEY_L && action == PRESS) showQuad = !showQuad;
}

void mouse_callback(double xpos, double ypos) {  // main.cpp:219-234
  if (firstMouse) {
    lastX = xpos;
    lastY = ypos;
    firstMouse = false;
  }
  float xoffset = lastX - xpos;
  float yoffset = lastY - ypos;
  lastX = xpos;
  lastY = ypos;
  mouse.ProcessMouseOffset(xoffset, yoffset);
  camera.setMouse(-xpos, -ypos);
}

uint32_t bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}
uint64_t bits64(double d) {
  uint64_t u;
  std::memcpy(&u, &d, 8);
  return u;
}

uint64_t rng = 0x9E3779B97F4A7C15ull;
uint32_t next() {
  rng = rng * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(rng >> 33);
}
double unit() { return next() / 2147483648.0; }

void emit_state() {
  glm::vec3 e = mouse.EulerAngles();
  std::printf("{\"axes\": [%d, %d, %d, %d], \"halfSpeed\": %u, \"AA\": %d, \"showQuad\": %d, "
              "\"bounce\": %d, \"close\": %d, \"deltaTime\": %u, \"lastFrame\": %u, "
              "\"lastX\": %u, \"lastY\": %u, \"firstMouse\": %d, \"yaw\": %u, \"pitch\": %u, "
              "\"euler\": [%u, %u, %u], \"cam_mouse\": [%u, %u], \"pos\": [%u, %u, %u], "
              "\"dir\": [%u, %u, %u], \"yAxis\": [%u, %u, %u], \"xAxis\": [%u, %u, %u]}",
              zaxisPos, zaxisNeg, xaxisPos, xaxisNeg, bits(halfSpeed), AA, showQuad, bounce,
              shouldClose, bits(deltaTime), bits(lastFrame), bits(lastX), bits(lastY), firstMouse,
              bits(mouse.yaw), bits(mouse.pitch), bits(e.x), bits(e.y), bits(e.z),
              bits(camera.xpos), bits(camera.ypos), bits(camera.cameraPos.x),
              bits(camera.cameraPos.y), bits(camera.cameraPos.z), bits(camera.forward.x),
              bits(camera.forward.y), bits(camera.forward.z), bits(camera.up.x), bits(camera.up.y),
              bits(camera.up.z), bits(camera.right.x), bits(camera.right.y), bits(camera.right.z));
}

int main() {
  std::printf("{\"generator\": \"oracle/gen_input_goldens.cpp against GLM 0.9.8.5 (reference "
              "includes/glm)\",\n \"screen\": [%u, %u],\n \"initial\": ",
              SCREEN_WIDTH, SCREEN_HEIGHT);
  emit_state();
  std::printf(",\n \"events\": [\n");
  const int keys[] = {KEY_UP, KEY_UP, KEY_UP, KEY_DOWN, KEY_DOWN, KEY_F1, KEY_L, KEY_W, 32, KEY_ESCAPE};
  double now = 0.0, mx = 700.25, my = 300.5;
  const int N = 600;
  for (int i = 0; i < N; ++i) {
    const uint32_t kind = next() % 8;
    std::printf("  {");
    if (kind < 3) {  // one frame: clock, then processInput with held keys
      now += 1.0 / 60.0 + 0.004 * unit();
      unsigned held = next() % 16;
      if (next() % 97 == 0) held |= HELD_ESC;
      held_now = held;
      float currentFrame = now;  // main.cpp:93-95
      deltaTime = currentFrame - lastFrame;
      lastFrame = currentFrame;
      processInput();
      std::printf("\"ev\": \"frame\", \"now\": %llu, \"held\": %u, ", (unsigned long long)bits64(now), held);
    } else if (kind < 6) {  // key event (repeats and releases included)
      int key = keys[next() % 10];
      int action = (int)(next() % 3);
      key_callback(key, action);
      std::printf("\"ev\": \"key\", \"key\": %d, \"action\": %d, ", key, action);
    } else {  // cursor motion; occasionally a big jump
      double s = next() % 11 == 0 ? 4000.0 : 60.0;
      mx += s * (unit() - 0.5);
      my += s * (unit() - 0.5);
      if (next() % 5 == 0) mx = std::floor(mx);
      mouse_callback(mx, my);
      std::printf("\"ev\": \"mouse\", \"x\": %llu, \"y\": %llu, ", (unsigned long long)bits64(mx),
                  (unsigned long long)bits64(my));
    }
    std::printf("\"state\": ");
    emit_state();
    std::printf("}%s\n", i + 1 < N ? "," : "");
  }
  std::printf(" ]\n}\n");
  return 0;
}
