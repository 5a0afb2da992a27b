// rm_host.cpp — host-side pieces of librm that need no GPU:
//   * Camera (source/camera.{hpp,cpp}) restated without GLM/GLFW, reproducing
//     GLM 0.9.8.5's operation order so the basis is bit-identical to what the
//     reference uploads (pinned by tests/golden/camera_goldens.json, which was
//     generated against the reference's vendored GLM by
//     oracle/gen_camera_goldens.cpp);
//   * the uniform block defaults and by-name lookup (shader.hpp:19-69 +
//     main.cpp:99-120);
//   * synthetic sweep frames and the row-shard map.
// Compiled with -ffp-contract=off: every float op is one IEEE binary32 op.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <initializer_list>
#include <limits>
#include <vector>

#include "rm_internal.hpp"
#include "rm_shard.hpp"

namespace {

// ---- GLM 0.9.8.5 restated (column-major mat4: m[col][row]) -------------------
struct vec3 {
  float x, y, z;
};
struct vec4 {
  float v[4];
};
struct mat4 {
  vec4 c[4];
};

// glm::radians  detail/func_trigonometric.inl:12-17
inline float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
// glm::dot (vec3)  detail/func_geometric.inl:54-61  -> (x + y) + z
inline float dot(vec3 a, vec3 b) {
  float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
  return tx + ty + tz;
}
// glm::normalize  detail/func_geometric.inl:88-96 + inversesqrt func_exponential.inl:130-133
inline vec3 normalize(vec3 v) {
  float s = 1.0f / std::sqrt(dot(v, v));
  return {v.x * s, v.y * s, v.z * s};
}
// glm::cross  detail/func_geometric.inl:74-86
inline vec3 cross(vec3 x, vec3 y) {
  return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline vec4 add4(vec4 a, vec4 b) {
  return {{a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3]}};
}
inline vec4 mul4s(vec4 a, float s) { return {{a.v[0] * s, a.v[1] * s, a.v[2] * s, a.v[3] * s}}; }

inline mat4 identity() {
  mat4 m;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) m.c[i].v[j] = (i == j) ? 1.0f : 0.0f;
  return m;
}

// glm::rotate(m, angle, v)  gtc/matrix_transform.inl:19-47
mat4 rotate(const mat4& m, float angle, vec3 v) {
  const float a = angle;
  const float c = std::cos(a);
  const float s = std::sin(a);
  vec3 axis = normalize(v);
  vec3 temp = {(1.0f - c) * axis.x, (1.0f - c) * axis.y, (1.0f - c) * axis.z};
  float R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = temp.x * axis.y + s * axis.z;
  R[0][2] = temp.x * axis.z - s * axis.y;
  R[1][0] = temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = temp.y * axis.z + s * axis.x;
  R[2][0] = temp.z * axis.x + s * axis.y;
  R[2][1] = temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  mat4 out;
  for (int i = 0; i < 3; ++i)
    out.c[i] = add4(add4(mul4s(m.c[0], R[i][0]), mul4s(m.c[1], R[i][1])), mul4s(m.c[2], R[i][2]));
  out.c[3] = m.c[3];
  return out;
}

// mat4 * mat4  detail/type_mat4x4.inl:595-613: ((A0*b0 + A1*b1) + A2*b2) + A3*b3
mat4 matmul(const mat4& a, const mat4& b) {
  mat4 r;
  for (int j = 0; j < 4; ++j)
    r.c[j] = add4(add4(add4(mul4s(a.c[0], b.c[j].v[0]), mul4s(a.c[1], b.c[j].v[1])),
                       mul4s(a.c[2], b.c[j].v[2])),
                  mul4s(a.c[3], b.c[j].v[3]));
  return r;
}

// mat4 * vec4  detail/type_mat4x4.inl:501-535: (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
vec4 matvec(const mat4& m, vec4 v) {
  vec4 add0 = add4(mul4s(m.c[0], v.v[0]), mul4s(m.c[1], v.v[1]));
  vec4 add1 = add4(mul4s(m.c[2], v.v[2]), mul4s(m.c[3], v.v[3]));
  return add4(add0, add1);
}

inline vec3 ld3(const float* p) { return {p[0], p[1], p[2]}; }
inline void st3(float* p, vec3 v) {
  p[0] = v.x;
  p[1] = v.y;
  p[2] = v.z;
}

}  // namespace

extern "C" {

int rm_api_version(void) { return RM_API_VERSION; }

// Camera::Camera(width, height, mouseSensitivity, keyboardSpeed, pos, lookAt, up)
// camera.cpp:8-14.  As in the reference, the constructor's `up` parameter
// shadows the member (camera.cpp:13 assigns the parameter), so the member `up`
// keeps its zero-initialised value (the reference instance is a global,
// main.cpp:40), as do angleX/angleY/xpos/ypos.  lookAt() overwrites the basis
// before the first dispatch (main.cpp:97).
int rm_camera_init(rm_camera_state* c, int32_t width, int32_t height, float mouseSensitivity,
                   float keyboardSpeed, const float pos[3], const float lookAt[3],
                   const float up[3]) {
  if (!c || !pos || !lookAt || !up) return RM_ERR_INVALID;
  std::memset(c, 0, sizeof(*c));
  c->width = width;
  c->height = height;
  c->mouseSensitivity = mouseSensitivity;
  c->keyboardSpeed = keyboardSpeed;
  st3(c->cameraPos, ld3(pos));
  vec3 p = ld3(pos), l = ld3(lookAt), u = ld3(up);
  vec3 fwd = normalize({l.x - p.x, l.y - p.y, l.z - p.z});
  vec3 right = normalize(cross(u, fwd));
  st3(c->forward, fwd);
  st3(c->right, right);
  return RM_OK;
}

// Camera::setMouse  camera.cpp:16-20
int rm_camera_set_mouse(rm_camera_state* c, float x, float y) {
  if (!c) return RM_ERR_INVALID;
  c->xpos = x;
  c->ypos = y;
  return RM_OK;
}

// Camera::lookAt  camera.cpp:22-51
int rm_camera_look_at(rm_camera_state* c, int zN, int zP, int xN, int xP, int halfSpeed,
                      float deltaTime) {
  if (!c) return RM_ERR_INVALID;
  c->angleX = c->xpos * c->mouseSensitivity;
  c->angleY = c->ypos * c->mouseSensitivity;
  mat4 rotateX = rotate(identity(), radians(c->angleY), {1.0f, 0.0f, 0.0f});
  mat4 rotateY = rotate(identity(), radians(c->angleX), {0.0f, 1.0f, 0.0f});
  mat4 R = matmul(rotateY, rotateX);
  vec4 f4 = matvec(R, {{0.0f, 0.0f, -1.0f, 0.0f}});
  vec4 u4 = matvec(R, {{0.0f, 1.0f, 0.0f, 0.0f}});
  vec3 fwd = normalize({f4.v[0], f4.v[1], f4.v[2]});
  vec3 up = normalize({u4.v[0], u4.v[1], u4.v[2]});
  vec3 right = normalize(cross(fwd, up));
  st3(c->forward, fwd);
  st3(c->up, up);
  st3(c->right, right);
  c->keyboardSpeed = halfSpeed ? 5.0f : 10.0f;
  vec3 pos = ld3(c->cameraPos);
  auto step = [&](vec3 axis, float sign) {
    // cameraPos += (keyboardSpeed * (+/-axis)) * deltaTime   camera.cpp:39-50
    vec3 a = {sign * axis.x, sign * axis.y, sign * axis.z};
    vec3 k = {c->keyboardSpeed * a.x, c->keyboardSpeed * a.y, c->keyboardSpeed * a.z};
    pos = {pos.x + k.x * deltaTime, pos.y + k.y * deltaTime, pos.z + k.z * deltaTime};
  };
  if (zN) step(fwd, 1.0f);
  if (zP) step(fwd, -1.0f);
  if (xN) step(right, -1.0f);
  if (xP) step(right, 1.0f);
  st3(c->cameraPos, pos);
  return RM_OK;
}

// main.cpp:103-106: setVec4("camera.pos"|"dir"|"yAxis"|"xAxis", v.x, v.y, v.z, 0)
int rm_camera_to_uniform(const rm_camera_state* c, rm_camera* out) {
  if (!c || !out) return RM_ERR_INVALID;
  for (int k = 0; k < 3; ++k) {
    out->pos[k] = c->cameraPos[k];
    out->dir[k] = c->forward[k];
    out->yAxis[k] = c->up[k];
    out->xAxis[k] = c->right[k];
  }
  out->pos[3] = out->dir[3] = out->yAxis[3] = out->xAxis[3] = 0.0f;
  return RM_OK;
}

// ---- interactive input: main.cpp's GLFW globals/callbacks ----
// The reference keeps this state in globals (main.cpp:23-39); here it is one
// struct per front-end.  The float/double conversions follow the reference's
// declared types exactly: lastX/lastY/deltaTime/lastFrame are float, GLFW hands
// doubles to the callbacks, and halfSpeed is a float holding a bool.

int rm_input_init(rm_input_state* s, int32_t screen_width, int32_t screen_height) {
  if (!s || screen_width <= 0 || screen_height <= 0) return RM_ERR_INVALID;
  std::memset(s, 0, sizeof(*s));
  s->AA = 1;                                      // main.cpp:27
  s->lastX = (float)(screen_width / 2.0);         // main.cpp:35 (SCREEN_WIDTH / 2.0)
  s->lastY = (float)(screen_height / 2.0);        // main.cpp:36
  s->firstMouse = 1;                              // main.cpp:37
  s->mouseSensitivity = (float)0.001;             // MousePosition.hpp:8 (double literal -> float)
  return RM_OK;                                   // pitch = yaw = 0: MousePosition.cpp:4-5
}

// main.cpp:93-95
int rm_input_begin_frame(rm_input_state* s, double now_seconds) {
  if (!s) return RM_ERR_INVALID;
  const float currentFrame = (float)now_seconds;
  s->deltaTime = currentFrame - s->lastFrame;
  s->lastFrame = currentFrame;
  return RM_OK;
}

// processInput  main.cpp:155-195
int rm_input_process(rm_input_state* s, uint32_t held, rm_camera_state* cam) {
  if (!s || !cam) return RM_ERR_INVALID;
  const bool W = held & RM_HELD_W, A = held & RM_HELD_A, S = held & RM_HELD_S,
             D = held & RM_HELD_D;
  if (held & RM_HELD_ESCAPE) s->shouldClose = 1;
  s->zaxisNeg = W;
  s->zaxisPos = S;
  s->xaxisPos = D;
  s->xaxisNeg = A;
  // diagonal pairs only: W+S or A+D alone keep full speed (main.cpp:185-188)
  const bool half = (W && A) || (W && D) || (A && S) || (S && D);
  s->halfSpeed = half ? 1.0f : 0.0f;
  return rm_camera_look_at(cam, s->zaxisNeg, s->zaxisPos, s->xaxisNeg, s->xaxisPos,
                           s->halfSpeed != 0.0f, s->deltaTime);
}

// key_callback  main.cpp:197-217
int rm_input_key(rm_input_state* s, int32_t key, int32_t action) {
  if (!s) return RM_ERR_INVALID;
  if (action != RM_PRESS) return RM_OK;
  if (key == RM_KEY_UP && s->bounce < 5) s->bounce += 1;
  if (key == RM_KEY_DOWN && s->bounce > 0) s->bounce -= 1;
  if (key == RM_KEY_F1) s->AA = !s->AA;
  if (key == RM_KEY_L) s->showQuad = !s->showQuad;  // glPolygonMode only: no render effect
  return RM_OK;
}

// mouse_callback  main.cpp:219-234 + MouseInput::ProcessMouseOffset MousePosition.cpp:10-22
int rm_input_mouse(rm_input_state* s, double xpos, double ypos, rm_camera_state* cam) {
  if (!s || !cam) return RM_ERR_INVALID;
  if (s->firstMouse) {
    s->lastX = (float)xpos;
    s->lastY = (float)ypos;
    s->firstMouse = 0;
  }
  float xoffset = (float)((double)s->lastX - xpos);  // float - double is a double subtraction
  float yoffset = (float)((double)s->lastY - ypos);
  s->lastX = (float)xpos;
  s->lastY = (float)ypos;
  xoffset *= s->mouseSensitivity;
  yoffset *= s->mouseSensitivity;
  s->yaw += xoffset;
  s->pitch += yoffset;
  return rm_camera_set_mouse(cam, (float)-xpos, (float)-ypos);
}

// MouseInput::EulerAngles  MousePosition.cpp:24-33.  As written there: cos/sin of
// the PRODUCT, and the unqualified cos/sin of a float resolve to the C library's
// double functions (no std:: float overload is visible), so the trig runs in
// double and each component is rounded to float on assignment.
int rm_input_euler_angles(const rm_input_state* s, float out[3]) {
  if (!s || !out) return RM_ERR_INVALID;
  const double ry = radians(s->yaw), rp = radians(s->pitch);
  vec3 front;
  front.x = (float)std::cos(ry * std::cos(rp));
  front.y = (float)std::sin(rp);
  front.z = (float)std::sin(ry * std::cos(rp));
  st3(out, normalize(front));
  return RM_OK;
}

// main.cpp:101-120, the uploads input drives
int rm_input_to_uniforms(const rm_input_state* s, const rm_camera_state* cam, rm_uniforms* u) {
  if (!s || !cam || !u) return RM_ERR_INVALID;
  rm_camera_to_uniform(cam, &u->camera);
  u->iTime = s->lastFrame;
  u->AA = s->AA ? 1 : 0;
  u->bounceVar = s->bounce;
  rm_input_euler_angles(s, u->mouse);
  u->iMouse[0] = s->yaw;
  u->iMouse[1] = s->pitch;
  return RM_OK;
}

// Defaults: main.cpp:27,30 (AA on, bounce 0), light block main.cpp:108-114,
// start-up camera main.cpp:40 after lookAt with zero mouse.
int rm_default_uniforms(rm_uniforms* u) {
  if (!u) return RM_ERR_INVALID;
  std::memset(u, 0, sizeof(*u));
  rm_camera_state cam;
  const float pos[3] = {0.0f, 0.0f, 0.0f}, look[3] = {0.0f, 0.0f, -1.0f}, up[3] = {0.0f, 1.0f, 0.0f};
  rm_camera_init(&cam, 1080, 1080, 0.025f, 10.0f, pos, look, up);
  rm_camera_look_at(&cam, 0, 0, 0, 0, 0, 0.0f);
  rm_camera_to_uniform(&cam, &u->camera);
  const float lp[3] = {-5.0f, 5.0f, -10.0f};
  const float la[3] = {0.03f, 0.04f, 0.1f};
  const float ld[3] = {0.8f, 0.8f, 0.8f};
  const float ls[3] = {0.5f, 0.5f, 0.5f};
  std::memcpy(u->light.position, lp, sizeof lp);
  std::memcpy(u->light.ambient, la, sizeof la);
  std::memcpy(u->light.diffuse, ld, sizeof ld);
  std::memcpy(u->light.specular, ls, sizeof ls);
  u->light.constant = 1.0f;
  u->light.linear = 0.009f;
  u->light.quadratic = 0.00032f;
  u->iTime = 0.0f;
  u->bounceVar = 0;
  u->AA = 1;
  u->workgroups = 39;  // local_size of computeShader.glsl:12 (ignored)
  u->mouse[0] = 1.0f;  // MouseInput::EulerAngles() at yaw = pitch = 0 (ignored)
  u->shadow_mode = RM_SHADOW_SOFT;
  return RM_OK;
}

int rm_sweep_uniforms(int32_t frame, int32_t nframes, int32_t bounceVar, int32_t AA,
                      int32_t shadow_mode, rm_uniforms* out) {
  if (!out || nframes <= 0 || frame >= nframes || bounceVar < 0 || bounceVar > 5)
    return RM_ERR_INVALID;
  rm_default_uniforms(out);
  rm_camera_state cam;
  const float look[3] = {0.0f, 0.0f, -1.0f}, up[3] = {0.0f, 1.0f, 0.0f};
  if (frame < 0) {  // default frame D: the reference's start-up view
    const float pos[3] = {0.0f, 0.0f, 0.0f};
    rm_camera_init(&cam, 1080, 1080, 0.025f, 10.0f, pos, look, up);
    out->iTime = 0.0f;
  } else {
    const float pos[3] = {0.0f, 0.0f, 15.0f};
    rm_camera_init(&cam, 1080, 1080, 0.025f, 10.0f, pos, look, up);
    double yaw = nframes > 1 ? -20.0 + 40.0 * (double)frame / (double)(nframes - 1) : 0.0;
    rm_camera_set_mouse(&cam, (float)(yaw / 0.025), (float)(-5.0 / 0.025));
    out->iTime = (float)frame / 60.0f;
  }
  rm_camera_look_at(&cam, 0, 0, 0, 0, 0, 0.0f);
  rm_camera_to_uniform(&cam, &out->camera);
  out->bounceVar = bounceVar;
  out->AA = AA ? 1 : 0;
  out->shadow_mode = shadow_mode;
  return RM_OK;
}

// ---- row sharding: the weighted interleave of rm_shard.hpp ------
// A valid map for (row_block, rank0_rows, nshards >= 2): rows per round fit in
// 2^30 (so every row index below stays in int32).
static bool shard_map(int32_t row_block, int32_t rank0_rows, int32_t nshards, rm::ShardMap* m) {
  if (row_block <= 0 || rank0_rows < 0 || nshards < 2) return false;
  m->rb = row_block;
  m->rb0 = rank0_rows ? rank0_rows : row_block;
  m->n = nshards;
  return (int64_t)m->rb0 + (int64_t)(nshards - 1) * row_block <= (int64_t)1 << 30;
}

int rm_shard_rows(int32_t height, int32_t row_block, int32_t rank0_rows, int32_t nshards, int32_t shard,
                  int32_t* rows, int32_t* rows_cap) {
  if (height <= 0 || height > 65536) return RM_ERR_INVALID;
  if (nshards <= 1) {
    if (shard != 0) return RM_ERR_INVALID;
    if (rows) *rows = height;
    if (rows_cap) *rows_cap = height;
    return RM_OK;
  }
  rm::ShardMap m;
  if (!shard_map(row_block, rank0_rows, nshards, &m) || shard < 0 || shard >= nshards) return RM_ERR_INVALID;
  if (rows) *rows = rm::shard_real_rows(m, height, shard);
  if (rows_cap) *rows_cap = rm::shard_rows_cap(m, height);
  return RM_OK;
}

int32_t rm_shard_to_global(int32_t height, int32_t row_block, int32_t rank0_rows, int32_t nshards, int32_t shard,
                           int32_t local_row) {
  if (local_row < 0 || height <= 0 || height > 65536) return -1;
  if (nshards <= 1) return (shard == 0 && local_row < height) ? local_row : -1;
  rm::ShardMap m;
  if (!shard_map(row_block, rank0_rows, nshards, &m) || shard < 0 || shard >= nshards) return -1;
  if (local_row >= rm::shard_rows_cap(m, height)) return -1;
  const int32_t g = rm::shard_row(m, shard, local_row);
  return g < height ? g : -1;
}

int rm_shard_owner(int32_t height, int32_t row_block, int32_t rank0_rows, int32_t nshards, int32_t row,
                   int32_t* shard, int32_t* local_row) {
  if (!shard || !local_row || height <= 0 || height > 65536 || row < 0 || row >= height) return RM_ERR_INVALID;
  if (nshards <= 1) {
    *shard = 0;
    *local_row = row;
    return RM_OK;
  }
  rm::ShardMap m;
  if (!shard_map(row_block, rank0_rows, nshards, &m)) return RM_ERR_INVALID;
  rm::shard_owner(m, row, shard, local_row);
  return RM_OK;
}

}  // extern "C"

// ---- runtime scene table ----------------------------------
namespace {
rm_primitive prim(int32_t type, int32_t swz, int32_t id, int32_t paint, float material,
                  std::initializer_list<float> color, std::initializer_list<float> center,
                  std::initializer_list<float> param) {
  rm_primitive p;
  std::memset(&p, 0, sizeof p);
  p.type = type;
  p.swizzle = swz;
  p.id = id;
  p.paint = paint;
  p.material = material;
  std::copy(color.begin(), color.end(), p.color);
  std::copy(center.begin(), center.end(), p.center);
  std::copy(param.begin(), param.end(), p.param);
  return p;
}
}  // namespace

extern "C" int rm_default_scene(rm_primitive* out, int32_t capacity, int32_t* n) {
  if (!n) return RM_ERR_INVALID;
  // computeShader.glsl:107-123, in opU order
  const rm_primitive scene[6] = {
      prim(RM_PRIM_SPHERE, RM_SWIZZLE_XYZ, 0, RM_PAINT_SOLID, 1.0f, {0.1804f, 0.6f, 0.2157f},
           {15.0f, 0.0f, -10.0f}, {3.0f}),                                         // :111
      prim(RM_PRIM_SPHERE, RM_SWIZZLE_XYZ, 1, RM_PAINT_SOLID, 1.0f, {0.0f, 0.851f, 1.0f},
           {-25.0f, 0.0f, -10.0f}, {3.0f}),                                        // :112
      prim(RM_PRIM_BLEND, RM_SWIZZLE_XYZ, 4, RM_PAINT_SOLID, 1.0f, {0.4863f, 0.3529f, 0.702f},
           {-5.0f, 0.0f, -10.0f}, {3.0f, 2.5f, 2.5f, 3.0f}),                       // :115-117
      prim(RM_PRIM_TORUS, RM_SWIZZLE_XZY, 5, RM_PAINT_SOLID, 1.0f, {0.9137f, 0.549f, 0.0f},
           {-5.0f, 0.0f, 10.0f}, {2.5f, 0.5f}),                                    // :119
      prim(RM_PRIM_CAPSULE, RM_SWIZZLE_XYZ, 6, RM_PAINT_SOLID, 1.0f, {0.8f, 0.0902f, 0.4824f},
           {-5.0f, -2.0f, -30.0f}, {-0.1f, 0.1f, -0.1f, 2.0f, 4.0f, 2.0f, 1.0f}),  // :120
      prim(RM_PRIM_PLANE, RM_SWIZZLE_XYZ, 7, RM_PAINT_CHECKERS, 0.0f, {0.0f, 0.0f, 0.0f},
           {0.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f, 5.5f}),                          // :121
  };
  *n = 6;
  if (out) {
    if (capacity < 6) return RM_ERR_INVALID;
    std::memcpy(out, scene, sizeof scene);
  }
  return RM_OK;
}

namespace rm {

// Exit header of a table (rm_internal.hpp ExitWord; used by rm_table.hip).  In
// exact arithmetic every entry's distance is bounded below by a ball or is
// linear:
//   sphere  |q| - r;  box (a >= 0)  >= |q| - |a|;  blend (a >= 0, weights in
//   [0, 1])  >= |q| - max(|a|, r);  torus  >= |q| - (|R| + r) (triangle
//   inequality);  capsule  >= |q - M| - (|ba|/2 + r), M = a + ba/2;
//   plane  = dot(q, n) + w, linear along a ray;
// q = swizzle(p - c) is an isometry of p - c, so the balls map back to world
// space.  C is the mean of the ball centres and R >= max_k(|C - c_k| + R_k),
// rounded up.  The float error of an entry's value at p is below
// 40 u N (|p|_1 + S_k) (u = 2^-24; S_k = |c_k|_1 + sum |params|; N = the largest
// plane |n|_1, >= 1); the device slack sigma (|p|_1 + S), sigma = 2^-12 N,
// S = max_k S_k + 1, is two orders of magnitude above it.
// The same balls serve the culling of the table kernels' sdf (word TW_BALL of
// each entry; planes and every entry of a table without valid bounds get +inf).
static void exit_bounds(const rm_primitive* prims, int32_t n, uint32_t* out) {
  uint32_t* hdr = out + (size_t)n * TABLE_WORDS;
  float h[EXIT_WORDS];
  std::memset(h, 0, sizeof h);
  std::vector<double> cx, cy, cz, rr;
  std::vector<int32_t> ball_of;  // entry of each ball
  // the bounded entries' box: each entry's value is at least its distance to
  // the solid it bounds (exact sdfs; a blend is above the lower of its box and
  // sphere), so at least the distance to the solid's box, per axis
  double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
  double S = 0.0, N = 1.0, lip = 1.0;
  int np = 0;
  bool ok = true;
  for (int32_t k = 0; k < n && ok; ++k) {
    const rm_primitive& p = prims[k];
    double a[7];
    for (int j = 0; j < 7; ++j) a[j] = p.param[j];
    double sk = std::fabs((double)p.center[0]) + std::fabs((double)p.center[1]) + std::fabs((double)p.center[2]);
    for (int j = 0; j < 7; ++j) sk += std::fabs(a[j]);
    if (!std::isfinite(sk)) ok = false;
    S = std::max(S, sk);
    // world offset of a q-space vector (the swizzle is its own inverse)
    auto world = [&](double x, double y, double z, double* o) {
      o[0] = x;
      o[1] = p.swizzle == RM_SWIZZLE_XZY ? z : y;
      o[2] = p.swizzle == RM_SWIZZLE_XZY ? y : z;
    };
    double m[3] = {0.0, 0.0, 0.0}, R = 0.0;
    double qlo[3] = {0.0, 0.0, 0.0}, qhi[3] = {0.0, 0.0, 0.0};  // the solid's box, q-space
    auto sym = [&](double hx, double hy, double hz) {
      const double hh[3] = {hx, hy, hz};
      for (int j = 0; j < 3; ++j) qlo[j] = -hh[j], qhi[j] = hh[j];
    };
    switch (p.type) {
      case RM_PRIM_SPHERE:
        R = a[0];
        sym(std::max(a[0], 0.0), std::max(a[0], 0.0), std::max(a[0], 0.0));
        break;
      case RM_PRIM_BOX:
      case RM_PRIM_BLEND:
        if (a[0] < 0.0 || a[1] < 0.0 || a[2] < 0.0) ok = false;
        R = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (p.type == RM_PRIM_BLEND) {
          R = std::max(R, a[3]);
          const double r = std::max(a[3], 0.0);
          sym(std::max(a[0], r), std::max(a[1], r), std::max(a[2], r));
        } else {
          sym(a[0], a[1], a[2]);
        }
        break;
      case RM_PRIM_TORUS: {
        // the ring in the q.xz plane: |q.xz| <= |R| + r, |q.y| <= r
        R = std::fabs(a[0]) + a[1];
        const double r = std::max(a[1], 0.0), w = std::fabs(a[0]) + r;
        sym(w, r, w);
        break;
      }
      case RM_PRIM_CAPSULE: {
        const double bx = a[3] - a[0], by = a[4] - a[1], bz = a[5] - a[2];
        const double bl = std::sqrt(bx * bx + by * by + bz * bz);
        // the kernel divides by the float dot(ba, ba); 0 gives NaN distances
        const float fbx = p.param[3] - p.param[0], fby = p.param[4] - p.param[1], fbz = p.param[5] - p.param[2];
        if (!((fbx * fbx + fby * fby) + fbz * fbz > 0.0f)) ok = false;
        world(a[0] + bx / 2, a[1] + by / 2, a[2] + bz / 2, m);
        R = bl / 2 + a[6];
        const double r = std::max(a[6], 0.0);
        for (int j = 0; j < 3; ++j) qlo[j] = std::min(a[j], a[3 + j]) - r, qhi[j] = std::max(a[j], a[3 + j]) + r;
        break;
      }
      default: {  // plane
        if (np == EX_MAX_PLANES) {
          ok = false;
          break;
        }
        double nw[3];
        world(a[0], a[1], a[2], nw);
        const double off = a[3] - (nw[0] * p.center[0] + nw[1] * p.center[1] + nw[2] * p.center[2]);
        float* pl = h + EX_PLANES + 4 * np++;
        for (int j = 0; j < 3; ++j) pl[j] = (float)nw[j];
        pl[3] = (float)off;
        N = std::max(N, std::fabs(nw[0]) + std::fabs(nw[1]) + std::fabs(nw[2]));
        lip = std::max(lip, std::sqrt(nw[0] * nw[0] + nw[1] * nw[1] + nw[2] * nw[2]));
        continue;
      }
    }
    cx.push_back(p.center[0] + m[0]);
    cy.push_back(p.center[1] + m[1]);
    cz.push_back(p.center[2] + m[2]);
    {
      double wl[3], wh[3];  // the swizzle permutes axes: the box maps to a box
      world(qlo[0], qlo[1], qlo[2], wl);
      world(qhi[0], qhi[1], qhi[2], wh);
      for (int j = 0; j < 3; ++j) {
        blo[j] = std::min(blo[j], (double)p.center[j] + wl[j]);
        bhi[j] = std::max(bhi[j], (double)p.center[j] + wh[j]);
      }
    }
    rr.push_back(R);
    ball_of.push_back(k);
  }
  double C[3] = {0.0, 0.0, 0.0}, RA = 0.0;
  if (!cx.empty()) {
    for (size_t k = 0; k < cx.size(); ++k) C[0] += cx[k], C[1] += cy[k], C[2] += cz[k];
    for (double& v : C) v = (double)(float)(v / (double)cx.size());  // the device's float centre
    for (size_t k = 0; k < cx.size(); ++k) {
      const double dx = cx[k] - C[0], dy = cy[k] - C[1], dz = cz[k] - C[2];
      RA = std::max(RA, std::sqrt(dx * dx + dy * dy + dz * dz) + rr[k]);
    }
  } else {
    RA = -1e30;  // no bounded entry: the ball bound never binds
  }
  const double sigma = 0x1p-12 * N;
  ok = ok && std::isfinite(RA) && std::isfinite(S) && std::isfinite(sigma) && S < 1e15;
  h[EX_VALID] = ok ? 1.0f : 0.0f;
  h[EX_CX] = (float)C[0], h[EX_CY] = (float)C[1], h[EX_CZ] = (float)C[2];
  h[EX_R] = (float)(RA * (1.0 + 0x1p-20) + 0x1p-20 * (1.0 + std::fabs(RA)));  // rounded up
  h[EX_SIGMA] = (float)(sigma * (1.0 + 0x1p-20));
  h[EX_S] = (float)((S + 1.0) * (1.0 + 0x1p-20));
  h[EX_NPLANES] = (float)np;
  h[EX_LIP] = (float)(lip * (1.0 + 0x1p-20));
  for (int j = 0; j < 3; ++j) {  // rounded outward (no bounded entry: an empty box)
    h[EX_BOX + j] = cx.empty() ? 0.0f : (float)(blo[j] - 0x1p-20 * (1.0 + std::fabs(blo[j])));
    h[EX_BOX + 3 + j] = cx.empty() ? 0.0f : (float)(bhi[j] + 0x1p-20 * (1.0 + std::fabs(bhi[j])));
  }
  uint32_t eval_mask = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
  int ns = 0;
  for (size_t j = 0; ok && j < ball_of.size() && ns < EX_MAX_SLOTS; ++j) {
    h[EX_SLOTS + ns++] = (float)ball_of[j];
    eval_mask &= ~(1u << ball_of[j]);
  }
  h[EX_NSLOTS] = (float)ns;
  std::memcpy(&h[EX_EVAL_MASK], &eval_mask, sizeof eval_mask);
  uint32_t plane_mask = 0;
  for (int32_t k = 0; k < n; ++k)
    if (prims[k].type == RM_PRIM_PLANE) plane_mask |= 1u << k;
  std::memcpy(&h[EX_PLANE_MASK], &plane_mask, sizeof plane_mask);
  std::memcpy(hdr, h, sizeof h);
  const float INF = std::numeric_limits<float>::infinity();
  for (int32_t k = 0; k < n; ++k) {
    float b[4] = {0.0f, 0.0f, 0.0f, INF};
    std::memcpy(out + (size_t)k * TABLE_WORDS + TW_BALL, b, sizeof b);
  }
  if (!ok) return;
  for (size_t j = 0; j < ball_of.size(); ++j) {
    // centre rounded to float; the radius absorbs that rounding and is rounded up
    const float c[3] = {(float)cx[j], (float)cy[j], (float)cz[j]};
    const double e = std::fabs(c[0] - cx[j]) + std::fabs(c[1] - cy[j]) + std::fabs(c[2] - cz[j]);
    const float b[4] = {c[0], c[1], c[2],
                        (float)((rr[j] + e) * (1.0 + 0x1p-20) + 0x1p-20 * (1.0 + std::fabs(rr[j])))};
    std::memcpy(out + (size_t)ball_of[j] * TABLE_WORDS + TW_BALL, b, sizeof b);
  }
}

int compile_scene(const rm_primitive* prims, int32_t n, uint32_t* out, const char** why) {
  auto bad = [&](const char* m) {
    if (why) *why = m;
    return RM_ERR_INVALID;
  };
  if (!prims || n < 1 || n > RM_MAX_PRIMITIVES)
    return bad("rm_set_scene: need 1..RM_MAX_PRIMITIVES primitives");
  for (int32_t k = 0; k < n; ++k) {
    const rm_primitive& p = prims[k];
    if (p.type < RM_PRIM_SPHERE || p.type > RM_PRIM_PLANE) return bad("rm_set_scene: unknown primitive type");
    if (p.swizzle != RM_SWIZZLE_XYZ && p.swizzle != RM_SWIZZLE_XZY) return bad("rm_set_scene: unknown swizzle");
    if (p.paint != RM_PAINT_SOLID && p.paint != RM_PAINT_CHECKERS) return bad("rm_set_scene: unknown paint");
    uint32_t* w = out + (size_t)k * TABLE_WORDS;
    float f[TABLE_WORDS];
    std::memset(f, 0, sizeof f);
    f[TW_MATERIAL] = p.material;
    for (int j = 0; j < 3; ++j) {
      f[TW_COLOR + j] = p.color[j];
      f[TW_CENTER + j] = p.center[j];
    }
    float* q = f + TW_P;
    const float* a = p.param;
    switch (p.type) {
      case RM_PRIM_CAPSULE: {  // glsl:100-101: ba = b - a, dot(ba, ba) = (x*x + y*y) + z*z
        const float bax = a[3] - a[0], bay = a[4] - a[1], baz = a[5] - a[2];
        q[0] = a[0], q[1] = a[1], q[2] = a[2];
        q[3] = bax, q[4] = bay, q[5] = baz;
        q[6] = (bax * bax + bay * bay) + baz * baz;
        q[7] = a[6];
        break;
      }
      default:
        for (int j = 0; j < 7; ++j) q[j] = a[j];
    }
    std::memcpy(w, f, sizeof f);
    w[TW_TYPE] = (uint32_t)p.type;
    w[TW_SWIZZLE] = (uint32_t)p.swizzle;
    w[TW_ID] = (uint32_t)p.id;
    w[TW_PAINT] = (uint32_t)p.paint;
  }
  exit_bounds(prims, n, out);
  return RM_OK;
}

}  // namespace rm

// ---- uniform lookup by GLSL name (shader.hpp:19-69 semantics) -----------------
namespace rm {

float* uniform_floats(rm_uniforms* u, const char* name, int* n) {
  struct Entry {
    const char* name;
    size_t off;
    int n;
  };
  static const Entry table[] = {
      {"camera.pos", offsetof(rm_uniforms, camera.pos), 4},
      {"camera.dir", offsetof(rm_uniforms, camera.dir), 4},
      {"camera.yAxis", offsetof(rm_uniforms, camera.yAxis), 4},
      {"camera.xAxis", offsetof(rm_uniforms, camera.xAxis), 4},
      {"light.position", offsetof(rm_uniforms, light.position), 3},
      {"light.ambient", offsetof(rm_uniforms, light.ambient), 3},
      {"light.diffuse", offsetof(rm_uniforms, light.diffuse), 3},
      {"light.specular", offsetof(rm_uniforms, light.specular), 3},
      {"light.constant", offsetof(rm_uniforms, light.constant), 1},
      {"light.linear", offsetof(rm_uniforms, light.linear), 1},
      {"light.quadratic", offsetof(rm_uniforms, light.quadratic), 1},
      {"iTime", offsetof(rm_uniforms, iTime), 1},
      {"drand48", offsetof(rm_uniforms, drand48), 1},
      {"mouse", offsetof(rm_uniforms, mouse), 3},
      {"iMouse", offsetof(rm_uniforms, iMouse), 2},
  };
  for (const Entry& e : table)
    if (std::strcmp(e.name, name) == 0) {
      *n = e.n;
      return reinterpret_cast<float*>(reinterpret_cast<char*>(u) + e.off);
    }
  return nullptr;
}

int32_t* uniform_ints(rm_uniforms* u, const char* name) {
  if (std::strcmp(name, "bounceVar") == 0) return &u->bounceVar;
  if (std::strcmp(name, "AA") == 0) return &u->AA;
  if (std::strcmp(name, "shadow_mode") == 0) return &u->shadow_mode;
  if (std::strcmp(name, "workgroups") == 0) return reinterpret_cast<int32_t*>(&u->workgroups);
  return nullptr;
}

}  // namespace rm
