// rm/texture.hpp — C++ mirror of the reference's Texture (source/texture.hpp:3-14,
// texture.cpp:10-21) and of the program/uniform helpers of source/shader.hpp:17-69
// and main.cpp:123-125, over librm's C-ABI.  `texOutput` is the librm context
// that owns the device image (the GL texture name in the reference).
#pragma once

#include <rm_api.h>

#include <string>

namespace rm {

class Texture {
 public:
  int texWidth;
  int texHeight;
  rm_ctx* texOutput = nullptr;

  Texture() noexcept : texWidth(720), texHeight(720) {}                 // texture.cpp:4-5
  Texture(unsigned int SCREEN_WIDTH, unsigned int SCREEN_HEIGHT) noexcept  // texture.cpp:7-8
      : texWidth((int)SCREEN_WIDTH), texHeight((int)SCREEN_HEIGHT) {}
  ~Texture() { rm_destroy(texOutput); }
  Texture(const Texture&) = delete;
  Texture& operator=(const Texture&) = delete;

  // texture.cpp:10-21: allocate the image (RGBA8 for display + the RGBA32F
  // storage format of the reference texture).  Returns 0 or an RM_ERR_*.
  // ngpus >= 1: the image is rendered by ngpus devices (device, device+1, ...),
  // one row-block shard each, gathered with RCCL onto the first.
  int GenerateTexture(int outputs = RM_OUT_RGBA8 | RM_OUT_RGBA32F, int kernel = RM_KERNEL_AUTO,
                      int device = -1, int ngpus = 0) {
    rm_config cfg;
    rm_config_init(&cfg, texWidth, texHeight);
    cfg.device = device;
    cfg.outputs = outputs;
    cfg.kernel = kernel;
    cfg.ngpus = ngpus;
    rm_destroy(texOutput);
    texOutput = nullptr;
    return rm_create(&texOutput, &cfg);
  }
};

// shader.hpp-style helpers: the "program" is the context bound to the texture.
// Unknown names are no-ops, as with GL location -1 (return value 1 reports it).
inline void useShader(rm_ctx*) {}
inline int setBool(rm_ctx* p, const std::string& n, bool v) { return rm_set_bool(p, n.c_str(), v); }
inline int setInt(rm_ctx* p, const std::string& n, int v) { return rm_set_int(p, n.c_str(), v); }
inline int setuInt(rm_ctx* p, const std::string& n, unsigned int* v) {
  return rm_set_uint(p, n.c_str(), v);
}
inline int setFloat(rm_ctx* p, const std::string& n, float v) { return rm_set_float(p, n.c_str(), v); }
inline int setVec2(rm_ctx* p, const std::string& n, float x, float y) {
  return rm_set_vec2(p, n.c_str(), x, y);
}
inline int setVec3(rm_ctx* p, const std::string& n, float x, float y, float z) {
  return rm_set_vec3(p, n.c_str(), x, y, z);
}
inline int setVec4(rm_ctx* p, const std::string& n, float x, float y, float z, float w) {
  return rm_set_vec4(p, n.c_str(), x, y, z, w);
}
// main.cpp:123 / :125
inline int dispatchCompute(rm_ctx* p) { return rm_dispatch(p); }
// n frames of uniforms in one launch (rm_dispatch_frames, API version 4): the
// images of n dispatchCompute calls; frame k via rm_read_frame_rgba8(p, k, ...)
inline int dispatchFrames(rm_ctx* p, const rm_uniforms* frames, int n) {
  return rm_dispatch_frames(p, frames, n);
}
inline int memoryBarrier(rm_ctx* p) { return rm_synchronize(p); }

}  // namespace rm
