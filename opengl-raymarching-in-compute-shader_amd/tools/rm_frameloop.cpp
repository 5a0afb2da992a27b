// rm_frameloop.cpp — headless replacement of the reference's frame loop
// (main.cpp:42-153): the same per-frame host step — camera update, uniform
// upload by name (main.cpp:99-120), dispatch (:123), barrier (:125) — driven by
// a synthetic camera sweep instead of a window, with the reference's FPS print
// (:136-143) and its runtime toggles as flags (bounce 0..5 :199-204, AA F1
// :206-207).  Optionally dumps the last frame as a PPM (top row first).
//
// --input FILE replays a recorded input script through rm::Input (the
// reference's processInput / key_callback / mouse_callback)
// instead of the sweep; one line per event, in order:
//   frame <now_seconds> <held>   begin a frame: clock, processInput(held), render
//   key <glfw_key> <action>      key_callback
//   mouse <xpos> <ypos>          mouse_callback
// held = OR of W 1, A 2, S 4, D 8, ESC 16.  The loop stops after ESC, like
// while (!glfwWindowShouldClose(window)) (main.cpp:92).
//
// --gpus N renders every frame on N GPUs of this node from this one process
// (rm_config.ngpus: one row-block shard per device, RCCL gather onto the first,
// SURVEY 8(e)); --graph replays each frame from captured hipGraphs.
//
//   rm_frameloop [--width W] [--height H] [--frames N] [--bounces B] [--aa 0|1]
//                [--hard-shadows] [--kernel auto|pixel] [--dump out.ppm]
//                [--input script.txt] [--gpus N] [--graph] [--batch B]
// --batch B renders B consecutive frames per launch (rm_dispatch_frames: the
// setters run per frame as before, the uniforms of B frames are collected and
// dispatched together; the last frame's image is the one dumped).
#include <rm/camera.hpp>
#include <rm/input.hpp>
#include <rm/texture.hpp>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  int W = 1080, H = 1080, frames = 120, bounce = 0, aa = 1, shadow = RM_SHADOW_SOFT;
  int kernel = RM_KERNEL_AUTO, ngpus = 0, graph = 0, batch = 1;
  const char* dump = nullptr;
  const char* script = nullptr;
  for (int i = 1; i < argc; ++i) {
    auto next = [&](const char* flag) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "%s needs a value\n", flag);
        std::exit(2);
      }
      return argv[++i];
    };
    if (!std::strcmp(argv[i], "--width")) W = std::atoi(next("--width"));
    else if (!std::strcmp(argv[i], "--height")) H = std::atoi(next("--height"));
    else if (!std::strcmp(argv[i], "--frames")) frames = std::atoi(next("--frames"));
    else if (!std::strcmp(argv[i], "--bounces")) bounce = std::atoi(next("--bounces"));
    else if (!std::strcmp(argv[i], "--aa")) aa = std::atoi(next("--aa"));
    else if (!std::strcmp(argv[i], "--hard-shadows")) shadow = RM_SHADOW_HARD;
    else if (!std::strcmp(argv[i], "--dump")) dump = next("--dump");
    else if (!std::strcmp(argv[i], "--input")) script = next("--input");
    else if (!std::strcmp(argv[i], "--gpus")) ngpus = std::atoi(next("--gpus"));
    else if (!std::strcmp(argv[i], "--graph")) graph = 1;
    else if (!std::strcmp(argv[i], "--batch")) batch = std::atoi(next("--batch"));
    else if (!std::strcmp(argv[i], "--kernel")) {
      std::string k = next("--kernel");
      kernel = k == "pixel" ? RM_KERNEL_PIXEL : RM_KERNEL_AUTO;
    } else {
      std::fprintf(stderr, "unknown flag %s\n", argv[i]);
      return 2;
    }
  }
  if (batch < 1 || batch > RM_MAX_BATCH || (batch > 1 && graph)) {
    std::fprintf(stderr, "--batch must be in 1..%d (and not with --graph)\n", RM_MAX_BATCH);
    return 2;
  }
  if (bounce < 0) bounce = 0;  // the key callback clamps to 0..5 (main.cpp:199-204)
  if (bounce > 5) bounce = 5;

  // main.cpp:40 — the global camera; the sweep moves it to (0,0,15)
  rm::Camera camera(W, H, 0.025f, 10.0f, rm::vec3(0, 0, 0), rm::vec3(0, 0, -1), rm::vec3(0, 1, 0));
  rm::Input input(camera, W, H);  // main.cpp:23-39 globals + callbacks
  FILE* events = nullptr;
  if (script) {
    events = std::fopen(script, "r");
    if (!events) {
      std::fprintf(stderr, "cannot open %s\n", script);
      return 2;
    }
    // the reference starts at bounce 0 / AA on; the flags seed the toggles
    for (int b = 0; b < bounce; ++b) input.key_callback(RM_KEY_UP, 0, RM_PRESS, 0);
    if (!aa) input.key_callback(RM_KEY_F1, 0, RM_PRESS, 0);
    frames = 1 << 30;
  } else {
    camera.cameraPos = rm::vec3(0.0f, 0.0f, 15.0f);
  }
  rm::Texture tex(W, H);  // main.cpp:70-71
  if (int rc = tex.GenerateTexture(RM_OUT_RGBA8, kernel, -1, ngpus); rc != RM_OK) {
    std::fprintf(stderr, "GenerateTexture failed (%d): %s\n", rc, rm_last_error(nullptr));
    return 1;
  }
  rm_ctx* marching = tex.texOutput;
  if (graph && rm_graph_enable(marching, 1) != RM_OK) {
    std::fprintf(stderr, "rm_graph_enable failed: %s\n", rm_last_error(marching));
    return 1;
  }
  unsigned int workgroups = 39;  // main.cpp:76-77 (ignored by librm)
  std::vector<rm_uniforms> pending((size_t)batch);
  int npending = 0;
  auto flush = [&]() {
    if (rm_dispatch_frames(marching, pending.data(), npending) != RM_OK || rm::memoryBarrier(marching) != RM_OK) {
      std::fprintf(stderr, "batch of %d frames failed: %s\n", npending, rm_last_error(marching));
      return false;
    }
    npending = 0;
    return true;
  };

  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  double lastTime = 0.0;
  unsigned counter = 0, total = 0;
  for (int f = 0; f < frames; ++f) {
    float iTime = (float)f / 60.0f;
    if (events) {  // recorded input: apply events up to and including the next frame line
      if (input.shouldClose()) break;
      char kind[16];
      bool frame_line = false;
      while (!frame_line && std::fscanf(events, "%15s", kind) == 1) {
        double a = 0.0, b = 0.0;
        if (std::fscanf(events, "%lf %lf", &a, &b) != 2) {
          std::fprintf(stderr, "bad input line after '%s'\n", kind);
          return 2;
        }
        if (!std::strcmp(kind, "frame")) {
          input.beginFrame(a);
          input.processInput((unsigned)b);
          frame_line = true;
        } else if (!std::strcmp(kind, "key")) {
          input.key_callback((int)a, 0, (int)b, 0);
        } else if (!std::strcmp(kind, "mouse")) {
          input.mouse_callback(a, b);
        } else {
          std::fprintf(stderr, "unknown input event '%s'\n", kind);
          return 2;
        }
      }
      if (!frame_line) break;  // script exhausted
      rm_uniforms u{};
      input.toUniforms(&u);
      iTime = u.iTime;
      aa = input.AA();
      bounce = input.bounce();
    } else {
      // synthetic input instead of processInput/mouse_callback (SURVEY 8(d) sweep)
      const double yaw = frames > 1 ? -20.0 + 40.0 * f / (frames - 1) : 0.0;
      camera.setMouse((float)(yaw / 0.025), (float)(-5.0 / 0.025));
      camera.lookAt(false, false, false, false, false, 0.0f);
    }
    const rm_camera cu = camera.toUniform();

    rm::useShader(marching);  // main.cpp:99-120
    rm::setFloat(marching, "iTime", iTime);
    rm::setuInt(marching, "workgroups", &workgroups);
    rm::setVec4(marching, "camera.pos", cu.pos[0], cu.pos[1], cu.pos[2], 0.0f);
    rm::setVec4(marching, "camera.dir", cu.dir[0], cu.dir[1], cu.dir[2], 0.0f);
    rm::setVec4(marching, "camera.yAxis", cu.yAxis[0], cu.yAxis[1], cu.yAxis[2], 0.0f);
    rm::setVec4(marching, "camera.xAxis", cu.xAxis[0], cu.xAxis[1], cu.xAxis[2], 0.0f);
    rm::setVec3(marching, "light.position", -5, 5, -10);
    rm::setVec3(marching, "light.ambient", 0.03f, 0.04f, 0.1f);
    rm::setVec3(marching, "light.diffuse", 0.8f, 0.8f, 0.8f);
    rm::setVec3(marching, "light.specular", 0.5f, 0.5f, 0.5f);
    rm::setFloat(marching, "light.constant", 1.0f);
    rm::setFloat(marching, "light.linear", 0.009f);
    rm::setFloat(marching, "light.quadratic", 0.00032f);
    rm::setBool(marching, "AA", aa != 0);
    rm::setInt(marching, "bounceVar", bounce);
    rm_uniforms mu{};  // main.cpp:118-119 (accepted, unused by the shader)
    input.toUniforms(&mu);
    rm::setVec3(marching, "mouse", mu.mouse[0], mu.mouse[1], mu.mouse[2]);
    rm::setVec2(marching, "iMouse", mu.iMouse[0], mu.iMouse[1]);
    rm::setInt(marching, "shadow_mode", shadow);

    if (batch > 1) {  // collect this frame's uniforms; dispatch B frames at once
      rm_get_uniforms(marching, &pending[npending++]);
      if (npending == batch && !flush()) return 1;
    } else {
      const int drc = graph ? rm_graph_dispatch(marching) : rm::dispatchCompute(marching);
      if (drc != RM_OK || rm::memoryBarrier(marching) != RM_OK) {
        std::fprintf(stderr, "frame %d failed: %s\n", f, rm_last_error(marching));
        return 1;
      }
    }
    ++counter;
    ++total;
    const double now = std::chrono::duration<double>(clk::now() - t0).count();
    if (now - lastTime >= 1.0) {  // main.cpp:136-143
      std::printf("FPS:\t%u\n", counter);
      ++lastTime;
      counter = 0;
    }
  }
  if (npending && !flush()) return 1;
  const double secs = std::chrono::duration<double>(clk::now() - t0).count();
  std::printf("frames %u  %.3f s  %.2f fps  %.2f Mpixels/s  (%dx%d, bounces %d, AA %d, gpus %d%s)\n",
              total, secs, total / secs, total * (double)W * H / secs / 1e6, W, H, bounce, aa,
              ngpus > 0 ? ngpus : 1, graph ? ", hipGraph" : "");
  if (dump) {
    std::vector<uint8_t> img((size_t)W * H * 4);
    if (rm_read_rgba8(marching, img.data(), 0, /*flip_y=*/1) != RM_OK) {
      std::fprintf(stderr, "readback failed: %s\n", rm_last_error(marching));
      return 1;
    }
    FILE* fp = std::fopen(dump, "wb");
    if (!fp) return 1;
    std::fprintf(fp, "P6\n%d %d\n255\n", W, H);
    for (size_t i = 0; i < (size_t)W * H; ++i) std::fwrite(&img[i * 4], 1, 3, fp);
    std::fclose(fp);
    std::printf("wrote %s\n", dump);
  }
  return 0;
}
