/*
 * rm_api.h — C-ABI of librm, the MI355X-native SDF ray marcher.
 *
 * This is the drop-in boundary that replaces the reference's GL compute
 * program + dispatch (Qirias/OpenGL-RayMarching-in-Compute-Shader):
 *
 *   reference                                   replaced by
 *   ------------------------------------------  ------------------------------------
 *   CreateCompute            shader.hpp:186-197  rm_create (kernels are compiled AOT)
 *   setBool/setInt/setuInt/  shader.hpp:19-69    rm_set_bool/int/uint/float/vec2/3/4
 *   setFloat/setVec2/3/4     (called by name from main.cpp:99-120)
 *   glDispatchCompute        main.cpp:123        rm_dispatch (async, on the ctx stream)
 *   glMemoryBarrier          main.cpp:125        rm_synchronize
 *   Texture::GenerateTexture texture.cpp:10-21   device image owned by rm_ctx
 *   (no readback in the ref; quad draw only)     rm_read_rgba8 / rm_read_rgba32f
 *   Camera ctor/setMouse/lookAt camera.cpp:8-51  rm_camera_* (glm-free, same formulas)
 *
 * Conventions: every entry point returns 0 (RM_OK) on success and a negative
 * RM_ERR_* on failure, with a message available from rm_last_error(ctx).  The
 * one non-error positive code is RM_WARN_UNKNOWN_UNIFORM: like GL's location
 * -1 (shader.hpp:21 glUniform*(-1, ...) is a silent no-op) an unknown uniform
 * name changes nothing, but the caller can see that it happened.
 * No C++ exception crosses this boundary.  One context per host thread (the
 * same constraint as the reference's thread-bound GL context, main.cpp:59).
 * The context owns its device buffers and stream; the caller owns host buffers.
 */
#ifndef RM_API_H
#define RM_API_H

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define RM_API_VERSION 6
#define RM_CONFIG_MAGIC 0x36434D52u /* "RMC6" little-endian: rm_config layout of API version 6 */

/* ---- status codes --------------------------------------------------------- */
#define RM_OK 0
#define RM_WARN_UNKNOWN_UNIFORM 1 /* name not in the uniform block: no-op */
#define RM_ERR_INVALID (-1)       /* bad argument / shape */
#define RM_ERR_HIP (-2)           /* HIP runtime error */
#define RM_ERR_NOMEM (-3)         /* device or host allocation failed */
#define RM_ERR_NO_DEVICE (-4)     /* no HIP device (librm never falls back to CPU) */
#define RM_ERR_STATE (-5)         /* call not valid in this state */
#define RM_ERR_COMM (-6)          /* RCCL error, or a communicator deadline passed (a peer rank
                                     failed, stalled or never joined): the communicator was
                                     aborted; the context reports RM_ERR_COMM from then on and
                                     can only be destroyed (rm_comm_set_timeout) */

/* ---- output image formats (bitmask for rm_config.outputs) ----------------- */
#define RM_OUT_RGBA8 1   /* display format (what the quad shows, Quad.glsl:21-25) */
#define RM_OUT_RGBA32F 2 /* the reference texture's true storage (texture.cpp:19) */

/* ---- RGBA8 shard image formats (rm_config.shard_format, API version 6) ----
 * The reference stores alpha = 1.0 in every pixel (finalColor = vec4(render(),
 * 1.0), and the mean of four such, computeShader.glsl:314-341), so a shard that
 * travels to rank 0 need not carry it: an RGB8 shard image is [rows_cap][width]
 * x 3 bytes (R, G, B), and the un-shard writes alpha 255.  The assembled frame
 * is the same RGBA8 image byte for byte; the gather moves 3/4 of the bytes. */
#define RM_SHARD_AUTO 0  /* RGB8 once the context gathers (rm_comm_init, ngpus), else RGBA8 */
#define RM_SHARD_RGBA8 1 /* 4 B per pixel, the display format */
#define RM_SHARD_RGB8 2  /* 3 B per pixel (sharded contexts only; whole frames stay RGBA8) */

/* ---- shadow modes (rm_uniforms.shadow_mode) ------------------------------- */
#define RM_SHADOW_SOFT 0 /* reference: softshadow(k = 2.0)  computeShader.glsl:185,236 */
#define RM_SHADOW_HARD 1 /* extension: k = +inf -> shadow in {0.05, 1}  (BASELINE cfg 1) */

/* ---- kernel variants (rm_config.kernel) ----------------------------------- */
#define RM_KERNEL_AUTO 0       /* the fastest measured variant: RM_KERNEL_PIXEL */
#define RM_KERNEL_PIXEL 1      /* one thread per pixel, 8x8 pixel tile per wave, culled sdf */

/* Uniform block of computeShader.glsl:7,59-66.  vec4s carry w = 0
 * (main.cpp:103-106).  Layout is plain C, not std140. */
typedef struct rm_camera {
  float pos[4];   /* camera.pos    glsl:16 */
  float dir[4];   /* camera.dir    glsl:17 (forward) */
  float yAxis[4]; /* camera.yAxis  glsl:18 (up) */
  float xAxis[4]; /* camera.xAxis  glsl:19 (right) */
} rm_camera;

typedef struct rm_light { /* glsl:22-32 */
  float position[3];
  float ambient[3];
  float diffuse[3];
  float specular[3];
  float constant;
  float linear;
  float quadratic;
} rm_light;

typedef struct rm_uniforms {
  rm_camera camera;     /* glsl:65 */
  rm_light light;       /* glsl:66 */
  float iTime;          /* glsl:62  drives the box/sphere blend, sin(iTime)/2+0.5 (glsl:117) */
  int32_t bounceVar;    /* glsl:60  0..5 (main.cpp:199-204) */
  int32_t AA;           /* glsl:59  4x supersampling on/off */
  uint32_t workgroups;  /* glsl:7   launch geometry only; ignored (librm picks its own) */
  float drand48;        /* glsl:61  unused by the shader; accepted and ignored */
  float mouse[3];       /* glsl:63  unused by the shader; accepted and ignored */
  float iMouse[2];      /* glsl:64  unused by the shader; accepted and ignored */
  int32_t shadow_mode;  /* extension: RM_SHADOW_SOFT (reference) or RM_SHADOW_HARD */
} rm_uniforms;

/* Work counters, in the reference's units (calls as written in the GLSL). */
typedef struct rm_counters {
  uint64_t rays;          /* castRay calls                       glsl:68 */
  uint64_t march_steps;   /* sdf() calls inside RayMarch         glsl:131-139 */
  uint64_t reflect_steps; /* sdf() calls inside reflectedRay     glsl:150-158 */
  uint64_t shadow_steps;  /* sdf() calls inside softshadow       glsl:205-213 */
  uint64_t normals;       /* GetNormal calls (4 sdf each)        glsl:278-288 */
  uint64_t lights;        /* getPointLight calls                 glsl:253-276 */
  uint64_t sdf_evals;     /* march + reflect + shadow + 4*normals */
} rm_counters;

typedef struct rm_config {
  /* sizeof(rm_config) and RM_CONFIG_MAGIC (rm_config_init sets both).  rm_create
   * refuses a config where either differs (RM_ERR_INVALID) instead of reading
   * a stale layout: a v1/v2 host's first two words are width and height, a v3
   * host's second word is its width (<= 65536), and none of them can equal the
   * magic, whatever the struct sizes happen to be (a v3 struct has
   * the same size as this one on LP64). */
  uint32_t struct_size;
  uint32_t magic;
  int32_t width;      /* image width  (SCREEN_WIDTH,  main.cpp:16) */
  int32_t height;     /* image height (SCREEN_HEIGHT, main.cpp:17) */
  int32_t device;     /* HIP device ordinal; -1 = current device */
  int32_t outputs;    /* RM_OUT_* bitmask; 0 = RM_OUT_RGBA8 */
  int32_t kernel;     /* RM_KERNEL_*; 0 = auto */
  int32_t counters;   /* nonzero: collect rm_counters + per-pixel sdf counts (slower) */
  /* Row sharding (multi-GPU): the image's rows are cut into
   * rounds; a round holds rank0_rows rows of shard 0, then row_block rows of
   * shard 1, 2, ..., nshards-1 (rank0_rows = row_block: block b belongs to
   * shard b % nshards).  This context renders only shard `shard`'s rows, packed
   * in round order, into a [rows_cap][width] image (rows_cap = rm_shard_rows()).
   * nshards <= 1 means the whole image. */
  int32_t row_block;
  int32_t shard;
  int32_t nshards;
  /* Rows of shard 0 per round (API version 5); 0 = row_block.  Shard 0 is the
   * rank that assembles every gathered frame (k_unshard), so fewer rows for it
   * balance its render + assembly against the other ranks' render
   * (rm_shard_rows; bench.py --rank0-share). */
  int32_t rank0_rows;
  /* RM_SHARD_* (API version 6): the layout of this context's RGBA8 shard images
   * (its own, a caller's rm_set_output_rgba8 buffer, the batch ring, rank 0's
   * gather buffer) and of the gathered input of rm_unshard_rgba8 /
   * rm_unshard_batch_rgba8.  rm_read_rgba8 / rm_read_frame_rgba8 of an RGB8 shard
   * return RGBA8 (alpha 255; the padding rows too).  Ignored unless sharded. */
  int32_t shard_format;
  /* Multi-GPU frames in one process.  ngpus >= 1 makes the
   * context drive ngpus devices: devices[0..ngpus), or device, device+1, ...
   * when devices is NULL (device -1 = the current device).  Device i renders
   * shard i of the interleaved row blocks (row_block rows per block, 0 = 8);
   * ncclGather over a single-process communicator (ncclCommInitRankConfig per device in one group) collects
   * the shards on devices[0], which assembles the frame (k_unshard).  The
   * setters, rm_dispatch, rm_synchronize, rm_read_rgba8, rm_set_scene and the
   * graph calls work as on a one-GPU context; the frame lives on devices[0].
   * RGBA8 and/or RGBA32F outputs, no counters, shard/nshards must be 0.
   * ngpus = 0: one device, no RCCL (API version 1 behaviour). */
  int32_t ngpus;
  const int32_t *devices;
} rm_config;

typedef struct rm_ctx rm_ctx;

/* ---- lifetime ------------------------------------------------------------- */
/* Zero-fills *cfg and sets struct_size, width, height, device = -1 (current),
 * outputs = RM_OUT_RGBA8, nshards = 1: a one-GPU context with the defaults. */
int rm_config_init(rm_config *cfg, int32_t width, int32_t height);
int rm_create(rm_ctx **out, const rm_config *cfg);
void rm_destroy(rm_ctx *ctx);
const char *rm_last_error(const rm_ctx *ctx);
int rm_api_version(void);
int rm_device_count(int *count);

/* ---- uniforms: by-name setters mirroring shader.hpp:19-69 ------------------
 * Names are the GLSL ones: "iTime", "workgroups", "AA", "bounceVar",
 * "drand48", "mouse", "iMouse", "camera.pos", "camera.dir", "camera.yAxis",
 * "camera.xAxis", "light.position", "light.ambient", "light.diffuse",
 * "light.specular", "light.constant", "light.linear", "light.quadratic",
 * plus the extension "shadow_mode". */
int rm_set_bool(rm_ctx *ctx, const char *name, int value);
int rm_set_int(rm_ctx *ctx, const char *name, int32_t value);
int rm_set_uint(rm_ctx *ctx, const char *name, const uint32_t *value);
int rm_set_float(rm_ctx *ctx, const char *name, float value);
int rm_set_vec2(rm_ctx *ctx, const char *name, float x, float y);
int rm_set_vec3(rm_ctx *ctx, const char *name, float x, float y, float z);
int rm_set_vec4(rm_ctx *ctx, const char *name, float x, float y, float z, float w);
int rm_set_uniforms(rm_ctx *ctx, const rm_uniforms *u);
int rm_get_uniforms(const rm_ctx *ctx, rm_uniforms *u);

/* Defaults of main.cpp:100-120 for the lights/flags and the reference's
 * start-up camera (pos 0, looking down -z): AA on, bounceVar 0, soft shadow. */
int rm_default_uniforms(rm_uniforms *u);

/* ---- dispatch / barrier / readback --------------------------------------- */
/* Render one frame with the current uniforms. Asynchronous on the context's
 * stream (== glDispatchCompute, main.cpp:123). */
int rm_dispatch(rm_ctx *ctx);
/* Render frames[0..n) (API version 4), n <= RM_MAX_BATCH: the same images as
 * rm_set_uniforms(frames[k]) + rm_dispatch for k = 0..n-1, in one launch.  The
 * frames of a batch render concurrently, so the waves of frame k+1 fill the
 * SIMDs that frame k's longest waves leave idle (one tail per batch instead of
 * one per frame).  Asynchronous on the context's stream.  Afterwards the
 * context's uniforms are frames[n-1], its image (rm_read_rgba8 / _rgba32f,
 * rm_get_output_rgba8) holds frame n-1, and rm_read_frame_rgba8 /
 * rm_read_frame_rgba32f read any frame k of the batch (frames 0..n-2 live in a
 * ring the context allocates, n-1 images of each enabled format).  On a
 * communicator context (rm_comm_init, rm_config.ngpus) every rank renders its
 * shards of the n frames in one launch, one ncclGather moves all n shards, and
 * rank 0 assembles the n frames; the gather runs on a second stream of the
 * context, so the next batch renders while this one gathers (a consumer on the
 * caller's own stream orders itself after it with rm_wait_output).  A runtime
 * scene table's frames batch the same way (API version 5; its specialised
 * kernels too).  Frames with a different AA setting, or (specialised tables) a
 * camera that needs the generic kernel, render in separate launches.  Not
 * available with cfg.counters.  Every frame's uniforms are checked before any
 * launch; a batch that still fails (a HIP or RCCL error part way) leaves the
 * context's uniforms as before the call, and its image and ring hold
 * undefined contents until the next successful dispatch. */
#define RM_MAX_BATCH 32
int rm_dispatch_frames(rm_ctx *ctx, const rm_uniforms *frames, int32_t n);
/* Wait for all work queued on the context (== glMemoryBarrier + the
 * implicit sync of the draw, main.cpp:125-134).  On a context with a
 * communicator this wait (and the one inside every readback) is a bounded
 * poll of the stream and of the communicator's asynchronous error: an RCCL
 * error or the deadline aborts the communicator and returns RM_ERR_COMM. */
int rm_synchronize(rm_ctx *ctx);
/* Synchronous readback. Row 0 of the image is the bottom row (py = 0,
 * quad.hpp:9); flip_y != 0 writes the top row first (image-file order).
 * row_pitch is in bytes; 0 = tightly packed. For a sharded context the
 * packed [rows_cap][width] shard image is read (flip_y must be 0). */
int rm_read_rgba8(rm_ctx *ctx, uint8_t *dst, size_t row_pitch, int flip_y);
int rm_read_rgba32f(rm_ctx *ctx, float *dst, size_t row_pitch, int flip_y);
/* Frame k of the last rm_dispatch_frames batch (k = n-1 is the context's image;
 * after a plain rm_dispatch only k = 0 exists).  Same layout rules as above. */
int rm_read_frame_rgba8(rm_ctx *ctx, int32_t k, uint8_t *dst, size_t row_pitch, int flip_y);
int rm_read_frame_rgba32f(rm_ctx *ctx, int32_t k, float *dst, size_t row_pitch, int flip_y);
/* Counters of the last dispatch (requires cfg.counters). */
int rm_get_counters(rm_ctx *ctx, rm_counters *out);
/* Per-pixel sdf() evaluation counts of the last dispatch, summed over the
 * pixel's samples, reference units (requires cfg.counters). */
int rm_read_sdf_counts(rm_ctx *ctx, uint32_t *dst);

/* ---- hipGraph frame replay (BASELINE cfg 5) ------------------------------ */
/* rm_graph_enable(ctx, 1) switches the context to graph replay: the first
 * rm_graph_dispatch captures the render-kernel launch into a graph; every
 * later rm_graph_dispatch writes the current frame constants into the kernel
 * node's by-value argument (hipGraphExecKernelNodeSetParams) and replays the
 * graph on the context's stream (re-captured only when AA toggles, which
 * changes the grid and kernel).  Same kernel and image as rm_dispatch.
 * Not available with cfg.counters. */
int rm_graph_enable(rm_ctx *ctx, int enable);
int rm_graph_dispatch(rm_ctx *ctx);

/* ---- runtime scene table ------------------------------
 * The reference's scene is the hard-coded sdf() of computeShader.glsl:107-123:
 * an opU chain of primitives, each a RayHit {distance, colour, id, material}.
 * rm_set_scene replaces it with a table of up to RM_MAX_PRIMITIVES such
 * entries, evaluated in table order with the same opU rule (a later entry wins
 * unless the running distance is strictly smaller, glsl:105).  The table is
 * staged in LDS by every workgroup of the table kernel.  rm_default_scene
 * returns the reference's scene as a table; rendered through the table kernel
 * it gives the same image as the built-in scene's specialised kernel.
 * The shading rules stay the reference's: id 7 takes the floor branch
 * (shadow, no bounce; glsl:240-247, 177) and material 0 (MATTE) stops the
 * bounce colour accumulation (glsl:189-190). */
#define RM_MAX_PRIMITIVES 32
#define RM_PRIM_SPHERE 0  /* sdSphere(q, r)                               glsl:83 */
#define RM_PRIM_BOX 1     /* sdBox(q, b)                                  glsl:87-91 */
#define RM_PRIM_BLEND 2   /* mix(sdBox(q, b), sdSphere(q, r), sin(iTime)/2 + 0.5)  glsl:115-117 */
#define RM_PRIM_TORUS 3   /* sdTorus(q, (R, r))                           glsl:93-96 */
#define RM_PRIM_CAPSULE 4 /* sdCapsule(q, a, b, r)                        glsl:98-103 */
#define RM_PRIM_PLANE 5   /* sdPlane(q, (nx, ny, nz, w))                  glsl:85 */
#define RM_SWIZZLE_XYZ 0  /* q = p - center */
#define RM_SWIZZLE_XZY 1  /* q = (p - center).xzy  (the torus of glsl:119) */
#define RM_PAINT_SOLID 0    /* RayHit.color = color */
#define RM_PAINT_CHECKERS 1 /* RayHit.color = checkers(p)                 glsl:77-80 */

typedef struct rm_primitive {
  int32_t type;    /* RM_PRIM_* */
  int32_t swizzle; /* RM_SWIZZLE_* */
  int32_t id;      /* RayHit.id (glsl:42) */
  int32_t paint;   /* RM_PAINT_* */
  float material;  /* RayHit.material: 1 REFLECTIVE, 0 MATTE (glsl:4-5) */
  float color[3];
  float center[3];
  /* sphere {r}; box {bx, by, bz}; blend {bx, by, bz, r}; torus {R, r};
   * capsule {ax, ay, az, bx, by, bz, r}; plane {nx, ny, nz, w} */
  float param[7];
} rm_primitive;

/* The reference scene (glsl:107-123) as 6 table entries (the blended box and
 * sphere of glsl:115-117 are one RM_PRIM_BLEND entry, id 4).  *n = 6. */
int rm_default_scene(rm_primitive *out, int32_t capacity, int32_t *n);
/* Render with `prims[0..n)` from the next dispatch on.  prims == NULL and
 * n == 0 return to the built-in scene (the specialised kernel). */
int rm_set_scene(rm_ctx *ctx, const rm_primitive *prims, int32_t n);
/* The table in use (*n = 0: the built-in scene). */
int rm_get_scene(const rm_ctx *ctx, rm_primitive *out, int32_t capacity, int32_t *n);
/* enable != 0: tables render with kernels compiled for the table itself
 * (hiprtc, at this call for the current table and at every later
 * rm_set_scene; the analogue of the reference compiling its shader at run time,
 * CreateCompute shader.hpp:186-197).  Same image as the generic table kernel;
 * compiles are cached per process and device.  A failed compile returns
 * RM_ERR_HIP with the compiler log in rm_last_error and leaves the scene as it
 * was.  A frame whose camera lies farther than 1e15 from the origin (or is not
 * finite) renders with the generic kernel: the specialised kernels take an
 * exact short form of sqrt(x) - R that needs bounded march points.
 * enable == 0: the generic (LDS-staged) table kernel. */
int rm_scene_specialize(rm_ctx *ctx, int enable);
/* The register bound of the specialised table kernels in use: *waves = the
 * waves per SIMD they were compiled for (8, 7 or 6: the most at which they need
 * no scratch), or 0 when the generic table kernel (or the built-in scene)
 * renders; a table that spills at 6 waves is not specialised, and neither is
 * one of more than 12 entries (not compiled at all: past a dozen entries the
 * compile takes minutes and fits no bound). */
int rm_scene_kernel_waves(const rm_ctx *ctx, int32_t *waves);
/* Diagnostics (API version 5): the table as rm_set_scene compiles it on the host
 * for the device (no device needed): the n entries' words, then the exit header
 * with the bounds of the provable exits and the culling balls.  *nwords = its
 * length; words == NULL queries the length only.  RM_ERR_INVALID (with the
 * reason in rm_last_error(NULL)) for a table rm_set_scene would refuse. */
int rm_scene_compile(const rm_primitive *prims, int32_t n, uint32_t *words, size_t capacity, size_t *nwords);
/* Diagnostics: the code object rm_scene_specialize would load for this table
 * on `arch` (e.g. "gfx950"), compiled without a device.  *size = its size;
 * out == NULL queries the size only; *size = 0: the table is not specialised
 * (see rm_scene_kernel_waves). */
int rm_jit_code_object(const rm_primitive *prims, int32_t n, const char *arch, void *out,
                       size_t capacity, size_t *size);

/* ---- device-side interop (plain pointers; for stream/collective plumbing) - */
/* Use an external stream (hipStream_t passed as void*); NULL = own stream. */
int rm_set_stream(rm_ctx *ctx, void *hip_stream);
/* Render RGBA8 into a caller-owned device buffer of >= rows*width*4 bytes
 * (rows = height, or rows_cap when sharded) instead of the context's own.
 * A sharded context with RGB8 shards writes rows of width*3 bytes there.
 * NULL restores the internal buffer. */
int rm_set_output_rgba8(rm_ctx *ctx, void *device_ptr);
/* Device pointer of the RGBA8 image the next dispatch writes (a shard of an
 * RGB8 context: packed rows of width*3 bytes, rm_config.shard_format). */
int rm_get_output_rgba8(rm_ctx *ctx, void **device_ptr);
/* Orders `hip_stream` (hipStream_t as void*; NULL = the null stream) after every
 * write to the context's images queued so far: work the caller enqueues on it
 * afterwards sees the last dispatch's frames (API version 5).  Needed on a
 * communicator context (rm_comm_init, rm_config.ngpus): a batch's gather and
 * rank 0's assembly run on the context's internal gather stream, so frame n-1
 * in rm_get_output_rgba8 / rm_set_output_rgba8's buffer (and the batch's ring)
 * is not ordered by rm_set_stream's stream alone.  rm_synchronize and the
 * readbacks wait for it as well.  Asynchronous: records events, waits on none. */
int rm_wait_output(rm_ctx *ctx, void *hip_stream);
/* Assemble a full image from nshards packed shard images laid out
 * back-to-back ([nshards][rows_cap][width] RGBA8, e.g. the result of an RCCL
 * gather; RGB8, 3 B per pixel, when the context's shard_format is RGB8) into
 * `frame` ([height][width] RGBA8), both device pointers, on the context's
 * stream. Uses the context's width/height/row_block/rank0_rows/nshards and
 * shard format. */
int rm_unshard_rgba8(rm_ctx *ctx, const void *gathered_dev, void *frame_dev);
/* The same for frame k of an n-frame batch gathered as rm_dispatch_frames
 * gathers it: [nshards][n][rows_cap][width] RGBA8 or RGB8 (each rank's n shards
 * back to back, ranks in order), e.g. by a host that moves the shards itself. */
int rm_unshard_batch_rgba8(rm_ctx *ctx, const void *gathered_dev, int32_t k, int32_t n, void *frame_dev);
/* Kernel timing: when enabled, HIP events bracket every render-kernel launch
 * on the launch stream; rm_kernel_time_ms returns the summed kernel time and
 * launch count since the last reset (synchronizes). */
int rm_enable_timing(rm_ctx *ctx, int enable);
int rm_kernel_time_ms(rm_ctx *ctx, double *total_ms, int64_t *launches, int reset);
/* Phases of the last rm_dispatch issued with timing enabled (synchronizes):
 * the render kernel, then on a communicator context the gather (render end to
 * gather end on this rank's stream, so it includes waiting for the slowest
 * peer's shard) and rank 0's assembly (0 elsewhere).  A multi-GPU context
 * reports device 0.  RM_ERR_STATE before such a dispatch. */
int rm_frame_phases(rm_ctx *ctx, double *render_ms, double *gather_ms, double *assemble_ms);

/* ---- one rank per process: RCCL-gathered frames -------------
 * The multi-process form of rm_config.ngpus, for hosts that run one process
 * per GPU (torch.distributed.run, MPI).  Rank 0 creates an id and broadcasts it
 * over the host's own channel; every rank then joins its sharded context
 * (cfg.nshards = nranks, cfg.shard = rank) to the communicator
 * (ncclCommInitRank: collective, every rank must call it).  From then on
 * rm_dispatch renders this rank's shard, gathers all shards on rank 0
 * (ncclGather into rank 0's [nranks][rows_cap][width] buffer; rank 0 renders
 * its own shard in place) and, on rank 0, assembles the frame (k_unshard), all
 * on the context's stream.  Rank 0's rm_read_rgba8 / rm_read_rgba32f /
 * rm_get_output_rgba8 / rm_set_output_rgba8 then refer to the full height x
 * width frame, the other ranks' to their packed shard; an output buffer set on
 * rank 0 before rm_comm_init (shard-sized) is dropped, so set or re-query output
 * pointers after it.  rm_dispatch and rm_graph_dispatch are collective: every
 * rank issues the same sequence.  rm_graph_dispatch captures render + gather +
 * assembly into one hipGraph per rank (cfg 5).  RGBA8 and/or RGBA32F (16 B/px
 * shards gathered as ncclFloat32), no counters.
 *
 * Failure detection: communicators are non-blocking; rm_comm_init, and every
 * wait on the context afterwards, polls progress and ncclCommGetAsyncError
 * against a deadline (rm_comm_set_timeout; default 120000 ms or the
 * RM_COMM_TIMEOUT_MS environment variable; 0 = none).  A rank that never
 * joins, an RCCL error or a frame that misses the deadline aborts the
 * communicator (ncclCommAbort) and returns RM_ERR_COMM with the reason in
 * rm_last_error; the process and its other contexts stay usable. */
#define RM_COMM_ID_BYTES 128 /* == NCCL_UNIQUE_ID_BYTES */
int rm_comm_unique_id(void *id, size_t size);
int rm_comm_init(rm_ctx *ctx, const void *id, int32_t nranks, int32_t rank);
/* Deadline in ms of rm_comm_init and of every later wait on the context. */
int rm_comm_set_timeout(rm_ctx *ctx, int32_t timeout_ms);
/* Non-blocking health check: RM_OK, or RM_ERR_COMM when the communicator has
 * an asynchronous error (it is then aborted) or was aborted before. */
int rm_comm_check(rm_ctx *ctx);
/* The context's communicator: rank / size (0 / 1 without one), and the devices
 * a multi-GPU context drives (*ngpus = 1 for a one-GPU context). */
int rm_comm_info(const rm_ctx *ctx, int32_t *rank, int32_t *nranks, int32_t *ngpus);
/* What RCCL itself reports for the context's communicator (API version 4):
 * ncclCommCount, ncclCommUserRank and ncclCommCuDevice of the communicator
 * (device 0's for a multi-GPU context, whose every device is checked to be user
 * rank i of ngpus on its own device) and ncclGetVersion.  RM_ERR_COMM when RCCL's
 * view differs from the context's (rank, nranks, device).  Without a
 * communicator: *count = 0, *user_rank = *hip_device = -1, *version = 0.  Any
 * pointer may be NULL. */
int rm_comm_rccl_info(rm_ctx *ctx, int32_t *count, int32_t *user_rank, int32_t *hip_device,
                      int32_t *version);

/* ---- row sharding helpers (pure functions) ------------------------------- */
/* The weighted interleave (API version 5).  Rows go in rounds of
 * P = rank0_rows + (nshards - 1) row_block rows: shard 0 owns rows
 * [kP, kP + rank0_rows) of round k, shard s >= 1 the row_block rows after
 * rank0_rows + (s - 1) row_block.  Shard s's rows are packed in round order into
 * a [rows_cap][width] image; rows_cap (the same for every shard, so one
 * ncclGather moves them) is the largest shard's rounds times its rows per round,
 * and *rows is shard s's own count of real rows.  rank0_rows = 0 means
 * row_block (the plain interleave: block b belongs to shard b % nshards).
 * nshards <= 1: the whole image (rows = rows_cap = height).
 * Every function below takes (height, row_block, rank0_rows, nshards, ...) in
 * this order (API version 6; version 5's rm_shard_row took shard before nshards,
 * and version 1's rm_shard_rows_cap / rm_shard_global_row knew only the plain
 * interleave: all three are gone, so a stale caller fails to bind instead of
 * reading the wrong rows). */
int rm_shard_rows(int32_t height, int32_t row_block, int32_t rank0_rows, int32_t nshards, int32_t shard,
                  int32_t *rows, int32_t *rows_cap);
/* Global row (py) of local row `local_row` of shard `shard`; -1 if padding or
 * out of range (including invalid arguments). */
int32_t rm_shard_to_global(int32_t height, int32_t row_block, int32_t rank0_rows, int32_t nshards, int32_t shard,
                           int32_t local_row);
/* The inverse: the shard and local row that own global row `row`. */
int rm_shard_owner(int32_t height, int32_t row_block, int32_t rank0_rows, int32_t nshards, int32_t row,
                   int32_t *shard, int32_t *local_row);

/* ---- Camera (source/camera.{hpp,cpp}), glm-free, same formulas ----------- */
typedef struct rm_camera_state { /* members of camera.hpp:14-27 */
  int32_t width, height;
  float angleY, angleX;
  float mouseSensitivity, keyboardSpeed;
  float xpos, ypos;
  float cameraPos[3];
  float forward[3];
  float up[3];
  float right[3];
} rm_camera_state;

/* Camera::Camera(w,h,sens,speed,pos,lookAt,up)  camera.cpp:8-14 */
int rm_camera_init(rm_camera_state *c, int32_t width, int32_t height, float mouseSensitivity,
                   float keyboardSpeed, const float pos[3], const float lookAt[3],
                   const float up[3]);
/* Camera::setMouse                              camera.cpp:16-20 */
int rm_camera_set_mouse(rm_camera_state *c, float x, float y);
/* Camera::lookAt                                camera.cpp:22-51 */
int rm_camera_look_at(rm_camera_state *c, int zN, int zP, int xN, int xP, int halfSpeed,
                      float deltaTime);
/* The four setVec4 calls of main.cpp:103-106 (w = 0). */
int rm_camera_to_uniform(const rm_camera_state *c, rm_camera *out);

/* ---- interactive input mapping ------------------------
 * The reference's GLFW input globals and callbacks (main.cpp:20-39, 93-95,
 * 155-234; source/MousePosition.cpp:4-22) as a state struct and four event
 * functions, so any windowing front-end can feed its key/mouse events and get
 * the reference's camera motion, bounce/AA toggles and uniforms.  Key and
 * action codes are GLFW's (glfw3.h) so a GLFW front-end passes them through. */
#define RM_KEY_A 65
#define RM_KEY_D 68
#define RM_KEY_L 76
#define RM_KEY_S 83
#define RM_KEY_W 87
#define RM_KEY_ESCAPE 256
#define RM_KEY_DOWN 264
#define RM_KEY_UP 265
#define RM_KEY_F1 290
#define RM_RELEASE 0
#define RM_PRESS 1
#define RM_REPEAT 2
/* keys held this frame (glfwGetKey(...) == GLFW_PRESS), for rm_input_process */
#define RM_HELD_W 1u
#define RM_HELD_A 2u
#define RM_HELD_S 4u
#define RM_HELD_D 8u
#define RM_HELD_ESCAPE 16u

typedef struct rm_input_state {
  int32_t zaxisPos, zaxisNeg, xaxisPos, xaxisNeg; /* main.cpp:23-26 */
  int32_t AA;                                     /* main.cpp:27 (true) */
  int32_t showQuad;                               /* main.cpp:28 wireframe toggle (display only) */
  float halfSpeed;                                /* main.cpp:29 (a float in the reference) */
  int32_t bounce;                                 /* main.cpp:30, 0..5 */
  float deltaTime, lastFrame;                     /* main.cpp:32-33 */
  float lastX, lastY;                             /* main.cpp:35-36 (screen centre) */
  int32_t firstMouse;                             /* main.cpp:37 */
  float pitch, yaw;                               /* MouseInput mouse, main.cpp:39 */
  float mouseSensitivity;                         /* MouseSensitivity, MousePosition.hpp:8 */
  int32_t shouldClose;                            /* glfwSetWindowShouldClose (main.cpp:157) */
} rm_input_state;

/* The globals' initial values for a screen_width x screen_height window. */
int rm_input_init(rm_input_state *s, int32_t screen_width, int32_t screen_height);
/* main.cpp:93-95: currentFrame = (float)now; deltaTime = currentFrame - lastFrame. */
int rm_input_begin_frame(rm_input_state *s, double now_seconds);
/* processInput  main.cpp:155-195: axis flags and halfSpeed from the held keys
 * (RM_HELD_*), ESC -> shouldClose, then camera.lookAt(..., deltaTime). */
int rm_input_process(rm_input_state *s, uint32_t held, rm_camera_state *cam);
/* key_callback  main.cpp:197-217: UP/DOWN bounce within 0..5, F1 toggles AA,
 * L toggles showQuad; only RM_PRESS acts (repeats are ignored). */
int rm_input_key(rm_input_state *s, int32_t key, int32_t action);
/* mouse_callback  main.cpp:219-234: MouseInput offsets, camera.setMouse(-x, -y). */
int rm_input_mouse(rm_input_state *s, double xpos, double ypos, rm_camera_state *cam);
/* MouseInput::EulerAngles  MousePosition.cpp:24-33 (the "mouse" uniform). */
int rm_input_euler_angles(const rm_input_state *s, float out[3]);
/* The per-frame uploads of main.cpp:101-120 that input drives: camera block,
 * AA, bounceVar, mouse = EulerAngles(), iMouse = (yaw, pitch), and
 * iTime = the frame's clock sample (lastFrame).  Other fields are untouched. */
int rm_input_to_uniforms(const rm_input_state *s, const rm_camera_state *cam, rm_uniforms *u);

/* ---- synthetic frames -------------------------------------- */
/* Sweep S(F): camera at (0,0,15), yaw -20..+20 deg over F frames, pitch -5 deg,
 * iTime = f/60; lights of main.cpp:108-114. frame < 0 selects the default
 * frame D (start-up view: pos 0, yaw = pitch = 0, iTime = 0). */
int rm_sweep_uniforms(int32_t frame, int32_t nframes, int32_t bounceVar, int32_t AA,
                      int32_t shadow_mode, rm_uniforms *out);

#ifdef __cplusplus
}
#endif

#endif /* RM_API_H */
