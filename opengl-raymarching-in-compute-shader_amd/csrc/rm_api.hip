// rm_api.hip — librm's C-ABI: context, uniforms, dispatch, readback, timing.
//
// Replaces the reference's GL program + dispatch (see include/rm_api.h for the
// call-by-call mapping).  There is no CPU backend: without a HIP device
// rm_create fails with RM_ERR_NO_DEVICE — librm never falls back to the CPU.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "rm_comm.hpp"
#include "rm_internal.hpp"
#include "rm_jit.hpp"
#include "rm_scene.hpp"

namespace rm {
void pixel_grid(int width, int rows, bool aa, int32_t* gx, int32_t* gy);
hipError_t launch_pixel(const rmd::Frame& F, bool counters, hipStream_t s);
hipError_t launch_table(const rmd::Frame& F, bool counters, hipStream_t s, int nslots, int shape);
hipError_t launch_table_frames(const rmd::FrameBatch& B, int n, hipStream_t s, int nslots, int shape);
int table_shape(const uint32_t* words, int32_t n);
hipError_t launch_unshard(const void* gathered, void* frame, int width, int height, int row_block,
                          int row_block0, int nshards, int rows_cap, hipStream_t s, size_t rank_stride_rows = 0,
                          bool rgb3 = false);
hipError_t launch_frames(const rmd::FrameBatch& B, int n, hipStream_t s);
}  // namespace rm
static_assert(RM_MAX_BATCH == rmd::kMaxBatch, "rm_api.h RM_MAX_BATCH == rm_scene.hpp kMaxBatch");

// The graph path: the captured frame (the render kernel, and for a rank of an
// RCCL-gathered frame the gather and the assembly after it) whose render node
// gets the frame's by-value constants per replay (hipGraphExecKernelNodeSetParams).
struct rm_graph_slot {
  hipGraph_t graph = nullptr;
  hipGraphNode_t render = nullptr;  // the render kernel's node (its argument is a Frame)
  hipGraphExec_t exec = nullptr;
  const void* send = nullptr;       // buffers the captured gather / assembly use
  const void* frame = nullptr;
};

struct rm_ctx {
  rm_config cfg{};
  int device = 0;
  int rows = 0;  // rows rendered per dispatch (height, or the shard's rows_cap)
  rm_uniforms u{};
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint8_t* d_rgba8 = nullptr;     // own RGBA8 image
  uint8_t* ext_rgba8 = nullptr;   // caller-provided RGBA8 image (rm_set_output_rgba8)
  // the RGBA8 shard images are packed RGB, 3 B per pixel (rm_config.shard_format:
  // RGB8, or AUTO once the context gathers): the render writes them, the gather
  // moves them, k_unshard expands them with alpha 255
  bool rgb3 = false;
  float* d_rgba32f = nullptr;
  uint32_t* d_counts = nullptr;
  unsigned long long* d_counters = nullptr;
  float* d_uv = nullptr;          // per-column / per-row uv table (Frame::uvx / uvy)
  bool uv_exact = false;          // lane_uv's arithmetic equals the table (uv_exact_check)
  float uv_lo[2] = {0, 0}, uv_hi[2] = {0, 0};  // range of the table's column / row values
  uint32_t* d_scene = nullptr;    // runtime scene table (rm_set_scene), compiled words
  int nprims = 0;                 // 0: the built-in scene and its specialised kernel
  std::vector<rm_primitive> scene;     // the table as given (rm_get_scene)
  std::vector<uint32_t> scene_words;   // host copy of d_scene (source of the async upload)
  bool specialize = false;             // rm_scene_specialize: tables render with hiprtc kernels
  const rm::JitTable* jit = nullptr;   // the current table's specialised kernels, or null
  bool dispatched = false;
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  std::vector<int> ev_frames;  // frames each timed launch rendered (a batch: n)
  size_t ev_used = 0;
  double total_ms = 0.0;
  int64_t launches = 0;
  bool graph_on = false;
  int graph_aa = -1;  // AA value the graphs were captured for (grid shape depends on it)
  int graph_table = -1;  // the kernel the graph holds: built-in (0), generic table kernel (1 + its slot instance)
  const rm::JitTable* graph_jit = nullptr;  // the specialised table kernels captured, if any
  rm_graph_slot gs;
  // RCCL-gathered frames (rm_comm_init, or one device of a multi-GPU context)
  ncclComm_t comm = nullptr;
  bool own_comm = false;      // destroyed with the context
  bool group_member = false;  // a device of a multi-GPU context: its parent issues the gather
  bool comm_warm = false;     // a gather has run eagerly (before any graph capture)
  int crank = 0, cranks = 1;
  uint8_t* d_gathered = nullptr;  // rank 0: [cranks][rows][width] RGBA8; its own shard renders into slot 0
  uint8_t* d_frame = nullptr;     // rank 0: the assembled [height][width] frame
  float* d_gathered32 = nullptr;  // the same two for RGBA32F (16 B/px)
  float* d_frame32 = nullptr;
  long comm_timeout_ms = 0;       // deadline of every wait on the communicator (0: none)
  bool comm_failed = false;       // the communicator was aborted (RM_ERR_COMM from then on)
  std::string comm_why;           // why it was aborted
  // phase events of the last timed eager dispatch: render start / end, gather end, assembly end
  hipEvent_t ph[4] = {nullptr, nullptr, nullptr, nullptr};
  bool ph_recorded = false, ph_comm = false;
  // frame batches (rm_dispatch_frames)
  int batch_n = 1;                  // frames of the last dispatch (a plain dispatch: 1)
  std::vector<uint8_t*> ring8;      // frames 0..n-2 of the last batch (rank 0 of a communicator: assembled)
  std::vector<float*> ring32;
  // communicator contexts: two batch slots, so batch j + 1 renders while batch j
  // gathers on gstream.  A slot's send8 / send32 hold this rank's shards of the
  // batch's frames, [n][rows][width]; rank 0's is the whole gather buffer,
  // [nranks][n][rows][width], its own shards rendering in place into [0].
  struct BatchSlot {
    uint8_t* send8 = nullptr;
    float* send32 = nullptr;
    int cap = 0;                   // frames the buffers hold
    hipEvent_t rendered = nullptr; // the batch's render, on stream
    hipEvent_t freed = nullptr;    // its gather and assembly, on gstream
    bool pending = false;          // freed recorded and not yet waited for
  } bslot[2];
  int bnext = 0, blast = -1;        // the next slot; the slot of the last batch
  hipStream_t gstream = nullptr;    // gathers + assembly of batches
  hipEvent_t gdone = nullptr;       // the last batch's work on gstream
  hipEvent_t out_ev = nullptr;      // rm_wait_output: the tail of the context's stream
  bool gdone_pending = false;       // plain dispatches order after it
  // a multi-GPU context (rm_config.ngpus): one shard context per device, subs[0] = rank 0
  std::vector<rm_ctx*> subs;
  std::string err;
};

namespace {

thread_local std::string g_create_error;

int fail(rm_ctx* c, int code, const std::string& msg) {
  if (c)
    c->err = msg;
  else
    g_create_error = msg;
  return code;
}

int hip_fail(rm_ctx* c, hipError_t e, const char* what) {
  return fail(c, RM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define RM_HIP(c, call)                              \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return hip_fail(c, e_, #call); \
  } while (0)

int set_device(rm_ctx* c) {
  RM_HIP(c, hipSetDevice(c->device));
  return RM_OK;
}

// ---- where images live --------------------------------------------------------------
// A plain context renders into its RGBA8 image (the caller's, or its own).  Rank 0
// of an RCCL-gathered frame renders its shard into slot 0 of the gather buffer and
// its readable image is the assembled frame; the other ranks' is their shard.
bool comm_root(const rm_ctx* c) { return c->comm && c->crank == 0; }
uint8_t* render_dst(const rm_ctx* c) {
  if (!(c->cfg.outputs & RM_OUT_RGBA8)) return nullptr;
  if (comm_root(c)) return c->d_gathered;
  return c->ext_rgba8 ? c->ext_rgba8 : c->d_rgba8;
}
uint8_t* image_rgba8(const rm_ctx* c) {
  if (!c->subs.empty()) return image_rgba8(c->subs[0]);
  if (comm_root(c)) return c->ext_rgba8 ? c->ext_rgba8 : c->d_frame;
  return render_dst(c);
}
float* render_dst32(const rm_ctx* c) {
  if (!(c->cfg.outputs & RM_OUT_RGBA32F)) return nullptr;
  return comm_root(c) ? c->d_gathered32 : c->d_rgba32f;
}
float* image_rgba32f(const rm_ctx* c) {
  if (!c->subs.empty()) return image_rgba32f(c->subs[0]);
  if (comm_root(c)) return c->d_frame32;
  return render_dst32(c);
}
int image_rows(const rm_ctx* c) {
  if (!c->subs.empty() || comm_root(c)) return c->cfg.height;
  return c->rows;
}
bool full_frame(const rm_ctx* c) { return c->cfg.nshards <= 1 || !c->subs.empty() || comm_root(c); }
// Bytes per pixel of the context's RGBA8 shard images (rm_config.shard_format).
size_t bpp8(const rm_ctx* c) { return c->rgb3 ? 3 : 4; }
// Shard 0's rows per round (rm_config.rank0_rows; 0 = row_block, rm_shard.hpp).
int row_block0(const rm_ctx* c) { return c->cfg.rank0_rows > 0 ? c->cfg.rank0_rows : c->cfg.row_block; }

int nccl_fail(rm_ctx* c, const rm::Rccl* r, ncclResult_t e, const char* what) {
  return fail(c, RM_ERR_COMM, std::string(what) + ": " + (r ? r->GetErrorString(e) : "RCCL"));
}

// ---- communicator failure detection --------------------------------------
// Every wait on a communicator context is a bounded poll: the stream's progress
// (hipStreamQuery) and the communicator's asynchronous error
// (ncclCommGetAsyncError), against c->comm_timeout_ms.  An RCCL error or a missed
// deadline (a peer that died, stalled or never joined) aborts the communicator
// (ncclCommAbort: the pending collectives quit) and the context reports
// RM_ERR_COMM from then on; it can still be read for its error and destroyed.
long default_comm_timeout_ms() {
  const char* s = std::getenv("RM_COMM_TIMEOUT_MS");
  if (s && *s) {
    char* end = nullptr;
    const long v = std::strtol(s, &end, 10);
    if (end && *end == '\0' && v >= 0) return v;
  }
  return 120000;
}

// The contexts whose communicators one frame uses: a multi-GPU context's devices,
// or the context itself.
std::vector<rm_ctx*> comm_members(rm_ctx* c) {
  if (!c->subs.empty()) return c->subs;
  return {c};
}

int comm_abort(rm_ctx* c, const std::string& why) {
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  for (rm_ctx* m : comm_members(c)) {
    if (m->comm && r) {
      (void)hipSetDevice(m->device);
      (void)r->CommAbort(m->comm);  // pending collectives see the abort flag and quit
    }
    m->comm = nullptr;
    m->comm_failed = true;
    m->comm_why = why;
  }
  c->comm_failed = true;
  c->comm_why = why;
  return fail(c, RM_ERR_COMM, why);
}

bool has_comm(const rm_ctx* c) { return c->comm || (!c->subs.empty() && c->subs[0]->comm); }

// A communicator context whose communicator was aborted.
int comm_dead(rm_ctx* c) {
  return fail(c, RM_ERR_COMM, "the communicator was aborted: " + c->comm_why);
}

// Waits until every stream of the frame's contexts has drained, polling the
// communicators' asynchronous errors, within the context's deadline.
int comm_wait_devs(rm_ctx* c);
// (the caller's current device is restored: a multi-GPU context's wait visits
// every device)
int comm_wait(rm_ctx* c) {
  int dev = 0;
  const bool have_dev = hipGetDevice(&dev) == hipSuccess;
  const int rc = comm_wait_devs(c);
  if (have_dev) (void)hipSetDevice(dev);
  return rc;
}
int comm_wait_devs(rm_ctx* c) {
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, err);
  const std::vector<rm_ctx*> ms = comm_members(c);
  const long tmo = c->comm_timeout_ms;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<bool> done(ms.size(), false);
  for (int spins = 0;; ++spins) {
    bool all = true;
    for (size_t i = 0; i < ms.size(); ++i) {
      if (done[i]) continue;
      rm_ctx* m = ms[i];
      (void)hipSetDevice(m->device);
      // the render stream and, after a batch, the gather stream
      hipError_t q = hipStreamQuery(m->stream);
      if (q == hipSuccess && m->gstream) q = hipStreamQuery(m->gstream);
      if (q == hipSuccess) {
        done[i] = true;
        continue;
      }
      if (q != hipErrorNotReady) return hip_fail(c, q, "hipStreamQuery");
      all = false;
      if (m->comm) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t e = r->CommGetAsyncError(m->comm, &st);
        if (e != ncclSuccess || (st != ncclSuccess && st != ncclInProgress))
          return comm_abort(c, std::string("RCCL asynchronous error on device ") + std::to_string(m->device) +
                                   ": " + r->GetErrorString(e != ncclSuccess ? e : st));
      }
    }
    if (all) return RM_OK;
    if (tmo > 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(tmo))
      return comm_abort(c, "the frame did not complete within " + std::to_string(tmo) +
                               " ms (rm_comm_set_timeout): a peer rank stalled, failed or never issued "
                               "its gather");
    rm::poll_pause(spins);
  }
}

// Waits for an RCCL call that returned ncclInProgress (non-blocking communicator).
int comm_enqueued(rm_ctx* c, const rm::Rccl* r, ncclResult_t e, const char* what) {
  if (e == ncclSuccess) return RM_OK;
  // an enqueue error aborts the communicator (rm_api.h: RM_ERR_COMM means aborted);
  // a partial group may already have launched gathers that would wait forever
  if (e != ncclInProgress) return comm_abort(c, std::string(what) + ": " + r->GetErrorString(e));
  std::vector<ncclComm_t> cs;
  for (rm_ctx* m : comm_members(c))
    if (m->comm) cs.push_back(m->comm);
  const ncclResult_t w = rm::wait_ready(r, cs.data(), (int)cs.size(), c->comm_timeout_ms);
  if (w == ncclSuccess) return RM_OK;
  if (w == ncclInProgress)
    return comm_abort(c, std::string(what) + ": not enqueued within " + std::to_string(c->comm_timeout_ms) + " ms");
  return comm_abort(c, std::string(what) + ": " + r->GetErrorString(w));
}

// The stream wait of every synchronising call: bounded on a communicator context.
int stream_wait(rm_ctx* c) {
  if (c->comm_failed) return comm_dead(c);
  if (has_comm(c)) return comm_wait(c);
  RM_HIP(c, hipStreamSynchronize(c->stream));
  return RM_OK;
}

// Step 0 of every primary ray (rm_scene.hpp PrepSlot), on the host: what the
// render kernels' scene_lazy would compute at the camera, with the same IEEE operations in the same order (x86-64 SSE floats,
// -ffp-contract=off), so d0 is bit-identical to the device's scene_exact at the
// camera (sqrt_core / sqrt_cr_nonneg / div_capbb are the IEEE sqrt and divide on
// the values reached here, rm_fastmath.hpp).  The bounds (slack, LB_k, b1, b2)
// only need to be valid: their 2^-12 / 2^-18 margins were made for v_sqrt's
// 1.5 ulp, and the IEEE sqrt is within them.
void prep_host(const float cam[3], float blend, float omblend, float out[16]) {
  using namespace rmd;
  const float px = cam[0], py = cam[1], pz = cam[2];
  const float ax = px - 15.0f, ay = py, az = pz + 10.0f, bx = px + 25.0f, cx = px + 5.0f;
  const float ay2 = ay * ay, az2 = az * az, cx2 = cx * cx;
  const float x0 = (ax * ax + ay2) + az2, x1 = (bx * bx + ay2) + az2, xs = (cx2 + ay2) + az2;
  const float d0s = std::sqrt(x0) - 3.0f, d1 = std::sqrt(x1) - 3.0f;
  const float qx = std::fabs(cx) - 3.0f, qy = std::fabs(ay) - 2.5f, qz = std::fabs(az) - 2.5f;
  const float mx = std::fmax(qx, 0.0f), my = std::fmax(qy, 0.0f), mz = std::fmax(qz, 0.0f);
  const float box = std::fmin(std::fmax(qx, std::fmax(qy, qz)), 0.0f) +
                    std::sqrt((mx * mx + my * my) + mz * mz);
  const float d4 = box * omblend + (std::sqrt(xs) - 3.0f) * blend;
  const float tz = pz - 10.0f;
  const float l = std::sqrt(cx2 + ay2) - 2.5f;
  const float d5 = std::sqrt(l * l + tz * tz) - 0.5f;
  const float cpx = cx - CAP_AX, cpy = (py + 2.0f) - CAP_AY, cpz = (pz + 30.0f) - CAP_AZ;
  const float hn = (cpx * CAP_BAX + cpy * CAP_BAY) + cpz * CAP_BAZ;
  const float h = std::fmin(std::fmax(hn / CAP_BB_HOST, 0.0f), 1.0f);
  const float ex = cpx - CAP_BAX * h, ey = cpy - CAP_BAY * h, ez = cpz - CAP_BAZ * h;
  const float d6 = std::sqrt((ex * ex + ey * ey) + ez * ez) - 1.0f;
  const float d7 = py + 5.5f;
  const float ds[6] = {d0s, d1, d4, d5, d6, d7};
  float d = ds[0];
  bool nan = false;
  for (float v : ds) {
    nan = nan || std::isnan(v);
    d = v < d ? v : d;
  }
  const float HI = 1.0f + 0x1p-12f;
  const float sl = 0x1p-14f * (((std::fabs(px) + std::fabs(py)) + std::fabs(pz)) * HI + 64.0f) * HI;
  const float sx = px - SH_CX, sy = py - SH_CY, sz = pz - SH_CZ;
  const float rc = std::fma(std::sqrt((sx * sx + sy * sy) + sz * sz), HI, 0x1p-18f);
  const float kx = px - CAP_MX, ky = py - CAP_MY, kz = pz - CAP_MZ;
  const float x[5] = {x0, x1, xs, (cx2 + ay2) + tz * tz, (kx * kx + ky * ky) + kz * kz};
  const float R[5] = {3.0f, 3.0f, R_BLEND_LO, R_TORUS, R_CAPSULE};
  std::memset(out, 0, 16 * sizeof(float));
  out[PREP_VALID] = (!nan && d > 0.0f && d <= 400.0f) ? 1.0f : 0.0f;
  out[PREP_D0] = d;
  out[PREP_SLACK] = sl;
  out[PREP_B1] = (rc + SH_RALL + sl + 0.0f) * HI;
  out[PREP_B2] = ((py + 5.5f) - sl - 0.0f * HI) - 0x1p-19f * (std::fabs(py) + 5.5f + 0.0f + sl);
  out[PREP_B3] = ((SH_YTOP - py) + sl + 0.0f * HI) + 0x1p-19f * (std::fabs(py) + SH_YTOP + 0.0f + sl);
  const float pl = (py + 5.5f) + sl;
  for (int k = 0; k < 5; ++k) {
    // the gaps of scene_lazy's re-test at the camera with U = d0, in its float
    // operations: g = (lb - d0) - slack, plane gap lb - pl
    const float lb = std::fma(std::sqrt(x[k]), CULL_REL_LO, -(CULL_ABS + R[k]));
    const float g = lb - d - sl;
    out[PREP_G + k] = g > 0.0f ? g : -INFINITY;
    out[PREP_H + k] = g > 0.0f ? lb - pl : -INFINITY;
  }
}

// Step 0 of a table's primary rays (rm_internal.hpp TablePrep), on the host:
// what the table kernel's first march step computes at the camera, with the
// device's float operations (rm_table.hip prim_dist: IEEE sqrt and divide,
// GLSL min/max, opU in table order; x86-64 SSE floats, -ffp-contract=off).
// The slot bounds only need to be valid: the 2^-12 margin made for v_sqrt
// covers the IEEE sqrt.  Invalid (TP_VALID = 0) when d0 is not in (0, 400].
namespace {
struct H3 {
  float x, y, z;
};
float hgmin(float x, float y) { return y < x ? y : x; }
float hgmax(float x, float y) { return x < y ? y : x; }
float hdot(H3 a, H3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
float hlen(H3 a) { return std::sqrt(hdot(a, a)); }
float hprim(const float* P, H3 p, float blend, float omblend) {
  int type, swz;
  std::memcpy(&type, &P[rm::TW_TYPE], 4);
  std::memcpy(&swz, &P[rm::TW_SWIZZLE], 4);
  H3 q{p.x - P[rm::TW_CENTER], p.y - P[rm::TW_CENTER + 1], p.z - P[rm::TW_CENTER + 2]};
  if (swz == RM_SWIZZLE_XZY) q = H3{q.x, q.z, q.y};
  const float* a = P + rm::TW_P;
  switch (type) {
    case RM_PRIM_SPHERE:
      return hlen(q) - a[0];
    case RM_PRIM_BOX:
    case RM_PRIM_BLEND: {
      const H3 d{std::fabs(q.x) - a[0], std::fabs(q.y) - a[1], std::fabs(q.z) - a[2]};
      const H3 m{hgmax(d.x, 0.0f), hgmax(d.y, 0.0f), hgmax(d.z, 0.0f)};
      const float box = hgmin(hgmax(d.x, hgmax(d.y, d.z)), 0.0f) + hlen(m);
      if (type == RM_PRIM_BOX) return box;
      return box * omblend + (hlen(q) - a[3]) * blend;
    }
    case RM_PRIM_TORUS: {
      const float l = std::sqrt(q.x * q.x + q.z * q.z) - a[0];
      return std::sqrt(l * l + q.y * q.y) - a[1];
    }
    case RM_PRIM_CAPSULE: {
      const H3 pa{q.x - a[0], q.y - a[1], q.z - a[2]}, ba{a[3], a[4], a[5]};
      const float h = hgmin(hgmax(hdot(pa, ba) / a[6], 0.0f), 1.0f);
      return hlen(H3{pa.x - ba.x * h, pa.y - ba.y * h, pa.z - ba.z * h}) - a[7];
    }
    default:
      return hdot(q, H3{a[0], a[1], a[2]}) + a[3];
  }
}
}  // namespace

// The lazy slots of the context's table (EX_NSLOTS of its compiled words): the
// generic table kernel's instance (rm_table.hip launch_table).
static int table_slots(const rm_ctx* c) {
  const float* ex = reinterpret_cast<const float*>(c->scene_words.data()) + (size_t)c->nprims * rm::TABLE_WORDS;
  return (int)ex[rm::EX_NSLOTS];
}
// The generic kernel's production march for the table (rm_table.hip
// table_shape): 1 the built-in shape (reference-shaped tables), 2 the block
// shape of any plane-bounded table, 0 TLazy.
static int table_sl(const rm_ctx* c) {
  return c->nprims ? rm::table_shape(c->scene_words.data(), c->nprims) : 0;
}
// Which kernel a frame renders with (the graph's key): 0 built-in, 1 + the
// generic table kernel's instance (slots, shape).
static int table_key(const rm_ctx* c) {
  return c->nprims ? 1 + (table_slots(c) <= rm::TABLE_FEW_SLOTS ? 0 : 1) + 2 * table_sl(c) : 0;
}

void table_prep_host(const uint32_t* words, int32_t n, const float cam[3], float blend, float omblend,
                     float out[16]) {
  const float* t = reinterpret_cast<const float*>(words);
  const float* ex = t + (size_t)n * rm::TABLE_WORDS;
  const H3 p{cam[0], cam[1], cam[2]};
  std::memset(out, 0, 16 * sizeof(float));
  float d = INFINITY, U = INFINITY;
  for (int32_t k = 0; k < n; ++k) {
    const float* P = t + (size_t)k * rm::TABLE_WORDS;
    const float dk = hprim(P, p, blend, omblend);
    d = d < dk ? d : dk;  // opU(d, dk) = (d < dk) ? d : dk
    int type;
    std::memcpy(&type, &P[rm::TW_TYPE], 4);
    if (type == RM_PRIM_PLANE) U = hgmin(U, dk);
  }
  out[rm::TP_VALID] = (d > 0.0f && d <= 400.0f) ? 1.0f : 0.0f;
  out[rm::TP_D0] = d;
  // TLazy::dist's step-0 re-test at p = camera (dprev = +inf: U = the planes)
  const float sig2 = 2.0f * ex[rm::EX_SIGMA];
  const float a1 = (std::fabs(p.x) + std::fabs(p.y)) + std::fabs(p.z);
  const float sl0 = (a1 + ex[rm::EX_S]) * (1.0f + 0x1p-16f);
  const float sl = sig2 * (a1 + sl0) * (1.0f + 0x1p-10f);
  const int ns = (int)ex[rm::EX_NSLOTS];
  for (int j = 0; j < ns && j < rm::EX_MAX_SLOTS; ++j) {
    const float* B = t + (size_t)(int)ex[rm::EX_SLOTS + j] * rm::TABLE_WORDS + rm::TW_BALL;
    const float bx = p.x - B[0], by = p.y - B[1], bz = p.z - B[2];
    const float lb = std::fma(std::sqrt((bx * bx + by * by) + bz * bz), 1.0f - 0x1p-12f, -B[3]);
    out[rm::TP_G + j] = lb - U - sl;
  }
}

// Frame::unit_rd: every primary ray of the frame has |rd| within 2^-20 of 1.
// castRay (glsl:68-74) normalises v = uvx X + uvy Y + RN(D persp) (vec4, then
// .xyz): with the w components of X, Y, D zero, v.w = +-0 and, when |v|^2 stays
// in the normal range, every operation of normalize() has relative error <= u =
// 2^-24, so |rd| is within ~4.5u of 1.  The host bounds |v|^2 over the uv table's
// range [uv_lo, uv_hi]^2 exactly (a quadratic in (uvx, uvy): corners, edges and
// the interior critical point, in double), and requires min |v|^2 >= 2^-38 M^2
// (the float error of v, <= 3 sqrt(3) u M with M >= |v| the triangle bound,
// then moves |v| by < 16 %), min |v|^2 >= 2^-80 and M^2 <= 2^100.
static bool unit_rd_check(const rm_ctx* c, const rm_uniforms& u, float persp) {
  const rm_camera& k = u.camera;
  if (k.xAxis[3] != 0.0f || k.yAxis[3] != 0.0f || k.dir[3] != 0.0f) return false;
  double X[3], Y[3], C[3];
  for (int i = 0; i < 3; ++i) {
    X[i] = k.xAxis[i];
    Y[i] = k.yAxis[i];
    C[i] = (double)(k.dir[i] * persp);  // the kernel's float product
    if (!std::isfinite(X[i]) || !std::isfinite(Y[i]) || !std::isfinite(C[i])) return false;
  }
  auto dotd = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  const double xx = dotd(X, X), yy = dotd(Y, Y), xy = dotd(X, Y), xc = dotd(X, C), yc = dotd(Y, C),
               cc = dotd(C, C);
  auto q = [&](double a, double b) { return a * a * xx + b * b * yy + 2 * a * b * xy + 2 * a * xc + 2 * b * yc + cc; };
  const double a0 = c->uv_lo[0], a1 = c->uv_hi[0], b0 = c->uv_lo[1], b1 = c->uv_hi[1];
  if (!(a0 <= a1) || !(b0 <= b1)) return false;
  auto clampd = [](double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); };
  double m = std::fmin(std::fmin(q(a0, b0), q(a0, b1)), std::fmin(q(a1, b0), q(a1, b1)));
  for (double a : {a0, a1})
    if (yy > 0) m = std::fmin(m, q(a, clampd(-(a * xy + yc) / yy, b0, b1)));
  for (double b : {b0, b1})
    if (xx > 0) m = std::fmin(m, q(clampd(-(b * xy + xc) / xx, a0, a1), b));
  const double det = xx * yy - xy * xy;
  if (det > 0) {
    const double a = (-xc * yy + yc * xy) / det, b = (-yc * xx + xc * xy) / det;
    if (a >= a0 && a <= a1 && b >= b0 && b <= b1) m = std::fmin(m, q(a, b));
  }
  const double M = std::fmax(std::fabs(a0), std::fabs(a1)) * std::sqrt(xx) +
                   std::fmax(std::fabs(b0), std::fabs(b1)) * std::sqrt(yy) + std::sqrt(cc);
  // (m carries the double rounding of the quadratic, relative ~1e-15 of M^2:
  // the 2^-38 M^2 floor is far above it)
  return m >= std::ldexp(M * M, -38) && m >= std::ldexp(1.0, -80) && M * M <= std::ldexp(1.0, 100);
}

rmd::Frame make_frame(const rm_ctx* c) {
  const rm_uniforms& u = c->u;
  rmd::Frame F;
  std::memset(&F, 0, sizeof F);
  std::memcpy(F.cam_pos, u.camera.pos, sizeof F.cam_pos);
  std::memcpy(F.cam_dir, u.camera.dir, sizeof F.cam_dir);
  std::memcpy(F.cam_y, u.camera.yAxis, sizeof F.cam_y);
  std::memcpy(F.cam_x, u.camera.xAxis, sizeof F.cam_x);
  std::memcpy(F.lpos, u.light.position, sizeof F.lpos);
  std::memcpy(F.lamb, u.light.ambient, sizeof F.lamb);
  std::memcpy(F.ldif, u.light.diffuse, sizeof F.ldif);
  std::memcpy(F.lspec, u.light.specular, sizeof F.lspec);
  F.lconst = u.light.constant;
  F.llin = u.light.linear;
  F.lquad = u.light.quadratic;
  // Uniform-only subexpressions, evaluated once on the host with the same
  // float operations the GLSL performs per call (glsl:70, 117, 185/236).
  F.blend = std::sin(u.iTime) / 2.0f + 0.5f;
  F.omblend = 1.0f - F.blend;
  F.k = (u.shadow_mode == RM_SHADOW_HARD) ? INFINITY : 2.0f;
  // the soft-shadow exit's ratio bound (rm_scene.hpp shadow_exit_init), the
  // device's former per-call expression in the same float operations
  F.shc = (F.k == INFINITY) ? 0.0f : (1.0f + 0x1p-9f) / F.k * (1.0f + 0x1p-12f);
  F.persp = 45.0f * static_cast<float>(0.01745329251994329576923690768489);
  F.uvx = c->d_uv;
  F.uvy = c->d_uv + (size_t)5 * c->cfg.width;
  F.uv_exact = c->uv_exact ? 1 : 0;
  F.unit_rd = unit_rd_check(c, u, F.persp) ? 1 : 0;
  const float uv_ox[4] = {0.25f, 0.75f, 0.25f, 0.75f}, uv_oy[4] = {0.25f, 0.25f, 0.75f, 0.75f};
  for (int a = 0; a < 2; ++a) {
    const float n = (float)(a ? c->cfg.height : c->cfg.width);
    F.uv_dims[a] = n;
    F.uv_rcp[a] = 1.0f / n;
    for (int k = 0; k < 4; ++k) F.uv_off[a][k] = (a ? uv_oy[k] : uv_ox[k]) / n;
  }
  F.bounces = u.bounceVar;
  F.aa = u.AA ? 1 : 0;
  F.width = c->cfg.width;
  F.height = c->cfg.height;
  F.row_block = c->cfg.row_block;
  F.row_block0 = row_block0(c);
  F.shard = c->cfg.shard;
  F.nshards = c->cfg.nshards > 1 ? c->cfg.nshards : 1;
  F.rows = c->rows;
  F.rgba8 = render_dst(c);
  F.rgb3 = c->rgb3 ? 1 : 0;
  F.rgba32f = render_dst32(c);
  F.sdf_counts = c->cfg.counters ? c->d_counts : nullptr;
  F.counters = c->cfg.counters ? c->d_counters : nullptr;
  if (c->nprims) table_prep_host(c->scene_words.data(), c->nprims, F.cam_pos, F.blend, F.omblend, F.prepv);
  else prep_host(F.cam_pos, F.blend, F.omblend, F.prepv);
  F.scene = c->nprims ? reinterpret_cast<const float*>(c->d_scene) : nullptr;
  F.nprims = c->nprims;
  rm::pixel_grid(F.width, F.rows, F.aa != 0, &F.grid_x, &F.grid_y);
  return F;
}

// The specialised table kernels for frame F, or null: they take sqrt(x) - R in
// the fast exact form for march and normal points (rm_table.hip sqrt_sub), which
// needs every such point within 2^53 of every entry.  Entries lie within 10^15
// of the origin (rm::exit_bounds), a march moves at most nmax tmax = 2.05e5
// along a unit ray and five bounces add 1.3e5 more, so a camera within 10^15
// of the origin keeps them there; a frame whose camera is farther out (or not
// finite) renders with the generic kernel.
//
// The light position is not bounded here: shadow rays (rd = light.position - pos,
// unnormalised, glsl:184, 235) march with the full-range form (TLazy::dist ->
// prim_dist<false>, rm_table.hip), so however far the light is, no shadow point
// reaches the short form (tests/test_gpu_scene.py far-light case).
const rm::JitTable* frame_jit(const rm_ctx* c, const rmd::Frame& F) {
  if (!c->jit) return nullptr;
  for (int i = 0; i < 3; ++i)
    if (!(std::fabs(F.cam_pos[i]) <= 1e15f)) return nullptr;
  return c->jit;
}

void graph_release(rm_ctx* c) {
  rm_graph_slot& g = c->gs;
  if (g.exec || g.graph) (void)hipStreamSynchronize(c->stream);
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g = rm_graph_slot();
  c->graph_aa = -1;
  c->graph_table = -1;
}

void free_all(rm_ctx* c) {
  graph_release(c);
  {
    // the communicators of this context (its own, or its devices'), torn down
    // together and within the deadline (rm_comm.cpp teardown)
    std::vector<ncclComm_t> cs;
    for (rm_ctx* m : c->subs.empty() ? std::vector<rm_ctx*>{c} : c->subs)
      if (m->own_comm && m->comm) {
        cs.push_back(m->comm);
        m->comm = nullptr;
      }
    std::string err;
    const rm::Rccl* r = cs.empty() ? nullptr : rm::rccl(&err);
    if (r) {
      int dev = 0;
      const bool have_dev = hipGetDevice(&dev) == hipSuccess;
      rm::teardown(r, cs.data(), (int)cs.size(), c->comm_timeout_ms);
      if (have_dev) (void)hipSetDevice(dev);
    }
  }
  for (rm_ctx* s : c->subs) rm_destroy(s);
  c->subs.clear();
  c->comm = nullptr;
  for (void* p : {(void*)c->d_gathered, (void*)c->d_frame, (void*)c->d_gathered32, (void*)c->d_frame32,
                  (void*)c->d_rgba8, (void*)c->d_rgba32f, (void*)c->d_counts, (void*)c->d_counters,
                  (void*)c->d_uv, (void*)c->d_scene})
    if (p) (void)hipFree(p);
  c->d_gathered = c->d_frame = nullptr;
  c->d_gathered32 = c->d_frame32 = nullptr;
  if (c->gstream) (void)hipStreamSynchronize(c->gstream);
  for (uint8_t* p : c->ring8) (void)hipFree(p);
  for (float* p : c->ring32) (void)hipFree(p);
  c->ring8.clear();
  c->ring32.clear();
  for (auto& b : c->bslot) {
    if (b.send8) (void)hipFree(b.send8);
    if (b.send32) (void)hipFree(b.send32);
    if (b.rendered) (void)hipEventDestroy(b.rendered);
    if (b.freed) (void)hipEventDestroy(b.freed);
    b = rm_ctx::BatchSlot();
  }
  if (c->gdone) (void)hipEventDestroy(c->gdone);
  c->gdone = nullptr;
  if (c->out_ev) (void)hipEventDestroy(c->out_ev);
  c->out_ev = nullptr;
  if (c->gstream) (void)hipStreamDestroy(c->gstream);
  c->gstream = nullptr;
  for (auto& p : c->ev_pool) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  c->ev_pool.clear();
  c->ev_frames.clear();
  for (hipEvent_t& e : c->ph) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  c->d_rgba8 = nullptr;
  c->d_rgba32f = nullptr;
  c->d_counts = nullptr;
  c->d_counters = nullptr;
  c->d_uv = nullptr;
  c->d_scene = nullptr;
  c->stream = nullptr;
}

int check_uniforms(rm_ctx* c, const rm_uniforms& u) {
  if (u.bounceVar < 0 || u.bounceVar > 5)
    return fail(c, RM_ERR_INVALID, "bounceVar must be in 0..5 (main.cpp:199-204)");
  if (u.shadow_mode != RM_SHADOW_SOFT && u.shadow_mode != RM_SHADOW_HARD)
    return fail(c, RM_ERR_INVALID, "shadow_mode must be RM_SHADOW_SOFT or RM_SHADOW_HARD");
  return RM_OK;
}

// Joins a sharded context to a communicator as `rank` of `n`: rank 0 gets the
// gather buffers (its shard renders into slot 0, so ncclGather runs in place) and
// the assembled frames, one pair per enabled output format.  Rank 0's readable
// image changes from its shard to the full frame, so a caller-set RGBA8 output
// (sized for the shard) is dropped: output pointers are set, or re-queried, after
// rm_comm_init (include/rm_api.h).
int comm_attach(rm_ctx* c, ncclComm_t comm, int rank, int n, bool own, bool member) {
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  c->comm = comm;
  c->own_comm = own;
  c->group_member = member;
  c->crank = rank;
  c->cranks = n;
  c->comm_failed = false;
  // the gathered shards travel as packed RGB unless the config asks for RGBA8
  if ((c->cfg.outputs & RM_OUT_RGBA8) && c->cfg.shard_format == RM_SHARD_AUTO) c->rgb3 = true;
  if (rank == 0) {
    const size_t px_shard = (size_t)c->rows * c->cfg.width, px_frame = (size_t)c->cfg.height * c->cfg.width;
    if (c->cfg.outputs & RM_OUT_RGBA8) {
      RM_HIP(c, hipMalloc(&c->d_gathered, px_shard * 4 * n));
      RM_HIP(c, hipMalloc(&c->d_frame, px_frame * 4));
      RM_HIP(c, hipMemsetAsync(c->d_gathered, 0, px_shard * 4 * n, c->stream));
      RM_HIP(c, hipMemsetAsync(c->d_frame, 0, px_frame * 4, c->stream));
    }
    if (c->cfg.outputs & RM_OUT_RGBA32F) {
      RM_HIP(c, hipMalloc(&c->d_gathered32, px_shard * 16 * n));
      RM_HIP(c, hipMalloc(&c->d_frame32, px_frame * 16));
      RM_HIP(c, hipMemsetAsync(c->d_gathered32, 0, px_shard * 16 * n, c->stream));
      RM_HIP(c, hipMemsetAsync(c->d_frame32, 0, px_frame * 16, c->stream));
    }
    RM_HIP(c, hipStreamSynchronize(c->stream));
    // rank 0 renders into the gather buffers
    if (c->d_rgba8) (void)hipFree(c->d_rgba8);
    if (c->d_rgba32f) (void)hipFree(c->d_rgba32f);
    c->d_rgba8 = nullptr;
    c->d_rgba32f = nullptr;
    c->ext_rgba8 = nullptr;  // a shard-sized caller buffer cannot hold the frame
  }
  graph_release(c);
  return RM_OK;
}

int check_comm_config(const rm_config& cfg, const char* who) {
  if ((cfg.outputs & ~(RM_OUT_RGBA8 | RM_OUT_RGBA32F)) != 0 || cfg.counters)
    return fail(nullptr, RM_ERR_INVALID, std::string(who) + ": RCCL-gathered frames are RGBA8 and/or "
                                         "RGBA32F, without counters");
  return RM_OK;
}

// rm_config.ngpus >= 1: one shard context per device plus a single-process
// communicator over the devices (one ncclCommInitRankConfig per device inside a
// group, non-blocking, waited for within the deadline).
int create_multi(rm_ctx** out, const rm_config* cfg) {
  const int n = cfg->ngpus;
  int rc = check_comm_config(*cfg, "rm_create");
  if (rc != RM_OK) return rc;
  if (cfg->nshards > 1 || cfg->shard != 0)
    return fail(nullptr, RM_ERR_INVALID, "rm_create: ngpus shards by itself (shard/nshards must be 0)");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(nullptr, RM_ERR_NO_DEVICE, "rm_create: no HIP device (librm has no CPU fallback)");
  std::vector<int> devs(n);
  int d0 = cfg->device;
  if (d0 < 0 && hipGetDevice(&d0) != hipSuccess) d0 = 0;
  for (int i = 0; i < n; ++i) {
    devs[i] = cfg->devices ? cfg->devices[i] : d0 + i;
    if (devs[i] < 0 || devs[i] >= ndev)
      return fail(nullptr, RM_ERR_INVALID, "rm_create: device " + std::to_string(devs[i]) +
                                               " out of range (" + std::to_string(ndev) + " devices)");
    for (int j = 0; j < i; ++j)
      if (devs[j] == devs[i])
        return fail(nullptr, RM_ERR_INVALID, "rm_create: devices must be distinct (one shard per GPU)");
  }
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(nullptr, RM_ERR_COMM, "rm_create: " + err);
  rm_ctx* c = new (std::nothrow) rm_ctx();
  if (!c) return fail(nullptr, RM_ERR_NOMEM, "rm_create: out of host memory");
  c->cfg = *cfg;
  if (c->cfg.outputs == 0) c->cfg.outputs = RM_OUT_RGBA8;
  c->cfg.row_block = cfg->row_block > 0 ? cfg->row_block : 8;
  c->cfg.nshards = n;
  c->cfg.shard = 0;
  c->cfg.devices = nullptr;  // not kept: the caller owns the array
  c->device = devs[0];
  c->rows = c->cfg.height;
  c->comm_timeout_ms = default_comm_timeout_ms();
  rm_default_uniforms(&c->u);
  auto bail = [&](int code) {
    g_create_error = c->err;
    free_all(c);
    delete c;
    return code;
  };
  for (int i = 0; i < n; ++i) {
    rm_config sc = c->cfg;
    sc.ngpus = 0;
    sc.device = devs[i];
    sc.shard = i;
    rm_ctx* sub = nullptr;
    if ((rc = rm_create(&sub, &sc)) != RM_OK) {
      c->err = "rm_create (device " + std::to_string(devs[i]) + "): " + g_create_error;
      return bail(rc);
    }
    c->subs.push_back(sub);
  }
  ncclUniqueId id;
  ncclResult_t e = r->GetUniqueId(&id);
  if (e != ncclSuccess) return bail(nccl_fail(c, r, e, "ncclGetUniqueId"));
  std::vector<ncclComm_t> comms(n, nullptr);
  e = r->GroupStart();
  for (int i = 0; i < n && (e == ncclSuccess || e == ncclInProgress); ++i) {
    ncclConfig_t nb = rm::nonblocking_config();
    (void)hipSetDevice(devs[i]);
    e = r->CommInitRankConfig(&comms[i], n, id, i, &nb);
  }
  const ncclResult_t eg = r->GroupEnd();
  if (e == ncclSuccess || e == ncclInProgress) e = eg;
  if (e == ncclSuccess || e == ncclInProgress) e = rm::wait_ready(r, comms.data(), n, c->comm_timeout_ms);
  if (e != ncclSuccess) {
    for (int i = 0; i < n; ++i)
      if (comms[i]) (void)r->CommAbort(comms[i]);
    c->err = e == ncclInProgress
                 ? "rm_create: the communicator was not ready within " + std::to_string(c->comm_timeout_ms) + " ms"
                 : std::string("rm_create: ncclCommInitRankConfig: ") + r->GetErrorString(e);
    return bail(RM_ERR_COMM);
  }
  for (int i = 0; i < n; ++i) {
    if ((rc = comm_attach(c->subs[i], comms[i], i, n, true, true)) != RM_OK) {
      //  abort every member, attached or not, and detach them, so the
      // teardown below neither finalizes a half-aborted group (and waits out the
      // deadline) nor leaks comms[i]
      c->err = c->subs[i]->err;
      for (int j = 0; j < n; ++j) {
        (void)hipSetDevice(devs[j]);
        (void)r->CommAbort(comms[j]);
        c->subs[j]->comm = nullptr;
        c->subs[j]->own_comm = false;
      }
      return bail(rc);
    }
    c->subs[i]->comm_timeout_ms = c->comm_timeout_ms;
  }
  c->stream = c->subs[0]->stream;  // the frame's stream (not owned)
  *out = c;
  return RM_OK;
}

// The gather of one rank (ncclGather to rank 0, in place on rank 0): the RGBA8
// and RGBA32F shards in one group.
int comm_gather(rm_ctx* c) {
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, err);
  const size_t px = (size_t)c->rows * c->cfg.width;
  const bool root = comm_root(c);
  ncclResult_t e = r->GroupStart();
  if (e == ncclSuccess && (c->cfg.outputs & RM_OUT_RGBA8))
    e = r->Gather(render_dst(c), root ? c->d_gathered : nullptr, px * bpp8(c), ncclUint8, 0, c->comm, c->stream);
  if ((e == ncclSuccess || e == ncclInProgress) && (c->cfg.outputs & RM_OUT_RGBA32F))
    e = r->Gather(render_dst32(c), root ? c->d_gathered32 : nullptr, px * 4, ncclFloat32, 0, c->comm,
                  c->stream);
  const ncclResult_t eg = r->GroupEnd();
  if (e == ncclSuccess || e == ncclInProgress) e = eg;
  const int rc = comm_enqueued(c, r, e, "ncclGather");
  if (rc != RM_OK) return rc;
  c->comm_warm = true;
  return RM_OK;
}

// Rank 0: the gathered shards -> the frame (k_unshard), on the same stream.  An
// RGBA32F row is 4 x width 32-bit words: the same row permutation as an RGBA8
// image 4 x as wide.
int comm_assemble(rm_ctx* c) {
  if (!comm_root(c)) return RM_OK;
  if (c->cfg.outputs & RM_OUT_RGBA8) {
    const hipError_t e = rm::launch_unshard(c->d_gathered, image_rgba8(c), c->cfg.width, c->cfg.height,
                                            c->cfg.row_block, row_block0(c), c->cranks, c->rows, c->stream, 0,
                                            c->rgb3);
    if (e != hipSuccess) return hip_fail(c, e, "unshard launch");
  }
  if (c->cfg.outputs & RM_OUT_RGBA32F) {
    const hipError_t e = rm::launch_unshard(c->d_gathered32, c->d_frame32, c->cfg.width * 4, c->cfg.height,
                                            c->cfg.row_block, row_block0(c), c->cranks, c->rows, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "unshard launch (RGBA32F)");
  }
  return RM_OK;
}

}  // namespace

#ifdef RM_STATS
namespace rm {
hipError_t debug_stats(unsigned long long* out, bool clear);
}
#endif

extern "C" {

#ifdef RM_STATS
/* Diagnostic builds only (-DRM_STATS, tools/build_variant.sh): the 64 wave /
 * lane counters of rm_scene.hpp's RM_STAT points, then cleared. */
int rm_debug_stats(unsigned long long *out64) {
  return rm::debug_stats(out64, true) == hipSuccess ? 0 : -1;
}
#endif


const char* rm_last_error(const rm_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int rm_device_count(int* count) {
  if (!count) return RM_ERR_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return RM_OK;
}

int rm_config_init(rm_config* cfg, int32_t width, int32_t height) {
  if (!cfg) return RM_ERR_INVALID;
  std::memset(cfg, 0, sizeof *cfg);
  cfg->struct_size = (uint32_t)sizeof(rm_config);
  cfg->magic = RM_CONFIG_MAGIC;
  cfg->width = width;
  cfg->height = height;
  cfg->device = -1;
  cfg->outputs = RM_OUT_RGBA8;
  cfg->nshards = 1;
  return RM_OK;
}

int rm_create(rm_ctx** out, const rm_config* cfg) {
  if (!out || !cfg) return fail(nullptr, RM_ERR_INVALID, "rm_create: null argument");
  *out = nullptr;
  // A host built against an older rm_api.h passes a smaller struct without this
  // field (its first word is the width): refuse it rather than read past its end.
  if (cfg->struct_size != (uint32_t)sizeof(rm_config) || cfg->magic != RM_CONFIG_MAGIC)
    return fail(nullptr, RM_ERR_INVALID,
                "rm_create: rm_config.struct_size must be sizeof(rm_config) = " +
                    std::to_string(sizeof(rm_config)) + " and rm_config.magic RM_CONFIG_MAGIC (rm_config_init; "
                    "API version " + std::to_string(RM_API_VERSION) + ")");
  if (cfg->width <= 0 || cfg->height <= 0 || cfg->width > 65536 || cfg->height > 65536)
    return fail(nullptr, RM_ERR_INVALID, "rm_create: width/height must be in 1..65536");
  if (cfg->ngpus < 0 || cfg->ngpus > 64)
    return fail(nullptr, RM_ERR_INVALID, "rm_create: ngpus must be in 0..64");
  if (cfg->shard_format < RM_SHARD_AUTO || cfg->shard_format > RM_SHARD_RGB8)
    return fail(nullptr, RM_ERR_INVALID, "rm_create: shard_format must be RM_SHARD_AUTO, _RGBA8 or _RGB8");
  if (cfg->ngpus >= 1) {
    if (cfg->kernel < RM_KERNEL_AUTO || cfg->kernel > RM_KERNEL_PIXEL)
      return fail(nullptr, RM_ERR_INVALID, "rm_create: unknown kernel variant");
    return create_multi(out, cfg);
  }
  if (cfg->outputs & ~(RM_OUT_RGBA8 | RM_OUT_RGBA32F))
    return fail(nullptr, RM_ERR_INVALID, "rm_create: unknown output bits");
  if (cfg->kernel < RM_KERNEL_AUTO || cfg->kernel > RM_KERNEL_PIXEL)
    return fail(nullptr, RM_ERR_INVALID, "rm_create: unknown kernel variant");
  if (cfg->nshards > 1 && rm_shard_rows(cfg->height, cfg->row_block, cfg->rank0_rows, cfg->nshards, cfg->shard,
                                         nullptr, nullptr) != RM_OK)
    return fail(nullptr, RM_ERR_INVALID, "rm_create: bad row_block/rank0_rows/shard/nshards (rm_shard_rows)");
  if (cfg->rank0_rows < 0) return fail(nullptr, RM_ERR_INVALID, "rm_create: rank0_rows must be >= 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(nullptr, RM_ERR_NO_DEVICE,
                "rm_create: no HIP device (librm has no CPU fallback; use a GPU box)");
  rm_ctx* c = new (std::nothrow) rm_ctx();
  if (!c) return fail(nullptr, RM_ERR_NOMEM, "rm_create: out of host memory");
  c->cfg = *cfg;
  c->cfg.devices = nullptr;  // not kept: the caller owns the array
  if (c->cfg.outputs == 0) c->cfg.outputs = RM_OUT_RGBA8;
  if (c->cfg.nshards <= 1) {
    c->cfg.nshards = 1;
    c->cfg.shard = 0;
    if (c->cfg.row_block <= 0) c->cfg.row_block = 1;
  }
  c->rgb3 = c->cfg.nshards > 1 && c->cfg.shard_format == RM_SHARD_RGB8 && (c->cfg.outputs & RM_OUT_RGBA8);
  if (cfg->device >= 0) {
    c->device = cfg->device;
  } else {
    if (hipGetDevice(&c->device) != hipSuccess) c->device = 0;
  }
  if (c->device >= ndev) {
    delete c;
    return fail(nullptr, RM_ERR_INVALID, "rm_create: device ordinal out of range");
  }
  int rc = RM_OK;
  auto bail = [&](int code) {
    g_create_error = c->err;
    free_all(c);
    delete c;
    return code;
  };
  if ((rc = set_device(c)) != RM_OK) return bail(rc);
  rm_shard_rows(c->cfg.height, c->cfg.row_block, c->cfg.rank0_rows, c->cfg.nshards, c->cfg.shard, nullptr,
                &c->rows);
  const size_t npx = (size_t)c->rows * (size_t)c->cfg.width;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) return bail(hip_fail(c, e, "hipStreamCreate"));
  c->own_stream = true;
  if (c->cfg.outputs & RM_OUT_RGBA8) {
    if ((e = hipMalloc(&c->d_rgba8, npx * 4)) != hipSuccess) return bail(hip_fail(c, e, "hipMalloc rgba8"));
    // on the context's own (non-blocking) stream: a NULL-stream memset is not
    // ordered before kernels on it and could land after the first dispatch
    if ((e = hipMemsetAsync(c->d_rgba8, 0, npx * 4, c->stream)) != hipSuccess)
      return bail(hip_fail(c, e, "hipMemset"));
  }
  if (c->cfg.outputs & RM_OUT_RGBA32F) {
    if ((e = hipMalloc(&c->d_rgba32f, npx * 16)) != hipSuccess) return bail(hip_fail(c, e, "hipMalloc rgba32f"));
    if ((e = hipMemsetAsync(c->d_rgba32f, 0, npx * 16, c->stream)) != hipSuccess)
      return bail(hip_fail(c, e, "hipMemset"));
  }
  if (c->cfg.counters) {
    if ((e = hipMalloc(&c->d_counts, npx * 4)) != hipSuccess) return bail(hip_fail(c, e, "hipMalloc counts"));
    if ((e = hipMalloc(&c->d_counters, 8 * sizeof(unsigned long long))) != hipSuccess)
      return bail(hip_fail(c, e, "hipMalloc counters"));
  }
  {
    // uv of the pixel columns and rows with the shader's float operations
    // (glsl:301-305 and the cumulative sub-sample offsets of :309-332)
    const int W = c->cfg.width, H = c->cfg.height;
    const float ox[4] = {0.25f, 0.75f, 0.25f, 0.75f}, oy[4] = {0.25f, 0.25f, 0.75f, 0.75f};
    std::vector<float> uv((size_t)5 * (W + H));
    for (int p = 0; p < W + H; ++p) {
      const bool col = p < W;
      const int i = col ? p : p - W, n = col ? W : H;
      float v = (float)(i * 2 - n) / (float)n;
      uv[(size_t)p * 5] = v;
      for (int k = 0; k < 4; ++k) {
        v += (col ? ox[k] : oy[k]) / (float)n;
        uv[(size_t)p * 5 + 1 + k] = v;
      }
    }
    // lane_uv (rm_scene.hpp) may form the same values arithmetically when, for every
    // column and row, RN(1/n)-times-a plus one fma remainder correction equals the
    // IEEE (2p - n) / n; the offsets' adds are the table's own operations
    for (int a = 0; a < 2; ++a) {
      c->uv_lo[a] = INFINITY;
      c->uv_hi[a] = -INFINITY;
    }
    for (int p = 0; p < W + H; ++p)
      for (int k = 0; k < 5; ++k) {
        const int a = p < W ? 0 : 1;
        c->uv_lo[a] = std::fmin(c->uv_lo[a], uv[(size_t)p * 5 + k]);
        c->uv_hi[a] = std::fmax(c->uv_hi[a], uv[(size_t)p * 5 + k]);
      }
    c->uv_exact = true;
    for (int p = 0; p < W + H && c->uv_exact; ++p) {
      const bool col = p < W;
      const int i = col ? p : p - W, n = col ? W : H;
      const float a = (float)(i * 2 - n), nf = (float)n, r = 1.0f / nf;
      const float q0 = a * r;
      const float q = std::fma(std::fma(-q0, nf, a), r, q0);
      c->uv_exact = q == uv[(size_t)p * 5] && std::signbit(q) == std::signbit(uv[(size_t)p * 5]);
    }
    if ((e = hipMalloc(&c->d_uv, uv.size() * sizeof(float))) != hipSuccess ||
        (e = hipMemcpy(c->d_uv, uv.data(), uv.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
      return bail(hip_fail(c, e, "uv table"));
  }
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return bail(hip_fail(c, e, "hipStreamSynchronize"));
  rm_default_uniforms(&c->u);
  c->comm_timeout_ms = default_comm_timeout_ms();
  *out = c;
  return RM_OK;
}

void rm_destroy(rm_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  // a collective that never completes must not hang the teardown: the bounded
  // wait aborts the communicator on its deadline, and the aborted gather quits
  if (has_comm(ctx) && !ctx->comm_failed && !ctx->group_member) (void)comm_wait(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->gstream) (void)hipStreamSynchronize(ctx->gstream);
  free_all(ctx);
  delete ctx;
}

// ---- uniforms -------------------------------------------------------------------
static int set_floats(rm_ctx* c, const char* name, const float* v, int n) {
  if (!c || !name) return RM_ERR_INVALID;
  int m = 0;
  float* dst = rm::uniform_floats(&c->u, name, &m);
  if (!dst) return RM_WARN_UNKNOWN_UNIFORM;
  // glUniform with a mismatched component count is a GL error that leaves the
  // uniform unchanged; report it instead of writing.
  if (m != n) return fail(c, RM_ERR_INVALID, std::string("uniform '") + name + "' has " +
                                                 std::to_string(m) + " components");
  std::memcpy(dst, v, sizeof(float) * n);
  return RM_OK;
}

static int set_int(rm_ctx* c, const char* name, int32_t v) {
  if (!c || !name) return RM_ERR_INVALID;
  int32_t* dst = rm::uniform_ints(&c->u, name);
  if (!dst) {
    int m = 0;
    if (rm::uniform_floats(&c->u, name, &m))
      return fail(c, RM_ERR_INVALID, std::string("uniform '") + name + "' is a float");
    return RM_WARN_UNKNOWN_UNIFORM;
  }
  rm_uniforms t = c->u;
  *rm::uniform_ints(&t, name) = v;
  int rc = check_uniforms(c, t);
  if (rc != RM_OK) return rc;
  *dst = v;
  return RM_OK;
}

int rm_set_bool(rm_ctx* c, const char* name, int value) { return set_int(c, name, value ? 1 : 0); }
int rm_set_int(rm_ctx* c, const char* name, int32_t value) { return set_int(c, name, value); }
int rm_set_uint(rm_ctx* c, const char* name, const uint32_t* value) {
  if (!value) return RM_ERR_INVALID;
  return set_int(c, name, (int32_t)*value);
}
int rm_set_float(rm_ctx* c, const char* name, float value) { return set_floats(c, name, &value, 1); }
int rm_set_vec2(rm_ctx* c, const char* name, float x, float y) {
  const float v[2] = {x, y};
  return set_floats(c, name, v, 2);
}
int rm_set_vec3(rm_ctx* c, const char* name, float x, float y, float z) {
  const float v[3] = {x, y, z};
  return set_floats(c, name, v, 3);
}
int rm_set_vec4(rm_ctx* c, const char* name, float x, float y, float z, float w) {
  const float v[4] = {x, y, z, w};
  return set_floats(c, name, v, 4);
}

int rm_set_uniforms(rm_ctx* c, const rm_uniforms* u) {
  if (!c || !u) return RM_ERR_INVALID;
  int rc = check_uniforms(c, *u);
  if (rc != RM_OK) return rc;
  c->u = *u;
  return RM_OK;
}

int rm_get_uniforms(const rm_ctx* c, rm_uniforms* u) {
  if (!c || !u) return RM_ERR_INVALID;
  *u = c->u;
  return RM_OK;
}

// ---- dispatch ---------------------------------------------------------------------
namespace {

// Timing events for the next launch (rm_enable_timing), or nulls.
int timing_events(rm_ctx* c, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (!c->timing) return RM_OK;
  if (c->ev_used == c->ev_pool.size()) {
    std::pair<hipEvent_t, hipEvent_t> p;
    RM_HIP(c, hipEventCreate(&p.first));
    RM_HIP(c, hipEventCreate(&p.second));
    c->ev_pool.push_back(p);
  }
  *e0 = c->ev_pool[c->ev_used].first;
  *e1 = c->ev_pool[c->ev_used].second;
  if (c->ev_frames.size() < c->ev_pool.size()) c->ev_frames.resize(c->ev_pool.size(), 1);
  c->ev_frames[c->ev_used] = 1;
  c->ev_used++;
  return RM_OK;
}

// A plain dispatch after a batch on a communicator context: its render may
// write the image the batch's assembly writes, and its gather must follow the
// batch's on the communicator, so the context's stream waits for the gather
// stream's last batch (rm_dispatch_frames).
int order_after_batch(rm_ctx* c) {
  c->batch_n = 1;
  if (!c->gdone_pending) return RM_OK;
  RM_HIP(c, hipStreamWaitEvent(c->stream, c->gdone, 0));
  c->gdone_pending = false;
  return RM_OK;
}

// The render kernel of one frame on the context's stream (== glDispatchCompute).
int render_launch(rm_ctx* c) {
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if ((rc = order_after_batch(c)) != RM_OK) return rc;
  if (c->cfg.counters) {
    RM_HIP(c, hipMemsetAsync(c->d_counters, 0, 8 * sizeof(unsigned long long), c->stream));
  }
  rmd::Frame F = make_frame(c);
  hipEvent_t e0, e1;
  if ((rc = timing_events(c, &e0, &e1)) != RM_OK) return rc;
  if (e0) RM_HIP(c, hipEventRecord(e0, c->stream));
  // a runtime scene table renders with the table kernel
  const rm::JitTable* jit = frame_jit(c, F);
  hipError_t e = c->nprims ? (jit ? rm::launch_table_jit(jit, F, c->cfg.counters != 0, c->stream)
                                  : rm::launch_table(F, c->cfg.counters != 0, c->stream, table_slots(c), table_sl(c)))
                           : rm::launch_pixel(F, c->cfg.counters != 0, c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "kernel launch");
  if (e1) RM_HIP(c, hipEventRecord(e1, c->stream));
  c->dispatched = true;
  return RM_OK;
}

int graph_frame(rm_ctx* c);

// Phase k of the frame (0 render start, 1 render end, 2 gather end, 3 assembly
// end) on the context's stream, when timing is on (rm_frame_phases).
int phase(rm_ctx* c, int k, hipStream_t st = nullptr) {
  if (!c->timing) return RM_OK;
  if (!c->ph[k]) RM_HIP(c, hipEventCreate(&c->ph[k]));
  RM_HIP(c, hipEventRecord(c->ph[k], st ? st : c->stream));
  return RM_OK;
}

// A multi-GPU context's frame: every device renders its shard (plainly or from
// its render-only graph), one grouped ncclGather collects the shards on device
// 0 (a single-process communicator needs the group), device 0 assembles.
int multi_frame(rm_ctx* c, bool graph) {
  if (c->comm_failed) return comm_dead(c);
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, err);
  const bool timed = !graph && c->subs[0]->timing;
  int rc = RM_OK;
  for (rm_ctx* s : c->subs) {
    s->u = c->u;
    if (timed && (rc = phase(s, 0)) != RM_OK) return fail(c, rc, s->err);
    rc = graph ? graph_frame(s) : render_launch(s);
    if (rc != RM_OK) return fail(c, rc, s->err);
    if (timed && (rc = phase(s, 1)) != RM_OK) return fail(c, rc, s->err);
  }
  ncclResult_t e = r->GroupStart();
  if (e != ncclSuccess) return comm_abort(c, std::string("ncclGroupStart: ") + r->GetErrorString(e));
  std::string why;
  for (rm_ctx* s : c->subs) {
    if ((rc = set_device(s)) != RM_OK || (rc = comm_gather(s)) != RM_OK) {
      why = s->err;
      break;
    }
  }
  e = r->GroupEnd();
  // a partial group: the gathers already queued on some devices can never
  // complete, so the communicator is aborted (not left to the deadline)
  if (rc != RM_OK) return comm_abort(c, "gather (partial group): " + why);
  if ((rc = comm_enqueued(c, r, e, "ncclGroupEnd (gather)")) != RM_OK) return rc;
  rm_ctx* s0 = c->subs[0];
  if ((rc = set_device(s0)) != RM_OK) return fail(c, rc, s0->err);
  if (timed && (rc = phase(s0, 2)) != RM_OK) return fail(c, rc, s0->err);
  if ((rc = comm_assemble(s0)) != RM_OK) return fail(c, rc, s0->err);
  if (timed && (rc = phase(s0, 3)) != RM_OK) return fail(c, rc, s0->err);
  s0->ph_recorded = timed || s0->ph_recorded;
  s0->ph_comm = true;
  c->dispatched = true;
  return RM_OK;
}


// ---- frame batches (rm_dispatch_frames) ------------------------------------------
// One launch renders n frames (grid.z = frame, rm_kernels.hip k_*_frames), so
// the waves of frame k + 1 fill the SIMDs that frame k's longest waves leave
// idle.  Frames 0..n-2 go to a ring of images the context keeps, frame n-1 to
// the context's image, so afterwards the context reads as after n rm_dispatch
// calls.  On a communicator context the n shards of one rank go to a batch slot
// and move in ONE ncclGather on the gather stream; rank 0 assembles the n
// frames there.  Two slots alternate, so batch j + 1 renders while batch j
// gathers, and all of a communicator's collectives stay on one stream in issue
// order.

// Images for frames 0..n-2 of a batch, `rows` x width, per enabled format.
int ensure_ring(rm_ctx* c, int n, int rows) {
  const size_t px = (size_t)rows * (size_t)c->cfg.width;
  while ((c->cfg.outputs & RM_OUT_RGBA8) && (int)c->ring8.size() < n - 1) {
    uint8_t* p = nullptr;
    RM_HIP(c, hipMalloc(&p, px * 4));
    c->ring8.push_back(p);
  }
  while ((c->cfg.outputs & RM_OUT_RGBA32F) && (int)c->ring32.size() < n - 1) {
    float* p = nullptr;
    RM_HIP(c, hipMalloc(&p, px * 16));
    c->ring32.push_back(p);
  }
  return RM_OK;
}

// The frame constants of frames[0..n) with their output pointers, launched in
// runs of one kernel: one AA setting, and for a runtime scene table one of its
// kernels (the specialised ones, or the generic one for a frame frame_jit
// refuses); one grid per run.  out8(k) / out32(k): frame k's destinations.
// (C++ linkage: this block sits inside the C-ABI's extern "C")
extern "C++" template <class O8, class O32>
int launch_batch(rm_ctx* c, const rm_uniforms* u, int n, O8 out8, O32 out32) {
  static thread_local rmd::FrameBatch B;  // 11.9 KB of kernel arguments
  int m = 0;
  const rm::JitTable* run_jit = nullptr;  // the run's table kernels: specialised, or null = generic
  auto flush = [&]() -> int {
    if (m == 0) return RM_OK;
    const hipError_t e = !c->nprims ? rm::launch_frames(B, m, c->stream)
                         : run_jit ? rm::launch_table_jit_frames(run_jit, B, m, c->stream)
                                   : rm::launch_table_frames(B, m, c->stream, table_slots(c), table_sl(c));
    m = 0;
    if (e != hipSuccess) return hip_fail(c, e, "batch launch");
    return RM_OK;
  };
  int rc = RM_OK;
  for (int k = 0; k < n; ++k) {
    c->u = u[k];
    rmd::Frame F = make_frame(c);
    F.rgba8 = out8(k);
    F.rgba32f = out32(k);
    F.sdf_counts = nullptr;
    F.counters = nullptr;
    const rm::JitTable* jit = c->nprims ? frame_jit(c, F) : nullptr;
    if (m > 0 && (B.f[0].aa != F.aa || jit != run_jit) && (rc = flush()) != RM_OK) return rc;
    run_jit = jit;
    B.f[m++] = F;
  }
  return flush();
}

int plain_batch(rm_ctx* c, const rm_uniforms* u, int n) {
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if ((rc = order_after_batch(c)) != RM_OK) return rc;
  if ((rc = ensure_ring(c, n, c->rows)) != RM_OK) return rc;
  uint8_t* dst8 = render_dst(c);
  float* dst32 = render_dst32(c);
  hipEvent_t e0, e1;
  if ((rc = timing_events(c, &e0, &e1)) != RM_OK) return rc;
  if (e0) RM_HIP(c, hipEventRecord(e0, c->stream));
  if ((rc = phase(c, 0)) != RM_OK) return rc;
  rc = launch_batch(
      c, u, n, [&](int k) { return dst8 ? (k < n - 1 ? c->ring8[k] : dst8) : nullptr; },
      [&](int k) { return dst32 ? (k < n - 1 ? c->ring32[k] : dst32) : nullptr; });
  if (rc != RM_OK) return rc;
  if ((rc = phase(c, 1)) != RM_OK) return rc;
  if (e1) {
    RM_HIP(c, hipEventRecord(e1, c->stream));
    c->ev_frames[c->ev_used - 1] = n;
  }
  if (c->timing) {
    c->ph_recorded = true;
    c->ph_comm = false;
  }
  c->batch_n = n;
  c->dispatched = true;
  return RM_OK;
}

// A communicator context's batch slot holding n frames: this rank's shards
// ([n][rows][width]), or on rank 0 the whole gather buffer ([nranks][n][rows]
// [width]).  Re-allocated only for a longer batch, after the slot's last
// gather has read it.
int slot_alloc(rm_ctx* c, rm_ctx::BatchSlot& b, int n) {
  if (!b.rendered) RM_HIP(c, hipEventCreateWithFlags(&b.rendered, hipEventDisableTiming));
  if (!b.freed) RM_HIP(c, hipEventCreateWithFlags(&b.freed, hipEventDisableTiming));
  if (b.cap >= n) return RM_OK;
  // the slot's last gather (gstream) and this rank's renders (stream) must be done
  // before its buffers go: on a communicator context that wait is the bounded poll
  // of every other communicator wait (a stalled peer is RM_ERR_COMM at the deadline,
  // ADVICE r04), not an unbounded event / stream synchronise
  if (c->comm) {
    const int rc = comm_wait(c);
    if (rc != RM_OK) return rc;
  } else {
    if (b.pending) RM_HIP(c, hipEventSynchronize(b.freed));
    RM_HIP(c, hipStreamSynchronize(c->stream));
  }
  if (b.send8) (void)hipFree(b.send8);
  if (b.send32) (void)hipFree(b.send32);
  b.send8 = nullptr;
  b.send32 = nullptr;
  b.cap = 0;
  const size_t px = (size_t)c->rows * (size_t)c->cfg.width * (size_t)n * (comm_root(c) ? c->cranks : 1);
  if (c->cfg.outputs & RM_OUT_RGBA8) RM_HIP(c, hipMalloc(&b.send8, px * 4));
  if (c->cfg.outputs & RM_OUT_RGBA32F) RM_HIP(c, hipMalloc(&b.send32, px * 16));
  b.cap = n;
  return RM_OK;
}

// Step 1 of a communicator batch: this rank's n shards in one launch, on the
// context's stream, into the next slot.
int batch_render(rm_ctx* c, const rm_uniforms* u, int n) {
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if ((rc = order_after_batch(c)) != RM_OK) return rc;
  if (!c->gstream) {
    RM_HIP(c, hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking));
    RM_HIP(c, hipEventCreateWithFlags(&c->gdone, hipEventDisableTiming));
  }
  rm_ctx::BatchSlot& b = c->bslot[c->bnext];
  if ((rc = slot_alloc(c, b, n)) != RM_OK) return rc;
  if (comm_root(c) && (rc = ensure_ring(c, n, c->cfg.height)) != RM_OK) return rc;
  // the slot's previous batch (two batches ago) has been gathered and assembled
  if (b.pending) RM_HIP(c, hipStreamWaitEvent(c->stream, b.freed, 0));
  const size_t px = (size_t)c->rows * (size_t)c->cfg.width;
  hipEvent_t e0, e1;
  if ((rc = timing_events(c, &e0, &e1)) != RM_OK) return rc;
  if (e0) RM_HIP(c, hipEventRecord(e0, c->stream));
  if ((rc = phase(c, 0)) != RM_OK) return rc;
  rc = launch_batch(
      c, u, n, [&](int k) { return b.send8 ? b.send8 + (size_t)k * px * bpp8(c) : nullptr; },
      [&](int k) { return b.send32 ? b.send32 + (size_t)k * px * 4 : nullptr; });
  if (rc != RM_OK) return rc;
  if ((rc = phase(c, 1)) != RM_OK) return rc;
  if (e1) {
    RM_HIP(c, hipEventRecord(e1, c->stream));
    c->ev_frames[c->ev_used - 1] = n;
  }
  RM_HIP(c, hipEventRecord(b.rendered, c->stream));
  return RM_OK;
}

// Step 2 (inside an RCCL group): the slot's n shards to rank 0 in one gather
// per format, on the gather stream once the render is done.
ncclResult_t batch_gather(rm_ctx* c, const rm::Rccl* r, int n) {
  if (set_device(c) != RM_OK) return ncclUnhandledCudaError;
  rm_ctx::BatchSlot& b = c->bslot[c->bnext];
  if (hipStreamWaitEvent(c->gstream, b.rendered, 0) != hipSuccess) return ncclUnhandledCudaError;
  const size_t px = (size_t)c->rows * (size_t)c->cfg.width * (size_t)n;
  const size_t count = px * 4;  // 4 floats per px
  const bool root = comm_root(c);
  ncclResult_t e = ncclSuccess;
  if (b.send8) e = r->Gather(b.send8, root ? b.send8 : nullptr, px * bpp8(c), ncclUint8, 0, c->comm, c->gstream);
  if ((e == ncclSuccess || e == ncclInProgress) && b.send32)
    e = r->Gather(b.send32, root ? b.send32 : nullptr, count, ncclFloat32, 0, c->comm, c->gstream);
  return e;
}

// Step 3, on the gather stream: rank 0 assembles the n frames (frames 0..n-2
// into its ring, frame n-1 into its image); another rank copies its last shard
// into its image, so the context reads as after n rm_dispatch calls.
int batch_finish(rm_ctx* c, int n) {
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  rm_ctx::BatchSlot& b = c->bslot[c->bnext];
  const size_t px = (size_t)c->rows * (size_t)c->cfg.width;
  if ((rc = phase(c, 2, c->gstream)) != RM_OK) return rc;
  if (comm_root(c)) {
    const int W = c->cfg.width, H = c->cfg.height, rb = c->cfg.row_block, rb0 = row_block0(c);
    const size_t stride = (size_t)n * (size_t)c->rows;  // rows between two ranks' blocks
    for (int k = 0; k < n; ++k) {
      if (b.send8) {
        void* dst = k < n - 1 ? (void*)c->ring8[k] : (void*)image_rgba8(c);
        const hipError_t e = rm::launch_unshard(b.send8 + (size_t)k * px * bpp8(c), dst, W, H, rb, rb0, c->cranks,
                                                c->rows, c->gstream, stride, c->rgb3);
        if (e != hipSuccess) return hip_fail(c, e, "unshard launch (batch)");
      }
      if (b.send32) {
        void* dst = k < n - 1 ? (void*)c->ring32[k] : (void*)c->d_frame32;
        const hipError_t e = rm::launch_unshard(b.send32 + (size_t)k * px * 4, dst, W * 4, H, rb, rb0,
                                                c->cranks, c->rows, c->gstream, stride);
        if (e != hipSuccess) return hip_fail(c, e, "unshard launch (batch, RGBA32F)");
      }
    }
  } else {
    if (b.send8 && render_dst(c))
      RM_HIP(c, hipMemcpyAsync(render_dst(c), b.send8 + (size_t)(n - 1) * px * bpp8(c), px * bpp8(c),
                               hipMemcpyDeviceToDevice, c->gstream));
    if (b.send32 && render_dst32(c))
      RM_HIP(c, hipMemcpyAsync(render_dst32(c), b.send32 + (size_t)(n - 1) * px * 4, px * 16,
                               hipMemcpyDeviceToDevice, c->gstream));
  }
  if ((rc = phase(c, 3, c->gstream)) != RM_OK) return rc;
  RM_HIP(c, hipEventRecord(b.freed, c->gstream));
  b.pending = true;
  RM_HIP(c, hipEventRecord(c->gdone, c->gstream));
  c->gdone_pending = true;
  if (c->timing) {
    c->ph_recorded = true;
    c->ph_comm = true;
  }
  c->blast = c->bnext;
  c->bnext ^= 1;
  c->batch_n = n;
  c->comm_warm = true;
  c->dispatched = true;
  return RM_OK;
}

// One rank's batch (rm_comm_init), or a multi-GPU context's (every device
// renders, one group gathers, device 0 assembles).
int comm_batch(rm_ctx* c, const rm_uniforms* u, int n) {
  if (c->comm_failed) return comm_dead(c);
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, err);
  const std::vector<rm_ctx*> ms = comm_members(c);
  int rc = RM_OK;
  for (rm_ctx* m : ms)
    if ((rc = batch_render(m, u, n)) != RM_OK) {
      if (m == c) return rc;
      // a member's communicator failed (its bounded slot wait): the frame's whole
      // group is aborted, as for any other member failure
      return rc == RM_ERR_COMM ? comm_abort(c, m->err) : fail(c, rc, m->err);
    }
  ncclResult_t e = r->GroupStart();
  if (e != ncclSuccess) return comm_abort(c, std::string("ncclGroupStart: ") + r->GetErrorString(e));
  for (rm_ctx* m : ms) {
    e = batch_gather(m, r, n);
    if (e != ncclSuccess && e != ncclInProgress) break;
  }
  const ncclResult_t eg = r->GroupEnd();
  if (e == ncclSuccess || e == ncclInProgress) e = eg;
  if ((rc = comm_enqueued(c, r, e, "ncclGather (batch)")) != RM_OK) return rc;
  for (rm_ctx* m : ms)
    if ((rc = batch_finish(m, n)) != RM_OK) return m == c ? rc : fail(c, rc, m->err);
  c->batch_n = n;
  c->dispatched = true;
  return RM_OK;
}
}  // namespace

int rm_dispatch(rm_ctx* c) {
  if (!c) return RM_ERR_INVALID;
  if (!c->subs.empty()) return multi_frame(c, false);
  if (c->comm_failed) return comm_dead(c);
  int rc;
  if ((rc = phase(c, 0)) != RM_OK) return rc;
  if ((rc = render_launch(c)) != RM_OK) return rc;
  if ((rc = phase(c, 1)) != RM_OK) return rc;
  // one rank of an RCCL-gathered frame: gather on rank 0, which assembles
  const bool comm = c->comm && !c->group_member;
  if (comm) {
    if ((rc = comm_gather(c)) != RM_OK) return rc;
    if ((rc = phase(c, 2)) != RM_OK) return rc;
    if ((rc = comm_assemble(c)) != RM_OK) return rc;
    if ((rc = phase(c, 3)) != RM_OK) return rc;
  }
  if (c->timing) {
    c->ph_recorded = true;
    c->ph_comm = comm;
  }
  return RM_OK;
}

int rm_dispatch_frames(rm_ctx* c, const rm_uniforms* u, int32_t n) {
  if (!c || !u) return RM_ERR_INVALID;
  if (n < 1 || n > RM_MAX_BATCH)
    return fail(c, RM_ERR_INVALID, "rm_dispatch_frames: n must be in 1.." + std::to_string(RM_MAX_BATCH));
  for (int k = 0; k < n; ++k) {
    const int rc = check_uniforms(c, u[k]);
    if (rc != RM_OK) return rc;
  }
  if (c->cfg.counters) return fail(c, RM_ERR_STATE, "rm_dispatch_frames: not available with counters");
  // launch_batch walks c->u (and every member's) through the frames; a failed
  // batch leaves the uniforms of the last successful dispatch
  const rm_uniforms before = c->u;
  int rc;
  if (has_comm(c) && !c->group_member) rc = comm_batch(c, u, n);
  else rc = plain_batch(c, u, n);
  const rm_uniforms& now = rc == RM_OK ? u[n - 1] : before;
  c->u = now;
  for (rm_ctx* s : c->subs) s->u = now;
  return rc;
}

int rm_synchronize(rm_ctx* c) {
  if (!c) return RM_ERR_INVALID;
  if (c->subs.empty()) {
    const int rc = set_device(c);
    if (rc != RM_OK) return rc;
  }
  return stream_wait(c);
}

// packed3: `dev` is an RGB8 shard image (rows of width x 3 bytes), read back as
// RGBA8 with alpha 255 (rm_config.shard_format).
static int read_image(rm_ctx* c, const void* dev, size_t bpp, void* dst, size_t row_pitch,
                      int flip_y, bool packed3 = false) {
  if (!c || !dst) return RM_ERR_INVALID;
  if (!dev) return fail(c, RM_ERR_STATE, "output format not enabled in rm_config.outputs");
  if (!c->dispatched) return fail(c, RM_ERR_STATE, "no dispatch yet");
  if (flip_y && !full_frame(c))
    return fail(c, RM_ERR_INVALID, "flip_y is not defined for a packed shard image");
  if (!c->subs.empty()) {  // the frame is on device 0, behind every device's stream
    const int rc = rm_synchronize(c);
    if (rc != RM_OK) return rc;
    c = c->subs[0];
  }
  const size_t w = (size_t)c->cfg.width * bpp;
  if (row_pitch == 0) row_pitch = w;
  if (row_pitch < w) return fail(c, RM_ERR_INVALID, "row_pitch smaller than a row");
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if ((rc = stream_wait(c)) != RM_OK) return rc;
  const size_t rows = (size_t)image_rows(c);
  if (packed3) {
    const size_t w3 = (size_t)c->cfg.width * 3;
    std::vector<uint8_t> tmp(w3 * rows);
    RM_HIP(c, hipMemcpy(tmp.data(), dev, tmp.size(), hipMemcpyDeviceToHost));
    for (size_t r = 0; r < rows; ++r) {
      const uint8_t* s3 = tmp.data() + r * w3;
      uint8_t* d4 = static_cast<uint8_t*>(dst) + r * row_pitch;
      for (int x = 0; x < c->cfg.width; ++x) {
        d4[4 * x] = s3[3 * x];
        d4[4 * x + 1] = s3[3 * x + 1];
        d4[4 * x + 2] = s3[3 * x + 2];
        d4[4 * x + 3] = 255;
      }
    }
    return RM_OK;  // (a shard image: flip_y was refused above)
  }
  RM_HIP(c, hipMemcpy2D(dst, row_pitch, dev, w, w, rows, hipMemcpyDeviceToHost));
  if (flip_y) {
    // Row 0 of the device image is the bottom row (quad.hpp:9); flip in place
    // so the top row comes first (image-file order).
    std::vector<char> tmp(w);
    char* base = static_cast<char*>(dst);
    for (size_t r = 0; r < rows / 2; ++r) {
      char* a = base + r * row_pitch;
      char* b = base + (rows - 1 - r) * row_pitch;
      std::memcpy(tmp.data(), a, w);
      std::memcpy(a, b, w);
      std::memcpy(b, tmp.data(), w);
    }
  }
  return RM_OK;
}

int rm_read_rgba8(rm_ctx* c, uint8_t* dst, size_t row_pitch, int flip_y) {
  if (!c) return RM_ERR_INVALID;
  return read_image(c, image_rgba8(c), 4, dst, row_pitch, flip_y, c->rgb3 && !full_frame(c));
}

int rm_read_rgba32f(rm_ctx* c, float* dst, size_t row_pitch, int flip_y) {
  if (!c) return RM_ERR_INVALID;
  return read_image(c, image_rgba32f(c), 16, dst, row_pitch, flip_y);
}

// Frame k of the last batch: the context's image for k = n-1; else rank 0's
// (or a plain context's) ring, or another rank's shard in the batch's slot.
static int read_frame(rm_ctx* c, int32_t k, bool f32, void* dst, size_t row_pitch, int flip_y) {
  if (!c) return RM_ERR_INVALID;
  rm_ctx* t = c->subs.empty() ? c : c->subs[0];
  const int n = t->batch_n;
  if (k < 0 || k >= n)
    return fail(c, RM_ERR_INVALID, "frame " + std::to_string(k) + " of a batch of " + std::to_string(n));
  if (k == n - 1) return f32 ? rm_read_rgba32f(c, (float*)dst, row_pitch, flip_y)
                             : rm_read_rgba8(c, (uint8_t*)dst, row_pitch, flip_y);
  const void* dev;
  if (t->comm && !comm_root(t)) {
    const rm_ctx::BatchSlot& b = t->bslot[t->blast];
    const size_t px = (size_t)t->rows * (size_t)t->cfg.width;
    dev = f32 ? (const void*)(b.send32 ? b.send32 + (size_t)k * px * 4 : nullptr)
              : (const void*)(b.send8 ? b.send8 + (size_t)k * px * bpp8(t) : nullptr);
  } else {
    dev = f32 ? (const void*)((size_t)k < t->ring32.size() ? t->ring32[k] : nullptr)
              : (const void*)((size_t)k < t->ring8.size() ? t->ring8[k] : nullptr);
  }
  return read_image(c, dev, f32 ? 16 : 4, dst, row_pitch, flip_y, !f32 && t->rgb3 && !full_frame(t));
}

int rm_read_frame_rgba8(rm_ctx* c, int32_t k, uint8_t* dst, size_t row_pitch, int flip_y) {
  return read_frame(c, k, false, dst, row_pitch, flip_y);
}

int rm_read_frame_rgba32f(rm_ctx* c, int32_t k, float* dst, size_t row_pitch, int flip_y) {
  return read_frame(c, k, true, dst, row_pitch, flip_y);
}

int rm_get_counters(rm_ctx* c, rm_counters* out) {
  if (!c || !out) return RM_ERR_INVALID;
  if (!c->cfg.counters) return fail(c, RM_ERR_STATE, "context created without counters");
  if (!c->dispatched) return fail(c, RM_ERR_STATE, "no dispatch yet");
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  unsigned long long h[8];
  RM_HIP(c, hipStreamSynchronize(c->stream));
  RM_HIP(c, hipMemcpy(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost));
  out->rays = h[0];
  out->march_steps = h[1];
  out->reflect_steps = h[2];
  out->shadow_steps = h[3];
  out->normals = h[4];
  out->lights = h[5];
  out->sdf_evals = h[1] + h[2] + h[3] + 4 * h[4];
  return RM_OK;
}

int rm_read_sdf_counts(rm_ctx* c, uint32_t* dst) {
  if (!c || !dst) return RM_ERR_INVALID;
  if (!c->cfg.counters) return fail(c, RM_ERR_STATE, "context created without counters");
  if (!c->dispatched) return fail(c, RM_ERR_STATE, "no dispatch yet");
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  RM_HIP(c, hipStreamSynchronize(c->stream));
  RM_HIP(c, hipMemcpy(dst, c->d_counts, (size_t)c->rows * c->cfg.width * 4, hipMemcpyDeviceToHost));
  return RM_OK;
}

// ---- hipGraph frame replay -----------------------------------------------------------
// Captures the frame once per AA setting / scene kernel / buffer set: the render
// kernel launch, and for one rank of an RCCL-gathered frame (rm_comm_init) the
// ncclGather and rank 0's assembly after it.  Each replay writes the frame's
// constants into the render node's by-value argument and launches the graph, so
// the graph path runs the same kernels as rm_dispatch at the same register
// budgets.  Counters and the wave-queue kernel are not available on this path.
static int graph_capture(rm_ctx* c, const rmd::Frame& F) {
  graph_release(c);
  rm_graph_slot& g = c->gs;
  const bool comm = c->comm && !c->group_member;
  hipStream_t cs = nullptr;
  RM_HIP(c, hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipStream_t keep = c->stream;
  int rc = RM_OK;
  hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
  if (e == hipSuccess) {
    e = !F.nprims ? rm::launch_pixel(F, false, cs)
        : frame_jit(c, F) ? rm::launch_table_jit(frame_jit(c, F), F, false, cs)
                  : rm::launch_table(F, false, cs, table_slots(c), table_sl(c));
    // the render node: the one node the next captured operation would depend on
    hipStreamCaptureStatus st;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    if (e == hipSuccess) e = hipStreamGetCaptureInfo_v2(cs, &st, nullptr, nullptr, &deps, &ndeps);
    if (e == hipSuccess && ndeps == 1) g.render = deps[0];
    else if (e == hipSuccess) e = hipErrorInvalidValue;
    if (e == hipSuccess && comm) {
      c->stream = cs;  // the gather and the assembly, captured after the render
      rc = comm_gather(c);
      if (rc == RM_OK) rc = comm_assemble(c);
      c->stream = keep;
    }
    hipGraph_t gr = nullptr;
    const hipError_t e2 = hipStreamEndCapture(cs, &gr);
    g.graph = gr;
    if (e == hipSuccess) e = e2;
  }
  if (e == hipSuccess && rc == RM_OK) e = hipGraphInstantiate(&g.exec, g.graph, nullptr, nullptr, 0);
  (void)hipStreamDestroy(cs);
  if (e != hipSuccess || rc != RM_OK) {
    if (rc == RM_OK) rc = hip_fail(c, e, "graph capture");
    graph_release(c);
    return rc;
  }
  g.send = render_dst(c);
  g.frame = image_rgba8(c);
  c->graph_aa = F.aa;
  c->graph_table = table_key(c);
  c->graph_jit = F.nprims ? frame_jit(c, F) : nullptr;
  return RM_OK;
}

int rm_graph_enable(rm_ctx* c, int enable) {
  if (!c) return RM_ERR_INVALID;
  for (rm_ctx* s : c->subs) {
    const int rc = rm_graph_enable(s, enable);
    if (rc != RM_OK) return fail(c, rc, s->err);
  }
  if (!c->subs.empty()) {
    c->graph_on = enable != 0;
    return RM_OK;
  }
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if (!enable) {
    graph_release(c);
    c->graph_on = false;
    return RM_OK;
  }
  if (c->cfg.counters) return fail(c, RM_ERR_STATE, "graph path does not collect counters");
  c->graph_on = true;
  return RM_OK;
}

namespace {
int graph_frame(rm_ctx* c) {
  if (c->comm_failed) return comm_dead(c);
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if ((rc = order_after_batch(c)) != RM_OK) return rc;
  rmd::Frame F = make_frame(c);
  const bool comm = c->comm && !c->group_member;
  if (comm && !c->comm_warm) {
    // RCCL sets a communicator's buffers up on its first operation, which must
    // not happen inside a capture: the first frame of a rank runs eagerly (every
    // rank takes the same branch, so the collective sequence matches)
    return rm_dispatch(c);
  }
  if ((F.aa != c->graph_aa || table_key(c) != c->graph_table ||
       (F.nprims ? frame_jit(c, F) : nullptr) != c->graph_jit || c->gs.send != render_dst(c) ||
       c->gs.frame != image_rgba8(c)) &&
      (rc = graph_capture(c, F)) != RM_OK)
    return rc;
  rm_graph_slot& g = c->gs;
  // a specialised table's render node is its batch kernel with one frame
  // (rm_jit.hpp launch_table_jit): its argument is a FrameBatch
  static thread_local rmd::FrameBatch GB;
  void* args[] = {&F};
  if (c->graph_jit) {
    GB.f[0] = F;
    args[0] = &GB;
  }
  hipKernelNodeParams kp;
  RM_HIP(c, hipGraphKernelNodeGetParams(g.render, &kp));
  kp.kernelParams = args;
  kp.extra = nullptr;
  RM_HIP(c, hipGraphExecKernelNodeSetParams(g.exec, g.render, &kp));
  hipEvent_t e0, e1;
  if ((rc = timing_events(c, &e0, &e1)) != RM_OK) return rc;
  if (e0) RM_HIP(c, hipEventRecord(e0, c->stream));
  RM_HIP(c, hipGraphLaunch(g.exec, c->stream));
  if (e1) RM_HIP(c, hipEventRecord(e1, c->stream));
  c->dispatched = true;
  return RM_OK;
}
}  // namespace

int rm_graph_dispatch(rm_ctx* c) {
  if (!c) return RM_ERR_INVALID;
  if (!c->graph_on) return fail(c, RM_ERR_STATE, "rm_graph_enable(ctx, 1) first");
  if (!c->subs.empty()) return multi_frame(c, true);
  return graph_frame(c);
}

// ---- runtime scene table ----------------------------------------------------------
int rm_set_scene(rm_ctx* c, const rm_primitive* prims, int32_t n) {
  if (!c) return RM_ERR_INVALID;
  if (!c->subs.empty()) {  // every device renders the same table
    for (rm_ctx* s : c->subs) {
      const int rc = rm_set_scene(s, prims, n);
      if (rc != RM_OK) return fail(c, rc, s->err);
    }
    c->nprims = c->subs[0]->nprims;
    c->scene = c->subs[0]->scene;
    return RM_OK;
  }
  if (!prims && n == 0) {  // back to the built-in scene
    c->nprims = 0;
    c->scene.clear();
    c->jit = nullptr;
    return RM_OK;
  }
  std::vector<uint32_t> words(rm::scene_words(n > 0 && n <= RM_MAX_PRIMITIVES ? n : 0));
  const char* why = "rm_set_scene: bad table";
  if (rm::compile_scene(prims, n, words.data(), &why) != RM_OK) return fail(c, RM_ERR_INVALID, why);
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  // compile first: a table whose specialisation fails leaves the context as it was
  const rm::JitTable* jit = nullptr;
  if (c->specialize) {
    std::string err;
    if ((rc = rm::jit_table(words.data(), n, &jit, err)) != RM_OK) return fail(c, rc, err);
    if (!jit->mod) jit = nullptr;  // no spill-free bound: the generic kernel
  }
  if (!c->d_scene) {
    RM_HIP(c, hipMalloc(&c->d_scene, rm::scene_words(RM_MAX_PRIMITIVES) * sizeof(uint32_t)));
  }
  // Ordered on the context's stream after the frames already queued (they keep
  // reading the previous table); the host copy must outlive the async copy, so
  // wait for it before the staging vector is replaced.
  RM_HIP(c, hipStreamSynchronize(c->stream));
  c->scene_words = std::move(words);
  RM_HIP(c, hipMemcpyAsync(c->d_scene, c->scene_words.data(), c->scene_words.size() * sizeof(uint32_t),
                           hipMemcpyHostToDevice, c->stream));
  c->scene.assign(prims, prims + n);
  c->nprims = n;
  c->jit = jit;
  return RM_OK;
}

int rm_scene_compile(const rm_primitive* prims, int32_t n, uint32_t* words, size_t capacity, size_t* nwords) {
  if (!nwords) return fail(nullptr, RM_ERR_INVALID, "rm_scene_compile: null nwords");
  *nwords = 0;
  if (n < 1 || n > RM_MAX_PRIMITIVES)
    return fail(nullptr, RM_ERR_INVALID, "rm_scene_compile: need 1..RM_MAX_PRIMITIVES primitives");
  std::vector<uint32_t> w(rm::scene_words(n));
  const char* why = "rm_scene_compile: bad table";
  if (rm::compile_scene(prims, n, w.data(), &why) != RM_OK) return fail(nullptr, RM_ERR_INVALID, why);
  *nwords = w.size();
  if (words) {
    if (capacity < w.size()) return fail(nullptr, RM_ERR_INVALID, "rm_scene_compile: capacity < *nwords");
    std::memcpy(words, w.data(), w.size() * sizeof(uint32_t));
  }
  return RM_OK;
}

int rm_scene_specialize(rm_ctx* c, int enable) {
  if (!c) return RM_ERR_INVALID;
  for (rm_ctx* s : c->subs) {
    const int rc = rm_scene_specialize(s, enable);
    if (rc != RM_OK) return fail(c, rc, s->err);
  }
  c->specialize = enable != 0;
  if (!c->subs.empty()) return RM_OK;
  if (!c->specialize) {
    c->jit = nullptr;
    return RM_OK;
  }
  if (!c->nprims || c->jit) return RM_OK;
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  std::string err;
  const rm::JitTable* jit = nullptr;
  if ((rc = rm::jit_table(c->scene_words.data(), c->nprims, &jit, err)) != RM_OK) {
    c->specialize = false;
    return fail(c, rc, err);
  }
  c->jit = jit->mod ? jit : nullptr;  // no spill-free bound: the generic kernel
  return RM_OK;
}

int rm_scene_kernel_waves(const rm_ctx* c, int32_t* waves) {
  if (!c || !waves) return RM_ERR_INVALID;
  const rm_ctx* r = c->subs.empty() ? c : c->subs[0];
  *waves = r->jit ? r->jit->waves : 0;
  return RM_OK;
}

int rm_get_scene(const rm_ctx* c, rm_primitive* out, int32_t capacity, int32_t* n) {
  if (!c || !n) return RM_ERR_INVALID;
  *n = c->nprims;
  if (out && c->nprims) {
    if (capacity < c->nprims) return RM_ERR_INVALID;
    std::memcpy(out, c->scene.data(), sizeof(rm_primitive) * c->nprims);
  }
  return RM_OK;
}

// ---- device interop ----------------------------------------------------------------
int rm_set_stream(rm_ctx* c, void* hip_stream) {
  if (!c) return RM_ERR_INVALID;
  if (!c->subs.empty())
    return fail(c, RM_ERR_STATE, "a multi-GPU context runs one stream per device (its own)");
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  if (c->own_stream && c->stream) {
    RM_HIP(c, hipStreamSynchronize(c->stream));
    (void)hipStreamDestroy(c->stream);
    c->stream = nullptr;
    c->own_stream = false;
  }
  if (hip_stream) {
    c->stream = static_cast<hipStream_t>(hip_stream);
  } else {
    RM_HIP(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  return RM_OK;
}

int rm_set_output_rgba8(rm_ctx* c, void* device_ptr) {
  if (!c) return RM_ERR_INVALID;
  if (!c->subs.empty()) {  // the frame's destination on device 0
    const int rc = rm_set_output_rgba8(c->subs[0], device_ptr);
    return rc == RM_OK ? rc : fail(c, rc, c->subs[0]->err);
  }
  if (!(c->cfg.outputs & RM_OUT_RGBA8))
    return fail(c, RM_ERR_STATE, "RGBA8 output not enabled in rm_config.outputs");
  c->ext_rgba8 = static_cast<uint8_t*>(device_ptr);
  return RM_OK;
}

int rm_get_output_rgba8(rm_ctx* c, void** device_ptr) {
  if (!c || !device_ptr) return RM_ERR_INVALID;
  *device_ptr = image_rgba8(c);
  return RM_OK;
}

// The images live on the context's device (a multi-GPU context's: device 0).
// Everything that writes them is on its stream, or for a communicator batch on
// its gather stream, which the stream itself waits for before any later write
// (order_after_batch); so the caller's stream waits for an event at the tail of
// each.
int rm_wait_output(rm_ctx* c, void* hip_stream) {
  if (!c) return RM_ERR_INVALID;
  rm_ctx* t = c->subs.empty() ? c : c->subs[0];
  if (t->comm_failed || c->comm_failed) return comm_dead(c);
  int rc = set_device(t);
  if (rc != RM_OK) return fail(c, rc, t->err);
  hipStream_t dst = static_cast<hipStream_t>(hip_stream);
  if (!t->out_ev) RM_HIP(c, hipEventCreateWithFlags(&t->out_ev, hipEventDisableTiming));
  RM_HIP(c, hipEventRecord(t->out_ev, t->stream));
  RM_HIP(c, hipStreamWaitEvent(dst, t->out_ev, 0));
  if (t->gstream) RM_HIP(c, hipStreamWaitEvent(dst, t->gdone, 0));
  return RM_OK;
}

int rm_unshard_rgba8(rm_ctx* c, const void* gathered_dev, void* frame_dev) {
  if (!c || !gathered_dev || !frame_dev) return RM_ERR_INVALID;
  if (!c->subs.empty()) return fail(c, RM_ERR_STATE, "a multi-GPU context assembles its own frames");
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  hipError_t e = rm::launch_unshard(gathered_dev, frame_dev, c->cfg.width, c->cfg.height,
                                    c->cfg.row_block, row_block0(c), c->cfg.nshards, c->rows, c->stream, 0,
                                    c->rgb3);
  if (e != hipSuccess) return hip_fail(c, e, "unshard launch");
  return RM_OK;
}

int rm_unshard_batch_rgba8(rm_ctx* c, const void* gathered_dev, int32_t k, int32_t n, void* frame_dev) {
  if (!c || !gathered_dev || !frame_dev) return RM_ERR_INVALID;
  if (n < 1 || k < 0 || k >= n) return fail(c, RM_ERR_INVALID, "rm_unshard_batch_rgba8: need 0 <= k < n");
  if (!c->subs.empty()) return fail(c, RM_ERR_STATE, "a multi-GPU context assembles its own frames");
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  const size_t px = (size_t)c->rows * (size_t)c->cfg.width;
  const uint8_t* src = static_cast<const uint8_t*>(gathered_dev) + (size_t)k * px * bpp8(c);
  hipError_t e = rm::launch_unshard(src, frame_dev, c->cfg.width, c->cfg.height, c->cfg.row_block,
                                    row_block0(c), c->cfg.nshards, c->rows, c->stream, (size_t)n * (size_t)c->rows,
                                    c->rgb3);
  if (e != hipSuccess) return hip_fail(c, e, "unshard launch");
  return RM_OK;
}

// A multi-GPU context times device 0's render kernel.
int rm_enable_timing(rm_ctx* c, int enable) {
  if (!c) return RM_ERR_INVALID;
  if (!c->subs.empty()) return rm_enable_timing(c->subs[0], enable);
  c->timing = enable != 0;
  return RM_OK;
}

int rm_kernel_time_ms(rm_ctx* c, double* total_ms, int64_t* launches, int reset) {
  if (!c) return RM_ERR_INVALID;
  if (!c->subs.empty()) {
    const int rc = rm_kernel_time_ms(c->subs[0], total_ms, launches, reset);
    return rc == RM_OK ? rc : fail(c, rc, c->subs[0]->err);
  }
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  for (size_t i = 0; i < c->ev_used; ++i) {
    RM_HIP(c, hipEventSynchronize(c->ev_pool[i].second));
    float ms = 0.0f;
    RM_HIP(c, hipEventElapsedTime(&ms, c->ev_pool[i].first, c->ev_pool[i].second));
    c->total_ms += ms;
    c->launches += i < c->ev_frames.size() ? c->ev_frames[i] : 1;  // a batch counts its frames
  }
  c->ev_used = 0;
  if (total_ms) *total_ms = c->total_ms;
  if (launches) *launches = c->launches;
  if (reset) {
    c->total_ms = 0.0;
    c->launches = 0;
  }
  return RM_OK;
}

// ---- one rank per process -------------------------------------------------------------
int rm_comm_unique_id(void* id, size_t size) {
  if (!id || size < sizeof(ncclUniqueId)) return fail(nullptr, RM_ERR_INVALID, "rm_comm_unique_id: buffer < 128 bytes");
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(nullptr, RM_ERR_HIP, "rm_comm_unique_id: " + err);
  ncclUniqueId u;
  const ncclResult_t e = r->GetUniqueId(&u);
  if (e != ncclSuccess) return fail(nullptr, RM_ERR_HIP, std::string("ncclGetUniqueId: ") + r->GetErrorString(e));
  std::memcpy(id, &u, sizeof u);
  return RM_OK;
}

namespace {
//  Every rank of a communicator must cut the frame the same way, or
// the gather's counts differ (a stall until the deadline) or k_unshard puts rows
// in the wrong places: the ranks exchange (width, height, row_block, rank 0's
// rows per round, outputs, shard format) with one ncclAllGather on the new
// communicator, and a rank that sees a difference aborts it (every rank sees the
// same table, so every rank fails the same way) with RM_ERR_INVALID.
int comm_check_layout(rm_ctx* c, const rm::Rccl* r) {
  constexpr int K = 6;
  const int32_t mine[K] = {c->cfg.width, c->cfg.height, c->cfg.row_block, row_block0(c), c->cfg.outputs,
                           c->rgb3 ? RM_SHARD_RGB8 : RM_SHARD_RGBA8};
  int32_t* d = nullptr;
  RM_HIP(c, hipMalloc(&d, sizeof(mine) * (size_t)c->cranks));
  std::vector<int32_t> all((size_t)K * c->cranks, 0);
  hipError_t he = hipMemcpyAsync(d + (size_t)K * c->crank, mine, sizeof mine, hipMemcpyHostToDevice, c->stream);
  ncclResult_t e = ncclSuccess;
  if (he == hipSuccess) e = r->AllGather(d + (size_t)K * c->crank, d, K, ncclInt32, c->comm, c->stream);
  int rc = he != hipSuccess ? hip_fail(c, he, "hipMemcpyAsync (layout)")
                            : comm_enqueued(c, r, e, "ncclAllGather (rm_comm_init layout check)");
  if (rc == RM_OK) rc = comm_wait(c);  // bounded: a rank that dies here is RM_ERR_COMM
  if (rc == RM_OK && (he = hipMemcpy(all.data(), d, all.size() * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess)
    rc = hip_fail(c, he, "hipMemcpy (layout)");
  (void)hipFree(d);
  if (rc != RM_OK) return rc;
  static const char* names[K] = {"width", "height", "row_block", "rank0_rows", "outputs", "shard_format"};
  for (int q = 0; q < c->cranks; ++q)
    for (int k = 0; k < K; ++k)
      if (all[(size_t)K * q + k] != all[k]) {
        const std::string why = std::string("rm_comm_init: ranks 0 and ") + std::to_string(q) + " disagree on " +
                                names[k] + " (" + std::to_string(all[k]) + " vs " +
                                std::to_string(all[(size_t)K * q + k]) + "): every rank must shard the frame alike";
        (void)comm_abort(c, why);
        return fail(c, RM_ERR_INVALID, why);
      }
  return RM_OK;
}
}  // namespace

int rm_comm_init(rm_ctx* c, const void* id, int32_t nranks, int32_t rank) {
  if (!c || !id) return RM_ERR_INVALID;
  if (!c->subs.empty()) return fail(c, RM_ERR_STATE, "a multi-GPU context has its own communicator");
  if (c->comm) return fail(c, RM_ERR_STATE, "the context already has a communicator");
  // an aborted context can only be destroyed (rm_api.h); a second init would
  // re-attach without freeing its gather buffers
  if (c->comm_failed) return comm_dead(c);
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return fail(c, RM_ERR_INVALID, "rm_comm_init: rank must be in 0..nranks-1");
  const int ns = c->cfg.nshards > 1 ? c->cfg.nshards : 1;
  if (ns != nranks || c->cfg.shard != rank)
    return fail(c, RM_ERR_INVALID, "rm_comm_init: the context must render shard `rank` of `nranks` "
                                   "(rm_config.shard / nshards)");
  if (check_comm_config(c->cfg, "rm_comm_init") != RM_OK) return fail(c, RM_ERR_INVALID, g_create_error);
  int rc = set_device(c);
  if (rc != RM_OK) return rc;
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, "rm_comm_init: " + err);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t comm = nullptr;
  // non-blocking init, polled against the deadline: a rank that never joins is
  // RM_ERR_COMM after comm_timeout_ms, not a host thread blocked forever
  ncclConfig_t nb = rm::nonblocking_config();
  ncclResult_t e = r->CommInitRankConfig(&comm, nranks, u, rank, &nb);
  if ((e == ncclSuccess || e == ncclInProgress) && comm) e = rm::wait_ready(r, &comm, 1, c->comm_timeout_ms);
  if (e != ncclSuccess) {
    if (comm) (void)r->CommAbort(comm);
    if (e == ncclInProgress)
      return fail(c, RM_ERR_COMM, "rm_comm_init: the communicator was not ready within " +
                                      std::to_string(c->comm_timeout_ms) +
                                      " ms (rm_comm_set_timeout): a rank never joined");
    return nccl_fail(c, r, e, "ncclCommInitRankConfig");
  }
  RM_HIP(c, hipStreamSynchronize(c->stream));  // frames already queued keep their buffers
  if ((rc = comm_attach(c, comm, rank, nranks, true, false)) != RM_OK) {
    (void)r->CommAbort(comm);  // this rank leaves: its peers see the abort
    c->comm = nullptr;
    return rc;
  }
  return comm_check_layout(c, r);
}

int rm_comm_set_timeout(rm_ctx* c, int32_t timeout_ms) {
  if (!c) return RM_ERR_INVALID;
  if (timeout_ms < 0) return fail(c, RM_ERR_INVALID, "rm_comm_set_timeout: timeout_ms must be >= 0");
  c->comm_timeout_ms = timeout_ms;
  for (rm_ctx* s : c->subs) s->comm_timeout_ms = timeout_ms;
  return RM_OK;
}

int rm_comm_check(rm_ctx* c) {
  if (!c) return RM_ERR_INVALID;
  if (c->comm_failed) return comm_dead(c);
  if (!has_comm(c)) return RM_OK;
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, err);
  for (rm_ctx* m : comm_members(c)) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t e = r->CommGetAsyncError(m->comm, &st);
    if (e != ncclSuccess || (st != ncclSuccess && st != ncclInProgress))
      return comm_abort(c, std::string("RCCL asynchronous error on device ") + std::to_string(m->device) + ": " +
                               r->GetErrorString(e != ncclSuccess ? e : st));
  }
  return RM_OK;
}

int rm_frame_phases(rm_ctx* c, double* render_ms, double* gather_ms, double* assemble_ms) {
  if (!c) return RM_ERR_INVALID;
  rm_ctx* t = c->subs.empty() ? c : c->subs[0];
  if (!t->ph_recorded) return fail(c, RM_ERR_STATE, "no timed eager dispatch yet (rm_enable_timing, rm_dispatch)");
  int rc = set_device(t);
  if (rc != RM_OK) return rc;
  if ((rc = stream_wait(c)) != RM_OK) return rc;
  (void)set_device(t);
  float ms[3] = {0.0f, 0.0f, 0.0f};
  RM_HIP(c, hipEventElapsedTime(&ms[0], t->ph[0], t->ph[1]));
  if (t->ph_comm) {
    RM_HIP(c, hipEventElapsedTime(&ms[1], t->ph[1], t->ph[2]));
    RM_HIP(c, hipEventElapsedTime(&ms[2], t->ph[2], t->ph[3]));
  }
  if (render_ms) *render_ms = ms[0];
  if (gather_ms) *gather_ms = ms[1];
  if (assemble_ms) *assemble_ms = ms[2];
  return RM_OK;
}

int rm_comm_info(const rm_ctx* c, int32_t* rank, int32_t* nranks, int32_t* ngpus) {
  if (!c) return RM_ERR_INVALID;
  if (rank) *rank = c->crank;
  if (nranks) *nranks = c->subs.empty() ? c->cranks : (int32_t)c->subs.size();
  if (ngpus) *ngpus = c->subs.empty() ? 1 : (int32_t)c->subs.size();
  return RM_OK;
}

int rm_comm_rccl_info(rm_ctx* c, int32_t* count, int32_t* user_rank, int32_t* hip_device, int32_t* version) {
  if (!c) return RM_ERR_INVALID;
  if (count) *count = 0;
  if (user_rank) *user_rank = -1;
  if (hip_device) *hip_device = -1;
  if (version) *version = 0;
  if (c->comm_failed) return comm_dead(c);
  if (!has_comm(c)) return RM_OK;
  std::string err;
  const rm::Rccl* r = rm::rccl(&err);
  if (!r) return fail(c, RM_ERR_COMM, err);
  int v = 0;
  if (version && r->GetVersion(&v) == ncclSuccess) *version = v;
  // every member communicator as RCCL formed it: a multi-GPU context's device i
  // must be user rank i of ngpus, a rank's communicator rank crank of cranks
  const std::vector<rm_ctx*> ms = comm_members(c);
  for (size_t i = 0; i < ms.size(); ++i) {
    int n = 0, ur = -1, dev = -1;
    ncclResult_t e = r->CommCount(ms[i]->comm, &n);
    if (e == ncclSuccess) e = r->CommUserRank(ms[i]->comm, &ur);
    if (e == ncclSuccess) e = r->CommCuDevice(ms[i]->comm, &dev);
    if (e != ncclSuccess) return nccl_fail(c, r, e, "ncclCommCount / ncclCommUserRank / ncclCommCuDevice");
    const int want_n = c->subs.empty() ? c->cranks : (int)ms.size();
    const int want_r = c->subs.empty() ? c->crank : (int)i;
    if (n != want_n || ur != want_r || dev != ms[i]->device)
      return fail(c, RM_ERR_COMM, "RCCL reports rank " + std::to_string(ur) + " of " + std::to_string(n) +
                                      " on device " + std::to_string(dev) + " for a member set up as rank " +
                                      std::to_string(want_r) + " of " + std::to_string(want_n) + " on device " +
                                      std::to_string(ms[i]->device));
    if (i == 0) {
      if (count) *count = n;
      if (user_rank) *user_rank = ur;
      if (hip_device) *hip_device = dev;
    }
  }
  return RM_OK;
}

}  // extern "C"
