// rm_jit.hip — per-table specialisation of the scene-table kernels (hiprtc).
//
// The reference compiles its compute shader from source at run time
// (CreateCompute, shader.hpp:186-197).  The analogue here: rm_scene_specialize
// makes rm_set_scene compile rm_table.hip once more, for the given table, with
// hiprtc.  The table's compiled words (rm::compile_scene) become a constant
// array of a generated header (RM_TABLE_STATIC, rm_table.hip), so every loop
// over the entries unrolls over compile-time types, masks and parameters.  The
// arithmetic is the same source under the same flags (-ffp-contract=off), so the
// image equals the generic table kernel's bit for bit (tests/test_gpu_scene.py).
//
// Register bound per table.  First compile: bounded to 8 waves per SIMD, kept
// when the production kernels spill at most kFewSpillBytes of scratch per lane
// (their kernel descriptors' private segment).  The reference scene's batch
// kernels need none there (round 6); in round 4 its single-frame kernels spilled
// 7 VGPRs (32 B) and still rendered a cfg3 frame 1.8 % faster than at the
// spill-free 7-wave bound (profiles/r04_spec_waves.txt), hence the allowance.  A
// table whose kernels fit 64 registers compiles the same as without a bound.  Otherwise the
// spill-free ladder: a compile without an occupancy bound (RM_TABLE_MIN_WAVES =
// 1), whose descriptors give each production kernel's VGPR allocation (a kernel
// allocating at most 512 / w registers runs at w waves with no scratch), and
// only for a table needing more than 80 registers one more, bounded to 6 waves,
// kept if it needs no scratch; one that spills even there is not specialised
// and renders with the generic (LDS-staged) kernel, whose registers do not grow
// with the table, and so does a table of more than kJitMaxEntries entries,
// without a compile (below).  The
// reference scene compiles once.  RM_JIT_LOG=1 prints one line
// per hiprtc compile (stderr).
//
// Modules are cached per (device, table words) for the life of the process:
// contexts rendering the same table (frames in flight) share one compile.
#include <elf.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "rm_internal.hpp"
#include "rm_jit.hpp"
#include "rm_scene.hpp"

namespace {
#include "rm_jit_src.inc"  // kJitSources: the table kernel's sources (build/, embed_sources.py)

std::mutex g_mu;
std::map<std::pair<int, std::string>, rm::JitTable*> g_cache;

// The counting kernels [aa] (JitTable::fnc), then the production batch kernels
// [aa] (JitTable::fnb).  A specialised table renders every production frame with
// the batch kernel, a single frame as a batch of one (round 6):
// the single-frame production kernel, whose whole Frame lives in SGPRs from the
// prologue on, spilled two VGPRs at the 8-wave bound (12 B of scratch per lane,
// 1.19x the image's HBM bytes) where the batch kernel, reading its frame at a
// run-time offset of the argument block, needs none.
const char* const kNames[2][2] = {{"rmd::k_table_pixel<true>", "rmd::k_table_sample<true>"},
                                  {"rmd::k_table_pixel_frames<>", "rmd::k_table_sample_frames<>"}};
constexpr int kProd[2] = {2, 3};  // the production kernels' indices in `lowered`
}  // namespace

namespace rm {

// The kernel descriptor `name`.kd of an AMDGPU code object (ELF64): the
// private_segment_fixed_size (u32 at offset 4; scratch bytes per lane) and the
// VGPR allocation per lane (compute_pgm_rsrc1 at offset 48, bits 5:0 =
// allocation / 8 - 1 on gfx950, VGPRs and AGPRs together).  false when absent.
bool kernel_desc(const std::vector<char>& code, const std::string& name, long* priv, int* vgprs) {
  if (code.size() < sizeof(Elf64_Ehdr)) return false;
  const char* base = code.data();
  const auto* eh = reinterpret_cast<const Elf64_Ehdr*>(base);
  if (std::memcmp(eh->e_ident, ELFMAG, SELFMAG) != 0 || eh->e_shoff == 0 ||
      eh->e_shoff + (size_t)eh->e_shnum * sizeof(Elf64_Shdr) > code.size())
    return false;
  const auto* sh = reinterpret_cast<const Elf64_Shdr*>(base + eh->e_shoff);
  const std::string kd = name + ".kd";
  for (int i = 0; i < eh->e_shnum; ++i) {
    if (sh[i].sh_type != SHT_SYMTAB || sh[i].sh_link >= eh->e_shnum) continue;
    const Elf64_Shdr& strs = sh[sh[i].sh_link];
    const size_t nsym = sh[i].sh_size / sizeof(Elf64_Sym);
    const auto* sym = reinterpret_cast<const Elf64_Sym*>(base + sh[i].sh_offset);
    for (size_t k = 0; k < nsym; ++k) {
      if (sym[k].st_name >= strs.sh_size || sym[k].st_shndx >= eh->e_shnum) continue;
      if (kd != base + strs.sh_offset + sym[k].st_name) continue;
      const Elf64_Shdr& sec = sh[sym[k].st_shndx];
      const size_t off = sec.sh_offset + (sym[k].st_value - sec.sh_addr);
      if (off + 64 > code.size()) return false;
      uint32_t p, rsrc1;
      std::memcpy(&p, base + off + 4, 4);
      std::memcpy(&rsrc1, base + off + 48, 4);
      *priv = (long)p;
      *vgprs = (int)((rsrc1 & 0x3fu) + 1u) * 8;
      return true;
    }
  }
  return false;
}

// Waves per SIMD a kernel allocating `vgprs` registers per lane can hold (512
// per SIMD lane, granule 8), capped at 8.
int waves_for(int vgprs) {
  const int w = vgprs > 0 ? 512 / vgprs : 8;
  return w < 8 ? w : 8;
}

// hiprtc: the table kernels for words[0..scene_words(n)) as a code object for
// `arch`, bounded to min_waves waves per SIMD.
int jit_compile_waves(const uint32_t* words, int32_t n, const std::string& arch, int min_waves,
                      std::vector<char>& code, std::vector<std::string>& lowered, std::string& err) {
  const size_t nw = scene_words(n);
  std::string hdr = "// generated by rm_jit.hip for one scene table\n#define RM_TS_N " + std::to_string(n) +
                    "\n__constant__ const unsigned int RM_TS_WORDS[" + std::to_string(nw) + "] = {";
  char buf[16];
  for (size_t i = 0; i < nw; ++i) {
    std::snprintf(buf, sizeof buf, "%s0x%08xu", i ? "," : "", words[i]);
    hdr += buf;
  }
  hdr += "};\n";
  const char* main_src = nullptr;
  std::vector<const char*> htext, hname;
  for (const auto& s : kJitSources) {
    if (std::strcmp(s.name, "rm_table.hip") == 0) {
      main_src = s.text;
    } else {
      htext.push_back(s.text);
      hname.push_back(s.name);
    }
  }
  htext.push_back(hdr.c_str());
  hname.push_back("rm_table_static.h");
  hiprtcProgram prog;
  if (!main_src || hiprtcCreateProgram(&prog, main_src, "rm_table.hip", (int)htext.size(), htext.data(),
                                       hname.data()) != HIPRTC_SUCCESS) {
    err = "rm_scene_specialize: hiprtcCreateProgram failed";
    return RM_ERR_HIP;
  }
  for (auto& row : kNames)
    for (const char* nm : row) hiprtcAddNameExpression(prog, nm);
  const std::string a = "--offload-arch=" + arch;
  const std::string w = "-DRM_TABLE_MIN_WAVES=" + std::to_string(min_waves);
  // -fno-slp-vectorize: as for librm's k_table_* and k_sample (Makefile): packed
  // f32 pairs measured 6.5 % slower for the reference scene's specialised kernel
#ifndef RM_JIT_EXTRA
#define RM_JIT_EXTRA "-DRM_JIT_PLAIN=1"  // diagnostic builds pass e.g. "-DRM_TDBL_SHADOW=1"
#endif
  const char* opts[] = {a.c_str(), "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
                        "-DRM_TABLE_STATIC=1", w.c_str(), RM_JIT_EXTRA};
  if (const char* lg = std::getenv("RM_JIT_LOG"); lg && *lg == '1')
    std::fprintf(stderr, "rm_jit: hiprtc compile, %d-entry table, occupancy bound %d waves\n", n, min_waves);
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)(sizeof opts / sizeof opts[0]), opts);
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    err = "rm_scene_specialize: hiprtc compile failed: " + log.substr(0, 4000);
    hiprtcDestroyProgram(&prog);
    return RM_ERR_HIP;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code.resize(cs);
  hiprtcGetCode(prog, code.data());
  lowered.clear();
  for (auto& row : kNames)
    for (const char* nm : row) {
      const char* low = nullptr;
      if (hiprtcGetLoweredName(prog, nm, &low) != HIPRTC_SUCCESS || !low) {
        hiprtcDestroyProgram(&prog);
        err = "rm_scene_specialize: kernel name not found";
        return RM_ERR_HIP;
      }
      lowered.emplace_back(low);
    }
  hiprtcDestroyProgram(&prog);
  return RM_OK;
}

// Waves per SIMD the production kernels (the batch kernels, kProd) of a
// compiled code object run at, or 0 when any needs scratch;
// -1 (with err) when a descriptor is missing: that is an error, not a spill, as
// silently falling back to the generic kernel would hide a code-object layout
// change.
int production_waves(const std::vector<char>& c, const std::vector<std::string>& l, std::string& err) {
  int w = 8;
  for (int k : kProd) {
    long priv = -1;
    int vg = 0;
    if (!kernel_desc(c, l[k], &priv, &vg)) {
      err = "rm_scene_specialize: kernel descriptor " + l[k] + ".kd not found in the compiled code object";
      return -1;
    }
    if (priv != 0) return 0;
    const int wk = waves_for(vg);
    w = wk < w ? wk : w;
  }
  return w;
}

// The largest scratch bytes per lane of the production kernels, or -1 (with
// err) when a descriptor is missing.
long production_scratch(const std::vector<char>& c, const std::vector<std::string>& l, std::string& err) {
  long most = 0;
  for (int k : kProd) {
    long priv = -1;
    int vg = 0;
    if (!kernel_desc(c, l[k], &priv, &vg)) {
      err = "rm_scene_specialize: kernel descriptor " + l[k] + ".kd not found in the compiled code object";
      return -1;
    }
    most = priv > most ? priv : most;
  }
  return most;
}

constexpr long kFewSpillBytes = 32;  // 8 spilled VGPRs per lane
// Larger tables are not compiled: the unrolled kernels' registers grow with the
// table, and past a dozen entries hiprtc spends minutes producing spill code that
// fits no bound (the reference scene's objects repeated, on the build host's
// CPU: 12 entries 26 s, one compile that fits 8 waves; 16 entries 261 s for the
// 8-wave compile alone, 3.7 MB of code, and 786 s for the ladder, which ends
// on the generic kernel; round 6, with the single-frame production kernels no
// longer compiled: 12 entries 22 s, 16 entries 509 s for the ladder, still ending
// on the generic kernel: 88 VGPRs and 400 B of scratch at 8 waves, spills at 6).
// They render with the generic kernel at once.  RM_JIT_MAX_ENTRIES (a build
// define) moves the cap for such measurements.
#ifndef RM_JIT_MAX_ENTRIES
#define RM_JIT_MAX_ENTRIES 12
#endif
constexpr int32_t kJitMaxEntries = RM_JIT_MAX_ENTRIES;

// The table kernels at their register bound (above): *waves is the waves per
// SIMD they run at, or 0 (code left empty) when no bound fits.
int jit_compile(const uint32_t* words, int32_t n, const std::string& arch, std::vector<char>& code,
                std::vector<std::string>& lowered, std::string& err, int* waves) {
  if (waves) *waves = 0;
  code.clear();
  if (n > kJitMaxEntries) return RM_OK;
  std::vector<char> c;
  std::vector<std::string> l;
  if (const char* fw = std::getenv("RM_JIT_FORCE_WAVES"); fw && *fw) {
    // diagnostic A/Bs only: this bound whatever scratch it costs
    const int wf = std::atoi(fw);
    const int rf = jit_compile_waves(words, n, arch, wf, c, l, err);
    if (rf != RM_OK) return rf;
    code.swap(c);
    lowered.swap(l);
    if (waves) *waves = wf;
    return RM_OK;
  }
  int rc = jit_compile_waves(words, n, arch, 8, c, l, err);
  if (rc != RM_OK) return rc;
  const long sc = production_scratch(c, l, err);
  if (sc < 0) return RM_ERR_HIP;
  if (const char* lg = std::getenv("RM_JIT_LOG"); lg && *lg == '1') {
    //  which kernels set the bound: the production batch kernels,
    // which render single frames too (kNames)
    for (int k : kProd) {
      long priv = 0;
      int vg = 0;
      if (kernel_desc(c, l[k], &priv, &vg))
        std::fprintf(stderr, "rm_jit:   8-wave bound: %s %d VGPRs, %ld B scratch\n", l[k].c_str(), vg, priv);
    }
  }
  if (sc <= kFewSpillBytes) {
    code.swap(c);
    lowered.swap(l);
    if (waves) *waves = 8;
    return RM_OK;
  }
  rc = jit_compile_waves(words, n, arch, 1, c, l, err);
  if (rc != RM_OK) return rc;
  int w = production_waves(c, l, err);
  if (w < 0) return RM_ERR_HIP;
  if (w >= 6) {  // usable as it is
    code.swap(c);
    lowered.swap(l);
  }
  if (w < 6) {
    // more than 80 registers unbounded: one compile bounded to 6 waves, kept
    // when it needs no scratch
    rc = jit_compile_waves(words, n, arch, 6, c, l, err);
    if (rc != RM_OK) return rc;
    const int wb = production_waves(c, l, err);
    if (wb < 0) return RM_ERR_HIP;
    if (wb >= 6) {
      code.swap(c);
      lowered.swap(l);
      w = wb;
    }
  }
  if (w < 6) {
    code.clear();
    w = 0;
  }
  if (waves) *waves = w;
  return RM_OK;
}

int jit_table(const uint32_t* words, int32_t n, const JitTable** out, std::string& err) {
  const size_t nw = scene_words(n);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    err = "rm_scene_specialize: hipGetDevice failed";
    return RM_ERR_HIP;
  }
  const auto key = std::make_pair(dev, std::string(reinterpret_cast<const char*>(words), nw * 4));
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    *out = it->second;
    return RM_OK;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    err = "rm_scene_specialize: hipGetDeviceProperties failed";
    return RM_ERR_HIP;
  }
  std::string arch = prop.gcnArchName;
  arch = arch.substr(0, arch.find(':'));  // gfx950
  std::vector<char> code;
  std::vector<std::string> lowered;
  int waves = 0;
  int rc = jit_compile(words, n, arch, code, lowered, err, &waves);
  if (rc != RM_OK) return rc;
  auto* j = new JitTable();
  j->waves = waves;
  if (waves == 0) {  // no spill-free bound: the generic kernel renders this table
    g_cache.emplace(key, j);
    *out = j;
    return RM_OK;
  }
  hipError_t e = hipModuleLoadData(&j->mod, code.data());
  for (int k = 0; k < 2 && e == hipSuccess; ++k)
    e = hipModuleGetFunction(&j->fnc[k], j->mod, lowered[k].c_str());
  for (int k = 0; k < 2 && e == hipSuccess; ++k)
    e = hipModuleGetFunction(&j->fnb[k], j->mod, lowered[kProd[k]].c_str());
  if (e != hipSuccess) {
    if (j->mod) (void)hipModuleUnload(j->mod);
    delete j;
    err = std::string("rm_scene_specialize: module load failed: ") + hipGetErrorString(e);
    return RM_ERR_HIP;
  }
  g_cache.emplace(key, j);
  *out = j;
  return RM_OK;
}

hipError_t launch_table_jit(const JitTable* j, const rmd::Frame& F, bool counters, hipStream_t s) {
  if (!counters) {
    // production: the batch kernel over a batch of one (kNames)
    static thread_local rmd::FrameBatch B;
    B.f[0] = F;
    return launch_table_jit_frames(j, B, 1, s);
  }
  void* args[] = {const_cast<rmd::Frame*>(&F)};
  if (F.aa)
    return hipModuleLaunchKernel(j->fnc[1], (F.width + 3) / 4, (F.rows + 3) / 4, 1, 64, 1, 1, 0, s, args, nullptr);
  return hipModuleLaunchKernel(j->fnc[0], (F.width + 7) / 8, (F.rows + 7) / 8, 1, 64, 1, 1, 0, s, args, nullptr);
}

hipError_t launch_table_jit_frames(const JitTable* j, const rmd::FrameBatch& B, int n, hipStream_t s) {
  if (n < 1 || n > rmd::kMaxBatch) return hipErrorInvalidValue;
  const rmd::Frame& F = B.f[0];
  void* args[] = {const_cast<rmd::FrameBatch*>(&B)};
  if (F.aa)
    return hipModuleLaunchKernel(j->fnb[1], (F.width + 3) / 4, (F.rows + 3) / 4, n, 64, 1, 1, 0, s, args, nullptr);
  return hipModuleLaunchKernel(j->fnb[0], (F.width + 7) / 8, (F.rows + 7) / 8, n, 64, 1, 1, 0, s, args, nullptr);
}

}  // namespace rm

// Diagnostics: the specialised code object for a table, compiled without a
// device (hiprtc cross-compiles), e.g. to inspect its ISA or to check on a
// machine without a GPU that a table specialises.  *size = 0 (RM_OK): the table
// fits no spill-free bound and would render with the generic kernel.
extern "C" int rm_jit_code_object(const rm_primitive* prims, int32_t n, const char* arch, void* out,
                                  size_t capacity, size_t* size) {
  if (!prims || !arch || !size || n < 1 || n > RM_MAX_PRIMITIVES) return RM_ERR_INVALID;
  std::vector<uint32_t> words(rm::scene_words(n));
  const char* why = nullptr;
  if (rm::compile_scene(prims, n, words.data(), &why) != RM_OK) return RM_ERR_INVALID;
  std::vector<char> code;
  std::vector<std::string> lowered;
  std::string err;
  const int rc = rm::jit_compile(words.data(), n, arch, code, lowered, err, nullptr);
  if (rc != RM_OK) {
    std::fprintf(stderr, "%s\n", err.c_str());
    return rc;
  }
  *size = code.size();
  if (code.empty()) return RM_OK;
  if (out && capacity >= code.size()) std::memcpy(out, code.data(), code.size());
  return out && capacity < code.size() ? RM_ERR_INVALID : RM_OK;
}
