// valu_peak.hip — the VALU issue peak that bench.py's roofline divides by,
// measured on the box ("verify both on the box").
//
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o tools/valu_peak tools/valu_peak.hip
//   (no SLP: plain v_fma_f32 / v_add_f32, not packed pairs, as k_sample is built)
//   tools/valu_peak            -> one line per instruction kind
//
// Each kernel runs 8 waves per SIMD on every CU (one-wave workgroups, 64
// VGPRs at most) and issues long streams of independent wave64 instructions of
// one kind (8 independent accumulators per lane, so no dependent stall): the
// rate is lane-instructions per second over the whole chip, to compare with
// 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz = 78.64 T (a wave64 plain VALU op issues
// over 2 cycles, MI355X_MICROARCH.md).  The clock under that load comes from
// s_memtime (shader cycles) against the HIP-event wall time.  A dependent chain
// (one accumulator per lane) at 8 waves/SIMD shows how far latency alone keeps
// the SIMD from its issue peak.  Diagnostic tool, not part of the product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kIters = 256;   // loop trips per wave
constexpr int kAcc = 8;       // independent accumulators per lane
constexpr int kRep = 16;      // kAcc-instruction groups per trip: 128 VALU between two
                              // branches, so the taken branch's refetch is amortised

enum Kind { FMA = 0, ADD = 1, SQRT = 2, MIX = 3, DEP = 4, ADDMUL = 5, FMAADD = 6,
            // one instruction kind each, written in asm so nothing folds
            A_MUL = 8, A_MIN = 9, A_MIN3 = 10, A_MOV = 11, A_CND = 12, A_CMP = 13, A_U32 = 14, A_E64 = 15,
            // operand sources: VGPR, SGPR, literal, inline constant
            O_VV = 16, O_VS = 17, O_VL = 18, O_VI = 19, O_FMAVVV = 20, O_FMAVSV = 21, O_FMAC = 22,
            O_MULL = 23, O_MAXVV = 24, O_CNDS = 25, O_SUB = 26, O_CMPS = 27, O_FMAVVL = 28,
            // integer min / max and bit operations on float bit patterns (round 6)
            I_MINI = 29, I_MAXI = 30, I_MINU = 31, I_MAXU = 32, I_AND = 33, I_OR = 34, I_MAX3I = 35,
            I_MED3 = 36, I_PKADD = 37 };

template <int K>
__global__ __launch_bounds__(64, 8) void k_issue(float* out, unsigned long long* clk, float s) {
  float a[kAcc];
#pragma unroll
  for (int j = 0; j < kAcc; ++j) a[j] = (float)(threadIdx.x + j) * 1e-3f + 1.0f;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int jj = 0; jj < kAcc * kRep; ++jj) {
      const int j = jj % kAcc;
      if (K == FMA) a[j] = __builtin_fmaf(a[j], s, 0.5f);
      if (K == ADD) a[j] = a[j] + s;
      if (K == SQRT) a[j] = __builtin_amdgcn_sqrtf(a[j]);
      if (K == MIX) a[j] = (j == 0) ? __builtin_amdgcn_sqrtf(a[j]) : __builtin_fmaf(a[j], s, 0.5f);
      if (K == DEP) a[0] = __builtin_fmaf(a[0], s, 0.5f);  // one dependent chain
      // mixed streams: does the SIMD issue two kinds of VALU op per slot?
      if (K == ADDMUL) a[j] = (j & 1) ? a[j] * s : a[j] + s;
      if (K == FMAADD) a[j] = (j & 1) ? __builtin_fmaf(a[j], s, 0.5f) : a[j] + s;
      const float b = a[(j + 1) % kAcc], c = a[(j + 2) % kAcc];
      if (K == A_MUL) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == A_MIN) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == A_MIN3) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (K == A_MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(b));
      if (K == A_CND) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b));
      if (K == A_CMP) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(a[j]), "v"(b) : "vcc");
      if (K == A_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == O_VV) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == O_VS) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[j]) : "s"(s));
      if (K == O_VL) asm volatile("v_add_f32 %0, 0x3f8ccccd, %0" : "+v"(a[j]));
      if (K == O_VI) asm volatile("v_add_f32 %0, 0.5, %0" : "+v"(a[j]));
      if (K == O_FMAVVV) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (K == O_FMAVSV) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "s"(s), "v"(c));
      if (K == O_FMAC) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (K == O_MULL) asm volatile("v_mul_f32 %0, 0x358637bd, %0" : "+v"(a[j]));
      if (K == O_MAXVV) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == O_CNDS) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[2:3]" : "+v"(a[j]) : "v"(b) : "s2", "s3");
      if (K == O_SUB) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == O_CMPS) asm volatile("v_cmp_lt_f32_e64 s[2:3], %0, %1" : : "v"(a[j]), "v"(b) : "s2", "s3");
      if (K == O_FMAVVL) asm volatile("v_fmamk_f32 %0, %0, 0x3f7ff000, %1" : "+v"(a[j]) : "v"(b));
      if (K == A_E64) asm volatile("v_add_f32_e64 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_MINI) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_MAXI) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_MINU) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_MAXU) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_AND) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_OR) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (K == I_MAX3I) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (K == I_MED3) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (K == I_PKADD && (j & 1) == 0) {
        // one v_pk_add_f32 per two accumulators (a wave64 packed op covers both)
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*reinterpret_cast<double*>(&a[j])) : "v"(*reinterpret_cast<const double*>(&a[(j + 2) % kAcc])));
      }
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  float r = 0.0f;
#pragma unroll
  for (int j = 0; j < kAcc; ++j) r += a[j];
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) clk[blockIdx.x] = c1 - c0;
}

template <int K>
void run(const char* name, int nblk, float* out, unsigned long long* clk) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_issue<K>, dim3(nblk), dim3(64), 0, 0, out, clk, 0.999f);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_issue<K>, dim3(nblk), dim3(64), 0, 0, out, clk, 0.999f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.0f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  unsigned long long* h = (unsigned long long*)std::malloc(sizeof(unsigned long long) * nblk);
  CK(hipMemcpy(h, clk, sizeof(unsigned long long) * nblk, hipMemcpyDeviceToHost));
  double cyc = 0.0, cmin = 1e30, cmax = 0.0;
  for (int b = 0; b < nblk; ++b) {
    cyc += (double)h[b];
    cmin = h[b] < cmin ? (double)h[b] : cmin;
    cmax = h[b] > cmax ? (double)h[b] : cmax;
  }
  cyc /= nblk;  // shader cycles per wave's loop (s_memtime counts shader clocks)
  std::free(h);
  // VALU instructions per wave in the loop: kAcc * kRep per trip (DEP: dependent ones)
  const double per_wave = (double)kIters * kAcc * kRep;
  const double lane_instr = per_wave * 64.0 * nblk;
  const double rate_T = lane_instr / (ms * 1e-3) / 1e12;
  // one wave's loop time against the kernel time: the clock the loop ran at
  // (all waves resident at once: nblk = 8 waves x SIMDs)
  const double ghz = cyc / (ms * 1e-3) / 1e9;
  const double cyc_per_instr_simd = cyc / (per_wave * 8.0);  // 8 waves share a SIMD
  std::printf("%-5s waves %d  kernel %.4f ms  %.2f T lane-instr/s  loop clock %.2f GHz  "
              "%.2f cycles per wave-instruction per SIMD  (wave loop min/max %.0f/%.0f)\n",
              name, nblk, ms, rate_T, ghz, cyc_per_instr_simd, cmin, cmax);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char**) {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int nblk = p.multiProcessorCount * 4 * 8;  // 8 one-wave workgroups per SIMD
  std::printf("device %s, %d CUs, peak clock %.2f GHz -> plain-VALU issue peak %.2f T lane-instr/s\n",
              p.gcnArchName, p.multiProcessorCount, p.clockRate / 1e6,
              p.multiProcessorCount * 4.0 * 32.0 * (p.clockRate / 1e6) / 1e3);
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, sizeof(float) * 64 * nblk));
  CK(hipMalloc(&clk, sizeof(unsigned long long) * nblk));
  if (argc > 1) {  // the round-6 kinds only
    run<I_MINI>("min.i32", nblk, out, clk);
    run<I_MAXI>("max.i32", nblk, out, clk);
    run<I_MINU>("min.u32", nblk, out, clk);
    run<I_MAXU>("max.u32", nblk, out, clk);
    run<I_AND>("and.b32", nblk, out, clk);
    run<I_OR>("or.b32", nblk, out, clk);
    run<I_MAX3I>("max3.i32", nblk, out, clk);
    run<I_MED3>("med3.f32", nblk, out, clk);
    run<I_PKADD>("pkadd(x2)", nblk, out, clk);
    run<O_MAXVV>("max.vv", nblk, out, clk);
    run<A_U32>("u32", nblk, out, clk);
    return 0;
  }
  run<FMA>("fma", nblk, out, clk);
  run<ADD>("add", nblk, out, clk);
  run<SQRT>("sqrt", nblk, out, clk);
  run<MIX>("mix", nblk, out, clk);  // 1 v_sqrt per 7 v_fma
  run<DEP>("dep", nblk, out, clk);
  run<ADDMUL>("a+m", nblk, out, clk);
  run<FMAADD>("f+a", nblk, out, clk);
  run<A_MUL>("mul", nblk, out, clk);
  run<A_MIN>("min", nblk, out, clk);
  run<A_MIN3>("min3", nblk, out, clk);
  run<A_MOV>("mov", nblk, out, clk);
  run<A_CND>("cnd", nblk, out, clk);
  run<A_CMP>("cmp", nblk, out, clk);
  run<A_U32>("u32", nblk, out, clk);
  run<A_E64>("adde64", nblk, out, clk);
  run<O_VV>("add.vv", nblk, out, clk);
  run<O_VS>("add.vs", nblk, out, clk);
  run<O_VL>("add.vlit", nblk, out, clk);
  run<O_VI>("add.vinl", nblk, out, clk);
  run<O_FMAVVV>("fma.vvv", nblk, out, clk);
  run<O_FMAVSV>("fma.vsv", nblk, out, clk);
  run<O_FMAC>("fmac.vv", nblk, out, clk);
  run<O_MULL>("mul.lit", nblk, out, clk);
  run<O_MAXVV>("max.vv", nblk, out, clk);
  run<O_CNDS>("cnd.sgpr", nblk, out, clk);
  run<O_SUB>("sub.vv", nblk, out, clk);
  run<O_CMPS>("cmp.sgpr", nblk, out, clk);
  run<O_FMAVVL>("fmamk", nblk, out, clk);
  CK(hipFree(out));
  CK(hipFree(clk));
  return 0;
}
