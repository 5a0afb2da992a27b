// exhaustive_fp.hip — exhaustive bit-exactness proofs for the cheap f32
// sequences used by k_wavequeue.  For every input of the
// stated domain, each candidate is compared bit-for-bit with the compiler's
// correctly-rounded operation (HIP default -fhip-fp32-correctly-rounded-divide-sqrt).
//   sqrt candidates: all non-negative finite floats (0x00000000..0x7f7fffff)
//   x / C candidates: all finite floats, for the capsule constant C = dot(ba, ba)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/exhaustive_fp.hip -o tools/exhaustive_fp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../opengl-raymarching-in-compute-shader_amd/csrc/rm_fastmath.hpp"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr float CAP_BB = rmd::CAP_BB_HOST;

__global__ void k_sqrt(unsigned long long* bad, unsigned* first) {
  const unsigned long long n = 0x7f800000ull;  // all non-negative finite floats
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    float x = __uint_as_float((unsigned)i);
    float ref = __builtin_sqrtf(x);  // correctly rounded (compiler default)
    float c0 = __builtin_amdgcn_sqrtf(x);  // raw v_sqrt_f32
    float c1 = rmd::sqrt_cr_nonneg(x);      // librm's exact sequence
    // sqrt_core: exact on {0} U [2^-96, FLT_MAX] (its documented domain)
    float c2 = rmd::sqrt_core(x);
    if (x == 0.0f || x >= rmd::SQRT_CORE_MIN) {
      if (__float_as_uint(c2) != __float_as_uint(ref)) {
        atomicAdd(&bad[2], 1ull);
        atomicMin(&first[2], (unsigned)i);
      }
    } else if (!(c2 >= 0.0f && c2 < 0x1p-47f)) {
      // below 2^-96 sqrt_core must stay in [0, 2^-47): then RN(s - R) = -R for
      // every R in {3, 2.5, 1, 0.5} (rm_scene.hpp)
      atomicAdd(&bad[3], 1ull);
      atomicMin(&first[3], (unsigned)i);
    }
    if (__float_as_uint(c0) != __float_as_uint(ref)) {
      atomicAdd(&bad[0], 1ull);
      atomicMin(&first[0], (unsigned)i);
    }
    if (__float_as_uint(c1) != __float_as_uint(ref)) {
      atomicAdd(&bad[1], 1ull);
      atomicMin(&first[1], (unsigned)i);
    }
  }
}

__global__ void k_div(unsigned long long* bad, unsigned* first) {
  const unsigned long long n = 0x100000000ull;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    unsigned u = (unsigned)i;
    if ((u & 0x7f800000u) == 0x7f800000u) continue;  // inf/nan
    float x = __uint_as_float(u);
    volatile float cc = CAP_BB;
    float ref = x / cc;  // correctly rounded
    float c1 = rmd::div_capbb(x);
    if (__float_as_uint(c1) != __float_as_uint(ref)) {
      // region 0: |x| < 2^-100 (guarded by a slow path in librm), 1: the rest
      const int reg = (fabsf(x) < 0x1p-100f) ? 0 : 1;
      atomicAdd(&bad[reg], 1ull);
      atomicMin(&first[reg], u & 0x7fffffffu);
      atomicMax(&first[2 + reg], u & 0x7fffffffu);
    }
    if (fabsf(x) < 0x1p-100f) {
      // below 2^-100 div_capbb need not be exact but must stay tiny and keep the
      // sign: |q| <= 2^-104 and q*x >= 0 (rm_scene.hpp's capsule argument)
      if (!(fabsf(c1) <= 0x1p-104f && !(c1 * x < 0.0f) && !(c1 > 0.0f && x < 0.0f) &&
            !(c1 < 0.0f && x > 0.0f)))
        atomicAdd(&bad[2], 1ull);
    }
  }
}

int main() {
  unsigned long long* bad;
  unsigned* first;
  CK(hipMalloc(&bad, 4 * sizeof(unsigned long long)));
  CK(hipMalloc(&first, 4 * sizeof(unsigned)));
  CK(hipMemset(bad, 0, 4 * sizeof(unsigned long long)));
  CK(hipMemset(first, 0xff, 4 * sizeof(unsigned)));
  hipLaunchKernelGGL(k_sqrt, dim3(4096), dim3(256), 0, 0, bad, first);
  CK(hipDeviceSynchronize());
  unsigned long long hb[4];
  unsigned hf[4];
  CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  printf("sqrt  raw v_sqrt_f32 mismatches: %llu (first 0x%08x)\n", hb[0], hf[0]);
  printf("sqrt  sqrt_cr_nonneg mismatches: %llu (first 0x%08x)\n", hb[1], hf[1]);
  printf("sqrt  sqrt_core on {0}U[2^-96,max] mismatches: %llu (first 0x%08x)\n", hb[2], hf[2]);
  printf("sqrt  sqrt_core on (0,2^-96) outside [0,2^-47): %llu (first 0x%08x)\n", hb[3], hf[3]);
  const bool sqrt_ok = hb[1] == 0 && hb[2] == 0 && hb[3] == 0;
  CK(hipMemset(bad, 0, 4 * sizeof(unsigned long long)));
  CK(hipMemset(first, 0xff, 2 * sizeof(unsigned)));
  CK(hipMemset(first + 2, 0, 2 * sizeof(unsigned)));
  hipLaunchKernelGGL(k_div, dim3(4096), dim3(256), 0, 0, bad, first);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  printf("div   x/CAP_BB (%.9g) div_capbb mismatches |x|<2^-100: %llu (|x| bits 0x%08x..0x%08x)\n",
         (double)CAP_BB, hb[0], hf[0], hf[2]);
  printf("div   x/CAP_BB div_capbb mismatches |x|>=2^-100: %llu (|x| bits 0x%08x..0x%08x)\n",
         hb[1], hf[1], hf[3]);
  printf("div   |x|<2^-100: results not tiny or sign-flipped: %llu\n", hb[2]);
  return (sqrt_ok && hb[1] == 0 && hb[2] == 0) ? 0 : 1;
}
