// exhaustive_fp.hip — exhaustive bit-exactness proofs for the cheap f32
// sequences used by the render kernels.  For every input of the
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

// Direction of raw v_sqrt_f32's error on [2^-96, FLT_MAX]: counts of inputs where
// the correctly rounded result is s (exact), s - 1 ulp (overshoot), s + 1 ulp
// (undershoot), or further away.  One-sided errors allow a one-fma correction.
__global__ void k_sqrt_dir(unsigned long long* cnt) {
  const unsigned long long lo = 0x0f800000ull, n = 0x7f800000ull;  // 2^-96 .. FLT_MAX
  unsigned long long c[4] = {0, 0, 0, 0};
  for (unsigned long long i = lo + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((unsigned)i);
    const int d = (int)__float_as_uint(__builtin_sqrtf(x)) - (int)__float_as_uint(__builtin_amdgcn_sqrtf(x));
    c[d == 0 ? 0 : d == -1 ? 1 : d == 1 ? 2 : 3]++;
  }
  for (int k = 0; k < 4; ++k) atomicAdd(&cnt[k], c[k]);
}

// Candidate cheaper exact sqrt sequences, counted against the CR sqrt on [2^-96, max].
__device__ __forceinline__ float cand_rsq_newton(float x) {  // rsq, s = x y, one Newton step
  const float y = __builtin_amdgcn_rsqf(x);
  const float s = x * y;
  const float h = 0.5f * y;
  const float r = __builtin_fmaf(-s, s, x);
  return __builtin_fmaf(h, r, s);
}
__device__ __forceinline__ float cand_sqrt_newton(float x) {  // v_sqrt, residual, rcp step
  const float s = __builtin_amdgcn_sqrtf(x);
  const float r = __builtin_fmaf(-s, s, x);
  return __builtin_fmaf(r, 0.5f * __builtin_amdgcn_rcpf(s), s);
}
__global__ void k_sqrt_cand(unsigned long long* cnt, unsigned* first) {
  const unsigned long long lo = 0x0f800000ull, n = 0x7f800000ull;
  unsigned long long c[2] = {0, 0};
  for (unsigned long long i = lo + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((unsigned)i);
    const unsigned ref = __float_as_uint(__builtin_sqrtf(x));
    if (__float_as_uint(cand_rsq_newton(x)) != ref) { c[0]++; atomicMin(&first[0], (unsigned)i); }
    if (__float_as_uint(cand_sqrt_newton(x)) != ref) { c[1]++; atomicMin(&first[1], (unsigned)i); }
  }
  atomicAdd(&cnt[0], c[0]);
  atomicAdd(&cnt[1], c[1]);
}

// 1/x candidate: v_rcp_f32 plus one Newton step, against the IEEE division.
__device__ __forceinline__ float cand_rcp_newton(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}
__global__ void k_rcp_cand(unsigned long long* cnt, unsigned* first) {
  unsigned long long c[2] = {0, 0};
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < 0x100000000ull;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned u = (unsigned)i;
    if ((u & 0x7f800000u) == 0x7f800000u || (u & 0x7fffffffu) == 0) continue;  // inf/nan/0
    const float x = __uint_as_float(u);
    volatile float one = 1.0f;
    const unsigned ref = __float_as_uint(one / x);
    const int reg = (fabsf(x) >= 0x1p-125f && fabsf(x) <= 0x1p125f) ? 0 : 1;
    if (__float_as_uint(cand_rcp_newton(x)) != ref) {
      c[reg]++;
      atomicMin(&first[reg], u & 0x7fffffffu);
    }
  }
  atomicAdd(&cnt[0], c[0]);
  atomicAdd(&cnt[1], c[1]);
}

// x / 3 and x / 5 (bounce weights 1/i, glsl:186-187) by the Markstein sequence
// (the candidate librm measured and did not adopt: rm_fastmath.hpp div_small is
// the IEEE division), against the IEEE division, over all finite x.
__device__ __forceinline__ float cand_div_small(float x, int i) {
  const float d = (float)i;
  const float y = (i == 3) ? (1.0f / 3.0f) : (1.0f / 5.0f);
  const float q = x * y;
  const float r = __builtin_fmaf(-q, d, x);
  return q == 0.0f ? q : __builtin_fmaf(r, y, q);  // keeps -0 / 3 == -0
}
__global__ void k_div_small(unsigned long long* cnt, unsigned* first) {
  unsigned long long c[4] = {0, 0, 0, 0};
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < 0x100000000ull;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned u = (unsigned)i;
    if ((u & 0x7f800000u) == 0x7f800000u) continue;
    const float x = __uint_as_float(u);
    volatile float d3 = 3.0f, d5 = 5.0f;
    const int reg = fabsf(x) >= 0x1p-100f ? 0 : 1;
    if (__float_as_uint(cand_div_small(x, 3)) != __float_as_uint(x / d3)) { c[reg]++; atomicMin(&first[reg], u & 0x7fffffffu); }
    if (__float_as_uint(cand_div_small(x, 5)) != __float_as_uint(x / d5)) { c[2 + reg]++; atomicMin(&first[2 + reg], u & 0x7fffffffu); }
  }
  for (int k = 0; k < 4; ++k) atomicAdd(&cnt[k], c[k]);
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
  hipLaunchKernelGGL(k_sqrt_dir, dim3(4096), dim3(256), 0, 0, bad);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  printf("sqrt  v_sqrt_f32 on [2^-96,max]: exact %llu, over by 1ulp %llu, under by 1ulp %llu, other %llu\n",
         hb[0], hb[1], hb[2], hb[3]);
  CK(hipMemset(bad, 0, 4 * sizeof(unsigned long long)));
  CK(hipMemset(first, 0xff, 4 * sizeof(unsigned)));
  hipLaunchKernelGGL(k_sqrt_cand, dim3(4096), dim3(256), 0, 0, bad, first);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  printf("sqrt  candidate rsq+Newton on [2^-96,max] mismatches: %llu (first 0x%08x)\n", hb[0], hf[0]);
  printf("sqrt  candidate sqrt+rcp Newton on [2^-96,max] mismatches: %llu (first 0x%08x)\n", hb[1], hf[1]);
  CK(hipMemset(bad, 0, 4 * sizeof(unsigned long long)));
  CK(hipMemset(first, 0xff, 4 * sizeof(unsigned)));
  hipLaunchKernelGGL(k_rcp_cand, dim3(4096), dim3(256), 0, 0, bad, first);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  printf("rcp   candidate rcp+Newton 1/x on 2^-125<=|x|<=2^125 mismatches: %llu (first |x| 0x%08x)\n", hb[0], hf[0]);
  printf("rcp   candidate rcp+Newton 1/x outside that range mismatches: %llu (first |x| 0x%08x)\n", hb[1], hf[1]);
  CK(hipMemset(bad, 0, 4 * sizeof(unsigned long long)));
  CK(hipMemset(first, 0xff, 4 * sizeof(unsigned)));
  hipLaunchKernelGGL(k_div_small, dim3(4096), dim3(256), 0, 0, bad, first);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
  printf("div   div_small x/3 mismatches |x|>=2^-100: %llu, |x|<2^-100: %llu (first |x| 0x%08x)\n", hb[0], hb[1], hf[1]);
  printf("div   div_small x/5 mismatches |x|>=2^-100: %llu, |x|<2^-100: %llu (first |x| 0x%08x)\n", hb[2], hb[3], hf[3]);
  const bool small_ok = hb[0] == 0 && hb[1] == 0 && hb[2] == 0 && hb[3] == 0;
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
  return (sqrt_ok && small_ok && hb[1] == 0 && hb[2] == 0) ? 0 : 1;
}
