// Diagnostic: wave clock cycles per render phase of k_sample (cfg 3 frame),
// from RM_PHASE_TIMING hooks in rm_kernels.hip.  Phase 8 is the whole
// per-wave render (ray setup .. AA reduce); the remainder is setup + gamma.
#define RM_PHASE_TIMING 1
#include "../opengl-raymarching-in-compute-shader_amd/csrc/rm_kernels.hip"
#include "../opengl-raymarching-in-compute-shader_amd/csrc/rm_api.hip"
#include "../opengl-raymarching-in-compute-shader_amd/csrc/rm_wavequeue.hip"
#include <cstdio>
#include <cstdlib>
int main(int argc, char** argv) {
  const int bounces = argc > 1 ? atoi(argv[1]) : 3;
  const int aa = argc > 2 ? atoi(argv[2]) : 1;
  const int W = argc > 3 ? atoi(argv[3]) : 3840, H = argc > 4 ? atoi(argv[4]) : 2160;
  rm_config cfg = {W, H, 0, RM_OUT_RGBA8, RM_KERNEL_PIXEL, 0, 0, 0, 1};
  rm_ctx* c;
  if (rm_create(&c, &cfg)) { printf("create failed %s\n", rm_last_error(nullptr)); return 1; }
  const char* nm[] = {"primary march", "primary normal", "primary light", "primary shadow",
                      "bounce march", "bounce normal", "bounce light", "bounce shadow", "whole render"};
  unsigned long long tot[16] = {0};
  for (int f = 0; f < 120; f += 12) {
    rm_uniforms u; rm_sweep_uniforms(f, 120, bounces, aa, 0, &u); rm_set_uniforms(c, &u);
    unsigned long long z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(rmd::g_phase), z, sizeof z);
    rm_dispatch(c); rm_synchronize(c);
    unsigned long long h[16];
    hipMemcpyFromSymbol(h, HIP_SYMBOL(rmd::g_phase), sizeof h);
    for (int k = 0; k < 16; ++k) tot[k] += h[k];
  }
  double sum = 0;
  for (int k = 0; k < 8; ++k) sum += (double)tot[k];
  printf("bounces %d aa %d %dx%d, 10 sweep frames\n", bounces, aa, W, H);
  for (int k = 0; k < 9; ++k)
    printf("%-16s %16llu  %5.1f%%\n", nm[k], tot[k], 100.0 * tot[k] / (double)tot[8]);
  printf("%-16s %16.0f  %5.1f%%\n", "other", (double)tot[8] - sum, 100.0 * ((double)tot[8] - sum) / tot[8]);
  rm_destroy(c);
  return 0;
}
