// Diagnostic: per-wave lifetimes of one cfg-3 k_sample launch (RM_WAVE_TIMES):
// concurrency over time (waves alive / 8 per SIMD), dispatch gaps, tail.
// Build with -DRM_WAVE_STATS for per-wave counts of the RM_STAT points as well
// (their atomics slow the launch ~10x: lifetimes are then only relative).
#define RM_WAVE_TIMES 1
#include "../opengl-raymarching-in-compute-shader_amd/csrc/rm_kernels.hip"
#include "../opengl-raymarching-in-compute-shader_amd/csrc/rm_api.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
int main(int argc, char** argv) {
  const int W = 3840, H = 2160;
  const int nsh = argc > 1 ? atoi(argv[1]) : 1;  // optional: row-block shards (rank 0's shard)
  rm_config cfg;
  rm_config_init(&cfg, W, H);
  cfg.device = 0;
  cfg.kernel = RM_KERNEL_PIXEL;
  cfg.row_block = nsh > 1 ? 8 : 0;
  cfg.nshards = nsh;
  rm_ctx* c;
  if (rm_create(&c, &cfg)) return 1;
  int rows = H;
  rm_shard_rows(H, 8, 0, nsh, 0, nullptr, &rows);
  if (nsh <= 1) rows = H;
  const size_t nw = (size_t)(W / 4) * ((rows + 3) / 4);
  unsigned long long* d;
  hipMalloc(&d, nw * 3 * 8);
  hipMemset(d, 0, nw * 3 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(rmd::g_wave_times), &d, sizeof d);
  unsigned long long* ds = nullptr;  // per-wave counts of the RM_STAT points (RM_WAVE_STATS)
  hipMalloc(&ds, nw * 32 * 8);
  hipMemset(ds, 0, nw * 32 * 8);
#ifdef RM_WAVE_STATS
  hipMemcpyToSymbol(HIP_SYMBOL(rmd::g_wave_stats), &ds, sizeof ds);
#endif
  rm_uniforms u;
  rm_sweep_uniforms(30, 120, 3, 1, 0, &u);
  rm_set_uniforms(c, &u);
  rm_dispatch(c);  // warm
  rm_synchronize(c);
  hipMemset(ds, 0, nw * 32 * 8);
  rm_dispatch(c);
  rm_synchronize(c);
  std::vector<unsigned long long> h(nw * 3), hs(nw * 32);
  hipMemcpy(h.data(), d, nw * 3 * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hs.data(), ds, nw * 32 * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, t1 = 0;
  for (size_t w = 0; w < nw; ++w) { t0 = std::min(t0, h[3 * w]); t1 = std::max(t1, h[3 * w + 1]); }
  const double span = (double)(t1 - t0);  // wall_clock64 ticks (100 MHz)
  printf("waves %zu, span %.1f us\n", nw, span / 100.0);
  // concurrency histogram over 40 time bins
  const int NB = 40;
  std::vector<double> alive(NB, 0.0);
  double life = 0;
  for (size_t w = 0; w < nw; ++w) {
    const double a = (double)(h[3 * w] - t0), b = (double)(h[3 * w + 1] - t0);
    life += b - a;
    for (int k = 0; k < NB; ++k) {
      const double lo = span * k / NB, hi = span * (k + 1) / NB;
      const double ov = std::max(0.0, std::min(b, hi) - std::max(a, lo));
      alive[k] += ov / (hi - lo);
    }
  }
  printf("mean wave life %.2f us; mean resident %.0f waves = %.2f per SIMD (1024 SIMDs)\n",
         life / nw / 100.0, life / span, life / span / 1024.0);
  for (int k = 0; k < NB; ++k) printf("bin %2d  %.2f waves/SIMD\n", k, alive[k] / 1024.0);
  // per-slot gaps: group by hardware id (SE/SH/CU/SIMD/wave slot)
  std::vector<std::pair<unsigned, std::pair<unsigned long long, unsigned long long>>> v;
  for (size_t w = 0; w < nw; ++w) v.push_back({(unsigned)h[3 * w + 2], {h[3 * w], h[3 * w + 1]}});
  std::sort(v.begin(), v.end());
  double gap = 0; size_t ng = 0; std::vector<double> gaps;
  for (size_t i = 1; i < v.size(); ++i)
    if (v[i].first == v[i - 1].first && v[i].second.first >= v[i - 1].second.second) {
      const double g = (double)(v[i].second.first - v[i - 1].second.second);
      gap += g; ++ng; gaps.push_back(g);
    }
  std::sort(gaps.begin(), gaps.end());
  if (ng) printf("slot refill gaps: %zu, mean %.2f us, median %.2f us, p90 %.2f us\n", ng, gap / ng / 100.0,
                 gaps[ng / 2] / 100.0, gaps[ng * 9 / 10] / 100.0);
  // the last waves to finish: their tile row / column and lifetime
  std::vector<std::pair<unsigned long long, size_t>> ends;
  for (size_t w = 0; w < nw; ++w) ends.push_back({h[3 * w + 1], w});
  std::sort(ends.begin(), ends.end());
  const size_t gx = W / 4;
  printf("last 12 waves to finish (tile row of %d, col, start us, life us; wave-level counts of "
         "primary steps, reflected steps, lazy blocks, re-tests, shadow steps, bounce iterations, "
         "normals, shadows):\n", (rows + 3) / 4);
  auto counts = [&](size_t w) {
    const unsigned long long* q = &hs[32 * w];
    printf("  prim %llu refl %llu blk %llu rt %llu sh %llu bnc %llu nrm %llu shd %llu", q[15], q[6], q[9], q[1],
           q[2], q[26], q[27], q[29]);
  };
  for (size_t i = nw - 12; i < nw; ++i) {
    const size_t w = ends[i].second;
    printf("  row %4zu col %4zu start %7.1f life %6.1f", w / gx, w % gx, (h[3 * w] - t0) / 100.0,
           (h[3 * w + 1] - h[3 * w]) / 100.0);
    counts(w);
    printf("\n");
  }
  {  // the mean wave for comparison
    std::vector<double> m(32, 0.0);
    for (size_t w = 0; w < nw; ++w)
      for (int k = 0; k < 32; ++k) m[k] += (double)hs[32 * w + k] / nw;
    printf("mean wave: prim %.1f refl %.1f blk %.1f rt %.1f sh %.1f bnc %.2f nrm %.2f shd %.2f\n", m[15], m[6], m[9],
           m[1], m[2], m[26], m[27], m[29]);
  }
  // lifetime by tile-row band (10 bands)
  for (int b = 0; b < 10; ++b) {
    double s = 0, mx = 0; size_t n = 0;
    for (size_t w = 0; w < nw; ++w) {
      const size_t row = w / gx;
      if (row * 10 / ((rows + 3) / 4) != (size_t)b) continue;
      const double l = (h[3 * w + 1] - h[3 * w]) / 100.0;
      s += l; mx = std::max(mx, l); ++n;
    }
    printf("rows band %d: mean life %.1f us, max %.1f us\n", b, s / n, mx);
  }
  rm_destroy(c);
  return 0;
}
