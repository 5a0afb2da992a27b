// rm_shard.hpp — the weighted row interleave of a sharded frame (SURVEY 8(e);
// include/rm_api.h rm_shard_rows).  One definition for the host (rm_host.cpp's
// pure functions, the shard sizes of rm_api.hip) and the device (rm_scene.hpp
// global_row, rm_kernels.hip k_unshard).
//
// Rows go in rounds of P = rb0 + (n - 1) rb rows: shard 0 owns the first rb0
// rows of a round, shard s >= 1 the rb rows after rb0 + (s - 1) rb.  Shard s
// packs its rows in round order.  Per-row cost varies ~50x around the horizon
// (SURVEY 8(e)), so rounds stay short (64 rows at n = 8, rb = 8) and every
// shard samples every band of the image.  Shard 0 is the root of the gather
// and also assembles the frame; rb0 < rb gives it that much less to render
// (DESIGN §7).  rb0 = rb is the plain interleave: block b to shard b % n.
#pragma once

#if defined(__HIP__) || defined(__HIPCC_RTC__)
#define RM_HD __host__ __device__ __forceinline__
#else
#define RM_HD inline
#endif

namespace rm {

struct ShardMap {
  int rb;   // rows per round of every shard but 0
  int rb0;  // rows per round of shard 0
  int n;    // shards (>= 2)
};

RM_HD int shard_period(const ShardMap& m) { return m.rb0 + (m.n - 1) * m.rb; }
RM_HD int shard_width(const ShardMap& m, int s) { return s == 0 ? m.rb0 : m.rb; }
RM_HD int shard_offset(const ShardMap& m, int s) { return s == 0 ? 0 : m.rb0 + (s - 1) * m.rb; }

// Global row of local row l of shard s (>= height for the padding rows at the
// end of a shard image).
RM_HD int shard_row(const ShardMap& m, int s, int l) {
  const int w = shard_width(m, s);
  const int k = l / w;
  return k * shard_period(m) + shard_offset(m, s) + (l - k * w);
}

// The shard and local row holding global row y (the inverse of shard_row).
RM_HD void shard_owner(const ShardMap& m, int y, int* s, int* l) {
  const int P = shard_period(m);
  const int k = y / P;
  int j = y - k * P;
  if (j < m.rb0) {
    *s = 0;
    *l = k * m.rb0 + j;
  } else {
    j -= m.rb0;
    const int q = j / m.rb;
    *s = 1 + q;
    *l = k * m.rb + (j - q * m.rb);
  }
}

// Real rows of shard s in a frame of `height` rows.
RM_HD int shard_real_rows(const ShardMap& m, int height, int s) {
  const int P = shard_period(m), K = height / P, rem = height - K * P;
  const int w = shard_width(m, s), part = rem - shard_offset(m, s);
  return K * w + (part <= 0 ? 0 : (part < w ? part : w));
}

// Rows of every shard image: the largest shard's rounds times its rows per
// round (shard 0, or shard 1, whose rounds reach at least as far as any later
// shard's), so the padding rows of every shard map past the frame.
RM_HD int shard_rows_cap(const ShardMap& m, int height) {
  const int P = shard_period(m), K = height / P, rem = height - K * P;
  const int c0 = (K + (rem > 0 ? 1 : 0)) * m.rb0;
  const int c1 = (K + (rem > m.rb0 ? 1 : 0)) * m.rb;
  return c0 > c1 ? c0 : c1;
}

}  // namespace rm
