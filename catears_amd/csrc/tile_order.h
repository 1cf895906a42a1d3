// tile_order.h -- XCD-aware, L2-friendly block -> output tile mapping shared
// by the GEMM kernels (device code).
#pragma once

#include <hip/hip_runtime.h>

namespace catears {

// XCD-aware tile order.  Blocks b, b+8, b+16, ... run on one XCD
// (round-robin dispatch), so each XCD gets a contiguous run of a global tile
// order, and that order walks compact 2-D blocks: groups of `group` column
// tiles, row blocks inside a group, columns inside a row.  For the 3072 x 1024
// layers at 64 x 128 tiles an XCD's 64 tiles are then a 16 x 4 block: it
// fetches 16 A row panels and 4 weight panels into its L2 (~19 MB) instead
// of all of A (51 MB) under a plain column-major order.  Bijective for any
// grid (a speed choice, never correctness).
__device__ __forceinline__ void tile_of(int b, int tiles_m, int tiles_n, int group, int *tm, int *tn) {
  const int nwg = tiles_m * tiles_n, q = nwg / 8, r = nwg % 8, xcd = b % 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
  const int per_group = group * tiles_m;
  const int g = t / per_group, rem = t - g * per_group;
  const int w = min(group, tiles_n - g * group);  // the last group may be narrower
  const int rb = rem / w;
  *tm = rb;
  *tn = g * group + (rem - rb * w);
}

}  // namespace catears
