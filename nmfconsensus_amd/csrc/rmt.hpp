// rmt.hpp -- R's default RNG (Mersenne-Twister, Inversion) for `set.seed(s); runif(N)` on the GPU.
//
// Used by the R-path initialisation of both engines: nmf.r:37-38 (`W = runif(m*k); H = runif(k*n)`
// under the BatchJobs job seed) for the MU engine, and NMF.div's `set.seed(rseed + i)` init for the
// Brunet engine.  Restates R's RNG.c: set.seed scrambles the seed with 50 LCG steps (69069 s + 1),
// fills the 625-word seed table with further LCG steps, and FixupSeeds sets mti = 624, so the first
// draw regenerates all 624 words; MT_genrand tempers and scales by 2^-32 and fixup() keeps the value
// inside (0, 1).  Bit-exact against R's published set.seed/runif values (tests/test_brunet_oracle.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rmt {

__device__ __forceinline__ uint32_t mt_step(uint32_t cur, uint32_t nxt, uint32_t far) {
  const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// set.seed(seed): mt[0..623] (thread 0 writes; caller synchronises)
__device__ __forceinline__ void seed_table(uint32_t* mt, uint32_t s) {
  for (int j = 0; j < 51; ++j) s = 69069u * s + 1u;   // 50 scrambling steps + the mti slot
  for (int j = 0; j < 624; ++j) {
    s = 69069u * s + 1u;
    mt[j] = s;
  }
}

// One 624-word regeneration by NT threads in four dependency phases: kk < 227 reads old words only;
// 227 <= kk < 454 and 454 <= kk < 623 read kk - 227 from the previous phase; kk = 623 reads 0 and 396.
template <int NT>
__device__ __forceinline__ void regenerate(uint32_t* mt) {
  static_assert(NT >= 227, "one word per thread and phase");
  const int tid = threadIdx.x;
  const int plo[4] = {0, 227, 454, 623}, phi[4] = {227, 454, 623, 624};
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    const int kk = plo[ph] + tid;
    const bool mine = kk < phi[ph];
    uint32_t v = 0;
    if (mine) v = mt_step(mt[kk], mt[kk == 623 ? 0 : kk + 1], mt[kk < 227 ? kk + 397 : kk - 227]);
    __syncthreads();
    if (mine) mt[kk] = v;
    __syncthreads();
  }
}

// tempering + MT_genrand scaling + fixup (unif_rand with min 0, max 1)
__device__ __forceinline__ double unif(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  double u = (double)y * 2.3283064365386963e-10;
  if (u <= 0.0) u = 0.5 * 2.328306437080797e-10;
  else if (1.0 - u <= 0.0) u = 1.0 - 0.5 * 2.328306437080797e-10;
  return u;
}

}  // namespace rmt
