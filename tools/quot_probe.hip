// Probe: how close the Brunet kernels' quotient sequences come to IEEE a / p on gfx950 (standalone; not part of
// the product library).  For N pseudo-random pairs (a >= 0, p > 0 over wide exponent ranges) it counts results
// that differ from the correctly rounded quotient for
//   q2: v_rcp_f64, two Newton steps, residual correction  (csrc/brunet.hip quot(), the shipped form)
//   q1: v_rcp_f64, ONE Newton step, residual correction
//   qb: the batched form (csrc/brunet.hip recip_batch): the reciprocals of 4 consecutive p from ONE v_rcp_f64 of their
//       product (prefix products, one Newton step, back-multiplication), then the same residual correction
// and reports the largest relative error of v_rcp_f64 itself (against 1 / p).  `rate` mode (argv[2] == "rate") times
// independent v_rcp_f64 against v_fma_f64 chains instead (issue cycles of the quarter-rate reciprocal).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <string>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// a double with a random 52-bit mantissa and an exponent uniform in [e0, e1]
__device__ __forceinline__ double rnd(uint64_t z, int e0, int e1) {
  const uint64_t man = z & ((1ull << 52) - 1);
  const int e = e0 + (int)((z >> 52) % (uint64_t)(e1 - e0 + 1));
  return __longlong_as_double((long long)(((uint64_t)(e + 1023) << 52) | man));
}

__global__ void probe(long n, uint64_t seed, int ea0, int ea1, int ep0, int ep1, unsigned long long* cnt,
                      double* maxrel) {
  unsigned long long c1 = 0, c2 = 0, cb = 0;
  double mr = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double a = rnd(mix(seed ^ (2 * i)), ea0, ea1);
    const double p = rnd(mix(seed ^ (2 * i + 1)), ep0, ep1);
    const double q = a / p;   // IEEE (the compiler's div_scale / div_fmas / div_fixup sequence)
    const double r0 = __builtin_amdgcn_rcp(p);
    mr = fmax(mr, fabs(fma(-p, r0, 1.0)));
    double e = fma(-p, r0, 1.0);
    const double r1 = fma(r0, e, r0);
    e = fma(-p, r1, 1.0);
    const double r2 = fma(r1, e, r1);
    const double t2 = a * r2, q2 = fma(fma(-p, t2, a), r2, t2);
    const double t1 = a * r1, q1 = fma(fma(-p, t1, a), r1, t1);
    c2 += q2 != q;
    c1 += q1 != q;
    // batch of 4: this p and the next three draws of the same stream
    double pb[4], rb[4], cpre[4];
    pb[0] = p;
#pragma unroll
    for (int j = 1; j < 4; ++j) pb[j] = rnd(mix(seed ^ (2 * i + 1 + 2 * (long)n * j)), ep0, ep1);
    cpre[0] = pb[0];
#pragma unroll
    for (int j = 1; j < 4; ++j) cpre[j] = cpre[j - 1] * pb[j];
    double u = __builtin_amdgcn_rcp(cpre[3]);
    u = fma(u, fma(-cpre[3], u, 1.0), u);
#pragma unroll
    for (int j = 3; j > 0; --j) {
      rb[j] = u * cpre[j - 1];
      u = u * pb[j];
    }
    rb[0] = u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double tb = a * rb[j], qb = fma(fma(-pb[j], tb, a), rb[j], tb);
      cb += qb != a / pb[j];
    }
  }
  atomicAdd(&cnt[0], c1);
  atomicAdd(&cnt[1], c2);
  atomicAdd(&cnt[2], cb);
  // the largest |1 - p r0| over the grid: doubles >= 0 order like their bit patterns
  atomicMax((unsigned long long*)maxrel, (unsigned long long)__double_as_longlong(mr));
}

// rate: every lane runs 8 independent chains of the same instruction (x = rcp(x) or x = fma(x, y, z)) for `it` steps
template <bool RCP>
__global__ __launch_bounds__(256) void rate(int it, double* out) {
  double x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = 1.0 + 1e-3 * (threadIdx.x + j);
  const double y = 0.999999, z = 1e-9;
  for (int s = 0; s < it; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = RCP ? __builtin_amdgcn_rcp(x[j]) : fma(x[j], y, z);
  }
  double v = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) v += x[j];
  if (v == 12345.0) out[threadIdx.x] = v;   // keeps the chains live
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : (1L << 30);
  if (argc > 2 && std::string(argv[2]) == "rate") {
    double* o;
    CK(hipMalloc(&o, 256 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = 20000, blocks = 256 * 8;   // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    for (int rep = 0; rep < 3; ++rep)
      for (int which = 0; which < 2; ++which) {
        CK(hipEventRecord(e0));
        if (which) rate<true><<<blocks, 256>>>(it, o); else rate<false><<<blocks, 256>>>(it, o);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // wave-instructions per SIMD: blocks * 4 waves / 1024 SIMDs * it * 8
        const double per_simd = (double)blocks * 4 / 1024 * it * 8;
        printf("%s: %.3f ms, %.3f ns per wave-instruction per SIMD\n", which ? "v_rcp_f64" : "v_fma_f64", ms,
               ms * 1e6 / per_simd);
      }
    return 0;
  }
  struct Range { const char* what; int ea0, ea1, ep0, ep1; } rs[] = {
      {"a in [2^-4, 2^4), p in [2^-4, 2^4)", -4, 3, -4, 3},
      {"a in [2^-30, 2^10), p in [2^-60, 2^10)", -30, 9, -60, 9},
      {"a in [2^-1, 2^1), p in [2^-1, 2^1)", -1, 0, -1, 0},
  };
  unsigned long long* cnt;
  double* mr;
  CK(hipMalloc(&cnt, 3 * sizeof(unsigned long long)));
  CK(hipMalloc(&mr, sizeof(double)));
  for (const Range& r : rs) {
    CK(hipMemset(cnt, 0, 3 * sizeof(unsigned long long)));
    CK(hipMemset(mr, 0, sizeof(double)));
    probe<<<4096, 256>>>(n, 0x5EEDull + (uint64_t)r.ep0, r.ea0, r.ea1, r.ep0, r.ep1, cnt, mr);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long h[3];
    double m;
    CK(hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&m, mr, sizeof m, hipMemcpyDeviceToHost));
    printf("%-42s %ld pairs: one Newton step %llu differ from a / p, two steps %llu, batches of 4 %llu (of %ld); "
           "max |1 - p rcp(p)| = %.3g (2^%.1f)\n",
           r.what, n, h[0], h[1], h[2], 4 * n, m, m > 0 ? std::log2(m) : -1e9);
  }
  return 0;
}
