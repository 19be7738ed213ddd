// Probe: how close the Brunet kernels' quotient sequences come to IEEE a / p on gfx950 (standalone; not part of
// the product library).  For N pseudo-random pairs (a >= 0, p > 0 over wide exponent ranges) it counts results
// that differ from the correctly rounded quotient for
//   q2: v_rcp_f64, two Newton steps, residual correction  (csrc/brunet.hip quot(), the shipped form)
//   q1: v_rcp_f64, ONE Newton step, residual correction
// and reports the largest relative error of v_rcp_f64 itself (against 1 / p).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
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
  unsigned long long c1 = 0, c2 = 0;
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
  }
  atomicAdd(&cnt[0], c1);
  atomicAdd(&cnt[1], c2);
  // the largest |1 - p r0| over the grid: doubles >= 0 order like their bit patterns
  atomicMax((unsigned long long*)maxrel, (unsigned long long)__double_as_longlong(mr));
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : (1L << 30);
  struct Range { const char* what; int ea0, ea1, ep0, ep1; } rs[] = {
      {"a in [2^-4, 2^4), p in [2^-4, 2^4)", -4, 3, -4, 3},
      {"a in [2^-30, 2^10), p in [2^-60, 2^10)", -30, 9, -60, 9},
      {"a in [2^-1, 2^1), p in [2^-1, 2^1)", -1, 0, -1, 0},
  };
  unsigned long long* cnt;
  double* mr;
  CK(hipMalloc(&cnt, 2 * sizeof(unsigned long long)));
  CK(hipMalloc(&mr, sizeof(double)));
  for (const Range& r : rs) {
    CK(hipMemset(cnt, 0, 2 * sizeof(unsigned long long)));
    CK(hipMemset(mr, 0, sizeof(double)));
    probe<<<4096, 256>>>(n, 0x5EEDull + (uint64_t)r.ep0, r.ea0, r.ea1, r.ep0, r.ep1, cnt, mr);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long h[2];
    double m;
    CK(hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&m, mr, sizeof m, hipMemcpyDeviceToHost));
    printf("%-42s %ld pairs: one Newton step %llu differ from a / p, two steps %llu; max |1 - p rcp(p)| = %.3g (2^%.1f)\n",
           r.what, n, h[0], h[1], m, m > 0 ? std::log2(m) : -1e9);
  }
  return 0;
}
