// Host check of the Brunet kernels' batched reciprocal (csrc/brunet.hip recip_batch + quot_r), CPU test
// infrastructure only (tests/test_brunet_recip.py builds and runs it).  The device sequence is restated with std::fma
// (the same fused operation as v_fma_f64) and v_rcp_f64 is emulated by a correctly rounded float reciprocal of the
// mantissa (relative error <= 2^-24, against v_rcp_f64's measured 2^-24.4: profiles/r05/brunet/quot_probe.txt), so the
// check is if anything pessimistic.  For batches of N = 1..5 it counts quotients that differ from the IEEE a / p and
// reports the largest |1 - p r| of the batched reciprocals (the residual correction needs it well below 2^-26).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

static double rcp_emul(double c) {
  int e = 0;
  const double m = std::frexp(c, &e);                  // c = m 2^e, m in [0.5, 1)
  return std::ldexp((double)(1.0f / (float)m), -e);   // float-accurate reciprocal, as v_rcp_f64
}

template <int N>
static void recip_batch(const double* p, double* r) {
  double c[N];
  c[0] = p[0];
  for (int i = 1; i < N; ++i) c[i] = c[i - 1] * p[i];
  double u = rcp_emul(c[N - 1]);
  u = std::fma(u, std::fma(-c[N - 1], u, 1.0), u);
  for (int i = N - 1; i > 0; --i) {
    r[i] = u * c[i - 1];
    u = u * p[i];
  }
  r[0] = u;
}

static double quot_r(double a, double p, double r) {
  const double q = a * r;
  return std::fma(std::fma(-p, q, a), r, q);
}

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint64_t next() {   // splitmix64
  uint64_t z = (s_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double rnd(int e0, int e1) {   // random 52-bit mantissa, exponent uniform in [e0, e1]
  const uint64_t z = next();
  const double man = 1.0 + (double)(z & ((1ull << 52) - 1)) / 4503599627370496.0;
  return std::ldexp(man, e0 + (int)((z >> 52) % (uint64_t)(e1 - e0 + 1)));
}

template <int N>
static int run(long batches, int ep0, int ep1) {
  long diff = 0;
  double worst = 0.0;
  for (long t = 0; t < batches; ++t) {
    double p[N], r[N];
    for (int i = 0; i < N; ++i) p[i] = rnd(ep0, ep1);
    recip_batch<N>(p, r);
    for (int i = 0; i < N; ++i) {
      const double a = rnd(-30, 10);
      diff += quot_r(a, p[i], r[i]) != a / p[i];
      const double err = std::fabs(std::fma(-p[i], r[i], 1.0));
      if (err > worst) worst = err;
    }
  }
  std::printf("N=%d p in [2^%d, 2^%d]: %ld quotients, %ld differ from a / p, max |1 - p r| = 2^%.1f\n", N, ep0, ep1,
              batches * N, diff, worst > 0 ? std::log2(worst) : -1e9);
  return diff != 0 || worst > std::ldexp(1.0, -44);
}

int main(int argc, char** argv) {
  const long b = argc > 1 ? std::atol(argv[1]) : 400000;
  int bad = 0;
  // VP of the KL updates: [eps^2 / T, T]; here a representative spread and the extremes of a batch
  bad |= run<1>(b, -60, 10);
  bad |= run<2>(b, -60, 10);
  bad |= run<3>(b, -60, 10);
  bad |= run<4>(b, -60, 10);
  bad |= run<5>(b, -60, 10);
  bad |= run<5>(b / 4, -204, -200);   // near the lower bound: a product of 5 near 2^-1020
  bad |= run<5>(b / 4, 96, 100);      // near the upper bound
  std::printf(bad ? "FAIL\n" : "OK\n");
  return bad;
}
