// Probe: can fp64 MFMA (v_mfma_f64_16x16x4_f64) and fp64 VALU FMA (v_fma_f64) run concurrently on
// gfx950?  Each workgroup has 8 waves (2 per SIMD); MODE selects which waves work:
//   0: MFMA waves only (even waves), 1: VALU waves only (odd waves), 2: both.
// If the DP VALU and the matrix core are separate pipes, mode 2 takes about max(mode 0, mode 1).
// Standalone; not part of the product library.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);              \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(512) void mix_k(double* out, int iters_mfma, int iters_valu, double seed) {
  const int w = threadIdx.x >> 6;
  double s = 0.0;
  if ((w & 1) == 0) {
    if (MODE == 1) return;
    d4 acc[4];
    for (int i = 0; i < 4; i++) acc[i] = (d4){seed, seed, seed, seed};
    const double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
    for (int it = 0; it < iters_mfma; it++) {
#pragma unroll
      for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    if (MODE == 0) return;
    double x[8];
    for (int i = 0; i < 8; i++) x[i] = seed + i + threadIdx.x;
    const double m = 1.0000001, c = 1e-9;
    for (int it = 0; it < iters_valu; it++) {
#pragma unroll
      for (int i = 0; i < 8; i++) x[i] = fma(x[i], m, c);
    }
    for (int i = 0; i < 8; i++) s += x[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* dout;
  const int blocks = 256 * 2;
  CK(hipMalloc(&dout, sizeof(double) * blocks * 512));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int im = 4000;
  // VALU iterations sized so the VALU waves alone take about as long as the MFMA waves alone
  for (int iv : {4000, 8000, 16000}) {
    float ms[3];
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      mix_k<0><<<blocks, 512>>>(dout, im, iv, 1.0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[0], e0, e1));
      CK(hipEventRecord(e0));
      mix_k<1><<<blocks, 512>>>(dout, im, iv, 1.0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[1], e0, e1));
      CK(hipEventRecord(e0));
      mix_k<2><<<blocks, 512>>>(dout, im, iv, 1.0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[2], e0, e1));
    }
    const double waves = blocks * 4.0;
    const double fl_m = waves * im * 4 * 2048.0, fl_v = waves * 64.0 * iv * 8 * 2.0;
    printf("valu iters %5d: mfma-only %.3f ms (%.1f TF)  valu-only %.3f ms (%.1f TF)  both %.3f ms (%.1f TF combined)\n",
           iv, ms[0], fl_m / ms[0] / 1e9, ms[1], fl_v / ms[1] / 1e9, ms[2], (fl_m + fl_v) / ms[2] / 1e9);
  }
  return 0;
}
