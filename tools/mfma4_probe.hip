// tools/mfma4_probe.hip -- operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950 (one-hot probes),
// its issue cost against v_mfma_f64_16x16x4_f64, and its K order (is it an in-order fma chain?).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma4_probe.hip -o tools/mfma4_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// mode 0: a one-hot at lane `hot`, b = 1 everywhere; mode 1: b one-hot, a = 1; mode 2: c = lane id, a = b = 0
__global__ void probe(int mode, int hot, double* out) {
  const int l = threadIdx.x;
  double a = 0, b = 0, c = 0;
  if (mode == 0) {
    a = (l == hot) ? 1.0 : 0.0;
    b = 1.0;
  } else if (mode == 1) {
    a = 1.0;
    b = (l == hot) ? 1.0 : 0.0;
  } else {
    c = (double)l;
  }
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// general product for a hypothesis check: a[l], b[l] given, c = 0
__global__ void prod(const double* a, const double* b, double* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}

template <int SMALL>
__global__ void rate(double* out, int n) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
  for (int i = 0; i < n; ++i) {
    if (SMALL) {
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    } else {
      e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e1, 0, 0, 0);
      e2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e2, 0, 0, 0);
      e3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e3, 0, 0, 0);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + e0[0] + e1[1] + e2[2] + e3[3];
}

int main() {
  double* d;
  CK(hipMalloc(&d, sizeof(double) * 64 * 1024 * 4));
  double h[64];
  for (int mode = 0; mode < 2; ++mode) {
    printf("mode %s: operand lane -> result lanes that become nonzero\n", mode == 0 ? "A one-hot" : "B one-hot");
    for (int hot = 0; hot < 64; ++hot) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, mode, hot, d);
      CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
      printf("  %2d:", hot);
      for (int l = 0; l < 64; ++l)
        if (h[l] != 0.0) printf(" %d", l);
      printf("\n");
    }
  }
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, 2, 0, d);
  CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
  printf("C passthrough:");
  for (int l = 0; l < 64; ++l) printf(" %g", h[l]);
  printf("\n");
  // K order: a = (1, 1e16, -1e16, 1) along K for every (block, row) if the layout is as inferred below
  // rate: 1024 waves (256 WGs x 4 waves), n iterations x 4 MFMAs
  for (int small = 0; small < 2; ++small) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int n = 4096;
    if (small)
      hipLaunchKernelGGL(rate<1>, dim3(1024), dim3(256), 0, 0, d, n);
    else
      hipLaunchKernelGGL(rate<0>, dim3(1024), dim3(256), 0, 0, d, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    if (small)
      hipLaunchKernelGGL(rate<1>, dim3(1024), dim3(256), 0, 0, d, n);
    else
      hipLaunchKernelGGL(rate<0>, dim3(1024), dim3(256), 0, 0, d, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double mfmas = 1024.0 * 4 * n * 4;   // waves x iterations x 4
    const double flop = mfmas * (small ? 512.0 : 2048.0);
    printf("%s: %.3f ms, %.2f TFLOP/s, %.1f cycles per MFMA per SIMD at 2.4 GHz (4 waves/SIMD... 1024 waves on 1024 SIMDs)\n",
           small ? "4x4x4_4b f64" : "16x16x4 f64", ms, flop / ms / 1e9, ms * 1e-3 * 2.4e9 / (4.0 * n));
  }
  printf("done\n");
  return 0;
}
