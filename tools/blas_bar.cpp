// Reference bar: rocBLAS dgemm on the two C3 full-load contraction shapes of one MU sweep-iteration
// (176 panels x 64 columns = 11264 stacked restart columns, m_pad = 20096, n_pad = 512):
//   G   = W^T A      (11264 x 512,   K = 20096)  -- what k_wta2 computes (plus Gram blocks)
//   F^T = H A^T      (11264 x 20096, K = 512)    -- what k_ahtw4 computes (plus the W update)
// Standalone timing tool; not part of the product library.
// Build: hipcc -O3 tools/blas_bar.cpp -lrocblas -o tools/blas_bar
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);        \
      exit(1);                                                         \
    }                                                                  \
  } while (0)
#define RB(x)                                                          \
  do {                                                                 \
    rocblas_status s = (x);                                            \
    if (s != rocblas_status_success) {                                 \
      printf("rocBLAS %d at %d\n", (int)s, __LINE__);                  \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

int main() {
  const long cols = 11264, m_pad = 20096, n_pad = 512;
  double *W, *A, *H, *Arm, *G, *F;
  CK(hipMalloc(&W, 8 * cols * m_pad));
  CK(hipMalloc(&A, 8 * n_pad * m_pad));
  CK(hipMalloc(&H, 8 * cols * n_pad));
  CK(hipMalloc(&Arm, 8 * m_pad * n_pad));
  CK(hipMalloc(&G, 8 * cols * n_pad));
  CK(hipMalloc(&F, 8 * cols * m_pad));
  {
    std::vector<double> h(cols * m_pad);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.25 + (double)((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(W, h.data(), 8 * cols * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(F, h.data(), 8 * cols * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(A, h.data(), 8 * n_pad * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Arm, h.data(), 8 * n_pad * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(H, h.data(), 8 * cols * n_pad, hipMemcpyHostToDevice));
  }
  rocblas_handle hd;
  RB(rocblas_create_handle(&hd));
  const double one = 1.0, zero = 0.0;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto f, double flops) {
    for (int w = 0; w < 3; ++w) f();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-34s %8.3f ms  %6.1f TF\n", name, ms, flops / ms / 1e9);
  };
  run("rocblas dgemm W^T A (TN)", [&] {
    RB(rocblas_dgemm(hd, rocblas_operation_transpose, rocblas_operation_none, cols, n_pad, m_pad, &one, W, m_pad, A,
                     m_pad, &zero, G, cols));
  }, 2.0 * cols * n_pad * m_pad);
  run("rocblas dgemm H A^T (TN, K=512)", [&] {
    RB(rocblas_dgemm(hd, rocblas_operation_transpose, rocblas_operation_none, cols, m_pad, n_pad, &one, H, n_pad, Arm,
                     n_pad, &zero, F, cols));
  }, 2.0 * cols * n_pad * m_pad);
  run("rocblas dgemm A h^T (NT, K=512)", [&] {
    RB(rocblas_dgemm(hd, rocblas_operation_transpose, rocblas_operation_none, m_pad, cols, n_pad, &one, Arm, n_pad, H,
                     n_pad, &zero, F, m_pad));
  }, 2.0 * cols * n_pad * m_pad);
  run("rocblas dgemm 8192^3 (NN)", [&] {
    RB(rocblas_dgemm(hd, rocblas_operation_none, rocblas_operation_none, 8192, 8192, 8192, &one, W, 8192, W + 8192L * 8192,
                     8192, &zero, F, 8192));
  }, 2.0 * 8192.0 * 8192.0 * 8192.0);
  return 0;
}
