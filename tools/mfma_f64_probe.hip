// Probe: fp64 MFMA (v_mfma_f64_16x16x4_f64) operand/result lane maps and issue rate on gfx950,
// plus the fp64 VALU FMA rate. Standalone; not part of the product library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)

__global__ void layout_k(const double* A, const double* B, double* C) {
  int l = threadIdx.x;
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) C[l * 4 + r] = acc[r];
}

// Is v_mfma_f64_16x16x4_f64 bit-for-bit the k-ordered fma chain D = fma(a3,b3,fma(a2,b2,fma(a1,b1,fma(a0,b0,C))))?
__global__ void chain_k(const double* A, const double* B, const double* C, double* D, double* Dref) {
  int l = threadIdx.x;
  d4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[((l >> 4) + 4 * r) * 16 + (l & 15)];
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    const int row = (l >> 4) + 4 * r, col = l & 15;
    D[row * 16 + col] = acc[r];
    double s = C[row * 16 + col];
    for (int k = 0; k < 4; ++k) s = fma(A[row * 4 + k], B[k * 16 + col], s);
    Dref[row * 16 + col] = s;
  }
}

// v_mfma_f64_4x4x4_4b: 4 blocks b of 4 x 4 outputs, K = 4.  Lane 16 K + 4 b + i holds X_b[i][K] and Y_b[K][i]
// (operand order: D_b = X_b Y_b + C_b); result lane 16 i + 4 b + j holds D_b[i][j].  Is it the k-ordered fma chain?
__global__ void chain4_k(const double* X, const double* Y, const double* C, double* D, double* Dref) {
  const int l = threadIdx.x, K = l >> 4, b = (l >> 2) & 3, i = l & 3;
  const int ri = l >> 4, rj = l & 3;   // result (i, j) of block b for this lane
  double acc = C[b * 16 + ri * 4 + rj];
  acc = __builtin_amdgcn_mfma_f64_4x4x4f64(X[b * 16 + i * 4 + K], Y[b * 16 + K * 4 + i], acc, 0, 0, 0);
  D[b * 16 + ri * 4 + rj] = acc;
  double s = C[b * 16 + ri * 4 + rj];
  for (int k = 0; k < 4; ++k) s = fma(X[b * 16 + ri * 4 + k], Y[b * 16 + k * 4 + rj], s);
  Dref[b * 16 + ri * 4 + rj] = s;
}

template <int NACC>
__global__ void rate4_k(double* out, int iters, double seed) {
  double acc[NACC];
  for (int i = 0; i < NACC; i++) acc[i] = seed;
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void rate_k(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; i++) acc[i] = (d4){seed, seed, seed, seed};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void valu_k(double* out, int iters, double seed) {
  double x[8];
  for (int i = 0; i < 8; i++) x[i] = seed + i + threadIdx.x;
  double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < 8; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double hA[64], hB[64], hC[256];
  for (int i = 0; i < 16; i++) for (int k = 0; k < 4; k++) hA[i * 4 + k] = (i + 1) * 1.0 + (k + 1) * 0.001;
  for (int k = 0; k < 4; k++) for (int j = 0; j < 16; j++) hB[k * 16 + j] = (k == 0 ? 1.0 : 0.0) * (j + 1) + (k + 1) * 100.0 * (j == 3);
  double *dA, *dB, *dC;
  CK(hipMalloc(&dA, 64 * 8)); CK(hipMalloc(&dB, 64 * 8)); CK(hipMalloc(&dC, 256 * 8));
  CK(hipMemcpy(dA, hA, 64 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, 64 * 8, hipMemcpyHostToDevice));
  layout_k<<<1, 64>>>(dA, dB, dC);
  CK(hipMemcpy(hC, dC, 256 * 8, hipMemcpyDeviceToHost));
  double ref[16][16];
  for (int i = 0; i < 16; i++) for (int j = 0; j < 16; j++) { double s = 0; for (int k = 0; k < 4; k++) s += hA[i * 4 + k] * hB[k * 16 + j]; ref[i][j] = s; }
  int ok_guide = 1, ok_f32 = 1;
  for (int l = 0; l < 64; l++) for (int r = 0; r < 4; r++) {
    int col = l & 15;
    int row_g = (l >> 4) + 4 * r, row_f = (l >> 4) * 4 + r;
    if (fabs(hC[l * 4 + r] - ref[row_g][col]) > 1e-9) ok_guide = 0;
    if (fabs(hC[l * 4 + r] - ref[row_f][col]) > 1e-9) ok_f32 = 0;
  }
  printf("layout: row=(lane>>4)+4*reg: %s ; row=(lane>>4)*4+reg: %s\n", ok_guide ? "MATCH" : "no", ok_f32 ? "MATCH" : "no");

  {
    double hA2[64], hB2[64], hC2[256];
    unsigned long long x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (double)(x >> 11) / 9007199254740992.0 * 2 - 1; };
    int same = 0, tot = 0;
    double *dA2, *dB2, *dC2, *dD, *dR;
    CK(hipMalloc(&dA2, 512)); CK(hipMalloc(&dB2, 512)); CK(hipMalloc(&dC2, 2048)); CK(hipMalloc(&dD, 2048)); CK(hipMalloc(&dR, 2048));
    for (int trial = 0; trial < 200; ++trial) {
      for (int i = 0; i < 64; ++i) { hA2[i] = rnd() * (1 << (trial % 20)); hB2[i] = rnd() / (1 + trial % 7); }
      for (int i = 0; i < 256; ++i) hC2[i] = rnd() * 1e3;
      CK(hipMemcpy(dA2, hA2, 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB2, hB2, 512, hipMemcpyHostToDevice));
      CK(hipMemcpy(dC2, hC2, 2048, hipMemcpyHostToDevice));
      chain_k<<<1, 64>>>(dA2, dB2, dC2, dD, dR);
      double hD[256], hR[256];
      CK(hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost)); CK(hipMemcpy(hR, dR, 2048, hipMemcpyDeviceToHost));
      for (int i = 0; i < 256; ++i) { tot++; same += (hD[i] == hR[i]); }
    }
    printf("f64 MFMA == k-ordered fma chain: %d / %d entries bit-identical\n", same, tot);
  }
  {
    double hX[64], hY[64], hC4[64], hD[64], hR[64];
    unsigned long long x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (double)(x >> 11) / 9007199254740992.0 * 2 - 1; };
    double *dX, *dY, *dC4, *dD4, *dR4;
    CK(hipMalloc(&dX, 512)); CK(hipMalloc(&dY, 512)); CK(hipMalloc(&dC4, 512)); CK(hipMalloc(&dD4, 512)); CK(hipMalloc(&dR4, 512));
    int same = 0, tot = 0;
    for (int trial = 0; trial < 400; ++trial) {
      for (int i = 0; i < 64; ++i) { hX[i] = rnd() * (1 << (trial % 20)); hY[i] = rnd() / (1 + trial % 7); hC4[i] = rnd() * 1e3; }
      CK(hipMemcpy(dX, hX, 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dY, hY, 512, hipMemcpyHostToDevice));
      CK(hipMemcpy(dC4, hC4, 512, hipMemcpyHostToDevice));
      chain4_k<<<1, 64>>>(dX, dY, dC4, dD4, dR4);
      CK(hipMemcpy(hD, dD4, 512, hipMemcpyDeviceToHost)); CK(hipMemcpy(hR, dR4, 512, hipMemcpyDeviceToHost));
      for (int i = 0; i < 64; ++i) { tot++; same += (hD[i] == hR[i]); }
    }
    printf("f64 MFMA 4x4x4 == k-ordered fma chain: %d / %d entries bit-identical\n", same, tot);
  }
  double* dout; CK(hipMalloc(&dout, 1 << 24));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int iters = 4000; float ms;
  for (int rep = 0; rep < 2; rep++) {
    int blocks = 256 * 4, threads = 256;
    CK(hipEventRecord(e0)); rate_k<4><<<blocks, threads>>>(dout, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    double fl = (double)blocks * (threads / 64) * iters * 4 * 2048.0;
    printf("mfma f64 16x16x4, 4 acc, %d WGx%d: %.3f ms  %.2f TFLOP/s\n", blocks, threads, ms, fl / ms / 1e9);
    CK(hipEventRecord(e0)); rate_k<1><<<blocks, threads>>>(dout, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = (double)blocks * (threads / 64) * iters * 1 * 2048.0;
    printf("mfma f64 16x16x4, 1 acc: %.3f ms  %.2f TFLOP/s\n", ms, fl / ms / 1e9);
    CK(hipEventRecord(e0)); rate_k<4><<<256, 64>>>(dout, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = 256.0 * iters * 4 * 2048.0;
    printf("mfma f64 one wave/CU 4 acc: %.3f ms -> %.1f cycles/mfma @2.4GHz\n", ms, ms * 1e-3 * 2.4e9 / (iters * 4.0));
    for (int na = 1; na <= 4; na *= 2) {   // one wave per SIMD: cycles per MFMA with na independent chains
      CK(hipEventRecord(e0));
      if (na == 1) rate_k<1><<<256, 256>>>(dout, iters, 1.0);
      if (na == 2) rate_k<2><<<256, 256>>>(dout, iters, 1.0);
      if (na == 4) rate_k<4><<<256, 256>>>(dout, iters, 1.0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("mfma f64 one wave/SIMD, %d chain(s): %.1f cycles/mfma @2.4GHz\n", na, ms * 1e-3 * 2.4e9 / (iters * (double)na));
    }
    for (int na = 1; na <= 4; na *= 2) {   // 4x4x4: one wave per SIMD
      CK(hipEventRecord(e0));
      if (na == 1) rate4_k<1><<<256, 256>>>(dout, iters, 1.0);
      if (na == 2) rate4_k<2><<<256, 256>>>(dout, iters, 1.0);
      if (na == 4) rate4_k<4><<<256, 256>>>(dout, iters, 1.0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("mfma f64 4x4x4 one wave/SIMD, %d chain(s): %.1f cycles/mfma @2.4GHz\n", na, ms * 1e-3 * 2.4e9 / (iters * (double)na));
    }
    CK(hipEventRecord(e0)); rate4_k<4><<<blocks, threads>>>(dout, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = (double)blocks * (threads / 64) * iters * 4 * 512.0;
    printf("mfma f64 4x4x4, 4 acc, %d WGx%d: %.3f ms  %.2f TFLOP/s\n", blocks, threads, ms, fl / ms / 1e9);
    CK(hipEventRecord(e0)); valu_k<<<blocks, threads>>>(dout, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = (double)blocks * threads * iters * 8 * 2.0;
    printf("valu fma f64: %.3f ms  %.2f TFLOP/s\n", ms, fl / ms / 1e9);
  }
  return 0;
}
