// tools/kvar.hip -- where the time of the full-load MFMA kernels goes (C3 shape, every restart live): A h^T
// (k_ahtw4) with its epilogue pieces switched off (VARIANT 1: no W0 loads, 2: no E, 3: no W stores, 4: no E and
// no rule) and at n = 2000 (K four times longer: the per-tile fixed cost amortised over 4x the MFMA work), and
// W^T A (k_wta2 big) with / without its Gram chains and at other ring depths.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kvar.hip -o tools/kvar     Usage: kvar [R=200] [reps=10]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "../nmfconsensus_amd/csrc/nmfc_kernels.hpp"

using namespace nmfc;

// ---------------------------------------------------------------------------------------------------------------
// k_ahtw_probe: a copy of the engine's k_ahtw4 in its full-load form (GTG = 128, 2-stage ring, one panel, LATE, KHALF),
// with probe arms that the product kernel does not carry (round 5: moved out of nmfc_kernels.hpp):
//   VARIANT 0  the engine's kernel (bit-identical output: checked in main against k_ahtw4)
//   VARIANT 1  no W0 loads (W0 = 1.0)      2  no E (E = 0)      3  no W stores      4  no E, no rule (raw F stored)
// epilogue forms (F flags):
//   F_BL  the W rule without branches (selects; the same bits as mu_rule for every input)
//   F_FD  ... and the divide as v_rcp_f64 + two Newton steps + the correction FMA, without v_div_scale / v_div_fmas /
//         v_div_fixup (the same bits as IEEE division wherever those are identities: no operand or quotient near
//         the denormal / overflow range) -- unguarded here, an upper bound for the guarded form
//   F_E4  E over the four K steps of its own 16-row block always (no lo / hi shuffles; exact zeros elsewhere)
//   F_EW  W0 blocks 0 and 1 issued with the last K stage's DMA (XL = 16 loads in flight across the last step)
// STAMP: per-wave s_memtime stamps (diagnostic build; read its shares, never its length):
//   [0] entry  [1] K loop done  [2] h h^T staged + first W0 blocks landed (barrier)  [3..6] block mb's stores issued
//   [7] HW_ID  [8] XCC_ID
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

constexpr int NSTAMP = 9;
constexpr int F_BL = 1, F_FD = 2, F_E4 = 4, F_EW = 8;

__device__ __forceinline__ double div_nr(double n, double d) {   // LLVM's f64 fdiv sequence without scale / fixup
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  const double q = n * r;
  const double res = fma(-d, q, n);
  return fma(res, r, q);
}

template <int FL>
__device__ __forceinline__ double rule_form(double old, double num, double den) {
  if constexpr (!(FL & F_BL)) return mu_rule(old, num, den);
  const double dd = den + DIV_BY_ZERO_AVOIDANCE;
  const double q = (FL & F_FD) ? div_nr(num, dd) : num / dd;
  const double t = old * q;
  return (old == 0.0 || num == 0.0 || t < 0.0) ? 0.0 : t;
}

template <int VARIANT, bool STAMP, bool KHALF, int FL = 0>
static __global__ __launch_bounds__(256, 3) void k_ahtw_probe(int iter, const double* __restrict__ H, long n_pad,
                                                              const double* __restrict__ Arm, long m_pad,
                                                              double* __restrict__ W, const double* __restrict__ SHP,
                                                              const ColInfo* __restrict__ ci, const int* __restrict__ colact,
                                                              int npanels, int ngt, unsigned long long* __restrict__ st) {
  constexpr int GTG = GT, NBUF = 2, NPT = 1, PR = PANEL, WC = 4;
  using TileW4 = GTile<PR * NPT, GTG, NPT, WC, NBUF>;
  constexpr int NTH = 64 * NPT * WC;
  constexpr bool EW = (FL & F_EW) != 0;
  __shared__ __attribute__((aligned(1024))) char smem[TileW4::LDS_BYTES];
  unsigned long long ts[NSTAMP] = {};
  if constexpr (STAMP) ts[0] = stamp();
  int pp, gt;
  ahtw_map(xcd_item(blockIdx.x, (npanels / NPT) * ngt), npanels / NPT, ngt, pp, gt);
  const int p0 = pp * NPT;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), wr = w / WC, wc = w % WC;
  const int p = p0 + wr;
  ColInfo cc;
  uint64_t actmask = 0;
  TileW4 tl;
  tl.zero();
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      W + (long)p * PR * m_pad + (long)gt * GTG + (GTG / WC) * wc, 0, (int)(PR * m_pad * 8), 0x00020000);
  const int wvoff = (int)(((lane >> 4) * m_pad + (lane & 15)) * 8);
  auto woff = [&](int mb, int reg, int nb) { return (int)(((16 * mb + 4 * reg) * m_pad + 16 * nb) * 8); };
  double w0[TileW4::MB][TileW4::NB][4];
  auto load_w0_block = [&](int mb) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
#pragma unroll
      for (int nb = 0; nb < TileW4::NB; ++nb)
        w0[mb][nb][reg] = (VARIANT == 1 || VARIANT == 4)
                              ? 1.0
                              : __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rw, wvoff, woff(mb, reg, nb), 0));
  };
  constexpr int NSH = NPT * PR * KMAX / 2 / NTH;
  d2 shv[NSH];
  const bool live = tl.template run<EW ? 2 * TileW4::NB * 4 : 0, KHALF ? 1 : 2>(
      H + (long)p0 * PR * n_pad, n_pad, Arm + (long)gt * GTG * n_pad, n_pad, 0, (int)n_pad, smem,
      [&] {
        cc = lane < PR ? ci[(long)p * PR + lane] : ColInfo{0, 0, 0, 0};
        const int ca = lane < PR ? colact[(long)p0 * PR + lane] : -1;
        const d2* src = reinterpret_cast<const d2*>(SHP + (long)p0 * PR * KMAX);
#pragma unroll
        for (int j = 0; j < NSH; ++j) shv[j] = src[tid + NTH * j];
        actmask = __ballot(ca == iter);
        return actmask != 0;
      },
      [](const char*) {},
      [&] {
        if constexpr (EW) {
          load_w0_block(0);
          load_w0_block(1);
        }
      });
  if (!live) return;
  if constexpr (STAMP) ts[1] = stamp();
  const int nst = (int)n_pad / BK2;
  double* SHl = reinterpret_cast<double*>(smem + ((nst - 2) % NBUF) * TileW4::STAGE_BYTES);
#pragma unroll
  for (int j = 0; j < NSH; ++j) reinterpret_cast<d2*>(SHl)[tid + NTH * j] = shv[j];
  if constexpr (!EW) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) load_w0_block(mb);
  }
  // F_E4 holds only where no active restart crosses a 16-column block (the engine's block packing): wave-uniform
  bool e4 = false;
  if constexpr ((FL & F_E4) != 0) {
    const bool cross = ((actmask >> lane) & 1) && cc.k > 0 && ((cc.lc0 & (PR - 1)) >> 4) != (((cc.lc0 & (PR - 1)) + cc.k - 1) >> 4);
    e4 = __ballot(cross) == 0;
  }
  __syncthreads();
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ts[2] = stamp();
  }
  const double* SHw = SHl + (long)wr * PR * KMAX;
#pragma unroll
  for (int mb = 0; mb < TileW4::MB; ++mb) {
    if (mb + 2 < TileW4::MB) load_w0_block(mb + 2);
    const int ra = 16 * mb + (lane & 15);
    const int alc = __shfl(cc.lc0, ra) & (PR - 1);
    const int ak = (VARIANT == 2 || VARIANT == 4 || !((actmask >> ra) & 1)) ? 0 : __shfl(cc.k, ra);
    d4 e[TileW4::NB];
#pragma unroll
    for (int nb = 0; nb < TileW4::NB; ++nb) e[nb] = d4{0.0, 0.0, 0.0, 0.0};
    if (e4) {
      if (VARIANT != 2 && VARIANT != 4) {
        double av[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int bb = 16 * mb + 4 * q + (lane >> 4) - alc;
          av[q] = (bb >= 0 && bb < ak) ? SHw[ra * KMAX + bb] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int nb = 0; nb < TileW4::NB; ++nb)
            e[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], w0[mb][nb][q], e[nb], 0, 0, 0);
      }
    } else {
      int lo = ak ? alc : PANEL, hi = ak ? alc + ak : 0;
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off));
        hi = max(hi, __shfl_xor(hi, off));
      }
      lo = __builtin_amdgcn_readfirstlane(lo);
      hi = __builtin_amdgcn_readfirstlane(hi);
#pragma unroll
      for (int q = (4 * mb - 4 > 0 ? 4 * mb - 4 : 0); q < (4 * mb + 8 < 4 * TileW4::MB ? 4 * mb + 8 : 4 * TileW4::MB); ++q) {
        if (4 * q + 3 < lo || 4 * q >= hi) continue;
        const int bb = 4 * q + (lane >> 4) - alc;
        const double av = (bb >= 0 && bb < ak) ? SHw[ra * KMAX + bb] : 0.0;
#pragma unroll
        for (int nb = 0; nb < TileW4::NB; ++nb)
          e[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, w0[q >> 2][nb][q & 3], e[nb], 0, 0, 0);
      }
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int c = 16 * mb + (lane >> 4) + 4 * reg;
      if (!((actmask >> c) & 1)) continue;
#pragma unroll
      for (int nb = 0; nb < TileW4::NB; ++nb) {
        const double v = VARIANT == 4 ? tl.acc[mb][nb][reg] : rule_form<FL>(w0[mb][nb][reg], tl.acc[mb][nb][reg], e[nb][reg]);
        if (VARIANT != 3 || v == (double)iter * 1.5e300)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rw, wvoff, woff(mb, reg, nb), 0);
      }
    }
    if constexpr (STAMP) ts[3 + mb] = stamp();
  }
  if constexpr (STAMP) {
    ts[7] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    ts[8] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11));   // HW_REG_XCC_ID
    if (lane < NSTAMP) {
      unsigned long long v = ts[0];
#pragma unroll
      for (int i = 1; i < NSTAMP; ++i)
        if (lane == i) v = ts[i];
      st[((long)blockIdx.x * 4 + w) * NSTAMP + lane] = v;
    }
  }
}


// ---------------------------------------------------------------------------------------------------------------
// FETCH_SIZE calibration (kvar cal): read a known number of bytes with the access patterns of the engine's MFMA kernels
// and compare with the counter (MI355X_MICROARCH.md: FETCH_SIZE under-counts wide coalesced streams up to 2x; the
// factor depends on the pattern).  k_cal_b64: the A h^T epilogue's W0 loads (buffer_load_b64, each instruction 4 rows
// x 128 B) over W; k_cal_dma: the GTile operand stream (buffer_load ... lds, 1 KiB per wave instruction) over W.
// ---------------------------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(256) void k_cal_b64(const double* __restrict__ W, long m_pad, int npanels, int ngt,
                                                        double* __restrict__ out) {
  const int b = blockIdx.x, p = b / ngt, gt = b % ngt, w = wave_id(), lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(W) + (long)p * PANEL * m_pad + (long)gt * GT + (GT / 4) * w, 0, (int)(PANEL * m_pad * 8), 0x00020000);
  const int wvoff = (int)(((lane >> 4) * m_pad + (lane & 15)) * 8);
  double acc = 0.0;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                              rw, wvoff, (int)(((16 * mb + 4 * reg) * m_pad + 16 * nb) * 8), 0));
  out[(long)b * 256 + threadIdx.x] = acc;
}

static __global__ __launch_bounds__(256) void k_cal_dma(const double* __restrict__ W, long m_pad, long cols,
                                                        double* __restrict__ out) {
  // workgroup b streams rows [64 b, 64 b + 64) of W (m_pad doubles each) through LDS in 1 KiB pieces
  __shared__ __attribute__((aligned(1024))) char lds[4096];
  const int w = wave_id(), lane = threadIdx.x & 63;
  const long row0 = (long)blockIdx.x * 64;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(W) + row0 * m_pad, 0,
                                                                     (int)(64 * m_pad * 8), 0x00020000);
  const long bytes = 64 * m_pad * 8;
  for (long off = (long)w * 1024; off < bytes; off += 4 * 1024) {
    lds_dma16(r, (uint32_t)(uintptr_t)lds + w * 1024, lane * 16, (int)off);
  }
  wait_vmcnt<0>();
  __syncthreads();
  out[(long)blockIdx.x * 256 + threadIdx.x] = reinterpret_cast<const double*>(lds)[threadIdx.x & 127];
  (void)cols;
}

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 200, reps = argc > 2 ? atoi(argv[2]) : 10;
  const bool pmc = argc > 3 && !strcmp(argv[3], "pmc");   // counter passes: n = 500, one round, no checks / stamps
  const bool cal = argc > 3 && !strcmp(argv[3], "cal");   // FETCH_SIZE calibration kernels only
  const int m = 20000;
  // packing of R restarts of every k = 10..2 as the engine packs them (engine.hip pack()): k descending, first fit
  // into 16-column blocks (no restart across a block), four blocks to a 64-column panel
  std::vector<ColInfo> ci;
  std::vector<RestartInfo> ri;
  std::vector<int> pfirst;
  int np = -1, sq = 0;
  double fk = 0, fk2 = 0;   // sum of k, k^2
  {
    std::vector<int> bfill;
    std::vector<std::vector<std::pair<int, int>>> bmem;   // (k, first column in block)
    for (int k = 10; k >= 2; --k)
      for (int r = 0; r < R; ++r) {
        size_t b = 0;
        while (b < bfill.size() && bfill[b] + k > 16) ++b;
        if (b == bfill.size()) {
          bfill.push_back(0);
          bmem.emplace_back();
        }
        bmem[b].push_back({k, bfill[b]});
        bfill[b] += k;
      }
    const int nblocks = (int)bfill.size();
    np = (nblocks + 3) / 4 - 1;
    ci.assign((size_t)(np + 1) * PANEL, ColInfo{0, 0, 0, 0});
    for (int b = 0; b < nblocks; ++b) {
      if (b % 4 == 0) pfirst.push_back((int)ri.size());
      for (auto [k, c0] : bmem[b]) {
        const int col0 = 16 * b + c0;
        ri.push_back({col0, k, (int)ri.size(), sq});
        for (int a = 0; a < k; ++a) ci[(size_t)col0 + a] = ColInfo{sq, col0 % PANEL, k, (int)ri.size() - 1};
        fk += k;
        fk2 += (double)k * k;
        sq += k * k;
      }
    }
  }
  const int live = np + 1, npanels = (live + 3) / 4 * 4;
  pfirst.push_back((int)ri.size());
  ci.resize((size_t)npanels * PANEL, ColInfo{0, 0, 0, 0});
  const long cols = (long)npanels * PANEL;
  const long m_pad = (m + GT - 1) / GT * GT;
  const int ngt = (int)(m_pad / GT);
  const int nall = (int)ri.size();
  printf("kvar: R=%d, %d restarts in %d panels (%d launched), %d gene tiles\n", R, nall, live, npanels, ngt);
  const long nmax = 2048;
  double *W, *Wb, *Hh, *Arm, *Ablk, *SHP, *Gpart, *SWpart;
  unsigned long long* dstamp;
  int *colact, *dprb, *dpre, *stop;
  ColInfo* dci;
  RestartInfo* dri;
  const long n_cols_max = nmax;
  const int kchunk = 2048, nsplit = (int)((m_pad + kchunk - 1) / kchunk);
  CK(hipMalloc(&W, sizeof(double) * cols * m_pad));
  CK(hipMalloc(&Wb, sizeof(double) * cols * m_pad));
  CK(hipMalloc(&dstamp, sizeof(unsigned long long) * (size_t)(np + 1) * (m_pad / GT) * 4 * NSTAMP));
  CK(hipMalloc(&Hh, sizeof(double) * cols * nmax));
  CK(hipMalloc(&Arm, sizeof(double) * m_pad * nmax));
  CK(hipMalloc(&Ablk, sizeof(double) * m_pad * n_cols_max));
  CK(hipMalloc(&SHP, sizeof(double) * cols * KMAX));
  CK(hipMalloc(&Gpart, sizeof(double) * nsplit * cols * n_cols_max));
  CK(hipMalloc(&SWpart, sizeof(double) * nsplit * sq));
  CK(hipMalloc(&colact, sizeof(int) * cols));
  CK(hipMalloc(&dci, sizeof(ColInfo) * cols));
  CK(hipMalloc(&dri, sizeof(RestartInfo) * nall));
  CK(hipMalloc(&dprb, sizeof(int) * npanels));
  CK(hipMalloc(&dpre, sizeof(int) * npanels));
  CK(hipMalloc(&stop, sizeof(int) * nall));
  {
    std::vector<double> h((size_t)std::max<long>(cols * m_pad, m_pad * nmax));
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.25 + (double)((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(W, h.data(), sizeof(double) * cols * m_pad, hipMemcpyHostToDevice));
    CK(hipMemcpy(Hh, h.data(), sizeof(double) * cols * nmax, hipMemcpyHostToDevice));
    CK(hipMemcpy(Arm, h.data(), sizeof(double) * m_pad * nmax, hipMemcpyHostToDevice));
    CK(hipMemcpy(Ablk, h.data(), sizeof(double) * m_pad * n_cols_max, hipMemcpyHostToDevice));
    std::vector<double> sp((size_t)cols * KMAX, 1e-3);
    CK(hipMemcpy(SHP, sp.data(), sizeof(double) * sp.size(), hipMemcpyHostToDevice));
    std::vector<int> ca(cols);
    for (long c = 0; c < cols; ++c) ca[c] = ci[c].k ? 1 : 0;
    CK(hipMemcpy(colact, ca.data(), sizeof(int) * cols, hipMemcpyHostToDevice));
    CK(hipMemcpy(dci, ci.data(), sizeof(ColInfo) * cols, hipMemcpyHostToDevice));
    CK(hipMemcpy(dri, ri.data(), sizeof(RestartInfo) * nall, hipMemcpyHostToDevice));
    std::vector<int> prb(npanels), pre(npanels);
    for (int p = 0; p < npanels; ++p) {
      prb[p] = p < live ? pfirst[p] : nall;
      pre[p] = p < live ? pfirst[p + 1] : nall;
    }
    CK(hipMemcpy(dprb, prb.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpre, pre.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    CK(hipMemset(stop, 0, sizeof(int) * nall));
  }
  auto report = [&](const char* name, float ms, double flop) {
    printf("  %-44s %8.4f ms  %6.2f TF\n", name, ms, flop / ms / 1e9);
  };
  if (cal) {   // each calibration kernel twice; the known bytes are printed for tools/pmc_cal.py
    double* o;
    CK(hipMalloc(&o, sizeof(double) * 256 * (size_t)live * ngt));
    for (int r = 0; r < 2; ++r) {
      hipLaunchKernelGGL(k_cal_b64, dim3(live * ngt), dim3(256), 0, 0, W, m_pad, live, ngt, o);
      hipLaunchKernelGGL(k_cal_dma, dim3(live), dim3(256), 0, 0, W, m_pad, cols, o);
    }
    CK(hipDeviceSynchronize());
    printf("cal k_cal_b64 bytes %.0f\ncal k_cal_dma bytes %.0f\n", (double)live * PANEL * m_pad * 8,
           (double)live * PANEL * m_pad * 8);
    return 0;
  }
  for (long n : {500L, 2000L}) {
    if (pmc && n != 500) break;
    const long n_pad = (n + BK - 1) / BK * BK;
    const double flop = 2.0 * m * n * fk + 2.0 * m * fk2;   // one contraction (+ its k^2 part), every restart
    printf("\n== A h^T, n = %ld (n_pad %ld)\n", n, n_pad);
#define AH_ARGS Hh, n_pad, Arm, m_pad, W, SHP, dci, colact, live, ngt
#define AP(V, S) hipLaunchKernelGGL((k_ahtw_probe<V, S, true>), dim3(live * ngt), dim3(256), 0, 0, 1, AH_ARGS, dstamp)
#define AF(FLG) hipLaunchKernelGGL((k_ahtw_probe<0, false, true, FLG>), dim3(live * ngt), dim3(256), 0, 0, 1, AH_ARGS, dstamp)
    std::vector<std::pair<std::string, std::function<void()>>> arms = {
        {"k_ahtw4 128 LATE KHALF (engine)", [&] {
           hipLaunchKernelGGL((k_ahtw4<GT, 2, 1, PANEL, 4, true, true>), dim3(live * ngt), dim3(256), 0, 0, 1, AH_ARGS);
         }},
        {"  probe V0 (= engine)", [&] { AP(0, false); }},
        {"  V1 no W0 loads", [&] { AP(1, false); }},
        {"  V2 no E", [&] { AP(2, false); }},
        {"  V3 no W stores", [&] { AP(3, false); }},
        {"  V4 no E, no rule (raw F stored)", [&] { AP(4, false); }},
        {"  form BL (branch-free rule)", [&] { AF(F_BL); }},
        {"  form BL+FD (fast divide, unguarded)", [&] { AF(F_BL | F_FD); }},
        {"  form E4 (4 K steps, no lo/hi)", [&] { AF(F_E4); }},
        {"  form EW (W0 0,1 with the last DMA)", [&] { AF(F_EW); }},
        {"  form BL+E4", [&] { AF(F_BL | F_E4); }},
        {"  form BL+FD+E4", [&] { AF(F_BL | F_FD | F_E4); }},
        {"  form BL+FD+E4+EW", [&] { AF(F_BL | F_FD | F_E4 | F_EW); }},
    };
    if (!pmc) {   // every arm that keeps the arithmetic (V0 and the forms): one launch from the same W as one engine launch
      std::vector<double> x((size_t)cols * m_pad), y((size_t)cols * m_pad);
      for (auto& [name, launch] : arms) {
        if (name.find("V0") == std::string::npos && name.find("form") == std::string::npos) continue;
        CK(hipMemcpy(Wb, W, sizeof(double) * cols * m_pad, hipMemcpyDeviceToDevice));
        arms[0].second();
        std::swap(W, Wb);
        launch();
        std::swap(W, Wb);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(x.data(), W, sizeof(double) * x.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(y.data(), Wb, sizeof(double) * y.size(), hipMemcpyDeviceToHost));
        const bool eq = memcmp(x.data(), y.data(), sizeof(double) * x.size()) == 0;
        printf("  %-44s output %s the engine's\n", name.c_str(), eq ? "bit-identical to" : "DIFFERS FROM");
      }
    }
    auto interleaved = [&](std::vector<std::pair<std::string, std::function<void()>>>& arms) {
      // interleaved rounds (the chip's clock drifts with load and temperature): median and min per arm
      for (int i = 0; i < (pmc ? 2 : 200); ++i) arms[0].second();   // ~1 s of load before the first round
      CK(hipDeviceSynchronize());
      const int rounds = pmc ? 1 : 7;
      std::vector<std::vector<float>> t(arms.size());
      for (int r = 0; r < rounds; ++r)
        for (size_t q = 0; q < arms.size(); ++q) t[q].push_back(timeit(arms[q].second, reps));
      printf("  %d interleaved rounds of %d launches per arm: median (min)\n", rounds, reps);
      for (size_t q = 0; q < arms.size(); ++q) {
        std::vector<float> v = t[q];
        std::sort(v.begin(), v.end());
        printf("  %-44s %8.4f ms  %6.2f TF   (%6.2f)\n", arms[q].first.c_str(), v[v.size() / 2], flop / v[v.size() / 2] / 1e9,
               flop / v[0] / 1e9);
      }
    };
    interleaved(arms);
    if (!pmc) {   // stamped probe: phase shares per wave and, per CU, how many of its workgroups are in their K loop
      const long nw = (long)live * ngt * 4;
      AP(0, true);
      AP(0, true);
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> t((size_t)nw * NSTAMP);
      CK(hipMemcpy(t.data(), dstamp, sizeof(unsigned long long) * t.size(), hipMemcpyDeviceToHost));
      double sum[8] = {};
      long cnt = 0;
      std::map<long, std::vector<std::pair<unsigned long long, int>>> ev;   // CU -> (time, +1/-1 K loop; +2/-2 epilogue)
      for (long i = 0; i < nw; ++i) {
        const unsigned long long* r = &t[(size_t)i * NSTAMP];
        if (r[6] == 0) continue;   // idle wave
        for (int j = 1; j <= 6; ++j) sum[j] += (double)(r[j] - r[j - 1]);
        sum[7] += (double)(r[6] - r[0]);
        ++cnt;
        if (i % 4 == 0) {
          const long cu = ((long)(r[8] & 0xf) << 16) | (long)((r[7] >> 8) & 0xff);
          ev[cu].push_back({r[0], 1});
          ev[cu].push_back({r[1], -1});
          ev[cu].push_back({r[1], 2});
          ev[cu].push_back({r[6], -2});
        }
      }
      const char* nm[8] = {"", "K loop", "hhT stage + W0 blocks 0,1 landed", "block 0 (E, rule, stores)", "block 1", "block 2",
                           "block 3", "whole tile"};
      printf("  stamped probe: %ld waves; mean cycles per wave-tile:\n", cnt);
      for (int j = 1; j <= 7; ++j) printf("    %-36s %9.0f  (%5.1f %%)\n", nm[j], sum[j] / cnt, 100.0 * sum[j] / sum[7]);
      // per CU: time with 0 / 1 / 2 / 3 workgroups in their K loop (between its first start and last end)
      double occ[5] = {}, epi_k0 = 0, tot = 0;
      for (auto& [cu, v] : ev) {
        std::sort(v.begin(), v.end());
        int nk = 0, ne = 0;
        for (size_t q = 0; q + 1 < v.size(); ++q) {
          if (v[q].second == 1 || v[q].second == -1) nk += v[q].second; else ne += v[q].second / 2;
          const double dt = (double)(v[q + 1].first - v[q].first);
          occ[nk < 4 ? nk : 4] += dt;
          if (nk == 0 && ne > 0) epi_k0 += dt;
          tot += dt;
        }
      }
      printf("  per CU, share of time with 0/1/2/3 workgroups in their K loop: %.1f / %.1f / %.1f / %.1f %% "
             "(%.1f %% with none in a K loop and one in its epilogue); %zu CUs\n", 100 * occ[0] / tot, 100 * occ[1] / tot,
             100 * occ[2] / tot, 100 * occ[3] / tot, 100 * epi_k0 / tot, ev.size());
    }
    const long n_cols_pad = (n + 127) / 128 * 128, g_ld = n_cols_pad, g_split = cols * g_ld;
    const int ntj = (int)(n_cols_pad / 128), ng = npanels / 4;
    printf("== W^T A, n = %ld (%d sample tiles)\n", n, ntj);
#define WA(...) WAT(512, __VA_ARGS__)
#define WAT(NTHR, ...) hipLaunchKernelGGL((k_wta2<__VA_ARGS__>), dim3(nsplit * ng * ntj), dim3(NTHR), 0, 0, W, Ablk, m_pad, ng, ntj, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, (long)sq)
    if (!pmc && ntj >= 4) {   // the 16-wave tile's G and Gram partials against the engine's 8-wave tile, bit for bit
      const size_t gn = (size_t)nsplit * g_split, sn = (size_t)nsplit * sq;
      std::vector<double> g1(gn), g2(gn), s1(sn), s2(sn);
      auto grab = [&](std::vector<double>& g, std::vector<double>& sw, auto launch) {
        CK(hipMemset(Gpart, 0xff, sizeof(double) * gn));
        CK(hipMemset(SWpart, 0xff, sizeof(double) * sn));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(g.data(), Gpart, sizeof(double) * gn, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sw.data(), SWpart, sizeof(double) * sn, hipMemcpyDeviceToHost));
      };
      grab(g1, s1, [&] { WA(4, 128, 4, 2, 1, 3, 1, true, true, false, true); });
      grab(g2, s2, [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, true); });
      printf("  16-wave GREG vs engine (block packing): G partials %s, Gram partials %s\n",
             memcmp(g1.data(), g2.data(), sizeof(double) * gn) ? "DIFFER" : "bit-identical",
             memcmp(s1.data(), s2.data(), sizeof(double) * sn) ? "DIFFER" : "bit-identical");
      // contiguous packing (restarts straddle 16-column blocks, never panels): every straddling Gram block through
      // the 16-wave tile's register chains against the 8-wave tile's LDS chains
      std::vector<ColInfo> cj((size_t)npanels * PANEL, ColInfo{0, 0, 0, 0});
      std::vector<RestartInfo> rj;
      std::vector<int> pb(npanels, 0), pe(npanels, 0);
      int col = 0, sqj = 0, nstr = 0;
      for (int k = 10; k >= 2; --k)
        for (int r = 0; r < R; ++r) {
          if (col % PANEL + k > PANEL) col = (col / PANEL + 1) * PANEL;
          if (col + k > npanels * PANEL) break;
          const int id = (int)rj.size();
          rj.push_back({col, k, id, sqj});
          for (int a = 0; a < k; ++a) cj[(size_t)col + a] = ColInfo{sqj, col % PANEL, k, id};
          nstr += (col >> 4) != ((col + k - 1) >> 4);
          sqj += k * k;
          col += k;
        }
      for (int p = 0; p < npanels; ++p) {
        pb[p] = (int)rj.size();
        pe[p] = (int)rj.size();
      }
      for (size_t q = rj.size(); q-- > 0;) pb[rj[q].col0 / PANEL] = (int)q;
      for (size_t q = 0; q < rj.size(); ++q) pe[rj[q].col0 / PANEL] = (int)q + 1;
      for (int p = 0; p < npanels; ++p)
        if (pe[p] < pb[p]) pe[p] = pb[p];
      std::vector<ColInfo> ci_save(cols);
      CK(hipMemcpy(ci_save.data(), dci, sizeof(ColInfo) * cols, hipMemcpyDeviceToHost));
      std::vector<RestartInfo> ri_save(nall);
      CK(hipMemcpy(ri_save.data(), dri, sizeof(RestartInfo) * nall, hipMemcpyDeviceToHost));
      std::vector<int> pbs(npanels), pes(npanels);
      CK(hipMemcpy(pbs.data(), dprb, sizeof(int) * npanels, hipMemcpyDeviceToHost));
      CK(hipMemcpy(pes.data(), dpre, sizeof(int) * npanels, hipMemcpyDeviceToHost));
      CK(hipMemcpy(dci, cj.data(), sizeof(ColInfo) * cols, hipMemcpyHostToDevice));
      CK(hipMemcpy(dri, rj.data(), sizeof(RestartInfo) * std::min<size_t>(rj.size(), nall), hipMemcpyHostToDevice));
      CK(hipMemcpy(dprb, pb.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
      CK(hipMemcpy(dpre, pe.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
      const size_t sj = std::min<size_t>((size_t)sqj, (size_t)sq);
      grab(g1, s1, [&] { WA(4, 128, 4, 2, 1, 3, 1, true); });
      grab(g2, s2, [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, true); });
      bool same_sw = true;
      for (int sp = 0; sp < nsplit; ++sp)
        same_sw = same_sw && !memcmp(s1.data() + (size_t)sp * sq, s2.data() + (size_t)sp * sq, sizeof(double) * sj);
      printf("  16-wave GREG vs 8-wave LDS Gram (contiguous packing, %d of %zu restarts straddle a block): Gram partials %s\n",
             nstr, rj.size(), same_sw ? "bit-identical" : "DIFFER");
      CK(hipMemcpy(dci, ci_save.data(), sizeof(ColInfo) * cols, hipMemcpyHostToDevice));
      CK(hipMemcpy(dri, ri_save.data(), sizeof(RestartInfo) * nall, hipMemcpyHostToDevice));
      CK(hipMemcpy(dprb, pbs.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
      CK(hipMemcpy(dpre, pes.data(), sizeof(int) * npanels, hipMemcpyHostToDevice));
    }
    // stream-K form (round 6): bit identity against the engine's big tile, the recompute path included
    double* fixb = nullptr;
    unsigned* flg = nullptr;
    unsigned epoch = 0;
    int ncu = 256;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&fixb, sizeof(double) * SK_FIX * ncu));
    CK(hipMalloc(&flg, sizeof(unsigned) * ncu));
    CK(hipMemset(flg, 0, sizeof(unsigned) * ncu));
    const long sk_stages = (long)ng * ntj * ((m_pad + 15) / 16);
    const int gsk = (int)std::min<long>(ncu, sk_stages / (kchunk / 16));
    auto SK = [&](int G, bool nowait, int dpx = 0) {
      ++epoch;
      const SkArgs a{W, Ablk, m_pad, ng, ntj, kchunk, dprb, dpre, dri, dci, stop, Gpart, g_ld, g_split, SWpart, (long)sq,
                     fixb, flg, epoch, nsplit, nullptr, dpx};
      if (nowait)
        hipLaunchKernelGGL((k_wta2_sk<3, true>), dim3(G), dim3(SK_THREADS), 0, 0, a);
      else
        hipLaunchKernelGGL((k_wta2_sk<3>), dim3(G), dim3(SK_THREADS), 0, 0, a);
    };
    if (!pmc && ntj >= 4) {
      const size_t gn = (size_t)nsplit * g_split, sn = (size_t)nsplit * sq;
      std::vector<double> g1(gn), g2(gn), s1(sn), s2(sn);
      auto grab = [&](std::vector<double>& g, std::vector<double>& sw, auto launch) {
        CK(hipMemset(Gpart, 0xff, sizeof(double) * gn));
        CK(hipMemset(SWpart, 0xff, sizeof(double) * sn));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(g.data(), Gpart, sizeof(double) * gn, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sw.data(), SWpart, sizeof(double) * sn, hipMemcpyDeviceToHost));
      };
      grab(g1, s1, [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, true); });
      for (int G : {gsk, gsk / 2 + 1, 37}) {
        for (int nw = 0; nw < 3; ++nw) {
          grab(g2, s2, [&] { SK(G, nw == 1, nw == 2); });
          printf("  stream-K G=%d%s vs engine big tile: G partials %s, Gram partials %s\n", G,
                 nw == 1 ? " (recompute path)" : nw == 2 ? " (XCD-contiguous rounds)" : "",
                 memcmp(g1.data(), g2.data(), sizeof(double) * gn) ? "DIFFER" : "bit-identical",
                 memcmp(s1.data(), s2.data(), sizeof(double) * sn) ? "DIFFER" : "bit-identical");
        }
      }
    }
    std::vector<std::pair<std::string, std::function<void()>>> warms;
    if (ntj >= 4) {
      warms = {
          {"k_wta2 big 4x128 nbuf3 GREG (8 waves)", [&] { WA(4, 128, 4, 2, 1, 3, 1, true, true, false, true); }},
          {"  16 waves, GREG (engine)", [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, true); }},
          {"  stream-K 16 waves GREG, G = CUs", [&] { SK(gsk, false); }},
          {"  stream-K, XCD-contiguous whole rounds", [&] { SK(gsk, false, 1); }},
          {"  stream-K, recompute path (no hand-off)", [&] { SK(gsk, true); }},
          {"  Gram in LDS chains (round 3 form)", [&] { WA(4, 128, 4, 2, 1, 3, 1, true); }},
          {"  no Gram chains", [&] { WA(4, 128, 4, 2, 1, 3, 1, true, false); }},
          {"  nbuf 2, LDS Gram", [&] { WA(4, 128, 4, 2, 1, 2, 1, true); }},
          {"  16 waves (4 x 4), no Gram", [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, false); }},
          {"  16 waves, GREG", [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, true); }},
          {"  16 waves, GREG, first 6 x 256 items only", [&] {
             hipLaunchKernelGGL((k_wta2<4, 128, 4, 4, 1, 3, 1, true, true, false, true>), dim3(std::min(6 * 256, nsplit * ng * ntj)),
                                dim3(1024), 0, 0, W, Ablk, m_pad, ng, ntj, nsplit, kchunk, dprb, dpre, dri, dci, stop, Gpart,
                                g_ld, g_split, SWpart, (long)sq);
           }},
          {"  16 waves, GREG, unsplit steps", [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, true, false); }},
          {"  16 waves, LDS Gram, unsplit steps", [&] { WAT(1024, 4, 128, 4, 4, 1, 3, 1, true, true, false, false, false); }},
          {"  8 waves, GREG, unsplit steps", [&] { WA(4, 128, 4, 2, 1, 3, 1, true, true, false, true, false); }},
      };
    } else {
      warms = {{"k_wta2 big 4x128 nbuf3 GPW2 (engine)", [&] { WA(4, 128, 4, 2, 2, 3, 1, true); }}};
    }
    interleaved(warms);
  }
  printf("done\n");
  return 0;
}
