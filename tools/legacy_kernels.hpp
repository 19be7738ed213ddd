// tools/legacy_kernels.hpp -- superseded kernel generations, kept ONLY for tools/kbench.hip's cost
// breakdowns (round 1: register-prefetch Tile core, k_wta, k_ahtw_t, k_ahtw2).  Not part of the
// product library: nmfconsensus_amd/csrc/nmfc_kernels.hpp holds the kernels the engine launches.
#pragma once
#include "../nmfconsensus_amd/csrc/nmfc_kernels.hpp"

namespace nmfc {
// ---------------------------------------------------------------------------------------------
// The MFMA tile: RP x RQ outputs, 4 waves arranged WR x WC, K range [kbeg, kend) in stages of BK.
// DB: double-buffered LDS stages; otherwise one stage buffer + register prefetch (less LDS, so two
// workgroups share a CU and one's epilogue overlaps the other's MFMA loop).
// ---------------------------------------------------------------------------------------------
template <int RP, int RQ, int WR, int WC, bool DB>
struct Tile {
  static_assert(WR * WC == 4, "4 waves");
  static constexpr int MB = RP / WR / 16;            // 16x16 blocks per wave, rows
  static constexpr int NB = RQ / WC / 16;            // 16x16 blocks per wave, cols
  static constexpr int PL = RP / 16;                 // 16-byte loads per lane per stage for P
  static constexpr int QL = RQ / 16;
  static constexpr int STAGE = (RP + RQ) * BK;       // doubles per LDS stage
  static constexpr int LDS_DOUBLES = DB ? 2 * STAGE : STAGE;

  d4 acc[MB][NB];
  d2 pr[DB ? 2 : 1][PL], qr[DB ? 2 : 1][QL];   // register prefetch sets (two: loads run 2 stages ahead)
  // operand blocks as buffer resources: one 32-bit row offset per load, the K position in soffset
  __amdgpu_buffer_rsrc_t rp, rq;
  int vop[PL], voq[QL];

  __device__ __forceinline__ void bind(const double* P, long ldp, const double* Q, long ldq) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(P), 0, (int)(RP * ldp * 8), 0x00020000);
    rq = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(Q), 0, (int)(RQ * ldq * 8), 0x00020000);
#pragma unroll
    for (int i = 0; i < PL; ++i) vop[i] = (int)(((long)(i * 16 + w * 4 + (l >> 4)) * ldp + (l & 15) * 2) * 8);
#pragma unroll
    for (int i = 0; i < QL; ++i) voq[i] = (int)(((long)(i * 16 + w * 4 + (l >> 4)) * ldq + (l & 15) * 2) * 8);
  }

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  }

  // one wave-instruction moves 4 rows x 256 B; lane l -> row (l >> 4), 16-byte slot (l & 15)
  template <int SET = 0>
  __device__ __forceinline__ void gload(int k0) {
    const int so = k0 * 8;
#pragma unroll
    for (int i = 0; i < PL; ++i)
      pr[SET][i] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rp, vop[i], so, 0));
#pragma unroll
    for (int i = 0; i < QL; ++i)
      qr[SET][i] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rq, voq[i], so, 0));
  }

  template <int SET = 0>
  __device__ __forceinline__ void swrite(double* __restrict__ st) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int slot = l & 15;
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      const int row = i * 16 + w * 4 + (l >> 4);
      *reinterpret_cast<d2*>(st + row * BK + ((slot ^ (row & 11)) << 1)) = pr[SET][i];
    }
    double* sq = st + RP * BK;
#pragma unroll
    for (int i = 0; i < QL; ++i) {
      const int row = i * 16 + w * 4 + (l >> 4);
      *reinterpret_cast<d2*>(sq + row * BK + ((slot ^ (row & 11)) << 1)) = qr[SET][i];
    }
  }

  // lane group g = l >> 4 covers k = 8g + 2*kk2 + {0,1}: one ds_read_b128 per fragment and k pair
  __device__ __forceinline__ void compute(const double* __restrict__ st) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int wr = w / WC, wc = w % WC;
    const int fr = l & 15, g = l >> 4;
    const int sw = fr & 11;
    const double* sp = st + (wr * (RP / WR) + fr) * BK;
    const double* sq = st + RP * BK + (wc * (RQ / WC) + fr) * BK;
#pragma unroll
    for (int kk2 = 0; kk2 < 4; ++kk2) {
      const int off = (((4 * g + kk2) ^ sw) << 1);
      d2 a[MB], b[NB];
#pragma unroll
      for (int i = 0; i < MB; ++i) a[i] = *reinterpret_cast<const d2*>(sp + i * 16 * BK + off);
#pragma unroll
      for (int j = 0; j < NB; ++j) b[j] = *reinterpret_cast<const d2*>(sq + j * 16 * BK + off);
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
      if (DB) __builtin_amdgcn_sched_barrier(0);   // keep fragment loads from hoisting across k pairs
    }
  }

  // Double-buffered LDS with loads two stages ahead (register sets 0/1 alternate with the stage
  // parity); `extra(stage)` lets a kernel add work on the staged tile (k_wta's Gram blocks).
  template <bool DEEP = true, class Extra>
  __device__ __forceinline__ void run_db(const double* __restrict__ P, long ldp, const double* __restrict__ Q,
                                         long ldq, int kbeg, int kend, double* __restrict__ smem, Extra extra) {
    const int nst = (kend - kbeg) / BK;
    double* b0 = smem;
    double* b1 = smem + STAGE;
    bind(P, ldp, Q, ldq);
    if (!DEEP) {   // loads one stage ahead, one register set (lower register pressure)
      gload<0>(kbeg);
      swrite<0>(b0);
      __syncthreads();
      for (int s = 0; s < nst; ++s) {
        const bool more = s + 1 < nst;
        if (more) gload<0>(kbeg + (s + 1) * BK);
        double* cur = (s & 1) ? b1 : b0;
        compute(cur);
        extra(cur);
        if (more) swrite<0>((s & 1) ? b0 : b1);
        __syncthreads();
      }
      return;
    }
    gload<0>(kbeg);
    if (nst > 1) gload<1>(kbeg + BK);
    swrite<0>(b0);
    __syncthreads();
    for (int s = 0; s < nst; s += 2) {
      if (s + 2 < nst) gload<0>(kbeg + (s + 2) * BK);
      compute(b0);
      extra(b0);
      if (s + 1 < nst) swrite<1>(b1);
      __syncthreads();
      if (s + 1 >= nst) break;
      if (s + 3 < nst) gload<1>(kbeg + (s + 3) * BK);
      compute(b1);
      extra(b1);
      if (s + 2 < nst) swrite<0>(b0);
      __syncthreads();
    }
  }

  __device__ __forceinline__ void run(const double* __restrict__ P, long ldp, const double* __restrict__ Q, long ldq,
                                      int kbeg, int kend, double* __restrict__ smem) {
    if (DB) {
      run_db(P, ldp, Q, ldq, kbeg, kend, smem, [](const double*) {});
      return;
    }
    const int nst = (kend - kbeg) / BK;
    bind(P, ldp, Q, ldq);
    gload(kbeg);
    swrite(smem);
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
      const bool more = s + 1 < nst;
      if (more) gload(kbeg + (s + 1) * BK);
      compute(smem);
      __syncthreads();
      if (more) {
        swrite(smem);
        __syncthreads();
      }
    }
  }

  // C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
  __device__ __forceinline__ static int row_of(int mb, int reg) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    return (w / WC) * (RP / WR) + mb * 16 + (l >> 4) + 4 * reg;
  }
  __device__ __forceinline__ static int col_of(int nb) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    return (w % WC) * (RQ / WC) + nb * 16 + (l & 15);
  }
};
// ---------------------------------------------------------------------------------------------
// K1 "wta":  G = W^T A  (nmf_mu.c:174), 128 x 128 tiles over (panel pair, sample tile); the gene
// range is cut into fixed chunks (a function of m only, so each entry's summation order is
// independent of batch composition); partials are summed in chunk order by k_hupdate.
// ---------------------------------------------------------------------------------------------
using TileH = Tile<128, 128, 2, 2, true>;

// Gram blocks of a panel pair needed by restarts with k <= 16: per panel the diagonal 16x16 blocks
// (b, b) and the straddling blocks (b, b+1); 14 candidates spread over the pair's ntj sample-tile
// workgroups and their 4 waves: wave w of tile t takes candidates t + ntj * (w + 4x).
constexpr int GRAM_CAND = 14;

__device__ __forceinline__ void gram_block_of(int cand, int& q, int& br, int& bc) {
  q = cand / 7;
  const int x = cand % 7;
  if (x < 4) {
    br = x;
    bc = x;
  } else {
    br = x - 4;
    bc = x - 3;
  }
}

// ---------------------------------------------------------------------------------------------
// K1 "wta":  G = W^T A  (nmf_mu.c:174), 128 x 128 tiles over (panel pair, sample tile), and the
// Gram W^T W (nmf_mu.c:176) restricted to the 16x16 blocks that carry restart-diagonal k x k blocks,
// from the same LDS-staged W tile (a few extra MFMAs per wave, spread evenly).  The gene range is cut into fixed
// chunks (a function of m only, so each entry's summation order is independent of batch
// composition); per-chunk partials are summed in chunk order by k_hupdate.
// ---------------------------------------------------------------------------------------------
// GRAM_PER_WAVE = ceil(14 / (4 * ntj)) candidates per wave (1 for n > 384), chosen by the host.
template <int GRAM_PER_WAVE, bool DEEP>
static __global__ __launch_bounds__(NT) void k_wta(const double* __restrict__ W, const double* __restrict__ Acm,
                                                   long m_pad, int npairs, int ntj, int nsplit, int kchunk,
                                                   const int* __restrict__ prb, const int* __restrict__ pre,
                                                   const RestartInfo* __restrict__ ri, const ColInfo* __restrict__ ci,
                                                   const int* __restrict__ stop_iter, double* __restrict__ Gpart,
                                                   long g_ld, long g_split, double* __restrict__ SWpart,
                                                   long sw_total) {
  __shared__ __attribute__((aligned(16))) double smem[TileH::LDS_DOUBLES];
  __shared__ int need[GRAM_CAND];
  const int nitems = nsplit * npairs * ntj;
  const int item = xcd_item(blockIdx.x, nitems);
  const int t = item % ntj;
  const int pp = (item / ntj) % npairs;
  const int s = item / (ntj * npairs);
  const bool live0 = panel_live(prb, pre, 2 * pp, ri, stop_iter, 0);
  const bool live1 = panel_live(prb, pre, 2 * pp + 1, ri, stop_iter, 0);
  if (!live0 && !live1) return;
  if (threadIdx.x < GRAM_CAND) {
    int q, br, bc;
    gram_block_of(threadIdx.x, q, br, bc);
    int nd = (q == 0) ? live0 : live1;
    if (nd && br != bc) {   // straddling block: needed only if a restart spans columns 16*bc-1 and 16*bc
      const ColInfo c = ci[(long)(2 * pp + q) * PANEL + 16 * bc];
      nd = (c.k > 0 && c.lc0 < 16 * bc);
    }
    need[threadIdx.x] = nd;
  }
  const double* P = W + (long)pp * 128 * m_pad;
  const double* Q = Acm + (long)t * 128 * m_pad;
  const int kbeg = s * kchunk;
  const int kend = (int)min((long)kbeg + kchunk, m_pad);
  TileH tl;
  tl.zero();
  d4 gacc[GRAM_PER_WAVE];
#pragma unroll
  for (int x = 0; x < GRAM_PER_WAVE; ++x) gacc[x] = (d4){0.0, 0.0, 0.0, 0.0};
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int fr = l & 15, g = l >> 4, sw = fr & 11;
  __syncthreads();   // need[] visible
  int my_need[GRAM_PER_WAVE];
  int my_ra[GRAM_PER_WAVE], my_rb[GRAM_PER_WAVE];
  bool gram = false;
#pragma unroll
  for (int x = 0; x < GRAM_PER_WAVE; ++x) {
    const int cand = t + ntj * (w + 4 * x);
    my_need[x] = 0;
    my_ra[x] = 0;
    my_rb[x] = 0;
    if (cand < GRAM_CAND) {
      int q, br, bc;
      gram_block_of(cand, q, br, bc);
      my_need[x] = need[cand];
      my_ra[x] = 64 * q + 16 * br;
      my_rb[x] = 64 * q + 16 * bc;
      gram = gram || my_need[x];
    }
  }
  tl.template run_db<DEEP>(P, m_pad, Q, m_pad, kbeg, kend, smem, [&](const double* stg) {
    if (!gram) return;
#pragma unroll
    for (int x = 0; x < GRAM_PER_WAVE; ++x) {
      if (!my_need[x]) continue;
      const double* pa = stg + (my_ra[x] + fr) * BK;
      const double* pb = stg + (my_rb[x] + fr) * BK;
#pragma unroll
      for (int kk2 = 0; kk2 < 4; ++kk2) {
        const int off = (((4 * g + kk2) ^ sw) << 1);
        const d2 a = *reinterpret_cast<const d2*>(pa + off);
        const d2 b = *reinterpret_cast<const d2*>(pb + off);
        gacc[x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b.x, gacc[x], 0, 0, 0);
        gacc[x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b.y, gacc[x], 0, 0, 0);
      }
    }
  });
  double* out = Gpart + (long)s * g_split + (long)pp * 128 * g_ld + (long)t * 128;
#pragma unroll
  for (int mb = 0; mb < TileH::MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < TileH::NB; ++nb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        out[(long)TileH::row_of(mb, reg) * g_ld + TileH::col_of(nb)] = tl.acc[mb][nb][reg];
  if (gram) {
    double* so = SWpart + (long)s * sw_total;
#pragma unroll
    for (int x = 0; x < GRAM_PER_WAVE; ++x) {
      if (!my_need[x]) continue;
      const int pnl = my_ra[x] >> 6;   // panel within the pair
      const ColInfo* cp = ci + (long)(2 * pp + pnl) * PANEL;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int lr = (my_ra[x] & 63) + g + 4 * reg;   // panel-local row column index
        const int lcn = (my_rb[x] & 63) + fr;           // panel-local col column index
        const ColInfo cr = cp[lr];
        if (cr.k == 0 || cr.lc0 != cp[lcn].lc0 || cp[lcn].k == 0) continue;   // not the same restart
        const int a = lr - cr.lc0, b = lcn - cr.lc0;
        so[cr.sq_off + a * cr.k + b] = gacc[x][reg];
        so[cr.sq_off + b * cr.k + a] = gacc[x][reg];
      }
    }
  }
}
// ---------------------------------------------------------------------------------------------
// K3 "ahtw": F = A h^T (nmf_mu.c:198) computed transposed per tile (rows = the 64 columns of panel
// p, cols = GT genes), fused with work2w = W0 (h h^T) (:202) and the W rule (:209-216), written in
// place.  The epilogue runs in the MFMA accumulator layout (F never leaves registers); the W0 tile is
// prefetched into registers during the last K stage and staged in LDS with the panel's h h^T blocks.
// ---------------------------------------------------------------------------------------------
using TileW = Tile<64, 128, 1, 4, false>;
constexpr int WLS = GT + 2;        // LDS row stride of the W0 tile (16-byte aligned rows)
constexpr int SHS = KMAX + 1;      // LDS row stride of the h h^T rows
constexpr int AHTW_EPI = PANEL * WLS + PANEL * SHS;
constexpr int AHTW_LDS = (TileW::LDS_DOUBLES > AHTW_EPI) ? TileW::LDS_DOUBLES : AHTW_EPI;

// One (panel, gene tile) item of K3.  Returns without touching memory when the panel is idle.
// VARIANT != 0 only in tools/kbench (cost breakdown): 1 no W0 prefetch, 2 no E, 3 no W store.
template <int VARIANT>
__device__ __forceinline__ void ahtw_item(int item, int iter, const double* __restrict__ H, long n_pad,
                                          const double* __restrict__ Arm, long m_pad, double* __restrict__ W,
                                          const double* __restrict__ SH, const int* __restrict__ prb,
                                          const int* __restrict__ pre, const RestartInfo* __restrict__ ri,
                                          const ColInfo* __restrict__ ci, const int* __restrict__ stop_iter,
                                          int npanels, int ngt, double* __restrict__ smem, int* __restrict__ c_lc0,
                                          int* __restrict__ c_k, int* __restrict__ c_act) {
  // bands of 8 panels, gene super-tiles of 8: neighbouring items share operands in L2
  int p, gt;
  {
    const int SP = 8, SG = 8;
    const int band = item / (SP * ngt);
    const int rem = item % (SP * ngt);
    const int bp = min(SP, npanels - band * SP);
    const int sg = rem / (bp * SG);
    const int gsz = min(SG, ngt - sg * SG);
    const int w2 = rem - sg * bp * SG;
    p = band * SP + w2 / gsz;
    gt = ngt - 1 - (sg * SG + w2 % gsz);   // high gene tiles first: W^T A streamed them last (MALL-warm)
  }
  if (!panel_live(prb, pre, p, ri, stop_iter, iter)) return;
  const int tid = threadIdx.x;
  const double* P = H + (long)p * PANEL * n_pad;
  const double* Q = Arm + (long)gt * GT * n_pad;
  const double* wsrc = W + (long)p * PANEL * m_pad + (long)gt * GT;
  TileW tl;
  tl.zero();
  d2 wpre[16];
  const int nst = (int)(n_pad / BK);
  tl.bind(P, n_pad, Q, n_pad);
  tl.gload(0);
  __syncthreads();   // the previous item's epilogue is done with smem
  tl.swrite(smem);
  __syncthreads();
  for (int st = 0; st + 1 < nst; ++st) {
    tl.gload((st + 1) * BK);
    tl.compute(smem);
    __syncthreads();
    tl.swrite(smem);
    __syncthreads();
  }
  // last stage: no staging load is in flight, so the W0 prefetch overlaps this stage's MFMAs
#pragma unroll
  for (int j = 0; j < 16; ++j)
    wpre[j] = VARIANT == 1 ? d2{1.0, 1.0}
                           : *reinterpret_cast<const d2*>(wsrc + (long)((tid >> 6) + 4 * j) * m_pad + (tid & 63) * 2);
  tl.compute(smem);
  __syncthreads();
  // epilogue staging: W0 tile, the panel's compact h h^T blocks, per-column restart info
  double* Wl = smem;
  double* SHl = smem + PANEL * WLS;
#pragma unroll
  for (int j = 0; j < 16; ++j) *reinterpret_cast<d2*>(Wl + ((tid >> 6) + 4 * j) * WLS + (tid & 63) * 2) = wpre[j];
  const int b0 = prb[p], e0 = pre[p];
  for (int q = b0; q < e0; ++q) {
    const RestartInfo r = ri[q];
    const int lc = r.col0 - p * PANEL;
    for (int idx = tid; idx < r.k * r.k; idx += NT) SHl[(lc + idx / r.k) * SHS + (idx % r.k)] = SH[r.sq_off + idx];
  }
  if (tid < PANEL) {
    const ColInfo c = ci[(long)p * PANEL + tid];
    c_lc0[tid] = c.lc0;
    c_k[tid] = c.k;
    int act = 0;
    if (c.k > 0) {
      const int sv = stop_iter[c.rid];
      act = (sv == 0 || sv == iter);
    }
    c_act[tid] = act;
  }
  __syncthreads();
  double* wdst = W + (long)p * PANEL * m_pad + (long)gt * GT;
  // E = S W0 on the MFMA pipe.  S is the panel's block-diagonal h h^T: row c holds SH_r[c - lc0][.]
  // on its restart's columns lc0..lc0+k-1 and zeros elsewhere (all zeros for idle columns).  The
  // f64 MFMA is a k-ordered fma chain, so E[c][i] = sum_b SH_r[c-lc0][b] W0[lc0+b][i] accumulates
  // exactly like the VALU chain b = 0..k-1 of nmf_mu.c:202: the zero terms around the block leave
  // the chain unchanged.  K runs only over the columns the 16 rows of a block touch.
  const int lane = tid & 63;
  d4 e[TileW::MB][TileW::NB];
  int kss[TileW::MB][4];
#pragma unroll
  for (int mb = 0; mb < TileW::MB; ++mb) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int c = TileW::row_of(mb, reg);
      kss[mb][reg] = c_act[c] ? c_k[c] : 0;
    }
    const int ra = mb * 16 + (lane & 15);   // MFMA A-operand row of this lane
    const int alc = c_lc0[ra];
    const int ak = (VARIANT == 2 || !c_act[ra]) ? 0 : c_k[ra];
    int lo = ak ? alc : PANEL, hi = ak ? alc + ak : 0;
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {
      lo = min(lo, __shfl_xor(lo, off));
      hi = max(hi, __shfl_xor(hi, off));
    }
    lo = __builtin_amdgcn_readfirstlane(lo) & ~3;
    hi = __builtin_amdgcn_readfirstlane(hi);
#pragma unroll
    for (int nb = 0; nb < TileW::NB; ++nb) e[mb][nb] = d4{0.0, 0.0, 0.0, 0.0};
    for (int kk = lo; kk < hi; kk += 4) {
      const int cp = kk + (lane >> 4);
      const int bb = cp - alc;
      const double av = (bb >= 0 && bb < ak) ? SHl[ra * SHS + bb] : 0.0;
#pragma unroll
      for (int nb = 0; nb < TileW::NB; ++nb) {
        const double bv = cp < hi ? Wl[cp * WLS + TileW::col_of(nb)] : 0.0;
        e[mb][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, e[mb][nb], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int mb = 0; mb < TileW::MB; ++mb)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      if (!kss[mb][reg]) continue;
      const int c = TileW::row_of(mb, reg);
#pragma unroll
      for (int nb = 0; nb < TileW::NB; ++nb) {
        const int i = TileW::col_of(nb);
        const double v = mu_rule(Wl[c * WLS + i], tl.acc[mb][nb][reg], e[mb][nb][reg]);
        if (VARIANT != 3 || v == (double)iter * 1.5e300) wdst[(long)c * m_pad + i] = v;
      }
    }
}

// One item per workgroup; two workgroups share a CU (one's epilogue overlaps the other's MFMA loop).
template <int VARIANT>
static __global__ __launch_bounds__(NT, 2) void k_ahtw_t(int iter, const double* __restrict__ H, long n_pad,
                                                       const double* __restrict__ Arm, long m_pad,
                                                       double* __restrict__ W, const double* __restrict__ SH,
                                                       const int* __restrict__ prb, const int* __restrict__ pre,
                                                       const RestartInfo* __restrict__ ri,
                                                       const ColInfo* __restrict__ ci,
                                                       const int* __restrict__ stop_iter, int npanels, int ngt) {
  __shared__ __attribute__((aligned(16))) double smem[AHTW_LDS];
  __shared__ int c_lc0[PANEL], c_k[PANEL], c_act[PANEL];
  ahtw_item<VARIANT>(xcd_item(blockIdx.x, npanels * ngt), iter, H, n_pad, Arm, m_pad, W, SH, prb, pre, ri, ci, stop_iter,
            npanels, ngt, smem, c_lc0, c_k, c_act);
}

#define k_ahtw k_ahtw_t<0>
using TileW2 = GTile<64, 128, 1, 4, 2>;
constexpr int AHTW2_SH = TileW2::LDS_BYTES;                    // h h^T rows: 64 x AHTW2_SHS doubles
constexpr int AHTW2_SHS = KMAX + 1;                             // LDS row stride of the h h^T rows
constexpr int AHTW2_CI = AHTW2_SH + PANEL * AHTW2_SHS * 8;     // c_lc0 / c_k / c_act: 3 x 64 ints
constexpr int AHTW2_LDS = AHTW2_CI + 3 * PANEL * 4;

// MAIN = 0: GTile 2-stage DMA ring main loop; MAIN = 1: the register-prefetch Tile (TileW) main loop
// (single 48 KiB stage).  Both keep two workgroups per CU.
constexpr int AHTW3_SH = TileW::LDS_DOUBLES * 8;
constexpr int AHTW3_CI = AHTW3_SH + PANEL * AHTW2_SHS * 8;
constexpr int AHTW3_LDS = AHTW3_CI + 3 * PANEL * 4;

template <int VARIANT, int MAIN = 0>
static __global__ __launch_bounds__(256, 2) void k_ahtw2(int iter, const double* __restrict__ H, long n_pad,
                                                         const double* __restrict__ Arm, long m_pad,
                                                         double* __restrict__ W, const double* __restrict__ SH,
                                                         const int* __restrict__ prb, const int* __restrict__ pre,
                                                         const RestartInfo* __restrict__ ri,
                                                         const ColInfo* __restrict__ ci,
                                                         const int* __restrict__ stop_iter, int npanels, int ngt) {
  __shared__ __attribute__((aligned(1024))) char smem[MAIN ? AHTW3_LDS : AHTW2_LDS];
  double* SHl = reinterpret_cast<double*>(smem + (MAIN ? AHTW3_SH : AHTW2_SH));
  int* c_lc0 = reinterpret_cast<int*>(smem + (MAIN ? AHTW3_CI : AHTW2_CI));
  int* c_k = c_lc0 + PANEL;
  int* c_act = c_k + PANEL;
  int p, gt;
  ahtw_map(xcd_item(blockIdx.x, npanels * ngt), npanels, ngt, p, gt);
  if (!panel_live(prb, pre, p, ri, stop_iter, iter)) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  {   // the panel's h h^T blocks (row c = panel column, AHTW2_SHS doubles per row) and column info;
      // entry (c, b) per thread, all loads independent
#pragma unroll
    for (int j = 0; j < PANEL * KMAX / 256; ++j) {
      const int idx = tid + 256 * j, c = idx >> 4, b = idx & 15;
      const ColInfo cc = ci[(long)p * PANEL + c];
      if (b < cc.k) SHl[c * AHTW2_SHS + b] = SH[cc.sq_off + (c - cc.lc0) * cc.k + b];
      if (b == 0) {
        c_lc0[c] = cc.lc0;
        c_k[c] = cc.k;
        c_act[c] = cc.k > 0 ? (stop_iter[cc.rid] == 0 || stop_iter[cc.rid] == iter) : 0;
      }
    }
  }
  // (the ring prologue's barrier publishes SHl / c_* to the workgroup)
  using TT = std::conditional_t<MAIN == 1, TileW, TileW2>;
  TT tl;
  tl.zero();
  const double* wsrc = W + (long)p * PANEL * m_pad + (long)gt * GT + 32 * w + (lane & 15);
  double w0[TT::MB][TT::NB][4];
  auto load_w0 = [&] {
#pragma unroll
    for (int mb = 0; mb < TT::MB; ++mb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
#pragma unroll
        for (int nb = 0; nb < TT::NB; ++nb)
          w0[mb][nb][reg] = (VARIANT == 1 || VARIANT == 4) ? 1.0 : wsrc[(long)(16 * mb + (lane >> 4) + 4 * reg) * m_pad + 16 * nb];
  };
  const double* P = H + (long)p * PANEL * n_pad;
  const double* Q = Arm + (long)gt * GT * n_pad;
  if constexpr (MAIN == 0) {
    tl.template run<TT::MB * TT::NB * 4>(P, n_pad, Q, n_pad, 0, (int)n_pad, smem, [](const char*) {}, load_w0);
  } else {
    double* st = reinterpret_cast<double*>(smem);
    const int nst = (int)(n_pad / BK);
    tl.bind(P, n_pad, Q, n_pad);
    tl.gload(0);
    if (nst == 1) load_w0();
    __syncthreads();   // SHl / c_* staged
    tl.swrite(st);
    __syncthreads();
    for (int s2 = 0; s2 < nst; ++s2) {
      const bool more = s2 + 1 < nst;
      if (more) {
        tl.gload((s2 + 1) * BK);
        if (s2 + 2 == nst) load_w0();   // after the last staging load: the epilogue's W0 overlaps 2 stages
      }
      tl.compute(st);
      __syncthreads();
      if (more) {
        tl.swrite(st);
        __syncthreads();
      }
    }
  }
  double* wdst = W + (long)p * PANEL * m_pad + (long)gt * GT + 32 * w + (lane & 15);
#pragma unroll
  for (int mb = 0; mb < TT::MB; ++mb) {
    // E rows 16*mb .. +15 = sum over the restart's columns b of S[c][b] * W0[b][i]; K runs over the
    // 4-column groups q the block's restarts touch (wave-uniform range)
    const int ra = 16 * mb + (lane & 15);
    const int alc = c_lc0[ra];
    const int ak = (VARIANT == 2 || VARIANT == 4 || !c_act[ra]) ? 0 : c_k[ra];
    int lo = ak ? alc : PANEL, hi = ak ? alc + ak : 0;
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {
      lo = min(lo, __shfl_xor(lo, off));
      hi = max(hi, __shfl_xor(hi, off));
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    d4 e[TT::NB];
#pragma unroll
    for (int nb = 0; nb < TT::NB; ++nb) e[nb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (4 * q + 3 < lo || 4 * q >= hi) continue;   // wave-uniform
      const int bb = 4 * q + (lane >> 4) - alc;
      const double av = (bb >= 0 && bb < ak) ? SHl[ra * AHTW2_SHS + bb] : 0.0;
#pragma unroll
      for (int nb = 0; nb < TT::NB; ++nb)
        e[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, w0[q >> 2][nb][q & 3], e[nb], 0, 0, 0);
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int c = 16 * mb + (lane >> 4) + 4 * reg;
      if (!c_act[c]) continue;
#pragma unroll
      for (int nb = 0; nb < TT::NB; ++nb) {
        const double v = VARIANT == 4 ? tl.acc[mb][nb][reg] : mu_rule(w0[mb][nb][reg], tl.acc[mb][nb][reg], e[nb][reg]);
        if (VARIANT != 3 || v == (double)iter * 1.5e300) wdst[(long)c * m_pad + 16 * nb] = v;
      }
    }
  }
}

}  // namespace nmfc

// ---------------------------------------------------------------------------------------------
// Round-2 experiment, not kept: a persistent A h^T kernel that pipelines ACROSS tiles (the next tile's
// setup loads, h h^T rows and first ring stages are issued before the current tile's epilogue; W0 via
// untracked loads so the compiler's vmcnt insertion does not drain that DMA).  Bit-identical, but on C3
// it measured 49.7 TF vs 50.4 TF for k_ahtw4 (and slower on the R = 25 shard): the static round-robin
// tile walk loses more to imbalance than the overlap wins (gpurun_out r02n).
// ---------------------------------------------------------------------------------------------
namespace nmfc {
// A global load the compiler's wait-count insertion does not see (the caller waits with wait_vmcnt).
__device__ __forceinline__ double load_untracked(const double* p) {
  double v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// p[0] and p[16] (one address register pair for both)
__device__ __forceinline__ void load_untracked2(const double* p, double& a, double& b) {
  asm volatile("global_load_dwordx2 %0, %2, off\n\tglobal_load_dwordx2 %1, %2, off offset:128"
               : "=&v"(a), "=&v"(b)
               : "v"(p)
               : "memory");
}

// ---------------------------------------------------------------------------------------------
// K3 persistent form "ahtw_p" (the full-load shape of k_ahtw4: 1 panel x GTG genes, 4 waves, 2 workgroups
// per CU): each workgroup walks the items v = blockIdx.x, + gridDim.x, ... (same item map) and pipelines
// ACROSS tiles -- right after a tile's last MFMA stage it issues the next live tile's setup loads and its
// first D ring stages, then runs the tile's epilogue (E = W0 (h h^T) on MFMA, W rule, W stores) while that
// DMA is in flight.  The per-tile ring fill latency and the epilogue no longer leave the matrix pipe idle
// between tiles.  The arithmetic of every output is exactly k_ahtw4's (same K order), so it is
// bit-identical to every other A h^T shape.  Needs n_pad / BK2 >= GT_NBUF - 1 (n_pad >= 32).
// ---------------------------------------------------------------------------------------------
template <int GTG = GT>
static __global__ __launch_bounds__(256, 2) void k_ahtw_p(int iter, const double* __restrict__ H, long n_pad,
                                                          const double* __restrict__ Arm, long m_pad,
                                                          double* __restrict__ W, const double* __restrict__ SHP,
                                                          const ColInfo* __restrict__ ci,
                                                          const int* __restrict__ colact, int npanels, int ngt) {
  using TL = GTile<PANEL, GTG, 1, 4, GT_NBUF>;
  constexpr int D = GT_NBUF - 1;
  constexpr int XL = TL::MB * TL::NB * 4;   // W0 loads per lane, issued with the tile's last ring stage
  static_assert(GT_NBUF >= 3 && PANEL * KMAX * 8 == 8192 && TL::STAGE_BYTES >= 8192, "SH rows staged in ring slot D");
  __shared__ __attribute__((aligned(1024))) char smem[TL::LDS_BYTES + PANEL * KMAX * 8];
  double* SHl = reinterpret_cast<double*>(smem + TL::LDS_BYTES);
  const uint32_t base = (uint32_t)(uintptr_t)smem;
  const int nitems = npanels * ngt;
  const int nst = (int)(n_pad / BK2);
  const int tid = threadIdx.x, lane = tid & 63, wc = tid >> 6;
  TL tl;
  int v = blockIdx.x, p = 0, gt = 0;
  int c_lc0 = 0, c_k = 0;   // this lane's column: first panel-local column and k of its restart
  uint64_t actmask = 0;
  // claim the next live item from v on: setup loads first, then the tile's h h^T rows (8 KiB, one LDS-DMA
  // copy into ring slot D, which the K loop refills only at its first step) and the D prologue stages, so
  // waiting on the setup loads leaves the DMA in flight.  An idle tile (no column updated at this
  // iteration) is drained and skipped; every wave sees the same ballot.
  auto claim = [&]() -> bool {
    for (; v < nitems; v += gridDim.x) {
      ahtw_map(xcd_item(v, nitems), npanels, ngt, p, gt);
      const ColInfo* cip = ci + (long)p * PANEL + lane;
      c_lc0 = cip->lc0;
      c_k = cip->k;
      const int ca = colact[(long)p * PANEL + lane];
      __builtin_amdgcn_sched_barrier(0);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<double*>(SHP + (long)p * PANEL * KMAX), 0, PANEL * KMAX * 8, 0x00020000);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        lds_dma16(rs, base + D * TL::STAGE_BYTES + (uint32_t)(wc + 4 * j) * 1024u, (wc + 4 * j) * 1024 + 16 * lane, 0);
      tl.bind(H + (long)p * PANEL * n_pad, n_pad, Arm + (long)gt * GTG * n_pad, n_pad, (int)n_pad);
#pragma unroll
      for (int q = 0; q < D; ++q) tl.issue(base + q * TL::STAGE_BYTES, q * BK2);
      __builtin_amdgcn_sched_barrier(0);
      // (c_k >= 0 keeps the ColInfo loads ahead of the DMA: they complete with ca, before the stages)
      actmask = __ballot(ca == iter && c_k >= 0);
      if (actmask != 0) return true;
      wait_vmcnt<0>();
    }
    return false;
  };
  if (!claim()) return;
  bool first = true;
  for (;;) {
    const int cp = p, cgt = gt;
    const int cc_lc0 = c_lc0, cc_k = c_k;
    const uint64_t cam = actmask;
    // laundered per tile: otherwise the 32 W0 / W row offsets are hoisted out of the tile loop (registers)
    long mp = m_pad;
    asm volatile("" : "+s"(mp));
    const double* wsrc = W + (long)cp * PANEL * mp + (long)cgt * GTG + (GTG / 4) * wc + (lane & 15);
    double w0[TL::MB][TL::NB][4];
    auto load_w0 = [&] {
#pragma unroll
      for (int mb = 0; mb < TL::MB; ++mb)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const double* rowp = wsrc + (long)(16 * mb + (lane >> 4) + 4 * reg) * mp;
          if constexpr (TL::NB == 2)
            load_untracked2(rowp, w0[mb][0][reg], w0[mb][1][reg]);
          else
            w0[mb][0][reg] = load_untracked(rowp);
        }
    };
    tl.zero();
    bool xl = first ? false : true;   // the previous tile's XL W stores are still in flight
    if (nst == D) {
      load_w0();
      xl = true;
    }
    TL::template wait_stages<D - 1, XL>(D - 1, xl);   // stage 0 and (older) the h h^T rows have landed
    step_barrier();   // ... for every wave; every wave is also past the previous tile's epilogue (SHl free)
    {
      const d2* stg = reinterpret_cast<const d2*>(smem + D * TL::STAGE_BYTES);
      const d2 a0 = stg[tid], a1 = stg[tid + 256];
      reinterpret_cast<d2*>(SHl)[tid] = a0;
      reinterpret_cast<d2*>(SHl)[tid + 256] = a1;
    }
    step_barrier();   // slot D read by every wave before step 0 refills it; SHl published
    int b = 0;
    for (int s = 0; s < nst; ++s) {
      if (s + D < nst) {
        const int bd = (b + D >= GT_NBUF) ? b + D - GT_NBUF : b + D;
        tl.issue(base + bd * TL::STAGE_BYTES, (s + D) * BK2);
        if (s + D + 1 == nst) {
          load_w0();
          xl = true;
        }
      }
      tl.compute(smem + b * TL::STAGE_BYTES);
      if (s + 1 < nst) {
        const int left = nst - s - 2;
        // the stores are older than stage D: from step 1 on, waiting for stage s + 1 covers them
        if (s + D + 1 < nst && s >= 1) xl = false;
        TL::template wait_stages<D - 1, XL>(left < D - 1 ? left : D - 1, xl);
        step_barrier();
      }
      b = (b + 1 == GT_NBUF) ? 0 : b + 1;
    }
    first = false;
    step_barrier();   // every wave is done with the ring: the next tile's prologue may refill it
    v += gridDim.x;
    const bool more = claim();
    // W0 came through untracked loads (the compiler would wait for them with vmcnt(0), draining the next
    // tile's DMA): they are older than the claim's 2 h h^T and D * PPW stage DMA operations
    if (more)
      wait_vmcnt<2 + D * TL::PPW>();
    else
      wait_vmcnt<0>();
    // ---- epilogue of (cp, cgt), overlapping the next tile's DMA ----
    double* wdst = W + (long)cp * PANEL * mp + (long)cgt * GTG + (GTG / 4) * wc + (lane & 15);
#pragma unroll
    for (int mb = 0; mb < TL::MB; ++mb) {
      const int ra = 16 * mb + (lane & 15);
      const int alc = __shfl(cc_lc0, ra);
      const int ak = ((cam >> ra) & 1) ? __shfl(cc_k, ra) : 0;
      int lo = ak ? alc : PANEL, hi = ak ? alc + ak : 0;
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off));
        hi = max(hi, __shfl_xor(hi, off));
      }
      lo = __builtin_amdgcn_readfirstlane(lo);
      hi = __builtin_amdgcn_readfirstlane(hi);
      d4 e[TL::NB];
#pragma unroll
      for (int nb = 0; nb < TL::NB; ++nb) e[nb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4 * TL::MB; ++q) {
        if (4 * q + 3 < lo || 4 * q >= hi) continue;   // wave-uniform
        const int bb = 4 * q + (lane >> 4) - alc;
        const double av = (bb >= 0 && bb < ak) ? SHl[ra * KMAX + bb] : 0.0;
#pragma unroll
        for (int nb = 0; nb < TL::NB; ++nb)
          e[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, w0[q >> 2][nb][q & 3], e[nb], 0, 0, 0);
      }
      // every lane stores (an idle column gets its W0 back, unchanged): a fixed XL stores per tile, so the
      // next tile's first waits can leave them in flight
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int c = 16 * mb + (lane >> 4) + 4 * reg;
        const bool act = (cam >> c) & 1;
#pragma unroll
        for (int nb = 0; nb < TL::NB; ++nb) {   // mu_rule, branch-free (no execz skips around the stores)
          const double o = w0[mb][nb][reg], f = tl.acc[mb][nb][reg];
          const double t = o * (f / (e[nb][reg] + DIV_BY_ZERO_AVOIDANCE));
          const double nw = (o == 0.0 || f == 0.0 || t < 0.0) ? 0.0 : t;
          __builtin_nontemporal_store(act ? nw : o, wdst + (long)c * mp + 16 * nb);
        }
        __builtin_amdgcn_sched_barrier(0);   // bounded live ranges: no spills
      }
    }
    if (!more) break;
  }
}

// Round 2 experiment (not in the product: 73 us vs 66 us per narrow launch for the 16-stage LDS ring,
// profiles/r02/narrow_stream_vs_lds_kstats.txt): the narrow W^T A with fragments streamed into registers.
// ---------------------------------------------------------------------------------------------
// K1 streaming form of the narrow tail (same outputs as k_wta_narrow, bit for bit): no LDS and no
// barriers -- each wave owns one (chunk, 16-row block, 16-sample block) and loads its MFMA fragments
// straight from global memory (buffer loads, 16 B per lane) PF K-steps ahead in a register ring.  In the
// tail at most a few waves share a SIMD, so a wave's throughput is set by how many loads it keeps in
// flight, not by LDS reuse: PF steps of 4 MFMAs cover PF x 256 matrix cycles of load latency.  The
// fragments are exactly GTile's: lane (fr, g) holds K = 8 kk + 2 g + {x, y} of row fr, and each
// accumulator sees kk = 0 (x, y) then kk = 1 (x, y) of every 16-K step in order (the canonical order).
// ---------------------------------------------------------------------------------------------
template <int PF>
static __global__ __launch_bounds__(256) void k_wta_stream(const double* __restrict__ W, const double* __restrict__ Acm,
                                                           long m_pad, int ntq, int nsplit, int kchunk, int nblk,
                                                           const ColInfo* __restrict__ ci, double* __restrict__ Gpart,
                                                           long g_ld, long g_split, double* __restrict__ SWpart,
                                                           long sw_total) {
  const int nw = nsplit * nblk * ntq;
  const int item = xcd_item(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);   // 4 consecutive items per CU
  if (item >= nw) return;
  const int t = item % ntq, bk = (item / ntq) % nblk, s = item / (ntq * nblk);
  const int kbeg = s * kchunk;
  const int nst = (int)((min((long)kbeg + kchunk, m_pad) - kbeg) / BK2);
  const int l = threadIdx.x & 63, fr = l & 15, g = l >> 4;
  const bool gram = t == 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(W + (long)bk * 16 * m_pad + kbeg), 0, (int)(16 * m_pad * 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(Acm + (long)t * 16 * m_pad + kbeg), 0, (int)(16 * m_pad * 8), 0x00020000);
  const int voff = (int)((fr * m_pad + 2 * g) * 8);
  d2 fa[PF][2], fb[PF][2];
  auto load = [&](int u, int st) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      fa[u][kk] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(ra, voff, (st * BK2 + 8 * kk) * 8, 0));
      fb[u][kk] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rb, voff, (st * BK2 + 8 * kk) * 8, 0));
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nst) load(u, u);
  d4 acc = (d4){0.0, 0.0, 0.0, 0.0}, gacc = (d4){0.0, 0.0, 0.0, 0.0};
  for (int s0 = 0; s0 < nst; s0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (s0 + u < nst) {   // wave-uniform
        const d2 a0 = fa[u][0], a1 = fa[u][1], b0 = fb[u][0], b1 = fb[u][1];
        if (s0 + u + PF < nst) load(u, s0 + u + PF);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.x, b0.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.y, b0.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.x, b1.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.y, b1.y, acc, 0, 0, 0);
        if (gram) {
          gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.x, a0.x, gacc, 0, 0, 0);
          gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.y, a0.y, gacc, 0, 0, 0);
          gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.x, a1.x, gacc, 0, 0, 0);
          gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.y, a1.y, gacc, 0, 0, 0);
        }
      }
    }
  }
  double* out = Gpart + (long)s * g_split + (long)bk * 16 * g_ld + (long)t * 16;
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) out[(long)(g + 4 * reg) * g_ld + fr] = acc[reg];
  if (gram) {
    double* so = SWpart + (long)s * sw_total;
    const ColInfo* cb = ci + (long)bk * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int lr = g + 4 * reg, lcn = fr;
      const ColInfo cr = cb[lr];
      if (cr.k == 0 || cr.lc0 != cb[lcn].lc0 || cb[lcn].k == 0) continue;   // not the same restart
      const int a = lr - (cr.lc0 & 15), b = lcn - (cr.lc0 & 15);
      so[cr.sq_off + a * cr.k + b] = gacc[reg];
      so[cr.sq_off + b * cr.k + a] = gacc[reg];
    }
  }
}

}  // namespace nmfc
