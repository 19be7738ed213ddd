// nmfc_kernels.hpp -- HIP kernels of the batched MU restart engine (gfx950 / CDNA4).
//
// Device layouts (DESIGN.md "Data layout in HBM"):
//   Ablk [m_pad/16][n_cols_pad][16]  16-gene blocks of every column j of A (operand of W^T A)
//   Acm [n_cols_pad][m_pad]  column j of A, gene-contiguous              (small-shape kernel only)
//   Arm [m_pad][n_pad]       row i of A, sample-contiguous              (operand of A h^T)
//   W   [cols][m_pad]        column c of the stacked W_all (restart owns columns col0..col0+k-1)
//   H   [cols][n_pad]        row c of the stacked H_all (sample-contiguous)
//   Restarts are packed into panels of 64 columns; a restart never straddles a panel.
// Both contractions are "TN" tiles C[r][c] = sum_k P[r][k] Q[c][k] over K-contiguous rows, computed
// with v_mfma_f64_16x16x4_f64 on the GTile core (LDS-DMA ring, see below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nmfc_tuning.hpp"
#include "rmt.hpp"

namespace nmfc {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));

constexpr int PANEL = 64;          // restart columns per panel
constexpr int BK = 32;             // padding multiple of the sample dimension (K of A h^T)
constexpr int NT = 256;            // threads per workgroup
constexpr int KMAX = 16;           // largest rank k
constexpr int GT = 128;            // genes per A h^T tile (and per Gram partial)
constexpr int STOP_FIXED = 0, STOP_REF_COMPAT = 1, STOP_ARGMAX_STABLE = 2, STOP_TOLX = 3;
constexpr double SQRTEPS = 1.0536712127723509e-08;   // sqrt(dlamch('E')), nmf_als.c sqrteps
constexpr double DIV_BY_ZERO_AVOIDANCE = 1E-09;   // nmf_mu.c:56

// nmf_mu.c:184-191 / :209-216: h = (h0 == 0 || num == 0) ? 0 : h0 * (num / (den + 1e-9)); clamp < 0
// (ZERO_THRESHOLD = 0.0, common.h:15).  Order add -> divide -> multiply is kept (no contraction).
__device__ __forceinline__ double mu_rule(double old, double num, double den) {
  if (old == 0.0 || num == 0.0) return 0.0;
  const double q = num / (den + DIV_BY_ZERO_AVOIDANCE);
  const double t = old * q;
  return t < 0.0 ? 0.0 : t;
}

// The wave's index in its workgroup as a wave-uniform (SGPR) value.  threadIdx.x >> 6 is uniform within a wave, but the
// compiler does not know it: a buffer resource or a base pointer derived from it would be kept in VGPRs and every
// buffer load / store through it wrapped in a readfirstlane "waterfall" loop (round 5: 64 such loops around k_ahtw4's
// W0 loads and W stores).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
// The lane index by v_mbcnt: recomputed where it is used (two VALU instructions) instead of a value derived from
// threadIdx.x before a K loop and held in a VGPR across it (the 16-wave W^T A tile has no register to spare).
__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// mu_rule without branches: the quotient and product are formed for every element and the zero cases selected after,
// so a wave's rule is one straight instruction stream (no exec-mask branch per element).  The same bits as mu_rule for
// every input: where mu_rule returns early, the select returns the same +0.0.
__device__ __forceinline__ double mu_rule_sel(double old, double num, double den) {
  const double q = num / (den + DIV_BY_ZERO_AVOIDANCE);
  const double t = old * q;
  return (old == 0.0 || num == 0.0 || t < 0.0) ? 0.0 : t;
}

// Workgroup id -> work item such that each XCD (blocks b, b+8, ... share one) receives a contiguous
// range of items (bijective for any count; a speed choice only, never correctness).
__device__ __forceinline__ int xcd_item(int b, int nblocks) {
  const int xcd = b & 7, idx = b >> 3;
  const int q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// ---------------------------------------------------------------------------------------------
// GTile: the LDS-DMA-staged MFMA tile (v2 core).  RP x RQ outputs over NW waves (WR x WC), K in
// stages of BK2 = 16 doubles (one 128 B row per tile row per stage) in a ring of 3 LDS buffers filled
// by buffer_load ... lds (16 B per lane, no VGPR round trip).  A stage is issued two steps ahead; each
// step ends with ONE counted vmcnt wait + a raw s_barrier, so the next stage's DMA stays in flight
// across it.  LDS image: row r at r*128 B, logical 16-byte slot s stored at physical slot
// s ^ ((r >> 1) & 7) -- the swizzle is applied on the per-lane SOURCE address (the DMA destination is
// lane-linear) and on the fragment reads; it makes the ds_read_b128 fragment reads conflict-free.
// Canonical K order (a function of the 16-aligned K block only): MFMA j = 2*kk + sub (kk, sub in
// {0,1}) consumes k = 8*kk + sub + 2*g for lane group g = 0..3.  Every GTile shape uses this order, so
// results are bit-identical across tile shapes (the tail variants) and batch compositions.
// ---------------------------------------------------------------------------------------------
constexpr int BK2 = 16;
constexpr int GT_NBUF = 3;
constexpr bool GT_PRIO = NMFC_GT_PRIO != 0;   // raise the wave priority around each MFMA block (experiment)

__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, uint32_t lds_addr, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(uintptr_t)lds_addr, 16, voff,
                                           soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void step_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// QBLK: the Q operand is K-blocked ([K/16][rows][16] doubles: one 16-gene block of every row
// contiguous, `ldq` = the total row count), so a stage of a tile is ONE contiguous RQ x 128 B run instead
// of RQ rows 8 * ldq bytes apart.  The same canonical K order either way.
// GREG: the wave may also accumulate one 16 x 16 Gram block of its own P rows -- row block `gi` against row block
// `gj` of its MB row blocks (gj = gi: a restart-diagonal block; gj = gi + 1: a block straddled by a restart) -- into
// `gacc`: W^T W from the W fragments already in registers for the tile MFMAs (the A operand lane map (row fr, k g)
// and the B operand map (k g, col fr) hold the same value for P = Q), in the canonical K order; gi < 0: none.
// SPLIT (NBUF >= 3): the split-step form (below); false: each step computes its whole stage between the barriers
// (one fragment set live instead of two: 24 VGPRs fewer at MB = 4, NB = 2, for the 16-wave tile).  Same order of
// accumulation either way (kk = 0 then kk = 1 of every stage), so the same bits.
// OPQ: the lane index comes from an opaque copy taken in bind() (per run), not from threadIdx.x: inside an outer loop
// (k_wta2_sk's pieces) the lane-derived offsets then stay inside each run instead of being hoisted out of the outer
// loop and held across every K loop.  The same values, the same code in the loop.
template <int RP, int RQ, int WR, int WC, int NBUF = GT_NBUF, bool QBLK = false, bool GREG = false, bool SPLIT = true,
          bool OPQ = false>
struct GTile {
  static_assert(NBUF >= 2 && NBUF <= 16, "ring of 2..16 stages");
  static constexpr int NW = WR * WC;
  static constexpr int NTH = NW * 64;
  static constexpr int STAGE_BYTES = (RP + RQ) * BK2 * 8;
  static constexpr int LDS_BYTES = NBUF * STAGE_BYTES;
  static constexpr int PIECES = (RP + RQ) / 8;   // 1 KiB DMA pieces (8 rows) per stage
  static constexpr int PPW = PIECES / NW;        // pieces per wave per stage
  static constexpr int PPW_P = RP / 8 / NW;      // of which rows of P
  static_assert(PIECES % NW == 0 && (RP / 8) % NW == 0, "pieces must split evenly over waves");
  static constexpr int MB = RP / WR / 16;
  static constexpr int NB = RQ / WC / 16;
  static_assert(!GREG || NBUF >= 3, "register Gram on the split-step ring only");

  d4 acc[MB][NB];
  d4 gacc;
  int gi = -1, gj = -1;   // GREG: wave-uniform
  __amdgpu_buffer_rsrc_t rp, rq;
  int voff[PPW];
  int qkm;
  int tix = 0;  // OPQ: the opaque lane index (bind)
  int wo = 0;   // wave offset: this tile's waves are wo .. wo + NW - 1 of the workgroup (several 1-wave tiles per workgroup)   // QBLK: bytes between consecutive K positions' blocks / 8 (= 8 * total rows); else 8

  // P rows are K-contiguous at P + row*ldp, Q rows at Q + row*ldq (doubles); QBLK: Q + (k/16)*16*ldq + row*16
  __device__ __forceinline__ int lane_ix() const { return OPQ ? tix : (int)(threadIdx.x & 63); }
  __device__ __forceinline__ void bind(const double* P, long ldp, const double* Q, long ldq, int kend) {
    if constexpr (OPQ) {
      tix = lane_id();
      asm volatile("" : "+v"(tix));
    }
    const int w = wave_id() - wo, l = lane_ix();
    rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(P), 0, (int)(RP * ldp * 8), 0x00020000);
    rq = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(Q), 0, QBLK ? (int)((long)kend * ldq * 8) : (int)(RQ * ldq * 8),
                                           0x00020000);
    qkm = QBLK ? (int)ldq * 8 : 8;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = w + NW * i;
      const bool isq = i >= PPW_P;
      const int row = (isq ? piece - RP / 8 : piece) * 8 + (l >> 3);
      const int slot = (l & 7) ^ ((row >> 1) & 7);
      voff[i] = (int)((long)row * (isq ? (QBLK ? 16 : ldq) : ldp) * 8 + slot * 16);
    }
  }

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
    gacc = (d4){0.0, 0.0, 0.0, 0.0};
  }

  // DMA of the stage starting at K position k0 into the LDS buffer at byte address `buf`
  __device__ __forceinline__ void issue(uint32_t buf, int k0) const {
#pragma unroll
    for (int i = 0; i < PPW; ++i) issue_piece(buf, k0, i);
  }
  // piece i of this wave (the wave index is wave-uniform: read into an SGPR so M0 is scalar arithmetic)
  __device__ __forceinline__ void issue_piece(uint32_t buf, int k0, int i) const {
    const int w = wave_id() - wo;
    const uint32_t dst = buf + (uint32_t)(w + NW * i) * 1024u;
    if (i >= PPW_P)
      lds_dma16(rq, dst, voff[i], k0 * qkm);
    else
      lds_dma16(rp, dst, voff[i], k0 * 8);
  }

  // byte offset of (row, logical slot) in a stage
  __device__ __forceinline__ static uint32_t off(int row, int slot) {
    return (uint32_t)(row * 128 + ((slot ^ ((row >> 1) & 7)) << 4));
  }

  // the split form of compute(): fragments of one kk half of a stage, then its MFMAs
  struct Frag {
    d2 a[MB], b[NB];
  };
  __device__ __forceinline__ void load_frag(const char* __restrict__ st, int kk, Frag& f) const {
    const int w = wave_id() - wo, l = lane_ix();
    const int wr = w / WC, wc = w % WC;
    const int fr = l & 15, g = l >> 4;
    const char* sp = st + (wr * (RP / WR) + fr) * 128;
    const char* sq = st + RP * 128 + (wc * (RQ / WC) + fr) * 128;
    const int so = ((4 * kk + g) ^ (fr >> 1)) << 4;
#pragma unroll
    for (int i = 0; i < MB; ++i) f.a[i] = *reinterpret_cast<const d2*>(sp + i * 16 * 128 + so);
#pragma unroll
    for (int j = 0; j < NB; ++j) f.b[j] = *reinterpret_cast<const d2*>(sq + j * 16 * 128 + so);
  }
  // GC: the wave's register Gram block.  GC_DYN: chosen at run time by gi (diagonal blocks only, a VGPR select of the
  // fragment); -1: none; gi * 4 + gj: fixed at compile time (a K-loop instantiation per block: no selects, no branches)
  static constexpr int GC_DYN = -2;
  template <int GC = GC_DYN>
  __device__ __forceinline__ void mfma_frag(const Frag& f) {
    if constexpr (GT_PRIO) __builtin_amdgcn_s_setprio(1);
    mfma_frag_body<GC>(f);
    if constexpr (GT_PRIO) __builtin_amdgcn_s_setprio(0);
  }
  template <int GC = GC_DYN>
  __device__ __forceinline__ void mfma_frag_body(const Frag& f) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[i].x, f.b[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[i].y, f.b[j].y, acc[i][j], 0, 0, 0);
    if constexpr (GREG && GC >= 0) {
      constexpr int i = GC >> 2, j = GC & 3;
      static_assert(i < MB && j < MB, "Gram block inside the wave's rows");
      gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[i].x, f.a[j].x, gacc, 0, 0, 0);
      gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[i].y, f.a[j].y, gacc, 0, 0, 0);
    } else if constexpr (GREG && GC == GC_DYN) {
      if (gi >= 0) {
        d2 v = f.a[0];
#pragma unroll
        for (int i = 1; i < MB; ++i)
          if (gi == i) v = f.a[i];
        gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(v.x, v.x, gacc, 0, 0, 0);
        gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(v.y, v.y, gacc, 0, 0, 0);
      }
    }
  }
  template <int NKK = 2>
  __device__ __forceinline__ void compute(const char* __restrict__ st) {
    const int w = wave_id() - wo, l = threadIdx.x & 63;
    const int wr = w / WC, wc = w % WC;
    const int fr = l & 15, g = l >> 4;
    const char* sp = st + (wr * (RP / WR) + fr) * 128;
    const char* sq = st + RP * 128 + (wc * (RQ / WC) + fr) * 128;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const int so = ((4 * kk + g) ^ (fr >> 1)) << 4;
      d2 a[MB], b[NB];
#pragma unroll
      for (int i = 0; i < MB; ++i) a[i] = *reinterpret_cast<const d2*>(sp + i * 16 * 128 + so);
#pragma unroll
      for (int j = 0; j < NB; ++j) b[j] = *reinterpret_cast<const d2*>(sq + j * 16 * 128 + so);
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
    }
  }

  // the pipelined K loop over [kbeg, kend) (multiple of BK2); `extra(stage_ptr)` runs after each
  // stage's MFMAs on the same staged data.  smem: GT_NBUF * STAGE_BYTES bytes.
  template <class Extra>
  __device__ __forceinline__ void run(const double* __restrict__ P, long ldp, const double* __restrict__ Q, long ldq,
                                      int kbeg, int kend, char* __restrict__ smem, Extra extra) {
    run(P, ldp, Q, ldq, kbeg, kend, smem, extra, [] {});
  }

  // as above with `at_last()`: a place to issue the epilogue's own XL global loads early (see below)
  // NBUF == 2: `at_last()` runs right after the last DMA issue and may issue XL vector-memory
  // operations of its own; the one wait that follows leaves those XL in flight.
  template <int XL = 0, class Extra, class AtLast>
  __device__ __forceinline__ void run(const double* __restrict__ P, long ldp, const double* __restrict__ Q, long ldq,
                                      int kbeg, int kend, char* __restrict__ smem, Extra extra, AtLast at_last) {
    (void)run<XL>(P, ldp, Q, ldq, kbeg, kend, smem, [] { return true; }, extra, at_last);
  }

  // with `pre()`: runs right after the prologue's first DMA issue, so the workgroup's own setup loads
  // overlap the first stages' latency; returning false abandons the tile (the DMA is drained first)
  // and run returns false.  All waves must return the same answer.
  // LASTKK (NBUF == 2) = 1: the last stage's second half (K positions 8..15) holds zeros in both operands (the K
  // padding) and is skipped -- adding exact zeros to sums of non-negative products would change no bit.
  template <int XL = 0, int LASTKK = 2, int GC = GC_DYN, class Pre, class Extra, class AtLast>
  __device__ __forceinline__ bool run(const double* __restrict__ P, long ldp, const double* __restrict__ Q, long ldq,
                                      int kbeg, int kend, char* __restrict__ smem, Pre pre, Extra extra, AtLast at_last) {
    static_assert(LASTKK == 2 || NBUF == 2, "half last stage on the two-stage ring only");
    const int nst = (kend - kbeg) / BK2;
    bind(P, ldp, Q, ldq, kend);
    const uint32_t base = (uint32_t)(uintptr_t)smem;
    if constexpr (NBUF == 2) {   // one stage in flight, issued after the barrier that freed its buffer
      issue(base, kbeg);
      if (!pre()) {
        wait_vmcnt<0>();
        return false;
      }
      wait_vmcnt<0>();
      step_barrier();
      if (nst == 1) at_last();
      for (int s = 0; s + 1 < nst; ++s) {
        const int b = s & 1;
        issue(base + (b ^ 1) * STAGE_BYTES, kbeg + (s + 1) * BK2);
        if (s + 2 == nst) at_last();
        const char* cur = smem + b * STAGE_BYTES;
        compute(cur);
        extra(cur);
        if (s + 2 == nst)
          wait_vmcnt<XL>();
        else
          wait_vmcnt<0>();
        step_barrier();
      }
      {   // last step
        const char* cur = smem + ((nst - 1) & 1) * STAGE_BYTES;
        compute<LASTKK>(cur);
        extra(cur);
      }
      return true;
    }
    // NBUF >= 3: a ring of NBUF stages with D = NBUF - 1 stages in flight; stage s + D is issued at step
    // s into the buffer that stage s - 1 freed (every wave passed the barrier after computing it).
    // `at_last()` runs right after the LAST DMA issue and may issue XL vector-memory operations; every
    // later wait leaves those XL in flight.  After step s the wait leaves min(D - 1, nst - s - 2) stages
    // in flight (each PPW pieces per wave), so stage s + 1 has landed for this wave; the barrier makes
    // it landed for all waves.
    constexpr int D = NBUF - 1;
    static_assert(PPW * (D - 1) + XL <= 63, "vmcnt holds at most 63 outstanding operations");
    const int npro = nst < D ? nst : D;
    bool xl = false;
    for (int q = 0; q < npro; ++q) issue(base + q * STAGE_BYTES, kbeg + q * BK2);
    if (!pre()) {
      wait_vmcnt<0>();
      return false;
    }
    if (nst <= D) {
      at_last();
      xl = true;
    }
    wait_stages<D - 1, XL>(npro - 1, xl);
    step_barrier();
    int b = 0;
    // split steps: the kk = 1 MFMAs of stage s are issued AFTER the barrier that publishes stage s + 1,
    // right behind the LDS reads of stage s + 1's kk = 0 fragments, so those reads (and the barrier) are
    // covered by matrix work instead of leaving the pipe idle at every step.  Each accumulator still sees
    // kk = 0 (x, y) then kk = 1 (x, y) of every stage in order: the same sums bit for bit.
    // (the last step is peeled: no branch around the barrier, so the compiler's lgkmcnt for the kk = 1
    // fragments leaves the next stage's reads in flight)
    if constexpr (!SPLIT) {
      for (int s = 0; s < nst; ++s) {
        const char* cur = smem + b * STAGE_BYTES;
        if (s + D < nst) {
          const int bd = (b + D >= NBUF) ? b + D - NBUF : b + D;
          issue(base + bd * STAGE_BYTES, kbeg + (s + D) * BK2);
          if (s + D + 1 == nst) {
            at_last();
            xl = true;
          }
        }
        Frag f;
        load_frag(cur, 0, f);
        mfma_frag<GC>(f);
        load_frag(cur, 1, f);
        mfma_frag<GC>(f);
        extra(cur);
        if (s + 1 < nst) {
          const int left = nst - s - 2;
          wait_stages<D - 1, XL>(left < D - 1 ? left : D - 1, xl);
          step_barrier();
        }
        b = (b + 1 == NBUF) ? 0 : b + 1;
      }
      return true;
    }
    Frag f0, f1;
    load_frag(smem, 0, f0);
    for (int s = 0; s + 1 < nst; ++s) {
      const char* cur = smem + b * STAGE_BYTES;
      // the stage's DMA pieces go out as one block at the step head (spreading them one by one between the
      // MFMAs was measured 2 % slower on both contractions: the data then lands later)
      if (s + D < nst) {
        const int bd = (b + D >= NBUF) ? b + D - NBUF : b + D;
        issue(base + bd * STAGE_BYTES, kbeg + (s + D) * BK2);
        if (s + D + 1 == nst) {
          at_last();
          xl = true;
        }
      }
      load_frag(cur, 1, f1);
      mfma_frag<GC>(f0);
      extra(cur);
      const int bn = (b + 1 == NBUF) ? 0 : b + 1;
      const int left = nst - s - 2;
      __builtin_amdgcn_sched_barrier(0);   // the kk = 1 MFMAs stay behind the barrier and the next reads
      wait_stages<D - 1, XL>(left < D - 1 ? left : D - 1, xl);
      step_barrier();   // also: every wave has read stage s (its kk = 1 fragments are in registers)
      load_frag(smem + bn * STAGE_BYTES, 0, f0);
      __builtin_amdgcn_sched_barrier(0);
      mfma_frag<GC>(f1);
      b = bn;
    }
    {   // last step (its DMA was issued D steps ago)
      const char* cur = smem + b * STAGE_BYTES;
      load_frag(cur, 1, f1);
      mfma_frag<GC>(f0);
      extra(cur);
      mfma_frag<GC>(f1);
    }
    return true;
  }

  // s_waitcnt vmcnt(PPW * j + (xl ? XL : 0)) for a wave-uniform j in [0, J] (the count is an immediate)
  template <int J, int XL>
  __device__ __forceinline__ static void wait_stages(int j, bool xl) {
    if (j >= J) {
      if (xl)
        wait_vmcnt<PPW * J + XL>();
      else
        wait_vmcnt<PPW * J>();
    } else if constexpr (J > 0) {
      wait_stages<J - 1, XL>(j, xl);
    }
  }

  // C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
  __device__ __forceinline__ static int row_of(int mb, int reg) {
    const int w = wave_id(), l = lane_id();
    return (w / WC) * (RP / WR) + mb * 16 + (l >> 4) + 4 * reg;
  }
  __device__ __forceinline__ static int col_of(int nb) {
    const int w = wave_id(), l = lane_id();
    return (w % WC) * (RQ / WC) + nb * 16 + (l & 15);
  }
};

// Per-restart metadata.  rid is the persistent restart index (stop state, Gram/SH offsets, output
// slot); col0 is its current first column in W/H (changes when the engine repacks live restarts).
struct RestartInfo {
  int col0;
  int k;
  int rid;
  int sq_off;   // offset of its k x k blocks in the compact Gram / SH arrays
};

// Per panel column: the owning restart's compact-block offset, its first panel-local column, k
// (k = 0: padding column) and its restart id.
struct ColInfo {
  int sq_off;
  int lc0;
  int k;
  int rid;
};

// A panel takes part when one of its restarts is still running, or (for the W update) stopped at
// exactly this iteration.  [prb[p], pre[p]) is the panel's range in the active restart list.
__device__ __forceinline__ bool panel_live(const int* __restrict__ prb, const int* __restrict__ pre, int p,
                                           const RestartInfo* __restrict__ ri, const int* __restrict__ stop_iter,
                                           int iter) {
  const int b = prb[p], e = pre[p];
  for (int q = b; q < e; ++q) {
    const int s = stop_iter[ri[q].rid];
    if (s == 0 || s == iter) return true;
  }
  return false;
}

// ---------------------------------------------------------------------------------------------
// K1 v2 "wta2": G = W^T A on the GTile core.  A tile = NPT panels (64*NPT restart columns) x RQ
// samples; waves WR x WC.  Gram blocks (per panel: 4 diagonal + 3 straddling 16x16 blocks) are spread
// over the ntj sample-tile workgroups of the panel group and their waves.
// ---------------------------------------------------------------------------------------------
// GRAM = false: no Gram blocks (a probe: a wave carrying a Gram chain sets every barrier step of its workgroup,
// 20-35 % of a 1-panel tile's time and 4-7 % of the 2- and 4-panel tiles', tools/tailbench.hip).
// GITEM (1-panel tiles): the Gram blocks run in 3 extra workgroups per (chunk, panel), their first three waves
// each one candidate block as a 1-wave GTile<16, 16> (P, Q = the block's W rows; the rest of the wave set exits),
// beside the W^T A workgroups instead of on their waves (bit-identical: see k_wta_narrow).
// Gram candidate blocks of an NPT-panel tile, diagonal blocks first: cand < 4 NPT is the diagonal block
// cand & 3 of panel cand >> 2; the rest are the 3 blocks per panel straddling two 16-column blocks (needed only
// when a restart crosses a block boundary, which the engine's 16-column block packing never produces).
// cand = t + ntj (w + NW x) then gives waves 0..3 of each sample-tile workgroup one diagonal block each when
// ntj = 4, one Gram chain per SIMD (a wave w shares its SIMD with w + 4): 4 MFMAs on the SIMD's 128 per stage,
// where the per-panel order (7 candidates per panel) put two chains on each of two SIMDs (+2.6 % W^T A, C3).
template <int NPT>
__device__ __forceinline__ void gram_cand(int cand, int& q, int& br, int& bc) {
  if (cand < 4 * NPT) {
    q = cand >> 2;
    br = bc = cand & 3;
  } else {
    const int s = cand - 4 * NPT;
    q = s / 3;
    br = s % 3;
    bc = br + 1;
  }
}

// GREG (4-panel tiles, ntj >= 4): each diagonal Gram block is accumulated by a wave of the wave row that holds the
// block's W rows, from the tile's own W fragments (GTile GREG) -- no LDS reads of its own; wave column (wr >> 1) & 1
// of wave row wr, so at ntj = 4 the four chains of a workgroup sit on four SIMDs.  The straddling candidates (never
// produced by the engine's 16-column block packing) keep the LDS form.  Same operands, same K order: bit-identical.
template <int NPT, int RQ, int WR, int WC, int GPW, int NBUF = GT_NBUF, int MINW = 1, bool ABLK = false, bool GRAM = true,
          bool GITEM = false, bool GREG = false, bool SPLIT = true>
static __global__ __launch_bounds__(WR * WC * 64, MINW) void k_wta2(const double* __restrict__ W, const double* __restrict__ Acm,
                                                              long m_pad, int ngroups, int ntj, int nsplit, int kchunk,
                                                              const int* __restrict__ prb, const int* __restrict__ pre,
                                                              const RestartInfo* __restrict__ ri,
                                                              const ColInfo* __restrict__ ci,
                                                              const int* __restrict__ stop_iter, double* __restrict__ Gpart,
                                                              long g_ld, long g_split, double* __restrict__ SWpart,
                                                              long sw_total) {
  using T = GTile<64 * NPT, RQ, WR, WC, NBUF, ABLK, GREG, SPLIT>;
  static_assert(!GREG || (WR == NPT && GPW == 1 && GRAM && !GITEM), "register Gram: one panel per wave row");
  constexpr int NCAND = 7 * NPT;
  __shared__ __attribute__((aligned(1024))) char smem[T::LDS_BYTES + 64];
  int* need = reinterpret_cast<int*>(smem + T::LDS_BYTES);
  constexpr int NGW = GITEM ? 3 : 0;   // Gram workgroups per (chunk, panel)
  const int ntt = ntj + NGW;
  const int nitems = nsplit * ngroups * ntt;
  const int item = xcd_item(blockIdx.x, nitems);
  const int t = item % ntt;
  const int pg = (item / ntt) % ngroups;
  const int s = item / (ntt * ngroups);
  if constexpr (GITEM) {
    static_assert(NPT == 1 && T::NW >= 3, "Gram items: 1-panel tiles of at least 3 waves");
    using TG = GTile<16, 16, 1, 1, NBUF, false>;
    static_assert(3 * TG::LDS_BYTES <= T::LDS_BYTES, "three Gram rings fit the tile's");
    if (t >= ntj) {
      const int w = wave_id(), l = threadIdx.x & 63, fr = l & 15, g = l >> 4;
      const int x = 3 * (t - ntj) + w;   // candidate: 4 diagonal, 3 straddling blocks
      if (w >= 3 || x >= 7) return;
      if (!panel_live(prb, pre, pg, ri, stop_iter, 0)) return;
      const int br = x < 4 ? x : x - 4, bc = x < 4 ? x : x - 3;
      const ColInfo* cp = ci + (long)pg * PANEL;
      if (br != bc) {   // a straddling block only when the restart at column 16 bc started before it
        const ColInfo c = cp[16 * bc];
        if (!(c.k > 0 && c.lc0 < 16 * bc)) return;
      }
      const int kbeg = s * kchunk;
      const int kend = (int)min((long)kbeg + kchunk, m_pad);
      TG tg;
      tg.wo = w;
      tg.zero();
      const double* Pr = W + ((long)pg * PANEL + 16 * br) * m_pad + kbeg;
      const double* Qr = W + ((long)pg * PANEL + 16 * bc) * m_pad + kbeg;
      tg.run(Pr, m_pad, Qr, m_pad, 0, kend - kbeg, smem + w * TG::LDS_BYTES, [](const char*) {});
      double* so = SWpart + (long)s * sw_total;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int lr = 16 * br + g + 4 * reg, lcn = 16 * bc + fr;
        const ColInfo cr = cp[lr];
        if (cr.k == 0 || cr.lc0 != cp[lcn].lc0 || cp[lcn].k == 0) continue;   // not the same restart
        const int a = lr - cr.lc0, b = lcn - cr.lc0;
        so[cr.sq_off + a * cr.k + b] = tg.acc[0][0][reg];
        so[cr.sq_off + b * cr.k + a] = tg.acc[0][0][reg];
      }
      return;
    }
  }
  bool live[NPT];
  bool any = false;
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    live[q] = panel_live(prb, pre, NPT * pg + q, ri, stop_iter, 0);
    any = any || live[q];
  }
  if (!any) return;
  if (threadIdx.x < NCAND) {
    int q, br, bc;
    gram_cand<NPT>(threadIdx.x, q, br, bc);
    int nd = live[q];
    if (nd && br != bc) {
      const ColInfo c = ci[(long)(NPT * pg + q) * PANEL + 16 * bc];
      nd = (c.k > 0 && c.lc0 < 16 * bc);
    }
    need[threadIdx.x] = nd;
  }
  // ABLK: Acm is K-blocked over all ntj * RQ sample rows.  Both operands are rebased to the chunk start, so the
  // buffer offsets stay within one chunk (32-bit for any n_cols_pad up to 2^17).
  const int kbeg = s * kchunk;
  const int kend = (int)min((long)kbeg + kchunk, m_pad);
  const long ldq = ABLK ? (long)ntj * RQ : m_pad;
  const double* Q = ABLK ? Acm + (long)kbeg * ldq + (long)t * RQ * 16 : Acm + (long)t * RQ * m_pad + kbeg;
  T tl;
  tl.zero();
  d4 gacc[GPW];
#pragma unroll
  for (int x = 0; x < GPW; ++x) gacc[x] = (d4){0.0, 0.0, 0.0, 0.0};
  const int w = wave_id(), l = threadIdx.x & 63;
  const int fr = l & 15, g = l >> 4;
  __syncthreads();   // need[] visible (no DMA in flight yet)
  int my_need[GPW], my_ra[GPW], my_rb[GPW];
  bool gram = false;
#pragma unroll
  for (int x = 0; x < GPW; ++x) {
    const int cand = t + ntj * (w + T::NW * x);
    my_need[x] = 0;
    my_ra[x] = 0;
    my_rb[x] = 0;
    if (cand < NCAND) {
      int q, br, bc;
      gram_cand<NPT>(cand, q, br, bc);
      my_need[x] = (GREG && (cand < 4 * NPT || WC == 4)) ? 0 : need[cand];
      my_ra[x] = 64 * q + 16 * br;
      my_rb[x] = 64 * q + 16 * bc;
      gram = GRAM && !GITEM && (gram || my_need[x]);
    }
  }
  if constexpr (GREG) {
    const int wr = w / WC, wc = w % WC;
    int gi = -1, gj = -1;
    if constexpr (WC == 4) {
      // 16 waves: every Gram candidate of panel wr that falls to this workgroup (cand % ntj == t: at most two per
      // panel for ntj >= 4) on its own wave of row wr, the k-th on wave column (t + wr + 2 k) & 3 -- the diagonal
      // chains of a workgroup on four SIMDs (wave w runs on SIMD w & 3), a straddling one two SIMDs away
      int kth = 0;
#pragma unroll
      for (int c = 0; c < 7; ++c) {   // panel wr's candidates: 4 diagonal blocks, then 3 straddling blocks
        const int cand = c < 4 ? 4 * wr + c : 4 * NPT + 3 * wr + (c - 4);
        if (cand % ntj != t) continue;
        if (wc == ((t + wr + 2 * kth) & 3) && need[cand]) {
          gi = c < 4 ? c : c - 4;
          gj = c < 4 ? c : c - 3;
        }
        ++kth;
      }
    } else if (wc == ((wr >> 1) & 1) % WC) {   // WC = 2: the diagonal blocks, wave column (wr >> 1) & 1 of row wr
#pragma unroll
      for (int br = 0; br < 4; ++br)
        if ((4 * wr + br) % ntj == t && need[4 * wr + br]) gi = gj = br;
    }
    tl.gi = __builtin_amdgcn_readfirstlane(gi);
    tl.gj = __builtin_amdgcn_readfirstlane(gj);
  }
  const double* P = W + (long)pg * 64 * NPT * m_pad + kbeg;
  auto lds_gram = [&](const char* stg) {
#pragma unroll
    for (int x = 0; x < GPW; ++x) {
      if (!my_need[x]) continue;
      const char* pa = stg + (my_ra[x] + fr) * 128;
      const char* pb = stg + (my_rb[x] + fr) * 128;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int so = ((4 * kk + g) ^ (fr >> 1)) << 4;
        const d2 a = *reinterpret_cast<const d2*>(pa + so);
        const d2 b = *reinterpret_cast<const d2*>(pb + so);
        gacc[x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b.x, gacc[x], 0, 0, 0);
        gacc[x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b.y, gacc[x], 0, 0, 0);
      }
    }
  };
  // two instantiations of the K loop: the LDS Gram chains' accumulators are live only in the loop that runs them
  // (a wave without an LDS chain -- every wave of a GREG tile under block packing -- keeps none of their registers)
  constexpr bool LDSG = GRAM && !GITEM && !(GREG && WC == 4);   // the 16-wave GREG tile keeps every chain in registers
  if constexpr (GREG && WC == 4) {
    // one K-loop instantiation per register Gram block (4 diagonal, 3 straddling, none): the block is a compile-time
    // constant in the MFMA stream, with no fragment select and no branch in the loop
    auto go = [&](auto gc) {
      tl.template run<0, 2, decltype(gc)::value>(P, m_pad, Q, ldq, 0, kend - kbeg, smem, [] { return true; },
                                                 [](const char*) {}, [] {});
    };
    switch (tl.gi < 0 ? -1 : 4 * tl.gi + tl.gj) {
      case 0: go(std::integral_constant<int, 0>{}); break;
      case 5: go(std::integral_constant<int, 5>{}); break;
      case 10: go(std::integral_constant<int, 10>{}); break;
      case 15: go(std::integral_constant<int, 15>{}); break;
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 6: go(std::integral_constant<int, 6>{}); break;
      case 11: go(std::integral_constant<int, 11>{}); break;
      default: go(std::integral_constant<int, -1>{}); break;
    }
  } else if (LDSG && gram) {
    tl.run(P, m_pad, Q, ldq, 0, kend - kbeg, smem, lds_gram);
  } else {
    tl.run(P, m_pad, Q, ldq, 0, kend - kbeg, smem, [](const char*) {});
  }
  double* out = Gpart + (long)s * g_split + (long)pg * 64 * NPT * g_ld + (long)t * RQ;
#pragma unroll
  for (int mb = 0; mb < T::MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < T::NB; ++nb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) out[(long)T::row_of(mb, reg) * g_ld + T::col_of(nb)] = tl.acc[mb][nb][reg];
  // the restart-diagonal entries of Gram block (rows ra .. ra + 15, columns rb .. rb + 15 of the tile)
  auto put_gram = [&](int ra, int rb, const d4& v) {
    double* so = SWpart + (long)s * sw_total;
    const int pnl = ra >> 6;
    const ColInfo* cp = ci + (long)(NPT * pg + pnl) * PANEL;
    const int ln = lane_id();   // not the pre-loop lane values: nothing lane-derived held across the K loop
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int lr = (ra & 63) + (ln >> 4) + 4 * reg;
      const int lcn = (rb & 63) + (ln & 15);
      const ColInfo cr = cp[lr];
      if (cr.k == 0 || cr.lc0 != cp[lcn].lc0 || cp[lcn].k == 0) continue;
      const int a = lr - cr.lc0, b = lcn - cr.lc0;
      so[cr.sq_off + a * cr.k + b] = v[reg];
      so[cr.sq_off + b * cr.k + a] = v[reg];
    }
  };
  if (gram) {
#pragma unroll
    for (int x = 0; x < GPW; ++x)
      if (my_need[x]) put_gram(my_ra[x], my_rb[x], gacc[x]);
  }
  if constexpr (GREG) {
    if (tl.gi >= 0) put_gram(64 * (w / WC) + 16 * tl.gi, 64 * (w / WC) + 16 * tl.gj, tl.gacc);
  }
}

// ---------------------------------------------------------------------------------------------
// K1 stream-K form of the 16-wave 4-panel x 128-sample W^T A tile (round 6).  The big tile's grid is nsplit x ng x
// ntj items of up to kchunk / 16 stages each; as one workgroup per item (one per CU: 144 KiB of LDS) the launch takes
// ceil(items / CUs) rounds for items / CUs rounds of work (C3 at full load: 1 720 items = 6.72 rounds, the short last
// chunk makes it 6.56 rounds of work for 7 rounds of time).  Here G <= #CU persistent workgroups each take an equal
// contiguous range of the S stages of all items (in the item order of k_wta2, ranges XCD-contiguous); a range starts
// and ends anywhere inside an item, so an item is cut at a stage boundary into at most two pieces (G <= S / longest
// item).  The canonical K order is kept exactly: the first piece accumulates stages [0, x) from zero, stores its
// accumulators (G tile and register Gram chain, fp64 stores are exact) and publishes them; the second piece loads them
// and continues the same MFMA chains over [x, end) -- the same chain, instruction for instruction, as one workgroup
// running the whole item, so G and the Gram partials are bit-identical to k_wta2's (tools/kvar.hip checks it).
// Deadlock freedom without any assumption on dispatch order: every range runs its first-piece (start) item FIRST
// and its continuation LAST, and a continuation waits a bounded time; if the start piece has not been published by
// then (its workgroup not yet dispatched), it recomputes the item from stage 0 -- the same bits again, only slower.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility; cdna_hip_programming.md split-K recipe): plain stores ->
// every wave vmcnt(0) -> barrier -> lane 0 agent release fence -> vmcnt(0) -> relaxed agent flag store (= epoch of
// this launch); reader lane 0 relaxed agent poll -> agent acquire fence -> vmcnt(0) -> barrier -> plain loads.
// fix: G slots of SK_FIX doubles (9 d4 per lane: the 8 accumulator blocks and the Gram chain); flags: G words.
// ---------------------------------------------------------------------------------------------
constexpr int SK_THREADS = 1024;              // the 4-panel tile's 16 waves (the 2-panel tile: 8, SK_THREADS / 2)
constexpr long SK_FIX = 9L * 4 * SK_THREADS;   // doubles per range slot (either tile: 8 blocks + the Gram chain per lane)
constexpr int SK_POLLS = 256;                  // x s_sleep 127 (~3.4 us each): ~0.9 ms before recomputing

// A wave-uniform copy of a value held in VGPRs (device-function arguments arrive in VGPRs): SGPR operands for the
// buffer resources and soffsets of the K loop (a VGPR resource would wrap every buffer access in a waterfall loop).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long uni(long v) {
  const unsigned long long u = (unsigned long long)v;
  return (long)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((int)(u & 0xffffffffu)));
}
template <class P>
__device__ __forceinline__ P* uni(P* p) {
  return reinterpret_cast<P*>(uni(reinterpret_cast<long>(p)));
}
// An SGPR value the compiler may not treat as loop-invariant (an empty asm that "redefines" it): what is computed from
// it stays inside the loop instead of being hoisted and held in registers across the whole loop.
template <class V>
__device__ __forceinline__ V opaque(V v) {
  asm volatile("" : "+s"(v));
  return v;
}

struct SkArgs {   // the launch's operands: k_wta2_sk's only kernel argument (offset 0 of the kernarg segment)
  const double* W;
  const double* Acm;
  long m_pad;
  int ngroups, ntj, kchunk;
  const int* prb;
  const int* pre;
  const RestartInfo* ri;
  const ColInfo* ci;
  const int* stop_iter;
  double* Gpart;
  long g_ld, g_split;
  double* SWpart;
  long sw_total;
  double* fix;
  unsigned* flags;
  unsigned epoch;
  int nsplit;
  unsigned* tcnt;   // LSUM: per-tile chunk-arrival counters (monotonic: nsplit arrivals per tile and launch)
  int dp_xcd;       // whole rounds: 0 round-robin (item k G + r), 1 XCD-contiguous blocks (a speed / DVFS probe)
};
typedef const SkArgs __attribute__((address_space(4)))* SkArgsK;   // the kernarg copy, read by scalar loads

// The kernarg segment as an opaque pointer: every operand is re-read (s_load) where it is used, instead of being held
// in SGPRs across the whole piece loop -- the K loop then keeps k_wta2's SGPR and VGPR budget (a first form spilled).
__device__ __forceinline__ SkArgsK sk_args() {
  unsigned long long u = (unsigned long long)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(u));
  return (SkArgsK)u;
}

// One piece of the stream-K range: item `item`, stages [s0, s1); mode 0 whole item, 1 start piece (publish its
// chains in slot r), 2 continuation (of slot r - 1).  Every operand is re-read through opaque() per piece, so the
// compiler cannot hoist per-piece scalars (buffer resources, row offsets of the eight K-loop instantiations) out of the
// piece loop and hold them all at once: the K loop keeps k_wta2's register budget (a first form spilled).
// LSUM (probe arm, NMFC_WTA_LASTSUM=1): the workgroup that writes a tile's last chunk partial sums
// the tile's nsplit partials in chunk order -- k_hupdate's order, the same bits -- into chunk slot 0, so k_hupdate
// reads one partial instead of nsplit.  Publication: every wave vmcnt(0) -> barrier -> lane 0 agent release -> ticket;
// the ticket that completes the tile -> agent acquire -> barrier -> plain loads.
// NPT: 4 (the 16-wave big tile) or 2 (the 8-wave 2-panel tile of k_wta2<2, 128, 2, 4, ...>: wave rows = panels, the same
// register Gram scheme, one workgroup per CU; round 6, for grids between one and two rounds of it -- the 8-GPU shard).
template <int NBUF, bool NOWAIT, bool LSUM = false, int NPT = 4>
__device__ __forceinline__ void wta_sk_piece(int r, int item_in, int s0_in, int s1_in, int mode_in,
                                             char* __restrict__ smem) {
  constexpr int RQ = 128, WC = 4;
  using T = GTile<64 * NPT, RQ, NPT, WC, NBUF, true, true, true, true>;
  static_assert(T::MB * T::NB == 8 && T::NTH <= SK_THREADS, "a slot holds 8 accumulator blocks + the Gram chain per lane");
  SkArgsK A = sk_args();
  const double* W = A->W;
  const double* Acm = A->Acm;
  const long m_pad = A->m_pad;
  const int ngroups = A->ngroups, ntj = A->ntj, kchunk = A->kchunk;
  const int* prb = A->prb;
  const int* pre = A->pre;
  const RestartInfo* ri = A->ri;
  const ColInfo* ci = A->ci;
  const int* stop_iter = A->stop_iter;
  r = uni(r);
  const int item = uni(item_in), s0 = uni(s0_in), s1 = uni(s1_in), mode = uni(mode_in);
  const unsigned epoch = A->epoch;
  // lane-derived values are computed from an opaque copy of the lane index where they are used: hoisted out of the
  // piece loop they would all be held across the K loop (one VGPR too many there)
  auto lane = [] {
    int v = lane_id();
    asm volatile("" : "+v"(v));
    return v;
  };
  int* need = reinterpret_cast<int*>(smem + T::LDS_BYTES);   // 28 Gram candidates
  int* okw = need + 7 * NPT;                                  // the continuation's "published" word
  const int w = wave_id();
  const int t = uni(item % ntj);
  const int pg = uni((item / ntj) % ngroups);
  const int s = uni(item / (ngroups * ntj));
  bool live[NPT];
  bool any = false;
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    live[q] = panel_live(prb, pre, NPT * pg + q, ri, stop_iter, 0);
    any = any || live[q];
  }
  if (!any) return;   // both pieces of a dead item see the same stop_iter: neither runs, nobody waits
  const int tid = 64 * w + lane();
  if (tid < 7 * NPT) {
    int q, br, bc;
    gram_cand<NPT>(tid, q, br, bc);
    int nd = live[q];
    if (nd && br != bc) {
      const ColInfo c = ci[(long)(NPT * pg + q) * PANEL + 16 * bc];
      nd = (c.k > 0 && c.lc0 < 16 * bc);
    }
    need[tid] = nd;
  }
  unsigned* flags = A->flags;
  double* fix = A->fix;
  if (mode == 2 && tid == 0) {
    int ok = 0;
    for (int i = 0; i < (NOWAIT ? 0 : SK_POLLS); ++i) {
      if (__hip_atomic_load(flags + (r - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(127);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *okw = ok;
  }
  const int kbeg = s * kchunk;
  const long ldq = (long)ntj * RQ;
  const double* Q = Acm + (long)kbeg * ldq + (long)t * RQ * 16;
  T tl;
  tl.zero();
  __syncthreads();   // need[] and okw visible
  // continuation: the chains come back from slot r - 1 in run()'s pre() hook, after the prologue's first DMA issue (held
  // in registers only from there on, where the K loop holds them anyway); not published: the whole item from stage 0
  const bool cont = mode == 2 && uni(*okw) != 0;
  const int resume = uni(cont ? s0 : (mode == 2 ? 0 : s0));
  auto load_chains = [&] {
    if (cont) {
      const double* src = fix + (long)(r - 1) * SK_FIX + 4L * (64 * w);
      const int ln = lane();
#pragma unroll
      for (int mb = 0; mb < T::MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < T::NB; ++nb)
          tl.acc[mb][nb] = *reinterpret_cast<const d4*>(src + ((long)(mb * T::NB + nb) * SK_THREADS + ln) * 4);
      tl.gacc = *reinterpret_cast<const d4*>(src + ((long)T::MB * T::NB * SK_THREADS + ln) * 4);
    }
    return true;
  };
  {
    const int wr = w / WC, wc = w % WC;
    int gi = -1, gj = -1, kth = 0;
#pragma unroll
    for (int c = 0; c < 7; ++c) {   // as k_wta2 (GREG, WC = 4)
      const int cand = c < 4 ? 4 * wr + c : 4 * NPT + 3 * wr + (c - 4);
      if (cand % ntj != t) continue;
      if (wc == ((t + wr + 2 * kth) & 3) && need[cand]) {
        gi = c < 4 ? c : c - 4;
        gj = c < 4 ? c : c - 3;
      }
      ++kth;
    }
    tl.gi = __builtin_amdgcn_readfirstlane(gi);
    tl.gj = __builtin_amdgcn_readfirstlane(gj);
  }
  const double* P = W + (long)pg * 64 * NPT * m_pad + kbeg;
  auto go = [&](auto gc) {
    tl.template run<0, 2, decltype(gc)::value>(P, m_pad, Q, ldq, BK2 * resume, BK2 * s1, smem, load_chains,
                                               [](const char*) {}, [] {});
  };
  switch (tl.gi < 0 ? -1 : 4 * tl.gi + tl.gj) {
    case 0: go(std::integral_constant<int, 0>{}); break;
    case 5: go(std::integral_constant<int, 5>{}); break;
    case 10: go(std::integral_constant<int, 10>{}); break;
    case 15: go(std::integral_constant<int, 15>{}); break;
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 6: go(std::integral_constant<int, 6>{}); break;
    case 11: go(std::integral_constant<int, 11>{}); break;
    default: go(std::integral_constant<int, -1>{}); break;
  }
  if (mode == 1) {   // publish the start piece's chains for range r + 1
    // lane index by mbcnt and the wave index in an SGPR: nothing derived from threadIdx.x is held across the K loop
    A = sk_args();
    fix = A->fix;
    flags = A->flags;
    double* dst = fix + (long)r * SK_FIX + 4L * (64 * w);
    const int ln = lane();
#pragma unroll
    for (int mb = 0; mb < T::MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < T::NB; ++nb)
        *reinterpret_cast<d4*>(dst + ((long)(mb * T::NB + nb) * SK_THREADS + ln) * 4) = tl.acc[mb][nb];
    *reinterpret_cast<d4*>(dst + ((long)T::MB * T::NB * SK_THREADS + ln) * 4) = tl.gacc;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w == 0 && ln == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(flags + r, A->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  A = sk_args();   // re-read after the K loop
  const long g_ld = A->g_ld, g_split = A->g_split;
  double* out = A->Gpart + (long)s * g_split + (long)pg * 64 * NPT * g_ld + (long)t * RQ;
  {   // T::row_of / T::col_of from the opaque lane
    const int ln = lane();
    const int r0 = (w / WC) * 64 + (ln >> 4), c0 = (w % WC) * (RQ / WC) + (ln & 15);
#pragma unroll
    for (int mb = 0; mb < T::MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < T::NB; ++nb)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) out[(long)(r0 + mb * 16 + 4 * reg) * g_ld + c0 + nb * 16] = tl.acc[mb][nb][reg];
  }
  if (tl.gi >= 0) {   // the restart-diagonal entries of the wave's Gram block (as k_wta2's put_gram)
    const int ra = 64 * (w / WC) + 16 * tl.gi, rb = 64 * (w / WC) + 16 * tl.gj;
    double* so = A->SWpart + (long)s * A->sw_total;
    const ColInfo* cp = ci + (long)(NPT * pg + (ra >> 6)) * PANEL;
    const int ln = lane();
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int lr = (ra & 63) + (ln >> 4) + 4 * reg;
      const int lcn = (rb & 63) + (ln & 15);
      const ColInfo cr = cp[lr];
      if (cr.k == 0 || cr.lc0 != cp[lcn].lc0 || cp[lcn].k == 0) continue;
      const int a = lr - cr.lc0, bq = lcn - cr.lc0;
      so[cr.sq_off + a * cr.k + bq] = tl.gacc[reg];
      so[cr.sq_off + bq * cr.k + a] = tl.gacc[reg];
    }
  }
  if constexpr (LSUM) {
    A = sk_args();   // everything from the kernarg copy and `item` again: nothing extra held across the K loop
    const int nsplit = A->nsplit;
    if (nsplit > 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int ntj2 = A->ntj, ng2 = A->ngroups;
      const int tile = item % (ng2 * ntj2), pg2 = (item / ntj2) % ng2, t2 = item % ntj2;
      if (w == 0 && lane() == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(A->tcnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (old + 1) % (unsigned)nsplit == 0;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *okw = last;
      }
      __syncthreads();
      if (uni(*okw)) {   // the tile's partials, chunk 0 first, summed as k_hupdate sums them, into chunk slot 0
        const long g_ld2 = A->g_ld, g_split2 = A->g_split;
        double* base = A->Gpart + (long)pg2 * 64 * NPT * g_ld2 + (long)t2 * RQ;
        const int ln = lane();
        const int r0 = (w / WC) * 64 + (ln >> 4), c0 = (w % WC) * (RQ / WC) + (ln & 15);
#pragma unroll
        for (int mb = 0; mb < T::MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < T::NB; ++nb) {
            double v[4];
            double* e0 = base + (long)(r0 + mb * 16) * g_ld2 + c0 + nb * 16;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) v[reg] = e0[(long)4 * reg * g_ld2];
            for (int c = 1; c < nsplit; ++c) {
              double u[4];
#pragma unroll
              for (int reg = 0; reg < 4; ++reg) u[reg] = e0[(long)c * g_split2 + (long)4 * reg * g_ld2];
#pragma unroll
              for (int reg = 0; reg < 4; ++reg) v[reg] = v[reg] + u[reg];
            }
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) e0[(long)4 * reg * g_ld2] = v[reg];
          }
      }
    }
  }
}

// NOWAIT (tools/kvar.hip only): every continuation takes the recompute path (tests its bits)
template <int NBUF = GT_NBUF, bool NOWAIT = false, bool LSUM = false, int NPT = 4>
static __global__ __launch_bounds__(64 * NPT * 4, 1) void k_wta2_sk(SkArgs args) {
  using T = GTile<64 * NPT, 128, NPT, 4, NBUF, true, true, true, true>;
  static_assert(NPT == 4 || NPT == 2, "the 16-wave 4-panel tile or the 8-wave 2-panel tile");
  __shared__ __attribute__((aligned(1024))) char smem[T::LDS_BYTES + 128];
  (void)args;   // read through sk_args() (the kernarg segment), see there
  SkArgsK A = sk_args();
  const int nsplit = A->nsplit;
  const int G = gridDim.x;
  const int r = __builtin_amdgcn_readfirstlane(xcd_item(blockIdx.x, G));
  // this workgroup's XCD (blocks b, b + 8, ... share one): its xcd_item range [xb, xb + xc) of the G ranges
  const int xq = G >> 3, xrem = G & 7, xcd = blockIdx.x & 7;
  const int xc = xq + (xcd < xrem ? 1 : 0), xb = xcd < xrem ? xcd * (xq + 1) : xrem * (xq + 1) + (xcd - xrem) * xq;
  const int ipc = A->ngroups * A->ntj;
  const int nitems = nsplit * ipc;
  const int nst_full = A->kchunk / BK2;
  const int nst_last = (int)((A->m_pad - (long)(nsplit - 1) * A->kchunk) / BK2);
  const int nst_max = nsplit > 1 ? nst_full : nst_last;
  const int c_last = ipc * (nsplit - 1);   // first item of the last chunk
  auto nst_of = [&](int item) { return item >= c_last ? nst_last : nst_full; };
  auto off = [&](int item) -> long {        // stage offset of an item in k_wta2's item order
    return item <= c_last ? (long)item * nst_full : (long)c_last * nst_full + (long)(item - c_last) * nst_last;
  };
  auto locate = [&](long x, int& item, int& st) {
    const long lc = (long)c_last * nst_full;
    const int it = x < lc ? (int)(x / nst_full) : c_last + (int)((x - lc) / nst_last);
    item = __builtin_amdgcn_readfirstlane(it);
    st = __builtin_amdgcn_readfirstlane((int)(x - off(it)));
  };
  // whole rounds first, item k G + r in round k (the dispatch order of k_wta2: the items a round runs at once are
  // neighbours that share their A chunk and W rows in L2); the items left after them -- between one and two rounds'
  // worth, at least G x the longest item in stages -- are split evenly over the G workgroups (stream-K)
  int D = (nitems / G - 1) * G;
  if (D < 0) D = 0;
  while (D > 0 && off(nitems) - off(D) < (long)G * nst_max) D -= G;
  D = __builtin_amdgcn_readfirstlane(D);
  const long base = off(D), S = off(nitems) - base;
  const long b = base + S * r / G, e = base + S * (r + 1) / G;
  int ib, sb, ie, se;
  locate(b, ib, sb);
  locate(e - 1, ie, se);
  ++se;   // the range's piece of item ie is [0, se)
  const bool head = sb > 0;                 // [sb, nst) of item ib: a continuation of range r - 1's start piece
  const bool tail = se < nst_of(ie);        // [0, se) of item ie: the start piece, published for range r + 1
  const int f0 = head ? ib + 1 : ib, f1 = tail ? ie - 1 : ie;   // whole items f0 .. f1 of the split part
  const int nfull = f1 >= f0 ? f1 - f0 + 1 : 0;
  const int ndp = D / G;
  const int t0 = tail ? 1 : 0;
  const int npieces = t0 + ndp + nfull + (head ? 1 : 0);
  for (int pc = 0; pc < npieces; ++pc) {
    // piece order: the whole rounds first -- every workgroup starts them together, so the workgroups that share an A
    // or W stage read it at the same time and L2 serves all but the first (starting with the split part's start pieces,
    // of every length, desynchronised them and tripled the L2-miss bytes) -- then the split part: the start piece (a
    // later range waits for it), its whole items, the continuation last.  With shares of at least one item the start
    // piece of range r - 1 ends before range r reaches its continuation, so nobody waits.
    int item, s0, s1, mode;
    if (pc < ndp) {
      item = A->dp_xcd ? ndp * xb + pc * xc + (r - xb) : pc * G + r;
      s0 = 0, s1 = nst_of(item), mode = 0;
    } else if (pc < ndp + t0) {
      item = ie, s0 = 0, s1 = se, mode = 1;
    } else if (head && pc == npieces - 1) {
      item = ib, s0 = sb, s1 = nst_of(ib), mode = 2;
    } else {
      item = f0 + pc - t0 - ndp, s0 = 0, s1 = nst_of(item), mode = 0;
    }
    __syncthreads();   // the previous piece's LDS ring, need[] and okw are free
    wta_sk_piece<NBUF, NOWAIT, LSUM, NPT>(r, item, s0, s1, mode, smem);
  }
}

// ---------------------------------------------------------------------------------------------
// K1 narrow form (the tail: the live restarts block-packed into the first nblk 16-column blocks, none
// straddling a block): G rows 16 b .. 16 b + 15 = W^T A over the same fixed gene chunks, one wave per
// (chunk, block, RQ-sample tile), RP = 16 rows -- only the live blocks' MFMA work, and many more, lighter
// workgroups than the 64-row tiles.  The accumulation is the canonical GTile K order, so the rows are
// bit-identical to every other shape.  Tile t == 0 of each (chunk, block) also forms the block's 16 x 16
// Gram block (nmf_mu.c:176); no restart crosses a block, so that is every Gram entry of its restarts.
// ---------------------------------------------------------------------------------------------
// Tile t == ntq of each (chunk, block) is the block's Gram item: its own wave runs the 16 x 16 W^T W block
// (P = Q = the block's W rows) beside the W^T A waves, instead of a W^T A wave carrying the Gram chain next
// to its own (that wave took 50 us where the others take 30).  A GTile MFMA with the same rows on both sides
// is the in-tile Gram MFMA operand for operand, in the same canonical K order: bit-identical partials.
template <int RQ, int NBUF, bool ABLK = false>
static __global__ __launch_bounds__(64) void k_wta_narrow(const double* __restrict__ W, const double* __restrict__ Acm,
                                                          long m_pad, int ntq, int nsplit, int kchunk, int nblk,
                                                          const ColInfo* __restrict__ ci, double* __restrict__ Gpart,
                                                          long g_ld, long g_split, double* __restrict__ SWpart,
                                                          long sw_total) {
  using T = GTile<16, RQ, 1, 1, NBUF, ABLK>;
  using TG = GTile<16, 16, 1, 1, NBUF, false>;
  static_assert(TG::LDS_BYTES <= T::LDS_BYTES, "the Gram item's ring fits the tile's");
  __shared__ __attribute__((aligned(1024))) char smem[T::LDS_BYTES];
  const int nt = ntq + 1;   // ntq W^T A tiles + the Gram item
  const int item = xcd_item(blockIdx.x, nsplit * nblk * nt);
  const int t = item % nt, bk = (item / nt) % nblk, s = item / (nt * nblk);
  const int kbeg = s * kchunk;
  const int kend = (int)min((long)kbeg + kchunk, m_pad);
  const int l = threadIdx.x, fr = l & 15, g = l >> 4;
  const double* Wb = W + (long)bk * 16 * m_pad + kbeg;
  if (t == ntq) {   // the Gram item
    TG tg;
    tg.zero();
    tg.run(Wb, m_pad, Wb, m_pad, 0, kend - kbeg, smem, [](const char*) {});
    double* so = SWpart + (long)s * sw_total;
    const ColInfo* cb = ci + (long)bk * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int lr = g + 4 * reg, lcn = fr;
      const ColInfo cr = cb[lr];
      if (cr.k == 0 || cr.lc0 != cb[lcn].lc0 || cb[lcn].k == 0) continue;   // not the same restart
      const int a = lr - (cr.lc0 & 15), b = lcn - (cr.lc0 & 15);
      so[cr.sq_off + a * cr.k + b] = tg.acc[0][0][reg];
      so[cr.sq_off + b * cr.k + a] = tg.acc[0][0][reg];
    }
    return;
  }
  T tl;
  tl.zero();
  const long ldq = ABLK ? (long)ntq * RQ : m_pad;   // operands rebased to the chunk start (see k_wta2)
  const double* Q = ABLK ? Acm + (long)kbeg * ldq + (long)t * RQ * 16 : Acm + (long)t * RQ * m_pad + kbeg;
  tl.run(Wb, m_pad, Q, ldq, 0, kend - kbeg, smem, [](const char*) {});
  double* out = Gpart + (long)s * g_split + (long)bk * 16 * g_ld + (long)t * RQ;
#pragma unroll
  for (int nb = 0; nb < T::NB; ++nb)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) out[(long)T::row_of(0, reg) * g_ld + T::col_of(nb)] = tl.acc[0][nb][reg];
}

// Loader / consumer form of k_wta_narrow (round 4): the same items and the same canonical K order (GTile's
// load_frag / mfma_frag on the same stages), but two waves per item: wave 1 only issues the LDS-DMA stages and waits
// for them to land, wave 0 only reads fragments and issues the MFMA chain; they meet at one barrier per stage.  In the
// one-wave form the wave's in-order issue serialises each stage's four 1-KiB DMA pieces (~60 cycles of issue each)
// with its four dependent MFMAs (~64 cycles each): here the two run on two SIMDs at once.  Bit-identical results.
template <int RQ, int NBUF, bool ABLK = false>
static __global__ __launch_bounds__(128) void k_wta_narrow_lc(const double* __restrict__ W, const double* __restrict__ Acm,
                                                             long m_pad, int ntq, int nsplit, int kchunk, int nblk,
                                                             const ColInfo* __restrict__ ci, double* __restrict__ Gpart,
                                                             long g_ld, long g_split, double* __restrict__ SWpart,
                                                             long sw_total) {
  static_assert(RQ == 16, "the Gram item shares the tile type: RQ = 16");
  using T = GTile<16, RQ, 1, 1, NBUF, ABLK>;
  __shared__ __attribute__((aligned(1024))) char smem[T::LDS_BYTES];
  const int nt = ntq + 1;   // ntq W^T A tiles + the Gram item
  const int item = xcd_item(blockIdx.x, nsplit * nblk * nt);
  const int t = item % nt, bk = (item / nt) % nblk, s = item / (nt * nblk);
  const int kbeg = s * kchunk;
  const int kend = (int)min((long)kbeg + kchunk, m_pad);
  const int wave = wave_id(), l = threadIdx.x & 63, fr = l & 15, g = l >> 4;
  const bool gram = t == ntq;
  const double* Wb = W + (long)bk * 16 * m_pad + kbeg;
  const long ldq = gram ? m_pad : (ABLK ? (long)ntq * RQ : m_pad);   // operands rebased to the chunk start
  const double* Q = gram ? Wb : (ABLK ? Acm + (long)kbeg * ldq + (long)t * RQ * 16 : Acm + (long)t * RQ * m_pad + kbeg);
  const int nst = (kend - kbeg) / BK2;
  constexpr int D = NBUF - 1;
  const uint32_t base = (uint32_t)(uintptr_t)smem;
  T tl;
  tl.wo = wave;   // each wave is wave 0 of its own 1-wave tile view
  if (wave == 1) {
    // loader: the K-blocked A operand only for the W^T A items (the Gram item stages W rows on both sides)
    if (gram) {
      GTile<16, RQ, 1, 1, NBUF, false> tg;
      tg.wo = 1;
      tg.bind(Wb, m_pad, Q, ldq, kend - kbeg);
      const int npro = nst < D ? nst : D;
      for (int q = 0; q < npro; ++q) tg.issue(base + q * T::STAGE_BYTES, q * BK2);
      T::template wait_stages<D - 1, 0>(npro - 1, false);
      step_barrier();
      for (int st = 0; st + 1 < nst; ++st) {
        if (st + D < nst) tg.issue(base + ((st + D) % NBUF) * T::STAGE_BYTES, (st + D) * BK2);
        const int left = nst - st - 2;
        T::template wait_stages<D - 1, 0>(left < D - 1 ? left : D - 1, false);
        step_barrier();
      }
    } else {
      tl.bind(Wb, m_pad, Q, ldq, kend - kbeg);
      const int npro = nst < D ? nst : D;
      for (int q = 0; q < npro; ++q) tl.issue(base + q * T::STAGE_BYTES, q * BK2);
      T::template wait_stages<D - 1, 0>(npro - 1, false);
      step_barrier();
      for (int st = 0; st + 1 < nst; ++st) {
        if (st + D < nst) tl.issue(base + ((st + D) % NBUF) * T::STAGE_BYTES, (st + D) * BK2);
        const int left = nst - st - 2;
        T::template wait_stages<D - 1, 0>(left < D - 1 ? left : D - 1, false);
        step_barrier();
      }
    }
    return;
  }
  // consumer: GTile::run's split steps (kk = 1 MFMAs of stage st behind the barrier publishing stage st + 1)
  tl.zero();
  step_barrier();
  typename T::Frag f0, f1;
  int b = 0;
  tl.load_frag(smem, 0, f0);
  for (int st = 0; st + 1 < nst; ++st) {
    const char* cur = smem + b * T::STAGE_BYTES;
    tl.load_frag(cur, 1, f1);
    tl.mfma_frag(f0);
    const int bn = (b + 1 == NBUF) ? 0 : b + 1;
    __builtin_amdgcn_sched_barrier(0);
    step_barrier();
    tl.load_frag(smem + bn * T::STAGE_BYTES, 0, f0);
    __builtin_amdgcn_sched_barrier(0);
    tl.mfma_frag(f1);
    b = bn;
  }
  {
    const char* cur = smem + b * T::STAGE_BYTES;
    tl.load_frag(cur, 1, f1);
    tl.mfma_frag(f0);
    tl.mfma_frag(f1);
  }
  if (gram) {
    double* so = SWpart + (long)s * sw_total;
    const ColInfo* cb = ci + (long)bk * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int lr = g + 4 * reg, lcn = fr;
      const ColInfo cr = cb[lr];
      if (cr.k == 0 || cr.lc0 != cb[lcn].lc0 || cb[lcn].k == 0) continue;   // not the same restart
      const int a = lr - (cr.lc0 & 15), bb = lcn - (cr.lc0 & 15);
      so[cr.sq_off + a * cr.k + bb] = tl.acc[0][0][reg];
      so[cr.sq_off + bb * cr.k + a] = tl.acc[0][0][reg];
    }
    return;
  }
  double* out = Gpart + (long)s * g_split + (long)bk * 16 * g_ld + (long)t * RQ;
#pragma unroll
  for (int nb = 0; nb < T::NB; ++nb)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) out[(long)T::row_of(0, reg) * g_ld + T::col_of(nb)] = tl.acc[0][nb][reg];
}

// ---------------------------------------------------------------------------------------------
// K2 "hupdate": one workgroup per active restart.
//   work1 = W0^T W0 = sum of the per-chunk Gram partials (nmf_mu.c:176); work2 = work1 H0 (:178);
//   H <- mu_rule(H, G, work2) (:184-191); SH = H H^T (:200); stability check (:253-282).
// ---------------------------------------------------------------------------------------------
constexpr int NTH = 512;           // threads of the H-update kernel (one sample per thread and round)
constexpr int HCH2 = NTH;          // samples per round

struct HupdSmem {
  double sw[KMAX * KMAX];
  double Hn[KMAX * HCH2];
  double win[KMAX * KMAX];
  double shp[NTH];
  int changed;
  unsigned long long dmax, omax;   // STOP_TOLX: max |h0 - h| and max |h0| (non-negative doubles as bits)
};

// The body for rank K (compile time).  Latency is what matters here (one workgroup per restart, often
// only a few restarts live): every load the workgroup needs is issued before its first use -- the stop
// state, the Gram partials and the first round's H and W^T A partials together -- and the split-K
// partials of one sample are loaded GS chunks at a time (GS*K <= 64 values in flight per thread).  The
// arithmetic order is fixed: chunk partials and Gram partials summed in chunk order, d = sum_b in b order,
// h h^T by T = f(k) threads per pair over j = pq (mod T) in j order, then the T partials in pq order.
template <int K, int GSV = 32>
__device__ __forceinline__ void hupdate_body(const RestartInfo me, int iter, int maxiter, int stop_rule, int n,
                                             long n_pad, const double* __restrict__ Gpart, long g_ld, long g_split,
                                             int gsplit, int nsplit, const double* __restrict__ SWpart, long sw_total,
                                             double* __restrict__ H, double* __restrict__ SH,
                                             int* __restrict__ stop_iter, int* __restrict__ stop_reason,
                                             int* __restrict__ unchanged, int* __restrict__ classes, long cls_ld,
                                             int* __restrict__ n_stopped, double* __restrict__ SHP,
                                             int* __restrict__ colact, double* __restrict__ Hstat, HupdSmem& sm) {
  // GSV: chunk-partial values in flight per thread (32: 128 VGPRs, two workgroups per CU).  Round 4 measured a
  // "latency form" <100, 2> (every chunk of a C3 restart in one group of loads, one workgroup per CU) for launches
  // of at most one restart per CU: the 8-GPU replay went 380.8 -> 373.3 per GPU, so it is not used.
  constexpr int GS = (GSV / K) < 1 ? 1 : (GSV / K) > 16 ? 16 : (GSV / K);
  double* sw = sm.sw;
  double* Hn = sm.Hn;
  double* win = sm.win;
  double* shp = sm.shp;
  int& changed = sm.changed;
  const int rid = me.rid;
  const int tid = threadIdx.x;
  constexpr int k = K;
  const int c0 = me.col0;
  const bool check = (stop_rule != STOP_FIXED) && iter > 1 && (iter % 2 == 0);
  const bool tolx = check && stop_rule == STOP_TOLX;
  double tdm = 0.0, tom = 0.0;   // this thread's max |h0 - h| and max |h0| (STOP_TOLX)
  // stop state, loaded now and used at the end
  const int u_prev = (tid == 0 && check) ? unchanged[rid] : 0;
  const int nwin = k < n ? k : n;
  const bool refc = check && stop_rule == STOP_REF_COMPAT;
  const int cl_prev = (refc && tid < nwin) ? classes[(long)rid * cls_ld + tid] : 0;
  // the sample rounds' loads: H and the split-K partials of W^T A (first group issued here)
  auto load_h = [&](int j, double* hc) {
#pragma unroll
    for (int a = 0; a < K; ++a) hc[a] = H[(long)(c0 + a) * n_pad + j];
  };
  auto sum_g = [&](int j, double* gs) {   // chunk partials of this sample, added in chunk order
    const double* gsrc = Gpart + (long)c0 * g_ld + j;
    for (int g0 = 0; g0 < gsplit; g0 += GS) {
      double v[GS][K];
#pragma unroll
      for (int u = 0; u < GS; ++u) {   // chunks past the end re-read the last one (not added)
        const double* q = gsrc + (long)min(g0 + u, gsplit - 1) * g_split;
#pragma unroll
        for (int a = 0; a < K; ++a) v[u][a] = q[(long)a * g_ld];
      }
#pragma unroll
      for (int u = 0; u < GS; ++u)
        if (g0 + u < gsplit) {
#pragma unroll
          for (int a = 0; a < K; ++a) gs[a] = (g0 + u == 0) ? v[u][a] : gs[a] + v[u][a];
        }
    }
  };
  if (tid == 0) {
    changed = 0;
    sm.dmax = 0ull;
    sm.omax = 0ull;
  }
  for (int idx = tid; idx < k * k; idx += NTH) {
    const double* src = SWpart + me.sq_off + idx;
    double sacc = 0.0;
    for (int g0 = 0; g0 < nsplit; g0 += 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = (g0 + u < nsplit) ? src[(long)(g0 + u) * sw_total] : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (g0 + u < nsplit) sacc = (g0 + u == 0) ? v[u] : sacc + v[u];
    }
    sw[(idx / k) * KMAX + (idx % k)] = sacc;
  }
  for (int idx = tid; idx < KMAX * KMAX; idx += NTH) win[idx] = 0.0;
  // h h^T: T threads per (pa, pb) pair (T a function of k only); thread pq of a pair sums the samples
  // j = pq (mod T) in order, and the T partials are added in pq order at the end.
  const int npairs = k * (k + 1) / 2;
  const int T = (npairs * 8 <= 256) ? 8 : (npairs * 4 <= 256) ? 4 : (npairs * 2 <= 256) ? 2 : 1;
  const int pid = tid / T, pq = tid % T;
  int pa = 0, pb = 0;
  if (pid < npairs) {
    int t = pid;
    while (t >= k - pa) {
      t -= k - pa;
      ++pa;
    }
    pb = pa + t;
  }
  double shacc = 0.0;

  for (int j0 = 0; j0 < n; j0 += HCH2) {
    const int j = j0 + tid;
    const bool valid = j < n;
    double hc[K], gs[K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
      hc[a] = 0.0;
      gs[a] = 0.0;
    }
    int cl_j = 0;
    if (valid) {
      load_h(j, hc);
      if (check && stop_rule == STOP_ARGMAX_STABLE) cl_j = classes[(long)rid * cls_ld + j];
      sum_g(j, gs);
    }
    __syncthreads();   // sw, win (first round) / Hn free (later rounds)
    int best = 0;
    double bestv = 0.0;
#pragma unroll
    for (int a = 0; a < K; ++a) {
      double hn = 0.0;
      if (valid) {
        double d = 0.0;
#pragma unroll
        for (int bb = 0; bb < K; ++bb) d = fma(sw[a * KMAX + bb], hc[bb], d);
        hn = mu_rule(hc[a], gs[a], d);
        H[(long)(c0 + a) * n_pad + j] = hn;
        if (tolx) {   // calculateMaxchange(h, h0) (calculatemaxchange.c:55-60): dlange('M') of h0 and h0 - h
          tdm = fmax(tdm, fabs(hc[a] - hn));
          tom = fmax(tom, fabs(hc[a]));
        }
        if (refc) {
          // flat column-major index of (a, j) in the k x n buffer; window i reads [i*n, i*n + k)
          const int tf = j * k + a;
          const int wi = tf / n;
          const int wj = tf - wi * n;
          if (wi < k && wj < k) win[wi * KMAX + wj] = hn;
        }
      }
      Hn[a * HCH2 + tid] = hn;
      if (a == 0 || hn > bestv) {   // first maximum
        best = a;
        bestv = hn;
      }
    }
    if (check && stop_rule == STOP_ARGMAX_STABLE && valid && cl_j != best) {
      classes[(long)rid * cls_ld + j] = best;
      changed = 1;
    }
    __syncthreads();
    if (pid < npairs) {
      const int cnt = min(HCH2, n - j0);
      const double* ha = Hn + pa * HCH2;
      const double* hb = Hn + pb * HCH2;
      // 8 samples' operands loaded ahead of their (in-order) FMAs: the LDS latency is paid once per 8 terms
      int q = pq;
      for (; q + 7 * T < cnt; q += 8 * T) {
        double xa[8], xb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          xa[u] = ha[q + u * T];
          xb[u] = hb[q + u * T];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) shacc = fma(xa[u], xb[u], shacc);
      }
      for (; q < cnt; q += T) shacc = fma(ha[q], hb[q], shacc);
    }
  }
  shp[tid] = shacc;
  if (tolx) {
    atomicMax(&sm.dmax, (unsigned long long)__double_as_longlong(tdm));
    atomicMax(&sm.omax, (unsigned long long)__double_as_longlong(tom));
  }
  __syncthreads();
  if (tolx && tid == 0)
    Hstat[rid] = __longlong_as_double((long long)sm.dmax) / (SQRTEPS + __longlong_as_double((long long)sm.omax));
  if (pid < npairs && pq == 0) {
    double s = shp[tid];
    for (int q = 1; q < T; ++q) s += shp[tid + q];
    SH[me.sq_off + pa * k + pb] = s;
    SH[me.sq_off + pb * k + pa] = s;
    if (SHP) {   // the panel-row copy for the W update: row = global column c0 + a, KMAX doubles
      SHP[(long)(c0 + pa) * KMAX + pb] = s;
      SHP[(long)(c0 + pb) * KMAX + pa] = s;
    }
  }
  if (colact && tid < k) colact[c0 + tid] = iter;   // this restart's columns take part in the W update
  if (refc && tid < nwin) {
    int c = 0;
    for (int jj = 1; jj < k; ++jj)
      if (win[tid * KMAX + jj] > win[tid * KMAX + jj - 1]) c = jj;
    if (cl_prev != c) {
      classes[(long)rid * cls_ld + tid] = c;
      changed = 1;
    }
  }
  __syncthreads();
  if (tid == 0) {
    int reason = 0;
    if (check && stop_rule != STOP_TOLX) {   // the TolX test runs after the W update (k_wstat)
      if (!changed) {
        const int u = u_prev + 1;
        unchanged[rid] = u;
        if (u >= 200) reason = 1;   // nmf_mu.c:269-271
      } else {
        unchanged[rid] = 0;
      }
    }
    if (!reason && iter >= maxiter) reason = 2;
    if (reason) {
      stop_iter[rid] = iter;
      stop_reason[rid] = reason;
      atomicAdd(n_stopped, 1);
    }
  }
}

// <32, 4>: 4 waves per SIMD, two 512-thread workgroups per CU (full-load launch 150 -> 118 us).
template <int GSV = 32, int MINW = 4>
static __global__ __launch_bounds__(NTH, MINW) void k_hupdate(int iter, int maxiter, int stop_rule,
                                                        const RestartInfo* __restrict__ ri, int n, long n_pad,
                                                        const double* __restrict__ Gpart, long g_ld, long g_split,
                                                        int gsplit, int nsplit, const double* __restrict__ SWpart,
                                                        long sw_total,
                                                        double* __restrict__ H, double* __restrict__ SH,
                                                        int* __restrict__ stop_iter, int* __restrict__ stop_reason,
                                                        int* __restrict__ unchanged, int* __restrict__ classes,
                                                        long cls_ld, int* __restrict__ n_stopped,
                                                        double* __restrict__ SHP, int* __restrict__ colact,
                                                        double* __restrict__ Hstat) {
  __shared__ HupdSmem sm;
  const RestartInfo me = ri[blockIdx.x];
  if (stop_iter[me.rid] != 0) return;
#define NMFC_HUPD_CASE(KK)                                                                                      \
  case KK:                                                                                                     \
    hupdate_body<KK, GSV>(me, iter, maxiter, stop_rule, n, n_pad, Gpart, g_ld, g_split, gsplit, nsplit, SWpart, sw_total, H, SH, \
                     stop_iter, stop_reason, unchanged, classes, cls_ld, n_stopped, SHP, colact, Hstat, sm);   \
    break;
  switch (me.k) {
    NMFC_HUPD_CASE(2) NMFC_HUPD_CASE(3) NMFC_HUPD_CASE(4) NMFC_HUPD_CASE(5) NMFC_HUPD_CASE(6)
    NMFC_HUPD_CASE(7) NMFC_HUPD_CASE(8) NMFC_HUPD_CASE(9) NMFC_HUPD_CASE(10) NMFC_HUPD_CASE(11)
    NMFC_HUPD_CASE(12) NMFC_HUPD_CASE(13) NMFC_HUPD_CASE(14) NMFC_HUPD_CASE(15) NMFC_HUPD_CASE(16)
    default: break;
  }
#undef NMFC_HUPD_CASE
}

constexpr bool AHTW_KSKIP = NMFC_AHTW_KSKIP != 0;   // A h^T: skip the K-padding half of the last stage (KHALF)

// ---------------------------------------------------------------------------------------------
// Item map of the A h^T kernels: (panel, gene tile) from the XCD-contiguous item index.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void ahtw_map(int item, int npanels, int ngt, int& p, int& gt) {
  // bands of SP panels, gene super-tiles of SG: neighbours share operands in L2
  const int SP = NMFC_AHTW_SP, SG = NMFC_AHTW_SG;
  const int band = item / (SP * ngt);
  const int rem = item % (SP * ngt);
  const int bp = min(SP, npanels - band * SP);
  const int sg = rem / (bp * SG);
  const int gsz = min(SG, ngt - sg * SG);
  const int w2 = rem - sg * bp * SG;
  p = band * SP + w2 / gsz;
  gt = ngt - 1 - (sg * SG + w2 % gsz);   // high gene tiles first: W^T A streamed them last
}

// ---------------------------------------------------------------------------------------------
// K3 v4 "ahtw4": F = A h^T on the GTile ring (NPT panels x GTG genes, 4 waves per panel: WR = NPT,
// WC = 4, each wave 64 panel rows x GTG/4 genes) + the panels' h h^T rows in LDS.  Engine default (LATE,
// NBUF = 2, GTG = 128): a 2 x 24 KiB ring and 160 VGPRs, so THREE workgroups share a CU and their K loops
// cover each other's prologues and epilogues (MFMA busy 75.5 -> 80.2 % at full load, +4.5 % kernel rate
// over the 3-stage, 80 KiB, two-per-CU form); the h h^T rows wait in registers until the loop is done,
// and W0 streams in by 16-row blocks during the epilogue.  Column state lives in registers: each wave reads its
// panel's 64 ColInfo entries (lane = column), the active set is a 64-bit ballot of colact[c] == iter
// (k_hupdate stamps its restart's columns with the iteration it ran) and the E-operand rows' (lc0, k)
// come by lane shuffles.  These setup loads are issued after the first DMA stages, so they overlap
// them.  The h h^T rows are read from SHP (panel-row layout written by k_hupdate), one coalesced
// block.  W0 is loaded in the D layout right after the last DMA issue and is the B operand of
// E = W0 (h h^T) directly.
// ---------------------------------------------------------------------------------------------
// GTG: genes per tile (128 at full load; 64 for small grids: half the MFMA chain per wave, twice the
// workgroups).  ngt = m_pad / GTG; npanels is a multiple of NPT.  Every shape accumulates in the
// canonical GTile K order.
// PR = 16 is the narrow (tail) form: only the first 16 columns of panel 0 are live, so the tile covers
// those 16 rows (WC waves along the genes): a quarter of the H / W bytes and MFMA work per gene tile.
// LATE: the h h^T rows stay in registers through the K loop and are staged afterwards into a ring buffer
// the last step no longer reads, and W0 is loaded after the loop: no LDS beyond the ring and no W0
// registers live in the loop, so more workgroups fit a CU (their K loops cover each other's epilogues).
template <int GTG = GT, int NBUF = GT_NBUF, int NPT = 1, int PR = PANEL, int WC = 4, bool LATE = false>
static constexpr int ahtw4_lds() {
  return GTile<PR * NPT, GTG, NPT, WC, NBUF>::LDS_BYTES + (LATE ? 0 : NPT * PR * KMAX * 8);
}
// KHALF: the last K stage's second half is padding (n_pad - n >= 8, decided on the host): skipped.
template <int GTG = GT, int NBUF = GT_NBUF, int NPT = 1, int PR = PANEL, int WC = 4, bool LATE = false, bool KHALF = false>
static __global__ __launch_bounds__(64 * NPT * WC,
                                    (163840 / ahtw4_lds<GTG, NBUF, NPT, PR, WC, LATE>()) * NPT * WC / 4 > 8
                                        ? 8
                                        : (163840 / ahtw4_lds<GTG, NBUF, NPT, PR, WC, LATE>()) * NPT * WC / 4)
void k_ahtw4(int iter, const double* __restrict__ H, long n_pad, const double* __restrict__ Arm, long m_pad,
             double* __restrict__ W, const double* __restrict__ SHP, const ColInfo* __restrict__ ci,
             const int* __restrict__ colact, int npanels, int ngt) {
  using TileW4 = GTile<PR * NPT, GTG, NPT, WC, NBUF>;
  constexpr int AHTW4_SH = TileW4::LDS_BYTES;
  constexpr int AHTW4_LDS = ahtw4_lds<GTG, NBUF, NPT, PR, WC, LATE>();
  static_assert(AHTW4_LDS <= 163840, "LDS of one CU");
  static_assert(PR == PANEL || (PR == 16 && NPT == 1), "narrow tiles: one 16-column block");
  static_assert(!LATE || TileW4::STAGE_BYTES >= NPT * PR * KMAX * 8, "h h^T rows fit one ring stage");
  constexpr int NTH = 64 * NPT * WC;
  __shared__ __attribute__((aligned(1024))) char smem[AHTW4_LDS];
  double* SHl = reinterpret_cast<double*>(smem + AHTW4_SH);   // !LATE; LATE: set after the K loop
  int pp, gt;
  ahtw_map(xcd_item(blockIdx.x, (npanels / NPT) * ngt), npanels / NPT, ngt, pp, gt);
  const int p0 = pp * NPT;   // first panel of the tile
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), wr = w / WC, wc = w % WC;
  const int p = p0 + wr;     // this wave's panel
  ColInfo cc;
  uint64_t actmask = 0;
  TileW4 tl;
  tl.zero();
  // PR = 16: the "panel" index p is a 16-column block (column 16 p of the stacked W / H).
  // W0 loads and W stores through a buffer resource over this wave's W rows: one 32-bit lane offset, the
  // (row block, nb) part wave-uniform in soffset -- no 64-bit row addresses held in VGPRs across the K loop
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
        w0[mb][nb][reg] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rw, wvoff, woff(mb, reg, nb), 0));
  };
  auto load_w0 = [&] {
#pragma unroll
    for (int mb = 0; mb < TileW4::MB; ++mb) load_w0_block(mb);
  };
  constexpr int NSH = NPT * PR * KMAX / 2 / NTH;
  static_assert(NSH * 2 * NTH == NPT * PR * KMAX, "h h^T rows split evenly over the threads");
  d2 shv[NSH];
  // W0 blocks 0 and 1 go out with the last K stage's DMA (EARLY, the 2-stage LATE form): their latency is covered by
  // the last step's MFMAs instead of opening the epilogue (round 5: +2 % at full load, tools/kvar.hip form EW)
  constexpr bool EARLY = LATE && NBUF == 2 && TileW4::MB >= 2;
  constexpr int XL = LATE ? (EARLY ? 2 * TileW4::NB * 4 : 0) : TileW4::MB * TileW4::NB * 4;
  const bool live = tl.template run<XL, KHALF ? 1 : 2>(
      H + (long)p0 * PR * n_pad, n_pad, Arm + (long)gt * GTG * n_pad, n_pad, 0, (int)n_pad, smem,
      [&] {   // setup loads, independent of each other, overlapping the first stages' DMA
        cc = lane < PR ? ci[(long)p * PR + lane] : ColInfo{0, 0, 0, 0};
        int ca[NPT];
#pragma unroll
        for (int q = 0; q < NPT; ++q) ca[q] = lane < PR ? colact[(long)(p0 + q) * PR + lane] : -1;
        const d2* src = reinterpret_cast<const d2*>(SHP + (long)p0 * PR * KMAX);
#pragma unroll
        for (int j = 0; j < NSH; ++j) shv[j] = src[tid + NTH * j];
        bool any = false;
#pragma unroll
        for (int q = 0; q < NPT; ++q) {
          const uint64_t mk = __ballot(ca[q] == iter);   // the column's restart ran k_hupdate at this iteration
          if (q == wr) actmask = mk;
          any = any || mk != 0;
        }
        if (!any) return false;   // every panel of the tile idle (the same answer in every wave)
        if constexpr (!LATE) {
#pragma unroll
          for (int j = 0; j < NSH; ++j) reinterpret_cast<d2*>(SHl)[tid + NTH * j] = shv[j];
        }
        return true;   // SHl is published by the ring prologue's barrier
      },
      [](const char*) {},
      [&] {
        if constexpr (!LATE) load_w0();
        if constexpr (EARLY) {
          load_w0_block(0);
          load_w0_block(1);
        }
      });
  if (!live) return;
  if constexpr (LATE) {
    // the ring buffer of stage nst - 2: every wave passed the barrier after reading it (nst >= 2)
    const int nst = (int)n_pad / BK2;
    SHl = reinterpret_cast<double*>(smem + ((nst - 2) % NBUF) * TileW4::STAGE_BYTES);
#pragma unroll
    for (int j = 0; j < NSH; ++j) reinterpret_cast<d2*>(SHl)[tid + NTH * j] = shv[j];
    // W0 by 16-row blocks, one block ahead of the epilogue's block loop (block mb's E reads blocks
    // mb - 1 .. mb + 1 only), so at most three blocks are live at once
    if constexpr (!EARLY) {
#pragma unroll
      for (int mb = 0; mb < (TileW4::MB < 2 ? TileW4::MB : 2); ++mb) load_w0_block(mb);
    }
  }
  // Block-aligned restarts (the engine's 16-column block packing: no active restart crosses a 16-column block) take
  // E over the four K steps of their own block, no shuffles for its K range; the K steps the restarts do not cover
  // add exact zeros (0 x finite W0), so the bits are those of the general form, which stays for any other packing.
  const bool cross = ((actmask >> lane) & 1) && ((cc.lc0 & (PR - 1)) >> 4) != (((cc.lc0 & (PR - 1)) + cc.k - 1) >> 4);
  const bool aligned = __ballot(cross) == 0;   // wave-uniform
  if constexpr (LATE) __syncthreads();
  if (actmask == 0) return;   // this wave's panel is idle (its partner panel is not)
  const double* SHw = SHl + (long)wr * PR * KMAX;
#pragma unroll
  for (int mb = 0; mb < TileW4::MB; ++mb) {
    if constexpr (LATE) {
      if (mb + 2 < TileW4::MB) load_w0_block(mb + 2);
    }
    const int ra = 16 * mb + (lane & 15);
    const int alc = __shfl(cc.lc0, ra) & (PR - 1);   // tile-local (a restart never straddles a tile)
    const int ak = ((actmask >> ra) & 1) ? __shfl(cc.k, ra) : 0;
    d4 e[TileW4::NB];
#pragma unroll
    for (int nb = 0; nb < TileW4::NB; ++nb) e[nb] = d4{0.0, 0.0, 0.0, 0.0};
    if (aligned) {
      double av[4];   // the block's four K steps' operands loaded ahead of the MFMA chain
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
    } else {
      int lo = ak ? alc : PANEL, hi = ak ? alc + ak : 0;
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off));
        hi = max(hi, __shfl_xor(hi, off));
      }
      lo = __builtin_amdgcn_readfirstlane(lo);
      hi = __builtin_amdgcn_readfirstlane(hi);
      // K = the rows of the restarts touching block mb: within [16 mb - 15, 16 mb + 31) (k <= 16, restarts never
      // leave the tile), i.e. K steps q in [4 mb - 4, 4 mb + 8)
#pragma unroll
      for (int q = (4 * mb - 4 > 0 ? 4 * mb - 4 : 0); q < (4 * mb + 8 < 4 * TileW4::MB ? 4 * mb + 8 : 4 * TileW4::MB); ++q) {
        if (4 * q + 3 < lo || 4 * q >= hi) continue;   // wave-uniform
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
        const double v = mu_rule_sel(w0[mb][nb][reg], tl.acc[mb][nb][reg], e[nb][reg]);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rw, wvoff, woff(mb, reg, nb), 0);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Small shapes (m_pad <= 1024, n <= 64: the bundled gct, BASELINE configs[0..1]): ONE persistent workgroup
// runs a 16-column block of restarts (restarts never straddle a block) through the whole MU loop and the
// stop rule in-kernel -- no per-iteration launches, A read from L2.  4 waves; wave w owns the gene blocks
// [w*GBW, (w+1)*GBW) and keeps its W rows in registers in the fp64 MFMA D layout
//   w[gb][r] = W[g = 16*(w*GBW + gb) + (lane>>4) + 4r][c = lane & 15],
// which is at once the A operand of G = W^T A and of W^T W (K = genes), and the D layout of
// F = A h^T, E = W0 (h h^T) and the W update, so W never moves.  Per iteration (nmf_mu.c:174-216):
//   G, W^T W   per wave over its genes (MFMA chains in gene order), the 4 wave partials summed in wave order
//   H update   h = mu_rule(H, G, (W^T W) H) per (column, sample), d summed over the restart's columns in order
//   h h^T      one wave, MFMA over the samples (zeroed across restarts)
//   F, E, W    per wave: F = A h^T (K = samples), E = W0 (h h^T) (W0 transposed through LDS), W rule
//   stop rule  every even iteration (REF_COMPAT windows / ARGMAX_STABLE classes), nmf_mu.c:253-282
// A restart that stops freezes its columns; the block ends when all its restarts have stopped.
// Deterministic: every reduction order is a function of (m, n) only, so a job gives the same bits in
// any block and any batch.
// ---------------------------------------------------------------------------------------------
constexpr int SMALL_PF = NMFC_SMALL_PF;
constexpr int SMALL_FPF = NMFC_SMALL_FPF;
constexpr int SMALL_NW = 4;
constexpr int SMALL_MAXR = 8;   // restarts per 16-column block (k >= 2)
constexpr int SMALL_GGMAX = 4;  // gene blocks per F/E group: 4 when GBW % 4 == 0, else 2 (GBW is even)

struct SmallBlock {
  int col0;                  // first stacked column of the block (W/H rows col0 .. col0 + 15)
  int nr;                    // restarts in the block
  int rid[SMALL_MAXR];       // persistent restart ids
  int k[SMALL_MAXR];
  int lc0[SMALL_MAXR];       // block-local first column
};

// One restart of a batched k_solo_mu launch (csrc/solo.hip; rank <= 4 on gct-sized shapes): its stacked W/H
// rows col0 .. col0 + k - 1 and its persistent restart id (stop iteration / reason slots).
struct SoloJob {
  int col0, k, rid, pad;
};

template <int JB, int NW = SMALL_NW>
struct SmallSmem {
  double H[2][16][16 * JB];        // H of the block (rows = columns c), double-buffered: the update writes the other one
  union {                          // G partials (G phase .. H update) and W0 transpositions (F/E phase) never overlap
    double Gp[NW][16][16 * JB];
    double T[NW][SMALL_GGMAX][16][17];   // per-wave W0 block transpositions (padded rows), SMALL_GG blocks
  } u;
  double SWp[NW][16][16];
  double SW[16][16];
  double S[16][16];                // h h^T, zero across restarts
  double win[SMALL_MAXR][16][16];  // REF_COMPAT windows
  int cls[SMALL_MAXR][64];         // classes (REF_COMPAT: windows i < k; ARGMAX_STABLE: samples)
  int colr[16];                    // restart slot of each column (-1: padding)
  int run[SMALL_MAXR];             // 1 while the restart runs
  int unch[SMALL_MAXR];
  int changed[SMALL_MAXR];
  int nrun;
};

// SKIP != 0 only in tools/smallbench.hip (phase cost breakdown): bit 0 no G/W^T W, 1 no H update,
// 2 no h h^T / stop rule, 3 no F/E/W update, 4 no E = W0 (h h^T), 5 W rule replaced by adds.
// NW waves (4 or 8); GBW = m_pad / (16 NW) gene blocks per wave.  The wave partials are summed in wave order, so
// the NW = 4 and NW = 8 forms differ in the last bits (each is a function of (m, n) only).
template <int GBW, int JB, int SKIP = 0, int NW = SMALL_NW>
static __global__ __launch_bounds__(64 * NW) void k_small_mu(
    const SmallBlock* __restrict__ blocks, const double* __restrict__ Arm, long ld_rm, const double* __restrict__ Acm,
    long m_pad, int n, long n_pad, double* __restrict__ W, double* __restrict__ H, int maxiter, int stop_rule,
    int* __restrict__ stop_iter, int* __restrict__ stop_reason) {
  constexpr int NP = 16 * JB;
  // prefetch distances: with eight waves (two per SIMD) the other wave covers part of the load latency, and the
  // registers are half (256 per lane)
  constexpr int PF = NW == 8 ? SMALL_PF / 2 : SMALL_PF, FPF = SMALL_FPF;   // 8 waves: PF 2 / 4 / 8 tied or slower, FPF 8 +1 %
  __shared__ SmallSmem<JB, NW> sm;
  __shared__ SmallBlock blk;   // in LDS: indexed by restart slot at run time
  if (threadIdx.x == 0) blk = blocks[blockIdx.x];
  __syncthreads();
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, lr = l >> 4, lc = l & 15;
  const int nr = blk.nr;
  // ---- state ----
  if (tid < 16) sm.colr[tid] = -1;
  __syncthreads();
  if (tid < nr)
    for (int a = 0; a < blk.k[tid]; ++a) sm.colr[blk.lc0[tid] + a] = tid;
  if (tid < SMALL_MAXR) {
    sm.run[tid] = tid < nr;
    sm.unch[tid] = 0;
  }
  for (int x = tid; x < SMALL_MAXR * 64; x += 64 * NW) (&sm.cls[0][0])[x] = 0;   // nmf_mu.c:132
  for (int x = tid; x < 16 * NP; x += 64 * NW) {
    const int c = x / NP, j = x % NP;
    sm.H[0][c][j] = (j < n) ? H[(long)(blk.col0 + c) * n_pad + j] : 0.0;
  }
  double wr[GBW][4];
#pragma unroll
  for (int gb = 0; gb < GBW; ++gb)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      wr[gb][r] = W[(long)(blk.col0 + lc) * m_pad + 16 * (w * GBW + gb) + 4 * r + lr];
  if (tid == 0) sm.nrun = nr;
  __syncthreads();
  int hb = 0;   // sm.H[hb]: the current H
  for (int iter = 1; iter <= maxiter; ++iter) {
    // the operand base pointers are laundered every iteration: otherwise the compiler hoists the
    // per-k-step addresses of all 4*GBW k-steps out of the iteration loop (hundreds of registers)
    // (a laundered zero OFFSET, not a laundered pointer: the pointers keep their global address space, so
    // the loads stay global_load -- a laundered pointer becomes flat and waits on lgkmcnt too)
    long zo = 0;
    asm volatile("" : "+s"(zo));
    const double* __restrict__ ArmI = Arm + zo;
    const double* __restrict__ AcmI = Acm + zo;
    // ---- G = W^T A, W^T W over this wave's genes ----
    d4 gacc[JB], sacc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) gacc[jb] = (d4){0.0, 0.0, 0.0, 0.0};
    // software-pipelined: the A rows of k-step t + PF are loaded at step t into a register ring
    // (the loads are L2 hits; issued just before their use they would expose the L2 latency every k-step)
    {
      constexpr int NKS = (SKIP & 1) ? 0 : 4 * GBW;
      double pf[PF][JB];
      constexpr long LDR = (JB <= 2) ? 32 : 64;   // == ld_rm (n_pad = round_up(n, 32), n <= 16 JB; host-checked)
      const double* __restrict__ arow = ArmI + (long)(16 * w * GBW + lr) * LDR + lc;
#pragma unroll
      for (int t = 0; t < PF; ++t)
        if (t < NKS) {
#pragma unroll
          for (int jb = 0; jb < JB; ++jb) pf[t][jb] = arow[(long)(4 * t) * LDR + 16 * jb];
        }
#pragma unroll
      for (int t = 0; t < NKS; ++t) {
        const int gb = t >> 2, r = t & 3;
        double av[JB];
#pragma unroll
        for (int jb = 0; jb < JB; ++jb) av[jb] = pf[t % PF][jb];
        if (t + PF < NKS) {
#pragma unroll
          for (int jb = 0; jb < JB; ++jb) pf[t % PF][jb] = arow[(long)(4 * (t + PF)) * LDR + 16 * jb];
        }
#pragma unroll
        for (int jb = 0; jb < JB; ++jb) gacc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(wr[gb][r], av[jb], gacc[jb], 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(wr[gb][r], wr[gb][r], sacc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);   // keep the issue order: prefetch distance PF k-steps
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int jb = 0; jb < JB; ++jb) sm.u.Gp[w][lr + 4 * r][16 * jb + lc] = gacc[jb][r];
      sm.SWp[w][lr + 4 * r][lc] = sacc[r];
    }
    __syncthreads();
    if (tid < 256) {   // W^T W: wave partials in wave order
      const int c = tid >> 4, d = tid & 15;
      double sw = sm.SWp[0][c][d];
#pragma unroll
      for (int v = 1; v < NW; ++v) sw += sm.SWp[v][c][d];
      sm.SW[c][d] = sw;
      if (tid < SMALL_MAXR) sm.changed[tid] = 0;
    }
    __syncthreads();
    // ---- H update (nmf_mu.c:178, 184-191) from sm.H[hb] into sm.H[hb ^ 1] ----
    // (the run flags for this iteration's W update are read here, before any thread can reach the bookkeeping below)
    int runmask = 0;
#pragma unroll
    for (int q = 0; q < SMALL_MAXR; ++q) runmask |= (q < nr && sm.run[q]) ? (1 << q) : 0;
    {
      const double(*Ho)[NP] = sm.H[hb];
      double(*Hn)[NP] = sm.H[hb ^ 1];
#pragma unroll
      for (int u = 0; u < (16 * NP + 64 * NW - 1) / (64 * NW); ++u) {
        const int x = tid + u * 64 * NW;
        if (x < 16 * NP) {
          const int c = x / NP, j = x % NP;
          const int q = sm.colr[c];
          const double h0 = Ho[c][j];
          double hv = h0;
          if (!(SKIP & 2) && q >= 0 && ((runmask >> q) & 1) && j < n) {
            double gsum = sm.u.Gp[0][c][j];
#pragma unroll
            for (int v = 1; v < NW; ++v) gsum += sm.u.Gp[v][c][j];
            const int b0 = blk.lc0[q], kq = blk.k[q];
            double dsum = 0.0;
            for (int b = 0; b < kq; ++b) dsum = fma(sm.SW[c][b0 + b], Ho[b0 + b][j], dsum);
            hv = mu_rule(h0, gsum, dsum);
          }
          Hn[c][j] = hv;
        }
      }
    }
    hb ^= 1;
    __syncthreads();
    const double(*Hc)[NP] = sm.H[hb];
    // ---- h h^T (nmf_mu.c:200) by wave 0; stop rule (nmf_mu.c:253-282) by the other waves at the same time ----
    const bool check = !(SKIP & 4) && stop_rule != STOP_FIXED && iter > 1 && (iter % 2 == 0);
    if (w == 0 && !(SKIP & 4)) {
      d4 hh = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < NP / 4; ++q) {
        const double hv = Hc[lc][4 * q + lr];
        hh = __builtin_amdgcn_mfma_f64_16x16x4f64(hv, hv, hh, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = lr + 4 * r, d = lc;
        const int qc = sm.colr[c];
        sm.S[c][d] = (qc >= 0 && qc == sm.colr[d]) ? hh[r] : 0.0;
      }
    } else if (check) {   // concurrently with wave 0's h h^T chain: both only read the new H
      const int t1 = tid - 64;
      if (stop_rule == STOP_REF_COMPAT) {
        // window i of restart q reads the flat k x n column-major buffer at [i*n, i*n + k)
        for (int x = t1; x < nr * 16; x += 64 * (NW - 1)) {
          const int q = x >> 4, i = x & 15, kq = blk.k[q];
          if (i >= kq || i >= n || !sm.run[q]) continue;
          int cl = 0;
          double prev = 0.0;
          for (int jj = 0; jj < kq; ++jj) {
            const int f = i * n + jj, j = f / kq, a = f - j * kq;
            const double v = Hc[blk.lc0[q] + a][j];
            if (jj > 0 && v > prev) cl = jj;
            prev = v;
          }
          if (sm.cls[q][i] != cl) {
            sm.cls[q][i] = cl;
            sm.changed[q] = 1;
          }
        }
      } else if (stop_rule == STOP_ARGMAX_STABLE) {
        for (int x = t1; x < nr * 64; x += 64 * (NW - 1)) {
          const int q = x >> 6, j = x & 63;
          if (j >= n || !sm.run[q]) continue;
          int best = 0;
          double bv = Hc[blk.lc0[q]][j];
          for (int a = 1; a < blk.k[q]; ++a) {
            const double v = Hc[blk.lc0[q] + a][j];
            if (v > bv) {
              bv = v;
              best = a;
            }
          }
          if (sm.cls[q][j] != best) {
            sm.cls[q][j] = best;
            sm.changed[q] = 1;
          }
        }
      }
    }
    __syncthreads();
    // ---- F = A h^T, E = W0 (h h^T), W update (nmf_mu.c:198-216) ----
    const int qmine = sm.colr[lc];
    const bool upd = qmine >= 0 && ((runmask >> qmine) & 1);
    constexpr int SMALL_GG = (NW == 4 && GBW % 4 == 0) ? 4 : 2;   // eight waves: two chains per wave, two waves per SIMD
    constexpr int NQ = NP / 4;                                    // K steps of F (samples, 4 per step)
    constexpr int NFS = (SKIP & 8) ? 0 : (GBW / SMALL_GG) * NQ;   // (group, K step) pairs of this wave
    constexpr long MP = 16L * NW * GBW;                           // == m_pad (host-checked)
    // the A columns of step t + PF are loaded at step t into a register ring (rows >= n are in
    // bounds: Acm holds round_up(n, 128) columns, zero past n)
    double fpf[FPF][SMALL_GG];
    double hvq[NQ];   // the B operand of every F step (h^T rows), the same for every gene group
#pragma unroll
    for (int q = 0; q < NQ; ++q) hvq[q] = Hc[lc][4 * q + lr];
    const double* __restrict__ acol = AcmI + (long)lr * MP + 16 * w * GBW + lc;
    auto f_load = [&](int t, double* dst) {
      const int g4 = (t / NQ) * SMALL_GG, q = t % NQ;
#pragma unroll
      for (int i = 0; i < SMALL_GG; ++i) dst[i] = acol[(long)(4 * q) * MP + 16 * (g4 + i)];
    };
#pragma unroll
    for (int t = 0; t < FPF; ++t)
      if (t < NFS) f_load(t, fpf[t]);
    // GG gene blocks at a time: GG independent MFMA chains for F and for E (a single chain per block would
    // leave the matrix pipe waiting on the dependent-issue latency)
#pragma unroll
    for (int g4 = 0; g4 < ((SKIP & 8) ? 0 : GBW); g4 += SMALL_GG) {
      d4 f[SMALL_GG], e[SMALL_GG];
#pragma unroll
      for (int i = 0; i < SMALL_GG; ++i) {
        f[i] = (d4){0.0, 0.0, 0.0, 0.0};
        e[i] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!(SKIP & 16)) sm.u.T[w][i][lr + 4 * r][lc] = wr[g4 + i][r];
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int t = (g4 / SMALL_GG) * NQ + q;
        double av[SMALL_GG];
#pragma unroll
        for (int i = 0; i < SMALL_GG; ++i) av[i] = fpf[t % FPF][i];
        if (t + FPF < NFS) f_load(t + FPF, fpf[t % FPF]);
        // every step, also past n (zero rows of h^T add exact zeros): a data-dependent skip here makes the
        // compiler shuttle the accumulators between AGPRs and VGPRs around each step
#pragma unroll
        for (int i = 0; i < SMALL_GG; ++i) f[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], hvq[q], f[i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);   // keep the prefetch distance
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < ((SKIP & 16) ? 0 : 4); ++q) {
        const double sv = sm.S[4 * q + lr][lc];
#pragma unroll
        for (int i = 0; i < SMALL_GG; ++i)
          e[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(sm.u.T[w][i][lc][4 * q + lr], sv, e[i], 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
      if ((SKIP & 32) && upd) {
#pragma unroll
        for (int i = 0; i < SMALL_GG; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) wr[g4 + i][r] += f[i][r] + e[i][r];
      } else if (upd) {
#pragma unroll
        for (int i = 0; i < SMALL_GG; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) wr[g4 + i][r] = mu_rule(wr[g4 + i][r], f[i][r], e[i][r]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- stop bookkeeping (one thread, right after its own W rule: every thread read this iteration's run flags
    // before the barrier ahead of the F phase, and nothing reads the stop state until the barrier below), then
    // every thread sees the new run flags ----
    if (tid == 0) {
      for (int q = 0; q < nr; ++q) {
        if (!sm.run[q]) continue;
        int reason = 0;
        if (check) {
          if (!sm.changed[q]) {
            if (++sm.unch[q] >= 200) reason = 1;   // nmf_mu.c:269-271
          } else {
            sm.unch[q] = 0;
          }
        }
        if (!reason && iter >= maxiter) reason = 2;
        if (reason) {
          sm.run[q] = 0;
          --sm.nrun;
          stop_iter[blk.rid[q]] = iter;
          stop_reason[blk.rid[q]] = reason;
        }
      }
    }
    __syncthreads();
    if (sm.nrun == 0) break;
  }
  // ---- final factors back to the stacked layout ----
#pragma unroll
  for (int gb = 0; gb < GBW; ++gb)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      W[(long)(blk.col0 + lc) * m_pad + 16 * (w * GBW + gb) + 4 * r + lr] = wr[gb][r];
  for (int x = tid; x < 16 * NP; x += 64 * NW) {
    const int c = x / NP, j = x % NP;
    if (j < n) H[(long)(blk.col0 + c) * n_pad + j] = sm.H[hb][c][j];
  }
}

// ---------------------------------------------------------------------------------------------
// Team form of the small-shape loop (k_team_mu, round 3).  One workgroup per 16-column block (k_small_mu)
// is bound by that CU's matrix pipe: ~512 MFMAs per wave per iteration, ~14 us, whatever k is.  Here a
// block is run by a TEAM of P = m_pad / 64 workgroups (up to 128); workgroup p owns genes [64p, 64p + 64) and keeps
// its slice of A in registers for the whole launch, in both operand layouts:
//   ag[s] = A[64p + 4s + (lane>>4)][16w + (lane&15)]   (B operand of G = W^T A, wave w = sample block w)
//   af[t] = A[64p + 16w + (lane&15)][4t + (lane>>4)]   (B operand of F^T = h A^T, wave w = genes 16w..)
// and its W rows as wg[s] = W[64p + 4s + (lane>>4)][c = lane&15] (A operand of G and W^T W) and in the
// D layout wd[r] = W[64p + 16w + (lane&15)][c = (lane>>4) + 4r] (B operand of E^T = S W^T, the W rule).
// Per iteration (nmf_mu.c:174-216) a workgroup forms its partial G and W^T W over its 64 genes (MFMA
// chains in gene order, W^T W's four wave partials summed in wave order) and publishes them; every
// workgroup then sums the P partials in workgroup order -- the same bits in every workgroup -- and repeats
// the H update, h h^T and the stop rule redundantly, so only G and W^T W cross workgroups.  F^T = h A^T
// (K = samples), E^T = (h h^T) W0^T and the W rule stay local.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the measured sc1 table): every
// partial is stored `sc1` (write-through), every storing wave waits vmcnt(0), the workgroup barrier, then ONE
// lane stores the workgroup's flag (`sc1`, the iteration's tag); a consumer polls all P flags at once (lane q
// (and q + 64) of wave 0 reads flag q, one coalesced `sc1` load per poll), meets at a workgroup barrier and reads the
// partials with `sc1` loads only.  (The data-tagged granule form, R2, was measured slower here: 16 producers'
// granules re-read per retry.)  Tags are tag_base + the team's iteration count (monotonic; a caller that
// carries tag_base across launches need not zero the flags again), and the partials alternate between two
// buffers by parity, so a workgroup one iteration ahead (flag = tag + 1) never overwrites what another still
// reads.  The grid holds only as many teams as are resident at once (host-sized); a team runs its blocks one
// after another.  Every wait is bounded: a team that cannot meet sets *err and ends (the host reports the
// failure) instead of hanging.
// Deterministic: every order is a function of (m_pad, n) only, so a job gives the same bits in any block.
// ---------------------------------------------------------------------------------------------
constexpr int TEAM_ROWS = 64;           // genes per workgroup of a team
constexpr int TEAM_PMAX = 128;          // workgroups per team (m_pad <= 8192)
constexpr int TEAM_LB = 16;             // partials loaded per batch (in flight at once) when summing
constexpr long TEAM_SPIN_MAX = 1L << 22;   // re-reads before a team gives up (seconds; teams are co-resident)

template <int NJ>
struct TeamSmem {
  double H[16][16 * NJ + 1];   // current H of the block (rows = columns c; padded: conflict-free row reads)
  double G[16][16 * NJ];    // team sum of W^T A
  double SWw[4][16][16];    // wave partials of W^T W
  double SW[16][17];        // team sum of W^T W (zero across restarts)
  double S[16][17];         // h h^T (zero across restarts)
  double Wt[TEAM_ROWS][17]; // updated W rows, (gene, column), padded rows
  int cls[SMALL_MAXR][64];  // classes (REF_COMPAT: windows i < k; ARGMAX_STABLE: samples)
  int colr[16];             // restart slot of each column (-1: padding)
  int run[SMALL_MAXR];
  int unch[SMALL_MAXR];
  int changed[SMALL_MAXR];
  int nrun, ncol, abort;
  SmallBlock blk;
};

typedef unsigned long long u64;
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<u64*>(p), (u64)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load(reinterpret_cast<u64*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// sum of the P partials of one entry (slots `stride` doubles apart) in workgroup order, in batches of TEAM_LB
// loads issued back to back (every slot of a batch loaded unconditionally: the buffers hold TEAM_PMAX slots,
// slots >= P are read but not summed), one wait per batch
__device__ __forceinline__ double team_sum(const double* g, long stride, int P) {
  double s = 0.0;
  for (int q0 = 0; q0 < P; q0 += TEAM_LB) {
    double v[TEAM_LB];
#pragma unroll
    for (int q = 0; q < TEAM_LB; ++q) v[q] = ld_sc1(g + (q0 + q) * stride);
    if (q0 == 0) s = v[0];
#pragma unroll
    for (int q = 0; q < TEAM_LB; ++q)
      if ((q0 > 0 || q > 0) && q0 + q < P) s += v[q];
  }
  return s;
}

// SKIP != 0 only in tools/teambench.hip (phase cost breakdown): bit 0 no exchange (each workgroup uses its own
// partials), 1 no G / W^T W MFMAs, 2 no h h^T, 3 no F / E MFMAs, 4 no stop check, 6 phase clock stamps.
template <int NJ, int SKIP = 0>
static __global__ __launch_bounds__(256) void k_team_mu(
    const SmallBlock* __restrict__ blocks, int nblocks, int P, const double* __restrict__ Acm, long m_pad, int n,
    long n_pad, double* __restrict__ W, double* __restrict__ H, int maxiter, int stop_rule,
    int* __restrict__ stop_iter, int* __restrict__ stop_reason, double* __restrict__ Gx, double* __restrict__ SWx,
    unsigned* __restrict__ flags, unsigned tag_base, int* __restrict__ err, long long* __restrict__ prof) {
  constexpr int NP = 16 * NJ;
  constexpr int NQ = NP / 4;
  constexpr int HU = (16 * NP + 255) / 256;
  __shared__ TeamSmem<NJ> sm;
  const int team = blockIdx.x / P, p = blockIdx.x - team * P;
  const int nteams = gridDim.x / P;
  if (team >= nteams) return;   // grid not a multiple of P (host sizes it exactly)
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, lr = l >> 4, lc = l & 15;
  const int sc = tid >> 4, sd = tid & 15;   // this thread's (c, d) entry of the 16 x 16 W^T W and h h^T
  const long g0 = (long)TEAM_ROWS * p;
  double* const gx = Gx + (long)team * 2 * TEAM_PMAX * 16 * NP;   // [team][buf][slot][16][NP]
  double* const swx = SWx + (long)team * 2 * TEAM_PMAX * 256;      // [team][buf][slot][256]
  unsigned* const fl = flags + (long)team * TEAM_PMAX;             // [team][slot]
  // this workgroup's slice of A, resident for the whole launch (Acm is zero past m and n)
  double ag[16], af[NQ];
#pragma unroll
  for (int s = 0; s < 16; ++s) ag[s] = (w < NJ) ? Acm[(long)(16 * w + lc) * m_pad + g0 + 4 * s + lr] : 0.0;
#pragma unroll
  for (int t = 0; t < NQ; ++t) af[t] = Acm[(long)(4 * t + lr) * m_pad + g0 + 16 * w + lc];
  if (tid == 0) sm.abort = 0;
  unsigned epoch = 0;
  long long prof_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, prof_t = 0;
#define TEAM_STAMP(i)                                             \
  if ((SKIP & 64) && p == 0 && tid == 0) {                        \
    const long long t_ = (long long)__builtin_readcyclecounter(); \
    if ((i) > 0) prof_acc[(i)] += t_ - prof_t;                    \
    prof_t = t_;                                                  \
  }
  for (int b = team; b < nblocks; b += nteams) {
    __syncthreads();   // the previous block's readers of sm are done
    if (tid == 0) {
      sm.blk = blocks[b];
      int nc = 0;
      for (int q = 0; q < sm.blk.nr; ++q) nc = max(nc, sm.blk.lc0[q] + sm.blk.k[q]);
      sm.ncol = nc;
      sm.nrun = sm.blk.nr;
    }
    if (tid < 16) sm.colr[tid] = -1;
    __syncthreads();
    const SmallBlock& blk = sm.blk;
    const int nr = blk.nr, ncol = sm.ncol;
    if (tid < nr)
      for (int a = 0; a < blk.k[tid]; ++a) sm.colr[blk.lc0[tid] + a] = tid;
    if (tid < SMALL_MAXR) {
      sm.run[tid] = tid < nr;
      sm.unch[tid] = 0;
    }
    for (int x = tid; x < SMALL_MAXR * 64; x += 256) (&sm.cls[0][0])[x] = 0;   // nmf_mu.c:132
    for (int x = tid; x < 16 * NP; x += 256) {
      const int c = x / NP, j = x % NP;
      sm.H[c][j] = (j < n) ? H[(long)(blk.col0 + c) * n_pad + j] : 0.0;
    }
    double wg[16], wd[4];
#pragma unroll
    for (int s = 0; s < 16; ++s) wg[s] = W[(long)(blk.col0 + lc) * m_pad + g0 + 4 * s + lr];
#pragma unroll
    for (int r = 0; r < 4; ++r) wd[r] = W[(long)(blk.col0 + lr + 4 * r) * m_pad + g0 + 16 * w + lc];
    __syncthreads();
    // per-thread constants of the block: the H entries (c, j) this thread updates (live columns, j < n) with
    // their restart's columns [b0, b0 + kq), and whether W^T W entry (sc, sd) lies inside one restart
    int he_c[HU], he_j[HU], he_q[HU], he_b0[HU], he_k[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int x = tid + 256 * u;
      const int c = x / n, j = x - (x / n) * n;
      const bool live = x < ncol * n;
      const int q = live ? sm.colr[c] : -1;
      he_c[u] = c;
      he_j[u] = j;
      he_q[u] = q;
      he_b0[u] = q >= 0 ? blk.lc0[q] : 0;
      he_k[u] = q >= 0 ? blk.k[q] : 0;
    }
    const int sq = sm.colr[sc];
    const bool sw_live = sc < ncol && sd < ncol && sq >= 0 && sq == sm.colr[sd];
    int wq[4];   // restart slot of this lane's W-rule columns lr + 4r
#pragma unroll
    for (int r = 0; r < 4; ++r) wq[r] = sm.colr[lr + 4 * r];
    int runmask = (1 << nr) - 1;   // restarts still running (register copy of sm.run)
    for (int iter = 1; iter <= maxiter; ++iter) {
      TEAM_STAMP(0);
      // ---- this workgroup's partials of G = W^T A (wave w: samples 16w..) and W^T W (wave w: genes 16w..) ----
      d4 gacc = (d4){0.0, 0.0, 0.0, 0.0}, sacc = (d4){0.0, 0.0, 0.0, 0.0};
      if (w < NJ && !(SKIP & 2)) {
#pragma unroll
        for (int s = 0; s < 16; ++s) gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(wg[s], ag[s], gacc, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < ((SKIP & 2) ? 0 : 4); ++s) {
        const double v = wg[4 * w + s];
        sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, sacc, 0, 0, 0);
      }
      ++epoch;
      const unsigned tag = tag_base + epoch;
      const int buf = epoch & 1;
      double* const gxb = gx + (long)buf * TEAM_PMAX * 16 * NP;
      double* const swb = swx + (long)buf * TEAM_PMAX * 256;
      if (w < NJ) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (lr + 4 * r < ncol) {
            if (SKIP & 1)
              sm.G[lr + 4 * r][16 * w + lc] = gacc[r];
            else
              st_sc1(gxb + ((long)p * 16 + lr + 4 * r) * NP + 16 * w + lc, gacc[r]);
          }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sm.SWw[w][lr + 4 * r][lc] = sacc[r];
      __syncthreads();
      TEAM_STAMP(1);
      const double sw_own = ((sm.SWw[0][sc][sd] + sm.SWw[1][sc][sd]) + sm.SWw[2][sc][sd]) + sm.SWw[3][sc][sd];
      if (sw_live && !(SKIP & 1)) st_sc1(swb + (long)p * 256 + tid, sw_own);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
      __syncthreads();
      if (tid == 0 && !(SKIP & 1)) __hip_atomic_store(fl + p, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      TEAM_STAMP(2);
      // ---- wait for the P flags (lane q of wave 0 polls flag q), then the team sums in workgroup order ----
      if (w == 0 && !(SKIP & 1)) {
        bool mine = l >= P, mine2 = l + 64 >= P;   // lane l polls flags l and l + 64
        for (long spins = 0;; ++spins) {
          if (!mine) mine = (int)(__hip_atomic_load(fl + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - tag) >= 0;
          if (!mine2) mine2 = (int)(__hip_atomic_load(fl + l + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - tag) >= 0;
          if (__all(mine && mine2)) break;
          if (spins > TEAM_SPIN_MAX) {
            if (l == 0) {
              sm.abort = 1;
              __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      TEAM_STAMP(3);
      if (sm.abort) break;
      if (!(SKIP & 1)) {
        if (w < NJ) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = lr + 4 * r;
            if (4 * r >= ncol) break;   // wave-uniform: no lane holds a live row from here on
            const double v = team_sum(gxb + (long)c * NP + 16 * w + lc, 16L * NP, P);
            if (c < ncol) sm.G[c][16 * w + lc] = v;
          }
        }
        double v = 0.0;
        if (sw_live) v = team_sum(swb + tid, 256, P);
        sm.SW[sc][sd] = v;
      } else {
        sm.SW[sc][sd] = sw_live ? sw_own : 0.0;
      }
      if (tid < SMALL_MAXR) sm.changed[tid] = 0;
      __syncthreads();
      TEAM_STAMP(4);
      if (sm.abort) break;
      // ---- H update (nmf_mu.c:178, 184-191): d summed over the restart's columns in order ----
      double hn[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int q = he_q[u];
        hn[u] = 0.0;
        if (q >= 0 && ((runmask >> q) & 1)) {
          const int c = he_c[u], j = he_j[u], b0 = he_b0[u];
          double dsum = 0.0;
          for (int bb = 0; bb < he_k[u]; ++bb) dsum = fma(sm.SW[c][b0 + bb], sm.H[b0 + bb][j], dsum);
          hn[u] = mu_rule(sm.H[c][j], sm.G[c][j], dsum);
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < HU; ++u)
        if (he_q[u] >= 0 && ((runmask >> he_q[u]) & 1)) sm.H[he_c[u]][he_j[u]] = hn[u];
      __syncthreads();
      TEAM_STAMP(5);
      // ---- h h^T (wave 0, MFMA over the samples); the stop rule (nmf_mu.c:253-282) on waves 1-3 ----
      const bool check = stop_rule != STOP_FIXED && iter > 1 && (iter % 2 == 0);
      if (w == 0) {
        double hv[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) hv[q] = sm.H[lc][4 * q + lr];
        __builtin_amdgcn_sched_barrier(0);
        d4 hh = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < ((SKIP & 4) ? 0 : NQ); ++q) hh = __builtin_amdgcn_mfma_f64_16x16x4f64(hv[q], hv[q], hh, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = lr + 4 * r;
          const int qc = sm.colr[c];
          sm.S[c][lc] = (qc >= 0 && qc == sm.colr[lc]) ? hh[r] : 0.0;
        }
      } else if (check && !(SKIP & 16)) {
        if (stop_rule == STOP_REF_COMPAT) {
          // window i of restart q reads the flat k x n column-major buffer at [i*n, i*n + k)
          for (int x = tid - 64; x < nr * 16; x += 192) {
            const int q = x >> 4, i = x & 15, kq = blk.k[q];
            if (i >= kq || i >= n || !((runmask >> q) & 1)) continue;
            int cl = 0;
            double prev = 0.0;
            for (int jj = 0; jj < kq; ++jj) {
              const int f = i * n + jj, j = f / kq, a = f - j * kq;
              const double v = sm.H[blk.lc0[q] + a][j];
              if (jj > 0 && v > prev) cl = jj;
              prev = v;
            }
            if (sm.cls[q][i] != cl) {
              sm.cls[q][i] = cl;
              sm.changed[q] = 1;
            }
          }
        } else if (stop_rule == STOP_ARGMAX_STABLE) {
          for (int x = tid - 64; x < nr * 64; x += 192) {
            const int q = x >> 6, j = x & 63;
            if (j >= n || !((runmask >> q) & 1)) continue;
            int best = 0;
            double bv = sm.H[blk.lc0[q]][j];
            for (int a = 1; a < blk.k[q]; ++a) {
              const double v = sm.H[blk.lc0[q] + a][j];
              if (v > bv) {
                bv = v;
                best = a;
              }
            }
            if (sm.cls[q][j] != best) {
              sm.cls[q][j] = best;
              sm.changed[q] = 1;
            }
          }
        }
      }
      __syncthreads();
      TEAM_STAMP(6);
      // ---- F^T = h A^T, E^T = (h h^T) W0^T, W rule (nmf_mu.c:198-216) on this wave's 16 genes ----
      {
        d4 f = (d4){0.0, 0.0, 0.0, 0.0}, e = (d4){0.0, 0.0, 0.0, 0.0};
        double hv[NQ], sv[4];   // every LDS operand read before the MFMA chains (one LDS latency, not one per step)
#pragma unroll
        for (int t = 0; t < NQ; ++t) hv[t] = sm.H[lc][4 * t + lr];
#pragma unroll
        for (int q = 0; q < 4; ++q) sv[q] = sm.S[lc][4 * q + lr];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < ((SKIP & 8) ? 0 : 4); ++q) e = __builtin_amdgcn_mfma_f64_16x16x4f64(sv[q], wd[q], e, 0, 0, 0);
#pragma unroll
        for (int t = 0; t < ((SKIP & 8) ? 0 : NQ); ++t) f = __builtin_amdgcn_mfma_f64_16x16x4f64(hv[t], af[t], f, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (wq[r] >= 0 && ((runmask >> wq[r]) & 1)) wd[r] = mu_rule(wd[r], f[r], e[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sm.Wt[16 * w + lc][lr + 4 * r] = wd[r];
      // ---- stop bookkeeping (wave 0, lane q = restart q; identical in every workgroup of the team) ----
      if (w == 0) {
        bool alive = false;
        if (l < nr && ((runmask >> l) & 1)) {
          int reason = 0;
          if (check) {
            if (!sm.changed[l]) {
              const int u = sm.unch[l] + 1;
              sm.unch[l] = u;
              if (u >= 200) reason = 1;   // nmf_mu.c:269-271
            } else {
              sm.unch[l] = 0;
            }
          }
          if (!reason && iter >= maxiter) reason = 2;
          if (reason) {
            sm.run[l] = 0;
            if (p == 0) {
              stop_iter[blk.rid[l]] = iter;
              stop_reason[blk.rid[l]] = reason;
            }
          } else {
            alive = true;
          }
        }
        const u64 am = __ballot(alive);
        if (l == 0) sm.nrun = (int)__popcll(am);
      }
      __syncthreads();   // every wave has applied its W rule under this iteration's run flags
      TEAM_STAMP(7);
#pragma unroll
      for (int s = 0; s < 16; ++s) wg[s] = sm.Wt[4 * s + lr][lc];
      if (sm.nrun == 0) break;
      int rm = 0;
#pragma unroll
      for (int q = 0; q < SMALL_MAXR; ++q) rm |= (q < nr && sm.run[q]) ? (1 << q) : 0;
      runmask = rm;
      TEAM_STAMP(8);
    }
    if (sm.abort) break;
    // ---- final factors of the block back to the stacked layout ----
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (lr + 4 * r < ncol) W[(long)(blk.col0 + lr + 4 * r) * m_pad + g0 + 16 * w + lc] = wd[r];
    if (p == 0)
      for (int x = tid; x < 16 * NP; x += 256) {
        const int c = x / NP, j = x % NP;
        if (c < ncol && j < n) H[(long)(blk.col0 + c) * n_pad + j] = sm.H[c][j];
      }
  }
  if ((SKIP & 64) && p == 0 && tid == 0 && prof)
    for (int i = 0; i < 9; ++i) prof[i] = prof_acc[i];
#undef TEAM_STAMP
}

// ---------------------------------------------------------------------------------------------
// Repacking (compaction of live restarts) and the final-factor archive: k rows per job.
// ---------------------------------------------------------------------------------------------
struct MoveJob {
  int src_row;
  int dst_row;
  int k;
};

static __global__ __launch_bounds__(NT) void k_move_rows(const MoveJob* __restrict__ jobs, const double* __restrict__ src,
                                                         long src_ld, double* __restrict__ dst, long dst_ld, long len) {
  const MoveJob jb = jobs[blockIdx.x];
  for (int a = 0; a < jb.k; ++a) {
    const double* s = src + (long)(jb.src_row + a) * src_ld;
    double* d = dst + (long)(jb.dst_row + a) * dst_ld;
    for (long x = (long)blockIdx.y * NT + threadIdx.x; x < len; x += (long)gridDim.y * NT) d[x] = s[x];
  }
}

// ---------------------------------------------------------------------------------------------
// Init: generateMatrix(ran) (generatematrix.c:131-137) with randnumber (randnumber.c:34) over the
// glibc TYPE_3 stream seeded per job.  Thread = (restart, chunk of 31 * rnb draws); the chunk's start
// state is J[c] * s_344 (mod 2^32), J[c] = M^(c * 31 * rnb) the 31x31 jump matrix of the lagged
// recurrence r[i] = r[i-31] + r[i-3].  The host picks rnb per run: long chunks (few jump products) when the
// sweep has draws enough to fill the GPU, short ones when it has not (C1's 73 000 draws were 74 threads).
// ---------------------------------------------------------------------------------------------
constexpr int RCHUNK = 31 * 32;   // longest chunk: draws per thread (a multiple of 31: a statically indexed ring)

struct InitJob {
  uint32_t seed;
  int col0;
  int k;
  int nchunks;
};

static __global__ __launch_bounds__(NT) void k_init(const InitJob* __restrict__ jobs, const int* __restrict__ chunk_job,
                                                    const int* __restrict__ chunk_idx, int total_chunks,
                                                    const uint32_t* __restrict__ jump, int rnb, int m, int n, long m_pad,
                                                    long n_pad, int min_init, int max_init, double* __restrict__ W,
                                                    double* __restrict__ H) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total_chunks) return;
  const InitJob jb = jobs[chunk_job[gid]];
  const int c = chunk_idx[gid];
  // srand(seed): r[0..30] by the Park-Miller LCG (Schrage), r[31..33] = r[0..2]
  uint32_t ring[31];
  int32_t word = (int32_t)(jb.seed ? jb.seed : 1u);
  ring[0] = (uint32_t)word;
#pragma unroll
  for (int i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long wv = 16807 * lo - 2836 * hi;
    if (wv < 0) wv += 2147483647;
    word = (int32_t)wv;
    ring[i] = (uint32_t)word;
  }
  // ring[q] holds r[q]; r[31..33] = r[0..2] occupy the same slots.  Steps i = 34..343 (10 x 31).
#pragma unroll 1
  for (int blk = 0; blk < 10; ++blk) {
#pragma unroll
    for (int q = 0; q < 31; ++q) {
      const int pos = (3 + q) % 31;
      ring[pos] = ring[pos] + ring[(pos + 28) % 31];
    }
  }
  // ordered window s[q] = r[313 + q] sits at ring[(3 + q) % 31]
  uint32_t s[31];
#pragma unroll
  for (int q = 0; q < 31; ++q) s[q] = ring[(3 + q) % 31];
  if (c > 0) {
    const uint32_t* J = jump + (long)c * 31 * 31;
#pragma unroll
    for (int q = 0; q < 31; ++q) {
      uint32_t v = 0;
#pragma unroll
      for (int pq = 0; pq < 31; ++pq) v += J[q * 31 + pq] * s[pq];
      ring[q] = v;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 31; ++q) ring[q] = s[q];
  }
  // ring[q] = r[i0 - 31 + q]; step jj overwrites slot jj % 31 with r[i0+jj] = slot + slot[(jj+28)%31].
  // Draw t goes to W (column-major m x k: row i, column a) while t < m k, then to H (k x n: row a, column jcol);
  // both positions advance incrementally (one division per thread, not two 64-bit divisions per draw).
  const int mk = m * jb.k;
  const int total = mk + jb.k * n;
  int t = c * 31 * rnb;
  int p0, p1;   // (i, a) in W, then (a, jcol) in H
  if (t < mk) {
    p1 = t / m;
    p0 = t - p1 * m;
  } else {
    p1 = (t - mk) / jb.k;
    p0 = (t - mk) - p1 * jb.k;
  }
#pragma unroll 1
  for (int blk = 0; blk < rnb; ++blk) {
#pragma unroll
    for (int q = 0; q < 31; ++q) {
      const uint32_t v = ring[q] + ring[(q + 28) % 31];
      ring[q] = v;
      if (t < total) {
        const int32_t o = (int32_t)(v >> 1);
        const int32_t prod = (int32_t)((uint32_t)(max_init - min_init) * (uint32_t)o);
        const double val = (double)min_init + (double)prod / 2147483647.0;
        if (t < mk) {
          W[(long)(jb.col0 + p1) * m_pad + p0] = val;
          if (++p0 == m) {
            p0 = 0;
            if (++p1 == jb.k) p1 = 0;   // t + 1 == mk: H starts at (a, jcol) = (0, 0)
          }
        } else {
          H[(long)(jb.col0 + p0) * n_pad + p1] = val;
          if (++p0 == jb.k) {
            p0 = 0;
            ++p1;
          }
        }
      }
      ++t;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Init, R path (nmf.r:37-38): the BatchJobs job seed s = seed + job_id - 1, then set.seed(s);
// W <- runif(m*k) (column-major m x k); H <- runif(k*n) (column-major k x n).  One workgroup per
// restart walks R's Mersenne-Twister stream (rmt.hpp) 624 draws at a time.
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_init_runif(const InitJob* __restrict__ jobs, int m, int n, long m_pad,
                                                          long n_pad, double* __restrict__ W, double* __restrict__ H) {
  __shared__ uint32_t mt[624];
  const InitJob jb = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  if (tid == 0) rmt::seed_table(mt, jb.seed);
  __syncthreads();
  const long mk = (long)m * jb.k, total = mk + (long)jb.k * n;
  for (long base = 0; base < total; base += 624) {
    rmt::regenerate<NT>(mt);
    for (int t = tid; t < 624; t += NT) {
      const long d = base + t;
      if (d >= total) break;
      const double u = rmt::unif(mt[t]);
      if (d < mk) {
        const long a = d / m, i = d - a * m;
        W[(long)(jb.col0 + a) * m_pad + i] = u;
      } else {
        const long tt = d - mk, jcol = tt / jb.k, a = tt - jcol * jb.k;
        H[(long)(jb.col0 + a) * n_pad + jcol] = u;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// STOP_TOLX, after the W update of an even iteration > 1 (nmf_als.c:304-349 applied to MU): one
// workgroup per live restart: dw = calculateMaxchange(W, W0) from the pre-update snapshot W0,
// delta = max(dh, dw) with dh from k_hupdate; stop if delta < TolX, or if TolFun >= 1 (the test
// dnorm <= TolFun * dnorm0 runs after dnorm0 = dnorm, nmf_als.c:330/:345, so it only fires then --
// or on an exactly-zero residual, which is not evaluated here).
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_wstat(int iter, const RestartInfo* __restrict__ ri,
                                                     const double* __restrict__ W, const double* __restrict__ W0,
                                                     long m_pad, int m, const int* __restrict__ colact,
                                                     const double* __restrict__ Hstat, double TolX, double TolFun,
                                                     int* __restrict__ stop_iter, int* __restrict__ stop_reason,
                                                     int* __restrict__ n_stopped) {
  __shared__ unsigned long long dmax, omax;
  const RestartInfo me = ri[blockIdx.x];
  if (stop_iter[me.rid] != 0 || colact[me.col0] != iter) return;   // stopped, or no W update this iteration
  if (threadIdx.x == 0) {
    dmax = 0ull;
    omax = 0ull;
  }
  __syncthreads();
  double tdm = 0.0, tom = 0.0;
  for (int a = 0; a < me.k; ++a) {
    const double* w = W + (long)(me.col0 + a) * m_pad;
    const double* w0 = W0 + (long)(me.col0 + a) * m_pad;
    for (int i = threadIdx.x; i < m; i += NT) {
      const double o = w0[i];
      tdm = fmax(tdm, fabs(o - w[i]));
      tom = fmax(tom, fabs(o));
    }
  }
  atomicMax(&dmax, (unsigned long long)__double_as_longlong(tdm));
  atomicMax(&omax, (unsigned long long)__double_as_longlong(tom));
  __syncthreads();
  if (threadIdx.x == 0) {
    const double dw = __longlong_as_double((long long)dmax) / (SQRTEPS + __longlong_as_double((long long)omax));
    const double dh = Hstat[me.rid];
    const double delta = dh > dw ? dh : dw;
    if (delta < TolX || TolFun >= 1.0) {
      stop_iter[me.rid] = iter;
      stop_reason[me.rid] = 3;
      atomicAdd(n_stopped, 1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Labels (nmf.r:128 / documented intent) and connectivity counts (nmf.r:140-141).
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(NT) void k_labels(const RestartInfo* __restrict__ ri, const int* __restrict__ slot,
                                                      const double* __restrict__ H, long n_pad, int n, int rule,
                                                      int32_t* __restrict__ labels) {
  const int r = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int c0 = ri[r].col0, k = ri[r].k;
  int best = 0;
  double bv = H[(long)c0 * n_pad + j];
  for (int a = 1; a < k; ++a) {
    const double v = H[(long)(c0 + a) * n_pad + j];
    if (rule == 0 ? (v > bv) : (v < bv)) {
      bv = v;
      best = a;
    }
  }
  labels[(long)slot[r] * n + j] = best + 1;
}

// counts[g][i + j*n] = sum over the group's restarts of [L[i] == L[j]] (nmf.r:140-141).  A workgroup owns a
// 64 x 64 block of (i, j); the two 64-label strips of CR restarts at a time are staged in LDS (each label
// read once per block) and every thread accumulates a 4 x 4 register block of exact integer counts.
constexpr int CNT_T = 64, CNT_R = 32;
static __global__ __launch_bounds__(NT) void k_counts(const int32_t* __restrict__ labels,
                                                      const int* __restrict__ grp_begin,
                                                      const int* __restrict__ grp_list, int n,
                                                      int32_t* __restrict__ counts) {
  __shared__ int32_t li[CNT_R][CNT_T], lj[CNT_R][CNT_T];
  const int gidx = blockIdx.z;
  const int i0 = blockIdx.x * CNT_T, j0 = blockIdx.y * CNT_T;
  const int tid = threadIdx.x, ti = (tid & 15) * 4, tj = (tid >> 4) * 4;
  const int b = grp_begin[gidx], e = grp_begin[gidx + 1];
  int32_t cnt[4][4] = {};
  for (int q0 = b; q0 < e; q0 += CNT_R) {
    const int nr = min(CNT_R, e - q0);
    for (int x = tid; x < nr * CNT_T; x += NT) {
      const int r = x / CNT_T, c = x % CNT_T;
      const int32_t* L = labels + (long)grp_list[q0 + r] * n;
      li[r][c] = (i0 + c < n) ? L[i0 + c] : -1;
      lj[r][c] = (j0 + c < n) ? L[j0 + c] : -2;
    }
    __syncthreads();
    for (int r = 0; r < nr; ++r) {
      int32_t a[4], bb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = li[r][ti + u];
        bb[u] = lj[r][tj + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) cnt[u][v] += (a[u] == bb[v]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int j = j0 + tj + v;
    if (j >= n) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + ti + u;
      if (i < n) counts[(long)gidx * n * n + (long)j * n + i] = cnt[u][v];
    }
  }
}

static __global__ void k_divide(const int32_t* __restrict__ counts, double denom, long len, double* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < len) out[i] = (double)counts[i] / denom;
}

// A (m x n, ld lda) -> Acm (column j at j*m_pad, zero padded) and Arm (row i at i*n_pad)
static __global__ void k_layout_a(const double* __restrict__ A, long lda, int m, int n, long m_pad, long n_pad,
                                  double* __restrict__ Acm, double* __restrict__ Arm) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (i >= m) return;
  const double v = A[(long)j * lda + i];
  if (Acm) Acm[(long)j * m_pad + i] = v;
  Arm[i * n_pad + j] = v;
}

// A -> Ablk, the K-blocked operand of W^T A: Ablk[(i / 16) * ld * 16 + j * 16 + i % 16] (ld = n_cols_pad rows),
// so the 16-gene block of a tile's sample rows is one contiguous run.  Block (x, y): NT genes x the 16
// sample columns 16 y ..; lanes run along the genes of one column (16 doubles = 128 B contiguous).
static __global__ __launch_bounds__(NT) void k_layout_ablk(const double* __restrict__ A, long lda, int m, int n, long ld,
                                                           double* __restrict__ Ablk) {
  const long i = (long)blockIdx.x * NT + threadIdx.x;   // gene
  if (i >= m) return;
  const long kb = i >> 4, r = i & 15;
#pragma unroll 4
  for (int jj = 0; jj < 16; ++jj) {
    const int j = 16 * blockIdx.y + jj;
    if (j < n) Ablk[kb * ld * 16 + (long)j * 16 + r] = A[(long)j * lda + i];
  }
}

// ---------------------------------------------------------------------------------------------
// calculateNorm (calculatenorm.c:44-78) and calculateMaxchange (calculatemaxchange.c:42-71)
// ---------------------------------------------------------------------------------------------
// grid (x: gene blocks of NT, y: column groups); block (x, y) covers genes x*NT.. of columns y, y + gridDim.y, ...
static __global__ __launch_bounds__(NT) void k_norm_partial(const double* __restrict__ a, const double* __restrict__ w,
                                                            const double* __restrict__ h, double* __restrict__ d, int m,
                                                            int n, int k, double* __restrict__ partial) {
  __shared__ double red[NT];
  const int i = blockIdx.x * NT + threadIdx.x;
  double ss = 0.0;
  if (i < m) {
    for (int j = blockIdx.y; j < n; j += gridDim.y) {
      const long idx = (long)j * m + i;
      double s = 0.0;
      for (int q = 0; q < k; ++q) s = fma(w[i + (long)q * m], h[q + (long)j * k], s);
      const double v = a[idx] - s;
      d[idx] = v;
      ss = fma(v, v, ss);
    }
  }
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

// The same pass for rank K <= 16 known at compile time: the thread's row of W is loaded once into
// registers, the column of H is wave-uniform (scalar loads), and 4 columns are in flight per step, so the
// pass streams A in and d out at HBM rate instead of re-reading W per element.  Per element the sum over
// q runs in q order with fma, as k_norm_partial (identical d); the per-block partial of v^2 likewise.
template <int K>
static __global__ __launch_bounds__(NT) void k_norm_partial_k(const double* __restrict__ a, const double* __restrict__ w,
                                                              const double* __restrict__ h, double* __restrict__ d, int m,
                                                              int n, double* __restrict__ partial) {
  __shared__ double red[NT];
  const int i = blockIdx.x * NT + threadIdx.x;
  double ss = 0.0;
  if (i < m) {
    double wr[K];
#pragma unroll
    for (int q = 0; q < K; ++q) wr[q] = w[i + (long)q * m];
    constexpr int U = 4;
    int j = blockIdx.y;
    for (; j + (U - 1) * (int)gridDim.y < n; j += U * gridDim.y) {
      double av[U], sv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) av[u] = a[(long)(j + u * gridDim.y) * m + i];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double* hc = h + (long)(j + u * gridDim.y) * K;
        double sacc = 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) sacc = fma(wr[q], hc[q], sacc);
        sv[u] = sacc;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double v = av[u] - sv[u];
        d[(long)(j + u * gridDim.y) * m + i] = v;
        ss = fma(v, v, ss);
      }
    }
    for (; j < n; j += gridDim.y) {
      const double* hc = h + (long)j * K;
      double sacc = 0.0;
#pragma unroll
      for (int q = 0; q < K; ++q) sacc = fma(wr[q], hc[q], sacc);
      const double v = a[(long)j * m + i] - sacc;
      d[(long)j * m + i] = v;
      ss = fma(v, v, ss);
    }
  }
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

static __global__ __launch_bounds__(NT) void k_maxchange_partial(const double* __restrict__ mat,
                                                                 double* __restrict__ mat0, long len,
                                                                 double* __restrict__ partial) {
  __shared__ double r0[NT], r1[NT];
  double mx0 = 0.0, mxd = 0.0;
  for (long idx = (long)blockIdx.x * NT + threadIdx.x; idx < len; idx += (long)gridDim.x * NT) {
    const double v0 = mat0[idx];
    mx0 = fmax(mx0, fabs(v0));
    const double dv = v0 - mat[idx];
    mat0[idx] = dv;
    mxd = fmax(mxd, fabs(dv));
  }
  r0[threadIdx.x] = mx0;
  r1[threadIdx.x] = mxd;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      r0[threadIdx.x] = fmax(r0[threadIdx.x], r0[threadIdx.x + off]);
      r1[threadIdx.x] = fmax(r1[threadIdx.x], r1[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = r0[0];
    partial[2 * blockIdx.x + 1] = r1[0];
  }
}

}  // namespace nmfc
