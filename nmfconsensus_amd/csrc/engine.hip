// engine.hip -- host side of the batched MU restart engine (C ABI in include/nmfc.h).
//
// Replaces the reference's restart driver (nmf.r:53-70, 106-113), its per-job nmf_mu loop
// (libnmf/nmf_mu.c:167-293) and the consensus reduction (nmf.r:121-144) with one batched sweep on
// one MI355X: all (k, restart) jobs of a shard are packed into 64-column panels of a stacked W/H,
// and every MU iteration is three launches on one HIP stream:
//   k_wta2    G = W^T A                                          (fp64 MFMA, fixed gene chunks)
//   k_wta2    also the restart-diagonal blocks of W^T W (nmf_mu.c:176) from the same staged W
//   k_hupdate W^T W from the chunk partials, H update, H H^T, stability check (one workgroup per restart)
//   k_ahtw4   A h^T fused with W0 (h h^T) and the W update (fp64 MFMA)
// Restarts that stop are archived and the live ones repacked into fewer panels as the sweep goes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/nmfc.h"
#include "nmfc_kernels.hpp"

using namespace nmfc;

// solo.hip: the batched one-workgroup-per-restart kernel for rank <= 4 on gct-sized shapes
int nmfc_solo_batch_rank(int n, int k);
int nmfc_solo_batch_launch(const double* Acm, long a_ld, int m, int n, double* W, long w_ld, double* H, long h_ld,
                           const nmfc::SoloJob* djobs, int njobs, int kp, int maxiter, int stop_rule, int* stop_iter,
                           int* stop_reason, int max_wgs, hipStream_t st);

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

#define HCHECK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return -1;                                                                            \
    }                                                                                       \
  } while (0)

long round_up(long v, long a) { return (v + a - 1) / a * a; }

// Device buffer, released on destruction (every early return frees what it allocated).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  int ensure(size_t need) {
    if (need <= bytes) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (need == 0) return 0;
    hipError_t e = hipMalloc(&p, need);
    if (e != hipSuccess) {
      set_err("hipMalloc(%zu) failed: %s", need, hipGetErrorString(e));
      p = nullptr;
      return -1;
    }
    bytes = need;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// 31x31 jump matrices J[c] = M^(c * rchunk) mod 2^32 of the recurrence r[i] = r[i-31] + r[i-3]
// acting on the ordered window (r[i-31], ..., r[i-1]).
void mat_mul31(const uint32_t* A, const uint32_t* B, uint32_t* C) {
  for (int i = 0; i < 31; ++i)
    for (int j = 0; j < 31; ++j) {
      uint32_t s = 0;
      for (int q = 0; q < 31; ++q) s += A[i * 31 + q] * B[q * 31 + j];
      C[i * 31 + j] = s;
    }
}

std::vector<uint32_t> make_jump_table(int nchunks, int rchunk) {
  std::vector<uint32_t> M(31 * 31, 0), P(31 * 31, 0), T(31 * 31);
  for (int q = 0; q < 30; ++q) M[q * 31 + q + 1] = 1;
  M[30 * 31 + 0] = 1;    // r[i-31]
  M[30 * 31 + 28] += 1;  // r[i-3]
  for (int i = 0; i < 31; ++i) P[i * 31 + i] = 1;
  std::vector<uint32_t> base = M;
  for (int e = rchunk; e > 0; e >>= 1) {   // P = M^rchunk
    if (e & 1) {
      mat_mul31(P.data(), base.data(), T.data());
      P = T;
    }
    mat_mul31(base.data(), base.data(), T.data());
    base = T;
  }
  std::vector<uint32_t> table((size_t)std::max(nchunks, 1) * 961, 0);
  for (int i = 0; i < 31; ++i) table[i * 31 + i] = 1;
  for (int c = 1; c < nchunks; ++c) mat_mul31(P.data(), &table[(size_t)(c - 1) * 961], &table[(size_t)c * 961]);
  return table;
}

enum { KID_WTA = 0, KID_HUPD = 1, KID_AHTW = 2, KID_INIT = 3, KID_OTHER = 4, KID_LABELS = 5, KID_COUNTS = 6, KID_SMALL = 7, KID_N = 8 };

// Packing of a restart list: first-fit decreasing (k descending, ties by rid) into 16-column blocks -- a restart
// never straddles a block -- and blocks, in order, four to a 64-column panel; panel count rounded up to a
// multiple of WTA_NPT (the large W^T A tile spans that many panels).  Against packing whole 64-column panels
// (rounds 1-2) this costs ~1 % more columns (R = 200: 682 blocks for 675 blocks' worth of columns) and removes
// every 16 x 16 block a restart shares with another: W^T A forms only the 4 diagonal Gram blocks per panel (not
// 4 + 3 straddling ones), A h^T's E = W0 (h h^T) runs 4 K steps per 16-row block (not up to 12), and the narrow
// tail kernels apply as soon as the live restarts fit their blocks.  Placement never changes a result bit
// (DESIGN.md "Determinism").
constexpr int WTA_NPT = 4;
constexpr int NARROW_NBUF = NMFC_NARROW_NBUF;      // LDS ring depth of the narrow (tail) W^T A kernel (16: +2 % on the R = 25 shard)
constexpr bool WTA_MID_GREG = NMFC_WTA_MID_GREG != 0;   // 2-panel W^T A tile: 2 x 4 waves, Gram chains in registers
constexpr bool SMALL_NW8 = NMFC_SMALL_NW8 != 0;    // k_small_mu with eight waves where m_pad % 256 == 0
constexpr bool WTA_GREG = NMFC_WTA_GREG != 0;      // 4-panel W^T A tiles: diagonal Gram blocks from the tile's W registers
constexpr bool WTA_W16 = NMFC_WTA_W16 != 0 && WTA_GREG;   // the 4-panel x 128-sample W^T A tile on 16 waves (4 per SIMD)
constexpr int WTA_MID_NBUF = NMFC_WTA_MID_NBUF;    // ring depth of the 2-panel W^T A tile
constexpr int WTA_MID_MINW = NMFC_WTA_MID_MINW;    // its launch-bounds waves per SIMD (4: two workgroups per CU)
constexpr int AHTW_NBUF = NMFC_AHTW_NBUF;          // LDS ring depth of the full-width A h^T tiles
constexpr bool AHTW_LATE = NMFC_AHTW_LATE != 0;    // h h^T rows / W0 staged after the K loop (k_ahtw4 LATE)
struct Packing {
  std::vector<RestartInfo> ri;   // active list, panel-contiguous
  std::vector<int> prb, pre;     // per panel: [begin, end) in ri
  std::vector<ColInfo> ci;       // per panel column
  int npanels = 0;
};

Packing pack(const std::vector<RestartInfo>& in) {
  std::vector<RestartInfo> srt(in);
  std::stable_sort(srt.begin(), srt.end(), [](const RestartInfo& a, const RestartInfo& b) {
    return a.k != b.k ? a.k > b.k : a.rid < b.rid;
  });
  std::vector<int> fill;
  std::vector<std::vector<RestartInfo>> members;
  size_t first_open = 0;   // blocks before it have fewer than 2 free columns (k >= 2)
  for (RestartInfo r : srt) {
    size_t b = first_open;
    while (b < fill.size() && fill[b] + r.k > 16) ++b;
    if (b == fill.size()) {
      fill.push_back(0);
      members.emplace_back();
    }
    r.col0 = (int)b * 16 + fill[b];
    fill[b] += r.k;
    members[b].push_back(r);
    while (first_open < fill.size() && fill[first_open] > 14) ++first_open;
  }
  const int nblocks = (int)members.size();
  Packing pk;
  pk.npanels = std::max(1, (nblocks + 3) / 4);
  for (int p = 0; p < pk.npanels; ++p) {   // a panel = 4 consecutive blocks
    pk.prb.push_back((int)pk.ri.size());
    for (int b = 4 * p; b < std::min(nblocks, 4 * p + 4); ++b)
      for (const RestartInfo& r : members[b]) pk.ri.push_back(r);
    pk.pre.push_back((int)pk.ri.size());
  }
  while (pk.npanels % WTA_NPT) {
    pk.prb.push_back((int)in.size());
    pk.pre.push_back((int)in.size());
    ++pk.npanels;
  }
  pk.ci.assign((size_t)pk.npanels * PANEL, ColInfo{0, 0, 0, 0});
  for (const RestartInfo& r : pk.ri)
    for (int a = 0; a < r.k; ++a) pk.ci[r.col0 + a] = ColInfo{r.sq_off, r.col0 % PANEL, r.k, r.rid};
  return pk;
}

// Narrow (end-of-sweep) form: every restart of the packing inside one 16-column block, all of them in the
// first nb <= maxb blocks -> nb (the narrow kernels run only those blocks); otherwise 0.
int narrow_blocks(const Packing& pk, int maxb) {
  if (pk.ri.empty()) return 0;
  int nb = 0;
  for (const RestartInfo& r : pk.ri) {
    if (r.col0 / 16 != (r.col0 + r.k - 1) / 16) return 0;
    nb = std::max(nb, (r.col0 + r.k + 15) / 16);
  }
  return nb <= maxb ? nb : 0;
}

// Small-shape path (k_small_mu): restarts packed first-fit decreasing into 16-column blocks (a restart never
// straddles a block, at most SMALL_MAXR per block); the Packing's panels only size the stacked buffers.
Packing pack_small(const std::vector<RestartInfo>& in, std::vector<SmallBlock>& blocks) {
  std::vector<RestartInfo> srt(in);
  std::stable_sort(srt.begin(), srt.end(), [](const RestartInfo& a, const RestartInfo& b) {
    return a.k != b.k ? a.k > b.k : a.rid < b.rid;
  });
  std::vector<int> fill;
  blocks.clear();
  Packing pk;
  for (RestartInfo r : srt) {
    size_t b = 0;
    while (b < fill.size() && (fill[b] + r.k > 16 || blocks[b].nr == SMALL_MAXR)) ++b;
    if (b == fill.size()) {
      fill.push_back(0);
      SmallBlock sb{};
      sb.col0 = (int)b * 16;
      blocks.push_back(sb);
    }
    SmallBlock& sb = blocks[b];
    r.col0 = sb.col0 + fill[b];
    sb.rid[sb.nr] = r.rid;
    sb.k[sb.nr] = r.k;
    sb.lc0[sb.nr] = fill[b];
    ++sb.nr;
    fill[b] += r.k;
    pk.ri.push_back(r);
  }
  pk.npanels = std::max(1, (int)((blocks.size() * 16 + PANEL - 1) / PANEL));
  while (pk.npanels % WTA_NPT) ++pk.npanels;
  pk.prb.assign(pk.npanels, 0);
  pk.pre.assign(pk.npanels, 0);
  pk.ci.assign((size_t)pk.npanels * PANEL, ColInfo{0, 0, 0, 0});
  return pk;
}

// panels holding at least one restart (the packing fills panels from 0; the rest pad the 4-panel groups)
int live_panels(const Packing& pk) {
  int np = 0;
  for (int p = 0; p < pk.npanels; ++p)
    if (pk.pre[p] > pk.prb[p]) np = p + 1;
  return np;
}

// Small-shape path, restarts that the one-workgroup solo kernels take (nmfc_mu_solo_fits(m, n, k): rank <= 8 on
// gct-sized shapes): each gets 4 (kernel rank <= 4) or 8 stacked columns of its own after the k_small_mu blocks
// (cols from col_base), highest kernel rank first, then rank descending, then restart id: the order the fused
// launch starts them in (costliest first).  Returns the solo jobs; pk grows to hold them.
std::vector<SoloJob> place_solo(Packing& pk, std::vector<RestartInfo> solo, int col_base, int n) {
  // costliest kernel rank first, and within it the higher ranks (k_solo8_mu takes k = 5..8 at one cost per
  // iteration, and higher ranks run longer on average): the dispatcher, which starts the workgroups in order, then
  // starts the likely stragglers first
  std::stable_sort(solo.begin(), solo.end(), [n](const RestartInfo& a, const RestartInfo& b) {
    const int ka = nmfc_solo_batch_rank(n, a.k), kb = nmfc_solo_batch_rank(n, b.k);
    return ka != kb ? ka > kb : a.k != b.k ? a.k > b.k : a.rid < b.rid;
  });
  std::vector<SoloJob> jobs;
  int col = col_base;
  for (RestartInfo r : solo) {
    r.col0 = col;
    col += nmfc_solo_batch_rank(n, r.k) <= 4 ? 4 : 8;
    pk.ri.push_back(r);
    jobs.push_back(SoloJob{r.col0, r.k, r.rid, 0});
  }
  pk.npanels = std::max(pk.npanels, (col + PANEL - 1) / PANEL);
  while (pk.npanels % WTA_NPT) ++pk.npanels;
  pk.prb.assign(pk.npanels, 0);
  pk.pre.assign(pk.npanels, 0);
  pk.ci.assign((size_t)pk.npanels * PANEL, ColInfo{0, 0, 0, 0});
  return jobs;
}

}  // namespace

// error slot shared with the other translation units of the library (brunet.hip)
__attribute__((visibility("hidden"))) void nmfc_set_error(const char* msg) { g_err = msg; }

struct nmfc_engine {
  int dev = 0;
  hipStream_t st = nullptr;
  int m = 0, n = 0;
  long m_pad = 0, n_pad = 0, n_cols_pad = 0;
  int kchunk = 0, nsplit = 0, ngt = 0;
  int ncu = 256;   // compute units (grid-size heuristics only)
  int force_wta = -1, force_ahtw = -1;   // tile-shape overrides (env NMFC_WTA_TILE / NMFC_AHTW_TILE)
  int repack_div = 20;                    // repack after nact / repack_div stops (env NMFC_REPACK_DIV; 5 / 10 / 20 / 40
                                          // measured 437.7 / 441.2 / 446.0 / 445.7 restarts/s on C3)
  bool narrow_ok = true;                  // narrow end-of-sweep kernels allowed (env NMFC_NARROW=0 disables)
  int narrow_maxb = 3;                    // narrow form up to this many 16-column blocks (env NMFC_NARROW_MAXB)
  bool small_ok = true;                   // small-shape persistent kernel allowed (env NMFC_SMALL=0 disables)
  int small_kernel = 0;                   // batched small shapes: 0/2 one workgroup per block (k_small_mu), 1 teams
                                          // (k_team_mu); env NMFC_SMALL_KERNEL=team|single (single also keeps
                                          // nmf_mu off the team path)
  DevBuf Acm, Arm, Ablk;   // Acm: small-shape kernel only; Ablk: K-blocked A for W^T A (see k_layout_a)
  // per-run buffers (grow-only)
  DevBuf W[2], H[2], Gpart, SWpart, SH, SHP, colact, Hfin, Wfin;
  DevBuf rinfo, stop_iter, stop_reason, unchanged, classes, n_stopped, Hstat, Wsnap;
  DevBuf prb, pre, colinfo, moves, finfo;
  DevBuf initjobs, chunk_job, chunk_idx, jump, labels, slot, grp_begin, grp_list, counts_tmp, cons_tmp, smallblk;
  DevBuf teamG, teamSW, teamFlag;   // k_team_mu: partial buffers, per-workgroup flags (+ the error word)
  DevBuf solojobs;                  // batched k_solo_mu jobs (small shapes, rank <= 4)
  bool narrow_lc = true;            // env NMFC_NARROW_LC=0: the one-wave narrow W^T A kernel
  bool wta_sk = true;               // env NMFC_WTA_SK=0: the big W^T A tile one item per workgroup (no stream-K)
  bool wta_sk_mid = true;           // env NMFC_WTA_SK_MID=0: the same for the 2-panel tile
  bool wta_lastsum = false;         // env NMFC_WTA_LASTSUM=1: k_wta2_sk sums each tile's chunk partials (probe arm)
  int sk_dp_xcd = 0;                // env NMFC_SK_DP_XCD=1: k_wta2_sk's whole rounds in XCD-contiguous blocks (probe)
  DevBuf skfix, skflag, sktcnt;     // k_wta2_sk: per-range hand-off slots and flags (zeroed once), per-tile tickets
  unsigned sk_epoch = 0;            // k_wta2_sk launches so far (the flag value of the current launch)
  bool gram_model = true;           // env NMFC_GRAM_MODEL=0: the tile cost model without the Gram workgroups
  bool solo_ok = true;              // env NMFC_SOLO=0: no solo kernel (every small-shape restart in k_small_mu blocks)
  hipStream_t aux[4] = {nullptr, nullptr, nullptr, nullptr};   // the solo launches (one per kernel rank: 2, 3, 4, 8)
  hipEvent_t fork_ev = nullptr, join_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  int team_occ = 0;                // resident k_team_mu workgroups per CU (occupancy query, once)
  // nmfc_engine_mu1 (one restart, the nmf_mu drop-in): device and pinned staging [block | stop | W | H],
  // its own partial buffers and flags (zeroed when allocated; tags continue from mu1_base, the iterations of
  // earlier calls)
  DevBuf mu1_dev, mu1_G, mu1_SW, mu1_flag;
  char* mu1_host = nullptr;
  size_t mu1_host_bytes = 0;
  int mu1_base = -1;   // -1: the flags must be zeroed
  int mu1_kprev = 16;  // staging rows [k, mu1_kprev) may hold a previous call's factors
  int jump_chunks = 0, jump_rchunk = 0;   // the jump table on the device: chunks, draws per chunk
  int* h_stopped = nullptr;   // pinned, 2 slots
  // timing
  bool timing = false;
  int timing_stride = 1;            // time the launches of every timing_stride-th MU iteration
  std::vector<hipEvent_t> ev_pool;
  struct Pending {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  double kms[KID_N] = {0};
  long long kcount[KID_N] = {0};    // timed launches (event pairs drained)
  long long klaunch[KID_N] = {0};   // every launch
  double kflops[KID_N] = {0};
  double kbytes[KID_N] = {0};       // bytes the kernel's design moves per launch (operands + partials)
  double kbytes_algo[KID_N] = {0};  // algorithmic bytes per launch (each operand once)
  int repacks = 0;
};

namespace {

// Tile shapes for one chunk of iterations, from a wave-quantised cost model: a shape's time is
// ceil(workgroups / resident slots) x its relative per-workgroup time.  Slots per CU and relative
// per-workgroup times (2048-gene chunk, 128 samples of W^T A) were measured on MI355X with
// tools/tailbench.hip over 1..172 live panels of the C3 shape (profiles/r02/tailbench_*.txt):
//   big  4 panels x 128 samples, 8 waves, 144 KiB   1 / CU   2.0
//   mid  2 panels x 128 samples, 8 waves,  96 KiB   1 / CU   1.0
//   small 1 panel x  64 samples, 4 waves,  48 KiB   3 / CU   0.8
//   tiny 1 panel x  32 samples, 4 waves,  36 KiB   4 / CU   0.6
// Ties go to the larger tile.  A h^T uses 64-gene tiles only on small grids (below).  Every shape accumulates in the canonical K order, so this never changes a bit.
struct TileChoice {
  int wta;          // 0 big, 3 mid, 1 small, 2 tiny
  bool ahtw_small;  // 64-gene A h^T tiles
};

// The stream-K big tile (k_wta2_sk): 16-wave GREG tiles (ntj >= 4), NMFC_WTA_SK not 0.  Its cost per round of items
// against the one-item-per-workgroup kernel's (hand-offs, per-piece prologues; tools/kvar.hip: 3.34 vs 3.51 ms at the
// C3 full-load grid of 6.72 rounds, i.e. ~1 % above the ideal 6.72 / 7 of the unsplit form's time)
constexpr double WTA_SK_COST = 1.01;
bool sk_big_ok(const nmfc_engine* e, int ntj) { return e->wta_sk && WTA_W16 && ntj >= 4; }
// the 2-panel tile's stream-K form (k_wta2_sk<..., 2>): its 8-wave register-Gram instantiation (ntj >= 4)
bool sk_mid_ok(const nmfc_engine* e, int ntj) { return e->wta_sk && e->wta_sk_mid && WTA_MID_GREG && ntj >= 4; }
// ... and the grid condition of either: at least one whole round of items, and every workgroup's even share of the
// stages at least one item long (so an item is cut into at most two pieces: k_wta2_sk's contract)
bool sk_grid_fits(const nmfc_engine* e, long ngroups, int ntj) {
  const long ipc = ngroups * ntj, nitems = ipc * e->nsplit;
  const long nst_full = e->kchunk / 16, nst_last = (e->m_pad - (long)(e->nsplit - 1) * e->kchunk) / 16;
  const long nst_max = e->nsplit > 1 ? nst_full : nst_last;
  const long S = ipc * (e->nsplit - 1) * nst_full + ipc * nst_last;
  return nitems >= e->ncu && S >= (long)e->ncu * nst_max;
}

TileChoice choose_tiles(const nmfc_engine* e, int np_live, int ntj) {
  const long ns = e->nsplit, cu = e->ncu;
  const long np = std::max(np_live, 1);
  // The 1-panel shapes launch 3 Gram workgroups per (chunk, panel) beside their tiles (GITEM): one 512-MFMA chain
  // per wave, about a quarter of a 1 x 64 tile's work and half of a 1 x 32 tile's, counted as such (round 4: without
  // them the model chose 1 x 64 tiles at 9..12 live panels, 295 us per launch on the R = 25 shard against 275 for
  // 2-panel tiles, and 1 x 32 tiles at 6, 191 us against ~165; profiles/r04/shard2_wta_shapes.txt).
  struct Cand {
    int id;
    double wgs;
    long slots;
    double t;
  } cands[4] = {{0, (double)(ns * ((np + 3) / 4) * ntj), cu, 2.0},
                {3, (double)(ns * ((np + 1) / 2) * ntj), cu, 1.0},
                {1, (double)(ns * np) * (2 * ntj + (e->gram_model ? 0.75 : 0.0)), 3 * cu, 0.8},
                {2, (double)(ns * np) * (4 * ntj + (e->gram_model ? 1.5 : 0.0)), 4 * cu, 0.6}};
  TileChoice tc{0, false};
  double best = 1e300;
  for (const Cand& c : cands) {
    // the big and 2-panel tiles in their stream-K form (k_wta2_sk, from one whole round of items on) take wgs / slots
    // rounds, not ceil(wgs / slots): the last round's items are split over every CU
    const bool sk = (c.id == 0 && sk_big_ok(e, ntj) && sk_grid_fits(e, (np + 3) / 4, ntj)) ||
                    (c.id == 3 && sk_mid_ok(e, ntj) && sk_grid_fits(e, (np + 1) / 2, ntj));
    const double est = sk ? c.wgs / (double)c.slots * c.t * WTA_SK_COST : std::ceil(c.wgs / (double)c.slots) * c.t;
    if (est < best - 1e-9) {
      best = est;
      tc.wta = c.id;
    }
  }
  // 64-gene A h^T tiles (5 workgroups / CU) beat the 128-gene ones (3 / CU) only on grids of a few
  // thousand tiles: R = 25 shard +3 %, R = 50 tied, R >= 100 128 genes ahead (tools/gpu_var_bench.sh)
  tc.ahtw_small = np * e->ngt < 16 * cu;
  if (e->force_wta >= 0) tc.wta = e->force_wta;   // NMFC_WTA_TILE (tests: every shape gives the same bits)
  if (e->force_ahtw >= 0) tc.ahtw_small = e->force_ahtw == 1;
  return tc;
}

// k_small_mu<GBW, JB, 0, NW> for this engine's shape (GBW = m_pad / (16 NW) gene blocks per wave, JB = sample blocks)
template <int GBW, int NW>
hipError_t launch_small_g(nmfc_engine* e, int nblocks, int maxiter, int stop_rule) {
  const int jb = (e->n + 15) / 16;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nblocks), dim3(64 * NW), 0, e->st, e->smallblk.as<SmallBlock>(),
                       e->Arm.as<double>(), e->n_pad, e->Acm.as<double>(), e->m_pad, e->n, e->n_pad,
                       e->W[0].as<double>(), e->H[0].as<double>(), maxiter, stop_rule, e->stop_iter.as<int>(),
                       e->stop_reason.as<int>());
  };
  switch (jb) {
    case 1: args(k_small_mu<GBW, 1, 0, NW>); break;
    case 2: args(k_small_mu<GBW, 2, 0, NW>); break;
    case 3: args(k_small_mu<GBW, 3, 0, NW>); break;
    default: args(k_small_mu<GBW, 4, 0, NW>); break;
  }
  return hipGetLastError();
}

// k_team_mu: teams of P = m_pad / 64 workgroups, as many teams as are resident at once (each team runs its
// blocks one after another); partial buffers two per team, flags and the error word zeroed per launch, tags from 1.
int team_count(nmfc_engine* e, int nblocks) {
  const int P = (int)(e->m_pad / TEAM_ROWS);
  if (!e->team_occ) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_team_mu<4>, 256, 0) != hipSuccess || occ < 1) occ = 1;
    // teams must be co-resident (their workgroups wait for each other); the API's answer can overstate
    // residency where SGPRs bind: at ~106 SGPRs at most 6 256-thread workgroups fit a CU (MI355X_MICROARCH.md,
    // residency).  A team that still cannot meet ends with an error, it does not hang.
    e->team_occ = std::min(occ, 6);
  }
  return std::max(1, std::min(nblocks, (int)((long)e->team_occ * e->ncu / P)));
}

int launch_team(nmfc_engine* e, int nblocks, int maxiter, int stop_rule) {
  const int jb = (e->n + 15) / 16;
  const int P = (int)(e->m_pad / TEAM_ROWS);
  if (e->m_pad % TEAM_ROWS != 0 || P > TEAM_PMAX || jb < 1 || jb > 4) {
    set_err("k_team_mu: m_pad %ld / n %d unsupported", e->m_pad, e->n);
    return -1;
  }
  auto kern = jb == 1 ? k_team_mu<1> : jb == 2 ? k_team_mu<2> : jb == 3 ? k_team_mu<3> : k_team_mu<4>;
  const int nteams = team_count(e, nblocks);
  const long np = 16L * jb;
  if (e->teamG.ensure(sizeof(double) * nteams * 2 * TEAM_PMAX * 16 * np) ||
      e->teamSW.ensure(sizeof(double) * nteams * 2 * TEAM_PMAX * 256) ||
      e->teamFlag.ensure(sizeof(unsigned) * (nteams * TEAM_PMAX + 16)))
    return -1;
  // flags zeroed per launch (tags start at 1); the error word sits behind them
  HCHECK(hipMemsetAsync(e->teamFlag.p, 0, sizeof(unsigned) * (nteams * TEAM_PMAX + 16), e->st));
  hipLaunchKernelGGL(kern, dim3(nteams * P), dim3(256), 0, e->st, e->smallblk.as<SmallBlock>(), nblocks, P,
                     e->Acm.as<double>(), e->m_pad, e->n, e->n_pad, e->W[0].as<double>(), e->H[0].as<double>(), maxiter,
                     stop_rule, e->stop_iter.as<int>(), e->stop_reason.as<int>(), e->teamG.as<double>(),
                     e->teamSW.as<double>(), e->teamFlag.as<unsigned>(), 0u,
                     reinterpret_cast<int*>(e->teamFlag.as<unsigned>() + nteams * TEAM_PMAX), nullptr);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_err("k_team_mu launch: %s", hipGetErrorString(err));
    return -1;
  }
  return 0;
}

// 1 if a k_team_mu launch reported a team that could not meet (bounded wait), after the stream is drained
int team_failed(nmfc_engine* e, int nblocks) {
  int v = 0;
  const unsigned* w = e->teamFlag.as<unsigned>() + team_count(e, nblocks) * TEAM_PMAX;
  if (hipMemcpy(&v, w, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  return v != 0;
}

// Kernel for a batch of small-shape blocks: the one-workgroup k_small_mu, whatever the batch size, so a job
// gives the same bits in any batch and on any number of GPUs (the consensus is then bit-identical at any GPU
// count).  Teams (k_team_mu) serve the single-restart nmf_mu drop-in (nmfc_engine_mu1): a team runs a block's
// iteration in ~7 us against ~25 us, but only team_count() teams are resident (one 256-VGPR workgroup per CU)
// and a team runs its blocks one after another, so on C2's 219 blocks they are 2.5x slower
// (profiles/r03/team/c2_kernels.txt).  NMFC_SMALL_KERNEL=team forces teams for batches too (tests).
bool use_team(nmfc_engine* e, int nblocks) {
  (void)nblocks;
  return e->small_kernel == 1;
}

int launch_small(nmfc_engine* e, int nblocks, int maxiter, int stop_rule) {
  if (use_team(e, nblocks)) return launch_team(e, nblocks, maxiter, stop_rule);
  hipError_t err;
  const int jb = (e->n + 15) / 16;
  if (e->m_pad % 64 != 0 || e->n_pad != (jb <= 2 ? 32 : 64)) {   // k_small_mu's compile-time strides
    set_err("k_small_mu: m_pad %ld / n_pad %ld unsupported for n = %d", e->m_pad, e->n_pad, e->n);
    return -1;
  }
  // eight waves where the genes split into an even number of 16-gene blocks per wave (m_pad a multiple of 256),
  // else four: a function of (m, n) only, so a job's bits stay independent of its batch
  if (SMALL_NW8 && e->m_pad % 256 == 0) {
    switch (e->m_pad / 128) {
      case 2: err = launch_small_g<2, 8>(e, nblocks, maxiter, stop_rule); break;
      case 4: err = launch_small_g<4, 8>(e, nblocks, maxiter, stop_rule); break;
      case 6: err = launch_small_g<6, 8>(e, nblocks, maxiter, stop_rule); break;
      case 8: err = launch_small_g<8, 8>(e, nblocks, maxiter, stop_rule); break;
      default: set_err("k_small_mu: m_pad %ld unsupported", e->m_pad); return -1;
    }
  } else {
    switch (e->m_pad / 64) {
      case 2: err = launch_small_g<2, 4>(e, nblocks, maxiter, stop_rule); break;
      case 4: err = launch_small_g<4, 4>(e, nblocks, maxiter, stop_rule); break;
      case 6: err = launch_small_g<6, 4>(e, nblocks, maxiter, stop_rule); break;
      case 8: err = launch_small_g<8, 4>(e, nblocks, maxiter, stop_rule); break;
      case 10: err = launch_small_g<10, 4>(e, nblocks, maxiter, stop_rule); break;
      case 12: err = launch_small_g<12, 4>(e, nblocks, maxiter, stop_rule); break;
      case 14: err = launch_small_g<14, 4>(e, nblocks, maxiter, stop_rule); break;
      case 16: err = launch_small_g<16, 4>(e, nblocks, maxiter, stop_rule); break;
      default: set_err("k_small_mu: m_pad %ld unsupported", e->m_pad); return -1;
    }
  }
  if (err != hipSuccess) {
    set_err("k_small_mu launch: %s", hipGetErrorString(err));
    return -1;
  }
  return 0;
}

hipEvent_t take_event(nmfc_engine* e) {
  if (!e->ev_pool.empty()) {
    hipEvent_t ev = e->ev_pool.back();
    e->ev_pool.pop_back();
    return ev;
  }
  hipEvent_t ev;
  if (hipEventCreate(&ev) != hipSuccess) return nullptr;
  return ev;
}

void drain_timing(nmfc_engine* e) {
  for (auto& pnd : e->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(pnd.b) == hipSuccess && hipEventElapsedTime(&ms, pnd.a, pnd.b) == hipSuccess) {
      e->kms[pnd.kid] += ms;
      e->kcount[pnd.kid] += 1;
    }
    e->ev_pool.push_back(pnd.a);
    e->ev_pool.push_back(pnd.b);
  }
  e->pending.clear();
}

// HIP events on the engine's stream around one launch (only when timing is enabled)
struct TimedLaunch {
  nmfc_engine* e;
  int kid;
  hipEvent_t a = nullptr;
  // sample = false: counted, not timed (the MU loop times every timing_stride-th iteration)
  TimedLaunch(nmfc_engine* e_, int kid_, bool sample = true) : e(e_), kid(kid_) {
    e->klaunch[kid] += 1;
    if (e->timing && sample) {
      a = take_event(e);
      if (a) (void)hipEventRecord(a, e->st);
    }
  }
  ~TimedLaunch() {
    if (a) {
      hipEvent_t b = take_event(e);
      if (b) {
        (void)hipEventRecord(b, e->st);
        e->pending.push_back({kid, a, b});
      } else {
        e->ev_pool.push_back(a);
      }
    }
  }
};

}  // namespace

extern "C" {

const char* nmfc_last_error(void) { return g_err.c_str(); }

const char* nmfc_build_tuning(void) { return NMFC_TUNING_MU; }
const char* nmfc_version(void) { return "nmfconsensus_amd 0.2 (gfx950, fp64 MFMA)"; }

void nmfc_default_opts(nmfc_sweep_opts* o) {
  memset(o, 0, sizeof *o);
  o->maxiter = 10000;                 // nmf.r:13, test_nmf.r:27
  o->stop_rule = NMFC_STOP_REF_COMPAT;
  o->label_rule = NMFC_LABEL_ARGMAX;
  o->seed = 123;                      // nmf.r:13
  o->min_init = 0;                    // setdefaultopts.c:42-43
  o->max_init = 1;
  o->job_begin = 0;
  o->job_end = -1;
  o->check_every = 4;   // C3: 16 -> 4 gives 437 -> 453 restarts/s (earlier repacks, less dead work)
  o->verbose = 0;
  o->TolX = 1.0E-04;                  // setdefaultopts.c (options_t.TolX / TolFun)
  o->TolFun = 1.0E-04;
}

nmfc_engine* nmfc_engine_create(int device, const double* A, int m, int n, int a_on_device) {
  if (!A || m <= 0 || n <= 0) {
    set_err("nmfc_engine_create: bad arguments (A=%p m=%d n=%d)", (const void*)A, m, n);
    return nullptr;
  }
  nmfc_engine* e = new nmfc_engine();
  auto fail = [&](const char* what, hipError_t err) -> nmfc_engine* {
    set_err("nmfc_engine_create: %s: %s", what, hipGetErrorString(err));
    nmfc_engine_destroy(e);
    return nullptr;
  };
  hipError_t err;
  if (device >= 0) {
    if ((err = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", err);
  }
  if ((err = hipGetDevice(&e->dev)) != hipSuccess) return fail("hipGetDevice", err);
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->dev) == hipSuccess && ncu > 0) e->ncu = ncu;
  }
  if (const char* s = getenv("NMFC_WTA_TILE")) {
    const std::string v(s);
    e->force_wta = v == "big" ? 0 : v == "small" ? 1 : v == "tiny" ? 2 : v == "mid" ? 3 : -1;
  }
  if (const char* s = getenv("NMFC_REPACK_DIV")) e->repack_div = std::max(1, atoi(s));
  if (const char* s = getenv("NMFC_NARROW")) e->narrow_ok = atoi(s) != 0;
  if (const char* s = getenv("NMFC_NARROW_MAXB")) e->narrow_maxb = std::min(8, std::max(1, atoi(s)));
  if (const char* s = getenv("NMFC_SMALL")) e->small_ok = atoi(s) != 0;
  if (const char* s = getenv("NMFC_SOLO")) e->solo_ok = atoi(s) != 0;
  if (const char* s = getenv("NMFC_NARROW_LC")) e->narrow_lc = atoi(s) != 0;
  if (const char* s = getenv("NMFC_WTA_SK")) e->wta_sk = atoi(s) != 0;
  if (const char* s = getenv("NMFC_WTA_SK_MID")) e->wta_sk_mid = atoi(s) != 0;
  if (const char* s = getenv("NMFC_WTA_LASTSUM")) e->wta_lastsum = atoi(s) != 0;
  if (const char* s = getenv("NMFC_SK_DP_XCD")) e->sk_dp_xcd = atoi(s) != 0;
  if (const char* s = getenv("NMFC_GRAM_MODEL")) e->gram_model = atoi(s) != 0;
  if (const char* s = getenv("NMFC_SMALL_KERNEL"))
    e->small_kernel = std::string(s) == "team" ? 1 : std::string(s) == "single" ? 2 : 0;
  if (const char* s = getenv("NMFC_AHTW_TILE")) {
    const std::string v(s);
    e->force_ahtw = v == "128" ? 0 : v == "64" ? 1 : -1;
  }
  if ((err = hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", err);
  if ((err = hipHostMalloc((void**)&e->h_stopped, 2 * sizeof(int), 0)) != hipSuccess) return fail("hipHostMalloc", err);
  e->m = m;
  e->n = n;
  e->m_pad = round_up(m, GT);          // gene tiles of A h^T and Gram partials
  e->n_pad = round_up(n, BK);          // K of A h^T
  e->n_cols_pad = round_up(n, 128);    // sample tiles of W^T A
  e->ngt = (int)(e->m_pad / GT);
  // fixed gene chunks of W^T A: a function of m only, so every entry's summation order is batch-independent
  int kchunk = 2048;   // canonical split-K chunk; NMFC_KCHUNK (512 | 1024 | 2048 | 4096) is a probe knob
  if (const char* v = getenv("NMFC_KCHUNK")) {
    const int x = atoi(v);
    if (x == 512 || x == 1024 || x == 2048 || x == 4096) kchunk = x;
  }
  e->kchunk = (int)std::min<long>(kchunk, e->m_pad);
  e->nsplit = (int)((e->m_pad + e->kchunk - 1) / e->kchunk);
  // Acm (column-major, padded) feeds only the small-shape kernel; the general path's W^T A reads the K-blocked Ablk
  // the column-major copy feeds the small-shape kernels: k_small_mu (m_pad <= 1024) and the team kernel
  // behind nmfc_engine_mu1 (m_pad <= TEAM_ROWS * TEAM_PMAX = 8192)
  const bool small_shape = e->m_pad <= (long)TEAM_ROWS * TEAM_PMAX && n <= 64;
  if ((small_shape && e->Acm.ensure(sizeof(double) * e->n_cols_pad * e->m_pad)) ||
      e->Ablk.ensure(sizeof(double) * e->n_cols_pad * e->m_pad) || e->Arm.ensure(sizeof(double) * e->m_pad * e->n_pad)) {
    nmfc_engine_destroy(e);
    return nullptr;
  }
  if (small_shape && (err = hipMemsetAsync(e->Acm.p, 0, e->Acm.bytes, e->st)) != hipSuccess) return fail("memset", err);
  if ((err = hipMemsetAsync(e->Ablk.p, 0, e->Ablk.bytes, e->st)) != hipSuccess) return fail("memset", err);
  if ((err = hipMemsetAsync(e->Arm.p, 0, e->Arm.bytes, e->st)) != hipSuccess) return fail("memset", err);
  const double* dA = A;
  DevBuf tmp;
  if (!a_on_device) {
    if (tmp.ensure(sizeof(double) * (size_t)m * n)) {
      nmfc_engine_destroy(e);
      return nullptr;
    }
    if ((err = hipMemcpyAsync(tmp.p, A, sizeof(double) * (size_t)m * n, hipMemcpyHostToDevice, e->st)) != hipSuccess)
      return fail("upload A", err);
    dA = tmp.as<double>();
  }
  dim3 grid((m + NT - 1) / NT, n);
  hipLaunchKernelGGL(k_layout_a, grid, dim3(NT), 0, e->st, dA, (long)m, m, n, e->m_pad, e->n_pad,
                     small_shape ? e->Acm.as<double>() : nullptr, e->Arm.as<double>());
  hipLaunchKernelGGL(k_layout_ablk, dim3((unsigned)((m + NT - 1) / NT), (unsigned)((n + 15) / 16)), dim3(NT), 0,
                     e->st, dA, (long)m, m, n, e->n_cols_pad, e->Ablk.as<double>());
  if ((err = hipGetLastError()) != hipSuccess) return fail("k_layout_a", err);
  if ((err = hipStreamSynchronize(e->st)) != hipSuccess) return fail("sync", err);
  tmp.release();
  return e;
}

void nmfc_engine_destroy(nmfc_engine* e) {
  if (!e) return;
  if (e->st) (void)hipStreamSynchronize(e->st);
  drain_timing(e);
  for (auto ev : e->ev_pool) (void)hipEventDestroy(ev);
  DevBuf* bufs[] = {&e->Acm,       &e->Arm,       &e->Ablk,      &e->W[0],      &e->W[1],     &e->H[0],       &e->H[1],
                    &e->Gpart,     &e->SWpart,    &e->SH,        &e->SHP,      &e->colact,     &e->Hfin,
                    &e->Wfin,      &e->rinfo,
                    &e->stop_iter, &e->stop_reason, &e->unchanged, &e->classes, &e->n_stopped, &e->prb,
                    &e->pre,       &e->colinfo,   &e->moves,     &e->finfo,     &e->initjobs, &e->chunk_job,  &e->chunk_idx,
                    &e->jump,      &e->labels,    &e->slot,      &e->grp_begin, &e->grp_list,  &e->counts_tmp,
                    &e->cons_tmp,  &e->Hstat,     &e->Wsnap,     &e->smallblk,  &e->teamG,    &e->teamSW,
                    &e->teamFlag,  &e->mu1_dev,   &e->mu1_G,     &e->mu1_SW,    &e->mu1_flag};
  for (DevBuf* b : bufs) b->release();
  e->solojobs.release();
  for (int q = 0; q < 4; ++q) {
    if (e->aux[q]) (void)hipStreamDestroy(e->aux[q]);
    if (e->join_ev[q]) (void)hipEventDestroy(e->join_ev[q]);
  }
  if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
  if (e->h_stopped) (void)hipHostFree(e->h_stopped);
  if (e->mu1_host) (void)hipHostFree(e->mu1_host);
  if (e->st) (void)hipStreamDestroy(e->st);
  delete e;
}

int nmfc_engine_device(const nmfc_engine* e) { return e ? e->dev : -1; }

int nmfc_current_device(void) {
  int d = -1;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}

void nmfc_engine_set_timing(nmfc_engine* e, int enable) {
  if (!e) return;
  e->timing = enable > 0;
  e->timing_stride = std::max(1, enable);
}

long long nmfc_engine_kernel_time(nmfc_engine* e, int kid, double* ms_out) {
  if (!e || kid < 0 || kid >= KID_N) return -1;
  if (ms_out) *ms_out = e->kms[kid];
  return e->kcount[kid];
}

double nmfc_engine_kernel_flops(nmfc_engine* e, int kid) {
  if (!e || kid < 0 || kid >= KID_N) return 0.0;
  return e->kflops[kid];
}

double nmfc_engine_kernel_bytes(nmfc_engine* e, int kid, double* algo_bytes_out) {
  if (!e || kid < 0 || kid >= KID_N) return 0.0;
  if (algo_bytes_out) *algo_bytes_out = e->kbytes_algo[kid];
  return e->kbytes[kid];
}

int nmfc_engine_run(nmfc_engine* e, const int* ks, int nk, int R, const nmfc_sweep_opts* opts_in,
                    const double* W_init, const double* H_init, nmfc_result* out) {
  if (!e || !ks || nk <= 0 || R <= 0) {
    set_err("nmfc_engine_run: bad arguments");
    return -1;
  }
  nmfc_sweep_opts opts;
  if (opts_in)
    opts = *opts_in;
  else
    nmfc_default_opts(&opts);
  if (opts.check_every <= 0) opts.check_every = 4;
  const int m = e->m, n = e->n;
  for (int q = 0; q < nk; ++q) {
    // nmf.r:107-108 rejects k = 1; the per-restart LDS blocks hold k <= KMAX.
    if (ks[q] < 2 || ks[q] > KMAX || ks[q] > n || ks[q] > m) {
      set_err("nmfc_engine_run: k=%d unsupported (need 2 <= k <= min(%d, m, n))", ks[q], KMAX);
      return -1;
    }
    // k_init walks a restart's m k + k n draws with 32-bit draw indices (one chunk of up to 31 x 32 past the end)
    if ((long)m * ks[q] + (long)ks[q] * n + 31L * 32 >= (long)INT_MAX) {
      set_err("nmfc_engine_run: m k + k n = %ld draws per restart exceeds the init kernel's 32-bit index range",
              (long)m * ks[q] + (long)ks[q] * n);
      return -1;
    }
  }
  if (opts.maxiter < 0) {
    set_err("nmfc_engine_run: maxiter must be >= 0");
    return -1;
  }
  if (opts.stop_rule < 0 || opts.stop_rule > 3 || opts.label_rule < 0 || opts.label_rule > 1 ||
      opts.init_stream < 0 || opts.init_stream > 1) {
    set_err("nmfc_engine_run: bad stop rule, label rule or init stream");
    return -1;
  }
  HCHECK(hipSetDevice(e->dev));
  auto t_start = std::chrono::steady_clock::now();
  for (int q = 0; q < KID_N; ++q) {
    e->kms[q] = 0;
    e->kcount[q] = 0;
    e->klaunch[q] = 0;
    e->kflops[q] = 0;
    e->kbytes[q] = 0;
    e->kbytes_algo[q] = 0;
  }
  e->repacks = 0;
  const long njobs_all = (long)nk * R;
  const long jb = std::max(0, opts.job_begin);
  const long je = (opts.job_end < 0) ? njobs_all : std::min<long>(opts.job_end, njobs_all);
  if (jb >= je) {
    set_err("nmfc_engine_run: empty job range [%ld, %ld)", jb, je);
    return -1;
  }
  const int nj = (int)(je - jb);
  auto job_k = [&](int s) { return ks[(jb + s) % nk]; };

  // ---- restart ids: shard jobs in k-descending order (packing order) ----
  std::vector<int> order(nj);
  for (int i = 0; i < nj; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return job_k(a) > job_k(b); });
  std::vector<RestartInfo> all(nj);
  std::vector<int> rslot(nj);          // rid -> shard job slot
  std::vector<int> hoff(nj + 1, 0);    // rid -> first archive row
  long sw_total = 0;
  for (int rid = 0; rid < nj; ++rid) {
    const int s = order[rid];
    all[rid].k = job_k(s);
    all[rid].rid = rid;
    all[rid].sq_off = (int)sw_total;
    all[rid].col0 = 0;
    rslot[rid] = s;
    sw_total += (long)all[rid].k * all[rid].k;
    hoff[rid + 1] = hoff[rid] + all[rid].k;
  }
  // small shapes: one persistent workgroup per 16-column block runs the whole loop (a function of m, n and
  // the stop rule only, so a job takes the same path -- and gives the same bits -- in any batch)
  const bool small = e->small_ok && e->m_pad <= 1024 && n <= 64 && opts.stop_rule != NMFC_STOP_TOLX;
  std::vector<SmallBlock> sblocks;
  // ... and there, a restart the solo kernels take (rank 2..8 on gct-sized shapes, nmfc_mu_solo_fits: k_solo_mu for
  // ranks 2..4, k_solo8_mu for 5..8) runs on one workgroup of its own, the others in k_small_mu blocks; the choice is a
  // function of (m, n, k) only, so a job gives the same bits in any batch and on any number of GPUs.  Through the
  // single-restart nmf_mu drop-in the bits are the same for ranks 2..4 only (the drop-in runs k_solo_mu there); it
  // runs ranks 5..8 on k_team_mu (faster for one restart), whose sums run in another order
  std::vector<RestartInfo> blk_jobs, solo_jobs;
  for (const RestartInfo& r : all) (small && e->solo_ok && nmfc_mu_solo_fits(m, n, r.k) ? solo_jobs : blk_jobs).push_back(r);
  Packing pk = small ? pack_small(blk_jobs, sblocks) : pack(all);
  std::vector<SoloJob> solo;
  if (small && !solo_jobs.empty()) solo = place_solo(pk, solo_jobs, (int)sblocks.size() * 16, n);
  const long cap_cols = (long)pk.npanels * PANEL;
  const int ntj = (int)(e->n_cols_pad / 128);
  const long g_ld = e->n_cols_pad;
  const long g_split = cap_cols * g_ld;
  const long cls_ld = std::max<long>(n, KMAX);
  const long fin_rows = hoff[nj];
  const bool want_w = out && out->W;

  // ---- device buffers ----
  if (e->W[0].ensure(sizeof(double) * cap_cols * e->m_pad) || e->H[0].ensure(sizeof(double) * cap_cols * e->n_pad) ||
      e->W[1].ensure(sizeof(double) * cap_cols * e->m_pad) || e->H[1].ensure(sizeof(double) * cap_cols * e->n_pad) ||
      e->Gpart.ensure(sizeof(double) * g_split * e->nsplit) || e->SWpart.ensure(sizeof(double) * sw_total * e->nsplit) ||
      e->SH.ensure(sizeof(double) * sw_total) || e->Hfin.ensure(sizeof(double) * fin_rows * e->n_pad) ||
      e->SHP.ensure(sizeof(double) * cap_cols * KMAX) || e->colact.ensure(sizeof(int) * cap_cols) ||
      (want_w && e->Wfin.ensure(sizeof(double) * fin_rows * e->m_pad)) || e->rinfo.ensure(sizeof(RestartInfo) * nj) ||
      e->finfo.ensure(sizeof(RestartInfo) * nj) || e->stop_iter.ensure(sizeof(int) * nj) ||
      e->stop_reason.ensure(sizeof(int) * nj) || e->unchanged.ensure(sizeof(int) * nj) ||
      e->classes.ensure(sizeof(int) * nj * cls_ld) || e->n_stopped.ensure(sizeof(int)) ||
      e->prb.ensure(sizeof(int) * pk.npanels) || e->pre.ensure(sizeof(int) * pk.npanels) ||
      e->colinfo.ensure(sizeof(ColInfo) * pk.npanels * PANEL) ||
      e->moves.ensure(sizeof(MoveJob) * nj) || e->labels.ensure(sizeof(int32_t) * (size_t)nj * n) ||
      e->slot.ensure(sizeof(int) * nj) || e->Hstat.ensure(sizeof(double) * nj))
    return -1;
  const bool tolx = opts.stop_rule == NMFC_STOP_TOLX;
  if (tolx && e->Wsnap.ensure(sizeof(double) * cap_cols * e->m_pad)) return -1;
  hipStream_t st = e->st;
  int cur = 0;
  auto upload_packing = [&](const Packing& p) -> int {
    HCHECK(hipMemcpyAsync(e->rinfo.p, p.ri.data(), sizeof(RestartInfo) * std::max<size_t>(p.ri.size(), 1),
                          hipMemcpyHostToDevice, st));
    HCHECK(hipMemcpyAsync(e->prb.p, p.prb.data(), sizeof(int) * p.npanels, hipMemcpyHostToDevice, st));
    HCHECK(hipMemcpyAsync(e->pre.p, p.pre.data(), sizeof(int) * p.npanels, hipMemcpyHostToDevice, st));
    HCHECK(hipMemcpyAsync(e->colinfo.p, p.ci.data(), sizeof(ColInfo) * p.ci.size(), hipMemcpyHostToDevice, st));
    return 0;
  };
  if (upload_packing(pk)) return -1;
  HCHECK(hipMemcpyAsync(e->slot.p, rslot.data(), sizeof(int) * nj, hipMemcpyHostToDevice, st));
  HCHECK(hipMemsetAsync(e->stop_iter.p, 0, sizeof(int) * nj, st));
  HCHECK(hipMemsetAsync(e->stop_reason.p, 0, sizeof(int) * nj, st));
  HCHECK(hipMemsetAsync(e->unchanged.p, 0, sizeof(int) * nj, st));
  HCHECK(hipMemsetAsync(e->classes.p, 0, sizeof(int) * nj * cls_ld, st));   // nmf_mu.c:132 zero start
  HCHECK(hipMemsetAsync(e->n_stopped.p, 0, sizeof(int), st));
  HCHECK(hipMemsetAsync(e->colact.p, 0, sizeof(int) * cap_cols, st));
  HCHECK(hipMemsetAsync(e->W[0].p, 0, sizeof(double) * cap_cols * e->m_pad, st));
  HCHECK(hipMemsetAsync(e->H[0].p, 0, sizeof(double) * cap_cols * e->n_pad, st));
  HCHECK(hipMemsetAsync(e->W[1].p, 0, sizeof(double) * cap_cols * e->m_pad, st));
  HCHECK(hipMemsetAsync(e->H[1].p, 0, sizeof(double) * cap_cols * e->n_pad, st));

  // ---- init ----
  if (W_init && H_init) {
    // caller-provided factors, shard-job-major: W_j (m x k), H_j (k x n)
    std::vector<long> woff(nj + 1, 0), ho(nj + 1, 0);
    for (int s = 0; s < nj; ++s) {
      woff[s + 1] = woff[s] + (long)m * job_k(s);
      ho[s + 1] = ho[s] + (long)job_k(s) * n;
    }
    std::vector<double> hrow;
    for (const RestartInfo& r : pk.ri) {
      const int s = rslot[r.rid], k = r.k;
      HCHECK(hipMemcpy2DAsync(e->W[0].as<double>() + (long)r.col0 * e->m_pad, sizeof(double) * e->m_pad,
                              W_init + woff[s], sizeof(double) * m, sizeof(double) * m, k, hipMemcpyHostToDevice, st));
      hrow.assign((size_t)k * n, 0.0);
      for (int j = 0; j < n; ++j)
        for (int a = 0; a < k; ++a) hrow[(size_t)a * n + j] = H_init[ho[s] + (long)j * k + a];
      HCHECK(hipMemcpy2DAsync(e->H[0].as<double>() + (long)r.col0 * e->n_pad, sizeof(double) * e->n_pad, hrow.data(),
                              sizeof(double) * n, sizeof(double) * n, k, hipMemcpyHostToDevice, st));
      HCHECK(hipStreamSynchronize(st));   // hrow is reused
    }
  } else if (opts.init_stream == NMFC_INIT_R_RUNIF) {
    // nmf.r:37-38 under the BatchJobs job seed (seed + job_id - 1)
    std::vector<InitJob> ij(nj);
    for (int q = 0; q < nj; ++q) {
      const RestartInfo& r = pk.ri[q];
      ij[q] = InitJob{(uint32_t)(opts.seed + (uint32_t)(jb + rslot[r.rid])), r.col0, r.k, 0};
    }
    if (e->initjobs.ensure(sizeof(InitJob) * nj)) return -1;
    HCHECK(hipMemcpyAsync(e->initjobs.p, ij.data(), sizeof(InitJob) * nj, hipMemcpyHostToDevice, st));
    {
      TimedLaunch tl(e, KID_INIT);
      hipLaunchKernelGGL(k_init_runif, dim3(nj), dim3(NT), 0, st, e->initjobs.as<InitJob>(), m, n, e->m_pad, e->n_pad,
                         e->W[0].as<double>(), e->H[0].as<double>());
    }
    HCHECK(hipGetLastError());
    HCHECK(hipStreamSynchronize(st));   // ij goes out of scope
  } else {
    std::vector<InitJob> ij(nj);
    std::vector<int> cj, ci;
    int maxch = 1;
    // draws per thread: halve the chunk (down to 62) while the sweep would run fewer than 65 536 threads -- the
    // draws of one chunk are a dependent sequence, and the jump product a thread starts with costs ~1 000 ops
    long draws = 0;
    for (int q = 0; q < nj; ++q) draws += (long)m * pk.ri[q].k + (long)pk.ri[q].k * n;
    int rchunk = RCHUNK;
    while (rchunk > 62 && draws / rchunk < 65536) rchunk /= 2;
    for (int q = 0; q < nj; ++q) {
      const RestartInfo& r = pk.ri[q];
      const long total = (long)m * r.k + (long)r.k * n;
      const int nch = (int)((total + rchunk - 1) / rchunk);
      ij[q].seed = (uint32_t)(opts.seed + (uint32_t)(jb + rslot[r.rid]));   // job seed = seed + job_id - 1
      ij[q].col0 = r.col0;
      ij[q].k = r.k;
      ij[q].nchunks = nch;
      maxch = std::max(maxch, nch);
      for (int c = 0; c < nch; ++c) {
        cj.push_back(q);
        ci.push_back(c);
      }
    }
    if (maxch > e->jump_chunks || rchunk != e->jump_rchunk) {
      std::vector<uint32_t> tab = make_jump_table(maxch, rchunk);
      if (e->jump.ensure(sizeof(uint32_t) * tab.size())) return -1;
      HCHECK(hipMemcpyAsync(e->jump.p, tab.data(), sizeof(uint32_t) * tab.size(), hipMemcpyHostToDevice, st));
      HCHECK(hipStreamSynchronize(st));
      e->jump_chunks = maxch;
      e->jump_rchunk = rchunk;
    }
    if (e->initjobs.ensure(sizeof(InitJob) * nj) || e->chunk_job.ensure(sizeof(int) * cj.size()) ||
        e->chunk_idx.ensure(sizeof(int) * ci.size()))
      return -1;
    HCHECK(hipMemcpyAsync(e->initjobs.p, ij.data(), sizeof(InitJob) * nj, hipMemcpyHostToDevice, st));
    HCHECK(hipMemcpyAsync(e->chunk_job.p, cj.data(), sizeof(int) * cj.size(), hipMemcpyHostToDevice, st));
    HCHECK(hipMemcpyAsync(e->chunk_idx.p, ci.data(), sizeof(int) * ci.size(), hipMemcpyHostToDevice, st));
    const int total_chunks = (int)cj.size();
    {
      TimedLaunch tl(e, KID_INIT);
      hipLaunchKernelGGL(k_init, dim3((total_chunks + NT - 1) / NT), dim3(NT), 0, st, e->initjobs.as<InitJob>(),
                         e->chunk_job.as<int>(), e->chunk_idx.as<int>(), total_chunks, e->jump.as<uint32_t>(), rchunk / 31,
                         m, n,
                         e->m_pad, e->n_pad, opts.min_init, opts.max_init, e->W[0].as<double>(), e->H[0].as<double>());
    }
    HCHECK(hipGetLastError());
    HCHECK(hipStreamSynchronize(st));   // host vectors cj/ci go out of scope
  }
  // archive rows of restarts (final H, and W when requested) from the current buffers
  std::vector<char> archived(nj, 0);
  auto archive = [&](const std::vector<RestartInfo>& list) -> int {
    if (list.empty()) return 0;
    std::vector<MoveJob> mv(list.size());
    for (size_t q = 0; q < list.size(); ++q) mv[q] = {list[q].col0, hoff[list[q].rid], list[q].k};
    HCHECK(hipMemcpyAsync(e->moves.p, mv.data(), sizeof(MoveJob) * mv.size(), hipMemcpyHostToDevice, st));
    {
      TimedLaunch tl(e, KID_OTHER);
      hipLaunchKernelGGL(k_move_rows, dim3((unsigned)mv.size(), 2), dim3(NT), 0, st, e->moves.as<MoveJob>(),
                         e->H[cur].as<double>(), e->n_pad, e->Hfin.as<double>(), e->n_pad, e->n_pad);
      if (want_w)
        hipLaunchKernelGGL(k_move_rows, dim3((unsigned)mv.size(), 16), dim3(NT), 0, st, e->moves.as<MoveJob>(),
                           e->W[cur].as<double>(), e->m_pad, e->Wfin.as<double>(), e->m_pad, e->m_pad);
    }
    HCHECK(hipGetLastError());
    HCHECK(hipStreamSynchronize(st));   // mv is a host temporary
    for (const RestartInfo& r : list) archived[r.rid] = 1;
    return 0;
  };

  // ---- iterate ----
  auto t_iter0 = std::chrono::steady_clock::now();
  int it = 0, q = 0, checked = 0;
  if (small) {
    if (!sblocks.empty()) {
      if (e->smallblk.ensure(sizeof(SmallBlock) * sblocks.size())) return -1;
      HCHECK(hipMemcpyAsync(e->smallblk.p, sblocks.data(), sizeof(SmallBlock) * sblocks.size(), hipMemcpyHostToDevice, st));
    }
    if (!solo.empty()) {
      if (e->solojobs.ensure(sizeof(SoloJob) * solo.size())) return -1;
      HCHECK(hipMemcpyAsync(e->solojobs.p, solo.data(), sizeof(SoloJob) * solo.size(), hipMemcpyHostToDevice, st));
      for (int q = 0; q < 4; ++q) {
        if (!e->aux[q]) HCHECK(hipStreamCreateWithFlags(&e->aux[q], hipStreamNonBlocking));
        if (!e->join_ev[q]) HCHECK(hipEventCreateWithFlags(&e->join_ev[q], hipEventDisableTiming));
      }
      if (!e->fork_ev) HCHECK(hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming));
    }
    {
      TimedLaunch tl(e, KID_SMALL);   // the whole small-shape phase: k_small_mu blocks and the solo launches
      const bool team = use_team(e, (int)sblocks.size());
      // the fork point is recorded BEFORE the block kernel: an event recorded after it would hold the solo launches
      // until the block kernel had finished (round 4: C1 24.7 ms = 9.9 + 14.8 ms serialised)
      if (!solo.empty() && !team) HCHECK(hipEventRecord(e->fork_ev, st));
      if (!sblocks.empty() && launch_small(e, (int)sblocks.size(), opts.maxiter, opts.stop_rule)) return -1;
      if (!solo.empty()) {
        // after k_small_mu when teams run (a team's workgroups must all be resident at once: nothing else may hold CUs
        // then), else beside it on streams of their own, one launch per kernel rank, taking at most the CUs it leaves
        // free (one workgroup of either kernel fills a CU), shared in proportion to jobs x cost per iteration
        // (tools/solo_iter_time.py: rank 2 ~3.7 us, 3..4 ~5.1, 5..8 ~10.1), each workgroup running its share of jobs
        // one after another: the block kernel's workgroups never wait for a CU behind solo workgroups (the budget
        // assumes this engine is the only one on the device; restart groups -- several engines on one GPU -- are a
        // large-shape tool and would oversubscribe it here; a speed matter only, the bits do not depend on it)
        const bool alone = sblocks.empty() || team;
        if (alone) {
          // the batch's solo jobs have the GPU to themselves: ONE launch of every kernel rank, one workgroup per job
          // in list order -- the costliest ranks first -- on the main stream (per-rank launches on streams of their
          // own were serialised by the hardware queues they shared: C2's rank-2 launch began when the rank-4 one ended)
          if (nmfc_solo_batch_launch(e->Acm.as<double>(), e->m_pad, m, n, e->W[0].as<double>(), e->m_pad,
                                     e->H[0].as<double>(), e->n_pad, e->solojobs.as<SoloJob>(), (int)solo.size(), 0,
                                     opts.maxiter, opts.stop_rule, e->stop_iter.as<int>(), e->stop_reason.as<int>(),
                                     (int)solo.size(), st))
            return -1;
        } else {
          const long free_cu = std::max<long>(1, e->ncu - (long)sblocks.size());
          auto wt = [](int kp) -> long { return kp <= 2 ? 4 : kp <= 4 ? 6 : 12; };
          long wsum = 0;
          for (const SoloJob& jb : solo) wsum += wt(nmfc_solo_batch_rank(n, jb.k));
          std::vector<std::pair<size_t, size_t>> groups;   // [g0, g1) of one kernel rank, highest rank first
          for (size_t g0 = 0; g0 < solo.size();) {
            const int kp = nmfc_solo_batch_rank(n, solo[g0].k);
            size_t g1 = g0;
            while (g1 < solo.size() && nmfc_solo_batch_rank(n, solo[g1].k) == kp) ++g1;
            groups.emplace_back(g0, g1);
            g0 = g1;
          }
          for (int q = 0; q < (int)groups.size(); ++q) {
            const size_t g0 = groups[q].first, g1 = groups[q].second;
            const int kp = nmfc_solo_batch_rank(n, solo[g0].k);
            const long nq = (long)(g1 - g0);
            const long share = std::min<long>(nq, std::max<long>(1, free_cu * nq * wt(kp) / wsum));
            HCHECK(hipStreamWaitEvent(e->aux[q], e->fork_ev, 0));
            if (nmfc_solo_batch_launch(e->Acm.as<double>(), e->m_pad, m, n, e->W[0].as<double>(), e->m_pad,
                                       e->H[0].as<double>(), e->n_pad, e->solojobs.as<SoloJob>() + g0, (int)nq, kp,
                                       opts.maxiter, opts.stop_rule, e->stop_iter.as<int>(), e->stop_reason.as<int>(),
                                       (int)share, e->aux[q]))
              return -1;
            HCHECK(hipEventRecord(e->join_ev[q], e->aux[q]));
          }
          // the main stream joins after every launch is enqueued
          for (int q = 0; q < (int)groups.size(); ++q) HCHECK(hipStreamWaitEvent(st, e->join_ev[q], 0));
        }
      }
    }
    HCHECK(hipStreamSynchronize(st));
    if (!sblocks.empty() && use_team(e, (int)sblocks.size()) && team_failed(e, (int)sblocks.size())) {
      set_err("k_team_mu: a team of workgroups could not meet (not co-resident?)");
      return -1;
    }
    if (e->timing) drain_timing(e);
    it = opts.maxiter;   // every restart records its own stop iteration
  }
  int nact = nj;
  int stopped_at_pack = 0;
  struct PollEvents {   // destroyed on every exit path, including HCHECK returns
    hipEvent_t ev[2] = {nullptr, nullptr};
    ~PollEvents() {
      for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    }
  } pe;
  hipEvent_t* ev = pe.ev;
  HCHECK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
  HCHECK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  std::vector<int> si(nj);
  for (; !small;) {
    if (it < opts.maxiter) {
      const int chunk = std::min(opts.check_every, opts.maxiter - it);
      // tile shapes by grid size (a speed choice only: every shape sums in the canonical K order)
      const TileChoice tc = choose_tiles(e, live_panels(pk), ntj);
      bool wta_big = tc.wta == 0, wta_mid = tc.wta == 3, wta_tiny = tc.wta == 2;
      bool ahtw_small = tc.ahtw_small;
      // narrow (end-of-sweep) form: the restarts block-packed into the first nblk 16-column blocks
      const int nblk = e->narrow_ok ? narrow_blocks(pk, e->narrow_maxb) : 0;
      const bool narrow = nblk > 0;
      const int ngt_ahtw = e->ngt * (ahtw_small ? 2 : 1);
      // panels holding restarts: the empty panels that pad the last 4-panel W^T A group get no A h^T
      // workgroups (each would fetch a prologue stage before finding its panel idle) and no 1-panel W^T A ones
      const int lp = std::max(1, live_panels(pk));
      const int grid_ahtw = lp * ngt_ahtw;
      for (int c = 1; c <= chunk; ++c) {
        const int iter = it + c;
        int gsplit = e->nsplit;
        {
          // W^T A on the GTile core: 4-panel x 128-sample tiles (8 waves) while the grid fills the chip
          // at least twice, else 1-panel x 64-sample tiles (4 waves).  Both accumulate every entry in
          // the same canonical K order, so the switch never changes a bit.
          TimedLaunch tl(e, KID_WTA, iter % e->timing_stride == 0);
          gsplit = e->nsplit;   // chunk partials k_hupdate sums (1 after a LASTSUM launch)
          if (narrow) {
            const int ntq = (int)(e->n_cols_pad / 16);
            if (e->narrow_lc)   // loader / consumer waves (bit-identical to the one-wave form)
              hipLaunchKernelGGL((k_wta_narrow_lc<16, NARROW_NBUF, true>), dim3(e->nsplit * nblk * (ntq + 1)), dim3(128), 0,
                                 st, e->W[cur].as<double>(), e->Ablk.as<double>(), e->m_pad, ntq, e->nsplit, e->kchunk,
                                 nblk, e->colinfo.as<ColInfo>(), e->Gpart.as<double>(), g_ld, g_split,
                                 e->SWpart.as<double>(), sw_total);
            else
              hipLaunchKernelGGL((k_wta_narrow<16, NARROW_NBUF, true>), dim3(e->nsplit * nblk * (ntq + 1)), dim3(64), 0, st,
                                 e->W[cur].as<double>(), e->Ablk.as<double>(), e->m_pad, ntq, e->nsplit, e->kchunk, nblk,
                                 e->colinfo.as<ColInfo>(),
                                 e->Gpart.as<double>(), g_ld, g_split, e->SWpart.as<double>(), sw_total);
          } else if ((wta_big && sk_big_ok(e, ntj) && sk_grid_fits(e, pk.npanels / WTA_NPT, ntj)) ||
                     (wta_mid && sk_mid_ok(e, ntj) && sk_grid_fits(e, (lp + 1) / 2, ntj))) {
            // stream-K form: ncu persistent workgroups, whole rounds of items then the rest split evenly (bit-identical
            // to the one-item-per-workgroup tile: the same MFMA chains, handed over at a stage boundary)
            if (!e->skflag.p) {
              if (e->skfix.ensure(sizeof(double) * SK_FIX * e->ncu) || e->skflag.ensure(sizeof(unsigned) * e->ncu)) return -1;
              HCHECK(hipMemsetAsync(e->skflag.p, 0, sizeof(unsigned) * e->ncu, st));
            }
            const int ng = wta_big ? pk.npanels / WTA_NPT : (lp + 1) / 2;
            const long tiles = (long)ng * ntj;
            const bool lastsum = e->wta_lastsum && wta_big;
            if (lastsum && e->sktcnt.bytes < sizeof(unsigned) * tiles) {
              if (e->sktcnt.ensure(sizeof(unsigned) * tiles)) return -1;   // fresh tickets: zero
              HCHECK(hipMemsetAsync(e->sktcnt.p, 0, sizeof(unsigned) * tiles, st));
            }
            const SkArgs a{e->W[cur].as<double>(), e->Ablk.as<double>(), e->m_pad, ng, ntj, e->kchunk,
                           e->prb.as<int>(), e->pre.as<int>(), e->rinfo.as<RestartInfo>(), e->colinfo.as<ColInfo>(),
                           e->stop_iter.as<int>(), e->Gpart.as<double>(), g_ld, g_split, e->SWpart.as<double>(), sw_total,
                           e->skfix.as<double>(), e->skflag.as<unsigned>(), ++e->sk_epoch, e->nsplit,
                           e->sktcnt.as<unsigned>(), e->sk_dp_xcd};
            if (!wta_big) {
              hipLaunchKernelGGL((k_wta2_sk<WTA_MID_NBUF, false, false, 2>), dim3(e->ncu), dim3(SK_THREADS / 2), 0, st, a);
            } else if (lastsum) {
              hipLaunchKernelGGL((k_wta2_sk<GT_NBUF, false, true>), dim3(e->ncu), dim3(SK_THREADS), 0, st, a);
              gsplit = 1;   // every tile's chunk partials summed into chunk slot 0
            } else {
              hipLaunchKernelGGL(k_wta2_sk<GT_NBUF>, dim3(e->ncu), dim3(SK_THREADS), 0, st, a);
            }
          } else if (wta_big) {
            const int ng = pk.npanels / WTA_NPT;
            // ntj >= 4: 16 waves (4 per SIMD, 64 x 32 outputs each; round 5: +2 % over 8 waves at full load, every
            // Gram chain in registers, tools/kvar.hip), else 8 waves carrying 2 / 4 Gram candidates each
            auto kw = (ntj >= 4)   ? (WTA_W16 ? k_wta2<WTA_NPT, 128, 4, 4, 1, GT_NBUF, 1, true, true, false, true>
                                              : k_wta2<WTA_NPT, 128, 4, 2, 1, GT_NBUF, 1, true, true, false, WTA_GREG>)
                      : (ntj >= 2) ? k_wta2<WTA_NPT, 128, 4, 2, 2, GT_NBUF, 1, true>
                                   : k_wta2<WTA_NPT, 128, 4, 2, 4, GT_NBUF, 1, true>;
            const int wthr = (ntj >= 4 && WTA_W16) ? 1024 : 512;
            hipLaunchKernelGGL(kw, dim3(e->nsplit * ng * ntj), dim3(wthr), 0, st, e->W[cur].as<double>(),
                               e->Ablk.as<double>(), e->m_pad, ng, ntj, e->nsplit, e->kchunk, e->prb.as<int>(),
                               e->pre.as<int>(), e->rinfo.as<RestartInfo>(), e->colinfo.as<ColInfo>(),
                               e->stop_iter.as<int>(), e->Gpart.as<double>(), g_ld, g_split, e->SWpart.as<double>(),
                               sw_total);
          } else if (wta_mid) {   // npanels is a multiple of WTA_NPT, so of 2
            const int ng = (lp + 1) / 2;
            // ntj >= 4: wave rows = panels (2 x 4 waves, 64 x 32 outputs each) with every Gram chain in registers
            // (the 16-wave big tile's scheme), else 4 x 2 waves carrying LDS Gram chains
            auto kw = (ntj >= 4 && WTA_MID_GREG) ? k_wta2<2, 128, 2, 4, 1, WTA_MID_NBUF, WTA_MID_MINW, true, true, false, true>
                      : (ntj >= 2)               ? k_wta2<2, 128, 4, 2, 1, WTA_MID_NBUF, WTA_MID_MINW, true>
                                                 : k_wta2<2, 128, 4, 2, 2, WTA_MID_NBUF, WTA_MID_MINW, true>;
            hipLaunchKernelGGL(kw, dim3(e->nsplit * ng * ntj), dim3(512), 0, st, e->W[cur].as<double>(),
                               e->Ablk.as<double>(), e->m_pad, ng, ntj, e->nsplit, e->kchunk, e->prb.as<int>(),
                               e->pre.as<int>(), e->rinfo.as<RestartInfo>(), e->colinfo.as<ColInfo>(),
                               e->stop_iter.as<int>(), e->Gpart.as<double>(), g_ld, g_split, e->SWpart.as<double>(),
                               sw_total);
          } else if (!wta_tiny) {   // 1-panel tiles: the Gram blocks in 3 workgroups of their own per (chunk, panel)
            hipLaunchKernelGGL((k_wta2<1, 64, 2, 2, 1, GT_NBUF, 1, true, true, true>), dim3(e->nsplit * lp * (2 * ntj + 3)), dim3(256),
                               0, st, e->W[cur].as<double>(), e->Ablk.as<double>(), e->m_pad, lp, 2 * ntj, e->nsplit,
                               e->kchunk, e->prb.as<int>(), e->pre.as<int>(), e->rinfo.as<RestartInfo>(),
                               e->colinfo.as<ColInfo>(), e->stop_iter.as<int>(), e->Gpart.as<double>(), g_ld, g_split,
                               e->SWpart.as<double>(), sw_total);
          } else {   // few live panels: 1-panel x 32-sample tiles, two 16x16 blocks per wave (short chains);
                     // at most one live workgroup per CU: an 8-stage ring (more DMA in flight per CU, 96 KiB)
            auto kw = (long)e->nsplit * live_panels(pk) * 4 * ntj <= e->ncu ? k_wta2<1, 32, 4, 1, 1, 8, 1, true, true, true>
                                                                             : k_wta2<1, 32, 4, 1, 1, GT_NBUF, 1, true, true, true>;
            hipLaunchKernelGGL(kw, dim3(e->nsplit * lp * (4 * ntj + 3)), dim3(256), 0, st,
                               e->W[cur].as<double>(), e->Ablk.as<double>(), e->m_pad, lp, 4 * ntj, e->nsplit,
                               e->kchunk, e->prb.as<int>(), e->pre.as<int>(), e->rinfo.as<RestartInfo>(),
                               e->colinfo.as<ColInfo>(), e->stop_iter.as<int>(), e->Gpart.as<double>(), g_ld, g_split,
                               e->SWpart.as<double>(), sw_total);
          }
        }
        {
          TimedLaunch tl(e, KID_HUPD, iter % e->timing_stride == 0);
          hipLaunchKernelGGL(k_hupdate<>, dim3(nact), dim3(NTH), 0, st, iter, opts.maxiter, opts.stop_rule,
                             e->rinfo.as<RestartInfo>(), n, e->n_pad, e->Gpart.as<double>(), g_ld, g_split, gsplit, e->nsplit,
                             e->SWpart.as<double>(), sw_total, e->H[cur].as<double>(), e->SH.as<double>(),
                             e->stop_iter.as<int>(), e->stop_reason.as<int>(), e->unchanged.as<int>(),
                             e->classes.as<int>(), cls_ld, e->n_stopped.as<int>(), e->SHP.as<double>(),
                             e->colact.as<int>(), e->Hstat.as<double>());
        }
        // STOP_TOLX (even iterations > 1): snapshot W before its update, test after it
        const bool tol_check = tolx && iter > 1 && iter % 2 == 0;
        if (tol_check)
          HCHECK(hipMemcpyAsync(e->Wsnap.p, e->W[cur].p, sizeof(double) * (size_t)pk.npanels * PANEL * e->m_pad,
                                hipMemcpyDeviceToDevice, st));
        {
          TimedLaunch tl(e, KID_AHTW, iter % e->timing_stride == 0);
          if (narrow) {   // per live 16-column block: 16 rows x 32 genes, 2 waves
            hipLaunchKernelGGL((k_ahtw4<GT / 4, GT_NBUF, 1, 16, 2>), dim3(4 * e->ngt * nblk), dim3(128), 0, st,
                               iter, e->H[cur].as<double>(), e->n_pad, e->Arm.as<double>(), e->m_pad,
                               e->W[cur].as<double>(), e->SHP.as<double>(), e->colinfo.as<ColInfo>(),
                               e->colact.as<int>(), nblk, 4 * e->ngt);
          } else {
            // the last K stage's second half is padding (samples >= n): the KHALF form skips it
            const bool kh = AHTW_KSKIP && AHTW_NBUF == 2 && e->n_pad - n >= 8;
            auto ka = ahtw_small ? (kh ? k_ahtw4<GT / 2, AHTW_NBUF, 1, PANEL, 4, AHTW_LATE, AHTW_NBUF == 2>
                                       : k_ahtw4<GT / 2, AHTW_NBUF, 1, PANEL, 4, AHTW_LATE>)
                                 : (kh ? k_ahtw4<GT, AHTW_NBUF, 1, PANEL, 4, AHTW_LATE, AHTW_NBUF == 2>
                                       : k_ahtw4<GT, AHTW_NBUF, 1, PANEL, 4, AHTW_LATE>);
            hipLaunchKernelGGL(ka, dim3(grid_ahtw), dim3(256), 0, st, iter,
                               e->H[cur].as<double>(), e->n_pad, e->Arm.as<double>(), e->m_pad, e->W[cur].as<double>(),
                               e->SHP.as<double>(), e->colinfo.as<ColInfo>(), e->colact.as<int>(), lp,
                               ngt_ahtw);
          }
        }
        if (tol_check) {
          TimedLaunch tl(e, KID_OTHER);
          hipLaunchKernelGGL(k_wstat, dim3(nact), dim3(NT), 0, st, iter, e->rinfo.as<RestartInfo>(),
                             e->W[cur].as<double>(), e->Wsnap.as<double>(), e->m_pad, m, e->colact.as<int>(),
                             e->Hstat.as<double>(), opts.TolX, opts.TolFun, e->stop_iter.as<int>(),
                             e->stop_reason.as<int>(), e->n_stopped.as<int>());
        }
      }
      HCHECK(hipGetLastError());
      it += chunk;
      HCHECK(hipMemcpyAsync(&e->h_stopped[q & 1], e->n_stopped.p, sizeof(int), hipMemcpyDeviceToHost, st));
      HCHECK(hipEventRecord(ev[q & 1], st));
      ++q;
    }
    // consume polls, keeping one chunk in flight while there is more to enqueue
    const int target = (it < opts.maxiter) ? q - 1 : q;
    bool done = false;
    int stopped = 0;
    while (checked < target) {
      HCHECK(hipEventSynchronize(ev[checked & 1]));
      stopped = e->h_stopped[checked & 1];
      if (stopped >= nj) done = true;
      ++checked;
    }
    if (e->timing) drain_timing(e);
    if (done || (it >= opts.maxiter && checked == q)) break;
    // repack when a fraction 1/repack_div of the live restarts have stopped since the last packing
    if (stopped - stopped_at_pack >= std::max(1, nact / e->repack_div)) {
      HCHECK(hipStreamSynchronize(st));
      if (e->timing) drain_timing(e);
      checked = q;   // every poll is now complete
      HCHECK(hipMemcpy(si.data(), e->stop_iter.p, sizeof(int) * nj, hipMemcpyDeviceToHost));
      std::vector<RestartInfo> gone, live;
      for (const RestartInfo& r : pk.ri) {
        if (!si[r.rid])
          live.push_back(r);
        else if (!archived[r.rid])   // stopped restarts a skipped repack (below) left in pk are archived once
          gone.push_back(r);
      }
      if (archive(gone)) return -1;
      Packing np = pack(live);
      if ((long)np.npanels * PANEL > cap_cols) {
        // first-fit decreasing is not monotone under removal: a (rare) larger packing would overrun
        // the buffers sized from the initial one, so keep the current placement until the next poll
        stopped_at_pack = stopped;
        continue;
      }
      std::vector<int> old_col(nj, -1);
      for (const RestartInfo& r : live) old_col[r.rid] = r.col0;
      std::vector<MoveJob> mv(np.ri.size());
      for (size_t x = 0; x < np.ri.size(); ++x) mv[x] = {old_col[np.ri[x].rid], np.ri[x].col0, np.ri[x].k};
      if (!mv.empty()) {
        HCHECK(hipMemcpyAsync(e->moves.p, mv.data(), sizeof(MoveJob) * mv.size(), hipMemcpyHostToDevice, st));
        {
          TimedLaunch tl(e, KID_OTHER);
          hipLaunchKernelGGL(k_move_rows, dim3((unsigned)mv.size(), 16), dim3(NT), 0, st, e->moves.as<MoveJob>(),
                             e->W[cur].as<double>(), e->m_pad, e->W[cur ^ 1].as<double>(), e->m_pad, e->m_pad);
          hipLaunchKernelGGL(k_move_rows, dim3((unsigned)mv.size(), 2), dim3(NT), 0, st, e->moves.as<MoveJob>(),
                             e->H[cur].as<double>(), e->n_pad, e->H[cur ^ 1].as<double>(), e->n_pad, e->n_pad);
        }
        HCHECK(hipGetLastError());
      }
      cur ^= 1;
      pk = np;
      if (upload_packing(pk)) return -1;
      HCHECK(hipStreamSynchronize(st));   // mv / pk host data uploaded
      nact = (int)pk.ri.size();
      stopped_at_pack = nj - nact;
      ++e->repacks;
      if (nact == 0) break;
    }
  }
  HCHECK(hipStreamSynchronize(st));
  if (e->timing) drain_timing(e);
  const int iters_enqueued = it;
  auto t_iter1 = std::chrono::steady_clock::now();
  {
    std::vector<RestartInfo> rest;
    for (const RestartInfo& r : pk.ri)
      if (!archived[r.rid]) rest.push_back(r);
    if (archive(rest)) return -1;
  }

  // ---- labels, counts (from the archive) ----
  std::vector<RestartInfo> fin(nj);
  for (int rid = 0; rid < nj; ++rid) fin[rid] = {hoff[rid], all[rid].k, rid, all[rid].sq_off};
  HCHECK(hipMemcpyAsync(e->finfo.p, fin.data(), sizeof(RestartInfo) * nj, hipMemcpyHostToDevice, st));
  {
    TimedLaunch tl(e, KID_LABELS);
    hipLaunchKernelGGL(k_labels, dim3((n + NT - 1) / NT, nj), dim3(NT), 0, st, e->finfo.as<RestartInfo>(),
                       e->slot.as<int>(), e->Hfin.as<double>(), e->n_pad, n, opts.label_rule, e->labels.as<int32_t>());
  }
  HCHECK(hipGetLastError());
  std::vector<int> gb(nk + 1, 0), gl;
  for (int g = 0; g < nk; ++g) {
    gb[g] = (int)gl.size();
    for (int s = 0; s < nj; ++s)
      if ((jb + s) % nk == g) gl.push_back(s);
  }
  gb[nk] = (int)gl.size();
  const size_t cnt_len = (size_t)nk * n * n;
  if (out && (out->counts || out->consensus)) {
    if (e->grp_begin.ensure(sizeof(int) * (nk + 1)) || e->grp_list.ensure(sizeof(int) * std::max<size_t>(gl.size(), 1)))
      return -1;
    HCHECK(hipMemcpyAsync(e->grp_begin.p, gb.data(), sizeof(int) * (nk + 1), hipMemcpyHostToDevice, st));
    if (!gl.empty()) HCHECK(hipMemcpyAsync(e->grp_list.p, gl.data(), sizeof(int) * gl.size(), hipMemcpyHostToDevice, st));
    int32_t* dcounts;
    if (out->counts && out->counts_on_device) {
      dcounts = out->counts;
    } else {
      if (e->counts_tmp.ensure(sizeof(int32_t) * cnt_len)) return -1;
      dcounts = e->counts_tmp.as<int32_t>();
    }
    {
      TimedLaunch tl(e, KID_COUNTS);
      hipLaunchKernelGGL(k_counts, dim3((n + CNT_T - 1) / CNT_T, (n + CNT_T - 1) / CNT_T, nk), dim3(NT), 0, st, e->labels.as<int32_t>(),
                         e->grp_begin.as<int>(), e->grp_list.as<int>(), n, dcounts);
    }
    HCHECK(hipGetLastError());
    if (out->consensus) {
      if (e->cons_tmp.ensure(sizeof(double) * cnt_len)) return -1;
      hipLaunchKernelGGL(k_divide, dim3((unsigned)((cnt_len + NT - 1) / NT)), dim3(NT), 0, st, dcounts, (double)R,
                         (long)cnt_len, e->cons_tmp.as<double>());
      HCHECK(hipGetLastError());
      HCHECK(hipMemcpyAsync(out->consensus, e->cons_tmp.p, sizeof(double) * cnt_len, hipMemcpyDeviceToHost, st));
    }
    if (out->counts && !out->counts_on_device)
      HCHECK(hipMemcpyAsync(out->counts, dcounts, sizeof(int32_t) * cnt_len, hipMemcpyDeviceToHost, st));
  }
  std::vector<int> sr(nj);
  HCHECK(hipMemcpyAsync(si.data(), e->stop_iter.p, sizeof(int) * nj, hipMemcpyDeviceToHost, st));
  HCHECK(hipMemcpyAsync(sr.data(), e->stop_reason.p, sizeof(int) * nj, hipMemcpyDeviceToHost, st));
  if (out && out->labels)
    HCHECK(hipMemcpyAsync(out->labels, e->labels.p, sizeof(int32_t) * (size_t)nj * n, hipMemcpyDeviceToHost, st));
  HCHECK(hipStreamSynchronize(st));
  if (e->timing) drain_timing(e);

  long long tot_iters = 0;
  int max_it = 0;
  double fl_wta = 0, fl_ahtw = 0;
  // bytes, summed over restart-iterations (each restart takes part in `itr` launches of each MU kernel)
  double b_wta = 0, ba_wta = 0, b_ahtw = 0, ba_ahtw = 0, b_hupd = 0, ba_hupd = 0, b_lab = 0, cols = 0;
  const double ns = e->nsplit;
  for (int rid = 0; rid < nj; ++rid) {
    const int itr = si[rid] ? si[rid] : iters_enqueued;
    tot_iters += itr;
    max_it = std::max(max_it, itr);
    const double k = all[rid].k;
    // algorithmic flops (nmf_mu.c:174-202 at 2*M*N*K each): W^T A + W^T W  |  A h^T + W0 (h h^T)
    fl_wta += (double)itr * (2.0 * m * n * k + 2.0 * m * k * k);
    fl_ahtw += (double)itr * (2.0 * m * n * k + 2.0 * m * k * k);
    // W^T A: W read + G written (algorithmic) | + the split-K partials and Gram partials (design)
    ba_wta += itr * 8.0 * k * (m + n);
    b_wta += itr * 8.0 * k * (m + ns * n + ns * k);
    // A h^T + W update: h, W0 read, W written
    ba_ahtw += itr * 8.0 * k * (2.0 * m + n);
    b_ahtw += itr * 8.0 * k * (2.0 * m + n + KMAX);
    // H update (SURVEY 8(d) B_ew, H side): H, numerator, denominator read, H written = 32 n k
    ba_hupd += itr * 32.0 * n * k;
    b_hupd += itr * 8.0 * (k * n * (ns + 2.0) + k * k * (ns + 2.0) + k * KMAX);
    b_lab += 8.0 * k * n + 4.0 * n;
    cols += k;
    if (out && out->iters) out->iters[rslot[rid]] = itr;
    if (out && out->stopped_early) out->stopped_early[rslot[rid]] = (sr[rid] == 1 || sr[rid] == 3);
  }
  const double a_bytes = 8.0 * m * n;   // A, read once per launch by each contraction
  if (const long long c = e->klaunch[KID_WTA]) {
    e->kflops[KID_WTA] = fl_wta / c;
    e->kbytes_algo[KID_WTA] = a_bytes + ba_wta / c;
    e->kbytes[KID_WTA] = a_bytes + b_wta / c;
  }
  if (const long long c = e->klaunch[KID_AHTW]) {
    e->kflops[KID_AHTW] = fl_ahtw / c;
    e->kbytes_algo[KID_AHTW] = a_bytes + ba_ahtw / c;
    e->kbytes[KID_AHTW] = a_bytes + b_ahtw / c;
  }
  if (const long long c = e->klaunch[KID_SMALL]) {   // the whole MU iteration in one persistent launch
    e->kflops[KID_SMALL] = (fl_wta + fl_ahtw) / c;
    e->kbytes_algo[KID_SMALL] = (ba_wta + ba_ahtw + ba_hupd) / c;
    e->kbytes[KID_SMALL] = e->kbytes_algo[KID_SMALL];
  }
  if (const long long c = e->klaunch[KID_HUPD]) {
    e->kbytes_algo[KID_HUPD] = ba_hupd / c;
    e->kbytes[KID_HUPD] = b_hupd / c;
  }
  if (e->klaunch[KID_LABELS]) e->kbytes[KID_LABELS] = e->kbytes_algo[KID_LABELS] = b_lab;   // one launch
  if (e->klaunch[KID_COUNTS]) {   // labels of each k group read once, n x n int32 counts written per k
    e->kbytes_algo[KID_COUNTS] = 4.0 * nj * n + 4.0 * nk * n * n;
    e->kbytes[KID_COUNTS] = e->kbytes_algo[KID_COUNTS];
  }
  (void)cols;

  if (out && (out->W || out->H)) {
    std::vector<long> woff(nj + 1, 0), ho(nj + 1, 0);
    for (int s = 0; s < nj; ++s) {
      woff[s + 1] = woff[s] + (long)m * job_k(s);
      ho[s + 1] = ho[s] + (long)job_k(s) * n;
    }
    std::vector<double> hrow;
    for (int rid = 0; rid < nj; ++rid) {
      const int s = rslot[rid], k = all[rid].k;
      if (out->W)
        HCHECK(hipMemcpy2DAsync(out->W + woff[s], sizeof(double) * m, e->Wfin.as<double>() + (long)hoff[rid] * e->m_pad,
                                sizeof(double) * e->m_pad, sizeof(double) * m, k, hipMemcpyDeviceToHost, st));
      if (out->H) {
        hrow.assign((size_t)k * n, 0.0);
        HCHECK(hipMemcpy2DAsync(hrow.data(), sizeof(double) * n, e->Hfin.as<double>() + (long)hoff[rid] * e->n_pad,
                                sizeof(double) * e->n_pad, sizeof(double) * n, k, hipMemcpyDeviceToHost, st));
        HCHECK(hipStreamSynchronize(st));
        for (int j = 0; j < n; ++j)
          for (int a = 0; a < k; ++a) out->H[ho[s] + (long)j * k + a] = hrow[(size_t)a * n + j];
      }
    }
    HCHECK(hipStreamSynchronize(st));
  }
  auto t_end = std::chrono::steady_clock::now();
  if (out) {
    out->seconds_total = std::chrono::duration<double>(t_end - t_start).count();
    out->seconds_iterate = std::chrono::duration<double>(t_iter1 - t_iter0).count();
    out->restart_iterations = tot_iters;
    out->max_iter_run = max_it;
  }
  if (opts.verbose) {
    fprintf(stderr, "[nmfc] %d restarts, %d iterations enqueued, max %d, mean %.1f, %d repacks, %.3f s\n", nj,
            iters_enqueued, max_it, (double)tot_iters / nj, e->repacks,
            std::chrono::duration<double>(t_end - t_start).count());
  }
  return 0;
}

// One restart of nmf_mu.c:84-315 with the fewest host round trips (the unchanged-R drop-in, nmf.r:41-45 calls
// nmf_mu once per restart): the job as one 16-column block on one k_team_mu team; one upload of
// [block | W0 | H0] from pinned staging, the launch, one download of [stop | W | H], one synchronisation.
// The flags are not zeroed per call: tags continue after the previous call's (mu1_base).
int nmfc_engine_mu1(nmfc_engine* e, int k, int maxiter, int stop_rule, const double* W0, const double* H0,
                    double* W_out, double* H_out, int* iters, int* early) {
  if (!e || !W0 || !H0 || !W_out || !H_out || maxiter < 0 || k < 1 || k > 16 || k > e->m || k > e->n ||
      (stop_rule != NMFC_STOP_FIXED && stop_rule != NMFC_STOP_REF_COMPAT && stop_rule != NMFC_STOP_ARGMAX_STABLE)) {
    set_err("nmfc_engine_mu1: bad arguments");
    return -1;
  }
  const int m = e->m, n = e->n;
  const int jb = (n + 15) / 16;
  const int P = (int)(e->m_pad / TEAM_ROWS);
  if (!e->small_ok || e->small_kernel == 2 || n > 64 || P > TEAM_PMAX) {
    set_err("nmfc_engine_mu1: shape %d x %d is not a team shape (m rounded up to 128 <= %d, n <= 64)", m, n,
            TEAM_ROWS * TEAM_PMAX);
    return -1;
  }
  HCHECK(hipSetDevice(e->dev));
  const long mp = e->m_pad, np = e->n_pad;
  const size_t off_stop = 256, off_w = 512, off_h = off_w + sizeof(double) * 16 * mp;
  const size_t total = off_h + sizeof(double) * 16 * np;
  if (e->mu1_host_bytes < total) {
    if (e->mu1_host) (void)hipHostFree(e->mu1_host);
    e->mu1_host = nullptr;
    e->mu1_host_bytes = 0;
    HCHECK(hipHostMalloc((void**)&e->mu1_host, total, 0));
    memset(e->mu1_host, 0, total);
    e->mu1_host_bytes = total;
    e->mu1_kprev = 16;
  }
  if (e->mu1_dev.ensure(total) || e->mu1_G.ensure(sizeof(double) * 2 * TEAM_PMAX * 16 * 16 * jb) ||
      e->mu1_SW.ensure(sizeof(double) * 2 * TEAM_PMAX * 256))
    return -1;
  if (!e->mu1_flag.p) e->mu1_base = -1;
  if (e->mu1_flag.ensure(sizeof(unsigned) * TEAM_PMAX)) return -1;
  if (e->mu1_base < 0 || e->mu1_base > (1 << 30)) {
    HCHECK(hipMemsetAsync(e->mu1_flag.p, 0, sizeof(unsigned) * TEAM_PMAX, e->st));
    e->mu1_base = 0;
  }
  char* hb = e->mu1_host;
  SmallBlock blk{};
  blk.col0 = 0;
  blk.nr = 1;
  blk.rid[0] = 0;
  blk.k[0] = k;
  blk.lc0[0] = 0;
  memcpy(hb, &blk, sizeof(blk));
  int* hstop = reinterpret_cast<int*>(hb + off_stop);
  hstop[0] = hstop[1] = hstop[2] = 0;   // stop iteration, reason, team error word
  double* hw = reinterpret_cast<double*>(hb + off_w);
  double* hh = reinterpret_cast<double*>(hb + off_h);
  for (int c = 0; c < k; ++c) memcpy(hw + c * mp, W0 + (long)c * m, sizeof(double) * m);   // W0 column c -> row c
  for (int c = 0; c < k; ++c)
    for (int j = 0; j < n; ++j) hh[c * np + j] = H0[c + (long)j * k];                     // k x n column-major
  if (e->mu1_kprev > k) {   // rows a larger previous k left behind
    memset(hw + k * mp, 0, sizeof(double) * (e->mu1_kprev - k) * mp);
    memset(hh + k * np, 0, sizeof(double) * (e->mu1_kprev - k) * np);
  }
  e->mu1_kprev = k;
  char* db = static_cast<char*>(e->mu1_dev.p);
  HCHECK(hipMemcpyAsync(db, hb, total, hipMemcpyHostToDevice, e->st));
  auto kern = jb == 1 ? k_team_mu<1> : jb == 2 ? k_team_mu<2> : jb == 3 ? k_team_mu<3> : k_team_mu<4>;
  int* dstop = reinterpret_cast<int*>(db + off_stop);
  hipLaunchKernelGGL(kern, dim3(P), dim3(256), 0, e->st, reinterpret_cast<const SmallBlock*>(db), 1, P, e->Acm.as<double>(),
                     mp, n, np, reinterpret_cast<double*>(db + off_w), reinterpret_cast<double*>(db + off_h), maxiter,
                     stop_rule, dstop, dstop + 1, e->mu1_G.as<double>(), e->mu1_SW.as<double>(),
                     e->mu1_flag.as<unsigned>(), (unsigned)e->mu1_base, dstop + 2, nullptr);
  HCHECK(hipGetLastError());
  HCHECK(hipMemcpyAsync(hb + off_stop, db + off_stop, total - off_stop, hipMemcpyDeviceToHost, e->st));
  HCHECK(hipStreamSynchronize(e->st));
  if (hstop[2]) {
    e->mu1_base = -1;
    set_err("k_team_mu: the team could not meet (not co-resident?)");
    return -1;
  }
  const int it = maxiter == 0 ? 0 : hstop[0];
  e->mu1_base += it;   // one tag per iteration run
  for (int c = 0; c < k; ++c) memcpy(W_out + (long)c * m, hw + c * mp, sizeof(double) * m);
  for (int c = 0; c < k; ++c)
    for (int j = 0; j < n; ++j) H_out[c + (long)j * k] = hh[c * np + j];
  if (iters) *iters = it;
  if (early) *early = hstop[1] == 1;
  return 0;
}

int nmfc_consensus(const double* Hs, int k, int n, int R, int label_rule, int32_t* labels, int32_t* counts,
                   double* consensus) {
  if (!Hs || k < 1 || n < 1 || R < 1 || label_rule < 0 || label_rule > 1) {
    set_err("nmfc_consensus: bad arguments");
    return -1;
  }
  std::vector<double> hrows((size_t)R * k * n);
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < n; ++j)
      for (int a = 0; a < k; ++a) hrows[((size_t)r * k + a) * n + j] = Hs[(size_t)r * k * n + (size_t)j * k + a];
  std::vector<RestartInfo> ri(R);
  std::vector<int> slot(R), gb = {0, R};
  for (int r = 0; r < R; ++r) {
    ri[r] = {r * k, k, r, 0};
    slot[r] = r;
  }
  DevBuf dH, dri, dslot, dgb, dlab, dcnt, dcons;
  if (dH.ensure(sizeof(double) * hrows.size()) || dri.ensure(sizeof(RestartInfo) * R) || dslot.ensure(sizeof(int) * R) ||
      dgb.ensure(sizeof(int) * 2) || dlab.ensure(sizeof(int32_t) * (size_t)R * n) ||
      dcnt.ensure(sizeof(int32_t) * (size_t)n * n) || dcons.ensure(sizeof(double) * (size_t)n * n))
    return -1;
  HCHECK(hipMemcpy(dH.p, hrows.data(), sizeof(double) * hrows.size(), hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(dri.p, ri.data(), sizeof(RestartInfo) * R, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(dslot.p, slot.data(), sizeof(int) * R, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(dgb.p, gb.data(), sizeof(int) * 2, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_labels, dim3((n + NT - 1) / NT, R), dim3(NT), 0, 0, dri.as<RestartInfo>(), dslot.as<int>(),
                     dH.as<double>(), (long)n, n, label_rule, dlab.as<int32_t>());
  HCHECK(hipGetLastError());
  hipLaunchKernelGGL(k_counts, dim3((n + CNT_T - 1) / CNT_T, (n + CNT_T - 1) / CNT_T, 1), dim3(NT), 0, 0, dlab.as<int32_t>(), dgb.as<int>(),
                     dslot.as<int>(), n, dcnt.as<int32_t>());
  HCHECK(hipGetLastError());
  hipLaunchKernelGGL(k_divide, dim3((unsigned)(((size_t)n * n + NT - 1) / NT)), dim3(NT), 0, 0, dcnt.as<int32_t>(),
                     (double)R, (long)n * n, dcons.as<double>());
  HCHECK(hipGetLastError());
  if (labels) HCHECK(hipMemcpy(labels, dlab.p, sizeof(int32_t) * (size_t)R * n, hipMemcpyDeviceToHost));
  if (counts) HCHECK(hipMemcpy(counts, dcnt.p, sizeof(int32_t) * (size_t)n * n, hipMemcpyDeviceToHost));
  if (consensus) HCHECK(hipMemcpy(consensus, dcons.p, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToHost));
  HCHECK(hipDeviceSynchronize());
  return 0;
}

int nmfc_sweep(const double* A, int m, int n, const int* ks, int nk, int R, const nmfc_sweep_opts* opts,
               nmfc_result* out) {
  nmfc_engine* e = nmfc_engine_create(-1, A, m, n, 0);
  if (!e) return -1;
  int rc = nmfc_engine_run(e, ks, nk, R, opts, nullptr, nullptr, out);
  nmfc_engine_destroy(e);
  return rc;
}

}  // extern "C"
