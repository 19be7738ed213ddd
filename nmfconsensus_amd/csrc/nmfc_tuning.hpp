// nmfc_tuning.hpp -- every compile-time A/B switch of the kernels, with its product default, in ONE place.
//
// The product build (nmfconsensus_amd/build.py) passes no -D flags, so every switch below takes the default written
// here; only tools/build_variant.sh (experiment builds for A/B runs) overrides them.  The library reports the values
// it was compiled with (nmfc_build_tuning() from engine.hip's translation unit, nmfc_build_tuning_brunet() from
// brunet.hip's), and tests/test_kernel_resources.py::test_product_build_uses_tuning_defaults fails the CPU suite when
// they differ from the defaults below -- a variant build can never ship.  The parity suites run the defaults only.
// Each value's measurement is cited where it is used.
#pragma once

// ---- MU engine (engine.hip / nmfc_kernels.hpp) ----
#ifndef NMFC_AHTW_NBUF
#define NMFC_AHTW_NBUF 2        // LDS ring stages of the A h^T tile (2: three workgroups per CU)
#endif
#ifndef NMFC_AHTW_LATE
#define NMFC_AHTW_LATE 1        // A h^T: W0 loaded after the K loop, one 16-row block ahead of the epilogue
#endif
#ifndef NMFC_AHTW_KSKIP
#define NMFC_AHTW_KSKIP 1       // A h^T: skip the K-padding half of the last stage
#endif
#ifndef NMFC_AHTW_SP
#define NMFC_AHTW_SP 32         // A h^T item map: bands of SP panels ...
#endif
#ifndef NMFC_AHTW_SG
#define NMFC_AHTW_SG 4          // ... by gene super-tiles of SG
#endif
#ifndef NMFC_NARROW_NBUF
#define NMFC_NARROW_NBUF 16     // LDS ring depth of the narrow (tail) W^T A kernel
#endif
#ifndef NMFC_WTA_MID_NBUF
#define NMFC_WTA_MID_NBUF 3     // ring depth of the 2-panel W^T A tile
#endif
#ifndef NMFC_WTA_MID_MINW
#define NMFC_WTA_MID_MINW 1     // its launch-bounds waves per SIMD
#endif
#ifndef NMFC_WTA_MID_GREG
#define NMFC_WTA_MID_GREG 1     // 2-panel W^T A tile: Gram chains in registers
#endif
#ifndef NMFC_WTA_GREG
#define NMFC_WTA_GREG 1         // 4-panel W^T A tiles: diagonal Gram blocks from the tile's W registers
#endif
#ifndef NMFC_WTA_W16
#define NMFC_WTA_W16 1          // the 4-panel x 128-sample W^T A tile on 16 waves (4 per SIMD)
#endif
#ifndef NMFC_SMALL_NW8
#define NMFC_SMALL_NW8 1        // k_small_mu with eight waves where m_pad % 256 == 0
#endif
#ifndef NMFC_SMALL_PF
#define NMFC_SMALL_PF 8         // k-steps of A rows in flight in the G phase of k_small_mu
#endif
#ifndef NMFC_SMALL_FPF
#define NMFC_SMALL_FPF 8        // F steps (4 gene blocks each) of A columns in flight
#endif
#ifndef NMFC_GT_PRIO
#define NMFC_GT_PRIO 0          // raise the wave priority around each GTile MFMA block (experiment; -1 %)
#endif

// ---- Brunet KL kernels (brunet.hip) ----
#ifndef NMFC_BRUNET_IEEEDIV
#define NMFC_BRUNET_IEEEDIV 0   // 1: the compiler's IEEE divide instead of rcp + Newton + residual correction
#endif
// Brunet per-rank kernel configuration, one table per kernel (H side k_br_hnum, W side k_br_wupd), nibble / bit k for
// rank k (ranks 0..15; rank 16 and any nibble 0 mean 1 restart per workgroup, no SPL, LDS operand rows).  Measured per
// k and kernel on the C5 shape (tools/brunet_kbench.py; profiles/r06/brunet_sload/).
#ifndef NMFC_BR_RGH
#define NMFC_BR_RGH 0x11121334500ULL   // restarts per workgroup (RG), H side: k = 2..10 -> 5 4 3 3 1 2 1 1 1
#endif
#ifndef NMFC_BR_RGW
#define NMFC_BR_RGW 0x21222334500ULL   // RG, W side: k = 2..10 -> 5 4 3 3 2 2 2 1 2
#endif
#ifndef NMFC_BR_SPLH
#define NMFC_BR_SPLH 0x300ULL          // bit k: 2 elements per lane (SPL), H side: k = 8, 9
#endif
#ifndef NMFC_BR_SPLW
#define NMFC_BR_SPLW 0x200ULL          // SPL, W side: k = 9
#endif
#ifndef NMFC_BR_SLH
#define NMFC_BR_SLH 0x6F0ULL           // bit k: operand rows by scalar loads (else LDS tiles), H side: k = 4..7, 9, 10
#endif
#ifndef NMFC_BR_SLW
#define NMFC_BR_SLW 0x7F0ULL           // scalar-load operand rows, W side: k = 4..10
#endif
#ifndef NMFC_BR_SMALL_B
#define NMFC_BR_SMALL_B 32      // batches of at most this many restarts use rg_small
#endif
#ifndef NMFC_BR_RG_SMALL_DIV
#define NMFC_BR_RG_SMALL_DIV 0  // 0: one restart per workgroup for small batches
#endif
#ifndef NMFC_BR_TL
#define NMFC_BR_TL 64           // operand tile rows
#endif
#ifndef NMFC_BR_UNROLL
#define NMFC_BR_UNROLL 0        // 0: the measured per-k, per-kernel unroll tables (brunet.hip br_unroll_h / _w)
#endif
#ifndef NMFC_BR_RCPH
#define NMFC_BR_RCPH 0x12221222200ULL  // nibble k: quotients sharing one v_rcp_f64 (brunet.hip recip_batch), H side: k = 2..10 -> 2 2 2 2 1 2 2 2 1
#endif
#ifndef NMFC_BR_RCPW
#define NMFC_BR_RCPW 0x22222242500ULL  // the same, W side: k = 2..10 -> 5 2 4 2 2 2 2 2 2
#endif

#define NMFC_TUNING_STR_(x) #x
#define NMFC_TUNING_STR(x) NMFC_TUNING_STR_(x)
// "NAME=value;" for every switch of one group, as the preprocessor saw it in this translation unit
#define NMFC_TUNING_MU                                                                                               \
  "NMFC_AHTW_NBUF=" NMFC_TUNING_STR(NMFC_AHTW_NBUF) ";NMFC_AHTW_LATE=" NMFC_TUNING_STR(NMFC_AHTW_LATE)               \
  ";NMFC_AHTW_KSKIP=" NMFC_TUNING_STR(NMFC_AHTW_KSKIP) ";NMFC_AHTW_SP=" NMFC_TUNING_STR(NMFC_AHTW_SP)                \
  ";NMFC_AHTW_SG=" NMFC_TUNING_STR(NMFC_AHTW_SG) ";NMFC_NARROW_NBUF=" NMFC_TUNING_STR(NMFC_NARROW_NBUF)              \
  ";NMFC_WTA_MID_NBUF=" NMFC_TUNING_STR(NMFC_WTA_MID_NBUF) ";NMFC_WTA_MID_MINW=" NMFC_TUNING_STR(NMFC_WTA_MID_MINW)  \
  ";NMFC_WTA_MID_GREG=" NMFC_TUNING_STR(NMFC_WTA_MID_GREG) ";NMFC_WTA_GREG=" NMFC_TUNING_STR(NMFC_WTA_GREG)          \
  ";NMFC_WTA_W16=" NMFC_TUNING_STR(NMFC_WTA_W16) ";NMFC_SMALL_NW8=" NMFC_TUNING_STR(NMFC_SMALL_NW8)                  \
  ";NMFC_SMALL_PF=" NMFC_TUNING_STR(NMFC_SMALL_PF) ";NMFC_SMALL_FPF=" NMFC_TUNING_STR(NMFC_SMALL_FPF)                \
  ";NMFC_GT_PRIO=" NMFC_TUNING_STR(NMFC_GT_PRIO)
#define NMFC_TUNING_BRUNET                                                                                           \
  "NMFC_BRUNET_IEEEDIV=" NMFC_TUNING_STR(NMFC_BRUNET_IEEEDIV) ";NMFC_BR_RGH=" NMFC_TUNING_STR(NMFC_BR_RGH)           \
  ";NMFC_BR_RGW=" NMFC_TUNING_STR(NMFC_BR_RGW) ";NMFC_BR_SPLH=" NMFC_TUNING_STR(NMFC_BR_SPLH)                        \
  ";NMFC_BR_SPLW=" NMFC_TUNING_STR(NMFC_BR_SPLW) ";NMFC_BR_SLH=" NMFC_TUNING_STR(NMFC_BR_SLH)                        \
  ";NMFC_BR_SLW=" NMFC_TUNING_STR(NMFC_BR_SLW) ";NMFC_BR_SMALL_B=" NMFC_TUNING_STR(NMFC_BR_SMALL_B)                  \
  ";NMFC_BR_RG_SMALL_DIV=" NMFC_TUNING_STR(NMFC_BR_RG_SMALL_DIV) ";NMFC_BR_TL=" NMFC_TUNING_STR(NMFC_BR_TL)          \
  ";NMFC_BR_UNROLL=" NMFC_TUNING_STR(NMFC_BR_UNROLL) ";NMFC_BR_RCPH=" NMFC_TUNING_STR(NMFC_BR_RCPH)              \
  ";NMFC_BR_RCPW=" NMFC_TUNING_STR(NMFC_BR_RCPW)
