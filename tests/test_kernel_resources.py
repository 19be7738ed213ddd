"""Register-spill guard for the hot kernels (CPU: compiles with hipcc, no GPU needed).

A spill in the MFMA tile kernels costs far more than any of their tuning gains (round 4: a branch in the A h^T
K loop spilled 182 VGPRs and cut the kernel 2.5x while every parity test stayed green), so the build itself is
checked: hipcc's kernel-resource-usage remarks for every kernel of engine.hip, brunet.hip and generic.hip must
show no VGPR spill and no scratch; solo.hip's measured spills (the one-workgroup kernel at the 256-VGPR edge,
DESIGN.md 5c) are pinned per instantiation (round 5: a new spill anywhere else, or a larger one in these four, fails)."""
import os
import re
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nmfconsensus_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
# spilled VGPRs per k_solo_mu<NC, K, ..., JOBS> / k_solo_batch<NC> instantiation (measured round 5, ROCm 7.2 hipcc);
# every other solo.hip kernel (k_solo8_mu included) must not spill
SOLO_SPILLS = {
    "k_solo_muILi10ELi2ELi0ELi0ELi0ELb0E": 10,   # k = 2 x 40 samples, single restart (the nmf_mu drop-in)
    "k_solo_muILi10ELi2ELi0ELi0ELi0ELb1E": 24,   # the same, batched job loop (C1 / C2)
    "k_solo_muILi8ELi3ELi0ELi0ELi0ELb1E": 2,     # k = 3 x 32, batched
    # k = 4 x 40, two gene steps in LDS, batched: ONE instantiation serves the fused solo launch (C1 / C2) and the
    # per-rank launches beside k_small_mu blocks (measured 3 spilled VGPRs, ROCm 7.2 hipcc, round 6)
    "k_solo_muILi10ELi4ELi0ELi0ELi2ELb1E": 3,
    "k_solo_batchILi10E": 37,                    # every rank x 40 samples in one launch (the rank-2 body's edge)
}


def _usage(src):
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-c", os.path.join(CSRC, src),
                            "-o", os.path.join(td, "x.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = {}
    for blk in r.stderr.split("Function Name: ")[1:]:
        name = blk.split()[0]
        g = lambda key: int(re.search(key + r": (\d+)", blk).group(1))
        out[name] = (g("VGPRs Spill"), g(r"ScratchSize \[bytes/lane\]"))
        OCC[name] = g(r"Occupancy \[waves/SIMD\]")
    return out


# engine kernels allowed a pinned spill count: k_wta2_sk (the stream-K W^T A tiles) reloads a few VGPRs once per piece,
# outside its K loops (test_wta_sk_k_loops_spill_free checks the loops themselves): 3 in the engine's 4-panel form (ROCm
# 7.2 hipcc, round 6 final), 12 in the LSUM probe arm (its last-arriver sum after the loop), 0 in the 2-panel form
ENGINE_SPILLS = {"k_wta2_skILi3ELb0ELb0ELi4E": 3, "k_wta2_skILi3ELb0ELb1ELi4E": 12}


def _short(mangled):
    m = re.search(r"L\d+(k_\w+?)I|L\d+(k_\w+?)E", mangled)
    return (m.group(1) or m.group(2)) if m else mangled


OCC = {}   # kernel -> waves per SIMD its registers allow (filled by _usage)
# the full-load MFMA tiles keep the occupancy their design rests on: A h^T three workgroups per CU
# (four waves each: 3 per SIMD), the 16-wave W^T A tile one workgroup of 4 waves per SIMD
OCC_MIN = {"k_ahtw4ILi128ELi2ELi1ELi64ELi4ELb1E": 3, "k_wta2ILi4ELi128ELi4ELi4E": 4}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_register_spills():
    srcs = ["engine.hip", "brunet.hip", "generic.hip", "solo.hip"]
    with ThreadPoolExecutor(4) as ex:
        res = dict(zip(srcs, ex.map(_usage, srcs)))
    for src in ("engine.hip", "brunet.hip", "generic.hip"):
        assert res[src], f"no kernels found in {src}"
        bad = {k: v for k, v in res[src].items()
               if v != (0, 0) and v[0] > max([n for key, n in ENGINE_SPILLS.items() if key in k], default=-1)}
        assert not bad, f"{src}: spilling kernels {bad}"
    def allowed(name):
        return next((v for key, v in SOLO_SPILLS.items() if key in name), 0)
    bad = {k: v for k, v in res["solo.hip"].items() if v[0] > allowed(k)}
    assert not bad, f"solo.hip: spills above the pinned counts {bad}"
    # the hot tile kernels are all there (the guard checks what the engine launches)
    for key, want in OCC_MIN.items():
        hits = {k: v for k, v in OCC.items() if key in k}
        assert hits, f"no {key} instantiation"
        assert all(v >= want for v in hits.values()), f"{key}: occupancy {hits} below {want} waves/SIMD"
    names = " ".join(res["engine.hip"])
    for k in ("k_wta2", "k_ahtw4", "k_hupdate", "k_wta_narrow_lc", "k_small_mu", "k_team_mu"):
        assert k in names, k


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_brunet_divide_op_count_matches_isa():
    """bench.py's C5 roofline prices each quotient at BRUNET_DIV_OPS fp64 VALU instructions beside the 2k rank-k FMAs
    (ADVICE r04): the innermost loop of k_br_hnum / k_br_wupd must hold exactly 2k + BRUNET_DIV_OPS fp64 VALU
    instructions per quotient, so the figure cannot drift from the compiled code.  Round 6: the RG x SPL quotients of a
    gene (sample) step share v_rcp_f64s in batches of the kernel's RCP table entry (brunet.hip recip_batch: 3 fp64
    instructions per quotient for the reciprocal either way), so a loop holds ceil(RG SPL / RCP) v_rcp_f64 per
    RG SPL quotients."""
    import re
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench import BRUNET_DIV_OPS
    import isa_loop

    defaults = _tuning_defaults()

    def rcp_batch(side, k):
        v = (int(defaults["NMFC_BR_RCP" + side].rstrip("ULul"), 0) >> (4 * k)) & 15
        return min(max(v, 1), 5)

    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "b.s")
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                            os.path.join(CSRC, "brunet.hip"), "-o", s], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = open(s).read().splitlines()
    # scalar-load operand rows (k = 10, 5) and the LDS-tile form (k = 2, 3)
    for kern in ("k_br_hnumILi10ELi1ELi1ELb1E", "k_br_wupdILi10ELi2ELi1ELb1E", "k_br_hnumILi5ELi3ELi1ELb1E",
                 "k_br_wupdILi5ELi3ELi1ELb1E", "k_br_hnumILi2ELi5ELi1ELb0E", "k_br_wupdILi3ELi4ELi1ELb0E"):
        k, rg, spl = (int(x) for x in re.findall(r"ILi(\d+)ELi(\d+)ELi(\d+)E", kern)[0])
        nq = rg * spl
        b = rcp_batch("H" if "hnum" in kern else "W", k)
        rcps_per_step = -(-nq // b)
        body = isa_loop.kernel_body(lines, kern)
        inner = isa_loop.innermost_loop_with(body, "v_rcp_f64")
        ops = [x.split()[0] for x in inner]
        n_rcp = sum(1 for o in ops if o.startswith("v_rcp_f64"))
        n_f64 = sum(1 for o in ops if o.startswith("v_") and "f64" in o and not o.startswith("v_mfma"))
        assert n_rcp > 0 and n_rcp % rcps_per_step == 0, (kern, n_rcp, rcps_per_step)
        n_quot = n_rcp // rcps_per_step * nq
        assert n_f64 == n_quot * (2 * k + BRUNET_DIV_OPS), (kern, n_f64, n_rcp, n_quot)


def _tuning_defaults():
    import re
    txt = open(os.path.join(CSRC, "nmfc_tuning.hpp")).read()
    return dict(re.findall(r"#ifndef (NMFC_\w+)\n#define \1 (.+?)(?:\s*//[^\n]*)?\n#endif", txt))


def test_tuning_switches_live_in_one_header():
    """Every compile-time A/B switch is declared in csrc/nmfc_tuning.hpp; no other product source
    opens its own #ifndef NMFC_* default, and the product build passes no -D."""
    import re
    defaults = _tuning_defaults()
    assert len(defaults) >= 26, sorted(defaults)
    for f in os.listdir(CSRC):
        if f == "nmfc_tuning.hpp" or not f.endswith((".hip", ".hpp", ".cpp")):
            continue
        txt = open(os.path.join(CSRC, f)).read()
        assert not re.search(r"#\s*if(n?def)\s+NMFC_|defined\s*\(\s*NMFC_", txt), f
    build_src = open(os.path.join(ROOT, "nmfconsensus_amd", "build.py")).read()
    assert '"-D' not in build_src and "'-D" not in build_src


def test_product_build_uses_tuning_defaults():
    """The built library reports, per translation unit, the values its switches had: they must be the header's
    defaults, so an experiment build (tools/build_variant.sh) can never ship.  Loads the .so; no GPU call."""
    import ctypes
    so = os.path.join(ROOT, "nmfconsensus_amd", "lib", "libnmf.so")
    if not os.path.exists(so):
        pytest.skip("libnmf.so not built")
    lib = ctypes.CDLL(so)
    defaults = _tuning_defaults()
    seen = set()
    for fn in ("nmfc_build_tuning", "nmfc_build_tuning_brunet"):
        f = getattr(lib, fn)
        f.restype = ctypes.c_char_p
        got = dict(kv.split("=", 1) for kv in f().decode().split(";"))
        for k, v in got.items():
            assert defaults[k] == v, (fn, k, v, defaults[k])
        seen |= set(got)
    assert seen == set(defaults), set(defaults) ^ seen


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_wta_sk_k_loops_spill_free():
    """k_wta2_sk runs eight K-loop instantiations inside its piece loop: no scratch access may sit in any of those inner
    loops (a first form reloaded a fragment offset every stage), and every inner loop carries the tile's MFMAs."""
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "e.s")
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                            os.path.join(CSRC, "engine.hip"), "-o", s], capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = open(s).read().splitlines()
    # the engine's forms: the 4-panel tile and the 2-panel tile (not the LSUM probe arm, k_wta2_sk<3, false, true>: it
    # reloads spilled values inside its K loops since the whole-round order, one reason it stays a probe)
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*k_wta2_sk\S*:", l) and "k_wta2_skILi3ELb0ELb1E" not in l]
    assert len(starts) >= 2, [lines[i] for i in starts]
    for start in starts:
        end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
        depth, inner_mfma, inner_scratch, blocks = 0, 0, 0, 0
        for l in lines[start:end]:
            if re.match(r"^\.LBB\w+:", l):
                m = re.search(r"Depth=(\d)", l)
                depth = int(m.group(1)) if m else 0
                blocks += depth >= 2
                continue
            m = re.match(r"^\s*; =>.*Loop Header: Depth=(\d)", l)
            if m:
                depth = int(m.group(1))
                continue
            if depth >= 2:
                inner_mfma += "v_mfma_f64_16x16x4" in l
                inner_scratch += "scratch_" in l
        assert blocks > 0 and inner_mfma >= 8 * 32, (lines[start], blocks, inner_mfma)
        assert inner_scratch == 0, f"{inner_scratch} scratch accesses inside the K loops of {lines[start]}"
