"""Host code under the sanitizers (SURVEY.md §5 "Race detection / sanitizers": ASan / UBSan builds of the host C).

CPU only, no GPU: the GPU pool runs no sanitizer builds, so the host-side C/C++ is checked here.
* csrc/hclust.cpp -- the product's cophenetic / cutree step (nmf.r:165-177) -- with tests/sanitize/hclust_driver.cpp:
  under AddressSanitizer + UndefinedBehaviorSanitizer, and under ThreadSanitizer for nmfc_cophenetic_batch's host
  threads (the batch must equal the one-matrix call bit for bit).
* the oracle's C restatements (oracle/nmf_oracle.c, oracle/brunet_oracle.c; test infrastructure, the parity
  anchor) built with ASan + UBSan and loaded in a child interpreter that then re-runs golden cases through it.
* the drop-in's host C (csrc/compat.hip) built with -Xarch_host -fsanitize=address,undefined and driven by
  tests/sanitize/compat_driver.c (argument / matrix checks, generateMatrix against the golden init).
"""
import os
import shutil
import subprocess
import sys
import tempfile

import pytest

from conftest import ROOT

GXX = shutil.which("g++")
GCC = shutil.which("gcc")
CSRC = os.path.join(ROOT, "nmfconsensus_amd", "csrc")
DRIVER = os.path.join(ROOT, "tests", "sanitize", "hclust_driver.cpp")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")


def _build_and_run(flags, td, name):
    exe = os.path.join(td, name)
    r = subprocess.run([GXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-pthread",
                        os.path.join(CSRC, "hclust.cpp"), DRIVER, "-o", exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0 and "hclust driver ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_hclust_asan_ubsan():
    with tempfile.TemporaryDirectory() as td:
        _build_and_run(["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], td, "hclust_asan")


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_hclust_tsan():
    with tempfile.TemporaryDirectory() as td:
        _build_and_run(["-fsanitize=thread"], td, "hclust_tsan")


CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[2])
sys.path.insert(0, sys.argv[3])
from pyoracle import Oracle
from conftest import relfro
o = Oracle(sys.argv[1])
with np.load(sys.argv[4], allow_pickle=False) as z:
    g = {k: z[k] for k in z.files}
A = g["A_gct"]
for k in (2, 3, 4, 5):
    W, H = o.init_restart(123, 1000, 40, k)
    assert np.array_equal(W, g[f"init_k{k}_W"]) and np.array_equal(H, g[f"init_k{k}_H"])
    W, H, it = o.nmf_mu(A, W, H, 10, 0)
    assert it == 10 and relfro(W, g[f"fixed_k{k}_T10_W"]) < 1e-9 and relfro(H, g[f"fixed_k{k}_T10_H"]) < 1e-9
    W, H, it = o.nmf_mu(A, g[f"init_k{k}_W"], g[f"init_k{k}_H"], 10000, 1)
    assert it == int(g[f"refc_k{k}_iter"]), (k, it)
    W, H, it = o.nmf_mu(A, g[f"init_k{k}_W"], g[f"init_k{k}_H"], 300, 2)
    lab = o.labels(H)
    cnt = o.counts(np.stack([lab, lab]))
    assert cnt.shape == (40, 40)
    o.calculate_norm(A, W, H)
    o.calculate_maxchange(W, g[f"init_k{k}_W"])
    W, H, it = o.nmf_mu_tol(A, g[f"init_k{k}_W"], g[f"init_k{k}_H"], 200)
# Brunet on a ragged small case (the C5 restatement)
rng = np.random.default_rng(5)
B = np.asfortranarray(rng.random((37, 11)) + 0.1)
for k in (2, 5):
    W0, H0 = o.brunet_init(7, 37, 11, k)
    o.brunet(B, W0, H0, 60)
print("oracle under sanitizers ok")
"""


@pytest.mark.skipif(GCC is None, reason="gcc not available")
def test_oracle_asan_ubsan():
    asan = subprocess.run([GCC, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("libasan runtime not found")
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, "liboracle_asan.so")
        r = subprocess.run([GCC, "-O1", "-g", "-fno-omit-frame-pointer", "-fPIC", "-shared", "-fno-fast-math",
                            "-ffp-contract=off", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                            os.path.join(ROOT, "oracle", "nmf_oracle.c"), os.path.join(ROOT, "oracle", "brunet_oracle.c"),
                            "-o", so, "-lm"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        env = dict(ENV, LD_PRELOAD=asan)
        r = subprocess.run([sys.executable, "-c", CHILD, so, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
                            os.path.join(ROOT, "tests", "golden", "golden.npz")],
                           capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0 and "oracle under sanitizers ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
        assert "runtime error" not in r.stderr, r.stderr[-4000:]


HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/llvm/bin/clang"
LIBDIR = os.path.join(ROOT, "nmfconsensus_amd", "lib")


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)), reason="hipcc / clang not available")
@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libnmf.so")), reason="libnmf.so not built")
def test_compat_host_asan_ubsan(golden):
    """The drop-in's host C (csrc/compat.hip: set_default_opts, checkArguments, checkMatrices, randnumber,
    generateMatrix) compiled with -Xarch_host -fsanitize=address,undefined, linked ahead of the product libnmf.so (its
    definitions interpose) with tests/sanitize/compat_driver.c: every predicate answers as the reference's, and
    generateMatrix(ran) after srand(123) equals the reference's golden init bit for bit.  No GPU entry point runs."""
    import numpy as np
    with tempfile.TemporaryDirectory() as td:
        obj, drv, exe, out = (os.path.join(td, x) for x in ("c.o", "d.o", "compat_drv", "out.bin"))
        hostsan = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"]
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-fPIC", "-std=c++17", *hostsan, "-c",
                            os.path.join(CSRC, "compat.hip"), "-o", obj], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        r = subprocess.run([CLANG, "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-c",
                            os.path.join(ROOT, "tests", "sanitize", "compat_driver.c"), "-o", drv],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        link = ["-fsanitize=address", "-fsanitize=undefined", "-fno-gpu-sanitize"]
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", *link, drv, obj, "-L" + LIBDIR, "-lnmf",
                            "-Wl,-rpath," + LIBDIR, "-o", exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        r = subprocess.run([exe, out], capture_output=True, text=True, timeout=300, env=ENV)
        assert r.returncode == 0 and "compat driver ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
        assert "runtime error" not in r.stderr, r.stderr[-4000:]
        got = np.fromfile(out, dtype=np.float64)
    m, n, off = 1000, 40, 0
    for k in (2, 3, 4, 5):
        W = got[off:off + m * k].reshape((m, k), order="F")
        off += m * k
        H = got[off:off + k * n].reshape((k, n), order="F")
        off += k * n
        assert np.array_equal(W, golden[f"init_k{k}_W"]) and np.array_equal(H, golden[f"init_k{k}_H"]), k
    assert off == got.size


LANE_DRIVER = os.path.join(ROOT, "tests", "sanitize", "lane_pool_driver.cpp")


@pytest.mark.skipif(GXX is None, reason="g++ not available")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_brunet_lane_pool_sanitized(san):
    """The Brunet sweep's lane scheduler (csrc/lane_pool.hpp: 4 host threads, one per HIP stream, taking k batches
    from one atomic counter; brunet.hip nmfc_brunet_run) with a stub job that grows per-lane scratch, sets the
    thread-local error string and writes its own output slot: under ThreadSanitizer and under ASan + UBSan, 1..8
    lanes, every job exactly once, outputs equal to a serial run, a failure reported with its own message."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "lane_pool_driver")
        extra = ["-fno-sanitize-recover=all"] if "undefined" in san else []
        r = subprocess.run([GXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", *extra,
                            "-pthread", LANE_DRIVER, "-o", exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
        assert r.returncode == 0 and "lane pool driver ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
        assert "WARNING: ThreadSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
