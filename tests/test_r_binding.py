"""CPU side of the R bindings (examples/r_nmfc.c): the shim builds as `R CMD SHLIB` would (C99, -fPIC -shared,
-lnmf), exports exactly the two .C entry points, and runExample()'s golden (tests/golden/golden_runexample.npz, the
reference's own nmf_mu on all 40 jobs) agrees with the first 40 jobs of the reference's C1 sweep in golden.npz (same
job ids and seeds, nmf.r:53-70).  The GPU calls are in tests/test_gpu_r_binding.py."""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ROOT

LIBDIR = os.path.join(ROOT, "nmfconsensus_amd", "lib")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libnmf.so")), reason="libnmf.so not built")
def test_r_shim_builds_and_exports():
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, "r_nmfc.so")
        r = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror", "-fPIC", "-shared",
                            "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "examples", "r_nmfc.c"),
                            "-L" + LIBDIR, "-lnmf", "-o", so], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
        exported = {l.split()[-1] for l in syms.splitlines() if " T " in l}
        assert exported == {"r_nmfc_sweep", "r_nmfc_brunet"}
        undef = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True).stdout
        lib = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIBDIR, "libnmf.so")], capture_output=True,
                             text=True).stdout
        provided = {l.split()[-1] for l in lib.splitlines()}
        for s in ("nmfc_sweep", "nmfc_default_opts", "nmfc_brunet_create", "nmfc_brunet_run", "nmfc_brunet_destroy",
                  "nmfc_brunet_default_opts"):
            assert s in undef and s in provided, s


def test_runexample_golden_is_the_c1_prefix(golden):
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_runexample.npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    assert list(g["rx_ks"]) == [2, 3, 4, 5] and int(g["rx_R"]) == 10 and int(g["rx_seed"]) == 123
    assert np.array_equal(g["rx_iters"], golden["c1_iters"][:40])
    assert np.array_equal(g["rx_job_seed"], golden["c1_job_seed"][:40])
    for rule in ("argmax", "rorder"):
        assert np.array_equal(g[f"rx_labels_{rule}"], golden[f"c1_labels_{rule}"][:40])
        assert g[f"rx_counts_{rule}"].dtype == np.int32
        assert np.array_equal(g[f"rx_consensus_{rule}"], g[f"rx_counts_{rule}"] / 10.0)
        assert all(np.all(np.diagonal(c) == 10) for c in g[f"rx_counts_{rule}"])
