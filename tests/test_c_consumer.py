"""The C ABI from plain C99 (CPU): examples/c_sweep.c compiles against include/*.h with -std=c99 -pedantic -Werror
and links against libnmf.so (every symbol it calls resolves).  The GPU run is tests/test_gpu_c_consumer.py."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "nmfconsensus_amd", "lib", "libnmf.so")


@pytest.mark.skipif(shutil.which("gcc") is None or not os.path.exists(LIB), reason="gcc or libnmf.so missing")
def test_c99_consumer_compiles_and_links(tmp_path):
    exe = tmp_path / "c_sweep"
    r = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror",
                        "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "examples", "c_sweep.c"),
                        "-L" + os.path.dirname(LIB), "-lnmf", "-Wl,--no-undefined", "-Wl,-rpath," + os.path.dirname(LIB),
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # every libnmf symbol the program uses is defined by libnmf.so
    nm = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
    used = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    ours = {s for s in used if s.startswith("nmfc_") or s in ("nmf_mu", "generateMatrix", "randnumber",
                                                                "set_default_opts")}
    assert {"nmfc_sweep", "nmf_mu", "generateMatrix", "nmfc_cophenetic_batch"} <= ours
    exported = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    have = {ln.split()[-1] for ln in exported.splitlines() if ln.strip()}
    assert ours <= have, ours - have
