"""The Brunet kernels' batched reciprocal on the host (CPU suite): tests/numerics/recip_check.cpp restates
csrc/brunet.hip recip_batch + quot_r with std::fma and a float-accurate stand-in for v_rcp_f64 (no worse than the
hardware's 2^-24.4), and checks that batches of 1..5 reciprocals -- at the spread of the KL updates' VP and at both
ends of the domain the library admits -- keep |1 - p r| below 2^-44 and give the IEEE quotient
a / p for every sampled pair.  The device form is checked the same way on the GPU by tools/quot_probe.hip
(profiles/r06/brunet_rcp/quot_probe.txt) and end to end by tests/test_gpu_brunet.py."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GXX = shutil.which("g++")


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_batched_reciprocal_gives_the_ieee_quotient():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "recip_check")
        # no FMA contraction: the restatement's fused operations are exactly its std::fma calls
        subprocess.run([GXX, "-O2", "-ffp-contract=off", "-std=c++17", os.path.join(HERE, "numerics", "recip_check.cpp"),
                        "-o", exe], check=True, capture_output=True, timeout=120)
        out = subprocess.run([exe, "2000000"], capture_output=True, text=True, timeout=300)
    lines = [l for l in out.stdout.splitlines() if l.startswith("N=")]
    assert out.returncode == 0 and out.stdout.strip().endswith("OK"), out.stdout
    assert len(lines) == 7
    for l in lines:
        m = re.search(r"(\d+) quotients, (\d+) differ .* = 2\^(-?[\d.]+)", l)
        assert m and int(m.group(1)) > 0 and int(m.group(2)) == 0 and float(m.group(3)) < -44, l
