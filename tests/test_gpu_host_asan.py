"""The engine's host code under AddressSanitizer + UndefinedBehaviorSanitizer on a real GPU.

tests/sanitize/engine_driver.c (C, no Python or torch in the process) drives the small-shape sweep, the MFMA engine
(two runs and a sharded run with caller init on one engine: packing, repacks, tile choices, tail kernels, stop
polling), the drop-in nmf_mu on the solo / team / generic paths, a Brunet sweep and the cophenetic step.  It is built
twice by `make -C tests/sanitize` (here, on the CPU): against the product library, and against a libnmf whose HOST
side is compiled with -Xarch_host -fsanitize=address,undefined (device code untouched -- the pool runs no GPU
sanitizer).  On the GPU both must exit 0, the sanitized one without a report, and their outputs (counts,
iterations, labels, W / H) must be identical bytes: instrumenting the host changes no result."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = os.path.join(ROOT, "tests", "sanitize", "build")
PLAIN, ASAN = os.path.join(B, "engine_driver"), os.path.join(B, "engine_driver_asan")
pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not (os.path.exists(PLAIN) and os.path.exists(ASAN)),
                    reason="host-sanitizer drivers not built (make -C tests/sanitize)")
def test_engine_host_code_under_asan_ubsan(tmp_path):
    outs = []
    for exe, tag in ((PLAIN, "plain"), (ASAN, "asan")):
        d = tmp_path / tag
        d.mkdir()
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:protect_shadow_gap=0",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
        r = subprocess.run([exe, str(d)], capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0 and "engine driver ok" in r.stdout, (tag, r.stdout[-2000:], r.stderr[-6000:])
        assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-6000:]
        outs.append((d / "engine_driver.bin").read_bytes())
    assert len(outs[0]) > 0 and outs[0] == outs[1]
