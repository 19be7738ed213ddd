import hashlib
import os

import numpy as np

from nmfconsensus_amd.gct import read_gct, write_gct


def test_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    X = rng.random((7, 3)) * 10
    p = str(tmp_path / "x.gct")
    write_gct(X, [f"g{i}" for i in range(7)], ["a", "b", "c"], p)
    g = read_gct(p)
    assert g.shape == (7, 3)
    assert np.array_equal(g.data, X)
    assert g.row_names[0] == "g0"
    # write.gct (nmf.r:384-391) writes the column indices 1..ncol and then the names into the header
    assert open(p).read().splitlines()[2] == "Name\tDescription\t1\t2\t3\ta\tb\tc"
    assert open(p).readline() == "#1.2\n"


def test_golden_matrix_is_the_bundled_gct(golden):
    path = "/root/reference/20+20x1000.gct"
    A = golden["A_gct"]
    assert A.shape == (1000, 40)
    assert 0.09 < A.min() and A.max() < 6.2
    if os.path.exists(path):   # build container only
        assert hashlib.sha256(open(path, "rb").read()).digest() == bytes(golden["gct_sha256"])
        assert np.array_equal(read_gct(path).data, A)
