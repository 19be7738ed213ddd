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


RES_TEXT = (
    "Description\tAccession\tS1\t\tS2\t\tS3\t\n"          # read.res header (nmf.r:355-358); trailing tab dropped
    "\tsample descriptions\t\t\t\t\t\n"
    "3\n"
    "gene one\tG1\t1.5\tP\t2\tA\t0.25\tM\n"
    "\n"                                                  # blank.lines.skip=T
    "gene two\tG2\t3\tP\t4.75\tP\t5\tP\n"
    "gene three\tG3\t-1e-3\tA\t6\tM\t7.125\tP\n"
)


def test_read_res(tmp_path):
    from nmfconsensus_amd.gct import read_dataset, read_res

    p = tmp_path / "x.RES"
    p.write_text(RES_TEXT)
    g = read_res(str(p))
    assert g.col_names == ["S1", "S2", "S3"]
    assert g.row_names == ["G1", "G2", "G3"]              # row.names = 2 (Accession)
    assert np.array_equal(g.data, [[1.5, 2, 0.25], [3, 4.75, 5], [-1e-3, 6, 7.125]])
    assert g.data.flags.f_contiguous
    assert np.array_equal(read_dataset(str(p)).data, g.data)   # suffix dispatch is case-insensitive


def test_read_res_errors(tmp_path):
    import pytest

    from nmfconsensus_amd.gct import read_dataset, read_res

    bad = tmp_path / "dup.res"
    bad.write_text(RES_TEXT.replace("\tG2\t", "\tG1\t"))
    with pytest.raises(ValueError, match="duplicate"):
        read_res(str(bad))
    ragged = tmp_path / "ragged.res"
    ragged.write_text(RES_TEXT.replace("\t0.25\tM", ""))
    with pytest.raises(ValueError, match="ragged"):
        read_res(str(ragged))
    other = tmp_path / "x.txt"
    other.write_text("x")
    with pytest.raises(ValueError, match="Input is not a res or gct file"):
        read_dataset(str(other))
