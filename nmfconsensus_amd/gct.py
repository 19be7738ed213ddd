"""GCT 1.2 / RES dataset I/O -- mirror of nmf.r's read.gct / read.res / write.gct / read.dataset.

read.gct  (nmf.r:371-377): read.delim(skip=2, header=T, row.names=1) then drop the Description column.
read.res  (nmf.r:351-369): sample labels = header fields 3, 5, 7, ... (1-based; R's strsplit drops a trailing
                           empty field); body after 3 skipped lines, row names from column 2 (Accession), values
                           from the even columns after it (the odd ones are the A/P/M calls, dropped).
write.gct (nmf.r:379-408): "#1.2", dims, a header "Name\tDescription\t1..ncol" + column names, then rows
                           with the row name repeated as Name and Description.
Values are parsed with Python's correctly rounded float(); R's own R_strtod is not pinned here
(no R in the image), see DESIGN.md.
"""
from __future__ import annotations

import numpy as np


class GCT:
    """A parsed GCT: `data` is an (genes x samples) float64 array in Fortran order (libnmf's layout)."""

    def __init__(self, data: np.ndarray, row_names: list[str], col_names: list[str]):
        self.data = np.asfortranarray(data, dtype=np.float64)
        self.row_names = list(row_names)
        self.col_names = list(col_names)

    @property
    def shape(self):
        return self.data.shape


def read_gct(path: str) -> GCT:
    with open(path, "r") as f:
        lines = f.read().splitlines()
    if not lines or not lines[0].startswith("#1.2"):
        raise ValueError(f"{path}: not a GCT 1.2 file")
    dims = lines[1].split("\t")
    nrow, ncol = int(dims[0]), int(dims[1])
    header = lines[2].split("\t")
    col_names = header[2:2 + ncol]
    rows, names = [], []
    for ln in lines[3:]:
        if not ln.strip():
            continue  # blank.lines.skip=T
        parts = ln.split("\t")
        names.append(parts[0])
        rows.append([float(x) for x in parts[2:2 + ncol]])
    data = np.array(rows, dtype=np.float64)
    if data.shape != (nrow, ncol):
        raise ValueError(f"{path}: header says {nrow}x{ncol}, body has {data.shape}")
    return GCT(data, names, col_names)


def read_res(path: str) -> GCT:
    with open(path, "r") as f:
        lines = f.read().splitlines()
    if len(lines) < 3:
        raise ValueError(f"{path}: not a RES file (fewer than 3 header lines)")
    head = lines[0].split("\t")
    while head and head[-1] == "":
        head.pop()                      # strsplit("a\tb\t", "\t") is c("a", "b")
    labels = head[2::2]
    rows, names = [], []
    for ln in lines[3:]:
        if not ln.strip():
            continue                    # blank.lines.skip=T
        parts = ln.split("\t")
        if len(parts) < 3:
            raise ValueError(f"{path}: data line with {len(parts)} fields")
        names.append(parts[1])          # row.names = 2
        rows.append([float(x) for x in parts[2::2]])
    if not rows:
        raise ValueError(f"{path}: no data lines")
    ncols = {len(r) for r in rows}
    if len(ncols) != 1:
        raise ValueError(f"{path}: ragged data lines ({sorted(ncols)} value columns)")
    if len(set(names)) != len(names):
        raise ValueError(f"{path}: duplicate row names (read.delim row.names=2 refuses them)")
    data = np.array(rows, dtype=np.float64)
    if data.shape[1] != len(labels):
        raise ValueError(f"{path}: {len(labels)} sample labels for {data.shape[1]} value columns")
    return GCT(data, names, labels)


def read_dataset(path: str) -> GCT:
    """nmf.r:261-269: dispatch on the file suffix, .gct first, then .res (case-insensitive)."""
    low = path.lower()
    if low.endswith(".gct"):
        return read_gct(path)
    if low.endswith(".res"):
        return read_res(path)
    raise ValueError("Input is not a res or gct file.")


def _fmt(v) -> str:
    if isinstance(v, (float, np.floating)):
        return repr(float(v)) if not float(v).is_integer() else str(int(v))
    return str(v)


def write_gct(data, row_names, col_names, path: str) -> None:
    """nmf.r:379-408 layout."""
    data = np.asarray(data)
    if data.ndim == 1:
        data = data[:, None]
    nr, nc = data.shape
    with open(path, "w") as f:
        f.write("#1.2\n")
        f.write(f"{nr}\t{nc}\n")
        f.write("Name\tDescription\t" + "\t".join(str(i + 1) for i in range(nc)))
        for c in col_names:
            f.write("\t" + str(c))
        f.write("\n")
        for i in range(nr):
            f.write(str(row_names[i]) + "\t" + str(row_names[i]) + "\t" + "\t".join(_fmt(v) for v in data[i]) + "\n")
