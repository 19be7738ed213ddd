"""Builds nmfconsensus_amd/libnmf.so (soname libnmf.so) for gfx950 with hipcc, in-tree.

The library is the product: HIP kernels + the C ABI of include/libnmf_compat.h and include/nmfc.h.
`python -m nmfconsensus_amd.build` or __graft_entry__.build().
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libnmf.so")
SOURCES = ["engine.hip", "compat.hip", "brunet.hip", "generic.hip", "solo.hip", "hclust.cpp"]
HEADERS = ["nmfc_kernels.hpp", "nmfc_tuning.hpp", "lane_pool.hpp", "rmt.hpp", "../../include/nmfc.h", "../../include/libnmf_compat.h"]
ARCH = os.environ.get("NMFC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def source_sha256() -> str:
    """Hash of the engine's kernel + host sources: tags PMC profiles with the code they measured."""
    import hashlib
    h = hashlib.sha256()
    for f in ("nmfc_kernels.hpp", "engine.hip", "nmfc_tuning.hpp"):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    if not force and not _stale(LIB, deps):
        return LIB
    from concurrent.futures import ThreadPoolExecutor

    def compile_one(src):
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ".o")
        lang = [] if src.endswith(".hip") else ["-x", "c++"]
        off = [f"--offload-arch={ARCH}"] if src.endswith(".hip") else []
        cmd = [HIPCC, *off, "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result", "-Wno-unused-function", *lang, "-c",
               os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=CSRC)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "6"))))
    with ThreadPoolExecutor(max_workers=jobs) as pool:   # one hipcc per translation unit, in parallel
        objs = list(pool.map(compile_one, SOURCES))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs,
           "-Wl,-soname,libnmf.so", "-Wl,-rpath,/opt/rocm/lib", "-Wl,-z,defs"]   # an unresolved symbol fails the build
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    for o in objs:
        os.remove(o)
    return LIB


def build_oracle(verbose: bool = True) -> None:
    """Builds the test-only checker: oracle/liboracle.so, and oracle/_ref/libnmf_ref.so when the
    reference sources are present (build container only; the GPU box uses the prebuilt file)."""
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", odir, "liboracle.so"], check=True)
    if os.path.isdir("/root/reference/libnmf"):
        subprocess.run(["make", "-s", "-C", odir, "ref"], check=True)


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    build_oracle()
