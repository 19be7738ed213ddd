"""nmfconsensus_amd -- MI355X-native engine for the NMF consensus restart sweep.

The product is nmfconsensus_amd/libnmf.so (HIP/gfx950, C ABI in include/).  This package holds its
Python bindings and the host-side mirror of the reference's R driver (nmf.r).
"""
from .gct import GCT, read_dataset, read_gct, read_res, write_gct  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not require the built library (CPU-side tooling, build())
    if name in ("Engine", "SweepResult", "doNMF", "createJobArray", "runNMFinJobs",
                "computeConsensusMatrixFromClusterings", "computeConsensusAndSaveFiles", "cophenetic", "cutree",
                "job_grid"):
        from . import nmf
        return getattr(nmf, name)
    raise AttributeError(name)
