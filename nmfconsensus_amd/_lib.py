"""ctypes binding of nmfconsensus_amd/libnmf.so (the HIP engine, C ABI of include/*.h).

There is no CPU fallback: if the library is missing, importing the bindings raises.  Build it with
`python -m nmfconsensus_amd.build` (hipcc, gfx950).
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NMFC_LIB", os.path.join(HERE, "lib", "libnmf.so"))

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)
c_int = ctypes.c_int

STOP_FIXED, STOP_REF_COMPAT, STOP_ARGMAX_STABLE, STOP_TOLX = 0, 1, 2, 3
LABEL_ARGMAX, LABEL_R_ORDER = 0, 1
INIT_LIBNMF, INIT_R_RUNIF = 0, 1
KID_WTA, KID_HUPD, KID_AHTW, KID_INIT, KID_OTHER, KID_LABELS, KID_COUNTS, KID_SMALL = 0, 1, 2, 3, 4, 5, 6, 7


class SweepOpts(ctypes.Structure):
    _fields_ = [("maxiter", c_int), ("stop_rule", c_int), ("label_rule", c_int), ("seed", ctypes.c_uint32),
                ("min_init", c_int), ("max_init", c_int), ("job_begin", c_int), ("job_end", c_int),
                ("check_every", c_int), ("verbose", c_int), ("TolX", ctypes.c_double), ("TolFun", ctypes.c_double),
                ("init_stream", c_int)]


class Result(ctypes.Structure):
    _fields_ = [("counts", _ip), ("counts_on_device", c_int), ("consensus", _dp), ("labels", _ip),
                ("iters", _ip), ("stopped_early", _ip), ("W", _dp), ("H", _dp),
                ("seconds_total", ctypes.c_double), ("seconds_iterate", ctypes.c_double),
                ("restart_iterations", ctypes.c_longlong), ("max_iter_run", c_int)]


class BrunetOpts(ctypes.Structure):
    _fields_ = [("maxiter", c_int), ("stopconv", c_int), ("stopfreq", c_int), ("seed", ctypes.c_uint32),
                ("restart_begin", c_int), ("restart_end", c_int), ("verbose", c_int), ("lanes", c_int)]


BK_HNUM, BK_HUPD, BK_WUPD = 0, 1, 2


class OptionsT(ctypes.Structure):
    """options_t (libnmf/include/common.h:92-105)."""
    _fields_ = [("rep", c_int), ("init", c_int), ("min_init", c_int), ("max_init", c_int),
                ("w_out", ctypes.c_char_p), ("h_out", ctypes.c_char_p), ("TolX", ctypes.c_double),
                ("TolFun", ctypes.c_double), ("nndsvd_maxiter", c_int), ("nndsvd_blocksize", c_int),
                ("nndsvd_tol", ctypes.c_double), ("nndsvd_ncv", c_int)]


EXPORTED = [
    # include/libnmf_compat.h
    "nmf_mu", "set_default_opts", "checkArguments", "checkMatrices", "randnumber", "generateMatrix",
    "calculateNorm", "calculateMaxchange",
    # include/nmfc.h
    "nmfc_engine_create", "nmfc_engine_destroy", "nmfc_engine_device", "nmfc_current_device", "nmfc_engine_mu1", "nmfc_mu_generic", "nmfc_mu_solo_fits", "nmfc_mu_solo", "nmfc_brunet_device", "nmfc_default_opts", "nmfc_engine_run", "nmfc_sweep",
    "nmfc_consensus", "nmfc_cophenetic", "nmfc_cophenetic_batch", "nmfc_cutree", "nmfc_last_error", "nmfc_version", "nmfc_engine_kernel_time",
    "nmfc_engine_set_timing", "nmfc_engine_kernel_flops", "nmfc_engine_kernel_bytes",
    "nmfc_calculate_norm_dev", "nmfc_calculate_maxchange_dev", "nmfc_nmf_mu_release",
    "nmfc_brunet_default_opts", "nmfc_brunet_create", "nmfc_brunet_destroy", "nmfc_brunet_run",
    "nmfc_brunet_set_timing", "nmfc_brunet_kernel_time", "nmfc_build_tuning", "nmfc_build_tuning_brunet",
]

_LIB = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    # One HIP runtime per process: libnmf.so and torch both bind the SONAME libamdhip64.so.7.  If torch
    # is importable, load it first so that a later torch.cuda call (bench.py, multi-GPU all-reduce) and
    # the engine share torch's already-loaded runtime instead of torch failing to initialise a second one.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: the HIP engine is not built (python -m nmfconsensus_amd.build)")
    L = ctypes.CDLL(LIB_PATH)
    ip = ctypes.POINTER(c_int)
    L.nmf_mu.argtypes = [_dp, _dp, _dp, ip, ip, ip, ip, _dp, _dp]
    L.nmf_mu.restype = ctypes.c_double
    L.set_default_opts.argtypes = [ctypes.POINTER(OptionsT)]
    L.set_default_opts.restype = None
    L.checkArguments.argtypes = [ctypes.c_char_p, c_int, c_int, ctypes.c_char_p, ctypes.c_char_p,
                                 ctypes.POINTER(OptionsT)]
    L.checkArguments.restype = c_int
    L.checkMatrices.argtypes = [_dp, _dp, _dp, c_int, c_int, c_int]
    L.checkMatrices.restype = c_int
    L.randnumber.argtypes = [c_int, c_int]
    L.randnumber.restype = ctypes.c_double
    L.generateMatrix.argtypes = [ip, ip, ip, ip, ip, ip, _dp, _dp, _dp, ctypes.c_void_p]
    L.generateMatrix.restype = None
    L.calculateNorm.argtypes = [_dp, _dp, _dp, _dp, c_int, c_int, c_int]
    L.calculateNorm.restype = ctypes.c_double
    L.calculateMaxchange.argtypes = [_dp, _dp, c_int, c_int, ctypes.c_double]
    L.calculateMaxchange.restype = ctypes.c_double
    L.nmfc_engine_create.argtypes = [c_int, ctypes.c_void_p, c_int, c_int, c_int]
    L.nmfc_engine_create.restype = ctypes.c_void_p
    L.nmfc_engine_destroy.argtypes = [ctypes.c_void_p]
    L.nmfc_engine_destroy.restype = None
    L.nmfc_engine_device.argtypes = [ctypes.c_void_p]
    L.nmfc_engine_device.restype = c_int
    L.nmfc_current_device.argtypes = []
    L.nmfc_current_device.restype = c_int
    L.nmfc_engine_mu1.argtypes = [ctypes.c_void_p, c_int, c_int, c_int, _dp, _dp, _dp, _dp, ip, ip]
    L.nmfc_engine_mu1.restype = c_int
    L.nmfc_mu_generic.argtypes = [_dp, c_int, c_int, c_int, c_int, c_int, _dp, _dp, ip, ip]
    L.nmfc_mu_generic.restype = c_int
    L.nmfc_mu_solo_fits.argtypes = [c_int, c_int, c_int]
    L.nmfc_mu_solo_fits.restype = c_int
    L.nmfc_mu_solo.argtypes = [_dp, c_int, c_int, c_int, c_int, c_int, _dp, _dp, _dp, _dp, ip, ip]
    L.nmfc_mu_solo.restype = c_int
    L.nmfc_brunet_device.argtypes = [ctypes.c_void_p]
    L.nmfc_brunet_device.restype = c_int
    L.nmfc_default_opts.argtypes = [ctypes.POINTER(SweepOpts)]
    L.nmfc_default_opts.restype = None
    L.nmfc_engine_run.argtypes = [ctypes.c_void_p, _ip, c_int, c_int, ctypes.POINTER(SweepOpts), _dp, _dp,
                                  ctypes.POINTER(Result)]
    L.nmfc_engine_run.restype = c_int
    L.nmfc_sweep.argtypes = [_dp, c_int, c_int, _ip, c_int, c_int, ctypes.POINTER(SweepOpts), ctypes.POINTER(Result)]
    L.nmfc_sweep.restype = c_int
    L.nmfc_consensus.argtypes = [_dp, c_int, c_int, c_int, c_int, _ip, _ip, _dp]
    L.nmfc_consensus.restype = c_int
    L.nmfc_cophenetic.argtypes = [_dp, c_int, _ip, _ip, _dp]
    L.nmfc_cophenetic.restype = ctypes.c_double
    L.nmfc_cophenetic_batch.argtypes = [_dp, c_int, c_int, c_int, _dp, _ip, _ip, _dp]
    L.nmfc_cophenetic_batch.restype = c_int
    L.nmfc_cutree.argtypes = [_ip, c_int, c_int, _ip]
    L.nmfc_cutree.restype = c_int
    L.nmfc_last_error.argtypes = []
    L.nmfc_last_error.restype = ctypes.c_char_p
    L.nmfc_version.argtypes = []
    L.nmfc_version.restype = ctypes.c_char_p
    L.nmfc_engine_kernel_time.argtypes = [ctypes.c_void_p, c_int, _dp]
    L.nmfc_engine_kernel_time.restype = ctypes.c_longlong
    L.nmfc_engine_set_timing.argtypes = [ctypes.c_void_p, c_int]
    L.nmfc_engine_set_timing.restype = None
    L.nmfc_engine_kernel_flops.argtypes = [ctypes.c_void_p, c_int]
    L.nmfc_engine_kernel_flops.restype = ctypes.c_double
    L.nmfc_engine_kernel_bytes.argtypes = [ctypes.c_void_p, c_int, _dp]
    L.nmfc_engine_kernel_bytes.restype = ctypes.c_double
    vp = ctypes.c_void_p
    L.nmfc_calculate_norm_dev.argtypes = [vp, vp, vp, vp, c_int, c_int, c_int, _dp, _dp, vp]
    L.nmfc_calculate_norm_dev.restype = c_int
    L.nmfc_calculate_maxchange_dev.argtypes = [vp, vp, c_int, c_int, ctypes.c_double, _dp, _dp, vp]
    L.nmfc_nmf_mu_release.argtypes = []
    L.nmfc_nmf_mu_release.restype = None
    L.nmfc_calculate_maxchange_dev.restype = c_int
    L.nmfc_brunet_default_opts.argtypes = [ctypes.POINTER(BrunetOpts)]
    L.nmfc_brunet_default_opts.restype = None
    L.nmfc_brunet_create.argtypes = [c_int, ctypes.c_void_p, c_int, c_int, c_int]
    L.nmfc_brunet_create.restype = ctypes.c_void_p
    L.nmfc_brunet_destroy.argtypes = [ctypes.c_void_p]
    L.nmfc_brunet_destroy.restype = None
    L.nmfc_brunet_run.argtypes = [ctypes.c_void_p, _ip, c_int, c_int, ctypes.POINTER(BrunetOpts), _dp, _dp,
                                  ctypes.POINTER(Result)]
    L.nmfc_brunet_run.restype = c_int
    L.nmfc_brunet_set_timing.argtypes = [ctypes.c_void_p, c_int]
    L.nmfc_brunet_set_timing.restype = None
    L.nmfc_brunet_kernel_time.argtypes = [ctypes.c_void_p, c_int, _dp, _dp]
    L.nmfc_brunet_kernel_time.restype = ctypes.c_longlong
    _LIB = L
    return L


def last_error() -> str:
    return lib().nmfc_last_error().decode()
