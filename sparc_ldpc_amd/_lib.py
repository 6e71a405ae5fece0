"""ctypes binding of the gfx950 HIP library ``libsparc_amp.so`` (include/sparc_amp.h).

The loader follows the reference's own native-boundary pattern
(ldpc/py/ldpc.py:859-872: ``ctypes.CDLL`` + ``ndarray.ctypes`` pointers,
caller-allocated outputs, int status codes) but resolves the library next to
this file instead of relative to the CWD.  There is no CPU fallback: if the
library is missing or no HIP device is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

LIB_NAME = "libsparc_amp.so"
LIB_PATH = os.environ.get("SPARC_AMP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

SA_OK = 0
SA_ERR_ARG = -1
SA_ERR_HIP = -2
SA_ERR_NOMEM = -3
SA_ERR_ORDERING = -4
SA_ERR_UNSUPPORTED = -5
SA_ERR_NO_DEVICE = -6

SA_BACKEND_HADAMARD = 0
SA_BACKEND_DENSE = 1
SA_BACKEND_HOST = 2
SA_BACKEND_MATRIX = 3
SA_PREC_F32 = 0
SA_PREC_F64 = 1
SA_FLAG_NO_EARLY_STOP = 1
SA_FLAG_BETA0 = 0x100
SA_PTR_DEVICE = 0x200

# sa_create_ex plan options (include/sparc_amp.h): overrides of the built-in
# kernel / layout choice rules, by name
SA_PLAN = {
    "SEC3": 1 << 0, "NO_SEC3": 1 << 1, "ROW16": 1 << 2, "NO_ROW16": 1 << 3, "NO_PT": 1 << 4,
    "ZIL": 1 << 5, "NO_ZIL": 1 << 6, "WB8": 1 << 7, "WB16": 1 << 8, "NO_BANKS": 1 << 9, "EAGER": 1 << 10,
    "ONE_PASS": 1 << 11,
}


def plan_bits(plan) -> int:
    """None / an int / an iterable of SA_PLAN names -> the option bits."""
    if plan is None:
        return 0
    if isinstance(plan, int):
        return plan
    if isinstance(plan, str):
        plan = [plan]
    bits = 0
    for name in plan:
        key = name.upper()
        if key not in SA_PLAN:
            raise ValueError(f"unknown plan option {name!r}; known: {sorted(SA_PLAN)}")
        bits |= SA_PLAN[key]
    return bits

# Every symbol include/sparc_amp.h declares (tests check the export table).
EXPORTS = (
    "sa_create", "sa_create_ex", "sa_create_matrix", "sa_create_matrix_random", "sa_subset", "sa_create_twin", "sa_destroy", "sa_Ab", "sa_Az", "sa_amp",
    "sa_reserve", "sa_stage", "sa_stage_power_batch", "sa_run", "sa_wait", "sa_fetch", "sa_fetch_z", "sa_run_event_ms",
    "sa_profile", "sa_profile_rep", "sa_profile_dispatch", "sa_profile_kinds", "sa_decide",
    "sa_decide_async", "sa_decide_collect", "sa_info", "sa_device_count", "sa_last_error", "sa_version",
    "sa_encode", "sa_stage_onehot", "sa_llr", "sa_soft_beta0", "sa_hard_cancel",
    "sa_threshold", "sa_cancel", "sa_plan", "sa_plan_batched", "sa_stage_onehot_scaled", "sa_cancel_scaled",
    "sa_host_init", "sa_host_tau", "sa_host_eta", "sa_host_residual",
    "sa_draw_reps", "sa_mc_stage", "sa_mc_run", "sa_make_ordering",
)

_P = ct.c_void_p
_I = ct.c_int
_D = ct.POINTER(ct.c_double)
_SIG = {
    "sa_create": (_I, [ct.POINTER(_P), _I, _I, _I, ct.POINTER(ct.c_uint32), _I, _I, _I]),
    "sa_create_ex": (_I, [ct.POINTER(_P), _I, _I, _I, ct.POINTER(ct.c_uint32), _I, _I, _I, _I]),
    "sa_create_matrix": (_I, [ct.POINTER(_P), _I, _I, _I, _D, _I, _I]),
    "sa_create_matrix_random": (_I, [ct.POINTER(_P), _I, _I, _I, ct.c_uint64, ct.c_double, _I, _I]),
    "sa_subset": (_I, [_P, ct.POINTER(ct.c_int64), _I, ct.POINTER(_P)]),
    "sa_create_twin": (_I, [_P, ct.POINTER(_P)]),
    "sa_destroy": (None, [_P]),
    "sa_Ab": (_I, [_P, _I, _D, _D]),
    "sa_Az": (_I, [_P, _I, _D, _D]),
    "sa_amp": (_I, [_P, _I, _D, _D, _I, _D, _D, ct.POINTER(ct.c_int), _I]),
    "sa_reserve": (_I, [_P, _I, _I]),
    "sa_stage": (_I, [_P, _I, _D, _D, _D]),
    "sa_stage_power_batch": (_I, [_P, _I, _D]),
    "sa_run": (_I, [_P, _I, _I, _I]),
    "sa_wait": (_I, [_P]),
    "sa_fetch": (_I, [_P, _I, _D, ct.POINTER(ct.c_int)]),
    "sa_fetch_z": (_I, [_P, _I, _D]),
    "sa_run_event_ms": (ct.c_double, [_P]),
    "sa_profile": (_I, [_P, _I, _I, _I, _D]),
    "sa_profile_rep": (_I, [_P, _I, _I, _I, _I, _D]),
    "sa_profile_dispatch": (_I, [_P, _I, _I, _I, _D]),
    "sa_profile_kinds": (_I, []),
    "sa_decide_async": (_I, [_P, _I, _I]),
    "sa_decide_collect": (_I, [_P, _I, _I, ct.POINTER(ct.c_int32)]),
    "sa_decide": (_I, [_P, _I, ct.POINTER(ct.c_int32)]),
    "sa_info": (_I, [_P, ct.POINTER(ct.c_int64)]),
    "sa_device_count": (_I, []),
    "sa_last_error": (ct.c_char_p, []),
    "sa_version": (ct.c_char_p, []),
    "sa_encode": (_I, [_P, _I, ct.POINTER(ct.c_int32), _D]),
    "sa_threshold": (_I, [_P, _I, _I, _I, _P, _I, ct.c_double, ct.POINTER(ct.c_int32)]),
    "sa_cancel": (_I, [_P, _I, ct.POINTER(ct.c_int32), _P]),
    "sa_plan": (_I, [_P, _I, ct.POINTER(ct.c_int64)]),
    "sa_plan_batched": (_I, [_P, _I, ct.POINTER(ct.c_int64)]),
    "sa_stage_onehot": (_I, [_P, _I, ct.POINTER(ct.c_int32)]),
    "sa_stage_onehot_scaled": (_I, [_P, _I, ct.POINTER(ct.c_int32), ct.c_double]),
    "sa_cancel_scaled": (_I, [_P, _I, ct.POINTER(ct.c_int32), ct.c_double, _P]),
    "sa_llr": (_I, [_P, _I, _I, _I, _P, _I]),
    "sa_soft_beta0": (_I, [_P, _I, _I, _I, _P, _I]),
    "sa_hard_cancel": (_I, [_P, _I, _I, _I, _P, _I, _P, ct.POINTER(ct.c_int32)]),
    "sa_host_init": (_I, [_P, _I, _I, _D, _D, _D, _D]),
    "sa_host_tau": (_I, [_P, _I, _I, _I, ct.POINTER(ct.c_int)]),
    "sa_host_eta": (_I, [_P, _I, _I, _I, _D]),
    "sa_host_residual": (_I, [_P, _I, _I, _I, _D]),
    "sa_draw_reps": (_I, [ct.POINTER(ct.c_uint32), _I, _I, _I, _I, ct.c_double, ct.POINTER(ct.c_int32), _D, _I]),
    "sa_mc_stage": (_I, [_P, _I, ct.POINTER(ct.c_int32), _D]),
    "sa_mc_run": (_I, [_P, _I, _I, _I, ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32), _D]),
    "sa_make_ordering": (_I, [_I, _I, _I, ct.c_uint32, ct.POINTER(ct.c_uint32)]),
}

_lib = None

_SRC_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
_INC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")


def source_hash() -> str:
    """SHA-256 (first 16 hex digits) over the HIP sources and headers the
    libraries are built from (csrc/*.hip, csrc/*.h, csrc/Makefile, include/*.h,
    in name order): the identity a committed profile records and bench.py compares
    against, so a roofline figure is only read from a profile of this build."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(_SRC_DIR) if f.endswith((".hip", ".h")) or f == "Makefile")
    paths = [os.path.join(_SRC_DIR, f) for f in files]
    if os.path.isdir(_INC_DIR):
        paths += [os.path.join(_INC_DIR, f) for f in sorted(os.listdir(_INC_DIR)) if f.endswith(".h")]
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


class SparcAmpError(RuntimeError):
    """A non-zero status from libsparc_amp.so."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libsparc_amp error {code}: {msg}")
        self.code = code


def load(path: str = LIB_PATH) -> ct.CDLL:
    """Load (once) and type the library; raises ImportError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ct.CDLL(path)
    for name, (res, args) in _SIG.items():
        # an older build (A/B runs against a previous library) may lack newer
        # entry points: they stay untyped and absent; the export test pins the
        # current build to the full list
        if not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != SA_OK:
        msg = load().sa_last_error().decode(errors="replace")
        if rc == SA_ERR_ARG:
            raise AssertionError(msg)
        raise SparcAmpError(rc, msg)


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_D)


def as_f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)
