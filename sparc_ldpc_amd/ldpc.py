"""LDPC outer code of the joint decoder: mirror of the reference's ``ldpc.code``
(ldpc/py/ldpc.py:6-943) with belief propagation running on the GPU.

``code(standard, rate, z, ptype)`` builds the same Tanner graph
(``vdeg``, ``cdeg``, ``intrlv``: identical arrays, ldpc.py:694-786) from the
same base matrices (``data/protographs.json``), encodes systematically
(ldpc.py:790-850) and decodes through ``libldpc_bp.so``
(include/ldpc_bp.h), the HIP replacement of ``bin/c_ldpc.so``.  The decoder
returns ``(app, it)`` like ldpc.py:855-930; ``decode_batch`` decodes many
words of one code in one launch.  There is no CPU decoder: without the
library or a HIP device, decoding raises.
"""
from __future__ import annotations

import ctypes as ct
import functools
import json
import os

import numpy as np

MAX_ITCOUNT = 200  # ldpc.py:4 / c_ldpc.c:7

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LDPC_BP_LIB") or os.path.join(_HERE, "libldpc_bp.so")

LB_SUMPROD2, LB_SUMPROD, LB_MINSUM = 0, 1, 2
_ALGOS = {"sumprod2": LB_SUMPROD2, "sumprod": LB_SUMPROD, "minsum": LB_MINSUM}

# Every symbol include/ldpc_bp.h declares (tests check the export table).
EXPORTS = (
    "sumprod", "sumprod2", "minsum", "Lxor", "Lxfb",
    "lb_create", "lb_destroy", "lb_decode", "lb_decode_device", "lb_stage", "lb_run", "lb_wait",
    "lb_fetch", "lb_run_event_ms", "lb_info", "lb_device_count", "lb_last_error", "lb_version",
    "lb_buffers", "lb_set_tail",
)

_P, _I, _D = ct.c_void_p, ct.c_int, ct.POINTER(ct.c_double)
_LP = ct.POINTER(ct.c_long)
_SIG = {
    "sumprod": (_I, [_D, _LP, _LP, _LP, _I, _I, _I, _D]),
    "sumprod2": (_I, [_D, _LP, _LP, _LP, _I, _I, _I, _D]),
    "minsum": (_I, [_D, _LP, _LP, _LP, _I, _I, _I, _D, ct.c_double]),
    "Lxor": (ct.c_double, [ct.c_double, ct.c_double, _I]),
    "Lxfb": (ct.c_double, [_D, ct.c_long, _I]),
    "lb_create": (_I, [ct.POINTER(_P), _LP, _LP, _LP, _I, _I, _I, _I]),
    "lb_destroy": (None, [_P]),
    "lb_decode": (_I, [_P, _I, _D, _D, ct.POINTER(ct.c_int), _I, ct.c_double, _I]),
    "lb_decode_device": (_I, [_P, _I, _P, _P, _P, _I, ct.c_double, _I]),
    "lb_stage": (_I, [_P, _I, _D]),
    "lb_buffers": (_I, [_P, _I, ct.POINTER(_P), ct.POINTER(_P), ct.POINTER(_P)]),
    "lb_run": (_I, [_P, _I, _I, ct.c_double, _I]),
    "lb_wait": (_I, [_P]),
    "lb_fetch": (_I, [_P, _I, _D, ct.POINTER(ct.c_int)]),
    "lb_run_event_ms": (ct.c_double, [_P]),
    "lb_info": (_I, [_P, ct.POINTER(ct.c_int64)]),
    "lb_set_tail": (_I, [_P, _I]),
    "lb_device_count": (_I, []),
    "lb_last_error": (ct.c_char_p, []),
    "lb_version": (ct.c_char_p, []),
}

_lib = None


class LdpcBpError(RuntimeError):
    """A negative status from libldpc_bp.so."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libldpc_bp error {code}: {msg}")
        self.code = code


def load_bp_library(path: str = LIB_PATH) -> ct.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with __graft_entry__.build() "
                          "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ct.CDLL(path)
    for name, (res, args) in _SIG.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older build (A/B runs): the entry point stays absent
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int) -> None:
    if rc < 0:
        msg = load_bp_library().lb_last_error().decode(errors="replace")
        if rc == -1:
            raise AssertionError(msg)
        raise LdpcBpError(rc, msg)


@functools.lru_cache(maxsize=None)
def _protographs():
    with open(os.path.join(_HERE, "data", "protographs.json")) as fh:
        return json.load(fh)["protographs"]


def assign_proto(standard, rate, z, ptype="A"):
    """Base matrix for (standard, rate[, ptype / z]) — ldpc.py:26-663, same errors."""
    tab = _protographs()
    if standard == "802.11n":
        if z not in (27, 54, 81):
            raise NameError("802.11n invalid z (must be 27,54 or 81)")
        by_rate = tab["802.11n"][str(z)]
        if rate not in by_rate:
            raise UnboundLocalError(f"no 802.11n protograph for rate {rate!r}")
        return np.array(by_rate[rate], dtype=np.int64)
    if standard not in tab["z_free"]:
        raise NameError("IEEE standard unknown")
    by_rate = tab["z_free"][standard]
    if rate not in by_rate:
        raise UnboundLocalError(f"no {standard} protograph for rate {rate!r}")
    by_type = by_rate[rate]
    if ptype not in by_type:
        if len(by_type) == 1:  # ptype is ignored for single-type rates (ldpc.py:43-45)
            return np.array(next(iter(by_type.values())), dtype=np.int64)
        raise UnboundLocalError(f"no {standard} rate {rate} protograph of type {ptype!r}")
    return np.array(by_type[ptype], dtype=np.int64)


def tanner_graph(proto: np.ndarray, z: int):
    """(vdeg, cdeg, intrlv) — the arrays of ldpc.py:694-786.

    The reference assigns ports while walking the protograph row by row
    (np.nonzero order), so check node (r, k)'s ports follow the columns of
    row r and variable node (c, k')'s ports follow the rows of column c.  With
    those two ranks the interleaver is written directly: entry (r, c) with
    shift s links check r*z+k to variable c*z+(k+s)%z."""
    proto = np.asarray(proto, dtype=np.int64)
    on = proto != -1
    cdeg = np.repeat(on.sum(1), z).astype(np.int64)
    vdeg = np.repeat(on.sum(0), z).astype(np.int64)
    cfirst = np.concatenate([[0], np.cumsum(cdeg)[:-1]])
    vfirst = np.concatenate([[0], np.cumsum(vdeg)[:-1]])
    cport = np.cumsum(on, 1) - 1
    vport = np.cumsum(on, 0) - 1
    r, c = np.nonzero(on)
    k = np.arange(z)[None, :]
    chk = r[:, None] * z + k
    var = c[:, None] * z + (k + proto[r, c][:, None]) % z
    intrlv = np.empty(int(cdeg.sum()), dtype=np.int64)
    intrlv[(vfirst[var] + vport[r, c][:, None]).ravel()] = (cfirst[chk] + cport[r, c][:, None]).ravel()
    return vdeg, cdeg, intrlv


def encode_batch(proto: np.ndarray, z: int, U) -> np.ndarray:
    """Systematic encoding of B information words (rows of U) — ldpc.py:790-850.

    Works on (B, Np, z) blocks: the systematic syndromes p_j, their sum gives
    the first parity block (after undoing the single surviving shift of column
    Kp), then the dual-diagonal recursion yields the remaining parity blocks."""
    proto = np.asarray(proto, dtype=np.int64)
    Mp, Np = proto.shape
    Kp = Np - Mp
    U = np.atleast_2d(np.asarray(U, dtype=np.int64))
    if U.shape[1] != Kp * z:
        raise NameError("information word length not compatible with proto and z")
    B = U.shape[0]
    x = np.zeros((B, Np, z), dtype=np.int64)
    x[:, :Kp] = U.reshape(B, Kp, z)
    p = np.zeros((B, Mp, z), dtype=np.int64)
    for j in range(Mp):
        for k in np.nonzero(proto[j, :Kp] != -1)[0]:
            p[:, j] ^= np.roll(x[:, k], -proto[j, k], axis=-1)
    col = proto[:, Kp]
    shifts = np.bincount(col[col != -1] % z, minlength=z) % 2
    nz = np.nonzero(shifts)[0]
    if len(nz) != 1:
        raise NameError("The offsets in colum Kp+1 of proto do not add to a single offset")
    x[:, Kp] = np.roll(np.bitwise_xor.reduce(p, axis=1), nz[0], axis=-1)
    for j in range(Mp - 1):
        m = Kp + j + 1
        acc = p[:, j].copy()
        for k in np.nonzero(proto[j, Kp:m] != -1)[0]:
            acc ^= np.roll(x[:, Kp + k], -proto[j, Kp + k], axis=-1)
        x[:, m] = acc
    return x.reshape(B, Np * z)


class code:
    """Drop-in for ``ldpc.code`` (ldpc/py/ldpc.py:6-24): same attributes
    (standard, rate, z, ptype, proto, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, N, K)
    and methods (assign_proto, pcmat, prepare_decoder, encode, decode, Lxor,
    Lxfb), plus ``encode_batch`` / ``decode_batch`` for Monte-Carlo."""

    def __init__(self, standard="802.11n", rate="1/2", z=27, ptype="A", device=None):
        self.standard = standard
        self.rate = rate
        self.z = z
        self.ptype = ptype
        self.proto = self.assign_proto()
        vdeg, cdeg, intrlv = self.prepare_decoder()
        self.vdeg = vdeg
        self.cdeg = cdeg
        self.intrlv = intrlv
        self.Nv = len(vdeg)
        self.Nc = len(cdeg)
        self.Nmsg = len(intrlv)
        self.N = self.Nv
        self.K = self.Nv - self.Nc
        self._device = device
        self._ctx = None

    # -- construction ---------------------------------------------------------
    def assign_proto(self):
        return assign_proto(self.standard, self.rate, self.z, self.ptype)

    def pcmat(self):
        """Dense parity-check matrix (ldpc.py:666-691)."""
        z = self.z
        H = np.zeros((z * self.proto.shape[0], z * self.proto.shape[1]), dtype=int)
        eye = np.eye(z, dtype=int)
        for r, c in zip(*np.nonzero(self.proto != -1)):
            H[r * z:(r + 1) * z, c * z:(c + 1) * z] = np.roll(eye, self.proto[r, c] % z, 1)
        return H

    def prepare_decoder(self):
        return tanner_graph(self.proto, self.z)

    def encode(self, info):
        return encode_batch(self.proto, self.z, np.asarray(info).reshape(1, -1))[0]

    def encode_batch(self, U):
        return encode_batch(self.proto, self.z, U)

    # -- decoding (GPU) ---------------------------------------------------------
    def _context(self):
        if self._ctx is None:
            lib = load_bp_library()
            dev = self._device
            if dev is None:
                ndev = lib.lb_device_count()
                if ndev <= 0:
                    raise LdpcBpError(-6, "no HIP device visible (MI355X required; no CPU decoder)")
                env = os.environ.get("SPARC_AMP_DEVICE", os.environ.get("LOCAL_RANK", "0"))
                dev = int(env) if 0 <= int(env) < ndev else 0
            ctx = ct.c_void_p()
            v = np.ascontiguousarray(self.vdeg, dtype=np.int64)
            c = np.ascontiguousarray(self.cdeg, dtype=np.int64)
            il = np.ascontiguousarray(self.intrlv, dtype=np.int64)
            _check(lib.lb_create(ct.byref(ctx), v.ctypes.data_as(_LP), c.ctypes.data_as(_LP),
                                 il.ctypes.data_as(_LP), self.Nv, self.Nc, self.Nmsg, int(dev)))
            self._ctx = ctx
        return self._ctx

    def decode_batch(self, CH, dectype="sumprod2", corr_factor=0.7, max_iter=MAX_ITCOUNT):
        """Decode B words (rows of CH, channel LLRs) -> (app (B, N) float64, it (B,) int)."""
        if dectype not in _ALGOS:
            raise NameError("Decoder type unknonwn")
        CH = np.ascontiguousarray(np.atleast_2d(CH), dtype=np.float64)
        if CH.shape[1] != self.Nv:
            raise NameError("Channel inputs not consistent with variable degrees")
        B = CH.shape[0]
        app = np.empty((B, self.Nv), dtype=np.float64)
        it = np.empty(B, dtype=np.intc)
        lib = load_bp_library()
        _check(lib.lb_decode(self._context(), B, CH.ctypes.data_as(_D), app.ctypes.data_as(_D),
                             it.ctypes.data_as(ct.POINTER(ct.c_int)), _ALGOS[dectype],
                             float(corr_factor), int(max_iter)))
        return app, it.astype(np.int64)

    def device_buffers(self, B):
        """Device pointers (ch, app, iters) of the decoder's buffers for B words."""
        ch, app, it = ct.c_void_p(), ct.c_void_p(), ct.c_void_p()
        _check(load_bp_library().lb_buffers(self._context(), int(B), ct.byref(ch), ct.byref(app), ct.byref(it)))
        return ch.value, app.value, it.value

    def run_buffers(self, B, dectype="sumprod2", corr_factor=0.7, max_iter=MAX_ITCOUNT):
        """Decode the B words in the device ch buffer into the app buffer (blocking)."""
        lib = load_bp_library()
        _check(lib.lb_run(self._context(), int(B), _ALGOS[dectype], float(corr_factor), int(max_iter)))
        _check(lib.lb_wait(self._context()))

    def fetch_buffers(self, B, app=True):
        """(app (B, N) or None, iters (B,)) from the device buffers."""
        a = np.empty((B, self.Nv)) if app else None
        it = np.empty(B, dtype=np.intc)
        _check(load_bp_library().lb_fetch(self._context(), int(B), None if a is None else a.ctypes.data_as(_D),
                                          it.ctypes.data_as(ct.POINTER(ct.c_int))))
        return a, it.astype(np.int64)

    def decode(self, ch, dectype="sumprod2", corr_factor=0.7):
        """ldpc.py:855-930: (app, it) for one word of channel LLRs."""
        ch = np.asarray(ch, dtype=np.float64).reshape(-1)
        if len(ch) != len(self.vdeg):
            raise NameError("Channel inputs not consistent with variable degrees")
        app, it = self.decode_batch(ch[None, :], dectype, corr_factor)
        return app[0], int(it[0])

    def info(self):
        out = (ct.c_int64 * 10)()
        _check(load_bp_library().lb_info(self._context(), out))
        keys = ("Nv", "Nc", "Nmsg", "max_vdeg", "max_cdeg", "lds_messages", "threads", "device", "fixed_dc",
                "tail_at")
        return dict(zip(keys, list(out)))

    def set_tail(self, tail_at=-1):
        """First iteration of the tail launches (words still running after it
        are spread over several workgroups each; bit-identical).  -1: the
        default, 0: off (include/ldpc_bp.h lb_set_tail)."""
        _check(load_bp_library().lb_set_tail(self._context(), int(tail_at)))

    def Lxor(self, L1, L2, corrflag=1):
        """ldpc.py:932-935 (evaluated on the GPU)."""
        r = load_bp_library().Lxor(float(L1), float(L2), int(corrflag))
        if r != r and not (np.isnan(L1) or np.isnan(L2)):
            _check(-2)
        return r

    def Lxfb(self, L, corrflag=1):
        """ldpc.py:937-943: (aggregate LLR, extrinsic LLRs)."""
        L = np.array(L, dtype=float)
        r = load_bp_library().Lxfb(L.ctypes.data_as(_D), len(L), int(corrflag))
        if r != r and not np.isnan(L).any():
            _check(-2)
        return r, L

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and _lib is not None:
            try:
                _lib.lb_destroy(ctx)
            except Exception:
                pass
            self._ctx = None
