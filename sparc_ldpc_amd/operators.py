"""Design operators on the MI355X: the drop-in for ldpc/sparc_ldpc.py:32-168.

``sparc_transforms`` / ``sparc_transforms_shorter`` / ``block_sub_fht`` /
``sub_fht`` keep the reference's names, argument order and return shapes.
The returned ``Ab``/``Az`` are callable objects (so ``x = Ab(β₀)``,
sparc_ldpc.py:439, and ``y - Ab(β)``, :514 / amp_exit.py:111, work
unchanged); each carries the device context that ``amp()`` uses to run the
whole iteration loop on the GPU.
"""
from __future__ import annotations

import hashlib
import os
from collections import OrderedDict

import numpy as np

from . import _lib
from ._lib import as_f64, check, dptr

__all__ = [
    "SparcOperator", "AbOp", "AzOp", "HostOperatorLoop", "make_ordering", "sub_fht", "block_sub_fht",
    "sparc_transforms", "sparc_transforms_shorter", "dense_transforms", "gaussian_transforms", "default_device",
]

_BACKENDS = {"hadamard": _lib.SA_BACKEND_HADAMARD, "dense": _lib.SA_BACKEND_DENSE}
_PRECS = {"fp32": _lib.SA_PREC_F32, "fp64": _lib.SA_PREC_F64}

# Process-wide defaults; bench/tests override through these env vars or kwargs.
DEFAULT_BACKEND = os.environ.get("SPARC_AMP_BACKEND", "hadamard")
DEFAULT_PRECISION = os.environ.get("SPARC_AMP_PRECISION", "fp32")


def default_device() -> int:
    """LOCAL_RANK (one process per GPU) if it names a visible device, else 0."""
    lib = _lib.load()
    ndev = lib.sa_device_count()
    if ndev <= 0:
        raise _lib.SparcAmpError(_lib.SA_ERR_NO_DEVICE, "no HIP device visible (MI355X required)")
    env = os.environ.get("SPARC_AMP_DEVICE", os.environ.get("LOCAL_RANK", "0"))
    d = int(env)
    return d if 0 <= d < ndev else 0


def _w_of(n: int, m: int) -> int:
    # sparc_ldpc.py:52 / :110
    return 2 ** int(np.ceil(np.log2(max(m + 1, n + 1))))


_ORDER_CACHE: "OrderedDict[tuple, np.ndarray]" = OrderedDict()


def make_ordering(L: int, M: int, n: int, seed: int = 0) -> np.ndarray:
    """The reference's row sub-sampling table (sparc_ldpc.py:107-117).

    Legacy ``RandomState(seed)`` (frozen by NEP 19), a *cumulative* shuffle
    of ``arange(1, w, uint32)`` per section, first n kept.  Host-side set-up,
    exactly as in the reference; memoised because every Monte-Carlo rep of
    the reference rebuilds the same seed-0 table (sparc_ldpc.py:433).
    """
    if seed is None:  # RandomState(None): a fresh design from OS entropy, never memoised
        w = _w_of(n, M)
        rng = np.random.RandomState(None)
        ordering = np.empty((L, n), dtype=np.uint32)
        idxs = np.arange(1, w, dtype=np.uint32)
        for ll in range(L):
            rng.shuffle(idxs)
            ordering[ll] = idxs[:n]
        return ordering
    key = (int(L), int(M), int(n), int(seed))
    hit = _ORDER_CACHE.get(key)
    if hit is not None:
        _ORDER_CACHE.move_to_end(key)
        return hit
    # the same shuffles restated natively (sa_make_ordering: NumPy's legacy
    # MT19937 and its 1-d shuffle, bit for bit; tests/test_host.py)
    if not 0 <= int(seed) < 2 ** 32:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    ordering = np.empty((int(L), int(n)), dtype=np.uint32)
    check(_lib.load().sa_make_ordering(int(L), int(M), int(n), int(seed),
                                       ordering.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_uint32))))
    ordering.setflags(write=False)
    _ORDER_CACHE[key] = ordering
    while len(_ORDER_CACHE) > 8:
        _ORDER_CACHE.popitem(last=False)
    return ordering


class SparcOperator:
    """A device-resident SPARC design operator (one ``sa_ctx``)."""

    def __init__(self, L, M, n, ordering, backend=None, precision=None, device=None, plan=None):
        """plan: None (the built-in kernel choice rules) or sa_create_ex plan
        options, an int or names such as ``("SEC3", "NO_ROW16")``."""
        lib = _lib.load()
        backend = backend or DEFAULT_BACKEND
        precision = precision or DEFAULT_PRECISION
        if backend not in _BACKENDS:
            raise ValueError(f"backend must be one of {sorted(_BACKENDS)}")
        if precision not in _PRECS:
            raise ValueError(f"precision must be one of {sorted(_PRECS)}")
        ordering = np.ascontiguousarray(ordering, dtype=np.uint32)
        assert ordering.shape == (L, n), "ordering must be (L, n)"
        self.L, self.M, self.n = int(L), int(M), int(n)
        self.w = _w_of(self.n, self.M)
        self.backend, self.precision = backend, precision
        self.device = default_device() if device is None else int(device)
        self.ordering = ordering
        self.plan_bits = _lib.plan_bits(plan)
        self._ctx = _lib.ct.c_void_p()
        ordp = ordering.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_uint32))
        if self.plan_bits:
            check(lib.sa_create_ex(_lib.ct.byref(self._ctx), self.L, self.M, self.n, ordp,
                                   _BACKENDS[backend], _PRECS[precision], self.device, self.plan_bits))
        else:
            check(lib.sa_create(_lib.ct.byref(self._ctx), self.L, self.M, self.n, ordp,
                                _BACKENDS[backend], _PRECS[precision], self.device))
        self._lib = lib

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                self._lib.sa_destroy(ctx)
            except Exception:
                pass
            self._ctx = None

    @classmethod
    def from_matrix(cls, A, L, M, precision=None, device=None):
        """A caller's own dense design (SA_BACKEND_MATRIX): A is n x (L*M);
        Ab(β) = A β and Az(z) = Aᵀ z as given (no 1/√n), on the device in
        `precision` (GEMVs below 4 codewords, MFMA GEMMs from 4)."""
        lib = _lib.load()
        precision = precision or DEFAULT_PRECISION
        if precision not in _PRECS:
            raise ValueError(f"precision must be one of {sorted(_PRECS)}")
        A = np.ascontiguousarray(A, dtype=np.float64)
        assert A.ndim == 2 and A.shape[1] == L * M, "A must be n x (L*M)"
        self = cls.__new__(cls)
        self.L, self.M, self.n = int(L), int(M), int(A.shape[0])
        self.w = None
        self.backend, self.precision = "matrix", precision
        self.device = default_device() if device is None else int(device)
        self.ordering = None
        self.plan_bits = 0
        self._ctx = _lib.ct.c_void_p()
        check(lib.sa_create_matrix(_lib.ct.byref(self._ctx), self.L, self.M, self.n, dptr(A), _PRECS[precision],
                                   self.device))
        self._lib = lib
        return self

    @classmethod
    def from_random(cls, L, M, n, seed=0, scale=None, precision=None, device=None):
        """An i.i.d. N(0, scale²) design generated on the device (default
        scale 1/√n): sa_create_matrix_random, Philox4x32-10 + Box–Muller,
        reproducible per (seed, element)."""
        lib = _lib.load()
        precision = precision or DEFAULT_PRECISION
        if precision not in _PRECS:
            raise ValueError(f"precision must be one of {sorted(_PRECS)}")
        self = cls.__new__(cls)
        self.L, self.M, self.n = int(L), int(M), int(n)
        self.w = None
        self.backend, self.precision = "matrix", precision
        self.device = default_device() if device is None else int(device)
        self.ordering = None
        self.plan_bits = 0
        self.scale = float(1.0 / np.sqrt(n) if scale is None else scale)
        self._ctx = _lib.ct.c_void_p()
        check(lib.sa_create_matrix_random(_lib.ct.byref(self._ctx), self.L, self.M, self.n, int(seed) & (2**64 - 1),
                                          self.scale, _PRECS[precision], self.device))
        self._lib = lib
        return self

    @property
    def ctx(self):
        return self._ctx

    # ---- operator products (fp64 at the boundary) -----------------------
    def Ab_batch(self, beta: np.ndarray) -> np.ndarray:
        """A β for a (B, L*M) batch -> (B, n)."""
        beta = as_f64(beta)
        B = beta.shape[0]
        assert beta.size == B * self.L * self.M
        out = np.empty((B, self.n))
        check(self._lib.sa_Ab(self._ctx, B, dptr(beta), dptr(out)))
        return out

    def Az_batch(self, z: np.ndarray) -> np.ndarray:
        """Aᵀ z for a (B, n) batch -> (B, L*M)."""
        z = as_f64(z)
        B = z.shape[0]
        assert z.size == B * self.n
        out = np.empty((B, self.L * self.M))
        check(self._lib.sa_Az(self._ctx, B, dptr(z), dptr(out)))
        return out

    # ---- AMP -------------------------------------------------------------
    def amp_batch(self, y, Pl, T, beta0=None, early_stop=True):
        """Decode B codewords: y (B, n) -> (β̂ (B, L*M), iters (B,)).

        iters[b] is the loop index at which the exact τ == last_τ stop fired
        (sparc_ldpc.py:204) or T when the loop ran out.
        """
        y = as_f64(y)
        B = y.shape[0] if y.ndim == 2 else 1
        assert y.size == B * self.n, "y must hold B x n values"
        Pl = as_f64(Pl).reshape(-1)
        assert Pl.size == self.L, "Pl must hold L section powers"
        T = int(T)
        assert T >= 0
        b0p = None
        if beta0 is not None:
            beta0 = as_f64(beta0)
            assert beta0.size == B * self.L * self.M, "β₀ must hold L*M values per codeword"
            b0p = dptr(beta0)
        out = np.empty((B, self.L * self.M))
        iters = np.empty(B, dtype=np.int32)
        flags = 0 if early_stop else _lib.SA_FLAG_NO_EARLY_STOP
        check(self._lib.sa_amp(self._ctx, B, dptr(y), dptr(Pl), T, b0p, dptr(out),
                               iters.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int)), flags))
        return out, iters

    def decide(self, B: int) -> np.ndarray:
        """Section argmax of the last decode (device-side), (B, L) int32."""
        idx = np.empty((B, self.L), dtype=np.int32)
        check(self._lib.sa_decide(self._ctx, B, idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32))))
        return idx

    DECIDE_SLOTS = 4  # SA_DECIDE_SLOTS

    def decide_async(self, B: int, slot: int) -> None:
        """Queue the section argmax of the decode on the stream and the copy of
        its (B, L) indices into pinned ring slot `slot`; returns at once."""
        check(self._lib.sa_decide_async(self._ctx, int(B), int(slot)))

    def decide_collect(self, B: int, slot: int) -> np.ndarray:
        """Wait for slot `slot`'s decisions (decide_async) and return them, (B, L) int32."""
        idx = np.empty((B, self.L), dtype=np.int32)
        check(self._lib.sa_decide_collect(self._ctx, int(B), int(slot),
                                          idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32))))
        return idx

    # ---- device-resident path (bench) -------------------------------------
    def reserve(self, B, T):
        check(self._lib.sa_reserve(self._ctx, int(B), int(T)))

    def stage(self, y, Pl=None, beta0=None):
        y = as_f64(y)
        B = y.shape[0] if y.ndim == 2 else 1
        Pl = None if Pl is None else as_f64(Pl)
        beta0 = None if beta0 is None else as_f64(beta0)
        check(self._lib.sa_stage(self._ctx, B, dptr(y), None if Pl is None else dptr(Pl),
                                 None if beta0 is None else dptr(beta0)))
        return B

    def run(self, B, T, early_stop=True, beta0=False):
        flags = (0 if early_stop else _lib.SA_FLAG_NO_EARLY_STOP) | (_lib.SA_FLAG_BETA0 if beta0 else 0)
        check(self._lib.sa_run(self._ctx, int(B), int(T), flags))

    def wait(self):
        check(self._lib.sa_wait(self._ctx))

    def last_run_ms(self) -> float:
        return float(self._lib.sa_run_event_ms(self._ctx))

    # kinds 2 / 4 are the int8 matrix-core GEMMs (k_gemm_i8) on the dense
    # backend's batched path, the fp32 GEMVs below kI8MinB codewords
    KERNEL_KINDS = ("k_sec", "k_row", "k_dense_az", "k_dense_den", "k_dense_ab", "k_i8_quant")

    def profile(self, B, T, early_stop=True, beta0=False, rep=1):
        """Eager decode with per-launch HIP events: {kind: (mean_ms, launches)}, total_ms.
        rep > 1: each launch issued rep times back to back between its events
        (mean = elapsed / rep; the staged results are then not a decode).
        rep = 0: every loop kernel once, timed by the start / stop events of
        its own dispatch (hipExtLaunchKernel; sa_profile_dispatch)."""
        flags = (0 if early_stop else _lib.SA_FLAG_NO_EARLY_STOP) | (_lib.SA_FLAG_BETA0 if beta0 else 0)
        nk = len(self.KERNEL_KINDS)
        if int(self._lib.sa_profile_kinds()) != nk:
            raise _lib.SparcAmpError(_lib.SA_ERR_UNSUPPORTED, f"libsparc_amp profiles {self._lib.sa_profile_kinds()} kernel kinds, "
                                f"this module knows {nk}: rebuild the library")
        out = np.zeros(2 * nk + 1)
        if rep == 0:
            check(self._lib.sa_profile_dispatch(self._ctx, int(B), int(T), flags, dptr(out)))
        else:
            check(self._lib.sa_profile_rep(self._ctx, int(B), int(T), flags, int(rep), dptr(out)))
        kinds = {k: (float(out[2 * i]), int(out[2 * i + 1])) for i, k in enumerate(self.KERNEL_KINDS)}
        return kinds, float(out[2 * nk])

    def fetch(self, B):
        out = np.empty((B, self.L * self.M))
        iters = np.empty(B, dtype=np.int32)
        check(self._lib.sa_fetch(self._ctx, B, dptr(out), iters.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int))))
        return out, iters

    def iters(self, B):
        """Stop index of each codeword of the last decode (T when the loop ran out)."""
        it = np.empty(B, dtype=np.int32)
        check(self._lib.sa_fetch(self._ctx, B, None, it.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int))))
        return it

    SECTION_KERNELS = ("k_sec", "k_sec2", "k_secb", "dense", "k_sec4", "k_sec43", "dense_mfma", "matrix_mfma",
                       "k_secg")

    def fetch_z(self, B):
        """Residual z after the last decode's final iteration, (B, n)."""
        z = np.empty((B, self.n))
        check(self._lib.sa_fetch_z(self._ctx, int(B), z.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_double))))
        return z

    def plan(self, B):
        """Which kernels a decode of B codewords runs (sa_plan)."""
        o = np.zeros(8, dtype=np.int64)
        check(self._lib.sa_plan(self._ctx, int(B), o.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int64))))
        return dict(section_kernel=self.SECTION_KERNELS[int(o[0])], partials=int(o[1]), row_splits=int(o[2]),
                    codewords_per_wg=int(o[3]), zz_partials=int(o[4]), w=int(o[5]),
                    row_kernel={1: "k_row2", 2: "k_rowv16B", 3: "k_rowv8B", 4: "k_row2_16", 5: "k_rowc"}.get(int(o[6]), "k_row"), cus=int(o[7]))

    # ---- Monte-Carlo rep stream (sa_mc_stage / sa_mc_run) -------------------
    def mc_supported(self, B):
        """Whether sa_mc_run can decode a stream through B slots on this operator
        (the batched codeword-interleaved Hadamard decode, 4 <= B <= 1024)."""
        if self.backend != "hadamard" or not 4 <= int(B) <= 1024:
            return False
        p = self.plan(B)
        return p["section_kernel"] == "k_secb" and p["row_kernel"] == "k_rowc"

    def mc_stage(self, idx, noise):
        """Stage reps for mc_run: section indices idx (R, L), noise (R, n) fp64."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        R = idx.shape[0]
        assert idx.shape == (R, self.L), "idx must be (R, L)"
        noise = as_f64(noise)
        assert noise.size == R * self.n, "noise must be (R, n)"
        check(self._lib.sa_mc_stage(self._ctx, R, idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32)), dptr(noise)))
        self._mc_reps = R
        return R

    def mc_run(self, B, T, early_stop=True, decisions=True):
        """Decode the staged reps through B slots with per-slot refill:
        -> (decisions (R, L) int32 or None, stop indices (R,) int32 (T: ran
        out), bit errors (R,) int32, device milliseconds of the stream)."""
        R = int(getattr(self, "_mc_reps", 0))
        i32 = _lib.ct.POINTER(_lib.ct.c_int32)
        dec = np.empty((R, self.L), dtype=np.int32) if decisions else None
        its = np.empty(R, dtype=np.int32)
        errs = np.empty(R, dtype=np.int32)
        ms = np.zeros(1)
        flags = 0 if early_stop else _lib.SA_FLAG_NO_EARLY_STOP
        check(self._lib.sa_mc_run(self._ctx, int(B), int(T), flags, None if dec is None else dec.ctypes.data_as(i32),
                                  its.ctypes.data_as(i32), errs.ctypes.data_as(i32), dptr(ms)))
        return dec, its, errs, float(ms[0])

    def plan_batched(self, B):
        """The batched section kernel's work order for B codewords
        (sa_plan_batched): section groups, sections per workgroup, groups per
        XCD per pass, passes per XCD."""
        o = np.zeros(4, dtype=np.int64)
        check(self._lib.sa_plan_batched(self._ctx, int(B), o.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int64))))
        return dict(groups=int(o[0]), sections_per_wg=int(o[1]), groups_per_pass=int(o[2]), passes=int(o[3]))

    def info(self):
        o = np.zeros(8, dtype=np.int64)
        check(self._lib.sa_info(self._ctx, o.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int64))))
        keys = ("L", "M", "n", "w", "backend", "precision", "device", "device_bytes")
        return dict(zip(keys, (int(v) for v in o)))

    # ---- SPARC <-> LDPC glue (device kernels, include/sparc_amp.h) ----------
    # llr / app arguments: a host float64 array, or an int device pointer
    # (e.g. the LDPC decoder's buffers from ldpc.code.device_buffers).
    @staticmethod
    def _ptr(x):
        if isinstance(x, int):
            return _lib.ct.c_void_p(x), _lib.SA_PTR_DEVICE
        return _lib.ct.c_void_p(x.ctypes.data), 0

    def stage_power(self, B, Pl):
        """Stage the section powers (c_l = sqrt(n Pl_l)) for a batch of B."""
        Pl = as_f64(Pl).reshape(-1)
        assert Pl.size == self.L, "Pl must hold L section powers"
        check(self._lib.sa_stage(self._ctx, int(B), None, dptr(Pl), None))

    def stage_power_batch(self, B, Pl):
        """Stage per-codeword section powers Pl (B, L) for the next run of up to B
        codewords; Pl = 0 drops a section (β stays 0: the shortened-operator decode
        of sparc_transforms_shorter as a per-codeword mask).  stage_power returns
        to one allocation."""
        Pl = as_f64(Pl)
        assert Pl.shape == (B, self.L), "Pl must be (B, L)"
        check(self._lib.sa_stage_power_batch(self._ctx, int(B), dptr(Pl)))

    def encode(self, idx, noise=None):
        """Stage y = A β(idx) + noise (sparc_ldpc.py:436-446); idx (B, L) section indices."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        B = idx.shape[0]
        assert idx.shape == (B, self.L)
        nz = None
        if noise is not None:
            noise = as_f64(noise)
            assert noise.size == B * self.n
            nz = dptr(noise)
        check(self._lib.sa_encode(self._ctx, B, idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32)), nz))
        return B

    def stage_onehot(self, idx, scale=None):
        """Stage the one-hot β₀ of section indices idx (B, L) for run(..., beta0=True):
        c_l at idx[b, l]; with ``scale``, scale * c_l and idx -1 = an all-zero section."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        p = idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32))
        if scale is None:
            check(self._lib.sa_stage_onehot(self._ctx, idx.shape[0], p))
        else:
            check(self._lib.sa_stage_onehot_scaled(self._ctx, idx.shape[0], p, float(scale)))

    def llr(self, B, l0, ns, out=None):
        """LDPC-bit LLRs of sections [l0, l0+ns) of the current β (sparc_ldpc.py:470-479).
        out: None (returns a (B, ns*log2 M) array) or a device pointer."""
        lgm = int(np.log2(self.M))
        if out is None:
            out = np.empty((B, ns * lgm))
        p, fl = self._ptr(out)
        check(self._lib.sa_llr(self._ctx, int(B), int(l0), int(ns), p, fl))
        return out

    def soft_beta0(self, B, l0, ns, app):
        """Stage β₀ = β with sections [l0, l0+ns) from the LDPC app (sparc_ldpc.py:683-698)."""
        if not isinstance(app, int):
            app = as_f64(app)
        p, fl = self._ptr(app)
        check(self._lib.sa_soft_beta0(self._ctx, int(B), int(l0), int(ns), p, fl))

    def hard_cancel(self, B, l0, ns, app, dst=None):
        """Hard LDPC decisions of sections [l0, l0+ns) -> (B, ns) indices; with dst,
        stage y - A β_hard as dst's input (sparc_ldpc.py:486-524)."""
        if not isinstance(app, int):
            app = as_f64(app)
        p, fl = self._ptr(app)
        idx = np.empty((B, ns), dtype=np.int32)
        check(self._lib.sa_hard_cancel(self._ctx, int(B), int(l0), int(ns), p, fl,
                                       None if dst is None else dst.ctx,
                                       idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32))))
        return idx

    def threshold(self, B, l0, ns, app, threshold):
        """Threshold decisions of sections [l0, l0+ns) from LLRs ``app`` -> (B, ns) int32, -1 undecided."""
        if not isinstance(app, int):
            app = as_f64(app)
        p, fl = self._ptr(app)
        idx = np.empty((B, ns), dtype=np.int32)
        check(self._lib.sa_threshold(self._ctx, int(B), int(l0), int(ns), p, fl, float(threshold),
                                     idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32))))
        return idx

    def cancel(self, idx, dst, scale=None):
        """Stage y - A β(idx) (idx (B, L), -1 = keep) as dst's input y; β(idx) has
        c_l at idx[b, l], or scale * c_l with ``scale``."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        assert idx.ndim == 2 and idx.shape[1] == self.L
        p = idx.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int32))
        if scale is None:
            check(self._lib.sa_cancel(self._ctx, idx.shape[0], p, dst.ctx))
        else:
            check(self._lib.sa_cancel_scaled(self._ctx, idx.shape[0], p, float(scale), dst.ctx))

    def twin(self) -> "SparcOperator":
        """A second operator context sharing this one's device tables
        (sa_create_twin): its own stream and workspace for a concurrent
        decode; keeps this operator alive."""
        if self.backend != "hadamard":
            raise ValueError("twin() needs a Hadamard-backend operator")
        tw = SparcOperator.__new__(SparcOperator)
        tw.L, tw.M, tw.n, tw.w = self.L, self.M, self.n, self.w
        tw.backend, tw.precision, tw.device = self.backend, self.precision, self.device
        tw.ordering, tw.plan_bits = self.ordering, self.plan_bits
        tw._src = self  # the tables' owner outlives the twin
        tw._ctx = _lib.ct.c_void_p()
        check(self._lib.sa_create_twin(self._ctx, _lib.ct.byref(tw._ctx)))
        tw._lib = self._lib
        return tw

    def subset(self, sections) -> "SparcOperator":
        """Operator over the given parent sections (sparc_transforms_shorter)."""
        sec = np.ascontiguousarray(np.asarray(sections, dtype=np.int64).reshape(-1))
        if self.ordering is None:
            raise ValueError("subset() needs a design built from an ordering")
        return SparcOperator(len(sec), self.M, self.n, self.ordering[sec],
                             self.backend, self.precision, self.device, self.plan_bits)


class HostOperatorLoop:
    """The AMP loop for operators that are not this package's
    (``amp(y, σ, Pl, L, M, T, Ab, Az)`` with any callables, as the reference's
    amp() accepts, sparc_ldpc.py:189-222): the caller's ``Ab``/``Az`` run where
    the caller wrote them; τ, the exact-τ stop, the section denoiser η and the
    Onsager residual run on the device in binary64 (an ``SA_BACKEND_HOST``
    context, ``sa_host_*`` in include/sparc_amp.h).  One codeword per call,
    the callables invoked exactly as often, and with the same shapes ((n, 1)
    and (L·M, 1) float64), as in the reference loop.
    """

    def __init__(self, L, M, n, precision="fp64", device=None):
        lib = _lib.load()
        self.L, self.M, self.n = int(L), int(M), int(n)
        self.precision = precision
        self.device = default_device() if device is None else int(device)
        self._ctx = _lib.ct.c_void_p()
        check(lib.sa_create(_lib.ct.byref(self._ctx), self.L, self.M, self.n, None, _lib.SA_BACKEND_HOST,
                            _PRECS[precision], self.device))
        self._lib = lib

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                self._lib.sa_destroy(ctx)
            except Exception:
                pass
            self._ctx = None

    def run(self, y, Pl, T, Ab, Az, beta0=None, early_stop=True):
        """-> (β̂ (L·M, 1), t): t = the loop index at which the exact-τ stop
        fired (sparc_ldpc.py:204), or T when the loop ran out."""
        L, M, n, lib = self.L, self.M, self.n, self._lib
        y = as_f64(y).reshape(-1)
        assert y.size == n, "y must be n long"
        Pl = as_f64(Pl).reshape(-1)
        assert Pl.size == L, "Pl must hold one power per section"
        ab0 = None
        if beta0 is not None:
            beta0 = as_f64(beta0).reshape(-1)
            ab0 = as_f64(Ab(beta0.reshape(-1, 1))).reshape(-1)  # sparc_ldpc.py:198
            assert ab0.size == n, "Ab must return n values"
        check(lib.sa_host_init(self._ctx, 1, int(T), dptr(y), dptr(Pl), None if beta0 is None else dptr(beta0),
                               None if ab0 is None else dptr(ab0)))
        flags = 0 if early_stop else _lib.SA_FLAG_NO_EARLY_STOP
        stopped = np.zeros(1, dtype=np.int32)
        z = np.empty((1, n))
        beta = np.empty((1, L * M))
        t_stop = int(T)
        for t in range(int(T)):
            check(lib.sa_host_tau(self._ctx, 1, t, flags, stopped.ctypes.data_as(_lib.ct.POINTER(_lib.ct.c_int))))
            if stopped[0]:
                t_stop = t
                break
            check(lib.sa_fetch_z(self._ctx, 1, dptr(z)))
            az = as_f64(Az(z.reshape(-1, 1))).reshape(-1)                  # :213
            assert az.size == L * M, "Az must return L*M values"
            check(lib.sa_host_eta(self._ctx, 1, t, flags, dptr(az)))
            check(lib.sa_fetch(self._ctx, 1, dptr(beta), None))
            ab = as_f64(Ab(beta.reshape(-1, 1))).reshape(-1)               # :220
            assert ab.size == n, "Ab must return n values"
            check(lib.sa_host_residual(self._ctx, 1, t, flags, dptr(ab)))
        check(lib.sa_fetch(self._ctx, 1, dptr(beta), None))
        return beta.reshape(-1, 1), t_stop


_HOST_LOOPS: "OrderedDict[tuple, HostOperatorLoop]" = OrderedDict()


def host_loop(L, M, n, device=None) -> HostOperatorLoop:
    """A cached host-operator loop context for (L, M, n)."""
    dev = default_device() if device is None else int(device)
    key = (int(L), int(M), int(n), dev)
    hit = _HOST_LOOPS.get(key)
    if hit is None:
        hit = HostOperatorLoop(L, M, n, device=dev)
        _HOST_LOOPS[key] = hit
        while len(_HOST_LOOPS) > 4:
            _HOST_LOOPS.popitem(last=False)
    else:
        _HOST_LOOPS.move_to_end(key)
    return hit


class AbOp:
    """``Ab(β)`` -> A β / (n, 1) float64 (sparc_ldpc.py:143-144)."""

    def __init__(self, op: SparcOperator):
        self.op = op

    def __call__(self, b):
        b = np.asarray(b)
        assert b.size == self.op.L * self.op.M  # block_sub_fht.Ax, sparc_ldpc.py:121
        return self.op.Ab_batch(b.reshape(1, -1)).reshape(-1, 1)


class AzOp:
    """``Az(z)`` -> Aᵀ z / (L*M, 1) float64 (sparc_ldpc.py:145-146)."""

    def __init__(self, op: SparcOperator):
        self.op = op

    def __call__(self, z):
        z = np.asarray(z)
        assert z.size == self.op.n  # block_sub_fht.Ay, sparc_ldpc.py:129
        return self.op.Az_batch(z.reshape(1, -1)).reshape(-1, 1)


_OP_CACHE: "OrderedDict[tuple, SparcOperator]" = OrderedDict()


def _cached_operator(L, M, n, ordering, backend, precision, device):
    backend = backend or DEFAULT_BACKEND
    precision = precision or DEFAULT_PRECISION
    device = default_device() if device is None else int(device)
    o = np.ascontiguousarray(ordering, dtype=np.uint32)
    key = (L, M, n, hashlib.sha1(o.tobytes()).hexdigest(), backend, precision, device)
    op = _OP_CACHE.get(key)
    if op is None:
        op = SparcOperator(L, M, n, o, backend, precision, device)
        _OP_CACHE[key] = op
        while len(_OP_CACHE) > 6:
            _OP_CACHE.popitem(last=False)
    else:
        _OP_CACHE.move_to_end(key)
    return op


def sparc_transforms(L, M, n, seed=0, *, backend=None, precision=None, device=None):
    """Drop-in for sparc_ldpc.py:140-147: returns (Ab, Az, ordering)."""
    ordering = make_ordering(L, M, n, seed)
    op = _cached_operator(L, M, n, ordering, backend, precision, device)
    return AbOp(op), AzOp(op), ordering


def dense_transforms(A, L, M, *, precision=None, device=None):
    """A caller's own dense n x (L*M) design (e.g. an i.i.d. Gaussian matrix)
    as device operators: returns (Ab, Az) with Ab(β) = A β, Az(z) = Aᵀ z —
    the callables a reference caller would write as ``lambda b: A @ b`` /
    ``lambda z: A.T @ z`` for amp() (sparc_ldpc.py:189,213,220) — so that
    ``amp(y, σ, Pl, L, M, T, Ab, Az)`` keeps the whole loop on the device.
    Not cached: each call copies A to the device."""
    op = SparcOperator.from_matrix(A, L, M, precision=precision, device=device)
    return AbOp(op), AzOp(op)


def gaussian_transforms(L, M, n, seed=0, *, scale=None, precision=None, device=None):
    """An i.i.d. Gaussian design N(0, scale²) (default scale 1/√n) generated on
    the device: (Ab, Az) device operators for amp(), as dense_transforms()
    gives for a host matrix.  The entries come from the device generator
    (SparcOperator.from_random), not from NumPy's stream."""
    op = SparcOperator.from_random(L, M, n, seed, scale, precision=precision, device=device)
    return AbOp(op), AzOp(op)


def sparc_transforms_shorter(L, M, n, ordering, *, backend=None, precision=None, device=None):
    """Drop-in for sparc_ldpc.py:154-168: operator over ``ordering[:L, :]``.

    Callers pass fancy-indexed subsets (amp_exit.py:113-116); any (≥L, n)
    array works.
    """
    ordering = np.asarray(ordering)
    op = _cached_operator(L, M, n, ordering[:L, :], backend, precision, device)
    return AbOp(op), AzOp(op)


def block_sub_fht(n, m, l, seed=0, ordering=None, *, backend=None, precision=None, device=None):
    """Drop-in for sparc_ldpc.py:81-136: unscaled (Ax, Ay, ordering).

    The device computes A·x / sqrt(n); Ax/Ay here undo the 1/sqrt(n) so the
    contract (no scaling) matches the reference.
    """
    assert n > 0, "n must be positive"
    assert m > 0, "m must be positive"
    assert l > 0, "l must be positive"
    if ordering is not None:
        assert ordering.shape == (l, n)
    else:
        ordering = make_ordering(l, m, n, seed)
    op = _cached_operator(l, m, n, ordering, backend, precision, device)
    s = np.sqrt(n)

    def Ax(x):
        assert np.asarray(x).size == l * m
        return op.Ab_batch(np.asarray(x).reshape(1, -1)).reshape(-1) * s

    def Ay(y):
        assert np.asarray(y).size == n
        return op.Az_batch(np.asarray(y).reshape(1, -1)).reshape(-1) * s

    return Ax, Ay, ordering


def sub_fht(n, m, seed=0, ordering=None, **kw):
    """Drop-in for sparc_ldpc.py:32-79 (one block): unscaled (Ax, Ay, ordering)."""
    assert n > 0, "n must be positive"
    assert m > 0, "m must be positive"
    if ordering is None:
        w = _w_of(n, m)
        rng = np.random.RandomState(seed)
        idxs = np.arange(1, w, dtype=np.uint32)
        rng.shuffle(idxs)
        ordering = idxs[:n]
    else:
        assert ordering.shape == (n,)
    Ax, Ay, _ = block_sub_fht(n, m, 1, ordering=np.asarray(ordering).reshape(1, n), **kw)
    return Ax, Ay, ordering
