"""Golden reps of the reference's joint SPARC + LDPC simulators (build container only).

Run from the repo root:  make -C oracle && python tests/golden/make_joint_golden.py

Executes ``amp_ldpc_sim`` (LDPC branch), ``soft_amp_ldpc_sim`` and
``hardinitbeta_amp_ldpc_sim`` of ldpc/sparc_ldpc.py:359-860 on seeded global
``np.random`` streams and records their outputs.  ``code.decode`` loads
``./bin/c_ldpc.so`` relative to the CWD (ldpc.py:859); here it is pointed at
the reference's own decoder built from ldpc/src/c_ldpc.c by oracle/Makefile,
and each call's LLR input and (app, it) output are recorded as well.  The
reference's other workarounds (bitarray stub, vectorised FHT of identical
butterfly order, NumPy-2 beta sentinel) are those of make_golden.py.
Output: tests/golden/joint.npz.
"""
from __future__ import annotations

import ctypes as ct
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)


class _Bits(list):  # bitarray is absent: bp2sp (sparc_ldpc.py:301-311) only needs ** and .invert()
    def __init__(self, s):
        super().__init__(c == "1" for c in s)

    def invert(self):
        self[:] = [not v for v in self]

    def __array__(self, dtype=None, copy=None):
        return np.array(list(self), dtype=bool if dtype is None else dtype)


def main():
    stub = types.ModuleType("bitarray")
    stub.bitarray = _Bits
    sys.modules["bitarray"] = stub
    import make_golden as mg
    ref = mg.load_reference()
    ref.fht_inplace = mg.fast_fht
    _amp = ref.amp

    def amp_np2(y, s, Pl, L, M, T, Ab, Az, β=None):
        if β is None or (isinstance(β, np.ndarray) and β.dtype == object):
            β = np.zeros((L * M, 1))
        return _amp(y, s, Pl, L, M, T, Ab, Az, β)

    ref.amp = amp_np2

    lib = ct.CDLL(os.path.join(ROOT, "oracle", "_ref", "c_ldpc.so"))
    calls = []

    def decode(self, ch, dectype="sumprod2", corr_factor=0.7):
        D, LP = ct.POINTER(ct.c_double), ct.POINTER(ct.c_long)
        ch = np.ascontiguousarray(ch, dtype=np.double)
        app = np.zeros(self.Nv, dtype=np.double)
        v, c, il = (np.ascontiguousarray(a, dtype=np.int64) for a in (self.vdeg, self.cdeg, self.intrlv))
        it = lib.sumprod2(ch.ctypes.data_as(D), v.ctypes.data_as(LP), c.ctypes.data_as(LP), il.ctypes.data_as(LP),
                          self.Nv, self.Nc, self.Nmsg, app.ctypes.data_as(D))
        calls.append((ch.copy(), app.copy(), it))
        return app, it

    ref.ldpc.code.decode = decode
    b2i = ref.bits2indices
    first_idx = []

    def bits2indices(bits, m):  # record the message indices of each rep (first call, :429)
        r = b2i(bits, m)
        first_idx.append(np.asarray(r))
        return r

    ref.bits2indices = bits2indices

    out = {}
    cases = [
        # tag, L, M, P, r, T, z, sigma, seeds, modes
        ("small", 64, 16, 4.0, 1.0, 30, 8, 1.0, (1, 2, 3, 4), ("originalHard", "soft", "hard")),
        ("noisy", 64, 16, 4.0, 1.0, 30, 8, 1.15, (1, 2, 3, 4), ("originalHard", "soft", "hard")),
        ("mid", 64, 16, 4.0, 1.0, 30, 8, 0.93, (1, 2, 3, 4, 5, 6, 7, 8), ("originalHard", "soft", "hard")),
        ("c5", 512, 512, 4.0, 1.0, 64, 192, None, (11, 12), ("soft",)),
    ]
    for tag, L, M, P, r, T, z, sigma, seeds, modes in cases:
        if sigma is None:  # waterfall's mapping at Eb/N0 = 6.89 dB, overall rate 5/6 (:1184-1200)
            R = 5 / 6
            sigma = float(np.sqrt(P / (10 ** (6.888888888888889 / 20) / (1 / (2 * R)))))
        sp = ref.SPARCParams(L, M, sigma, P, r, T)
        lp = ref.LDPCParams("802.16", "5/6", z)
        out[f"{tag}|cfg"] = np.array([L, M, P, r, T, z, sigma])
        for mode in modes:
            for s in seeds:
                calls.clear()
                first_idx.clear()
                np.random.seed(s)
                t0 = time.time()
                if mode == "originalHard":
                    ba, bl, bla, R = ref.amp_ldpc_sim(sp, lp)
                    res = [ba, bl, -1.0 if bla is None else bla]
                elif mode == "soft":
                    ba, bl, R = ref.soft_amp_ldpc_sim(sp, lp, 2)
                    res = list(ba) + list(bl)
                else:
                    ba, bl, R = ref.hardinitbeta_amp_ldpc_sim(sp, lp)
                    res = list(ba) + list(bl)
                key = f"{tag}|{mode}|{s}"
                out[key + "|ber"] = np.array(res)
                out[key + "|R"] = np.array([R])
                out[key + "|idx"] = first_idx[0]
                for k, (ch, app, it) in enumerate(calls):
                    out[key + f"|llr{k}"] = ch
                    out[key + f"|app{k}"] = app
                    out[key + f"|it{k}"] = np.array([it])
                print(key, np.round(res, 5), [c[2] for c in calls], f"{time.time() - t0:.1f}s", flush=True)
    # amp_exit.py does `from sparc_ldpc import *` while sparc_ldpc imports amp_exit:
    # imported as a module (not run as a script) amp_exit sees a half-initialised
    # sparc_ldpc.  Give it the names a script run would have bound.
    ae = ref.ae
    for name in dir(ref):
        if not name.startswith("_") and not hasattr(ae, name):
            setattr(ae, name, getattr(ref, name))
    ae.amp = amp_np2

    # ---- threshold-initialised exchange (sparc_ldpc.py:862-1047) -------------------
    for tag, L, M, P, r, T, z, sigma, seeds, thr in (("thr", 64, 16, 4.0, 1.0, 30, 8, 0.93, (1, 2, 3, 4, 5, 6, 7, 8), 0.7),):
        sp = ref.SPARCParams(L, M, sigma, P, r, T)
        lp = ref.LDPCParams("802.16", "5/6", z)
        out[f"{tag}|cfg"] = np.array([L, M, P, r, T, z, sigma, thr])
        for s in seeds:
            calls.clear()
            first_idx.clear()
            np.random.seed(s)
            ba, bl, R = ref.soft_amp_ldpc_hardinit(sp, lp, 3, thr)
            key = f"{tag}|hardinit|{s}"
            out[key + "|ber"] = np.array(list(ba) + list(bl))
            out[key + "|R"] = np.array([R])
            out[key + "|idx"] = first_idx[0]
            for k, (ch, app, it) in enumerate(calls):
                out[key + f"|llr{k}"] = ch
                out[key + f"|app{k}"] = app
                out[key + f"|it{k}"] = np.array([it])
            print(key, np.round(list(ba) + list(bl), 5), [c[2] for c in calls], flush=True)

    # ---- EXIT: calc_E (amp_exit.py:185-270) ------------------------------------------
    _spo = np.set_printoptions

    def _spo_np2(*a, **k):  # amp_exit.py:261 passes threshold=np.nan, rejected by NumPy 2
        if k.get("threshold", 0) != k.get("threshold", 0):
            k["threshold"] = sys.maxsize
        return _spo(*a, **k)

    np.set_printoptions = _spo_np2
    L, M, P, r, T = 64, 16, 4.0, 1.0, 30
    sp = ref.SPARCParams(L, M, None, P, r, T)
    out["exit|cfg"] = np.array([L, M, P, r, T])
    for s, (I_a, snr_db, thr) in enumerate(((0.3, 12.0, 0.5), (0.6, 11.0, 0.7), (0.8, 10.0, 0.5), (0.95, 13.0, 0.9))):
        np.random.seed(100 + s)
        X = ae.gen_bits(int(L * np.log2(M)))
        E = ae.calc_E(X, I_a, snr_db, sp, None, thr)
        key = f"exit|{s}"
        out[key + "|X"] = X
        out[key + "|E"] = E
        out[key + "|par"] = np.array([I_a, snr_db, thr])
        PE_pos, PE_neg, mp, mn, vp, vn, bw = ae.hist_E(X, E)
        out[key + "|hist"] = np.array([mp, mn, vp, vn, bw, ae.calc_I_e(PE_pos, PE_neg, bw)])
        print(key, np.round(out[key + "|hist"], 4), flush=True)
    np.set_printoptions = _spo
    np.set_printoptions(threshold=1000)

    np.savez_compressed(os.path.join(HERE, "joint.npz"), **out)


if __name__ == "__main__":
    main()
