"""Generate the LDPC fixtures by running the reference (build container only).

Run from the repo root:  make -C oracle && python tests/golden/make_ldpc_golden.py

Touches /root/reference only to execute ``ldpc/py/ldpc.py`` (the ``code``
class) and the reference's own C decoder built from ``ldpc/src/c_ldpc.c`` by
``oracle/Makefile`` into ``oracle/_ref/c_ldpc.so``; it records their outputs as
data.  Outputs:

* ``sparc_ldpc_amd/data/protographs.json`` -- the base (proto) matrices the
  reference's ``code.assign_proto`` returns (ldpc.py:26-663) for every
  (standard, rate, ptype[, z]) it defines: the IEEE 802.16e / 802.11n LDPC
  base matrices and the reference author's own threshold-designed protographs.
  These numbers are the code definitions (data), needed at run time to build
  the Tanner graph; the graph construction, encoder and decoder are this
  repo's own.
* ``tests/golden/ldpc.npz`` -- per code: SHA-256 of (vdeg, cdeg, intrlv) of
  ``code.prepare_decoder`` (ldpc.py:694-786); full arrays for the small codes;
  encoder KATs (``code.encode``, ldpc.py:790-850); decoder KATs of the
  reference C ``sumprod2`` / ``sumprod`` / ``minsum`` (c_ldpc.c:32-381) on
  seeded noisy BPSK LLRs and on saturated (+-DBL_MAX, i.e. ``nan_to_num``'d
  SPARC) LLRs: inputs, app, iteration counts.
"""
from __future__ import annotations

import ctypes as ct
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_PY = "/root/reference/ldpc/py"
REF_SO = os.path.join(ROOT, "oracle", "_ref", "c_ldpc.so")

STANDARDS_Z_FREE = {
    "802.16": [("1/2", "A"), ("2/3", "A"), ("2/3", "B"), ("3/4", "A"), ("3/4", "B"), ("5/6", "A")],
    "2_7_12_good": [("1/2", "A")],
    "2_7_12_good_dc6": [("1/2", "A"), ("0.45", "A")],
    "2_5_12_good_threshold08": [("0.45", "A"), ("3/8", "A")],
    "2_7_12_bad": [("1/2", "A")],
}
RATES_11N = ["1/2", "2/3", "3/4", "5/6"]


def sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
    return h.hexdigest()


def c_decoder():
    lib = ct.CDLL(REF_SO)
    for f in (lib.sumprod, lib.sumprod2, lib.minsum):
        f.restype = ct.c_int
    return lib


def ref_decode(lib, code, ch, algo, corr=0.7):
    """What code.decode (ldpc.py:855-930) does, with the library path made explicit."""
    ch = np.ascontiguousarray(ch, dtype=np.double)
    app = np.zeros(code.Nv, dtype=np.double)
    D, Lp = ct.POINTER(ct.c_double), ct.POINTER(ct.c_long)
    vdeg = np.ascontiguousarray(code.vdeg, dtype=np.int64)
    cdeg = np.ascontiguousarray(code.cdeg, dtype=np.int64)
    il = np.ascontiguousarray(code.intrlv, dtype=np.int64)
    args = [ch.ctypes.data_as(D), vdeg.ctypes.data_as(Lp), cdeg.ctypes.data_as(Lp), il.ctypes.data_as(Lp),
            code.Nv, code.Nc, code.Nmsg, app.ctypes.data_as(D)]
    if algo == "sumprod2":
        it = lib.sumprod2(*args)
    elif algo == "sumprod":
        it = lib.sumprod(*args)
    else:
        it = lib.minsum(*args, ct.c_double(corr))
    return app, it


def main():
    sys.path.insert(0, REF_PY)
    import ldpc as ref

    # ---- protographs ------------------------------------------------------
    protos = {"z_free": {}, "802.11n": {}}
    for std, lst in STANDARDS_Z_FREE.items():
        for rate, ptype in lst:
            c = ref.code(std, rate, 96, ptype)
            protos["z_free"].setdefault(std, {}).setdefault(rate, {})[ptype] = c.proto.astype(int).tolist()
            # the table must not depend on z
            assert np.array_equal(ref.code(std, rate, 24, ptype).proto, c.proto)
    for z in (27, 54, 81):
        for rate in RATES_11N:
            c = ref.code("802.11n", rate, z, "A")
            protos["802.11n"].setdefault(str(z), {})[rate] = c.proto.astype(int).tolist()
    os.makedirs(os.path.join(ROOT, "sparc_ldpc_amd", "data"), exist_ok=True)
    with open(os.path.join(ROOT, "sparc_ldpc_amd", "data", "protographs.json"), "w") as fh:
        json.dump({"source": "IEEE 802.16e-2005 / 802.11n-2009 LDPC base matrices and the "
                             "reference's designed protographs, as returned by ldpc.py:26-663 "
                             "code.assign_proto (captured by tests/golden/make_ldpc_golden.py)",
                   "protographs": protos}, fh, separators=(",", ":"))

    # ---- graph hashes: every case of the reference's test_ldpc.py + SPARC codes ----
    cases = []
    for z in (3, 27, 54, 81):
        for rate, ptype in STANDARDS_Z_FREE["802.16"]:
            cases.append(("802.16", rate, z, ptype))
    for z in (27, 54, 81):
        for rate in RATES_11N:
            cases.append(("802.11n", rate, z, "A"))
    cases += [("802.16", "5/6", 192, "A"), ("802.16", "1/2", 24, "A")]
    for std, lst in STANDARDS_Z_FREE.items():
        if std != "802.16":
            for rate, ptype in lst:
                cases.append((std, rate, 32, ptype))
    graphs = {}
    out = {}
    for std, rate, z, ptype in cases:
        c = ref.code(std, rate, z, ptype)
        key = f"{std}|{rate}|{z}|{ptype}"
        graphs[key] = {"sha": sha(c.vdeg, c.cdeg, c.intrlv), "N": int(c.N), "K": int(c.K),
                       "Nmsg": int(c.Nmsg)}
        if z == 3:
            out[f"graph|{key}|vdeg"] = np.asarray(c.vdeg, np.int64)
            out[f"graph|{key}|cdeg"] = np.asarray(c.cdeg, np.int64)
            out[f"graph|{key}|intrlv"] = np.asarray(c.intrlv, np.int64)

    # ---- encoder KATs -------------------------------------------------------
    rs = np.random.RandomState(20240611)
    enc_codes = [("802.16", "5/6", 192, "A"), ("802.16", "1/2", 24, "A"), ("802.16", "2/3", 27, "B"),
                 ("802.16", "3/4", 54, "A"), ("802.11n", "1/2", 27, "A"), ("802.11n", "5/6", 81, "A")]
    # the designed protographs are not dual-diagonal: the reference encoder
    # raises NameError for them (ldpc.py:834-835); record which do
    enc_raises = []
    for std, lst in STANDARDS_Z_FREE.items():
        for rate, ptype in lst:
            c = ref.code(std, rate, 32, ptype)
            try:
                c.encode([0] * c.K)
            except NameError:
                enc_raises.append(f"{std}|{rate}|32|{ptype}")
    for std, rate, z, ptype in enc_codes:
        c = ref.code(std, rate, z, ptype)
        U = rs.randint(0, 2, (3, c.K))
        X = np.stack([c.encode(u.tolist()) for u in U])
        key = f"{std}|{rate}|{z}|{ptype}"
        out[f"enc|{key}|info"] = U.astype(np.uint8)
        out[f"enc|{key}|code"] = X.astype(np.uint8)

    # ---- decoder KATs (the reference C decoder) --------------------------------
    lib = c_decoder()
    dec = []
    dec_codes = [("802.16", "5/6", 192, "A", [3.2, 3.6, 4.2]), ("802.16", "1/2", 24, "A", [1.0, 1.6]),
                 ("802.11n", "3/4", 27, "A", [2.4, 3.0]), ("802.11n", "5/6", 81, "A", [3.4])]
    for std, rate, z, ptype, snrs in dec_codes:
        c = ref.code(std, rate, z, ptype)
        key = f"{std}|{rate}|{z}|{ptype}"
        for si, ebno in enumerate(snrs):
            u = rs.randint(0, 2, c.K)
            x = np.asarray(c.encode(u.tolist()))
            r = c.K / c.N
            sigma = np.sqrt(1.0 / (2 * r * 10 ** (ebno / 10)))
            y = (1 - 2 * x) + sigma * rs.randn(c.N)
            ch = 2 * y / sigma ** 2
            algos = ["sumprod2", "sumprod"]
            if len(set(np.asarray(c.cdeg).tolist())) == 1:
                algos.append("minsum")  # c_ldpc.c:364 advances by cdeg[j+1]: exact only when check-regular
            for algo in algos:
                app, it = ref_decode(lib, c, ch, algo)
                tag = f"dec|{key}|{si}|{algo}"
                out[tag + "|ch"] = ch
                out[tag + "|app"] = app
                out[tag + "|it"] = np.array([it])
                out[tag + "|x"] = x.astype(np.uint8)
                dec.append(tag)
    # saturated LLRs as produced by nan_to_num(log(1-p) - log(p)) (sparc_ldpc.py:477-479)
    c = ref.code("802.16", "5/6", 192, "A")
    u = rs.randint(0, 2, c.K)
    x = np.asarray(c.encode(u.tolist()))
    ch = np.where(x == 0, 1.0, -1.0) * rs.exponential(6.0, c.N)
    flip = rs.rand(c.N) < 0.04
    ch[flip] = -ch[flip]
    sat = rs.rand(c.N) < 0.3
    ch[sat] = np.sign(ch[sat]) * np.finfo(np.float64).max
    for algo in ("sumprod2",):
        app, it = ref_decode(lib, c, ch, algo)
        tag = f"dec|802.16|5/6|192|A|sat|{algo}"
        out[tag + "|ch"] = ch
        out[tag + "|app"] = app
        out[tag + "|it"] = np.array([it])
        out[tag + "|x"] = x.astype(np.uint8)
        dec.append(tag)

    # ---- sp2bp / bp2sp / LLR glue (sparc_ldpc.py:257-314, 470-479) ------------------
    import types
    import matplotlib
    matplotlib.use("Agg")

    class _Bits(list):  # stand-in for bitarray (absent): bp2sp only needs ** and .invert()
        def __init__(self, s):
            super().__init__(c == "1" for c in s)

        def invert(self):
            self[:] = [not v for v in self]

        def __array__(self, dtype=None, copy=None):
            return np.array(list(self), dtype=bool if dtype is None else dtype)

    stub = types.ModuleType("bitarray")
    stub.bitarray = _Bits
    sys.modules["bitarray"] = stub
    sys.path.insert(0, os.path.dirname(REF_PY))
    import warnings
    warnings.simplefilter("ignore")
    import sparc_ldpc as sref
    for L, M in ((6, 8), (4, 64), (3, 512)):
        e = rs.exponential(1.0, (L, M)) ** 4
        beta = (e / e.sum(1, keepdims=True)).reshape(-1)
        beta[:M] = 0.0
        beta[rs.randint(0, M)] = 1.0  # a decided section: p in {0, 1} -> infinite LLRs
        p = sref.sp2bp(beta, L, M)
        out[f"sp2bp|{L}|{M}|beta"] = beta
        out[f"sp2bp|{L}|{M}|p"] = p
        with np.errstate(divide="ignore"):
            out[f"sp2bp|{L}|{M}|llr"] = np.nan_to_num(np.log(1 - p) - np.log(p))
        if M <= 64:
            v = rs.rand(L * int(np.log2(M)))
            out[f"bp2sp|{L}|{M}|v"] = v
            out[f"bp2sp|{L}|{M}|sp"] = sref.bp2sp(v, L, M)

    np.savez_compressed(os.path.join(HERE, "ldpc.npz"), **out)
    with open(os.path.join(HERE, "ldpc_meta.json"), "w") as fh:
        json.dump({"graphs": graphs, "decode_cases": dec,
                   "encode_codes": [f"{s}|{r}|{z}|{p}" for s, r, z, p in enc_codes],
                   "encode_raises": enc_raises}, fh, indent=1)
    print("wrote", len(out), "arrays;", len(graphs), "graphs;", len(dec), "decode cases")
    for t in dec:
        print(t, int(out[t + "|it"][0]), int(np.sum((out[t + "|app"] < 0) != out[t + "|x"])))


if __name__ == "__main__":
    main()
