"""CPU: the LDPC oracle against the reference's own fixtures (tests/golden/ldpc.npz,
captured from ldpc/py/ldpc.py and the reference C decoder) and, when built by
oracle/Makefile, against oracle/_ref/c_ldpc.so itself."""
import ctypes as ct
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden
from oracle import ldpc_oracle as lo

REF_SO = os.path.join(ROOT, "oracle", "_ref", "c_ldpc.so")


def _meta():
    with open(os.path.join(GOLDEN, "ldpc_meta.json")) as fh:
        return json.load(fh)


def _key(k):
    std, rate, z, ptype = k.split("|")
    return std, rate, int(z), ptype


def _sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
    return h.hexdigest()


def test_graphs_match_reference_prepare_decoder():
    g = golden("ldpc.npz")
    for key, info in _meta()["graphs"].items():
        std, rate, z, ptype = _key(key)
        proto = lo.protograph(std, rate, z, ptype)
        vdeg, cdeg, il = lo.prepare_decoder(proto, z)
        assert _sha(vdeg, cdeg, il) == info["sha"], key
        assert len(vdeg) == info["N"] and len(vdeg) - len(cdeg) == info["K"] and len(il) == info["Nmsg"]
        if z == 3:
            assert np.array_equal(il, g[f"graph|{key}|intrlv"])


@pytest.mark.parametrize("key", ["802.16|1/2|3|A", "802.16|2/3|3|B", "802.11n|3/4|27|A", "802.16|5/6|3|A"])
def test_pcmat_degrees(key):
    std, rate, z, ptype = _key(key)
    proto = lo.protograph(std, rate, z, ptype)
    H = lo.pcmat(proto, z)
    vdeg, cdeg, il = lo.prepare_decoder(proto, z)
    assert H.sum() == len(il) and np.array_equal(H.sum(0), vdeg) and np.array_equal(H.sum(1), cdeg)


def test_encoder_kats():
    g = golden("ldpc.npz")
    meta = _meta()
    for key in meta["encode_codes"]:
        std, rate, z, ptype = _key(key)
        proto = lo.protograph(std, rate, z, ptype)
        H = lo.pcmat(proto, z) if z <= 54 else None
        for u, x in zip(g[f"enc|{key}|info"], g[f"enc|{key}|code"]):
            got = lo.encode(proto, z, u)
            assert np.array_equal(got, x), key
            if H is not None:
                assert not np.any(H.dot(got) % 2)
    for key in meta["encode_raises"]:
        std, rate, z, ptype = _key(key)
        proto = lo.protograph(std, rate, z, ptype)
        with pytest.raises(NameError):
            lo.encode(proto, z, np.zeros((proto.shape[1] - proto.shape[0]) * z, dtype=int))


def _decode_cases():
    return _meta()["decode_cases"]


@pytest.mark.parametrize("tag", _decode_cases())
def test_decoder_kats(tag):
    g = golden("ldpc.npz")
    parts = tag.split("|")
    std, rate, z, ptype, algo = parts[1], parts[2], int(parts[3]), parts[4], parts[-1]
    proto = lo.protograph(std, rate, z, ptype)
    vdeg, cdeg, il = lo.prepare_decoder(proto, z)
    ch = g[tag + "|ch"]
    ref_app, ref_it = g[tag + "|app"], int(g[tag + "|it"][0])
    app, it = lo._decode(ch, vdeg, cdeg, il, algo)
    assert it == ref_it
    if ref_it < lo.MAX_ITCOUNT:
        # converged decodes: NumPy vs glibc exp/log differ by ulps at most
        assert np.array_equal(app < 0, ref_app < 0)
        # tanh/atanh (sumprod) is ill-conditioned near +-1 and amplifies ulps more
        tol = 1e-3 if algo == "sumprod" else 1e-9
        np.testing.assert_allclose(app, ref_app, rtol=tol, atol=tol)
    else:
        # 200 non-converging iterations amplify ulp differences; decisions stay close
        assert np.mean((app < 0) != (ref_app < 0)) < 0.02


def _ref_lib():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/c_ldpc.so not built (make -C oracle; needs /root/reference)")
    lib = ct.CDLL(REF_SO)
    lib.Lxor.restype = ct.c_double
    lib.Lxor.argtypes = [ct.c_double, ct.c_double, ct.c_int]
    lib.Lxfb.restype = ct.c_double
    lib.Lxfb.argtypes = [ct.POINTER(ct.c_double), ct.c_long, ct.c_int]
    return lib


def test_lxor_lxfb_against_reference_c():
    lib = _ref_lib()
    rs = np.random.RandomState(3)
    a = rs.randn(200) * 5
    b = rs.randn(200) * 5
    a[:5] = [0.0, -0.0, 1e300, -1e308, 40.0]
    for corr in (0, 1):
        ref = np.array([lib.Lxor(x, y, corr) for x, y in zip(a, b)])
        np.testing.assert_allclose(lo.lxor(a, b, bool(corr)), ref, rtol=1e-14, atol=1e-15)
    for dc in (2, 3, 7, 20, 25):
        L = rs.randn(dc) * 3
        Lr = L.copy()
        agg_ref = lib.Lxfb(Lr.ctypes.data_as(ct.POINTER(ct.c_double)), dc, 1)
        Lm = L[None, :].copy()
        agg = lo.lxfb(Lm, True)
        np.testing.assert_allclose(Lm[0], Lr, rtol=1e-13, atol=1e-14)
        assert abs(agg[0] - agg_ref) <= 1e-13 * max(1, abs(agg_ref))


def test_sp2bp_bp2sp_llr_against_reference():
    g = golden("ldpc.npz")
    for L, M in ((6, 8), (4, 64), (3, 512)):
        beta = g[f"sp2bp|{L}|{M}|beta"]
        p = lo.sp2bp(beta, L, M)
        assert np.array_equal(p, g[f"sp2bp|{L}|{M}|p"])
        with np.errstate(divide="ignore"):
            llr = np.nan_to_num(np.log(1 - p) - np.log(p))
        assert np.array_equal(llr, g[f"sp2bp|{L}|{M}|llr"])
        if M <= 64:
            np.testing.assert_allclose(lo.bp2sp(g[f"bp2sp|{L}|{M}|v"], L, M), g[f"bp2sp|{L}|{M}|sp"],
                                       rtol=1e-14, atol=0)
