"""GPU: the HIP belief-propagation decoder (libldpc_bp.so) against the
reference C decoder — its recorded KATs (tests/golden/ldpc.npz), the library
itself when oracle/_ref/c_ldpc.so travelled with the snapshot, and the NumPy
oracle (oracle/ldpc_oracle.py).  Tolerances: iteration counts and hard
decisions exact on converged words; app within 1e-9 relative (sumprod2,
minsum) or 1e-3 (sumprod, whose tanh/atanh product form amplifies the
last-ulp exp/log/tanh differences between ROCm and glibc)."""
import ctypes as ct
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden
from oracle import ldpc_oracle as lo

pytestmark = pytest.mark.gpu
REF_SO = os.path.join(ROOT, "oracle", "_ref", "c_ldpc.so")
TOL = {"sumprod2": 1e-9, "minsum": 1e-9, "sumprod": 1e-3}


@pytest.fixture(scope="module")
def bp():
    from sparc_ldpc_amd import ldpc
    lib = ldpc.load_bp_library()
    assert lib.lb_device_count() > 0, "no HIP device visible: -m gpu tests need an MI355X"
    return ldpc


def _meta():
    with open(os.path.join(GOLDEN, "ldpc_meta.json")) as fh:
        return json.load(fh)


def _agree(app, it, ref_app, ref_it, algo, max_it=200):
    assert it == ref_it
    if ref_it < max_it:
        assert np.array_equal(app < 0, ref_app < 0)
        np.testing.assert_allclose(app, ref_app, rtol=TOL[algo], atol=TOL[algo])
    else:
        assert np.mean((app < 0) != (ref_app < 0)) < 0.02


@pytest.mark.parametrize("tag", _meta()["decode_cases"])
def test_decode_matches_reference_kats(bp, tag):
    g = golden("ldpc.npz")
    parts = tag.split("|")
    c = bp.code(parts[1], parts[2], int(parts[3]), parts[4])
    algo = parts[-1]
    app, it = c.decode(g[tag + "|ch"], algo)
    _agree(app, it, g[tag + "|app"], int(g[tag + "|it"][0]), algo)


def _awgn(c, rs, ebno, B):
    U = rs.randint(0, 2, (B, c.K))
    X = c.encode_batch(U)
    r = c.K / c.N
    sigma = np.sqrt(1.0 / (2 * r * 10 ** (ebno / 10)))
    Y = (1 - 2 * X) + sigma * rs.randn(B, c.N)
    return X, 2 * Y / sigma ** 2


def test_batch_equals_single_bitwise(bp):
    c = bp.code("802.16", "5/6", 192)
    rs = np.random.RandomState(11)
    X, CH = _awgn(c, rs, 3.4, 24)
    A, IT = c.decode_batch(CH)
    for b in (0, 7, 23):
        a, it = c.decode(CH[b])
        assert it == IT[b] and np.array_equal(a, A[b])


def test_check_regular_code_runs_the_straight_line_check_kernel(bp):
    """802.16 rate 5/6 (every check of degree 20, the joint decoder's outer
    code) runs lxfb_fixed: the reference's forward / backward chains side by
    side; the irregular rate-1/2 code keeps the general kernel.  Both are
    checked against the reference C library in test_against_reference_library."""
    assert bp.code("802.16", "5/6", 192).info()["fixed_dc"] == 20
    assert bp.code("802.16", "1/2", 96).info()["fixed_dc"] == 0


def test_batch_against_oracle(bp):
    c = bp.code("802.16", "5/6", 192)
    rs = np.random.RandomState(12)
    X, CH = _awgn(c, rs, 3.3, 16)
    A, IT = c.decode_batch(CH)
    for b in range(16):
        app, it = lo.sumprod2(CH[b], c.vdeg, c.cdeg, c.intrlv)
        _agree(A[b], IT[b], app, it, "sumprod2")


@pytest.mark.parametrize("algo", ["sumprod2", "sumprod", "minsum"])
def test_against_reference_library(bp, algo):
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/c_ldpc.so not built")
    lib = ct.CDLL(REF_SO)
    D, LP = ct.POINTER(ct.c_double), ct.POINTER(ct.c_long)
    rs = np.random.RandomState(13)
    for std, rate, z, ebno in (("802.16", "5/6", 192, 3.5), ("802.11n", "1/2", 81, 1.4), ("802.16", "3/4", 27, 2.6)):
        c = bp.code(std, rate, z)
        if algo == "minsum" and len(set(c.cdeg.tolist())) != 1:
            continue
        X, CH = _awgn(c, rs, ebno, 6)
        A, IT = c.decode_batch(CH, algo)
        v, cd, il = (np.ascontiguousarray(a, dtype=np.int64) for a in (c.vdeg, c.cdeg, c.intrlv))
        for b in range(len(CH)):
            ch = np.ascontiguousarray(CH[b])
            app = np.zeros(c.N)
            args = [ch.ctypes.data_as(D), v.ctypes.data_as(LP), cd.ctypes.data_as(LP), il.ctypes.data_as(LP),
                    c.Nv, c.Nc, c.Nmsg, app.ctypes.data_as(D)]
            it = lib.minsum(*args, ct.c_double(0.7)) if algo == "minsum" else getattr(lib, algo)(*args)
            _agree(A[b], IT[b], app, it, algo)


def test_reference_signature_dropins(bp):
    """The c_ldpc.c entry points exported under the reference's own names."""
    lib = bp.load_bp_library()
    c = bp.code("802.16", "1/2", 24)
    rs = np.random.RandomState(14)
    X, CH = _awgn(c, rs, 1.6, 2)
    D, LP = ct.POINTER(ct.c_double), ct.POINTER(ct.c_long)
    v, cd, il = (np.ascontiguousarray(a, dtype=np.int64) for a in (c.vdeg, c.cdeg, c.intrlv))
    for b in range(2):
        ch = np.ascontiguousarray(CH[b])
        app = np.zeros(c.N)
        it = lib.sumprod2(ch.ctypes.data_as(D), v.ctypes.data_as(LP), cd.ctypes.data_as(LP), il.ctypes.data_as(LP),
                          c.Nv, c.Nc, c.Nmsg, app.ctypes.data_as(D))
        a2, it2 = c.decode(ch)
        assert it == it2 and np.array_equal(app, a2)
    r = rs.randn(40) * 4
    for corr in (0, 1):
        got = np.array([c.Lxor(x, y, corr) for x, y in zip(r[:20], r[20:])])
        np.testing.assert_allclose(got, lo.lxor(r[:20], r[20:], bool(corr)), rtol=1e-14, atol=1e-15)
    for dc in (2, 5, 20, 25):
        L = rs.randn(dc) * 3
        agg, out = c.Lxfb(L)
        Lm = L[None, :].copy()
        agg_o = lo.lxfb(Lm, True)
        np.testing.assert_allclose(out, Lm[0], rtol=1e-13, atol=1e-14)
        assert abs(agg - agg_o[0]) <= 1e-13 * max(1.0, abs(agg))


def test_messages_in_hbm_path(bp):
    """Nmsg * 8 B > LDS: the per-codeword HBM message slices give the same result."""
    c = bp.code("802.16", "5/6", 300)  # 24000 edges = 187.5 KB
    assert c.info()["lds_messages"] == 0
    rs = np.random.RandomState(15)
    X, CH = _awgn(c, rs, 3.4, 3)
    A, IT = c.decode_batch(CH)
    for b in range(3):
        app, it = lo.sumprod2(CH[b], c.vdeg, c.cdeg, c.intrlv)
        _agree(A[b], IT[b], app, it, "sumprod2")


def test_reference_test_ldpc_decode_property(bp):
    """test_ldpc.py:51-56: noiseless +-5 LLRs decode in 0 iterations to the codeword."""
    rs = np.random.RandomState(16)
    for std, rate, z, p in (("802.16", "2/3", 27, "B"), ("802.11n", "5/6", 54, "A"), ("802.16", "1/2", 3, "A")):
        c = bp.code(std, rate, z, p)
        X = c.encode_batch(rs.randint(0, 2, (8, c.K)))
        A, IT = c.decode_batch(10 * (0.5 - X))
        assert not IT.any() and np.array_equal((A < 0).astype(int), X)


def test_max_iter_and_errors(bp):
    c = bp.code("802.16", "5/6", 192)
    rs = np.random.RandomState(17)
    X, CH = _awgn(c, rs, 2.0, 2)  # too noisy to converge
    A, IT = c.decode_batch(CH, max_iter=5)
    assert (IT == 5).all()
    with pytest.raises(NameError):
        c.decode(np.zeros(c.N + 1))
    with pytest.raises(NameError):
        c.decode(CH[0], "bitflip")


@pytest.mark.parametrize("std,rate,z,ebno", [("802.16", "5/6", 192, 3.2), ("802.11n", "1/2", 81, 1.2),
                                             ("802.16", "1/2", 96, 1.3), ("802.16", "5/6", 300, 3.2)])
def test_tail_launches_bit_identical(bp, std, rate, z, ebno):
    """The tail launches (words still running after tail_at iterations spread
    over several workgroups, a variable and a check launch per iteration)
    against whole decodes in one workgroup per word: app and iteration
    counts identical for every word, every decoder,
    with words that stop before, at and after the hand-off and words that run
    to max_iter; the straight-line (5/6), general (1/2: variable degrees up to
    11 and 6) and HBM-message (z = 300) kernels."""
    c = bp.code(std, rate, z)
    rs = np.random.RandomState(18)
    X, CH = _awgn(c, rs, ebno, 24)
    CH[:4] = 10 * (0.5 - X[:4])  # stop at iteration 0
    algos = ["sumprod2", "sumprod"] + (["minsum"] if len(set(c.cdeg.tolist())) == 1 else [])
    try:
        for algo in algos:
            c.set_tail(0)
            assert c.info()["tail_at"] == 0
            for mi in (200, 9):
                A0, I0 = c.decode_batch(CH, algo, max_iter=mi)
                if mi == 200:
                    its = I0
                for at in (1, 3, 8):
                    c.set_tail(at)
                    A1, I1 = c.decode_batch(CH, algo, max_iter=mi)
                    assert np.array_equal(I0, I1), (algo, mi, at)
                    # sumprod's tanh product saturates (atanh(+-1) = +-inf, then inf - inf) on words
                    # that do not converge: NaN in both, at the same places
                    assert np.array_equal(A0, A1, equal_nan=True), (
                        algo, mi, at, np.isnan(A0).sum(), np.isnan(A1).sum(),
                        np.nanmax(np.abs(np.where(np.isnan(A0) | np.isnan(A1), 0, A0 - A1))))
                c.set_tail(0)
            if algo == "sumprod2":
                assert (its > 8).any() and (its < 3).any()  # words on both sides of the hand-off
    finally:
        c.set_tail(-1)
    assert c.info()["tail_at"] == 8


def test_large_batch_runs_without_the_tail(bp):
    """More than 65535 words in one call: the decode runs whole in k_bp (the
    tail's grid has the words on its y dimension), same results as smaller
    calls for the same words."""
    c = bp.code("802.16", "1/2", 24)
    rs = np.random.RandomState(19)
    X, CH = _awgn(c, rs, 1.6, 8)
    CH = np.repeat(CH, 8193, axis=0)  # 65544 words
    A, IT = c.decode_batch(CH, max_iter=20)
    a8, it8 = c.decode_batch(CH[::8193], max_iter=20)
    assert np.array_equal(IT[::8193], it8) and np.array_equal(A[::8193], a8)
    assert np.array_equal(IT.reshape(8, 8193), np.repeat(it8[:, None], 8193, axis=1))



@pytest.mark.parametrize("std,rate,z,ebno", [("802.16", "5/6", 192, 3.2), ("802.16", "1/2", 96, 1.3)])
def test_device_sized_tail_bit_identical(bp, std, rate, z, ebno):
    """lb_run (the tail sized on the device, every iteration queued, no host
    wait; what the joint decoder uses) against lb_decode (the tail sized on
    the host from one read-back): app and iteration counts identical, for
    batches whose share of words entering the tail differs from the previous
    call's estimate (all, some, none), and for max_iter cut inside the tail."""
    c = bp.code(std, rate, z)
    rs = np.random.RandomState(21)
    X, CH = _awgn(c, rs, ebno, 40)
    CH[:6] = 10 * (0.5 - X[:6])  # stop at iteration 0
    easy = 10 * (0.5 - X)  # every word done before the tail
    for algo in ["sumprod2", "sumprod"]:
        for ch, mi in ((CH, 200), (easy, 200), (CH[6:], 200), (CH, 13)):
            A0, I0 = c.decode_batch(ch, algo, max_iter=mi)
            B = ch.shape[0]
            d_ch, d_app, d_it = c.device_buffers(B)
            lib = bp.load_bp_library()
            assert lib.lb_stage(c._context(), B, np.ascontiguousarray(ch).ctypes.data_as(ct.POINTER(ct.c_double))) == 0
            c.run_buffers(B, algo, max_iter=mi)
            A1, I1 = c.fetch_buffers(B)
            assert np.array_equal(I0, I1), (algo, mi)
            assert np.array_equal(A0, A1, equal_nan=True), (algo, mi)


def test_set_tail_default_restores_create_choice(bp, monkeypatch):
    """lb_set_tail(-1) restores the tail chosen at lb_create, including an
    LDPC_BP_TAIL override read there."""
    monkeypatch.setenv("LDPC_BP_TAIL", "5")
    c = bp.code("802.16", "5/6", 24)
    assert c.info()["tail_at"] == 5
    c.set_tail(0)
    assert c.info()["tail_at"] == 0
    c.set_tail(-1)
    assert c.info()["tail_at"] == 5
