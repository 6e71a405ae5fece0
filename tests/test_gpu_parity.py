"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden vectors.

Tolerances (BASELINE.json north_star: "within 1e-5 relative fp32"):
  * fp32 device precision: ‖x − ref‖₂ / ‖ref‖₂ ≤ 1e-5 and identical section
    argmax (SURVEY §0.4 — per-element relative error is meaningless for the
    ~e^-50 saturated entries);
  * fp64 device precision: ‖x − ref‖₂ / ‖ref‖₂ ≤ 1e-11 (only the summation
    order differs from the reference's).
"""
import numpy as np
import pytest

from conftest import golden
from oracle import amp_oracle as orc

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-5, "fp64": 1e-11}


def argmax_agree(a, ref, L, M, margin=1e-5):
    """Section argmax equality wherever the reference's top two entries are
    separated by more than `margin` (relative): a near-tie may legitimately
    flip under a different summation order."""
    a = np.asarray(a).reshape(L, M)
    r = np.asarray(ref).reshape(L, M)
    top = np.sort(r, axis=1)
    clear = (top[:, -1] - top[:, -2]) > margin * np.maximum(top[:, -1], 1e-300)
    return np.array_equal(a.argmax(1)[clear], r.argmax(1)[clear])


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def sp(lib_gpu):
    import sparc_ldpc_amd
    return sparc_ldpc_amd


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_operator_small_golden(sp, prec):
    g = golden("small.npz")
    L, M, n = int(g["L"]), int(g["M"]), int(g["n"])
    Ab, Az, ordering = sp.sparc_transforms(L, M, n, precision=prec)
    assert np.array_equal(ordering, g["ordering"])
    assert rel(Ab(g["brand"]), g["Ab_brand"]) <= TOL[prec]
    assert rel(Az(g["zrand"]), g["Az_zrand"]) <= TOL[prec]
    assert Ab(g["brand"]).shape == (n, 1) and Az(g["zrand"]).shape == (L * M, 1)
    sub = g["sub"]
    Ab_s, Az_s = sp.sparc_transforms_shorter(len(sub), M, n, ordering[sub], precision=prec)
    assert rel(Ab_s(g["bsub"]), g["Ab_sub"]) <= TOL[prec]
    assert rel(Az_s(g["zrand"]), g["Az_sub"]) <= TOL[prec]


@pytest.mark.parametrize("L,M,R", [(12, 2, 1.0), (40, 4, 1.0), (16, 64, 1.0), (9, 128, 0.8),
                                   (6, 256, 1.0), (5, 512, 5 / 6), (3, 1024, 1.0), (2, 4096, 1.0)])
@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_operator_sizes_vs_oracle(sp, L, M, R, prec):
    n = int(L * np.log2(M) / R)
    Ab, Az, ordering = sp.sparc_transforms(L, M, n, precision=prec)
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    assert np.array_equal(ordering, oord)
    rs = np.random.RandomState(L * 1000 + M)
    b = rs.randn(L * M, 1)
    z = rs.randn(n, 1)
    assert rel(Ab(b), oAb(b)) <= TOL[prec]
    assert rel(Az(z), oAz(z)) <= TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_amp_small_trajectory(sp, prec):
    g = golden("small.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, _ = sp.sparc_transforms(L, M, n, precision=prec)
    Pl = float(g["P"]) / L * np.ones(L)
    for t in (1, 2, 3, 5, 8):
        b = sp.amp(g["y"], 0, Pl, L, M, t, Ab, Az)
        assert b.shape == (L * M, 1)
        assert rel(b, g["traj"][t - 1]) <= TOL[prec], t
    b, t = sp.amp_test(g["y"], 0, Pl, L, M, T, Ab, Az, precision="operator")
    assert rel(b, g["beta_final"]) <= TOL[prec]
    assert np.array_equal(orc.section_argmax(b, L, M), orc.section_argmax(g["beta_final"], L, M))
    b, t = sp.amp_test(g["y"], 0, Pl, L, M, T, Ab, Az, g["beta0_soft"], precision="operator")
    assert rel(b, g["beta_soft"]) <= TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c1_reps(sp, prec):
    g = golden("c1.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, _ = sp.sparc_transforms(L, M, n, precision=prec)
    Pl = float(g["P"]) / L * np.ones(L)
    for r in range(4):
        y = g[f"y_{r}"]
        for k, t in enumerate((1, 2, 5)):
            assert rel(sp.amp(y, 0, Pl, L, M, t, Ab, Az), g[f"traj_{r}"][k]) <= TOL[prec]
        b, t = sp.amp_test(y, 0, Pl, L, M, T, Ab, Az, precision="operator")
        assert np.array_equal(orc.section_argmax(b, L, M), orc.section_argmax(g[f"beta_{r}"], L, M))
        assert rel(b, g[f"beta_{r}"]) <= TOL[prec]


def check_f64(b, g, key, NS, M, k=None):
    """A binary64 estimate against the reference's binary64 fixture (c2_f64 /
    c4_f64.npz): its first NS sections and the norm of the whole vector, both
    at TOL["fp64"] = 1e-11."""
    sfx = "" if k is None else f"_{k}"
    b = np.asarray(b).reshape(-1)
    assert rel(b[:NS * M], g[f"{key}{sfx}"]) <= TOL["fp64"], key
    assert abs(np.linalg.norm(b) / float(g[f"{key}_norm{sfx}"]) - 1) <= TOL["fp64"], key


# per-section bars of check_sections (tests/golden/make_section_stats.py):
# |stat - ref| <= bar * the section's scale (c_l^2, c_l M, c_l)
SEC_TOL = {"fp32": 2e-4, "fp64": 1e-10}


def check_sections(b, prefix, L, M, c, prec):
    """EVERY section of a full-size estimate against the reference's
    per-section statistics (sections.npz): energy sum_j beta_j^2, first moment
    sum_j j beta_j and max_j beta_j of each of the L sections, each within
    SEC_TOL[prec] of the section's scale, and the L-vectors norm-relative
    within TOL[prec].  Pins the sections past the element-wise fixtures' first
    NS, which were otherwise held only through the vector norm."""
    S = golden("sections.npz")
    bb = np.asarray(b, dtype=np.float64).reshape(L, M)
    got = {"e2": (bb * bb).sum(axis=1), "m1": (bb * np.arange(M)[None, :]).sum(axis=1), "mx": bb.max(axis=1)}
    scale = {"e2": c * c, "m1": c * M, "mx": c}
    for k, v in got.items():
        ref = S[f"{prefix}_{k}"]
        worst = float(np.max(np.abs(v - ref) / scale[k]))
        assert worst <= SEC_TOL[prec], (prefix, k, worst, int(np.argmax(np.abs(v - ref))))
        assert rel(v, ref) <= TOL[prec], (prefix, k, rel(v, ref))


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c2_golden(sp, prec):
    """L=M=512 R=1 P=4, snr 10 dB (amp_test.py:161-176), T=64.  binary32
    against the binary32 fixture at 1e-5; binary64 against the reference's
    binary64 beta (c2_f64.npz) at 1e-11, at t = 1, t = 8 and the stop."""
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, _ = sp.sparc_transforms(L, M, n, precision=prec)
    Pl = float(g["P"]) / L * np.ones(L)
    y = g["y"]
    b1 = sp.amp(y, 0, Pl, L, M, 1, Ab, Az)
    b, t = sp.amp_test(y, 0, Pl, L, M, T, Ab, Az, precision="operator")
    if prec == "fp32":
        assert rel(b1, g["beta_t1"]) <= TOL[prec]
        assert rel(b, g["beta_final"]) <= TOL[prec]
    else:
        g64 = golden("c2_f64.npz")
        NS = int(g64["NS"])
        assert np.array_equal(g64["y"], y)
        check_f64(b1, g64, "beta_t1", NS, M)
        b8 = sp.amp(y, 0, Pl, L, M, 8, Ab, Az, early_stop=False)
        check_f64(b8, g64, "beta_t8", NS, M)
        check_f64(b, g64, "beta_final", NS, M)
        check_sections(b8, "c2_t8", L, M, np.sqrt(n * Pl[0]), prec)
    c = np.sqrt(n * Pl[0])
    check_sections(b1, "c2_t1", L, M, c, prec)
    check_sections(b, "c2_final", L, M, c, prec)
    assert np.array_equal(orc.section_argmax(b, L, M), g["argmax_final"])
    # hard and soft initialisation of amp_test.py:202-240
    Lz = int(g["Lz"])
    beta = np.zeros((L * M, 1)); beta[np.arange(L) * M + g["idx"], 0] = np.sqrt(n * Pl[0])
    beta_0 = beta / np.sqrt(n * float(g["P"]) / L); beta_0[:Lz * M] = 0
    y_new = y - Ab(beta_0)
    Ab_n, Az_n = sp.sparc_transforms_shorter(Lz, M, n, _ordering(sp, L, M, n), precision=prec)
    bh, _ = sp.amp_test(y_new, 0, Pl[:Lz], Lz, M, T, Ab_n, Az_n, precision="operator")
    assert np.array_equal(orc.section_argmax(bh, Lz, M), g["argmax_hard"])
    assert abs(np.linalg.norm(bh) - float(g["beta_hard_norm"])) <= 1e-5 * float(g["beta_hard_norm"])
    bs, _ = sp.amp_test(y, 0, Pl, L, M, T, Ab, Az, beta_0, precision="operator")
    assert np.array_equal(orc.section_argmax(bs, L, M), g["argmax_soft"])
    assert abs(np.linalg.norm(bs) - float(g["beta_soft_norm"])) <= 1e-5 * float(g["beta_soft_norm"])


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c4_golden(sp, prec):
    """BASELINE configs[3], L=768 M=512 R=5/6 P=1.8 (n=8294, w=16384), one
    codeword each at sigma 0.8 (97 % of the sections right) and 0.6 (all
    right): t=1 and the estimate at the exact-tau stop on
    the fixture's first NS sections, the norms of the whole vectors, and the
    per-section decisions (tests/golden/make_c4_golden.py)."""
    g = golden("c4.npz")
    L, M, n, T, NS = (int(g[k]) for k in ("L", "M", "n", "T", "NS"))
    Ab, Az, _ = sp.sparc_transforms(L, M, n, precision=prec)
    Pl = float(g["P"]) / L * np.ones(L)
    g64 = golden("c4_f64.npz") if prec == "fp64" else None
    for k in (0, 1):
        y = g[f"y_{k}"]
        b1 = sp.amp(y, 0, Pl, L, M, 1, Ab, Az)
        c = np.sqrt(n * Pl[0])
        check_sections(b1, f"c4_{k}_t1", L, M, c, prec)
        if g64 is not None:
            check_f64(b1, g64, "beta_t1", NS, M, k)
            b8 = sp.amp(y, 0, Pl, L, M, 8, Ab, Az, early_stop=False)
            check_f64(b8, g64, "beta_t8", NS, M, k)
            check_sections(b8, f"c4_{k}_t8", L, M, c, prec)
        else:
            assert rel(b1[:NS * M], g[f"beta_t1_{k}"]) <= TOL[prec]
            assert abs(np.linalg.norm(b1) / float(g[f"beta_t1_norm_{k}"]) - 1) <= TOL[prec]
        # the stop index in the operator's precision (bounds: see
        # test_stop_index_vs_reference; measured 38 / 7 in fp32, 63 / 9 in fp64
        # against the reference's 63 / 11) and the estimate it stops at
        b, t = sp.amp_test(y, 0, Pl, L, M, T, Ab, Az, precision="operator")
        t_ref = int(g[f"t_stop_{k}"])
        assert t_ref - (STOP32_EARLY if prec == "fp32" else STOP64) <= t <= t_ref + STOP64, (k, t, t_ref)
        if g64 is not None:
            check_f64(b, g64, "beta_final", NS, M, k)
        else:
            assert rel(b[:NS * M], g[f"beta_final_{k}"]) <= TOL[prec]
            assert abs(np.linalg.norm(b) / float(g[f"beta_final_norm_{k}"]) - 1) <= TOL[prec]
        check_sections(b, f"c4_{k}_final", L, M, c, prec)
        assert np.array_equal(orc.section_argmax(b, L, M), g[f"argmax_final_{k}"])
    # the same two codewords in one batch of 8 (the batched section kernel)
    Y = np.stack([g["y_0"].reshape(-1), g["y_1"].reshape(-1)] * 4)
    bb, it = sp.amp_batch(Y, Pl, T, Ab, Az)
    for i in range(8):
        k = i % 2
        if g64 is not None:
            check_f64(bb[i], g64, "beta_final", NS, M, k)
        else:
            assert rel(bb[i, :NS * M], g[f"beta_final_{k}"]) <= TOL[prec]
        check_sections(bb[i], f"c4_{k}_final", L, M, np.sqrt(n * Pl[0]), prec)
        assert np.array_equal(orc.section_argmax(bb[i], L, M), g[f"argmax_final_{k}"])


def _ordering(sp, L, M, n):
    return sp.make_ordering(L, M, n, 0)


def test_c5_decisions(sp):
    """Plain SPARC L=M=512 R=5/6 at Eb/N0 5.33 dB: the reference's own y
    (from amp_ldpc_sim's draws) decodes to the reference's decisions."""
    g = golden("c5_reps.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, _ = sp.sparc_transforms(L, M, n, precision="fp64")
    Ab32, Az32, _ = sp.sparc_transforms(L, M, n, precision="fp32")
    Pl = float(g["P"]) / L * np.ones(L)
    for s in range(3):
        b = sp.amp(g[f"y_{s}"], 0, Pl, L, M, T, Ab, Az)
        assert np.array_equal(orc.section_argmax(b, L, M), g[f"rx_{s}"])
        b32 = sp.amp(g[f"y_{s}"], 0, Pl, L, M, T, Ab32, Az32)
        rx32 = orc.section_argmax(b32, L, M)
        # fp32 may flip a section whose two largest posteriors tie to ~1e-7
        assert (rx32 != g[f"rx_{s}"]).sum() <= 1
        assert abs(sp.ber_of(g[f"idx_{s}"], rx32, L * 9) - float(g[f"ber_{s}"])) <= 9 / (L * 9)


def test_harness_draws_match_reference(sp):
    """amp_ldpc_sim consumes np.random like the reference (sparc_ldpc.py:423-446)."""
    g = golden("c5_reps.npz")
    L, M, T = int(g["L"]), int(g["M"]), int(g["T"])
    np.random.seed(1)
    ber, _, _, R = sp.amp_ldpc_sim(sp.SPARCParams(L, M, float(g["sigma"]), float(g["P"]), float(g["R"]), T),
                                   precision="fp64")
    assert abs(ber - float(g["ber_1"])) <= 9 / (L * 9)
    assert abs(R - L * 9 / int(g["n"])) < 1e-12


def test_amp_edge_cases(sp):
    g = golden("small.npz")
    L, M, n = int(g["L"]), int(g["M"]), int(g["n"])
    Ab, Az, _ = sp.sparc_transforms(L, M, n)
    Pl = float(g["P"]) / L * np.ones(L)
    y = g["y"]
    # T = 0: the loop never runs
    assert np.array_equal(sp.amp(y, 0, Pl, L, M, 0, Ab, Az), np.zeros((L * M, 1)))
    b0 = g["beta0_soft"]
    assert np.allclose(sp.amp(y, 0, Pl, L, M, 0, Ab, Az, b0), b0.reshape(-1, 1))
    # the reference's default sentinel and None both mean "zero start"
    a1 = sp.amp(y, 0, Pl, L, M, 4, Ab, Az, np.array([None]))
    a2 = sp.amp(y, 0, Pl, L, M, 4, Ab, Az)
    a3 = sp.amp(y, 0, Pl, L, M, 4, Ab, Az, np.zeros((L * M, 1)))
    assert np.array_equal(a1, a2) and np.allclose(a2, a3, rtol=0, atol=1e-6)
    # y (n,) and (n, 1) are the same
    assert np.array_equal(sp.amp(y.reshape(-1), 0, Pl, L, M, 4, Ab, Az), a2)
    # y == 0: tau == last_tau == 0 at t = 0 -> returns the zero start
    bz, t = sp.amp_test(np.zeros(n), 0, Pl, L, M, 10, Ab, Az, precision="operator")
    assert t == 0 and not np.any(bz)
    # bad sizes raise AssertionError like the reference
    with pytest.raises(AssertionError):
        Ab(np.zeros(L * M + 1))
    with pytest.raises(AssertionError):
        Az(np.zeros(n - 1))
    with pytest.raises(AssertionError):
        sp.amp(np.zeros(n + 1), 0, Pl, L, M, 3, Ab, Az)
    # the caller's own callables must return the reference's shapes
    with pytest.raises(AssertionError):
        sp.amp(y, 0, Pl, L, M, 3, lambda b: b, lambda z: z)
    with pytest.raises(TypeError):
        sp.amp(y, 0, Pl, L, M, 3, Ab, None)
    # bad orderings are rejected by the library
    bad = np.tile(np.arange(1, n + 1, dtype=np.uint32), (L, 1))
    bad[0, 1] = bad[0, 0]
    with pytest.raises(sp.SparcAmpError):
        sp.SparcOperator(L, M, n, bad)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("L,M,B", [(64, 64, 5), (48, 512, 7), (20, 8, 9)])
def test_batch_matches_single_and_deterministic(sp, prec, L, M, B):
    """B >= 4 runs the batched section kernel (codewords interleaved in LDS,
    16-section Ab accumulation); it must agree with per-codeword decodes
    (single-codeword kernel) to rounding and be bitwise reproducible."""
    P, R, T = 2.0, 1.0, 20
    n = int(L * np.log2(M) / R)
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)
    Pl = P / L * np.ones(L)
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.6, Ab, 50 + i)[1].reshape(-1) for i in range(B)])
    # fixed iteration count: the exact tau == last_tau stop (sparc_ldpc.py:204)
    # may fire at different t under different fp32 summation orders
    bb, it = op.amp_batch(ys, Pl, T, early_stop=False)
    for i in range(B):
        b1, i1 = op.amp_batch(ys[i:i + 1], Pl, T, early_stop=False)
        assert rel(bb[i], b1[0]) <= 2 * TOL[prec] or (prec == "fp32" and M < 64 and rel(bb[i], b1[0]) <= 1e-4)
        assert argmax_agree(bb[i], b1[0], L, M)
    bb2, it2 = op.amp_batch(ys, Pl, T, early_stop=False)
    assert np.array_equal(bb, bb2) and np.array_equal(it, it2)
    be, ie = op.amp_batch(ys, Pl, T)
    be2, ie2 = op.amp_batch(ys, Pl, T)
    assert np.array_equal(be, be2) and np.array_equal(ie, ie2)
    # against the oracle, codeword by codeword, before convergence
    for i in (0, B - 1):
        ref, t = orc.amp_test(ys[i], 0, Pl, L, M, 6, Ab, Az)
        assert t == 5
        b6, _ = op.amp_batch(ys, Pl, 6, early_stop=False)
        assert rel(b6[i], ref) <= TOL[prec]


@pytest.mark.parametrize("prec,n,want,zil", [("fp32", 1024, "k_rowv16B", "0"), ("fp32", 1026, "k_rowv8B", "0"),
                                             ("fp64", 1026, "k_rowv16B", "0"), ("fp32", 1025, "k_row", "0"),
                                             ("fp64", 1025, "k_row", "0"), ("fp32", 1024, "k_rowc", "1"),
                                             ("fp32", 1025, "k_rowc", "1"), ("fp64", 1026, "k_rowc", "1"),
                                             ("fp64", 1025, "k_rowc", "1"), ("fp32", 1024, "k_rowc", None),
                                             ("fp64", 1026, "k_rowc", None)])
def test_row_kernel_variants_vs_oracle(sp, prec, n, want, zil):
    """Every batched row kernel (the Onsager residual of sparc_ldpc.py:220 and
    the A beta sum of :143-146): with z and the Ab partials codeword-interleaved
    (k_rowc: the default in both precisions) and, with
    NO_ZIL, k_rowv with 16-byte rows (binary32 n % 4 == 0, binary64 n
    even), with 8-byte rows (binary32 n even), k_row for odd n; each chosen at
    B = 128 and checked against the oracle codeword by codeword."""
    L, M, B, P, T = 128, 256, 128, 2.0, 4
    plan = None if zil is None else ("ZIL" if zil == "1" else "NO_ZIL")
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec, plan=plan)
    assert op.plan(B)["row_kernel"] == want, op.plan(B)
    Pl = P / L * np.ones(L)
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.6, Ab, 900 + i)[1].reshape(-1) for i in range(B)])
    bb, _ = op.amp_batch(ys, Pl, T, early_stop=False)
    for i in (0, 1, 63, B - 1):
        ref = orc._amp_core(ys[i].reshape(-1, 1), Pl, L, M, T, Ab, Az, None, early_stop=False)[0]
        assert rel(bb[i], ref) <= TOL[prec], i
        assert argmax_agree(bb[i], ref, L, M)
    ab = op.Ab_batch(bb)  # the row kernel's A beta output mode
    for i in (0, B - 1):
        assert rel(ab[i], Ab(bb[i].reshape(-1, 1))) <= TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c2_batched_golden(sp, prec):
    """The golden C2 codeword decoded inside a batch of 6 (batched kernel)."""
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)
    Pl = float(g["P"]) / L * np.ones(L)
    rs = np.random.RandomState(9)
    ys = np.stack([g["y"].reshape(-1)] + [g["y"].reshape(-1) + 0.1 * rs.randn(n) for _ in range(5)])
    bb, it = op.amp_batch(ys, Pl, T)
    assert np.array_equal(orc.section_argmax(bb[0], L, M), g["argmax_final"])
    bt1, _ = op.amp_batch(ys, Pl, 1)
    if prec == "fp64":
        g64 = golden("c2_f64.npz")
        NS = int(g64["NS"])
        check_f64(bb[0], g64, "beta_final", NS, M)
        check_f64(bt1[0], g64, "beta_t1", NS, M)
        bt8, _ = op.amp_batch(ys, Pl, 8, early_stop=False)
        check_f64(bt8[0], g64, "beta_t8", NS, M)
    else:
        assert rel(bb[0], g["beta_final"]) <= TOL[prec]
        assert rel(bt1[0], g["beta_t1"]) <= TOL[prec]


def test_dense_backend_matches_hadamard(sp):
    for (L, M, R) in [(16, 8, 1.0), (24, 512, 1.0), (64, 64, 5 / 6)]:
        n = int(L * np.log2(M) / R)
        Abh, Azh, _ = sp.sparc_transforms(L, M, n, backend="hadamard", precision="fp64")
        Abd, Azd, _ = sp.sparc_transforms(L, M, n, backend="dense")
        rs = np.random.RandomState(1)
        b = rs.randn(L * M, 1); z = rs.randn(n, 1)
        assert rel(Abd(b), Abh(b)) <= 1e-5
        assert rel(Azd(z), Azh(z)) <= 1e-5
        Pl = 2.0 / L * np.ones(L)
        oAb, _, _ = orc.sparc_transforms(L, M, n)
        _, y = orc.rep_inputs(L, M, n, Pl, 0.5, oAb, 7)
        bh = sp.amp(y, 0, Pl, L, M, 12, Abh, Azh)
        bd = sp.amp(y, 0, Pl, L, M, 12, Abd, Azd)
        assert rel(bd, bh) <= 1e-5
        assert np.array_equal(orc.section_argmax(bd, L, M), orc.section_argmax(bh, L, M))


def test_full_size_properties_c4(sp):
    """L=768 M=512 R=5/6 (n=8294): size-independent properties at full size —
    linearity and adjointness of the operator, and an encode -> channel ->
    decode round trip that recovers every section at high SNR."""
    L, M, P = 768, 512, 1.8
    n = int(L * np.log2(M) / (5 / 6))
    Ab, Az, _ = sp.sparc_transforms(L, M, n)
    rs = np.random.RandomState(5)
    x1, x2 = rs.randn(L * M, 1), rs.randn(L * M, 1)
    z = rs.randn(n, 1)
    assert rel(Ab(2.5 * x1 + x2), 2.5 * Ab(x1) + Ab(x2)) <= 1e-5
    lhs = float((Ab(x1) * z).sum()); rhs = float((x1 * Az(z)).sum())
    assert abs(lhs - rhs) <= 1e-4 * (abs(lhs) + 1e-3 * np.linalg.norm(x1) * np.linalg.norm(z))
    Pl = P / L * np.ones(L)
    idx = rs.randint(0, M, L)
    b0 = np.zeros((L * M, 1)); b0[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
    y = Ab(b0) + 0.3 * rs.randn(n, 1)
    b, t = sp.amp_test(y, 0.3, Pl, L, M, 64, Ab, Az, precision="operator")
    assert np.array_equal(orc.section_argmax(b, L, M), idx)
    # β̂ is a per-section posterior scaled by sqrt(n Pl): rows sum to that
    assert np.allclose(b.reshape(L, M).sum(1), np.sqrt(n * Pl), rtol=1e-4)


@pytest.mark.parametrize("prec,L,M,n", [("fp32", 6, 512, 38000),    # w = 65536, z fills the LDS
                                         ("fp32", 3, 4096, 24000),   # M at its maximum, w = 32768
                                         ("fp64", 5, 512, 18000)])   # w = 32768
def test_maximum_sizes_vs_oracle(sp, prec, L, M, n):
    """The largest n the section kernels stage in LDS (w up to 65536, the
    uint16 table limit): operator, single-codeword and batched decodes
    against the oracle; one step past the LDS limit runs on k_secg (z from
    global memory, test_big_n_vs_oracle); the dense backend keeps the 16-bit
    row limit and refuses n = 65535 with an error, never launched."""
    Ab, Az, ordering = sp.sparc_transforms(L, M, n, precision=prec)
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    assert np.array_equal(ordering, oord)
    rs = np.random.RandomState(n)
    b = rs.randn(L * M, 1); z = rs.randn(n, 1)
    assert rel(Ab(b), oAb(b)) <= TOL[prec]
    assert rel(Az(z), oAz(z)) <= TOL[prec]
    Pl = 3.0 / L * np.ones(L)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 40.0, oAb, 70 + i)[1].reshape(-1) for i in range(5)])
    ref, t = orc.amp_test(ys[0], 0, Pl, L, M, 4, oAb, oAz)
    assert t == 3
    b1 = sp.amp(ys[0], 0, Pl, L, M, 4, Ab, Az)
    assert rel(b1, ref) <= TOL[prec] and argmax_agree(b1, ref, L, M)
    op = sp.SparcOperator(L, M, n, ordering, precision=prec)
    if M <= 1024:  # the batched kernel's range
        bb, _ = op.amp_batch(ys, Pl, 4, early_stop=False)
        assert rel(bb[0], ref) <= TOL[prec]
        ref4, _ = orc.amp_test(ys[4], 0, Pl, L, M, 4, oAb, oAz)
        assert rel(bb[4], ref4) <= TOL[prec]
    assert op.plan(1)["section_kernel"] != "k_secg"
    too_big = {"fp32": 40000, "fp64": 19000}[prec] if M == 512 else 25000
    big = sp.SparcOperator(L, M, too_big, sp.make_ordering(L, M, too_big), precision=prec)
    assert big.plan(1)["section_kernel"] == "k_secg" and big.plan(8)["section_kernel"] == "k_secg"
    if prec == "fp32":
        with pytest.raises(sp.SparcAmpError):
            sp.SparcOperator(2, 8, 65535, sp.make_ordering(2, 8, 65535), backend="dense", precision=prec)


@pytest.mark.parametrize("prec,L,M,n", [("fp32", 6, 512, 70000),   # n past 16-bit rows, w = 131072
                                         ("fp64", 4, 256, 40000),   # z past the binary64 LDS image
                                         ("fp32", 5, 64, 100000)])  # E = 1, w = 131072
def test_big_n_vs_oracle(sp, prec, L, M, n):
    """the Hadamard operator past the 16-bit row tables
    and the LDS image of z (k_secg: z from global memory, 32-bit bucket
    entries): operator products, a T = 3 decode single and batched, and the
    early stop against the oracle (sparc_ldpc.py:54 takes any n)."""
    Ab, Az, ordering = sp.sparc_transforms(L, M, n, precision=prec)
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    assert np.array_equal(ordering, oord)
    op = sp.SparcOperator(L, M, n, ordering, precision=prec)
    assert op.plan(1)["section_kernel"] == "k_secg"
    rs = np.random.RandomState(n + L)
    b = rs.randn(L * M, 1); z = rs.randn(n, 1)
    assert rel(Ab(b), oAb(b)) <= TOL[prec]
    assert rel(Az(z), oAz(z)) <= TOL[prec]
    Pl = 3.0 / L * np.ones(L)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 40.0, oAb, 90 + i)[1].reshape(-1) for i in range(3)])
    for T in (1, 3):
        ref = orc.amp(ys[0], 0, Pl, L, M, T, oAb, oAz)
        b1 = sp.amp(ys[0], 0, Pl, L, M, T, Ab, Az)
        assert rel(b1, ref) <= TOL[prec] and argmax_agree(b1, ref, L, M), T
    bb, _ = op.amp_batch(ys, Pl, 3, early_stop=False)
    for i in range(3):
        assert rel(bb[i], orc.amp(ys[i], 0, Pl, L, M, 3, oAb, oAz)) <= TOL[prec], i
    # converged decode: the transmitted sections at high SNR
    idx = rs.randint(0, M, L)
    b0 = np.zeros((L * M, 1)); b0[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
    y = oAb(b0) + 0.1 * rs.randn(n, 1)
    bf, t = sp.amp_test(y, 0.1, Pl, L, M, 20, Ab, Az, precision="operator")
    assert np.array_equal(orc.section_argmax(bf, L, M), idx)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("L,M,n", [(258, 512, 2580), (257, 256, 2284), (300, 512, 6000)])
def test_triple_section_kernel(sp, prec, L, M, n):
    """k_sec43 (three sections per workgroup, chosen by default for L = 768 on
    256 CUs) forced on, incl. a missing third section (L % 3 != 0) and n past
    one row pass (n > 4608): against the oracle per iteration and against the
    pair kernel k_sec4."""
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    Pl = 2.0 / L * np.ones(L)
    ys = [orc.rep_inputs(L, M, n, Pl, 0.9, oAb, 300 + i)[1].reshape(-1) for i in range(2)]
    ops = {}
    for flag in ("1", "0"):
        ops[flag] = sp.SparcOperator(L, M, n, oord, precision=prec, plan="SEC3" if flag == "1" else "NO_SEC3")
    assert ops["1"].plan(1)["section_kernel"] == "k_sec43"
    assert ops["1"].plan(1)["partials"] == (L + 2) // 3
    assert ops["0"].plan(1)["section_kernel"] == "k_sec4"
    for y in ys:
        for t in (1, 2, 5):
            ref, _ = orc.amp_test(y, 0, Pl, L, M, t, oAb, oAz)
            b3, _ = ops["1"].amp_batch(y.reshape(1, -1), Pl, t, early_stop=False)
            b2, _ = ops["0"].amp_batch(y.reshape(1, -1), Pl, t, early_stop=False)
            assert rel(b3[0], ref) <= TOL[prec], t
            assert rel(b3[0], b2[0]) <= 2 * TOL[prec], t
        b3, i3 = ops["1"].amp_batch(y.reshape(1, -1), Pl, 30)
        b3b, i3b = ops["1"].amp_batch(y.reshape(1, -1), Pl, 30)
        assert np.array_equal(b3, b3b) and np.array_equal(i3, i3b)  # bitwise reproducible
        assert argmax_agree(b3[0], orc.amp(y, 0, Pl, L, M, 30, oAb, oAz), L, M)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("L,M,n,sec3", [(512, 512, 4608, "0"), (300, 512, 6007, "1"), (258, 256, 2581, "0")])
def test_partial_layouts_bit_identical(sp, prec, L, M, n, sec3):
    """The row-block-major Ab partials between k_sec4 / k_sec43 and k_row2
    (the default) and the [G][n] layout (plan option NO_PT) hold the same sums in
    the same order: decodes bit-identical, incl. n not a multiple of the
    32-row block; and against the oracle.  The default 16-row k_row2 blocks
    (ceil(n / 16) <= 320; 32 partial groups instead of 16) against the oracle."""
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    Pl = 2.0 / L * np.ones(L)
    y = orc.rep_inputs(L, M, n, Pl, 0.9, oAb, 77)[1].reshape(-1)
    s3 = "SEC3" if sec3 == "1" else "NO_SEC3"
    ops = {}
    for flag in ("1", "0"):  # 32-row blocks in both layouts: the same sums
        ops[flag] = sp.SparcOperator(L, M, n, oord, precision=prec,
                                     plan=(s3, "NO_ROW16") if flag == "1" else (s3, "NO_ROW16", "NO_PT"))
    # 16-row blocks where they fit (the binary32 default)
    ops["16"] = sp.SparcOperator(L, M, n, oord, precision=prec, plan=(s3, "ROW16"))
    dflt = sp.SparcOperator(L, M, n, oord, precision=prec, plan=s3)
    assert ops["1"].plan(1)["section_kernel"] == ("k_sec43" if sec3 == "1" else "k_sec4")
    assert ops["1"].plan(1)["row_kernel"] == "k_row2"
    fits16 = (n + 15) // 16 <= 320
    assert ops["16"].plan(1)["row_kernel"] == ("k_row2_16" if fits16 else "k_row2")
    # binary64 keeps 32-row blocks (faster there)
    assert dflt.plan(1)["row_kernel"] == ("k_row2_16" if fits16 and prec == "fp32" else "k_row2")
    for t in (1, 4):
        b1, i1 = ops["1"].amp_batch(y.reshape(1, -1), Pl, t, early_stop=False)
        b0, i0 = ops["0"].amp_batch(y.reshape(1, -1), Pl, t, early_stop=False)
        assert np.array_equal(b1, b0) and np.array_equal(i1, i0), t
        ref, _ = orc.amp_test(y, 0, Pl, L, M, t, oAb, oAz)
        assert rel(b1[0], ref) <= TOL[prec], t
        b16, _ = ops["16"].amp_batch(y.reshape(1, -1), Pl, t, early_stop=False)
        b16b, _ = ops["16"].amp_batch(y.reshape(1, -1), Pl, t, early_stop=False)
        assert np.array_equal(b16, b16b), t  # bitwise reproducible
        assert rel(b16[0], ref) <= TOL[prec], t


def test_c4_single_uses_triples(sp):
    """L=768 M=512 R=5/6 (n=8294) single codeword: the triple kernel is the
    default where pairs overfill the chip (ceil(L/2) > CUs >= ceil(L/3))."""
    L, M = 768, 512
    n = int(L * np.log2(M) / (5 / 6))
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n))
    plan = op.plan(1)
    cus = plan["cus"]
    want = "k_sec43" if (L + 1) // 2 > cus >= (L + 2) // 3 else "k_sec4"
    assert plan["section_kernel"] == want
    assert plan["partials"] == (256 if want == "k_sec43" else 384)


@pytest.mark.parametrize("B", [1, 6])
def test_profile_rep_and_plan(sp, B):
    """sa_profile / sa_profile_rep (the bench's roofline timing): positive
    per-kernel means, one section + one row launch per iteration, and a
    subsequent run still decodes correctly (rep mode leaves garbage behind)."""
    L, M, T = 64, 512, 6
    n = int(L * np.log2(M))
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n))
    Pl = 2.0 / L * np.ones(L)
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.5, Ab, 70 + i)[1].reshape(-1) for i in range(B)])
    op.reserve(B, T)
    op.stage(ys, Pl)
    plan = op.plan(B)
    assert plan["section_kernel"] in op.SECTION_KERNELS and plan["partials"] > 0
    kinds, total = op.profile(B, T, early_stop=False)
    assert kinds["k_sec"][1] == T and kinds["k_row"][1] == T + 1 and total > 0
    kinds_rep, _ = op.profile(B, 2, early_stop=False, rep=8)
    assert kinds_rep["k_sec"][0] > 0 and kinds_rep["k_sec"][1] == 2
    with pytest.raises(AssertionError):  # SA_ERR_ARG: the reference's AssertionError cases
        op.profile(B, T, rep=-1)
    # dispatch-bound events (sa_profile_dispatch): one pair per loop launch,
    # and the decode it leaves behind is a decode (bit-identical to sa_run's)
    kinds_d, total_d = op.profile(B, T, early_stop=False, rep=0)
    assert kinds_d["k_sec"][1] == T and kinds_d["k_row"][1] == T + 1 and total_d > 0
    assert 0 < kinds_d["k_sec"][0] <= total_d and 0 < kinds_d["k_row"][0] <= total_d
    prof_beta, _ = op.fetch(B)
    op.run(B, T, early_stop=False)
    run_beta, _ = op.fetch(B)
    assert np.array_equal(prof_beta, run_beta)
    bb, _ = op.amp_batch(ys, Pl, T, early_stop=False)
    for i in range(B):
        ref, _ = orc.amp_test(ys[i], 0, Pl, L, M, T, Ab, Az)
        assert rel(bb[i], ref) <= TOL["fp32"]


def test_power_batch_errors(sp):
    """sa_stage_power_batch: shape, sign and backend checks; a later shared
    allocation returns to it (graphs keyed on the mode)."""
    L, M, T = 16, 8, 8
    n = int(L * np.log2(M))
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp64")
    Pl = 2.0 / L * np.ones(L)
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    _, y = orc.rep_inputs(L, M, n, Pl, 0.4, Ab, 3)
    op.reserve(1, T)
    op.stage(y.reshape(1, -1), Pl)
    with pytest.raises(AssertionError):
        op.stage_power_batch(1, Pl)  # must be (B, L)
    bad = Pl.copy()[None, :]
    bad[0, 3] = -1.0
    with pytest.raises(AssertionError):
        op.stage_power_batch(1, bad)
    op.stage_power_batch(1, Pl[None, :])
    op.run(1, T)
    op.wait()
    b_pb, _ = op.fetch(1)
    op.stage_power(1, Pl)
    op.run(1, T)
    op.wait()
    b_sh, _ = op.fetch(1)
    assert np.array_equal(b_pb, b_sh)
    dense = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense")
    dense.reserve(1, T)
    with pytest.raises(sp.SparcAmpError):  # SA_ERR_UNSUPPORTED
        dense.stage_power_batch(1, Pl[None, :])


def test_amp_init_test(sp, capsys):
    """amp_test.py:53-110: started from the transmitted beta, AMP keeps every
    section and stops almost at once; the zero start at high SNR also decodes."""
    np.random.seed(4)
    b_init, b_no = sp.amp_init_test(64, 64, 15.0, 4.0, 1.0)
    assert b_init == [0.0] and b_no == [0.0]
    out = capsys.readouterr().out
    assert "For initialised amp, BER=  [0.0]" in out and "all zero beta_0" in out


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c2_batch256_golden(sp, prec):
    """BASELINE configs[2] at its own batch size: 256 codewords of C2 in one
    decode, which runs the batched section kernel k_secb and the
    codeword-interleaved row kernel k_rowc (the launch shape of the c3 bench
    line; in binary64 k_secb<double> + k_rowc<double>, the kernels of the
    joint decoder).  Slot 0 holds the golden y: t = 1 and the converged
    estimate against the reference's (binary64: c2_f64.npz element-wise on
    its first sections at 1e-11, and every section's statistics); other slots
    (seeded reps) against the oracle at fixed t = 2."""
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    B = 256
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)
    plan = op.plan(B)
    assert plan["section_kernel"] == "k_secb" and plan["row_kernel"] == "k_rowc", plan  # the c3 bench line's kernels
    Pl = float(g["P"]) / L * np.ones(L)
    c = np.sqrt(n * Pl[0])
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    sigma = float(g["sigma"])
    Y = np.empty((B, n))
    Y[0] = g["y"].reshape(-1)
    slots = (1, 77, 128, 255)
    for s in range(1, B):
        rs = np.random.RandomState(5000 + s)
        b0 = np.zeros(L * M)
        b0[np.arange(L) * M + rs.randint(0, M, L)] = np.sqrt(n * Pl)
        Y[s] = rs.randn(n) * sigma  # noise; the codeword part added below
        if s in slots:
            Y[s] += oAb(b0).reshape(-1)
        else:
            Y[s] += op.Ab_batch(b0[None, :])[0]
    b1, _ = op.amp_batch(Y, Pl, 1)
    bf, it = op.amp_batch(Y, Pl, T)
    if prec == "fp32":
        assert rel(b1[0], g["beta_t1"]) <= TOL["fp32"]
        assert rel(bf[0], g["beta_final"]) <= TOL["fp32"]
    else:
        g64 = golden("c2_f64.npz")
        NS = int(g64["NS"])
        check_f64(b1[0], g64, "beta_t1", NS, M)
        check_f64(bf[0], g64, "beta_final", NS, M)
        b8, _ = op.amp_batch(Y, Pl, 8, early_stop=False)
        check_f64(b8[0], g64, "beta_t8", NS, M)
        check_sections(b8[0], "c2_t8", L, M, c, prec)
    check_sections(b1[0], "c2_t1", L, M, c, prec)
    check_sections(bf[0], "c2_final", L, M, c, prec)
    assert np.array_equal(orc.section_argmax(bf[0], L, M), g["argmax_final"])
    assert np.all((it >= 0) & (it <= T))  # T: the loop ran out
    b2, _ = op.amp_batch(Y, Pl, 2, early_stop=False)
    for s in slots:
        ref = orc.amp(Y[s], 0, Pl, L, M, 2, oAb, oAz)
        assert rel(b2[s], ref) <= TOL[prec], s
        assert argmax_agree(b2[s], ref, L, M), s


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c4_batch256_golden(sp, prec):
    """BASELINE configs[3] at the benched launch shape: 256 codewords of C4
    (L=768 M=512 R=5/6, n=8294) in one decode, which runs k_secb + k_rowc
    with 48 section groups in two passes per XCD (the c4 bench line).  The
    reference's two C4 codewords (c4.npz) sit in slots 0 and 1 and codeword 0
    again in slot 255 (the last codeword chunk): t = 1, t = 8 (binary64) and
    the estimate at the exact-tau stop against the reference's (binary32: the
    fixture's first NS sections at 1e-5 and the norm; binary64: c4_f64.npz at
    1e-11) and every section's statistics (sections.npz); four seeded slots
    spread over the chunks against the oracle at t = 2
    (sparc_ldpc.py:189-222, amp_test.py:14-50)."""
    g = golden("c4.npz")
    L, M, n, T, NS = (int(g[k]) for k in ("L", "M", "n", "T", "NS"))
    B = 256
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)
    plan = op.plan(B)
    assert plan["section_kernel"] == "k_secb" and plan["row_kernel"] == "k_rowc", plan
    wo = op.plan_batched(B)
    assert wo["groups"] == 48 and wo["passes"] == 2, wo  # 6 groups per XCD in 2 passes of 3
    Pl = float(g["P"]) / L * np.ones(L)
    c = np.sqrt(n * Pl[0])
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    gold = {0: 0, 1: 1, 255: 0}  # slot -> c4.npz codeword
    seeded = (2, 77, 130, 254)   # chunks 0, 19, 32, 63
    Y = np.empty((B, n))
    for s in range(B):
        if s in gold:
            Y[s] = g[f"y_{gold[s]}"].reshape(-1)
            continue
        rs = np.random.RandomState(7000 + s)
        b0 = np.zeros(L * M)
        b0[np.arange(L) * M + rs.randint(0, M, L)] = c
        Y[s] = rs.randn(n) * 0.7
        Y[s] += (oAb(b0).reshape(-1) if s in seeded else op.Ab_batch(b0[None, :])[0])
    g64 = golden("c4_f64.npz") if prec == "fp64" else None
    b1, _ = op.amp_batch(Y, Pl, 1)
    bf, it = op.amp_batch(Y, Pl, T)
    b8 = op.amp_batch(Y, Pl, 8, early_stop=False)[0] if g64 is not None else None
    for s, k in gold.items():
        check_sections(b1[s], f"c4_{k}_t1", L, M, c, prec)
        check_sections(bf[s], f"c4_{k}_final", L, M, c, prec)
        assert np.array_equal(orc.section_argmax(bf[s], L, M), g[f"argmax_final_{k}"]), s
        if g64 is not None:
            check_f64(b1[s], g64, "beta_t1", NS, M, k)
            check_f64(b8[s], g64, "beta_t8", NS, M, k)
            check_sections(b8[s], f"c4_{k}_t8", L, M, c, prec)
            check_f64(bf[s], g64, "beta_final", NS, M, k)
        else:
            assert rel(b1[s, :NS * M], g[f"beta_t1_{k}"]) <= TOL[prec], s
            assert abs(np.linalg.norm(b1[s]) / float(g[f"beta_t1_norm_{k}"]) - 1) <= TOL[prec], s
            assert rel(bf[s, :NS * M], g[f"beta_final_{k}"]) <= TOL[prec], s
            assert abs(np.linalg.norm(bf[s]) / float(g[f"beta_final_norm_{k}"]) - 1) <= TOL[prec], s
    # the same codeword in the first and the last chunk: the same decode bit for bit
    assert np.array_equal(bf[0], bf[255]) and it[0] == it[255]
    assert np.all((it >= 0) & (it <= T))
    b2, _ = op.amp_batch(Y, Pl, 2, early_stop=False)
    for s in seeded:
        ref = orc.amp(Y[s], 0, Pl, L, M, 2, oAb, oAz)
        assert rel(b2[s], ref) <= TOL[prec], s
        assert argmax_agree(b2[s], ref, L, M), s


def test_c4_fp64_stop_index(sp):
    """The exact-tau stop (sparc_ldpc.py:204, amp_test.py:14-50) in binary64
    at C4: the estimate after the reference's own stop index t_ref (t_ref
    updates, the early stop off) matches the reference's returned estimate,
    and this build's stop index lies within STOP_BOUND iterations of t_ref.
    The index itself cannot be bit-pinned: tau repeats exactly only once the
    iterates reach a fixed point to the last ulp, and the summation order of
    Ab / sum(z^2) differs from NumPy's."""
    STOP_BOUND = 3
    g = golden("c4.npz")
    L, M, n, T, NS = (int(g[k]) for k in ("L", "M", "n", "T", "NS"))
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp64")
    Pl = float(g["P"]) / L * np.ones(L)
    for k in (0, 1):
        y = g[f"y_{k}"].reshape(1, -1)
        t_ref = int(g[f"t_stop_{k}"])
        # t_ref = T-1 is also what amp_test returns when its loop ran out (T
        # updates, no stop): then the estimate after T updates is the match
        cands = (t_ref, T) if t_ref == T - 1 else (t_ref,)
        errs = []
        for upd in cands:
            b, _ = op.amp_batch(y, Pl, upd, early_stop=False)
            errs.append((rel(b[0, :NS * M], g[f"beta_final_{k}"]),  # the fixture stores fp32
                         abs(np.linalg.norm(b[0]) / float(g[f"beta_final_norm_{k}"]) - 1)))
        assert any(e1 <= 1e-7 and e2 <= 1e-11 for e1, e2 in errs), (k, errs)
        _, it = op.amp_batch(y, Pl, T)
        # amp_test returns T-1 when the loop ran out (the reference's t after its loop)
        t_ours = min(int(it[0]), T - 1)
        assert abs(t_ours - t_ref) <= STOP_BOUND, (k, t_ours, t_ref)


# Stop-index bounds of amp_test against the reference's own t (amp_test.py:
# 29-35, 50) on every golden that records it.  Binary64 (amp_test's default):
# within STOP64 iterations.  Binary32 iterates (precision="operator" on an fp32
# operator) reach their exact fixed point earlier, never later than the
# reference's plus STOP64; how much earlier is the measured STOP32_EARLY bound
# of these goldens (C4 codeword 0: 38 against 63).
STOP64, STOP32_EARLY = 3, 30


def _stop_cases(sp):
    """(name, operator args, y, Pl, L, T, beta0, t_ref) for every golden t."""
    cases = []
    g = golden("c1.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Pl = float(g["P"]) / L * np.ones(L)
    for r in range(4):
        cases.append((f"c1_{r}", (L, M, n, None), g[f"y_{r}"], Pl, T, None, int(g[f"t_{r}"])))
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Pl = float(g["P"]) / L * np.ones(L)
    y = g["y"]
    cases.append(("c2", (L, M, n, None), y, Pl, T, None, int(g["t_stop"])))
    Lz = int(g["Lz"])
    beta = np.zeros((L * M, 1)); beta[np.arange(L) * M + g["idx"], 0] = np.sqrt(n * Pl[0])
    beta_0 = beta / np.sqrt(n * float(g["P"]) / L); beta_0[:Lz * M] = 0
    Ab, _, _ = sp.sparc_transforms(L, M, n, precision="fp64")
    y_new = y - Ab(beta_0)
    cases.append(("c2_hard", (Lz, M, n, _ordering(sp, L, M, n)), y_new, Pl[:Lz], T, None, int(g["t_hard"])))
    cases.append(("c2_soft", (L, M, n, None), y, Pl, T, beta_0, int(g["t_soft"])))
    g = golden("c4.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Pl = float(g["P"]) / L * np.ones(L)
    for k in (0, 1):
        cases.append((f"c4_{k}", (L, M, n, None), g[f"y_{k}"], Pl, T, None, int(g[f"t_stop_{k}"])))
    return cases


def test_stop_index_vs_reference(sp):
    """amp_test's returned t against the reference's t (C1 x4, C2 plain /
    hard-init / soft-init, C4 x2): the drop-in default (an fp32
    sparc_transforms operator, amp_test's binary64 stop semantics) within
    STOP64; binary32 iterates within [t_ref - STOP32_EARLY, t_ref + STOP64]."""
    got = {}
    for name, (L, M, n, order), y, Pl, T, b0, t_ref in _stop_cases(sp):
        if order is None:
            Ab, Az, _ = sp.sparc_transforms(L, M, n)  # the drop-in default: fp32 operator
        else:
            Ab, Az = sp.sparc_transforms_shorter(L, M, n, order)
        assert Ab.op.precision == "fp32"
        _, t64 = sp.amp_test(y, 0, Pl, L, M, T, Ab, Az, b0)
        _, t32 = sp.amp_test(y, 0, Pl, L, M, T, Ab, Az, b0, precision="operator")
        got[name] = (t_ref, t64, t32)
        assert abs(t64 - t_ref) <= STOP64, (name, t_ref, t64)
        assert t_ref - STOP32_EARLY <= t32 <= t_ref + STOP64, (name, t_ref, t32)
    print("stop index (t_ref, fp64, fp32):", got)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_cached_operator_two_powers(sp, prec):
    """One cached operator (sparc_transforms' _OP_CACHE) decoding at two total
    powers P at the same (B, T): the replayed hipGraph must read the new P
    (the Onsager term z/tau^2 (P - sum(beta^2)/n), sparc_ldpc.py:220)."""
    L, M, T = 64, 64, 10
    n = int(L * np.log2(M))
    Ab, Az, _ = sp.sparc_transforms(L, M, n, precision=prec)
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    outs = {}
    for P in (2.0, 4.0, 2.0):
        Pl = P / L * np.ones(L)
        _, y = orc.rep_inputs(L, M, n, Pl, 0.7, oAb, 11)
        b = sp.amp(y, 0, Pl, L, M, T, Ab, Az)
        ref = orc.amp(y, 0, Pl, L, M, T, oAb, oAz)
        assert rel(b, ref) <= TOL[prec], P
        if P in outs:
            assert np.array_equal(b, outs[P])
        outs[P] = b


def test_row16_general_loop_for_kernel_partials(sp):
    """k_row2 in 16-row blocks after a one-codeword decode must still read the
    [G][n] partials of k_sec (sa_Ab; the beta0 start) through its general
    loop: at ceil(L / 4) = 256 partials (L = 1024) its constant-stride fast
    path, which assumes row-block-major partials, used to be taken (ADVICE r03
    high).  Ab(beta) and a beta0 decode against the oracle."""
    L, M, n, P = 1024, 256, 4096, 4.0
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp32")
    assert op.plan(1)["row_kernel"] == "k_row2_16"
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    Pl = P / L * np.ones(L)
    _, y = orc.rep_inputs(L, M, n, Pl, 0.8, oAb, 41)
    b1, _ = op.amp_batch(y.reshape(1, -1), Pl, 3, early_stop=False)  # leaves row_kind = 16-row k_row2
    ref3 = orc._amp_core(y.reshape(-1, 1), Pl, L, M, 3, oAb, oAz, None, early_stop=False)[0]
    assert rel(b1[0], ref3) <= TOL["fp32"]
    rs = np.random.RandomState(3)
    x = rs.randn(L * M)
    assert rel(op.Ab_batch(x.reshape(1, -1))[0], oAb(x.reshape(-1, 1))) <= TOL["fp32"]
    b0 = b1[0].reshape(-1, 1)
    bb, _ = op.amp_batch(y.reshape(1, -1), Pl, 2, beta0=b0.reshape(1, -1), early_stop=False)
    ref = orc._amp_core(y.reshape(-1, 1), Pl, L, M, 2, oAb, oAz, b0, early_stop=False)[0]
    assert rel(bb[0], ref) <= TOL["fp32"]


def test_fetch_z_layout_follows_every_run(sp):
    """sa_fetch_z after a batched decode (z codeword-interleaved), a
    one-codeword decode, and the same batched decode again from its cached
    graph: the layout flag follows every run, not only graph captures (ADVICE
    r03 medium), so both batched fetches agree bit for bit, and with the
    one-codeword residual."""
    L, M, n, B, P, T = 128, 256, 1024, 8, 2.0, 5
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp32")
    assert op.plan(B)["row_kernel"] == "k_rowc"
    oAb, _, _ = orc.sparc_transforms(L, M, n)
    Pl = P / L * np.ones(L)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.6, oAb, 500 + i)[1].reshape(-1) for i in range(B)])
    op.amp_batch(ys, Pl, T, early_stop=False)
    za = op.fetch_z(B)
    op.amp_batch(ys[:1], Pl, T, early_stop=False)
    z1 = op.fetch_z(1)
    op.amp_batch(ys, Pl, T, early_stop=False)  # replays the cached B = 8 graph
    zb = op.fetch_z(B)
    assert np.array_equal(za, zb)
    assert rel(zb[0], z1[0]) <= 1e-4


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_batched_work_order_passes_bit_identical(sp, prec):
    """C4 geometry (L = 768: 48 batched section groups, 6 per XCD): the
    default work order in two passes of 3 groups per XCD (one pass's tables
    fit the XCD's L2) and the single pass (plan option ONE_PASS) give the
    same decode bit for bit (the placement changes no sum)."""
    L, M = 768, 512
    n = int(L * np.log2(M) / (5 / 6))
    B, T, P = 8, 3, 1.8
    oAb, _, oord = orc.sparc_transforms(L, M, n)
    Pl = P / L * np.ones(L)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.6, oAb, 60 + i)[1].reshape(-1) for i in range(B)])
    a = sp.SparcOperator(L, M, n, oord, precision=prec)
    b = sp.SparcOperator(L, M, n, oord, precision=prec, plan="ONE_PASS")
    assert a.plan(B)["section_kernel"] == "k_secb"
    ba, ia = a.amp_batch(ys, Pl, T, early_stop=False)
    bb, ib = b.amp_batch(ys, Pl, T, early_stop=False)
    assert np.array_equal(ba, bb) and np.array_equal(ia, ib)


@pytest.mark.parametrize("B", [1, 8])
def test_decide_async_matches_decide(sp, B):
    """sa_decide_async / sa_decide_collect (the bench's pipelined decision):
    the same indices as sa_decide, per slot, with decode k + 1 queued before
    the decisions of decode k are collected; a slot holds one batch and a
    collect of an empty slot is refused."""
    L, M, T = 32, 64, 12
    n = int(L * np.log2(M))
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n))
    Pl = 4.0 / L * np.ones(L)
    Ab, _, _ = orc.sparc_transforms(L, M, n)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.3, Ab, 300 + i)[1].reshape(-1) for i in range(B)])
    op.reserve(B, T)
    op.stage(ys, Pl)
    op.run(B, T)
    ref = op.decide(B)
    op.run(B, T)
    op.decide_async(B, 0)
    op.run(B, T)
    op.decide_async(B, 1)
    a = op.decide_collect(B, 0)
    b = op.decide_collect(B, 1)
    assert np.array_equal(a, ref) and np.array_equal(b, ref)
    with pytest.raises(AssertionError):
        op.decide_collect(B, 0)  # already collected
    with pytest.raises(AssertionError):
        op.decide_async(B, op.DECIDE_SLOTS)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_twin_operator_bit_identical(sp, prec):
    """sa_create_twin (SparcOperator.twin, the joint pipeline's slices): a
    second context over the source's device tables decodes a batch bit for bit
    like the source (the batched kernel, with the bank-aware tables built
    before the twin borrows them), and the source keeps decoding after the
    twin is destroyed (the twin frees none of the borrowed tables)."""
    import gc
    L, M = 64, 256
    n = int(L * np.log2(M))
    B, T = 8, 6
    Ab, _, ordering = orc.sparc_transforms(L, M, n)
    Pl = 4.0 / L * np.ones(L)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.4, Ab, 700 + i)[1].reshape(-1) for i in range(B)])
    op = sp.SparcOperator(L, M, n, ordering, precision=prec)
    assert op.plan(B)["section_kernel"] == "k_secb"
    ref, iref = op.amp_batch(ys, Pl, T, early_stop=False)
    tw = op.twin()
    assert tw.plan(B) == op.plan(B)
    got, igot = tw.amp_batch(ys, Pl, T, early_stop=False)
    assert np.array_equal(got, ref) and np.array_equal(igot, iref)
    del tw
    gc.collect()
    again, _ = op.amp_batch(ys, Pl, T, early_stop=False)
    assert np.array_equal(again, ref)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("L,M,n", [(16, 100, 120), (24, 100, 700), (32, 384, 2048), (8, 3, 40)])
def test_hadamard_any_section_size_vs_oracle(sp, prec, L, M, n):
    """The matrix-free Hadamard operator for M not a power of two (VERDICT r05
    item 7): the reference keeps the last M of w = 2^ceil(log2 max(M+1, n+1))
    columns (sparc_ldpc.py:54, 65-77); the device pads each section to
    2^ceil(log2 M) columns whose first ones never carry an estimate.  Operator
    products, T = 3 decodes (one codeword and a batch of 5) and the section
    decisions against the oracle on the reference's own ordering, including
    w = 2^ceil(log2 M) (n < M: one bucket step)."""
    ordering = sp.make_ordering(L, M, n)
    op = sp.SparcOperator(L, M, n, ordering, backend="hadamard", precision=prec)
    assert op.info()["M"] == M and op.plan(5)["section_kernel"] == "k_sec"
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    assert np.array_equal(oord, ordering)
    rs = np.random.RandomState(L + M)
    x = rs.randn(3, L * M)
    z = rs.randn(3, n)
    for b in range(3):
        assert rel(op.Ab_batch(x[b:b + 1])[0], oAb(x[b].reshape(-1, 1))) <= TOL[prec]
        assert rel(op.Az_batch(z[b:b + 1])[0], oAz(z[b].reshape(-1, 1))) <= TOL[prec]
    P = 2.0
    Pl = P / L * np.ones(L)
    Y = np.stack([orc.rep_inputs(L, M, n, Pl, 0.4, oAb, 300 + i)[1].reshape(-1) for i in range(5)])
    for B in (1, 5):
        bb, it = op.amp_batch(Y[:B], Pl, 3, early_stop=False)
        for i in range(B):
            ref = orc._amp_core(Y[i].reshape(-1, 1), Pl, L, M, 3, oAb, oAz, None, early_stop=False)[0]
            assert rel(bb[i], ref) <= TOL[prec], (B, i)
            assert argmax_agree(bb[i], ref, L, M), (B, i)
        np.testing.assert_array_equal(op.decide(B), bb.reshape(B, L, M).argmax(axis=2))


@pytest.mark.parametrize("fixture,passes", [("c2.npz", 1), ("c4.npz", 2)])
def test_batch256_fp32_every_element_vs_f64_oracle(sp, fixture, passes):
    """the binary32 estimate at the benched launch shapes
    (configs[2] C2/C3 and configs[3] C4 at B = 256: k_secb + k_rowc, one / two
    passes per XCD) pinned element by element on EVERY section, not only the
    fixtures' first NS: slots 0 and 255 hold the reference's codeword 0 of
    the fixture, decoded T = 1, 8 and 16 iterations without the stop, against
    the binary64 oracle (itself pinned bit-exactly to the reference,
    test_oracle.py) on the same y.  Bars: the north-star contract (1e-5
    norm-relative) on the whole vector, and 1e-5 of the section scale
    c = sqrt(n P_l) for every section's error norm and every element (C4
    measured: 4.6e-7 / 4.3e-7 at T = 1, 2.9e-6 / 2.1e-6 at T = 8)."""
    g = golden(fixture)
    L, M, n = (int(g[k]) for k in ("L", "M", "n"))
    B = 256
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp32")
    assert op.plan(B)["section_kernel"] == "k_secb" and op.plan_batched(B)["passes"] == passes
    Pl = float(g["P"]) / L * np.ones(L)
    c = np.sqrt(n * Pl[0])
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    y0 = (g["y_0"] if "y_0" in g else g["y"]).reshape(-1)
    Y = np.empty((B, n))
    for s in range(B):
        rs = np.random.RandomState(9000 + s)
        Y[s] = y0 if s in (0, B - 1) else y0[rs.permutation(n)]
    for T in (1, 8, 16):
        b, _ = op.amp_batch(Y, Pl, T, early_stop=False)
        ref = orc.amp(y0.reshape(-1, 1), 0, Pl, L, M, T, oAb, oAz).reshape(-1)
        for s in (0, B - 1):
            d = (b[s] - ref).reshape(L, M)
            assert rel(b[s], ref) <= TOL["fp32"], (T, s, rel(b[s], ref))
            per_sec = np.linalg.norm(d, axis=1) / c
            per_el = np.abs(d).max() / c
            print(f"T={T} slot {s}: norm-rel {rel(b[s], ref):.3e}, worst section {per_sec.max():.3e} "
                  f"(section {int(per_sec.argmax())}), worst element {per_el:.3e}")
            assert per_sec.max() <= 1e-5, (T, s, per_sec.max())
            assert per_el <= 1e-5, (T, s, per_el)
        assert np.array_equal(b[0], b[B - 1])


@pytest.mark.parametrize("fixture", ["c2.npz", "c4.npz"])
def test_batch256_fp64_every_element_vs_oracle(sp, fixture):
    """The binary64 batched path (k_secb<double> + k_rowc<double>, CB = 2: 128
    codeword chunks) at B = 256, the launch shape of the fp64 legs and of the
    joint step's AMP, pinned element by element on every section: slots 0,
    129 and 255 (first, a middle and the last chunk) hold the fixture's
    codeword 0, the rest permuted copies, decoded T = 1 and 16 iterations
    without the stop against the binary64 oracle on the same y.  Bars:
    TOL["fp64"] on the whole vector and 1e-11 of the section scale on every
    section's error norm and every element; the three slots bit-identical
    (a codeword's decode does not depend on its slot)."""
    g = golden(fixture)
    L, M, n = (int(g[k]) for k in ("L", "M", "n"))
    B = 256
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp64")
    assert op.plan(B)["section_kernel"] == "k_secb"
    Pl = float(g["P"]) / L * np.ones(L)
    c = np.sqrt(n * Pl[0])
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    y0 = (g["y_0"] if "y_0" in g else g["y"]).reshape(-1)
    slots = (0, 129, B - 1)
    Y = np.empty((B, n))
    for s in range(B):
        rs = np.random.RandomState(9000 + s)
        Y[s] = y0 if s in slots else y0[rs.permutation(n)]
    for T in (1, 16):
        b, _ = op.amp_batch(Y, Pl, T, early_stop=False)
        ref = orc.amp(y0.reshape(-1, 1), 0, Pl, L, M, T, oAb, oAz).reshape(-1)
        for s in slots:
            d = (b[s] - ref).reshape(L, M)
            assert rel(b[s], ref) <= TOL["fp64"], (T, s, rel(b[s], ref))
            per_sec = np.linalg.norm(d, axis=1) / c
            per_el = np.abs(d).max() / c
            print(f"T={T} slot {s}: norm-rel {rel(b[s], ref):.3e}, worst section {per_sec.max():.3e}, "
                  f"worst element {per_el:.3e}")
            assert per_sec.max() <= 1e-11, (T, s, per_sec.max())
            assert per_el <= 1e-11, (T, s, per_el)
        assert np.array_equal(b[0], b[129]) and np.array_equal(b[0], b[B - 1])
