"""CPU: the oracle (oracle/amp_oracle.py) against the reference's own outputs.

The fixtures under tests/golden/ were produced by tests/golden/make_golden.py
importing ldpc/sparc_ldpc.py itself.  fp64, bit-exact comparisons.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle import amp_oracle as orc


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_fht_matches_reference_fallback_bitwise():
    g = golden("fht.npz")
    for w in (8, 64, 512, 2048):
        x = g[f"fht_in_{w}"].copy()
        orc.fht_inplace(x)
        assert np.array_equal(x, g[f"fht_out_{w}"])


def test_small_operator_and_trajectory_bitwise():
    g = golden("small.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, ordering = orc.sparc_transforms(L, M, n)
    assert np.array_equal(ordering, g["ordering"])
    assert np.array_equal(Ab(g["brand"]), g["Ab_brand"])
    assert np.array_equal(Az(g["zrand"]), g["Az_zrand"])
    P = float(g["P"])
    Pl = P / L * np.ones(L)
    for t in range(1, T + 1):
        b = orc.amp(g["y"], 0, Pl, L, M, t, Ab, Az)
        assert np.array_equal(b.reshape(-1), g["traj"][t - 1]), t
    b, t = orc.amp_test(g["y"], 0, Pl, L, M, T, Ab, Az)
    assert np.array_equal(b, g["beta_final"]) and t == int(g["t_stop"])
    b, t = orc.amp_test(g["y"], 0, Pl, L, M, T, Ab, Az, g["beta0_soft"])
    assert np.array_equal(b, g["beta_soft"]) and t == int(g["t_soft"])
    sub = g["sub"]
    Ab_s, Az_s = orc.sparc_transforms_shorter(len(sub), M, n, ordering[sub])
    assert np.array_equal(Ab_s(g["bsub"]), g["Ab_sub"])
    assert np.array_equal(Az_s(g["zrand"]), g["Az_sub"])
    assert np.array_equal(Ab(g["beta0_soft"]), g["Ab_b0"])


def test_c1_reps_bitwise():
    g = golden("c1.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, ordering = orc.sparc_transforms(L, M, n)
    assert np.array_equal(ordering, g["ordering"])
    Pl = float(g["P"]) / L * np.ones(L)
    for r in range(4):
        # the synthetic rep generator reproduces the stored inputs
        idx, y = orc.rep_inputs(L, M, n, Pl, float(g["sigma"]), Ab, 1000 + r)
        assert np.array_equal(idx, g[f"idx_{r}"]) and np.array_equal(y, g[f"y_{r}"])
        for k, t in enumerate((1, 2, 5)):
            assert np.array_equal(orc.amp(y, 0, Pl, L, M, t, Ab, Az).reshape(-1), g[f"traj_{r}"][k])
        b, t = orc.amp_test(y, 0, Pl, L, M, T, Ab, Az)
        assert np.array_equal(b, g[f"beta_{r}"]) and t == int(g[f"t_{r}"])


def test_ordering_hashes_all_configs():
    with open(os.path.join(GOLDEN, "meta.json")) as fh:
        meta = json.load(fh)
    for key, h in meta["ordering_sha256"].items():
        L, M, n = (int(p[1:]) for p in key.split("_"))
        assert sha(orc.make_ordering(L, M, n, 0)) == h, key


def test_c2_decode_matches_reference():
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, ordering = orc.sparc_transforms(L, M, n)
    assert sha(ordering) == str(g["ordering_sha256"])
    Pl = float(g["P"]) / L * np.ones(L)
    idx, y = orc.rep_inputs(L, M, n, Pl, float(g["sigma"]), Ab, 1000)
    assert np.array_equal(y, g["y"]) and np.array_equal(idx, g["idx"])
    b1 = orc.amp(y, 0, Pl, L, M, 1, Ab, Az)
    assert np.array_equal(b1.astype(np.float32), g["beta_t1"])
    b, t = orc.amp_test(y, 0, Pl, L, M, T, Ab, Az)
    assert np.array_equal(b.astype(np.float32), g["beta_final"]) and t == int(g["t_stop"])
    assert np.array_equal(orc.section_argmax(b, L, M), g["argmax_final"])


def test_c2_section_stats_match_reference():
    """sections.npz (make_section_stats.py, the reference's own decode): the
    oracle's per-section statistics of every C2 section at t = 1 and 8 are
    the reference's bit for bit (the GPU tests hold the device to them)."""
    g = golden("c2.npz")
    S = golden("sections.npz")
    L, M, n = int(g["L"]), int(g["M"]), int(g["n"])
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    Pl = float(g["P"]) / L * np.ones(L)
    for t in (1, 8):
        b = orc.amp(g["y"], 0, Pl, L, M, t, Ab, Az).reshape(L, M)
        assert np.array_equal((b * b).sum(axis=1), S[f"c2_t{t}_e2"]), t
        assert np.array_equal((b * np.arange(M)[None, :]).sum(axis=1), S[f"c2_t{t}_m1"]), t
        assert np.array_equal(b.max(axis=1), S[f"c2_t{t}_mx"]), t
    assert int(S["c2_t_stop"]) == int(g["t_stop"])


def test_c5_draw_order_and_one_decode():
    """The harness draw order (np.random.seed -> randint bits -> randn noise,
    sparc_ldpc.py:423-446) and one full decode against amp_ldpc_sim."""
    g = golden("c5_reps.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    Pl = float(g["P"]) / L * np.ones(L)
    for s in range(3):
        np.random.seed(s)
        bits = np.random.randint(0, 2, L * 9).tolist()
        assert np.array_equal(np.array(bits, dtype=np.uint8), g[f"bits_{s}"])
        idx = orc.bits2indices(bits, M)
        assert np.array_equal(idx, g[f"idx_{s}"])
        b0 = np.zeros((L * M, 1)); b0[np.arange(L) * M + np.array(idx), 0] = np.sqrt(n * Pl)
        y = (Ab(b0) + np.random.randn(n, 1) * float(g["sigma"])).reshape(-1, 1)
        assert np.array_equal(y, g[f"y_{s}"])
    b = orc.amp(g["y_0"], 0, Pl, L, M, T, Ab, Az)
    rx = orc.section_argmax(b, L, M)
    assert np.array_equal(rx, g["rx_0"])
    assert orc.ber_indices(g["idx_0"], rx, L * 9) == float(g["ber_0"])


def test_dense_matrix_and_factorisation():
    """A[r, l*M+c] from the popcount formula equals the FWHT operator, and it
    factorises as sgn(o >> log2 M) * H_M[o & (M-1), c] / sqrt(n) (DESIGN.md §2:
    the identity the HIP kernels are built on)."""
    g = golden("small.npz")
    L, M, n = int(g["L"]), int(g["M"]), int(g["n"])
    ordering = g["ordering"]
    A = orc.dense_design_matrix(L, M, n, ordering)
    assert np.allclose(A @ g["brand"], g["Ab_brand"], rtol=0, atol=1e-13)
    assert np.allclose(A.T @ g["zrand"], g["Az_zrand"], rtol=0, atol=1e-13)
    lg = int(np.log2(M))
    H = np.array([[(-1) ** bin(i & j).count("1") for j in range(M)] for i in range(M)], dtype=float)
    for l in range(L):
        o = ordering[l].astype(np.int64)
        sgn = np.array([(-1) ** bin(int(h)).count("1") for h in (o >> lg)], dtype=float)
        F = sgn[:, None] * H[o & (M - 1)] / np.sqrt(n)
        assert np.array_equal(np.sign(F), np.sign(A[:, l * M:(l + 1) * M]))


@pytest.mark.parametrize("L,M,R", [(16, 8, 1.0), (32, 64, 1.0), (8, 256, 0.75)])
def test_bucket_factorisation_model(L, M, R):
    """NumPy model of the kernel algorithm (inverse-table bucket gather +
    M-point FWHT for Az; M-point FWHT + signed gather for Ab) equals the
    oracle to fp64 rounding.  Documents the math of sparc_amp.hip."""
    n = int(L * np.log2(M) / R)
    Ab, Az, ordering = orc.sparc_transforms(L, M, n)
    w = orc._w_of(n, M)
    lg = int(np.log2(M))
    rs = np.random.RandomState(3)
    z = rs.randn(n)
    b = rs.randn(L * M)
    zs = np.append(z, 0.0)
    az = np.empty(L * M)
    ab = np.zeros(n)
    for l in range(L):
        inv = np.full(w, n)
        inv[ordering[l]] = np.arange(n)
        hi = np.arange(w // M)
        sg = np.array([(-1) ** bin(int(h)).count("1") for h in hi], dtype=float)
        v = (sg[:, None] * zs[inv.reshape(w // M, M)]).sum(axis=0)
        orc.fht_inplace(v)
        az[l * M:(l + 1) * M] = v
        t = b[l * M:(l + 1) * M].copy()
        orc.fht_inplace(t)
        o = ordering[l].astype(np.int64)
        sgr = np.array([(-1) ** bin(int(h)).count("1") for h in (o >> lg)], dtype=float)
        ab += sgr * t[o & (M - 1)]
    assert np.allclose(az / np.sqrt(n), Az(z).reshape(-1), rtol=0, atol=1e-12)
    assert np.allclose(ab / np.sqrt(n), Ab(b).reshape(-1), rtol=0, atol=1e-12)


def test_c4_oracle_matches_reference():
    """BASELINE configs[3] (L=768 M=512 R=5/6, w=16384): inputs, t=1 and the
    converged decode at sigma=0.6 bit for bit (tests/golden/make_c4_golden.py)."""
    g = golden("c4.npz")
    L, M, n, T, NS = (int(g[k]) for k in ("L", "M", "n", "T", "NS"))
    Ab, Az, ordering = orc.sparc_transforms(L, M, n)
    assert sha(ordering) == str(g["ordering_sha256"])
    Pl = float(g["P"]) / L * np.ones(L)
    for k in (0, 1):
        idx, y = orc.rep_inputs(L, M, n, Pl, float(g[f"sigma_{k}"]), Ab, 2000 + k)
        assert np.array_equal(y, g[f"y_{k}"]) and np.array_equal(idx, g[f"idx_{k}"])
        b1 = orc.amp(y, 0, Pl, L, M, 1, Ab, Az).astype(np.float32)
        assert np.array_equal(b1[:NS * M], g[f"beta_t1_{k}"])
        assert float(np.linalg.norm(b1.astype(np.float64))) == float(g[f"beta_t1_norm_{k}"])
    b, t = orc.amp_test(g["y_1"], 0, Pl, L, M, T, Ab, Az)
    assert t == int(g["t_stop_1"])
    assert np.array_equal(b[:NS * M].astype(np.float32), g["beta_final_1"])
    assert np.array_equal(orc.section_argmax(b, L, M), g["argmax_final_1"])
    assert float(np.linalg.norm(b)) == float(g["beta_final_norm_1"])


def test_oracle_amp_test_reps_golden():
    """The oracle reproduces the reference's seeded amp_test.py reps (first 3 of
    the small case of tests/golden/amp_test_reps.npz): hard / soft / no-init
    error counts, with the draws of amp_test.py:185-199."""
    import json
    with open(os.path.join(GOLDEN, "amp_test_reps.json")) as fh:
        m = json.load(fh)["small"]
    g = golden("amp_test_reps.npz")
    L, M, Lz, P, T = m["L"], m["M"], m["L_zero"], m["P"], m["T"]
    n, sigma = m["n"], m["sigma"]
    tb = int(L * np.log2(M))
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = orc.sparc_transforms(L, M, n)
    Ab_n, Az_n = orc.sparc_transforms_shorter(Lz, M, n, ordering)
    np.random.seed(m["seed"])
    for r in range(3):
        idx = np.asarray(orc.bits2indices(np.random.randint(0, 2, tb).tolist(), M))
        noise = np.random.randn(n, 1) * sigma
        beta = np.zeros((L * M, 1)); beta[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
        y = Ab(beta) + noise
        b0 = beta / np.sqrt(n * P / L); b0[:Lz * M] = 0
        bh = orc.amp(y - Ab(b0), sigma, Pl[:Lz], Lz, M, T, Ab_n, Az_n)
        bs = orc.amp(y, sigma, Pl, L, M, T, Ab, Az, b0)
        bz = orc.amp(y, sigma, Pl, L, M, T, Ab, Az)
        got = [round(orc.ber_indices(idx[:Lz], orc.section_argmax(bh, Lz, M), 1)),
               round(orc.ber_indices(idx, orc.section_argmax(bs, L, M), 1)),
               round(orc.ber_indices(idx, orc.section_argmax(bz, L, M), 1))]
        assert got == g["small_counts"][r].tolist(), (r, got)
