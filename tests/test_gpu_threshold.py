"""GPU: threshold-initialised exchange (soft_amp_ldpc_hardinit,
sparc_ldpc.py:862-1047) and the AMP EXIT measurement calc_E (amp_exit.py:185-270)
against reps of the reference itself (tests/golden/joint.npz, seeded np.random,
fp64).  BERs exactly when the reference's BP calls converged, else within
0.03; extrinsic LLRs E within 1e-8 relative where |E| < 50 (the clip at +-55
and saturated values compared by sign), histogram statistics within 1e-6."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _keys(prefix):
    g = golden("joint.npz")
    depth = prefix.count("|") + 1  # key fields + the array name
    return sorted({k.rsplit("|", 1)[0] for k in g
                   if k.startswith(prefix) and k.count("|") == depth and not k.endswith("|cfg")})


@pytest.mark.parametrize("key", _keys("thr|hardinit|"))
def test_hardinit_reps_match_reference(key):
    import sparc_ldpc_amd as sp
    g = golden("joint.npz")
    L, M, P, r, T, z, sigma, thr = g["thr|cfg"]
    spp = sp.SPARCParams(int(L), int(M), float(sigma), float(P), float(r), int(T))
    lp = sp.LDPCParams("802.16", "5/6", int(z))
    np.random.seed(int(key.split("|")[-1]))
    ba, bl, R = sp.soft_amp_ldpc_hardinit(spp, lp, 3, float(thr))
    got = np.array(list(ba) + list(bl))
    ref = g[key + "|ber"]
    assert got.shape == ref.shape and abs(R - g[key + "|R"][0]) < 1e-15
    assert got[0] == ref[0]
    its = [int(g[key + f"|it{k}"][0]) for k in range(3) if key + f"|it{k}" in g]
    if all(i < 200 for i in its):
        np.testing.assert_array_equal(got, ref)
    else:
        assert np.max(np.abs(got - ref)) <= 0.03


@pytest.mark.parametrize("key", _keys("exit|"))
def test_calc_E_matches_reference(key):
    import sparc_ldpc_amd as sp
    g = golden("joint.npz")
    L, M, P, r, T = g["exit|cfg"]
    spp = sp.SPARCParams(int(L), int(M), None, float(P), float(r), int(T))
    I_a, snr_db, thr = g[key + "|par"]
    s = int(key.split("|")[1])
    np.random.seed(100 + s)
    X = sp.threshold.gen_bits(int(L * np.log2(M)))
    assert np.array_equal(X, g[key + "|X"])
    E = sp.calc_E(X, float(I_a), float(snr_db), spp, None, float(thr))
    Er = g[key + "|E"]
    mid = np.abs(Er) < 50
    np.testing.assert_allclose(E[mid], Er[mid], rtol=1e-8, atol=1e-8)
    assert np.array_equal(np.sign(E[~mid]), np.sign(Er[~mid]))
    h = sp.hist_E(X, E)
    got = np.array([h[2], h[3], h[4], h[5], h[6], sp.calc_I_e(h[0], h[1], h[6])])
    np.testing.assert_allclose(got, g[key + "|hist"], rtol=1e-6, atol=1e-9)


def test_hard_initialisation_dropin():
    """amp_exit.hard_initialisation with the reference's signature: decided
    sections cancelled through the device Ab, the rest on a shortened operator."""
    import sparc_ldpc_amd as sp
    L, M, n = 32, 16, 128
    Ab, Az, ordering = sp.sparc_transforms(L, M, n, precision="fp64")
    Pl = 4.0 / L * np.ones(L)
    rs = np.random.RandomState(3)
    beta = rs.dirichlet(np.ones(M) * 0.05, L).reshape(-1, 1)
    y = rs.randn(n, 1)
    b = beta.copy()
    y_new, Ab_new, Az_new, secs, Ls = sp.hard_initialisation(b, L, M, n, ordering, y, Pl, Ab, 0.6, 20)
    # decided = LDPC sections (last 20) with exactly one entry > 0.6
    dec = [l for l in range(L - 20, L) if (beta[l * M:(l + 1) * M, 0] > 0.6).sum() == 1]
    assert secs == [l for l in range(L) if l not in dec] and Ls == len(secs)
    ref = np.zeros((L * M, 1))
    for l in dec:
        ref[l * M + int(np.argmax(beta[l * M:(l + 1) * M, 0]))] = np.sqrt(n * Pl[l])
    assert np.array_equal(b, ref)
    np.testing.assert_allclose(y_new, y - Ab(ref), rtol=0, atol=1e-12)
    v = rs.randn(Ls * M, 1)
    Ab_s, _ = sp.sparc_transforms_shorter(Ls, M, n, ordering[secs], precision="fp64")
    np.testing.assert_allclose(Ab_new(v), Ab_s(v), rtol=0, atol=1e-12)


def test_hardinit_batched_matches_reference():
    """The same reference reps decoded as ONE batch (JointDecoder mode
    "threshold": every codeword's undecided sections as a per-codeword mask on
    one full-size operator) instead of per-codeword shortened operators."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd.joint import joint_decoder
    g = golden("joint.npz")
    L, M, P, r, T, z, sigma, thr = g["thr|cfg"]
    L, M, T = int(L), int(M), int(T)
    n = int(L * np.log2(M) / float(r))
    keys = _keys("thr|hardinit|")
    seeds = [int(k.split("|")[-1]) for k in keys]
    jd = joint_decoder(L, M, n, sp.LDPCParams("802.16", "5/6", int(z)), T, precision="fp64")
    idx, noise = jd.draw([np.random.RandomState(s) for s in seeds], len(seeds), float(sigma))
    out = jd.run(idx, noise, float(P) / L * np.ones(L), "threshold", 3, float(thr))
    tb = jd.total_bits
    for i, key in enumerate(keys):
        assert np.array_equal(idx[i], g[key + "|idx"].astype(np.int32))
        got = np.concatenate([out["amp"][i], out["ldpc"][i]]) / tb
        ref = g[key + "|ber"]
        assert got.shape == ref.shape and got[0] == ref[0]
        its = [int(g[key + f"|it{k}"][0]) for k in range(3) if key + f"|it{k}" in g]
        if all(it < 200 for it in its):
            np.testing.assert_array_equal(got, ref)
        else:
            assert np.max(np.abs(got - ref)) <= 0.03


@pytest.mark.parametrize("L,M,n,B", [(64, 32, 320, 5), (64, 32, 320, 2), (256, 256, 2048, 1)])
def test_power_batch_mask_equals_shortened_operator(L, M, n, B):
    """Pl = 0 sections of a per-codeword power allocation = the reference's
    sparc_transforms_shorter decode over the other sections (fp64, different
    summation grouping only); equal rows reproduce the shared allocation
    bit for bit.  Batched (k_secb), unbatched (k_sec) and k_sec4 paths."""
    import sparc_ldpc_amd as sp
    T = 16
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp64", device=0)
    Pl = 4.0 / L * np.ones(L)
    rs = np.random.RandomState(11)
    idx = rs.randint(0, M, (B, L)).astype(np.int32)
    op.reserve(B, T)
    op.stage_power(B, Pl)
    op.encode(idx, 0.4 * rs.randn(B, n))
    op.run(B, T)
    op.wait()
    ref_shared, it_shared = op.fetch(B)
    op.stage_power_batch(B, np.tile(Pl, (B, 1)))
    op.run(B, T)
    op.wait()
    got, it = op.fetch(B)
    assert np.array_equal(got, ref_shared) and np.array_equal(it, it_shared)
    # masks: codeword b drops a different random subset of sections
    masks = rs.rand(B, L) < 0.3
    op.stage_power_batch(B, np.where(masks, 0.0, Pl[None, :]))
    op.run(B, T)
    op.wait()
    got, it = op.fetch(B)
    assert all(np.all(got[b].reshape(L, M)[masks[b]] == 0) for b in range(B))
    # the masked decode equals AMP over the kept sections on the host operator
    from oracle import amp_oracle as orc
    oAb, oAz, oord = orc.sparc_transforms(L, M, n)
    rs2 = np.random.RandomState(11)
    _ = rs2.randint(0, M, (B, L))
    noise = 0.4 * rs2.randn(B, n)
    c = np.sqrt(n * Pl)
    for b in range(B):
        beta0 = np.zeros((L * M, 1))
        beta0[np.arange(L) * M + idx[b], 0] = c
        yb = oAb(beta0) + noise[b].reshape(-1, 1)
        keep = np.nonzero(~masks[b])[0]
        sAb, sAz = orc.sparc_transforms_shorter(len(keep), M, n, oord[keep])
        refb = orc.amp(yb, 0, Pl[keep], len(keep), M, T, sAb, sAz).reshape(len(keep), M)
        np.testing.assert_allclose(got[b].reshape(L, M)[keep], refb, rtol=0, atol=1e-9 * np.abs(refb).max())


def test_calc_E_batch_matches_reference():
    """The reference's calc_E reps (tests/golden/joint.npz) decoded as one batch
    (calc_E_batch: per-codeword section masks), draws replayed by exit_draws."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd import threshold as th
    g = golden("joint.npz")
    L, M, P, r, T = g["exit|cfg"]
    L, M, T = int(L), int(M), int(T)
    spp = sp.SPARCParams(L, M, None, float(P), float(r), T)
    n = int(L * np.log2(M) / float(r))
    keys = _keys("exit|")
    Xs, As, ws, thrs = [], [], [], []
    for key in keys:
        I_a, snr_db, thr = g[key + "|par"]
        s = int(key.split("|")[1])
        X, A, w = th.exit_draws([(float(I_a), float(snr_db))], L, M, n, float(P), np.random.RandomState(100 + s))
        assert np.array_equal(X[0], g[key + "|X"])
        Xs.append(X[0]); As.append(A[0]); ws.append(w[0]); thrs.append(float(thr))
    E = np.empty((len(keys), len(Xs[0])))
    for thr in set(thrs):  # one batch per threshold
        sel = [b for b in range(len(keys)) if thrs[b] == thr]
        E[sel] = th.calc_E_batch(np.stack([Xs[b] for b in sel]), np.stack([As[b] for b in sel]),
                                 np.stack([ws[b] for b in sel]), spp, thr)
    for b, key in enumerate(keys):
        Er = g[key + "|E"]
        mid = np.abs(Er) < 50
        np.testing.assert_allclose(E[b][mid], Er[mid], rtol=1e-8, atol=1e-8)
        assert np.array_equal(np.sign(E[b][~mid]), np.sign(Er[~mid]))


def test_amp_exit_curve_matches_sequential_calc_E():
    """amp_exit_curve (amp_exit.py:520-631), batched, against the same sweep
    made of per-codeword calc_E calls in the reference's draw order."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd import threshold as th
    spp = sp.SPARCParams(64, 16, None, 4.0, 1.0, 30)
    reps, pts, thr = 2, 4, 0.7
    np.random.seed(123)
    I_a, snr, I_e, poly = th.amp_exit_curve(spp, 6.0, 12.0, reps, pts, thr, bin_number=125, batch=11)
    assert I_e.shape == (4, pts) and np.all((I_e >= 0) & (I_e <= 1)) and poly.shape == (4,)
    np.random.seed(123)
    ref = np.zeros((4, pts))
    for k in range(reps):
        for j, s in enumerate(snr):
            for i, ia in enumerate(I_a):
                X = th.gen_bits(64 * 4)
                E = th.calc_E(X, ia, s, spp, None, thr)
                h = th.hist_E(X, E, bin_number=125, max_bin=60, min_bin=-60)
                ref[j, i] += th.calc_I_e(h[0], h[1], h[6])
    ref /= reps
    np.testing.assert_allclose(I_e, ref, rtol=0, atol=1e-6)
    assert I_e[:, -1].mean() > I_e[:, 0].mean()  # more a-priori information, more extrinsic
