"""CPU: host side of the joint SPARC + LDPC decoder — the reference's draw
order (message bits, LDPC encoding, section indices) and the sp2bp / bp2sp
helpers, against fixtures captured from the reference (tests/golden/joint.npz,
tests/golden/ldpc.npz)."""
import numpy as np

from conftest import golden


def _cases(g):
    keys = sorted({k.rsplit("|", 1)[0] for k in g if k.count("|") == 3
                   and k.split("|")[1] in ("originalHard", "soft", "hard")})
    for key in keys:
        tag, mode, seed = key.split("|")
        yield key, tag, mode, int(seed)


def test_draws_match_reference_indices():
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd.joint import draw_reps
    g = golden("joint.npz")
    codes = {}
    for key, tag, mode, seed in _cases(g):
        L, M, P, r, T, z, sigma = g[f"{tag}|cfg"]
        L, M, z = int(L), int(M), int(z)
        n = int(L * np.log2(M) / r)
        code = codes.setdefault(z, sp.code("802.16", "5/6", z))
        np.random.seed(seed)
        idx, noise = draw_reps(code, L, M, n, np.random, 1, sigma)
        assert np.array_equal(idx[0], g[key + "|idx"]), key
        assert noise.shape == (1, n)


def test_rate_of_joint_code():
    g = golden("joint.npz")
    for key, tag, mode, seed in _cases(g):
        L, M, P, r, T, z, sigma = g[f"{tag}|cfg"]
        n = int(L * np.log2(M) / r)
        nl, kl = 24 * int(z), 20 * int(z)
        assert abs(g[key + "|R"][0] - (L * np.log2(M) - (nl - kl)) / n) < 1e-15


def test_host_sp2bp_bp2sp_helpers():
    import sparc_ldpc_amd as sp
    g = golden("ldpc.npz")
    for L, M in ((6, 8), (4, 64), (3, 512)):
        p = sp.sp2bp(g[f"sp2bp|{L}|{M}|beta"], L, M)
        assert np.array_equal(p, g[f"sp2bp|{L}|{M}|p"])
        if M <= 64:
            np.testing.assert_allclose(sp.bp2sp(g[f"bp2sp|{L}|{M}|v"], L, M), g[f"bp2sp|{L}|{M}|sp"],
                                       rtol=1e-13, atol=0)
