"""CPU: the host-side EXIT helpers (amp_exit.py:28-351) on the reference's own
calc_E outputs (tests/golden/joint.npz)."""
import numpy as np

from conftest import golden


def test_hist_and_mutual_information_match_reference():
    from sparc_ldpc_amd import threshold as th
    g = golden("joint.npz")
    for s in range(4):
        key = f"exit|{s}"
        X, E = g[key + "|X"], g[key + "|E"]
        PE_pos, PE_neg, mp, mn, vp, vn, bw = th.hist_E(X, E)
        got = np.array([mp, mn, vp, vn, bw, th.calc_I_e(PE_pos, PE_neg, bw)])
        np.testing.assert_allclose(got, g[key + "|hist"], rtol=1e-12, atol=0)


def test_J_functions_roundtrip():
    from sparc_ldpc_amd import threshold as th
    for I in (0.05, 0.2, 0.3646, 0.5, 0.9):
        s = th.J_inverse(I)
        assert abs(th.J(s) - I) < 0.02
    c = th.polynomial(np.linspace(0, 1, 9), np.linspace(0, 1, 9) ** 2)
    np.testing.assert_allclose(c, [0, 0, 1, 0], atol=1e-12)
