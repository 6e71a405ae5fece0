"""GPU: the joint SPARC + LDPC decoder (AMP <-> BP on the device) against reps
of the reference's own simulators (tests/golden/joint.npz: amp_ldpc_sim with an
LDPC code, soft_amp_ldpc_sim, hardinitbeta_amp_ldpc_sim on seeded np.random,
their decoder calls through the reference C sumprod2).

Precision fp64 (the reference's).  Bars: the first AMP stage's BER exactly;
the LLRs handed to BP within 1e-9 relative wherever the bit posterior is not
within 1e-6 of 0 or 1 (1 - p cancels there), same saturation elsewhere; BP
iteration counts exactly; and every later BER exactly whenever the
reference's BP calls converged (< 200 iterations).  After a non-converging
200-iteration BP the app values amplify last-ulp differences, so those later
stages are held to |dBER| <= 0.03."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _cases():
    g = golden("joint.npz")
    keys = sorted({k.rsplit("|", 1)[0] for k in g if k.count("|") == 3
                   and k.split("|")[1] in ("originalHard", "soft", "hard")})
    return [k for k in keys]


@pytest.fixture(scope="module")
def G():
    return golden("joint.npz")


def _params(G, tag):
    from sparc_ldpc_amd import SPARCParams, LDPCParams
    L, M, P, r, T, z, sigma = G[f"{tag}|cfg"]
    return SPARCParams(int(L), int(M), float(sigma), float(P), float(r), int(T)), LDPCParams("802.16", "5/6", int(z))


@pytest.mark.parametrize("key", _cases())
def test_joint_reps_match_reference(G, key):
    import sparc_ldpc_amd as sp
    tag, mode, seed = key.split("|")
    spp, lp = _params(G, tag)
    np.random.seed(int(seed))
    if mode == "originalHard":
        ba, bl, bla, R = sp.amp_ldpc_sim(spp, lp, precision="fp64")
        got = [ba, bl, -1.0 if bla is None else bla]
    elif mode == "soft":
        ba, bl, R = sp.soft_amp_ldpc_sim(spp, lp, 2, precision="fp64")
        got = list(ba) + list(bl)
    else:
        ba, bl, R = sp.hardinitbeta_amp_ldpc_sim(spp, lp, precision="fp64")
        got = list(ba) + list(bl)
    ref = G[key + "|ber"]
    assert abs(R - G[key + "|R"][0]) < 1e-15
    assert got[0] == ref[0]
    its = [int(G[key + f"|it{k}"][0]) for k in range(4) if key + f"|it{k}" in G]
    if all(i < 200 for i in its):
        np.testing.assert_array_equal(np.array(got), ref)
    else:
        assert np.max(np.abs(np.array(got) - ref)) <= 0.03


@pytest.mark.parametrize("key", [k for k in _cases() if k.endswith("|soft|1") or k.startswith("c5|")])
def test_llr_and_bp_on_reference_inputs(G, key):
    """First BP call: our device LLRs vs the reference's, and our BP on the
    reference's LLRs vs the reference's app / iteration count."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd.joint import joint_decoder
    tag, mode, seed = key.split("|")
    spp, lp = _params(G, tag)
    L, M = spp.L, spp.M
    n = int(L * np.log2(M) / spp.r)
    jd = joint_decoder(L, M, n, lp, spp.t, precision="fp64")
    np.random.seed(int(seed))
    idx, noise = jd.draw(np.random, 1, spp.sigma)
    Pl = spp.p / L * np.ones(L)
    op = jd.op
    op.reserve(1, spp.t)
    op.stage_power(1, Pl)
    op.encode(idx, noise)
    op.run(1, spp.t)
    op.wait()
    llr = op.llr(1, jd.l0, jd.ns)[0]
    ref_llr = G[key + "|llr0"]
    with np.errstate(over="ignore"):
        p = 1.0 / (1.0 + np.exp(ref_llr))
    good = (p > 1e-6) & (p < 1 - 1e-6)
    np.testing.assert_allclose(llr[good], ref_llr[good], rtol=1e-9, atol=1e-9)
    assert np.array_equal(np.sign(llr[~good]), np.sign(ref_llr[~good]))
    sat = np.abs(ref_llr) == np.finfo(np.float64).max
    assert np.array_equal(np.abs(llr) == np.finfo(np.float64).max, sat)
    app, it = jd.code.decode(ref_llr)
    assert it == int(G[key + "|it0"][0])
    ref_app = G[key + "|app0"]
    if it < 200:
        assert np.array_equal(app < 0, ref_app < 0)
        np.testing.assert_allclose(app, ref_app, rtol=1e-9, atol=1e-9)


def test_batched_joint_equals_per_rep():
    """mc_joint over seeds == the per-rep pipeline on the same seeds (batch independence)."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd.joint import joint_decoder, mc_joint
    spp = sp.SPARCParams(64, 16, 0.93, 4.0, 1.0, 30)
    lp = sp.LDPCParams("802.16", "5/6", 8)
    jd = joint_decoder(64, 16, 256, lp, 30, precision="fp64")
    Pl = 4.0 / 64 * np.ones(64)
    for mode in ("originalHard", "soft", "hard"):
        allr = mc_joint(jd, Pl, spp.sigma, range(100, 112), mode, batch=5)
        for j, s in enumerate((100, 107, 111)):
            one = mc_joint(jd, Pl, spp.sigma, [s], mode, batch=1)
            for k in one:
                assert np.array_equal(one[k][0], allr[k][s - 100]), (mode, k)


def test_sim_ldpc_bpsk_runs():
    import sparc_ldpc_amd as sp
    lp = sp.LDPCParams("802.16", "5/6", 192)
    ber_hi = sp.sim_ldpc(lp, np.sqrt((1 / 10 ** (3.0 / 20)) / 2), MIN_ERRORS=20, MAX_BLOCKS=2000, batch=256, seed=1)
    ber_lo = sp.sim_ldpc(lp, np.sqrt((1 / 10 ** (5.0 / 20)) / 2), MIN_ERRORS=20, MAX_BLOCKS=512, batch=256, seed=1)
    assert ber_hi > ber_lo >= 0.0


def _batch_cases():
    keys = _cases()
    out = sorted({(k.split("|")[0], k.split("|")[1]) for k in keys})
    return out


def _per_rep_bers(r, j, mode, tb):
    if mode == "originalHard":
        return [r["amp"][j, 0] / tb, r["ldpc"][j, 0] / tb, r["ldpc_amp"][j] / tb if "ldpc_amp" in r else -1.0]
    return [e / tb for e in r["amp"][j]] + [e / tb for e in r["ldpc"][j]]


@pytest.mark.parametrize("tag,mode", _batch_cases())
def test_joint_reps_as_one_batch(G, tag, mode):
    """every reference rep of a (config, scheme) decoded
    in ONE batch padded to 256 codewords (mc_joint: the benched shape, two
    concurrent halves of 128 on their own streams), against the reference's
    per-rep BERs with the bars of test_joint_reps_match_reference; at full
    size (c5) also as one 256-codeword decoder."""
    from sparc_ldpc_amd import joint
    keys = [k for k in _cases() if k.startswith(f"{tag}|{mode}|")]
    seeds = [int(k.split("|")[2]) for k in keys]
    pad = [900_000 + i for i in range(256 - len(seeds))]
    spp, lp = _params(G, tag)
    jd, Pl = joint._setup(spp, lp, precision="fp64")
    tb = jd.total_bits
    runs = [True] + ([False] if tag == "c5" else [])
    for pipe in runs:
        r = joint.mc_joint(jd, Pl, spp.sigma, seeds + pad, mode, soft_iter=2, batch=256, pipeline=pipe)
        assert r["amp"].shape[0] == 256
        for j, key in enumerate(keys):
            got = np.array(_per_rep_bers(r, j, mode, tb))
            ref = G[key + "|ber"]
            assert got[0] == ref[0], (key, pipe)
            its = [int(G[key + f"|it{k}"][0]) for k in range(4) if key + f"|it{k}" in G]
            if all(i < 200 for i in its):
                np.testing.assert_array_equal(got, ref, err_msg=f"{key} pipeline={pipe}")
            else:
                assert np.max(np.abs(got - ref)) <= 0.03, (key, pipe)


def test_pipeline_equals_one_decoder():
    """JointPipeline (two halves, two threads, own streams) == one decoder over
    the batch, every per-rep count, for the three schemes and an odd batch."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd.joint import joint_decoder, mc_joint
    spp = sp.SPARCParams(64, 16, 0.95, 4.0, 1.0, 30)
    lp = sp.LDPCParams("802.16", "5/6", 8)
    jd = joint_decoder(64, 16, 256, lp, 30, precision="fp64")
    Pl = 4.0 / 64 * np.ones(64)
    for mode in ("originalHard", "soft", "hard"):
        a = mc_joint(jd, Pl, spp.sigma, range(300, 371), mode, batch=71, pipeline=False)
        b = mc_joint(jd, Pl, spp.sigma, range(300, 371), mode, batch=71, pipeline=True)
        for k in a:
            assert np.array_equal(a[k], b[k]), (mode, k)


def test_pipeline_slices_share_a_seeded_design():
    """A JointDecoder on the design of ordering seed 3, pipelined with and
    without twin slices: every slice decodes against the decoder's own design
    (untwinned slices re-derived the seed-0 ordering), so the
    per-rep results equal one decoder's over the batch."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd import joint
    lp = sp.LDPCParams("802.16", "5/6", 8)
    code = sp.code(lp.standard, lp.r_ldpc, lp.z)
    jd = joint.JointDecoder(64, 16, 256, code, 30, precision="fp64", seed=3)
    assert not np.array_equal(jd.op.ordering, sp.make_ordering(64, 16, 256, 0))
    Pl = 4.0 / 64 * np.ones(64)
    a = joint.mc_joint(jd, Pl, 0.95, range(400, 471), "soft", batch=71, pipeline=False)
    twin = joint.TWIN_SLICES
    try:
        for tw in (True, False):
            joint.TWIN_SLICES = tw
            jd._pipeline = None
            b = joint.mc_joint(jd, Pl, 0.95, range(400, 471), "soft", batch=71, pipeline=True)
            for p in jd._pipeline.parts:
                assert np.array_equal(p.op.ordering, jd.op.ordering)
            for k in a:
                assert np.array_equal(a[k], b[k]), (tw, k)
            jd._pipeline.close()
    finally:
        joint.TWIN_SLICES = twin
