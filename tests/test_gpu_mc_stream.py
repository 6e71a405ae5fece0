"""GPU: the Monte-Carlo rep stream (sa_mc_stage / sa_mc_run, sa_mc.hip) — the
reps of BASELINE configs[3] decoded through refilled slots — against the
batch-by-batch decode of the same seeds (mc_decode_batched: sa_encode +
sa_run with the exact-tau stop + sa_decide, sparc_ldpc.py:189-222 /
amp_test.py:183-246).  A codeword's decode does not depend on its slot or on
the other codewords, so every rep's bit errors and stop index must be
identical (bit for bit), whatever the slot count, the rep count, T or the
precision."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sp(lib_gpu):
    import sparc_ldpc_amd
    return sparc_ldpc_amd


def _op(sp, L, M, R, prec):
    n = int(L * np.log2(M) / R)
    return sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)


def test_l768_sweep_stream_equals_batches(sp):
    """A reduced configs[3] sweep (L=768 M=512 at the sweep's rate R=0.8765,
    n=7885, P=1.8, T=64): 3 sigma points x 96 reps as ONE stream through 64
    slots (the points' reps interleave in the slots) against mc_decode_batched
    at batch 64 per point: identical per-rep bit errors and stop indices, and
    the stream's BER column equal to the batched one."""
    L, M, P, T = 768, 512, 1.8, 64
    R = (L * 9 - 9 * 569 * (1 - 5 / 6)) / (L * 9)
    op = _op(sp, L, M, R, "fp32")
    n = op.n
    assert n == 7885 and op.mc_supported(64)
    Pl = P / L * np.ones(L)
    sigmas = (0.8, 0.6, 0.45)
    seeds = [list(range(i * 100000, i * 100000 + 96)) for i in range(len(sigmas))]
    idx = np.concatenate([sp.draw_reps(s, L, M, n, sg)[0] for s, sg in zip(seeds, sigmas)])
    noise = np.concatenate([sp.draw_reps(s, L, M, n, sg)[1] for s, sg in zip(seeds, sigmas)])
    be, it, ms = sp.mc_stream(op, Pl, T, idx, noise, batch=64)
    assert ms > 0
    for i, sg in enumerate(sigmas):
        be0, it0 = sp.mc_decode_batched(op, Pl, sg, T, seeds[i], batch=64)
        np.testing.assert_array_equal(be[i * 96:(i + 1) * 96], be0, err_msg=f"bit errors, sigma {sg}")
        np.testing.assert_array_equal(it[i * 96:(i + 1) * 96], it0, err_msg=f"stop index, sigma {sg}")
    assert it.min() >= 0 and it.max() <= T
    assert (it < T).any() and be[-96:].sum() <= be[:96].sum()  # stops fire; the waterfall falls


@pytest.mark.parametrize("prec,B,nreps,T,es", [
    ("fp32", 16, 5, 20, True),     # fewer reps than slots: empty slots from the start
    ("fp32", 8, 37, 3, True),      # T = 3: most reps run out; reps not a multiple of the slots
    ("fp32", 12, 40, 12, False),   # no early stop: every rep runs T iterations
    ("fp64", 8, 30, 25, True),     # binary64 (CB = 2)
])
def test_stream_edge_cases(sp, prec, B, nreps, T, es):
    """Small L=128 M=256 R=1 streams over the slot / rep / T / precision edge
    cases against mc_decode_batched (batch 8), twice on one operator (the
    cached stream graph) with a plain batched decode in between (the per-slot
    iteration pointer must not leak into the ordinary graphs)."""
    L, M = 128, 256
    op = _op(sp, L, M, 1.0, prec)
    n = op.n
    assert op.mc_supported(B)
    Pl = 2.0 / L * np.ones(L)
    seeds = list(range(500, 500 + nreps))
    sg = 0.55
    ref_be, ref_it = sp.mc_decode_batched(op, Pl, sg, T, seeds, batch=8, early_stop=es)
    idx, noise = sp.draw_reps(seeds, L, M, n, sg)
    for rnd in range(2):
        be, it, _ = sp.mc_stream(op, Pl, T, idx, noise, batch=B, early_stop=es)
        np.testing.assert_array_equal(be, ref_be, err_msg=f"round {rnd}")
        np.testing.assert_array_equal(it, ref_it, err_msg=f"round {rnd}")
        # an ordinary batched decode between the streams, checked against its first run
        b1, i1 = op.amp_batch(noise[:8] * 4.0, Pl, T)
        if rnd == 0:
            first = (b1, i1)
        else:
            assert np.array_equal(b1, first[0]) and np.array_equal(i1, first[1])
    if not es:
        assert np.all(it == T)


def test_stream_decisions_are_the_decode_argmax(sp):
    """The stream's decisions are the section argmax of the decode's estimate
    (sparc_ldpc.py:452-455): per rep equal to sa_decide after amp_batch of the
    same y (sa_encode of the same indices and noise)."""
    L, M, T = 64, 64, 15
    op = _op(sp, L, M, 1.0, "fp32")
    n = op.n
    Pl = 2.0 / L * np.ones(L)
    seeds = list(range(9000, 9024))
    idx, noise = sp.draw_reps(seeds, L, M, n, 0.7)
    op.reserve(24, T)
    op.stage_power(24, Pl)
    op.mc_stage(idx, noise)
    dec, its, errs, _ = op.mc_run(8, T)
    op.encode(idx, noise)
    op.run(24, T)
    np.testing.assert_array_equal(dec, op.decide(24))
    np.testing.assert_array_equal(its, op.iters(24))
    np.testing.assert_array_equal(errs, sp.ber_of(idx, dec, 1).astype(np.int64))


def test_stream_refuses_unsupported(sp):
    """A stream needs the batched codeword-interleaved decode: the dense
    backend, a single slot and an unstaged power allocation are refused."""
    L, M = 32, 64
    n = int(L * np.log2(M))
    dense = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense", precision="fp32")
    assert not dense.mc_supported(8)
    op = _op(sp, L, M, 1.0, "fp32")
    idx, noise = sp.draw_reps([1, 2, 3], L, M, n, 0.5)
    op.mc_stage(idx, noise)
    with pytest.raises((AssertionError, sp.SparcAmpError)):  # SA_ERR_ARG raises AssertionError
        op.mc_run(2, 10)          # B < 4
    with pytest.raises((AssertionError, sp.SparcAmpError)):
        op.mc_run(8, 10)          # no power allocation staged
