"""The amp_test.py reps loop (amp_test.py:161-253) batched on the device and
sharded over ranks, against the reference's own seeded reps
(tests/golden/make_amp_test_golden.py): per rep the bit errors of the hard
init (shortened operator after the 0/1 cancellation), the soft init (0/1
beta_0) and the zero start, and the three BERs the loop prints."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

pytestmark = pytest.mark.gpu


def _case(name):
    with open(os.path.join(GOLDEN, "amp_test_reps.json")) as fh:
        meta = json.load(fh)[name]
    g = golden("amp_test_reps.npz")
    kw = {k: meta[k] for k in ("L", "M", "L_zero", "P", "snr_dB", "r_sparc", "T", "repeats")}
    return meta, kw, g


@pytest.fixture(scope="module")
def sp(lib_gpu):
    import sparc_ldpc_amd
    return sparc_ldpc_amd


@pytest.mark.parametrize("name,batch", [("main", 8), ("main", 3), ("small", 24), ("small", 5)])
def test_amp_test_reps_fp64_matches_reference(sp, name, batch):
    """binary64: every rep's three error counts and the three BERs exactly
    (batch 3 / 5: several device rounds, a ragged last one)."""
    meta, kw, g = _case(name)
    np.random.seed(meta["seed"])
    bers, counts = sp.amp_test_reps(**kw, precision="fp64", batch=batch, return_counts=True)
    assert np.array_equal(counts, g[f"{name}_counts"]), (counts.tolist(), g[f"{name}_counts"].tolist())
    assert bers == (meta["ber_hard"], meta["ber_soft"], meta["ber_no_init"])


def test_amp_test_reps_fp32(sp):
    """binary32 (north_star's 1e-5 contract): a section whose two largest
    posteriors tie to ~1e-7 may flip, so per-rep counts within 1 % + 9 bits."""
    meta, kw, g = _case("small")
    np.random.seed(meta["seed"])
    bers, counts = sp.amp_test_reps(**kw, precision="fp32", batch=24, return_counts=True)
    ref = g["small_counts"]
    assert np.all(np.abs(counts - ref) <= 0.01 * ref + 9), (counts.tolist(), ref.tolist())


def test_amp_test_reps_sharded_equals_single(sp):
    """world = 2 (each rank decodes reps i % 2 == rank; the per-rep counts are
    summed over ranks): identical to one process, for every rank."""
    meta, kw, g = _case("small")
    parts = {}
    for rank in (1, 0):
        np.random.seed(meta["seed"])
        other = parts.get(1)
        red = (lambda c: c) if other is None else (lambda c, o=other: c + o)
        bers, counts = sp.amp_test_reps(**kw, precision="fp64", batch=8, rank=rank, world=2,
                                        allreduce=red, return_counts=True)
        own = np.zeros_like(counts)
        own[rank::2] = counts[rank::2]
        parts[rank] = own
        if rank == 0:
            assert np.array_equal(counts, g["small_counts"])
            assert bers == (meta["ber_hard"], meta["ber_soft"], meta["ber_no_init"])
    with pytest.raises(ValueError):
        np.random.seed(meta["seed"])
        sp.amp_test_reps(**kw, precision="fp64", rank=0, world=2)
