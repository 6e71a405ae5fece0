"""GPU: the BER curve overlays the reference's published curves (statistical
parity).  The reference never seeded its simulations, so agreement is in
distribution: our BER must fall inside the spread of the reference's three
independent runs widened by 1.5x at every point whose BER is >= 1e-3."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_plain_waterfall_overlays_reference(lib_gpu):
    import sparc_ldpc_amd as sp
    with open(os.path.join(GOLDEN, "published_ber.json")) as fh:
        pub = json.load(fh)["waterfall_plain"]
    c = pub["config"]
    ebno = np.array(pub["EbN0_dB"][:4])
    rows = sp.waterfall_plain(c["L"], c["M"], c["P"], c["R"], c["T"], ebno, c["MIN_ERRORS"],
                              c["MAX_BLOCKS"], batch=64)
    runs = np.array(list(pub["BER_plain_runs"].values()))  # 3 x 10
    for i, r in enumerate(rows):
        lo, hi = runs[:, i].min() / 1.5, runs[:, i].max() * 1.5
        assert lo <= r["BER_plain"] <= hi, (r["EbN0_dB"], r["BER_plain"], lo, hi)
        assert r["blocks"] <= c["MAX_BLOCKS"]
