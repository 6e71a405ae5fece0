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


@pytest.mark.parametrize("init", ["soft", "hard"])
def test_joint_waterfall_overlays_reference(lib_gpu, init):
    """configs[4]: L=M=512 with the 802.16 rate-5/6 code over all sections,
    AMP <-> BP exchange; the points where every column is >= 1e-3 (3.0 and
    6.89 dB) fall within 1.5x of the reference run of the same scheme."""
    import sparc_ldpc_amd as sp
    with open(os.path.join(GOLDEN, "published_ber.json")) as fh:
        pub = json.load(fh)["waterfall_joint"]
    c = pub["config"]
    ref = pub["runs"][init]
    pts = [0, 5]
    ebno = np.linspace(3, 10, 10)[pts]
    spp = sp.SPARCParams(c["L"], c["M"], None, c["P"], c["r_sparc"], c["T"])
    rows = sp.waterfall(spp, sp.LDPCParams("802.16", "5/6", None), init=init, MIN_ERRORS=c["MIN_ERRORS"],
                        MAX_BLOCKS=c["MAX_BLOCKS"], bpsk=True, batch=64, ebno_dbs=ebno)
    for i, r in zip(pts, rows):
        for col in ("BER_amp_1", "BER_ldpc", "BER_amp_2", "BER_plain"):
            lo, hi = ref[col][i] / 1.5, ref[col][i] * 1.5
            assert lo <= r[col] <= hi, (init, r["EbN0_dB"], col, r[col], ref[col][i])
        if i == 0:
            assert ref["BER_bpsk"][i] / 1.5 <= r["BER_bpsk"] <= ref["BER_bpsk"][i] * 1.5
