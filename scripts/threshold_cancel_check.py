"""Diagnostic: the threshold-initialised exchange at L=M=512 (802.16 5/6, all
sections, soft_iter=2, threshold 0.6) with the decided sections cancelled as
the current reference does (one-hot sqrt(n Pl_l), amp_exit.py:96-99) and as
its own comment says it used to (one-hot 1: "previously I was setting this to
1 which was an error", amp_exit.py:98).  Prints mean BERs per round for both
next to the published runs (thresholdinit_*_threshold0_6.csv)."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sparc_ldpc_amd as sp
from sparc_ldpc_amd.joint import joint_decoder

pub = json.load(open(os.path.join(ROOT, "tests/golden/published_ber.json")))["threshold_init"]
L = M = 512; P = 4.0; T = 64; logm = 9; n = 4608
jd = joint_decoder(L, M, n, sp.LDPCParams("802.16", "5/6", 192), T, precision="fp64")
Pl = P / L * np.ones(L)
c = np.sqrt(n * Pl)
mk = jd.op.subset(np.arange(L))
B = 100
sig_all = np.linspace(0.9, 1.4, 10)
for pi in [int(a) for a in (sys.argv[1:] or ["2", "4", "6"])]:
    sigma = sig_all[pi]
    res = {}
    for variant in ("current", "unit"):
        idx, noise = jd.draw([np.random.RandomState(1000 + s) for s in range(B)], B, sigma)
        op = jd.op
        jd.stage(idx, noise, Pl)
        beta0 = np.zeros((B, L * M))
        beta0[np.arange(B)[:, None], np.arange(L)[None, :] * M + idx] = c
        y = op.Ab_batch(beta0) + noise
        op.run(B, T); op.wait()
        rx = op.decide(B)
        e_amp = [jd._errs(idx, rx)]
        LLR = op.llr(B, 0, L)
        app, _ = jd.code.decode_batch(LLR)
        LLR[:] = app
        e_ldpc = [jd._llr_errs(idx, LLR)]
        dec = op.threshold(B, 0, L, app, 0.6)
        und = dec < 0
        bc = np.zeros((B, L * M))
        val = c[None, :] if variant == "current" else np.ones((1, L))
        rows, secs = np.nonzero(~und)
        bc[rows, secs * M + dec[rows, secs]] = np.broadcast_to(val, (B, L))[rows, secs]
        yn = y - op.Ab_batch(bc)
        mk.reserve(B, T)
        mk.stage(yn, Pl)
        mk.stage_power_batch(B, np.where(und, Pl[None, :], 0.0))
        mk.run(B, T); mk.wait()
        llr = mk.llr(B, 0, L).reshape(B, L, logm)
        LLR.reshape(B, L, logm)[und] = llr[und]
        e_amp.append(jd._llr_errs(idx, LLR))
        app2, _ = jd.code.decode_batch(LLR)
        LLR[:] = app2
        e_ldpc.append(jd._llr_errs(idx, LLR))
        tb = L * logm
        res[variant] = [float(np.mean(e) / tb) for e in (e_amp[0], e_amp[1], e_ldpc[0], e_ldpc[1])]
    refs = [(r["BER_amp"][pi], r["BER_ldpc"][pi]) for r in pub["runs"] if r["threshold"] == 0.6]
    print(f"sigma {sigma:.3f}: [amp0 amp1 ldpc0 ldpc1] current {np.round(res['current'], 5)} unit {np.round(res['unit'], 5)}"
          f" | published {refs}", flush=True)
