"""Diagnostic: BP inputs/outputs of the batched threshold exchange vs the
reference reps in tests/golden/joint.npz (thr|hardinit|s)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparc_ldpc_amd as sp
from sparc_ldpc_amd.joint import joint_decoder
g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/joint.npz"))
L, M, P, r, T, z, sigma, thr = g["thr|cfg"]
L, M, T = int(L), int(M), int(T)
n = int(L * np.log2(M) / float(r))
seeds = [1, 2, 5]
jd = joint_decoder(L, M, n, sp.LDPCParams("802.16", "5/6", int(z)), T, precision="fp64")
rec = []
orig = jd.code.decode_batch
def spy(CH, *a, **k):
    app, it = orig(CH, *a, **k)
    rec.append((CH.copy(), app.copy(), it.copy()))
    return app, it
jd.code.decode_batch = spy
idx, noise = jd.draw([np.random.RandomState(s) for s in seeds], len(seeds), float(sigma))
out = jd.run(idx, noise, float(P) / L * np.ones(L), "threshold", 3, float(thr))
tb = jd.total_bits
for i, s in enumerate(seeds):
    key = f"thr|hardinit|{s}"
    print("seed", s, "ours", np.concatenate([out["amp"][i], out["ldpc"][i]]) / tb, "ref", g[key + "|ber"])
    for k in range(3):
        if key + f"|llr{k}" not in g:
            continue
        ch, app, it = rec[k][0][i], rec[k][1][i], rec[k][2][i]
        rl, ra, ri = g[key + f"|llr{k}"], g[key + f"|app{k}"], int(g[key + f"|it{k}"][0])
        big = np.abs(rl) < 1e300
        print(f"  BP{k}: in maxdiff {np.max(np.abs(ch[big] - rl[big])):.3e} (sat eq {np.array_equal(np.sign(ch[~big]), np.sign(rl[~big]))}, n_sat {(~big).sum()} vs ours {(np.abs(ch) >= 1e300).sum()}) "
              f"sign mismatches {(np.sign(ch) != np.sign(rl)).sum()}  it {it} vs {ri}  app sign mism {(np.sign(app) != np.sign(ra)).sum()}")
