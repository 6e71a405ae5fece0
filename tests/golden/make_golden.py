"""Generate golden fixtures by importing the reference itself (build container only).

Run from the repo root:  python tests/golden/make_golden.py

This script is the ONLY code in the repo that touches /root/reference, and only
to *execute* the reference's own functions on seeded inputs and record their
outputs as data (.npz / .json).  It never copies reference source.  It is not
run by the test suite, smoke() or bench.py (the GPU box has no /root/reference).

Workarounds needed to import ``ldpc/sparc_ldpc.py`` here, all outside the
reference tree:
  * ``bitarray`` is not installed: a stub module is registered before import.
    It is used only by ``bp2sp`` (sparc_ldpc.py:283-314), not on the AMP path.
  * ``pyfht`` is not installed: the module uses its in-file pure-Python
    fallback (sparc_ldpc.py:16-29).  For the large cases we replace
    ``sparc_ldpc.fht_inplace`` with a vectorised transform that performs the
    same butterflies in the same order; this script first checks that the two
    agree bit for bit in fp64 and records the check.
  * NumPy 2 breaks the ``β.all()==None`` default sentinel (sparc_ldpc.py:192),
    so the zero start is requested with an explicit zeros β₀ (bit-identical:
    y - Ab(0) == y).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/ldpc"


def load_reference():
    import matplotlib
    matplotlib.use("Agg")
    stub = types.ModuleType("bitarray")
    stub.bitarray = list
    sys.modules.setdefault("bitarray", stub)
    sys.path.insert(0, REF)
    import warnings
    warnings.simplefilter("ignore")
    import sparc_ldpc as ref
    return ref


def fast_fht(x):
    """Same butterfly order as sparc_ldpc.py:19-29, vectorised over blocks."""
    N = x.shape[0]
    i = N >> 1
    while i:
        v = x.reshape(N // (2 * i), 2, i)
        a = v[:, 0].copy()
        b = v[:, 1]
        v[:, 0] = a + b
        v[:, 1] = a - b
        i >>= 1


def sigma_from_snr_db(P, snr_db):
    # amp_test.py:167-169 (20*log10 convention)
    return float(np.sqrt(P / 10 ** (snr_db / 20)))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rep_inputs(ref, L, M, n, Pl, sigma, Ab, seed):
    rs = np.random.RandomState(seed)
    idx = rs.randint(0, M, L)
    b0 = np.zeros((L * M, 1))
    for l in range(L):
        b0[l * M + idx[l]] = np.sqrt(n * Pl[l])
    x = Ab(b0)
    y = (x + rs.randn(n, 1) * sigma).reshape(-1, 1)
    return idx, y


def zeros(L, M):
    return np.zeros((L * M, 1))


def main():
    ref = load_reference()
    slow_fht = ref.fht_inplace
    meta = {"generated_by": "tests/golden/make_golden.py", "numpy": np.__version__}

    # ---- 1. FHT: fallback vs vectorised, bitwise --------------------------
    rs = np.random.RandomState(7)
    fht_cases = {}
    for w in (8, 64, 512, 2048):
        x = rs.randn(w)
        a = x.copy(); slow_fht(a)
        b = x.copy(); fast_fht(b)
        assert np.array_equal(a, b), w
        fht_cases[f"fht_in_{w}"] = x
        fht_cases[f"fht_out_{w}"] = a
    np.savez_compressed(os.path.join(HERE, "fht.npz"), **fht_cases)
    meta["fht_vectorised_equals_fallback_bitwise"] = True

    # ---- 2. small case, pure-Python FHT (as shipped) -----------------------
    L, M, P, R, T = 16, 8, 2.0, 1.0, 30
    n = int(L * np.log2(M) / R)
    sigma = sigma_from_snr_db(P, 10)
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    idx, y = rep_inputs(ref, L, M, n, Pl, sigma, Ab, 1000)
    brand = rs.randn(L * M, 1); zrand = rs.randn(n, 1)
    traj = []
    for t in range(1, T + 1):
        traj.append(ref.amp(y, 0, Pl, L, M, t, Ab, Az, zeros(L, M)).reshape(-1))
    import amp_test as ref_amp_test
    bfin, tstop = ref_amp_test.amp_test(y, 0, Pl, L, M, T, Ab, Az, zeros(L, M))
    # soft init: 0/1 β₀ with the first 5 sections zeroed (amp_test.py:203-204)
    b0 = np.zeros((L * M, 1)); b0[np.arange(L) * M + idx] = 1.0; b0[:5 * M] = 0
    bsoft, tsoft = ref_amp_test.amp_test(y, 0, Pl, L, M, T, Ab, Az, b0)
    # shorter operator on a fancy-indexed subset (amp_exit.py:113-116 pattern)
    sub = np.array([3, 1, 7, 0, 12])
    Ab_s, Az_s = ref.sparc_transforms_shorter(len(sub), M, n, ordering[sub])
    bsub = rs.randn(len(sub) * M, 1)
    np.savez_compressed(
        os.path.join(HERE, "small.npz"), L=L, M=M, n=n, P=P, sigma=sigma, T=T,
        ordering=ordering, idx=idx, y=y, brand=brand, zrand=zrand,
        Ab_brand=Ab(brand), Az_zrand=Az(zrand), traj=np.array(traj),
        beta_final=bfin, t_stop=tstop, beta0_soft=b0, beta_soft=bsoft, t_soft=tsoft,
        sub=sub, bsub=bsub, Ab_sub=Ab_s(bsub), Az_sub=Az_s(zrand),
        Ab_b0=Ab(b0))

    # Everything below uses the vectorised FHT (bitwise-equal, checked above).
    ref.fht_inplace = fast_fht
    # amp_ldpc_sim calls amp() without β (sparc_ldpc.py:449); under NumPy 2 the
    # default sentinel crashes.  Supply the bit-identical zero
    # start for that call form only.
    _amp = ref.amp

    def amp_np2(y, s, Pl, L, M, T, Ab, Az, β=None):
        return _amp(y, s, Pl, L, M, T, Ab, Az, np.zeros((L * M, 1)) if β is None else β)
    ref.amp = amp_np2

    # ---- 3. C1: L=128 M=4 R=1 P=2 T=20, snr 10 dB, 4 reps ------------------
    L, M, P, R, T = 128, 4, 2.0, 1.0, 20
    n = int(L * np.log2(M) / R)
    sigma = sigma_from_snr_db(P, 10)
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    c1 = dict(L=L, M=M, n=n, P=P, sigma=sigma, T=T, ordering=ordering)
    for r in range(4):
        idx, y = rep_inputs(ref, L, M, n, Pl, sigma, Ab, 1000 + r)
        traj = [ref.amp(y, 0, Pl, L, M, t, Ab, Az, zeros(L, M)).reshape(-1) for t in (1, 2, 5)]
        bfin, tstop = ref_amp_test.amp_test(y, 0, Pl, L, M, T, Ab, Az, zeros(L, M))
        c1[f"idx_{r}"] = idx; c1[f"y_{r}"] = y
        c1[f"traj_{r}"] = np.array(traj); c1[f"beta_{r}"] = bfin; c1[f"t_{r}"] = tstop
    np.savez_compressed(os.path.join(HERE, "c1.npz"), **c1)

    # ---- 4. C2: L=M=512 R=1 P=4 T=64, snr 10 dB (amp_test.py:161-176) ------
    L, M, P, R, T = 512, 512, 4.0, 1.0, 64
    n = int(L * np.log2(M) / R)
    sigma = sigma_from_snr_db(P, 10)
    Pl = P / L * np.ones(L)
    t0 = time.time()
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    meta["c2_ordering_seconds"] = time.time() - t0
    idx, y = rep_inputs(ref, L, M, n, Pl, sigma, Ab, 1000)
    b1 = ref.amp(y, 0, Pl, L, M, 1, Ab, Az, zeros(L, M))
    t0 = time.time()
    bfin, tstop = ref_amp_test.amp_test(y, 0, Pl, L, M, T, Ab, Az, zeros(L, M))
    meta["c2_reference_decode_seconds"] = time.time() - t0
    meta["c2_reference_decode_iters"] = int(tstop)
    # amp_test.py:202-214 hard init, :231 soft init (L_zero = 154)
    Lz = 154
    beta = np.zeros((L * M, 1)); beta[np.arange(L) * M + idx] = np.sqrt(n * Pl[0])
    beta_0 = beta / np.sqrt(n * P / L); beta_0[:Lz * M] = 0
    y_new = y - Ab(beta_0)
    Ab_n, Az_n = ref.sparc_transforms_shorter(Lz, M, n, ordering)
    bhard, thard = ref_amp_test.amp_test(y_new, sigma, Pl[:Lz], Lz, M, T, Ab_n, Az_n, zeros(Lz, M))
    bsoft, tsoft = ref_amp_test.amp_test(y, sigma, Pl, L, M, T, Ab, Az, beta_0)
    np.savez_compressed(
        os.path.join(HERE, "c2.npz"), L=L, M=M, n=n, P=P, sigma=sigma, T=T,
        ordering_sha256=sha(ordering), idx=idx, y=y,
        beta_t1=b1.astype(np.float32),
        beta_final=bfin.astype(np.float32), t_stop=tstop,
        argmax_final=bfin.reshape(L, M).argmax(1),
        beta_final_norm=float(np.linalg.norm(bfin)),
        Lz=Lz, argmax_hard=bhard.reshape(Lz, M).argmax(1), t_hard=thard,
        beta_hard_norm=float(np.linalg.norm(bhard)),
        argmax_soft=bsoft.reshape(L, M).argmax(1), t_soft=tsoft,
        beta_soft_norm=float(np.linalg.norm(bsoft)))

    # ---- 5. ordering hashes for every BASELINE config ----------------------
    hashes = {}
    for (L, M, n) in [(128, 4, 256), (512, 512, 4608), (768, 512, 8294), (512, 512, 5529)]:
        _, _, o = ref.block_sub_fht(n, M, L, seed=0)
        hashes[f"L{L}_M{M}_n{n}"] = sha(o)
    meta["ordering_sha256"] = hashes

    # ---- 6. C5 plain SPARC reps through amp_ldpc_sim (sparc_ldpc.py:359) ----
    # waterfall's plain branch: L=M=512, P=4, R=5/6, T=64, Eb/N0 point 3 of
    # linspace(3,10,10) (sparc_ldpc.py:1166-1200).
    L, M, P, T = 512, 512, 4.0, 64
    R = 5 / 6
    ebno_db = float(np.linspace(3, 10, 10)[3])
    ebno = 10 ** (ebno_db / 20)
    snr = ebno / (1 / (2 * R))
    sigma = float(np.sqrt(P / snr))
    n = int(L * np.log2(M) / R)
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    c5 = dict(L=L, M=M, n=n, P=P, R=R, T=T, sigma=sigma, ebno_db=ebno_db)
    for s in range(3):
        np.random.seed(s)
        ber_ref, _, _, _ = ref.amp_ldpc_sim(ref.SPARCParams(L, M, sigma, P, R, T))
        # replicate the draw order of sparc_ldpc.py:423-446 for the same seed
        np.random.seed(s)
        bits = np.random.randint(0, 2, int(L * np.log2(M))).tolist()
        ind = ref.bits2indices(bits, M)
        b0 = np.zeros((L * M, 1))
        for l in range(L):
            b0[l * M + ind[l]] = np.sqrt(n * Pl[l])
        y = (Ab(b0) + np.random.randn(n, 1) * sigma).reshape(-1, 1)
        bh = ref.amp(y, sigma, Pl, L, M, T, Ab, Az, zeros(L, M)).reshape(-1)
        rx = bh.reshape(L, M).argmax(1)
        ber = sum(bin(a ^ b).count("1") for a, b in zip(ind, rx)) / (L * 9)
        assert ber == ber_ref, (s, ber, ber_ref)
        c5[f"bits_{s}"] = np.array(bits, dtype=np.uint8)
        c5[f"idx_{s}"] = np.array(ind)
        c5[f"y_{s}"] = y
        c5[f"rx_{s}"] = rx
        c5[f"ber_{s}"] = ber_ref
    np.savez_compressed(os.path.join(HERE, "c5_reps.npz"), **c5)
    meta["c5_draw_order_replicated"] = True

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
