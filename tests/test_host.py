"""CPU: the C-ABI library's export table, the host-side mirror of the
reference interface, and the multi-rank Monte-Carlo logic (gloo)."""
import hashlib
import json
import os
import re
import socket
import ctypes as ct

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden
from oracle import amp_oracle as orc


# ---- C ABI --------------------------------------------------------------

def _header_symbols():
    with open(os.path.join(ROOT, "include", "sparc_amp.h")) as fh:
        txt = fh.read()
    return sorted(set(re.findall(r"\b(sa_[a-z0-9_A-Z]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from sparc_ldpc_amd import _lib
    lib = ct.CDLL(_lib.LIB_PATH)
    syms = _header_symbols()
    assert syms, "no declarations parsed"
    for name in syms:
        assert hasattr(lib, name), f"{name} declared in include/sparc_amp.h but not exported"
    assert sorted(_lib.EXPORTS) == syms


def test_library_loads_without_gpu_and_fails_loudly():
    import sparc_ldpc_amd as sp
    lib = sp.load_library()
    assert lib.sa_version().startswith(b"sparc_amp")
    if lib.sa_device_count() == 0:
        ctx = ct.c_void_p()
        o = np.ones((2, 8), dtype=np.uint32)
        rc = lib.sa_create(ct.byref(ctx), 2, 4, 8, o.ctypes.data_as(ct.POINTER(ct.c_uint32)), 0, 0, 0)
        assert rc == -6  # SA_ERR_NO_DEVICE: no silent CPU fallback
        assert b"device" in lib.sa_last_error()
        with pytest.raises(sp.SparcAmpError):
            sp.SparcOperator(2, 4, 8, o)


def test_null_context_is_an_argument_error():
    import sparc_ldpc_amd as sp
    lib = sp.load_library()
    assert lib.sa_Ab(None, 1, None, None) == -1
    assert lib.sa_run(None, 1, 1, 0) == -1
    lib.sa_destroy(None)  # no-op


# ---- host mirror of the reference interface ------------------------------

def test_make_ordering_matches_reference_hashes():
    import sparc_ldpc_amd as sp
    with open(os.path.join(GOLDEN, "meta.json")) as fh:
        meta = json.load(fh)
    for key, h in meta["ordering_sha256"].items():
        L, M, n = (int(p[1:]) for p in key.split("_"))
        o = sp.make_ordering(L, M, n, 0)
        assert hashlib.sha256(o.tobytes()).hexdigest() == h
        assert o is sp.make_ordering(L, M, n, 0)  # memoised like the reference's seed-0 reuse


def test_bits_indices_ber_against_oracle():
    import sparc_ldpc_amd as sp
    rs = np.random.RandomState(4)
    for M in (2, 4, 512):
        logm = int(np.log2(M))
        bits = rs.randint(0, 2, 37 * logm).tolist()
        assert sp.bits2indices(bits, M) == orc.bits2indices(bits, M)
        a = rs.randint(0, M, 37)
        b = rs.randint(0, M, 37)
        assert sp.ber_of(a, b, 37 * logm) == orc.ber_indices(a, b, 37 * logm)


def test_ebno_mapping_matches_reference_fixture():
    import sparc_ldpc_amd as sp
    g = golden("c5_reps.npz")
    assert sp.ebno_to_sigma(float(g["ebno_db"]), float(g["P"]), float(g["R"])) == float(g["sigma"])


def test_pa_parameterised_matches_oracle():
    import sparc_ldpc_amd as sp
    a = sp.pa_parameterised(64, 1.3, 4.0, 0.8, 0.7)
    b = orc.pa_parameterised(64, 1.3, 4.0, 0.8, 0.7)
    assert np.array_equal(a, b) and abs(a.sum() - 4.0) < 1e-12


def test_beta0_sentinels():
    from sparc_ldpc_amd.amp import _beta0
    assert _beta0(None, 2, 4) is None
    assert _beta0(np.array([None]), 2, 4) is None  # the reference's default (sparc_ldpc.py:189)
    z = _beta0(np.zeros((8, 1)), 2, 4)
    assert z.shape == (1, 8) and not z.any()
    with pytest.raises(AssertionError):
        _beta0(np.zeros(7), 2, 4)


def test_amp_rejects_non_callable_operators():
    """amp() takes any callables (sparc_ldpc.py:189); anything else is a
    TypeError before the device is touched."""
    import sparc_ldpc_amd as sp
    with pytest.raises(TypeError):
        sp.amp(np.zeros(8), 0, np.ones(2), 2, 4, 3, "Ab", None)


# ---- Monte-Carlo stopping rule and sharding --------------------------------

def _fake_round(seeds):
    """Deterministic stand-in for mc_decode: bit errors as a function of the seed."""
    s = np.asarray(seeds, dtype=np.int64)
    be = np.where(s % 3 == 0, (s * 7) % 11, 0).astype(np.int64)
    return be, (s % 5 + 10).astype(np.int64)


def _reference_loop(seed_base, total_bits, min_errors, max_blocks):
    """sparc_ldpc.py:1217-1245 written out block by block."""
    ber_cum = 0.0
    nerr = nblocks = 0
    s = seed_base
    while nerr < min_errors:
        be, _ = _fake_round([s])
        ber = be[0] / total_bits
        ber_cum += ber
        if ber:
            nerr += 1
        nblocks += 1
        s += 1
        if nblocks >= max_blocks:
            break
    return ber_cum / nblocks, nblocks, nerr


@pytest.mark.parametrize("min_errors,max_blocks,batch", [(5, 250, 8), (200, 37, 16), (3, 1000, 1)])
def test_ber_point_matches_sequential_reference_rule(min_errors, max_blocks, batch):
    import sparc_ldpc_amd as sp
    r = sp.ber_point(_fake_round, 4608, min_errors, max_blocks, batch, seed_base=100)
    ber, nb, ne = _reference_loop(100, 4608, min_errors, max_blocks)
    assert r["blocks"] == nb and r["block_errors"] == ne
    assert abs(r["BER"] - ber) <= 1e-15


def test_shard_seeds_partition():
    from sparc_ldpc_amd.dist import shard_seeds
    for world in (1, 2, 8):
        allseeds = []
        for rnd in range(3):
            for rank in range(world):
                allseeds += shard_seeds(50, rnd, 4, rank, world)
        assert sorted(allseeds) == list(range(50, 50 + 3 * 4 * world))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd import dist
    dist.init("socket")
    assert dist.backend() == "socket"
    res = sp.ber_point(_fake_round, 4608, 7, 250, 4, rank, world, dist.allreduce_sum, seed_base=100)
    c = dist.allreduce_sum(np.array([rank + 1], dtype=np.int64))
    m = dist.allreduce_max(np.array([0.5 * rank, -rank], dtype=np.float64))
    f = dist.allreduce_sum(np.array([0.1 * (rank + 1)] * 3, dtype=np.float64))
    dist.barrier()
    out.put((rank, res, int(c[0]), m.tolist(), f.tolist()))
    dist.finalize()


@pytest.mark.parametrize("world", [2, 3])
def test_ber_point_ranks_socket_equals_single(world):
    """The counter all-reduce over the dist module's TCP star (the CPU backend;
    RCCL carries the same calls on GPUs): a sharded ber_point equals the
    single-process one over the same seeds."""
    import multiprocessing as mp
    import sparc_ldpc_amd as sp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = sp.ber_point(_fake_round, 4608, 7, 250, 4 * world, seed_base=100)
    for rank, res, csum, mx, fs in got:
        assert csum == world * (world + 1) // 2  # the counter all-reduce itself
        assert mx == [0.5 * (world - 1), 0.0]
        assert fs == got[0][4]  # rank-order float sums: every rank gets the same bits
        assert res["blocks"] == single["blocks"] and res["block_errors"] == single["block_errors"]
        assert abs(res["BER"] - single["BER"]) <= 1e-15


def test_allreduce_refuses_without_communicator(monkeypatch):
    """WORLD_SIZE > 1 without dist.init(): never this rank's counts as the job's."""
    from sparc_ldpc_amd import dist
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(dist, "_COMM", None)
    with pytest.raises(dist.DistError):
        dist.allreduce_sum(np.array([1], dtype=np.int64))
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert dist.allreduce_sum(np.array([5], dtype=np.int64)).tolist() == [5]


def test_amp_refuses_operators_of_two_contexts():
    """Ab of one operator with Az of another is a caller's mistake: ValueError,
    not the foreign-callable host loop (object stand-ins; no device needed)."""
    from sparc_ldpc_amd.operators import AbOp, AzOp
    import sparc_ldpc_amd as sp

    class _Op:  # attribute holder in place of two SparcOperators
        L, M, n = 4, 4, 8
    with pytest.raises(ValueError, match="different operators"):
        sp.amp(np.zeros(8), 1.0, np.ones(4), 4, 4, 3, AbOp(_Op()), AzOp(_Op()))
    with pytest.raises(ValueError, match="different operators"):
        sp.amp_test(np.zeros(8), 1.0, np.ones(4), 4, 4, 3, AbOp(_Op()), AzOp(_Op()))


@pytest.mark.parametrize("L,M,n,sigma", [(768, 512, 7885, 0.6), (16, 100, 33, 1.3), (5, 1, 7, 0.5),
                                         (64, 16, 256, 0.95), (3, 3, 0, 1.0)])
def test_native_draws_match_numpy(L, M, n, sigma):
    """sa_draw_reps (libsparc_amp's host restatement of NumPy's legacy
    RandomState: MT19937 integer seeding, masked bounded integers, the polar
    Gaussian) against harness._draw_reps itself — RandomState(s).randint(0, M, L)
    then .randn(n) * sigma — bit for bit, including a non-power-of-two M (the
    rejection loop), M = 1 (no draw), n = 0 and the seeds 0 and 2**32 - 1,
    single- and multi-threaded."""
    from sparc_ldpc_amd.harness import _draw_reps, draw_reps
    seeds = list(range(40)) + [2**32 - 1, 123456789]
    a_idx, a_noise = _draw_reps(seeds, L, M, n, sigma)
    for th in (1, 3):
        b_idx, b_noise = draw_reps(seeds, L, M, n, sigma, threads=th)
        assert np.array_equal(a_idx, b_idx)
        assert np.array_equal(a_noise, b_noise)


@pytest.mark.parametrize("L,M,n,seed", [(768, 512, 8294, 0), (64, 16, 256, 3), (20, 100, 37, 2**32 - 1), (4, 4, 1, 7)])
def test_native_ordering_matches_numpy(L, M, n, seed):
    """sa_make_ordering against the reference's own construction
    (sparc_ldpc.py:107-117: RandomState(seed).shuffle of arange(1, w) per
    section, cumulatively, the first n kept), restated in NumPy here."""
    from sparc_ldpc_amd import _lib
    from sparc_ldpc_amd.operators import _w_of
    w = _w_of(n, M)
    rng = np.random.RandomState(seed)
    ref = np.empty((L, n), dtype=np.uint32)
    idxs = np.arange(1, w, dtype=np.uint32)
    for ll in range(L):
        rng.shuffle(idxs)
        ref[ll] = idxs[:n]
    got = np.empty((L, n), dtype=np.uint32)
    _lib.check(_lib.load().sa_make_ordering(L, M, n, seed, got.ctypes.data_as(ct.POINTER(ct.c_uint32))))
    assert np.array_equal(got, ref)
