"""World-2 RCCL bootstrap of ``dist.RcclComm`` on the CPU.

Two spawned processes join a job exactly as two GPU ranks would
(``dist.init("rccl")``), but ``dist._load_rocm`` hands them a stub library
(``tests/stub/rocm_stub.c``, built here with gcc) in place of libamdhip64 /
librccl.  The stub logs every call and really reduces across the two processes,
so this checks, without GPUs:
  * the ncclUniqueId broadcast carries all 128 bytes (the id is full of NULs);
  * ``ncclCommInitRank(world, rank)`` on every rank with rank 0's id;
  * the ncclDataType_t / ncclRedOp_t codes of int64 / float64 sums and maxima;
  * the H2D copy -> all-reduce -> D2H copy -> stream sync sequence per call;
  * the results of the sums / maxima themselves.
The reps loop this serves is amp_test.py:183-246, sharded over ranks.
"""
import ctypes as ct
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def stub_lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("stub") / "librocm_stub.so"
    subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-fPIC", "-shared", "-o", str(out),
                    os.path.join(HERE, "stub", "rocm_stub.c")], check=True)
    return str(out)


def _rank_worker(rank, world, port, stub, logdir, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          STUB_LOG=os.path.join(logdir, f"log{rank}.txt"), STUB_DIR=logdir)
        sys.path.insert(0, ROOT)
        from sparc_ldpc_amd import dist
        loaded = []

        def fake_load(stem):
            loaded.append(stem)
            return ct.CDLL(stub)
        dist._load_rocm = fake_load
        dist.init("rccl", device=rank)
        assert dist.backend() == "rccl"
        s = dist.allreduce_sum(np.array([rank + 1, 10 * (rank + 1), -rank], dtype=np.int64))
        m = dist.allreduce_max(np.array([0.5 * rank, -float(rank)], dtype=np.float64))
        f = dist.allreduce_sum(np.full(700, 0.25 * (rank + 1)))  # > 4 KB: the buffer grows
        dist.barrier()
        dist.finalize()
        q.put((rank, sorted(set(loaded)), s.tolist(), m.tolist(), float(f.sum()), None))
    except Exception as e:  # report to the parent, never hang it
        q.put((rank, None, None, None, None, repr(e)))


def test_rccl_world2_bootstrap_and_allreduce(stub_lib, tmp_path):
    import multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_worker, args=(r, world, port, stub_lib, str(tmp_path), q))
          for r in range(world)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, loaded, s, m, fsum, err in got:
        assert err is None, f"rank {rank}: {err}"
        assert loaded == ["libamdhip64", "librccl"]
        assert s == [3, 30, -1]
        assert m == [0.5, 0.0]
        assert fsum == pytest.approx(700 * 0.75)

    pattern = bytes(0 if i % 3 == 2 else (i * 7 + 1) & 0xFF for i in range(128))
    for rank in range(world):
        log = open(tmp_path / f"log{rank}.txt").read().splitlines()
        assert log[0] == f"hipSetDevice {rank}"
        assert ("ncclGetUniqueId" in log) == (rank == 0)  # only rank 0 draws the id
        init = [ln for ln in log if ln.startswith("ncclCommInitRank")]
        assert len(init) == 1
        _, nr, r, verdict, hexid = init[0].split()
        assert (int(nr), int(r), verdict) == (world, rank, "uid-ok")
        assert bytes.fromhex(hexid) == pattern  # all 128 bytes, NULs included
        # per collective: H2D copy, all-reduce, D2H copy, stream sync
        calls = [ln for ln in log if ln.startswith(("hipMemcpyAsync", "ncclAllReduce", "hipStreamSynchronize"))]
        seq = [tuple(ln.split()) for ln in calls]
        assert len(seq) == 4 * 4 + 1  # sum, max, big sum, barrier; then close()'s sync
        assert seq[-1] == ("hipStreamSynchronize",)
        expect = [("3", "4", "0"), ("2", "8", "2"), ("700", "8", "0"), ("1", "4", "0")]
        for k, (cnt, dt, op) in enumerate(expect):
            h2d, ar, d2h, sync = seq[4 * k:4 * k + 4]
            nbytes = str(int(cnt) * 8)
            assert h2d == ("hipMemcpyAsync", nbytes, "1")
            assert ar == ("ncclAllReduce", cnt, dt, op)
            assert d2h == ("hipMemcpyAsync", nbytes, "2")
            assert sync == ("hipStreamSynchronize",)
        assert log[-1] in ("hipStreamDestroy",) and "ncclCommDestroy" in log


def test_uid_roundtrip_keeps_nul_bytes():
    from sparc_ldpc_amd import dist
    uid = dist._UniqueId()
    raw = bytes([7, 9, 0, 0, 5] + [0] * 120 + [1, 2, 3])
    ct.memmove(ct.addressof(uid), raw, 128)
    assert bytes(uid.internal) == bytes([7, 9])  # the c_char-array pitfall
    assert dist.uid_bytes(uid) == raw
    assert dist.uid_bytes(dist.uid_from_bytes(raw)) == raw
    with pytest.raises(dist.DistError):
        dist.uid_from_bytes(raw[:2])


def test_bench_refuses_gpus_world_mismatch():
    """A --gpus N launch without N ranks must fail loudly, before any GPU work."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr and r.stdout == ""
