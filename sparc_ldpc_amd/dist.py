"""Multi-GPU Monte-Carlo plumbing: one process per GPU, reps
sharded by rank, one all-reduce of int64 error counters per round.

The data path has no collective: every rank decodes its own codewords on its
own device with the same operator (seed-0 ordering).  The only exchange is
the sum of the per-block ``[bit_errors, iters]`` vectors (a few KB) — over
**RCCL** (``librccl.so``, ``ncclAllReduce`` on a device buffer, xGMI between
the GPUs of a node) bound here with ctypes, no PyTorch anywhere.

Bootstrap: the launcher (``torch.distributed.run`` / torchrun, or any other)
only provides ``RANK``/``WORLD_SIZE``/``LOCAL_RANK``/``MASTER_ADDR``/
``MASTER_PORT``.  Rank 0 listens on the first free TCP port of
``[MASTER_PORT + 1, MASTER_PORT + 16]`` (``SPARC_DIST_PORT`` overrides the
start; torchrun's own store holds ``MASTER_PORT`` itself); the other ranks
connect and are checked by a hello carrying a run token, world size and rank.
Rank 0 draws the ``ncclUniqueId`` and sends it over those sockets; then every
rank joins the communicator with ``ncclCommInitRank``.

The same star of sockets is the ``"socket"`` backend: a CPU all-reduce
through rank 0 (reduction in rank order, so float sums are deterministic),
used by the CPU tests and by rehearsals that put several ranks on one GPU
(RCCL refuses two ranks on one device).
"""
from __future__ import annotations

import ctypes as ct
import hashlib
import os
import socket
import struct
import time

import numpy as np

__all__ = ["env_rank", "init", "allreduce_sum", "allreduce_max", "barrier", "shard_seeds", "finalize",
           "backend", "DistError"]

_MAGIC = b"SPARCRDV"
_PORT_SPAN = 16


class DistError(RuntimeError):
    pass


def env_rank():
    """(rank, world, local_rank) from the launcher's environment (defaults 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _token() -> bytes:
    run = os.environ.get("TORCHELASTIC_RUN_ID", "") + "|" + os.environ.get("MASTER_PORT", "")
    return hashlib.sha1(run.encode()).digest()[:8]


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            raise DistError("peer closed the rendezvous socket")
        buf += chunk
    return bytes(buf)


def _send_msg(s, data: bytes):
    s.sendall(struct.pack("<Q", len(data)) + data)


def _recv_msg(s) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(s, 8))
    return _recv_exact(s, n)


class Rendezvous:
    """A star of TCP sockets through rank 0 (bootstrap and CPU collectives)."""

    def __init__(self, rank, world, addr=None, port=None, timeout=300.0):
        self.rank, self.world = rank, world
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("SPARC_DIST_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        self.peers = {}
        self.sock = None
        hello = _MAGIC + _token() + struct.pack("<ii", rank, world)
        deadline = time.time() + timeout
        if rank == 0:
            srv = None
            for p in range(port, port + _PORT_SPAN):
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                try:
                    s.bind((addr, p))
                except OSError:
                    s.close()
                    continue
                srv = s
                break
            if srv is None:
                raise DistError(f"rank 0: no free port in [{port}, {port + _PORT_SPAN}) on {addr}")
            srv.listen(max(8, world))
            srv.settimeout(1.0)
            while len(self.peers) < world - 1:
                if time.time() > deadline:
                    raise DistError(f"rank 0: only {len(self.peers)} of {world - 1} peers joined")
                try:
                    c, _ = srv.accept()
                except socket.timeout:
                    continue
                c.settimeout(30.0)
                try:
                    h = _recv_exact(c, len(hello))
                except (OSError, DistError):
                    c.close()
                    continue
                r, w = struct.unpack("<ii", h[16:])
                if h[:16] != hello[:16] or w != world or not (0 < r < world) or r in self.peers:
                    c.close()  # a foreign or duplicate connection
                    continue
                c.sendall(b"OK")
                c.settimeout(None)
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                self.peers[r] = c
            srv.close()
        else:
            while self.sock is None:
                for p in range(port, port + _PORT_SPAN):
                    try:
                        c = socket.create_connection((addr, p), timeout=2.0)
                    except OSError:
                        continue
                    try:
                        c.sendall(hello)
                        if _recv_exact(c, 2) == b"OK":
                            c.settimeout(None)
                            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                            self.sock = c
                            break
                    except (OSError, DistError):
                        pass
                    c.close()
                if self.sock is None:
                    if time.time() > deadline:
                        raise DistError(f"rank {rank}: could not reach rank 0 at {addr}:{port}+")
                    time.sleep(0.2)

    def bcast(self, data: bytes | None) -> bytes:
        if self.rank == 0:
            for r in sorted(self.peers):
                _send_msg(self.peers[r], data)
            return data
        return _recv_msg(self.sock)

    def allreduce(self, arr: np.ndarray, op: str) -> np.ndarray:
        arr = np.ascontiguousarray(arr)
        if self.rank == 0:
            acc = arr.copy()
            for r in sorted(self.peers):  # rank order: deterministic float sums
                other = np.frombuffer(_recv_msg(self.peers[r]), dtype=arr.dtype).reshape(arr.shape)
                acc = acc + other if op == "sum" else np.maximum(acc, other)
            out = acc.tobytes()
            for r in sorted(self.peers):
                _send_msg(self.peers[r], out)
            return acc
        _send_msg(self.sock, arr.tobytes())
        return np.frombuffer(_recv_msg(self.sock), dtype=arr.dtype).reshape(arr.shape).copy()

    def close(self):
        for c in self.peers.values():
            c.close()
        self.peers = {}
        if self.sock is not None:
            self.sock.close()
            self.sock = None


class SocketComm:
    name = "socket"

    def __init__(self, rdv: Rendezvous):
        self.rdv = rdv

    def allreduce(self, arr, op):
        return self.rdv.allreduce(arr, op)

    def barrier(self):
        self.rdv.allreduce(np.zeros(1, dtype=np.int64), "sum")

    def close(self):
        self.rdv.close()


class _UniqueId(ct.Structure):
    _fields_ = [("internal", ct.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES, rccl.h:40-43


_NCCL_INT64, _NCCL_FLOAT64 = 4, 8    # ncclDataType_t (rccl.h)
_NCCL_SUM, _NCCL_MAX = 0, 2          # ncclRedOp_t (rccl.h)
_H2D, _D2H = 1, 2                    # hipMemcpyKind


def _load_rocm(stem):
    """Load a ROCm library by its unversioned stem (``libamdhip64``,
    ``librccl``): the development symlink ``<stem>.so`` first, then any
    versioned ``<stem>.so.N`` on the loader path or under ``$ROCM_PATH/lib``
    (highest major first), so no ROCm major version is hard-coded."""
    import glob
    libdir = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
    cands = [stem + ".so", os.path.join(libdir, stem + ".so")]

    def major(p):
        tail = p.rsplit(".so.", 1)[-1].split(".")[0]
        return int(tail) if tail.isdigit() else -1
    cands += sorted(glob.glob(os.path.join(libdir, stem + ".so.*")), key=major, reverse=True)
    for cand in cands:
        try:
            return ct.CDLL(cand)
        except OSError:
            continue
    raise DistError(f"cannot load {stem}.so (tried {len(cands)} paths)")


_UID_BYTES = ct.sizeof(_UniqueId)


def uid_bytes(uid: _UniqueId) -> bytes:
    """All 128 bytes of an ncclUniqueId.  (``bytes(uid.internal)`` would stop
    at the first NUL: a c_char array field reads as a C string.)"""
    return ct.string_at(ct.addressof(uid), _UID_BYTES)


def uid_from_bytes(raw: bytes) -> _UniqueId:
    if len(raw) != _UID_BYTES:
        raise DistError(f"ncclUniqueId: got {len(raw)} bytes, expected {_UID_BYTES}")
    uid = _UniqueId()
    ct.memmove(ct.addressof(uid), raw, _UID_BYTES)
    return uid


class RcclComm:
    """One RCCL communicator over all ranks (ncclCommInitRank), device buffers
    on this rank's GPU, collectives on a stream of its own."""
    name = "rccl"

    def __init__(self, rdv: Rendezvous, device: int):
        self.rdv = rdv
        self.hip = hip = _load_rocm("libamdhip64")
        self.rccl = rccl = _load_rocm("librccl")
        rccl.ncclGetErrorString.restype = ct.c_char_p
        rccl.ncclGetErrorString.argtypes = [ct.c_int]
        rccl.ncclGetUniqueId.argtypes = [ct.POINTER(_UniqueId)]
        rccl.ncclCommInitRank.argtypes = [ct.POINTER(ct.c_void_p), ct.c_int, _UniqueId, ct.c_int]
        rccl.ncclAllReduce.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_size_t, ct.c_int, ct.c_int,
                                       ct.c_void_p, ct.c_void_p]
        rccl.ncclCommDestroy.argtypes = [ct.c_void_p]
        hip.hipSetDevice.argtypes = [ct.c_int]
        hip.hipMalloc.argtypes = [ct.POINTER(ct.c_void_p), ct.c_size_t]
        hip.hipStreamCreate.argtypes = [ct.POINTER(ct.c_void_p)]
        hip.hipMemcpyAsync.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_size_t, ct.c_int, ct.c_void_p]
        hip.hipStreamSynchronize.argtypes = [ct.c_void_p]
        hip.hipFree.argtypes = [ct.c_void_p]
        hip.hipStreamDestroy.argtypes = [ct.c_void_p]
        self._hip_ok(hip.hipSetDevice(int(device)), "hipSetDevice")
        if rdv.rank == 0:
            uid = _UniqueId()
            self._nccl_ok(rccl.ncclGetUniqueId(ct.byref(uid)), "ncclGetUniqueId")
            rdv.bcast(uid_bytes(uid))
        else:
            uid = uid_from_bytes(rdv.bcast(None))
        self.comm = ct.c_void_p()
        self._nccl_ok(rccl.ncclCommInitRank(ct.byref(self.comm), rdv.world, uid, rdv.rank), "ncclCommInitRank")
        self.stream = ct.c_void_p()
        self._hip_ok(hip.hipStreamCreate(ct.byref(self.stream)), "hipStreamCreate")
        self.buf = ct.c_void_p()
        self.cap = 0

    def _hip_ok(self, rc, what):
        if rc != 0:
            raise DistError(f"{what} failed: hipError {rc}")

    def _nccl_ok(self, rc, what):
        if rc != 0:
            raise DistError(f"{what} failed: {self.rccl.ncclGetErrorString(rc).decode()}")

    def _ensure(self, nbytes):
        if nbytes <= self.cap:
            return
        if self.buf.value:
            self.hip.hipFree(self.buf)
        cap = max(4096, 1 << (int(nbytes) - 1).bit_length())
        self._hip_ok(self.hip.hipMalloc(ct.byref(self.buf), ct.c_size_t(cap)), "hipMalloc")
        self.cap = cap

    def allreduce(self, arr, op):
        arr = np.ascontiguousarray(arr)
        if arr.dtype == np.int64:
            dt = _NCCL_INT64
        elif arr.dtype == np.float64:
            dt = _NCCL_FLOAT64
        else:
            raise DistError(f"allreduce: int64 or float64 only, got {arr.dtype}")
        self._ensure(arr.nbytes)
        out = np.empty_like(arr)
        h = self.hip
        self._hip_ok(h.hipMemcpyAsync(self.buf, arr.ctypes.data, arr.nbytes, _H2D, self.stream), "hipMemcpyAsync")
        self._nccl_ok(self.rccl.ncclAllReduce(self.buf, self.buf, arr.size, dt,
                                              _NCCL_SUM if op == "sum" else _NCCL_MAX, self.comm, self.stream),
                      "ncclAllReduce")
        self._hip_ok(h.hipMemcpyAsync(out.ctypes.data, self.buf, arr.nbytes, _D2H, self.stream), "hipMemcpyAsync")
        self._hip_ok(h.hipStreamSynchronize(self.stream), "hipStreamSynchronize")
        return out

    def barrier(self):
        self.allreduce(np.zeros(1, dtype=np.int64), "sum")

    def close(self):
        if self.comm.value:
            self.hip.hipStreamSynchronize(self.stream)
            self.rccl.ncclCommDestroy(self.comm)
            self.comm = ct.c_void_p()
        if self.buf.value:
            self.hip.hipFree(self.buf)
            self.buf = ct.c_void_p()
        if self.stream.value:
            self.hip.hipStreamDestroy(self.stream)
            self.stream = ct.c_void_p()
        self.rdv.close()


_COMM = None


def _gpu_count() -> int:
    try:
        from . import _lib
        return max(0, int(_lib.load().sa_device_count()))
    except Exception:
        return 0


def init(backend=None, device=None):
    """Join the job when WORLD_SIZE > 1; returns (rank, world, local).

    backend: "rccl" (the default where a GPU is visible), "socket" (CPU; the
    default without a GPU), or None (``SPARC_DIST_BACKEND`` or the default).
    device: this rank's GPU for RCCL (default LOCAL_RANK)."""
    global _COMM
    rank, world, local = env_rank()
    if world > 1 and _COMM is None:
        backend = backend or os.environ.get("SPARC_DIST_BACKEND") or ("rccl" if _gpu_count() > 0 else "socket")
        if backend == "gloo":  # the old name of the CPU path
            backend = "socket"
        if backend not in ("rccl", "socket"):
            raise DistError(f"unknown backend {backend!r}")
        rdv = Rendezvous(rank, world)
        _COMM = RcclComm(rdv, local if device is None else device) if backend == "rccl" else SocketComm(rdv)
    return rank, world, local


def backend():
    """Name of the active backend ("rccl", "socket"), or None outside a job."""
    return None if _COMM is None else _COMM.name


def _reduce(arr, op):
    arr = np.ascontiguousarray(arr)
    world = env_rank()[1]
    if world <= 1:
        return arr.copy()
    if _COMM is None:
        raise DistError(f"WORLD_SIZE={world} but dist.init() was never called: "
                        "refusing to return this rank's counts as the job's")
    return _COMM.allreduce(arr, op)


def allreduce_sum(arr: np.ndarray) -> np.ndarray:
    """Sum an int64 / float64 array over all ranks (a copy when WORLD_SIZE = 1;
    raises when WORLD_SIZE > 1 and no communicator exists)."""
    return _reduce(arr, "sum")


def allreduce_max(arr: np.ndarray) -> np.ndarray:
    """Element-wise max over all ranks (the bench's slowest-rank time)."""
    return _reduce(arr, "max")


def barrier():
    if _COMM is not None:
        _COMM.barrier()


def shard_seeds(base: int, rnd: int, batch: int, rank: int, world: int):
    """Seeds of round `rnd` for `rank`: base + rnd*batch*world + rank + world*i.
    Disjoint across ranks and rounds; the union over ranks is contiguous."""
    start = base + rnd * batch * world
    return [start + rank + world * i for i in range(batch)]


def finalize():
    global _COMM
    if _COMM is not None:
        _COMM.close()
        _COMM = None
