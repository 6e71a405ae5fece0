"""The RCCL binding of sparc_ldpc_amd.dist on a real GPU (one rank: RCCL
refuses two ranks on one device; the multi-rank protocol itself is covered by
the socket backend's CPU tests in test_host.py, and the driver's 8-GPU runs
go through the same calls)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_allreduce(lib_gpu):
    from sparc_ldpc_amd import dist
    rdv = dist.Rendezvous(0, 1)
    comm = dist.RcclComm(rdv, 0)
    try:
        a = np.arange(-5, 2000, dtype=np.int64)
        assert np.array_equal(comm.allreduce(a, "sum"), a)
        f = np.linspace(-1, 1, 33)
        assert np.array_equal(comm.allreduce(f, "max"), f)
        big = np.arange(70000, dtype=np.int64)  # grows the device buffer
        assert np.array_equal(comm.allreduce(big, "sum"), big)
        comm.barrier()
        with pytest.raises(dist.DistError):
            comm.allreduce(np.zeros(3, dtype=np.float32), "sum")
    finally:
        comm.close()
