"""bench.py's N-rank flow on the CPU: two and four ranks over the dist module's socket
backend drive bench.main() end to end with a stand-in device operator (the
bench's own timing, barriers, max-over-ranks, per-rank spread, binary64 leg,
roofline assembly and the CPU baseline run after the timed region on rank 0).
The device kernels are not exercised here (no GPU); the keys and their
consistency are: an N-rank line carries its own cpu_baseline / gpu_over_cpu
and the per-rank min / max."""
import json
import os
import socket
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeOp:
    """Stands in for SparcOperator: every call returns at once with plausible
    plan / profile data (a k_sec4 + k_row2 decode of T iterations)."""
    KERNEL_KINDS = ("k_sec", "k_row", "k_dense_az", "k_dense_den", "k_dense_ab", "k_i8_quant")

    def __init__(self, L, M, n, backend, precision, device, plan):
        self.L, self.M, self.n = L, M, n
        self.w = 2 ** int(np.ceil(np.log2(max(M + 1, n + 1))))
        self.backend, self.precision = backend, precision
        self.runs = 0

    def Ab_batch(self, beta):
        return np.zeros((beta.shape[0], self.n))

    def reserve(self, B, T):
        self.T = T

    def stage(self, y, Pl=None, beta0=None):
        return y.shape[0]

    def run(self, B, T, early_stop=True, beta0=False):
        self.runs += 1
        time.sleep(0.001)

    def wait(self):
        pass

    def plan(self, B):
        return dict(section_kernel="k_sec4", partials=256, row_splits=1, codewords_per_wg=1, zz_partials=288,
                    w=self.w, row_kernel="k_row2_16", cus=256)

    def profile(self, B, T, early_stop=True, beta0=False, rep=1):
        kinds = {k: (0.0, 0) for k in self.KERNEL_KINDS}
        kinds["k_sec"] = (0.0065, T)
        kinds["k_row"] = (0.0032, T + 1)
        return kinds, 1.6


def _rank(rank, world, port, out, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SPARC_DIST_BACKEND="socket")
    sys.path.insert(0, ROOT)
    import bench
    res = bench.main(argv, make_op=FakeOp)
    out.put((rank, json.dumps(res)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_n_rank_bench_line_carries_cpu_baseline_and_spread(world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    argv = ["--gpus", str(world), "--steps", "4", "--warmup", "1", "--no-dense", "--cpu-procs", "1", "--cpu-iters", "1"]
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, argv)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    line = json.loads(got[0])
    assert line["n_gpus"] == world and line["scaling"] == "weak"
    assert line["value"] > 0 and line["ms_per_step"] > 0
    # per-rank spread of a weak-scaling job
    pr = line["per_rank"]
    assert 0 < pr["value_min"] <= pr["value_max"] and len(pr["ms_per_step"]) == world
    assert max(pr["ms_per_step"]) <= line["ms_per_step"] + 1e-6  # the line's time is the max over ranks
    # the CPU baseline of an N-rank line, run on rank 0 after the timed region
    cb = line["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0
    assert abs(cb["gpu_over_cpu"] - line["value"] / cb["value"]) <= 0.05 * cb["gpu_over_cpu"] + 0.1
    # roofline assembly: live events, consistency check, the binary64 leg's own roofline
    r = line["roofline"]
    assert r["kernel"] == "k_sec4" and r["bound"] == "hbm" and 0 < r["frac"] < 1
    assert r["consistency"]["T"] == 64 and r["consistency"]["per_iteration_ms"] > 0
    assert "sources" in r and line["fp64_leg"]["roofline"]["kernel"] == "k_sec4"
    # the other ranks return the same line without printing it
    for r in range(1, world):
        assert json.loads(got[r])["value"] == line["value"]
    # value = every rank's codewords over the slowest rank's time
    assert abs(line["value"] - world * pr["value_min"]) <= 1e-3 * line["value"]
