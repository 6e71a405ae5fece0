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

    DECIDE_SLOTS = 4

    def __init__(self, L, M, n, backend, precision, device, plan):
        self.L, self.M, self.n = L, M, n
        self.w = 2 ** int(np.ceil(np.log2(max(M + 1, n + 1))))
        self.backend, self.precision = backend, precision
        self.runs = 0
        self.log = []  # (call, perf_counter) of run / decide_async / decide_collect
        self.slots = {}

    def Ab_batch(self, beta):
        return np.zeros((beta.shape[0], self.n))

    def reserve(self, B, T):
        self.T = T

    def stage(self, y, Pl=None, beta0=None):
        return y.shape[0]

    def run(self, B, T, early_stop=True, beta0=False):
        self.runs += 1
        self.log.append(("run", time.perf_counter()))
        time.sleep(0.001)

    def decide_async(self, B, slot):
        assert slot not in self.slots, "slot reused before it was collected"
        self.slots[slot] = B
        self.log.append(("decide_async", time.perf_counter()))

    def decide_collect(self, B, slot):
        assert self.slots.pop(slot) == B
        self.log.append(("decide_collect", time.perf_counter()))
        return np.zeros((B, self.L), dtype=np.int32)

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
    assert r["frac_dispatch"] > 0 and r["frac_events"] > 0 and "timing" in r
    # every rank's timed steps were decided and counted
    assert line["decisions"]["decided_steps"] == world * 4
    assert line["decode_only"]["value"] > 0
    # the other ranks return the same line without printing it
    for r in range(1, world):
        assert json.loads(got[r])["value"] == line["value"]
    # value = every rank's codewords over the slowest rank's time
    assert abs(line["value"] - world * pr["value_min"]) <= 1e-3 * line["value"]
    # the batched legs of the default line: configs[2] in
    # both precisions and configs[3], each timed over every rank with its own
    # decisions and roofline
    legs = line["batched_legs"]
    assert set(legs) == {"c3", "c3_fp64", "c4"}
    for tag, leg in legs.items():
        assert leg["value"] > 0 and leg["ms_per_step"] > 0 and leg["codewords_per_step_per_gpu"] == 256, tag
        assert leg["decided_steps_rank0"] == leg["steps"] and "frac" in leg["roofline"], tag
        assert abs(leg["value"] - 256 * leg["steps"] * world / (leg["ms_per_step"] * leg["steps"] / 1e3)) \
            <= 1e-2 * leg["value"], tag
    assert legs["c3_fp64"]["dtype"] == "f64" and legs["c4"]["workload"].startswith("BASELINE configs[3]")
    # the whole-iteration figures: minimal bytes = section + row bytes less the
    # Ab-partial hand-off; the dense GEMM formulation's 4 n L M B flops
    import bench
    for tag, wl in (("c3", "c3"), ("c4", "c4")):
        r = legs[tag]["roofline"]
        w = bench.WORKLOADS[wl]
        n, L, M = bench.n_of(w), w["L"], w["M"]
        it, de = r["iteration"], r["dense_equivalent"]
        assert it["minimal_bytes"] > 0 and it["partials_bytes"] > 0 and 0 < it["frac_minimal"] < r["frac"] + 1, tag
        assert de["flops_per_iteration"] == 4.0 * n * L * M * 256, tag
        assert abs(de["tflops"] - de["flops_per_iteration"] / (it["ms"] * 1e-3) / 1e12) <= 0.1 + 1e-3 * de["tflops"], tag


def test_timed_step_includes_the_decision():
    """a benched step is sa_run + the device argmax + the
    copy of the L section indices to the host; every timed step's decisions
    are collected inside the timed region, the decisions of step k while
    decode k + 1 is queued."""
    sys.path.insert(0, ROOT)
    import bench
    op = FakeOp(8, 4, 32, "hadamard", "fp32", 0, None)
    sent = np.zeros((3, 8), dtype=np.int32)
    sent[1, 2] = 1  # one section of one codeword differs from the stand-in's all-zero decisions
    steps, warmup = 5, 2
    ts = bench.timed_steps(op, 3, 64, steps, warmup, sent)
    inside = [(k, t) for k, t in op.log if ts["t0"] <= t <= ts["t1"]]
    assert [k for k, _ in inside].count("run") == steps
    assert [k for k, _ in inside].count("decide_async") == steps
    assert [k for k, _ in inside].count("decide_collect") == steps
    assert ts["decided_steps"] == steps and ts["section_errors"] == steps  # one error per step, scored
    # pipelined: decode k + 1 is queued before the decisions of decode k are collected
    seq = [k for k, _ in inside]
    assert seq[:4] == ["run", "decide_async", "run", "decide_async"] and seq[4] == "decide_collect"
    assert not op.slots  # nothing left uncollected
    # decode-only timing: no decisions
    op.log.clear()
    ts0 = bench.timed_steps(op, 3, 64, steps, 0, decide=False)
    assert [k for k, _ in op.log].count("decide_async") == 0 and ts0["decided_steps"] == 0


def test_load_trace_reads_the_exclusive_duration():
    """load_trace returns the exclusive in-graph median too (a
    committed trace line carries both)."""
    sys.path.insert(0, ROOT)
    import bench
    tr = bench.load_trace("c2", "k_sec4")
    assert tr is not None and tr["duration_ns"] > 0 and tr["launches"] > 0
    assert tr["exclusive_ns"] is not None and tr["exclusive_ns"] > 0


def test_plan_with_matrix_backend_is_refused():
    """--plan with --backend matrix used to be silently ignored
    (the device-generated design takes no plan); it is an argument error now."""
    import bench
    with pytest.raises(SystemExit):
        bench.parse_args(["--backend", "matrix", "--plan", "ONE_PASS"])
    assert bench.parse_args(["--backend", "matrix"]).plan == ""
    assert bench.parse_args(["--plan", "ONE_PASS"]).plan == "ONE_PASS"
