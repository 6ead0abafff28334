"""bench.py's N > 1 flow cannot lose its headline: the steps after the timed
frames -- the frame-end gather, its check and the other split -- run guarded, every collective has
a timeout (MCPT_DIST_TIMEOUT_S), and rank 0 prints the JSON line with the failure in
gather.error / <split>.error.  Two gloo ranks on the CPU run bench.main() end to end with a
stand-in tracer (the allocation rules of runtime.cpp, tests/test_dist.py::_FakeTracer); the gather
is the real point-to-point transport of mcpt/parallel.py, and one rank is made to fail in it."""
import contextlib
import io
import json
import os
import socket
import types

import torch.multiprocessing as mp

from test_dist import _FakeTracer


class _Tracer(_FakeTracer):
    device_name = "fake (CPU)"

    def set_work_counters(self, on=True):
        pass

    def trace_profile(self, reset=True):
        return None

    def hbm_copy_gbps(self, *a, **kw):
        return 0.0

    def close(self):
        pass


def _fake_torch():
    import torch

    cuda = types.SimpleNamespace(synchronize=lambda: None, set_device=lambda d: None, device_count=lambda: 1)
    return types.SimpleNamespace(cuda=cuda, tensor=torch.tensor, zeros_like=torch.zeros_like, float64=torch.float64,
                                 float32=torch.float32, device=torch.device, empty=torch.empty)


def _worker(rank, world, port, fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), MCPT_BENCH_BACKEND="gloo", MCPT_DIST_TIMEOUT_S="8")
    import torch

    import bench
    from mcpt import parallel

    def gather_film_to_root(pt, rank, world, tile=256):
        if rank == fail_rank:
            raise RuntimeError("injected gather failure")
        n = len(parallel.tiles_for_rank(rank, world, pt.W, pt.H, tile)) * tile * tile
        import torch.distributed as dist

        return parallel.gather_packed_to_root(torch.zeros((n, 4)), rank, world, dist, pt.W, pt.H, tile)

    parallel.gather_film_to_root = gather_film_to_root
    out = io.StringIO()
    err = None
    try:
        with contextlib.redirect_stdout(out):
            bench.main(["--gpus", str(world), "--steps", "1", "--warmup", "0", "--no-verify-gather",
                        "--no-work-counters"], tracer=lambda *a: (_Tracer(), None, None), torch_mod=_fake_torch())
    except BaseException as e:  # noqa: BLE001
        import traceback

        err = traceback.format_exc()
    q.put((rank, out.getvalue(), err))


def _run(world, fail_rank):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, text, err = q.get(timeout=180)
        res[r] = (text, err)
    for p in procs:
        p.join(60)
    return res


def test_gather_failure_still_prints_the_headline_gloo_world2():
    res = _run(2, fail_rank=1)
    text, err = res[0]
    assert err is None and res[1][1] is None
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    assert "error" in d["gather"]  # rank 0 timed out in its receive, or saw rank 1's failure
    assert d["weak"]["error"].startswith("skipped")  # the other split is not attempted after a failure
    assert d["config"]["product"] is False and "MCPT_BENCH_BACKEND" in d["config"]["knobs"]
    assert res[1][0] == ""  # only rank 0 prints


def test_gather_success_gloo_world2():
    res = _run(2, fail_rank=-1)
    d = json.loads([ln for ln in res[0][0].splitlines() if ln.startswith("{")][0])
    assert "error" not in d["gather"] and d["gather"]["gather_backend"] == "gloo"
    assert "error" not in d["weak"] and d["weak"]["frame"] == [1920, 2160]
