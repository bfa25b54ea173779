"""The N > 1 bench lines explain their own time and the end-to-end line runs at
N GPUs -- the CPU-checkable parts:

* ``bench.py --e2e --e2e-mode shm`` routes to the sharded shm ingest at world > 1 (and with
  ``--e2e-mode shm_shard`` at any world), other e2e modes refuse world > 1;
* ``bench.time_attribution``'s arithmetic (kernel ms by rank, exposed collective ms, per-wave
  all-gather span / GB/s) on hand-made gather timings;
* ``flame_amd.shard.GATHER_TIMING`` is filled by the real in-place gathers over a world-2 gloo
  group on CPU, and ``time_attribution`` all-gathers both ranks' numbers.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("world,mode,want", [
    (2, "shm", "sharded"), (8, "shm", "sharded"), (1, "shm", "e2e"), (1, "shm_shard", "sharded"),
    (2, "shm_shard", "sharded"), (1, "zerocopy", "e2e"), (2, "zerocopy", "refused"), (4, "copy", "refused"),
])
def test_e2e_routing(monkeypatch, world, mode, want):
    seen = []
    monkeypatch.setenv("WORLD_SIZE", str(world))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setattr(bench, "setup_dist", lambda force=False: (world, 0, 0))
    monkeypatch.setattr(bench, "bench_e2e_shm_sharded", lambda args, w, r, dev, n, P: seen.append(("sharded", w, n, P)))
    monkeypatch.setattr(bench, "bench_e2e", lambda args, n, P, dev: seen.append(("e2e", 1, n, P)))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", str(world), "--e2e", "--e2e-mode", mode,
                                      "--clients", "64", "--params", "2000000"])
    if want == "refused":
        with pytest.raises(SystemExit) as e:
            bench.main()
        assert "one-GPU mode" in str(e.value) and "--e2e-mode shm" in str(e.value)
        assert seen == []
        return
    bench.main()
    assert seen == [(want, world, 64, 2_000_000)]


def test_time_attribution_arithmetic():
    # host-time marks (seconds): wave 0 twice (2 ms, 4 ms spans), wave 1 once (1 ms)
    gt = [(0, 8_000_000, 1.0, 1.002), (1, 2_000_000, 2.0, 2.001), (0, 8_000_000, 3.0, 3.004)]
    a = bench.time_attribution(1, 10.0, 12.5, gt)
    assert a["kernel_ms_by_rank"] == [10.0] and a["kernel_ms_max"] == a["kernel_ms_min"] == 10.0
    assert a["exposed_collective_ms"] == pytest.approx(2.5)
    w0, w1 = a["allgather"]
    assert w0["wave"] == 0 and w0["bytes_received_per_rank"] == 8_000_000
    assert w0["span_ms_by_rank"][0] == pytest.approx(3.0)
    assert w0["GBps"] == pytest.approx(8e6 / 3e-3 / 1e9)
    assert w1["GBps"] == pytest.approx(2e6 / 1e-3 / 1e9)
    assert a["last_wave_exposed_gather_ms"] == pytest.approx(1.0)
    none = bench.time_attribution(1, None, 5.0, [])
    assert none["exposed_collective_ms"] is None and none["allgather"] == []


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from flame_amd import shard
        model = {"w": torch.zeros(world * 4096 * 2, dtype=torch.float32)}
        plan = shard.ShardPlan(model, world, rank, align=64, fracs=(0.75, 0.25))
        comm = shard._Comm()
        shard.GATHER_TIMING = []
        flat = model["w"]
        for w in range(plan.n_waves):
            pairs = []
            for s in plan.subs:
                if s.wave == w and not s.tail:
                    flat[s.lo:s.hi] = rank + 1.0
                    pairs.append((flat[s.g0:s.g1], flat[s.lo:s.hi]))
            comm.all_gather_inplace(pairs, w)
        comm.wait()
        gt = shard.GATHER_TIMING
        shard.GATHER_TIMING = None
        ok = len(gt) == plan.n_waves == 2
        for w, recv, t0, t1 in gt:
            piece = sum(s.g1 - s.g0 for s in plan.subs if s.wave == w and not s.tail)
            ok &= recv == piece * 4 * (world - 1) // world and t1 >= t0
        # every rank's range arrived in place
        ok &= all(float(flat[s.g0 + r * ((s.g1 - s.g0) // world)]) == r + 1.0
                  for s in plan.subs if not s.tail for r in range(world))
        import bench as B
        a = B.time_attribution(world, 1.0 + rank, 10.0, gt)
        ok &= a["kernel_ms_by_rank"] == [1.0, 2.0] and a["exposed_collective_ms"] == pytest.approx(8.0)
        ok &= [x["wave"] for x in a["allgather"]] == [0, 1] and all(
            len(x["span_ms_by_rank"]) == world and x["bytes_received_per_rank"] > 0 for x in a["allgather"])
        dist.destroy_process_group()
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put((rank, repr(e)))


def test_gather_timing_over_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}, res
