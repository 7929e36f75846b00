"""Multi-rank bench logic on CPU (gloo, world size 2): each rank encodes its own
frames (distinct seeds, weak scaling, no data-path collective); the process group
only provides barriers, the max-over-ranks time and the sum of pixels."""
import os
import time
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import bench

    r, local, w, pg = bench.dist_setup(world)
    bench.barrier(pg)
    mx = bench.max_over_ranks(pg, float(rank + 1) * 0.5)
    sm = bench.sum_over_ranks(pg, 1000.0)
    seeds = [bench.frame_seed(r, i) for i in range(16)]
    q.put((r, local, w, mx, sm, seeds))
    pg.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_bench_reductions_and_frame_sharding():
    mp = pytest.importorskip("torch.multiprocessing")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    (r0, l0, w0, mx0, sm0, s0), (r1, l1, w1, mx1, sm1, s1) = res
    assert (r0, r1, w0, w1, l0, l1) == (0, 1, 2, 2, 0, 1)
    assert mx0 == mx1 == 1.0          # slowest rank's time
    assert sm0 == sm1 == 2000.0       # whole-job pixels
    assert not set(s0) & set(s1)      # every rank encodes its own frames
    assert s0[0] == 3                 # rank 0 frame 0 = the config-3 seed


def test_single_rank_needs_no_process_group():
    sys.path.insert(0, ROOT)
    import bench

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    rank, local, world, pg = bench.dist_setup(1)
    assert (rank, local, world, pg) == (0, 0, 1, None)
    assert bench.max_over_ranks(pg, 2.5) == 2.5 and bench.sum_over_ranks(pg, 7.0) == 7.0


@pytest.mark.timeout(180)
def test_bench_gpus_n_spawns_ranks_without_a_launcher():
    """VERDICT r1 / ADVICE r1: `bench.py --gpus N` without torchrun starts N rank
    processes itself (before any GPU call); only rank 0 prints one JSON line."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["JPGE_BENCH_DEVICE_COUNT"] = "3"  # (mocked: a node with 3 GPUs)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--workload", "dist-check"],
                       env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["value"] == 3.0
    assert d["batch_frames"] == 256.0 and d["rank0_first"] == [0, 3, 6]
    assert d["devices"] == {"ranks": 3, "devices_visible": 3, "devices_distinct": 3, "ranks_per_device": 1,
                            "shared": False}


@pytest.mark.timeout(150)
def test_bench_refuses_more_ranks_than_gpus():
    """--gpus N on a node with fewer than N GPUs refuses (no fake
    scaling point); --allow-shared-gpu rehearses it and the line says the ranks share."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["JPGE_BENCH_DEVICE_COUNT"] = "1"  # (mocked: one GPU)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "dist-check"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "need 2 GPU(s), this node shows 1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    r = subprocess.run(cmd + ["--allow-shared-gpu"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["devices"] == {"ranks": 2, "devices_visible": 1, "devices_distinct": 1, "ranks_per_device": 2,
                            "shared": True}


@pytest.mark.timeout(150)
def test_bench_spawn_propagates_a_failing_rank():
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["JPGE_BENCH_FAIL_RANK"] = "1"  # rank 1 exits 3; rank 0 would wait in a barrier forever
    env["JPGE_BENCH_DEVICE_COUNT"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "dist-check"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(150)
def test_bench_phase_watchdog_names_a_stuck_rank():
    """A rank stuck in one phase (a first 8-GPU run that stalls in RCCL
    setup or a transfer) exits with status 124 once the phase outlives --phase-timeout, and
    says which rank and phase; the launcher ends the others and returns that status."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["JPGE_BENCH_HANG_RANK"] = "1"  # rank 1 sleeps inside a named phase; rank 0 waits in a barrier
    env["JPGE_BENCH_DEVICE_COUNT"] = "2"
    env["JPGE_BENCH_HANG_LIMIT"] = "4"  # the stuck phase's own limit; start-up keeps --phase-timeout
    t = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "dist-check",
                        "--phase-timeout", "40", "--pg-timeout", "60"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 124, r.stderr[-2000:]
    assert "rank 1: phase 'dist-check: stuck (test hook)' exceeded its 4 s limit" in r.stderr
    assert time.monotonic() - t < 60
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_records_the_cgroup_quota():
    sys.path.insert(0, ROOT)
    import bench

    q = bench.cgroup_quota_cpus()
    assert q is None or q > 0
    h = bench.host_cpu_use({"usage_usec": 0}, {"usage_usec": 4_000_000}, 2.0, 2)
    assert h["cpus_used"] == 2.0 and h["cpus_per_rank"] == 1.0 and "quota_cpus" in h


def test_batch_share_deals_every_frame_once():
    sys.path.insert(0, ROOT)
    import bench

    for world in (1, 2, 3, 4, 8):
        shares = [bench.batch_share(256, r, world) for r in range(world)]
        assert sorted(i for s in shares for i in s) == list(range(256))
        assert max(map(len, shares)) - min(map(len, shares)) <= 1
    assert bench.batch_seed(0) == 1000  # config 4 seeds


def _gather_worker(rank, world, port, q, B=37):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from jpgenc_amd.gather import BatchGather

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cap = 300  # (B: a batch that does not divide over the ranks; some empty segments)
    g = BatchGather(dist.new_group(backend="gloo"), dist.new_group(backend="gloo"), rank, world, B,
                    ((B + world - 1) // world) * cap, "cpu")

    def frame_bytes(step, i):  # deterministic stand-in .jpg bytes of frame i at a step
        gen = torch.Generator().manual_seed(1000 * step + i)
        n = int(torch.randint(0, cap, (1,), generator=gen)) if i % 7 else 0
        return torch.randint(0, 256, (n,), dtype=torch.uint8, generator=gen)

    ok = []
    for step in range(3):  # three posts: both pack buffers, one reused
        share = g.share(rank)
        segs, lens = [], []
        for i in share:
            b = frame_bytes(step, i)
            seg = torch.full((cap,), 0xEE, dtype=torch.uint8)  # (slot padding past the bytes)
            seg[:len(b)] = b
            segs.append(seg)
            lens.append(len(b))
        s = g.acquire()
        assert s == step % 2
        g.post(segs, lens)
        if rank == 0:
            g.wait()
            ok.append(all(torch.equal(g.frame(i), frame_bytes(step, i)) for i in range(B)))
    g.wait()
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world,B", [(2, 37), (3, 37), (3, 2)])
def test_batch_gather_is_byte_equal(world, B):
    """Config 4's gather: each rank packs its frames' bytes into one
    message; rank 0 finds every frame of the batch byte-equal, over three batches
    (both pack buffers used, one reused).  B=2 over 3 ranks: a rank with no frames
    (ADVICE r4)."""
    mp = pytest.importorskip("torch.multiprocessing")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q, B)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert res[0] == [True, True, True]
