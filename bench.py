"""jpge benchmark — BASELINE.json metric: MPixels/s encode (4K 4:2:0 Q=90).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 4k-frames|batch1080|16k-striped|ppm-files]

Launch: `--gpus N` under torch.distributed.run uses its RANK/WORLD_SIZE; without a
launcher (WORLD_SIZE unset) and N > 1 this script starts the N rank processes
itself, before anything touches a GPU, and exits with the worst rank's status.
Only rank 0 prints.

Workloads (a step = one pass of the full encode path over a batch of synthetic
frames resident in HBM: colour/4:2:0/FDCT/quantise + statistics kernels, host
Huffman-table build, entropy code + pack kernels, finished .jpg bytes in HBM):
  4k-frames  (default; BASELINE metric, SURVEY 8(e) frames): F = 3072 frames of
             3840x2160 Q90 per GPU per step, cycling over D = 32 distinct inputs
             (800 MB > the 256 MB Infinity Cache, so K1 reads from HBM); frames are
             independent, each rank encodes its own (weak scaling, no data-path
             collective; the gloo group only carries barriers and the max time).
  batch1080  (config 4): one batch of 256 distinct 1920x1080 Q90 frames (seeds
             1000+i) per step, dealt over the ranks (frame i -> rank i mod N:
             strong scaling); each rank's .jpg bytes go to rank 0 in one transfer
             (RCCL send/recv; HIP IPC when ranks share a GPU), overlapped with the
             next step's encode.
  16k-striped (config 5): one 16384^2 frame per step, row-striped over the ranks.
  ppm-files  (SURVEY 8(f) rank 1): PPM files -> .jpg files (PCIe-inclusive).

The 4k-frames line carries: `roofline` = the dominant kernel alone on the GPU (its
exclusive time: a 1-lane encoder after the timed region, HIP events bound to the
kernel's own dispatch; checked against the step: launches x duration <= ms_per_step),
`roofline_dct_stage` = K1 alone (the BASELINE figure, with its HBM-read-only
fraction), `latency` (one frame per jpge_encode_rgb8 call, device and pinned-host
buffers: the reference's one-image-per-call path), `roofline_pipeline`, per-kernel rooflines in situ (`stages`, overlapping
lanes: diagnostic) and alone (`stages_solo`; algorithmic bytes per launch, DESIGN.md
§4), `devices` (ranks, distinct GPUs, ranks per GPU), `verified` (every output of
the last timed step byte-compared with the host-path encode of its frame, and a
sample with the CPU oracle), `d2h` (device RGB -> .jpg bytes in pinned host
memory, SURVEY 8(d)'s end-to-end definition) and `cpu_baseline` (the test-only
oracle on the host cores, rank 0 at N=1; the reference's own figure from this
container's BASELINE.md beside it).
"""
from __future__ import annotations

import argparse
import collections
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W4K, H4K = 3840, 2160
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# The reference's own encoder (writeJPEG) at 4K 4:2:0 Q90, timed in the survey
# container (1874 ms on 8 vCPU = 4.4 MPix/s); the reference needs
# Boost, absent here and on the GPU box, so it cannot be rebuilt beside the GPU.
REF_CPU_4K_Q90 = {"value": 4.4, "unit": "MPix/s", "cores": 8, "kind": "reference",
                  "source": "BASELINE.md §2 (reference writeJPEG, 3840x2160 Q90, 8 vCPU Xeon, survey container)"}
REF_CPU_1080_Q90 = {"value": 3.8, "unit": "MPix/s", "cores": 8, "kind": "reference",
                    "source": "BASELINE.md §2 (reference writeJPEG, 1920x1080 Q90: 550 ms, 8 vCPU Xeon, survey container)"}
REF_CPU_16K_Q90 = {"value": 3.6, "unit": "MPix/s", "cores": 8, "kind": "reference",
                   "source": "BASELINE.md §2 (reference writeJPEG, 16384x16384 Q90, single interval: 74.5 s, 8 vCPU "
                             "Xeon, survey container)"}


# subsampling modes (jpge.h JPGE_S*) -> the name in the metric / workload
SUB_NAMES = {420: "4:2:0", 444: "4:4:4", 422: "4:2:2", 411: "4:1:1", 4200: "4:2:0 S420", 4201: "4:2:0 S420_lm"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per GPU per step (4k-frames: 3072, so the default 20 steps span ~3 s; "
                         "batch1080: the whole batch, 256)")
    ap.add_argument("--distinct", type=int, default=32, help="4k-frames: distinct input frames the step cycles over")
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--width", type=int, default=W4K)
    ap.add_argument("--height", type=int, default=H4K)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the post-timing output verification")
    ap.add_argument("--d2h-steps", type=int, default=5, help="steps of the D2H-inclusive pass (0 = skip)")
    ap.add_argument("--solo-batches", type=int, default=2,
                    help="batches through a 1-lane encoder after the timed region (kernel times alone; 0 = skip)")
    ap.add_argument("--solo-warmup", type=int, default=8, help="untimed batches before the solo pass's timed ones")
    ap.add_argument("--latency-calls", type=int, default=128,
                    help="4k-frames: single-frame jpge_encode_rgb8 calls timed for the latency key (0 = skip)")
    ap.add_argument("--lanes", type=int, default=0, help="encoder lanes (0 = library default)")
    ap.add_argument("--workload", choices=["4k-frames", "batch1080", "16k-striped", "ppm-files", "dist-check"],
                    default="4k-frames",
                    help="4k-frames: the BASELINE metric (frames sharded over ranks); batch1080: config 4 (256 "
                         "1080p frames per step dealt over the ranks, segments gathered to rank 0); 16k-striped: "
                         "one 16384x16384 frame per step, row-striped over the ranks (config 5); ppm-files: PPM "
                         "files -> .jpg files through the ingest pipeline (PCIe-inclusive); dist-check: the "
                         "launcher and reductions only, no GPU (CPU tests)")
    ap.add_argument("--restart", type=int, default=None,
                    help="restart interval in MCUs (16k-striped: default 1024 = one interval per MCU row, "
                         "the config's 'tiled with restart intervals'; 0 = the reference's single interval)")
    ap.add_argument("--subsampling", type=int, choices=sorted(SUB_NAMES), default=420,
                    help="4k-frames: subsampling mode (jpge.h JPGE_S*: 420 = the reference's S420_m; "
                         "444, 422, 411, 4200 = S420, 4201 = S420_lm are extensions)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="rehearse N ranks on fewer than N GPUs (ranks share devices; the line says so). "
                         "Without it, --gpus N refuses to run on a node with fewer than N GPUs")
    ap.add_argument("--no-kernel-events", action="store_true", help="diagnostic: time without per-kernel events")
    ap.add_argument("--pg-timeout", type=float, default=120.0,
                    help="seconds a gloo / RCCL collective may wait before it fails (process groups' timeout)")
    ap.add_argument("--phase-timeout", type=float, default=420.0,
                    help="seconds a rank may spend in one phase (setup, warm-up, timed steps, ...) before it "
                         "exits with status 124, naming the phase (0 = no watchdog)")
    ap.add_argument("--event-every", type=int, default=1024,
                    help="in the timed region, launch the kernels of the frame set holding every N-th frame with "
                         "timing events (the in-situ diagnostic; events cost throughput and host CPU: a HIP "
                         "runtime thread waits on their signals, 0.69 CPU at every 64th frame, 0.04 at every "
                         "1024th)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- launch / ranks

def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(n: int, argv: list[str]) -> int:
    """Start n rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* as
    torch.distributed.run sets them) and wait for them.  Called before anything
    touches a GPU.  A rank that fails ends the others; returns the worst status."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    # (children reaped in the order they end, so the rank that failed first names the
    # status, not a peer that failed because it vanished)
    rc = 0
    live = {p.pid: p for p in procs}
    while live:
        pid, status = os.waitpid(-1, 0)
        p = live.pop(pid, None)
        if p is None:
            continue
        code = os.waitstatus_to_exitcode(status)
        p.returncode = code
        if code != 0 and rc == 0:
            rc = code if code > 0 else 128 - code
            for q in live.values():  # (our own children, by handle)
                q.terminate()
    return rc


class PhaseWatch:
    """Names the phase each rank is in and ends a rank stuck in one: a
    daemon thread checks once a second; a phase older than its limit prints the rank, the
    phase and the time to stderr and exits the process with status 124, so a first
    multi-GPU run that stalls (RCCL setup, a p2p transfer, a barrier) ends well inside the
    driver's own limit and says where.  (os._exit: no GPU teardown, no exec.)"""

    def __init__(self, limit_s: float):
        import threading

        self.limit = limit_s
        self.rank = int(os.environ.get("RANK", "0"))
        self.name, self.t0 = "start", time.monotonic()
        self.extra = {}
        self.lock = threading.Lock()
        if limit_s > 0:
            threading.Thread(target=self._run, daemon=True).start()

    def __call__(self, name: str, limit_s: float | None = None) -> None:
        with self.lock:
            self.name, self.t0 = name, time.monotonic()
            self.extra[name] = limit_s

    def _run(self):
        while True:
            time.sleep(1.0)
            with self.lock:
                name, t0 = self.name, self.t0
                lim = self.extra.get(name) or self.limit
            dt = time.monotonic() - t0
            if dt > lim:
                print(f"bench: rank {self.rank}: phase '{name}' exceeded its {lim:.0f} s limit ({dt:.0f} s); "
                      f"exiting with status 124", file=sys.stderr, flush=True)
                os._exit(124)


PHASE = PhaseWatch(0)  # (main() replaces it with the --phase-timeout watch)


def pg_timeout(args):
    import datetime

    return datetime.timedelta(seconds=max(10, int(args.pg_timeout)))


def dist_setup(n_gpus: int, args=None):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and n_gpus > 1 and n_gpus != world:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    pg = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        PHASE("init_process_group (gloo rendezvous)")
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=pg_timeout(args) if args is not None else None)
        pg = dist
    return rank, local, world, pg


def barrier(pg):
    if pg is not None:
        name = PHASE.name
        PHASE(f"barrier after '{name}'")
        pg.barrier()
        PHASE(name)


def max_over_ranks(pg, v: float) -> float:
    if pg is None:
        return v
    import torch

    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(pg, v: float) -> float:
    if pg is None:
        return v
    import torch

    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def all_gather_floats(pg, v: float, world: int) -> list[float]:
    """Every rank's value, in rank order (on rank 0; a list of one without a group)."""
    if pg is None:
        return [v]
    import torch

    out = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    pg.all_gather(out, torch.tensor([v], dtype=torch.float64))
    return [float(t.item()) for t in out]


def process_cpu_s() -> float:
    """CPU seconds used by this process (every thread, user + system)."""
    t = os.times()
    return t.user + t.system


GATHER_NAMES = {"p2p": "RCCL isend/irecv over xGMI",
                "ipc": "HIP IPC into rank 0's buffers: the ranks share one GPU, which RCCL refuses",
                "gloo (host-staged)": "gloo through host memory"}


def visible_devices() -> int:
    """GPUs this node shows (torch.cuda.device_count() does not initialise the GPU on
    this image; JPGE_BENCH_DEVICE_COUNT overrides it for the CPU tests)."""
    if os.environ.get("JPGE_BENCH_DEVICE_COUNT"):
        return int(os.environ["JPGE_BENCH_DEVICE_COUNT"])
    import torch

    return torch.cuda.device_count()


def device_plan(world: int, allow_shared: bool) -> dict:
    """One GPU per rank, or a refusal: N ranks on fewer than N GPUs would publish a
    scaling point that no N-GPU run produced.  --allow-shared-gpu rehearses N ranks on
    fewer GPUs (rank r on GPU r mod count); the line then says so (`devices`)."""
    n = visible_devices()
    if world > n and not allow_shared:
        raise SystemExit(f"bench: {world} rank(s) need {world} GPU(s), this node shows {n}; "
                         f"--allow-shared-gpu rehearses ranks sharing GPUs (not a scaling point)")
    distinct = min(world, max(n, 1))
    return {"ranks": world, "devices_visible": n, "devices_distinct": distinct,
            "ranks_per_device": -(-world // distinct), "shared": world > distinct}


def device_for(local: int) -> int:
    """This rank's GPU: LOCAL_RANK (wrapped only under --allow-shared-gpu, which
    device_plan checked before any GPU work)."""
    return local % max(1, visible_devices())


def rank_lanes(args, world: int) -> int:
    """Encoder lanes of this rank: --lanes, else the library default (4) on a GPU of its
    own.  Ranks sharing a GPU (--allow-shared-gpu) split ~6 lanes between them: config 4
    on 2 ranks sharing one GPU ran at 0.88x one rank on it with 3 lanes each, 0.82x with
    4 and 0.74x with 2 (one box)."""
    if args.lanes:
        return args.lanes
    per_device = -(-world // max(1, visible_devices()))
    return max(1, 6 // per_device) if per_device > 1 else 0


def gather_group(world: int, args=None):
    """Process group for the data-path collectives: RCCL ("nccl") when every rank
    has its own GPU, else gloo (ranks sharing a GPU; tensors staged through the host)."""
    import torch
    import torch.distributed as dist

    backend = "nccl" if visible_devices() >= world else "gloo"
    PHASE(f"new_group ({backend})")
    return dist.new_group(backend=backend, timeout=pg_timeout(args) if args is not None else None)


def frame_seed(rank: int, i: int) -> int:
    return 3 + 1000 * rank + i  # config 3 seed family, distinct per rank and frame


def batch_seed(i: int) -> int:
    return 1000 + i  # config 4: 256 x 1080p, seeds 1000+i


def batch_share(total: int, rank: int, world: int) -> list[int]:
    """Frames of a config-4 batch that `rank` encodes (frame i -> rank i mod world)."""
    return list(range(rank, total, world))


# ---------------------------------------------------------------- CPU baseline

def cpu_baseline(args) -> tuple[dict, dict]:
    """The 4k-frames workload's baseline: whole frames of the step's inputs (seeds 3..)."""
    import jpgenc_amd as J

    ref = REF_CPU_4K_Q90 if (args.width, args.height, args.quality, args.subsampling) == (W4K, H4K, 90, 420) else None
    return oracle_cpu_baseline(args, lambda i: J.synth_rgb8(frame_seed(0, i), args.width, args.height),
                               f"{args.width}x{args.height} {sub_name(args)} Q{args.quality} frames (seeds 3..)", ref,
                               subsampling=args.subsampling, want_hashes=True)


def sub_name(args) -> str:
    return SUB_NAMES[getattr(args, "subsampling", 420)]


def cgroup_cpu_stat() -> dict:
    """The process cgroup's CPU accounting (usage and quota throttling), if visible."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f)}
    except (OSError, ValueError):
        return {}


def thread_cpu() -> dict:
    """CPU seconds per thread of this process, keyed (tid, name)."""
    out = {}
    tick = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
            name = st[st.index("(") + 1:st.rindex(")")]
            fields = st[st.rindex(")") + 2:].split()
            out[(tid, name)] = (int(fields[11]) + int(fields[12])) / tick
        except (OSError, ValueError, IndexError):
            pass
    return out


def thread_report(th0: dict, dt: float):
    """Diagnostic (JPGE_BENCH_THREADS): each thread's CPUs over the timed region, to stderr."""
    if not th0:
        return
    th1 = thread_cpu()
    use = collections.Counter()
    for k, v in th1.items():
        use[k] += (v - th0.get(k, 0.0)) / dt
    print(f"threads: {len(th1)}; busiest:", {f"{k[1]}/{k[0]}": round(v, 2) for k, v in use.most_common(24)},
          file=sys.stderr)


class ThreadSampler:
    """Diagnostic (JPGE_BENCH_THREADS=2): samples every thread's scheduler state and
    kernel wait channel every 2 ms; stop() prints each busy thread's distribution."""

    def __init__(self):
        import threading

        self.counts = collections.defaultdict(collections.Counter)
        self.done = threading.Event()
        self.th = threading.Thread(target=self.run, daemon=True)
        self.th.start()

    def run(self):
        while not self.done.wait(0.002):
            for tid in os.listdir("/proc/self/task"):
                try:
                    with open(f"/proc/self/task/{tid}/stat") as f:
                        st = f.read()
                    with open(f"/proc/self/task/{tid}/wchan") as f:
                        wc = f.read().strip() or "0"
                    name = st[st.index("(") + 1:st.rindex(")")]
                    state = st[st.rindex(")") + 2]
                    self.counts[f"{name}/{tid}"][f"{state}:{wc}"] += 1
                except (OSError, ValueError):
                    pass

    def stop(self):
        self.done.set()
        self.th.join()
        for k, c in self.counts.items():
            if sum(n for s, n in c.items() if s.startswith("R")) > 0:
                print(f"sampler {k}: {dict(c.most_common(6))}", file=sys.stderr)


def load_pmc_traffic(profile_dir: str, width: int, height: int) -> dict:
    """Per-launch HBM bytes per stage from the newest committed rocprofv3 PMC summary of this
    frame size (profiles/pmc_rNN.json for 4K, profiles/rNN_pmc_<size>.json for others; the
    entropy stage = its code, placement-scan and pack kernels)."""
    def round_of(f):
        return f[5:7] if f.startswith("pmc_r") else f[1:3]
    try:
        names = sorted((f for f in os.listdir(profile_dir) if f.endswith(".json") and
                        (f.startswith("pmc_r") or (f.startswith("r") and "_pmc_" in f))),
                       key=round_of, reverse=True)
    except OSError:
        return {}
    per = None
    for name in names:
        try:
            with open(os.path.join(profile_dir, name)) as f:
                d = json.load(f)
            if d.get("width") == width and d.get("height") == height:
                per = {k.split("<")[0]: v["hbm_bytes_per_launch"] for k, v in d["kernels"].items()}
                if "stats_wave_kernel" in per:  # (round 4's statistics kernel reports as stats_kernel)
                    per["stats_kernel"] = per.pop("stats_wave_kernel")
                break
        except (OSError, ValueError, KeyError, TypeError):
            continue
    if per is None:
        return {}
    out = {k: v for k, v in per.items() if not k.startswith("entropy_")}
    ent = [v for k, v in per.items() if k.startswith("entropy_")]
    if ent:
        out["entropy_kernel"] = sum(ent)
    return out


def cgroup_quota_cpus():
    """The cgroup's CPU quota in CPUs (cpu.max: quota / period), None when unlimited or
    not visible."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def host_cpu_use(cg0: dict, cg1: dict, dt: float, world: int = 1):
    """The cgroup's CPU use over the timed region (every rank of this box shares it), its
    quota and throttling, and CPUs per rank."""
    if not cg0:
        return {"cpus_used": None, "quota_cpus": cgroup_quota_cpus(), "reason": "cgroup cpu.stat not visible"}
    used = (cg1.get("usage_usec", 0) - cg0.get("usage_usec", 0)) / 1e6 / dt
    return {"cpus_used": round(used, 2), "quota_cpus": cgroup_quota_cpus(),
            "cpus_per_rank": round(used / max(1, world), 2), "ranks_in_cgroup": world,
            "throttled_periods": cg1.get("nr_throttled", 0) - cg0.get("nr_throttled", 0),
            "throttled_ms": round((cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0)) / 1e3, 1)}



# ---------------------------------------------------------------- kernel rooflines

def solo_timing(J, local, frames, outd, args, fset: int, restart: int = 0):
    """After the timed region: the given frames through a 1-lane encoder (nothing else on
    the GPU), every launch with its own HIP events bound to its dispatch, in frame sets of
    `fset` (the pipeline's launch shape; 1 = one frame per launch).  Returns the encoder's
    timing and the CLOCK_MONOTONIC window (rocprofv3 timestamps use the same clock)."""
    env = {"JPGE_SET": str(fset)}
    if fset > 1:  # (a 1-lane encoder places by the pack kernels unless told otherwise; sets place in the code kernel)
        env["JPGE_EXT_PLACE"] = "1"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        solo = J.Encoder(local, lanes=1)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    solo.set_subsampling(getattr(args, "subsampling", 420))
    if restart:
        solo.set_restart(restart)
    # warm-up batches first: right after a multi-lane region the chip's clock is still
    # settling (K1, fp64 VALU, ran its first solo batch ~1-2 us slower)
    for _ in range(max(1, args.solo_warmup)):
        solo.encode_batch_dev(frames, outd, quality=args.quality)
    solo.set_timing(1)
    solo.reset_timing()
    s0 = time.monotonic_ns()
    for _ in range(args.solo_batches):
        solo.encode_batch_dev(frames, outd, quality=args.quality)
    win = [s0, time.monotonic_ns()]
    tm = solo.timing()
    solo.close()
    return tm, win


def record_bytes(counts) -> float:
    """K2's symbol records of one frame (kernels.hpp): 2 bytes per Huffman-coded symbol,
    and a 2-byte continuation for each symbol whose size (AC) or category (DC) is above 6;
    counts = the frame's four histograms (Encoder.symbol_stats)."""
    c = np.asarray(counts, np.int64).reshape(4, 256)
    s = np.arange(256)
    size = np.where((np.arange(4)[:, None] & 1) == 1, s & 15, s)
    return 2.0 * float(c.sum() + c[size > 6].sum())


REC_WHAT = "16-bit symbol records (2 B per symbol, +2 B per size > 6)"


def alg_bytes(npx: float, cb: float, rec_bytes: float, avg_jpeg: float):
    """Per-kernel and entropy-stage algorithmic bytes per frame: K1 reads
    RGB8 and writes int16 coefficients; K2 reads the coefficients and writes its 16-bit
    symbol records (record_bytes); the code kernel reads the records and writes the bit
    stream (~ the .jpg size); the pack kernel reads it and writes the stuffed bytes."""
    alg = {
        "fdct_kernel": ((3.0 + cb) * npx, f"RGB8 read 3 B/px + int16 coefficients written {cb:g} B/px"),
        "stats_kernel": (cb * npx + rec_bytes, f"coefficients read {cb:g} B/px + {REC_WHAT} written"),
        "entropy_code_kernel": (rec_bytes + avg_jpeg, f"{REC_WHAT} read + bit stream written (~.jpg size)"),
        "entropy_pack_kernel": (2.0 * avg_jpeg, "bit stream read + stuffed .jpg bytes written"),
    }
    stage = {"entropy_stage": (rec_bytes + avg_jpeg, f"{REC_WHAT} read + .jpg bytes written")}
    return alg, stage


TM_KEY = {"fdct_kernel": "fdct_sum", "stats_kernel": "dc_stats_sum", "entropy_code_kernel": "code_sum",
          "entropy_pack_kernel": "pack_sum", "entropy_stage": "entropy_sum"}
PMC_KEY = {"entropy_stage": "entropy_kernel"}


def kernel_rooflines(tm, alg, stage_alg, traffic, npx):
    """Per launch (a frame set's launch covers frames_per_launch frames: its bytes and its
    duration both); traffic (PMC, profiles/) is per frame."""
    nl = max(1, tm.get("launches") or tm["frames"])
    fpl = tm["frames"] / nl if tm["frames"] else 1.0
    out = {}
    timed = bool(tm.get("launches") or tm["frames"])
    for name, (b, what) in list(alg.items()) + list(stage_alg.items()):
        ms = tm[TM_KEY[name]] / nl
        bl = b * fpl
        tr = traffic.get(PMC_KEY.get(name, name))
        if not timed or ms <= 0:  # (no launch of this pass was timed: no figure, not a zero)
            out[name] = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                         "traffic": int(tr * fpl) if tr else tr, "alg_bytes_per_launch": int(bl),
                         "alg_bytes": what, "avg_kernel_ms": None, "timed_launches": 0,
                         "reason": "no launch of this kernel was timed in this pass (kernel events off or "
                                   "no sampled frame)"}
            continue
        ach = bl / (ms * 1e-3) / 1e9
        out[name] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": int(tr * fpl) if tr else tr,
                     "alg_bytes_per_launch": int(bl), "alg_bytes": what, "avg_kernel_ms": round(ms, 5),
                     "timed_launches": nl, "frames_per_launch": round(fpl, 3)}
    # the north star's "HBM-read roofline": K1's RGB8 read alone (3 B/px)
    k1 = out["fdct_kernel"]
    ms1 = tm["fdct_sum"] / nl
    if ms1 > 0:
        rd = 3.0 * npx * fpl / (ms1 * 1e-3) / 1e9
        k1["read_achieved"] = round(rd, 1)
        k1["read_frac"] = round(rd / HBM_PEAK_GBS, 4)
    return out


def solo_headline(stages_solo, alg, frames_per_step: float, ms_step: float):
    """The headline roofline: the dominant kernel (longest exclusive time) ALONE on the GPU
    (the solo pass), checked against the step: its launches per step x its duration cannot
    exceed the step, or the run fails."""
    dominant = max(alg, key=lambda k: stages_solo[k]["avg_kernel_ms"] or 0.0)
    roofline = dict(kernel=dominant, timing="solo (1-lane encoder after the timed region; HIP events bound "
                                            "to the kernel's dispatch, hipExtLaunchKernel)", **stages_solo[dominant])
    lps = frames_per_step / roofline["frames_per_launch"]
    spent = lps * roofline["avg_kernel_ms"]
    roofline["check"] = {"launches_per_step": round(lps, 1), "launches_x_avg_ms": round(spent, 3),
                         "ms_per_step": round(ms_step, 3), "ok": spent <= ms_step}
    if spent > ms_step:
        raise SystemExit(f"bench: roofline check failed: {lps:.1f} launches x {roofline['avg_kernel_ms']} ms "
                         f"= {spent:.3f} ms > {ms_step:.3f} ms per step")
    return roofline


def oracle_cpu_baseline(args, make_frame, label: str, reference: dict | None, restart: int = 0,
                        subsampling: int = 420, want_hashes: bool = False):
    """The test-only oracle (CPU restatement of the reference path) on a bounded sample of
    the workload: frames from make_frame(i) until ~cpu_seconds of encode time (synthesis
    excluded).  Returns the cpu_baseline object and {i: sha256 of the oracle's bytes}."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # noqa: E402

    PHASE("cpu baseline (oracle)")
    threads = min(16, os.cpu_count() or 1)
    _oracle.orc().orc_set_threads(threads)
    enc_times, hashes, px = [], {}, 0
    for i in range(64):
        rgb = make_frame(i)
        t = time.perf_counter()
        out = _oracle.encode(rgb, args.quality, restart=restart, subsampling=subsampling)
        enc_times.append(time.perf_counter() - t)
        px += rgb.shape[0] * rgb.shape[1]
        if want_hashes:
            hashes[i] = hashlib.sha256(out).hexdigest()
        if sum(enc_times) >= args.cpu_seconds:
            break
    return {
        "value": round(px / sum(enc_times) / 1e6, 3),
        "unit": "MPix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(enc_times)} x {label}, oracle/jpge_oracle.cpp restatement, OpenMP {threads} threads "
                  f"(DCT/quant parallel, like the reference)",
        "reference": reference,
    }, hashes


# ---------------------------------------------------------------- workloads

def run_dist_check(args, rank, local, world, pg):
    """The launcher and the reductions without a GPU (CPU tests of --gpus N;
    JPGE_BENCH_FAIL_RANK=r makes rank r fail before the first barrier)."""
    if os.environ.get("JPGE_BENCH_FAIL_RANK") == str(rank):
        raise SystemExit(3)
    if os.environ.get("JPGE_BENCH_HANG_RANK") == str(rank):  # (the phase watchdog's test)
        # (its own limit: under a loaded test host the other phases keep --phase-timeout's slack)
        PHASE("dist-check: stuck (test hook)", float(os.environ.get("JPGE_BENCH_HANG_LIMIT", "0")) or None)
        time.sleep(3600)
    barrier(pg)
    dt = max_over_ranks(pg, 0.001 * (rank + 1))
    n = sum_over_ranks(pg, 1.0)
    share = batch_share(256, rank, world)
    frames = sum_over_ranks(pg, float(len(share)))
    if rank == 0:
        print(json.dumps({"metric": "dist-check", "value": n, "unit": "ranks", "n_gpus": world, "max_time": dt,
                          "batch_frames": frames, "rank0_first": share[:3], "devices": args.devices}), flush=True)


def run_striped16k(args, rank, local, world, pg):
    """One 16384^2 frame per step: whole-frame encode on one GPU; on N GPUs each
    rank holds and encodes its row stripe, with the three RCCL exchanges and the
    segment gather of SURVEY 8(e) inside the timed step (output identical to 1 GPU).
    After the timed region each rank's frame (or stripe) runs through a 1-lane encoder
    with kernel events (the roofline), and at N = 1 the CPU oracle encodes row stripes
    of the same frame (the CPU baseline)."""
    import torch

    import jpgenc_amd as J
    from jpgenc_amd import stripes

    local = device_for(local)
    torch.cuda.set_device(local)
    W = H = 16384
    restart = 1024 if args.restart is None else args.restart
    PHASE("setup (16K frame, encoder)")
    rgb = J.synth_rgb8(5, W, H)  # SURVEY 8(d) config 5 seed
    cap = J.max_jpeg_bytes(W, H)
    out = torch.empty(cap, dtype=torch.uint8, device=f"cuda:{local}")
    if world == 1:
        r0, nr = 0, H // 16
        enc = J.Encoder(local)
        enc.set_restart(restart)
        src = torch.from_numpy(rgb.reshape(-1)).to(f"cuda:{local}")

        def step():
            return enc.encode_batch_dev([(src.data_ptr(), W, H, W * 3)], [(out.data_ptr(), cap)],
                                        quality=args.quality)[0]
    else:
        import torch.distributed as dist

        rccl = gather_group(world, args)  # the exchanges and the gather ride RCCL over xGMI
        r0, nr = stripes.stripe_rows(H // 16, world, stripes.restart_align(W, restart))[rank]
        src = torch.from_numpy(np.ascontiguousarray(rgb[16 * r0:16 * (r0 + nr)]).reshape(-1)).to(f"cuda:{local}")
        del rgb
        enc = J.Encoder(local, lanes=1)
        enc.set_restart(restart)

        def step():
            return stripes.encode_stripe_dist(enc, src.data_ptr(), W * 3, W, H, args.quality, out, group=rccl,
                                              restart=restart)
    PHASE("warm-up steps (first RCCL exchanges)" if world > 1 else "warm-up steps")
    for _ in range(args.warmup):
        n = step()
    torch.cuda.synchronize()
    barrier(pg)
    PHASE("timed steps")
    cg0 = cgroup_cpu_stat()
    pc0 = process_cpu_s()
    win0 = time.monotonic_ns()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n = step()
    torch.cuda.synchronize()
    barrier(pg)
    dt = time.perf_counter() - t0
    win1 = time.monotonic_ns()
    cg1 = cgroup_cpu_stat()
    rank_cpus = all_gather_floats(pg, (process_cpu_s() - pc0) / dt, world)
    dt = max_over_ranks(pg, dt)
    ms_step = dt / args.steps * 1e3
    # per-kernel rooflines: this rank's rows (the whole frame at N = 1) as one frame through
    # a 1-lane encoder with kernel events (the same kernels over the same pixels; a stripe's
    # own phases run them with the exchanges between)
    roofline = stages_solo = None
    solo_win = None
    hs = 16 * nr if world > 1 else H
    # the output against the oracle's hash of this configuration (tests/golden/large_frames.json)
    verified = None
    if rank == 0 and not args.no_verify:
        PHASE("verification")
        with open(os.path.join(ROOT, "tests", "golden", "large_frames.json")) as f:
            gold = [g for g in json.load(f)["frames"] if (g["width"], g["height"], g["seed"], g["quality"],
                                                          g.get("restart", 0)) == (W, H, 5, args.quality, restart)]
        if gold:
            got = hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()
            verified = {"sha256_match": got == gold[0]["sha256"] and int(n) == gold[0]["len"],
                        "method": "sha256 of the last step's .jpg (gathered on rank 0) against the oracle's "
                                  "(tests/golden/large_frames.json)"}
            if not verified["sha256_match"]:
                raise SystemExit(f"16k-striped: output differs from the oracle's ({got} vs {gold[0]['sha256']})")
        else:
            verified = {"sha256_match": None, "method": "no oracle hash recorded for this quality/restart"}
    if args.solo_batches > 0 and not args.no_kernel_events and rank == 0:
        PHASE("solo kernel timing")
        enc.close()
        tm_solo, solo_win = solo_timing(J, local, [(src.data_ptr(), W, hs, W * 3)], [(out.data_ptr(), cap)], args, 1,
                                        restart=restart)
        sym_enc = J.Encoder(local, lanes=1)
        hrows = rgb if world == 1 else src.view(hs, W, 3).cpu().numpy()
        rb = record_bytes(sym_enc.symbol_stats(hrows, quality=args.quality)[0])
        sym_enc.close()
        del hrows
        alg, stage_alg = alg_bytes(W * hs, 3.0, rb, float(n) * hs / H)
        stages_solo = kernel_rooflines(tm_solo, alg, stage_alg, {}, W * hs)
        roofline = solo_headline(stages_solo, alg, 1, ms_step)
    else:
        enc.close()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rows = 1024  # a bounded sample: 16384 x 1024 row stripes of the same frame, the same restart interval
        cpu, _ = oracle_cpu_baseline(args, lambda i: np.ascontiguousarray(rgb[rows * (i % (H // rows)):
                                                                              rows * (i % (H // rows) + 1)]),
                                     f"{W}x{rows} row stripes of the 16384^2 frame (seed 5), "
                                     + (f"restart interval {restart} MCUs" if restart else "single interval"),
                                     REF_CPU_16K_Q90 if args.quality == 90 and not restart else None, restart=restart)
        if cpu["reference"] is None and args.quality == 90:
            cpu["reference_single_interval"] = REF_CPU_16K_Q90
    if rank == 0:
        line = {
            "metric": f"MPixels/s encode (16K 4:2:0 Q={args.quality})",
            "value": round(W * H * args.steps / dt / 1e6, 1), "unit": "MPix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (deterministic splitmix64 photo-like frame, seed 5, HBM-resident)",
            "config": {"workload": f"16384x16384 4:2:0 Q{args.quality}, one frame per step, "
                                   + (f"restart interval {restart} MCUs, " if restart else "single interval, ")
                                   + ("whole frame on one GPU" if world == 1 else
                                      f"row-striped over {world} GPUs (RCCL: "
                                      + ("histogram sum/min, segment lengths; segments gathered to rank 0)"
                                         if restart else
                                         "DC seeds, histogram sum/min, summaries; segments gathered to rank 0)")),
                       "restart_mcus": restart, "jpeg_bytes": int(n)},
            "roofline": roofline,
            "roofline_dct_stage": dict(kernel="fdct_kernel", timing="solo", **stages_solo["fdct_kernel"])
            if stages_solo else None,
            "stages_solo": stages_solo,
            "solo_rows": hs,
            "verified": verified,
            "host_cpu": host_cpu_use(cg0, cg1, dt, world),
            "rank_cpus": [round(c, 2) for c in rank_cpus],
            "windows_monotonic_ns": {"timed": [win0, win1], "solo": solo_win},
            "devices": args.devices,
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)


def run_ppm_files(args, rank, local, world, pg):
    """F synthetic P6 files (in /dev/shm, i.e. the page cache) ->
    .jpg files per step through jpge_encode_files: file read + parse into pinned
    memory, H2D, kernels, D2H and file write all inside the timed step."""
    import shutil
    import tempfile

    import torch

    import jpgenc_amd as J

    local = device_for(local)
    torch.cuda.set_device(local)
    W, H, F = args.width, args.height, args.frames or 16
    tmp = tempfile.mkdtemp(prefix=f"jpge_ppm_{rank}_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        ins, outs = [], []
        for i in range(F):
            p = os.path.join(tmp, f"f{i}.ppm")
            with open(p, "wb") as f:
                f.write(f"P6\n{W} {H}\n255\n".encode())
                f.write(J.synth_rgb8(frame_seed(rank, i), W, H).tobytes())
            ins.append(p)
            outs.append(os.path.join(tmp, f"f{i}.jpg"))
        enc = J.Encoder(local)
        for _ in range(args.warmup):
            enc.encode_files(ins, outs, quality=args.quality)
        barrier(pg)
        t0 = time.perf_counter()
        nbytes = 0
        for _ in range(args.steps):
            nbytes += sum(enc.encode_files(ins, outs, quality=args.quality))
        barrier(pg)
        dt = max_over_ranks(pg, time.perf_counter() - t0)
        pixels = sum_over_ranks(pg, float(W * H * F * args.steps))
        if rank == 0:
            print(json.dumps({
                "metric": f"MPixels/s encode from PPM files ({W}x{H} 4:2:0 Q={args.quality})",
                "value": round(pixels / dt / 1e6, 1), "unit": "MPix/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic P6 files (deterministic splitmix64 photo-like frames) in /dev/shm",
                "config": {"workload": f"{F} PPM files -> .jpg files per GPU per step (jpge_encode_files: read + "
                                       f"parse into pinned memory, H2D, kernels, D2H, write)",
                           "width": W, "height": H, "quality": args.quality, "files_per_step_per_gpu": F,
                           "avg_jpeg_bytes": int(nbytes / (args.steps * F)),
                           "parallelism": f"files sharded over {world} GPU(s)"},
                "devices": args.devices,
            }), flush=True)
        enc.close()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def out_capacity(J, w: int, h: int) -> int:
    """Device output bytes per frame slot: half the RGB size (a Q90 4K frame codes to
    ~3 MB of 24.9 MB) within the library's worst-case bound; a frame that does not fit
    fails with JPGE_E_NOSPACE (the pack kernel checks the capacity)."""
    return min(J.max_jpeg_bytes(w, h), (w * h * 3 // 2 + 4095) // 4096 * 4096)


def run_batch1080(args, rank, local, world, pg):
    """Config 4: a batch of B (256) distinct 1920x1080 Q90 frames per step, frame i
    encoded by rank i mod N; every rank's .jpg bytes go to rank 0 packed in one RCCL
    message per rank (jpgenc_amd/gather.py), posted at the end of the step and moving
    while the next step encodes; the timed region ends once the last batch is on
    rank 0.  Strong scaling (the batch is fixed)."""
    import torch

    import jpgenc_amd as J

    local = device_for(local)
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"
    W, H, B = 1920, 1080, args.frames or 256
    share = batch_share(B, rank, world)
    cap = out_capacity(J, W, H)
    PHASE("setup (frames, encoder, gather)")
    host = {i: J.synth_rgb8(batch_seed(i), W, H) for i in share}
    ins = {i: torch.from_numpy(host[i].reshape(-1)).to(dev) for i in share}
    frames = [(ins[i].data_ptr(), W, H, W * 3) for i in share]
    enc = J.Encoder(local, lanes=rank_lanes(args, world))
    gather, transport = None, None
    nsets = 1
    if world > 1 and not os.environ.get("JPGE_BENCH_NO_GATHER"):  # (diagnostic: encode only, no gather)
        import torch.distributed as dist

        from jpgenc_amd.gather import BatchGather

        PHASE("new_group (gloo, lengths)")
        meta = dist.new_group(backend="gloo", timeout=pg_timeout(args))
        if args.devices["shared"]:  # ranks on one GPU: RCCL refuses them; rank 0's buffers over HIP IPC
            PHASE("gather setup (HIP IPC handles)")
            gather = BatchGather(None, meta, rank, world, B, len(share) * cap, dev, transport="ipc")
            if gather.transport != "ipc":  # (no IPC: stage through the host over gloo)
                gather = BatchGather(dist.new_group(backend="gloo", timeout=pg_timeout(args)), meta, rank, world, B,
                                     len(share) * cap, "cpu")
        else:
            gather = BatchGather(gather_group(world, args), meta, rank, world, B, len(share) * cap, dev)
        transport = gather.transport if gather.cuda else "gloo (host-staged)"
        nsets = 2  # output slots alternate, so the next encode never waits for this step's pack
    outbuf = torch.empty(nsets * len(share) * cap, dtype=torch.uint8, device=dev)
    base = len(share) * cap
    outd = [[(outbuf.data_ptr() + s * base + k * cap, cap) for k in range(len(share))] for s in range(nsets)]
    segs = [[outbuf[s * base + k * cap:s * base + (k + 1) * cap] for k in range(len(share))] for s in range(nsets)]
    phase = collections.Counter()

    def step():
        # encode this rank's share; then pack its .jpg bytes and post them to rank 0 as
        # one transfer, which moves while the next step encodes (jpgenc_amd/gather.py)
        t0 = time.perf_counter()
        s = gather.acquire() if gather is not None else 0
        t1 = time.perf_counter()
        lens = enc.encode_batch_dev(frames, outd[s], quality=args.quality)
        t2 = time.perf_counter()
        if gather is not None:
            if gather.cuda:
                gather.post(segs[s], lens)
            else:
                gather.post([segs[s][k][:n].cpu() for k, n in enumerate(lens)], lens)
        t3 = time.perf_counter()
        phase["acquire"] += t1 - t0
        phase["encode"] += t2 - t1
        phase["gather_post"] += t3 - t2
        return lens, s

    PHASE("warm-up steps (first RCCL transfers)" if gather is not None else "warm-up steps")
    for _ in range(args.warmup):
        step()
    if gather is not None:
        gather.wait()
    torch.cuda.synchronize()
    barrier(pg)
    PHASE("timed steps")
    phase.clear()
    if gather is not None:
        gather.lens_wait_s = 0.0
    cg0 = cgroup_cpu_stat()
    pc0 = process_cpu_s()
    th0 = thread_cpu() if os.environ.get("JPGE_BENCH_THREADS") else {}
    win0 = time.monotonic_ns()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lens, s_last = step()
    t1 = time.perf_counter()
    if gather is not None:
        gather.wait()
    torch.cuda.synchronize()
    barrier(pg)
    dt = time.perf_counter() - t0
    win1 = time.monotonic_ns()
    phase["final_wait"] = dt - (t1 - t0)
    cg1 = cgroup_cpu_stat()
    pcpu = (process_cpu_s() - pc0) / dt
    thread_report(th0, dt)
    dt_max = max_over_ranks(pg, dt)
    nbytes = sum_over_ranks(pg, float(sum(lens)))
    rank_cpus = all_gather_floats(pg, pcpu, world)
    if gather is not None and rank == 0:
        phase["lengths_wait"] = gather.lens_wait_s
    # verification: every frame of the last step, as rank 0 holds it, equals the
    # host-path encode of that frame (rank 0's own frames are in its output slots)
    bad = 0
    if not args.no_verify and (world == 1 or gather is not None):
        PHASE("verification")
        if rank == 0:
            for i in range(B):
                ref = enc.encode(host[i] if i in host else J.synth_rgb8(batch_seed(i), W, H), quality=args.quality)
                if i in host:
                    k = share.index(i)
                    got = segs[s_last][k][:lens[k]]
                else:
                    got = gather.frame(i).to(dev)
                if not torch.equal(got, torch.frombuffer(bytearray(ref), dtype=torch.uint8).to(dev)):
                    bad += 1
        bad = int(sum_over_ranks(pg, float(bad)))
    # per-kernel rooflines: this rank's frames through a 1-lane encoder after the timed
    # region, in the pipeline's launch shape (sets of 4 1080p frames) and one per launch
    ms_step = dt_max / args.steps * 1e3
    stages_solo = stages_solo1 = roofline = None
    solo_win = solo1_win = None
    if args.solo_batches > 0 and not args.no_kernel_events and share and rank == 0:
        PHASE("solo kernel timing")
        sfr = frames[:min(len(frames), 32)]
        sout = outd[0][:len(sfr)]
        fset = max(1, min(4, (4 * 3840 * 2160) // (W * H)))
        tm_solo, solo_win = solo_timing(J, local, sfr, sout, args, fset)
        tm_solo1, solo1_win = solo_timing(J, local, sfr, sout, args, 1)
        rbs = [record_bytes(enc.symbol_stats(host[i], quality=args.quality)[0]) for i in share[:len(sfr)]]
        avg_jpeg_rank = sum(lens) / max(1, len(lens))
        alg, stage_alg = alg_bytes(W * H, 3.0, sum(rbs) / len(rbs), avg_jpeg_rank)
        traffic = load_pmc_traffic(os.path.join(ROOT, "profiles"), W, H)
        stages_solo = kernel_rooflines(tm_solo, alg, stage_alg, traffic, W * H)
        stages_solo1 = kernel_rooflines(tm_solo1, alg, stage_alg, traffic, W * H)
        roofline = solo_headline(stages_solo, alg, len(share), ms_step)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, _ = oracle_cpu_baseline(args, lambda i: host[i] if i in host else J.synth_rgb8(batch_seed(i), W, H),
                                     f"{W}x{H} 4:2:0 Q{args.quality} frames of the batch (seeds 1000..)",
                                     REF_CPU_1080_Q90 if args.quality == 90 else None)
    if rank == 0:
        line = {
            "metric": f"MPixels/s encode (batch of {B} x 1920x1080 4:2:0 Q={args.quality})",
            "value": round(W * H * B * args.steps / dt_max / 1e6, 1), "unit": "MPix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (deterministic splitmix64 photo-like frames, seeds 1000+i, HBM-resident)",
            "config": {"workload": f"config 4: {B} x {W}x{H} 4:2:0 Q{args.quality} per step, frame i on rank i mod "
                                   f"{world}" + (f", each rank's .jpg bytes packed and moved to rank 0 in one transfer "
                                                 f"({GATHER_NAMES.get(transport, transport)}), overlapped with the "
                                                 f"next step's encode" if world > 1 else ""),
                       "batch": B, "width": W, "height": H, "quality": args.quality,
                       "avg_jpeg_bytes": int(nbytes / B), "parallelism": f"frames dealt over {world} GPU(s)"},
            "verified": None if args.no_verify else {
                "frames": B, "mismatches": bad,
                "method": "every frame of the last step, as gathered on rank 0, byte-compared with the host-path "
                          "encode of the same frame"},
            "host_cpu": host_cpu_use(cg0, cg1, dt, world),
            "rank_cpus": [round(c, 2) for c in rank_cpus],
            "rank0_phases_ms_per_step": {k: round(v / args.steps * 1e3, 3) for k, v in phase.items()},
            "lanes_per_rank": enc.lanes(),
            "devices": args.devices,
            # the dominant kernel alone (rank 0's frames; exclusive time, checked against the step)
            "roofline": roofline,
            "roofline_dct_stage": dict(kernel="fdct_kernel", timing="solo", **stages_solo["fdct_kernel"])
            if stages_solo else None,
            "stages_solo": stages_solo,
            "stages_solo_single_frame": stages_solo1,
            "windows_monotonic_ns": {"timed": [win0, win1], "solo": solo_win, "solo_single": solo1_win},
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    enc.close()
    if bad:
        raise SystemExit(f"batch1080: {bad} frames differ from the host-path encode")


def run_frames(args, rank, local, world, pg):
    """The BASELINE metric: 4K frames, F per GPU per step over D distinct inputs."""
    import torch

    import jpgenc_amd as J

    local = device_for(local)
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"
    enc = J.Encoder(local, lanes=rank_lanes(args, world))
    enc.set_subsampling(args.subsampling)
    W, H = args.width, args.height
    F = args.frames or 3072
    D = max(1, min(args.distinct, F))
    pitch = W * 3
    cap = out_capacity(J, W, H)
    # HBM-resident input ring and output slots (torch = device-memory plumbing)
    PHASE("setup (frames, encoder)")
    host = [J.synth_rgb8(frame_seed(rank, i), W, H) for i in range(D)]
    ins = [torch.from_numpy(h.reshape(-1)).to(dev) for h in host]
    outbuf = torch.empty(F * cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    frames = [(ins[i % D].data_ptr(), W, H, pitch) for i in range(F)]
    outd = [(outbuf.data_ptr() + i * cap, cap) for i in range(F)]

    PHASE("warm-up steps")
    for _ in range(args.warmup):
        enc.encode_batch_dev(frames, outd, quality=args.quality)
    torch.cuda.synchronize()

    PHASE("timed steps")
    enc.set_timing(0 if args.no_kernel_events else args.event_every)
    enc.reset_timing()
    barrier(pg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    win0 = time.monotonic_ns()
    total_bytes = 0
    step_t = []
    cg0 = cgroup_cpu_stat()
    pc0 = process_cpu_s()
    th0 = thread_cpu() if os.environ.get("JPGE_BENCH_THREADS") else {}
    sampler = ThreadSampler() if os.environ.get("JPGE_BENCH_THREADS") == "2" else None
    for _ in range(args.steps):
        ts = time.perf_counter()
        lens = enc.encode_batch_dev(frames, outd, quality=args.quality)
        step_t.append(time.perf_counter() - ts)  # (encode_batch returns with every byte in place)
        total_bytes += sum(lens)
    torch.cuda.synchronize()
    barrier(pg)
    dt = time.perf_counter() - t0
    win1 = time.monotonic_ns()
    cg1 = cgroup_cpu_stat()
    rank_cpus = all_gather_floats(pg, (process_cpu_s() - pc0) / dt, world)
    if sampler:
        sampler.stop()
    thread_report(th0, dt)
    tm = enc.timing()
    enc.set_timing(False)

    dt_max = max_over_ranks(pg, dt)
    pixels = sum_over_ranks(pg, float(W * H * F * args.steps))
    value = pixels / dt_max / 1e6

    # Verification (after timing): every output slot of the last timed step equals
    # the host-path encode of its input frame (byte compare on the device).
    verified = None
    refs = {}
    if not args.no_verify:
        PHASE("verification")
        for d in range(D):
            refs[d] = enc.encode(host[d], quality=args.quality)
        bad = 0
        ref_dev = [torch.frombuffer(bytearray(refs[d]), dtype=torch.uint8).to(dev) for d in range(D)]
        for i in range(F):
            r = ref_dev[i % D]
            if lens[i] != r.numel() or not torch.equal(outbuf[i * cap:i * cap + lens[i]], r):
                bad += 1
        del ref_dev
        verified = {"frames": F, "distinct_inputs": D, "mismatches": bad,
                    "method": "every output of the last timed step byte-compared (on the device) with the "
                              "host-path encode of its input frame"}
        if bad:
            raise SystemExit(f"bench: {bad} of {F} outputs differ from the host-path encode")

    # D2H-inclusive pass (device RGB -> .jpg bytes in host memory): the
    # D distinct frames per step, outputs copied into pinned host buffers.
    d2h = None
    if args.d2h_steps > 0:
        PHASE("d2h pass")
        hostout = torch.empty(D * cap, dtype=torch.uint8, pin_memory=True)
        hfr = frames[:D]
        hout = [(hostout.data_ptr() + i * cap, cap) for i in range(D)]
        enc.encode_batch_dev(hfr, hout, quality=args.quality, flags=J.JPGE_DEVICE_INPUT)
        barrier(pg)
        t1 = time.perf_counter()
        for _ in range(args.d2h_steps):
            hl = enc.encode_batch_dev(hfr, hout, quality=args.quality, flags=J.JPGE_DEVICE_INPUT)
        d2 = max_over_ranks(pg, time.perf_counter() - t1)
        d2h_ok = all(hostout[i * cap:i * cap + hl[i]].numpy().tobytes() == refs[i] for i in range(D)) if refs else None
        d2h = {"value": round(sum_over_ranks(pg, float(W * H * D * args.d2h_steps)) / d2 / 1e6, 1), "unit": "MPix/s",
               "frames_per_step_per_gpu": D, "steps": args.d2h_steps, "bytes_match": d2h_ok,
               "what": "device-resident RGB -> finished .jpg bytes in pinned host memory (D2H inside the step)"}
        del hostout

    # Solo pass (after the timed region, not part of `value`): the distinct frames
    # through a single-lane encoder with events around every frame's kernels, so each
    # kernel's duration is its own, without other lanes' kernels beside it.
    # Two solo passes: launches as the pipeline makes them (frame sets of `set_size`
    # frames, encoder.cpp batch_set_size; the headline roofline) and one frame per launch.
    tm_solo = tm_solo1 = None
    solo_win = solo1_win = None
    set_size = max(1, min(4, (4 * 3840 * 2160) // (W * H))) if D >= 2 else 1
    # (rank 0 only: the other ranks' kernels would share its GPU in a shared-GPU rehearsal)
    if args.solo_batches > 0 and not args.no_kernel_events and rank == 0:
        PHASE("solo kernel timing")
        tm_solo, solo_win = solo_timing(J, local, frames[:D], outd[:D], args, set_size)
        tm_solo1, solo1_win = solo_timing(J, local, frames[:D], outd[:D], args, 1) if set_size > 1 else (tm_solo, solo_win)

    # Single-image latency on the drop-in path (main.cpp:29 -> Image::writeJPEG, one image
    # per call): jpge_encode_rgb8 on a 1-lane context, one frame per call, wall time per
    # call; device-in/device-out and pinned host-in/host-out (PCIe copies inside the call)
    latency = None
    if args.latency_calls > 0 and rank == 0:
        PHASE("latency calls")
        lat = J.Encoder(local, lanes=1)
        lat.set_subsampling(args.subsampling)
        hin = [torch.from_numpy(host[d].reshape(-1)).pin_memory() for d in range(min(D, 8))]
        hout = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
        dout = torch.empty(cap, dtype=torch.uint8, device=dev)  # (not an output slot: those are verified below)

        def series(call):
            for i in range(8):
                call(i)
            ts = []
            for i in range(args.latency_calls):
                t = time.perf_counter()
                call(i)
                ts.append((time.perf_counter() - t) * 1e3)
            ts.sort()
            return {"median_ms": round(ts[len(ts) // 2], 4), "p99_ms": round(ts[min(len(ts) - 1, int(0.99 * len(ts)))], 4),
                    "min_ms": round(ts[0], 4), "calls": len(ts)}

        latency = {
            "device_in_device_out": series(lambda i: lat.encode_ptr(frames[i % D][0], W, H, pitch, dout.data_ptr(), cap,
                                                                    quality=args.quality)),
            "host_in_host_out": series(lambda i: lat.encode_ptr(hin[i % len(hin)].data_ptr(), W, H, pitch,
                                                                hout.data_ptr(), cap, quality=args.quality, flags=0)),
            "what": f"one {W}x{H} frame per jpge_encode_rgb8 call on a 1-lane context (the reference's one image per "
                    f"writeJPEG call), wall time per call; host buffers pinned",
        }
        lat.close()
        del hin, hout, dout

    # per-kernel rooflines (HBM-bound integer/fp64 work; algorithmic bytes per launch)
    npx = W * H
    avg_jpeg = total_bytes / (args.steps * F)
    traffic = load_pmc_traffic(os.path.join(ROOT, "profiles"), W, H) if args.subsampling == 420 else {}
    yh, yv = J.SUBSAMPLING[args.subsampling]
    cb = 2.0 * 64 * (yh * yv + 2) / (64 * yh * yv)  # int16 coefficient bytes per pixel (4:2:0: 3)
    # symbol records (record_bytes): written by K2, read by K3; per frame from every
    # distinct input's histograms (whether or not a pass sampled it), averaged over the
    # step's frames (frame i = input i mod D)
    rbs = [record_bytes(enc.symbol_stats(host[d], quality=args.quality)[0]) for d in range(D)] if rank == 0 else [0.0]
    rec_bytes = sum(rbs[i % len(rbs)] for i in range(F)) / F
    alg, stage_alg = alg_bytes(npx, cb, rec_bytes, avg_jpeg)

    stages = kernel_rooflines(tm, alg, stage_alg, traffic, npx)  # in situ (lanes overlap: diagnostic)
    stages_solo = kernel_rooflines(tm_solo, alg, stage_alg, traffic, npx) if tm_solo else None
    stages_solo1 = kernel_rooflines(tm_solo1, alg, stage_alg, traffic, npx) if tm_solo1 else None
    ms_step = dt_max / args.steps * 1e3
    # The headline roofline: the dominant kernel (longest exclusive time) ALONE on the GPU
    # (the solo pass), its duration from events bound to its own dispatch, so the figure
    # can be recomputed from a rocprofv3 kernel trace.  In the timed region four lanes'
    # kernels overlap, so an in-situ duration is wall time shared with the other lanes.
    roofline = None
    if stages_solo:
        roofline = solo_headline(stages_solo, alg, F, ms_step)
    elif stages["fdct_kernel"]["avg_kernel_ms"]:
        # no solo pass (--solo-batches 0): the in-situ figure, labelled as such (lanes
        # overlap, so it is shared wall time and carries no per-step check)
        dominant = max(alg, key=lambda k: stages[k]["avg_kernel_ms"] or 0.0)
        roofline = dict(kernel=dominant, timing="in situ (4 lanes overlap: shared wall time, not exclusive; "
                                                "run with --solo-batches > 0 for the exclusive figure)",
                        **stages[dominant])
    # whole pipeline: every kernel's algorithmic bytes per frame, over the wall time
    pipe_bytes = sum(b for b, _ in alg.values())
    pipe_ach = pipe_bytes * F * args.steps * world / dt_max / 1e9
    pipeline = {"bound": "hbm", "achieved": round(pipe_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(pipe_ach / HBM_PEAK_GBS, 4), "alg_bytes_per_frame": int(pipe_bytes),
                "note": "sum of the kernels' algorithmic bytes per frame x frames / wall time (per GPU)"}

    if rank == 0:
        line = {
            "metric": f"MPixels/s encode ({'4K' if (W, H) == (W4K, H4K) else f'{W}x{H}'} {sub_name(args)} Q={args.quality})",
            "value": round(value, 1),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic splitmix64 photo-like frames, HBM-resident)",
            "config": {
                "workload": f"{W}x{H} {sub_name(args)} Q{args.quality} full encode (RGB8 in HBM -> .jpg bytes in HBM), "
                            f"{F} frames per GPU per step over {D} distinct inputs",
                "width": W, "height": H, "quality": args.quality, "subsampling": sub_name(args),
                "frames_per_step_per_gpu": F, "distinct_inputs_per_gpu": D,
                "parallelism": f"frames sharded over {world} GPU(s), no data-path collective",
                "avg_jpeg_bytes": int(avg_jpeg),
            },
            # dominant kernel alone (exclusive time; see above)
            "roofline": roofline,
            # BASELINE.json's "% HBM roofline on DCT stage" (6 B/px; read-only 3 B/px): the kernel alone
            "roofline_dct_stage": dict(kernel="fdct_kernel", timing="solo", **stages_solo["fdct_kernel"])
            if stages_solo else dict(kernel="fdct_kernel", timing="in situ", **stages["fdct_kernel"]),
            "roofline_pipeline": pipeline,
            "stages": stages,
            "stages_solo": stages_solo,
            "stages_solo_single_frame": stages_solo1,
            "kernel_events": f"each kernel launch of a sampled frame (set) launched with its own HIP events bound "
                             f"to its dispatch (hipExtLaunchKernel); figures per launch, a frame set's launch "
                             f"covering frames_per_launch frames. stages: in situ, the set of every "
                             f"{args.event_every}th frame in the timed region (4 lanes overlap: a diagnostic, not "
                             f"exclusive time); stages_solo: every launch of {args.solo_batches} batches of {D} on a "
                             f"1-lane encoder after the timed region, in the pipeline's frame sets of {set_size}; "
                             f"stages_solo_single_frame: the same, one frame per launch",
            "step_ms": {"min": round(min(step_t) * 1e3, 3), "median": round(sorted(step_t)[len(step_t) // 2] * 1e3, 3),
                        "max": round(max(step_t) * 1e3, 3)},
            "lanes": enc.lanes(),
            "verified": verified,
            "d2h": d2h,
            "latency": latency,
            # CLOCK_MONOTONIC windows (rocprofv3 timestamps use the same clock): tools/rocprof_window.py
            "windows_monotonic_ns": {"timed": [win0, win1], "solo": solo_win, "solo_single": solo1_win},
            # host CPU use over the timed region; quota throttling stalls the pipeline
            "host_cpu": host_cpu_use(cg0, cg1, dt, world),
            "rank_cpus": [round(c, 2) for c in rank_cpus],
            "devices": args.devices,
        }
        if world == 1 and not args.no_cpu_baseline:
            cpu, hashes = cpu_baseline(args)
            if verified is not None and args.subsampling == 420:
                # the oracle's bytes of the sampled frames against the GPU's (slot i = input i)
                ok = sum(hashlib.sha256(outbuf[i * cap:i * cap + lens[i]].cpu().numpy().tobytes()).hexdigest() == h
                         for i, h in hashes.items() if i < D)
                verified["vs_oracle"] = f"{ok}/{sum(1 for i in hashes if i < D)} sampled frames equal the CPU oracle"
                if ok != sum(1 for i in hashes if i < D):
                    raise SystemExit("bench: GPU output differs from the CPU oracle")
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    enc.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        device_plan(args.gpus, args.allow_shared_gpu)  # refuse before starting any rank
        sys.exit(spawn(args.gpus, argv))  # (the parent never touches a GPU)
    global PHASE
    PHASE = PhaseWatch(args.phase_timeout)
    rank, local, world, pg = dist_setup(args.gpus, args)
    args.devices = device_plan(world, args.allow_shared_gpu)
    run = {"4k-frames": run_frames, "batch1080": run_batch1080, "16k-striped": run_striped16k,
           "ppm-files": run_ppm_files, "dist-check": run_dist_check}[args.workload]
    try:
        run(args, rank, local, world, pg)
    finally:
        if pg is not None:
            pg.destroy_process_group()


if __name__ == "__main__":
    main()
