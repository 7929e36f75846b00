"""jpge benchmark — BASELINE.json metric: MPixels/s encode (4K 4:2:0 Q=90).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--quality Q]

A step = one pass of the full encode path (RGB8 in HBM -> finished .jpg bytes in
HBM: colour/4:2:0/FDCT/quantise + statistics kernels, host Huffman-table build,
entropy+stuffing kernel) over a batch of F distinct synthetic 3840x2160 frames
resident in HBM (F=16 by default: 16 x 24.9 MB > the 256 MB Infinity Cache, so
the colour/DCT stage reads from HBM).  Frames are independent, so with N GPUs
each rank encodes its own F frames (weak scaling, no data-path collective);
the gloo process group only provides the barriers and the max-over-ranks time.

Prints ONE JSON line (rank 0).  `roofline` is the dominant kernel (largest
HIP-event time per frame on its own stream inside the timed region); `stages`
carries all three kernels, each with its algorithmic bytes per launch:
  fdct_kernel    RGB8 read 3 B/px + int16 coefficients written 3 B/px
  stats_kernel   coefficients read 3 B/px
  entropy_kernel coefficients read 3 B/px + entropy-coded bytes written
`traffic` = HBM bytes per launch from the committed rocprofv3 PMC summary
(profiles/pmc_r01.json, FETCH_SIZE doubled on gfx950).  The CPU baseline is the
test-only oracle on the host cores, rank 0 at N=1.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W4K, H4K = 3840, 2160
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


# subsampling modes (jpge.h JPGE_S*) -> the name in the metric / workload
SUB_NAMES = {420: "4:2:0", 444: "4:4:4", 422: "4:2:2", 411: "4:1:1", 4200: "4:2:0 S420", 4201: "4:2:0 S420_lm"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--width", type=int, default=W4K)
    ap.add_argument("--height", type=int, default=H4K)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--solo-batches", type=int, default=2,
                    help="batches through a 1-lane encoder after the timed region (kernel times alone; 0 = skip)")
    ap.add_argument("--lanes", type=int, default=0, help="encoder lanes (0 = library default)")
    ap.add_argument("--workload", choices=["4k-frames", "16k-striped", "ppm-files"], default="4k-frames",
                    help="4k-frames: the BASELINE metric (frames sharded over ranks); 16k-striped: one "
                         "16384x16384 frame per step, row-striped over the ranks (SURVEY 8(e) config 5); "
                         "ppm-files: PPM files -> .jpg files through the ingest pipeline (PCIe-inclusive)")
    ap.add_argument("--restart", type=int, default=None,
                    help="restart interval in MCUs (16k-striped: default 1024 = one interval per MCU row, "
                         "the config's 'tiled with restart intervals'; 0 = the reference's single interval)")
    ap.add_argument("--subsampling", type=int, choices=sorted(SUB_NAMES), default=420,
                    help="4k-frames: subsampling mode (jpge.h JPGE_S*: 420 = the reference's S420_m; "
                         "444, 422, 411, 4200 = S420, 4201 = S420_lm are extensions)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-kernel-events", action="store_true", help="diagnostic: time without per-kernel events")
    ap.add_argument("--event-every", type=int, default=4,
                    help="bracket the kernels of every N-th frame with HIP events (each event costs GPU time)")
    return ap.parse_args()


def dist_setup(n_gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist
    return rank, local, world, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


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


def frame_seed(rank: int, i: int) -> int:
    return 3 + 1000 * rank + i  # config 3 seed family, distinct per rank and frame


def cpu_baseline(args) -> dict:
    """The test-only oracle (CPU restatement of the reference path) on a bounded
    sample of the same workload: whole 4K Q90 frames until ~cpu_seconds."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle  # noqa: E402
    import jpgenc_amd as J

    threads = min(16, os.cpu_count() or 1)
    _oracle.orc().orc_set_threads(threads)
    enc_times = []  # encode-only time per frame (synthesis excluded)
    for i in range(16):
        rgb = J.synth_rgb8(frame_seed(0, i), args.width, args.height)
        s = time.perf_counter()
        _oracle.encode(rgb, args.quality, subsampling=args.subsampling)
        enc_times.append(time.perf_counter() - s)
        if sum(enc_times) >= args.cpu_seconds:
            break
    px = args.width * args.height * len(enc_times)
    return {
        "value": round(px / sum(enc_times) / 1e6, 3),
        "unit": "MPix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(enc_times)} x {args.width}x{args.height} {sub_name(args)} Q{args.quality} frames (seeds 3..), "
                  f"oracle/jpge_oracle.cpp restatement, OpenMP {threads} threads (DCT/quant parallel, "
                  f"like the reference)",
    }


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


def load_pmc_traffic(profile_dir: str, width: int, height: int) -> dict:
    """Per-launch HBM bytes per stage from the committed rocprofv3 PMC summary (the
    entropy stage = its code, placement-scan and pack kernels)."""
    try:
        with open(os.path.join(profile_dir, "pmc_r01.json")) as f:
            d = json.load(f)
        if d.get("width") != width or d.get("height") != height:
            return {}
        per = {k.split("<")[0]: v["hbm_bytes_per_launch"] for k, v in d["kernels"].items()}
    except (OSError, ValueError, KeyError):
        return {}
    out = {k: v for k, v in per.items() if not k.startswith("entropy_")}
    ent = [v for k, v in per.items() if k.startswith("entropy_")]
    if ent:
        out["entropy_kernel"] = sum(ent)
    return out


def run_striped16k(args, rank, local, world, pg):
    """One 16384^2 frame per step: whole-frame encode on one GPU; on N GPUs each
    rank holds and encodes its row stripe, with the three RCCL exchanges and the
    segment gather of SURVEY 8(e) inside the timed step (output identical to 1 GPU)."""
    import torch

    import jpgenc_amd as J
    from jpgenc_amd import stripes

    torch.cuda.set_device(local)
    W = H = 16384
    restart = 1024 if args.restart is None else args.restart
    rgb = J.synth_rgb8(5, W, H)  # SURVEY 8(d) config 5 seed
    cap = J.max_jpeg_bytes(W, H)
    out = torch.empty(cap, dtype=torch.uint8, device=f"cuda:{local}")
    if world == 1:
        enc = J.Encoder(local)
        enc.set_restart(restart)
        src = torch.from_numpy(rgb.reshape(-1)).to(f"cuda:{local}")
        del rgb

        def step():
            return enc.encode_batch_dev([(src.data_ptr(), W, H, W * 3)], [(out.data_ptr(), cap)],
                                        quality=args.quality)[0]
    else:
        import torch.distributed as dist

        rccl = dist.new_group(backend="nccl")  # the exchanges and the gather ride RCCL over xGMI
        r0, nr = stripes.stripe_rows(H // 16, world, stripes.restart_align(W, restart))[rank]
        src = torch.from_numpy(np.ascontiguousarray(rgb[16 * r0:16 * (r0 + nr)]).reshape(-1)).to(f"cuda:{local}")
        del rgb
        enc = J.Encoder(local, lanes=1)
        enc.set_restart(restart)

        def step():
            return stripes.encode_stripe_dist(enc, src.data_ptr(), W * 3, W, H, args.quality, out, group=rccl,
                                              restart=restart)
    for _ in range(args.warmup):
        n = step()
    torch.cuda.synchronize()
    barrier(pg)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n = step()
    torch.cuda.synchronize()
    barrier(pg)
    dt = max_over_ranks(pg, time.perf_counter() - t0)
    if rank == 0:
        print(json.dumps({
            "metric": "MPixels/s encode (16K 4:2:0 Q=90)",
            "value": round(W * H * args.steps / dt / 1e6, 1), "unit": "MPix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
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
        }), flush=True)
    enc.close()


def run_ppm_files(args, rank, local, world, pg):
    """F synthetic P6 files (in /dev/shm, i.e. the page cache) ->
    .jpg files per step through jpge_encode_files: file read + parse into pinned
    memory, H2D, kernels, D2H and file write all inside the timed step."""
    import shutil
    import tempfile

    import torch

    import jpgenc_amd as J

    torch.cuda.set_device(local)
    W, H, F = args.width, args.height, args.frames
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
            }), flush=True)
        enc.close()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    args = parse()
    rank, local, world, pg = dist_setup(args.gpus)
    if args.workload == "ppm-files":
        run_ppm_files(args, rank, local, world, pg)
        if pg is not None:
            pg.destroy_process_group()
        return
    if args.workload == "16k-striped":
        run_striped16k(args, rank, local, world, pg)
        if pg is not None:
            pg.destroy_process_group()
        return
    import torch

    import jpgenc_amd as J

    torch.cuda.set_device(local)
    enc = J.Encoder(local, lanes=args.lanes)
    enc.set_subsampling(args.subsampling)
    W, H, F = args.width, args.height, args.frames
    pitch = W * 3
    cap = J.max_jpeg_bytes(W, H)
    # HBM-resident input ring and output buffers (torch = device-memory plumbing)
    ins = []
    for i in range(F):
        host = J.synth_rgb8(frame_seed(rank, i), W, H)
        ins.append(torch.from_numpy(host.reshape(-1)).to(f"cuda:{local}"))
    outs = [torch.empty(cap, dtype=torch.uint8, device=f"cuda:{local}") for _ in range(F)]
    torch.cuda.synchronize()
    frames = [(t.data_ptr(), W, H, pitch) for t in ins]
    outd = [(o.data_ptr(), cap) for o in outs]

    # correctness guard on the timed configuration: the first frame must match the
    # host-path encode (which the parity tests pin to the oracle)
    lens = enc.encode_batch_dev(frames[:1], outd[:1], quality=args.quality)
    dev_bytes = outs[0][: lens[0]].cpu().numpy().tobytes()
    if dev_bytes != enc.encode(J.synth_rgb8(frame_seed(rank, 0), W, H), quality=args.quality):
        raise RuntimeError("device-resident path differs from the host path")

    for _ in range(args.warmup):
        enc.encode_batch_dev(frames, outd, quality=args.quality)
    torch.cuda.synchronize()

    enc.set_timing(0 if args.no_kernel_events else args.event_every)
    enc.reset_timing()
    barrier(pg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    win0 = time.monotonic_ns()
    total_bytes = 0
    step_t = []
    cg0 = cgroup_cpu_stat()
    th0 = thread_cpu() if os.environ.get("JPGE_BENCH_THREADS") else {}
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
    if th0:
        th1 = thread_cpu()
        use = collections.Counter()
        for k, v in th1.items():
            use[k] += (v - th0.get(k, 0.0)) / dt
        print(f"threads: {len(th1)}; busiest:", {f"{k[1]}/{k[0]}": round(v, 2) for k, v in use.most_common(24)},
              file=sys.stderr)
    tm = enc.timing()
    enc.set_timing(False)

    dt_max = max_over_ranks(pg, dt)
    pixels = sum_over_ranks(pg, float(W * H * F * args.steps))
    value = pixels / dt_max / 1e6

    # Solo pass (after the timed region, not part of `value`): the same frames through
    # a single-lane encoder with events around every frame's kernels, so each kernel's
    # duration is its own, without other lanes' kernels beside it.
    tm_solo = None
    solo_win = None
    if args.solo_batches > 0 and not args.no_kernel_events:
        solo = J.Encoder(local, lanes=1)
        solo.set_subsampling(args.subsampling)
        solo.encode_batch_dev(frames, outd, quality=args.quality)
        solo.set_timing(1)
        solo.reset_timing()
        s0 = time.monotonic_ns()
        for _ in range(args.solo_batches):
            solo.encode_batch_dev(frames, outd, quality=args.quality)
        solo_win = [s0, time.monotonic_ns()]
        tm_solo = solo.timing()
        solo.close()

    # per-kernel rooflines (HBM-bound integer/fp64 work; algorithmic bytes per launch)
    npx = W * H
    avg_jpeg = total_bytes / (args.steps * F)
    traffic = load_pmc_traffic(os.path.join(ROOT, "profiles"), W, H) if args.subsampling == 420 else {}
    yh, yv = J.SUBSAMPLING[args.subsampling]
    cb = 2.0 * 64 * (yh * yv + 2) / (64 * yh * yv)  # int16 coefficient bytes per pixel (4:2:0: 3)
    alg = {
        "fdct_kernel": ((3.0 + cb) * npx, f"RGB8 read 3 B/px + int16 coefficients written {cb:g} B/px"),
        "stats_kernel": (cb * npx, f"coefficients read {cb:g} B/px"),
        "entropy_kernel": (cb * npx + avg_jpeg, f"coefficients read {cb:g} B/px + entropy-coded bytes written"),
    }

    def rooflines(tm):
        nfr = max(1, tm["frames"])
        ms = {"fdct_kernel": tm["fdct_sum"] / nfr, "stats_kernel": tm["dc_stats_sum"] / nfr,
              "entropy_kernel": tm["entropy_sum"] / nfr}
        out = {}
        for name, (b, what) in alg.items():
            ach = b / (ms[name] * 1e-3) / 1e9 if ms[name] > 0 else 0.0  # (0: --no-kernel-events)
            out[name] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic.get(name),
                         "alg_bytes_per_launch": int(b), "alg_bytes": what, "avg_kernel_ms": round(ms[name], 5),
                         "timed_launches": tm["frames"]}
        return out

    stages = rooflines(tm)  # in situ: the timed region, lanes side by side
    stages_solo = rooflines(tm_solo) if tm_solo else None
    dominant = max(stages, key=lambda k: stages[k]["avg_kernel_ms"])
    # whole pipeline: every kernel's algorithmic bytes per frame, over the wall time
    pipe_bytes = sum(b for b, _ in alg.values())
    pipe_ach = pipe_bytes * F * args.steps * world / dt_max / 1e9
    pipeline = {"bound": "hbm", "achieved": round(pipe_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(pipe_ach / HBM_PEAK_GBS, 4), "alg_bytes_per_frame": int(pipe_bytes),
                "note": "sum of the kernels' algorithmic bytes per frame x frames / wall time (per GPU)"}

    if rank == 0:
        line = {
            "metric": f"MPixels/s encode (4K {sub_name(args)} Q=90)",
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
                            f"{F} distinct frames per GPU per step",
                "width": W, "height": H, "quality": args.quality, "subsampling": sub_name(args),
                "frames_per_step_per_gpu": F,
                "parallelism": f"frames sharded over {world} GPU(s), no data-path collective",
                "avg_jpeg_bytes": int(total_bytes / (args.steps * F)),
            },
            # dominant kernel, timed in situ (HIP events on its lane's stream, lanes side by side)
            "roofline": dict(kernel=dominant, timing="in situ", **stages[dominant]),
            # BASELINE.json's "% HBM roofline on DCT stage" (6 B/px): the kernel alone
            "roofline_dct_stage": dict(kernel="fdct_kernel", timing="solo", **stages_solo["fdct_kernel"])
            if stages_solo else dict(kernel="fdct_kernel", timing="in situ", **stages["fdct_kernel"]),
            "roofline_pipeline": pipeline,
            "stages": stages,
            "stages_solo": stages_solo,
            "kernel_events": f"in situ: HIP events around every {args.event_every}th frame's kernels on its lane's "
                             f"stream; solo: every frame of {args.solo_batches} batches on a 1-lane encoder after "
                             f"the timed region",
            "step_ms": {"min": round(min(step_t) * 1e3, 3), "median": round(sorted(step_t)[len(step_t) // 2] * 1e3, 3),
                        "max": round(max(step_t) * 1e3, 3)},
            "lanes": enc.lanes(),
            # CLOCK_MONOTONIC windows (rocprofv3 timestamps use the same clock): tools/rocprof_window.py
            "windows_monotonic_ns": {"timed": [win0, win1], "solo": solo_win},
            # host CPU use over the timed region; quota throttling stalls the pipeline
            "host_cpu": {"cpus_used": round((cg1.get("usage_usec", 0) - cg0.get("usage_usec", 0)) / 1e6 / dt, 2),
                         "throttled_periods": cg1.get("nr_throttled", 0) - cg0.get("nr_throttled", 0),
                         "throttled_ms": round((cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0)) / 1e3,
                                               1)} if cg0 else None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(line), flush=True)
    enc.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
