"""Probe: P independent encoder processes on ONE GPU (each its own stream and host
pipeline), started together behind a barrier; prints each process's and the
aggregate MPix/s.  Measures how much headroom concurrent frames would find.

    python tools/concurrency_probe.py --procs 2 --steps 20
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, args, bar, q):
    sys.path.insert(0, ROOT)
    import torch

    import bench
    import jpgenc_amd as J

    enc = J.Encoder(0)
    W, H, F = 3840, 2160, args.frames
    cap = J.max_jpeg_bytes(W, H)
    ins = [torch.from_numpy(J.synth_rgb8(bench.frame_seed(rank, i), W, H).reshape(-1)).cuda() for i in range(F)]
    outs = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(F)]
    frames = [(t.data_ptr(), W, H, W * 3) for t in ins]
    outd = [(o.data_ptr(), cap) for o in outs]
    for _ in range(3):
        enc.encode_batch_dev(frames, outd, quality=90)
    torch.cuda.synchronize()
    bar.wait()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        enc.encode_batch_dev(frames, outd, quality=90)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    q.put((rank, dt, W * H * F * args.steps))
    bar.wait()
    enc.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=16)
    args = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    bar, q = ctx.Barrier(args.procs), ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, args, bar, q)) for r in range(args.procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
    tmax = max(r[1] for r in res)
    for r, dt, px in sorted(res):
        print(f"proc {r}: {px / dt / 1e6:9.1f} MPix/s")
    print(f"aggregate ({args.procs} procs): {sum(r[2] for r in res) / tmax / 1e6:9.1f} MPix/s")


if __name__ == "__main__":
    main()
