"""Single-frame profiling loop (no cross-frame overlap): encodes one HBM-resident
frame `--iters` times through the batch API with a batch of 1, and prints the
per-kernel HIP-event times.  Used under rocprofv3 for kernel traces / PMC."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402  (device-memory plumbing)

import jpgenc_amd as J  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--quality", type=int, default=90)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--kind", type=int, default=0)
ap.add_argument("--frames", type=int, default=1, help="distinct HBM-resident frames, encoded in turn")
ap.add_argument("--subsampling", type=int, default=420, choices=[420, 444])
a = ap.parse_args()

enc = J.Encoder(0)
enc.set_subsampling(a.subsampling)
devs = [torch.from_numpy(J.synth_rgb8(3 + i, a.width, a.height, a.kind).reshape(-1)).cuda() for i in range(a.frames)]
cap = J.max_jpeg_bytes(a.width, a.height)
out = torch.empty(cap, dtype=torch.uint8, device="cuda")
allframes = [[(d.data_ptr(), a.width, a.height, a.width * 3)] for d in devs]
outs = [(out.data_ptr(), cap)]
enc.encode_batch_dev(allframes[0], outs, quality=a.quality)
enc.set_timing(True)
enc.reset_timing()
for it in range(a.iters):
    n = enc.encode_batch_dev(allframes[it % a.frames], outs, quality=a.quality)
t = enc.timing()
f = max(1, t["frames"])
print(f"{a.width}x{a.height} Q{a.quality} kind{a.kind}: {n[0]} bytes; fdct {t['fdct_sum']/f*1e3:.1f} us, "
      f"dc {t['dc_stats_sum']/f*1e3:.1f} us, entropy {t['entropy_sum']/f*1e3:.1f} us")
enc.close()
