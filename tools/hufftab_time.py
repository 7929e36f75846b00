"""Device table build latency (run under rocprofv3 --kernel-trace): one histogram set
(a frame's four tables) per launch, for a few frame kinds; the kernel trace gives
each launch's duration."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import _oracle  # noqa: E402

import jpgenc_amd as J  # noqa: E402

for seed, (w, h), q, kind in [(3, (3840, 2160), 90, 0), (4, (1920, 1080), 90, 1), (5, (1920, 1080), 100, 1)]:
    c, f = _oracle.stage_hist(J.synth_rgb8(seed, w, h, kind), q)
    print(w, h, q, kind, "symbols per table", [(int((c[t] > 0).sum())) for t in range(4)], flush=True)
    for _ in range(5):
        J.huffman_tables_device(c[None], f[None])
