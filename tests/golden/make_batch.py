"""Golden SHA-256 + length of every frame of BASELINE config 4 (a batch of 256
synthetic 1920x1080 frames, 4:2:0 Q90, seeds 1000+i), made by the
TEST-ONLY oracle (oracle/jpge_oracle.cpp restatement) in this container.  Writes
tests/golden/batch1080.json; tests/test_gpu_configs.py checks every frame the GPU
batch path produces against it.

    python tests/golden/make_batch.py
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import _oracle  # noqa: E402
import jpgenc_amd as J  # noqa: E402

W, H, Q, B, SEED0 = 1920, 1080, 90, 256, 1000


def main():
    _oracle.orc().orc_set_threads(os.cpu_count() or 1)
    t = time.time()
    frames = []
    for i in range(B):
        jpg = _oracle.encode(J.synth_rgb8(SEED0 + i, W, H), Q)
        frames.append([len(jpg), hashlib.sha256(jpg).hexdigest()])
    print(f"{B} frames in {time.time() - t:.1f} s", flush=True)
    with open(os.path.join(HERE, "batch1080.json"), "w") as f:
        json.dump({"generator": "oracle/jpge_oracle.cpp via tests/_oracle.encode; frames from jpge_synth_rgb8",
                   "width": W, "height": H, "quality": Q, "seed0": SEED0, "frames": frames}, f, indent=0)


if __name__ == "__main__":
    main()
