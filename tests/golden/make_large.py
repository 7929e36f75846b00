"""Golden SHA-256 + length of whole-frame encodes too large to commit as bytes,
made by the TEST-ONLY oracle (oracle/jpge_oracle.cpp restatement) in this
container: 16384x16384 synthetic frame (seed 5) at Q90 and
Q50, and at Q90 with a restart interval of 1024 MCUs (one per MCU row: config 5
"tiled with restart intervals", the oracle's restart variant).  Writes
tests/golden/large_frames.json; entries already there are kept.

    python tests/golden/make_large.py
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


def main():
    _oracle.orc().orc_set_threads(os.cpu_count() or 1)
    path = os.path.join(HERE, "large_frames.json")
    out = json.load(open(path))["frames"] if os.path.exists(path) else []
    have = {(f["width"], f["height"], f["seed"], f["quality"], f.get("restart", 0)) for f in out}
    for (w, h, seed, q, rst) in [(16384, 16384, 5, 90, 0), (16384, 16384, 5, 50, 0), (16384, 16384, 5, 90, 1024)]:
        if (w, h, seed, q, rst) in have:
            continue
        rgb = J.synth_rgb8(seed, w, h)
        t = time.time()
        jpg = _oracle.encode(rgb, q, restart=rst)
        out.append({"width": w, "height": h, "seed": seed, "kind": 0, "quality": q, "len": len(jpg),
                    "sha256": hashlib.sha256(jpg).hexdigest()})
        if rst:
            out[-1]["restart"] = rst
        print(out[-1], f"{time.time() - t:.1f} s", flush=True)
        del rgb, jpg
    with open(path, "w") as f:
        json.dump({"generator": "oracle/jpge_oracle.cpp via tests/_oracle.encode; frames from jpge_synth_rgb8",
                   "frames": out}, f, indent=1)


if __name__ == "__main__":
    main()
