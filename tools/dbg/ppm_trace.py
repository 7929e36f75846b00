import os, sys, time, tempfile, shutil
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import jpgenc_amd as J
W, H, F = 3840, 2160, 16
tmp = tempfile.mkdtemp(dir="/dev/shm")
ins, outs = [], []
for i in range(F):
    p = os.path.join(tmp, f"f{i}.ppm")
    with open(p, "wb") as f:
        f.write(f"P6\n{W} {H}\n255\n".encode()); f.write(J.synth_rgb8(3 + i, W, H).tobytes())
    ins.append(p); outs.append(os.path.join(tmp, f"f{i}.jpg"))
enc = J.Encoder(0)
enc.encode_files(ins, outs, 90)
os.environ["JPGE_INGEST_TRACE"] = "1"
t = time.perf_counter(); enc.encode_files(ins, outs, 90); print("total ms", (time.perf_counter()-t)*1e3, flush=True)
rgb = J.synth_rgb8(3, W, H)
enc.encode(rgb, 90)
t = time.perf_counter()
for _ in range(5): enc.encode(rgb, 90)
print("single encode (pageable host in/out) ms", (time.perf_counter()-t)*1e3/5, flush=True)
shutil.rmtree(tmp)
