import os, sys, time, tempfile, shutil
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import jpgenc_amd as J
W, H, F = 3840, 2160, 32
tmp = tempfile.mkdtemp(dir="/dev/shm")
ins, outs = [], []
for i in range(F):
    p = os.path.join(tmp, f"f{i}.ppm")
    with open(p, "wb") as f:
        f.write(f"P6\n{W} {H}\n255\n".encode()); f.write(J.synth_rgb8(3 + i, W, H).tobytes())
    ins.append(p); outs.append(os.path.join(tmp, f"f{i}.jpg"))
enc = J.Encoder(0)
for g in (16, 8, 4, 2):
    enc.encode_files(ins, outs, 90, group=g)
    t = time.perf_counter()
    for _ in range(3):
        enc.encode_files(ins, outs, 90, group=g)
    dt = (time.perf_counter() - t) / 3
    print(f"group {g}: {dt*1e3:.1f} ms per {F} files = {W*H*F/dt/1e6:.0f} MPix/s, {dt/F*1e3:.2f} ms/file", flush=True)
# stage costs alone
import numpy as np
t = time.perf_counter()
for p in ins:
    with open(p, 'rb') as f: f.read()
print(f"python read of {F} files: {(time.perf_counter()-t)*1e3:.1f} ms")
shutil.rmtree(tmp)
