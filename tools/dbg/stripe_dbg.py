import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'tests'))
import numpy as np, torch
import jpgenc_amd as J
from jpgenc_amd import stripes
w = h = 512; n = 2
rgb = J.synth_rgb8(77 + n, w, h)
dev = torch.from_numpy(rgb.reshape(-1)).cuda()
stride = w * 3
rows = stripes.stripe_rows((h + 15) // 16, n)
encs = [J.Encoder(0, lanes=1) for _ in range(n)]
last = [encs[r].stripe_transform(dev.data_ptr() + rows[r][0] * 16 * stride, stride, w, h, rows[r][0], rows[r][1], 90) for r in range(n)]
st = [encs[r].stripe_stats(stripes.seeds_from(last, r)) for r in range(n)]
counts, first = stripes.combine_stats([s[0] for s in st], [s[1] for s in st])
codes = [encs[r].stripe_code(counts, first) for r in range(n)]
print("summaries", codes)
summ = [c[0] for c in codes]
for r in range(n):
    print(r, J.stripe_place(summ, r, codes[0][1]))
cap = J.max_jpeg_bytes(w, h)
out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
for r in range(n):
    try:
        print("pack", r, encs[r].stripe_pack(summ, r, out.data_ptr(), cap))
    except Exception as e:
        print("pack", r, "ERR", e)
