import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'tests'))
import numpy as np, torch
import jpgenc_amd as J, _oracle
from jpgenc_amd import stripes
def run(w, h, n, kind, q):
    rgb = J.synth_rgb8(77 + n + kind, w, h, kind=kind)
    dev = torch.from_numpy(rgb.reshape(-1)).cuda()
    stride = w * 3
    rows = stripes.stripe_rows((h + 15) // 16, n)
    encs = [J.Encoder(0, lanes=1) for _ in range(n)]
    last = [encs[r].stripe_transform(dev.data_ptr() + rows[r][0] * 16 * stride, stride, w, h, rows[r][0], rows[r][1], q) for r in range(n)]
    st = [encs[r].stripe_stats(stripes.seeds_from(last, r)) for r in range(n)]
    counts, first = stripes.combine_stats([s[0] for s in st], [s[1] for s in st])
    codes = [encs[r].stripe_code(counts, first) for r in range(n)]
    summ = [c[0] for c in codes]
    cap = J.max_jpeg_bytes(w, h)
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    res = []
    for r in range(n):
        try:
            res.append(encs[r].stripe_pack(summ, r, out.data_ptr(), cap))
        except Exception as e:
            res.append(str(e))
    tot = res[-1][2] if isinstance(res[-1], tuple) else 0
    ok = tot and out[:tot].cpu().numpy().tobytes() == _oracle.encode(rgb, q)
    print(w, h, n, "ok" if ok else "BAD", "last", [l.tolist() for l in last], "summ", [(s[0], s[2], s[3], s[4]) for s in summ], res)
    for e in encs: e.close()
for i in range(3):
    run(33, 17, 2, 0, 90)
    run(640, 48, 3, 1, 100)
    run(512, 512, 2, 0, 90)
