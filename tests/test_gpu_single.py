"""Single images on a 1-lane context (jpge_encode_rgb8, the reference's one image per
writeJPEG call, Image.cpp:831-976).  With device output the pack kernel hands the
result over once every workgroup's write-through stores have completed, and the call
returns without waiting for the kernel's formal end (encoder.cpp encode(), entropy.hip
pack_done).  The bytes must then be readable at once from another stream: each call's
output buffer is poisoned first, read back on torch's stream right after the call and
compared with the oracle; host output and a frame too big for its buffer as well."""
import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lone():
    enc = J.Encoder(0, lanes=1)
    yield enc
    enc.close()


@pytest.mark.parametrize("w,h,q", [(3840, 2160, 90), (1920, 1080, 100), (200, 136, 50), (17, 9, 90)])
def test_device_output_readable_on_return(lone, w, h, q):
    import torch

    rgb = J.synth_rgb8(77 + w, w, h)
    want = _oracle.encode(rgb, q)
    d_in = torch.from_numpy(rgb.reshape(-1)).cuda()
    cap = J.max_jpeg_bytes(w, h)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        out.fill_(0xA5)
        torch.cuda.synchronize()
        n = lone.encode_ptr(d_in.data_ptr(), w, h, w * 3, out.data_ptr(), cap, quality=q)
        assert out[:n].cpu().numpy().tobytes() == want  # (torch's stream, no synchronisation)
    assert lone.encode(rgb, quality=q) == want  # host output on the same context


def test_device_output_too_small(lone):
    import torch

    w, h = 640, 480
    rgb = J.synth_rgb8(5, w, h, kind=1)
    d_in = torch.from_numpy(rgb.reshape(-1)).cuda()
    out = torch.empty(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(J.JpgeError):
        lone.encode_ptr(d_in.data_ptr(), w, h, w * 3, out.data_ptr(), out.numel(), quality=100)
    assert lone.encode(rgb, quality=90) == _oracle.encode(rgb, 90)  # the context still works
