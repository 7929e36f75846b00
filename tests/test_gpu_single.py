"""Single images on a 1-lane context (jpge_encode_rgb8, the reference's one image per
writeJPEG call, Image.cpp:831-976).  With device output the pack kernel hands the
result over once every workgroup's write-through stores have completed, and the call
returns without waiting for the kernel's formal end (encoder.cpp encode(), entropy.hip
pack_done).  The bytes must then be readable at once from another stream: each call's
output buffer is poisoned first, read back on torch's stream right after the call and
compared with the oracle; host output and a frame too big for its buffer as well.

The tables' copy and the code kernel wait behind a stream gate the host opens once the
tables are built (encode()'s gate); a call that fails after queueing them (the header
does not fit the buffer) must still open it, and the context must keep working.  With
JPGE_GATE=0 (no gate) and 2 (the runtime's stream wait and copy instead of the library's
wait-and-copy workgroup) the same bytes come out."""
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


def test_header_does_not_fit(lone):
    import torch

    w, h = 320, 240
    rgb = J.synth_rgb8(9, w, h)
    d_in = torch.from_numpy(rgb.reshape(-1)).cuda()
    out = torch.empty(64, dtype=torch.uint8, device="cuda")  # (a header takes ~600 bytes)
    for _ in range(2):
        with pytest.raises(J.JpgeError):
            lone.encode_ptr(d_in.data_ptr(), w, h, w * 3, out.data_ptr(), out.numel(), quality=90)
    cap = J.max_jpeg_bytes(w, h)
    big = torch.empty(cap, dtype=torch.uint8, device="cuda")
    n = lone.encode_ptr(d_in.data_ptr(), w, h, w * 3, big.data_ptr(), cap, quality=90)
    assert big[:n].cpu().numpy().tobytes() == _oracle.encode(rgb, 90)


@pytest.mark.parametrize("mode", ["0", "2"])  # no gate; the runtime's stream wait
def test_gate_modes_same_bytes(monkeypatch, mode):
    monkeypatch.setenv("JPGE_GATE", mode)
    enc = J.Encoder(0, lanes=1)
    try:
        for w, h, q in [(1920, 1080, 90), (200, 136, 50)]:
            rgb = J.synth_rgb8(31 + w, w, h)
            assert enc.encode(rgb, quality=q) == _oracle.encode(rgb, q)
    finally:
        enc.close()


def test_gate_timeout_recodes(monkeypatch):
    """The gate kernel's time-out path: the device waits at
    most 300 us for the gate, the host opens it 30 ms after building the tables, so every
    call's gate times out and its code kernel runs on the previous call's tables (zeros for
    the first).  The call must notice (the gate's fail word), code the frame again behind a
    plain copy of the tables, and return the oracle's bytes; the context keeps working."""
    import torch

    monkeypatch.setenv("JPGE_TEST_GATE_TIMEOUT_US", "300")
    monkeypatch.setenv("JPGE_TEST_GATE_DELAY_US", "30000")
    enc = J.Encoder(0, lanes=1)
    monkeypatch.delenv("JPGE_TEST_GATE_TIMEOUT_US")
    monkeypatch.delenv("JPGE_TEST_GATE_DELAY_US")
    try:
        cases = [(1920, 1080, 90), (200, 136, 50), (640, 480, 100), (1920, 1080, 90)]
        for k, (w, h, q) in enumerate(cases):
            rgb = J.synth_rgb8(131 + k, w, h)
            assert enc.encode(rgb, quality=q) == _oracle.encode(rgb, q)
        w, h = 1280, 720
        rgb = J.synth_rgb8(7, w, h)
        d_in = torch.from_numpy(rgb.reshape(-1)).cuda()
        cap = J.max_jpeg_bytes(w, h)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        n = enc.encode_ptr(d_in.data_ptr(), w, h, w * 3, out.data_ptr(), cap, quality=90)
        assert out[:n].cpu().numpy().tobytes() == _oracle.encode(rgb, 90)
        # every call ran into the time-out (frames >= 1 MPix build tables with the helper
        # thread; all of them open the gate 30 ms late)
        assert enc.timing()["gate_timeouts"] == len(cases) + 1
    finally:
        enc.close()
    plain = J.Encoder(0, lanes=1)  # (no hooks: the gate opens in time)
    try:
        rgb = J.synth_rgb8(8, 1920, 1080)
        assert plain.encode(rgb, quality=90) == _oracle.encode(rgb, 90)
        assert plain.timing()["gate_timeouts"] == 0
    finally:
        plain.close()


def test_serialised_launches_skip_the_gate(monkeypatch):
    """AMD_SERIALIZE_KERNEL / HIP_LAUNCH_BLOCKING block the host in each launch until the
    kernel ends, so a gated call could never open its gate in time: such a context takes
    the ungated path (no time-outs, the same bytes).  The runtime reads these variables at
    its own start, so here only the library's reaction is checked."""
    monkeypatch.setenv("AMD_SERIALIZE_KERNEL", "3")
    enc = J.Encoder(0, lanes=1)
    monkeypatch.delenv("AMD_SERIALIZE_KERNEL")
    try:
        rgb = J.synth_rgb8(9, 1920, 1080)
        assert enc.encode(rgb, quality=90) == _oracle.encode(rgb, 90)
        assert enc.timing()["gate_timeouts"] == 0
    finally:
        enc.close()
