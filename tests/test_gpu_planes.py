"""The plane stage kernels (planes.hip) — the reference's Image stage methods on fp64
planes — bit-exact against the oracle and against plain fp64 restatements of the
reference's loops; writeJPEG on planes (jpge_encode_planes) against the oracle's
bytes; and the drop-in facade's GPU part (tests/cpp/test_facade.cpp gpu)."""
import os
import subprocess

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PPM = os.path.join(ROOT, "tests", "golden", "ppm")
FACADE = os.path.join(ROOT, "tests", "cpp", "bin", "test_facade")
f32 = lambda v: float(np.float32(v))  # noqa: E731  (the reference's float literals, widened)


def _planes(rng, h, w, kind):
    if kind == "bytes":  # loadPPM planes: byte * 255 / maxval
        mv = 255
        return [rng.integers(0, 256, (h, w)).astype(np.float64) * (255. / mv) for _ in range(3)]
    if kind == "scaled":
        mv = 15
        return [rng.integers(0, 16, (h, w)).astype(np.float64) * (255. / mv) for _ in range(3)]
    return [rng.normal(128, 90, (h, w)) for _ in range(3)]


@pytest.mark.parametrize("kind", ["bytes", "scaled", "float"])
def test_color_convert_matches_reference_loop(encoder, kind):
    rng = np.random.default_rng(11)
    r, g, b = _planes(rng, 24, 40, kind)
    y, cb, cr = encoder.color_convert(r, g, b, J.JPGE_TO_YCBCR)
    # Image.cpp:141-143, in fp64 with the float constants widened
    wy = f32(0) + (f32(.299) * r + f32(.587) * g + f32(.114) * b) - 128
    wcb = f32(128) + (f32(-.1687) * r + f32(-.3312) * g + f32(.5) * b) - 128
    wcr = f32(128) + (f32(.5) * r + f32(-.4186) * g + f32(-.0813) * b) - 128
    assert np.array_equal(y, wy) and np.array_equal(cb, wcb) and np.array_equal(cr, wcr)
    out = np.zeros(3)
    for i in range(0, r.size, 37):  # and the oracle's to_ycc
        _oracle.orc().orc_ycc(r.flat[i], g.flat[i], b.flat[i], _oracle._p(out))
        assert (y.flat[i], cb.flat[i], cr.flat[i]) == tuple(out)
    # back to RGB (Image.cpp:165-171)
    R, G, B = encoder.color_convert(y, cb, cr, J.JPGE_TO_RGB)
    yy, cc, rr = y + 128, cb + 128, cr + 128
    assert np.array_equal(R, f32(1) * yy + f32(0) * cc + f32(1.402) * rr)
    assert np.array_equal(G, f32(1) * yy + f32(-.344) * cc + f32(-.714) * rr)
    assert np.array_equal(B, f32(1) * yy + f32(1.772) * cc + f32(0) * rr)


@pytest.mark.parametrize("mode", [444, 422, 411, 4200, 420, 4201])
@pytest.mark.parametrize("shape", [(16, 16), (48, 64), (34, 20)])
def test_subsample_plane_matches_oracle(encoder, mode, shape):
    h, w = shape
    if mode == 411 and w % 4:
        pytest.skip("S411 needs whole runs of 4")
    rng = np.random.default_rng(h * w + mode)
    p = rng.normal(0, 60, (h, w))
    assert np.array_equal(encoder.subsample_plane(p, mode), _oracle.subsample_mode(p, mode))


def test_subsample_plane_rejects_partial_runs(encoder):
    with pytest.raises(J.JpgeError):
        encoder.subsample_plane(np.zeros((16, 18)), 411)
    with pytest.raises(J.JpgeError):
        encoder.subsample_plane(np.zeros((15, 16)), 420)


def _dct_blocks(plane, fn):
    out = np.empty_like(plane)
    for by in range(0, plane.shape[0], 8):
        for bx in range(0, plane.shape[1], 8):
            out[by:by + 8, bx:bx + 8] = fn(np.ascontiguousarray(plane[by:by + 8, bx:bx + 8]))
    return out


def _arai_oracle(blk):
    o = np.zeros(64)
    _oracle.orc().orc_dct_arai(_oracle._p(blk.reshape(64).copy()), _oracle._p(o))
    return o.reshape(8, 8)


def _dct_matrix_A():
    import math
    A = np.zeros((8, 8))
    for k in range(8):
        for n in range(8):
            A[k, n] = (1. / math.sqrt(2) if k == 0 else 1.) * math.sqrt(2. / 8) * math.cos(
                (2. * n + 1.) * ((k * math.pi) / (2. * 8)))
    return A


def _mat_restated(X, A):
    """dctMat (Dct.hpp:264-276): first = X A^T, Y = A first, uBLAS sums k ascending."""
    first = np.zeros((8, 8))
    Y = np.zeros((8, 8))
    for i in range(8):
        for j in range(8):
            s = 0.0
            for k in range(8):
                s += X[i, k] * A[j, k]
            first[i, j] = s
    for i in range(8):
        for j in range(8):
            s = 0.0
            for k in range(8):
                s += A[i, k] * first[k, j]
            Y[i, j] = s
    return Y


def _direct_restated(X, A):
    """dctDirect (Dct.hpp:238-262)."""
    Y = np.zeros((8, 8))
    for i in range(8):
        for j in range(8):
            s = 0.0
            for x in range(8):
                for y in range(8):
                    s += X[y, x] * A[i, x] * A[j, y]
            Y[j, i] = s
    return Y


def test_dct_plane_arai_matches_oracle(encoder):
    rng = np.random.default_rng(5)
    p = rng.normal(0, 70, (32, 48))
    assert np.array_equal(encoder.dct_plane(p, J.DCT_ARAI), _dct_blocks(p, _arai_oracle))


@pytest.mark.parametrize("mode", [J.DCT_MATRIX, J.DCT_SIMPLE])
def test_dct_plane_matrix_and_direct_match_restatement(encoder, mode):
    rng = np.random.default_rng(6 + mode)
    p = rng.normal(0, 70, (16, 16))
    A = _dct_matrix_A()
    fn = (lambda b: _mat_restated(b, A)) if mode == J.DCT_MATRIX else (lambda b: _direct_restated(b, A))
    got = encoder.dct_plane(p, mode)
    assert np.array_equal(got, _dct_blocks(p, fn))
    # DctTest.cpp:22-39: the three transforms agree within the reference's tolerance
    assert np.allclose(got, encoder.dct_plane(p, J.DCT_ARAI), atol=1e-9)


def test_quantize_plane_matches_oracle(encoder):
    rng = np.random.default_rng(8)
    qy, _ = J.quality_tables(75)
    p = rng.normal(0, 300, (24, 40))
    p[::3, ::5] = (np.round(p[::3, ::5]) + 0.5) * 3  # some exact halves (a multiple of q only where q = 1, 3)
    got = encoder.quantize_plane(p, qy)
    q32 = qy.astype(np.int32)
    for by in range(0, 24, 8):
        for bx in range(0, 40, 8):
            w = np.zeros(64, np.int32)
            _oracle.orc().orc_quantize(_oracle._p(np.ascontiguousarray(p[by:by + 8, bx:bx + 8]).reshape(64)),
                                       _oracle._p(q32), _oracle._p(w))
            assert np.array_equal(got[by:by + 8, bx:bx + 8].reshape(64), w)


def _padded_planes(rgb, maxval=255):
    """loadPPM's planes (Image.cpp:393-531): byte * 255/maxval, edge-replicated to x16."""
    h, w = rgb.shape[:2]
    H, W = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    ys = np.minimum(np.arange(H), h - 1)
    xs = np.minimum(np.arange(W), w - 1)
    p = rgb[ys][:, xs].astype(np.float64) * (255. / maxval)
    return [np.ascontiguousarray(p[..., c]) for c in range(3)]


@pytest.mark.parametrize("w,h,quality,maxval", [(64, 48, 50, 255), (26, 19, 90, 255), (333, 211, 75, 255),
                                                (100, 60, 50, 15), (1920, 1080, 90, 255)])
def test_encode_planes_matches_oracle(encoder, w, h, quality, maxval):
    rgb = (J.synth_rgb8(w + h, w, h).astype(np.uint32) * maxval // 255).astype(np.uint8)
    want = _oracle.encode(rgb, quality, maxval=maxval)
    planes = _padded_planes(rgb, maxval)
    assert encoder.encode_planes(*planes, w, h, J.JPGE_TO_RGB, quality) == want
    # the same image handed over in YCbCr (convertToColorSpace done first, on the GPU)
    ycc = encoder.color_convert(*planes, J.JPGE_TO_YCBCR)
    assert encoder.encode_planes(*ycc, w, h, J.JPGE_TO_YCBCR, quality) == want


def test_encode_planes_restart(encoder):
    rgb = J.synth_rgb8(3, 160, 96)
    encoder.set_restart(7)
    try:
        got = encoder.encode_planes(*_padded_planes(rgb), 160, 96, J.JPGE_TO_RGB, 90)
    finally:
        encoder.set_restart(0)
    assert got == _oracle.encode(rgb, 90, restart=7)


def _entropy_segment(jpg: bytes) -> bytes:
    i = jpg.index(b"\xff\xda")
    n = (jpg[i + 2] << 8) | jpg[i + 3]
    return jpg[i + 2 + n:-2]


@pytest.mark.timeout(240)
def test_facade_cpp_reference_unit_tests_gpu(tmp_path):
    """ImageTest.cpp:47-73, 75-199, 347-353 through the facade; the stage chain of
    writeJPEG; writeJPEG on the fused and the plane paths; two threads at once."""
    assert os.path.exists(FACADE), "run make"
    r = subprocess.run([FACADE, "gpu", PPM, str(tmp_path)], capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert ", 0 failed" in r.stdout

    def ppm(name):
        with open(os.path.join(PPM, name), "rb") as f:
            return J.parse_ppm(f.read())

    def read(name):
        with open(tmp_path / name, "rb") as f:
            return f.read()

    for name in ("tester_p3.ppm", "tester_RGB_26x19.ppm", "tester_text_32x32.ppm", "tester_p6.ppm"):
        p = ppm(name)
        want = _oracle.encode(p.rgb, 50, maxval=p.maxval)
        assert read(name + ".frame.jpg") == want, name
        assert read(name + ".planes.jpg") == want, name
    p = ppm("tester_RGB_26x19.ppm")
    assert read("tester_RGB_26x19.q90.jpg") == _oracle.encode(p.rgb, 90, maxval=p.maxval)
    # the stage chain: quantised planes and the entropy-coded segment
    y, cb, cr = _oracle.stage_coeffs(p.rgb, 50, maxval=p.maxval)
    with open(tmp_path / "stage_q.txt") as f:
        rows = [list(map(int, ln.split())) for ln in f]
    for (got, want) in zip(rows, (y, cb, cr)):
        H, W = got[0], got[1]
        plane = np.array(got[2:], np.int32).reshape(H, W)
        blocks = plane.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        assert np.array_equal(blocks, want.astype(np.int32))
    assert read("stage_entropy.bin") == _entropy_segment(_oracle.encode(p.rgb, 50, maxval=p.maxval))
    # built images (Image(w, h, RGB) with written planes), RGB and YCbCr
    yy, xx = np.mgrid[0:32, 0:48]
    built = np.stack([(xx * 5) % 256, (yy * 7) % 256, ((xx + yy) * 3) % 256], -1).astype(np.uint8)
    assert read("built_rgb.jpg") == _oracle.encode(built, 50)
    assert read("built_ycc.jpg") == _oracle.encode(built, 50)
    # two threads sharing the default context
    t = ppm("tester_text_32x32.ppm")
    assert read("thread_a.jpg") == _oracle.encode(t.rgb, 75, maxval=t.maxval)
    assert read("thread_b.jpg") == _oracle.encode(p.rgb, 75, maxval=p.maxval)
