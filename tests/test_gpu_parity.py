"""GPU parity: the HIP path (libjpge.so through the C ABI) against the oracle,
bit-exact — quantised coefficients, symbol statistics and whole .jpg files."""
import io
import os

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu


def _scaled(rgb, maxval):
    return (rgb.astype(np.uint32) * maxval // 255).astype(np.uint8)


def _ppm_files():
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ppm")
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".ppm"))


@pytest.mark.parametrize("path", _ppm_files(), ids=lambda p: os.path.basename(p))
@pytest.mark.parametrize("quality", [50, 90])
def test_reference_images_bit_exact(encoder, path, quality):
    img = J.load_ppm(path)
    got = encoder.encode(img.rgb, quality=quality, maxval=img.maxval)
    want = _oracle.encode(img.rgb, quality, img.maxval)
    assert got == want


SIZES = [(1, 1), (4, 4), (8, 8), (16, 16), (17, 33), (26, 19), (64, 64), (100, 60), (200, 136), (333, 211),
         (512, 512)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("quality", [50, 90, 100])
def test_synthetic_bit_exact(encoder, w, h, quality):
    rgb = J.synth_rgb8(w * 1000 + h, w, h)
    assert encoder.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)


@pytest.mark.parametrize("kind", [1, 2])
@pytest.mark.parametrize("quality", [10, 50, 100])
def test_stress_kinds_bit_exact(encoder, kind, quality):
    # kind 1 = random bytes (long codes, many 0xFF), kind 2 = flat (one-symbol tables)
    rgb = J.synth_rgb8(77 + kind, 160, 96, kind=kind)
    assert encoder.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)


@pytest.mark.parametrize("maxval", [1, 15, 100, 254])
def test_maxval_scaling_bit_exact(encoder, maxval):
    rgb = _scaled(J.synth_rgb8(5, 120, 72), maxval)
    for q in (50, 90):
        assert encoder.encode(rgb, quality=q, maxval=maxval) == _oracle.encode(rgb, q, maxval)


@pytest.mark.parametrize("w,h,maxval", [(64, 48, 255), (130, 70, 255), (512, 512, 255), (96, 64, 100)])
def test_stage_coefficients_bit_exact(encoder, w, h, maxval):
    rgb = _scaled(J.synth_rgb8(w + h, w, h), maxval)
    for q in (50, 90, 100):
        gy, gcb, gcr = encoder.fdct_quant(rgb, quality=q, maxval=maxval)
        oy, ocb, ocr = _oracle.stage_coeffs(rgb, q, maxval)
        assert np.array_equal(gy, oy) and np.array_equal(gcb, ocb) and np.array_equal(gcr, ocr)


@pytest.mark.parametrize("w,h", [(64, 48), (200, 136), (512, 512)])
def test_symbol_statistics(encoder, w, h):
    rgb = J.synth_rgb8(w * h, w, h)
    for q in (50, 90):
        counts, first = encoder.symbol_stats(rgb, quality=q)
        ocounts, ofirst = _oracle.stage_hist(rgb, q)
        assert np.array_equal(counts, ocounts)
        for t in range(4):
            present = np.nonzero(ocounts[t])[0]
            # first-occurrence ORDER is what the table build consumes
            assert list(present[np.argsort(first[t][present], kind="stable")]) == \
                list(present[np.argsort(ofirst[t][present], kind="stable")])


def test_config2_1080p_q90_coefficients_and_file(encoder):
    rgb = J.synth_rgb8(2, 1920, 1080)
    gy, gcb, gcr = encoder.fdct_quant(rgb, quality=90)
    oy, ocb, ocr = _oracle.stage_coeffs(rgb, 90)
    assert np.array_equal(gy, oy) and np.array_equal(gcb, ocb) and np.array_equal(gcr, ocr)
    assert encoder.encode(rgb, quality=90) == _oracle.encode(rgb, 90)


@pytest.mark.parametrize("quality", [50, 90, 100])
def test_config3_4k_bit_exact(encoder, quality):
    rgb = J.synth_rgb8(3, 3840, 2160)
    assert encoder.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)


def test_batch_matches_single(encoder):
    frames = [J.synth_rgb8(1000 + i, 320 + 16 * (i % 3), 200 + 8 * i) for i in range(7)]
    outs = encoder.encode_batch(frames, quality=90)
    for f, o in zip(frames, outs):
        assert o == encoder.encode(f, quality=90)
        assert o == _oracle.encode(f, 90)


def _encoder_with_env(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return J.Encoder(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _encoder_with_wgs(wgs):
    return _encoder_with_env(JPGE_ENTROPY_WGS=wgs)


# Lane streams with a hardware queue each (CU-masked, the multi-lane default) and
# from HIP's shared pool give the same bytes; batches spread over every lane.
@pytest.mark.parametrize("cumask", [0, 1])
@pytest.mark.parametrize("lanes", [2, 4])
def test_lane_streams_bit_exact(cumask, lanes):
    enc = _encoder_with_env(JPGE_CU_MASK_STREAMS=cumask, JPGE_LANES=lanes)
    try:
        frames = [J.synth_rgb8(700 + i, 256 + 32 * (i % 4), 136 + 16 * (i % 3), kind=i % 3) for i in range(12)]
        outs = enc.encode_batch(frames, quality=90)
        for f, o in zip(frames, outs):
            assert o == _oracle.encode(f, 90)
    finally:
        enc.close()


# The entropy kernel splits the frame's 128-block tiles into contiguous runs of
# 2..4 tiles per workgroup; every split must give the same bytes.  Widths of
# 65 and 129 MCUs leave a final tile of 6 blocks (a few bits).
@pytest.mark.parametrize("wgs", [1, 3, 5, 100000])
@pytest.mark.parametrize("w,h,kind,quality", [(500, 300, 0, 90), (500, 300, 1, 100), (500, 300, 2, 50),
                                              (1040, 16, 0, 75), (2064, 16, 1, 95), (16, 1040, 0, 50),
                                              (128, 128, 1, 100)])
def test_entropy_workgroup_partitions(wgs, w, h, kind, quality):
    enc = _encoder_with_wgs(wgs)
    try:
        rgb = J.synth_rgb8(31 + kind + w, w, h, kind=kind)
        assert enc.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)
    finally:
        enc.close()


@pytest.mark.parametrize("wgs", [1, 100000])
def test_entropy_workgroup_partitions_4k(wgs):
    enc = _encoder_with_wgs(wgs)
    try:
        rgb = J.synth_rgb8(11, 3840, 2160, kind=1)
        assert enc.encode(rgb, quality=90) == _oracle.encode(rgb, 90)
    finally:
        enc.close()


# Placement computed once for all workgroups — by the code kernel's last workgroup
# (in_code=1, the pipeline's default) or by the placement kernel (in_code=0) — must
# agree with the pack kernel's own scan at every partition.
@pytest.mark.parametrize("in_code", [0, 1])
@pytest.mark.parametrize("wgs", [1, 5, 100000])
@pytest.mark.parametrize("w,h,kind,quality", [(500, 300, 1, 100), (1040, 16, 0, 75), (16, 1040, 0, 50),
                                              (1920, 1080, 0, 90)])
def test_entropy_scan_kernel_placement(in_code, wgs, w, h, kind, quality):
    enc = _encoder_with_env(JPGE_ENTROPY_WGS=wgs, JPGE_EXT_PLACE=1, JPGE_PLACE_IN_CODE=in_code)
    try:
        rgb = J.synth_rgb8(57 + kind + w, w, h, kind=kind)
        assert enc.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)
    finally:
        enc.close()


# The largest grid placed by the code kernel's last workgroup (kPlaceInCodeMaxWgs = 4096
# entropy workgroups, an 8K frame's 6 075 tiles over 4 096 workgroups): that path relies
# on gfx950's write-through record stores plus vmcnt(0) before the completion count
# (kernels.hpp), so it is pinned at its maximum size on flat
# data and on dense data (photo-like and random frames at Q100, where
# every workgroup writes many records, so a stale record would show).
@pytest.mark.parametrize("kind,quality", [(2, 90), (0, 100), (1, 100)])
def test_placement_in_code_at_max_grid(kind, quality):
    enc = _encoder_with_env(JPGE_ENTROPY_WGS=4096, JPGE_EXT_PLACE=1, JPGE_PLACE_IN_CODE=1)
    try:
        rgb = J.synth_rgb8(8081 + kind, 7680, 4320, kind=kind)
        assert enc.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)
    finally:
        enc.close()


def _large_golden(w, h, quality):
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large_frames.json")) as f:
        for fr in json.load(f)["frames"]:
            if (fr["width"], fr["height"], fr["quality"], fr.get("restart", 0)) == (w, h, quality, 0):
                return fr
    raise KeyError((w, h, quality))


# SURVEY 8(d) config 5 on one GPU: 16384x16384 (12288 entropy workgroups, placed by
# the scan kernel), against the oracle's SHA-256 (tests/golden/make_large.py).
@pytest.mark.parametrize("quality", [90, 50])
def test_16k_frame_matches_oracle_hash(encoder, quality):
    import hashlib
    g = _large_golden(16384, 16384, quality)
    rgb = J.synth_rgb8(g["seed"], 16384, 16384, kind=g["kind"])
    jpg = encoder.encode(rgb, quality=quality)
    assert len(jpg) == g["len"]
    assert hashlib.sha256(jpg).hexdigest() == g["sha256"]


def test_output_decodes(encoder):
    Image = pytest.importorskip("PIL.Image")
    rgb = J.synth_rgb8(42, 640, 480)
    data = encoder.encode(rgb, quality=90)
    im = Image.open(io.BytesIO(data))
    im.load()
    assert im.size == (640, 480)
    dec = np.asarray(im.convert("RGB"), np.float64)
    assert 10 * np.log10(255 ** 2 / np.mean((dec - rgb) ** 2)) > 28


def test_deterministic_repeat(encoder):
    rgb = J.synth_rgb8(9, 1280, 720, kind=1)
    a = encoder.encode(rgb, quality=95)
    b = encoder.encode(rgb, quality=95)
    assert a == b


def test_facade_cli_roundtrip(tmp_path):
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "tests", "golden", "ppm", "tester_RGB_26x19.ppm")
    out = tmp_path / "o.jpg"
    r = subprocess.run([os.path.join(root, "jpgenc_amd", "bin", "jpgenc"), src, str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Processing image size: 26x19" in r.stdout and "Encoding duration:" in r.stdout
    img = J.load_ppm(src)
    assert out.read_bytes() == _oracle.encode(img.rgb, 50, img.maxval)


def _write_ppm(path, rgb, maxval=255, ascii=False):
    h, w = rgb.shape[:2]
    if ascii:
        body = "\n".join(" ".join(str(int(v)) for v in row.reshape(-1)) for row in rgb) + "\n"
        data = f"P3\n# jpge test\n{w} {h}\n{maxval}\n".encode() + body.encode()
    else:
        data = f"P6\n{w} {h}\n{maxval}\n".encode() + np.ascontiguousarray(rgb, np.uint8).tobytes()
    with open(path, "wb") as f:
        f.write(data)


# the PPM ingest pipeline (read + parse into pinned memory, H2D
# queued ahead of the kernels, D2H + write) — every file's bytes must be the
# oracle's, across group boundaries and with P3/P6 and maxval < 255 mixed.
@pytest.mark.parametrize("group", [0, 3])
def test_encode_files_pipeline(encoder, tmp_path, group):
    ins, outs, want = [], [], []
    for i, path in enumerate(_ppm_files()):
        img = J.load_ppm(path)
        ins.append(path)
        outs.append(str(tmp_path / f"ref{i}.jpg"))
        want.append(_oracle.encode(img.rgb, 90, img.maxval))
    for i, (w, h, mv, asc) in enumerate([(640, 480, 255, False), (333, 211, 255, True), (1920, 1080, 255, False),
                                         (100, 60, 100, False), (64, 48, 15, True)]):
        rgb = _scaled(J.synth_rgb8(600 + i, w, h), mv)
        p = str(tmp_path / f"s{i}.ppm")
        _write_ppm(p, rgb, mv, asc)
        ins.append(p)
        outs.append(str(tmp_path / f"s{i}.jpg"))
        want.append(_oracle.encode(rgb, 90, mv))
    lens = encoder.encode_files(ins, outs, quality=90, group=group)
    for o, wnt, n in zip(outs, want, lens):
        with open(o, "rb") as f:
            assert f.read() == wnt
        assert n == len(wnt)


def test_encode_files_reports_bad_file(encoder, tmp_path):
    good = str(tmp_path / "g.ppm")
    _write_ppm(good, J.synth_rgb8(1, 32, 32))
    bad = str(tmp_path / "b.ppm")
    with open(bad, "wb") as f:
        f.write(b"P5\n2 2\n255\n....")
    with pytest.raises(J.JpgeError) as e:
        encoder.encode_files([good, bad, str(tmp_path / "missing.ppm")],
                             [str(tmp_path / "g.jpg"), str(tmp_path / "b.jpg"), str(tmp_path / "m.jpg")], quality=50)
    assert "[0, 5, 6]" in str(e.value)
    with open(str(tmp_path / "g.jpg"), "rb") as f:
        assert f.read() == _oracle.encode(J.synth_rgb8(1, 32, 32), 50)


# Single frames and batches over the lanes (each frame its own tables) at ragged
# sizes and entropy partitions: one workgroup, 7, and the default.
@pytest.mark.parametrize("wgs", [0, 1, 7])
@pytest.mark.parametrize("w,h,kind,quality", [(1, 1, 0, 90), (16, 16, 1, 100), (37, 23, 0, 50), (200, 136, 2, 90),
                                              (500, 300, 1, 95), (1040, 48, 0, 75), (1920, 1080, 0, 90)])
def test_pipeline_shapes_bit_exact(wgs, w, h, kind, quality):
    enc = _encoder_with_env(JPGE_ENTROPY_WGS=wgs)
    try:
        rgb = J.synth_rgb8(77 + kind + w, w, h, kind=kind)
        assert enc.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)
        if w * h <= 200 * 136:  # a batch over the lanes, each frame its own tables
            frames = [J.synth_rgb8(90 + i, w, h, kind=kind) for i in range(5)]
            assert enc.encode_batch(frames, quality=quality) == [_oracle.encode(f, quality) for f in frames]
    finally:
        enc.close()


def _extreme_frame(w, h, seed):
    # 8x8 blocks alternating black and white (DC differences of +-2040 at Q100: category
    # 11, the largest; the DC continuation record) with single-pixel impulses and sharp
    # edges inside some blocks (AC sizes up to 10: continuations of 1..4 bits)
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = (((y // 8) + (x // 8)) & 1).astype(np.uint8) * 255
    rgb = np.repeat(base[:, :, None], 3, axis=2)
    mask = rng.random((h, w)) < 0.02
    rgb[mask] = 255 - rgb[mask]
    edge = ((x % 8) < (y % 8)) & (((y // 8) * 3 + (x // 8)) % 5 == 0)
    rgb[edge, 0] = 255 - rgb[edge, 0]
    step = (((y // 8) * 7 + (x // 8)) % 11 == 0)  # blocks split into a black and a white half (AC size 10)
    rgb[step] = np.where((x[step] % 8) < 4, 0, 255)[:, None]
    return np.ascontiguousarray(rgb)


@pytest.mark.parametrize("quality", [100, 97, 90, 50])
@pytest.mark.parametrize("w,h", [(64, 48), (256, 136), (1000, 504)])
def test_extreme_sizes_bit_exact(encoder, w, h, quality):
    """The 16-bit symbol records' continuations (kernels.hpp): DC categories up to 11 and
    AC sizes up to 10 (Coding.hpp:197-230), through the fast path's fix-up and the
    general path, in single frames and a batch."""
    rgb = _extreme_frame(w, h, w + h + quality)
    want = _oracle.encode(rgb, quality)
    assert encoder.encode(rgb, quality=quality) == want
    assert encoder.encode_batch([rgb, rgb[::-1].copy()], quality=quality) == [want, _oracle.encode(rgb[::-1].copy(), quality)]


def test_extreme_frame_reaches_the_largest_categories():
    """(host) the frame above does reach DC category 11 and AC size 10 at Q100."""
    rgb = _extreme_frame(256, 136, 1)
    counts, _ = _oracle.stage_hist(rgb, 100)
    counts = np.asarray(counts).reshape(4, 256)
    assert counts[0, 11] > 0 or counts[2, 11] > 0
    assert any(counts[1, (r << 4) | 10] or counts[3, (r << 4) | 10] for r in range(16))
