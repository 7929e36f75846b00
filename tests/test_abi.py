"""The C-ABI library loads and exports exactly what include/jpge.h declares
(no GPU work here), and the product never links the oracle."""
import os
import re
import subprocess

import jpgenc_amd as J

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "jpge.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(jpge_[a-z0-9_]+)\s*\(", src))


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_header_matches_python_binding_list():
    assert _declared() == set(J.EXPORTS)


def test_library_exports_every_declared_symbol():
    assert J.lib() is not None
    exported = _exported(J.LIB_PATH)
    missing = _declared() - exported
    assert not missing, missing
    for name in _declared():
        assert hasattr(J.lib(), name)


def test_product_does_not_link_oracle():
    out = subprocess.run(["ldd", J.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc" not in out and "libref" not in out
    syms = _exported(J.LIB_PATH)
    assert not any(s.startswith(("orc_", "ref_")) for s in syms)


def test_strerror_and_version():
    assert J.lib().jpge_strerror(0) == b"ok"
    assert J.lib().jpge_strerror(5) == b"Only P3 and P6 format is supported!"
    assert J.lib().jpge_version() >= 100


def test_cli_without_arguments_matches_reference():
    # main.cpp:10-13: no arguments -> message, exit code 0 (no GPU touched)
    cli = os.path.join(ROOT, "jpgenc_amd", "bin", "jpgenc")
    r = subprocess.run([cli], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "No filename was written"


def test_max_jpeg_bytes_covers_worst_case():
    # 1665 bits/block worst case, doubled for stuffing, + headers
    assert J.max_jpeg_bytes(16, 16) >= 2048 + 6 * 2 * 209
