"""Process exit with contexts and device groups left open.

libjpge closes whatever is still open from its own exit handler (jpgenc_amd/csrc/
live.hpp), registered at the first jpge_open and again after RCCL loads, so it runs
before the HIP runtime's, RCCL's and a profiler tool's teardown.  The subprocesses
below unregister the Python package's own atexit hook, so the library's handler is
the one that closes them; they must exit with status 0 and print no fault.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import atexit, sys
import numpy as np
import jpgenc_amd as J
atexit.unregister(J._close_live_encoders)   # leave everything to the library's exit handler
rgb = J.synth_rgb8(3, 640, 360)
e = J.Encoder(0)
a = e.encode(rgb, quality=90)
b = e.encode_batch([rgb, rgb[:200, :300].copy()], quality=75)
g1 = J.Group([0])          # a one-member RCCL clique (loads RCCL)
s = g1.encode_striped(rgb, quality=90)
g2 = J.Group([0, 0])       # host exchanges
c = g2.encode_batch([rgb, rgb], quality=90)
assert s == a and c[0] == a, "group output differs"
mode = sys.argv[1]
if mode == "exit":
    sys.exit(0)
elif mode == "raise":
    raise SystemExit(0)
print("ok", len(a), len(b[1]), flush=True)
"""


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["end", "exit"])
def test_exit_with_open_encoder_and_groups(mode):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", _CHILD, mode], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"rc {r.returncode}\n{out[-3000:]}"
    if mode == "end":
        assert "ok" in r.stdout
    assert "Segmentation" not in out and "Aborted" not in out, out[-3000:]


@pytest.mark.gpu
def test_caller_close_after_library_exit_handler():
    """a C caller whose atexit cleanup was registered before jpge_open closes
    its context and group after the library released them at exit: no-ops, no double
    free; other calls on the released handles return JPGE_E_ARG."""
    exe = os.path.join(ROOT, "tests", "cpp", "bin", "test_exit_close")
    assert os.path.exists(exe), "build with make"
    r = subprocess.run([exe], cwd=ROOT, capture_output=True, text=True, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"rc {r.returncode}\n{out[-3000:]}"
    assert "encoded" in r.stdout and "cleanup ok" in r.stdout, out[-3000:]
