"""the host C++ runtime under AddressSanitizer (host code only - GPU ASan is not
available on this pool).  Builds the ASan variant of the extension into a temp dir (the in-tree
module is untouched), loads it into a plain python with the clang ASan runtime preloaded and
drives host-side paths: MLP shape planning for every supported width, the exception paths of
bad shapes, the exchange slab sizing and the device query without a GPU.  Any heap overflow /
use-after-free in those paths aborts the child with an ASan report."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, {out!r})
import _dct_native as n
for dims in ([5, 64, 2], [5, 128, 128, 2], [256, 1024, 1024, 1024, 2], [7, 20, 2], [32, 128, 128, 4]):
    for bmax in (1, 4, 16):
        p = n.MlpPlan(dims, bmax)
        assert p.num_params == sum(a * b + b for a, b in zip(dims[:-1], dims[1:]))
for bad in ([5], [5, 0, 2], [5, 99999, 2], [1, 2, 3, 4, 5, 6, 7]):
    try:
        n.MlpPlan(bad, 4)
        raise SystemExit("bad dims accepted: %r" % (bad,))
    except (ValueError, RuntimeError):
        pass
assert n.mlp_xg_slab_granules([5, 64, 2]) > 0
print("device_count", n.device_count())
print("ASAN-CHILD-OK")
"""


@pytest.mark.slow
def test_host_runtime_under_asan(tmp_path):
    sys.path.insert(0, ROOT)
    import dct_amd  # noqa: F401
    from dct_amd import _build

    out = _build.build_sanitized(str(tmp_path / "asan"))
    rt = _build.asan_runtime()
    assert os.path.exists(rt), rt
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-c", CHILD.format(out=os.path.dirname(out))], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ASAN-CHILD-OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "AddressSanitizer" not in r.stderr
