"""Binary provenance: libdcamd.so carries the hash of the sources it was built from (dc_build_id), and the
loader refuses a library whose id differs from the tree it runs from (CPU; no GPU call)."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _load_in(root: Path) -> subprocess.CompletedProcess:
    code = "from depth_completion_amd import _lib; _lib.load(); print(_lib.build_id())"
    return subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120,
                          env={"PATH": "/usr/bin:/bin", "PYTHONPATH": str(root)})


def test_build_id_matches_tree():
    from depth_completion_amd import _lib, build
    lib = _lib.load()
    assert _lib.build_id(lib) == build.source_hash()


@pytest.mark.parametrize("flip", [False, True])
def test_stale_library_refused(tmp_path, flip):
    """A copy of the package loads; after one source byte changes (library not rebuilt) load() raises."""
    pkg = tmp_path / "depth_completion_amd"
    shutil.copytree(REPO / "depth_completion_amd", pkg, ignore=shutil.ignore_patterns("build_obj", "__pycache__"))
    shutil.copytree(REPO / "include", tmp_path / "include")
    if flip:
        src = pkg / "csrc" / "guidance.hip"
        b = bytearray(src.read_bytes())
        b[-2] ^= 0x01   # inside the trailing text: a different source, same size
        src.write_bytes(bytes(b))
    r = _load_in(tmp_path)
    if flip:
        assert r.returncode != 0 and "built from other sources" in r.stderr, r.stderr[-2000:]
    else:
        assert r.returncode == 0, r.stderr[-2000:]
        assert len(r.stdout.strip()) == 16
