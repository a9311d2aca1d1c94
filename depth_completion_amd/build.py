"""Build libdcamd.so (all HIP kernels + the C ABI of include/dcamd.h) for gfx950, in-tree.

``python -m depth_completion_amd.build`` or ``__graft_entry__.build()``.  hipcc cross-compiles
without a GPU, so this runs in the CPU container too.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "libdcamd.so"
OBJ_DIR = PKG / "build_obj"
SOURCES = ["conv_gemm.hip", "conv_skinny9.hip", "conv_skinny1.hip", "conv_skinny9_gn.hip", "conv_skinny9_gnb.hip",
           "conv_skinny1_gn.hip", "conv_skinny1_gnb.hip", "conv_gemm_gn.hip", "conv_gemm_gnb.hip", "conv_gemm_ln.hip", "norms.hip", "attention.hip", "crossattn.hip", "elementwise.hip", "guidance.hip", "metrics.hip", "vae_kl.hip",
           "rowsets.hip", "ensemble.hip", "host_tables.cpp", "session.cpp", "version.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DC_OFFLOAD_ARCH", "gfx950")
HEADERS = [CSRC / h for h in ("common.h", "gn_acc.h", "conv_gemm_impl.h", "conv_skinny.h", "json_mini.h", "safetensors_mini.h")] + \
    [PKG.parent / "include" / "dcamd.h"]
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]
# per-file additions: the attention softmax's fp32 row sums must stay scalar v_add_f32 -- the SLP vectoriser pairs
# them into v_pk_add_f32 behind register moves, which issue slower beside the partner wave's MFMAs
# (MI355X_MICROARCH.md cycle constants, 'packed f32 VALU')
FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"]}


def source_files() -> list[Path]:
    """Every file libdcamd.so is compiled from (the build id hashes exactly these)."""
    return [CSRC / s for s in SOURCES] + HEADERS


def source_hash() -> str:
    """sha256 (first 16 hex digits) over the library's sources: the build id compiled into libdcamd.so
    (dc_build_id) and checked by _lib.load() against the tree it runs from."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


CONV_FAMILY = ["conv_gemm.hip", "conv_gemm_gn.hip", "conv_gemm_gnb.hip", "conv_gemm_ln.hip", "conv_skinny9.hip",
               "conv_skinny1.hip", "conv_skinny9_gn.hip", "conv_skinny9_gnb.hip", "conv_skinny1_gn.hip",
               "conv_skinny1_gnb.hip", "conv_gemm_impl.h", "conv_skinny.h", "gn_acc.h", "common.h"]


def conv_family_hash() -> str:
    """sha256 prefix over the conv family's kernel sources and the tuned variant table: the provenance a committed PMC
    record of that family carries (tools/pmc_step.py), so that bench.py pairs its counters only with the same kernels
    and variant choices (any other change to the library leaves the conv counters valid)."""
    h = hashlib.sha256()
    for name in CONV_FAMILY:
        h.update(name.encode() + b"\0" + (CSRC / name).read_bytes() + b"\0")
    h.update((PKG / "tuned_gfx950.json").read_bytes())
    return h.hexdigest()[:16]


def _includes(src: Path, seen: set | None = None) -> set:
    """The repo headers a source includes, transitively (#include "..."): a header edit rebuilds only its users."""
    seen = set() if seen is None else seen
    for line in src.read_text(errors="ignore").splitlines():
        line = line.strip()
        if line.startswith("#include \""):
            h = (src.parent / line.split('"')[1]).resolve()
            if h.exists() and h not in seen:
                seen.add(h)
                _includes(h, seen)
    return seen


def _needs(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(verbose: bool = False, force: bool = False) -> Path:
    OBJ_DIR.mkdir(exist_ok=True)
    headers = HEADERS
    bid = source_hash()
    jobs = []
    for src in SOURCES:
        s = CSRC / src
        o = OBJ_DIR / (src + ".o")
        extra = list(FILE_FLAGS.get(src, []))
        deps = [s, *_includes(s)]
        if src == "version.hip":   # carries the build id: rebuilt whenever any source changes
            extra = [f'-DDC_BUILD_ID="{bid}"']
            deps = source_files()
        if force or _needs(o, deps):
            jobs.append([HIPCC, *FLAGS, *extra, "-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    with ThreadPoolExecutor(max_workers=min(len(jobs), 6) or 1) as ex:
        list(ex.map(run, jobs))
    objs = [str(OBJ_DIR / (s + ".o")) for s in SOURCES]
    if force or jobs or not LIB.exists():
        run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", str(LIB), *objs])
    return LIB


if __name__ == "__main__":
    p = build(verbose=True, force="--force" in sys.argv)
    print("built", p)
