"""Builds libisr.so (the HIP kernels + C-ABI) in-tree with hipcc for gfx950.

No cmake/ninja: one hipcc invocation per .hip file (run in parallel), then a
link.  The output lands in image_super_resolution_amd/lib/ so it travels with
the repository snapshot to the GPU box.

`python -m image_super_resolution_amd._build --tuning` builds lib/libisr_tuning.so
with -DISR_TUNING (adds timing-only ablation variants whose outputs are wrong);
tools load it with ISR_LIB=<path>.  The production libisr.so never contains them.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
LIB = LIBDIR / "libisr.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
         "-I", str(ROOT / "include"), "-I", str(CSRC)]


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = sources() + list(CSRC.glob("*.h")) + [ROOT / "include" / "isr.h", Path(__file__)]
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = False, tuning: bool = False) -> Path:
    lib_path = LIBDIR / "libisr_tuning.so" if tuning else LIB
    if not tuning and not force and not _needs_build():
        return LIB
    objdir = PKG / ("build_tuning" if tuning else "build")
    flags = FLAGS + (["-DISR_TUNING"] if tuning else [])
    objdir.mkdir(exist_ok=True)
    LIBDIR.mkdir(exist_ok=True)

    headers = list(CSRC.glob("*.h")) + [ROOT / "include" / "isr.h", Path(__file__)]
    newest_header = max(p.stat().st_mtime for p in headers)

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        if not force and obj.exists() and obj.stat().st_mtime > max(src.stat().st_mtime, newest_header):
            return obj  # incremental: object newer than its source and every header
        cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(sources()))) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib_path)
    return lib_path


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, tuning="--tuning" in sys.argv))
