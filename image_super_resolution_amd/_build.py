"""Builds libisr.so (the HIP kernels + C-ABI) in-tree with hipcc for gfx950.

No cmake/ninja: one hipcc invocation per .hip file (run in parallel), then a
link.  The output lands in image_super_resolution_amd/lib/ so it travels with
the repository snapshot to the GPU box.

`python -m image_super_resolution_amd._build --tuning` builds lib/libisr_tuning.so
with -DISR_TUNING (adds timing-only ablation variants whose outputs are wrong);
tools load it with ISR_LIB=<path>.  The production libisr.so never contains them.
`--interleave` builds lib/libisr_interleave.so: the production objects with trunk.hip rebuilt
under -DISR_TRUNK_INTERLEAVE=1 (the trunk's refill pieces issued one per step-0 MFMA; kept for
the parity run tests/test_gpu_chain.py gets with ISR_LIB pointing at it).
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


# sources whose kernels read LDS through inline asm with hand-counted waits: their device assembly
# is checked on every full build (tools/check_lds_waits.py)
WAIT_CHECKED = ("wgrad3x3.hip", "conv9x9.hip")


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

    def check_waits(src: Path) -> list[str]:
        """the hand-counted LDS waits of the asm-read kernels, checked on the gfx950
        assembly hipcc produces for them (tools/check_lds_waits.py: no read of an LDS destination
        before its wait, no SMEM load under a counted wait, no scratch)."""
        sys.path.insert(0, str(ROOT / "tools"))
        try:
            import check_lds_waits
        finally:
            sys.path.pop(0)
        asm = check_lds_waits.device_asm(src, ["-DISR_TUNING"] if tuning else [])
        errs = check_lds_waits.check_asm(asm, src.name)
        if tuning and errs:
            # the tuning library also carries A/B forms that never ship (measured slower; some are
            # timing probes): a hazard there is reported, and fatal only in a production kernel
            prod = set(check_lds_waits.kernels(check_lds_waits.device_asm(src, []))[0])
            for e in errs:
                if e.split(":", 1)[0] not in prod:
                    print(f"[build] tuning-only kernel, not fatal: {e}", file=sys.stderr)
            errs = [e for e in errs if e.split(":", 1)[0] in prod]
        return errs

    checked = [CSRC / n for n in WAIT_CHECKED] if (force or tuning or not LIB.exists()) else []
    with ThreadPoolExecutor(max_workers=min(8, len(sources()) + len(checked))) as ex:
        waits = [ex.submit(check_waits, src) for src in checked]
        objs = list(ex.map(compile_one, sources()))
        errs = [e for w in waits for e in w.result()]
    if errs:
        raise RuntimeError("LDS wait check failed (tools/check_lds_waits.py):\n" + "\n".join(errs))
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib_path)
    return lib_path


def build_interleave(verbose: bool = False) -> Path:
    """libisr_interleave.so: production objects, trunk.hip with -DISR_TRUNK_INTERLEAVE=1."""
    build(verbose=verbose)
    objdir = PKG / "build_interleave"
    objdir.mkdir(exist_ok=True)
    trunk_obj = objdir / "trunk.o"
    cmd = [HIPCC, *FLAGS, "-DISR_TRUNK_INTERLEAVE=1", "-c", str(CSRC / "trunk.hip"), "-o", str(trunk_obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on trunk.hip (interleave):\n{r.stderr}")
    objs = [trunk_obj if src.stem == "trunk" else PKG / "build" / (src.stem + ".o") for src in sources()]
    lib_path = LIBDIR / "libisr_interleave.so"
    tmp = lib_path.with_suffix(".so.tmp")
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib_path)
    return lib_path


def build_probe16(verbose: bool = False) -> Path:
    """libisr_probe16.so: production objects, trunk.hip with -DISR_TRUNK_MFMA16_PROBE=1 (timing
    probe, outputs wrong: each growth-chunk MFMA as two 16x16x32 of the same FLOPs)."""
    build(verbose=verbose)
    objdir = PKG / "build_probe16"
    objdir.mkdir(exist_ok=True)
    trunk_obj = objdir / "trunk.o"
    cmd = [HIPCC, *FLAGS, "-DISR_TRUNK_MFMA16_PROBE=1", "-c", str(CSRC / "trunk.hip"), "-o", str(trunk_obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on trunk.hip (probe16):\n{r.stderr}")
    objs = [trunk_obj if src.stem == "trunk" else PKG / "build" / (src.stem + ".o") for src in sources()]
    lib_path = LIBDIR / "libisr_probe16.so"
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib_path), *map(str, objs)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return lib_path


def build_trunk_alt(tag: str, defines: list[str], verbose: bool = False) -> Path:
    """lib/libisr_<tag>.so: the production objects with trunk.hip rebuilt under `defines` (A/B of a
    production trunk option in alternating processes, e.g. tag "xcd", ["-DISR_TRUNK_XCD=1"])."""
    build(verbose=verbose)
    objdir = PKG / f"build_{tag}"
    objdir.mkdir(exist_ok=True)
    trunk_obj = objdir / "trunk.o"
    r = subprocess.run([HIPCC, *FLAGS, *defines, "-c", str(CSRC / "trunk.hip"), "-o", str(trunk_obj)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on trunk.hip ({tag}):\n{r.stderr}")
    objs = [trunk_obj if src.stem == "trunk" else PKG / "build" / (src.stem + ".o") for src in sources()]
    lib_path = LIBDIR / f"libisr_{tag}.so"
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib_path), *map(str, objs)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return lib_path


if __name__ == "__main__":
    if "--probe16" in sys.argv:
        print(build_probe16(verbose=True))
    elif "--interleave" in sys.argv:
        print(build_interleave(verbose=True))
    else:
        print(build(force="--force" in sys.argv, verbose=True, tuning="--tuning" in sys.argv))
