#!/usr/bin/env python3
"""Static check of hand-counted LDS waits in the device assembly of a libisr source.

The production weight-gradient forms (wgrad3x3.hip) and the 9x9 tail (conv9x9.hip) issue their
LDS reads (`ds_read_b64_tr_b16`, `ds_read_b128`) through inline asm, which hipcc treats as
complete once issued; the kernels then wait with hand-counted `s_waitcnt lgkmcnt(N)`.  Their
correctness rests on what the compiler does around those asm statements, so this check reads the
gfx950 assembly hipcc produced for the source (`hipcc --cuda-device-only -S`) and, per kernel,
walks the instruction stream in program order modelling the lgkm counter:

* every `ds_*` instruction enters the lgkm queue in order (its destination VGPRs, if any, are
  pending until a wait retires it); every `s_load*` / `s_buffer_load*` enters it as an SMEM entry;
* `s_waitcnt lgkmcnt(N)` retires all but the N youngest entries — and is an ERROR if an SMEM
  entry is still queued and N > 0 (SMEM completes out of order, so a count says nothing then);
* an instruction that READS a VGPR of a pending LDS destination, or a non-LDS instruction that
  overwrites one, is an ERROR: a stale fragment would be used (or the late load would clobber the
  newer value); a second LDS read into the same register is not (a wave's LDS reads return in
  issue order);
* a kernel with a private (scratch) segment is an ERROR (a spilled fragment register is exactly
  what would break a hand-counted wait).

The walk follows the kernel's control-flow graph path-sensitively (each basic block once per
distinct queue it can be entered with), so reads issued ahead across a loop back-edge are checked
against the waits at the top of the next iteration.  The walk
applies to compiler-generated LDS reads too: hipcc's own waits must pass it, which is the check's
self-test.  Exit status 1 on any error.

    python tools/check_lds_waits.py image_super_resolution_amd/csrc/wgrad3x3.hip [more.hip ...]
    python tools/check_lds_waits.py --asm build/wgrad3x3.s
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-I", str(ROOT / "include"),
         "-I", str(ROOT / "image_super_resolution_amd" / "csrc")]

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
KERNEL = re.compile(r"^(_Z\w+):\s*(;.*)?$")
WAIT = re.compile(r"lgkmcnt\((\d+)\)")
LABEL = re.compile(r"^(\.LBB\w+|\w+):")
BRANCH = re.compile(r"^s_(?:c)?branch\w*\s+(\.LBB\w+)")
STORE_PREFIXES = ("global_store", "buffer_store", "ds_write", "ds_add", "ds_max", "ds_min", "flat_store",
                  "scratch_store", "global_atomic", "buffer_atomic", "ds_swizzle", "ds_bpermute", "ds_permute")


def regs(text: str) -> set[tuple[str, int]]:
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_ops(line: str) -> tuple[str, list[str]]:
    line = line.split(";")[0].strip()
    if not line:
        return "", []
    parts = line.split(None, 1)
    op = parts[0]
    if len(parts) == 1:
        return op, []
    # operands separated by commas at depth 0 (register ranges contain ':' only)
    return op, [o.strip() for o in parts[1].split(",")]


def _instructions(lines):
    """[(line no, text, op, args, in_asm)] and {label: index of the next instruction}."""
    ins, labels, in_asm = [], {}, False
    for no, raw in lines:
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = LABEL.match(s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op, args = split_ops(s)
        if op:
            ins.append((no, s, op, args, in_asm))
    return ins, labels


def check_kernel(name: str, lines: list[tuple[int, str]], max_states: int = 256) -> tuple[list[str], list[str], dict]:
    """Path-sensitive walk of one kernel's control-flow graph: basic blocks split at labels and
    branches; every (block, lgkm queue on entry) pair is explored once, so each path's queue — also
    around loop back-edges, where reads issued at the bottom of an iteration are still queued at
    the top of the next — is checked against the waits actually on that path."""
    ins, labels = _instructions(lines)
    starts = sorted({0, *labels.values(), *(i + 1 for i, x in enumerate(ins) if x[2].startswith(("s_branch",
                                                                                                  "s_cbranch",
                                                                                                  "s_endpgm",
                                                                                                  "s_setpc")))})
    starts = [b for b in starts if b < len(ins)]
    block_end = {b: (starts[k + 1] if k + 1 < len(starts) else len(ins)) for k, b in enumerate(starts)}
    stats = {"asm_lds_reads": sum(1 for x in ins if x[4] and x[2].startswith("ds_read")),
             "lds_ops": sum(1 for x in ins if x[2].startswith("ds_")),
             "waits": sum(1 for x in ins if x[2].startswith("s_waitcnt") and "lgkmcnt" in x[1]),
             "states": 0}
    errors: list[str] = []
    notes: list[str] = []
    seen: dict[int, set] = {}
    work = [(0, ())]
    while work:
        b, q = work.pop()
        if q in seen.setdefault(b, set()):
            continue
        if len(seen[b]) >= max_states:
            notes.append(f"{name}: block at line {ins[b][0]}: more than {max_states} queue states, not explored "
                         "further")
            continue
        seen[b].add(q)
        stats["states"] += 1
        q = list(q)
        succ = []
        for i in range(b, block_end[b]):
            no, s, op, args, in_asm = ins[i]
            q = _step(name, no, s, op, args, in_asm, q, errors)
            if op == "s_branch" and args and args[0] in labels:
                succ = [labels[args[0]]]
                break
            if op.startswith("s_cbranch") and args and args[0] in labels:
                succ = [labels[args[0]]]
            if op in ("s_endpgm", "s_setpc_b64"):
                succ = None
                break
        else:
            if block_end[b] < len(ins):
                succ = succ + [block_end[b]]
        for t in succ or []:
            work.append((t, tuple(q)))
    return sorted(set(errors), key=errors.index), notes, stats


def _step(name, no, s, op, args, in_asm, q, errors):
    """One instruction against the lgkm queue q (list of (kind, dest regs, line no)); returns the new q."""
    if op.startswith("s_waitcnt"):
        m = WAIT.search(s)
        if m:
            n = int(m.group(1))
            if n > 0 and any(k == "smem" for k, _, _ in q):
                smem_lines = [l for k, _, l in q if k == "smem"]
                errors.append(f"{name}: line {no}: counted wait lgkmcnt({n}) with SMEM load(s) still queued "
                              f"(issued at line(s) {smem_lines}): SMEM completes out of order")
            q = q[len(q) - n:] if n else []
        return q
    pend = set()
    for k, d, _ in q:
        if k == "lds":
            pend |= d
    is_store = op.startswith(STORE_PREFIXES)
    if op.startswith("ds_"):
        dest = frozenset() if (is_store or not args) else frozenset(regs(args[0]))
        srcs = regs(",".join(args[1:] if dest else args))
        hz = srcs & pend
        if hz:
            errors.append(f"{name}: line {no}: '{s}' reads {sorted(hz)[:4]} before the LDS read that writes it has "
                          "been waited for")
        # (a second LDS read into a register with an older one in flight is fine: one wave's LDS
        # reads return in issue order, so the younger value lands last)
        return q + [("lds", dest, no)]
    if op.startswith(("s_load", "s_buffer_load")):
        return q + [("smem", frozenset(), no)]
    if op.startswith("s_") or not args:
        return q  # scalar instructions read no VGPRs (v_readlane / v_writelane are VALU)
    lds_dma = op.startswith("global_load_lds") or (op.startswith("buffer_load") and re.search(r"\blds\b", s))
    if is_store or lds_dma:
        dest, srcs = set(), regs(",".join(args))
    else:
        dest, srcs = regs(args[0]), regs(",".join(args[1:]))
    hz = srcs & pend
    if hz:
        errors.append(f"{name}: line {no}: '{s}' reads {sorted(hz)[:4]} before the LDS read that writes it has been "
                      "waited for")
    waw = dest & pend
    if waw:
        errors.append(f"{name}: line {no}: '{s}' writes {sorted(waw)[:4]} while an LDS read into it is still in "
                      "flight")
    return q


def kernels(asm: str):
    lines = asm.splitlines()
    cur, body, out, scratch = None, [], {}, {}
    for no, ln in enumerate(lines, 1):
        m = KERNEL.match(ln)
        if m:
            if cur is not None:
                out[cur] = body
            cur, body = m.group(1), []
            continue
        if cur is not None and ln.strip().startswith(".Lfunc_end"):
            out[cur] = body
            cur, body = None, []
            continue
        if cur is not None:
            body.append((no, ln))
    for m in re.finditer(r"\.amdhsa_kernel (\w+)(.*?)\.end_amdhsa_kernel", asm, re.S):
        sm = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(2))
        scratch[m.group(1)] = int(sm.group(1)) if sm else 0
    return out, scratch


def device_asm(src: Path, extra: list[str]) -> str:
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / (src.stem + ".s")
        r = subprocess.run([HIPCC, *FLAGS, *extra, "--cuda-device-only", "-S", str(src), "-o", str(out)],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc -S failed on {src}:\n{r.stderr}")
        return out.read_text()


def check_asm(asm: str, label: str, verbose: bool = False) -> list[str]:
    ks, scratch = kernels(asm)
    errors = []
    for name, body in ks.items():
        e, notes, st = check_kernel(name, body)
        if scratch.get(name, 0) > 0:
            e.append(f"{name}: private segment {scratch[name]} B (scratch): a spilled register breaks counted waits")
        errors += e
        if verbose:
            print(f"{label}: {name[:90]}: {st['asm_lds_reads']} asm LDS reads, {st['lds_ops']} LDS ops, "
                  f"{st['waits']} lgkm waits, {st['states']} block states, scratch {scratch.get(name, 0)} B, "
                  f"{len(e)} errors")
    return errors


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("--asm", action="append", default=[], help="an existing device assembly file")
    ap.add_argument("-D", action="append", default=[], help="extra -D define for the compile")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    errors = []
    for s in a.sources:
        errors += check_asm(device_asm(Path(s), [f"-D{d}" for d in a.D]), Path(s).name, a.verbose)
    for f in a.asm:
        errors += check_asm(Path(f).read_text(), Path(f).name, a.verbose)
    for e in errors:
        print("ERROR:", e)
    print(f"check_lds_waits: {len(errors)} error(s)")
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main())
