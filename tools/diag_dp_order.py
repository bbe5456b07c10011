"""World-2 enqueue-order diagnostic.

Runs the SRGAN data-parallel rehearsal of tests/test_gpu_dist_train.py (2 gloo ranks on one GPU,
and the 1-rank reference with per-half discriminator BatchNorm, `_PerRankD`) with the
generator's optimiser step enqueued after (default) or before (ISR_TRAIN_G_FIRST=1) the
discriminator step, twice each, with trainer.TAPS on: every tap (sr, losses, G gradients after
the bucketed all-reduce, after clip, G parameters after Adam, D gradients before / after their
all-reduce, D parameters) is a device clone taken on the enqueuing stream, so the schedule under
test is unchanged.  For each pair of runs it names the FIRST tap that differs bit for bit and,
inside it, the tensor and element count — the first differing tensor names the state that
depends on the order or on the run.

    python tools/diag_dp_order.py [--steps 1] [--out gpurun_out/diag_dp_order.txt]
"""
from __future__ import annotations

import argparse
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def first_diff(a, b, names):
    """(tap index, tap name, tensor name, #differing, max |d|, max |d| / max |ref|) of the first
    differing tap, or None; plus a per-tap summary list."""
    rows, first = [], None
    for i, ((na, ta), (nb, tb)) in enumerate(zip(a["taps"], b["taps"])):
        assert na == nb, (na, nb)
        diff_t = []
        for k, (x, y) in enumerate(zip(ta, tb)):
            if x is None or y is None:
                continue
            if x.shape != y.shape or not np.array_equal(x, y):
                d = np.abs(x.astype(np.float64) - y.astype(np.float64))
                nm = names.get(na, [])
                diff_t.append((nm[k] if k < len(nm) else str(k), int((d > 0).sum()), float(d.max()),
                               float(d.max() / max(np.abs(y).max(), 1e-30))))
        rows.append((i, na, len(diff_t), diff_t[:3]))
        if diff_t and first is None:
            first = (i, na, diff_t[0])
    return first, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "diag_dp_order.txt"))
    a = ap.parse_args()
    # (a --round5-guard option re-created the round-5 chain-less guard path for one run,
    # profiles/r06_diag_dp_order_s2_r5guard.txt: identical to the current path at every tap, so
    # the knob was removed from train_engine)
    import test_gpu_dist_train as T

    runs = {}
    with tempfile.TemporaryDirectory() as tmp:
        for world in (1, 2):
            for g_first in (False, True):
                for rep in range(a.repeats):
                    print(f"running world {world} g_first {g_first} repeat {rep}", flush=True)
                    res = T._run("srgan", world, Path(tmp) / f"w{world}g{int(g_first)}r{rep}", "0", g_first,
                                 taps=True, steps=a.steps)
                    runs[(world, g_first, rep)] = res[0]
                    if world == 2:
                        runs[(world, g_first, rep, 1)] = res[1]
    n0 = runs[(2, False, 0)]["names"]
    names = {"sr": ["sr"], "g_loss": ["perceptual", "adversarial", "content"], "g_grad": n0["g"],
             "g_grad_clipped": n0["g"], "g_param": n0["g"], "d_grad_local": n0["d"], "d_grad": n0["d"],
             "d_param": n0["d"]}
    pairs = []
    for world in (1, 2):
        for g_first in (False, True):
            for rep in range(1, a.repeats):
                pairs.append((f"world {world} g_first {g_first}: run 0 vs run {rep}", (world, g_first, 0),
                              (world, g_first, rep)))
        pairs.append((f"world {world}: default vs g_first", (world, False, 0), (world, True, 0)))
    pairs.append(("world 2 default: rank 0 vs rank 1", (2, False, 0), (2, False, 0, 1)))
    pairs.append(("world 2 g_first: rank 0 vs rank 1", (2, True, 0), (2, True, 0, 1)))
    lines = []
    for what, ka, kb in pairs:
        first, rows = first_diff(runs[ka], runs[kb], names)
        lines.append(f"== {what}: " + ("bitwise identical at every tap" if first is None else
                                       f"first differing tap #{first[0]} '{first[1]}': {first[2]}"))
        for i, na, nd, ex in rows:
            if nd:
                lines.append(f"   tap #{i} {na}: {nd} tensors differ, e.g. {ex}")
    text = "\n".join(lines)
    print(text)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(text + "\n")


if __name__ == "__main__":
    main()
