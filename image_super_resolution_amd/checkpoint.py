"""Checkpoint I/O for the drop-in generator modules.

The reference pickles whole modules (`torch.save({'gen_net': deepcopy(model).half(),
'ema': ..., 'optimizer': ..., 'epoch': ...})`, train.py:239-244, 294-302,
376-388) and restores them with `ckpt['ema'].float().state_dict()`
(utils/models.py:659-665, train.py:276-290).  Here the same dictionary keys hold
**state_dicts** (fp16 like the reference's `.half()`), so every load goes through
`torch.load(..., weights_only=True)` and never executes code from the file.
`.safetensors` files holding one state_dict are accepted as well.
"""
from __future__ import annotations

import re
from pathlib import Path

import torch
from torch import nn


def _as_state_dict(v):
    if isinstance(v, nn.Module):
        return {k: t.detach().clone() for k, t in v.state_dict().items()}
    return v


def intersect_dicts(da: dict, db: dict, exclude=()) -> dict:
    """utils/general.py:129-131 — keys of `da` present in `db` with equal shapes."""
    return {k: v for k, v in da.items() if k in db and not any(x in k for x in exclude) and v.shape == db[k].shape}


def load_checkpoint(path) -> dict:
    """Read a checkpoint dictionary (or a bare state_dict) with the safe loader."""
    path = Path(path)
    if path.suffix == ".safetensors":
        from safetensors.torch import load_file
        return load_file(path.as_posix(), device="cpu")
    try:
        return torch.load(path.as_posix(), map_location="cpu", weights_only=True)
    except Exception as e:  # a pickled nn.Module (reference format) is refused by the safe loader
        raise RuntimeError(f"{path}: not loadable with weights_only=True ({type(e).__name__}). Reference "
                           "checkpoints that pickle whole modules must be re-exported as state_dicts") from e


def load_module_state(path, key: str | tuple[str, ...] = ("ema", "gen_net")) -> dict:
    """Return the fp32 state_dict stored under the first present `key`
    (the reference reads 'ema' for resume / SRGAN init, 'gen_net' otherwise);
    a bare state_dict file is returned as is."""
    ck = load_checkpoint(path)
    keys = (key,) if isinstance(key, str) else tuple(key)
    sd = None
    for k in keys:
        if isinstance(ck.get(k), dict):
            sd = ck[k]
            break
    if sd is None:
        if all(isinstance(v, torch.Tensor) for v in ck.values()):
            sd = ck
        else:
            raise KeyError(f"{path}: none of {keys} holds a state_dict (keys: {sorted(ck)})")
    return {k: (v.float() if v.is_floating_point() else v) for k, v in sd.items()}


def save_checkpoint(path, **entries) -> None:
    """train.py-style checkpoint: nn.Module entries are stored as fp16
    state_dicts (the reference stores `.half()` modules), optimiser/scaler
    states and scalars as given."""
    out = {}
    for k, v in entries.items():
        v = _as_state_dict(v)
        if k in ("gen_net", "dis_net", "ema") and isinstance(v, dict):
            v = {n: (t.half() if t.is_floating_point() else t) for n, t in v.items()}
        out[k] = v
    torch.save(out, Path(path).as_posix())


_RES = re.compile(r"^(?:res_net\.)?residual\.(\d+)\.")
_SCL = re.compile(r"^(?:res_net\.)?scaler\.(\d+)\.")


def generator_from_state(sd: dict, add_rate: float = 0.2) -> nn.Module:
    """Instantiate the generator class a state_dict belongs to: ResNet when the
    RDB convs carry BatchNorm keys, EResNet otherwise; depth from `residual.N`,
    scale from the number of `scaler.N` stages (scaleRate = 2·stages,
    utils/models.py:595,624).  Keys under `res_net.` give an SRGAN."""
    from . import models
    blocks = {int(m.group(1)) for k in sd if (m := _RES.match(k))}
    stages = {int(m.group(1)) for k in sd if (m := _SCL.match(k))}
    if not blocks or not stages:
        raise ValueError("state_dict does not look like a ResNet/EResNet generator")
    enchant = not any(k.endswith("conv0.bn.weight") and ".net.0." in k for k in sd)
    deep, scale = max(blocks) + 1, 2 * (max(stages) + 1)
    if any(k.startswith("res_net.") for k in sd):
        net = models.SRGAN(deep, add_rate, enchant=enchant, scaleRate=scale)
    elif enchant:
        net = models.EResNet(deep, add_rate, scale)
    else:
        net = models.ResNet(deep, add_rate, scaleRate=scale)
    net.load_state_dict(sd)
    return net
