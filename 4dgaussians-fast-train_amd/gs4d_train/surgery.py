"""Per-Gaussian row surgery: densification (clone / split) and pruning as ROW PLANS.

Reference behaviour (scene/gaussian_model.py:316-506): each event edits every per-Gaussian tensor -- the six
parameters, their Adam moments exp_avg / exp_avg_sq, the densification statistics and the deformation table --
by concatenation (densification_postfix) and boolean indexing (prune_points), one tensor and one torch op at a
time, and a split does it twice (append the children, then drop the parents).  The rows it produces, in order:

  prune(mask)     the rows where mask is False;
  densify(...)    the rows not chosen for a split, then one copy of each row chosen for cloning, then the
                  split children: N copies of the chosen rows, copy after copy (gaussian_model.py:415-457),
                  with positions and scales the caller computes; new rows' moments zero; all statistics zero.

Here an event is described once, as a plan over the OLD rows -- `keep` (old row indices, output order) and the
appended rows (old row indices to copy, and per tensor the trailing appended rows the caller computed) -- and
every per-Gaussian tensor is rebuilt from it in one pass: on the GPU one launch for all of them
(gs4d_rows_assemble, csrc/train_tail.hip), on the CPU the same plan as torch index ops.  Both are copies, so the
result is bitwise the reference's tensors.  The optimizer keeps its state objects (the "step" entry included):
each parameter is replaced by a new nn.Parameter whose state holds the rebuilt moments.
"""
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch
import torch.nn as nn

# optimizer group name -> GaussianModel attribute of the per-Gaussian parameters (gaussian_model.py:181-190)
PARAMS = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
          "scaling": "_scaling", "rotation": "_rotation"}
STATS = ("xyz_gradient_accum", "denom", "max_radii2D", "_deformation_accum")

GATHER, ZERO_NEW, ZERO = 0, 1, 2  # gs4d_rows_tensor modes (include/gs4d_train.h)


@dataclass
class RowPlan:
    """keep: old row indices that survive, in output order.  append: old row indices the appended rows copy
    (the first len(append) appended rows of every copied tensor).  computed: {group name: rows} -- the LAST
    appended rows of that parameter, given by the caller instead of copied.  n_new: appended row count.
    stats: "carry" (rows keep their statistics, appended rows zero) or "reset" (all zero)."""
    keep: torch.Tensor
    append: Optional[torch.Tensor] = None
    computed: Dict[str, torch.Tensor] = field(default_factory=dict)
    n_new: int = 0
    stats: str = "carry"


def _torch_rows(src, mode, given, keep, append, n_new):
    """One tensor of a plan with torch ops (the CPU path; the GPU path is gs4d_rows_assemble)."""
    shape = (keep.numel() + n_new,) + tuple(src.shape[1:])
    if mode == ZERO:
        return torch.zeros(shape, dtype=src.dtype, device=src.device)
    parts = [src.index_select(0, keep)]
    if n_new:
        if mode == ZERO_NEW:
            parts.append(torch.zeros((n_new,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device))
        else:
            n_copy = n_new - (0 if given is None else given.shape[0])
            if n_copy:
                parts.append(src.index_select(0, append[:n_copy]))
            if given is not None:
                parts.append(given.to(src.dtype))
    return torch.cat(parts, 0) if len(parts) > 1 else parts[0]


def apply(model, plan: RowPlan):
    """Rebuild every per-Gaussian tensor of `model` (a GaussianModel with its optimizer) by `plan`."""
    opt = model.optimizer
    groups = {g["name"]: g for g in opt.param_groups if g["name"] in PARAMS}
    srcs, modes, givens, slots = [], [], [], []
    for name, g in groups.items():
        p = g["params"][0]
        st = opt.state.get(p)
        srcs.append(p.detach()), modes.append(GATHER), givens.append(plan.computed.get(name)), slots.append(("p", name))
        if st and "exp_avg" in st:
            for key in ("exp_avg", "exp_avg_sq"):
                srcs.append(st[key]), modes.append(ZERO_NEW), givens.append(None), slots.append((key, name))
    srcs.append(model._deformation_table), modes.append(GATHER), givens.append(None), slots.append(("attr", "_deformation_table"))
    for name in STATS:
        srcs.append(getattr(model, name)), modes.append(ZERO_NEW if plan.stats == "carry" else ZERO)
        givens.append(None), slots.append(("attr", name))
    dev = srcs[0].device
    if getattr(model, "fused", False) and dev.type == "cuda":
        from . import _C
        table = srcs[len(srcs) - 1 - len(STATS)]
        as_u8 = table.dtype == torch.bool
        if as_u8:  # bool rows as bytes (the kernel copies 1- or 4-byte elements)
            srcs[len(srcs) - 1 - len(STATS)] = table.view(torch.uint8)
        keep32 = plan.keep.to(device=dev, dtype=torch.int32)
        app32 = (plan.append if plan.append is not None else plan.keep[:0]).to(device=dev, dtype=torch.int32)
        out = _C.rows_assemble([s.contiguous() for s in srcs], givens, modes, keep32, app32, plan.n_new)
        if as_u8:
            out[len(out) - 1 - len(STATS)] = out[len(out) - 1 - len(STATS)].view(torch.bool)
    else:
        keep = plan.keep.to(device=dev, dtype=torch.long)
        app = None if plan.append is None else plan.append.to(device=dev, dtype=torch.long)
        out = [_torch_rows(s, m, g, keep, app, plan.n_new) for s, m, g in zip(srcs, modes, givens)]
    # install: a new Parameter per group, its state object carried over with the rebuilt moments
    new = {}
    for (kind, name), t in zip(slots, out):
        if kind == "p":
            g = groups[name]
            old = g["params"][0]
            st = opt.state.pop(old, None)
            q = nn.Parameter(t.requires_grad_(True))
            g["params"][0] = q
            if st is not None:
                opt.state[q] = st
            new[name] = q
        elif kind in ("exp_avg", "exp_avg_sq"):
            opt.state[new[name]][kind] = t
        else:
            setattr(model, name, t)
    for name, attr in PARAMS.items():
        if name in new:
            setattr(model, attr, new[name])


def replace_param(model, name, tensor):
    """A parameter's values replaced wholesale with fresh (zero) moments, the state object kept
    (gaussian_model.py:316-329, used by reset_opacity)."""
    opt = model.optimizer
    for g in opt.param_groups:
        if g["name"] != name:
            continue
        st = opt.state.pop(g["params"][0], None)
        q = nn.Parameter(tensor.requires_grad_(True))
        g["params"][0] = q
        if st is not None:
            st["exp_avg"] = torch.zeros_like(tensor)
            st["exp_avg_sq"] = torch.zeros_like(tensor)
            opt.state[q] = st
        setattr(model, PARAMS[name], q)
        return q
    raise KeyError(name)
