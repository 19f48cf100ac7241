"""One-view-per-GPU data parallelism: per-rank gradient buffers and the gradient exchange.

The reference trains on one view per optimizer step (gs_lightning_module.py:139-141); an N-view batch
rendered one view per rank needs, per step:

* the SUM over views of every per-Gaussian parameter gradient (means3D, scales, rotations, opacities,
  SH coefficients), and
* the densification statistics of gaussian_model.py:175-181, formed PER VIEW before the exchange:
  sum of ||dL/dmeans2D[:, :2]|| and of the visibility count (radii > 0), plus the MAX of radii.

Two exchange modes:

``dense``   one SUM all-reduce of a flat column-block buffer [means3D 3 | scales 3 | rotations 4 | opacity 1 |
            shs 3M | stats 2] floats per Gaussian (61 floats = 244 B at SH degree 3).
``compact`` the SH gradient of one view is rank one per Gaussian -- basis(dir_v) (x) dRGB_v -- so ranks
            all-gather the 3-float factors dRGB_v (clamp-masked colour gradient) plus their camera
            positions and each rank expands sum_v on the GPU (gsr_sh_backward_views).  The all-reduce carries
            the other 13 floats.  Per-rank ring traffic at 8 ranks and SH degree 3: 2*(7/8)*52 B + (7/8)*96 B
            = 175 B per Gaussian instead of 2*(7/8)*244 B = 427 B.

Both modes give the sum of the single-view gradients (fp32 summation order aside); tests/test_multiview.py
checks them on world_size 2 with gloo, tests/test_gpu_parity.py checks the expansion kernel on the GPU.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist

from .rasterizer import sh_backward_views

FIELDS_DENSE = ("means3D", "scales", "rotations", "opacities", "shs", "stats")
FIELDS_COMPACT = ("means3D", "scales", "rotations", "opacities", "stats")


class ViewGradReducer:
    """Gradient destinations for backward_raw(out=...) and the cross-rank exchange for one step.

    Usage per step (one view per rank)::

        st = forward_raw(...)
        backward_raw(st, settings, dcolor, dinv, out=red.backward_out(), compact_sh=red.compact)
        red.record_view(red.means2D, radii, stats_written=True)  # stats come from the backward kernel
        red.reduce(means3D, campos)          # collectives + SH expansion
        red.grads["shs"], red.grads["means3D"], red.stats, red.radii_max, ...
    """

    def __init__(self, n: int, M: int, sh_degree: int, device, mode: str = "compact", group=None,
                 world_size: Optional[int] = None,
                 sh_views_fn: Optional[Callable[..., torch.Tensor]] = None):
        if mode not in ("dense", "compact"):
            raise ValueError(f"mode must be 'dense' or 'compact', got {mode!r}")
        self.n, self.M, self.D = int(n), int(M), int(sh_degree)
        self.device = torch.device(device)
        self.mode = mode
        self.compact = mode == "compact"
        self.group = group
        self.world = int(world_size if world_size is not None else
                         (dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1))
        self._sh_views = sh_views_fn or sh_backward_views
        widths = dict(means3D=3, scales=3, rotations=4, opacities=1, shs=3 * self.M, stats=2)
        fields = FIELDS_COMPACT if self.compact else FIELDS_DENSE
        cols = sum(widths[k] for k in fields)
        f32 = dict(dtype=torch.float32, device=self.device)
        # column-block layout [field][Gaussian][width]: every destination is a contiguous (n, w) view
        self.flat = torch.zeros(cols * self.n, **f32)
        self.views: Dict[str, torch.Tensor] = {}
        off = 0
        for k in fields:
            w = widths[k]
            self.views[k] = self.flat[off * self.n:(off + w) * self.n].view(self.n, w)
            off += w
        self.means2D = torch.zeros(self.n, 3, **f32)
        self.radii_max = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        if self.compact:
            self.colors_sh = torch.zeros(self.n, 3, **f32)
            self.colors_sh_all = torch.zeros(self.world, self.n, 3, **f32)
            self.campos_all = torch.zeros(self.world, 3, **f32)
            self.shs = torch.zeros(self.n, self.M, 3, **f32)
        else:
            self.shs = self.views["shs"].view(self.n, self.M, 3)

    # ---- per view ----
    def backward_out(self) -> Dict[str, torch.Tensor]:
        out = dict(means3D=self.views["means3D"], scales=self.views["scales"], rotations=self.views["rotations"],
                   opacities=self.views["opacities"], means2D=self.means2D, densify_stats=self.views["stats"])
        if self.compact:
            out["colors_sh"] = self.colors_sh
        else:
            out["shs"] = self.shs
        return out

    def record_view(self, dmeans2D: torch.Tensor, radii: torch.Tensor, stats_written: bool = False) -> None:
        """Densification statistics of this rank's view (gaussian_model.py:175-181), before the exchange.
        backward_raw(out=backward_out()) already wrote them (gsr_backward's densify_stats) unless
        stats_written is False and they are formed here from dmeans2D / radii."""
        if not stats_written:
            st = self.views["stats"]
            torch.linalg.vector_norm(dmeans2D[:, :2], dim=1, out=st[:, 0])
            st[:, 1].copy_(radii > 0)
        if self.world > 1:
            self.radii_max.copy_(radii)
        else:
            self.radii_max = radii

    # ---- exchange ----
    def reduce(self, means3D: torch.Tensor, campos: torch.Tensor) -> None:
        if self.world > 1:
            work = [dist.all_reduce(self.flat, group=self.group, async_op=True),
                    dist.all_reduce(self.radii_max, op=dist.ReduceOp.MAX, group=self.group, async_op=True)]
            if self.compact:
                work.append(_all_gather(self.colors_sh_all, self.colors_sh, self.group))
                work.append(_all_gather(self.campos_all, campos.reshape(3).to(torch.float32), self.group))
            for w in work:
                if w is not None:
                    w.wait()
        elif self.compact:
            self.colors_sh_all[0].copy_(self.colors_sh)
            self.campos_all[0].copy_(campos.reshape(3))
        if self.compact:
            self._sh_views(means3D, self.campos_all, self.colors_sh_all, self.D, self.M, out=self.shs)

    @property
    def grads(self) -> Dict[str, torch.Tensor]:
        return dict(means3D=self.views["means3D"], scales=self.views["scales"], rotations=self.views["rotations"],
                    opacities=self.views["opacities"], shs=self.shs)

    @property
    def stats(self) -> torch.Tensor:
        """(n, 2): [sum over views of ||dL/dmeans2D[:, :2]||, number of views with radii > 0]."""
        return self.views["stats"]


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group):
    """all_gather into a (world, ...) tensor; gloo lacks the single-tensor form on some builds."""
    inp = inp.contiguous()
    if dist.get_backend(group) == "nccl":
        return dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=group, async_op=True)
    dist.all_gather(list(out.unbind(0)), inp.view(out.shape[1:]), group=group)
    return None
