"""One-view-per-GPU data parallelism: per-rank gradient buffers and the gradient exchange.

The reference trains on one view per optimizer step (gs_lightning_module.py:139-141); an N-view batch
rendered one view per rank needs, per step:

* the SUM over views of every per-Gaussian parameter gradient (means3D, scales, rotations, opacities,
  SH coefficients), and
* the densification statistics of gaussian_model.py:175-181, formed PER VIEW: the sum of
  ||dL/dmeans2D[:, :2]|| and of the visibility count (radii > 0), plus the MAX of radii.

The statistics are only read when the model densifies (every densification_interval steps), and sums and maxima
commute with the exchange, so every rank accumulates its own views' statistics in the backward kernel
(gsr_backward's densify_accumulate / max_radii2D) and ``sync_densify_stats`` reduces them once, when densifying.
Per step only the parameter gradients cross the links:

``dense``   one SUM all-reduce of a flat column-block buffer [means3D 3 | scales 3 | rotations 4 | opacity 1 |
            shs 3M] floats per Gaussian (59 floats = 236 B at SH degree 3).
``compact`` the SH gradient of one view is rank one per Gaussian -- basis(dir_v) (x) dRGB_v -- so ranks
            all-gather the 3-float factors dRGB_v (clamp-masked colour gradient) together with their camera
            position (one buffer) and each rank expands sum_v on the GPU (gsr_sh_backward_views).  The all-reduce
            carries the other 11 floats.  Per-rank ring traffic at 8 ranks and SH degree 3:
            2*(7/8)*44 B + (7/8)*96 B = 161 B per Gaussian instead of 2*(7/8)*236 B = 413 B.

Both modes give the sum of the single-view gradients (fp32 summation order aside); tests/test_multiview.py
checks them on world_size 2 with gloo, tests/test_gpu_parity.py checks the expansion kernel on the GPU.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist

from .rasterizer import sh_backward_views

FIELDS_DENSE = ("means3D", "scales", "rotations", "opacities", "shs")
FIELDS_COMPACT = ("means3D", "scales", "rotations", "opacities")


class ViewGradReducer:
    """Gradient destinations for backward_raw(out=...) and the cross-rank exchange for one step.

    Usage per step (one view per rank)::

        st = forward_raw(...)
        backward_raw(st, settings, dcolor, dinv, out=red.backward_out(), compact_sh=red.compact,
                     accumulate_stats=True)    # statistics and max radii accumulate in the kernel
        red.reduce(means3D, campos)          # collectives + SH expansion
        red.grads["shs"], red.grads["means3D"], ...
        # when densifying:
        stats, max_radii = red.sync_densify_stats()   # summed / maxed over ranks (and steps)
        ... densify ...; red.reset_densify_stats()
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
        widths = dict(means3D=3, scales=3, rotations=4, opacities=1, shs=3 * self.M)
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
        # densification statistics of this rank's views since the last reset (local until sync_densify_stats)
        self.stats_accum = torch.zeros(self.n, 2, **f32)
        self.radii_max = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        if self.compact:
            # one all-gather buffer per rank: [dRGB (n, 3) | campos (3)]
            self.gather_in = torch.zeros(3 * self.n + 3, **f32)
            self.gather_all = torch.zeros(self.world, 3 * self.n + 3, **f32)
            self.colors_sh = self.gather_in[:3 * self.n].view(self.n, 3)
            self.shs = torch.zeros(self.n, self.M, 3, **f32)
        else:
            self.shs = self.views["shs"].view(self.n, self.M, 3)

    # ---- per view ----
    def backward_out(self) -> Dict[str, torch.Tensor]:
        """Destinations for backward_raw(out=..., accumulate_stats=True)."""
        out = dict(means3D=self.views["means3D"], scales=self.views["scales"], rotations=self.views["rotations"],
                   opacities=self.views["opacities"], means2D=self.means2D, densify_stats=self.stats_accum,
                   max_radii2D=self.radii_max)
        if self.compact:
            out["colors_sh"] = self.colors_sh
        else:
            out["shs"] = self.shs
        return out

    def record_view(self, dmeans2D: torch.Tensor, radii: torch.Tensor) -> None:
        """Accumulate one view's densification statistics (gaussian_model.py:175-181) when the backward did not
        (backward_raw without backward_out()'s densify_stats / max_radii2D)."""
        self.stats_accum[:, 0] += torch.linalg.vector_norm(dmeans2D[:, :2], dim=1)
        self.stats_accum[:, 1] += (radii > 0).to(torch.float32)
        torch.maximum(self.radii_max, radii.to(torch.int32), out=self.radii_max)

    # ---- exchange ----
    def reduce(self, means3D: torch.Tensor, campos: torch.Tensor) -> None:
        """The per-step exchange: SUM of the parameter gradients over ranks (and the SH expansion)."""
        if self.compact:
            self.gather_in[3 * self.n:].copy_(campos.reshape(3))
        # the all-gather is issued first: the collectives run in issue order on the communicator's stream, so the
        # SH expansion (which needs only the gathered factors) overlaps the all-reduce
        gather = None
        if self.world > 1 and self.compact:
            gather = _all_gather(self.gather_all, self.gather_in, self.group)
        reduce = dist.all_reduce(self.flat, group=self.group, async_op=True) if self.world > 1 else None
        if self.compact:
            if gather is not None:
                gather.wait()
            elif self.world == 1:
                self.gather_all[0].copy_(self.gather_in)
            colors_all = self.gather_all[:, :3 * self.n].view(self.world, self.n, 3)
            campos_all = self.gather_all[:, 3 * self.n:]
            self._sh_views(means3D, campos_all, colors_all, self.D, self.M, out=self.shs)
        if reduce is not None:
            reduce.wait()

    def sync_densify_stats(self):
        """SUM the accumulated statistics and MAX the radii over ranks, in place; returns (stats, radii_max):
        stats (n, 2) = [sum of ||dL/dmeans2D[:, :2]||, number of visible views] since the last reset."""
        if self.world > 1:
            work = [dist.all_reduce(self.stats_accum, group=self.group, async_op=True),
                    dist.all_reduce(self.radii_max, op=dist.ReduceOp.MAX, group=self.group, async_op=True)]
            for w in work:
                w.wait()
        return self.stats_accum, self.radii_max

    def reset_densify_stats(self) -> None:
        """After densifying (the reference zeroes xyz_gradient_accum, denom and max_radii2D there)."""
        self.stats_accum.zero_()
        self.radii_max.zero_()

    @property
    def grads(self) -> Dict[str, torch.Tensor]:
        return dict(means3D=self.views["means3D"], scales=self.views["scales"], rotations=self.views["rotations"],
                    opacities=self.views["opacities"], shs=self.shs)

    @property
    def stats(self) -> torch.Tensor:
        """(n, 2) accumulated statistics (this rank's until sync_densify_stats, then the global ones)."""
        return self.stats_accum


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group):
    """all_gather into a (world, ...) tensor; gloo lacks the single-tensor form on some builds."""
    inp = inp.contiguous()
    if dist.get_backend(group) == "nccl":
        return dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=group, async_op=True)
    dist.all_gather(list(out.unbind(0)), inp.view(out.shape[1:]), group=group)
    return None
