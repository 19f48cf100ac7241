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

``dense``   one SUM all-reduce of the per-Gaussian gradient block [means3D 3 | scales 3 | rotations 4 | opacity 1 |
            shs 3M] floats per Gaussian (59 floats = 236 B at SH degree 3).
``compact`` the SH gradient of one view is rank one per Gaussian -- basis(dir_v) (x) dRGB_v -- so ranks
            all-gather the 3-float factors dRGB_v (clamp-masked colour gradient) and their camera positions, and
            each rank expands sum_v on the GPU (gsr_sh_backward_views).  The all-reduce carries the other 11 floats.
            Per-rank ring traffic at 8 ranks and SH degree 3: 2*(7/8)*44 B + (7/8)*96 B = 161 B per Gaussian
            instead of 2*(7/8)*236 B = 413 B.

Overlap with the backward (``chunks`` = K > 1): the Gaussians are split into K contiguous ranges and the
gradient buffer is laid out chunk-major -- chunk c's block holds [means3D | scales | rotations | opacity (| shs)]
of its Gaussians only -- so a chunk's exchange is ONE all-reduce (+ one all-gather of its colour factors).  The
backward runs its per-Gaussian stage chunk by chunk (rasterizer.backward_chunked) and the exchange of chunk c is
issued as soon as chunk c is enqueued; RCCL runs it on its own stream while the GPU computes chunk c + 1.  The SH
expansions follow once each chunk's gather has arrived.  Results are bitwise those of K = 1: every element is the
same sum of the same per-rank values (tests/test_multiview.py checks K = 1 against K = 4 on world_size 2).

Both modes give the sum of the single-view gradients (fp32 summation order aside); tests/test_multiview.py
checks them on world_size 2 with gloo, tests/test_gpu_parity.py checks the expansion kernel on the GPU.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .rasterizer import sh_backward_views

FIELDS_DENSE = ("means3D", "scales", "rotations", "opacities", "shs")
FIELDS_COMPACT = ("means3D", "scales", "rotations", "opacities")


def chunk_bounds(n: int, k: int, align: int = 256) -> List[Tuple[int, int]]:
    """K contiguous Gaussian ranges covering [0, n), boundaries on multiples of `align` (whole preprocess blocks)."""
    k = max(1, int(k))
    step = -(-n // k)
    step = max(align, -(-step // align) * align)
    out = []
    g = 0
    while g < n or not out:
        out.append((g, min(n, g + step)))
        g += step
    return out


class ViewGradReducer:
    """Gradient destinations for the backward and the cross-rank exchange for one step.

    Usage per step (one view per rank)::

        st = forward_raw(...)
        red.begin_step(campos)
        backward_chunked(st, settings, dcolor, dinv, red.chunk_outputs(), on_chunk=red.start_chunk,
                         compact_sh=red.compact, accumulate_stats=True)
        red.finish(means3D)                  # SH expansion, waits for the collectives
        red.grads["shs"], red.grads["means3D"], ...
        # when densifying:
        stats, max_radii = red.sync_densify_stats()   # summed / maxed over ranks (and steps)
        ... densify ...; red.reset_densify_stats()

    With chunks == 1, ``backward_raw(..., out=red.backward_out(), ...)`` followed by ``red.reduce(means3D, campos)``
    is the same exchange without overlap.
    """

    def __init__(self, n: int, M: int, sh_degree: int, device, mode: str = "compact", group=None,
                 world_size: Optional[int] = None,
                 sh_views_fn: Optional[Callable[..., torch.Tensor]] = None, chunks: int = 1,
                 distributed: Optional[bool] = None):
        if mode not in ("dense", "compact"):
            raise ValueError(f"mode must be 'dense' or 'compact', got {mode!r}")
        self.n, self.M, self.D = int(n), int(M), int(sh_degree)
        self.device = torch.device(device)
        self.mode = mode
        self.compact = mode == "compact"
        self.group = group
        # Collectives run whenever a process group exists, even of one rank (the RCCL code path then executes on a
        # single GPU exactly as it does on eight); distributed=False keeps a reducer local inside a process group.
        if distributed is None:
            distributed = bool(dist.is_available() and dist.is_initialized())
        self.distributed = bool(distributed)
        self.world = int(world_size if world_size is not None else
                         (dist.get_world_size(group) if self.distributed else 1))
        self._sh_views = sh_views_fn or sh_backward_views
        self.widths = dict(means3D=3, scales=3, rotations=4, opacities=1, shs=3 * self.M)
        self.fields = FIELDS_COMPACT if self.compact else FIELDS_DENSE
        cols = sum(self.widths[k] for k in self.fields)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.bounds = chunk_bounds(self.n, chunks)
        # chunk-major blocks, each [field][Gaussian of the chunk][width]: every destination is a contiguous view
        self.flat = torch.zeros(cols * self.n, **f32)
        self.chunk_flat: List[torch.Tensor] = []
        self.chunk_views: List[Dict[str, torch.Tensor]] = []
        off = 0
        for g0, g1 in self.bounds:
            L = g1 - g0
            blk = self.flat[off:off + cols * L]
            views, o = {}, 0
            for k in self.fields:
                w = self.widths[k]
                views[k] = blk[o * L:(o + w) * L].view(L, w)
                o += w
            self.chunk_flat.append(blk)
            self.chunk_views.append(views)
            off += cols * L
        self.means2D = torch.zeros(self.n, 3, **f32)
        # densification statistics of this rank's views since the last reset (local until sync_densify_stats)
        self.stats_accum = torch.zeros(self.n, 2, **f32)
        self.radii_max = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        if self.compact:
            # per chunk: this rank's colour factors and everyone's; camera positions once per step
            self.gather_in = [torch.zeros(g1 - g0, 3, **f32) for g0, g1 in self.bounds]
            self.gather_all = [torch.zeros(self.world, g1 - g0, 3, **f32) for g0, g1 in self.bounds]
            self.campos_in = torch.zeros(3, **f32)
            self.campos_all = torch.zeros(self.world, 3, **f32)
            self.shs = torch.zeros(self.n, self.M, 3, **f32)
        elif len(self.bounds) == 1:
            self.shs = self.chunk_views[0]["shs"].view(self.n, self.M, 3)
        else:
            self.shs = None  # materialised by `grads`
        self._pending: List[tuple] = []
        self._campos_work = None
        self._materialised: Optional[Dict[str, torch.Tensor]] = None
        self._stats_synced = False  # sync_densify_stats has reduced the statistics since the last reset

    @property
    def chunks(self) -> int:
        return len(self.bounds)

    # ---- destinations ----
    def backward_out(self) -> Dict[str, torch.Tensor]:
        """Whole-range destinations for backward_raw(out=..., accumulate_stats=True) (chunks == 1 only)."""
        if self.chunks != 1:
            raise RuntimeError("backward_out() is the unchunked form; use chunk_outputs() with backward_chunked")
        self._check_not_synced()
        v = self.chunk_views[0]
        out = dict(means3D=v["means3D"], scales=v["scales"], rotations=v["rotations"], opacities=v["opacities"],
                   means2D=self.means2D, densify_stats=self.stats_accum, max_radii2D=self.radii_max)
        if self.compact:
            out["colors_sh"] = self.gather_in[0]
        else:
            out["shs"] = self.shs
        return out

    def backward_kwargs(self) -> Dict[str, object]:
        """Keyword arguments of backward_raw for this reducer (chunks == 1): the destinations, the SH mode and
        accumulate_stats=True -- the statistics destinations are running sums over views and steps, so a plain
        backward_out() with accumulate_stats left False would overwrite them."""
        return dict(out=self.backward_out(), compact_sh=self.compact, accumulate_stats=True)

    def chunk_outputs(self) -> List[Tuple[int, int, Dict[str, torch.Tensor]]]:
        """(g_begin, g_end, destinations) per chunk, for rasterizer.backward_chunked."""
        self._check_not_synced()
        res = []
        for c, (g0, g1) in enumerate(self.bounds):
            v = self.chunk_views[c]
            out = dict(means3D=v["means3D"], scales=v["scales"], rotations=v["rotations"], opacities=v["opacities"],
                       means2D=self.means2D[g0:g1], densify_stats=self.stats_accum[g0:g1],
                       max_radii2D=self.radii_max[g0:g1])
            if self.compact:
                out["colors_sh"] = self.gather_in[c]
            else:
                out["shs"] = v["shs"]
            res.append((g0, g1, out))
        return res

    def record_view(self, dmeans2D: torch.Tensor, radii: torch.Tensor) -> None:
        """Accumulate one view's densification statistics (gaussian_model.py:175-181) when the backward did not
        (backward_raw without backward_out()'s densify_stats / max_radii2D)."""
        self._check_not_synced()
        self.stats_accum[:, 0] += torch.linalg.vector_norm(dmeans2D[:, :2], dim=1)
        self.stats_accum[:, 1] += (radii > 0).to(torch.float32)
        torch.maximum(self.radii_max, radii.to(torch.int32), out=self.radii_max)

    # ---- exchange ----
    def begin_step(self, campos: torch.Tensor) -> None:
        """Start of a step's exchange: the camera positions of every rank's view (compact mode)."""
        self._check_not_synced()
        self._pending = []
        self._materialised = None
        if not self.compact:
            return
        self.campos_in.copy_(campos.reshape(3))
        if self.distributed:
            self._campos_work = _all_gather(self.campos_all, self.campos_in, self.group)
        else:
            self.campos_all[0].copy_(self.campos_in)
            self._campos_work = None

    def start_chunk(self, c: int) -> None:
        """Chunk c's gradients have been enqueued on the current stream: issue its collectives (async).  The
        all-gather goes first, so the SH expansion that needs it can start while the all-reduce still runs."""
        gather = reduce = None
        if self.distributed:
            if self.compact:
                gather = _all_gather(self.gather_all[c], self.gather_in[c], self.group)
            reduce = dist.all_reduce(self.chunk_flat[c], group=self.group, async_op=True)
        self._pending.append((c, gather, reduce))

    def finish(self, means3D: torch.Tensor) -> None:
        """SH expansion per chunk (after its gather) and the wait for every collective of the step."""
        if self._campos_work is not None:
            self._campos_work.wait()
            self._campos_work = None
        for c, gather, _ in self._pending:
            if not self.compact:
                continue
            if gather is not None:
                gather.wait()
            g0, g1 = self.bounds[c]
            factors = self.gather_all[c] if self.distributed else self.gather_in[c].unsqueeze(0)
            self._sh_views(means3D[g0:g1], self.campos_all, factors, self.D, self.M, out=self.shs[g0:g1])
        for _, _, reduce in self._pending:
            if reduce is not None:
                reduce.wait()
        self._pending = []

    def reduce(self, means3D: torch.Tensor, campos: torch.Tensor) -> None:
        """The whole exchange after an unchunked backward (backward_out()): every chunk at once."""
        self.begin_step(campos)
        for c in range(self.chunks):
            self.start_chunk(c)
        self.finish(means3D)

    def sync_densify_stats(self):
        """SUM the accumulated statistics and MAX the radii over ranks, in place; returns (stats, radii_max):
        stats (n, 2) = [sum of ||dL/dmeans2D[:, :2]||, number of visible views] since the last reset.  Reduces once
        per reset_densify_stats(); accumulating further views before that reset raises (a second reduction would
        count the other ranks' views twice)."""
        if self.distributed and not self._stats_synced:  # idempotent until reset: a second call must not re-add
            work = [dist.all_reduce(self.stats_accum, group=self.group, async_op=True),
                    dist.all_reduce(self.radii_max, op=dist.ReduceOp.MAX, group=self.group, async_op=True)]
            for w in work:
                w.wait()
        self._stats_synced = True
        return self.stats_accum, self.radii_max

    def _check_not_synced(self) -> None:
        if self._stats_synced and self.distributed:
            raise RuntimeError("densification statistics were reduced over ranks (sync_densify_stats); call "
                               "reset_densify_stats() before accumulating more views")

    def reset_densify_stats(self) -> None:
        """After densifying (the reference zeroes xyz_gradient_accum, denom and max_radii2D there)."""
        self.stats_accum.zero_()
        self.radii_max.zero_()
        self._stats_synced = False

    @property
    def grads(self) -> Dict[str, torch.Tensor]:
        """Per-field (n, w) gradients: views of the exchange buffer with one chunk, else gathered from the chunk
        blocks once per step (one copy of 11 (compact) / 59 (dense) floats per Gaussian)."""
        if self.chunks == 1:
            v = self.chunk_views[0]
            return dict(means3D=v["means3D"], scales=v["scales"], rotations=v["rotations"],
                        opacities=v["opacities"], shs=self.shs)
        if self._materialised is None:
            m = {k: torch.cat([v[k] for v in self.chunk_views], 0) for k in self.fields}
            m["shs"] = self.shs if self.compact else m["shs"].view(self.n, self.M, 3)
            self._materialised = m
        return dict(self._materialised)

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
