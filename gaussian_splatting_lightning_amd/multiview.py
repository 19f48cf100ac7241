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
            all-gather the 3-float factors dRGB_v (clamp-masked colour gradient) and each rank expands sum_v on the
            GPU (gsr_sh_backward_views_chunked).  The all-reduce carries the other 11 floats, plus one (world, 3)
            block of camera positions (each rank writes its own row, zeros elsewhere: the sum is every rank's
            campos, exactly), so no separate camera gather runs.  Per-rank ring traffic at 8 ranks and SH degree 3:
            2*(7/8)*44 B + (7/8)*96 B = 161 B per Gaussian instead of 2*(7/8)*236 B = 413 B.

``sharded`` (ZeRO-style: every Gaussian's reduced gradient is needed on ONE rank, its owner, which runs the optimizer
            for its shard and all-gathers the updated parameters): the 11 non-SH floats go in one reduce-scatter
            (rank r receives the sum over views for its Gaussian shard [r S, (r + 1) S)), and the colour factors in
            one all-to-all (rank r receives every view's factors for its shard only), plus the cameras in the
            reduce-scatter group.  Per-rank traffic at 8 ranks: (7/8)*(44 + 12) B = 49 B per Gaussian; the SH
            expansion (or the fused SH Adam) covers the shard only.  The training step then all-gathers the updated
            parameters, (7/8)*236 B per Gaussian, instead of every rank running the whole optimizer.

Overlap with the backward (``chunks`` = K > 1): the Gaussians are split into K contiguous ranges and the
gradient buffer is laid out chunk-major -- chunk c's block holds [means3D | scales | rotations | opacity (| shs)]
of its Gaussians only -- so a chunk's exchange is ONE all-reduce (+ one all-gather of its colour factors), issued
as one RCCL group (ncclGroupStart/End through the process group's coalescing calls) as soon as chunk c is
enqueued, on the reducer's side stream behind an event on the compute stream, so it runs while the GPU computes
chunk c + 1.  (With one chunk the group is issued blocking on the compute stream itself: no hand-off.)  The SH
expansion runs per chunk as
each group lands (``expand="chunk"``), or once over the chunk-major gather buffer after the last one
(``expand="once"``).  Results are bitwise those of K = 1: every element is the same sum of the same per-rank values
(tests/test_multiview.py checks K = 1 against K = 4 on world_size 2).

``plan_exchange`` picks the mode, K and the expansion schedule from a cost model (measured per-Gaussian kernel
times, the measured fixed cost of one collective group, an assumed xGMI bus bandwidth) and predicts the step.

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
NON_SH_FLOATS = 11  # means3D 3 + scales 3 + rotations 4 + opacity 1

# Cost-model constants, measured on one MI355X at cfg 3 (1M Gaussians, SH degree 3) with a one-rank RCCL group
# (tools/dist_overhead.py, interleaved rounds, and its rocprofv3 kernel trace split into steps by tools/trace_steps.py;
# profiles/r6c_*): kernel times per 1e6 Gaussians, and the GPU-timeline cost of the stream hand-offs -- a blocking
# group on the compute stream (K = 1: the gap before the next kernel), and for K > 1 chunks the extra chunk's launches
# with its event record (each event marker holds the next kernel ~6 us) plus one fixed cross-stream hand-off (the
# compute stream's waits for the side stream's events).  Fitted to the one-rank steps: compact K = 1 / 2 / 4 at
# +20 / +54 / +81 us over the plain step.  The bus bandwidth is an ASSUMPTION (no 8-GPU node has run this code): 7 xGMI
# links x 153 GB/s per direction at `bus_efficiency` of RCCL's ring schedules.
EXCHANGE_COSTS = dict(
    pb_dense_ms=0.104,       # preprocess_bwd writing dL/dsh (192 B/G)
    pb_compact_ms=0.080,     # preprocess_bwd writing the 12-B colour factor instead
    exp_ms=0.036,            # gsr_sh_backward_views: 192 B/G written + means + one view's factors
    exp_view_ms=0.002,       # + 12 B/G read per further view
    group_sync_ms=0.008,     # one blocking collective group on the compute stream (K = 1)
    chunk_ms=0.0135,         # per extra chunk: per-Gaussian and expansion launches + the chunk's event hand-off
    side_fixed_ms=0.0205,    # K > 1: the compute stream's waits for the side stream
    sharded_fixed_ms=0.030,  # sharded: the camera rows' fill and two blocking ops (reduce-scatter group, all-to-all),
                             # ~12 us of compute-queue gap each in the one-rank trace (profiles/r6z_*)
    link_GBps=153.0,
    links=7,
    bus_efficiency=0.6,
)


def exchange_bytes_per_gaussian(mode: str, world: int, M: int = 16) -> float:
    """Per-rank bytes over the links per Gaussian for one step's exchange (ring algorithms: all-reduce 2(N-1)/N of
    the buffer, all-gather (N-1)/N of the gathered output)."""
    N = max(1, int(world))
    if mode == "dense":
        return 2.0 * (N - 1) / N * 4 * (NON_SH_FLOATS + 3 * M)
    if mode == "sharded":  # reduce-scatter of the 11 floats + all-to-all of the 3-float factors
        return (N - 1) / N * (4 * NON_SH_FLOATS + 12.0)
    return 2.0 * (N - 1) / N * 4 * NON_SH_FLOATS + (N - 1) / N * 12.0 * N


def simulate_exchange(n: int, world: int, mode: str, chunks: int, expand: str = "chunk", M: int = 16,
                      costs: Optional[dict] = None) -> Dict[str, float]:
    """Timeline of the backward's per-Gaussian stage + the exchange (ms after the compositing backward ends).

    K = 1: the group runs blocking on the compute stream after the per-Gaussian stage, then the SH expansion.
    K > 1: the compute stream runs K per-Gaussian chunks; the side stream runs chunk k's group once chunk k is done and
    group k - 1 has finished (the links are the bottleneck); the SH expansion (compact) follows each landed chunk on the
    compute stream ("chunk"), or all of it after the last ("once"; "side" is modelled as "chunk": measured alike).
    The hand-offs cost chunk_ms per extra chunk and side_fixed_ms once (EXCHANGE_COSTS)."""
    c = dict(EXCHANGE_COSTS, **(costs or {}))
    scale = n / 1e6
    K = max(1, int(chunks))
    N = max(1, int(world))
    pb = (c["pb_dense_ms"] if mode == "dense" else c["pb_compact_ms"]) * scale
    bus = c["link_GBps"] * c["links"] * c["bus_efficiency"] * 1e9  # B/s
    link_bytes = exchange_bytes_per_gaussian(mode, N, M) * n
    comm = link_bytes / bus * 1e3 if N > 1 else 0.0  # one rank: in-place collectives move nothing
    exp = (c["exp_ms"] + c["exp_view_ms"] * (N - 1)) * scale if mode != "dense" else 0.0
    if mode == "sharded":  # K = 1: the reduce-scatter group and the all-to-all, then the shard's expansion
        exp /= N
        end = pb + c["sharded_fixed_ms"] + comm + exp
        return {"mode": mode, "chunks": 1, "expand": "once", "per_gaussian_stage_ms": round(pb, 4),
                "link_MB": round(link_bytes / 1e6, 1), "comm_ms": round(comm, 4), "end_ms": round(end, 4),
                "exposed_ms": round(end - pb, 4)}
    if K == 1:
        end = pb + c["group_sync_ms"] + comm + exp
    else:
        comp_end = comm_end = 0.0
        landed = []
        for k in range(K):
            comp_end += pb / K + (c["chunk_ms"] if k > 0 else 0.0)
            comm_end = max(comp_end, comm_end) + comm / K
            landed.append(comm_end)
        t = comp_end + c["side_fixed_ms"]
        if exp and expand == "once":
            t = max(t, landed[-1]) + exp
        elif exp:
            for k in range(K):
                t = max(t, landed[k]) + exp / K
        end = max(t, comm_end + c["side_fixed_ms"])
    return {"mode": mode, "chunks": K, "expand": expand, "per_gaussian_stage_ms": round(pb, 4),
            "link_MB": round(link_bytes / 1e6, 1), "comm_ms": round(comm, 4), "end_ms": round(end, 4),
            "exposed_ms": round(end - pb, 4)}


def plan_exchange(n: int, world: int, M: int = 16, costs: Optional[dict] = None,
                  modes=("compact", "dense", "sharded"), chunk_options=(1, 2, 4, 8),
                  margin: float = 0.15) -> Dict[str, float]:
    """The (mode, chunks, expand) with the smallest predicted end time -- but the fewest chunks whose prediction is
    within `margin` (relative) of the best: every extra chunk's hand-offs are measured costs, while the overlap they
    buy rests on the ASSUMED bus bandwidth (ties: fewer chunks, compact first)."""
    cands = []
    for mode in modes:
        for K in chunk_options:
            if K > 1 and (n < 256 * K or mode == "sharded"):
                continue
            for expand in (("chunk", "once") if (mode == "compact" and K > 1) else ("once",)):
                cands.append(simulate_exchange(n, world, mode, K, expand, M, costs))
    best = min(c["end_ms"] for c in cands)
    ok = [c for c in cands if c["end_ms"] <= best * (1.0 + margin) + 1e-9]
    return min(ok, key=lambda c: (c["chunks"], c["end_ms"]))


def chunk_bounds(n: int, k: int, align: int = 256) -> List[Tuple[int, int]]:
    """K contiguous Gaussian ranges covering [0, n), boundaries on multiples of `align` (whole preprocess blocks).
    Every range but the last has the same length (the chunk-major gather layout relies on it)."""
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

    mode="sharded" (and mode="auto" when the cost model picks it): ``grads`` and ``sh_views_gradient`` cover only this
    rank's shard ``self.shard`` = [g0, g1); the caller steps those rows of its parameters (padded to
    ``padded_rows()``) and calls ``gather_shards(params)``; ``reduce`` takes this view's campos.

    mode="auto" / chunks=None take ``plan_exchange``'s choice for this world size.  coalesce (default: on for the
    nccl backend) issues a chunk's all-gather and all-reduce as one RCCL group; sync_ops (default: on when there is
    one chunk) issues them as blocking ops, which torch's RCCL process group enqueues on the current stream -- with
    nothing to overlap, that saves the hand-off to the communication stream and back.
    """

    def __init__(self, n: int, M: int, sh_degree: int, device, mode: str = "compact", group=None,
                 world_size: Optional[int] = None,
                 sh_views_fn: Optional[Callable[..., torch.Tensor]] = None, chunks: Optional[int] = 1,
                 distributed: Optional[bool] = None, expand: Optional[str] = None,
                 coalesce: Optional[bool] = None, sync_ops: Optional[bool] = None, comm_stream: Optional[str] = None,
                 plan_world: Optional[int] = None, handoff: Optional[str] = None,
                 one_group: Optional[bool] = None):
        if mode not in ("dense", "compact", "sharded", "auto"):
            raise ValueError(f"mode must be 'dense', 'compact', 'sharded' or 'auto', got {mode!r}")
        self.n, self.M, self.D = int(n), int(M), int(sh_degree)
        self.device = torch.device(device)
        self.group = group
        # Collectives run whenever a process group exists, even of one rank (the RCCL code path then executes on a
        # single GPU exactly as it does on eight); distributed=False keeps a reducer local inside a process group.
        if distributed is None:
            distributed = bool(dist.is_available() and dist.is_initialized())
        self.distributed = bool(distributed)
        self.world = int(world_size if world_size is not None else
                         (dist.get_world_size(group) if self.distributed else 1))
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.plan = None
        if mode == "auto" or chunks is None:
            # plan_world: plan for that many ranks (a one-rank rehearsal of the N-GPU schedule, bench.py --plan-world)
            self.plan = plan_exchange(self.n, int(plan_world or self.world), self.M,
                                      modes=("compact", "dense", "sharded") if mode == "auto" else (mode,),
                                      chunk_options=(1, 2, 4, 8) if chunks is None else (int(chunks),))
            mode = self.plan["mode"]
            chunks = self.plan["chunks"]
            if expand is None:
                expand = self.plan["expand"]
        self.mode = mode
        self.sharded = mode == "sharded"
        if self.sharded and chunks not in (None, 1):
            raise ValueError("the sharded exchange runs unchunked (chunks=1)")
        self.compact = mode == "compact"
        self.expand = expand or "chunk"
        if self.expand not in ("chunk", "once", "side"):
            raise ValueError(f"expand must be 'chunk', 'once' or 'side', got {self.expand!r}")
        self._sh_views = sh_views_fn or sh_backward_views
        self.widths = dict(means3D=3, scales=3, rotations=4, opacities=1, shs=3 * self.M)
        self.fields = FIELDS_DENSE if mode == "dense" else FIELDS_COMPACT
        cols = sum(self.widths[k] for k in self.fields)
        f32 = dict(dtype=torch.float32, device=self.device)
        if self.sharded:
            self._init_sharded(cols, f32, coalesce, one_group)
            return
        self.bounds = chunk_bounds(self.n, chunks)
        self.chunk_len = self.bounds[0][1] - self.bounds[0][0]
        # compact: chunk 0's all-reduce block ends with a (world, 3) camera-position block
        cam_floats = 3 * self.world if self.compact else 0
        # chunk-major blocks, each [field][Gaussian of the chunk][width]: every destination is a contiguous view
        self.flat = torch.zeros(cols * self.n + cam_floats, **f32)
        self.chunk_flat: List[torch.Tensor] = []
        self.chunk_views: List[Dict[str, torch.Tensor]] = []
        off = 0
        for c, (g0, g1) in enumerate(self.bounds):
            L = g1 - g0
            extra = cam_floats if c == 0 else 0
            blk = self.flat[off:off + cols * L + extra]
            views, o = {}, 0
            for k in self.fields:
                w = self.widths[k]
                views[k] = blk[o * L:(o + w) * L].view(L, w)
                o += w
            self.chunk_flat.append(blk)
            self.chunk_views.append(views)
            off += cols * L + extra
        self.means2D = torch.zeros(self.n, 3, **f32)
        # densification statistics of this rank's views since the last reset (local until sync_densify_stats)
        self.stats_accum = torch.zeros(self.n, 2, **f32)
        self.radii_max = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        if self.compact:
            L0 = self.bounds[0][1] - self.bounds[0][0]
            self.campos_all = self.chunk_flat[0][NON_SH_FLOATS * L0:].view(self.world, 3)
            self._campos_onehot = torch.zeros(self.world, 1, **f32)
            self._campos_onehot[self.rank, 0] = 1.0
            # everyone's colour factors, chunk-major: chunk c = (world, L_c, 3); this rank's (L_c, 3) factors are its
            # row of the gathered block, written there by the backward (an in-place all-gather: nothing to copy)
            self.gather_all_flat = torch.zeros(self.world * self.n * 3, **f32)
            self.gather_all = [self.gather_all_flat[3 * self.world * g0:3 * self.world * g1].view(self.world, g1 - g0, 3)
                               for g0, g1 in self.bounds]
            self.gather_in = [blk[self.rank] for blk in self.gather_all]
            self.shs = torch.zeros(self.n, self.M, 3, **f32)
        elif len(self.bounds) == 1:
            self.shs = self.chunk_views[0]["shs"].view(self.n, self.M, 3)
        else:
            self.shs = None  # materialised by `grads`
        nccl = self.distributed and dist.get_backend(group) == "nccl"
        self.coalesce = nccl if coalesce is None else (bool(coalesce) and nccl)
        # decided once, before any group starts: a group that failed half-way could not be re-issued safely (the
        # process group would flush the ops queued before the failure and the fallback would issue them again)
        if self.coalesce and not _coalescing_supported(self._pg()):
            self.coalesce = False
        self.one_group = False  # (sharded exchange only)
        self.sync_ops = (self.chunks == 1) if sync_ops is None else bool(sync_ops)
        # comm_stream="side" (chunked exchange on a HIP device): the reducer's own stream carries the
        # collectives as blocking ops behind one event per chunk, and the compute stream waits for chunk c's group
        # only before chunk c's SH expansion.  torch's RCCL process group otherwise runs async ops on its pool stream,
        # which can share the compute stream's hardware queue (then the chunks serialise behind each hand-off).
        self.comm_stream = None
        if comm_stream not in (None, "pg", "side"):
            raise ValueError(f"comm_stream must be 'pg' or 'side', got {comm_stream!r}")
        if comm_stream is None:  # measured (one rank, 4 chunks): side 0.901 ms/step against 0.923 for the pg stream
            comm_stream = "side" if self.chunks > 1 else "pg"
        # handoff between the two streams: "event" (hipEvent record / wait) or "value" (a device word written and
        # waited on in stream order, gsr_stream_signal / gsr_stream_wait: no event marker on the compute stream)
        self.handoff = None
        if handoff not in (None, "event", "value"):
            raise ValueError(f"handoff must be 'event' or 'value', got {handoff!r}")
        if comm_stream == "side" and self.distributed and self.device.type == "cuda":
            self.comm_stream = torch.cuda.Stream(self.device)
            self.handoff = handoff or "event"
            if self.handoff == "value":
                from . import _native
                with torch.cuda.device(self.device):
                    if not _native.load().gsr_stream_values_supported():
                        self.handoff = "event"
            if self.handoff == "value":
                # [ready(c) for c] + [landed(c) for c]: step s signals s (monotone, never reset)
                self._flags = torch.zeros(2 * len(self.bounds), dtype=torch.int32, device=self.device)
                self._seq = 0
            else:
                self._ready = [torch.cuda.Event() for _ in self.bounds]   # chunk c's gradients are written
                self._landed = [torch.cuda.Event() for _ in self.bounds]  # chunk c's collectives are done
            self.sync_ops = True
        self._pending: List[tuple] = []
        self._side_means: Optional[torch.Tensor] = None  # begin_step(means3D=...): expansions on the side stream
        self._expanded: set = set()
        # who writes this step's camera block (compact): "backward" once backward_out()/chunk_outputs() handed
        # campos_rows to the backward, "begin_step" when the caller passed campos; finish() refuses a step with
        # neither (the block would still hold the previous step's all-reduced cameras, summed again)
        self._camera_source: Optional[str] = None
        self._sh_expanded = True  # finish(expand_sh=False) leaves dL/dshs in factored form (sh_views_gradient)
        self._materialised: Optional[Dict[str, torch.Tensor]] = None
        self._stats_synced = False  # sync_densify_stats has reduced the statistics since the last reset

    def _init_sharded(self, cols: int, f32: dict, coalesce: Optional[bool], one_group: Optional[bool]) -> None:
        """Buffers of the sharded exchange: the backward writes the full (n, w) gradient fields (padded to N S rows)
        and the (n, 3) colour factors; each field is reduce-scattered to its (S, w) shard, the factors go through one
        all-to-all into (N, S, 3), and the cameras ride in the reduce-scatter group as an (N, N, 3) block whose block j
        holds every rank's camera in its own row (block j's sum, rank j's share, is every camera)."""
        N, n = self.world, self.n
        S = max(256, -(-(-(-n // N)) // 256) * 256)
        self.shard_len = S
        self.shard = (min(n, self.rank * S), min(n, self.rank * S + S))
        L = self.shard[1] - self.shard[0]
        Np = N * S
        self.bounds = [(0, n)]
        self.chunk_len = n
        self.flat = torch.zeros(cols * Np, **f32)
        self.full: Dict[str, torch.Tensor] = {}
        self.shard_views: Dict[str, torch.Tensor] = {}
        self.shard_flat = torch.zeros(cols * S, **f32)
        o = 0
        for k in self.fields:
            w = self.widths[k]
            self.full[k] = self.flat[o * Np:(o + w) * Np].view(Np, w)
            self.shard_views[k] = self.shard_flat[o * S:(o + w) * S].view(S, w)
            o += w
        self.chunk_flat = [self.flat]
        self.chunk_views = [{k: v[:n] for k, v in self.full.items()}]
        self.cam_rs = torch.zeros(N * N * 3, **f32)
        self.campos_all = torch.zeros(N, 3, **f32)
        self.colors = torch.zeros(Np, 3, **f32)
        self.factors_all = torch.zeros(N, S, 3, **f32)
        self.shs = torch.zeros(L, self.M, 3, **f32)
        self.means2D = torch.zeros(n, 3, **f32)
        self.stats_accum = torch.zeros(n, 2, **f32)
        self.radii_max = torch.zeros(n, dtype=torch.int32, device=self.device)
        nccl = self.distributed and dist.get_backend(self.group) == "nccl"
        self.coalesce = nccl if coalesce is None else (bool(coalesce) and nccl)  # the reduce-scatters as one group
        self.one_group = self.coalesce and (True if one_group is None else bool(one_group))  # + the all-to-all
        self.sync_ops = True
        self.comm_stream = None
        self.handoff = None
        self._pending = []
        self._side_means = None
        self._expanded = set()
        self._camera_source = None
        self._sh_expanded = True
        self._materialised = None
        self._stats_synced = False

    def _sharded_exchange(self, means3D: torch.Tensor, campos: Optional[torch.Tensor], expand_sh: bool) -> None:
        if campos is None:
            raise RuntimeError("sharded exchange: pass this view's campos to reduce() (it rides in the reduce-scatter)")
        N, S = self.world, self.shard_len
        self.cam_rs.view(N, N, 3)[:, self.rank].copy_(campos.reshape(1, 3).to(torch.float32).expand(N, 3))
        pairs = [(self.shard_views[k], self.full[k]) for k in self.fields]
        pairs.append((self.campos_all, self.cam_rs))
        if not self.distributed:  # one rank without a group: the shard is everything
            for out, inp in pairs:
                out.copy_(inp.view_as(out))
            self.factors_all.view(-1).copy_(self.colors.view(-1))
        else:
            if self.coalesce:
                # torch's coalesced fast path (reduce_scatter_tensor_coalesced, one RCCL group; FSDP's path); with
                # one_group the all-to-all is issued inside the process group's own coalescing block too, so the
                # reduce-scatters and it leave as ONE RCCL group (one launch, one hand-off to the compute stream)
                dev = self.device if self.one_group else None
                with dist.distributed_c10d._coalescing_manager(group=self.group, device=dev):
                    for out, inp in pairs:
                        dist.reduce_scatter_tensor(out.view(-1), inp.reshape(-1), group=self.group)
                    if self.one_group:
                        dist.all_to_all_single(self.factors_all.view(-1), self.colors.view(-1), group=self.group)
            else:
                for out, inp in pairs:
                    dist.reduce_scatter_tensor(out.view(-1), inp.reshape(-1), group=self.group)
            if not (self.coalesce and self.one_group):
                dist.all_to_all_single(self.factors_all.view(-1), self.colors.view(-1), group=self.group)
        self._sh_expanded = bool(expand_sh)
        if expand_sh and self.shs.shape[0] > 0:
            g0, g1 = self.shard
            self._sh_views(means3D[g0:g1], self.campos_all, self._shard_factors(), self.D, self.M, out=self.shs,
                           chunk_len=0)

    def padded_rows(self) -> int:
        """Rows of a parameter tensor the sharded training step all-gathers in place (N S >= n; the rasterizer reads
        the first n)."""
        return self.world * self.shard_len if self.sharded else self.n

    def gather_shards(self, tensors) -> None:
        """Sharded training step, after this rank's optimizer stepped its shard: every rank's updated rows to every
        rank, in place, for tensors of padded_rows() rows (one coalesced RCCL all-gather group)."""
        if not self.sharded:
            raise RuntimeError("gather_shards: only the sharded exchange leaves the parameters sharded")
        if not self.distributed:
            return
        S, r = self.shard_len, self.rank
        for t in tensors:
            if t.shape[0] != self.padded_rows() or not t.is_contiguous():
                raise ValueError("gather_shards: contiguous tensors of padded_rows() rows expected")
        if self.coalesce:  # torch's coalesced fast path (allgather_into_tensor_coalesced): one RCCL group
            with dist.distributed_c10d._coalescing_manager(group=self.group):
                for t in tensors:
                    dist.all_gather_into_tensor(t.view(-1), t[r * S:(r + 1) * S].reshape(-1), group=self.group)
        else:  # gloo has no in-place form
            for t in tensors:
                dist.all_gather_into_tensor(t.view(-1), t[r * S:(r + 1) * S].reshape(-1).clone(), group=self.group)

    def _shard_factors(self) -> torch.Tensor:
        """(N, L, 3) every view's colour factors of this rank's L Gaussians (a copy only for a short last shard)."""
        L = self.shard[1] - self.shard[0]
        f = self.factors_all
        return f if L == self.shard_len else f[:, :L].contiguous()

    @property
    def chunks(self) -> int:
        return len(self.bounds)

    def describe(self) -> str:
        if self.sharded:
            return (f"sharded (reduce-scatter of 11 floats + cameras{' as one group' if self.coalesce else ''}, "
                    f"all-to-all of the colour factors; this rank owns Gaussians [{self.shard[0]}, {self.shard[1]}))")
        return (f"{self.mode}, {self.chunks} chunk(s), expand={self.expand if self.compact else '-'}, "
                f"{'one RCCL group per chunk' if self.coalesce else 'separate collectives'}, "
                f"{'blocking' if self.sync_ops else 'async'} ops"
                f"{f' on a side stream ({self.handoff} hand-off)' if self.comm_stream is not None else ''}")

    # ---- destinations ----
    def backward_out(self) -> Dict[str, torch.Tensor]:
        """Whole-range destinations for backward_raw(out=..., accumulate_stats=True) (chunks == 1 only)."""
        if self.chunks != 1:
            raise RuntimeError("backward_out() is the unchunked form; use chunk_outputs() with backward_chunked")
        self._check_not_synced()
        v = self.chunk_views[0]
        out = dict(means3D=v["means3D"], scales=v["scales"], rotations=v["rotations"], opacities=v["opacities"],
                   means2D=self.means2D, densify_stats=self.stats_accum, max_radii2D=self.radii_max)
        if self.sharded:
            out["colors_sh"] = self.colors[:self.n]
        elif self.compact:
            out["colors_sh"] = self.gather_in[0]
            out["campos_rows"] = (self.campos_all, self.rank)
            self._camera_source = "backward"
        else:
            out["shs"] = self.shs
        return out

    def backward_kwargs(self) -> Dict[str, object]:
        """Keyword arguments of backward_raw for this reducer (chunks == 1): the destinations, the SH mode and
        accumulate_stats=True -- the statistics destinations are running sums over views and steps, so a plain
        backward_out() with accumulate_stats left False would overwrite them."""
        return dict(out=self.backward_out(), compact_sh=self.compact or self.sharded, accumulate_stats=True)

    def chunk_outputs(self) -> List[Tuple[int, int, Dict[str, torch.Tensor]]]:
        """(g_begin, g_end, destinations) per chunk, for rasterizer.backward_chunked."""
        if self.sharded:
            raise RuntimeError("the sharded exchange is unchunked: use backward_kwargs() and reduce()")
        self._check_not_synced()
        res = []
        for c, (g0, g1) in enumerate(self.bounds):
            v = self.chunk_views[c]
            out = dict(means3D=v["means3D"], scales=v["scales"], rotations=v["rotations"], opacities=v["opacities"],
                       means2D=self.means2D[g0:g1], densify_stats=self.stats_accum[g0:g1],
                       max_radii2D=self.radii_max[g0:g1])
            if self.compact:
                out["colors_sh"] = self.gather_in[c]
                if c == 0:  # the camera block rides in chunk 0's all-reduce; chunk 0's backward call writes it
                    out["campos_rows"] = (self.campos_all, self.rank)
                    self._camera_source = "backward"
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
    def begin_step(self, campos: Optional[torch.Tensor] = None, means3D: Optional[torch.Tensor] = None,
                   expand_sh: bool = True) -> None:
        """Start of a step's exchange.  The camera block that chunk 0's all-reduce carries (this rank's campos in its
        row, zeros elsewhere) is written by the backward call that receives backward_out() / chunk_outputs()
        ("campos_rows"); a caller whose backward does not (a custom gradient source) passes campos here instead (one
        elementwise launch).

        means3D (expand="side": the side stream, compact mode): each chunk's SH expansion runs on the side stream right
        behind its group, overlapping the compute stream's next chunks, and finish() only waits; expand_sh=False for
        the factored form (see finish).  Without means3D, "side" expands in finish() like "chunk"."""
        self._check_not_synced()
        self._pending = []
        self._materialised = None
        side = self.compact and self.distributed and self.comm_stream is not None and self.expand == "side"
        self._side_means = means3D if (side and expand_sh and means3D is not None) else None
        self._expanded = set()
        if self.compact and campos is not None:
            torch.mul(self._campos_onehot, campos.reshape(1, 3).to(self.campos_all.dtype), out=self.campos_all)
            self._camera_source = "begin_step"

    def _check_camera_block(self) -> None:
        if self._camera_source is None:
            raise RuntimeError("compact exchange: nothing wrote this step's camera block -- pass the destinations of "
                               "backward_out()/chunk_outputs() to the backward, or campos to begin_step()/reduce()")

    def _pg(self):
        return self.group if self.group is not None else dist.distributed_c10d._get_default_group()

    def _issue(self, c: int):
        """Chunk c's collectives: (gather work, reduce work); None for a completed blocking op."""
        if self.coalesce:
            return self._issue_group(c)
        gather = None
        if self.compact:
            gather = _all_gather(self.gather_all[c], self.gather_in[c], self.group, not self.sync_ops)
        reduce = dist.all_reduce(self.chunk_flat[c], group=self.group, async_op=not self.sync_ops)
        return gather, reduce

    def _issue_group(self, c: int):
        """One ncclGroupStart/End around the chunk's all-gather and all-reduce (torch's _coalescing_manager only
        coalesces collectives of one kind, so the process group's coalescing calls are used directly)."""
        pg = self._pg()
        asynchronous = not self.sync_ops
        pg._start_coalescing(self.device)
        try:
            if self.compact:
                go = dist.distributed_c10d.AllgatherOptions()
                go.asyncOp = asynchronous
                pg._allgather_base(self.gather_all[c].view(-1), self.gather_in[c].reshape(-1), go)
            ro = dist.AllreduceOptions()
            ro.reduceOp = dist.ReduceOp.SUM
            ro.asyncOp = asynchronous
            pg.allreduce([self.chunk_flat[c]], ro)
        finally:
            work = pg._end_coalescing(self.device)
        if not asynchronous:
            if work is not None:
                work.wait()
            return None, None
        return work, work

    def start_chunk(self, c: int) -> None:
        """Chunk c's gradients have been enqueued on the current stream: issue its collectives (one group, or the
        all-gather first, so the SH expansion that needs it can start while the all-reduce still runs)."""
        if self.sharded:
            raise RuntimeError("the sharded exchange is unchunked: use backward_kwargs() and reduce()")
        if c == 0 and self.compact:
            self._check_camera_block()  # before chunk 0's all-reduce sums the camera block
        gather = reduce = None
        if self.distributed and self.comm_stream is not None:
            cur = torch.cuda.current_stream(self.device)
            value = self.handoff == "value"
            if value:
                from . import _native
                lib = _native.load()
                if c == 0:
                    self._seq = (self._seq + 1) & 0x7FFFFFFF
                ready = self._flags[c:c + 1].data_ptr()
                landed = self._flags[len(self.bounds) + c:len(self.bounds) + c + 1].data_ptr()
                _native.check(lib.gsr_stream_signal(cur.cuda_stream, ready, self._seq), "gsr_stream_signal")
            else:
                self._ready[c].record(cur)
            with torch.cuda.stream(self.comm_stream):
                if value:
                    _native.check(lib.gsr_stream_wait(self.comm_stream.cuda_stream, ready, self._seq),
                                  "gsr_stream_wait")
                else:
                    self.comm_stream.wait_event(self._ready[c])
                self._issue(c)  # blocking ops: they run on the side stream itself
                if self._side_means is not None:  # the SH expansion behind the group, off the compute stream
                    g0, g1 = self.bounds[c]
                    self._expand(self._side_means, g0, g1, self.gather_all[c], 0)
                    self._expanded.add(c)
                if value:
                    _native.check(lib.gsr_stream_signal(self.comm_stream.cuda_stream, landed, self._seq),
                                  "gsr_stream_signal")
                else:
                    self._landed[c].record(self.comm_stream)
            gather = reduce = (_StreamValueWork(landed, self._seq, self.device) if value else
                               _StreamEventWork(self._landed[c], self.device))
        elif self.distributed:
            gather, reduce = self._issue(c)
        self._pending.append((c, gather, reduce))

    def _expand(self, means3D: torch.Tensor, g0: int, g1: int, factors: torch.Tensor, chunk_len: int) -> None:
        self._sh_views(means3D[g0:g1], self.campos_all, factors, self.D, self.M, out=self.shs[g0:g1],
                       chunk_len=chunk_len)

    def finish(self, means3D: torch.Tensor, expand_sh: bool = True) -> None:
        """SH expansion (per chunk after its gather, or once after the last) and the wait for every collective.

        expand_sh=False (compact mode): no expansion -- the optimizer takes the SH gradient in factored form
        (sh_views_gradient() with GaussianAdam.step(sh_views=...), which forms it inside the update); grads["shs"] is
        then None for this step.

        Every work object is waited exactly once: a chunk's gather and reduce are often ONE object (a coalesced group,
        or the side stream's event), and dense mode has no gather to wait on, so each is tracked by identity."""
        waited = set()

        def wait(w) -> None:
            if w is not None and id(w) not in waited:
                waited.add(id(w))
                w.wait()

        if self.compact and self._pending:
            self._check_camera_block()
            todo = [c for c, _, _ in self._pending if c not in self._expanded] if expand_sh else []
            if todo:
                wait(self._pending[0][2])  # the camera block rides in chunk 0's all-reduce
            for c, gather, _ in self._pending:
                if c not in todo:
                    continue
                wait(gather)
                if self.expand != "once" or self.chunks == 1:
                    g0, g1 = self.bounds[c]
                    self._expand(means3D, g0, g1, self.gather_all[c], 0)
            if todo and self.expand == "once" and self.chunks > 1:
                self._expand(means3D, 0, self.n, self.gather_all_flat, self.chunk_len)
        self._sh_expanded = expand_sh or not self.compact
        if self.comm_stream is not None and self._pending:
            # the side stream runs every chunk's group (and expansion) in order: its last event covers them all
            wait(self._pending[-1][2])
            waited.update(id(w) for _, g, r in self._pending for w in (g, r))
        for _, gather, reduce in self._pending:
            wait(gather)
            wait(reduce)
        self._pending = []
        self._camera_source = None

    def reduce(self, means3D: torch.Tensor, campos: Optional[torch.Tensor] = None, expand_sh: bool = True) -> None:
        """The whole exchange after an unchunked backward (backward_out()): every chunk at once.  campos: only when
        the backward did not write the camera block (see begin_step); the sharded exchange always takes it here."""
        if self.sharded:
            self._check_not_synced()
            self._materialised = None
            self._sharded_exchange(means3D, campos, expand_sh)
            return
        self.begin_step(campos)
        for c in range(self.chunks):
            self.start_chunk(c)
        self.finish(means3D, expand_sh)

    def sh_views_gradient(self, means3D: torch.Tensor):
        """The step's summed SH gradient in factored form (compact mode, after finish()): every rank's colour factors
        (the chunk-major gather buffer) and cameras, for GaussianAdam.step(sh_views=(features_dc, features_rest,
        this)), which expands it inside the update instead of reading a (P, M, 3) gradient."""
        from .optim import ShViewsGradient
        if self.sharded:  # this rank's shard: every view's factors and camera
            g0, g1 = self.shard
            return ShViewsGradient(means3D=means3D[g0:g1].contiguous(), campos=self.campos_all,
                                   factors=self._shard_factors(), sh_degree=self.D, chunk_len=0)
        if not self.compact:
            raise RuntimeError("sh_views_gradient: the dense exchange carries dL/dshs itself")
        return ShViewsGradient(means3D=means3D.contiguous(), campos=self.campos_all, factors=self.gather_all_flat,
                               sh_degree=self.D, chunk_len=self.chunk_len if self.chunks > 1 else 0)

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
        shs = self.shs if self._sh_expanded else None
        if self.sharded:  # this rank's shard [g0, g1) of every field
            L = self.shard[1] - self.shard[0]
            return dict(means3D=self.shard_views["means3D"][:L], scales=self.shard_views["scales"][:L],
                        rotations=self.shard_views["rotations"][:L], opacities=self.shard_views["opacities"][:L],
                        shs=shs)
        if self.chunks == 1:
            v = self.chunk_views[0]
            return dict(means3D=v["means3D"], scales=v["scales"], rotations=v["rotations"],
                        opacities=v["opacities"], shs=shs)
        if self._materialised is None:
            m = {k: torch.cat([v[k] for v in self.chunk_views], 0) for k in self.fields}
            m["shs"] = shs if self.compact else m["shs"].view(self.n, self.M, 3)
            self._materialised = m
        return dict(self._materialised)

    @property
    def stats(self) -> torch.Tensor:
        """(n, 2) accumulated statistics (this rank's until sync_densify_stats, then the global ones)."""
        return self.stats_accum


def _coalescing_supported(pg) -> bool:
    """The process group's coalescing calls and the async flag on both option structs (torch builds differ)."""
    try:
        return (hasattr(pg, "_start_coalescing") and hasattr(pg, "_end_coalescing")
                and hasattr(pg, "_allgather_base")
                and hasattr(dist.distributed_c10d.AllgatherOptions(), "asyncOp")
                and hasattr(dist.AllreduceOptions(), "asyncOp"))
    except Exception:  # noqa: BLE001
        return False


class _StreamEventWork:
    """work.wait() for a collective run on the reducer's side stream: the current stream waits for its event."""

    def __init__(self, event, device):
        self.event, self.device = event, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.event)


class _StreamValueWork:
    """work.wait() for a collective run on the reducer's side stream, value hand-off: the current stream waits until
    the side stream has written the step's sequence number to the chunk's landed word."""

    def __init__(self, flag_ptr: int, value: int, device):
        self.flag_ptr, self.value, self.device = flag_ptr, value, device

    def wait(self):
        from . import _native
        _native.check(_native.load().gsr_stream_wait(torch.cuda.current_stream(self.device).cuda_stream,
                                                     self.flag_ptr, self.value), "gsr_stream_wait")


def unchunk_factors(flat: torch.Tensor, V: int, n: int, chunk_len: int) -> torch.Tensor:
    """(V, n, 3) colour factors from the chunk-major gather layout (test / oracle helper)."""
    if not chunk_len or chunk_len >= n:
        return flat.reshape(V, n, 3)
    parts = []
    for g0 in range(0, n, chunk_len):
        L = min(chunk_len, n - g0)
        parts.append(flat.reshape(-1)[3 * V * g0:3 * V * (g0 + L)].view(V, L, 3))
    return torch.cat(parts, 1)


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group, async_op: bool = True):
    """all_gather into a (world, ...) tensor; gloo lacks the single-tensor form on some builds."""
    if dist.get_backend(group) == "nccl":  # in place: inp is this rank's row of out
        return dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1), group=group, async_op=async_op)
    dist.all_gather(list(out.unbind(0)), inp.clone().view(out.shape[1:]), group=group)
    return None
