"""The 25-step EulerDiscrete denoising loop, MI355X-native and frame-window sharded over GPUs.

Reference: Pose2VideoLongSVDPipeline.__call__ step x window loop
(src/pipelines/pipeline_svd_audio_adapter_motionexp_idembed_vasa_two_ip.py:670-756) with diffusers
0.29.2 EulerDiscreteScheduler (Karras sigmas, v-prediction, continuous timesteps 0.25*ln(sigma);
mirror src/schedulers/scheduling_euler_discrete.py).

Work decomposition. Within a step every window is independent (overlap = 0 gives disjoint frame
sets, pipeline:684-751) and so is every CFG branch until guidance (:731-733). A *unit* is one
(window, CFG branch) pair = one 14-frame UNet batch element. Units are dealt to ranks in contiguous
blocks (N = 112 -> 9 windows x 4 branches = 36 units -> 5/5/5/5/4/4/4/4 over 8 GPUs); each rank runs
its units in as few UNet calls as the kernels' buffer extents allow (6 x 14 frames at 576x1024; the
reference's call is 4 units = 56 frames), then ONE all-gather of the fp32 noise predictions per step (RCCL over xGMI; torch's
"nccl" backend is RCCL on ROCm) gives every rank all branches, and every rank applies guidance +
Euler + window accumulation for all windows (tiny, replicated) so the latent state stays identical
everywhere without a second collective. Frames of one window never split across ranks (temporal
attention and the temporal GroupNorm span the window).

State: latents_all is fp32 token-major (T*h*w, 4) on device for the whole loop (the reference keeps
it in the UNet dtype, pipeline:674-681; fp32 here is strictly more accurate).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch


# ------------------------------------------------------------------------------------------ scheduler
def karras_sigmas(num_inference_steps: int = 25, sigma_min: float = 0.002, sigma_max: float = 700.0,
                  rho: float = 7.0) -> Tuple[List[float], List[float]]:
    """EulerDiscreteScheduler.set_timesteps (use_karras_sigmas, timestep_type='continuous',
    prediction_type='v_prediction'): returns (sigmas[steps+1] with a final 0, timesteps 0.25*ln(sigma))."""
    ramp = np.linspace(0, 1, num_inference_steps)
    min_inv = sigma_min ** (1 / rho)
    max_inv = sigma_max ** (1 / rho)
    sig = torch.from_numpy((max_inv + ramp * (min_inv - max_inv)) ** rho).to(torch.float32)
    ts = [float(0.25 * s.log()) for s in sig]
    return [float(s) for s in sig] + [0.0], ts


# ------------------------------------------------------------------------------------------ planning
def window_frames_raw(T: int, fpb: int, overlap: int, shift: int) -> List[List[int]]:
    """Unwrapped frame indices of every window at a step (pipeline:684-694): start - shift + j."""
    return [[index_start - shift + j for j in range(fpb)] for index_start in range(0, T, fpb - overlap)]


def window_frames(T: int, fpb: int, overlap: int, shift: int) -> List[List[int]]:
    """Frame indices of every window at a step, wrapped mod T (indice_slice, pipeline:687-693)."""
    return [[r % T for r in win] for win in window_frames_raw(T, fpb, overlap, shift)]


def assign_units(n_windows: int, world: int, rank: int, n_branch: int = 4,
                 branches: Optional[Sequence[int]] = None) -> Tuple[List[Tuple[int, int]], int]:
    """Contiguous block of (window, branch) units for ``rank``; also returns the per-rank capacity
    (max units on any rank) used to size the all-gather. ``branches``: the CFG branches evaluated
    (default all ``n_branch``); a branch whose inputs duplicate another's is left out (see
    ``HipBackend.branch_twins``)."""
    br = list(range(n_branch)) if branches is None else list(branches)
    nb = len(br)
    n = n_windows * nb
    cap = math.ceil(n / world)
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    units = [(u // nb, br[u % nb]) for u in range(start, start + count)]
    return units, cap


def unit_owner(n_windows: int, world: int, n_branch: int = 4,
               branches: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """For every global unit u = window*len(branches) + branch position: (rank, slot within that rank)."""
    owners = []
    for r in range(world):
        units, _ = assign_units(n_windows, world, r, n_branch, branches)
        for slot, (w, c) in enumerate(units):
            owners.append((r, slot))
    return owners


def window_twins(frame_eq: Optional[torch.Tensor], frames: Sequence[int], global_twins: dict) -> dict:
    """{branch: earlier branch} for one window: branch c reads branch e's noise prediction when their UNet inputs are
    bitwise equal on every frame of the window (``frame_eq[c, e, f]``, HipBackend.frame_equal). Besides the
    run-wide twins (mode 0: "cond" = "drop vasa"), this finds the windows that lie wholly in the fpb padding frames
    past N: there every CFG branch but the unconditional one carries the same ID embedding and image latents and
    the same uncond audio / VASA pad (pipeline:175-184), so branches 2 and 3 are branch 1's twins in every mode.
    ``frame_eq`` None: the run-wide twins only."""
    if frame_eq is None:
        return dict(global_twins)
    twins = {}
    idx = torch.as_tensor(list(frames), dtype=torch.long)
    for c in range(1, frame_eq.shape[0]):
        for e in range(c):
            if e not in twins and bool(frame_eq[c, e, idx].all()):
                twins[c] = e
                break
    return twins


def step_units(n_windows: int, twins_per_window: Sequence[dict], n_branch: int = 4) -> List[Tuple[int, int]]:
    """The (window, branch) units a step evaluates, window-major: every branch that is not a twin in its window."""
    return [(w, c) for w in range(n_windows) for c in range(n_branch) if c not in twins_per_window[w]]


def split_units(units: Sequence[Tuple[int, int]], world: int, rank: int) -> Tuple[List[Tuple[int, int]], int]:
    """Contiguous block of ``units`` for ``rank`` and the per-rank capacity (the all-gather slot count)."""
    n = len(units)
    cap = math.ceil(n / world)
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return list(units[start:start + count]), cap


def call_splits(n_units: int, max_per_call: int) -> List[Tuple[int, int]]:
    """[start, end) unit ranges: the fewest UNet calls of at most ``max_per_call`` units, sizes
    differing by at most one (5 units, max 4 -> 3 + 2 rather than 4 + 1)."""
    if n_units <= 0:
        return []
    n_calls = -(-n_units // max(1, max_per_call))
    base, extra = divmod(n_units, n_calls)
    out, c0 = [], 0
    for i in range(n_calls):
        c1 = c0 + base + (1 if i < extra else 0)
        out.append((c0, c1))
        c0 = c1
    return out


def gate_masks(gate, face_mask: torch.Tensor, mouth_mask: torch.Tensor, exp_mask: torch.Tensor):
    """ip_adapter_masks for a gate (pipeline:702-711): [1,1] -> [mouth, exp]; [1,0] -> [face, 0];
    [0,1] -> [0, face]."""
    if gate[0] == 1 and gate[1] == 1:
        return [mouth_mask, exp_mask]
    if gate[0] == 1 and gate[1] == 0:
        return [face_mask, torch.zeros_like(face_mask)]
    if gate[0] == 0 and gate[1] == 1:
        return [torch.zeros_like(face_mask), face_mask]
    raise ValueError(f"unsupported gate {gate}")


# ------------------------------------------------------------------------------------------ backend
def _bits_equal(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Per leading index (frame), whether the two tensors' elements are bitwise equal (so -0.0 != +0.0, unlike
    ``==``): the raw bits compared as integers of the element width."""
    it = {2: torch.int16, 4: torch.int32, 8: torch.int64}[a.element_size()]
    n = a.shape[0]
    return (a.reshape(n, -1).view(it) == b.reshape(n, -1).view(it)).all(-1)


def _same_bits(a: torch.Tensor, b: torch.Tensor) -> bool:
    return a.shape == b.shape and a.dtype == b.dtype and bool(_bits_equal(a.reshape(1, -1), b.reshape(1, -1)).all())


class HipBackend:
    """Runs units through the HIP UNet (forward_tokens) and the fused guidance/Euler kernel.
    ``masks`` = (face_mask, mouth_mask, exp_mask), each (1, 1, H_px, W_px) (pipeline:636-646)."""

    def __init__(self, unet, H: int, W: int, masks, gate, added_time_ids: torch.Tensor, T: int, fpb: int,
                 image_latents, image_embeddings, audio_prompts, vasa_prompts, pose_fea):
        from . import ops
        self.ops = ops
        self.unet = unet
        dev = unet.device
        self.dev = dev
        self.H, self.W, self.S = H, W, H * W
        self.T, self.F = T, fpb
        self.masks = gate_masks(gate, *masks)
        self.gate = list(gate)
        # run the UNet prefix once per (window, prefix class) inside a call (LoopConfig.share_cfg_prefix)
        self.share_prefix = True
        nb = image_latents.shape[0]
        # the UNet's activation dtype (bf16, or fp16 for an fp16 UNet: unet.compute_dtype())
        cdt = unet.compute_dtype() if hasattr(unet, "compute_dtype") else torch.bfloat16
        self.cdt = cdt
        # conditioning in device layouts, converted once per run
        self.img = ops.nchw_to_tokens(image_latents.to(dev).float(), out_dtype=torch.float32)     # (nb*T*S, 4)
        self.ide = image_embeddings.to(dev, cdt).reshape(nb, T, -1)                               # (nb, T, 1024)
        # gated prompts (pipeline:724); "+ 0.0" turns the -0.0 of a negative prompt times gate 0 into +0.0, so branches
        # whose gated prompts are equal are also bitwise equal (frame_equal / branch_twins compare bits)
        self.aud = (audio_prompts.to(dev, torch.float32) * self.gate[0] + 0.0).to(cdt)            # (nb, T, 32, 1024)
        self.n_audio = self.aud.shape[2]
        self.vas = (vasa_prompts.to(dev, torch.float32) * self.gate[1] + 0.0).to(cdt).reshape(nb, T, -1)
        with ops.compute_dtype(cdt):
            self.pose = ops.nchw_to_tokens(pose_fea.to(dev))                                        # (P*S, 320)
        # pose features may hold P != T frames (the pipeline's pose list has N frames): the reference
        # indexes them with the raw window index mod P (indice_slice, pipeline:687-693), not mod T
        self.pose_P = pose_fea.shape[1]
        self._raw = None
        self.added = added_time_ids.to(dev, torch.float32)                                          # (nb, 3)

    def max_units_per_call(self) -> int:
        """Largest UNet call (in 14-frame units) the kernels take: GEMM rows < 2^22 (the epilogues'
        float-reciprocal row division) at level 0, whose widest row count is the Mamba sequence (33
        condition tokens per frame, counted with margin as 64). Operands past the 2 GiB buffer extent
        (the 112-frame mode-2 call's 2.7 GB Mamba xz rows) are taken in row chunks by acth_gemm.
        576x1024: 32 units (448 frames)."""
        per_unit = self.F * (self.S + 64)
        return max(1, ((1 << 22) - 1) // per_unit)

    def prefix_classes(self) -> List[int]:
        """Per CFG branch, the first branch whose UNet prefix inputs are bitwise equal (image latents and
        added time ids; the window's noisy latents, timestep and pose rows are shared by construction).
        Branches 1-3 (drop audio+vasa, drop vasa, cond) share them (pipeline:162-200, 186-205), so the
        UNet prefix before the first IP-adapter input runs once per window for them."""
        if getattr(self, "_prefix_cls", None) is None:
            nb = self.ide.shape[0]
            img = self.img.reshape(nb, -1)
            cls = list(range(nb))
            for c in range(1, nb):
                for e in range(c):
                    if cls[e] == e and _same_bits(img[c], img[e]) and _same_bits(self.added[c], self.added[e]):
                        cls[c] = e
                        break
            self._prefix_cls = cls
        return self._prefix_cls

    def branch_twins(self) -> dict:
        """{branch: earlier branch with bitwise-identical UNet inputs}. The 4 CFG branches
        (pipeline:162-200: uncond, drop audio+vasa, drop vasa, cond) differ only in the ID embedding,
        image latents and the gated audio / VASA prompts (pipeline:724). Under gate [1, 0] (mode 0)
        every VASA prompt is multiplied by 0, so "drop vasa" and "cond" receive identical inputs;
        under gate [0, 1] (mode 1) the audio prompts vanish and "drop audio+vasa" equals "drop vasa".
        The UNet treats batch elements independently and every kernel is deterministic, so such a
        branch's noise prediction is bitwise the twin's: it is evaluated once and read twice by
        guidance (whose g3 / g2 term is then exactly zero, as in the reference)."""
        nb = self.ide.shape[0]
        img = self.img.reshape(nb, -1)
        twins = {}
        for c in range(1, nb):
            for e in range(c):
                if e in twins:
                    continue
                if (_same_bits(self.ide[c], self.ide[e]) and _same_bits(img[c], img[e])
                        and _same_bits(self.aud[c], self.aud[e]) and _same_bits(self.vas[c], self.vas[e])
                        and _same_bits(self.added[c], self.added[e])):
                    twins[c] = e
                    break
        return twins

    def frame_equal(self) -> torch.Tensor:
        """(nb, nb, T) bool on the host: [c, e, f] = CFG branches c and e receive bitwise-equal UNet inputs at latent
        frame f -- ID embedding, image latents, gated audio and VASA prompts of that frame, and the added time ids
        (the window's noisy latents, timestep, pose rows and masks are shared by construction). A window whose frames
        are all equal for (c, e) has c's noise prediction = e's (every kernel is deterministic and the UNet treats
        batch elements independently), so c is read from e's rows (pipeline.window_twins)."""
        if getattr(self, "_frame_eq", None) is None:
            nb, T = self.ide.shape[0], self.T
            img = self.img.reshape(nb, T, -1)
            eq = torch.zeros((nb, nb, T), dtype=torch.bool)
            for c in range(nb):
                for e in range(c):
                    if not _same_bits(self.added[c], self.added[e]):
                        continue
                    m = (_bits_equal(img[c], img[e]) & _bits_equal(self.ide[c], self.ide[e])
                         & _bits_equal(self.aud[c], self.aud[e]) & _bits_equal(self.vas[c], self.vas[e]))
                    eq[c, e] = m.cpu()
            self._frame_eq = eq
        return self._frame_eq

    def begin_schedule(self, timesteps: Sequence[float]):
        """The sampler's timesteps, uploaded once per denoise() call (one host -> device copy) and handed out to the
        UNet calls as device scalars."""
        vals = [float(v) for v in timesteps]
        dev_t = torch.tensor(vals, dtype=torch.float32).to(self.dev)
        self._t_table = {v: dev_t[k:k + 1] for k, v in enumerate(vals)}

    def begin_step(self, raw_frames: List[List[int]]):
        self._raw = raw_frames

    def new_state(self, latents_all: torch.Tensor) -> torch.Tensor:
        return self.ops.nchw_to_tokens(latents_all.to(self.dev).float(), out_dtype=torch.float32)  # (T*S, 4)

    def _dev_ints(self, values, dtype) -> torch.Tensor:
        """Device copy of a small host index list, cached by content: the loop's index lists repeat every
        step, and a host -> device copy from pageable memory blocks the host until the stream drains."""
        cache = self.__dict__.setdefault("_ints", {})
        key = (tuple(values), dtype)
        t = cache.get(key)
        if t is None:
            t = cache[key] = torch.tensor(values, dtype=dtype).to(self.dev)
        return t

    def run_units(self, lat: torch.Tensor, units: Sequence[Tuple[int, int]], frames: List[List[int]],
                  t: float, sigma: float, out: torch.Tensor, row0: int):
        """UNet on ``units``; noise rows written to out[row0 : row0 + U*F*S]."""
        with self.ops.compute_dtype(self.cdt):
            self._run_units(lat, units, frames, t, sigma, out, row0)

    def _run_units(self, lat, units, frames, t, sigma, out, row0):
        ops, F, S = self.ops, self.F, self.S
        U = len(units)
        fl_h = [f for (w, _c) in units for f in frames[w]]
        fidx_d = self._dev_ints(fl_h, torch.int32)
        br_d = self._dev_ints([c for (_w, c) in units], torch.int64)
        br32_d = self._dev_ints([c for (_w, c) in units], torch.int32)
        x = ops.window_input(lat, fidx_d, self.img, br32_d, 1.0 / math.sqrt(sigma * sigma + 1.0), U, F, S, self.T)
        # the units' conditioning rows (ID / audio / VASA prompts, added time ids): fixed for the whole sampling
        # run, and the loop's (frames, branches) layouts repeat (the window shift cycles), so each layout is
        # gathered once and reused -- no index kernels inside the steady-state step
        ckey = (tuple(fl_h), tuple(c for (_w, c) in units))
        cache = self.__dict__.setdefault("_ctx_rows", {})
        got = cache.get(ckey)
        if got is None:
            fl = fidx_d.long()
            bl = br_d.repeat_interleave(F)
            got = cache[ckey] = (self.ide[bl, fl], self.aud[bl, fl], self.vas[bl, fl], self.added[br_d])
        ide_r, aud_r, vas_r, added_r = got
        ehs = (ide_r, [aud_r, vas_r])
        cak = {"ip_adapter_masks": self.masks, "acth_gate": self.gate}
        # the step's timestep as a device scalar: a view into the schedule's table (begin_schedule) when the loop
        # announced it -- no fill kernel per call
        tt = self._t_table.get(t) if getattr(self, "_t_table", None) else None
        if tt is None:
            tt = torch.full((1,), t, device=self.dev, dtype=torch.float32)
        prmap, pmax = fidx_d, max(fl_h)
        if self.pose_P != self.T:
            pr = [r % self.pose_P for (w, _c) in units for r in self._raw[w]]
            prmap, pmax = self._dev_ints(pr, torch.int32), max(pr)
        prefix_src = None
        if self.share_prefix:
            cls = self.prefix_classes()
            first = {}
            prefix_src = [first.setdefault((w, cls[c]), b) for b, (w, c) in enumerate(units)]
        # conv_out writes the noise prediction straight into this call's rows of the loop buffer
        self.unet.forward_tokens(x, U, F, self.H, self.W, tt, ehs, added_r, self.pose, cak,
                                 spatial_condition_rmap=prmap, out_f32=True, spatial_condition_rmap_max=pmax,
                                 prefix_src=prefix_src, out=out[row0:row0 + U * F * S])

    def step_windows(self, lat, gathered, unit_rows: List[List[int]], frames, guidance, sigma, sigma_next):
        """Guidance + Euler + accumulate for every window, then average (pipeline:731-756)."""
        ops = self.ops
        acc = torch.zeros_like(lat)
        cnt = torch.zeros(self.T, device=self.dev, dtype=torch.float32)
        for w, rows in enumerate(unit_rows):
            offs = self._dev_ints(rows, torch.int64)
            fidx = self._dev_ints(frames[w], torch.int32)
            ops.cfg_euler_accum(gathered, offs, lat, fidx, guidance[0], guidance[1], guidance[2], sigma, sigma_next,
                                acc, cnt, self.F, self.S)
        return ops.div_counter(acc, cnt, torch.empty_like(lat), self.T, self.S)

    def finish(self, lat: torch.Tensor) -> torch.Tensor:
        out = self.ops.tokens_to_nchw(lat, self.T, self.H, self.W)
        return out.reshape(1, self.T, 4, self.H, self.W)


# ------------------------------------------------------------------------------------------ loop
def broadcast_from_rank0(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place broadcast of ``t`` from rank 0 of ``group``. RCCL ("nccl") needs device tensors,
    gloo host tensors: the tensor is staged through the backend's device when it lives elsewhere."""
    import torch.distributed as dist
    on_gpu = dist.get_backend(group) == "nccl"
    if t.is_cuda == on_gpu:
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return t
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    tmp = t.to(dev)
    dist.broadcast(tmp, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    t.copy_(tmp)
    return t


def all_gather_rows(dst: torch.Tensor, src: torch.Tensor, group=None):
    """``dst`` = every rank's ``src`` rows, rank-major (all_gather_into_tensor). RCCL ("nccl") gathers device
    tensors in place; another backend (gloo: the CPU tests, and ranks sharing one device) gathers host copies."""
    import torch.distributed as dist
    on_gpu = dist.get_backend(group) == "nccl"
    if src.is_cuda == on_gpu:
        dist.all_gather_into_tensor(dst, src, group=group)
        return dst
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    tmp = torch.empty(dst.shape, dtype=dst.dtype, device=dev)
    dist.all_gather_into_tensor(tmp, src.to(dev), group=group)
    dst.copy_(tmp)
    return dst


@dataclass
class LoopConfig:
    num_frames: int
    frames_per_batch: int = 14
    overlap: int = 0
    shift_offset: int = 7
    num_inference_steps: int = 25
    guidance: Tuple[float, float, float] = (2.0, 7.5, 3.0)
    # per-step (g1, g2, g3) = linspace(min, max, steps)[i] (pipeline:640-657); None: constant ``guidance``
    guidance_schedule: Optional[List[Tuple[float, float, float]]] = None
    sigma_min: float = 0.002
    sigma_max: float = 700.0
    # (window, branch) units per UNet call; 0 = auto: the fewest calls the backend's size limit
    # allows (backend.max_units_per_call), split evenly. Measured on MI355X, mode 0 at N = 14
    # (6 units per step): one 84-frame call 406.8 ms/step vs 4 + 2 units 444.0 ms, 3 + 3 430.1 ms
    # (profiles/r1_step11_bench.log, profiles/r1_step12_bench_upc{3,6}.log): fewer, larger launches fill the lower UNet levels better
    units_per_call: int = 0
    # a rank's UNet calls of one step are independent (disjoint units, disjoint output rows): run up
    # to this many of them on their own HIP streams. Off by default: measured on MI355X at N = 14
    # (2 calls per step), two streams ran 0.5 % slower (the GEMM / attention blocks occupy every
    # CU's registers or LDS, so kernels of the two calls cannot co-reside)
    concurrent_calls: int = 1
    # evaluate a CFG branch whose inputs are bitwise those of another branch once (backend.branch_twins)
    dedup_branches: bool = True
    # run the UNet prefix before the first IP-adapter input once per window for the CFG branches that
    # share its inputs (backend.prefix_classes; branches 1-3), inside each UNet call
    share_cfg_prefix: bool = True


def denoise(backend, latents_all: torch.Tensor, cfg: LoopConfig, rank: int = 0, world: int = 1,
            group=None, step_callback: Optional[Callable[[int], None]] = None, steps: Optional[int] = None,
            plan_log: Optional[list] = None):
    """Run the sampler loop. ``latents_all``: (1, T, 4, h, w) (already ``add_noise``d, pipeline:586-598).

    With world > 1, torch.distributed must be initialised; each rank runs its unit block and one
    ``all_gather_into_tensor`` per step exchanges the noise predictions. The units are planned per step
    (window_twins: which CFG branches of each window have another branch's inputs); ``plan_log``, when given,
    receives one {units, rank_units} entry per step."""
    T = cfg.num_frames + cfg.frames_per_batch
    F = cfg.frames_per_batch
    sigmas, timesteps = karras_sigmas(cfg.num_inference_steps, cfg.sigma_min, cfg.sigma_max)
    lat = backend.new_state(latents_all)
    if world > 1:
        # guidance / Euler / accumulation are replicated on every rank with no second collective, so
        # the latent state must start bitwise identical everywhere: rank 0's copy wins (a caller that
        # drew its noise from an unseeded per-rank RNG would otherwise run incoherent ranks)
        broadcast_from_rank0(lat, group)
    n_windows = len(range(0, T, F - cfg.overlap))
    twins = backend.branch_twins() if (cfg.dedup_branches and hasattr(backend, "branch_twins")) else {}
    frame_eq = backend.frame_equal() if (cfg.dedup_branches and hasattr(backend, "frame_equal")) else None
    if frame_eq is not None and world > 1:
        # every rank must plan the same units (the all-gather sizes depend on them): a pair of branches counts as
        # equal at a frame only if it is equal on every rank
        import torch.distributed as dist
        flags = frame_eq.to(torch.int32)
        if dist.get_backend(group) == "nccl":
            flags = flags.to(lat.device)
        dist.all_reduce(flags, op=dist.ReduceOp.MIN, group=group)
        frame_eq = flags.cpu().bool()
    if hasattr(backend, "share_prefix"):
        backend.share_prefix = cfg.share_cfg_prefix
    if hasattr(backend, "begin_schedule"):
        backend.begin_schedule(timesteps)
    S = backend.S
    rows_per_unit = F * S
    cap_max = math.ceil(n_windows * 4 / world)
    local = torch.zeros((cap_max * rows_per_unit, 4), device=lat.device, dtype=torch.float32)
    gathered = torch.empty((world * cap_max * rows_per_unit, 4), device=lat.device, dtype=torch.float32) \
        if world > 1 else local
    shift = 0
    n_steps = cfg.num_inference_steps if steps is None else steps
    upc = cfg.units_per_call
    if upc <= 0:
        upc = backend.max_units_per_call() if hasattr(backend, "max_units_per_call") else 4
    streams = []
    for i in range(n_steps):
        frames = window_frames(T, F, cfg.overlap, shift)
        # this step's units: per window, the CFG branches whose inputs are not another branch's (window_twins)
        tw = [window_twins(frame_eq, frames[w], twins) for w in range(n_windows)]
        units = step_units(n_windows, tw)
        my_units, cap = split_units(units, world, rank)
        if plan_log is not None:
            plan_log.append(dict(units=len(units), rank_units=len(my_units)))
        index = {u: k for k, u in enumerate(units)}
        base, extra = divmod(len(units), world)
        # row offset of global unit k inside the gathered buffer: rank r's block starts at r * cap units
        owner_row = []
        for r in range(world):
            cnt = base + (1 if r < extra else 0)
            owner_row += [(r * cap + slot) * rows_per_unit for slot in range(cnt)]
        calls = call_splits(len(my_units), upc)
        if cfg.concurrent_calls > 1 and len(calls) > 1 and lat.is_cuda and len(streams) < min(cfg.concurrent_calls,
                                                                                               len(calls)):
            streams += [torch.cuda.Stream(device=lat.device)
                        for _ in range(min(cfg.concurrent_calls, len(calls)) - len(streams))]
        if hasattr(backend, "begin_step"):
            backend.begin_step(window_frames_raw(T, F, cfg.overlap, shift))
        if streams and len(calls) > 1:
            main = torch.cuda.current_stream(lat.device)
            for s in streams:
                s.wait_stream(main)                  # this step's latent state is ready
            for ci, (c0, c1) in enumerate(calls):
                chunk = my_units[c0:c1]
                with torch.cuda.stream(streams[ci % len(streams)]):
                    backend.run_units(lat, chunk, frames, timesteps[i], sigmas[i], local, c0 * rows_per_unit)
            for s in streams:
                main.wait_stream(s)                  # every noise row written before the gather / step
        else:
            for c0, c1 in calls:
                chunk = my_units[c0:c1]
                backend.run_units(lat, chunk, frames, timesteps[i], sigmas[i], local, c0 * rows_per_unit)
        if world > 1:
            n = cap * rows_per_unit
            all_gather_rows(gathered[:world * n], local[:n], group)
        unit_rows = [[owner_row[index[(w, tw[w].get(c, c))]] for c in range(4)] for w in range(n_windows)]
        g = cfg.guidance if cfg.guidance_schedule is None else cfg.guidance_schedule[i]
        lat = backend.step_windows(lat, gathered, unit_rows, frames, g, sigmas[i], sigmas[i + 1])
        shift = (shift + cfg.shift_offset) % F
        if step_callback is not None:
            step_callback(i)
    return backend.finish(lat)
