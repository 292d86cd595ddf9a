"""CPU: the frame-window sharded sampler loop (actalker_amd.pipeline.denoise) over 1, 2 and 3 gloo
ranks against the oracle's single-process loop (pipeline:670-756 semantics).

The backend here is test-only and runs on the CPU: the UNet is a deterministic stand-in (a fixed
function of the window's frames, the CFG branch and the timestep that mixes frames within the
window), so the test isolates what the multi-GPU path adds: the (window, CFG-branch) unit
assignment, the all-gather layout of the noise predictions and the replicated guidance + Euler +
window accumulation. The UNet itself is parity-tested on the GPU (tests/test_model_gpu.py).
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from actalker_amd import pipeline as pl
from oracle import reference_cpu as ref


def fake_unet(x, branch, t):
    """(F, 8, h, w) window input (+ branch id, timestep) -> (F, 4, h, w) 'noise'. Mixes frames with
    a window-relative weighting so a wrong frame order or window split changes the result."""
    F = x.shape[0]
    w = torch.linspace(0.5, 1.5, F).view(F, 1, 1, 1)
    mean = (x[:, :4] * w).mean(0, keepdim=True)
    return torch.tanh(0.01 * x[:, :4] + 0.3 * x[:, 4:] + 0.05 * mean + 0.1 * (branch + 1) + 0.01 * t)


class CpuBackend:
    """Mirror of pipeline.HipBackend's interface on torch CPU tensors."""

    def __init__(self, image_latents, h, w, T, fpb):
        self.img = image_latents               # (4, T, 4, h, w)
        self.h, self.w, self.S = h, w, h * w
        self.T, self.F = T, fpb

    def new_state(self, latents_all):
        return latents_all.clone().float()     # (1, T, 4, h, w)

    def run_units(self, lat, units, frames, t, sigma, out, row0):
        F, S = self.F, self.S
        for u, (wdx, c) in enumerate(units):
            idx = frames[wdx]
            x = torch.cat([lat[0, idx] / math.sqrt(sigma * sigma + 1.0), self.img[c, idx]], dim=1)
            noise = fake_unet(x, c, t)                                        # (F, 4, h, w)
            out[row0 + u * F * S: row0 + (u + 1) * F * S] = noise.permute(0, 2, 3, 1).reshape(-1, 4)

    def step_windows(self, lat, gathered, unit_rows, frames, guidance, sigma, sigma_next):
        F, S, h, w = self.F, self.S, self.h, self.w
        acc = torch.zeros_like(lat)
        cnt = torch.zeros(1, self.T, 1, 1, 1)
        g1, g2, g3 = guidance
        for wdx, rows in enumerate(unit_rows):
            br = [gathered[r:r + F * S].view(F, h, w, 4).permute(0, 3, 1, 2) for r in rows]
            u, dav, dv, c = br
            eps = u + g1 * (dav - u) + g2 * (dv - dav) + g3 * (c - dv)
            idx = frames[wdx]
            out = ref.euler_step_v(eps[None], sigma, sigma_next, lat[:, idx])
            for j, f in enumerate(idx):
                acc[:, f] += out[:, j]
                cnt[:, f] += 1
        return acc / cnt

    def finish(self, lat):
        return lat


class TwinCpuBackend(CpuBackend):
    """Mode-0-like conditioning: branch 3 ("cond") receives exactly branch 2's inputs ("drop vasa",
    VASA prompts gated to zero), so its stand-in noise is branch 2's."""

    COND = (0, 1, 2, 2)

    def run_units(self, lat, units, frames, t, sigma, out, row0):
        F, S = self.F, self.S
        for u, (wdx, c) in enumerate(units):
            idx = frames[wdx]
            x = torch.cat([lat[0, idx] / math.sqrt(sigma * sigma + 1.0), self.img[c, idx]], dim=1)
            noise = fake_unet(x, self.COND[c], t)
            out[row0 + u * F * S: row0 + (u + 1) * F * S] = noise.permute(0, 2, 3, 1).reshape(-1, 4)

    def branch_twins(self):
        return {3: 2}


class PadTwinCpuBackend(CpuBackend):
    """The pipeline's padding structure (pipeline:175-184): past frame N every CFG branch but the unconditional one
    carries the same conditioning, so in a window made only of padding frames branches 2 and 3 have branch 1's
    inputs. The stand-in UNet sees a per-(branch, frame) condition code instead of the branch id, so equal inputs
    give equal outputs, and the backend reports the per-frame input equality (HipBackend.frame_equal)."""

    def __init__(self, image_latents, h, w, T, fpb, N):
        super().__init__(image_latents, h, w, T, fpb)
        self.cond = torch.arange(4, dtype=torch.float32)[:, None].repeat(1, T)
        self.cond[1:, N:] = 1.0
        self.img[2:, N:] = self.img[1, N:]

    def run_units(self, lat, units, frames, t, sigma, out, row0):
        F, S = self.F, self.S
        for u, (wdx, c) in enumerate(units):
            idx = frames[wdx]
            x = torch.cat([lat[0, idx] / math.sqrt(sigma * sigma + 1.0), self.img[c, idx]], dim=1)
            noise = fake_unet(x + self.cond[c, idx].view(-1, 1, 1, 1), 0, t)
            out[row0 + u * F * S: row0 + (u + 1) * F * S] = noise.permute(0, 2, 3, 1).reshape(-1, 4)

    def frame_equal(self):
        nb, T = 4, self.T
        eq = torch.zeros(nb, nb, T, dtype=torch.bool)
        for c in range(nb):
            for e in range(c):
                eq[c, e] = (self.img[c] == self.img[e]).reshape(T, -1).all(-1) & (self.cond[c] == self.cond[e])
        return eq


def oracle_loop(latents, imgl, N, fpb, shift_offset, steps):
    sig, ts = ref.euler_karras_tables(25)
    T = N + fpb
    lat = latents.clone()
    shift = 0
    for i in range(steps):
        pred = torch.zeros_like(lat)
        cnt = torch.zeros(1, T, 1, 1, 1)
        for index_start in range(0, T, fpb):
            s0 = index_start - shift
            idx = [j % T for j in range(s0, s0 + fpb)]
            noise = [fake_unet(torch.cat([lat[0, idx] / ((sig[i] ** 2 + 1) ** 0.5), imgl[c, idx]], 1), c, ts[i])
                     for c in range(4)]
            u, dav, dv, c = noise
            eps = u + 2.0 * (dav - u) + 7.5 * (dv - dav) + 3.0 * (c - dv)
            out = ref.euler_step_v(eps[None], sig[i], sig[i + 1], lat[:, idx])
            for j in range(fpb):
                pred[:, (s0 + j) % T] += out[:, j]
                cnt[:, (s0 + j) % T] += 1
        shift = (shift + shift_offset) % fpb
        lat = pred / cnt
    return lat


def make_case(N=6, fpb=3, h=2, w=3, seed=5):
    g = torch.Generator().manual_seed(seed)
    T = N + fpb
    latents = 0.18215 * torch.randn(1, 1, 4, h, w, generator=g) + 700.0 * torch.randn(1, T, 4, h, w, generator=g)
    imgl = torch.randn(4, T, 4, h, w, generator=g)
    imgl[0] = 0
    return latents, imgl


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, N, fpb, steps, q, twin=False, pad=False, shift=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        latents, imgl = make_case(N, fpb)
        if twin:
            imgl[3] = imgl[2]
        if pad:
            backend = PadTwinCpuBackend(imgl, latents.shape[3], latents.shape[4], N + fpb, fpb, N)
        else:
            backend = (TwinCpuBackend if twin else CpuBackend)(imgl, latents.shape[3], latents.shape[4], N + fpb, fpb)
        cfg = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=shift, units_per_call=2)
        out = pl.denoise(backend, latents, cfg, rank, world, steps=steps)
        # by value (numpy): a tensor put on the queue travels through shared memory whose descriptor
        # the parent fetches from this process, which may have exited by then
        q.put((rank, out.detach().cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_unit_assignment_covers_every_unit_once():
    for n_windows in (1, 2, 3, 9):
        for world in (1, 2, 3, 8):
            seen = []
            caps = set()
            for r in range(world):
                units, cap = pl.assign_units(n_windows, world, r)
                assert len(units) <= cap
                caps.add(cap)
                seen += units
            assert sorted(seen) == [(w, c) for w in range(n_windows) for c in range(4)]
            assert len(caps) == 1
    # N = 112 -> 9 windows x 4 branches over 8 GPUs = 5,5,5,5,4,4,4,4
    assert [len(pl.assign_units(9, 8, r)[0]) for r in range(8)] == [5, 5, 5, 5, 4, 4, 4, 4]


def test_window_frames_wrap_and_shift():
    assert pl.window_frames(6, 3, 0, 0) == [[0, 1, 2], [3, 4, 5]]
    assert pl.window_frames(6, 3, 0, 1) == [[5, 0, 1], [2, 3, 4]]      # (start - shift) mod T


def test_single_process_loop_matches_oracle():
    N, fpb, steps = 6, 3, 4
    latents, imgl = make_case(N, fpb)
    backend = CpuBackend(imgl, latents.shape[3], latents.shape[4], N + fpb, fpb)
    cfg = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=1, units_per_call=2)
    got = pl.denoise(backend, latents, cfg, steps=steps)
    want = oracle_loop(latents, imgl, N, fpb, 1, steps)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("world,N,fpb", [(2, 6, 3), (3, 6, 3), (8, 16, 2)])
def test_sharded_loop_matches_single_process(world, N, fpb):
    """world ranks (gloo), contiguous unit blocks + one all-gather per step == 1 process == oracle. The world-8
    case has C5's unit layout (BASELINE configs[4]: N + fpb = 9 windows x 4 CFG branches = 36 units dealt
    5, 5, 5, 5, 4, 4, 4, 4 over 8 ranks), at stand-in sizes."""
    steps = 4
    if world == 8:
        assert [len(pl.assign_units(len(range(0, N + fpb, fpb)), 8, r)[0]) for r in range(8)] == [5, 5, 5, 5, 4, 4, 4, 4]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, fpb, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {r: torch.from_numpy(a) for r, a in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    latents, imgl = make_case(N, fpb)
    want = oracle_loop(latents, imgl, N, fpb, 1, steps)
    for r in range(world):
        torch.testing.assert_close(outs[r], want, rtol=1e-5, atol=1e-3)
    # every rank holds the identical latent state (replicated guidance/Euler)
    for r in range(1, world):
        assert torch.equal(outs[r], outs[0])


def test_unit_assignment_with_deduplicated_branch():
    """Branches [0, 1, 2] (mode 0: branch 3 is branch 2's twin): N = 112 -> 27 units over 8 GPUs."""
    for n_windows, world in ((2, 1), (9, 8), (3, 2)):
        seen = []
        for r in range(world):
            units, cap = pl.assign_units(n_windows, world, r, branches=[0, 1, 2])
            assert len(units) <= cap
            seen += units
        assert sorted(seen) == [(w, c) for w in range(n_windows) for c in range(3)]
    assert [len(pl.assign_units(9, 8, r, branches=[0, 1, 2])[0]) for r in range(8)] == [4, 4, 4, 3, 3, 3, 3, 3]
    assert pl.assign_units(2, 1, 0, branches=[0, 2, 3])[0] == [(0, 0), (0, 2), (0, 3), (1, 0), (1, 2), (1, 3)]


@pytest.mark.parametrize("world", [1, 2])
def test_twin_branch_evaluated_once_matches_four_branch_loop(world):
    """Dedup (3 branches evaluated, branch 3 read from branch 2's rows) == all 4 evaluated, exactly,
    on 1 process and on 2 gloo ranks."""
    N, fpb, steps = 6, 3, 3
    latents, imgl = make_case(N, fpb)
    imgl[3] = imgl[2]
    calls = []

    class Counting(TwinCpuBackend):
        def run_units(self, lat, units, frames, t, sigma, out, row0):
            calls.extend(units)
            super().run_units(lat, units, frames, t, sigma, out, row0)

    cfg = pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=1, units_per_call=2)
    b4 = Counting(imgl, latents.shape[3], latents.shape[4], N + fpb, fpb)
    want = pl.denoise(b4, latents, pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=1,
                                                 units_per_call=2, dedup_branches=False), steps=steps)
    assert len(calls) == 3 * 4 * steps
    calls.clear()
    if world == 1:
        got = pl.denoise(Counting(imgl, latents.shape[3], latents.shape[4], N + fpb, fpb), latents, cfg, steps=steps)
        assert len(calls) == 3 * 3 * steps and all(c != 3 for _w, c in calls)
        assert torch.equal(got, want)
        return
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, fpb, steps, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {r: torch.from_numpy(a) for r, a in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        torch.testing.assert_close(outs[r], want, rtol=0, atol=0)


def test_window_twins_and_step_units():
    T, N = 6, 3
    eq = torch.zeros(4, 4, T, dtype=torch.bool)
    eq[3, 2] = True                                     # run-wide twin (mode 0)
    eq[2, 1, N:] = eq[3, 1, N:] = True                  # padding frames: branches 1-3 equal
    assert pl.window_twins(eq, [0, 1, 2], {}) == {3: 2}
    assert pl.window_twins(eq, [3, 4, 5], {}) == {2: 1, 3: 1}
    assert pl.window_twins(eq, [2, 3, 4], {}) == {3: 2}          # mixed window
    assert pl.window_twins(None, [3, 4, 5], {3: 2}) == {3: 2}    # no per-frame table: run-wide twins only
    tw = [pl.window_twins(eq, f, {}) for f in ([0, 1, 2], [3, 4, 5])]
    assert pl.step_units(2, tw) == [(0, 0), (0, 1), (0, 2), (1, 0), (1, 1)]
    units = pl.step_units(2, tw)
    got = [pl.split_units(units, 2, r) for r in range(2)]
    assert got == [([(0, 0), (0, 1), (0, 2)], 3), ([(1, 0), (1, 1)], 3)]


@pytest.mark.parametrize("world,N,fpb", [(1, 6, 3), (2, 6, 3), (8, 16, 2)])
def test_padding_window_twins_match_four_branch_loop(world, N, fpb):
    """Per-window twins (a padding-only window evaluates branches 0 and 1; 2 and 3 read branch 1's rows) == all
    four branches evaluated everywhere, bit for bit, on 1 process and on 2 and 8 gloo ranks. N = 6, fpb = 3,
    shift 1: the padding window [6, 7, 8] occurs every third step. World 8 at N = 16, fpb = 2 has C5's 9 windows:
    36 units dealt 5,5,5,5,4,4,4,4 on the odd steps and 34 units dealt 5,5,4,4,4,4,4,4 on the even ones."""
    steps = 6
    latents, imgl = make_case(N, fpb)
    calls = []

    class Counting(PadTwinCpuBackend):
        def run_units(self, lat, units, frames, t, sigma, out, row0):
            calls.extend(units)
            super().run_units(lat, units, frames, t, sigma, out, row0)

    b4 = Counting(imgl.clone(), latents.shape[3], latents.shape[4], N + fpb, fpb, N)
    want = pl.denoise(b4, latents, pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=1,
                                                 units_per_call=2, dedup_branches=False), steps=steps)
    assert len(calls) == len(range(0, N + fpb, fpb)) * 4 * steps
    calls.clear()
    if world == 1:
        plan = []
        got = pl.denoise(Counting(imgl.clone(), latents.shape[3], latents.shape[4], N + fpb, fpb, N), latents,
                         pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=1, units_per_call=2),
                         steps=steps, plan_log=plan)
        # shift 0 at steps 0 and 3: windows [0,1,2] [3,4,5] [6,7,8] -> the last is padding-only (2 units, not 4)
        assert [p["units"] for p in plan] == [10, 12, 12, 10, 12, 12]
        assert len(calls) == sum(p["units"] for p in plan)
        assert torch.equal(got, want)
        return
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    if world == 8:
        units = [pl.step_units(9, [{2: 1, 3: 1} if w == 8 else {} for w in range(9)])]
        assert [len(pl.split_units(units[0], 8, r)[0]) for r in range(8)] == [5, 5, 4, 4, 4, 4, 4, 4]
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, fpb, steps, q, False, True))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = {r: torch.from_numpy(a) for r, a in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        torch.testing.assert_close(outs[r], want, rtol=0, atol=0)


def test_call_splits_fewest_even_calls():
    assert pl.call_splits(6, 6) == [(0, 6)]
    assert pl.call_splits(8, 6) == [(0, 4), (4, 8)]
    assert pl.call_splits(5, 4) == [(0, 3), (3, 5)]
    assert pl.call_splits(1, 4) == [(0, 1)]
    assert pl.call_splits(0, 4) == []
    for n in range(1, 20):
        for m in range(1, 8):
            sp = pl.call_splits(n, m)
            assert sp[0][0] == 0 and sp[-1][1] == n and all(a[1] == b[0] for a, b in zip(sp, sp[1:]))
            sizes = [b - a for a, b in sp]
            assert max(sizes) <= m and max(sizes) - min(sizes) <= 1 and len(sp) == -(-n // m)


def test_auto_units_per_call_uses_backend_limit():
    """units_per_call = 0: calls sized by backend.max_units_per_call(); same result as fixed sizes."""
    N, fpb, steps = 6, 3, 3
    latents, imgl = make_case(N, fpb)
    sizes = []

    class Limited(CpuBackend):
        def max_units_per_call(self):
            return 5

        def run_units(self, lat, units, frames, t, sigma, out, row0):
            sizes.append(len(units))
            super().run_units(lat, units, frames, t, sigma, out, row0)

    b = Limited(imgl, latents.shape[3], latents.shape[4], N + fpb, fpb)
    got = pl.denoise(b, latents, pl.LoopConfig(num_frames=N, frames_per_batch=fpb, shift_offset=1), steps=steps)
    assert sizes == [4, 4, 4] * steps          # 12 units per step, at most 5 per call -> 4 + 4 + 4
    want = oracle_loop(latents, imgl, N, fpb, 1, steps)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-3)


def test_max_units_per_call_stays_under_row_limit():
    """HipBackend.max_units_per_call: level-0 GEMM rows (33 Mamba condition tokens per frame, with
    margin 64) below 2^22; 576x1024 -> 32 units (the 8-unit mode-2 call fits in one), 576x576 -> 57.
    Operands past 2 GiB are row-chunked by acth_gemm (tests/test_kernels_gpu.py::test_gemm_over_2gib)."""
    from types import SimpleNamespace
    for (h, w), want in (((72, 128), 32), ((72, 72), 57)):
        fake = SimpleNamespace(unet=SimpleNamespace(config=SimpleNamespace(block_out_channels=(320, 640, 1280, 1280))),
                               F=14, S=h * w)
        u = pl.HipBackend.max_units_per_call(fake)
        assert u == want
        assert u * 14 * (h * w + 33) < 2 ** 22


# ------------------------------------------------------------------------------------------
# Pose2VideoLongSVDPipeline on 2 gloo ranks with generator=None: the ranks draw their
# noise from different global RNG states; rank 0's draws must win everywhere.
class _Obj:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class _FakeVae:
    """encode(x) -> latent_dist with mean / mode(): 8x average-pooled first 4 'channels'."""

    def encode(self, x):
        lat = torch.nn.functional.avg_pool2d(x.float(), 8)
        lat = torch.cat([lat, lat[:, :1]], 1)[:, :4]
        return _Obj(latent_dist=_Obj(mean=lat, mode=lambda: lat))


class _FakeUnet:
    device = torch.device("cpu")
    config = _Obj(addition_time_embed_dim=256)
    add_embedding = _Obj(linear_1=_Obj(in_features=768))


class _SvdCpuBackend(CpuBackend):
    """pipeline.HipBackend's constructor signature over the CPU stand-in UNet."""

    def __init__(self, unet, H, W, masks, gate, added_time_ids, T, fpb, image_latents, image_embeddings,
                 audio_prompts, vasa_prompts, pose_fea):
        super().__init__(image_latents.float(), H, W, T, fpb)


def _svd_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from actalker_amd import pipeline_svd as ps
        ps.HipBackend = _SvdCpuBackend
        torch.manual_seed(1000 + rank)                       # deliberately different per-rank RNG state
        N, fpb, H, W = 4, 2, 16, 24
        pipe = ps.Pose2VideoLongSVDPipeline(vae=_FakeVae(), unet=_FakeUnet(),
                                            id_proj_model=lambda x: x.float().mean() * torch.ones(1, 1, 1024),
                                            pose_guider=lambda p: torch.zeros(1, 320, p.shape[2], H // 8, W // 8))
        ref = torch.linspace(-1, 1, 3 * H * W).view(1, 3, H, W)
        pose = [torch.ones(3, H, W) for _ in range(N)]
        masks = [torch.ones(1, H, W) for _ in range(N)]
        a = [torch.zeros(32, 1024) for _ in range(N)]
        v = [torch.zeros(1024) for _ in range(N)]
        out = pipe(ref, torch.zeros(1, 512), pose, masks, masks, a, a, v, v, height=H, width=W, num_frames=N,
                   num_inference_steps=3, frames_per_batch=fpb, overlap=0, shift_offset=1, output_type="latent",
                   generator=None, world=world, rank=rank).frames
        # by value (numpy): a tensor put on the queue travels through shared memory whose descriptor
        # the parent fetches from this process, which may have exited by then
        q.put((rank, out.detach().cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_svd_pipeline_ranks_agree_without_generator():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_svd_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {r: torch.from_numpy(a) for r, a in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])
