"""Worker of tests/test_dist_gpu.py (not a test module): the sampler loop on the REAL HIP backend over
``WORLD_SIZE`` ranks that share the box's one GPU, gloo transport (RCCL refuses two ranks on one device:
ncclInvalidUsage "Duplicate GPU detected", tools/probes/rccl_same_gpu.py), against the same loop on one rank.

Everything the multi-GPU path adds runs on device tensors: the rank-0 broadcast of the latent state (staged
through the host for gloo), the MIN all-reduce of the per-frame branch-equality table, the per-step
all-gather of every rank's fp32 noise predictions, and the replicated guidance + Euler + accumulation.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/dist_loop_gpu.py OUT.pt [mode] [steps]
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    mode = sys.argv[2] if len(sys.argv) > 2 else "mode2"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    import __graft_entry__ as ge
    from actalker_amd import pipeline as pl
    from tests import golden_loop as gl
    unet, _ = ge._tiny_unet(seed=gl.UNET_SEED)
    unet = unet.to(dev)
    latents, imgl, ide, aud, vas, pose, added, masks = gl.loop_inputs()
    # the pipeline's padding (pipeline:175-184): uncond pads past N for every branch, so padding windows have twins
    T = gl.N + gl.FPB
    aud[:, gl.N:] = aud[0:1, :1]
    vas[:, gl.N:] = vas[0:1, :1]
    lc = pl.LoopConfig(num_frames=gl.N, frames_per_batch=gl.FPB, overlap=0, shift_offset=gl.SHIFT,
                       num_inference_steps=25)

    def run(w, r):
        be = pl.HipBackend(unet, gl.H, gl.W, masks, gl.GATES[mode], added, T, gl.FPB, imgl, ide, aud, vas, pose)
        plan = []
        with torch.no_grad():
            got = pl.denoise(be, latents, lc, rank=r, world=w, steps=steps, plan_log=plan)
        torch.cuda.synchronize()
        return got.cpu(), plan

    multi, plan = run(world, rank)
    if rank == 0:
        single, plan1 = run(1, 0)
        torch.save({"multi": multi, "single": single, "rank_units": [p["rank_units"] for p in plan],
                    "units": [p["units"] for p in plan], "units1": [p["units"] for p in plan1]}, out_path)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
