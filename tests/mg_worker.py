"""One rank of the multi-GPU frame (include/gsm_multigpu.h) as its own process: the worker that
tests/test_multigpu_ipc.py starts W times on one GPU.  Handles are exchanged over torch.distributed
(gloo, 127.0.0.1); everything in the frame -- counts, records pushed into the peers' receive buffers
through their IPC mappings, the flag barriers across the processes, the slab render, the band written
straight into rank 0's gathered frame -- is the product path of libgsm_amd.so.

Frames (same scene every rank, generated from the seed):
  A  gathered with depth into the library frames (MultiGpuRenderer.frame() / frame_depth()), read
     back on rank 0
  B  the next camera, gathered with depth into caller tensors (the library's copies)
  C  not gathered: every rank writes its band into its own colour/depth targets
  D  rank 1 passes a width over the maximum: it alone refuses the frame, but still performs every
     barrier step (arrivals marked failed); the others finish it
  E  the frame of A again on every rank: bit-exact, the ranks still in step after D
With --pipelined 1 (GSM_MG_PIPELINE=1) instead: P0-P3, three views issued back to back without host
synchronisation, each gathered with depth into its own caller tensors on rank 0; then PD (rank 1
alone refuses, as D) and PE (the view of P0) issued back to back after them.
Rank 0 writes A, B and E (or P0-P3 and PE), and every rank its band of C, as .npy files into --out, plus status.json."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rank", type=int, required=True)
    p.add_argument("--world", type=int, required=True)
    p.add_argument("--port", type=int, required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--n", type=int, default=40_000)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--height", type=int, default=360)
    p.add_argument("--sh", type=int, default=16)
    p.add_argument("--precision", type=int, default=1)
    p.add_argument("--seed", type=int, default=11)
    p.add_argument("--cap", type=int, default=0, help="max_gaussians of this rank (0: n)")
    p.add_argument("--pipelined", type=int, default=0,
                   help="GSM_MG_PIPELINE=1: only frames P0-P3 (three views, issued back to back, gathered with "
                        "depth into caller tensors on rank 0)")
    a = p.parse_args()
    if a.pipelined:
        os.environ["GSM_MG_PIPELINE"] = "1"  # read at gsm_multigpu_prepare
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    import torch
    import torch.distributed as dist

    import gsm_amd
    from gsm_amd import scenes

    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, w, h = a.n, a.width, a.height
    world_np, harm_np, cam_d = scenes.gen_scene(n, w, h, a.sh, a.precision, seed=a.seed)
    wt = torch.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).to(dev)
    ht = torch.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).to(dev)
    inp = gsm_amd.GaussianInput(wt, ht, n, a.sh)
    cfg = gsm_amd.RendererConfig(max_gaussians=a.cap or n, max_width=w, max_height=h, precision=a.precision,
                                 gaussian_color_space=0)
    rend = gsm_amd.GlobalRenderer(device=0, config=cfg)
    mg = gsm_amd.MultiGpuRenderer.connect(rend, a.rank, a.world, gsm_amd.MultiGpuRenderer.torch_allgather)
    mg.set_timeout_ms(20000)
    result = {"rank": a.rank}
    stream = torch.cuda.current_stream(dev)
    try:
        if a.cap and a.cap < n:  # every rank must refuse the frame alike, before any barrier
            try:
                mg.render(None, None, inp, gsm_amd.CameraParams.from_dict(cam_d), w, h, gather=True, stream=stream)
                result["refused"] = False
            except gsm_amd.RendererError as e:
                result["refused"] = e.status == gsm_amd.Status.INVALID_GAUSSIAN_COUNT
            return
        if a.pipelined:
            cams = [cam_d, scenes.orbit_camera(w, h, 3.0), scenes.orbit_camera(w, h, 6.0), cam_d]
            cols = [torch.full((h, w, 4), float("nan"), dtype=torch.float16, device=dev) for _ in cams]
            deps = [torch.full((h, w), float("nan"), dtype=torch.float16, device=dev) for _ in cams]
            for i, cm in enumerate(cams):  # no host synchronisation between the frames
                mg.render(cols[i] if a.rank == 0 else None, deps[i] if a.rank == 0 else None, inp,
                          gsm_amd.CameraParams.from_dict(cm), w, h, gather=True, stream=stream, gather_depth=True)
            torch.cuda.synchronize()
            if a.rank == 0:
                for i in range(len(cams)):
                    np.save(os.path.join(a.out, f"frame_p{i}.npy"), cols[i].view(torch.int16).cpu().numpy().view(np.uint16))
                    np.save(os.path.join(a.out, f"depth_p{i}.npy"), deps[i].view(torch.int16).cpu().numpy().view(np.uint16))
            result["timeouts"] = mg.status()
            if a.world > 1:
                # D (rank 1 refuses: width over the maximum) then E (the first view again), pipelined and
                # back to back: the ranks stay in step, E is bit-exact
                for i, wd in enumerate((w + (1 if a.rank == 1 else 0), w)):
                    try:
                        mg.render(cols[i] if a.rank == 0 else None, deps[i] if a.rank == 0 else None, inp,
                                  gsm_amd.CameraParams.from_dict(cam_d), wd, h, gather=True, stream=stream,
                                  gather_depth=True)
                        result[f"pd{i}_status"] = 0
                    except gsm_amd.RendererError as e:
                        result[f"pd{i}_status"] = int(e.status)
                torch.cuda.synchronize()
                if a.rank == 0:
                    np.save(os.path.join(a.out, "frame_pe.npy"), cols[1].view(torch.int16).cpu().numpy().view(np.uint16))
                    np.save(os.path.join(a.out, "depth_pe.npy"), deps[1].view(torch.int16).cpu().numpy().view(np.uint16))
                result["timeouts_de"], result["failed_peer_arrivals"] = mg.errors()
            return
        frame_ptr, _ = mg.frame()
        # A: into the library frames (zero copy), colour and depth
        for _ in range(2):  # a second frame reuses every mapping and flag
            mg.render(None, None, inp, gsm_amd.CameraParams.from_dict(cam_d), w, h, gather=True, stream=stream,
                      gather_target=frame_ptr if a.rank == 0 else None, gather_depth=True)
        torch.cuda.synchronize()
        dist.barrier()
        if a.rank == 0:
            np.save(os.path.join(a.out, "frame_a.npy"), mg.copy_frame(w, h))
            np.save(os.path.join(a.out, "depth_a.npy"), mg.copy_depth(w, h))
        # B: the next camera, gathered into caller tensors on rank 0
        cam_b = scenes.orbit_camera(w, h, 3.0)
        color = torch.full((h, w, 4), float("nan"), dtype=torch.float16, device=dev) if a.rank == 0 else None
        depth = torch.full((h, w), float("nan"), dtype=torch.float16, device=dev) if a.rank == 0 else None
        mg.render(color, depth, inp, gsm_amd.CameraParams.from_dict(cam_b), w, h, gather=True, stream=stream,
                  gather_depth=True)
        torch.cuda.synchronize()
        if a.rank == 0:
            np.save(os.path.join(a.out, "frame_b.npy"), color.view(torch.int16).cpu().numpy().view(np.uint16))
            np.save(os.path.join(a.out, "depth_b.npy"), depth.view(torch.int16).cpu().numpy().view(np.uint16))
        # C: no gather -- every rank's band in its own targets
        color = torch.full((h, w, 4), float("nan"), dtype=torch.float16, device=dev)
        depth = torch.full((h, w), float("nan"), dtype=torch.float16, device=dev)
        mg.render(color, depth, inp, gsm_amd.CameraParams.from_dict(cam_d), w, h, gather=False, stream=stream)
        torch.cuda.synchronize()
        np.save(os.path.join(a.out, f"band_c_color_{a.rank}.npy"), color.view(torch.int16).cpu().numpy().view(np.uint16))
        np.save(os.path.join(a.out, f"band_c_depth_{a.rank}.npy"), depth.view(torch.int16).cpu().numpy().view(np.uint16))
        result["counts"] = mg.counts().tolist()
        result["timeouts"] = mg.status()
        if a.world > 1:
            # D: rank 1 alone refuses the frame (width over the maximum); every rank stays in step
            torch.cuda.synchronize()
            dist.barrier()
            try:
                mg.render(None, None, inp, gsm_amd.CameraParams.from_dict(cam_d), w + (1 if a.rank == 1 else 0), h,
                          gather=True, stream=stream, gather_target=frame_ptr if a.rank == 0 else None,
                          gather_depth=True)
                result["d_status"] = 0
            except gsm_amd.RendererError as e:
                result["d_status"] = int(e.status)
            torch.cuda.synchronize()
            # E: the frame of A on every rank again
            mg.render(None, None, inp, gsm_amd.CameraParams.from_dict(cam_d), w, h, gather=True, stream=stream,
                      gather_target=frame_ptr if a.rank == 0 else None, gather_depth=True)
            torch.cuda.synchronize()
            if a.rank == 0:
                np.save(os.path.join(a.out, "frame_e.npy"), mg.copy_frame(w, h))
                np.save(os.path.join(a.out, "depth_e.npy"), mg.copy_depth(w, h))
            result["timeouts_de"], result["failed_peer_arrivals"] = mg.errors()
    finally:
        torch.cuda.synchronize()
        dist.barrier()  # no rank unmaps its exchange memory while a peer may still write into it
        mg.close()
        rend.close()
        with open(os.path.join(a.out, f"status_{a.rank}.json"), "w") as f:
            json.dump(result, f)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
