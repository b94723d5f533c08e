#!/usr/bin/env python3
"""Benchmark: GlobalRenderer frames/sec on MI355X (BASELINE.json metric).

A step = one full frame of the hot path (project/cull/SH -> duplicate-with-keys ->
radix sort -> tile headers -> front-to-back fp16 blend) over one synthetic scene
resident in HBM.  Default workload = BASELINE.json configs[1]: 1M gaussians, SH3,
1920x1080, PackedWorldGaussianHalf (fp16).

N>1 (torch.distributed.run, one rank per GPU, RCCL over xGMI), --multi:
  alltoall (default): rank r projects ids [r*N/n, (r+1)*N/n) once and packs a
      48-byte record per (gaussian, slab it meets); all_to_all of the counts and of the
      records (gsm_amd.exchange); every rank renders its band of tile rows from the records;
  replicas: every rank projects all gaussians and keeps its band's assignments.
Either way the bands are gathered on rank 0 inside the timed step.  The frame is fixed as N
grows -> "scaling": "strong".

Prints ONE JSON line on rank 0 (contract in the task statement), including
"roofline" for the dominant kernel (the blend) and "cpu_baseline" (the C oracle
timed on this host's cores, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); measured copy ceiling ~6290
BLEND_EVENT_PERIOD = 5  # timed frames per bracketed blend (HIP events), see the timed loop
VALU_PEAK_GIPS = 1024 * 2.4 / 4  # wave64 packed-fp16 VALU instructions per ns, whole chip


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="cfg2_1m_sh3_1080p_f16")
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the C oracle (rank 0, N=1)")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--parity", type=int, default=1, help="compare the frame with the oracle")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"),
                   help="blend HBM bytes and VALU instructions per launch (tools/traffic.py)")
    p.add_argument("--stereo-path", choices=("depthfirst", "global"), default="depthfirst",
                   help="stereo configs: DepthFirst semantics (SURVEY 8f rank 1) or two Global views")
    p.add_argument("--traffic-json-df", default=os.path.join(ROOT, "profiles", "traffic_cfg5_r01.json"),
                   help="blend PMC traffic / VALU count of the DepthFirst config (tools/gpu_df_pmc.sh)")
    p.add_argument("--df-max-gaussians", type=int, default=6_000_000,
                   help="DepthFirst RendererConfig.maxGaussians (reference default 6M -> 24M instances)")
    p.add_argument("--multi", choices=("alltoall", "replicas"), default="alltoall",
                   help="N>1 partition: all-to-all of projected records (8e) or projection replicas")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import gsm_amd
    from gsm_amd import exchange, scenes, slabs

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo rehearses the N>1 protocol with several ranks on one GPU (CPU-staged
    # collectives; timings meaningless).  The driver's multi-GPU runs use RCCL ("nccl").
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    gpu = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    if world_size > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu if world_size > 1 else 0)
    torch.cuda.set_device(dev)

    c = scenes.CONFIGS[args.config]
    n, W, H, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
    stereo = c.get("stereo")  # config 5: W is per eye, the target is 2W wide
    if stereo and world_size > 1:
        raise SystemExit("the stereo config runs on one GPU")
    world_np, harm_np, cam_d = scenes.gen_scene(n, W, H, sh, prec, seed=42)
    world = torch.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).to(dev)
    harm = torch.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).to(dev)
    if stereo and args.stereo_path == "depthfirst":
        return run_depthfirst(args, c, world_np, harm_np, world, harm, dev)

    cfg = gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H, precision=prec,
                                 gaussian_color_space=gsm_amd.GaussianColorSpace.LINEAR)
    renderer = gsm_amd.GlobalRenderer(device=dev.index, config=cfg)
    tiles_y = (H + 15) // 16
    slab = slabs.partition(tiles_y, H, world_size, rank)
    all_sl = slabs.all_slabs(tiles_y, H, world_size)
    if world_size > 1:
        renderer.set_tile_rows(slab.row_begin, slab.row_end)
    TW = 2 * W if stereo else W  # target width
    pitch_c, pitch_d = TW * 8, TW * 2
    # band buffers; the renderer addresses absolute rows, so hand it base - y0 * pitch
    color = torch.zeros((slab.rows_padded, TW, 4), dtype=torch.float16, device=dev)
    depth = torch.zeros((slab.rows_padded, TW), dtype=torch.float16, device=dev)
    cptr = color.data_ptr() - slab.y0 * pitch_c
    dptr = depth.data_ptr() - slab.y0 * pitch_d
    gather = [torch.empty_like(color) for _ in range(world_size)] if (world_size > 1 and rank == 0) else None
    inp = gsm_amd.GaussianInput(world, harm, n, sh)
    cam = gsm_amd.CameraParams.from_dict(cam_d)
    stream = torch.cuda.current_stream(dev)

    alltoall = world_size > 1 and args.multi == "alltoall"
    if alltoall:
        first, cnt = exchange.id_range(n, world_size, rank)
        rows = exchange.slab_rows(tiles_y, H, world_size)
        send_cap = max(cnt, 1) * world_size
        send = torch.empty(send_cap * exchange.RECORD_BYTES, dtype=torch.uint8, device=dev)
        send_counts = torch.zeros(world_size, dtype=torch.int32, device=dev)
        recv = torch.empty(max(n, 1) * exchange.RECORD_BYTES, dtype=torch.uint8, device=dev)

    if stereo:
        cam_l = gsm_amd.CameraParams.from_dict(scenes.make_camera(W, H, -stereo))
        cam_r = gsm_amd.CameraParams.from_dict(scenes.make_camera(W, H, stereo))

    def step():
        if stereo:
            renderer.render_stereo_sbs(cptr, dptr, inp, cam_l, cam_r, W, H, stream=stream,
                                       color_pitch=pitch_c, depth_pitch=pitch_d)
        elif alltoall:
            renderer.project_partition(inp, cam, W, H, first, cnt, rows, send, send_cap, send_counts,
                                       stream=stream)
            nrec = exchange.exchange(send, send_counts, recv, staged=backend != "nccl")
            renderer.render_records(cptr, dptr, recv, nrec, W, H, stream=stream, color_pitch=pitch_c,
                                    depth_pitch=pitch_d)
        else:
            renderer.render(cptr, dptr, inp, cam, W, H, stream=stream, color_pitch=pitch_c, depth_pitch=pitch_d)
        if world_size > 1:
            if backend == "nccl":
                dist.gather(color, gather_list=gather, dst=0)
            else:  # rehearsal: gloo collectives take host tensors
                gl = [g.cpu() for g in gather] if gather else None
                dist.gather(color.cpu(), gather_list=gl, dst=0)

    for _ in range(args.warmup):
        step()
    # timed region: only the blend (the roofline kernel) is bracketed by HIP events on the render
    # stream -- two events on every BLEND_EVENT_PERIOD-th frame (each bracketed frame costs ~10 us
    # of event overhead, tools/exp_events.py); the per-stage breakdown comes from a separate pass below
    renderer.set_profiling(stage_events=False, blend_events=True, blend_event_period=BLEND_EVENT_PERIOD)
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    blend_ms_timed = renderer.stage_times_ms()["blend"]
    # per-stage breakdown: 10 more frames with every stage bracketed (not part of `value`)
    renderer.set_profiling(stage_events=True)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    stage_ms = renderer.stage_times_ms()
    stage_ms["blend_timed_region"] = blend_ms_timed
    counters = renderer.counters()
    ms_per_step = elapsed / args.steps * 1e3
    fps = 1e3 / ms_per_step

    if rank != 0:
        renderer.close()
        dist.destroy_process_group()
        return

    A = counters["total_assignments"]
    T = counters["tile_count"]
    P = W * H
    # B_blend = A*20 + P*10 + T*8 (index + render record per assignment,
    # rgba16f + r16f per pixel, header per tile) -- algorithmic bytes of one blend launch.
    b_blend = A * 20 + P * 10 + T * 8
    t_blend = blend_ms_timed * 1e-3
    achieved = b_blend / t_blend / 1e9 if t_blend > 0 else 0.0
    traffic = None
    valu_insts = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("config") == args.config and world_size == 1:  # measured on this workload only
                traffic = tj.get("blend_hbm_bytes_per_launch")
                valu_insts = tj.get("blend_valu_insts_per_launch")
        except Exception:
            traffic = None
    sort_gkeys = A / (stage_ms["sort"] * 1e-3) / 1e9 if stage_ms["sort"] > 0 else 0.0

    parity = None
    cpu = None
    if world_size == 1 and (args.parity or args.cpu_baseline):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline + parity checker only
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        views = [scenes.make_camera(W, H, -stereo), scenes.make_camera(W, H, stereo)] if stereo else [cam_d]
        times = []
        refs = None
        reps = 3 if args.cpu_baseline else 1
        for _ in range(reps):  # one frame = every view (both eyes for config 5)
            t = time.perf_counter()
            refs = [O.render(world_np, harm_np, sh, cv, W, H, max_gaussians=n, nthreads=threads) for cv in views]
            times.append(time.perf_counter() - t)
        if args.parity:
            got = color[:H].view(torch.int16).cpu().numpy().view(np.uint16)
            parity = all(bool(np.array_equal(got[:, v * W:(v + 1) * W], r["color"])) for v, r in enumerate(refs)) \
                and int(refs[-1]["total_assignments"]) == A
        if args.cpu_baseline:
            med = float(np.median(times))
            cpu = {"value": 1.0 / med, "unit": "frames/s", "cores": threads, "kind": "port",
                   "sample": f"{reps} full frames of {args.config} ({n} gaussians, {len(views)} view(s) of "
                             f"{W}x{H}) with the C oracle (oracle/gsm_oracle.c, pthreads), median "
                             f"{med:.2f} s/frame",
                   "stages_s": {k: round(v, 4) for k, v in refs[-1]["times"].items()}}

    out = {
        "metric": "frames/sec @ N Gaussians × W×H (1/2/4/8 GPU); sort Gkeys/s; blend HBM GB/s",
        "value": fps,
        "unit": "frames/s",
        "n_gpus": world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp16",
        "data": "synthetic",
        "config": {"workload": f"{args.config}: {n} gaussians SH{ {1: 0, 4: 1, 9: 2, 16: 3}[sh] } "
                               f"{'2x' if stereo else ''}{W}x{H}{' side-by-side stereo' if stereo else ''} "
                               f"{'fp16 PackedWorldGaussianHalf' if prec else 'fp32 PackedWorldGaussian'}",
                   "gaussians": n, "width": W, "height": H, "sh_components": sh,
                   "assignments": A, "tiles": T,
                   "parallelism": (f"dp{world_size} tile-row slabs, "
                                   + ("all-to-all of projected records" if alltoall else "projection replicas"))
                                  if world_size > 1 else "single GPU"},
        "roofline": {"bound": "hbm", "kernel": "k_blend", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes": b_blend, "launch_timing": f"HIP events around the blend on every {BLEND_EVENT_PERIOD}th frame of the timed region", "avg_launch_ms": blend_ms_timed,
                     "note": "blend is VALU/LDS-bound (fp16 math per pixel per entry); HBM fraction "
                             "reported per the metric"},
        # the blend's real bound: packed-fp16 VALU issue.  Peak = 1024 SIMDs x one wave64
        # v_pk_* instruction per 4 cycles x 2.4 GHz (measured issue cost of v_pk_mul_f16 with
        # >= 2 waves per SIMD: tools/exp/valu_lat.hip); instructions per launch from the
        # SQ_INSTS_VALU PMC pass of tools/gpu_round.sh (config 2 only).
        "roofline_valu": ({"bound": "valu", "kernel": "k_blend", "unit": "G wave-instr/s",
                           "achieved": valu_insts / t_blend / 1e9, "peak": VALU_PEAK_GIPS,
                           "frac": valu_insts / t_blend / 1e9 / VALU_PEAK_GIPS,
                           "insts_per_launch": valu_insts}
                          if (valu_insts and t_blend > 0) else None),
        "cpu_baseline": cpu,
        "stages_ms": stage_ms,
        "sort_gkeys_per_s": sort_gkeys,
        "blend_gb_per_s": achieved,
        "parity_vs_oracle": parity,
    }
    print(json.dumps(out))
    renderer.close()
    if world_size > 1:
        dist.destroy_process_group()


def run_depthfirst(args, c, world_np, harm_np, world, harm, dev):
    """Config 5 with DepthFirst stereo semantics (gsm_depthfirst_render_stereo_sbs): one frame =
    both eyes side by side, projected once, 16x16 tiles blended for both eyes together."""
    import torch

    import gsm_amd
    from gsm_amd import scenes
    n, W, H, sh, prec, stereo = c["count"], c["width"], c["height"], c["sh"], c["precision"], c["stereo"]
    cfg = gsm_amd.RendererConfig(max_gaussians=max(n, args.df_max_gaussians), max_width=W, max_height=H,
                                 precision=prec, gaussian_color_space=gsm_amd.GaussianColorSpace.LINEAR)
    renderer = gsm_amd.DepthFirstRenderer(device=dev.index, config=cfg)
    color = torch.zeros((H, 2 * W, 4), dtype=torch.float16, device=dev)
    inp = gsm_amd.GaussianInput(world, harm, n, sh)
    cams = [scenes.make_camera(W, H, -stereo), scenes.make_camera(W, H, stereo)]
    cam_l, cam_r = (gsm_amd.CameraParams.from_dict(x) for x in cams)
    stream = torch.cuda.current_stream(dev)

    def step():
        renderer.render_stereo_sbs(color, inp, cam_l, cam_r, W, H, stream=stream)

    for _ in range(args.warmup):
        step()
    renderer.set_profiling(stage_events=False, blend_events=True, blend_event_period=BLEND_EVENT_PERIOD)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    blend_ms_timed = renderer.stage_times_ms()["blend"]
    renderer.set_profiling(stage_events=True)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    stage_ms = renderer.stage_times_ms()
    stage_ms["blend_timed_region"] = blend_ms_timed
    renderer.set_profiling(stage_events=False, blend_stats=True)  # one more frame: walk statistics
    step()
    torch.cuda.synchronize()
    walk = [int(x) for x in renderer.copy_buffer(gsm_amd.DepthFirstBuffer.BLEND_STATS)]
    cnt = renderer.counters()
    ms_per_step = elapsed / args.steps * 1e3
    A, T, P = cnt["total_instances"], cnt["tile_count"], 2 * W * H
    # blend algorithmic bytes: 4 B id + 32 B StereoTiledRenderData per instance, rgba16f per
    # pixel of both eyes, 8 B header per tile
    b_blend = A * 36 + P * 8 + T * 8
    t_blend = blend_ms_timed * 1e-3
    achieved = b_blend / t_blend / 1e9 if t_blend > 0 else 0.0
    traffic, valu_insts = None, None
    tj_path = args.traffic_json_df
    if os.path.exists(tj_path):
        try:
            with open(tj_path) as f:
                tj = json.load(f)
            if tj.get("config") == args.config:  # measured on this workload only
                traffic = tj.get("blend_hbm_bytes_per_launch")
                valu_insts = tj.get("blend_valu_insts_per_launch")
        except Exception:
            traffic = None
    parity, cpu = None, None
    if args.parity or args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline + parity checker only
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        times, ref = [], None
        for _ in range(2 if args.cpu_baseline else 1):
            t = time.perf_counter()
            ref = O.df_render_stereo(world_np, harm_np, sh, cams[0], cams[1], W, H,
                                     max_gaussians=max(n, args.df_max_gaussians), nthreads=threads)
            times.append(time.perf_counter() - t)
        if args.parity:
            got = color.view(torch.int16).cpu().numpy().view(np.uint16)
            parity = bool(np.array_equal(got, ref["color"])) and int(ref["total_instances"]) == A
        if args.cpu_baseline:
            med = float(np.median(times))
            cpu = {"value": 1.0 / med, "unit": "frames/s", "cores": threads, "kind": "port",
                   "sample": f"{len(times)} full DepthFirst stereo frames of {args.config} with the C oracle "
                             f"(og_df_render_stereo, pthreads), median {med:.2f} s/frame",
                   "stages_s": {k: round(v, 4) for k, v in ref["times"].items()}}
    out = {
        "metric": "frames/sec @ N Gaussians × W×H (1/2/4/8 GPU); sort Gkeys/s; blend HBM GB/s",
        "value": 1e3 / ms_per_step, "unit": "frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "fp16", "data": "synthetic",
        "config": {"workload": f"{args.config}: {n} gaussians SH{ {1: 0, 4: 1, 9: 2, 16: 3}[sh] } 2x{W}x{H} "
                               f"side-by-side stereo, DepthFirst semantics (16x16 tiles, shared SH colour, "
                               f"union bounds), fp16 PackedWorldGaussianHalf",
                   "gaussians": n, "width": W, "height": H, "sh_components": sh, "instances": A,
                   "visible": cnt["visible"], "tiles": T, "max_gaussians": cfg.max_gaussians,
                   "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "kernel": "k_df_blend_eye", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes": b_blend, "launch_timing": f"HIP events around the blend on every {BLEND_EVENT_PERIOD}th frame of the timed region", "avg_launch_ms": blend_ms_timed,
                     "note": "blend is VALU/LDS-bound (fp16 math per pixel per (tile, eye) unit)"},
        "roofline_valu": ({"bound": "valu", "kernel": "k_df_blend_eye", "unit": "G wave-instr/s",
                           "achieved": valu_insts / t_blend / 1e9, "peak": VALU_PEAK_GIPS,
                           "frac": valu_insts / t_blend / 1e9 / VALU_PEAK_GIPS, "insts_per_launch": valu_insts}
                          if (valu_insts and t_blend > 0) else None),
        "blend_walk": {"walked": walk[0], "with_mean": walk[1], "blended": walk[2], "list_entries": walk[3]},
        "cpu_baseline": cpu, "stages_ms": stage_ms, "blend_gb_per_s": achieved, "parity_vs_oracle": parity,
    }
    print(json.dumps(out))
    renderer.close()


if __name__ == "__main__":
    main()
