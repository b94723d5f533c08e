#!/usr/bin/env python3
"""Benchmark: GlobalRenderer frames/sec on MI355X (BASELINE.json metric).

A step = one full frame of the hot path (project/cull/SH -> duplicate-with-keys ->
radix sort -> tile headers -> front-to-back fp16 blend) over one synthetic scene
resident in HBM.  Default workload = BASELINE.json configs[1]: 1M gaussians, SH3,
1920x1080, PackedWorldGaussianHalf (fp16).

N>1 (torch.distributed.run, one rank per GPU), --multi:
  alltoall (default): the whole partitioned frame inside libgsm_amd.so
      (gsm_multigpu_render; exchange handles all-gathered once at set-up over torch.distributed,
      no collective in a frame): rank r projects ids [r*N/n, (r+1)*N/n) once, its per-slab counts
      are stored into every rank's count matrix by the scan kernel, each 48-byte record is written
      straight into its slab owner's receive buffer over xGMI, every rank renders its band of tile
      rows into rank 0's frame, ordered by device-side flag barriers the producing kernels arrive
      at themselves; if any rank cannot create that frame, every rank takes the
      library's RCCL transport (grouped send / recv of the same runs, "multi_transport": "rccl"),
      and only without an NCCL backend the torch all-to-all of gsm_amd.exchange ("multi_fallback");
  replicas: every rank projects all gaussians and keeps its band's assignments.
Either way the bands are gathered on rank 0 inside the timed step.  The frame is fixed as N
grows -> "scaling": "strong".  The line also carries "config4": BASELINE configs[3], the 4K
scene of config 3 partitioned over the same N GPUs, timed the same way.

Prints ONE JSON line on rank 0 (contract in the task statement), including
"roofline" for the dominant kernel (the blend) and "cpu_baseline" (the C oracle
timed on this host's cores, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gsm-renderer_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); measured copy ceiling ~6290
BLEND_EVENT_PERIOD = 5  # timed frames per bracketed blend (HIP events), see the timed loop
# Packed-fp16 VALU issue peak (the blend's bound), measured by tools/exp/valu_peak.hip
# (profiles/r02_valu_peak.txt): independent v_pk_fma_f16 on every SIMD reach 566 G wave-instr/s
# at 8 waves per SIMD (4.19 cycles per instruction at the 2.3 GHz held under load; 32-bit VALU
# ops issue at ~2.3 cycles, so packed 16-bit ops issue at half their rate).  At the 2 waves per
# SIMD the Global blend runs with (one 512-thread workgroup per CU) the same probe reaches 509
# (v_pk_fma) / 400 (v_pk_mul).  Spec-derived ceiling: 1024 SIMDs x 2.4 GHz / 4 cycles = 614.4.
VALU_PEAK_GIPS = 566.0
VALU_PEAK_SPEC_GIPS = 1024 * 2.4 / 4
VALU_PEAK_2WPS_GIPS = 508.5
# Mix-weighted VALU roofline (r03): each class of the blend's VALU instructions (SQ_INSTS_VALU_*
# counters, tools/traffic.py valu_mix_per_launch) priced at its issue cost in cycles per
# wave-instruction per SIMD, measured with 8 independent waves per SIMD by tools/exp/valu_peak.hip
# (profiles/r03_valu_peak.txt): packed 16-bit ops, v_perm_b32, DPP moves, v_max_u32, v_pk_max_u16 and
# v_cvt_f32_f16 issue at half the 32-bit rate (4.1-4.3 cycles against 2.25), v_exp_f32 at a quarter.
# "other" = the instructions no SQ_INSTS_VALU_* class counts; in the blends these are v_pk_min_f16,
# v_perm_b32 (exp-table pairing), DPP / SDWA max (group break), v_pk_max_u16, readlane and moves (static
# ISA histogram), priced at the half rate; roofline_valu also reports the fraction with "other" at the
# full 32-bit rate (a lower bound).  Minimal issue time of a launch = sum(n_c * cost_c) / (SIMDs * clock).
VALU_ISSUE_CYCLES = {"f16": 4.20, "f32": 2.28, "int32": 2.25, "int64": 4.5, "cvt": 4.11, "trans": 8.14, "other": 4.2}
VALU_SIMDS = 1024
VALU_CLOCK_GHZ = 2.3  # held under load (s_memtime against s_memrealtime in the probe)


def valu_roofline(kernel, insts, mix, t_blend):
    """roofline_valu of a blend launch: issue rate against the mix-weighted peak (None without PMC)."""
    if not insts or t_blend <= 0:
        return None
    out = {"bound": "valu", "kernel": kernel, "unit": "G wave-instr/s", "achieved": insts / t_blend / 1e9,
           "insts_per_launch": insts, "frac_of_packed_fp16_peak": insts / t_blend / 1e9 / VALU_PEAK_GIPS,
           "peak_source": "tools/exp/valu_peak.hip, profiles/r03_valu_peak.txt"}
    if mix:
        cycles = sum(n * VALU_ISSUE_CYCLES[c] for c, n in mix.items())
        t_min = cycles / (VALU_SIMDS * VALU_CLOCK_GHZ * 1e9)
        lower = (cycles - mix.get("other", 0) * (VALU_ISSUE_CYCLES["other"] - 2.25)) / (VALU_SIMDS * VALU_CLOCK_GHZ * 1e9)
        out.update({"peak": insts / t_min / 1e9, "frac": t_min / t_blend, "issue_time_us": t_min * 1e6,
                    "frac_if_other_full_rate": lower / t_blend,
                    "mix_per_launch": mix, "issue_cycles": VALU_ISSUE_CYCLES, "clock_ghz": VALU_CLOCK_GHZ,
                    "peak_note": "mix-weighted: each instruction class at its measured issue cost (8 waves/SIMD)"})
    else:
        out.update({"peak": VALU_PEAK_GIPS, "frac": insts / t_blend / 1e9 / VALU_PEAK_GIPS,
                    "peak_note": "no instruction mix measured: every instruction priced as packed fp16 (upper bound)"})
    return out
# FETCH_SIZE corrections calibrated on MI355X (tools/exp/fetch_calib.hip, profiles/r02_fetch_calibration.json)
FETCH_TABLE_RAW_BYTES = 514.5 * 1024  # the blend's 128 KiB LDS table load: 8 XCD L2 misses, tallied at 1/2


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="cfg2_1m_sh3_1080p_f16")
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the C oracle (rank 0, N=1)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="oracle threads of cpu_baseline (0: every CPU of this process's affinity mask)")
    p.add_argument("--cpu-one-thread", type=int, default=1, help="also time one oracle frame on 1 thread (<= 1M)")
    p.add_argument("--orbit-steps", type=int, default=50,
                   help="moving-camera frames timed after the static ones (single GPU, mono); 0 = off")
    p.add_argument("--parity", type=int, default=1, help="compare the frame with the oracle")
    p.add_argument("--inflight-steps", type=int, default=50,
                   help="frames timed with two renderers on two streams (single GPU, mono); 0 = off")
    p.add_argument("--traffic-json", default=None,
                   help="blend PMC numbers per launch (tools/traffic.py), used when measured on --config; "
                        "default profiles/PMC_TAG_pmc_blend_<cfgN>.json")
    p.add_argument("--pmc-tag", default="r05", help="round tag of the default PMC files in profiles/")
    p.add_argument("--stereo-path", choices=("depthfirst", "global"), default="depthfirst",
                   help="stereo configs: DepthFirst semantics (SURVEY 8f rank 1) or two Global views")
    p.add_argument("--df-max-gaussians", type=int, default=6_000_000,
                   help="DepthFirst RendererConfig.maxGaussians (reference default 6M -> 24M instances)")
    p.add_argument("--virtual-ranks", type=int, default=8,
                   help="N=1: also run BASELINE config 4's frame (5M/SH3/4K) split over this many virtual "
                        "ranks on the one GPU (tools/exp_virtual_ranks.py, a child process): per-rank device "
                        "frame and its speedup over the same frame on one renderer; 0 = off")
    p.add_argument("--mg-pipeline", type=int, default=0,
                   help="N > 1: the pipelined multi-GPU frame (GSM_MG_PIPELINE=1: a frame's projection and push "
                        "beside the previous frame's slab render; rank 0 gathers into its own tensors)")
    p.add_argument("--multi", choices=("alltoall", "replicas"), default="alltoall",
                   help="N>1 partition: all-to-all of projected records (8e) or projection replicas")
    p.add_argument("--multi-extra-config", default="cfg3_5m_sh3_4k_f16",
                   help="N>1: also time this config's frame on the N GPUs (BASELINE config 4: the 4K scene), "
                        "reported under 'config4'; 'none' = off")
    a = p.parse_args()
    if a.traffic_json is None:
        a.traffic_json = os.path.join(ROOT, "profiles", f"{a.pmc_tag}_pmc_blend_{a.config.split('_')[0]}.json")
    return a


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes (torch.distributed.run,
    one per GPU, 127.0.0.1) from this process, which has made no GPU call, and return their exit
    code.  Fails loudly when the node has fewer than N GPUs (BENCH_SAME_GPU=1: a rehearsal with the
    ranks sharing the visible GPUs)."""
    import socket
    import subprocess

    import torch
    have = torch.cuda.device_count()  # counts devices without initialising the GPU on this image
    if have < args.gpus and os.environ.get("BENCH_SAME_GPU") != "1":
        print(f"bench: --gpus {args.gpus} needs {args.gpus} GPUs, this node has {have}", file=sys.stderr)
        return 3
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def virtual_ranks_entry(world: int):
    """BASELINE config 4 (5M / SH3 / 3840x2160 over `world` ranks) measured without a multi-GPU node:
    the product's multi-GPU frame (gsm_multigpu_render_phase) for `world` virtual ranks on this GPU,
    each rank's phases timed alone with the whole GPU -- the device part of one rank's frame, no xGMI
    -- against the same frame on one renderer (tools/exp_virtual_ranks.py, run as a child process so
    this process's GPU state stays as it is).  None when the child fails."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "tools", "exp_virtual_ranks.py"), "--config", "cfg3_5m_sh3_4k_f16",
           "--world", str(world), "--frames", "5", "--stages", "0", "--single", "1", "--interval", "20"]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001 -- reported, never fatal for the bench line
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    # the pipelined frame (GSM_MG_PIPELINE=1): frames issued back to back, phases 0-1 of frame f + 1
    # beside phases 2-3 of frame f; only the frame interval is meaningful there
    pipe = None
    try:
        pp = subprocess.run(cmd[:4] + ["--world", str(world), "--interval", "20"], capture_output=True, text=True,
                            timeout=300, env=dict(os.environ, GSM_MG_PIPELINE="1"))
        pipe = json.loads([ln for ln in pp.stdout.splitlines() if ln.startswith("{")][-1]).get("interval")
    except Exception as e:  # noqa: BLE001
        pipe = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    return {"workload": "cfg3_5m_sh3_4k_f16 frame (BASELINE configs[3]) over %d virtual ranks" % world,
            "world": world, "device_frame_ms": d["device_frame_ms"], "max_phase_ms": d["max_phase_ms"],
            "interval_serial": d.get("interval"), "interval_pipelined": pipe,
            "one_gpu_frame_ms": d.get("one_gpu_frame_ms"), "device_speedup": d.get("device_speedup"),
            "barrier_timeouts": d.get("timeouts"), "xgmi_model": d.get("xgmi_model"),
            "modelled_speedup_with_xgmi": (round(d["one_gpu_frame_ms"] / d["xgmi_model"]["modelled_frame_ms"], 3)
                                           if d.get("one_gpu_frame_ms") and d.get("xgmi_model") else None),
            "note": "each rank's phases run alone on this GPU (an upper bound for a rank's own GPU); the pushes "
                    "and the gathered pixels stay local (no xGMI time); each timed frame is enqueued while the GPU "
                    "spins, so the per-phase event pairs time device work only (r06: before, rank 0's phase 0 also "
                    "timed the host's enqueue, ~35 us); device_speedup = one-renderer frame / "
                    "per-rank device frame (one-frame latency); interval_*: the group's frame interval / world "
                    "for frames issued back to back under a moving camera, serial and pipelined (GSM_MG_PIPELINE=1)"}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print(f"bench: WORLD_SIZE={os.environ.get('WORLD_SIZE')} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    import gsm_amd
    from gsm_amd import exchange, scenes, slabs

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_SAME_GPU=1 maps every rank onto the visible GPUs round robin: an N-rank rehearsal of the
    # multi-GPU frame (IPC-mapped exchange memory, cross-process flag barriers) on a one-GPU box.
    # Ranks sharing a GPU cannot form an RCCL communicator ("Duplicate GPU detected"), so the host
    # side (handle exchange, timing barriers) then runs over gloo; the frame itself uses neither.
    same_gpu = os.environ.get("BENCH_SAME_GPU") == "1" or os.environ.get("BENCH_DIST_BACKEND") == "gloo"
    backend = os.environ.get("BENCH_DIST_BACKEND", "gloo" if same_gpu else "nccl")
    gpu = local_rank % max(1, torch.cuda.device_count()) if same_gpu else local_rank
    # BENCH_FORCE_MULTI=1 runs the N>1 code path (C-ABI multi-GPU frame over an RCCL communicator)
    # at world size 1 -- a one-GPU rehearsal of what the driver's 8-GPU runs execute
    force_multi = os.environ.get("BENCH_FORCE_MULTI") == "1"
    if world_size > 1 or force_multi:
        if world_size == 1:  # plain `python bench.py`: a world of one without a launcher
            for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533")):
                os.environ.setdefault(k, v)
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

    alltoall = (world_size > 1 or force_multi) and args.multi == "alltoall"
    # N > 1: the whole partitioned frame runs inside libgsm_amd.so (gsm_multigpu_render,
    # include/gsm_multigpu.h): counts stored into every rank's count matrix by the scan kernel,
    # records pushed to their slab owners over xGMI, bands written into rank 0's frame by the slab
    # blends, device flag barriers -- no host round trip and no collective in a frame (the exchange
    # handles travel once, at set-up, over torch.distributed with any backend).
    native_multi = alltoall
    multi_fallback = multi_transport = None
    gtargets = (None, None)
    if native_multi:
        mg, multi_transport, multi_fallback = connect_multi(gsm_amd, renderer, rank, world_size, backend, dev, args)
        if mg is None:
            native_multi = False
            print(f"bench: native multi-GPU frame unavailable ({multi_fallback}); "
                  "records move through gsm_amd.exchange (torch all-to-all, host-read counts)", file=sys.stderr)
        else:
            frame_ptr = mg.frame()[0]  # rank 0: the gathered frame (library memory, zero copy)
            if args.mg_pipeline and rank == 0:  # pipelined: the library frames alternate, gather into ours
                gtargets = (torch.empty((H, W, 4), dtype=torch.float16, device=dev),
                            torch.empty((H, W), dtype=torch.float16, device=dev))
    if alltoall and not native_multi:
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
        elif native_multi:
            # colour and depth gathered into rank 0's library frames (the reference writes depth with
            # every frame, GlobalRenderer.swift:350; the one-GPU step renders both too)
            if gtargets[0] is not None:
                mg.render(gtargets[0], gtargets[1], inp, cam, W, H, gather=True, stream=stream, gather_depth=True)
            else:
                mg.render(None, None, inp, cam, W, H, gather=True, stream=stream,
                          gather_target=frame_ptr if rank == 0 else None, gather_depth=True)
            return
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
    elapsed, blend_ms_timed = timed_loop(args.steps, step, renderer, world_size, dev, backend)
    # per-stage breakdown: 10 more frames with every stage bracketed (not part of `value`)
    renderer.set_profiling(stage_events=True)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    stage_ms = renderer.stage_times_ms()
    stage_ms["blend_timed_region"] = blend_ms_timed
    counters = renderer.counters()
    # the blend kernel the library launched for this frame (not re-derived here, so a
    # GSM_BLEND_WAVES / GSM_BLEND_PAIRS override is attributed to the kernel that actually ran)
    blend_kernel = renderer.blend_kernel() or "k_blend_px"
    ms_per_step = elapsed / args.steps * 1e3
    fps = 1e3 / ms_per_step
    # two frames in flight (single GPU, mono): a second renderer handle on a second stream, frames
    # alternating between the two -- the double-buffered use of the public API, so one frame's
    # sort and projection overlap the other's blend tail.  A separate line, not `value`.
    inflight = None
    inflight_color = None
    if world_size == 1 and not stereo and not native_multi and args.inflight_steps > 0:
        r2 = gsm_amd.GlobalRenderer(device=dev.index, config=cfg)
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        tg = [(color, depth, cptr, dptr), None]
        c2 = torch.zeros_like(color)
        d2 = torch.zeros_like(depth)
        tg[1] = (c2, d2, c2.data_ptr() - slab.y0 * pitch_c, d2.data_ptr() - slab.y0 * pitch_d)
        rs = [renderer, r2]
        renderer.set_profiling(stage_events=False)
        k = [0]

        def step_inflight():
            i = k[0] & 1
            k[0] += 1
            rs[i].render(tg[i][2], tg[i][3], inp, cam, W, H, stream=streams[i], color_pitch=pitch_c,
                         depth_pitch=pitch_d)
        torch.cuda.synchronize()
        for _ in range(args.warmup * 2):
            step_inflight()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.inflight_steps):
            step_inflight()
        torch.cuda.synchronize()
        t_if = time.perf_counter() - t0
        inflight = {"value": args.inflight_steps / t_if, "unit": "frames/s", "steps": args.inflight_steps,
                    "ms_per_step": t_if / args.inflight_steps * 1e3, "renderers": 2, "streams": 2,
                    "note": "two renderer handles on two HIP streams, frames alternating (double-buffered "
                            "targets); frames overlap across the handles, each frame is the full hot path",
                    "parity_both_targets": None}
        inflight_color = c2
        r2.close()

    # the same frame under camera motion (single GPU, mono): every step a new view, 0.25 degrees
    # further along an orbit about the scene centre, so the blend schedule (last frame's walk
    # lengths, k_unit_order) is always one frame stale -- what the static `value` cannot show
    orbit = None
    orbit_last_cam = None
    if world_size == 1 and not stereo and not native_multi and args.orbit_steps > 0:
        cams = [gsm_amd.CameraParams.from_dict(scenes.orbit_camera(W, H, 0.25 * (i + 1)))
                for i in range(args.warmup + args.orbit_steps)]
        it = iter(cams)

        def step_orbit():
            renderer.render(cptr, dptr, inp, next(it), W, H, stream=stream, color_pitch=pitch_c,
                            depth_pitch=pitch_d)
        for _ in range(args.warmup):
            step_orbit()
        o_elapsed, o_blend = timed_loop(args.orbit_steps, step_orbit, renderer, 1, dev)
        orbit_last_cam = scenes.orbit_camera(W, H, 0.25 * (args.warmup + args.orbit_steps))
        orbit = {"value": args.orbit_steps / o_elapsed, "unit": "frames/s", "steps": args.orbit_steps,
                 "ms_per_step": o_elapsed / args.orbit_steps * 1e3, "blend_ms": o_blend,
                 "camera": "orbit about (0, 0, 5.5), +0.25 deg about y per frame (scenes.orbit_camera)",
                 "parity_last_frame": None}

    multi_parity = None
    if native_multi and args.parity:  # the gathered N-GPU frame against the oracle (rank 0)
        step()
        torch.cuda.synchronize()
        dist.barrier()
        if rank == 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O  # parity checker only
            ref = O.render(world_np, harm_np, sh, cam_d, W, H, max_gaussians=n, nthreads=min(16, cpu_thread_candidates(args)[0]))
            multi_parity = bool(np.array_equal(mg.copy_frame(W, H), ref["color"])) and \
                bool(np.array_equal(mg.copy_depth(W, H), ref["depth"]))
    # BASELINE config 4 (the 4K scene of config 3 on N GPUs): timed the same way after `value`
    multi_4k = None
    if native_multi and args.multi_extra_config not in ("", "none", args.config):
        multi_4k = multi_extra_frame(args, gsm_amd, scenes, dev, gpu, rank, world_size, backend)
    barrier_timeouts = failed_arrivals = None
    if native_multi:
        t = torch.tensor(list(mg.errors()), dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t)  # every rank's barrier timeouts and failed peer arrivals (0, 0 when healthy)
        barrier_timeouts, failed_arrivals = int(t[0].item()), int(t[1].item())
        torch.cuda.synchronize()
        dist.barrier()  # no rank unmaps its exchange memory while a peer may still write into it
        mg.close()
    if rank != 0:
        renderer.close()
        dist.destroy_process_group()
        return
    if force_multi:
        dist.destroy_process_group()

    A = counters["total_assignments"]
    T = counters["tile_count"]
    P = W * H
    # B_blend = A*20 + P*10 + T*8 (index + render record per assignment,
    # rgba16f + r16f per pixel, header per tile) -- algorithmic bytes of one blend launch.
    b_blend = A * 20 + P * 10 + T * 8
    t_blend = blend_ms_timed * 1e-3
    achieved = b_blend / t_blend / 1e9 if t_blend > 0 else 0.0
    # blend units per tile (gsm_blend.hip blend_pairs_per_lane): half tiles while the frame's tiles
    # outnumber 8 waves x CUs, quadrants otherwise; every unit reads the tile's whole list
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    units_per_tile = 2 if T > 8 * n_cus else 4
    traffic = valu_insts = traffic_note = valu_mix = None
    tj = load_pmc(args.traffic_json, args.config, world_size, blend_kernel)
    if tj:
        raw_fetch = tj["fetch_size_kib"] * 1024
        write = tj["write_size_kib"] * 1024
        # the wide parts of the blend's reads are doubled (FETCH counts half of a wide stream):
        # the table prologue (calibrated raw bytes) and the tile lists (4 B/lane coalesced, read
        # once per unit); the record gathers (random 16 B + 4 B) count one 64-B unit per
        # fetched segment and stay as counted (tools/exp/fetch_calib.hip)
        list_bytes = units_per_tile * A * 4
        traffic = int(raw_fetch + FETCH_TABLE_RAW_BYTES + list_bytes / 2 + write)
        traffic_note = (f"FETCH_SIZE {tj['fetch_size_kib']:.0f} KiB + WRITE_SIZE {tj['write_size_kib']:.0f} KiB "
                        f"per launch ({tj['source']}); wide parts doubled: table {FETCH_TABLE_RAW_BYTES:.0f} B, "
                        f"lists {list_bytes // 2} B; gathers as counted (profiles/r02_fetch_calibration.json); "
                        f"upper bound if every gather segment were 128 B: {int(2 * raw_fetch + write)} B")
        valu_insts = tj.get("valu_insts_per_launch")
        valu_mix = tj.get("valu_mix_per_launch")
    stage_sum = sum(v for k, v in stage_ms.items() if k != "blend_timed_region")
    sort_gkeys = A / (stage_ms["sort"] * 1e-3) / 1e9 if stage_ms["sort"] > 0 else 0.0

    parity = None
    cpu = None
    if world_size == 1 and not native_multi and (args.parity or args.cpu_baseline):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline + parity checker only
        cands = cpu_thread_candidates(args)
        views = [scenes.make_camera(W, H, -stereo), scenes.make_camera(W, H, stereo)] if stereo else [cam_d]
        reps = 3 if args.cpu_baseline else 1
        # one frame = every view (both eyes for config 5); the baseline is the best thread count the box grants
        threads, times, per_threads, refs = time_oracle(
            lambda nt: [O.render(world_np, harm_np, sh, cv, W, H, max_gaussians=n, nthreads=nt) for cv in views],
            cands if args.cpu_baseline else cands[:1], reps)
        if args.parity:
            if orbit is not None:  # the buffer holds the last orbit frame: check it, then redo the static one
                ro = O.render(world_np, harm_np, sh, orbit_last_cam, W, H, max_gaussians=n, nthreads=threads)
                got = color[:H].view(torch.int16).cpu().numpy().view(np.uint16)
                orbit["parity_last_frame"] = bool(np.array_equal(got, ro["color"]))
                renderer.render(cptr, dptr, inp, cam, W, H, stream=stream, color_pitch=pitch_c, depth_pitch=pitch_d)
                torch.cuda.synchronize()
            got = color[:H].view(torch.int16).cpu().numpy().view(np.uint16)
            parity = all(bool(np.array_equal(got[:, v * W:(v + 1) * W], r["color"])) for v, r in enumerate(refs)) \
                and int(refs[-1]["total_assignments"]) == A
            if inflight is not None and inflight_color is not None:
                got2 = inflight_color[:H].view(torch.int16).cpu().numpy().view(np.uint16)
                inflight["parity_both_targets"] = bool(np.array_equal(got2, refs[-1]["color"]))
        if args.cpu_baseline:
            med = float(np.median(times))
            cpu = cpu_baseline_entry(med, threads, f"{reps} full frames of {args.config} ({n} gaussians, "
                                     f"{len(views)} view(s) of {W}x{H}) with the C oracle (oracle/gsm_oracle.c, "
                                     f"pthreads), median {med:.2f} s/frame", refs[-1]["times"], per_threads)
            if 16 not in per_threads:  # the r01-r03 figure (16 threads), for comparison
                t = time.perf_counter()
                O.render(world_np, harm_np, sh, cam_d, W, H, max_gaussians=n, nthreads=16)
                t16 = time.perf_counter() - t
                cpu["threads_16"] = {"value": 1.0 / t16, "unit": "frames/s", "cores": 16,
                                     "sample": f"1 full frame of {args.config}, 16 threads, {t16:.2f} s"}
            if args.cpu_one_thread and not stereo and n <= 1_000_000:
                t = time.perf_counter()
                O.render(world_np, harm_np, sh, cam_d, W, H, max_gaussians=n, nthreads=1)
                t1 = time.perf_counter() - t
                cpu["one_thread"] = {"value": 1.0 / t1, "unit": "frames/s", "cores": 1,
                                     "sample": f"1 full frame of {args.config}, 1 thread, {t1:.2f} s"}

    # SURVEY.md 8(d) B_frame: the minimal dataflow of one frame (inputs of all N, SH of the visible
    # V, render data, assignment write, K = 4 sort passes of key + value read and write, blend reads,
    # targets, headers), against the whole frame's time
    V = visible_count(renderer, gsm_amd)
    s_w = 32 if prec else 48
    s_sh = 3 * sh * (2 if prec else 4)
    b_frame = n * s_w + V * s_sh + V * 16 + A * 8 + 4 * A * 16 + A * 20 + P * 10 + T * 8
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
                   "visible": V, "assignments": A, "tiles": T,
                   "parallelism": (f"dp{world_size} tile-row slabs, "
                                   + ("records pushed to slab owners over xGMI inside libgsm_amd (gsm_multigpu_render)"
                                      if native_multi else
                                      ("all-to-all of projected records" if alltoall else "projection replicas")))
                                  if world_size > 1 else "single GPU"},
        "roofline": {"bound": "hbm", "kernel": blend_kernel, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_over_algorithmic": (traffic / b_blend) if traffic else None,
                     "traffic_note": traffic_note,
                     "algorithmic_bytes": b_blend, "launch_timing": f"HIP events around the blend on every {BLEND_EVENT_PERIOD}th frame of the timed region", "avg_launch_ms": blend_ms_timed,
                     "note": "blend is bound by packed-fp16 VALU issue (roofline_valu); HBM fraction "
                             "reported per the metric"},
        "roofline_valu": valu_roofline(blend_kernel, valu_insts, valu_mix, t_blend),
        "roofline_frame": {"bound": "hbm", "achieved": b_frame / (ms_per_step * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": b_frame / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "algorithmic_bytes": b_frame,
                           "formula": "N*S_w + V*S_sh + V*16 + A*8 + 4*A*16 + A*20 + P*10 + T*8 (SURVEY.md 8d)"},
        "cpu_baseline": cpu,
        "stages_ms": stage_ms,
        "stages_sum_ms": stage_sum,
        "sort_gkeys_per_s": sort_gkeys,
        "blend_gb_per_s": achieved,
        "orbit": orbit,
        "inflight2": inflight,
        "parity_vs_oracle": multi_parity if native_multi else parity,
    }
    if multi_fallback:
        out["multi_fallback"] = multi_fallback
    if multi_transport:
        out["multi_transport"] = multi_transport
    if barrier_timeouts is not None:
        out["barrier_timeouts"] = barrier_timeouts
        out["mg_pipelined"] = bool(args.mg_pipeline)
        out["failed_peer_arrivals"] = failed_arrivals
    if multi_4k:
        out["config4"] = multi_4k
    if world_size == 1 and not stereo and args.virtual_ranks > 1:
        out["virtual_ranks_config4"] = virtual_ranks_entry(args.virtual_ranks)
    print(json.dumps(out))
    renderer.close()
    if world_size > 1:
        dist.destroy_process_group()


def multi_extra_frame(args, gsm_amd, scenes, dev, gpu, rank, world_size, backend):
    """BASELINE.json configs[3]: config 3's 4K scene partitioned over the N GPUs by tile-row slab
    (gsm_multigpu_render), timed like `value` (barriers, max over ranks); rank 0 gathers the frame.
    Parity of the partitioned frame is checked on the main config; this is a throughput line."""
    import torch
    import torch.distributed  # noqa: F401 (the create check below is collective)
    c = scenes.CONFIGS[args.multi_extra_config]
    n, W, H, sh, prec = c["count"], c["width"], c["height"], c["sh"], c["precision"]
    world_np, harm_np, cam_d = scenes.gen_scene(n, W, H, sh, prec, seed=42)
    world = torch.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).to(dev)
    harm = torch.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).to(dev)
    del world_np, harm_np
    cfg = gsm_amd.RendererConfig(max_gaussians=n, max_width=W, max_height=H, precision=prec,
                                 gaussian_color_space=gsm_amd.GaussianColorSpace.LINEAR)
    r = gsm_amd.GlobalRenderer(device=dev.index, config=cfg)
    mg, transport, err = connect_multi(gsm_amd, r, rank, world_size, backend, dev, args)
    if mg is None:
        r.close()
        return {"error": err}
    frame_ptr = mg.frame()[0]
    inp = gsm_amd.GaussianInput(world, harm, n, sh)
    cam = gsm_amd.CameraParams.from_dict(cam_d)
    stream = torch.cuda.current_stream(dev)
    gcol = gdep = None
    if args.mg_pipeline and rank == 0:  # pipelined: rank 0 gathers into its own tensors
        gcol = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
        gdep = torch.empty((H, W), dtype=torch.float16, device=dev)

    def step():
        if gcol is not None:
            mg.render(gcol, gdep, inp, cam, W, H, gather=True, stream=stream, gather_depth=True)
            return
        mg.render(None, None, inp, cam, W, H, gather=True, stream=stream, gather_target=frame_ptr if rank == 0 else None,
                  gather_depth=True)
    for _ in range(3):
        step()
    steps = max(1, min(args.steps, 20))
    elapsed, _ = timed_loop(steps, step, r, world_size, dev, backend)
    timeouts = mg.status()
    torch.cuda.synchronize()
    torch.distributed.barrier()
    mg.close()
    r.close()
    return {"value": steps / elapsed, "unit": "frames/s", "n_gpus": world_size, "steps": steps, "warmup": 3,
            "barrier_timeouts": timeouts, "transport": transport,
            "ms_per_step": elapsed / steps * 1e3, "workload": f"{args.multi_extra_config}: {n} gaussians "
            f"{W}x{H} partitioned by tile-row slab over {world_size} GPUs (BASELINE config 4)"}


def connect_multi(gsm_amd, renderer, rank, world_size, backend, dev, args):
    """The partitioned frame inside libgsm_amd (gsm_multigpu_options, include/gsm_multigpu.h): the peer-stores
    transport first (exchange handles all-gathered over torch.distributed, any backend; no collective in a
    frame); if any rank cannot open it (e.g. exchange memory that cannot be mapped on this node, or the
    connect-time mapping check refusing), the in-library RCCL transport over torch's NCCL communicator
    (grouped send / recv, host-read counts).  Collective: every rank takes the same transport.  Returns
    (MultiGpuRenderer or None, transport name, reason of the fallback or None)."""
    import torch
    import torch.distributed as dist

    def agree(mg):  # create is collective: every rank takes this transport or none does
        ok = torch.tensor([0 if mg is None else 1], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0 and mg is not None:
            mg.close()
        return int(ok.item()) == 1
    reason = None
    mg = None
    try:
        opts = gsm_amd.MultiGpuOptions(pipelined=bool(args.mg_pipeline))
        mg = gsm_amd.MultiGpuRenderer.connect(renderer, rank, world_size, gsm_amd.MultiGpuRenderer.torch_allgather,
                                              options=opts)
    except gsm_amd.RendererError as e:
        reason = f"peer stores, rank {rank}: {e}"
    if agree(mg):
        return mg, "peer_stores", None
    reason = reason or "peer stores: another rank's connect failed"
    if backend != "nccl":
        return None, None, reason
    mg = None
    try:
        mg = gsm_amd.MultiGpuRenderer(renderer, gsm_amd.MultiGpuRenderer.torch_comm(dev.index), rank, world_size,
                                      options=gsm_amd.MultiGpuOptions(transport="rccl"))
    except gsm_amd.RendererError as e:
        reason += f"; rccl, rank {rank}: {e}"
    if agree(mg):
        return mg, "rccl", reason
    return None, None, reason + "; rccl: unavailable"


def timed_loop(steps, step, renderer, world_size, dev, backend="nccl"):
    """K steps between barriers and device syncs; returns (max-over-ranks seconds, blend ms)."""
    import torch
    import torch.distributed as dist
    renderer.set_profiling(stage_events=False, blend_events=True, blend_event_period=BLEND_EVENT_PERIOD)
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, renderer.stage_times_ms()["blend"]


def load_pmc(path, config, world_size, kernel):
    """PMC numbers of tools/traffic.py, only when measured on this very workload and kernel."""
    if not path or not os.path.exists(path) or world_size != 1:
        return None
    try:
        with open(path) as f:
            tj = json.load(f)
    except Exception:
        return None
    ok = tj.get("config") == config and "fetch_size_kib" in tj and kernel in tj.get("kernel", "")
    return tj if ok else None


def visible_count(renderer, gsm_amd):
    """V of SURVEY 8(d): gaussians that passed every cull (non-empty tile rect) in the last frame."""
    b = renderer.copy_buffer(gsm_amd.BufferId.BOUNDS).reshape(-1, 4)
    return int(np.count_nonzero((b[:, 0] <= b[:, 1]) & (b[:, 2] <= b[:, 3])))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_thread_candidates(args):
    """Oracle thread counts to time for cpu_baseline: --cpu-threads alone, else the CPUs of this
    process's affinity mask and the cgroup quota rounded up (on the GPU box 256 affine CPUs share a
    16-CPU quota: 256 threads there measure the throttling, not the host) -- the best one is `value`."""
    if args.cpu_threads > 0:
        return [args.cpu_threads]
    try:
        aff = max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        aff = max(1, os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    cands = [aff]
    if quota is not None and math.ceil(quota) < aff:
        cands.insert(0, max(1, math.ceil(quota)))
    return cands


def time_oracle(render, cands, reps):
    """Median seconds per frame of `render(nthreads)` over `reps` frames for each thread count;
    returns (best thread count, its frame times, {threads: frames/s}, the last frame's result)."""
    best, per, out = None, {}, None
    for nt in cands:
        times = []
        for _ in range(reps):
            t = time.perf_counter()
            out = render(nt)
            times.append(time.perf_counter() - t)
        per[nt] = 1.0 / float(np.median(times))
        if best is None or per[nt] > per[best[0]]:
            best = (nt, times)
    return best[0], best[1], per, out


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants (cpu.max quota / period), None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline_entry(median_s, threads, sample, stage_times, per_threads=None):
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    quota = cgroup_cpu_quota()
    out = {"value": 1.0 / median_s, "unit": "frames/s", "cores": threads, "kind": "port",
           "host_cpus": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
           "cpu_model": cpu_model(), "sample": sample, "stages_s": {k: round(v, 4) for k, v in stage_times.items()}}
    for nt, v in sorted((per_threads or {}).items()):
        out[f"threads_{nt}"] = {"value": v, "unit": "frames/s", "cores": nt}
    if per_threads and len(per_threads) > 1:
        out["note"] = (f"oracle timed at {sorted(per_threads)} threads (affinity mask {affinity} CPUs, cgroup quota "
                       f"{quota} CPUs); value = the best, {threads} threads")
    return out


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
    traffic = valu_insts = traffic_note = valu_mix = None
    tj = load_pmc(args.traffic_json, args.config, 1, "k_df_blend_eye")
    if tj:
        raw_fetch, write = tj["fetch_size_kib"] * 1024, tj["write_size_kib"] * 1024
        list_bytes = 2 * A * 4  # one unit per (tile, eye): each tile list is read twice
        traffic = int(raw_fetch + FETCH_TABLE_RAW_BYTES + list_bytes / 2 + write)
        traffic_note = (f"FETCH_SIZE {tj['fetch_size_kib']:.0f} KiB + WRITE_SIZE {tj['write_size_kib']:.0f} KiB per "
                        f"launch; wide parts doubled (table, lists), gathers as counted "
                        f"(profiles/r02_fetch_calibration.json); upper bound {int(2 * raw_fetch + write)} B")
        valu_insts = tj.get("valu_insts_per_launch")
        valu_mix = tj.get("valu_mix_per_launch")
    parity, cpu = None, None
    if args.parity or args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline + parity checker only
        cands = cpu_thread_candidates(args)
        threads, times, per_threads, ref = time_oracle(
            lambda nt: O.df_render_stereo(world_np, harm_np, sh, cams[0], cams[1], W, H,
                                          max_gaussians=max(n, args.df_max_gaussians), nthreads=nt),
            cands if args.cpu_baseline else cands[:1], 2 if args.cpu_baseline else 1)
        if args.parity:
            got = color.view(torch.int16).cpu().numpy().view(np.uint16)
            parity = bool(np.array_equal(got, ref["color"])) and int(ref["total_instances"]) == A
        if args.cpu_baseline:
            med = float(np.median(times))
            cpu = cpu_baseline_entry(med, threads, f"{len(times)} full DepthFirst stereo frames of {args.config} "
                                     f"with the C oracle (og_df_render_stereo, pthreads), median {med:.2f} s/frame",
                                     ref["times"], per_threads)
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
                     "traffic_over_algorithmic": (traffic / b_blend) if traffic else None, "traffic_note": traffic_note,
                     "algorithmic_bytes": b_blend, "launch_timing": f"HIP events around the blend on every {BLEND_EVENT_PERIOD}th frame of the timed region", "avg_launch_ms": blend_ms_timed,
                     "note": "blend is bound by packed-fp16 VALU issue (fp16 math per pixel per (tile, eye) unit)"},
        "roofline_valu": valu_roofline("k_df_blend_eye", valu_insts, valu_mix, t_blend),
        "blend_walk": {"walked": walk[0], "with_mean": walk[1], "blended": walk[2], "list_entries": walk[3]},
        "cpu_baseline": cpu, "stages_ms": stage_ms, "blend_gb_per_s": achieved, "parity_vs_oracle": parity,
    }
    print(json.dumps(out))
    renderer.close()


if __name__ == "__main__":
    main()
