"""Where does the uncached exchange memory go wrong?

The virtual-rank product frame (W renderers of one process, the product kernels) runs three ways on the
same scene and cameras, the exchange memory filled with 0xAB at prepare (GSM_MG_POISON) so that a word
nobody wrote is recognisable:
  fine     fine-grained exchange memory (the product default), gathered into rank 0's frame;
  uc       uncached exchange memory (GSM_MG_MEM=uncached-ab), gathered into rank 0's frame;
  uc_own   uncached exchange memory, NOT gathered: every rank renders its slab into its own ordinary
           device-memory target (so no pixel crosses the uncached memory).
After every frame each rank's exchange memory is copied out and compared with the fine run's, buffer by
buffer in pipeline order: the count matrix of the frame's parity (row = source), then each owner's
received records (48-B SplatRecords, sources concatenated in rank order), then the pixels against the
oracle.  Prints the first buffer that holds a wrong word, its rank, and which source rank wrote it.

usage: python tools/exp/mg_uncached_diag.py [rounds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")]
import torch  # noqa: E402

import gsm_amd as gsm  # noqa: E402
import oracle as O  # noqa: E402  (checker only)
from gsm_amd import scenes  # noqa: E402

K_MAX = 16
COUNTS_BYTE = 256 * 4
RECORDS_BYTE = 4096
REC = 48


def align(v, a):
    return (v + a - 1) // a * a


def run(kind, gather, world, n, w, h, sh, prec, cams, seed=78):
    os.environ["GSM_MG_MEM"] = kind
    os.environ["GSM_MG_POISON"] = "1"
    world_np, harm_np, _ = scenes.gen_scene(n, w, h, sh, prec, seed=seed)
    wt = torch.from_numpy(world_np.view(np.uint8).reshape(-1).copy()).cuda()
    ht = torch.from_numpy(harm_np.view(np.uint8).reshape(-1).copy()).cuda()
    inp = gsm.GaussianInput(wt, ht, n, sh)
    cfg = gsm.RendererConfig(max_gaussians=n, max_width=w, max_height=h, precision=prec, gaussian_color_space=0)
    rends = [gsm.GlobalRenderer(device=0, config=cfg) for _ in range(world)]
    pre = [gsm.MultiGpuRenderer.prepare(r, k, world) for k, r in enumerate(rends)]
    mgs = [m.connect_handles([hd for _, hd in pre]) for m, _ in pre]
    frame_ptr, _ = mgs[0].frame()
    stream = torch.cuda.current_stream()
    rec_bytes = 2 * align(n * REC, 4096)
    out = []
    own = [torch.zeros((h, w, 4), dtype=torch.float16, device="cuda") for _ in range(world)] if not gather else None
    for cam in cams:
        cp = gsm.CameraParams.from_dict(cam)
        for ph in range(4):
            for k, m in enumerate(mgs):
                if gather:
                    m.render_phases([ph], None, None, inp, cp, w, h, gather=True, stream=stream,
                                    gather_target=frame_ptr if k == 0 else None, gather_depth=False)
                else:
                    m.render_phases([ph], own[k], None, inp, cp, w, h, gather=False, stream=stream)
        torch.cuda.synchronize()
        ex = [m.copy_exchange(RECORDS_BYTE + rec_bytes) for m in mgs]
        if gather:
            pix = mgs[0].copy_frame(w, h)
        else:  # each band from its owner's target (contiguous rows: rank r owns tile rows [r p, (r + 1) p))
            tiles_y = (h + 15) // 16
            per = (tiles_y + world - 1) // world
            pix = np.zeros((h, w, 4), np.uint16)
            for k in range(world):
                y0, y1 = min(h, k * per * 16), min(h, (k + 1) * per * 16)
                pix[y0:y1] = own[k][y0:y1].view(torch.int16).cpu().numpy().view(np.uint16)
        out.append({"ex": ex, "pix": pix, "timeouts": [m.status() for m in mgs]})
    if os.environ.get("DIAG_KEEP") == "1":  # keep every allocation alive: no virtual address is reused
        KEEP.append((mgs, rends, wt, ht, own))
    else:
        for m in mgs:
            m.close()
        for r in rends:
            r.close()
    return out


KEEP = []


def counts_of(ex, par, world):
    words = ex[COUNTS_BYTE:COUNTS_BYTE + 2 * K_MAX * K_MAX * 4].view(np.uint32)
    return words[par * K_MAX * K_MAX:par * K_MAX * K_MAX + world * world].reshape(world, world).astype(np.int64)


def records_of(ex, par, n, nrec):
    base = RECORDS_BYTE + par * align(n * REC, 4096)
    return ex[base:base + nrec * REC].reshape(nrec, REC)


def compare(label, ref, got, refs_img, world, n, h):
    lines = []
    for f, (a, b) in enumerate(zip(ref, got)):
        par = 1 if f % 2 == 0 else 0  # frame 1, 2, ... of a fresh renderer: parity 1, 0, ...
        bad_rows = np.nonzero(np.any(b["pix"] != refs_img[f], axis=(1, 2)))[0]
        ca = [counts_of(x, par, world) for x in a["ex"]]
        cb = [counts_of(x, par, world) for x in b["ex"]]
        first = None
        # 1. the count matrix each owner holds (row = source)
        for r in range(world):
            if not np.array_equal(ca[r], cb[r]):
                d = np.argwhere(ca[r] != cb[r])[0]
                first = f"count matrix of rank {r}: [src {d[0]}][slab {d[1]}] {cb[r][d[0], d[1]]} (fine {ca[r][d[0], d[1]]})"
                break
        # 2. each owner's received records, in source order
        rec_info = []
        if first is None:
            for r in range(world):
                nrec = int(ca[0][:, r].sum())
                ra, rb = records_of(a["ex"][r], par, n, nrec), records_of(b["ex"][r], par, n, nrec)
                diff = np.nonzero(np.any(ra != rb, axis=1))[0]
                if len(diff):
                    starts = np.concatenate([[0], np.cumsum(ca[0][:, r])])
                    src = int(np.searchsorted(starts, diff[0], side="right") - 1)
                    poison = int(np.count_nonzero(np.all(rb[diff] == 0xAB, axis=1)))
                    rec_info.append(f"rank {r}: {len(diff)} of {nrec} records differ, first #{diff[0]} from source rank {src} "
                                    f"(offset {diff[0] - starts[src]} in its run); {poison} still poison")
            if rec_info:
                first = "received records -- " + "; ".join(rec_info)
        # 3. pixels
        if first is None and len(bad_rows):
            first = f"pixels only (records and counts equal): rows {bad_rows.min()}-{bad_rows.max()} ({len(bad_rows)})"
        lines.append(f"{label} frame {f}: timeouts {sum(b['timeouts'])}, bad rows {len(bad_rows)}"
                     + (f" ({bad_rows.min()}-{bad_rows.max()})" if len(bad_rows) else "")
                     + f"; first wrong buffer: {first or 'none'}")
    return lines


def main():
    """usage: mg_uncached_diag.py ROUNDS KINDS OUT  -- KINDS: comma list of fine | uc | uc_own run in this
    order in ONE process (each run a fresh set of renderers and exchange allocations); every frame's
    counts, received records and pixels are saved to OUT (npz) and its pixels compared with the oracle."""
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    kinds = (sys.argv[2] if len(sys.argv) > 2 else "fine,uc,uc_own").split(",")
    outp = sys.argv[3] if len(sys.argv) > 3 else None
    O.build()
    cases = [(8, 50_000, 640, 360, 0), (3, 60_000, 1280, 720, 1)]
    spec = {"fine": ("fine", True), "uc": ("uncached-ab", True), "uc_own": ("uncached-ab", False)}
    save = {}
    refs = {}
    for it in range(rounds):
        for world, n, w, h, prec in cases:
            sh = 16 if prec else 4
            cams = [scenes.make_camera(w, h), scenes.orbit_camera(w, h, 5.0)]
            key = (world, n, w, h, prec)
            if key not in refs:
                wn, hn, _ = scenes.gen_scene(n, w, h, sh, prec, seed=78)
                refs[key] = [O.render(wn, hn, sh, c, w, h, max_gaussians=n)["color"] for c in cams]
            for label in kinds:
                kind, gather = spec[label]
                got = run(kind, gather, world, n, w, h, sh, prec, cams)
                for f, fr in enumerate(got):
                    par = 1 if f % 2 == 0 else 0
                    bad = np.nonzero(np.any(fr["pix"] != refs[key][f], axis=(1, 2)))[0]
                    cts = [counts_of(x, par, world) for x in fr["ex"]]
                    consistent = all(np.array_equal(cts[0], c) for c in cts)
                    print(it, key, label, "frame", f, "timeouts", sum(fr["timeouts"]), "bad rows", len(bad),
                          (f"{bad.min()}-{bad.max()}" if len(bad) else ""), "count matrices equal on all ranks", consistent,
                          flush=True)
                    tag = f"{it}_{world}_{label}_{f}"
                    save[tag + "_counts"] = np.stack(cts)
                    save[tag + "_pix"] = fr["pix"]
                    for r in range(world):
                        nrec = int(cts[0][:, r].sum())
                        save[tag + f"_rec{r}"] = records_of(fr["ex"][r], par, n, nrec).copy()
    if outp:
        np.savez_compressed(outp, **save)


if __name__ == "__main__":
    main()
