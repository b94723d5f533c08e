"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's PLY ingestion, used by
tests/test_ply.py as the checker of the product loader (gsm-renderer_amd/csrc/gsm_ply.cpp via
include/gsm_ply.h).  Never imported by the product.

Follows Sources/Renderer/Utils/PLYLoader.swift (header :115-201, load :254-287, compressed
:291-514, standard :518-741) and Sources/Renderer/Utils/Scene.swift (bounds :172-196, Morton
sort :45-138) line by line in float32, with two declared choices shared with the product:
stable sorts where Swift's sort is unstable (SH property order, Morton ties).
Parity unpinned against the reference itself: the reference ships no PLY file or PLY test
vector (its PLY tests read a local file path and skip when it is absent,
Tests/RendererTests/PLYBenchmarkTests.swift:80-100), and Swift cannot run here.
"""
from __future__ import annotations

import re

import numpy as np

F32 = np.float32
_TYPES = {"int8": "<i1", "char": "<i1", "uint8": "<u1", "uchar": "<u1", "int16": "<i2", "short": "<i2",
          "uint16": "<u2", "ushort": "<u2", "int32": "<i4", "int": "<i4", "uint32": "<u4", "uint": "<u4",
          "float32": "<f4", "float": "<f4", "float64": "<f8", "double": "<f8"}


class PLYError(Exception):
    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


def decode_header(text: str):
    """PLYHeader.decodeASCII (PLYLoader.swift:115-201) -> (format, [(name, count, [(prop, type|('list', ct, vt))])])."""
    fmt = None
    elements = []
    for line in re.split(r"\r\n|\n|\r", text):
        toks = line.split()
        if not toks:
            continue
        kw = toks[0]
        if kw in ("ply", "comment", "obj_info"):
            continue
        if kw == "format":
            if fmt is not None:
                raise PLYError("headerUnexpectedKeyword")
            m = re.fullmatch(r"[ \t]*format[ \t]+(\w+?)[ \t]+(\S+?)", line)
            if not m:
                raise PLYError("headerInvalidLine")
            if m.group(1) not in ("ascii", "binary_little_endian", "binary_big_endian"):
                raise PLYError("headerInvalidFileFormatType")
            fmt = m.group(1)
        elif kw == "element":
            if fmt is None:
                raise PLYError("headerUnexpectedKeyword")
            m = re.fullmatch(r"[ \t]*element[ \t]+(\S+?)[ \t]+(\d+?)", line)
            if not m or int(m.group(2)) > 0xFFFFFFFF:
                raise PLYError("headerInvalidLine")
            elements.append((m.group(1), int(m.group(2)), []))
        elif kw == "property":
            if fmt is None or not elements:
                raise PLYError("headerUnexpectedKeyword")
            ml = re.fullmatch(r"[ \t]*property[ \t]+list[ \t]+(\w+?)[ \t]+(\w+?)[ \t]+(\S+)", line)
            mp = re.fullmatch(r"[ \t]*property[ \t]+(\w+?)[ \t]+(\S+)", line)
            if ml:
                if ml.group(1) not in _TYPES or ml.group(2) not in _TYPES:
                    raise PLYError("headerUnknownPropertyType")
                elements[-1][2].append((ml.group(3), ("list", ml.group(1), ml.group(2))))
            elif mp:
                if mp.group(1) not in _TYPES:
                    raise PLYError("headerUnknownPropertyType")
                elements[-1][2].append((mp.group(2), mp.group(1)))
            else:
                raise PLYError("headerInvalidLine")
        elif kw == "end_header":
            break
        else:
            raise PLYError("headerUnknownKeyword")
    if fmt is None:
        raise PLYError("headerFormatMissing")
    return fmt, elements


def _width(t):
    return 0 if isinstance(t, tuple) else np.dtype(_TYPES[t]).itemsize


def _recenter(pos):
    if len(pos) == 0:
        return pos
    ctr = (pos.min(0) + pos.max(0)) * F32(0.5)
    ln = np.sqrt((ctr[0] * ctr[0] + ctr[1] * ctr[1]) + ctr[2] * ctr[2])
    return pos - ctr if ln > F32(1e-6) else pos


def load(data: bytes) -> dict:
    """PLYLoader.load (PLYLoader.swift:254-287) -> dict(pos, scale, rot(xyzw), opacity, harmonics, sh, compressed)."""
    end = data.find(b"end_header\n")
    end = end + 11 if end >= 0 else (data.find(b"end_header\r\n") + 12 if data.find(b"end_header\r\n") >= 0 else -1)
    if end < 0:
        raise PLYError("invalidHeader")
    try:
        text = data[:end].decode("ascii")
    except UnicodeDecodeError:
        raise PLYError("headerInvalidCharacters")
    fmt, elements = decode_header(text)
    if fmt != "binary_little_endian":
        raise PLYError("unsupportedFormat")
    vertex = next((e for e in elements if e[0] == "vertex"), None)
    if vertex is None:
        raise PLYError("missingVertexElement")
    names = [p[0] for p in vertex[2]]
    if any(e[0] == "chunk" for e in elements) and all(
            k in names for k in ("packed_position", "packed_rotation", "packed_scale", "packed_color")):
        return _load_compressed(data, elements, end)
    return _load_standard(data, vertex, end)


def _unorm(v, bits):
    mask = (1 << bits) - 1
    return (v & mask).astype(F32) / F32(mask)


def _load_compressed(data, elements, body):
    """loadCompressed (PLYLoader.swift:291-514)."""
    chunk = next((e for e in elements if e[0] == "chunk"), None)
    vertex = next((e for e in elements if e[0] == "vertex"), None)
    sh = next((e for e in elements if e[0] == "sh"), None)
    cst = sum(_width(t) for _, t in chunk[2])
    vst = sum(_width(t) for _, t in vertex[2])
    sst = sum(_width(t) for _, t in sh[2]) if sh else 0
    nc, nv = chunk[1], vertex[1]
    vstart = body + cst * nc
    if len(data) < vstart + vst * nv + sst * nv:
        raise PLYError("insufficientData")
    if nv and (nv - 1) // 256 >= nc:
        raise PLYError("insufficientData")

    def col(elem, stride, start, count, name, dt):
        off = 0
        for n, t in elem[2]:
            if n == name:
                raw = np.frombuffer(data, np.uint8, count * stride, start).reshape(count, stride)
                return raw[:, off:off + 4].copy().view(dt).reshape(count)
            off += _width(t)
        return np.zeros(count, dt)

    cidx = np.arange(nv) // 256
    cf = {k: col(chunk, cst, body, nc, k, "<f4")[cidx] for k in (
        "min_x", "min_y", "min_z", "max_x", "max_y", "max_z", "min_scale_x", "min_scale_y", "min_scale_z",
        "max_scale_x", "max_scale_y", "max_scale_z", "min_r", "min_g", "min_b", "max_r", "max_g", "max_b")}
    pp, pr, ps, pc = (col(vertex, vst, vstart, nv, k, "<u4") for k in
                      ("packed_position", "packed_rotation", "packed_scale", "packed_color"))

    def lerp(a, b, t):
        return a * (F32(1) - t) + b * t

    pos = np.stack([lerp(cf["min_x"], cf["max_x"], _unorm(pp >> 21, 11)),
                    lerp(cf["min_y"], cf["max_y"], _unorm(pp >> 11, 10)),
                    lerp(cf["min_z"], cf["max_z"], _unorm(pp, 11))], 1)
    norm = F32(1) / (np.sqrt(F32(2)) * F32(0.5))
    a = (_unorm(pr >> 20, 10) - F32(0.5)) * norm
    b = (_unorm(pr >> 10, 10) - F32(0.5)) * norm
    c = (_unorm(pr, 10) - F32(0.5)) * norm
    m = np.sqrt(np.maximum(F32(0), F32(1) - ((a * a + b * b) + c * c)))
    which = pr >> 30
    rot = np.where((which == 0)[:, None], np.stack([a, b, c, m], 1),
                   np.where((which == 1)[:, None], np.stack([m, b, c, a], 1),
                            np.where((which == 2)[:, None], np.stack([b, m, c, a], 1), np.stack([b, c, m, a], 1))))
    scale = np.stack([np.exp(lerp(cf["min_scale_x"], cf["max_scale_x"], _unorm(ps >> 21, 11))),
                      np.exp(lerp(cf["min_scale_y"], cf["max_scale_y"], _unorm(ps >> 11, 10))),
                      np.exp(lerp(cf["min_scale_z"], cf["max_scale_z"], _unorm(ps, 11)))], 1)
    c0 = F32(0.28209479177387814)
    harm = np.stack([(lerp(cf["min_r"], cf["max_r"], _unorm(pc >> 24, 8)) - F32(0.5)) / c0,
                     (lerp(cf["min_g"], cf["max_g"], _unorm(pc >> 16, 8)) - F32(0.5)) / c0,
                     (lerp(cf["min_b"], cf["max_b"], _unorm(pc >> 8, 8)) - F32(0.5)) / c0], 1).reshape(-1)
    return dict(pos=_recenter(pos.astype(F32)), scale=scale.astype(F32), rot=rot.astype(F32),
                opacity=_unorm(pc, 8), harmonics=harm.astype(F32), sh=1, compressed=True)


def _sh_key(name):
    def num(s):
        return int(s) if s.isdigit() and len(s) < 10 else 0
    if name.startswith("f_dc_"):
        return num(name[5:])
    if name.startswith("f_rest_"):
        return 3 + num(name[7:])
    if name.startswith("sh_"):
        return num(name[3:])
    return 2 ** 31 - 1


def _load_standard(data, vertex, body):
    """loadStandard (PLYLoader.swift:518-741)."""
    props = vertex[2]
    if any(isinstance(t, tuple) for _, t in props):
        raise PLYError("listPropertiesNotSupported")
    n = vertex[1]
    dt = np.dtype([(f"p{i}", _TYPES[t]) for i, (_, t) in enumerate(props)])
    if len(data) - body < dt.itemsize * n:
        raise PLYError("insufficientData")
    rec = np.frombuffer(data, dt, n, body)
    idx = {}
    sh = []
    alias = {"x": ("x", "px", "pos_x", "position_x"), "y": ("y", "py", "pos_y", "position_y"),
             "z": ("z", "pz", "pos_z", "position_z"), "s0": ("scale_0", "scale0", "sx", "scale_x"),
             "s1": ("scale_1", "scale1", "sy", "scale_y"), "s2": ("scale_2", "scale2", "sz", "scale_z"),
             "r0": ("rot_0", "rot0", "qw", "rotation_w"), "r1": ("rot_1", "rot1", "qx", "rotation_x"),
             "r2": ("rot_2", "rot2", "qy", "rotation_y"), "r3": ("rot_3", "rot3", "qz", "rotation_z"),
             "op": ("opacity", "alpha")}
    for i, (name, _) in enumerate(props):
        ln = name.lower()
        for k, al in alias.items():
            if ln in al:
                idx[k] = i
                break
        else:
            if ln.startswith(("f_dc_", "f_rest_", "sh_", "spherical_harmonics_")):
                sh.append((ln, i))
    if not all(k in idx for k in "xyz"):
        raise PLYError("missingRequiredProperties")
    sh.sort(key=lambda p: _sh_key(p[0]))  # stable (declared choice)

    def get(k):
        if isinstance(k, str):
            if k not in idx:
                return np.zeros(n, F32)
            k = idx[k]
        v = rec[f"p{k}"]
        t = props[k][1]
        if _TYPES[t] == "<u1":
            return v.astype(F32) / F32(255)
        return v.astype(F32)  # f64 -> f32 rounds to nearest, ints convert

    s0, s1, s2, opr = get("s0"), get("s1"), get("s2"), get("op")
    log_scale, logit = True, True
    ns = min(100, n)
    if "s0" in idx and ns:
        smp = s0[:ns]
        tot = F32(0)
        for x in smp:
            tot = F32(tot + x)
        avg = F32(tot / F32(ns))
        if (smp < 0).any():
            log_scale = True
        elif not (smp > 1).any() and F32(0) < avg < F32(0.5):
            log_scale = False
    if "op" in idx and ns:
        logit = bool(opr[:ns].min() < 0 or opr[:ns].max() > 1)
    keep = ~((s0 == 2) & (s1 == 2) & (s2 == 2) & (np.abs(opr - F32(4.8402)) < F32(0.001)))
    pos = np.stack([get("x"), get("y"), get("z")], 1)[keep]
    sc = np.stack([s0, s1, s2], 1)[keep]
    scale = np.exp(sc) if log_scale else sc
    q = np.stack([get("r1"), get("r2"), get("r3"), get("r0")], 1)[keep]
    ln = np.sqrt(((q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1]) + q[:, 2] * q[:, 2]) + q[:, 3] * q[:, 3])
    rot = q / ln[:, None]
    op = opr[keep]
    opacity = F32(1) / (F32(1) + np.exp(-op)) if logit else op
    coeffs = np.stack([get(i) for _, i in sh], 1)[keep] if sh else np.zeros((int(keep.sum()), 0), F32)
    stride = len(sh)
    k = stride // 3 if stride else 0
    if k > 0:
        hoc = k - 1
        out = np.zeros((len(coeffs), stride), F32)
        out[:, 0] = coeffs[:, 0]
        out[:, 1:1 + hoc] = coeffs[:, 3:3 + hoc]
        out[:, k] = coeffs[:, 1]
        out[:, k + 1:k + 1 + hoc] = coeffs[:, 3 + hoc:3 + 2 * hoc]
        out[:, 2 * k] = coeffs[:, 2]
        out[:, 2 * k + 1:2 * k + 1 + hoc] = coeffs[:, 3 + 2 * hoc:3 + 3 * hoc]
        harm = out.reshape(-1)
    else:
        harm = np.zeros(0, F32)
    return dict(pos=_recenter(pos.astype(F32)), scale=scale.astype(F32), rot=rot.astype(F32),
                opacity=opacity.astype(F32), harmonics=harm, sh=k, compressed=False)


def bounds(pos, scale):
    """GaussianSceneBuilder.bounds(of:) (Scene.swift:172-196)."""
    if len(pos) == 0:
        return np.zeros(3, F32), 1.0
    mn, mx = pos.min(0), pos.max(0)
    ctr = (mn + mx) * F32(0.5)
    d = pos - ctr
    ln = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    r = F32(max(F32(0), (ln + scale.max(1)).max()))
    e = mx - ctr
    r = max(r, np.sqrt((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]))
    return ctr, float(max(r, F32(0.5)))


def _expand(v):
    x = v.astype(np.uint64) & np.uint64(0x1FFFFF)
    for sh, m in ((32, 0x1F00000000FFFF), (16, 0x1F0000FF0000FF), (8, 0x100F00F00F00F00F),
                  (4, 0x10C30C30C30C30C3), (2, 0x1249249249249249)):
        x = (x | (x << np.uint64(sh))) & np.uint64(m)
    return x


def morton_order(pos):
    """sortByMortonCode's permutation (Scene.swift:74-117), stable for equal codes."""
    mn, mx = pos.min(0), pos.max(0)
    ext = mx - mn
    inv = np.where(ext > F32(1e-6), F32(1) / np.where(ext > 0, ext, F32(1)), F32(0)).astype(F32)
    t = (pos - mn) * inv
    sc = F32((1 << 21) - 1)
    q = np.maximum(F32(0), np.minimum(sc, t * sc)).astype(np.uint64)
    code = _expand(q[:, 0]) | (_expand(q[:, 1]) << np.uint64(1)) | (_expand(q[:, 2]) << np.uint64(2))
    return np.argsort(code, kind="stable")
