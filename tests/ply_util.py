"""Test helpers: write PLY files in the layouts the reference's loader reads
(standard 3DGS binary_little_endian; PlayCanvas splat-transform compressed)."""
import numpy as np

_NP = {"float": "<f4", "float32": "<f4", "double": "<f8", "float64": "<f8", "uchar": "<u1", "uint8": "<u1",
       "char": "<i1", "int8": "<i1", "short": "<i2", "int16": "<i2", "ushort": "<u2", "uint16": "<u2",
       "int": "<i4", "int32": "<i4", "uint": "<u4", "uint32": "<u4"}


def header(elements, fmt="binary_little_endian", eol="\n", extra=()):
    lines = ["ply", f"format {fmt} 1.0", "comment written by tests/ply_util.py", *extra]
    for name, count, props in elements:
        lines.append(f"element {name} {count}")
        for pname, ptype in props:
            lines.append(f"property {ptype} {pname}")
    lines.append("end_header")
    return (eol.join(lines) + eol).encode("ascii")


def standard(columns, eol="\n", extra_header=()):
    """columns: list of (name, type, values[n]) in file order."""
    n = len(columns[0][2]) if columns else 0
    dt = np.dtype([(name, _NP[t]) for name, t, _ in columns])
    rec = np.zeros(n, dt)
    for name, t, v in columns:
        rec[name] = np.asarray(v).astype(_NP[t])
    return header([("vertex", n, [(c, t) for c, t, _ in columns])], eol=eol, extra=extra_header) + rec.tobytes()


def gaussian_columns(rng, n, sh_components=16, log_scale=True, logit=True, shuffle=False):
    """A standard 3DGS vertex layout: x y z, f_dc_*, f_rest_*, opacity, scale_*, rot_*."""
    pos = rng.normal(0, 2, (n, 3)).astype(np.float32) + np.float32(5)
    sc = rng.uniform(-6, -2, (n, 3)).astype(np.float32) if log_scale else rng.uniform(0.01, 0.2, (n, 3)).astype(np.float32)
    op = rng.normal(0, 2, n).astype(np.float32) if logit else rng.uniform(0.05, 0.95, n).astype(np.float32)
    rot = rng.normal(0, 1, (n, 4)).astype(np.float32)
    cols = [("x", "float", pos[:, 0]), ("y", "float", pos[:, 1]), ("z", "float", pos[:, 2])]
    cols += [("nx", "float", np.zeros(n)), ("ny", "float", np.zeros(n)), ("nz", "float", np.zeros(n))]
    for i in range(3):
        cols.append((f"f_dc_{i}", "float", rng.normal(0, 1, n)))
    for i in range(3 * (sh_components - 1)):
        cols.append((f"f_rest_{i}", "float", rng.normal(0, 0.1, n)))
    cols.append(("opacity", "float", op))
    for i in range(3):
        cols.append((f"scale_{i}", "float", sc[:, i]))
    for i in range(4):
        cols.append((f"rot_{i}", "float", rot[:, i]))
    if shuffle:
        order = rng.permutation(len(cols))
        cols = [cols[i] for i in order]
    return cols


CHUNK_PROPS = ["min_x", "min_y", "min_z", "max_x", "max_y", "max_z", "min_scale_x", "min_scale_y", "min_scale_z",
               "max_scale_x", "max_scale_y", "max_scale_z", "min_r", "min_g", "min_b", "max_r", "max_g", "max_b"]


def compressed(rng, n, with_sh=True):
    """PlayCanvas compressed PLY: chunk element (18 floats per 256 vertices), packed vertices, sh."""
    nc = (n + 255) // 256
    ch = np.zeros((nc, 18), np.float32)
    lo = rng.uniform(-5, 0, (nc, 3)).astype(np.float32)
    ch[:, 0:3] = lo
    ch[:, 3:6] = lo + rng.uniform(0.5, 4, (nc, 3)).astype(np.float32)
    ch[:, 6:9] = rng.uniform(-7, -4, (nc, 3)).astype(np.float32)
    ch[:, 9:12] = ch[:, 6:9] + rng.uniform(0.5, 3, (nc, 3)).astype(np.float32)
    ch[:, 12:15] = rng.uniform(0, 0.3, (nc, 3)).astype(np.float32)
    ch[:, 15:18] = ch[:, 12:15] + rng.uniform(0.3, 0.7, (nc, 3)).astype(np.float32)
    packed = rng.integers(0, 2 ** 32, (n, 4), dtype=np.uint64).astype(np.uint32)
    els = [("chunk", nc, [(p, "float") for p in CHUNK_PROPS]),
           ("vertex", n, [("packed_position", "uint"), ("packed_rotation", "uint"), ("packed_scale", "uint"),
                          ("packed_color", "uint")])]
    body = ch.tobytes() + packed.tobytes()
    if with_sh:
        els.append(("sh", n, [(f"f_rest_{i}", "uchar") for i in range(9)]))
        body += rng.integers(0, 256, (n, 9), dtype=np.uint8).tobytes()
    return header(els) + body
