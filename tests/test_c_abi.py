"""The C-ABI call sequence of the Swift host layer (swift/Sources/GsmRendererHIP, unverified: no Swift
toolchain here) made from C: tests/c/abi_sequence.c, built by __graft_entry__.build().  The frame it
renders through the C ABI alone (no Python, no torch in that process) must equal the oracle's."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c", "abi_sequence")


def test_c_source_uses_only_declared_entry_points():
    """CPU: every gsm_* call in the C program is declared in include/ (it builds against them)."""
    import re
    src = open(os.path.join(HERE, "c", "abi_sequence.c")).read()
    hdrs = "".join(open(os.path.join(HERE, "..", "include", h)).read()
                   for h in ("gsm_renderer.h", "gsm_debug.h"))
    for name in set(re.findall(r"\b(gsm_\w+)\(", src)):
        assert re.search(rf"\b{name}\(", hdrs), name


@pytest.mark.gpu
def test_c_abi_sequence_renders_the_oracle_frame(tmp_path, oracle):
    sys.path.insert(0, os.path.join(HERE, "..", "gsm-renderer_amd"))
    from gsm_amd import scenes
    assert os.path.exists(BIN), "tests/c/abi_sequence not built (__graft_entry__.build)"
    n, W, H, sh = 20_000, 320, 180, 16
    world, harm, cam = scenes.gen_scene(n, W, H, sh, 1, seed=9)
    (tmp_path / "w.bin").write_bytes(world.tobytes())
    (tmp_path / "h.bin").write_bytes(harm.tobytes())
    cf = np.concatenate([cam["view"], cam["proj"], cam["position"],
                         np.array([cam["focal_x"], cam["focal_y"], cam["near"], cam["far"]], np.float32)])
    (tmp_path / "c.bin").write_bytes(cf.astype(np.float32).tobytes())
    out = tmp_path / "color.bin"
    p = subprocess.run([BIN, str(tmp_path / "w.bin"), str(tmp_path / "h.bin"), str(n), str(sh), str(W), str(H),
                        str(tmp_path / "c.bin"), str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr + p.stdout
    ref = oracle.render(world, harm, sh, cam, W, H, max_gaussians=n)
    got = np.frombuffer(out.read_bytes(), np.uint16).reshape(H, W, 4)
    assert np.array_equal(got, ref["color"])
    assert f"total_assignments {ref['total_assignments']}" in p.stdout
